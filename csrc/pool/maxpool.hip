// Channels-last (NHWC) max pooling for gfx950: the ResNet stem's 3x3/s2/p1
// pool (any k, s, p) without PyTorch's int64 index tensor.
//
// PyTorch's NHWC max_pool2d_with_indices writes an int64 argmax per output
// element (822 MB at ResNet-50 batch 256) and its backward scatters through
// it: 0.25 ms forward + 0.62 ms backward on MI355X (profiles/r50_*_v5.md).
// Here:
//   forward : one lane = one output pixel x one 16-B channel vector; the k*k
//             window is read as 16-B vectors (neighbouring lanes share input
//             lines in L2) and the winning tap per channel is stored as ONE
//             byte (k*k <= 255), 1/8 of the int64 index traffic.
//   backward: a GATHER per input pixel (no atomics, no zero-fill pass): the
//             <= ceil(k/s)^2 windows that contain it are enumerated, their
//             argmax bytes compared with the pixel's tap id, matching dy
//             summed -- every dx element written exactly once.
// Tie-breaking matches PyTorch (first maximum in window order; NaN wins).
#include <cstdlib>
#include <type_traits>

#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include "../common.h"

namespace dmp {
namespace {

// 128 lanes per block: a 112-wide bf16 row of 64 channels is 896 lanes = 7 blocks.
constexpr int kPoolThreads = 128;

struct PoolGeo {
  int N, C, H, W, Ho, Wo, k, s, p, cv;  // cv = C / VEC
};

template <typename T>
__global__ __launch_bounds__(kPoolThreads) void maxpool_fwd_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                          uint8_t* __restrict__ idx, PoolGeo g,
                                                          int row_len) {
  constexpr int VEC = Vec16<T>::N;
  // blockIdx.x = one output row (n, oh), uniform per block: no per-lane 64-bit
  // div/mod chain; lanes run over (ow, channel vector) of that row.
  const int j = blockIdx.y * blockDim.x + threadIdx.x;
  if (j >= row_len) return;
  const int row = blockIdx.x;
  const int n = row / g.Ho, oh = row - n * g.Ho;
  const int ow = j / g.cv, cvi = j - ow * g.cv;
  const int64_t pix = (int64_t)row * g.Wo + ow;
  const int c0 = cvi * VEC;
  const int h0 = oh * g.s - g.p, w0 = ow * g.s - g.p;
  // argmax starts at the first IN-BOUNDS tap (PyTorch semantics): an all -inf
  // window at a border must still route its gradient to a real input pixel
  const uint8_t tap0 = (uint8_t)(max(0, -h0) * g.k + max(0, -w0));
  float m[VEC];
  uint8_t am[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) { m[j] = -INFINITY; am[j] = tap0; }
  for (int a = 0; a < g.k; ++a) {
    const int ih = h0 + a;
    if (ih < 0 || ih >= g.H) continue;
    for (int b = 0; b < g.k; ++b) {
      const int iw = w0 + b;
      if (iw < 0 || iw >= g.W) continue;
      float v[VEC];
      Vec16<T>::load(x + (((int64_t)n * g.H + ih) * g.W + iw) * g.C + c0, v);
      const uint8_t tap = (uint8_t)(a * g.k + b);
#pragma unroll
      for (int j = 0; j < VEC; ++j)
        if (v[j] > m[j] || (v[j] != v[j] && m[j] == m[j])) { m[j] = v[j]; am[j] = tap; }
    }
  }
  Vec16<T>::store(y + pix * g.C + c0, m);
  uint8_t* ip = idx + pix * g.C + c0;
#pragma unroll
  for (int j = 0; j < VEC; ++j) ip[j] = am[j];
}

template <typename T>
__global__ __launch_bounds__(kPoolThreads) void maxpool_bwd_kernel(const T* __restrict__ dy,
                                                          const uint8_t* __restrict__ idx,
                                                          T* __restrict__ dx, PoolGeo g,
                                                          int row_len) {
  constexpr int VEC = Vec16<T>::N;
  // blockIdx.x = one input row (n, ih): the window range in oh is uniform per block.
  const int j = blockIdx.y * blockDim.x + threadIdx.x;
  if (j >= row_len) return;
  const int row = blockIdx.x;
  const int n = row / g.H, ih = row - n * g.H;
  const int iw = j / g.cv, cvi = j - iw * g.cv;
  const int64_t pix = (int64_t)row * g.W + iw;
  const int c0 = cvi * VEC;
  float acc[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) acc[j] = 0.f;
  // windows oh with oh*s - p <= ih <= oh*s - p + k - 1
  const int oh_lo = max(0, (ih + g.p - g.k + g.s) / g.s), oh_hi = min(g.Ho - 1, (ih + g.p) / g.s);
  const int ow_lo = max(0, (iw + g.p - g.k + g.s) / g.s), ow_hi = min(g.Wo - 1, (iw + g.p) / g.s);
  for (int oh = oh_lo; oh <= oh_hi; ++oh) {
    const int a = ih - (oh * g.s - g.p);
    if (a < 0 || a >= g.k) continue;
    for (int ow = ow_lo; ow <= ow_hi; ++ow) {
      const int b = iw - (ow * g.s - g.p);
      if (b < 0 || b >= g.k) continue;
      const uint8_t tap = (uint8_t)(a * g.k + b);
      const int64_t o = (((int64_t)n * g.Ho + oh) * g.Wo + ow) * g.C + c0;
      uint8_t am[VEC];
      if constexpr (VEC == 8) {
        const uint64_t w = *reinterpret_cast<const uint64_t*>(idx + o);
#pragma unroll
        for (int j = 0; j < 8; ++j) am[j] = (uint8_t)(w >> (8 * j));
      } else {
        const uint32_t w = *reinterpret_cast<const uint32_t*>(idx + o);
#pragma unroll
        for (int j = 0; j < 4; ++j) am[j] = (uint8_t)(w >> (8 * j));
      }
      bool any = false;
#pragma unroll
      for (int j = 0; j < VEC; ++j) any |= am[j] == tap;
      if (!any) continue;
      float v[VEC];
      Vec16<T>::load(dy + o, v);
#pragma unroll
      for (int j = 0; j < VEC; ++j)
        if (am[j] == tap) acc[j] += v[j];
    }
  }
  Vec16<T>::store(dx + pix * g.C + c0, acc);
}

// Fixed-geometry fast paths (the ResNet stem's k=3, s=2).  Every tap of the
// forward window and every candidate window of the backward is loaded
// unconditionally from a clamped address and masked afterwards, so all loads
// of a lane are in flight together instead of one dependent round trip per
// tap (the runtime-k kernels above branch around each load).
template <typename T, int K, int S>
__global__ __launch_bounds__(kPoolThreads) void maxpool_fwd_fixed_kernel(const T* __restrict__ x,
                                                                       T* __restrict__ y,
                                                                       uint8_t* __restrict__ idx,
                                                                       PoolGeo g, int row_len) {
  constexpr int VEC = Vec16<T>::N;
  const int j = blockIdx.y * blockDim.x + threadIdx.x;
  if (j >= row_len) return;
  const int row = blockIdx.x;
  const int n = row / g.Ho, oh = row - n * g.Ho;
  const int ow = j / g.cv, cvi = j - ow * g.cv;
  const int c0 = cvi * VEC;
  const int h0 = oh * S - g.p, w0 = ow * S - g.p;
  const T* xn = x + (int64_t)n * g.H * g.W * g.C + c0;
  float v[K][K][VEC];
#pragma unroll
  for (int a = 0; a < K; ++a) {
    const int ih = min(max(h0 + a, 0), g.H - 1);
#pragma unroll
    for (int b = 0; b < K; ++b) {
      const int iw = min(max(w0 + b, 0), g.W - 1);
      Vec16<T>::load(xn + ((int64_t)ih * g.W + iw) * g.C, v[a][b]);
    }
  }
  const uint8_t tap0 = (uint8_t)(max(0, -h0) * K + max(0, -w0));  // first in-bounds tap
  float m[VEC];
  uint8_t am[VEC];
#pragma unroll
  for (int c = 0; c < VEC; ++c) { m[c] = -INFINITY; am[c] = tap0; }
#pragma unroll
  for (int a = 0; a < K; ++a) {
    const bool ha = (unsigned)(h0 + a) < (unsigned)g.H;
#pragma unroll
    for (int b = 0; b < K; ++b) {
      const bool ok = ha && (unsigned)(w0 + b) < (unsigned)g.W;
#pragma unroll
      for (int c = 0; c < VEC; ++c) {
        const float t = v[a][b][c];
        if (ok && (t > m[c] || (t != t && m[c] == m[c]))) { m[c] = t; am[c] = (uint8_t)(a * K + b); }
      }
    }
  }
  const int64_t pix = (int64_t)row * g.Wo + ow;
  Vec16<T>::store(y + pix * g.C + c0, m);
  uint8_t* ip = idx + pix * g.C + c0;
  if constexpr (VEC == 8) {
    uint64_t w = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) w |= (uint64_t)am[c] << (8 * c);
    *reinterpret_cast<uint64_t*>(ip) = w;
  } else {
    uint32_t w = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) w |= (uint32_t)am[c] << (8 * c);
    *reinterpret_cast<uint32_t*>(ip) = w;
  }
}

template <typename T, int K, int S>
__global__ __launch_bounds__(kPoolThreads) void maxpool_bwd_fixed_kernel(const T* __restrict__ dy,
                                                                       const uint8_t* __restrict__ idx,
                                                                       T* __restrict__ dx, PoolGeo g,
                                                                       int row_len) {
  constexpr int VEC = Vec16<T>::N;
  constexpr int MW = (K + S - 1) / S;  // windows containing a pixel, per dim
  const int j = blockIdx.y * blockDim.x + threadIdx.x;
  if (j >= row_len) return;
  const int row = blockIdx.x;
  const int n = row / g.H, ih = row - n * g.H;
  const int iw = j / g.cv, cvi = j - iw * g.cv;
  const int c0 = cvi * VEC;
  const int oh_hi = (ih + g.p) / S, ow_hi = (iw + g.p) / S;
  const int64_t nbase = (int64_t)n * g.Ho * g.Wo * g.C + c0;
  using IdxW = typename std::conditional<VEC == 8, uint64_t, uint32_t>::type;
  IdxW w[MW][MW];
  float v[MW][MW][VEC];
  bool ok[MW][MW];
#pragma unroll
  for (int t = 0; t < MW; ++t) {
    const int oh = oh_hi - t;
    const int a = ih - (oh * S - g.p);
    const bool okh = oh >= 0 && oh < g.Ho && a >= 0 && a < K;
    const int ohc = min(max(oh, 0), g.Ho - 1);
#pragma unroll
    for (int u = 0; u < MW; ++u) {
      const int ow = ow_hi - u;
      const int b = iw - (ow * S - g.p);
      ok[t][u] = okh && ow >= 0 && ow < g.Wo && b >= 0 && b < K;
      const int owc = min(max(ow, 0), g.Wo - 1);
      const int64_t o = nbase + ((int64_t)ohc * g.Wo + owc) * g.C;
      w[t][u] = *reinterpret_cast<const IdxW*>(idx + o);
      Vec16<T>::load(dy + o, v[t][u]);
    }
  }
  float acc[VEC];
#pragma unroll
  for (int c = 0; c < VEC; ++c) acc[c] = 0.f;
#pragma unroll
  for (int t = 0; t < MW; ++t) {
    const int a = ih - ((oh_hi - t) * S - g.p);
#pragma unroll
    for (int u = 0; u < MW; ++u) {
      const int b = iw - ((ow_hi - u) * S - g.p);
      const uint8_t tap = (uint8_t)(a * K + b);
#pragma unroll
      for (int c = 0; c < VEC; ++c)
        if (ok[t][u] && (uint8_t)(w[t][u] >> (8 * c)) == tap) acc[c] += v[t][u][c];
    }
  }
  Vec16<T>::store(dx + ((int64_t)row * g.W + iw) * g.C + c0, acc);
}

// ---------------------------------------------------------------------------
// Stem fusion: training-mode BN + ReLU applied INSIDE the k3/s2 pool.
// The pool's input is the raw conv output x; every tap is normalised on load
// (relu(x * sc[c] + sh[c]), rounded to bf16 exactly as the unfused BN apply
// would store it), so the BN output tensor is never written nor re-read.
// The backward gathers the pool gradient per input pixel as usual, then does
// the BN backward's reductions on the spot: ReLU mask from x through the same
// affine, dz stored, (sum dz, sum dz*(x - mean)) accumulated per thread over a
// grid-stride row loop and folded per block into [2][blocks][C] partials.
// ---------------------------------------------------------------------------
template <int K, int S>
__global__ __launch_bounds__(kPoolThreads) void bnpool_fwd_kernel(
    const __bf16* __restrict__ x, const float* __restrict__ sc, const float* __restrict__ sh,
    __bf16* __restrict__ y, uint8_t* __restrict__ idx, PoolGeo g, int row_len) {
  constexpr int VEC = 8;
  const int j = blockIdx.y * blockDim.x + threadIdx.x;
  if (j >= row_len) return;
  const int row = blockIdx.x;
  const int n = row / g.Ho, oh = row - n * g.Ho;
  const int ow = j / g.cv, cvi = j - ow * g.cv;
  const int c0 = cvi * VEC;
  const int h0 = oh * S - g.p, w0 = ow * S - g.p;
  const __bf16* xn = x + (int64_t)n * g.H * g.W * g.C + c0;
  float v[K][K][VEC];
#pragma unroll
  for (int a = 0; a < K; ++a) {
    const int ih = min(max(h0 + a, 0), g.H - 1);
#pragma unroll
    for (int b = 0; b < K; ++b) {
      const int iw = min(max(w0 + b, 0), g.W - 1);
      Vec16<__bf16>::load(xn + ((int64_t)ih * g.W + iw) * g.C, v[a][b]);
    }
  }
  float s8[VEC], t8[VEC];
  {
    const f32x4 s0 = *reinterpret_cast<const f32x4*>(sc + c0), s1 = *reinterpret_cast<const f32x4*>(sc + c0 + 4);
    const f32x4 t0 = *reinterpret_cast<const f32x4*>(sh + c0), t1 = *reinterpret_cast<const f32x4*>(sh + c0 + 4);
#pragma unroll
    for (int c = 0; c < 4; ++c) { s8[c] = s0[c]; s8[c + 4] = s1[c]; t8[c] = t0[c]; t8[c + 4] = t1[c]; }
  }
  const uint8_t tap0 = (uint8_t)(max(0, -h0) * K + max(0, -w0));
  float m[VEC];
  uint8_t am[VEC];
#pragma unroll
  for (int c = 0; c < VEC; ++c) { m[c] = -INFINITY; am[c] = tap0; }
#pragma unroll
  for (int a = 0; a < K; ++a) {
    const bool ha = (unsigned)(h0 + a) < (unsigned)g.H;
#pragma unroll
    for (int b = 0; b < K; ++b) {
      const bool ok = ha && (unsigned)(w0 + b) < (unsigned)g.W;
#pragma unroll
      for (int c = 0; c < VEC; ++c) {
        // the BN+ReLU output as the unfused apply pass would have stored it
        const float t = (float)(__bf16)fmaxf(fmaf(v[a][b][c], s8[c], t8[c]), 0.f);
        if (ok && (t > m[c] || (t != t && m[c] == m[c]))) { m[c] = t; am[c] = (uint8_t)(a * K + b); }
      }
    }
  }
  const int64_t pix = (int64_t)row * g.Wo + ow;
  Vec16<__bf16>::store(y + pix * g.C + c0, m);
  uint64_t w = 0;
#pragma unroll
  for (int c = 0; c < 8; ++c) w |= (uint64_t)am[c] << (8 * c);
  *reinterpret_cast<uint64_t*>(idx + pix * g.C + c0) = w;
}

// Two vertically adjacent output rows per thread (K = 3, S = 2): the five
// input rows they span are loaded once (15 taps for 2 outputs instead of 18),
// as raw bf16 vectors all in flight together, then normalised and pooled.
template <int K, int S>
__global__ __launch_bounds__(kPoolThreads) void bnpool_fwd2_kernel(
    const __bf16* __restrict__ x, const float* __restrict__ sc, const float* __restrict__ sh,
    __bf16* __restrict__ y, uint8_t* __restrict__ idx, PoolGeo g, int row_len) {
  static_assert(K == 3 && S == 2, "two-row stem pool: 3x3 / stride 2");
  constexpr int VEC = 8, NR = K + S;  // 5 input rows
  const int j = blockIdx.y * blockDim.x + threadIdx.x;
  if (j >= row_len) return;
  const int prow = blockIdx.x;           // output row pair
  const int hp = (g.Ho + 1) / 2;
  const int n = prow / hp, oh0 = (prow - n * hp) * 2;
  const int ow = j / g.cv, cvi = j - ow * g.cv;
  const int c0 = cvi * VEC;
  const int h0 = oh0 * S - g.p, w0 = ow * S - g.p;
  const __bf16* xn = x + (int64_t)n * g.H * g.W * g.C + c0;
  bf16x8 raw[NR][K];
#pragma unroll
  for (int a = 0; a < NR; ++a) {
    const int ih = min(max(h0 + a, 0), g.H - 1);
#pragma unroll
    for (int b = 0; b < K; ++b) {
      const int iw = min(max(w0 + b, 0), g.W - 1);
      raw[a][b] = *reinterpret_cast<const bf16x8*>(xn + ((int64_t)ih * g.W + iw) * g.C);
    }
  }
  float s8[VEC], t8[VEC];
  {
    const f32x4 s0 = *reinterpret_cast<const f32x4*>(sc + c0), s1 = *reinterpret_cast<const f32x4*>(sc + c0 + 4);
    const f32x4 t0 = *reinterpret_cast<const f32x4*>(sh + c0), t1 = *reinterpret_cast<const f32x4*>(sh + c0 + 4);
#pragma unroll
    for (int c = 0; c < 4; ++c) { s8[c] = s0[c]; s8[c + 4] = s1[c]; t8[c] = t0[c]; t8[c + 4] = t1[c]; }
  }
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int oh = oh0 + r;
    if (oh >= g.Ho) break;
    const int hr = h0 + r * S;
    const uint8_t tap0 = (uint8_t)(max(0, -hr) * K + max(0, -w0));
    float m[VEC];
    uint8_t am[VEC];
#pragma unroll
    for (int c = 0; c < VEC; ++c) { m[c] = -INFINITY; am[c] = tap0; }
#pragma unroll
    for (int a = 0; a < K; ++a) {
      const bool ha = (unsigned)(hr + a) < (unsigned)g.H;
#pragma unroll
      for (int b = 0; b < K; ++b) {
        const bool ok = ha && (unsigned)(w0 + b) < (unsigned)g.W;
        const f32x8 v = __builtin_convertvector(raw[r * S + a][b], f32x8);
#pragma unroll
        for (int c = 0; c < VEC; ++c) {
          // the BN+ReLU output as the unfused apply pass would have stored it
          const float t = (float)(__bf16)fmaxf(fmaf(v[c], s8[c], t8[c]), 0.f);
          if (ok && (t > m[c] || (t != t && m[c] == m[c]))) { m[c] = t; am[c] = (uint8_t)(a * K + b); }
        }
      }
    }
    const int64_t pix = ((int64_t)n * g.Ho + oh) * g.Wo + ow;
    Vec16<__bf16>::store(y + pix * g.C + c0, m);
    uint64_t w = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) w |= (uint64_t)am[c] << (8 * c);
    *reinterpret_cast<uint64_t*>(idx + pix * g.C + c0) = w;
  }
}

template <int K, int S>
__global__ __launch_bounds__(kPoolThreads) void bnpool_bwd_kernel(
    const __bf16* __restrict__ dy, const uint8_t* __restrict__ idx, const __bf16* __restrict__ x,
    const float* __restrict__ sc, const float* __restrict__ sh, const float* __restrict__ mean,
    __bf16* __restrict__ dz, float* __restrict__ part, double* __restrict__ zsums, PoolGeo g, int row_len,
    int rows) {
  constexpr int VEC = 8;
  constexpr int MW = (K + S - 1) / S;
  zero_moments(zsums, 2 * g.C);
  const int j = blockIdx.y * blockDim.x + threadIdx.x;
  const bool active = j < row_len;
  const int iw = active ? j / g.cv : 0, cvi = active ? j - (j / g.cv) * g.cv : 0;
  const int c0 = cvi * VEC;
  float s8[VEC], t8[VEC], mu[VEC], msum[VEC], msq[VEC];
#pragma unroll
  for (int c = 0; c < VEC; ++c) {
    s8[c] = sc[c0 + c]; t8[c] = sh[c0 + c]; mu[c] = mean[c0 + c];
    msum[c] = 0.f; msq[c] = 0.f;
  }
  using IdxW = uint64_t;
  for (int row = blockIdx.x; active && row < rows; row += gridDim.x) {
    const int n = row / g.H, ih = row - n * g.H;
    const int oh_hi = (ih + g.p) / S, ow_hi = (iw + g.p) / S;
    const int64_t nbase = (int64_t)n * g.Ho * g.Wo * g.C + c0;
    IdxW w[MW][MW];
    float v[MW][MW][VEC];
    bool ok[MW][MW];
#pragma unroll
    for (int t = 0; t < MW; ++t) {
      const int oh = oh_hi - t;
      const int a = ih - (oh * S - g.p);
      const bool okh = oh >= 0 && oh < g.Ho && a >= 0 && a < K;
      const int ohc = min(max(oh, 0), g.Ho - 1);
#pragma unroll
      for (int u = 0; u < MW; ++u) {
        const int ow = ow_hi - u;
        const int b = iw - (ow * S - g.p);
        ok[t][u] = okh && ow >= 0 && ow < g.Wo && b >= 0 && b < K;
        const int owc = min(max(ow, 0), g.Wo - 1);
        const int64_t o = nbase + ((int64_t)ohc * g.Wo + owc) * g.C;
        w[t][u] = *reinterpret_cast<const IdxW*>(idx + o);
        Vec16<__bf16>::load(dy + o, v[t][u]);
      }
    }
    const int64_t xo = ((int64_t)row * g.W + iw) * g.C + c0;
    float xv[VEC];
    Vec16<__bf16>::load(x + xo, xv);
    float acc[VEC];
#pragma unroll
    for (int c = 0; c < VEC; ++c) acc[c] = 0.f;
#pragma unroll
    for (int t = 0; t < MW; ++t) {
      const int a = ih - ((oh_hi - t) * S - g.p);
#pragma unroll
      for (int u = 0; u < MW; ++u) {
        const int b = iw - ((ow_hi - u) * S - g.p);
        const uint8_t tap = (uint8_t)(a * K + b);
#pragma unroll
        for (int c = 0; c < VEC; ++c)
          if (ok[t][u] && (uint8_t)(w[t][u] >> (8 * c)) == tap) acc[c] += v[t][u][c];
      }
    }
#pragma unroll
    for (int c = 0; c < VEC; ++c) {
      const float gq = (float)(__bf16)acc[c];  // the pool gradient as the unfused pass stores it
      const float d = fmaf(xv[c], s8[c], t8[c]) > 0.f ? gq : 0.f;
      acc[c] = d;
      msum[c] += d;
      msq[c] = fmaf(d, xv[c] - mu[c], msq[c]);
    }
    Vec16<__bf16>::store(dz + xo, acc);
  }
  // fold the threads of this block that share a channel vector (tid % cv, host
  // guarantees kPoolThreads % cv == 0) into one [2][C] partial row
  __shared__ float red[2][kPoolThreads][VEC];
#pragma unroll
  for (int c = 0; c < VEC; ++c) {
    red[0][threadIdx.x][c] = active ? msum[c] : 0.f;
    red[1][threadIdx.x][c] = active ? msq[c] : 0.f;
  }
  __syncthreads();
  const int rb = gridDim.x * gridDim.y, prow = blockIdx.y * gridDim.x + blockIdx.x;
  for (int c = threadIdx.x; c < g.C; c += kPoolThreads) {
    const int cv = c / VEC, e = c - cv * VEC;
    float a0 = 0.f, a1 = 0.f;
    for (int t = cv; t < kPoolThreads; t += g.cv) {
      a0 += red[0][t][e];
      a1 += red[1][t][e];
    }
    part[(int64_t)prow * g.C + c] = a0;
    part[(int64_t)(rb + prow) * g.C + c] = a1;
  }
}

// Global average pool backward, channels-last: dx[n, hw, c] = g[n, c] / HW.
// PyTorch returns an expanded gradient here that the next backward
// materialises with a strided copy (~1.3 TB/s, profiles finding 13); this is
// one 16-B vector store per lane, g read from L2.
template <typename T>
__global__ __launch_bounds__(256) void gap_bwd_kernel(const T* __restrict__ g, T* __restrict__ dx,
                                                      int HW, int cv, float inv, int64_t total) {
  constexpr int VEC = Vec16<T>::N;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int64_t row = i / cv;               // n * HW + hw
  const int cvi = (int)(i - row * cv);
  const int n = (int)(row / HW);
  float v[VEC];
  Vec16<T>::load(g + ((int64_t)n * cv + cvi) * VEC, v);
#pragma unroll
  for (int j = 0; j < VEC; ++j) v[j] *= inv;
  Vec16<T>::store(dx + i * VEC, v);
}

PoolGeo make_geo(const at::Tensor& x, int64_t k, int64_t s, int64_t p, int vec) {
  PoolGeo g;
  g.N = (int)x.size(0); g.C = (int)x.size(1); g.H = (int)x.size(2); g.W = (int)x.size(3);
  g.k = (int)k; g.s = (int)s; g.p = (int)p;
  g.Ho = (g.H + 2 * g.p - g.k) / g.s + 1;
  g.Wo = (g.W + 2 * g.p - g.k) / g.s + 1;
  g.cv = g.C / vec;
  return g;
}

// set_pool_generic(true) routes every geometry through the runtime-k kernels
// (A/B timing, tools/pool_bench.py).
bool g_pool_generic = false;
bool fixed_geometry_disabled() { return g_pool_generic; }

void check_x(const at::Tensor& x, const char* name) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 4, name, " must be a 4-D GPU tensor");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kFloat,
              name, " must be bf16 or fp32");
  TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast), name, " must be channels_last");
  const int vec = x.scalar_type() == at::kBFloat16 ? 8 : 4;
  TORCH_CHECK(x.size(1) % vec == 0, name, ": channels must be a multiple of ", vec);
}

}  // namespace

// Returns (y, argmax-tap bytes [N, Ho, Wo, C] uint8).
std::vector<at::Tensor> maxpool2d_forward(const at::Tensor& x, int64_t k, int64_t s, int64_t p) {
  check_x(x, "x");
  TORCH_CHECK(k >= 1 && k * k <= 255 && s >= 1 && p >= 0 && 2 * p <= k, "unsupported pool geometry");
  const int vec = x.scalar_type() == at::kBFloat16 ? 8 : 4;
  PoolGeo g = make_geo(x, k, s, p, vec);
  TORCH_CHECK(g.Ho > 0 && g.Wo > 0, "pool output is empty");
  auto y = at::empty({g.N, g.C, g.Ho, g.Wo}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto idx = at::empty({(int64_t)g.N * g.Ho * g.Wo * g.C}, x.options().dtype(at::kByte));
  const int row_len = g.Wo * g.cv;
  if ((int64_t)g.N * g.Ho * row_len == 0) return {y, idx};
  auto stream = at::hip::getCurrentHIPStream();
  const dim3 blocks((unsigned)(g.N * g.Ho), (unsigned)((row_len + kPoolThreads - 1) / kPoolThreads));
  const bool fixed = k == 3 && s == 2 && !fixed_geometry_disabled();
  if (fixed && x.scalar_type() == at::kBFloat16)
    hipLaunchKernelGGL((maxpool_fwd_fixed_kernel<__bf16, 3, 2>), blocks, dim3(kPoolThreads), 0, stream,
                       reinterpret_cast<const __bf16*>(x.data_ptr()), reinterpret_cast<__bf16*>(y.data_ptr()),
                       idx.data_ptr<uint8_t>(), g, row_len);
  else if (fixed)
    hipLaunchKernelGGL((maxpool_fwd_fixed_kernel<float, 3, 2>), blocks, dim3(kPoolThreads), 0, stream,
                       x.data_ptr<float>(), y.data_ptr<float>(), idx.data_ptr<uint8_t>(), g, row_len);
  else if (x.scalar_type() == at::kBFloat16)
    hipLaunchKernelGGL(maxpool_fwd_kernel<__bf16>, blocks, dim3(kPoolThreads), 0, stream,
                       reinterpret_cast<const __bf16*>(x.data_ptr()), reinterpret_cast<__bf16*>(y.data_ptr()),
                       idx.data_ptr<uint8_t>(), g, row_len);
  else
    hipLaunchKernelGGL(maxpool_fwd_kernel<float>, blocks, dim3(kPoolThreads), 0, stream,
                       x.data_ptr<float>(), y.data_ptr<float>(), idx.data_ptr<uint8_t>(), g, row_len);
  return {y, idx};
}

at::Tensor maxpool2d_backward(const at::Tensor& dy, const at::Tensor& idx, int64_t H, int64_t W,
                              int64_t k, int64_t s, int64_t p) {
  check_x(dy, "dy");
  const int vec = dy.scalar_type() == at::kBFloat16 ? 8 : 4;
  PoolGeo g;
  g.N = (int)dy.size(0); g.C = (int)dy.size(1); g.H = (int)H; g.W = (int)W;
  g.k = (int)k; g.s = (int)s; g.p = (int)p;
  g.Ho = (int)dy.size(2); g.Wo = (int)dy.size(3);
  g.cv = g.C / vec;
  TORCH_CHECK(g.Ho == (g.H + 2 * g.p - g.k) / g.s + 1 && g.Wo == (g.W + 2 * g.p - g.k) / g.s + 1,
              "dy does not match the pool geometry");
  TORCH_CHECK(idx.numel() == dy.numel() && idx.scalar_type() == at::kByte, "bad argmax tensor");
  auto dx = at::empty({g.N, g.C, g.H, g.W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int row_len = g.W * g.cv;
  if ((int64_t)g.N * g.H * row_len == 0) return dx;
  auto stream = at::hip::getCurrentHIPStream();
  const dim3 blocks((unsigned)(g.N * g.H), (unsigned)((row_len + kPoolThreads - 1) / kPoolThreads));
  const bool fixed = k == 3 && s == 2 && !fixed_geometry_disabled();
  if (fixed && dy.scalar_type() == at::kBFloat16)
    hipLaunchKernelGGL((maxpool_bwd_fixed_kernel<__bf16, 3, 2>), blocks, dim3(kPoolThreads), 0, stream,
                       reinterpret_cast<const __bf16*>(dy.data_ptr()), idx.data_ptr<uint8_t>(),
                       reinterpret_cast<__bf16*>(dx.data_ptr()), g, row_len);
  else if (fixed)
    hipLaunchKernelGGL((maxpool_bwd_fixed_kernel<float, 3, 2>), blocks, dim3(kPoolThreads), 0, stream,
                       dy.data_ptr<float>(), idx.data_ptr<uint8_t>(), dx.data_ptr<float>(), g, row_len);
  else if (dy.scalar_type() == at::kBFloat16)
    hipLaunchKernelGGL(maxpool_bwd_kernel<__bf16>, blocks, dim3(kPoolThreads), 0, stream,
                       reinterpret_cast<const __bf16*>(dy.data_ptr()), idx.data_ptr<uint8_t>(),
                       reinterpret_cast<__bf16*>(dx.data_ptr()), g, row_len);
  else
    hipLaunchKernelGGL(maxpool_bwd_kernel<float>, blocks, dim3(kPoolThreads), 0, stream,
                       dy.data_ptr<float>(), idx.data_ptr<uint8_t>(), dx.data_ptr<float>(), g, row_len);
  return dx;
}

// batchnorm.hip
void bn_reduce_partials_launch(const float* part, int rb, int C, double* sums, double count,
                               hipStream_t stream);

namespace {
void check_bnpool(const at::Tensor& x, const at::Tensor& scale, const at::Tensor& shift, int64_t k,
                  int64_t s, int64_t p) {
  check_x(x, "x");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && k == 3 && s == 2 && p <= 1,
              "fused BN+pool covers bf16 3x3/s2 pools");
  TORCH_CHECK(kPoolThreads % (x.size(1) / 8) == 0, "fused BN+pool: C/8 must divide ", kPoolThreads);
  for (const auto* t : {&scale, &shift})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous() && t->numel() == x.size(1),
                "BN coefficients must be contiguous fp32 [C]");
}
}  // namespace

// y, argmax = maxpool(relu(x * scale + shift)) -- BN apply + ReLU fused into the pool.
std::vector<at::Tensor> maxpool2d_bn_forward(const at::Tensor& x, const at::Tensor& scale,
                                             const at::Tensor& shift, int64_t k, int64_t s, int64_t p) {
  check_bnpool(x, scale, shift, k, s, p);
  PoolGeo g = make_geo(x, k, s, p, 8);
  TORCH_CHECK(g.Ho > 0 && g.Wo > 0, "pool output is empty");
  auto y = at::empty({g.N, g.C, g.Ho, g.Wo}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto idx = at::empty({(int64_t)g.N * g.Ho * g.Wo * g.C}, x.options().dtype(at::kByte));
  const int row_len = g.Wo * g.cv;
  if ((int64_t)g.N * g.Ho * row_len == 0) return {y, idx};
  static const bool one_row = [] { const char* e = std::getenv("DMP_POOL_FWD1"); return e && e[0] == '1'; }();
  if (one_row) {  // A/B: one output row per thread
    const dim3 blocks((unsigned)(g.N * g.Ho), (unsigned)((row_len + kPoolThreads - 1) / kPoolThreads));
    hipLaunchKernelGGL((bnpool_fwd_kernel<3, 2>), blocks, dim3(kPoolThreads), 0, at::hip::getCurrentHIPStream(),
                       reinterpret_cast<const __bf16*>(x.data_ptr()), scale.data_ptr<float>(), shift.data_ptr<float>(),
                       reinterpret_cast<__bf16*>(y.data_ptr()), idx.data_ptr<uint8_t>(), g, row_len);
  } else {
    const dim3 blocks((unsigned)(g.N * ((g.Ho + 1) / 2)), (unsigned)((row_len + kPoolThreads - 1) / kPoolThreads));
    hipLaunchKernelGGL((bnpool_fwd2_kernel<3, 2>), blocks, dim3(kPoolThreads), 0, at::hip::getCurrentHIPStream(),
                       reinterpret_cast<const __bf16*>(x.data_ptr()), scale.data_ptr<float>(), shift.data_ptr<float>(),
                       reinterpret_cast<__bf16*>(y.data_ptr()), idx.data_ptr<uint8_t>(), g, row_len);
  }
  DMP_HIP_CHECK(hipGetLastError());
  return {y, idx};
}

// dz = relu_mask(x) * maxpool_backward(dy), plus fp64 [2C+1] = (sum dz, sum dz*(x-mean), rows)
std::vector<at::Tensor> maxpool2d_bn_backward(const at::Tensor& dy, const at::Tensor& idx, const at::Tensor& x,
                                              const at::Tensor& scale, const at::Tensor& shift,
                                              const at::Tensor& mean, int64_t k, int64_t s, int64_t p) {
  check_bnpool(x, scale, shift, k, s, p);
  check_x(dy, "dy");
  TORCH_CHECK(mean.is_cuda() && mean.scalar_type() == at::kFloat && mean.is_contiguous() &&
                  mean.numel() == x.size(1), "mean must be contiguous fp32 [C]");
  PoolGeo g = make_geo(x, k, s, p, 8);
  TORCH_CHECK(dy.size(0) == g.N && dy.size(1) == g.C && dy.size(2) == g.Ho && dy.size(3) == g.Wo,
              "dy does not match the pool geometry");
  TORCH_CHECK(idx.numel() == dy.numel() && idx.scalar_type() == at::kByte, "bad argmax tensor");
  auto dz = at::empty_like(x, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto sums = at::empty({2 * (int64_t)g.C + 1}, x.options().dtype(at::kDouble));
  // (one thread per 2 x 2 input quad -- a quarter of the dy / argmax loads --
  // measured 2.54 vs 2.15 ms at batch 2048 with 164 VGPRs; profiles finding 68)
  const int row_len = g.W * g.cv;
  const int rows = g.N * g.H;
  const unsigned gx = (unsigned)std::min(rows, 1024), gy = (unsigned)((row_len + kPoolThreads - 1) / kPoolThreads);
  const int rb = (int)(gx * gy);
  auto part = at::empty({2, rb, (int64_t)g.C}, x.options().dtype(at::kFloat));
  auto stream = at::hip::getCurrentHIPStream();
  hipLaunchKernelGGL((bnpool_bwd_kernel<3, 2>), dim3(gx, gy), dim3(kPoolThreads), 0, stream,
                     reinterpret_cast<const __bf16*>(dy.data_ptr()), idx.data_ptr<uint8_t>(),
                     reinterpret_cast<const __bf16*>(x.data_ptr()), scale.data_ptr<float>(),
                     shift.data_ptr<float>(), mean.data_ptr<float>(), reinterpret_cast<__bf16*>(dz.data_ptr()),
                     part.data_ptr<float>(), moments_zero_target(sums.data_ptr<double>(), rb), g, row_len, rows);
  DMP_HIP_CHECK(hipGetLastError());
  bn_reduce_partials_launch(part.data_ptr<float>(), rb, g.C, sums.data_ptr<double>(), (double)g.N * g.H * g.W,
                            stream);
  return {dz, sums};
}

at::Tensor global_avgpool_backward(const at::Tensor& g, int64_t H, int64_t W) {
  TORCH_CHECK(g.is_cuda() && g.dim() == 2 && g.is_contiguous(), "g must be a contiguous [N, C] GPU tensor");
  TORCH_CHECK(g.scalar_type() == at::kBFloat16 || g.scalar_type() == at::kFloat, "g must be bf16 or fp32");
  const int vec = g.scalar_type() == at::kBFloat16 ? 8 : 4;
  const int64_t N = g.size(0), C = g.size(1);
  TORCH_CHECK(C % vec == 0 && H > 0 && W > 0, "channels must be a multiple of ", vec);
  auto dx = at::empty({N, C, H, W}, g.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int64_t total = N * H * W * (C / vec);
  if (total == 0) return dx;
  const unsigned blocks = (unsigned)((total + 255) / 256);
  const float inv = 1.f / (float)(H * W);
  auto stream = at::hip::getCurrentHIPStream();
  if (g.scalar_type() == at::kBFloat16)
    hipLaunchKernelGGL(gap_bwd_kernel<__bf16>, dim3(blocks), dim3(256), 0, stream,
                       reinterpret_cast<const __bf16*>(g.data_ptr()), reinterpret_cast<__bf16*>(dx.data_ptr()),
                       (int)(H * W), (int)(C / vec), inv, total);
  else
    hipLaunchKernelGGL(gap_bwd_kernel<float>, dim3(blocks), dim3(256), 0, stream, g.data_ptr<float>(),
                       dx.data_ptr<float>(), (int)(H * W), (int)(C / vec), inv, total);
  return dx;
}

void set_pool_generic(bool on) { g_pool_generic = on; }

}  // namespace dmp
