// Channels-last 3x3 depthwise convolution (groups == channels, padding 1,
// stride 1 or 2) -- forward, data gradient and weight gradient -- for the
// MobileNetV2 inverted-residual blocks (reference model/mobilenetv2.py:19,
// "3x3 depthwise conv: memory-bound; LDS-tiled direct conv").
//
// Measured motivation (profiles/mnv2_bs512_1gpu_v1.md): MIOpen runs bf16 NHWC
// depthwise as naive_conv forward / data-grad and a grouped-GEMM weight-grad
// that together take 315 of 326 ms per CIFAR bs512 step.
//
// Design (memory-bound, so: every byte once, 16-B accesses, fp32 math):
//   * a lane owns one 16-byte channel vector (8 bf16 / 4 fp32 channels) and a
//     strip of TW consecutive output columns of one output row; the 3 x
//     (TW-1)*stride+3 input window is streamed through registers, so each input
//     vector is loaded once per strip instead of 9 times;
//   * consecutive lanes take consecutive channel vectors of the same pixel, so a
//     wave reads/writes whole 16-B-aligned pixel rows of C channels;
//   * the 9 taps x 8 channels of weights (read from the module's own [C][9]
//     tensor and transposed in registers) live in
//     registers for the whole launch;
//   * forward can emit per-block BatchNorm moment partials of its OUTPUT
//     (sum, sum^2) for the following BN -- same partial format the BN and GEMM
//     kernels use, reduced by bn_reduce_partials_launch;
//   * weight gradient: each lane accumulates its 9 x 8 products in fp32 over
//     the pixels it visits, the block combines lanes of the same channel vector
//     in LDS and writes one fp32 partial row; a column-reduce kernel sums the
//     partials deterministically (no atomics).
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include "../common.h"

namespace dmp {

void bn_reduce_partials_launch(const float* part, int rb, int C, double* sums, double count,
                               hipStream_t stream);

namespace {

constexpr int kThreads = 256;
constexpr int TW = 4;  // output columns per lane

struct Geo {
  int N, H, W, C, OH, OW, stride;
  int cv;      // channel vectors
  int tc;      // channel vectors per block row
  int spp;     // strips per block pass (kThreads / tc)
  int strips;  // OW / TW (ceil)
};

template <typename T>
__device__ __forceinline__ void ldv(const T* p, float (&v)[Vec16<T>::N]) { Vec16<T>::load(p, v); }

// Window loads are issued unconditionally from clamped addresses and the
// out-of-range ones zeroed afterwards (a select, not a branch): a load under a
// per-column branch is waited for before the next one is issued, which made
// every column of the 3 x (TW+2) window a full memory round trip (ISA showed
// 18-54 serialized load -> vmcnt(0) pairs per kernel).
template <typename T>
__device__ __forceinline__ typename Vec16<T>::raw ldraw(const T* p) {
  return *reinterpret_cast<const typename Vec16<T>::raw*>(p);
}

template <typename T>
__device__ __forceinline__ void cvt_masked(typename Vec16<T>::raw r, bool ok, float (&v)[Vec16<T>::N]) {
  using R = typename Vec16<T>::raw;
  r = ok ? r : R{};
  if constexpr (Vec16<T>::N == 8) {
    const f32x8 f = __builtin_convertvector(r, f32x8);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = f[i];
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = r[i];
  }
}

__device__ __forceinline__ int clampi(int v, int hi) { return v < 0 ? 0 : (v > hi ? hi : v); }

// The lane's VEC channels x 9 taps straight from the [C][9] weight (the
// module's own [C,1,3,3] tensor, bf16 or fp32): channels c0..c0+VEC-1 are one
// contiguous run of 9*VEC elements, read as 16-B (or 8-B) vectors and
// transposed in registers -- no per-call fp32 [9][C] copy (two torch launches
// per forward and per data gradient).  The host checks 16-B base alignment.
template <typename WT, int VEC>
__device__ __forceinline__ void load_taps(const WT* __restrict__ wc, int c0, float (&wr)[9][VEC]) {
  constexpr int NE = 9 * VEC, NB = NE * (int)sizeof(WT);
  using U = typename std::conditional<NB % 16 == 0, uint4, uint2>::type;
  constexpr int NU = NB / (int)sizeof(U);
  const U* p = reinterpret_cast<const U*>(wc + (int64_t)c0 * 9);
  U r[NU];
#pragma unroll
  for (int i = 0; i < NU; ++i) r[i] = p[i];
  WT e[NE];
  __builtin_memcpy(e, r, NB);
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int j = 0; j < VEC; ++j) wr[t][j] = (float)e[j * 9 + t];
}

// ---------------------------------------------------------------------------
// forward: y[n,oh,ow,c] = sum_{kh,kw} x[n, oh*s-1+kh, ow*s-1+kw, c] * w[kh,kw,c]
// grid.x = ceil(N*OH*strips / spp), grid.y = channel chunks
// ---------------------------------------------------------------------------
// S = stride as a template constant: every tap index in the unrolled loops is
// then a compile-time constant, so wr/acc stay in registers (a runtime stride
// made the compiler index them dynamically -> scratch memory, measured 2-4x).
template <typename T, typename WT, bool MOMENTS, int S>
__global__ __launch_bounds__(kThreads) void dw_fwd_kernel(const T* __restrict__ x,
                                                         const WT* __restrict__ wc,
                                                         T* __restrict__ y, Geo g,
                                                         float* __restrict__ part,
                                                         double* __restrict__ zsums) {
  if (MOMENTS) zero_moments(zsums, 2 * g.C);
  constexpr int VEC = Vec16<T>::N;
  const int tid = threadIdx.x;
  const int lc = tid % g.tc, ls = tid / g.tc;
  const int cvec = blockIdx.y * g.tc + lc;
  const bool active_c = ls < g.spp && cvec < g.cv;
  const int c0 = cvec * VEC;
  float wr[9][VEC];
  float ms[VEC], mq[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) { ms[j] = 0.f; mq[j] = 0.f; }
  const int64_t total = (int64_t)g.N * g.OH * g.strips;
  const int64_t sidx = (int64_t)blockIdx.x * g.spp + ls;
  if (active_c && sidx < total) {
    load_taps<WT, VEC>(wc, c0, wr);
    const int st = (int)(sidx % g.strips);
    const int64_t nr = sidx / g.strips;
    const int oh = (int)(nr % g.OH);
    const int n = (int)(nr / g.OH);
    const int ow0 = st * TW;
    float acc[TW][VEC];
#pragma unroll
    for (int o = 0; o < TW; ++o)
#pragma unroll
      for (int j = 0; j < VEC; ++j) acc[o][j] = 0.f;
    constexpr int NCI = (TW - 1) * S + 3;  // input columns touched
    const int iw0 = ow0 * S - 1;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int ih = oh * S - 1 + kh;
      if (ih < 0 || ih >= g.H) continue;
      const T* row = x + (((int64_t)n * g.H + ih) * g.W) * g.C + c0;
      typename Vec16<T>::raw raw[NCI];
#pragma unroll
      for (int ci = 0; ci < NCI; ++ci) raw[ci] = ldraw<T>(row + (int64_t)clampi(iw0 + ci, g.W - 1) * g.C);
#pragma unroll
      for (int ci = 0; ci < NCI; ++ci) {
        const int iw = iw0 + ci;
        float v[VEC];
        cvt_masked<T>(raw[ci], iw >= 0 && iw < g.W, v);
#pragma unroll
        for (int o = 0; o < TW; ++o) {
          const int kw = ci - o * S;
          if (kw < 0 || kw > 2) continue;
#pragma unroll
          for (int j = 0; j < VEC; ++j) acc[o][j] = fmaf(v[j], wr[kh * 3 + kw][j], acc[o][j]);
        }
      }
    }
#pragma unroll
    for (int o = 0; o < TW; ++o) {
      const int ow = ow0 + o;
      if (ow >= g.OW) break;
      T* dst = y + (((int64_t)n * g.OH + oh) * g.OW + ow) * g.C + c0;
      Vec16<T>::store(dst, acc[o]);
      if (MOMENTS) {
        float r[VEC];
        Vec16<T>::load(dst, r);  // moments of the ROUNDED stored values (L1 hit)
#pragma unroll
        for (int j = 0; j < VEC; ++j) { ms[j] += r[j]; mq[j] = fmaf(r[j], r[j], mq[j]); }
      }
    }
  }
  if (MOMENTS) {
    __shared__ float lds[2][kThreads * VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      lds[0][j * kThreads + tid] = ms[j];
      lds[1][j * kThreads + tid] = mq[j];
    }
    __syncthreads();
    const int nout = g.tc * VEC;
    for (int o = tid; o < nout; o += kThreads) {
      const int c_l = o % g.tc, e = o / g.tc;
      const int cg = (blockIdx.y * g.tc + c_l) * VEC + e;
      if (cg >= g.C) continue;
      float s = 0.f, q = 0.f;
      for (int r = 0; r < g.spp; ++r) {
        s += lds[0][e * kThreads + r * g.tc + c_l];
        q += lds[1][e * kThreads + r * g.tc + c_l];
      }
      part[(int64_t)blockIdx.x * g.C + cg] = s;
      part[(int64_t)(gridDim.x + blockIdx.x) * g.C + cg] = q;
    }
  }
}

// ---------------------------------------------------------------------------
// data gradient: dx[n,ih,iw,c] = sum over (kh,kw) with oh = (ih+1-kh)/s,
// ow = (iw+1-kw)/s integral and in range of dy[n,oh,ow,c] * w[kh,kw,c].
// One lane: 8 channels x TW consecutive input columns of one input row.
// ---------------------------------------------------------------------------
template <typename T, typename WT, int S>
__global__ __launch_bounds__(kThreads) void dw_dgrad_kernel(const T* __restrict__ dy,
                                                           const WT* __restrict__ wc,
                                                           T* __restrict__ dx, Geo g,
                                                           int istrips) {
  constexpr int VEC = Vec16<T>::N;
  const int tid = threadIdx.x;
  const int lc = tid % g.tc, ls = tid / g.tc;
  const int cvec = blockIdx.y * g.tc + lc;
  if (ls >= g.spp || cvec >= g.cv) return;
  const int64_t total = (int64_t)g.N * g.H * istrips;
  const int64_t sidx = (int64_t)blockIdx.x * g.spp + ls;
  if (sidx >= total) return;
  const int c0 = cvec * VEC;
  float wr[9][VEC];
  load_taps<WT, VEC>(wc, c0, wr);
  const int st = (int)(sidx % istrips);
  const int64_t nr = sidx / istrips;
  const int ih = (int)(nr % g.H);
  const int n = (int)(nr / g.H);
  const int iw0 = st * TW;
  float acc[TW][VEC];
#pragma unroll
  for (int o = 0; o < TW; ++o)
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[o][j] = 0.f;
  static_assert(TW % 2 == 0, "stride-2 column mapping assumes an even strip start");
  // stride 1: output columns iw0-1 .. iw0+TW feed the strip; stride 2: only
  // the even taps hit, output columns iw0/2 .. iw0/2+2
  constexpr int NCO = S == 1 ? TW + 2 : TW / 2 + 1;
  const int owb = S == 1 ? iw0 - 1 : iw0 / 2;
#pragma unroll
  for (int kh = 0; kh < 3; ++kh) {
    const int th = ih + 1 - kh;
    if (th < 0 || th % S) continue;
    const int oh = th / S;
    if (oh >= g.OH) continue;
    const T* row = dy + (((int64_t)n * g.OH + oh) * g.OW) * g.C + c0;
    typename Vec16<T>::raw raw[NCO];
#pragma unroll
    for (int ci = 0; ci < NCO; ++ci) raw[ci] = ldraw<T>(row + (int64_t)clampi(owb + ci, g.OW - 1) * g.C);
#pragma unroll
    for (int ci = 0; ci < NCO; ++ci) {
      const int ow = owb + ci;
      float v[VEC];
      cvt_masked<T>(raw[ci], ow >= 0 && ow < g.OW, v);
#pragma unroll
      for (int o = 0; o < TW; ++o) {
        // iw = ow*S - 1 + kw  ->  kw = iw0 + o + 1 - ow*S
        const int kw = S == 1 ? o + 1 - (ci - 1) : o + 1 - 2 * ci;
        if (kw < 0 || kw > 2) continue;
#pragma unroll
        for (int j = 0; j < VEC; ++j) acc[o][j] = fmaf(v[j], wr[kh * 3 + kw][j], acc[o][j]);
      }
    }
  }
#pragma unroll
  for (int o = 0; o < TW; ++o) {
    const int iw = iw0 + o;
    if (iw >= g.W) break;
    Vec16<T>::store(dx + (((int64_t)n * g.H + ih) * g.W + iw) * g.C + c0, acc[o]);
  }
}

// ---------------------------------------------------------------------------
// weight gradient partials: part[block][t*C + c] = sum over the block's output
// strips of dy * x (tap t).  Lanes of one channel vector combine in LDS.
// ---------------------------------------------------------------------------
template <typename T, int S>
__global__ __launch_bounds__(kThreads) void dw_wgrad_kernel(const T* __restrict__ dy,
                                                           const T* __restrict__ x, Geo g,
                                                           int strips_per_lane,
                                                           float* __restrict__ part) {
  constexpr int VEC = Vec16<T>::N;
  const int tid = threadIdx.x;
  const int lc = tid % g.tc, ls = tid / g.tc;
  const int cvec = blockIdx.y * g.tc + lc;
  const bool active = ls < g.spp && cvec < g.cv;
  const int c0 = cvec * VEC;
  float acc[9][VEC];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[t][j] = 0.f;
  const int64_t total = (int64_t)g.N * g.OH * g.strips;
  if (active) {
    for (int k = 0; k < strips_per_lane; ++k) {
      const int64_t sidx = ((int64_t)blockIdx.x * strips_per_lane + k) * g.spp + ls;
      if (sidx >= total) break;
      const int st = (int)(sidx % g.strips);
      const int64_t nr = sidx / g.strips;
      const int oh = (int)(nr % g.OH);
      const int n = (int)(nr / g.OH);
      const int ow0 = st * TW;
      float gv[TW][VEC];
      {
        const T* grow = dy + (((int64_t)n * g.OH + oh) * g.OW) * g.C + c0;
        typename Vec16<T>::raw graw[TW];
#pragma unroll
        for (int o = 0; o < TW; ++o) graw[o] = ldraw<T>(grow + (int64_t)min(ow0 + o, g.OW - 1) * g.C);
#pragma unroll
        for (int o = 0; o < TW; ++o) cvt_masked<T>(graw[o], ow0 + o < g.OW, gv[o]);
      }
      constexpr int NCI = (TW - 1) * S + 3;
      const int iw0 = ow0 * S - 1;
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        const int ih = oh * S - 1 + kh;
        if (ih < 0 || ih >= g.H) continue;
        const T* row = x + (((int64_t)n * g.H + ih) * g.W) * g.C + c0;
        typename Vec16<T>::raw raw[NCI];
#pragma unroll
        for (int ci = 0; ci < NCI; ++ci) raw[ci] = ldraw<T>(row + (int64_t)clampi(iw0 + ci, g.W - 1) * g.C);
#pragma unroll
        for (int ci = 0; ci < NCI; ++ci) {
          const int iw = iw0 + ci;
          float v[VEC];
          cvt_masked<T>(raw[ci], iw >= 0 && iw < g.W, v);
#pragma unroll
          for (int o = 0; o < TW; ++o) {
            const int kw = ci - o * S;
            if (kw < 0 || kw > 2) continue;
#pragma unroll
            for (int j = 0; j < VEC; ++j) acc[kh * 3 + kw][j] = fmaf(v[j], gv[o][j], acc[kh * 3 + kw][j]);
          }
        }
      }
    }
  }
  __shared__ float lds[kThreads * VEC];
  for (int t = 0; t < 9; ++t) {
#pragma unroll
    for (int j = 0; j < VEC; ++j) lds[j * kThreads + tid] = acc[t][j];
    __syncthreads();
    const int nout = g.tc * VEC;
    for (int o = tid; o < nout; o += kThreads) {
      const int c_l = o % g.tc, e = o / g.tc;
      const int cg = (blockIdx.y * g.tc + c_l) * VEC + e;
      if (cg < g.C) {
        float s = 0.f;
        for (int r = 0; r < g.spp; ++r) s += lds[e * kThreads + r * g.tc + c_l];
        part[(int64_t)blockIdx.x * 9 * g.C + t * g.C + cg] = s;
      }
    }
    __syncthreads();
  }
}

// out[c] = sum_b part[b][c]  (fp64 accumulation, 32 row-groups x 32 columns per block)
template <typename OT>
__global__ __launch_bounds__(1024) void column_reduce_kernel(const float* __restrict__ part, int rb,
                                                             int ncol, int C, OT* __restrict__ out, int acc) {
  const int cl = threadIdx.x % 32, g = threadIdx.x / 32;
  const int c = blockIdx.x * 32 + cl;
  double a = 0.0;
  if (c < ncol)
    for (int i = g; i < rb; i += 32) a += (double)part[(int64_t)i * ncol + c];
  __shared__ double l[1024];
  l[threadIdx.x] = a;
  __syncthreads();
  for (int s = 16; s > 0; s >>= 1) {
    if (g < s) l[threadIdx.x] += l[threadIdx.x + s * 32];
    __syncthreads();
  }
  if (g == 0 && c < ncol) {  // [C][9] = [C,1,3,3]; acc: add into the existing gradient
    OT* o = out + (c % C) * 9 + c / C;
    *o = (OT)(acc ? l[threadIdx.x] + (double)(float)*o : l[threadIdx.x]);
  }
}

Geo make_geo(const at::Tensor& x4, int stride, int VEC) {
  Geo g;
  g.N = (int)x4.size(0);
  g.C = (int)x4.size(1);
  g.H = (int)x4.size(2);
  g.W = (int)x4.size(3);
  g.stride = stride;
  g.OH = (g.H + 2 - 3) / stride + 1;
  g.OW = (g.W + 2 - 3) / stride + 1;
  g.cv = g.C / VEC;
  g.tc = g.cv < kThreads ? g.cv : kThreads;
  g.spp = kThreads / g.tc;
  g.strips = (g.OW + TW - 1) / TW;
  return g;
}

void check_nhwc(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.dim() == 4, name, " must be a 4-D GPU tensor");
  TORCH_CHECK(t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kFloat, name,
              " must be bf16 or fp32");
  TORCH_CHECK(t.is_contiguous(at::MemoryFormat::ChannelsLast), name, " must be channels-last");
  const int vec = t.scalar_type() == at::kBFloat16 ? 8 : 4;
  TORCH_CHECK(t.size(1) % vec == 0, name, ": channels must be a multiple of ", vec);
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-B aligned");
}

// The weight as the kernels read it: [C][9] contiguous, bf16 or fp32, 16-B
// aligned -- the module's own tensor when it already is (flat parameter views
// are padded to 8 elements), else one converted copy.
at::Tensor taps(const at::Tensor& w) {
  TORCH_CHECK(w.dim() == 4 && w.size(1) == 1 && w.size(2) == 3 && w.size(3) == 3,
              "depthwise weight must be [C,1,3,3]");
  TORCH_CHECK(w.is_cuda(), "depthwise weight must be a GPU tensor");
  if (w.is_contiguous() && (w.scalar_type() == at::kBFloat16 || w.scalar_type() == at::kFloat) &&
      reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0)
    return w;
  return w.to(at::kFloat).contiguous();
}

template <typename F>
void dispatch_w(const at::Tensor& w, F&& f) {
  if (w.scalar_type() == at::kBFloat16) f(__bf16{});
  else f(float{});
}

template <typename F>
void dispatch_t(const at::Tensor& x, F&& f) {
  if (x.scalar_type() == at::kBFloat16) f(__bf16{});
  else f(float{});
}

}  // namespace

// Forward.  Returns (y, moments-or-undefined); moments = fp64 [2C+1] of y.
std::vector<at::Tensor> dwconv3x3_forward(const at::Tensor& x, const at::Tensor& w, int64_t stride,
                                          bool moments) {
  check_nhwc(x, "x");
  TORCH_CHECK(stride == 1 || stride == 2, "stride must be 1 or 2");
  const int VEC = x.scalar_type() == at::kBFloat16 ? 8 : 4;
  Geo g = make_geo(x, (int)stride, VEC);
  auto y = at::empty({g.N, g.C, g.OH, g.OW}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  const auto wt = taps(w);
  TORCH_CHECK(wt.size(0) == g.C, "weight channels do not match x");
  auto stream = at::hip::getCurrentHIPStream();
  const int64_t total = (int64_t)g.N * g.OH * g.strips;
  const int cchunks = (g.cv + g.tc - 1) / g.tc;
  dim3 grid((unsigned)((total + g.spp - 1) / g.spp), (unsigned)cchunks);
  at::Tensor mom, part;
  double* zt = nullptr;
  if (moments) {
    part = at::empty({2, (int64_t)grid.x, g.C}, x.options().dtype(at::kFloat));
    mom = at::empty({2 * (int64_t)g.C + 1}, x.options().dtype(at::kDouble));
    zt = moments_zero_target(mom.data_ptr<double>(), (int)grid.x);
  }
  dispatch_t(x, [&](auto tag) {
    using T = decltype(tag);
    dispatch_w(wt, [&](auto wtag) {
      using WT = decltype(wtag);
      const WT* wp = reinterpret_cast<const WT*>(wt.data_ptr());
      if (moments)
        hipLaunchKernelGGL((g.stride == 1 ? dw_fwd_kernel<T, WT, true, 1> : dw_fwd_kernel<T, WT, true, 2>), grid,
                           dim3(kThreads), 0, stream, reinterpret_cast<const T*>(x.data_ptr()), wp,
                           reinterpret_cast<T*>(y.data_ptr()), g, part.data_ptr<float>(), zt);
      else
        hipLaunchKernelGGL((g.stride == 1 ? dw_fwd_kernel<T, WT, false, 1> : dw_fwd_kernel<T, WT, false, 2>), grid,
                           dim3(kThreads), 0, stream, reinterpret_cast<const T*>(x.data_ptr()), wp,
                           reinterpret_cast<T*>(y.data_ptr()), g, nullptr, nullptr);
    });
  });
  if (moments) {
    bn_reduce_partials_launch(part.data_ptr<float>(), (int)grid.x, g.C, mom.data_ptr<double>(),
                              (double)g.N * g.OH * g.OW, stream);
  }
  return {y, mom};
}

// Data gradient: dx [N,C,H,W] channels-last.
at::Tensor dwconv3x3_dgrad(const at::Tensor& dy, const at::Tensor& w, int64_t stride, int64_t H,
                           int64_t W) {
  check_nhwc(dy, "dy");
  const int VEC = dy.scalar_type() == at::kBFloat16 ? 8 : 4;
  auto shape_x = at::empty({dy.size(0), dy.size(1), H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  Geo g = make_geo(shape_x, (int)stride, VEC);
  TORCH_CHECK(g.OH == dy.size(2) && g.OW == dy.size(3), "dy shape does not match the input size");
  const auto wt = taps(w);
  TORCH_CHECK(wt.size(0) == g.C, "weight channels do not match dy");
  auto stream = at::hip::getCurrentHIPStream();
  const int istrips = (g.W + TW - 1) / TW;
  const int64_t total = (int64_t)g.N * g.H * istrips;
  const int cchunks = (g.cv + g.tc - 1) / g.tc;
  dim3 grid((unsigned)((total + g.spp - 1) / g.spp), (unsigned)cchunks);
  dispatch_t(dy, [&](auto tag) {
    using T = decltype(tag);
    dispatch_w(wt, [&](auto wtag) {
      using WT = decltype(wtag);
      hipLaunchKernelGGL((g.stride == 1 ? dw_dgrad_kernel<T, WT, 1> : dw_dgrad_kernel<T, WT, 2>), grid,
                         dim3(kThreads), 0, stream, reinterpret_cast<const T*>(dy.data_ptr()),
                         reinterpret_cast<const WT*>(wt.data_ptr()), reinterpret_cast<T*>(shape_x.data_ptr()), g,
                         istrips);
    });
  });
  return shape_x;
}

// Weight gradient: returns [C,1,3,3] in `out_dtype`.
at::Tensor acc_target(const c10::optional<at::Tensor>& out, int64_t numel, at::ScalarType dtype,
                      const char* who);

at::Tensor dwconv3x3_wgrad(const at::Tensor& dy, const at::Tensor& x, int64_t stride,
                           at::ScalarType out_dtype, const c10::optional<at::Tensor>& acc_out) {
  check_nhwc(dy, "dy");
  check_nhwc(x, "x");
  const int VEC = x.scalar_type() == at::kBFloat16 ? 8 : 4;
  Geo g = make_geo(x, (int)stride, VEC);
  TORCH_CHECK(g.OH == dy.size(2) && g.OW == dy.size(3), "dy shape does not match x");
  auto stream = at::hip::getCurrentHIPStream();
  const int64_t total = (int64_t)g.N * g.OH * g.strips;
  const int cchunks = (g.cv + g.tc - 1) / g.tc;
  // ~1024 blocks total, each lane walking several strips
  const int64_t lanes_needed = (total + g.spp - 1) / g.spp;
  const int target = std::max(1, 1024 / cchunks);
  const int spl = (int)std::max<int64_t>(1, (lanes_needed + target - 1) / target);
  dim3 grid((unsigned)((lanes_needed + spl - 1) / spl), (unsigned)cchunks);
  auto part = at::empty({(int64_t)grid.x, 9 * (int64_t)g.C}, x.options().dtype(at::kFloat));
  dispatch_t(x, [&](auto tag) {
    using T = decltype(tag);
    hipLaunchKernelGGL((g.stride == 1 ? dw_wgrad_kernel<T, 1> : dw_wgrad_kernel<T, 2>), grid, dim3(kThreads), 0, stream,
                       reinterpret_cast<const T*>(dy.data_ptr()),
                       reinterpret_cast<const T*>(x.data_ptr()), g, spl, part.data_ptr<float>());
  });
  // reduced straight into [C,1,3,3] in the parameter dtype (no transpose / cast launches)
  TORCH_CHECK(out_dtype == at::kBFloat16 || out_dtype == at::kFloat, "weight gradient must be bf16 or fp32");
  at::Tensor acc = acc_target(acc_out, 9 * (int64_t)g.C, out_dtype, "dwconv3x3_wgrad");
  TORCH_CHECK(!acc.defined() || acc.is_contiguous(), "dwconv3x3_wgrad: the accumulation target must be [C,1,3,3] contiguous");
  auto out = acc.defined() ? acc : at::empty({(int64_t)g.C, 1, 3, 3}, x.options().dtype(out_dtype));
  const int ncol = 9 * g.C;
  if (out_dtype == at::kBFloat16)
    hipLaunchKernelGGL((column_reduce_kernel<__bf16>), dim3((ncol + 31) / 32), dim3(1024), 0, stream,
                       part.data_ptr<float>(), (int)grid.x, ncol, g.C, reinterpret_cast<__bf16*>(out.data_ptr()),
                       (int)acc.defined());
  else
    hipLaunchKernelGGL((column_reduce_kernel<float>), dim3((ncol + 31) / 32), dim3(1024), 0, stream,
                       part.data_ptr<float>(), (int)grid.x, ncol, g.C, out.data_ptr<float>(), (int)acc.defined());
  return out;
}

}  // namespace dmp
