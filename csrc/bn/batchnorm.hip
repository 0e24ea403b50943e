// Channels-last (NHWC / [M, C]) batch normalisation for gfx950, with the
// activation and the residual add fused in, plus the split-phase entry points
// SyncBatchNorm needs (local moments -> RCCL all-reduce -> apply).
//
// Capability parity: upstream BatchNorm2d / SyncBatchNorm as studied in the
// reference README (Readme.md:151 "prepare for sync batch norm layers",
// SURVEY.md D11).  Design is MI355X-first and launch-lean (ResNet-50 runs 53
// BN layers per step; BN is ~60 GB of HBM traffic per step at batch 256, so
// every kernel here is a pure streaming pass):
//   * x is viewed as a row-major [M, C] matrix (M = N*H*W).  Each lane owns ONE
//     16-byte channel vector (8 bf16 or 4 f32) for the whole launch, so its
//     per-channel coefficients live in registers and every global access is a
//     16-B coalesced load; a block walks a contiguous slab of rows with two
//     rows in flight per lane.
//   * moments: fp32 per-lane partial sums -> LDS combine -> one fp32 partial
//     row per block ([2][blocks][C]) -> a 2-D fp64 reduce kernel into a [2C+1]
//     fp64 buffer (sum, sum of squares, row count).  Same-address fp64 atomics
//     from ~1000 blocks serialise (~100 ns each, measured), hence the partials.
//     fp64 accumulation across blocks avoids E[x^2]-E[x]^2 cancellation at
//     M = 3.2M rows; the buffer is what SyncBN all-reduces.
//   * the apply kernel derives scale/shift from the moments itself (no
//     finalize launch); the blocks of row-slab 0 also write the saved
//     mean/invstd and update the running statistics.
//   * backward: pass 1 accumulates sum(dz) and sum(dz*(x-mean)) the same way
//     (dz = dy * [y > 0] -- ReLU re-derived from the saved OUTPUT, nothing
//     extra stored); pass 2 computes dx = a*dz + b*x + c with per-lane
//     coefficients, writes d(residual) = dz when the residual was fused, and
//     row-slab-0 blocks write dweight/dbias.
// Forward = moments + reduce + apply, backward = moments + reduce + apply (the
// moments pass disappears when the producing GEMM/depthwise kernel emits them).
#include <cstdlib>

#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include "../common.h"

namespace dmp {
namespace {

// ones / zeros an absent BN weight / bias is read from (branch-free loads)
__device__ float g_bn_ones[16] = {1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f};
__device__ float g_bn_zeros[16] = {};

constexpr int kThreads = 256;

struct Layout {
  int cv;    // channel vectors per row (C / VEC)
  int tc;    // channel vectors handled by one block (<= 256)
  int rpi;   // rows per block iteration = 256 / tc
};

__host__ __device__ inline Layout make_layout(int C, int vec) {
  Layout l;
  l.cv = C / vec;
  l.tc = l.cv < kThreads ? l.cv : kThreads;
  l.rpi = kThreads / l.tc;
  return l;
}

// Combine the rpi row-lanes of each channel through LDS and write the block's
// totals to its partial row: part[blockIdx.x][c] (sum) and part[rb + blockIdx.x][c].
// (Same-address fp64 atomics from ~1000 blocks serialise at ~100 ns each at
// the memory side -- measured 115 us per call -- so the cross-block sum is a
// separate wide, deterministic reduce kernel instead.)
template <int VEC>
__device__ __forceinline__ void block_combine_store(const float (&s)[VEC], const float (&q)[VEC],
                                                    const Layout& L, int C, float* part) {
  __shared__ float lds_s[kThreads * VEC];
  __shared__ float lds_q[kThreads * VEC];
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    lds_s[i * kThreads + tid] = s[i];
    lds_q[i * kThreads + tid] = q[i];
  }
  __syncthreads();
  const int nout = L.tc * VEC;
  for (int o = tid; o < nout; o += kThreads) {
    const int c_l = o % L.tc, e = o / L.tc;
    const int cg = (blockIdx.y * L.tc + c_l) * VEC + e;
    if (cg >= C) continue;
    float ss = 0.f, qq = 0.f;
    for (int rr = 0; rr < L.rpi; ++rr) {
      ss += lds_s[e * kThreads + rr * L.tc + c_l];
      qq += lds_q[e * kThreads + rr * L.tc + c_l];
    }
    part[(int64_t)blockIdx.x * C + cg] = ss;
    part[(int64_t)(gridDim.x + blockIdx.x) * C + cg] = qq;
  }
}

// fp64 reduction of the [2][rb][C] partials into sums[0:2C].  Grid is
// (ceil(C/32), ceil(rb/kRedRows)): each 1024-thread block (32 row-groups x 32
// channels) folds kRedRows partial rows.  With one row-chunk the block stores
// the result (deterministic); otherwise the caller zeroes sums and each chunk
// adds with an fp64 atomic (<= rb/kRedRows adds per address, so no same-address
// serialisation worth speaking of; the producer zeroed sums, see common.h).
// Writes sums[2C] = count when count >= 0.
constexpr int kRedCh = 32, kRedGroups = 32, kRedRows = kBnRedRows;
__global__ __launch_bounds__(1024) void bn_reduce_partials_kernel(const float* __restrict__ part,
                                                                  int rb, int C,
                                                                  double* __restrict__ sums,
                                                                  double count) {
  const int cl = threadIdx.x % kRedCh, g = threadIdx.x / kRedCh;
  const int c = blockIdx.x * kRedCh + cl;
  const int r0 = blockIdx.y * kRedRows, r1 = min(rb, r0 + kRedRows);
  double a = 0.0, b = 0.0;
  if (c < C) {
    const float* pa = part + c;
    const float* pb = part + (int64_t)rb * C + c;
    int i = r0 + g;
    // four rows (8 loads) in flight per iteration: at a micro-batch's ~100-400
    // partial rows that is one or two round trips per thread (round 6: a
    // 2-row loop made this ~5 us launch latency-bound)
    for (; i + 3 * kRedGroups < r1; i += 4 * kRedGroups) {
      float va[4], vb[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        va[u] = pa[(int64_t)(i + u * kRedGroups) * C];
        vb[u] = pb[(int64_t)(i + u * kRedGroups) * C];
      }
      a += ((double)va[0] + (double)va[1]) + ((double)va[2] + (double)va[3]);
      b += ((double)vb[0] + (double)vb[1]) + ((double)vb[2] + (double)vb[3]);
    }
    for (; i < r1; i += kRedGroups) {
      a += (double)pa[(int64_t)i * C];
      b += (double)pb[(int64_t)i * C];
    }
  }
  __shared__ double la[1024], lb[1024];
  la[threadIdx.x] = a;
  lb[threadIdx.x] = b;
  __syncthreads();
  for (int s = kRedGroups / 2; s > 0; s >>= 1) {
    if (g < s) {
      la[threadIdx.x] += la[threadIdx.x + s * kRedCh];
      lb[threadIdx.x] += lb[threadIdx.x + s * kRedCh];
    }
    __syncthreads();
  }
  if (g == 0 && c < C) {
    if (gridDim.y == 1) {
      sums[c] = la[threadIdx.x];
      sums[C + c] = lb[threadIdx.x];
    } else {
      atomicAdd(sums + c, la[threadIdx.x]);
      atomicAdd(sums + C + c, lb[threadIdx.x]);
    }
  }
  if (count >= 0.0 && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) sums[2 * C] = count;
}

// -------------------------------------------------------------------------
// Forward moments, phase 1: per-block partial sum / sum of squares.
// grid = (row_blocks, channel_chunks); 4 rows in flight per lane.
// -------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(kThreads) void bn_moments_kernel(
    const T* __restrict__ x, int64_t M, int C, int64_t rows_per_block, float* __restrict__ part,
    double* __restrict__ zsums) {
  zero_moments(zsums, 2 * C);
  constexpr int VEC = Vec16<T>::N;
  const Layout L = make_layout(C, VEC);
  const int tid = threadIdx.x;
  const int lc = tid % L.tc, lr = tid / L.tc;
  const int cvec = blockIdx.y * L.tc + lc;
  const bool active = lr < L.rpi && cvec < L.cv;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(M, r0 + rows_per_block);

  float s[VEC], q[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) { s[i] = 0.f; q[i] = 0.f; }
  if (active) {
    const T* p = x + (int64_t)cvec * VEC;
    const int64_t st = (int64_t)L.rpi * C;
    int64_t r = r0 + lr;
    for (; r + 3 * L.rpi < r1; r += 4 * L.rpi) {
      float a[VEC], b[VEC], c[VEC], d[VEC];
      const T* pr = p + r * C;
      Vec16<T>::load(pr, a);
      Vec16<T>::load(pr + st, b);
      Vec16<T>::load(pr + 2 * st, c);
      Vec16<T>::load(pr + 3 * st, d);
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        s[i] += (a[i] + b[i]) + (c[i] + d[i]);
        q[i] = fmaf(a[i], a[i], fmaf(b[i], b[i], fmaf(c[i], c[i], fmaf(d[i], d[i], q[i]))));
      }
    }
    for (; r < r1; r += L.rpi) {
      float a[VEC];
      Vec16<T>::load(p + r * C, a);
#pragma unroll
      for (int i = 0; i < VEC; ++i) { s[i] += a[i]; q[i] = fmaf(a[i], a[i], q[i]); }
    }
  }
  block_combine_store<VEC>(s, q, L, C, part);
}

// Per-channel forward coefficients from (possibly all-reduced) moments.
__device__ __forceinline__ void fwd_coeffs(const double* __restrict__ sums, int C, int c,
                                           const float* __restrict__ w, const float* __restrict__ b,
                                           float eps, float& mean, float& invstd, float& var_b,
                                           float& scale, float& shift) {
  const double n = sums[2 * C];
  const double m = sums[c] / n;
  double v = sums[C + c] / n - m * m;
  v = v < 0.0 ? 0.0 : v;
  mean = (float)m;
  var_b = (float)v;
  invstd = (float)(1.0 / sqrt(v + (double)eps));
  const float ww = w ? w[c] : 1.f, bb = b ? b[c] : 0.f;
  scale = ww * invstd;
  shift = bb - mean * scale;
}

// Coefficients only (no pass over x): when the BN apply + ReLU is fused into
// the consuming GEMM's operand staging (ops/fused.py bn_relu_conv1x1), the BN
// output is never materialised.  coef = [scale, shift, mean, invstd] x C;
// running stats and the step counter are updated here.
__global__ __launch_bounds__(256) void bn_finalize_kernel(
    const double* __restrict__ sums, const float* __restrict__ weight,
    const float* __restrict__ bias, float* __restrict__ running_mean,
    float* __restrict__ running_var, float momentum, float eps, int C, float* __restrict__ coef,
    int64_t* __restrict__ num_batches_tracked) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (num_batches_tracked != nullptr && c == 0) *num_batches_tracked += 1;
  if (c >= C) return;
  float mean, invstd, var_b, sc, sh;
  fwd_coeffs(sums, C, c, weight, bias, eps, mean, invstd, var_b, sc, sh);
  coef[c] = sc;
  coef[C + c] = sh;
  coef[2 * C + c] = mean;
  coef[3 * C + c] = invstd;
  if (running_mean) {
    const double n = sums[2 * C];
    const float unb = n > 1.0 ? (float)((double)var_b * n / (n - 1.0)) : var_b;
    running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mean;
    running_var[c] = (1.f - momentum) * running_var[c] + momentum * unb;
  }
}

// -------------------------------------------------------------------------
// Forward apply: y = act(x*scale + shift [+ residual]); act = ReLU clipped at
// `clip` (+inf: ReLU; 6: ReLU6, the 224-px MobileNetV2's activation).
// FROM_SUMS: training mode -- coefficients from the moments; row-slab-0 blocks
// also save mean/invstd and update running stats.  Otherwise eval mode --
// coefficients from running stats.
// -------------------------------------------------------------------------
template <typename T, bool RELU, bool RES, bool FROM_SUMS, bool NT, bool OSUM>
__device__ __forceinline__ void bn_apply_rows(
    const T* __restrict__ x, const T* __restrict__ res, const double* __restrict__ sums,
    const float* __restrict__ weight, const float* __restrict__ bias,
    float* __restrict__ running_mean, float* __restrict__ running_var, float momentum, float eps,
    int64_t M, int C, int64_t rows_per_block, T* __restrict__ y, float* __restrict__ save_mean,
    float* __restrict__ save_invstd, const Layout& L, int lr, int cvec,
    float (&os)[Vec16<T>::N], float (&oq)[Vec16<T>::N], float clip);

// OSUM: also reduce per-block partials of the column sums (and sums of
// squares) of the STORED output -- the colsum a BN-folded consumer needs
// (ops/bn_fold.py: the next BN's mean is W @ colsum(y) / M) without a pass.
template <typename T, bool RELU, bool RES, bool FROM_SUMS, bool NT = false, bool OSUM = false>
__global__ __launch_bounds__(kThreads) void bn_apply_kernel(
    const T* __restrict__ x, const T* __restrict__ res, const double* __restrict__ sums,
    const float* __restrict__ weight, const float* __restrict__ bias,
    float* __restrict__ running_mean, float* __restrict__ running_var, float momentum, float eps,
    int64_t M, int C, int64_t rows_per_block, T* __restrict__ y, float* __restrict__ save_mean,
    float* __restrict__ save_invstd, int64_t* __restrict__ num_batches_tracked,
    float* __restrict__ opart = nullptr, double* __restrict__ ozsums = nullptr,
    float clip = __builtin_inff()) {
  // BatchNorm's step counter rides along (one lane), instead of its own launch
  if (num_batches_tracked != nullptr && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)
    *num_batches_tracked += 1;
  constexpr int VEC = Vec16<T>::N;
  const Layout L = make_layout(C, VEC);
  const int tid = threadIdx.x;
  const int lc = tid % L.tc, lr = tid / L.tc;
  const int cvec = blockIdx.y * L.tc + lc;
  if constexpr (OSUM) {
    zero_moments(ozsums, 2 * C);
    float os[VEC], oq[VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) { os[i] = 0.f; oq[i] = 0.f; }
    if (lr < L.rpi && cvec < L.cv)
      bn_apply_rows<T, RELU, RES, FROM_SUMS, NT, true>(x, res, sums, weight, bias, running_mean, running_var,
                                                       momentum, eps, M, C, rows_per_block, y, save_mean,
                                                       save_invstd, L, lr, cvec, os, oq, clip);
    block_combine_store<VEC>(os, oq, L, C, opart);
    return;
  }
  if (lr >= L.rpi || cvec >= L.cv) return;
  float os[VEC], oq[VEC];
  bn_apply_rows<T, RELU, RES, FROM_SUMS, NT, false>(x, res, sums, weight, bias, running_mean, running_var,
                                                    momentum, eps, M, C, rows_per_block, y, save_mean,
                                                    save_invstd, L, lr, cvec, os, oq, clip);
}

template <typename T, bool RELU, bool RES, bool FROM_SUMS, bool NT, bool OSUM>
__device__ __forceinline__ void bn_apply_rows(
    const T* __restrict__ x, const T* __restrict__ res, const double* __restrict__ sums,
    const float* __restrict__ weight, const float* __restrict__ bias,
    float* __restrict__ running_mean, float* __restrict__ running_var, float momentum, float eps,
    int64_t M, int C, int64_t rows_per_block, T* __restrict__ y, float* __restrict__ save_mean,
    float* __restrict__ save_invstd, const Layout& L, int lr, int cvec,
    float (&os)[Vec16<T>::N], float (&oq)[Vec16<T>::N], float clip) {
  constexpr int VEC = Vec16<T>::N;
  float sc[VEC], sh[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    const int c = cvec * VEC + i;
    float mean, invstd, var_b;
    if (FROM_SUMS) {
      fwd_coeffs(sums, C, c, weight, bias, eps, mean, invstd, var_b, sc[i], sh[i]);
    } else {
      mean = running_mean[c];
      invstd = rsqrtf(running_var[c] + eps);
      const float ww = weight ? weight[c] : 1.f, bb = bias ? bias[c] : 0.f;
      sc[i] = ww * invstd;
      sh[i] = bb - mean * sc[i];
    }
    if (blockIdx.x == 0 && lr == 0) {
      save_mean[c] = mean;
      save_invstd[c] = invstd;
      if (FROM_SUMS && running_mean) {
        const double n = sums[2 * C];
        const float unb = n > 1.0 ? (float)((double)var_b * n / (n - 1.0)) : var_b;
        running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mean;
        running_var[c] = (1.f - momentum) * running_var[c] + momentum * unb;
      }
    }
  }
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(M, r0 + rows_per_block);
  const int64_t off0 = (int64_t)cvec * VEC;
  int64_t r = r0 + lr;
  for (; r + L.rpi < r1; r += 2 * L.rpi) {
    const int64_t o = r * C + off0, o2 = o + (int64_t)L.rpi * C;
    float v[VEC], v2[VEC], rv[VEC], rv2[VEC];
    ld16<NT>(x + o, v);
    ld16<NT>(x + o2, v2);
    if (RES) {
      ld16<NT>(res + o, rv);
      ld16<NT>(res + o2, rv2);
    }
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      float t = fmaf(v[i], sc[i], sh[i]), t2 = fmaf(v2[i], sc[i], sh[i]);
      if (RES) { t += rv[i]; t2 += rv2[i]; }
      if (RELU) { t = fminf(fmaxf(t, 0.f), clip); t2 = fminf(fmaxf(t2, 0.f), clip); }
      if constexpr (OSUM) {  // moments of the values as stored
        t = (float)(T)t;
        t2 = (float)(T)t2;
        os[i] += t + t2;
        oq[i] = fmaf(t, t, fmaf(t2, t2, oq[i]));
      }
      v[i] = t;
      v2[i] = t2;
    }
    st16<NT>(y + o, v);
    st16<NT>(y + o2, v2);
  }
  if (r < r1) {
    const int64_t o = r * C + off0;
    float v[VEC], rv[VEC];
    ld16<NT>(x + o, v);
    if (RES) ld16<NT>(res + o, rv);
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      float t = fmaf(v[i], sc[i], sh[i]);
      if (RES) t += rv[i];
      if (RELU) t = fminf(fmaxf(t, 0.f), clip);
      if constexpr (OSUM) {
        t = (float)(T)t;
        os[i] += t;
        oq[i] = fmaf(t, t, oq[i]);
      }
      v[i] = t;
    }
    st16<NT>(y + o, v);
  }
}

// -------------------------------------------------------------------------
// Backward pass 1 (per-block partials of sum dz and sum dz*(x-mean)).
// -------------------------------------------------------------------------
// RELU: 0 none; 1 mask from the saved output (y > 0); 2 mask re-derived from
// x and the forward's per-channel affine (x*w*invstd + b - mean*w*invstd > 0)
// -- one full-tensor read fewer, used whenever no residual was fused.
template <typename T, int RELU>
__global__ __launch_bounds__(kThreads) void bn_bwd_moments_kernel(
    const T* __restrict__ dy, const T* __restrict__ x, const T* __restrict__ y,
    const float* __restrict__ mean, const float* __restrict__ weight,
    const float* __restrict__ bias, const float* __restrict__ invstd, int64_t M, int C,
    int64_t rows_per_block, float* __restrict__ part, double* __restrict__ zsums, float clip) {
  zero_moments(zsums, 2 * C);
  constexpr int VEC = Vec16<T>::N;
  const Layout L = make_layout(C, VEC);
  const int tid = threadIdx.x;
  const int lc = tid % L.tc, lr = tid / L.tc;
  const int cvec = blockIdx.y * L.tc + lc;
  const bool active = lr < L.rpi && cvec < L.cv;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(M, r0 + rows_per_block);
  float s[VEC], q[VEC], mu[VEC], msc[VEC], msh[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) { s[i] = 0.f; q[i] = 0.f; mu[i] = 0.f; msc[i] = 0.f; msh[i] = 0.f; }
  if (active) {
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      const int ch = cvec * VEC + i;
      mu[i] = mean[ch];
      if (RELU == 2) {
        msc[i] = (weight ? weight[ch] : 1.f) * invstd[ch];
        msh[i] = (bias ? bias[ch] : 0.f) - mu[i] * msc[i];
      }
    }
    const int64_t off0 = (int64_t)cvec * VEC;
    for (int64_t r = r0 + lr; r < r1; r += L.rpi) {
      const int64_t o = r * C + off0;
      float g[VEC], xv[VEC];
      Vec16<T>::load(dy + o, g);
      Vec16<T>::load(x + o, xv);
      if (RELU == 1) {
        float yv[VEC];
        Vec16<T>::load(y + o, yv);
#pragma unroll
        for (int i = 0; i < VEC; ++i) g[i] = (yv[i] > 0.f && yv[i] < clip) ? g[i] : 0.f;
      } else if (RELU == 2) {
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
          const float t = fmaf(xv[i], msc[i], msh[i]);
          g[i] = (t > 0.f && t < clip) ? g[i] : 0.f;
        }
      }
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        s[i] += g[i];
        q[i] = fmaf(g[i], xv[i] - mu[i], q[i]);
      }
    }
  }
  block_combine_store<VEC>(s, q, L, C, part);
}

// -------------------------------------------------------------------------
// Backward pass 2: dx = a*dz + b*x + c ; dres = dz (residual fused); the
// row-slab-0 blocks write dweight = sum(dz*(x-mean))*invstd, dbias = sum(dz).
// -------------------------------------------------------------------------
template <typename T, int RELU, bool DRES, bool NT = false>
__global__ __launch_bounds__(kThreads) void bn_bwd_apply_kernel(
    const T* __restrict__ dy, const T* __restrict__ x, const T* __restrict__ y,
    const double* __restrict__ sums, const double* __restrict__ count_ptr,
    const float* __restrict__ weight, const float* __restrict__ bias, const float* __restrict__ mean,
    const float* __restrict__ invstd, int training, int64_t M, int C, int64_t rows_per_block,
    T* __restrict__ dx, T* __restrict__ dres, float* __restrict__ dweight,
    float* __restrict__ dbias, float clip, int acc) {
  constexpr int VEC = Vec16<T>::N;
  const Layout L = make_layout(C, VEC);
  const int tid = threadIdx.x;
  const int lc = tid % L.tc, lr = tid / L.tc;
  const int cvec = blockIdx.y * L.tc + lc;
  if (lr >= L.rpi || cvec >= L.cv) return;
  const double n = *count_ptr;
  float a[VEC], b[VEC], c[VEC], msc[VEC], msh[VEC];
  // per-channel constants: every load issued up front and branch-free (an
  // absent weight / bias reads ones / zeros) -- a `weight ? weight[ch] : 1`
  // per element made the compiler wait for each load before the next, eight
  // dependent round trips before a block's first row
  const int ch0 = cvec * VEC;
  const float* wp = weight ? weight + ch0 : g_bn_ones;
  const float* bp = bias ? bias + ch0 : g_bn_zeros;
  float wv[VEC], bv[VEC], isv[VEC], muv[VEC];
  double s1[VEC], s2[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    wv[i] = wp[i];
    bv[i] = bp[i];
    isv[i] = invstd[ch0 + i];
    muv[i] = mean[ch0 + i];
    s1[i] = sums[ch0 + i];
    s2[i] = sums[C + ch0 + i];
  }
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    const int ch = ch0 + i;
    const double sdz = s1[i], sdzx = s2[i];
    const double is = isv[i];
    const double aa = (double)wv[i] * is;
    if (RELU == 2) {  // the forward's affine, as in bn_bwd_moments_kernel
      msc[i] = wv[i] * isv[i];
      msh[i] = bv[i] - muv[i] * msc[i];
    } else {
      msc[i] = msh[i] = 0.f;
    }
    if (training) {
      const double bb = -aa * is * is * sdzx / n;
      a[i] = (float)aa;
      b[i] = (float)bb;
      c[i] = (float)(-aa * sdz / n - bb * (double)muv[i]);
    } else {
      a[i] = (float)aa;
      b[i] = 0.f;
      c[i] = 0.f;
    }
    if (blockIdx.x == 0 && lr == 0) {
      if (dweight) dweight[ch] = (float)(sdzx * is) + (acc ? dweight[ch] : 0.f);
      if (dbias) dbias[ch] = (float)sdz + (acc ? dbias[ch] : 0.f);
    }
  }
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(M, r0 + rows_per_block);
  const int64_t off0 = (int64_t)cvec * VEC;
  for (int64_t r = r0 + lr; r < r1; r += L.rpi) {
    const int64_t o = r * C + off0;
    float g[VEC], xv[VEC];
    ld16<NT>(dy + o, g);
    ld16<NT>(x + o, xv);
    if (RELU == 1) {
      float yv[VEC];
      ld16<NT>(y + o, yv);
#pragma unroll
      for (int i = 0; i < VEC; ++i) g[i] = (yv[i] > 0.f && yv[i] < clip) ? g[i] : 0.f;
    } else if (RELU == 2) {
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        const float t = fmaf(xv[i], msc[i], msh[i]);
        g[i] = (t > 0.f && t < clip) ? g[i] : 0.f;
      }
    }
    if (DRES) st16<NT>(dres + o, g);
#pragma unroll
    for (int i = 0; i < VEC; ++i) xv[i] = fmaf(a[i], g[i], fmaf(b[i], xv[i], c[i]));
    st16<NT>(dx + o, xv);
  }
}

// ---------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------
struct Grid {
  dim3 grid;
  int64_t rows_per_block;
};

// ~`target` blocks: grid.y chunks channels, grid.x slabs rows (>= 8 rows per lane).
Grid plan(int64_t M, int C, int vec, int target = 1024, int64_t min_rows_per_lane = 8) {
  Layout L = make_layout(C, vec);
  int cchunks = (L.cv + L.tc - 1) / L.tc;
  int64_t max_rb = std::max<int64_t>(1, (M + (int64_t)L.rpi * min_rows_per_lane - 1) /
                                            ((int64_t)L.rpi * min_rows_per_lane));
  int64_t rb = std::max<int64_t>(1, std::min<int64_t>(max_rb, std::max(1, target / cchunks)));
  int64_t rows = (M + rb - 1) / rb;
  rb = (M + rows - 1) / rows;
  Grid g;
  g.grid = dim3((unsigned)rb, (unsigned)cchunks);
  g.rows_per_block = rows;
  return g;
}

void check_input(const at::Tensor& x, int64_t C, const char* name) {
  TORCH_CHECK(x.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16,
              name, " must be float32 or bfloat16");
  TORCH_CHECK(x.is_contiguous(), name, " must be a contiguous [M, C] view");
  const int vec = x.scalar_type() == at::kBFloat16 ? 8 : 4;
  TORCH_CHECK(C % vec == 0, "channels must be a multiple of ", vec);
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0, name, " must be 16-B aligned");
}

int vec_of(const at::Tensor& x) { return x.scalar_type() == at::kBFloat16 ? 8 : 4; }

template <typename F>
void dispatch_t(const at::Tensor& x, F&& f) {
  if (x.scalar_type() == at::kBFloat16) f(__bf16{});
  else f(float{});
}

template <typename T> T* ptr(const at::Tensor& t) { return reinterpret_cast<T*>(t.data_ptr()); }

// Non-temporal streaming for the apply passes over tensors much larger than
// the Infinity Cache (set_bn_streaming(false) disables it, for A/B runs).
bool g_bn_streaming = true;
bool streaming(int64_t M, int64_t C) { return g_bn_streaming && M * C * 2 >= (int64_t)256 << 20; }
float* fptr(const c10::optional<at::Tensor>& t) {
  return (t.has_value() && t->defined()) ? t->data_ptr<float>() : nullptr;
}

}  // namespace

// Shared with the GEMM moments epilogue (csrc/conv/gemm_bf16.hip).
void bn_reduce_partials_launch(const float* part, int rb, int C, double* sums, double count,
                               hipStream_t stream) {
  const int chunks = (rb + kRedRows - 1) / kRedRows;  // > 1: producer zeroed sums
  hipLaunchKernelGGL(bn_reduce_partials_kernel, dim3((C + kRedCh - 1) / kRedCh, chunks), dim3(1024),
                     0, stream, part, rb, C, sums, count);
}

// Local moments: fp64 [2C+1] = (sum x, sum x^2, rows) over the local rows.
at::Tensor bn_local_moments(const at::Tensor& x, int64_t C) {
  check_input(x, C, "x");
  const int64_t M = x.numel() / C;
  auto stream = at::hip::getCurrentHIPStream();
  if (M == 0) return at::zeros({2 * C + 1}, x.options().dtype(at::kDouble));
  auto sums = at::empty({2 * C + 1}, x.options().dtype(at::kDouble));
  Grid g = plan(M, (int)C, vec_of(x));
  auto part = at::empty({2, (int64_t)g.grid.x, C}, x.options().dtype(at::kFloat));
  dispatch_t(x, [&](auto tag) {
    using T = decltype(tag);
    hipLaunchKernelGGL(bn_moments_kernel<T>, g.grid, dim3(kThreads), 0, stream, ptr<T>(x), M,
                       (int)C, g.rows_per_block, part.data_ptr<float>(),
                       moments_zero_target(sums.data_ptr<double>(), (int)g.grid.x));
  });
  bn_reduce_partials_launch(part.data_ptr<float>(), (int)g.grid.x, (int)C, sums.data_ptr<double>(),
                            (double)M, stream);
  return sums;
}

// Training-mode apply from moments.  Returns (y, save_mean, save_invstd).
std::vector<at::Tensor> bn_forward_apply(const at::Tensor& x, const at::Tensor& sums,
                                         const c10::optional<at::Tensor>& weight,
                                         const c10::optional<at::Tensor>& bias,
                                         const c10::optional<at::Tensor>& running_mean,
                                         const c10::optional<at::Tensor>& running_var,
                                         double momentum, double eps,
                                         const c10::optional<at::Tensor>& residual, bool relu,
                                         int64_t C,
                                         const c10::optional<at::Tensor>& num_batches_tracked,
                                         bool out_moments, double clip) {
  check_input(x, C, "x");
  TORCH_CHECK(sums.scalar_type() == at::kDouble && sums.numel() == 2 * C + 1, "bad moments");
  int64_t* nbt = nullptr;
  if (num_batches_tracked.has_value() && num_batches_tracked->defined()) {
    TORCH_CHECK(num_batches_tracked->scalar_type() == at::kLong && num_batches_tracked->numel() == 1 &&
                    num_batches_tracked->is_cuda(), "num_batches_tracked must be a 1-element int64 GPU tensor");
    nbt = num_batches_tracked->data_ptr<int64_t>();
  }
  const int64_t M = x.numel() / C;
  auto y = at::empty_like(x);
  auto saved = at::empty({2, C}, x.options().dtype(at::kFloat));
  auto stream = at::hip::getCurrentHIPStream();
  const bool has_res = residual.has_value() && residual->defined();
  if (has_res) check_input(*residual, C, "residual");
  at::Tensor osums;
  if (out_moments) {
    TORCH_CHECK(relu && !has_res && x.scalar_type() == at::kBFloat16,
                "out_moments: bf16 BN + ReLU without residual only");
    osums = at::empty({2 * C + 1}, x.options().dtype(at::kDouble));
    if (M == 0) osums.zero_();
  }
  if (M > 0 && out_moments) {
    Grid g = plan(M, (int)C, vec_of(x));
    auto part = at::empty({2, (int64_t)g.grid.x, C}, x.options().dtype(at::kFloat));
    double* zt = moments_zero_target(osums.data_ptr<double>(), (int)g.grid.x);
    using T = __bf16;
#define DMP_BN_FWD_OS(NT)                                                                          \
  hipLaunchKernelGGL((bn_apply_kernel<T, true, false, true, NT, true>), g.grid, dim3(kThreads), 0,   \
                     stream, ptr<T>(x), nullptr, sums.data_ptr<double>(), fptr(weight), fptr(bias), \
                     fptr(running_mean), fptr(running_var), (float)momentum, (float)eps, M, (int)C, \
                     g.rows_per_block, ptr<T>(y), saved.data_ptr<float>(), saved.data_ptr<float>() + C, \
                     nbt, part.data_ptr<float>(), zt, (float)clip)
    if (streaming(M, C)) DMP_BN_FWD_OS(true);
    else DMP_BN_FWD_OS(false);
#undef DMP_BN_FWD_OS
    bn_reduce_partials_launch(part.data_ptr<float>(), (int)g.grid.x, (int)C, osums.data_ptr<double>(),
                              (double)M, stream);
  } else if (M > 0) {
    Grid g = plan(M, (int)C, vec_of(x));
    dispatch_t(x, [&](auto tag) {
      using T = decltype(tag);
      const T* r = has_res ? ptr<T>(*residual) : nullptr;
#define DMP_BN_FWD1(RELU, RES, NT)                                                               \
  hipLaunchKernelGGL((bn_apply_kernel<T, RELU, RES, true, NT>), g.grid, dim3(kThreads), 0, stream, \
                     ptr<T>(x), r, sums.data_ptr<double>(), fptr(weight), fptr(bias),            \
                     fptr(running_mean), fptr(running_var), (float)momentum, (float)eps, M,      \
                     (int)C, g.rows_per_block, ptr<T>(y), saved.data_ptr<float>(),               \
                     saved.data_ptr<float>() + C, nbt, nullptr, nullptr, (float)clip)
#define DMP_BN_FWD(RELU, RES) \
  do { if (streaming(M, C)) DMP_BN_FWD1(RELU, RES, true); else DMP_BN_FWD1(RELU, RES, false); } while (0)
      if (relu && has_res) DMP_BN_FWD(true, true);
      else if (relu) DMP_BN_FWD(true, false);
      else if (has_res) DMP_BN_FWD(false, true);
      else DMP_BN_FWD(false, false);
#undef DMP_BN_FWD
#undef DMP_BN_FWD1
    });
  }
  if (out_moments) return {y, saved[0], saved[1], osums};
  return {y, saved[0], saved[1]};
}

// Training-mode coefficients from (global) moments without touching x.
// Returns coef [4, C] fp32 = (scale, shift, mean, invstd).
at::Tensor bn_finalize(const at::Tensor& sums, const c10::optional<at::Tensor>& weight,
                       const c10::optional<at::Tensor>& bias,
                       const c10::optional<at::Tensor>& running_mean,
                       const c10::optional<at::Tensor>& running_var, double momentum, double eps,
                       int64_t C, const c10::optional<at::Tensor>& num_batches_tracked) {
  TORCH_CHECK(sums.is_cuda() && sums.scalar_type() == at::kDouble && sums.numel() == 2 * C + 1,
              "bad moments");
  auto coef = at::empty({4, C}, sums.options().dtype(at::kFloat));
  int64_t* nbt = nullptr;
  if (num_batches_tracked.has_value() && num_batches_tracked->defined()) {
    TORCH_CHECK(num_batches_tracked->scalar_type() == at::kLong && num_batches_tracked->numel() == 1,
                "num_batches_tracked must be a 1-element int64 tensor");
    nbt = num_batches_tracked->data_ptr<int64_t>();
  }
  auto stream = at::hip::getCurrentHIPStream();
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, stream,
                     sums.data_ptr<double>(), fptr(weight), fptr(bias), fptr(running_mean),
                     fptr(running_var), (float)momentum, (float)eps, (int)C, coef.data_ptr<float>(),
                     nbt);
  return coef;
}

// Eval-mode apply from running statistics.  Returns (y, mean, invstd).
std::vector<at::Tensor> bn_eval_apply(const at::Tensor& x, const at::Tensor& running_mean,
                                      const at::Tensor& running_var,
                                      const c10::optional<at::Tensor>& weight,
                                      const c10::optional<at::Tensor>& bias, double eps,
                                      const c10::optional<at::Tensor>& residual, bool relu,
                                      int64_t C, double clip) {
  check_input(x, C, "x");
  const int64_t M = x.numel() / C;
  auto y = at::empty_like(x);
  auto saved = at::empty({2, C}, x.options().dtype(at::kFloat));
  auto stream = at::hip::getCurrentHIPStream();
  const bool has_res = residual.has_value() && residual->defined();
  if (has_res) check_input(*residual, C, "residual");
  auto rm = running_mean.to(at::kFloat).contiguous();
  auto rv = running_var.to(at::kFloat).contiguous();
  if (M > 0) {
    Grid g = plan(M, (int)C, vec_of(x));
    dispatch_t(x, [&](auto tag) {
      using T = decltype(tag);
      const T* r = has_res ? ptr<T>(*residual) : nullptr;
#define DMP_BN_EVAL(RELU, RES)                                                                   \
  hipLaunchKernelGGL((bn_apply_kernel<T, RELU, RES, false>), g.grid, dim3(kThreads), 0, stream,  \
                     ptr<T>(x), r, nullptr, fptr(weight), fptr(bias), rm.data_ptr<float>(),      \
                     rv.data_ptr<float>(), 0.f, (float)eps, M, (int)C, g.rows_per_block,         \
                     ptr<T>(y), saved.data_ptr<float>(), saved.data_ptr<float>() + C, nullptr,   \
                     nullptr, nullptr, (float)clip)
      if (relu && has_res) DMP_BN_EVAL(true, true);
      else if (relu) DMP_BN_EVAL(true, false);
      else if (has_res) DMP_BN_EVAL(false, true);
      else DMP_BN_EVAL(false, false);
#undef DMP_BN_EVAL
    });
  }
  return {y, saved[0], saved[1]};
}

// Backward local moments: fp64 [2C] = (sum dz, sum dz*(x-mean)).
// relu with y undefined: the ReLU mask is re-derived from x with the forward's
// affine (needs invstd; weight/bias optional) -- see bn_bwd_moments_kernel.
at::Tensor bn_backward_moments(const at::Tensor& dy, const at::Tensor& x,
                               const c10::optional<at::Tensor>& y, const at::Tensor& mean,
                               bool relu, int64_t C, const c10::optional<at::Tensor>& weight,
                               const c10::optional<at::Tensor>& bias,
                               const c10::optional<at::Tensor>& invstd, double clip) {
  check_input(dy, C, "grad");
  check_input(x, C, "x");
  const int64_t M = x.numel() / C;
  auto stream = at::hip::getCurrentHIPStream();
  if (M == 0) return at::zeros({2 * C}, x.options().dtype(at::kDouble));
  auto sums = at::empty({2 * C}, x.options().dtype(at::kDouble));
  Grid g = plan(M, (int)C, vec_of(x));
  auto part = at::empty({2, (int64_t)g.grid.x, C}, x.options().dtype(at::kFloat));
  float* pp = part.data_ptr<float>();
  double* zt = moments_zero_target(sums.data_ptr<double>(), (int)g.grid.x);
  const bool from_y = relu && y.has_value() && y->defined();
  if (relu && !from_y)
    TORCH_CHECK(invstd.has_value() && invstd->defined(), "relu mask from x needs invstd");
  const float* ip = fptr(invstd);
  dispatch_t(x, [&](auto tag) {
    using T = decltype(tag);
    const T* yp = from_y ? ptr<T>(*y) : nullptr;
#define DMP_BN_BM(MODE)                                                                          \
  hipLaunchKernelGGL((bn_bwd_moments_kernel<T, MODE>), g.grid, dim3(kThreads), 0, stream,        \
                     ptr<T>(dy), ptr<T>(x), yp, mean.data_ptr<float>(), fptr(weight), fptr(bias), \
                     ip, M, (int)C, g.rows_per_block, pp, zt, (float)clip)
    if (!relu) DMP_BN_BM(0);
    else if (from_y) DMP_BN_BM(1);
    else DMP_BN_BM(2);
#undef DMP_BN_BM
  });
  bn_reduce_partials_launch(pp, (int)g.grid.x, (int)C, sums.data_ptr<double>(), -1.0, stream);
  return sums;
}

// Backward apply.  Returns (dx, dweight, dbias, dresidual-or-undefined).
std::vector<at::Tensor> bn_backward_apply(const at::Tensor& dy, const at::Tensor& x,
                                          const c10::optional<at::Tensor>& y,
                                          const at::Tensor& sums, const at::Tensor& count,
                                          const c10::optional<at::Tensor>& weight,
                                          const at::Tensor& mean, const at::Tensor& invstd,
                                          bool training, bool relu, bool want_dres, int64_t C,
                                          const c10::optional<at::Tensor>& bias, double clip,
                                          const c10::optional<at::Tensor>& acc_weight,
                                          const c10::optional<at::Tensor>& acc_bias) {
  TORCH_CHECK(count.scalar_type() == at::kDouble && count.numel() >= 1, "count must be fp64");
  check_input(dy, C, "grad");
  const int64_t M = x.numel() / C;
  auto stream = at::hip::getCurrentHIPStream();
  // acc_weight / acc_bias (fp32 [C] gradients, both or neither): the affine
  // gradients are ADDED into them (micro-batch accumulation, ops/grad_accum.py)
  const bool acc = acc_weight.has_value() && acc_weight->defined();
  TORCH_CHECK(acc == (acc_bias.has_value() && acc_bias->defined()), "bn_backward_apply: acc_weight and acc_bias together");
  if (acc)
    TORCH_CHECK(acc_weight->scalar_type() == at::kFloat && acc_bias->scalar_type() == at::kFloat &&
                    acc_weight->is_contiguous() && acc_bias->is_contiguous() && acc_weight->numel() == C &&
                    acc_bias->numel() == C,
                "bn_backward_apply: accumulation targets must be contiguous fp32 [C]");
  auto dwb = acc ? at::Tensor() : at::empty({2, C}, x.options().dtype(at::kFloat));
  float* dwp = acc ? acc_weight->data_ptr<float>() : dwb.data_ptr<float>();
  float* dbp = acc ? acc_bias->data_ptr<float>() : dwb.data_ptr<float>() + C;
  auto dx = at::empty_like(x);
  at::Tensor dres;
  if (want_dres) dres = at::empty_like(x);
  if (M > 0) {
    Grid g = plan(M, (int)C, vec_of(x));
    dispatch_t(x, [&](auto tag) {
      using T = decltype(tag);
      const bool from_y = relu && y.has_value() && y->defined();
      const T* yp = from_y ? ptr<T>(*y) : nullptr;
      T* dr = want_dres ? ptr<T>(dres) : nullptr;
#define DMP_BN_BWD(RELU, DRES) \
  do { if (streaming(M, C)) DMP_BN_BWD1(RELU, DRES, true); else DMP_BN_BWD1(RELU, DRES, false); } while (0)
#define DMP_BN_BWD1(RELU, DRES, NT)                                                               \
  hipLaunchKernelGGL((bn_bwd_apply_kernel<T, RELU, DRES, NT>), g.grid, dim3(kThreads), 0, stream, \
                     ptr<T>(dy), ptr<T>(x), yp, sums.data_ptr<double>(), count.data_ptr<double>(), \
                     fptr(weight), fptr(bias), mean.data_ptr<float>(), invstd.data_ptr<float>(),  \
                     (int)training, M, (int)C, g.rows_per_block, ptr<T>(dx), dr,                  \
                     dwp, dbp, (float)clip, (int)acc)
      const int mode = !relu ? 0 : (from_y ? 1 : 2);
      if (mode == 1 && want_dres) DMP_BN_BWD(1, true);
      else if (mode == 1) DMP_BN_BWD(1, false);
      else if (mode == 2 && want_dres) DMP_BN_BWD(2, true);
      else if (mode == 2) DMP_BN_BWD(2, false);
      else if (want_dres) DMP_BN_BWD(0, true);
      else DMP_BN_BWD(0, false);
#undef DMP_BN_BWD
#undef DMP_BN_BWD1
    });
  }
  if (acc) return {dx, at::Tensor(), at::Tensor(), dres};
  return {dx, dwb[0], dwb[1], dres};
}

void set_bn_streaming(bool on) { g_bn_streaming = on; }

}  // namespace dmp
