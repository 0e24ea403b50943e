// Channels-last (NHWC / [M, C]) batch normalisation for gfx950, with the
// activation and the residual add fused in, plus the split-phase entry points
// SyncBatchNorm needs (local partial moments -> RCCL all-reduce -> finalize).
//
// Capability parity: upstream BatchNorm2d / SyncBatchNorm as studied in the
// reference README (Readme.md:151 "prepare for sync batch norm layers",
// SURVEY.md D11).  Design is MI355X-first:
//   * x is viewed as a row-major [M, C] matrix (M = N*H*W).  Each lane owns ONE
//     16-byte channel vector (8 bf16 or 4 f32) for the whole launch, so its
//     scale/shift live in registers and every global access is a 16-B
//     coalesced load; a block walks a contiguous slab of rows.
//   * moments: fp32 per-lane partial sums -> per-block partials in HBM ->
//     one reduce kernel that sums the partials in fp64 (no E[x^2]-E[x]^2
//     catastrophic cancellation at M = 3.2M rows) and finalises
//     mean/invstd/scale/shift/running stats in the same launch.
//   * backward needs 2 passes (moments of dz, then dx); ReLU is re-derived from
//     the saved OUTPUT (y > 0), so nothing extra is stored.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include "../common.h"

namespace dmp {
namespace {

constexpr int kThreads = 256;
constexpr int kRedCh = 32;     // channels per block in the partial-reduce kernel
constexpr int kRedGroups = 8;  // row groups per block in the partial-reduce kernel

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

// -------------------------------------------------------------------------
// Phase 1 (forward): per-block partial sum / sum of squares per channel.
// grid = (row_blocks, channel_chunks)
// -------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(kThreads) void bn_moments_partial_kernel(
    const T* __restrict__ x, int64_t M, int C, int64_t rows_per_block,
    float* __restrict__ psum, float* __restrict__ psq) {
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
    int64_t r = r0 + lr;
    // 2 rows in flight per lane per iteration for memory-level parallelism.
    for (; r + L.rpi < r1; r += 2 * L.rpi) {
      float a[VEC], b[VEC];
      Vec16<T>::load(p + r * C, a);
      Vec16<T>::load(p + (r + L.rpi) * C, b);
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        s[i] += a[i] + b[i];
        q[i] = fmaf(a[i], a[i], fmaf(b[i], b[i], q[i]));
      }
    }
    if (r < r1) {
      float a[VEC];
      Vec16<T>::load(p + r * C, a);
#pragma unroll
      for (int i = 0; i < VEC; ++i) { s[i] += a[i]; q[i] = fmaf(a[i], a[i], q[i]); }
    }
  }
  // Combine the rpi row-lanes of each channel through LDS.
  __shared__ float lds_s[kThreads * VEC];
  __shared__ float lds_q[kThreads * VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    lds_s[tid * VEC + i] = s[i];
    lds_q[tid * VEC + i] = q[i];
  }
  __syncthreads();
  const int nout = L.tc * VEC;
  for (int o = tid; o < nout; o += kThreads) {
    const int c_l = o / VEC, e = o % VEC;
    const int cg = (blockIdx.y * L.tc + c_l) * VEC + e;
    if (cg >= C) continue;
    float ss = 0.f, qq = 0.f;
    for (int rr = 0; rr < L.rpi; ++rr) {
      ss += lds_s[(rr * L.tc + c_l) * VEC + e];
      qq += lds_q[(rr * L.tc + c_l) * VEC + e];
    }
    psum[(int64_t)blockIdx.x * C + cg] = ss;
    psq[(int64_t)blockIdx.x * C + cg] = qq;
  }
}

// -------------------------------------------------------------------------
// Phase 2: fp64 reduction of the per-block partials.  One block per 32
// channels, 8 row groups.  Writes sums[c] / sums[C + c] (fp64) and, when
// `finalize` is set, the forward or backward per-channel coefficients.
// -------------------------------------------------------------------------
__global__ __launch_bounds__(kThreads) void bn_reduce_partials_kernel(
    const float* __restrict__ pa, const float* __restrict__ pb, int nb, int C,
    double* __restrict__ sums, double count) {
  const int cl = threadIdx.x % kRedCh, g = threadIdx.x / kRedCh;
  const int c = blockIdx.x * kRedCh + cl;
  double a = 0.0, b = 0.0;
  if (c < C) {
    int i = g;
    for (; i + 3 * kRedGroups < nb; i += 4 * kRedGroups) {
      float a0 = pa[(int64_t)i * C + c], a1 = pa[(int64_t)(i + kRedGroups) * C + c];
      float a2 = pa[(int64_t)(i + 2 * kRedGroups) * C + c], a3 = pa[(int64_t)(i + 3 * kRedGroups) * C + c];
      float b0 = pb[(int64_t)i * C + c], b1 = pb[(int64_t)(i + kRedGroups) * C + c];
      float b2 = pb[(int64_t)(i + 2 * kRedGroups) * C + c], b3 = pb[(int64_t)(i + 3 * kRedGroups) * C + c];
      a += (double)a0 + (double)a1 + (double)a2 + (double)a3;
      b += (double)b0 + (double)b1 + (double)b2 + (double)b3;
    }
    for (; i < nb; i += kRedGroups) {
      a += (double)pa[(int64_t)i * C + c];
      b += (double)pb[(int64_t)i * C + c];
    }
  }
  __shared__ double la[kThreads], lb[kThreads];
  la[threadIdx.x] = a;
  lb[threadIdx.x] = b;
  __syncthreads();
  if (g == 0 && c < C) {
    for (int k = 1; k < kRedGroups; ++k) {
      a += la[k * kRedCh + cl];
      b += lb[k * kRedCh + cl];
    }
    sums[c] = a;
    sums[C + c] = b;
  }
  if (count >= 0.0 && blockIdx.x == 0 && threadIdx.x == 0) sums[2 * C] = count;
}

// Forward finalize from global moments sums[0:C] = sum x, sums[C:2C] = sum x^2,
// sums[2C] = number of rows summed (all ranks) -- read on device, so SyncBN
// never needs a host round-trip for the global count.
__global__ void bn_forward_finalize_kernel(
    const double* __restrict__ sums, int C,
    const float* __restrict__ weight, const float* __restrict__ bias,
    float* __restrict__ running_mean, float* __restrict__ running_var,
    float momentum, float eps, float* __restrict__ save_mean,
    float* __restrict__ save_invstd, float* __restrict__ scale,
    float* __restrict__ shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const double count = sums[2 * C];
  const double mean = sums[c] / count;
  double var = sums[C + c] / count - mean * mean;
  var = var < 0.0 ? 0.0 : var;
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  save_mean[c] = (float)mean;
  save_invstd[c] = invstd;
  const float w = weight ? weight[c] : 1.f;
  const float b = bias ? bias[c] : 0.f;
  const float sc = w * invstd;
  scale[c] = sc;
  shift[c] = b - (float)mean * sc;
  if (running_mean) {
    const double unbiased = count > 1.0 ? var * count / (count - 1.0) : var;
    running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * (float)mean;
    running_var[c] = (1.f - momentum) * running_var[c] + momentum * (float)unbiased;
  }
}

// Eval-mode coefficients from running statistics.
__global__ void bn_eval_coeffs_kernel(const float* __restrict__ rm, const float* __restrict__ rv,
                                      const float* __restrict__ weight, const float* __restrict__ bias,
                                      float eps, int C, float* __restrict__ save_mean,
                                      float* __restrict__ save_invstd, float* __restrict__ scale,
                                      float* __restrict__ shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float invstd = rsqrtf(rv[c] + eps);
  const float w = weight ? weight[c] : 1.f, b = bias ? bias[c] : 0.f;
  save_mean[c] = rm[c];
  save_invstd[c] = invstd;
  scale[c] = w * invstd;
  shift[c] = b - rm[c] * w * invstd;
}

// -------------------------------------------------------------------------
// Elementwise apply: y = act(x*scale + shift [+ residual])
// -------------------------------------------------------------------------
template <typename T, bool RELU, bool RES>
__global__ __launch_bounds__(kThreads) void bn_apply_kernel(
    const T* __restrict__ x, const T* __restrict__ res, const float* __restrict__ scale,
    const float* __restrict__ shift, int64_t M, int C, int64_t rows_per_block, T* __restrict__ y) {
  constexpr int VEC = Vec16<T>::N;
  const Layout L = make_layout(C, VEC);
  const int tid = threadIdx.x;
  const int lc = tid % L.tc, lr = tid / L.tc;
  const int cvec = blockIdx.y * L.tc + lc;
  if (lr >= L.rpi || cvec >= L.cv) return;
  float sc[VEC], sh[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) { sc[i] = scale[cvec * VEC + i]; sh[i] = shift[cvec * VEC + i]; }
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(M, r0 + rows_per_block);
  const int64_t off0 = (int64_t)cvec * VEC;
  for (int64_t r = r0 + lr; r < r1; r += L.rpi) {
    const int64_t o = r * C + off0;
    float v[VEC];
    Vec16<T>::load(x + o, v);
    float rv[VEC];
    if (RES) Vec16<T>::load(res + o, rv);
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      float t = fmaf(v[i], sc[i], sh[i]);
      if (RES) t += rv[i];
      if (RELU) t = fmaxf(t, 0.f);
      v[i] = t;
    }
    Vec16<T>::store(y + o, v);
  }
}

// -------------------------------------------------------------------------
// Backward phase 1: partial sums of dz and dz*(x - mean), dz = dy * [y > 0].
// -------------------------------------------------------------------------
template <typename T, bool RELU>
__global__ __launch_bounds__(kThreads) void bn_bwd_partial_kernel(
    const T* __restrict__ dy, const T* __restrict__ x, const T* __restrict__ y,
    const float* __restrict__ mean, int64_t M, int C, int64_t rows_per_block,
    float* __restrict__ pdz, float* __restrict__ pdzx) {
  constexpr int VEC = Vec16<T>::N;
  const Layout L = make_layout(C, VEC);
  const int tid = threadIdx.x;
  const int lc = tid % L.tc, lr = tid / L.tc;
  const int cvec = blockIdx.y * L.tc + lc;
  const bool active = lr < L.rpi && cvec < L.cv;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(M, r0 + rows_per_block);
  float s[VEC], q[VEC], mu[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) { s[i] = 0.f; q[i] = 0.f; mu[i] = 0.f; }
  if (active) {
#pragma unroll
    for (int i = 0; i < VEC; ++i) mu[i] = mean[cvec * VEC + i];
    const int64_t off0 = (int64_t)cvec * VEC;
    for (int64_t r = r0 + lr; r < r1; r += L.rpi) {
      const int64_t o = r * C + off0;
      float g[VEC], xv[VEC];
      Vec16<T>::load(dy + o, g);
      Vec16<T>::load(x + o, xv);
      if (RELU) {
        float yv[VEC];
        Vec16<T>::load(y + o, yv);
#pragma unroll
        for (int i = 0; i < VEC; ++i) g[i] = yv[i] > 0.f ? g[i] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        s[i] += g[i];
        q[i] = fmaf(g[i], xv[i] - mu[i], q[i]);
      }
    }
  }
  __shared__ float lds_s[kThreads * VEC];
  __shared__ float lds_q[kThreads * VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    lds_s[tid * VEC + i] = s[i];
    lds_q[tid * VEC + i] = q[i];
  }
  __syncthreads();
  const int nout = L.tc * VEC;
  for (int o = tid; o < nout; o += kThreads) {
    const int c_l = o / VEC, e = o % VEC;
    const int cg = (blockIdx.y * L.tc + c_l) * VEC + e;
    if (cg >= C) continue;
    float ss = 0.f, qq = 0.f;
    for (int rr = 0; rr < L.rpi; ++rr) {
      ss += lds_s[(rr * L.tc + c_l) * VEC + e];
      qq += lds_q[(rr * L.tc + c_l) * VEC + e];
    }
    pdz[(int64_t)blockIdx.x * C + cg] = ss;
    pdzx[(int64_t)blockIdx.x * C + cg] = qq;
  }
}

// Backward finalize: dx = a*dz + b*x + c per channel; dweight, dbias.
__global__ void bn_backward_finalize_kernel(
    const double* __restrict__ sums, const double* __restrict__ count_ptr, int C, const float* __restrict__ weight,
    const float* __restrict__ mean, const float* __restrict__ invstd, int training,
    float* __restrict__ coef_a, float* __restrict__ coef_b, float* __restrict__ coef_c,
    float* __restrict__ dweight, float* __restrict__ dbias) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const double count = *count_ptr;
  const double sdz = sums[c], sdzx = sums[C + c];
  const float w = weight ? weight[c] : 1.f;
  const double is = invstd[c];
  if (dweight) dweight[c] = (float)(sdzx * is);
  if (dbias) dbias[c] = (float)sdz;
  const double a = (double)w * is;
  if (training) {
    const double b = -a * is * is * sdzx / count;
    const double cc = -a * sdz / count - b * (double)mean[c];
    coef_a[c] = (float)a;
    coef_b[c] = (float)b;
    coef_c[c] = (float)cc;
  } else {
    coef_a[c] = (float)a;
    coef_b[c] = 0.f;
    coef_c[c] = 0.f;
  }
}

// Backward phase 2: dx = a*dz + b*x + c ; dres = dz (when the residual was fused).
template <typename T, bool RELU, bool DRES>
__global__ __launch_bounds__(kThreads) void bn_bwd_apply_kernel(
    const T* __restrict__ dy, const T* __restrict__ x, const T* __restrict__ y,
    const float* __restrict__ ca, const float* __restrict__ cb, const float* __restrict__ cc,
    int64_t M, int C, int64_t rows_per_block, T* __restrict__ dx, T* __restrict__ dres) {
  constexpr int VEC = Vec16<T>::N;
  const Layout L = make_layout(C, VEC);
  const int tid = threadIdx.x;
  const int lc = tid % L.tc, lr = tid / L.tc;
  const int cvec = blockIdx.y * L.tc + lc;
  if (lr >= L.rpi || cvec >= L.cv) return;
  float a[VEC], b[VEC], c[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    a[i] = ca[cvec * VEC + i];
    b[i] = cb[cvec * VEC + i];
    c[i] = cc[cvec * VEC + i];
  }
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(M, r0 + rows_per_block);
  const int64_t off0 = (int64_t)cvec * VEC;
  for (int64_t r = r0 + lr; r < r1; r += L.rpi) {
    const int64_t o = r * C + off0;
    float g[VEC], xv[VEC];
    Vec16<T>::load(dy + o, g);
    Vec16<T>::load(x + o, xv);
    if (RELU) {
      float yv[VEC];
      Vec16<T>::load(y + o, yv);
#pragma unroll
      for (int i = 0; i < VEC; ++i) g[i] = yv[i] > 0.f ? g[i] : 0.f;
    }
    if (DRES) Vec16<T>::store(dres + o, g);
#pragma unroll
    for (int i = 0; i < VEC; ++i) xv[i] = fmaf(a[i], g[i], fmaf(b[i], xv[i], c[i]));
    Vec16<T>::store(dx + o, xv);
  }
}

// ---------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------
struct Grid {
  dim3 grid;
  int64_t rows_per_block;
};

// Pick a 2-D grid with ~`target` blocks: grid.y chunks channels, grid.x slabs rows.
Grid plan(int64_t M, int C, int vec, int target = 2048, int64_t min_rows_per_lane = 4) {
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

void check_input(const at::Tensor& x, const char* name) {
  TORCH_CHECK(x.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16,
              name, " must be float32 or bfloat16");
}

// x viewed as [M, C] (channels-last contiguous); returns C.
int64_t rows_of(const at::Tensor& x, int64_t C) { return x.numel() / C; }

int vec_of(const at::Tensor& x) { return x.scalar_type() == at::kBFloat16 ? 8 : 4; }

template <typename F>
void dispatch_t(const at::Tensor& x, F&& f) {
  if (x.scalar_type() == at::kBFloat16) f(__bf16{});
  else f(float{});
}

template <typename T> T* ptr(const at::Tensor& t) { return reinterpret_cast<T*>(t.data_ptr()); }
const float* fptr_or_null(const c10::optional<at::Tensor>& t) {
  return (t.has_value() && t->defined()) ? t->data_ptr<float>() : nullptr;
}
float* fptr_or_null_mut(const c10::optional<at::Tensor>& t) {
  return (t.has_value() && t->defined()) ? t->data_ptr<float>() : nullptr;
}

}  // namespace

// Local moments: returns fp64 [2C+1] = (sum x, sum x^2, row count) over the local rows.
at::Tensor bn_local_moments(const at::Tensor& x, int64_t C) {
  check_input(x, "x");
  TORCH_CHECK(C % vec_of(x) == 0, "channels must be a multiple of the vector width");
  const int64_t M = rows_of(x, C);
  auto stream = at::hip::getCurrentHIPStream();
  auto fopt = x.options().dtype(at::kFloat);
  Grid g = plan(M, (int)C, vec_of(x));
  auto part = at::empty({2, (int64_t)g.grid.x, C}, fopt);
  auto sums = at::empty({2 * C + 1}, x.options().dtype(at::kDouble));
  float* ps = part.data_ptr<float>();
  float* pq = ps + (int64_t)g.grid.x * C;
  dispatch_t(x, [&](auto tag) {
    using T = decltype(tag);
    hipLaunchKernelGGL(bn_moments_partial_kernel<T>, g.grid, dim3(kThreads), 0, stream,
                       ptr<T>(x), M, (int)C, g.rows_per_block, ps, pq);
  });
  hipLaunchKernelGGL(bn_reduce_partials_kernel, dim3((C + kRedCh - 1) / kRedCh), dim3(kThreads), 0,
                     stream, ps, pq, (int)g.grid.x, (int)C, sums.data_ptr<double>(), (double)M);
  return sums;
}

// Finalize forward statistics from (possibly all-reduced) fp64 moments.
// Returns (save_mean, save_invstd, scale, shift), all fp32 [C].
std::vector<at::Tensor> bn_forward_finalize(const at::Tensor& sums, int64_t C,
                                            const c10::optional<at::Tensor>& weight,
                                            const c10::optional<at::Tensor>& bias,
                                            const c10::optional<at::Tensor>& running_mean,
                                            const c10::optional<at::Tensor>& running_var,
                                            double momentum, double eps) {
  auto stream = at::hip::getCurrentHIPStream();
  auto fopt = sums.options().dtype(at::kFloat);
  auto coeffs = at::empty({4, C}, fopt);
  float* base = coeffs.data_ptr<float>();
  hipLaunchKernelGGL(bn_forward_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, stream,
                     sums.data_ptr<double>(), (int)C, fptr_or_null(weight), fptr_or_null(bias),
                     fptr_or_null_mut(running_mean), fptr_or_null_mut(running_var), (float)momentum,
                     (float)eps, base, base + C, base + 2 * C, base + 3 * C);
  return {coeffs[0], coeffs[1], coeffs[2], coeffs[3]};
}

std::vector<at::Tensor> bn_eval_coeffs(const at::Tensor& running_mean, const at::Tensor& running_var,
                                       const c10::optional<at::Tensor>& weight,
                                       const c10::optional<at::Tensor>& bias, double eps) {
  const int64_t C = running_mean.numel();
  auto stream = at::hip::getCurrentHIPStream();
  auto coeffs = at::empty({4, C}, running_mean.options().dtype(at::kFloat));
  float* base = coeffs.data_ptr<float>();
  hipLaunchKernelGGL(bn_eval_coeffs_kernel, dim3((C + 255) / 256), dim3(256), 0, stream,
                     running_mean.data_ptr<float>(), running_var.data_ptr<float>(),
                     fptr_or_null(weight), fptr_or_null(bias), (float)eps, (int)C, base, base + C,
                     base + 2 * C, base + 3 * C);
  return {coeffs[0], coeffs[1], coeffs[2], coeffs[3]};
}

// y = act(x*scale + shift [+ residual]); x, residual channels-last contiguous.
at::Tensor bn_apply(const at::Tensor& x, const at::Tensor& scale, const at::Tensor& shift,
                    const c10::optional<at::Tensor>& residual, bool relu, int64_t C) {
  check_input(x, "x");
  const int64_t M = rows_of(x, C);
  auto y = at::empty_like(x);
  if (M == 0) return y;
  auto stream = at::hip::getCurrentHIPStream();
  Grid g = plan(M, (int)C, vec_of(x));
  const bool has_res = residual.has_value() && residual->defined();
  dispatch_t(x, [&](auto tag) {
    using T = decltype(tag);
    const T* r = has_res ? ptr<T>(*residual) : nullptr;
#define DMP_BN_APPLY(RELU, RES)                                                                    \
  hipLaunchKernelGGL((bn_apply_kernel<T, RELU, RES>), g.grid, dim3(kThreads), 0, stream, ptr<T>(x), \
                     r, scale.data_ptr<float>(), shift.data_ptr<float>(), M, (int)C,               \
                     g.rows_per_block, ptr<T>(y))
    if (relu && has_res) DMP_BN_APPLY(true, true);
    else if (relu) DMP_BN_APPLY(true, false);
    else if (has_res) DMP_BN_APPLY(false, true);
    else DMP_BN_APPLY(false, false);
#undef DMP_BN_APPLY
  });
  return y;
}

// Backward local moments: fp64 [2C] = (sum dz, sum dz*(x-mean)).
at::Tensor bn_backward_moments(const at::Tensor& dy, const at::Tensor& x,
                               const c10::optional<at::Tensor>& y, const at::Tensor& mean,
                               bool relu, int64_t C) {
  check_input(dy, "grad");
  const int64_t M = rows_of(x, C);
  auto stream = at::hip::getCurrentHIPStream();
  Grid g = plan(M, (int)C, vec_of(x));
  auto part = at::empty({2, (int64_t)g.grid.x, C}, x.options().dtype(at::kFloat));
  auto sums = at::empty({2 * C}, x.options().dtype(at::kDouble));
  float* ps = part.data_ptr<float>();
  float* pq = ps + (int64_t)g.grid.x * C;
  dispatch_t(x, [&](auto tag) {
    using T = decltype(tag);
    if (relu) {
      TORCH_CHECK(y.has_value() && y->defined(), "relu backward needs the saved output");
      hipLaunchKernelGGL((bn_bwd_partial_kernel<T, true>), g.grid, dim3(kThreads), 0, stream,
                         ptr<T>(dy), ptr<T>(x), ptr<T>(*y), mean.data_ptr<float>(), M, (int)C,
                         g.rows_per_block, ps, pq);
    } else {
      hipLaunchKernelGGL((bn_bwd_partial_kernel<T, false>), g.grid, dim3(kThreads), 0, stream,
                         ptr<T>(dy), ptr<T>(x), (const T*)nullptr, mean.data_ptr<float>(), M,
                         (int)C, g.rows_per_block, ps, pq);
    }
  });
  hipLaunchKernelGGL(bn_reduce_partials_kernel, dim3((C + kRedCh - 1) / kRedCh), dim3(kThreads), 0,
                     stream, ps, pq, (int)g.grid.x, (int)C, sums.data_ptr<double>(), -1.0);
  return sums;
}

// Backward finalize + apply.  Returns (dx, dweight, dbias, dresidual-or-undefined).
std::vector<at::Tensor> bn_backward_apply(const at::Tensor& dy, const at::Tensor& x,
                                          const c10::optional<at::Tensor>& y,
                                          const at::Tensor& sums, const at::Tensor& count,
                                          const c10::optional<at::Tensor>& weight,
                                          const at::Tensor& mean, const at::Tensor& invstd,
                                          bool training, bool relu, bool want_dres, int64_t C) {
  TORCH_CHECK(count.scalar_type() == at::kDouble && count.numel() >= 1, "count must be fp64");
  const int64_t M = rows_of(x, C);
  auto stream = at::hip::getCurrentHIPStream();
  auto fopt = x.options().dtype(at::kFloat);
  auto coef = at::empty({5, C}, fopt);
  float* cb = coef.data_ptr<float>();
  hipLaunchKernelGGL(bn_backward_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, stream,
                     sums.data_ptr<double>(), count.data_ptr<double>(), (int)C, fptr_or_null(weight),
                     mean.data_ptr<float>(), invstd.data_ptr<float>(), (int)training, cb, cb + C,
                     cb + 2 * C, cb + 3 * C, cb + 4 * C);
  auto dx = at::empty_like(x);
  at::Tensor dres;
  if (want_dres) dres = at::empty_like(x);
  if (M > 0) {
    Grid g = plan(M, (int)C, vec_of(x));
    dispatch_t(x, [&](auto tag) {
      using T = decltype(tag);
      const T* yp = relu ? ptr<T>(*y) : nullptr;
      T* dr = want_dres ? ptr<T>(dres) : nullptr;
#define DMP_BN_BWD(RELU, DRES)                                                                    \
  hipLaunchKernelGGL((bn_bwd_apply_kernel<T, RELU, DRES>), g.grid, dim3(kThreads), 0, stream,     \
                     ptr<T>(dy), ptr<T>(x), yp, cb, cb + C, cb + 2 * C, M, (int)C,                 \
                     g.rows_per_block, ptr<T>(dx), dr)
      if (relu && want_dres) DMP_BN_BWD(true, true);
      else if (relu) DMP_BN_BWD(true, false);
      else if (want_dres) DMP_BN_BWD(false, true);
      else DMP_BN_BWD(false, false);
#undef DMP_BN_BWD
    });
  }
  return {dx, coef[3], coef[4], dres};
}

}  // namespace dmp
