// LayerNorm over the last dim (ViT-B/16: D = 768) for gfx950, forward and
// backward, with the per-column dgamma / dbeta reduced in-kernel per block.
//
// Capability: torch.nn.LayerNorm as used by the BASELINE.json ViT-B/16 config
// (SURVEY.md §2.4 lists the reference workloads' device kernels).  Measured on
// MI355X (profiles/vit_b16_bs128_1gpu_v1.md): PyTorch-ROCm spends 3.6 ms of a
// 38 ms ViT-B/16 step in layer_norm forward / grad-input / grad-gamma-beta.
//
// Design:
//   * one wave64 per row, rows strided over the grid; a lane owns the 16-byte
//     column vectors c = lane, lane+64, ... (D/8 <= 64*MAXV), kept in
//     registers between the statistics and the normalise pass (x read once);
//   * two-pass mean/variance in fp32 from registers (no E[x^2]-E[x]^2);
//   * backward: dx = rstd * (g - xhat*mean(g*xhat) - mean(g)), g = dy*gamma,
//     plus per-lane running sums of dy*xhat and dy for the lane's columns ->
//     one partial row per block -> a column reduce launch.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include "../colreduce.h"
#include "../common.h"

namespace dmp {
namespace {

constexpr int kLnThreads = 256;  // 4 waves, one row each per iteration
constexpr int kMaxVMax = 4;      // 16-B vectors per lane -> D <= 64*4*8 = 2048
// (kernels are instantiated with 2 vectors per lane for D <= 1024: fewer registers)

template <typename T> struct PVec;  // parameter vector loads (fp32 or bf16 params)
template <> struct PVec<float> {
  __device__ static void load(const float* p, float (&v)[8]) {
    const f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) { v[i] = a[i]; v[i + 4] = b[i]; }
  }
};
template <> struct PVec<__bf16> {
  __device__ static void load(const __bf16* p, float (&v)[8]) {
    const f32x8 f = __builtin_convertvector(*reinterpret_cast<const bf16x8*>(p), f32x8);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = f[i];
  }
};

// activations: 8 elements per vector (bf16 16 B, fp32 2 x 16 B)
template <typename T> __device__ __forceinline__ void ld8(const T* p, float (&v)[8]);
template <> __device__ __forceinline__ void ld8<__bf16>(const __bf16* p, float (&v)[8]) {
  PVec<__bf16>::load(p, v);
}
template <> __device__ __forceinline__ void ld8<float>(const float* p, float (&v)[8]) {
  PVec<float>::load(p, v);
}
template <typename T> __device__ __forceinline__ void st8(T* p, const float (&v)[8]);
template <> __device__ __forceinline__ void st8<__bf16>(__bf16* p, const float (&v)[8]) {
  f32x8 f;
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = v[i];
  *reinterpret_cast<bf16x8*>(p) = __builtin_convertvector(f, bf16x8);
}
template <> __device__ __forceinline__ void st8<float>(float* p, const float (&v)[8]) {
  f32x4 a, b;
#pragma unroll
  for (int i = 0; i < 4; ++i) { a[i] = v[i]; b[i] = v[i + 4]; }
  *reinterpret_cast<f32x4*>(p) = a;
  *reinterpret_cast<f32x4*>(p + 4) = b;
}

// raw 8-element activation vectors held across a row (the prefetch buffer)
template <typename T> struct Raw8;
template <> struct Raw8<__bf16> {
  bf16x8 v;
  __device__ void load(const __bf16* p) { v = *reinterpret_cast<const bf16x8*>(p); }
  __device__ void get(float (&o)[8]) const {
    const f32x8 f = __builtin_convertvector(v, f32x8);
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = f[i];
  }
};
template <> struct Raw8<float> {
  f32x4 a, b;
  __device__ void load(const float* p) {
    a = *reinterpret_cast<const f32x4*>(p);
    b = *reinterpret_cast<const f32x4*>(p + 4);
  }
  __device__ void get(float (&o)[8]) const {
#pragma unroll
    for (int i = 0; i < 4; ++i) { o[i] = a[i]; o[i + 4] = b[i]; }
  }
};

// Sum over the LPR lanes of a row group (xor offsets < LPR stay inside it).
template <int LPR>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int off = LPR / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// RPW rows per wave pass: LPR = 64 / RPW lanes per row, lane l serves vectors
// (l % LPR) + LPR k of row 2 pass + l / LPR.  RPW = 2 for D = 768 (ViT-B): 32
// lanes x 3 vectors cover a row exactly (one row per wave left half the lanes
// idle on the third vector) and a wave keeps two rows = 3 KB of loads in
// flight instead of one.
template <typename T, typename P, int kMaxV, int RPW = 1>
__global__ __launch_bounds__(kLnThreads) void ln_fwd_kernel(const T* __restrict__ x,
                                                            const P* __restrict__ w,
                                                            const P* __restrict__ b, int64_t rows,
                                                            int D, float eps, T* __restrict__ y,
                                                            float* __restrict__ mean_out,
                                                            float* __restrict__ rstd_out) {
  constexpr int LPR = 64 / RPW;
  const int lane = (threadIdx.x & 63) % LPR, sub = (threadIdx.x & 63) / LPR;
  const int nv = D / 8;
  const int64_t wave = ((int64_t)blockIdx.x * (kLnThreads / 64) + (threadIdx.x >> 6)) * RPW + sub;
  const int64_t nwaves = (int64_t)gridDim.x * (kLnThreads / 64) * RPW;
  // w / b are never null (the host passes ones / zeros for an absent one) and
  // every load below goes to a clamped valid address with no branch around
  // it: a load under a lane- or row-guard is waited for before the next one
  // issues (the ISA had 8 serialized load -> vmcnt(0) round trips per row).
  float gw[kMaxV][8], gb[kMaxV][8];
#pragma unroll
  for (int k = 0; k < kMaxV; ++k) {
    const int c = min(lane + LPR * k, nv - 1);
    PVec<P>::load(w + c * 8, gw[k]);
    PVec<P>::load(b + c * 8, gb[k]);
  }
  // the next row's vectors are loaded before this row is reduced and written
  // (as ln_bwd_kernel): one row of loads always in flight per wave instead of
  // a dependent HBM round trip at the head of every row
  Raw8<T> nx[kMaxV];
  auto fetch = [&](int64_t r) {
    const T* xr = x + min(r, rows - 1) * D;
#pragma unroll
    for (int k = 0; k < kMaxV; ++k) nx[k].load(xr + min(lane + LPR * k, nv - 1) * 8);
  };
  fetch(wave);
  for (int64_t r = wave; r < rows; r += nwaves) {
    float v[kMaxV][8];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < kMaxV; ++k) {
      const int c = lane + LPR * k;
      if (c < nv) {
        nx[k].get(v[k]);
#pragma unroll
        for (int i = 0; i < 8; ++i) s += v[k][i];
      }
    }
    fetch(r + nwaves);
    const float mean = group_sum<LPR>(s) / (float)D;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < kMaxV; ++k) {
      const int c = lane + LPR * k;
      if (c < nv) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float d = v[k][i] - mean;
          q = fmaf(d, d, q);
        }
      }
    }
    const float rstd = rsqrtf(group_sum<LPR>(q) / (float)D + eps);
    T* yr = y + r * D;
#pragma unroll
    for (int k = 0; k < kMaxV; ++k) {
      const int c = lane + LPR * k;
      if (c < nv) {
        float o[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = fmaf((v[k][i] - mean) * rstd, gw[k][i], gb[k][i]);
        st8<T>(yr + c * 8, o);
      }
    }
    if (lane == 0) {
      mean_out[r] = mean;
      rstd_out[r] = rstd;
    }
  }
}

// dgamma/dbeta partials: part[block][0:D] = sum dy*xhat, part[block][D:2D] = sum dy.
// The next row's x / dy / residual-gradient vectors are loaded before the
// current row is reduced and written (one row of loads always in flight per
// wave): with one wave per row the kernel is otherwise latency-bound, not
// bandwidth-bound (85 us -> see profiles/vit_b16_bs128_1gpu_v3.md).
template <typename T, typename P, int kMaxV, int RPW = 1>
__global__ __launch_bounds__(kLnThreads) void ln_bwd_kernel(
    const T* __restrict__ dy, const T* __restrict__ x, const P* __restrict__ w,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in, int64_t rows, int D,
    T* __restrict__ dx, float* __restrict__ part, const T* __restrict__ dres) {
  constexpr int LPR = 64 / RPW;  // lanes per row (see ln_fwd_kernel)
  const int lane = (threadIdx.x & 63) % LPR, sub = (threadIdx.x & 63) / LPR, wid = threadIdx.x >> 6;
  const int nv = D / 8;
  const int64_t wave = ((int64_t)blockIdx.x * (kLnThreads / 64) + wid) * RPW + sub;
  const int64_t nwaves = (int64_t)gridDim.x * (kLnThreads / 64) * RPW;
  float gw[kMaxV][8], accw[kMaxV][8], accb[kMaxV][8];
#pragma unroll
  for (int k = 0; k < kMaxV; ++k) {
    const int c = lane + LPR * k;
#pragma unroll
    for (int i = 0; i < 8; ++i) { accw[k][i] = 0.f; accb[k][i] = 0.f; }
    PVec<P>::load(w + min(c, nv - 1) * 8, gw[k]);  // never null (see ln_fwd_kernel)
  }
  Raw8<T> nx[kMaxV], ndy[kMaxV], nres[kMaxV];
  float nmean = 0.f, nrstd = 0.f;
  auto fetch = [&](int64_t r) {  // clamped, branch-free loads (see ln_fwd_kernel)
    r = min(r, rows - 1);
    nmean = mean_in[r];
    nrstd = rstd_in[r];
#pragma unroll
    for (int k = 0; k < kMaxV; ++k) {
      const int64_t o = r * D + min(lane + LPR * k, nv - 1) * 8;
      nx[k].load(x + o);
      ndy[k].load(dy + o);
    }
    if (dres) {
#pragma unroll
      for (int k = 0; k < kMaxV; ++k) nres[k].load(dres + r * D + min(lane + LPR * k, nv - 1) * 8);
    }
  };
  fetch(wave);
  for (int64_t r = wave; r < rows; r += nwaves) {
    const float mean = nmean, rstd = nrstd;
    float xh[kMaxV][8], g[kMaxV][8], rv[kMaxV][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < kMaxV; ++k) {
      const int c = lane + LPR * k;
      if (c < nv) {
        float dv[8];
        nx[k].get(xh[k]);
        ndy[k].get(dv);
        if (dres) nres[k].get(rv[k]);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          xh[k][i] = (xh[k][i] - mean) * rstd;
          g[k][i] = dv[i] * gw[k][i];
          s1 = fmaf(g[k][i], xh[k][i], s1);
          s2 += g[k][i];
          accw[k][i] = fmaf(dv[i], xh[k][i], accw[k][i]);
          accb[k][i] += dv[i];
        }
      }
    }
    fetch(r + nwaves);  // next row in flight during the reduce + store
    const float c1 = group_sum<LPR>(s1) / (float)D, c2 = group_sum<LPR>(s2) / (float)D;
#pragma unroll
    for (int k = 0; k < kMaxV; ++k) {
      const int c = lane + LPR * k;
      if (c < nv) {
        float o[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = rstd * (g[k][i] - xh[k][i] * c1 - c2);
        if (dres) {  // + the residual branch's gradient of the same input (one pass)
#pragma unroll
          for (int i = 0; i < 8; ++i) o[i] += rv[k][i];
        }
        st8<T>(dx + r * D + c * 8, o);
      }
    }
  }
  // combine the column partials of the 4 waves x RPW row groups through LDS,
  // one partial row per block
  constexpr int G = kLnThreads / 64 * RPW;
  __shared__ float red[2][G][LPR * 8];
#pragma unroll
  for (int k = 0; k < kMaxV; ++k) {
    const int c = lane + LPR * k;
    if (k * LPR >= nv) break;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      red[0][wid * RPW + sub][lane * 8 + i] = accw[k][i];
      red[1][wid * RPW + sub][lane * 8 + i] = accb[k][i];
    }
    __syncthreads();
    for (int e = threadIdx.x; e < LPR * 8; e += kLnThreads) {
      const int col = (k * LPR + e / 8) * 8 + (e % 8);
      if (col < D) {
        float sw = 0.f, sb = 0.f;
#pragma unroll
        for (int q = 0; q < G; ++q) { sw += red[0][q][e]; sb += red[1][q][e]; }
        part[(int64_t)blockIdx.x * 2 * D + col] = sw;
        part[(int64_t)blockIdx.x * 2 * D + D + col] = sb;
      }
    }
    __syncthreads();
    (void)c;
  }
}


void check_ln(const at::Tensor& x, int64_t D, const char* name) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous(), name, " must be a contiguous GPU tensor");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kFloat,
              name, " must be bf16 or fp32");
  TORCH_CHECK(x.numel() % D == 0, name, " is not a multiple of the normalised size");
}

int ln_blocks(int64_t rows, int64_t cap = 2048) {
  return (int)std::max<int64_t>(1, std::min<int64_t>((rows + 3) / 4, cap));
}

}  // namespace

bool layernorm_supported(int64_t D) { return D % 8 == 0 && D / 8 <= 64 * kMaxVMax; }

// Returns (y, mean[rows], rstd[rows]); x viewed as [rows, D].
std::vector<at::Tensor> layernorm_forward(const at::Tensor& x, const c10::optional<at::Tensor>& w,
                                          const c10::optional<at::Tensor>& b, int64_t D,
                                          double eps) {
  check_ln(x, D, "x");
  TORCH_CHECK(layernorm_supported(D), "layernorm: D must be a multiple of 8 and <= 2048");
  const bool hw = w.has_value() && w->defined(), hb = b.has_value() && b->defined();
  TORCH_CHECK(!hw || (w->is_contiguous() && w->numel() == D), "bad weight");
  TORCH_CHECK(!hb || (b->is_contiguous() && b->numel() == D), "bad bias");
  TORCH_CHECK(!hw || !hb || w->scalar_type() == b->scalar_type(), "weight/bias dtype mismatch");
  const int64_t rows = x.numel() / D;
  auto y = at::empty_like(x);
  auto mean = at::empty({rows}, x.options().dtype(at::kFloat));
  auto rstd = at::empty({rows}, x.options().dtype(at::kFloat));
  if (rows == 0) return {y, mean, rstd};
  auto stream = at::hip::getCurrentHIPStream();
  const bool pbf = (hw && w->scalar_type() == at::kBFloat16) || (!hw && hb && b->scalar_type() == at::kBFloat16);
  // an absent weight / bias is passed as ones / zeros (branch-free kernel loads)
  const auto popt = x.options().dtype(pbf ? at::kBFloat16 : at::kFloat);
  const at::Tensor wt = hw ? *w : at::ones({D}, popt), bt = hb ? *b : at::zeros({D}, popt);
  const dim3 grid(ln_blocks(rows)), block(kLnThreads);
#define DMP_LN_FWD(T, P)                                                                       \
  hipLaunchKernelGGL((D == 768 ? ln_fwd_kernel<T, P, 3, 2> : D <= 1024 ? ln_fwd_kernel<T, P, 2> : ln_fwd_kernel<T, P, 4>), grid, block, 0, stream, \
                     reinterpret_cast<const T*>(x.data_ptr()),                                 \
                     reinterpret_cast<const P*>(wt.data_ptr()),                                \
                     reinterpret_cast<const P*>(bt.data_ptr()), rows, (int)D,                  \
                     (float)eps, reinterpret_cast<T*>(y.data_ptr()), mean.data_ptr<float>(),   \
                     rstd.data_ptr<float>())
  if (x.scalar_type() == at::kBFloat16) {
    if (pbf) DMP_LN_FWD(__bf16, __bf16); else DMP_LN_FWD(__bf16, float);
  } else {
    if (pbf) DMP_LN_FWD(float, __bf16); else DMP_LN_FWD(float, float);
  }
#undef DMP_LN_FWD
  return {y, mean, rstd};
}

// Returns (dx, dweight, dbias) -- dweight/dbias in the parameter dtype (fp32 if none).
std::vector<at::Tensor> layernorm_backward(const at::Tensor& dy, const at::Tensor& x,
                                           const c10::optional<at::Tensor>& w,
                                           const at::Tensor& mean, const at::Tensor& rstd,
                                           int64_t D, at::ScalarType param_dtype,
                                           const c10::optional<at::Tensor>& dres) {
  check_ln(x, D, "x");
  check_ln(dy, D, "dy");
  TORCH_CHECK(dy.scalar_type() == x.scalar_type(), "dy/x dtype mismatch");
  TORCH_CHECK(layernorm_supported(D), "layernorm: D must be a multiple of 8 and <= 2048");
  const bool hw = w.has_value() && w->defined();
  const bool hr = dres.has_value() && dres->defined();
  if (hr) {
    check_ln(*dres, D, "dres");
    TORCH_CHECK(dres->scalar_type() == x.scalar_type() && dres->numel() == x.numel(), "bad dres");
  }
  const int64_t rows = x.numel() / D;
  auto dx = at::empty_like(x);
  auto dwb = at::empty({2, D}, x.options().dtype(param_dtype));
  if (rows == 0) return {dx, dwb[0].zero_(), dwb[1].zero_()};
  auto stream = at::hip::getCurrentHIPStream();
  // 4 blocks (16 waves) per CU: enough rows in flight to reach the HBM rate;
  // each block writes one dgamma/dbeta partial row
  const int nb = ln_blocks(rows, 1024);
  auto part = at::empty({nb, 2 * D}, x.options().dtype(at::kFloat));
  const bool pbf = hw && w->scalar_type() == at::kBFloat16;
  const at::Tensor wt = hw ? *w : at::ones({D}, x.options().dtype(at::kFloat));  // see forward
#define DMP_LN_BWD(T, P)                                                                        \
  hipLaunchKernelGGL((D == 768 ? ln_bwd_kernel<T, P, 3, 2> : D <= 1024 ? ln_bwd_kernel<T, P, 2> : ln_bwd_kernel<T, P, 4>), dim3(nb), dim3(kLnThreads), 0, stream, \
                     reinterpret_cast<const T*>(dy.data_ptr()),                                 \
                     reinterpret_cast<const T*>(x.data_ptr()),                                  \
                     reinterpret_cast<const P*>(wt.data_ptr()),                                 \
                     mean.data_ptr<float>(), rstd.data_ptr<float>(), rows, (int)D,               \
                     reinterpret_cast<T*>(dx.data_ptr()), part.data_ptr<float>(),             \
                     hr ? reinterpret_cast<const T*>(dres->data_ptr()) : nullptr)
  if (x.scalar_type() == at::kBFloat16) {
    if (pbf) DMP_LN_BWD(__bf16, __bf16); else DMP_LN_BWD(__bf16, float);
  } else {
    if (pbf) DMP_LN_BWD(float, __bf16); else DMP_LN_BWD(float, float);
  }
#undef DMP_LN_BWD
  const int n = (int)(2 * D);
  if (param_dtype == at::kBFloat16)
    colreduce::launch(part.data_ptr<float>(), nb, n, reinterpret_cast<__bf16*>(dwb.data_ptr()), stream);
  else
    colreduce::launch(part.data_ptr<float>(), nb, n, dwb.data_ptr<float>(), stream);
  return {dx, dwb[0], dwb[1]};
}

}  // namespace dmp
