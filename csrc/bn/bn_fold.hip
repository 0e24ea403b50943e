// Coefficient kernels of the BN fold (distributed_model_parallel_amd/ops/bn_fold.py):
// the small [Cout, Cin] / [Cin, Cin] algebra that turns the Gram matrix
// G = a^T a, colsum(a) and D = dz^T a into BN statistics, the weight gradient
// and the folded data-gradient operand -- two launches per direction instead
// of ~25 tiny framework ops per bottleneck.
//
//   forward   fold_fwd_kernel       WG = W G (fp32), sums = [W s, rowdot(WG, W), M] (fp64)
//   backward  fold_bwd_sums_kernel  local = [sdz, rowdot(D, W) - mean * sdz] (fp64)
//             fold_bwd_coef_kernel  al, be, c per channel from the (all-reduced) sums, then
//                 role A  dW = al o D + be o WG + c (x) s,  Bm[:, :Cout] = (al o W)^T,  dgamma, dbeta
//                 role B  Bm[:, Cout:] = W^T diag(be) W
//                 role C  ebias = c^T W
// W is bf16 [Cout, Cin] with Cin <= 512 (ResNet bottlenecks: 64..512); fp64
// where sums over many rows or channels meet (row dots, coefficients).
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include "../common.h"

namespace dmp {
namespace {

using bf16 = __bf16;
constexpr int kFoldThreads = 256;
constexpr int kFwdRows = 16;     // output channels per forward block
constexpr int kMaxCin = 512;

__device__ __forceinline__ double block_sum_d(double v, double* lds) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) lds[wave] = v;
  __syncthreads();
  double t = 0.0;
  for (int w = 0; w < kFoldThreads / 64; ++w) t += lds[w];
  return t;
}

// grid = Cout / kFwdRows.  Thread t owns columns j = t, t + 256 of WG rows k0..k0+15.
__global__ __launch_bounds__(kFoldThreads) void fold_fwd_kernel(const bf16* __restrict__ W,
                                                                const float* __restrict__ G,
                                                                const double* __restrict__ asums, int Cout,
                                                                int Cin, float* __restrict__ WG,
                                                                double* __restrict__ sums) {
  __shared__ __attribute__((aligned(16))) float wl[kFwdRows][kMaxCin];
  __shared__ double red[kFoldThreads / 64];
  const int tid = threadIdx.x, k0 = blockIdx.x * kFwdRows;
  for (int idx = tid; idx < kFwdRows * Cin; idx += kFoldThreads) {
    const int r = idx / Cin, i = idx - r * Cin;
    wl[r][i] = (float)W[(int64_t)(k0 + r) * Cin + i];
  }
  __syncthreads();
  const int j0 = tid, j1 = tid + kFoldThreads;
  const bool v0 = j0 < Cin, v1 = j1 < Cin;
  float acc0[kFwdRows], acc1[kFwdRows];
#pragma unroll
  for (int r = 0; r < kFwdRows; ++r) acc0[r] = acc1[r] = 0.f;
  for (int i = 0; i < Cin; i += 4) {
    float g0[4], g1[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      g0[u] = v0 ? G[(int64_t)(i + u) * Cin + j0] : 0.f;
      g1[u] = v1 ? G[(int64_t)(i + u) * Cin + j1] : 0.f;
    }
#pragma unroll
    for (int r = 0; r < kFwdRows; ++r) {
      const f32x4 w4 = *reinterpret_cast<const f32x4*>(&wl[r][i]);  // LDS broadcast
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        acc0[r] = fmaf(w4[u], g0[u], acc0[r]);
        acc1[r] = fmaf(w4[u], g1[u], acc1[r]);
      }
    }
  }
  for (int r = 0; r < kFwdRows; ++r) {
    const int k = k0 + r;
    double q = 0.0, m = 0.0;
    if (v0) { WG[(int64_t)k * Cin + j0] = acc0[r]; q += (double)acc0[r] * wl[r][j0]; m += (double)wl[r][j0] * asums[j0]; }
    if (v1) { WG[(int64_t)k * Cin + j1] = acc1[r]; q += (double)acc1[r] * wl[r][j1]; m += (double)wl[r][j1] * asums[j1]; }
    m = block_sum_d(m, red);
    q = block_sum_d(q, red);
    if (tid == 0) {
      sums[k] = m;         // sum_m y[m, k]
      sums[Cout + k] = q;  // sum_m y[m, k]^2
    }
  }
  if (blockIdx.x == 0 && tid == 0) sums[2 * Cout] = asums[2 * Cin];  // rows
}

// One wave per output channel.  local = [sdz, sum dz*(y - mean)].
__global__ __launch_bounds__(kFoldThreads) void fold_bwd_sums_kernel(const float* __restrict__ D,
                                                                     const bf16* __restrict__ W,
                                                                     const double* __restrict__ sdz,
                                                                     const float* __restrict__ mean, int Cout,
                                                                     int Cin, double* __restrict__ local) {
  const int k = blockIdx.x * (kFoldThreads / 64) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (k >= Cout) return;
  double acc = 0.0;
  for (int i = lane; i < Cin; i += 64) acc += (double)D[(int64_t)k * Cin + i] * (double)(float)W[(int64_t)k * Cin + i];
  acc = wave_sum(acc);
  if (lane == 0) {
    local[k] = sdz[k];
    local[Cout + k] = acc - (double)mean[k] * sdz[k];
  }
}

struct FoldBwdArgs {
  const double* sums;   // [2Cout] (all-reduced) sdz, sdzx
  const double* local;  // [2Cout] this rank's, for dgamma / dbeta
  const double* count;  // [1] global rows
  const float *invstd, *mean, *gamma;  // [Cout] (gamma may be null)
  const float *D, *WG;  // [Cout, Cin] fp32
  const double* s;      // [Cin] colsum(a)
  const bf16* W;        // [Cout, Cin]
  bf16* dW;             // [Cout, Cin]
  float *dgamma, *dbeta;
  bf16* Bm;             // [Cin, Cout + Cin]
  float* ebias;         // [Cin]
  int Cout, Cin;
  int nA, nB;           // role A / B block counts (role C: the last block)
};

__device__ __forceinline__ void fold_coef(const FoldBwdArgs& p, int k, double& al, double& be, double& c) {
  const double istd = p.invstd[k];
  const double cnt = p.count[0];
  al = istd * (p.gamma ? (double)p.gamma[k] : 1.0);
  be = -al * istd * istd * p.sums[p.Cout + k] / cnt;
  c = -al * p.sums[k] / cnt - be * (double)p.mean[k];
}

constexpr int kTK = 16, kTI = 64;  // role A tile: 16 channels x 64 input columns
constexpr int kTR = 8;             // role B: Bm rows (input channels i) per block
constexpr int kKC = 64;            // role B: channels staged per LDS round

__global__ __launch_bounds__(kFoldThreads) void fold_bwd_coef_kernel(const FoldBwdArgs p) {
  const int tid = threadIdx.x;
  const int Cout = p.Cout, Cin = p.Cin, LDB = Cout + Cin;
  if ((int)blockIdx.x < p.nA) {
    // ---- role A: 16 x 64 tile of dW and of the transposed (al o W) block of Bm ----
    __shared__ float tr[kTI][kTK + 1];
    const int itiles = Cin / kTI;
    const int k0 = (blockIdx.x / itiles) * kTK, i0 = (blockIdx.x % itiles) * kTI;
    const int il = tid % kTI, rq = tid / kTI;  // rows rq, rq + 4, ...
#pragma unroll
    for (int rr = 0; rr < kTK / 4; ++rr) {
      const int r = rq + rr * 4, k = k0 + r, i = i0 + il;
      double al, be, c;
      fold_coef(p, k, al, be, c);
      const int64_t o = (int64_t)k * Cin + i;
      const double dw = al * (double)p.D[o] + be * (double)p.WG[o] + c * p.s[i];
      p.dW[o] = (bf16)(float)dw;
      tr[il][r] = (float)(al * (double)(float)p.W[o]);
      if (i0 == 0 && il == 0) {
        p.dgamma[k] = (float)(p.local[Cout + k] * (double)p.invstd[k]);
        p.dbeta[k] = (float)p.local[k];
      }
    }
    __syncthreads();
    // Bm[i, k0 .. k0+15]: 4 threads per row, 4 channels each
    const int i = tid / 4, kq = (tid % 4) * 4;
    if (i < kTI) {
#pragma unroll
      for (int u = 0; u < 4; ++u) p.Bm[(int64_t)(i0 + i) * LDB + k0 + kq + u] = (bf16)tr[i][kq + u];
    }
    return;
  }
  if ((int)blockIdx.x < p.nA + p.nB) {
    // ---- role B: rows i0..i0+7 of W^T diag(be) W; thread t owns columns j = t, t + 256 ----
    __shared__ float wb[kKC][kTR];
    const int i0 = (blockIdx.x - p.nA) * kTR;
    const int j0 = tid, j1 = tid + kFoldThreads;
    const bool v0 = j0 < Cin, v1 = j1 < Cin;
    float acc0[kTR], acc1[kTR];
#pragma unroll
    for (int r = 0; r < kTR; ++r) acc0[r] = acc1[r] = 0.f;
    for (int kc = 0; kc < Cout; kc += kKC) {
      __syncthreads();
      for (int idx = tid; idx < kKC * kTR; idx += kFoldThreads) {
        const int kk = idx / kTR, r = idx - kk * kTR, k = kc + kk;
        double al, be, c;
        fold_coef(p, k, al, be, c);
        wb[kk][r] = (float)(be * (double)(float)p.W[(int64_t)k * Cin + i0 + r]);
      }
      __syncthreads();
      for (int kk = 0; kk < kKC; ++kk) {
        const int64_t row = (int64_t)(kc + kk) * Cin;
        const float w0 = v0 ? (float)p.W[row + j0] : 0.f, w1 = v1 ? (float)p.W[row + j1] : 0.f;
#pragma unroll
        for (int r = 0; r < kTR; ++r) {
          acc0[r] = fmaf(wb[kk][r], w0, acc0[r]);
          acc1[r] = fmaf(wb[kk][r], w1, acc1[r]);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < kTR; ++r) {
      if (v0) p.Bm[(int64_t)(i0 + r) * LDB + Cout + j0] = (bf16)acc0[r];
      if (v1) p.Bm[(int64_t)(i0 + r) * LDB + Cout + j1] = (bf16)acc1[r];
    }
    return;
  }
  // ---- role C: ebias = c^T W ----
  for (int i = tid; i < Cin; i += kFoldThreads) {
    double e = 0.0;
    for (int k = 0; k < Cout; ++k) {
      double al, be, c;
      fold_coef(p, k, al, be, c);
      e += c * (double)(float)p.W[(int64_t)k * Cin + i];
    }
    p.ebias[i] = (float)e;
  }
}

void check_f32(const at::Tensor& t, int64_t n, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous() && t.numel() == n, name,
              " must be a contiguous fp32 GPU tensor of ", n, " elements");
}
void check_f64(const at::Tensor& t, int64_t n, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kDouble && t.is_contiguous() && t.numel() >= n, name,
              " must be a contiguous fp64 GPU tensor of >= ", n, " elements");
}
void check_w(const at::Tensor& W) {
  TORCH_CHECK(W.is_cuda() && W.scalar_type() == at::kBFloat16 && W.dim() == 2 && W.is_contiguous(),
              "W must be a contiguous bf16 [Cout, Cin] GPU tensor");
  TORCH_CHECK(W.size(1) % kTI == 0 && W.size(1) <= kMaxCin && W.size(0) % kFwdRows == 0 &&
                  W.size(0) % kKC == 0,
              "bn fold: Cin % 64 == 0, Cin <= 512, Cout % 64 == 0");
}

}  // namespace

bool bn_fold_supported(int64_t cout, int64_t cin) {
  return cin % kTI == 0 && cin <= kMaxCin && cout % kFwdRows == 0 && cout % kKC == 0;
}

// Forward: (sums fp64 [2Cout+1], WG fp32 [Cout, Cin]) from W, G = a^T a and
// asums = (colsum a, colsum a^2, rows) fp64 [2Cin+1].
std::vector<at::Tensor> bn_fold_fwd(const at::Tensor& W, const at::Tensor& G, const at::Tensor& asums) {
  check_w(W);
  const int64_t Cout = W.size(0), Cin = W.size(1);
  check_f32(G, Cin * Cin, "G");
  check_f64(asums, 2 * Cin + 1, "asums");
  auto sums = at::empty({2 * Cout + 1}, W.options().dtype(at::kDouble));
  auto WG = at::empty({Cout, Cin}, W.options().dtype(at::kFloat));
  hipLaunchKernelGGL(fold_fwd_kernel, dim3((unsigned)(Cout / kFwdRows)), dim3(kFoldThreads), 0,
                     at::hip::getCurrentHIPStream(), reinterpret_cast<const bf16*>(W.data_ptr()),
                     G.data_ptr<float>(), asums.data_ptr<double>(), (int)Cout, (int)Cin, WG.data_ptr<float>(),
                     sums.data_ptr<double>());
  DMP_HIP_CHECK(hipGetLastError());
  return {sums, WG};
}

// Backward local sums [sdz, sum dz*(y - mean)] fp64 [2Cout] from D = dz^T a.
at::Tensor bn_fold_bwd_sums(const at::Tensor& D, const at::Tensor& W, const at::Tensor& sdz,
                            const at::Tensor& mean) {
  check_w(W);
  const int64_t Cout = W.size(0), Cin = W.size(1);
  check_f32(D, Cout * Cin, "D");
  check_f64(sdz, Cout, "sdz");
  check_f32(mean, Cout, "mean");
  auto local = at::empty({2 * Cout}, W.options().dtype(at::kDouble));
  hipLaunchKernelGGL(fold_bwd_sums_kernel, dim3((unsigned)((Cout + 3) / 4)), dim3(kFoldThreads), 0,
                     at::hip::getCurrentHIPStream(), D.data_ptr<float>(),
                     reinterpret_cast<const bf16*>(W.data_ptr()), sdz.data_ptr<double>(), mean.data_ptr<float>(),
                     (int)Cout, (int)Cin, local.data_ptr<double>());
  DMP_HIP_CHECK(hipGetLastError());
  return local;
}

// Backward coefficients: (dW bf16 [Cout, Cin], dgamma, dbeta fp32 [Cout],
// Bm bf16 [Cin, Cout + Cin] = [(al o W)^T | W^T diag(be) W], ebias fp32 [Cin]).
std::vector<at::Tensor> bn_fold_bwd_coef(const at::Tensor& sums, const at::Tensor& local, const at::Tensor& count,
                                         const at::Tensor& invstd, const at::Tensor& mean,
                                         const c10::optional<at::Tensor>& gamma, const at::Tensor& D,
                                         const at::Tensor& WG, const at::Tensor& s, const at::Tensor& W) {
  check_w(W);
  const int64_t Cout = W.size(0), Cin = W.size(1);
  check_f64(sums, 2 * Cout, "sums");
  check_f64(local, 2 * Cout, "local");
  check_f64(count, 1, "count");
  check_f32(invstd, Cout, "invstd");
  check_f32(mean, Cout, "mean");
  check_f32(D, Cout * Cin, "D");
  check_f32(WG, Cout * Cin, "WG");
  check_f64(s, Cin, "s");
  const bool hg = gamma.has_value() && gamma->defined();
  if (hg) check_f32(*gamma, Cout, "gamma");
  auto dW = at::empty({Cout, Cin}, W.options());
  auto dgb = at::empty({2, Cout}, W.options().dtype(at::kFloat));
  auto Bm = at::empty({Cin, Cout + Cin}, W.options());
  auto ebias = at::empty({Cin}, W.options().dtype(at::kFloat));
  FoldBwdArgs p{};
  p.sums = sums.data_ptr<double>(); p.local = local.data_ptr<double>(); p.count = count.data_ptr<double>();
  p.invstd = invstd.data_ptr<float>(); p.mean = mean.data_ptr<float>();
  p.gamma = hg ? gamma->data_ptr<float>() : nullptr;
  p.D = D.data_ptr<float>(); p.WG = WG.data_ptr<float>(); p.s = s.data_ptr<double>();
  p.W = reinterpret_cast<const bf16*>(W.data_ptr());
  p.dW = reinterpret_cast<bf16*>(dW.data_ptr());
  p.dgamma = dgb.data_ptr<float>(); p.dbeta = p.dgamma + Cout;
  p.Bm = reinterpret_cast<bf16*>(Bm.data_ptr());
  p.ebias = ebias.data_ptr<float>();
  p.Cout = (int)Cout; p.Cin = (int)Cin;
  p.nA = (int)((Cout / kTK) * (Cin / kTI));
  p.nB = (int)(Cin / kTR);
  hipLaunchKernelGGL(fold_bwd_coef_kernel, dim3((unsigned)(p.nA + p.nB + 1)), dim3(kFoldThreads), 0,
                     at::hip::getCurrentHIPStream(), p);
  DMP_HIP_CHECK(hipGetLastError());
  return {dW, dgb[0], dgb[1], Bm, ebias};
}

}  // namespace dmp
