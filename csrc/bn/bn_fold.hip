// Coefficient kernels of the BN fold (distributed_model_parallel_amd/ops/bn_fold.py):
// the small [Cout, Cin] / [Cin, Cin] algebra that turns the Gram matrix
// G = a^T a, colsum(a) and D = dz^T a into BN statistics, the weight gradient
// and the folded data-gradient operand -- two launches per direction instead
// of ~25 tiny framework ops per bottleneck.
//
//   forward   fold_fwd_kernel       WG = W G (fp32), sums = [W s, rowdot(WG, W), M] (fp64)
//   backward  fold_bwd_sums_kernel  local = [sdz, rowdot(D, W) - mean * sdz] (fp64)
//             fold_coef_kernel      al, be, c per channel from the (all-reduced) sums
//             fold_bwd_coef_kernel  role A  dW = al o D + be o WG + c (x) s,  Bm[:, :Cout] = (al o W)^T,
//                                           dgamma, dbeta
//                                   role B  Bm[:, Cout:] = W^T diag(be) W, ebias = c^T W
// W is bf16 [Cout, Cin] with Cin <= 1024 (ResNet: 64..1024); fp64
// where sums over many rows or channels meet (row dots, coefficients).
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include "../common.h"

namespace dmp {

void bn_reduce_partials_launch(const float* part, int rb, int C, double* sums, double count,
                               hipStream_t stream);

namespace {

using bf16 = __bf16;
constexpr int kFoldThreads = 256;
constexpr int kFwdRows = 8;      // output channels per forward block (2 blocks / CU)
constexpr int kMaxCin = 1024;
// How the two [Cout x Cin x Cin] / [Cin x Cin x Cout] products of the fold
// (W G forward, W^T diag(be) W and c^T W backward) run:
//   0  the fused VALU kernels (fold_fwd_kernel, role B of fold_bwd_coef_kernel):
//      one block per CU, ~8 TF/s, 2.4 ms of a 23 ms batch-256 ResNet-50 step
//      (the algebra does not shrink with the batch);
//   1  library fp32 GEMMs (hipBLASLt): fast kernels, but 30-280 us of host
//      time per call stalls the launch-bound batch-256 forward;
//   2  fold_sgemm_kernel: a 64 x 64-tiled fp32 GEMM reading W (bf16) and G /
//      the coefficients directly (no fp32 copies, no concatenated operand),
//      with the backward's epilogue writing Bm's bf16 block and ebias in place.
//      On fp32 MFMAs since round 6 (VALU before).
// Default 1: batch-256 step 22.0 ms (1) vs 23.3 (0) vs 24.3 (2, VALU), round 4
// (profiles/raw_r4/fold_gemm_ab_r4i.md); round 6 with the MFMA form of 2:
// 20.67 (1) vs 21.03 (2) at batch 256, 113.77 vs 114.16 at 2048
// (tools/fold_gemm_ab.py): its 16-deep K stages leave the few blocks of these
// small products waiting on load round trips (29 / 23 us per call).
int g_fold_gemm = 1;

// grid = Cout / kFwdRows.  Thread t owns columns j = t + 256 q (q < NQ) of WG rows
// k0..k0+7; G streams through LDS in 4-row chunks (double buffered), so the
// FMAs read LDS instead of waiting on L2 per row of G.
template <int NQ>
__global__ __launch_bounds__(kFoldThreads, 2) void fold_fwd_kernel(const bf16* __restrict__ W,
                                                                const float* __restrict__ G,
                                                                const double* __restrict__ asums, int Cout,
                                                                int Cin, float* __restrict__ WG,
                                                                double* __restrict__ sums) {
  constexpr int GR = 4;  // rows of G per LDS chunk
  __shared__ __attribute__((aligned(16))) float wl[kFwdRows][NQ * kFoldThreads];
  __shared__ __attribute__((aligned(16))) float gl[2][GR][NQ * kFoldThreads];
  __shared__ double red[2][kFoldThreads / 64][kFwdRows];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, k0 = blockIdx.x * kFwdRows;
  for (int idx = tid; idx < kFwdRows * Cin; idx += kFoldThreads) {
    const int r = idx / Cin, i = idx - r * Cin;
    wl[r][i] = (float)W[(int64_t)(k0 + r) * Cin + i];
  }
  auto stage = [&](int i0, int buf) {  // G rows i0..i0+7 -> gl[buf] (16-B vectors)
    const int nv = GR * Cin / 4;
    for (int v = tid; v < nv; v += kFoldThreads) {
      const int r = v / (Cin / 4), c = (v - r * (Cin / 4)) * 4;
      *reinterpret_cast<f32x4*>(&gl[buf][r][c]) = *reinterpret_cast<const f32x4*>(G + (int64_t)(i0 + r) * Cin + c);
    }
  };
  float acc[kFwdRows][NQ];
#pragma unroll
  for (int r = 0; r < kFwdRows; ++r)
#pragma unroll
    for (int q = 0; q < NQ; ++q) acc[r][q] = 0.f;
  stage(0, 0);
  __syncthreads();
  for (int i0 = 0; i0 < Cin; i0 += GR) {
    const int buf = (i0 / GR) & 1;
    if (i0 + GR < Cin) stage(i0 + GR, buf ^ 1);
#pragma unroll
    for (int u = 0; u < GR; u += 4) {
      float g[4][NQ];
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int q = 0; q < NQ; ++q) g[e][q] = gl[buf][u + e][tid + q * kFoldThreads];
#pragma unroll
      for (int r = 0; r < kFwdRows; ++r) {
        const f32x4 w4 = *reinterpret_cast<const f32x4*>(&wl[r][i0 + u]);  // LDS broadcast
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int q = 0; q < NQ; ++q) acc[r][q] = fmaf(w4[e], g[e][q], acc[r][q]);
      }
    }
    __syncthreads();
  }
  // WG and this thread's share of the two row dots, one wave reduction each,
  // one LDS exchange for the whole block
#pragma unroll
  for (int r = 0; r < kFwdRows; ++r) {
    double qd = 0.0, md = 0.0;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int j = tid + q * kFoldThreads;
      if (j < Cin) {
        WG[(int64_t)(k0 + r) * Cin + j] = acc[r][q];
        qd += (double)acc[r][q] * wl[r][j];
        md += (double)wl[r][j] * asums[j];
      }
    }
    qd = wave_sum(qd);
    md = wave_sum(md);
    if (lane == 0) { red[0][wave][r] = md; red[1][wave][r] = qd; }
  }
  __syncthreads();
  if (tid < 2 * kFwdRows) {
    const int which = tid / kFwdRows, r = tid % kFwdRows;
    double t = 0.0;
#pragma unroll
    for (int w = 0; w < kFoldThreads / 64; ++w) t += red[which][w][r];
    sums[which * Cout + k0 + r] = t;  // sum_m y[m, k] | sum_m y[m, k]^2
  }
  if (blockIdx.x == 0 && tid == 0) sums[2 * Cout] = asums[2 * Cin];  // rows
}

// ---- fold_sgemm_kernel: C[m][n] = sum_k A(m, k) B(k, n), fp32 accumulation ----
// 64 x 64 tile per 256-thread block on fp32 MFMAs (four waves, 32 x 32 each),
// K staged through LDS 16 at a time (register-prefetched one chunk ahead; 64-deep
// stages measured slower in-step: 21.35 vs 21.03 ms at batch 256).
//   FWD: A(m, k) = W[m][k] (bf16 [Cout, Cin]), B(k, n) = G[k][n] (fp32 [Cin, Cin]);
//        C = WG fp32 [Cout, Cin]
//   BWD: A(m, k) = be[k] W[k][m] for m < Cin, c[k] for m == Cin (the rows of
//        [W^T diag(be) ; c^T], built on load from W and the coefficients),
//        B(k, n) = W[k][n]; rows m < Cin go to Bm[m][Cout + n] (bf16), row Cin
//        to ebias[n]  (W^T diag(be) W is symmetric: its rows are Bm's columns)
constexpr int kSgT = 64, kSgK = 16, kSgU = kSgT * kSgK / kFoldThreads;  // elements per thread per operand
// BWD splits K (= Cout, up to 2048, while M x N = Cin^2 is small) over
// gridDim.z: split z writes its fp32 partials to C[z] ([Cin][Cin] rows) and
// ebias[z] ([Cin]), summed into Bm / ebias by fold_bwd_reduce_kernel.
template <bool BWD>
__global__ __launch_bounds__(kFoldThreads) void fold_sgemm_kernel(const bf16* __restrict__ W,
                                                                  const float* __restrict__ G,
                                                                  const float* __restrict__ be,
                                                                  const float* __restrict__ cc, int M, int N,
                                                                  int K, float* __restrict__ C,
                                                                  bf16* __restrict__ Bm, int ldbm, int bm_off,
                                                                  float* __restrict__ ebias) {
  const int kchunk = K / gridDim.z, kbeg = blockIdx.z * kchunk, kend = kbeg + kchunk;
  if constexpr (BWD) {
    C += (int64_t)blockIdx.z * N * N;
    ebias += (int64_t)blockIdx.z * N;
  }
  __shared__ __attribute__((aligned(16))) float As[kSgK][kSgT + 4];
  __shared__ __attribute__((aligned(16))) float Bs[kSgK][kSgT + 4];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int m0 = blockIdx.y * kSgT, n0 = blockIdx.x * kSgT;
  // loaders: A as [kk][m], B as [kk][n] (kSgU elements each per thread)
  float ra[kSgU], rb[kSgU];
  auto load = [&](int k0) {
#pragma unroll
    for (int u = 0; u < kSgU; ++u) {
      const int e = tid + u * kFoldThreads;  // 0 .. kSgT * kSgK - 1
      if constexpr (BWD) {
        const int kk = e / kSgT, m = e % kSgT, k = k0 + kk, mm = m0 + m;  // coalesced along m
        float v = 0.f;
        if (k < kend) v = mm < N ? be[k] * (float)W[(int64_t)k * N + mm] : (mm == N ? cc[k] : 0.f);
        ra[u] = v;
      } else {
        const int m = e / kSgK, kk = e % kSgK, k = k0 + kk, mm = m0 + m;  // kSgK consecutive k per row
        ra[u] = (mm < M && k < kend) ? (float)W[(int64_t)mm * K + k] : 0.f;
      }
      const int kk = e / kSgT, n = e % kSgT, k = k0 + kk;
      if constexpr (BWD) rb[u] = k < kend ? (float)W[(int64_t)k * N + n0 + n] : 0.f;
      else rb[u] = k < kend ? G[(int64_t)k * N + n0 + n] : 0.f;
    }
  };
  auto store = [&] {
#pragma unroll
    for (int u = 0; u < kSgU; ++u) {
      const int e = tid + u * kFoldThreads;
      if constexpr (BWD) As[e / kSgT][e % kSgT] = ra[u];
      else As[e % kSgK][e / kSgK] = ra[u];
      Bs[e / kSgT][e % kSgT] = rb[u];
    }
  };
  // fp32 MFMA (v_mfma_f32_16x16x4_f32): wave w owns the 32 x 32 quadrant
  // (w >> 1, w & 1) as 2 x 2 16x16 blocks; per k4 step lane l feeds A(row
  // l & 15, k l >> 4) and B(k l >> 4, col l & 15) from the LDS stage and gets
  // back rows 4 (l >> 4) + v, column l & 15 of each block.
  (void)tx; (void)ty;
  const int lane = tid & 63, wave = tid >> 6, wr = wave >> 1, wc = wave & 1;
  const int lr = lane & 15, lk = lane >> 4;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  load(kbeg);
  for (int k0 = kbeg; k0 < kend; k0 += kSgK) {
    __syncthreads();
    store();
    __syncthreads();
    if (k0 + kSgK < kend) load(k0 + kSgK);  // next chunk in flight during this one's MFMAs
#pragma unroll
    for (int s4 = 0; s4 < kSgK; s4 += 4) {
      const int kk = s4 + lk;
      float a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = As[kk][wr * 32 + i * 16 + lr];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = Bs[kk][wc * 32 + j * 16 + lr];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int m = m0 + wr * 32 + i * 16 + 4 * lk + v;
      if (m >= M) continue;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = n0 + wc * 32 + j * 16 + lr;
        if constexpr (BWD) {
          float* dst = m < N ? C + (int64_t)m * N + n : ebias + n;
          *dst = acc[i][j][v];
        } else {
          C[(int64_t)m * N + n] = acc[i][j][v];
        }
      }
    }
}

// Forward row sums from WG = W G (fold_gemm modes 1, 2): one wave per
// output channel, sums = [W s, rowdot(WG, W)] in fp64, plus the row count.
// Finalize fused in (FoldFin set, no cross-rank moment reduce in between):
// the same per-channel coefficients as batchnorm.hip's bn_finalize_kernel
// (coef = [scale, shift, mean, invstd] x Cout, running statistics and the
// step counter) from the moments this wave just formed -- one launch fewer
// per folded BN.
struct FoldFin {
  const float *w, *b;
  float *rm, *rv, *coef;
  int64_t* nbt;
  float momentum, eps;
};

__global__ __launch_bounds__(kFoldThreads) void fold_fwd_sums_kernel(const bf16* __restrict__ W,
                                                                     const float* __restrict__ WG,
                                                                     const double* __restrict__ asums, int Cout,
                                                                     int Cin, double* __restrict__ sums,
                                                                     FoldFin fin) {
  const int k = blockIdx.x * (kFoldThreads / 64) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (k >= Cout) return;
  double qd = 0.0, md = 0.0;
  for (int i = lane; i < Cin; i += 64) {
    const double w = (double)(float)W[(int64_t)k * Cin + i];
    qd += (double)WG[(int64_t)k * Cin + i] * w;
    md += w * asums[i];
  }
  qd = wave_sum(qd);
  md = wave_sum(md);
  if (lane == 0) {
    const double n = asums[2 * Cin];  // rows
    sums[k] = md;          // sum_m y[m, k]
    sums[Cout + k] = qd;   // sum_m y[m, k]^2
    if (k == 0) sums[2 * Cout] = n;
    if (fin.coef) {
      const double m = md / n;
      double v = qd / n - m * m;
      v = v < 0.0 ? 0.0 : v;
      const float mean = (float)m, var_b = (float)v, invstd = (float)(1.0 / sqrt(v + (double)fin.eps));
      const float ww = fin.w ? fin.w[k] : 1.f, bb = fin.b ? fin.b[k] : 0.f;
      const float sc = ww * invstd;
      fin.coef[k] = sc;
      fin.coef[Cout + k] = bb - mean * sc;
      fin.coef[2 * Cout + k] = mean;
      fin.coef[3 * Cout + k] = invstd;
      if (fin.rm) {
        const float unb = n > 1.0 ? (float)((double)var_b * n / (n - 1.0)) : var_b;
        fin.rm[k] = (1.f - fin.momentum) * fin.rm[k] + fin.momentum * mean;
        fin.rv[k] = (1.f - fin.momentum) * fin.rv[k] + fin.momentum * unb;
      }
      if (fin.nbt && k == 0) *fin.nbt += 1;
    }
  }
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
  const double* local;  // [2Cout] this rank's sums, for dgamma / dbeta
  const float* coef;    // [3, Cout] al, be, c (fold_coef_kernel)
  const float* invstd;  // [Cout]
  const float *D, *WG;  // [Cout, Cin] fp32
  const double* s;      // [2Cin+1] (colsum a, colsum a^2, local rows) of a
  const bf16* W;        // [Cout, Cin]
  bf16* dW;             // [Cout, Cin]
  float *dgamma, *dbeta;
  bf16* Bm;             // [Cin, Cout + Cin]
  float* ebias;         // [Cin]
  int Cout, Cin;
  int nA;               // role A blocks; the rest are role B
  int ksplit;           // role B: channel (K) range split over this many blocks per row group
  float* bpart;         // role B partials [ksplit][Cin][Cin]
  float* epart;         // role B ebias partials [ksplit][Cin]
  float* Wf;            // fold_gemm 1: fp32 copy of W [Cout, Cin] (role A writes it)
  float* R;             // fold_gemm 1: [Cout, Cin + 1] = [be o W | c] (role A writes it)
};

// al, be, c per output channel from the (all-reduced) backward sums -- once,
// so the role kernels never repeat the fp64 divisions.
__global__ __launch_bounds__(kFoldThreads) void fold_coef_kernel(const double* __restrict__ sums,
                                                                 const double* __restrict__ count,
                                                                 const float* __restrict__ invstd,
                                                                 const float* __restrict__ mean,
                                                                 const float* __restrict__ gamma, int Cout,
                                                                 float* __restrict__ coef) {
  const int k = blockIdx.x * kFoldThreads + threadIdx.x;
  if (k >= Cout) return;
  const double rc = 1.0 / count[0];
  const double istd = invstd[k];
  const double al = istd * (gamma ? (double)gamma[k] : 1.0);
  const double be = -al * istd * istd * sums[Cout + k] * rc;
  const double c = -al * sums[k] * rc - be * (double)mean[k];
  coef[k] = (float)al;
  coef[Cout + k] = (float)be;
  coef[2 * Cout + k] = (float)c;
}

constexpr int kTK = 16, kTI = 64;  // role A tile: 16 channels x 64 input columns
constexpr int kTR = 8;             // role B: Bm rows (input channels i) per block (+1: ebias)
constexpr int kKC = 32;            // role B: channels staged per LDS round

template <int NQ>
__global__ __launch_bounds__(kFoldThreads) void fold_bwd_coef_kernel(const FoldBwdArgs p) {
  const int tid = threadIdx.x;
  const int Cout = p.Cout, Cin = p.Cin, LDB = Cout + Cin;
  const float* al_ = p.coef;
  const float* be_ = p.coef + Cout;
  const float* c_ = p.coef + 2 * Cout;
  if ((int)blockIdx.x < p.nA) {
    // ---- role A: 16 x 64 tile of dW and of the transposed (al o W) block of Bm ----
    __shared__ float tr[kTI][kTK + 1];
    const int itiles = Cin / kTI;
    const int k0 = (blockIdx.x / itiles) * kTK, i0 = (blockIdx.x % itiles) * kTI;
    const int il = tid % kTI, rq = tid / kTI;  // rows rq, rq + 4, ...
#pragma unroll
    for (int rr = 0; rr < kTK / 4; ++rr) {
      const int r = rq + rr * 4, k = k0 + r, i = i0 + il;
      const float al = al_[k], be = be_[k], c = c_[k];
      const int64_t o = (int64_t)k * Cin + i;
      const float dw = fmaf(al, p.D[o], fmaf(be, p.WG[o], (float)((double)c * p.s[i])));
      p.dW[o] = (bf16)dw;
      const float w = (float)p.W[o];
      tr[il][r] = al * w;
      if (p.R) {  // operands of the library product [W^T diag(be) W ; c^T W] = [be o W | c]^T W
        p.Wf[o] = w;
        p.R[(int64_t)k * (Cin + 1) + i] = be * w;
        if (i == Cin - 1) p.R[(int64_t)k * (Cin + 1) + Cin] = c;
      }
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
  // ---- role B: rows i0..i0+7 of B = W^T diag(be) W; thread t owns columns
  // j = t + 256 q.  W rows of a channel chunk are staged in LDS as fp32 with
  // the per-row factors applied.  ebias for the block's rows: c^T W[:, i].
  __shared__ __attribute__((aligned(16))) float wj[kKC][NQ * kFoldThreads];
  __shared__ float wb[kKC][kTR];
  __shared__ float rsum[kFoldThreads / 64][kTR];
  const int rb = blockIdx.x - p.nA, rgroups = Cin / kTR;
  const int i0 = (rb % rgroups) * kTR, ks = rb / rgroups;
  const int kchunk = Cout / p.ksplit, kbeg = ks * kchunk, kend = kbeg + kchunk;
  const int lane = tid & 63, wave = tid >> 6;
  float acc[kTR][NQ];
#pragma unroll
  for (int r = 0; r < kTR; ++r)
#pragma unroll
    for (int q = 0; q < NQ; ++q) acc[r][q] = 0.f;
  for (int kc = kbeg; kc < kend; kc += kKC) {
    __syncthreads();
    for (int v = tid; v < kKC * Cin / 8; v += kFoldThreads) {  // 16-B bf16 vectors
      const int kk = v / (Cin / 8), c = (v - kk * (Cin / 8)) * 8;
      const bf16x8 w8 = *reinterpret_cast<const bf16x8*>(p.W + (int64_t)(kc + kk) * Cin + c);
      const f32x8 f = __builtin_convertvector(w8, f32x8);
#pragma unroll
      for (int e = 0; e < 8; ++e) wj[kk][c + e] = f[e];
    }
    for (int idx = tid; idx < kKC * kTR; idx += kFoldThreads) {
      const int kk = idx / kTR, r = idx - kk * kTR, k = kc + kk;
      wb[kk][r] = be_[k] * (float)p.W[(int64_t)k * Cin + i0 + r];
    }
    __syncthreads();
#pragma unroll 4
    for (int kk = 0; kk < kKC; ++kk) {
      float w[NQ];
#pragma unroll
      for (int q = 0; q < NQ; ++q) w[q] = wj[kk][tid + q * kFoldThreads];
#pragma unroll
      for (int r = 0; r < kTR; ++r)
#pragma unroll
        for (int q = 0; q < NQ; ++q) acc[r][q] = fmaf(wb[kk][r], w[q], acc[r][q]);
    }
  }
  // this channel range's partial rows of B, and its share of ebias = c^T W[:, i]
  float* bp = p.bpart + (int64_t)ks * Cin * Cin;
  float part[kTR];
#pragma unroll
  for (int r = 0; r < kTR; ++r) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int j = tid + q * kFoldThreads;
      if (j < Cin) bp[(int64_t)(i0 + r) * Cin + j] = acc[r][q];
    }
    float e = 0.f;
    for (int k = kbeg + tid; k < kend; k += kFoldThreads) e = fmaf(c_[k], (float)p.W[(int64_t)k * Cin + i0 + r], e);
    part[r] = e;
  }
#pragma unroll
  for (int r = 0; r < kTR; ++r) {
    const float v = wave_sum(part[r]);
    if (lane == 0) rsum[wave][r] = v;
  }
  __syncthreads();
  if (tid < kTR) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < kFoldThreads / 64; ++w) t += rsum[w][tid];
    p.epart[(int64_t)ks * Cin + i0 + tid] = t;
  }
}

// Sum role B's channel-split partials: Bm[:, Cout:] = bf16(sum_s part[s]), ebias = sum_s epart[s].
__global__ __launch_bounds__(kFoldThreads) void fold_bwd_reduce_kernel(const float* __restrict__ bpart,
                                                                       const float* __restrict__ epart, int ksplit,
                                                                       int Cout, int Cin, bf16* __restrict__ Bm,
                                                                       float* __restrict__ ebias) {
  const int64_t n = (int64_t)Cin * Cin;
  for (int64_t v = (int64_t)blockIdx.x * kFoldThreads + threadIdx.x; v < n + Cin;
       v += (int64_t)gridDim.x * kFoldThreads) {
    if (v < n) {
      float t = 0.f;
      for (int s = 0; s < ksplit; ++s) t += bpart[(int64_t)s * n + v];
      const int i = (int)(v / Cin), j = (int)(v - (int64_t)i * Cin);
      Bm[(int64_t)i * (Cout + Cin) + Cout + j] = (bf16)t;
    } else {
      const int i = (int)(v - n);
      float t = 0.f;
      for (int s = 0; s < ksplit; ++s) t += epart[(int64_t)s * Cin + i];
      ebias[i] = t;
    }
  }
}

// Column sums and sums of squares of the rows of x [N*Hi*Wi, C] sampled at
// stride s ((n, oh*s, ow*s) for the N*Ho*Wo logical rows; s = 1: every row):
// the colsum a folded downsample's BN statistics need, per-block partials
// [2][blocks][C] reduced deterministically by bn_reduce_partials_launch.
// grid = (row blocks); 256 threads = (256 / cv) row lanes x cv channel vectors.
// MASK: x is dL/dout of a ReLU output y; the pass writes dz = [y > 0] dL/dout
// to out and reduces dz (the fold's backward when no consumer epilogue did it).
template <bool MASK>
__global__ __launch_bounds__(kFoldThreads) void fold_colsum_kernel(const bf16* __restrict__ x, int C, int64_t M,
                                                                   int s, int ho, int wo, int hi, int wi,
                                                                   int64_t rows_per_block, float* __restrict__ part,
                                                                   double* __restrict__ zsums,
                                                                   const bf16* __restrict__ y = nullptr,
                                                                   bf16* __restrict__ out = nullptr) {
  zero_moments(zsums, 2 * C);
  __shared__ float ls[kFoldThreads * 8], lq[kFoldThreads * 8];
  const int cv = C / 8, rpi = kFoldThreads / cv;
  const int tid = threadIdx.x, lc = tid % cv, lr = tid / cv;
  float su[8], sq[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) su[e] = sq[e] = 0.f;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block, r1 = min(M, r0 + rows_per_block);
  if (lr < rpi) {
    for (int64_t m = r0 + lr; m < r1; m += rpi) {
      int64_t pm = m;
      if (s != 1) {
        const int64_t hw = (int64_t)ho * wo;
        const int64_t n = m / hw;
        const int r = (int)(m - n * hw), oh = r / wo, ow = r - oh * wo;
        pm = (n * hi + (int64_t)oh * s) * wi + (int64_t)ow * s;
      }
      f32x8 f = __builtin_convertvector(*reinterpret_cast<const bf16x8*>(x + pm * C + lc * 8), f32x8);
      if constexpr (MASK) {
        const bf16x8 yv = *reinterpret_cast<const bf16x8*>(y + pm * C + lc * 8);
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = (float)yv[e] > 0.f ? f[e] : 0.f;
        *reinterpret_cast<bf16x8*>(out + pm * C + lc * 8) = __builtin_convertvector(f, bf16x8);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) { su[e] += f[e]; sq[e] = fmaf(f[e], f[e], sq[e]); }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) { ls[e * kFoldThreads + tid] = su[e]; lq[e * kFoldThreads + tid] = sq[e]; }
  __syncthreads();
  for (int o = tid; o < C; o += kFoldThreads) {
    const int c_l = o / 8, e = o % 8;
    float a = 0.f, b = 0.f;
    for (int r = 0; r < rpi; ++r) {
      a += ls[e * kFoldThreads + r * cv + c_l];
      b += lq[e * kFoldThreads + r * cv + c_l];
    }
    part[(int64_t)blockIdx.x * C + o] = a;
    part[(int64_t)(gridDim.x + blockIdx.x) * C + o] = b;
  }
}

// Bf = [s3 o W3 | sd o Wd] (bf16 [Cout, C3 + Cd]) and shift = t3 + td: the
// operand and epilogue constant of a bottleneck whose bn3 and downsample BN
// are both folded into one GEMM over [a | x_s].
__global__ __launch_bounds__(kFoldThreads) void fold_scale_concat_kernel(
    const bf16* __restrict__ W3, const float* __restrict__ s3, const float* __restrict__ t3, int C3,
    const bf16* __restrict__ Wd, const float* __restrict__ sd, const float* __restrict__ td, int Cd, int Cout,
    bf16* __restrict__ Bf, float* __restrict__ shift) {
  const int ld = C3 + Cd;
  const int64_t n = (int64_t)Cout * ld;
  for (int64_t v = (int64_t)blockIdx.x * kFoldThreads + threadIdx.x; v < n; v += (int64_t)gridDim.x * kFoldThreads) {
    const int k = (int)(v / ld), c = (int)(v - (int64_t)k * ld);
    const float w = c < C3 ? s3[k] * (float)W3[(int64_t)k * C3 + c] : sd[k] * (float)Wd[(int64_t)k * Cd + c - C3];
    Bf[v] = (bf16)w;
    if (c == 0) shift[k] = t3[k] + td[k];
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
              "bn fold: Cin % 64 == 0, Cin <= 1024, Cout % 64 == 0");
}

}  // namespace

bool bn_fold_supported(int64_t cout, int64_t cin) {
  return cin % kTI == 0 && cin <= kMaxCin && cout % kFwdRows == 0 && cout % kKC == 0;
}

// Forward: (sums fp64 [2Cout+1], WG fp32 [Cout, Cin]) from W, G = a^T a and
// asums = (colsum a, colsum a^2, rows) fp64 [2Cin+1].
// Wf (optional): fp32 W, e.g. the copy the optimizer keeps (ops/wt_cache.py),
// read by the library product instead of a cast per call (fold_gemm mode 1)
namespace {
std::vector<at::Tensor> fold_fwd_impl(const at::Tensor& W, const at::Tensor& G, const at::Tensor& asums,
                                      const c10::optional<at::Tensor>& Wf, const FoldFin& fin) {
  check_w(W);
  const int64_t Cout = W.size(0), Cin = W.size(1);
  check_f32(G, Cin * Cin, "G");
  check_f64(asums, 2 * Cin + 1, "asums");
  auto sums = at::empty({2 * Cout + 1}, W.options().dtype(at::kDouble));
  if (g_fold_gemm == 2) {
    auto WG = at::empty({Cout, Cin}, W.options().dtype(at::kFloat));
    hipStream_t stream = at::hip::getCurrentHIPStream();
    hipLaunchKernelGGL(fold_sgemm_kernel<false>, dim3((unsigned)(Cin / kSgT), (unsigned)((Cout + kSgT - 1) / kSgT)),
                       dim3(kFoldThreads), 0, stream, reinterpret_cast<const bf16*>(W.data_ptr()), G.data_ptr<float>(),
                       nullptr, nullptr, (int)Cout, (int)Cin, (int)Cin, WG.data_ptr<float>(), nullptr, 0, 0, nullptr);
    hipLaunchKernelGGL(fold_fwd_sums_kernel, dim3((unsigned)((Cout + 3) / 4)), dim3(kFoldThreads), 0, stream,
                       reinterpret_cast<const bf16*>(W.data_ptr()), WG.data_ptr<float>(), asums.data_ptr<double>(),
                       (int)Cout, (int)Cin, sums.data_ptr<double>(), fin);
    DMP_HIP_CHECK(hipGetLastError());
    return {sums, WG};
  }
  if (g_fold_gemm == 1) {
    const bool cached = Wf.has_value() && Wf->defined();
    if (cached)
      TORCH_CHECK(Wf->scalar_type() == at::kFloat && Wf->numel() == Cout * Cin && Wf->is_contiguous() &&
                      Wf->device() == W.device(), "bn_fold_fwd: Wf must be a contiguous fp32 [Cout, Cin]");
    auto WG = at::mm(cached ? Wf->view({Cout, Cin}) : W.to(at::kFloat), G.view({Cin, Cin}));
    hipLaunchKernelGGL(fold_fwd_sums_kernel, dim3((unsigned)((Cout + 3) / 4)), dim3(kFoldThreads), 0,
                       at::hip::getCurrentHIPStream(), reinterpret_cast<const bf16*>(W.data_ptr()),
                       WG.data_ptr<float>(), asums.data_ptr<double>(), (int)Cout, (int)Cin, sums.data_ptr<double>(),
                       fin);
    DMP_HIP_CHECK(hipGetLastError());
    return {sums, WG};
  }
  auto WG = at::empty({Cout, Cin}, W.options().dtype(at::kFloat));
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3((unsigned)(Cout / kFwdRows)), dim3(kFoldThreads), 0,
                       at::hip::getCurrentHIPStream(), reinterpret_cast<const bf16*>(W.data_ptr()),
                       G.data_ptr<float>(), asums.data_ptr<double>(), (int)Cout, (int)Cin, WG.data_ptr<float>(),
                       sums.data_ptr<double>());
  };
  if (Cin <= 256) go(fold_fwd_kernel<1>);
  else if (Cin <= 512) go(fold_fwd_kernel<2>);
  else go(fold_fwd_kernel<4>);
  DMP_HIP_CHECK(hipGetLastError());
  return {sums, WG};
}
}  // namespace

std::vector<at::Tensor> bn_fold_fwd(const at::Tensor& W, const at::Tensor& G, const at::Tensor& asums,
                                    const c10::optional<at::Tensor>& Wf) {
  return fold_fwd_impl(W, G, asums, Wf, FoldFin{});
}

// bn_fold_fwd plus the BN finalize of its moments in the same launch (fold_gemm
// modes 1 / 2; no cross-rank moment reduce may sit in between): returns (sums,
// WG, coef [4, Cout] = scale, shift, mean, invstd), updates the running
// statistics and num_batches_tracked as bn_finalize does.
std::vector<at::Tensor> bn_fold_fwd_finalize(const at::Tensor& W, const at::Tensor& G, const at::Tensor& asums,
                                             const c10::optional<at::Tensor>& Wf,
                                             const c10::optional<at::Tensor>& weight,
                                             const c10::optional<at::Tensor>& bias,
                                             const c10::optional<at::Tensor>& running_mean,
                                             const c10::optional<at::Tensor>& running_var, double momentum,
                                             double eps, const c10::optional<at::Tensor>& num_batches_tracked) {
  const int64_t Cout = W.size(0);
  TORCH_CHECK(g_fold_gemm == 1 || g_fold_gemm == 2, "bn_fold_fwd_finalize: fold_gemm modes 1 / 2 only");
  auto f32 = [&](const c10::optional<at::Tensor>& t, const char* name) -> float* {
    if (!t.has_value() || !t->defined()) return nullptr;
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous() && t->numel() == Cout, name,
                " must be a contiguous fp32 [Cout] GPU tensor");
    return t->data_ptr<float>();
  };
  auto coef = at::empty({4, Cout}, W.options().dtype(at::kFloat));
  FoldFin fin{};
  fin.w = f32(weight, "weight");
  fin.b = f32(bias, "bias");
  fin.rm = f32(running_mean, "running_mean");
  fin.rv = f32(running_var, "running_var");
  TORCH_CHECK((fin.rm == nullptr) == (fin.rv == nullptr), "running_mean and running_var together");
  fin.coef = coef.data_ptr<float>();
  if (num_batches_tracked.has_value() && num_batches_tracked->defined()) {
    TORCH_CHECK(num_batches_tracked->scalar_type() == at::kLong && num_batches_tracked->numel() == 1,
                "num_batches_tracked must be a 1-element int64 tensor");
    fin.nbt = num_batches_tracked->data_ptr<int64_t>();
  }
  fin.momentum = (float)momentum;
  fin.eps = (float)eps;
  auto r = fold_fwd_impl(W, G, asums, Wf, fin);
  return {r[0], r[1], coef};
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
  check_f64(s, 2 * Cin + 1, "s (asums)");
  const bool hg = gamma.has_value() && gamma->defined();
  if (hg) check_f32(*gamma, Cout, "gamma");
  auto dW = at::empty({Cout, Cin}, W.options());
  auto dgb = at::empty({2, Cout}, W.options().dtype(at::kFloat));
  auto Bm = at::empty({Cin, Cout + Cin}, W.options());
  auto ebias = at::empty({Cin}, W.options().dtype(at::kFloat));
  auto coef = at::empty({3, Cout}, W.options().dtype(at::kFloat));
  hipStream_t stream = at::hip::getCurrentHIPStream();
  hipLaunchKernelGGL(fold_coef_kernel, dim3((unsigned)((Cout + kFoldThreads - 1) / kFoldThreads)),
                     dim3(kFoldThreads), 0, stream, sums.data_ptr<double>(), count.data_ptr<double>(),
                     invstd.data_ptr<float>(), mean.data_ptr<float>(), hg ? gamma->data_ptr<float>() : nullptr,
                     (int)Cout, coef.data_ptr<float>());
  FoldBwdArgs p{};
  p.local = local.data_ptr<double>();
  p.coef = coef.data_ptr<float>();
  p.invstd = invstd.data_ptr<float>();
  p.D = D.data_ptr<float>(); p.WG = WG.data_ptr<float>(); p.s = s.data_ptr<double>();
  p.W = reinterpret_cast<const bf16*>(W.data_ptr());
  p.dW = reinterpret_cast<bf16*>(dW.data_ptr());
  p.dgamma = dgb.data_ptr<float>(); p.dbeta = p.dgamma + Cout;
  p.Bm = reinterpret_cast<bf16*>(Bm.data_ptr());
  p.ebias = ebias.data_ptr<float>();
  p.Cout = (int)Cout; p.Cin = (int)Cin;
  p.nA = (int)((Cout / kTK) * (Cin / kTI));
  if (g_fold_gemm == 2) {
    // role A in the coefficient kernel; [W^T diag(be) W ; c^T W] in the tiled
    // kernel, straight into Bm's second block and ebias
    hipLaunchKernelGGL(fold_bwd_coef_kernel<1>, dim3((unsigned)p.nA), dim3(kFoldThreads), 0, stream, p);
    const int tiles = (int)((Cin / kSgT) * ((Cin + 1 + kSgT - 1) / kSgT));
    int ks = 1;  // split K (= Cout) until ~2 blocks per CU, chunks of >= 64 channels
    while (tiles * ks < 512 && Cout % (2 * ks * kSgK) == 0 && Cout / (2 * ks) >= 64) ks *= 2;
    auto bpart = at::empty({ks, Cin, Cin}, W.options().dtype(at::kFloat));
    auto epart = at::empty({ks, Cin}, W.options().dtype(at::kFloat));
    hipLaunchKernelGGL(fold_sgemm_kernel<true>,
                       dim3((unsigned)(Cin / kSgT), (unsigned)((Cin + 1 + kSgT - 1) / kSgT), (unsigned)ks),
                       dim3(kFoldThreads), 0, stream, p.W, nullptr, coef.data_ptr<float>() + Cout,
                       coef.data_ptr<float>() + 2 * Cout, (int)(Cin + 1), (int)Cin, (int)Cout,
                       bpart.data_ptr<float>(), nullptr, 0, 0, epart.data_ptr<float>());
    const int64_t nred = Cin * Cin + Cin;
    hipLaunchKernelGGL(fold_bwd_reduce_kernel,
                       dim3((unsigned)std::min<int64_t>(1024, (nred + kFoldThreads - 1) / kFoldThreads)),
                       dim3(kFoldThreads), 0, stream, bpart.data_ptr<float>(), epart.data_ptr<float>(), ks,
                       (int)Cout, (int)Cin, p.Bm, p.ebias);
    DMP_HIP_CHECK(hipGetLastError());
    return {dW, dgb[0], dgb[1], Bm, ebias};
  }
  if (g_fold_gemm == 1) {
    // role A in the kernel (also writing fp32 W and R = [be o W | c]); role B and
    // ebias as ONE library fp32 product R^T W = [W^T diag(be) W ; c^T W]
    // (W^T diag(be) W is symmetric, so its rows are Bm's columns as they are)
    auto Wf = at::empty({Cout, Cin}, W.options().dtype(at::kFloat));
    auto R = at::empty({Cout, Cin + 1}, W.options().dtype(at::kFloat));
    p.Wf = Wf.data_ptr<float>();
    p.R = R.data_ptr<float>();
    hipLaunchKernelGGL(fold_bwd_coef_kernel<1>, dim3((unsigned)p.nA), dim3(kFoldThreads), 0, stream, p);
    DMP_HIP_CHECK(hipGetLastError());
    const auto out = at::mm(R.t(), Wf);  // [Cin + 1, Cin]
    Bm.narrow(1, Cout, Cin).copy_(out.narrow(0, 0, Cin));
    return {dW, dgb[0], dgb[1], Bm, out.select(0, Cin)};
  }
  // split the channel range until role B has >= 256 blocks (one per CU), chunks of kKC channels
  int ksplit = 1;
  while ((Cin / kTR) * ksplit < 256 && Cout % (2 * ksplit * kKC) == 0) ksplit *= 2;
  p.ksplit = ksplit;
  auto bpart = at::empty({ksplit, Cin, Cin}, W.options().dtype(at::kFloat));
  auto epart = at::empty({ksplit, Cin}, W.options().dtype(at::kFloat));
  p.bpart = bpart.data_ptr<float>();
  p.epart = epart.data_ptr<float>();
  const unsigned blocks = (unsigned)(p.nA + (Cin / kTR) * ksplit);
  if (Cin <= 256) hipLaunchKernelGGL(fold_bwd_coef_kernel<1>, dim3(blocks), dim3(kFoldThreads), 0, stream, p);
  else if (Cin <= 512) hipLaunchKernelGGL(fold_bwd_coef_kernel<2>, dim3(blocks), dim3(kFoldThreads), 0, stream, p);
  else hipLaunchKernelGGL(fold_bwd_coef_kernel<4>, dim3(blocks), dim3(kFoldThreads), 0, stream, p);
  const int64_t nred = Cin * Cin + Cin;
  hipLaunchKernelGGL(fold_bwd_reduce_kernel, dim3((unsigned)std::min<int64_t>(1024, (nred + kFoldThreads - 1) / kFoldThreads)),
                     dim3(kFoldThreads), 0, stream, p.bpart, p.epart, ksplit, (int)Cout, (int)Cin,
                     p.Bm, p.ebias);
  DMP_HIP_CHECK(hipGetLastError());
  return {dW, dgb[0], dgb[1], Bm, ebias};
}

void set_fold_gemm(int mode) {
  TORCH_CHECK(mode >= 0 && mode <= 2, "fold gemm mode: 0 VALU kernels, 1 library, 2 tiled kernel");
  g_fold_gemm = mode;
}
int get_fold_gemm() { return g_fold_gemm; }

// fp64 [2C+1] = (colsum, colsum of squares, rows) of x's rows sampled through
// map [s, Ho, Wo, Hi, Wi] (empty: all rows).
at::Tensor bn_fold_colsum(const at::Tensor& x, const std::vector<int64_t>& map) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 2 && x.is_contiguous(),
              "x must be a contiguous bf16 [rows, C] GPU tensor");
  const int64_t C = x.size(1);
  TORCH_CHECK(C % 8 == 0 && C <= 8 * kFoldThreads, "C % 8 == 0, C <= 2048");
  int s = 1, ho = 1, wo = 1, hi = 1, wi = 1;
  int64_t M = x.size(0);
  if (!map.empty()) {
    TORCH_CHECK(map.size() == 5, "map must be [stride, Ho, Wo, Hi, Wi]");
    s = (int)map[0]; ho = (int)map[1]; wo = (int)map[2]; hi = (int)map[3]; wi = (int)map[4];
    TORCH_CHECK(x.size(0) % ((int64_t)hi * wi) == 0 && (ho - 1) * s < hi && (wo - 1) * s < wi, "bad map");
    M = x.size(0) / ((int64_t)hi * wi) * ho * wo;
  }
  auto sums = at::empty({2 * C + 1}, x.options().dtype(at::kDouble));
  if (M == 0) return sums.zero_();
  const int rpi = kFoldThreads / (int)(C / 8);
  int64_t blocks = std::min<int64_t>(1024, (M + (int64_t)rpi * 16 - 1) / ((int64_t)rpi * 16));
  const int64_t rpb = (M + blocks - 1) / blocks;
  blocks = (M + rpb - 1) / rpb;
  auto part = at::empty({2, blocks, C}, x.options().dtype(at::kFloat));
  hipStream_t stream = at::hip::getCurrentHIPStream();
  hipLaunchKernelGGL(fold_colsum_kernel<false>, dim3((unsigned)blocks), dim3(kFoldThreads), 0, stream,
                     reinterpret_cast<const bf16*>(x.data_ptr()), (int)C, M, s, ho, wo, hi, wi, rpb,
                     part.data_ptr<float>(), moments_zero_target(sums.data_ptr<double>(), (int)blocks),
                     nullptr, nullptr);
  bn_reduce_partials_launch(part.data_ptr<float>(), (int)blocks, (int)C, sums.data_ptr<double>(), (double)M, stream);
  DMP_HIP_CHECK(hipGetLastError());
  return sums;
}

// (dz = [y > 0] dy bf16 [rows, C], fp64 [2C+1] = (sum dz, sum dz^2, rows)):
// the ReLU mask and dz column sum of the folded bn3's backward in one pass
// (ops/bn_fold.py, when no consumer data-gradient epilogue applied them).
std::vector<at::Tensor> bn_fold_relu_mask(const at::Tensor& dy, const at::Tensor& y) {
  for (const at::Tensor* t : {&dy, &y})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kBFloat16 && t->dim() == 2 && t->is_contiguous(),
                "dy / y must be contiguous bf16 [rows, C] GPU tensors");
  TORCH_CHECK(dy.sizes() == y.sizes(), "dy / y shape mismatch");
  const int64_t C = dy.size(1), M = dy.size(0);
  TORCH_CHECK(C % 8 == 0 && C <= 8 * kFoldThreads, "C % 8 == 0, C <= 2048");
  auto dz = at::empty_like(dy);
  auto sums = at::empty({2 * C + 1}, dy.options().dtype(at::kDouble));
  if (M == 0) return {dz, sums.zero_()};
  const int rpi = kFoldThreads / (int)(C / 8);
  int64_t blocks = std::min<int64_t>(1024, (M + (int64_t)rpi * 16 - 1) / ((int64_t)rpi * 16));
  const int64_t rpb = (M + blocks - 1) / blocks;
  blocks = (M + rpb - 1) / rpb;
  auto part = at::empty({2, blocks, C}, dy.options().dtype(at::kFloat));
  hipStream_t stream = at::hip::getCurrentHIPStream();
  hipLaunchKernelGGL(fold_colsum_kernel<true>, dim3((unsigned)blocks), dim3(kFoldThreads), 0, stream,
                     reinterpret_cast<const bf16*>(dy.data_ptr()), (int)C, M, 1, 1, 1, 1, 1, rpb,
                     part.data_ptr<float>(), moments_zero_target(sums.data_ptr<double>(), (int)blocks),
                     reinterpret_cast<const bf16*>(y.data_ptr()), reinterpret_cast<bf16*>(dz.data_ptr()));
  bn_reduce_partials_launch(part.data_ptr<float>(), (int)blocks, (int)C, sums.data_ptr<double>(), (double)M, stream);
  DMP_HIP_CHECK(hipGetLastError());
  return {dz, sums};
}

// (Bf bf16 [Cout, C3 + Cd] = [s3 o W3 | sd o Wd], shift fp32 [Cout] = t3 + td).
std::vector<at::Tensor> bn_fold_scale_concat(const at::Tensor& W3, const at::Tensor& s3, const at::Tensor& t3,
                                             const at::Tensor& Wd, const at::Tensor& sd, const at::Tensor& td) {
  for (const at::Tensor* w : {&W3, &Wd})
    TORCH_CHECK(w->is_cuda() && w->scalar_type() == at::kBFloat16 && w->dim() == 2 && w->is_contiguous(),
                "weights must be contiguous bf16 [Cout, C] GPU tensors");
  const int64_t Cout = W3.size(0), C3 = W3.size(1), Cd = Wd.size(1);
  TORCH_CHECK(Wd.size(0) == Cout, "W3 / Wd Cout mismatch");
  check_f32(s3, Cout, "s3"); check_f32(t3, Cout, "t3"); check_f32(sd, Cout, "sd"); check_f32(td, Cout, "td");
  auto Bf = at::empty({Cout, C3 + Cd}, W3.options());
  auto shift = at::empty({Cout}, W3.options().dtype(at::kFloat));
  const int64_t n = Cout * (C3 + Cd);
  const unsigned blocks = (unsigned)std::min<int64_t>(2048, (n + kFoldThreads - 1) / kFoldThreads);
  hipLaunchKernelGGL(fold_scale_concat_kernel, dim3(blocks), dim3(kFoldThreads), 0, at::hip::getCurrentHIPStream(),
                     reinterpret_cast<const bf16*>(W3.data_ptr()), s3.data_ptr<float>(), t3.data_ptr<float>(), (int)C3,
                     reinterpret_cast<const bf16*>(Wd.data_ptr()), sd.data_ptr<float>(), td.data_ptr<float>(), (int)Cd,
                     (int)Cout, reinterpret_cast<bf16*>(Bf.data_ptr()), shift.data_ptr<float>());
  DMP_HIP_CHECK(hipGetLastError());
  return {Bf, shift};
}

}  // namespace dmp
