// MFMA bf16 GEMM for channels-last 1x1 convolutions with fused BatchNorm
// prologues / epilogues (gfx950, v_mfma_f32_16x16x32_bf16).
//
//   C[M, N] = A'[M, K] * B[N, K]^T          (both operands K-contiguous, "NT")
//
// A 1x1 convolution on an NHWC activation is exactly this GEMM with
// A = x viewed [N*H*W, Cin], B = weight [Cout, Cin], C = y [N*H*W, Cout]; its
// data gradient is the same GEMM with A = dy, B = weight^T.  The fusions are
// what a library GEMM cannot do (north star: "MFMA conv+BN+ReLU fused kernel"):
//
//   prologue  PRO_BN : A' = relu(A * s[k] + t[k])   -- the previous layer's BN
//                      apply + ReLU, done while staging A, so the normalised
//                      activation is never written to / re-read from HBM;
//   epilogue  EPI_STORE     : C = bf16(acc)
//             EPI_MOMENTS   : C = bf16(acc) and per-column partial (sum, sum^2)
//                             of the STORED values per M-tile -> BN statistics
//                             without a separate read pass over C;
//             EPI_AFFINE    : C = act(acc * s[n] + t[n] (+ R))  -- eval-mode
//                             conv + folded BN (+ residual) + ReLU in one kernel.
//
// Structure (cdna_hip_programming.md §5): 256 threads = 4 waves in a
// WAVES_M x WAVES_N grid, each wave owning a (BM/WAVES_M) x (BN/WAVES_N) tile
// of 16x16 accumulators; BK = 64 (two MFMA k-steps); A/B tiles staged through
// registers into double-buffered LDS (ONE __shared__ array) with a row-pair XOR
// swizzle so each 16-lane ds_read_b128 group hits distinct banks; the next
// K-tile's global loads are issued before the current tile's MFMAs.  The
// epilogue restages the accumulator tile through LDS so C is written with
// 16-byte row-contiguous stores.  Blocks are remapped XCD-aware (T1).
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include "../common.h"

namespace dmp {

// batchnorm.hip: deterministic fp64 reduce of [2][rb][C] partials into [2C+1] moments
void bn_reduce_partials_launch(const float* part, int rb, int C, double* sums, double count,
                               hipStream_t stream);

namespace {

using bf16 = __bf16;
constexpr int BK = 64;
constexpr int kThreads = 256;

enum Epi { EPI_STORE = 0, EPI_MOMENTS = 1, EPI_AFFINE = 2 };

// Logical GEMM row -> physical activation row for strided 1x1 convs: logical
// row (n, oh, ow) of an [N, Ho, Wo] output grid reads/writes physical row
// (n, oh*s, ow*s) of an [N, Hi, Wi] tensor.  s == 1 is the identity, so the
// stride-2 ResNet shortcut needs no subsample copy (forward / wgrad) and no
// scatter pass (dgrad).
struct RowMap {
  int s = 1, ho = 1, wo = 1, hi = 1, wi = 1;
};

__device__ __forceinline__ int64_t map_row(const RowMap& g, int64_t m) {
  if (g.s == 1) return m;
  const int64_t hw = (int64_t)g.ho * g.wo;
  const int64_t n = m / hw;
  const int r = (int)(m - n * hw);
  const int oh = r / g.wo, ow = r - oh * g.wo;
  return (n * g.hi + (int64_t)oh * g.s) * g.wi + (int64_t)ow * g.s;
}

__device__ __forceinline__ int swz(int row, int kvec) {
  // byte offset of 16-B vector `kvec` (0..7) of row `row` in a [rows][64] bf16 tile
  return row * (BK * 2) + ((kvec ^ ((row >> 1) & 7)) << 4);
}

template <int BM, int BN, int WAVES_M, int WAVES_N, bool PRO_BN, int EPI>
__global__ __launch_bounds__(kThreads, 2) void gemm_nt_kernel(
    const bf16* __restrict__ A, int64_t lda, const bf16* __restrict__ B, int64_t ldb,
    bf16* __restrict__ C, int64_t ldc, int M, int N, int K,
    const float* __restrict__ pro_s, const float* __restrict__ pro_t,
    const float* __restrict__ epi_s, const float* __restrict__ epi_t,
    const bf16* __restrict__ R, int64_t ldr, int epi_relu, float* __restrict__ part, RowMap amap,
    RowMap cmap) {
  constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
  constexpr int MI = WTM / 16, NI = WTN / 16;
  constexpr int A_VECS = BM * BK / 8 / kThreads;  // 16-B vectors per thread per A tile
  constexpr int B_VECS = BN * BK / 8 / kThreads;
  static_assert(A_VECS >= 1 && B_VECS >= 1, "tile too small for 256 threads");
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int STAGE_BYTES = A_BYTES + B_BYTES;
  constexpr int CT_STRIDE = BN + 8;  // +16 B per row: epilogue tile writes spread over banks
  constexpr int EPI_BYTES = BM * CT_STRIDE * 2;
  constexpr int LDS_BYTES = (2 * STAGE_BYTES > EPI_BYTES ? 2 * STAGE_BYTES : EPI_BYTES);
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int mtiles = (M + BM - 1) / BM, ntiles = (N + BN - 1) / BN;
  const int nblocks = mtiles * ntiles;
  const int bid = xcd_remap(blockIdx.x, nblocks);
  // N-tiles of one M-tile are adjacent (they share the A panel in L2)
  const int mt = bid / ntiles, nt = bid % ntiles;
  const int m0 = mt * BM, n0 = nt * BN;
  const int ktiles = (K + BK - 1) / BK;

  // ---- per-thread staging coordinates (fixed k-vector per thread) ----
  const int kv = tid % (BK / 8);  // 0..7
  const int r0 = tid / (BK / 8);  // 0..31, rows r0 + i*32
  constexpr int ROWS_PER_PASS = kThreads / (BK / 8);

  bf16x8 ra[A_VECS], rb[B_VECS];
  const bf16* arow[A_VECS];  // this thread's A rows are fixed for the whole K loop
#pragma unroll
  for (int i = 0; i < A_VECS; ++i) {
    const int row = m0 + r0 + i * ROWS_PER_PASS;
    arow[i] = row < M ? A + map_row(amap, row) * lda : nullptr;
  }

  auto load_tile = [&](int kt) {
    const int k = kt * BK + kv * 8;
    const bool kin = k < K;
#pragma unroll
    for (int i = 0; i < A_VECS; ++i) {
      if (kin && arow[i]) ra[i] = *reinterpret_cast<const bf16x8*>(arow[i] + k);
      else ra[i] = bf16x8{};
    }
#pragma unroll
    for (int i = 0; i < B_VECS; ++i) {
      const int col = n0 + r0 + i * ROWS_PER_PASS;
      if (kin && col < N) rb[i] = *reinterpret_cast<const bf16x8*>(B + (int64_t)col * ldb + k);
      else rb[i] = bf16x8{};
    }
    if constexpr (PRO_BN) {
      if (kin) {
        float s[8], t[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) { s[j] = pro_s[k + j]; t[j] = pro_t[k + j]; }
#pragma unroll
        for (int i = 0; i < A_VECS; ++i) {
          const int row = m0 + r0 + i * ROWS_PER_PASS;
          f32x8 f = __builtin_convertvector(ra[i], f32x8);
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = fmaxf(fmaf(f[j], s[j], t[j]), 0.f);
          // rows beyond M stay exactly zero (they are never stored)
          ra[i] = row < M ? __builtin_convertvector(f, bf16x8) : bf16x8{};
        }
      }
    }
  };
  auto store_tile = [&](int buf) {
    char* as = smem + buf * STAGE_BYTES;
    char* bs = as + A_BYTES;
#pragma unroll
    for (int i = 0; i < A_VECS; ++i)
      *reinterpret_cast<bf16x8*>(as + swz(r0 + i * ROWS_PER_PASS, kv)) = ra[i];
#pragma unroll
    for (int i = 0; i < B_VECS; ++i)
      *reinterpret_cast<bf16x8*>(bs + swz(r0 + i * ROWS_PER_PASS, kv)) = rb[i];
  };

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  load_tile(0);
  store_tile(0);
  __syncthreads();
  const int lrow = lane & 15, lk = lane >> 4;
  for (int kt = 0; kt < ktiles; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < ktiles) load_tile(kt + 1);  // global loads in flight under the MFMAs
    const char* as = smem + cur * STAGE_BYTES;
    const char* bs = as + A_BYTES;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      bf16x8 fa[MI], fb[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i)
        fa[i] = *reinterpret_cast<const bf16x8*>(as + swz(wm * WTM + i * 16 + lrow, ks * 4 + lk));
#pragma unroll
      for (int j = 0; j < NI; ++j)
        fb[j] = *reinterpret_cast<const bf16x8*>(bs + swz(wn * WTN + j * 16 + lrow, ks * 4 + lk));
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < ktiles) {
      store_tile(cur ^ 1);
    }
    __syncthreads();
  }

  // ---- epilogue: accumulators -> bf16 tile in LDS (row-major [BM][BN]) ----
  bf16* ct = reinterpret_cast<bf16*>(smem);
  // (the last loop iteration ended with a barrier, staging buffers are free)
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int col = wn * WTN + j * 16 + (lane & 15);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = wm * WTM + i * 16 + (lane >> 4) * 4 + e;
        // affine / residual / activation are applied in the row-contiguous store pass
        ct[row * CT_STRIDE + col] = (bf16)acc[i][j][e];
      }
    }
  __syncthreads();

  // ---- store pass: each thread moves 8 contiguous columns of a row ----
  constexpr int CV = BN / 8;                  // 16-B vectors per row
  constexpr int RPP = kThreads / CV;          // rows per pass
  const int cvi = tid % CV, rr0 = tid / CV;
  const int col = n0 + cvi * 8;
  const bool col_ok = col < N;
  float es[8], et[8];
  if constexpr (EPI == EPI_AFFINE) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      es[j] = col_ok ? epi_s[col + j] : 0.f;
      et[j] = col_ok ? epi_t[col + j] : 0.f;
    }
  }
  float msum[8], msq[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { msum[j] = 0.f; msq[j] = 0.f; }
#pragma unroll
  for (int p = 0; p < BM / RPP; ++p) {
    const int lr = rr0 + p * RPP;
    const int row = m0 + lr;
    bf16x8 v = *reinterpret_cast<const bf16x8*>(ct + lr * CT_STRIDE + cvi * 8);
    if (row < M && col_ok) {
      if constexpr (EPI == EPI_AFFINE) {
        f32x8 f = __builtin_convertvector(v, f32x8);
        f32x8 r{};
        if (R) r = __builtin_convertvector(*reinterpret_cast<const bf16x8*>(R + (int64_t)row * ldr + col), f32x8);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float t = fmaf(f[j], es[j], et[j]) + r[j];
          f[j] = epi_relu ? fmaxf(t, 0.f) : t;
        }
        v = __builtin_convertvector(f, bf16x8);
      }
      *reinterpret_cast<bf16x8*>(C + map_row(cmap, row) * ldc + col) = v;
      if constexpr (EPI == EPI_MOMENTS) {
        f32x8 f = __builtin_convertvector(v, f32x8);
#pragma unroll
        for (int j = 0; j < 8; ++j) { msum[j] += f[j]; msq[j] = fmaf(f[j], f[j], msq[j]); }
      }
    }
  }
  if constexpr (EPI == EPI_MOMENTS) {
    // combine the RPP row-groups of each column through LDS, one partial per M-tile
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);  // [2][RPP][BN]
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[(0 * RPP + rr0) * BN + cvi * 8 + j] = msum[j];
      red[(1 * RPP + rr0) * BN + cvi * 8 + j] = msq[j];
    }
    __syncthreads();
    for (int c = tid; c < BN; c += kThreads) {
      float s = 0.f, q = 0.f;
      for (int g = 0; g < RPP; ++g) {
        s += red[(0 * RPP + g) * BN + c];
        q += red[(1 * RPP + g) * BN + c];
      }
      if (n0 + c < N) {
        part[(int64_t)mt * N + n0 + c] = s;
        part[(int64_t)(mtiles + mt) * N + n0 + c] = q;
      }
    }
  }
}

template <int BM, int BN, int WM, int WN, bool PRO, int EPI>
void launch(const at::Tensor& A, const at::Tensor& B, at::Tensor& C, int M, int N, int K,
            const float* ps, const float* pt, const float* es, const float* et, const bf16* R,
            int64_t ldr, bool relu, float* part, const RowMap& am, const RowMap& cm,
            hipStream_t stream) {
  const int mtiles = (M + BM - 1) / BM, ntiles = (N + BN - 1) / BN;
  hipLaunchKernelGGL((gemm_nt_kernel<BM, BN, WM, WN, PRO, EPI>), dim3(mtiles * ntiles),
                     dim3(kThreads), 0, stream, reinterpret_cast<const bf16*>(A.data_ptr()),
                     A.stride(0), reinterpret_cast<const bf16*>(B.data_ptr()), B.stride(0),
                     reinterpret_cast<bf16*>(C.data_ptr()), C.stride(0), M, N, K, ps, pt, es, et, R,
                     ldr, (int)relu, part, am, cm);
}

template <bool PRO, int EPI>
void dispatch_tile(const at::Tensor& A, const at::Tensor& B, at::Tensor& C, int M, int N, int K,
                   const float* ps, const float* pt, const float* es, const float* et,
                   const bf16* R, int64_t ldr, bool relu, float* part, const RowMap& am,
                   const RowMap& cm, int bm, hipStream_t s) {
  // bm selects the M tile (128 or 256 rows) ; BN follows N.
  if (N <= 64) {
    if (bm == 256) launch<256, 64, 4, 1, PRO, EPI>(A, B, C, M, N, K, ps, pt, es, et, R, ldr, relu, part, am, cm, s);
    else launch<128, 64, 2, 2, PRO, EPI>(A, B, C, M, N, K, ps, pt, es, et, R, ldr, relu, part, am, cm, s);
  } else {
    launch<128, 128, 2, 2, PRO, EPI>(A, B, C, M, N, K, ps, pt, es, et, R, ldr, relu, part, am, cm, s);
  }
}

RowMap parse_map(const std::vector<int64_t>& g, const char* name) {
  RowMap m;
  if (g.empty()) return m;
  TORCH_CHECK(g.size() == 5, name, " must be [stride, Ho, Wo, Hi, Wi]");
  m.s = (int)g[0]; m.ho = (int)g[1]; m.wo = (int)g[2]; m.hi = (int)g[3]; m.wi = (int)g[4];
  TORCH_CHECK(m.s >= 1 && (m.ho - 1) * m.s < m.hi && (m.wo - 1) * m.s < m.wi && m.ho > 0 && m.wo > 0,
              name, ": output grid does not fit the input grid");
  return m;
}

int tile_m_for(int N) { return N <= 64 ? 256 : 128; }

// ---------------------------------------------------------------------------
// Weight gradient of a 1x1 conv: C[N, K] = sum_m A[m, n] * B[m, k]
// (A = dy [M, N], B = x [M, K], both row-major).  The reduction runs over the
// huge M = batch*H*W, the output is tiny, so the M range is split across
// blocks (split-M) and each block writes an fp32 partial tile; a column
// reduce sums the partials deterministically.  MFMA operands need 8
// consecutive m per lane, i.e. a transpose of the row-major tiles: staged
// row-major in LDS (16-B writes) and read with ds_read_b64_tr_b16 (gfx950's
// transposing LDS read, cdna_hip_programming.md §5.5 T10), with a 32-B chunk
// XOR swizzle so the 4-row x 32-B blocks of the two 16-lane groups of a
// half-wave hit distinct banks.
// ---------------------------------------------------------------------------
constexpr int TN_BM = 64;  // m rows per LDS stage (two MFMA k-steps)

__device__ __forceinline__ int tn_off(int row, int col, int row_bytes) {
  // byte offset of element (row, col) [bf16] with the 32-B-chunk swizzle; the
  // XOR stays inside the row (row_bytes / 32 chunks: 8 for 256-B, 4 for 128-B rows)
  const int byte = col * 2;
  const int mask = (row_bytes >> 5) - 1;
  const int chunk = (byte >> 5) ^ ((row + 4 * (row >> 3)) & mask);
  return row * row_bytes + (chunk << 5) + (byte & 31);
}

template <int BNT, int BKT>
__global__ __launch_bounds__(kThreads, 2) void gemm_tn_kernel(
    const bf16* __restrict__ A, int64_t lda, const bf16* __restrict__ B, int64_t ldb, int M, int N,
    int K, int64_t rows_per_split, float* __restrict__ part, RowMap bmap) {
  // 4 waves as 2 x 2, each wave (BNT/2) x (BKT/2) outputs
  constexpr int WTN = BNT / 2, WTK = BKT / 2;
  constexpr int MI = WTN / 16, NI = WTK / 16;
  constexpr int A_ROWB = BNT * 2, B_ROWB = BKT * 2;  // LDS row bytes
  constexpr int A_BYTES = TN_BM * A_ROWB, B_BYTES = TN_BM * B_ROWB;
  constexpr int A_VPR = BNT / 8, B_VPR = BKT / 8;    // 16-B vectors per row
  constexpr int A_VECS = TN_BM * A_VPR / kThreads, B_VECS = TN_BM * B_VPR / kThreads;
  static_assert(A_VECS >= 1 && B_VECS >= 1, "tile too small");
  __shared__ __attribute__((aligned(16))) char smem[2 * (A_BYTES + B_BYTES)];
  using v4i16 = short __attribute__((ext_vector_type(4)));
  using lds_v4 = __attribute__((address_space(3))) v4i16;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave >> 1, wk = wave & 1;
  const int ntiles = (N + BNT - 1) / BNT, ktiles = (K + BKT - 1) / BKT;
  const int tile = blockIdx.x % (ntiles * ktiles);
  const int split = blockIdx.x / (ntiles * ktiles);
  const int n0 = (tile / ktiles) * BNT, k0 = (tile % ktiles) * BKT;
  const int64_t mb = (int64_t)split * rows_per_split;
  const int64_t me = min((int64_t)M, mb + rows_per_split);
  const int nstages = (int)((me - mb + TN_BM - 1) / TN_BM);

  bf16x8 ra[A_VECS], rb[B_VECS];
  auto load = [&](int s) {
    const int64_t m0 = mb + (int64_t)s * TN_BM;
#pragma unroll
    for (int i = 0; i < A_VECS; ++i) {
      const int v = tid + i * kThreads, r = v / A_VPR, c = (v % A_VPR) * 8;
      const int64_t m = m0 + r;
      ra[i] = (m < me && n0 + c < N) ? *reinterpret_cast<const bf16x8*>(A + m * lda + n0 + c) : bf16x8{};
    }
#pragma unroll
    for (int i = 0; i < B_VECS; ++i) {
      const int v = tid + i * kThreads, r = v / B_VPR, c = (v % B_VPR) * 8;
      const int64_t m = m0 + r;
      rb[i] = (m < me && k0 + c < K)
                  ? *reinterpret_cast<const bf16x8*>(B + map_row(bmap, m) * ldb + k0 + c)
                  : bf16x8{};
    }
  };
  auto store = [&](int buf) {
    char* as = smem + buf * (A_BYTES + B_BYTES);
    char* bs = as + A_BYTES;
#pragma unroll
    for (int i = 0; i < A_VECS; ++i) {
      const int v = tid + i * kThreads, r = v / A_VPR, c = (v % A_VPR) * 8;
      *reinterpret_cast<bf16x8*>(as + tn_off(r, c, A_ROWB)) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < B_VECS; ++i) {
      const int v = tid + i * kThreads, r = v / B_VPR, c = (v % B_VPR) * 8;
      *reinterpret_cast<bf16x8*>(bs + tn_off(r, c, B_ROWB)) = rb[i];
    }
  };

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // tr-read lane roles: group g = lane>>4 covers m rows 8g..8g+7 of a k-step,
  // lane i = 4q+p of the group addresses row q, columns 4p..4p+3 of the block
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  if (nstages > 0) {
    load(0);
    store(0);
  }
  __syncthreads();
  for (int s = 0; s < nstages; ++s) {
    const int cur = s & 1;
    if (s + 1 < nstages) load(s + 1);
    const char* as = smem + cur * (A_BYTES + B_BYTES);
    const char* bs = as + A_BYTES;
#pragma unroll
    for (int ks = 0; ks < TN_BM / 32; ++ks) {
      bf16x8 fa[MI], fb[NI];
      const int rbase = ks * 32 + 8 * g + q;
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int col = wn * WTN + i * 16 + 4 * p;
        v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(as + tn_off(rbase, col, A_ROWB)));
        v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(as + tn_off(rbase + 4, col, A_ROWB)));
        short __attribute__((ext_vector_type(8))) t8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        fa[i] = __builtin_bit_cast(bf16x8, t8);
      }
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int col = wk * WTK + j * 16 + 4 * p;
        v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(bs + tn_off(rbase, col, B_ROWB)));
        v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(bs + tn_off(rbase + 4, col, B_ROWB)));
        short __attribute__((ext_vector_type(8))) t8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        fb[j] = __builtin_bit_cast(bf16x8, t8);
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if (s + 1 < nstages) store(cur ^ 1);
    __syncthreads();
  }
  // fp32 partial tile: part[split][n][k]
  float* out = part + (int64_t)split * N * K;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int k = k0 + wk * WTK + j * 16 + (lane & 15);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int n = n0 + wn * WTN + i * 16 + (lane >> 4) * 4 + e;
        if (n < N && k < K) out[(int64_t)n * K + k] = acc[i][j][e];
      }
    }
}

// out[c] = sum_s part[s][c], written as bf16 or fp32.  A 256-thread block owns
// 256/SL float4 columns and splits them over SL "split lanes" (thread t reads
// splits t/cols, t/cols + SL, ...), then folds the SL lanes in LDS.  SL is
// chosen on the host so small outputs with many splits still fill the chip
// (a 64x64 weight with 1024 splits would otherwise be 4 blocks of serial loads).
template <typename OT>
__global__ __launch_bounds__(256) void split_reduce_kernel(const float* __restrict__ part, int splits,
                                                           int64_t n, int sl, OT* __restrict__ out) {
  const int cols = 256 / sl;
  const int cl = threadIdx.x % cols, lane_s = threadIdx.x / cols;
  const int64_t i = ((int64_t)blockIdx.x * cols + cl) * 4;
  f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f};
  if (i < n) {
    int s = lane_s;
    for (; s + sl < splits; s += 2 * sl) {
      const f32x4 p0 = *reinterpret_cast<const f32x4*>(part + (int64_t)s * n + i);
      const f32x4 p1 = *reinterpret_cast<const f32x4*>(part + (int64_t)(s + sl) * n + i);
      a += p0 + p1;
    }
    if (s < splits) a += *reinterpret_cast<const f32x4*>(part + (int64_t)s * n + i);
  }
  __shared__ f32x4 red[256];
  red[threadIdx.x] = a;
  __syncthreads();
  for (int h = sl / 2; h > 0; h >>= 1) {
    if (lane_s < h) red[threadIdx.x] += red[threadIdx.x + h * cols];
    __syncthreads();
  }
  if (lane_s == 0 && i < n) {
    a = red[threadIdx.x];
#pragma unroll
    for (int e = 0; e < 4; ++e) out[i + e] = (OT)a[e];
  }
}

void check_operand(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16, name, " must be a bf16 GPU tensor");
  TORCH_CHECK(t.dim() == 2 && t.stride(1) == 1, name, " must be a row-major 2-D view");
  TORCH_CHECK(t.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name,
              " rows must be 16-B aligned");
}

template <int BNT, int BKT>
void launch_tn(const at::Tensor& A, const at::Tensor& B, int M, int N, int K, float* part,
               int splits, int64_t rps, const RowMap& bm, hipStream_t s) {
  const int tiles = ((N + BNT - 1) / BNT) * ((K + BKT - 1) / BKT);
  hipLaunchKernelGGL((gemm_tn_kernel<BNT, BKT>), dim3(tiles * splits), dim3(kThreads), 0, s,
                     reinterpret_cast<const bf16*>(A.data_ptr()), A.stride(0),
                     reinterpret_cast<const bf16*>(B.data_ptr()), B.stride(0), M, N, K, rps, part, bm);
}

}  // namespace

// Weight gradient of a 1x1 conv: C[N, K] = A^T B with A [M, N], B [M, K] (bf16,
// row-major).  Output dtype bf16 or fp32.  b_map ([s, Ho, Wo, Hi, Wi]) reads
// B's logical row m from the strided physical row (stride-s 1x1 conv input).
at::Tensor gemm_tn(const at::Tensor& A, const at::Tensor& B, at::ScalarType out_dtype,
                   const std::vector<int64_t>& b_map) {
  check_operand(A, "A");
  check_operand(B, "B");
  const RowMap bmap = parse_map(b_map, "b_map");
  if (bmap.s == 1) {
    TORCH_CHECK(A.size(0) == B.size(0), "A/B M mismatch");
  } else {
    TORCH_CHECK(B.size(0) % ((int64_t)bmap.hi * bmap.wi) == 0 &&
                    A.size(0) == B.size(0) / ((int64_t)bmap.hi * bmap.wi) * bmap.ho * bmap.wo,
                "b_map does not match the A/B row counts");
  }
  const int M = (int)A.size(0), N = (int)A.size(1), K = (int)B.size(1);
  TORCH_CHECK(N % 8 == 0 && K % 8 == 0, "N and K must be multiples of 8");
  auto stream = at::hip::getCurrentHIPStream();
  auto out = at::empty({N, K}, A.options().dtype(out_dtype));
  if (M == 0) return out.zero_();
  const int bnt = N >= 128 ? 128 : 64, bkt = K >= 128 ? 128 : 64;
  const int tiles = ((N + bnt - 1) / bnt) * ((K + bkt - 1) / bkt);
  // ~4 blocks per CU, but keep the fp32 partial traffic well under the operand
  // traffic (the GEMM streams (N+K)*M bf16; partials cost 2 * splits*N*K*4 B).
  const int max_splits = std::max(1, (M + TN_BM - 1) / TN_BM);
  const int64_t operand_bytes = (int64_t)M * (N + K) * 2;
  const int64_t part_cap = std::max<int64_t>(operand_bytes / 4, 8 << 20);
  const int by_bytes = (int)std::max<int64_t>(1, part_cap / ((int64_t)N * K * 8));
  int splits = std::min({max_splits, by_bytes, std::max(1, (1024 + tiles - 1) / tiles)});
  int64_t rps = ((int64_t)M + splits - 1) / splits;
  rps = (rps + TN_BM - 1) / TN_BM * TN_BM;
  splits = (int)(((int64_t)M + rps - 1) / rps);
  auto part = at::empty({splits, N, K}, A.options().dtype(at::kFloat));
  float* pp = part.data_ptr<float>();
  if (bnt == 128 && bkt == 128) launch_tn<128, 128>(A, B, M, N, K, pp, splits, rps, bmap, stream);
  else if (bnt == 128) launch_tn<128, 64>(A, B, M, N, K, pp, splits, rps, bmap, stream);
  else if (bkt == 128) launch_tn<64, 128>(A, B, M, N, K, pp, splits, rps, bmap, stream);
  else launch_tn<64, 64>(A, B, M, N, K, pp, splits, rps, bmap, stream);
  const int64_t n = (int64_t)N * K;
  int sl = 1;  // split lanes per column: grow until >= 512 blocks or lanes cover the splits
  while (sl < 64 && sl < splits && (n / 4 + 256 / sl - 1) / (256 / sl) < 512) sl *= 2;
  const unsigned blocks = (unsigned)((n / 4 + 256 / sl - 1) / (256 / sl));
  if (out_dtype == at::kBFloat16)
    hipLaunchKernelGGL((split_reduce_kernel<bf16>), dim3(blocks), dim3(256), 0, stream, pp, splits, n,
                       sl, reinterpret_cast<bf16*>(out.data_ptr()));
  else
    hipLaunchKernelGGL((split_reduce_kernel<float>), dim3(blocks), dim3(256), 0, stream, pp, splits, n,
                       sl, out.data_ptr<float>());
  return out;
}

// C = prologue(A) @ B^T with an optional fused epilogue.  Returns (C, moments-or-undefined).
//   A [M, K] bf16, B [N, K] bf16 (both K-contiguous), K % 8 == 0, N % 8 == 0.
//   pro_scale/pro_shift [K] fp32: A' = relu(A*s + t)
//   mode "store" | "moments" (returns fp64 [2N+1] = (sum, sumsq, M)) | "affine"
//   (epi_scale/epi_shift [N], optional residual [M, N], relu flag).
std::vector<at::Tensor> gemm_nt(const at::Tensor& A, const at::Tensor& B,
                                const c10::optional<at::Tensor>& pro_scale,
                                const c10::optional<at::Tensor>& pro_shift, const std::string& mode,
                                const c10::optional<at::Tensor>& epi_scale,
                                const c10::optional<at::Tensor>& epi_shift,
                                const c10::optional<at::Tensor>& residual, bool relu,
                                const std::vector<int64_t>& a_map,
                                const std::vector<int64_t>& c_map) {
  check_operand(A, "A");
  check_operand(B, "B");
  const RowMap am = parse_map(a_map, "a_map"), cm = parse_map(c_map, "c_map");
  int64_t m64 = A.size(0);
  if (am.s != 1) {
    TORCH_CHECK(m64 % ((int64_t)am.hi * am.wi) == 0, "a_map does not match A's rows");
    m64 = m64 / ((int64_t)am.hi * am.wi) * am.ho * am.wo;
  }
  const int M = (int)m64, K = (int)A.size(1), N = (int)B.size(0);
  TORCH_CHECK(B.size(1) == K, "A/B K mismatch");
  TORCH_CHECK(K % 8 == 0 && N % 8 == 0, "K and N must be multiples of 8");
  auto stream = at::hip::getCurrentHIPStream();
  at::Tensor C;
  if (cm.s == 1) {
    C = at::empty({M, N}, A.options());
  } else {
    // rows the strided scatter does not reach are exactly zero (dgrad of a strided 1x1 conv)
    TORCH_CHECK(M % ((int64_t)cm.ho * cm.wo) == 0, "c_map does not match the GEMM rows");
    C = at::zeros({(int64_t)M / ((int64_t)cm.ho * cm.wo) * cm.hi * cm.wi, N}, A.options());
  }
  const bool pro = pro_scale.has_value() && pro_scale->defined();
  const float* ps = pro ? pro_scale->data_ptr<float>() : nullptr;
  const float* pt = pro ? pro_shift->data_ptr<float>() : nullptr;
  at::Tensor moments;
  if (M == 0) return {C, moments};
  const int bm = tile_m_for(N);
  if (mode == "store") {
    if (pro) dispatch_tile<true, EPI_STORE>(A, B, C, M, N, K, ps, pt, nullptr, nullptr, nullptr, 0, false, nullptr, am, cm, bm, stream);
    else dispatch_tile<false, EPI_STORE>(A, B, C, M, N, K, ps, pt, nullptr, nullptr, nullptr, 0, false, nullptr, am, cm, bm, stream);
  } else if (mode == "moments") {
    const int mtiles = (M + bm - 1) / bm;
    auto part = at::empty({2, mtiles, N}, A.options().dtype(at::kFloat));
    if (pro) dispatch_tile<true, EPI_MOMENTS>(A, B, C, M, N, K, ps, pt, nullptr, nullptr, nullptr, 0, false, part.data_ptr<float>(), am, cm, bm, stream);
    else dispatch_tile<false, EPI_MOMENTS>(A, B, C, M, N, K, ps, pt, nullptr, nullptr, nullptr, 0, false, part.data_ptr<float>(), am, cm, bm, stream);
    moments = at::empty({2 * (int64_t)N + 1}, A.options().dtype(at::kDouble));
    bn_reduce_partials_launch(part.data_ptr<float>(), mtiles, N, moments.data_ptr<double>(),
                              (double)M, stream);
  } else if (mode == "affine") {
    TORCH_CHECK(epi_scale.has_value() && epi_shift.has_value(), "affine epilogue needs scale/shift");
    const bf16* R = nullptr;
    int64_t ldr = 0;
    if (residual.has_value() && residual->defined()) {
      check_operand(*residual, "residual");
      TORCH_CHECK(residual->size(0) == M && residual->size(1) == N, "residual shape");
      R = reinterpret_cast<const bf16*>(residual->data_ptr());
      ldr = residual->stride(0);
    }
    if (pro) dispatch_tile<true, EPI_AFFINE>(A, B, C, M, N, K, ps, pt, epi_scale->data_ptr<float>(), epi_shift->data_ptr<float>(), R, ldr, relu, nullptr, am, cm, bm, stream);
    else dispatch_tile<false, EPI_AFFINE>(A, B, C, M, N, K, ps, pt, epi_scale->data_ptr<float>(), epi_shift->data_ptr<float>(), R, ldr, relu, nullptr, am, cm, bm, stream);
  } else {
    TORCH_CHECK(false, "unknown epilogue mode ", mode);
  }
  return {C, moments};
}

}  // namespace dmp
