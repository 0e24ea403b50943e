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
    const bf16* __restrict__ R, int64_t ldr, int epi_relu, float* __restrict__ part) {
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

  auto load_tile = [&](int kt) {
    const int k = kt * BK + kv * 8;
    const bool kin = k < K;
#pragma unroll
    for (int i = 0; i < A_VECS; ++i) {
      const int row = m0 + r0 + i * ROWS_PER_PASS;
      if (kin && row < M) ra[i] = *reinterpret_cast<const bf16x8*>(A + (int64_t)row * lda + k);
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
      *reinterpret_cast<bf16x8*>(C + (int64_t)row * ldc + col) = v;
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
            int64_t ldr, bool relu, float* part, hipStream_t stream) {
  const int mtiles = (M + BM - 1) / BM, ntiles = (N + BN - 1) / BN;
  hipLaunchKernelGGL((gemm_nt_kernel<BM, BN, WM, WN, PRO, EPI>), dim3(mtiles * ntiles),
                     dim3(kThreads), 0, stream, reinterpret_cast<const bf16*>(A.data_ptr()),
                     A.stride(0), reinterpret_cast<const bf16*>(B.data_ptr()), B.stride(0),
                     reinterpret_cast<bf16*>(C.data_ptr()), C.stride(0), M, N, K, ps, pt, es, et, R,
                     ldr, (int)relu, part);
}

template <bool PRO, int EPI>
void dispatch_tile(const at::Tensor& A, const at::Tensor& B, at::Tensor& C, int M, int N, int K,
                   const float* ps, const float* pt, const float* es, const float* et,
                   const bf16* R, int64_t ldr, bool relu, float* part, int bm, hipStream_t s) {
  // bm selects the M tile (128 or 256 rows) ; BN follows N.
  if (N <= 64) {
    if (bm == 256) launch<256, 64, 4, 1, PRO, EPI>(A, B, C, M, N, K, ps, pt, es, et, R, ldr, relu, part, s);
    else launch<128, 64, 2, 2, PRO, EPI>(A, B, C, M, N, K, ps, pt, es, et, R, ldr, relu, part, s);
  } else {
    launch<128, 128, 2, 2, PRO, EPI>(A, B, C, M, N, K, ps, pt, es, et, R, ldr, relu, part, s);
  }
}

int tile_m_for(int N) { return N <= 64 ? 256 : 128; }

void check_operand(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16, name, " must be a bf16 GPU tensor");
  TORCH_CHECK(t.dim() == 2 && t.stride(1) == 1, name, " must be a row-major 2-D view");
  TORCH_CHECK(t.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name,
              " rows must be 16-B aligned");
}

}  // namespace

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
                                const c10::optional<at::Tensor>& residual, bool relu) {
  check_operand(A, "A");
  check_operand(B, "B");
  const int M = (int)A.size(0), K = (int)A.size(1), N = (int)B.size(0);
  TORCH_CHECK(B.size(1) == K, "A/B K mismatch");
  TORCH_CHECK(K % 8 == 0 && N % 8 == 0, "K and N must be multiples of 8");
  auto stream = at::hip::getCurrentHIPStream();
  auto C = at::empty({M, N}, A.options());
  const bool pro = pro_scale.has_value() && pro_scale->defined();
  const float* ps = pro ? pro_scale->data_ptr<float>() : nullptr;
  const float* pt = pro ? pro_shift->data_ptr<float>() : nullptr;
  at::Tensor moments;
  if (M == 0) return {C, moments};
  const int bm = tile_m_for(N);
  if (mode == "store") {
    if (pro) dispatch_tile<true, EPI_STORE>(A, B, C, M, N, K, ps, pt, nullptr, nullptr, nullptr, 0, false, nullptr, bm, stream);
    else dispatch_tile<false, EPI_STORE>(A, B, C, M, N, K, ps, pt, nullptr, nullptr, nullptr, 0, false, nullptr, bm, stream);
  } else if (mode == "moments") {
    const int mtiles = (M + bm - 1) / bm;
    auto part = at::empty({2, mtiles, N}, A.options().dtype(at::kFloat));
    if (pro) dispatch_tile<true, EPI_MOMENTS>(A, B, C, M, N, K, ps, pt, nullptr, nullptr, nullptr, 0, false, part.data_ptr<float>(), bm, stream);
    else dispatch_tile<false, EPI_MOMENTS>(A, B, C, M, N, K, ps, pt, nullptr, nullptr, nullptr, 0, false, part.data_ptr<float>(), bm, stream);
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
    if (pro) dispatch_tile<true, EPI_AFFINE>(A, B, C, M, N, K, ps, pt, epi_scale->data_ptr<float>(), epi_shift->data_ptr<float>(), R, ldr, relu, nullptr, bm, stream);
    else dispatch_tile<false, EPI_AFFINE>(A, B, C, M, N, K, ps, pt, epi_scale->data_ptr<float>(), epi_shift->data_ptr<float>(), R, ldr, relu, nullptr, bm, stream);
  } else {
    TORCH_CHECK(false, "unknown epilogue mode ", mode);
  }
  return {C, moments};
}

}  // namespace dmp
