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
//                             (s, t null: C = acc + R -- a data gradient
//                             summed with another branch's, see ops/fused.py)
//                             conv + folded BN (+ residual) + ReLU in one kernel.
//             EPI_BNBWD     : the data gradient G = bf16(acc (+ R)) of a layer
//                             whose input is a training-mode BN+ReLU output:
//                             C = dz = G * relu_mask (mask from the BN output y
//                             when a residual was fused before the ReLU, else
//                             re-derived from the BN input x as x*sc + sh > 0)
//                             and per-column partial (sum dz, sum dz*(x-mean))
//                             per M-tile -> the BN backward's reductions
//                             without its separate read pass over dy and x.
//
// Structure (cdna_hip_programming.md §5): 256 threads = 4 waves in a
// WAVES_M x WAVES_N grid, each wave owning a (BM/WAVES_M) x (BN/WAVES_N) tile
// of 16x16 accumulators; BK = 64 (two MFMA k-steps); A/B tiles staged through
// registers into double-buffered LDS (ONE __shared__ array) with a row-pair XOR
// swizzle so each 16-lane ds_read_b128 group hits distinct banks; the next
// K-tile's global loads are issued before the current tile's MFMAs.  The
// epilogue restages the accumulator tile through LDS so C is written with
// 16-byte row-contiguous stores.  Blocks are remapped XCD-aware (T1).
#include <cstdlib>
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

// zeros an absent per-column coefficient vector is read from (branch-free epilogue loads)
__device__ __attribute__((aligned(32))) float g_nt_zero[16] = {};

enum Epi { EPI_STORE = 0, EPI_MOMENTS = 1, EPI_AFFINE = 2, EPI_BNBWD = 3,
           // EPI_BNBWD with the mask taken from the BN output y, fixed at compile
           // time (with / without the x moments); plain EPI_BNBWD = mask from x
           // (gemm_xl.hip finding 55: the runtime operand flags cost the epilogue)
           EPI_BNBWD_Y = 4, EPI_BNBWD_YO = 5 };
__host__ __device__ constexpr bool nt_bnbwd(int e) { return e == EPI_BNBWD || e == EPI_BNBWD_Y || e == EPI_BNBWD_YO; }

// Logical GEMM row -> physical activation row for strided 1x1 convs: logical
// row (n, oh, ow) of an [N, Ho, Wo] output grid reads/writes physical row
// (n, oh*s, ow*s) of an [N, Hi, Wi] tensor.  s == 1 is the identity, so the
// stride-2 ResNet shortcut needs no subsample copy (forward / wgrad) and no
// scatter pass (dgrad).
struct RowMap {
  int s = 1, ho = 1, wo = 1, hi = 1, wi = 1;
  int oy = 0, ox = 0;  // phase offset: logical (oh, ow) -> physical (oh*s + oy, ow*s + ox)
};

__device__ __forceinline__ int64_t map_row(const RowMap& g, int64_t m) {
  if (g.s == 1) return m;
  const int64_t hw = (int64_t)g.ho * g.wo;
  const int64_t n = m / hw;
  const int r = (int)(m - n * hw);
  const int oh = r / g.wo, ow = r - oh * g.wo;
  return (n * g.hi + (int64_t)oh * g.s + g.oy) * g.wi + (int64_t)ow * g.s + g.ox;
}

__device__ __forceinline__ int swz(int row, int kvec) {
  // byte offset of 16-B vector `kvec` (0..7) of row `row` in a [rows][64] bf16 tile
  return row * (BK * 2) + ((kvec ^ ((row >> 1) & 7)) << 4);
}

// Implicit-GEMM convolution geometry (kh x kw taps, NHWC activations).
// GEMM rows are the pixels of the (ho, wo) grid; A is the (hi, wi) tensor.
//   forward    : A pixel = (oh*stride - pad + r, ow*stride - pad + c)
//   transposed : A pixel = ((oh + pad - r) / stride, ...) when divisible --
//                the data gradient of a strided conv, no flipped weights.
// kc = channels per tap (a multiple of BK so a K tile never straddles taps).
// transposed == 2 is the STRIDE-PHASE data gradient: one launch per output
// phase (py, px) of a stride-s conv; its rows are the phase's sub-grid pixels
// (a, b) (physical (a*s + py, b*s + px), written through the C row map) and its
// K runs over only the taps that reach that phase -- ptr/ptc[i] -- each a
// dense dy pixel (a + (py + pad - tr)/s, ...): no multiply-by-zero taps (the
// plain transposed gather wastes (s*s - 1)/(s*s) of its K on them).
struct ConvMap {
  int kw = 1, stride = 1, pad = 0, hi = 1, wi = 1, ho = 1, wo = 1, kc = 0, transposed = 0;
  int py = 0, px = 0;
  int8_t ptr[16] = {}, ptc[16] = {};
  int amap = 0;  // TN only: A rows mapped like B's tap (0, 0) -- the Gram x_s^T x_s of a strided sample
};

struct NtArgs {
  const bf16* A; int64_t lda;
  const bf16* B; int64_t ldb;
  bf16* C; int64_t ldc;
  int M, N, K;
  const float *pro_s, *pro_t;   // PRO_BN prologue (per A channel)
  const float *epi_s, *epi_t;   // EPI_AFFINE (per output column)
  const bf16* R; int64_t ldr;   // EPI_AFFINE residual
  int epi_relu;
  float* part;                  // EPI_MOMENTS partials [2][mtiles][N]
  double* zsums;                // EPI_MOMENTS: fp64 moments to zero (see common.h) or null
  RowMap amap, cmap;            // strided 1x1 row maps (non-CONV)
  ConvMap cv;                   // implicit-GEMM conv geometry (CONV)
  // EPI_BNBWD: BN input x [M, N] and (optional) BN output y [M, N], per-column
  // mean and the forward affine (sc, sh) for the mask when y is absent
  const bf16* bx; int64_t ldbx;
  const bf16* bny; int64_t ldby;
  // mask affine x*sc + sh > 0 with sc = invstd * w, sh = b - mean * sc (w, b optional),
  // computed per column in the epilogue (no coefficient kernels on the host side)
  const float *bmean, *binv, *bw, *bb;
  CompactMap rmap;              // EPI_BNBWD residual R in compact stride-s form
  // Second A source (non-CONV): K columns k >= K1 read A2[row, k - K1] -- the
  // operand [dz | a] of a BN-folded data gradient (ops/bn_fold.py).  K1 % 8 == 0.
  const bf16* A2; int64_t lda2; int K1;
  RowMap a2map;                 // A2 rows through a strided map (the x_s of a folded downsample)
  const float* ebias;           // EPI_BNBWD: per-column bias added to the GEMM output
};

// NT = WAVES_M*WAVES_N*64 threads: 4 waves (2 blocks/CU) or 8 waves (256-row
// tiles, 1 block/CU: 1.36x the FLOPs per staged byte of 128x128, for the
// L2-bandwidth-bound deep-K shapes).
template <int BM, int BN, int WAVES_M, int WAVES_N, bool PRO_BN, int EPI, bool CONV, int NSTAGE>
__global__ __launch_bounds__(WAVES_M * WAVES_N * 64, (WAVES_M * WAVES_N == 8 ? 1 : 2))
void gemm_nt_kernel(const NtArgs p) {
  constexpr int kThreads = WAVES_M * WAVES_N * 64;
  const bf16* __restrict__ A = p.A;
  const bf16* __restrict__ B = p.B;
  bf16* __restrict__ C = p.C;
  const int64_t lda = p.lda, ldb = p.ldb, ldc = p.ldc, ldr = p.ldr;
  const int M = p.M, N = p.N, K = p.K;
  const float* __restrict__ pro_s = p.pro_s;
  const float* __restrict__ pro_t = p.pro_t;
  const float* __restrict__ epi_s = p.epi_s;
  const float* __restrict__ epi_t = p.epi_t;
  const bf16* __restrict__ R = p.R;
  const int epi_relu = p.epi_relu;
  float* __restrict__ part = p.part;
  const RowMap& amap = p.amap;
  const RowMap& cmap = p.cmap;
  const ConvMap& cv = p.cv;
  if constexpr (EPI == EPI_MOMENTS || nt_bnbwd(EPI)) zero_moments(p.zsums, 2 * N);
  constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
  constexpr int MI = WTM / 16, NI = WTN / 16;
  constexpr int A_VECS = BM * BK / 8 / kThreads;  // 16-B vectors per thread per A tile
  constexpr int B_VECS = BN * BK / 8 / kThreads;
  static_assert(A_VECS >= 1 && B_VECS >= 1, "tile too small for 256 threads");
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int STAGE_BYTES = A_BYTES + B_BYTES;
  constexpr int CT_STRIDE = BN + 8;  // +16 B per row: epilogue tile writes spread over banks
  constexpr int EPI_BYTES = BM * CT_STRIDE * 2;
  // NSTAGE == 1: the host guarantees K <= BK (one K tile), so no second
  // staging buffer -- half the LDS, more resident blocks for these
  // memory-bound shapes
  constexpr int LDS_BYTES = (NSTAGE * STAGE_BYTES > EPI_BYTES ? NSTAGE * STAGE_BYTES : EPI_BYTES);
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
  // This thread's A rows are fixed for the whole K loop.  Plain / strided 1x1:
  // one row pointer each.  Implicit-GEMM conv: the output pixel (n, oh, ow) of
  // each row; the tap of a K tile picks the input pixel (or zero padding).
  const bf16* arow[A_VECS];
  const bf16* arow2[A_VECS];
  int pn[A_VECS], ph[A_VECS], pw[A_VECS];
#pragma unroll
  for (int i = 0; i < A_VECS; ++i) {
    const int row = m0 + r0 + i * ROWS_PER_PASS;
    if constexpr (CONV) {
      if (row < M) {
        const int hw = cv.ho * cv.wo;
        pn[i] = row / hw;
        const int r = row - pn[i] * hw;
        ph[i] = r / cv.wo;
        pw[i] = r - ph[i] * cv.wo;
      } else {
        pn[i] = -1; ph[i] = pw[i] = 0;
      }
    } else {
      arow[i] = row < M ? A + map_row(amap, row) * lda : nullptr;
      arow2[i] = (row < M && p.A2) ? p.A2 + map_row(p.a2map, row) * p.lda2 - p.K1 : nullptr;
    }
  }
  bool aval[A_VECS];

  auto load_tile = [&](int kt) {
    const int k = kt * BK + kv * 8;
    const bool kin = k < K;
    int kch = k;  // channel index of this thread's 8-vector (prologue coefficients)
    int bk = k;   // column of B this 8-vector multiplies (differs only for phase taps)
    if constexpr (CONV) {
      // K = taps * kc with kc % BK == 0: a K tile lies inside one tap
      const int tap = (kt * BK) / cv.kc;
      kch = k - tap * cv.kc;
      int tr, tc;
      if (cv.transposed == 2) {
        tr = cv.ptr[tap];
        tc = cv.ptc[tap];
        bk = (tr * cv.kw + tc) * cv.kc + kch;  // the phase's taps are a subset of the weight's
      } else {
        tr = tap / cv.kw;
        tc = tap - tr * cv.kw;
      }
#pragma unroll
      for (int i = 0; i < A_VECS; ++i) {
        int ih, iw;
        bool ok = kin && pn[i] >= 0;
        if (cv.transposed == 2) {  // exact by construction: (py + pad - tr) % stride == 0
          ih = ph[i] + (cv.py + cv.pad - tr) / cv.stride;
          iw = pw[i] + (cv.px + cv.pad - tc) / cv.stride;
          ok = ok && ih >= 0 && iw >= 0;
        } else if (cv.transposed) {  // data gradient: input pixel (ph, pw) gathers dy at (ph+pad-r)/s
          const int th = ph[i] + cv.pad - tr, tw = pw[i] + cv.pad - tc;
          ih = th / cv.stride;
          iw = tw / cv.stride;
          ok = ok && th >= 0 && tw >= 0 && ih * cv.stride == th && iw * cv.stride == tw;
        } else {
          ih = ph[i] * cv.stride - cv.pad + tr;
          iw = pw[i] * cv.stride - cv.pad + tc;
          ok = ok && ih >= 0 && iw >= 0;
        }
        ok = ok && ih < cv.hi && iw < cv.wi;
        aval[i] = ok;
        if (ok)
          ra[i] = *reinterpret_cast<const bf16x8*>(
              A + (((int64_t)pn[i] * cv.hi + ih) * cv.wi + iw) * lda + kch);
        else
          ra[i] = bf16x8{};
      }
    } else {
      const bool second = p.A2 && k >= p.K1;  // [A | A2] K concatenation
#pragma unroll
      for (int i = 0; i < A_VECS; ++i) {
        aval[i] = kin && arow[i];
        if (aval[i]) ra[i] = *reinterpret_cast<const bf16x8*>((second ? arow2[i] : arow[i]) + k);
        else ra[i] = bf16x8{};
      }
    }
#pragma unroll
    for (int i = 0; i < B_VECS; ++i) {
      const int col = n0 + r0 + i * ROWS_PER_PASS;
      if (kin && col < N) rb[i] = *reinterpret_cast<const bf16x8*>(B + (int64_t)col * ldb + bk);
      else rb[i] = bf16x8{};
    }
    if constexpr (PRO_BN) {
      if (kin) {
        float s[8], t[8];
        {  // 4 x 16-B loads instead of 16 scalar ones (kch is a multiple of 8)
          const f32x4 s0 = *reinterpret_cast<const f32x4*>(pro_s + kch);
          const f32x4 s1 = *reinterpret_cast<const f32x4*>(pro_s + kch + 4);
          const f32x4 t0 = *reinterpret_cast<const f32x4*>(pro_t + kch);
          const f32x4 t1 = *reinterpret_cast<const f32x4*>(pro_t + kch + 4);
#pragma unroll
          for (int j = 0; j < 4; ++j) { s[j] = s0[j]; s[j + 4] = s1[j]; t[j] = t0[j]; t[j + 4] = t1[j]; }
        }
#pragma unroll
        for (int i = 0; i < A_VECS; ++i) {
          f32x8 f = __builtin_convertvector(ra[i], f32x8);
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = fmaxf(fmaf(f[j], s[j], t[j]), 0.f);
          // rows beyond M and zero-padding taps stay exactly zero
          ra[i] = aval[i] ? __builtin_convertvector(f, bf16x8) : bf16x8{};
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
      // operands swapped: acc[i][j] holds the C^T block (lane = output row,
      // registers = 4 consecutive output columns) -> 8-B row pieces in the epilogue
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < ktiles) {
      store_tile(cur ^ 1);
    }
    __syncthreads();
  }

  // ---- epilogue: accumulators -> bf16 tile in LDS (row-major [BM][BN]) ----
  bf16* ct = reinterpret_cast<bf16*>(smem);
  // (the last loop iteration ended with a barrier, staging buffers are free)
  // Per-column affine on the fp32 accumulator before the bf16 staging
  // (EPI_AFFINE scale/shift, EPI_BNBWD's folded-BN constant): a shift that
  // nearly cancels acc must not meet a bf16-rounded acc (finding 33).
  // Transposed accumulators: lane l holds row l & 15 and columns 4 (l >> 4) + e
  // of each 16 x 16 block -> one 8-B LDS write per block (host: N % 8 == 0, so
  // a 4-column group is wholly in or out; coefficient vectors 16-B aligned).
  // Residual / activation are applied in the row-contiguous store pass.
  // every per-column coefficient first, with branch-free loads (an absent
  // vector reads zeros, columns past N read column N - 4, selects pick the
  // defaults): a load under a runtime condition made the compiler wait for
  // each one before the next -- 4-8 dependent round trips per tile.  The
  // BN-backward constants of the store pass go out in the same batch.
  constexpr int CVS = BN / 8;
  const int colb = n0 + (tid % CVS) * 8;
  const int colbc = min(colb, N - 8);
  f32x4 csa[NI], cba[NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int gcc = min(n0 + wn * WTN + j * 16 + (lane >> 4) * 4, N - 4);
    f32x4 cs = {1.f, 1.f, 1.f, 1.f}, cb = {0.f, 0.f, 0.f, 0.f};
    if constexpr (EPI == EPI_AFFINE) {
      const f32x4 sl = *reinterpret_cast<const f32x4*>(epi_s ? epi_s + gcc : g_nt_zero);
      cs = epi_s ? sl : cs;
      cb = *reinterpret_cast<const f32x4*>(epi_t ? epi_t + gcc : g_nt_zero);
    }
    if constexpr (nt_bnbwd(EPI)) cb = *reinterpret_cast<const f32x4*>(p.ebias ? p.ebias + gcc : g_nt_zero);
    csa[j] = cs;
    cba[j] = cb;
  }
  f32x8 bmu8 = {}, biv8 = {}, bw8 = {}, bb8 = {};
  if constexpr (nt_bnbwd(EPI)) {
    bmu8 = *reinterpret_cast<const f32x8*>(p.bmean ? p.bmean + colbc : g_nt_zero);
    if constexpr (EPI == EPI_BNBWD) {
      biv8 = *reinterpret_cast<const f32x8*>(p.binv ? p.binv + colbc : g_nt_zero);
      bw8 = *reinterpret_cast<const f32x8*>(p.bw ? p.bw + colbc : g_nt_zero);
      bb8 = *reinterpret_cast<const f32x8*>(p.bb ? p.bb + colbc : g_nt_zero);
    }
  }
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int lc = wn * WTN + j * 16 + (lane >> 4) * 4;
    const f32x4 cs = csa[j], cb = cba[j];
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int row = wm * WTM + i * 16 + (lane & 15);
      f32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = fmaf(acc[i][j][e], cs[e], cb[e]);
      *reinterpret_cast<bf16x4*>(ct + row * CT_STRIDE + lc) = __builtin_convertvector(v, bf16x4);
    }
  }
  __syncthreads();

  // ---- store pass: each thread moves 8 contiguous columns of a row ----
  constexpr int CV = BN / 8;                  // 16-B vectors per row
  constexpr int RPP = kThreads / CV;          // rows per pass
  const int cvi = tid % CV, rr0 = tid / CV;
  const int col = n0 + cvi * 8;
  const bool col_ok = col < N;
  const bf16* __restrict__ bnx = p.bx;
  const bf16* __restrict__ bny = p.bny;
  const int64_t ldbx = p.ldbx, ldby = p.ldby;
  const CompactMap rmap = p.rmap;
  constexpr bool kMom = EPI == EPI_MOMENTS || nt_bnbwd(EPI);
  static_assert(!kMom || 2 * RPP * BN * 4 <= LDS_BYTES, "moments scratch exceeds LDS");
  float msum[8], msq[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { msum[j] = 0.f; msq[j] = 0.f; }
  float bmu[8], bsc[8], bsh[8];
  if constexpr (nt_bnbwd(EPI)) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      bmu[j] = bmu8[j];
      bsc[j] = EPI == EPI_BNBWD ? biv8[j] * (p.bw ? bw8[j] : 1.f) : 0.f;
      bsh[j] = EPI == EPI_BNBWD ? bb8[j] - bmu[j] * bsc[j] : 0.f;
    }
  }
  // Phase 1 issues every global operand load of the tile's row passes
  // (residual / BN input / BN output), phase 2 computes and stores: loads that
  // sit behind possibly-aliasing stores would keep ~2 per lane in flight
  // (tools/epi_bench.py; same structure as gemm_xl.hip's conv epilogues).
  constexpr int NP = BM / RPP;
  constexpr bool kLR = nt_bnbwd(EPI) || EPI == EPI_AFFINE;
  // branch-free operand loads (dummy row 0 of C when an operand is absent; see gemm_xl.hip)
  const bf16* rbase = R ? R : C;
  const int64_t rld = R ? ldr : 0;
  const bf16* xbase = bnx ? bnx : C;
  const int64_t xld = bnx ? ldbx : 0;
  const bf16* ybase = bny ? bny : C;
  const int64_t yld = bny ? ldby : 0;
  bf16x8 l0[NP], l1[NP], l2[NP];
  unsigned rok = 0;
  const int colc = col_ok ? col : 0;
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int row = min(m0 + rr0 + i * RPP, M - 1);
    if constexpr (kLR) {
      int64_t rr = row;
      if constexpr (nt_bnbwd(EPI)) {
        rr = R ? compact_row(rmap, row) : -1;
        rok |= (rr >= 0 ? 1u : 0u) << i;
        rr = rr >= 0 ? rr : 0;
      }
      l0[i] = *reinterpret_cast<const bf16x8*>(rbase + rr * rld + colc);
    }
    if constexpr (EPI == EPI_BNBWD || EPI == EPI_BNBWD_Y)
      l1[i] = *reinterpret_cast<const bf16x8*>(xbase + (int64_t)row * xld + colc);
    if constexpr (EPI == EPI_BNBWD_Y || EPI == EPI_BNBWD_YO)
      l2[i] = *reinterpret_cast<const bf16x8*>(ybase + (int64_t)row * yld + colc);
  }
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int lr = rr0 + i * RPP;
    const int row = m0 + lr;
    bf16x8 v = *reinterpret_cast<const bf16x8*>(ct + lr * CT_STRIDE + cvi * 8);
    if (row < M && col_ok) {
      if constexpr (EPI == EPI_AFFINE) {  // v = bf16(acc * s + t) (staged)
        f32x8 f = __builtin_convertvector(v, f32x8);
        if (R) f += __builtin_convertvector(l0[i], f32x8);
        if (epi_relu) {
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = fmaxf(f[j], 0.f);
        }
        v = __builtin_convertvector(f, bf16x8);
      }
      if constexpr (nt_bnbwd(EPI)) {
        f32x8 g = __builtin_convertvector(v, f32x8);  // ebias already in (staging)
        if (R) {  // the other branch's gradient, summed in fp32 then rounded once (as "add")
          if ((rok >> i) & 1u) g += __builtin_convertvector(l0[i], f32x8);
          v = __builtin_convertvector(g, bf16x8);
          g = __builtin_convertvector(v, f32x8);
        }
        // bnx null (the BN input was never materialised, ops/bn_fold.py): mask
        // from y, only sum dz is reduced (sum dz*(x-mean) is formed from dz^T a)
        // the operand set is compile-time: EPI_BNBWD = mask from x (run_nt maps
        // any set with y to _Y / _YO), _Y = mask from y with x moments, _YO = y only
        constexpr bool kX = EPI != EPI_BNBWD_YO, kY = EPI != EPI_BNBWD;
        f32x8 xv = {}, yv = {};
        if constexpr (kX) xv = __builtin_convertvector(l1[i], f32x8);
        if constexpr (kY) yv = __builtin_convertvector(l2[i], f32x8);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          bool on;
          if constexpr (kY) on = yv[j] > 0.f;
          else on = fmaf(xv[j], bsc[j], bsh[j]) > 0.f;
          const float dz = on ? g[j] : 0.f;
          g[j] = dz;
          msum[j] += dz;
          if constexpr (kX) msq[j] = fmaf(dz, xv[j] - bmu[j], msq[j]);
        }
        v = __builtin_convertvector(g, bf16x8);  // exact: dz is G or 0
      }
      *reinterpret_cast<bf16x8*>(C + map_row(cmap, row) * ldc + col) = v;
      if constexpr (EPI == EPI_MOMENTS) {
        f32x8 f = __builtin_convertvector(v, f32x8);
#pragma unroll
        for (int j = 0; j < 8; ++j) { msum[j] += f[j]; msq[j] = fmaf(f[j], f[j], msq[j]); }
      }
    }
  }
  if constexpr (kMom) {
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

template <int BM, int BN, int WM, int WN, bool PRO, int EPI, bool CONV>
void launch(const NtArgs& a, hipStream_t stream) {
  const int mtiles = (a.M + BM - 1) / BM, ntiles = (a.N + BN - 1) / BN;
  constexpr int threads = WM * WN * 64;
  if constexpr (!CONV) {
    if (a.K <= BK) {
      hipLaunchKernelGGL((gemm_nt_kernel<BM, BN, WM, WN, PRO, EPI, CONV, 1>), dim3(mtiles * ntiles),
                         dim3(threads), 0, stream, a);
      return;
    }
  }
  hipLaunchKernelGGL((gemm_nt_kernel<BM, BN, WM, WN, PRO, EPI, CONV, 2>), dim3(mtiles * ntiles),
                     dim3(threads), 0, stream, a);
}

// Tile override for experiments (set_gemm_tile; -1 = automatic).
int g_tile_override = -1;
// Strided transposed convs (data gradients) as stride-phase launches (default)
// or the plain zero-tap gather (set_phase_dgrad(false), for A/B runs).
bool g_phase_dgrad = true;
// Wide (128 x 256) TN tiles for deep weight gradients; set_tn_wide for A/B runs.
bool g_tn_wide = true;

template <bool PRO, int EPI, bool CONV>
void dispatch_tile(const NtArgs& a, int bm, hipStream_t s) {
  int t = g_tile_override;
  if (t < 0) t = a.N <= 64 ? (bm == 256 ? 0 : 1) : 2;
  switch (t) {
    case 0: launch<256, 64, 4, 1, PRO, EPI, CONV>(a, s); break;
    case 1: launch<128, 64, 2, 2, PRO, EPI, CONV>(a, s); break;
    case 3: launch<128, 64, 4, 1, PRO, EPI, CONV>(a, s); break;
    case 4: launch<64, 128, 2, 2, PRO, EPI, CONV>(a, s); break;
    case 5: launch<64, 64, 2, 2, PRO, EPI, CONV>(a, s); break;
    case 6: launch<256, 128, 4, 2, PRO, EPI, CONV>(a, s); break;
    default: launch<128, 128, 2, 2, PRO, EPI, CONV>(a, s); break;
  }
}

// M tile of the selected variant (moments partial rows = M tiles)
int tile_bm(int N, int bm) {
  int t = g_tile_override;
  if (t < 0) t = N <= 64 ? (bm == 256 ? 0 : 1) : 2;
  switch (t) {
    case 0: return 256;
    case 4: case 5: return 64;
    case 6: return 256;
    default: return 128;
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
  // ds_read_b64_tr_b16 banks per 32-lane half: lanes l and l+16 read rows r
  // and r+8, which must land on different banks (MI355X_MICROARCH.md §LDS).
  // 256-/512-B rows: the +4*(row>>3) term moves rows 8-15 to the other half of
  // the chunk range; 128-B rows (4 chunks, rows q and q+2 already share a bank
  // half) need an XOR with bit 3 of the row instead.
  const int byte = col * 2;
  const int mask = (row_bytes >> 5) - 1;
  const int f = mask == 3 ? ((row & 3) ^ ((row >> 3) & 1)) : ((row + 4 * (row >> 3)) & mask);
  const int chunk = (byte >> 5) ^ f;
  return row * row_bytes + (chunk << 5) + (byte & 31);
}

// PRO_B: B' = relu(B * s[k] + t[k]) applied while staging B (the weight
// gradient of a conv whose input is a BN+ReLU output that was never
// materialised -- ops/fused.py bn_relu_conv1x1).
template <int BNT, int BKT, bool PRO_B, int MINB = 2>
__global__ __launch_bounds__(kThreads, MINB) void gemm_tn_kernel(
    const bf16* __restrict__ A, int64_t lda, const bf16* __restrict__ B, int64_t ldb, int M, int N,
    int K, int64_t rows_per_split, float* __restrict__ part, ConvMap bmap,
    const float* __restrict__ bps, const float* __restrict__ bpt) {
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
  // XCD-aware order: the ntiles*ktiles output tiles of one M split are
  // consecutive logical ids on ONE XCD and run together, so the dy rows they
  // all stream (and, for a 3x3 wgrad, the neighbouring taps' x rows) come
  // from that XCD's L2 instead of HBM once per tile.
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = bid % (ntiles * ktiles);
  const int split = bid / (ntiles * ktiles);
  const int n0 = (tile / ktiles) * BNT, k0 = (tile % ktiles) * BKT;
  const int64_t mb = (int64_t)split * rows_per_split;
  const int64_t me = min((int64_t)M, mb + rows_per_split);
  const int nstages = (int)((me - mb + TN_BM - 1) / TN_BM);
  // implicit-GEMM wgrad: K = taps * kc, this block's K tile lies in one tap
  int tr = 0, tc = 0, kc0 = k0;
  if (bmap.kc != 0) {
    const int tap = k0 / bmap.kc;
    tr = tap / bmap.kw;
    tc = tap - tr * bmap.kw;
    kc0 = k0 - tap * bmap.kc;
  }

  __shared__ __attribute__((aligned(16))) float pro_lds[PRO_B ? 2 * BKT : 4];
  if constexpr (PRO_B) {
    const int kb = bmap.kc == 0 ? k0 : kc0;
    for (int j = threadIdx.x; j < BKT; j += kThreads) {
      const bool in = k0 + j < K;
      pro_lds[j] = in ? bps[kb + j] : 0.f;
      pro_lds[BKT + j] = in ? bpt[kb + j] : 0.f;
    }
    __syncthreads();
  }
  bf16x8 ra[A_VECS], rb[B_VECS];
  auto load = [&](int s) {
    const int64_t m0 = mb + (int64_t)s * TN_BM;
#pragma unroll
    for (int i = 0; i < A_VECS; ++i) {
      const int v = tid + i * kThreads, r = v / A_VPR, c = (v % A_VPR) * 8;
      const int64_t m = m0 + r;
      int64_t am = m;
      if (bmap.amap) {  // physical pixel (n, oh*s, ow*s)
        const int hw = bmap.ho * bmap.wo;
        const int n = (int)(m / hw);
        const int rr = (int)(m - (int64_t)n * hw);
        const int oh = rr / bmap.wo, ow = rr - oh * bmap.wo;
        am = ((int64_t)n * bmap.hi + oh * bmap.stride) * bmap.wi + ow * bmap.stride;
      }
      ra[i] = (m < me && n0 + c < N) ? *reinterpret_cast<const bf16x8*>(A + am * lda + n0 + c) : bf16x8{};
    }
#pragma unroll
    for (int i = 0; i < B_VECS; ++i) {
      const int v = tid + i * kThreads, r = v / B_VPR, c = (v % B_VPR) * 8;
      const int64_t m = m0 + r;
      const bf16* src = nullptr;
      if (m < me && k0 + c < K) {
        if (bmap.kc == 0) {
          src = B + m * ldb + k0 + c;
        } else {  // conv input pixel feeding output pixel m through tap (tr, tc), or padding
          const int hw = bmap.ho * bmap.wo;
          const int n = (int)(m / hw);
          const int rr = (int)(m - (int64_t)n * hw);
          const int oh = rr / bmap.wo, ow = rr - oh * bmap.wo;
          const int ih = oh * bmap.stride - bmap.pad + tr, iw = ow * bmap.stride - bmap.pad + tc;
          if (ih >= 0 && iw >= 0 && ih < bmap.hi && iw < bmap.wi)
            src = B + (((int64_t)n * bmap.hi + ih) * bmap.wi + iw) * ldb + kc0 + c;
        }
      }
      rb[i] = src ? *reinterpret_cast<const bf16x8*>(src) : bf16x8{};
      if constexpr (PRO_B) {
        if (src) {  // coefficients of this 8-vector's channels, staged in LDS once per block
          const f32x4 s0 = *reinterpret_cast<const f32x4*>(pro_lds + c);
          const f32x4 s1 = *reinterpret_cast<const f32x4*>(pro_lds + c + 4);
          const f32x4 t0 = *reinterpret_cast<const f32x4*>(pro_lds + BKT + c);
          const f32x4 t1 = *reinterpret_cast<const f32x4*>(pro_lds + BKT + c + 4);
          f32x8 f = __builtin_convertvector(rb[i], f32x8);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            f[j] = fmaxf(fmaf(f[j], s0[j], t0[j]), 0.f);
            f[j + 4] = fmaxf(fmaf(f[j + 4], s1[j], t1[j]), 0.f);
          }
          rb[i] = __builtin_convertvector(f, bf16x8);
        }
      }
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
                                                           int64_t n, int sl, OT* __restrict__ out, int acc) {
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
    for (int e = 0; e < 4; ++e) out[i + e] = (OT)(acc ? a[e] + (float)out[i + e] : a[e]);
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
               int splits, int64_t rps, const ConvMap& bm, const float* bps, const float* bpt,
               hipStream_t s) {
  const int tiles = ((N + BNT - 1) / BNT) * ((K + BKT - 1) / BKT);
  // the 128 x 256 tile holds 128 accumulator VGPRs per lane and 96 KB of LDS: 1 block/CU
  constexpr int MINB = BKT * BNT > 128 * 128 ? 1 : 2;
  if constexpr (MINB == 1) {
    TORCH_CHECK(bps == nullptr, "wide TN tile has no B prologue variant");
    hipLaunchKernelGGL((gemm_tn_kernel<BNT, BKT, false, 1>), dim3(tiles * splits), dim3(kThreads), 0, s,
                       reinterpret_cast<const bf16*>(A.data_ptr()), A.stride(0),
                       reinterpret_cast<const bf16*>(B.data_ptr()), B.stride(0), M, N, K, rps, part,
                       bm, nullptr, nullptr);
  } else if (bps) {
    hipLaunchKernelGGL((gemm_tn_kernel<BNT, BKT, true>), dim3(tiles * splits), dim3(kThreads), 0, s,
                       reinterpret_cast<const bf16*>(A.data_ptr()), A.stride(0),
                       reinterpret_cast<const bf16*>(B.data_ptr()), B.stride(0), M, N, K, rps, part,
                       bm, bps, bpt);
  } else {
    hipLaunchKernelGGL((gemm_tn_kernel<BNT, BKT, false>), dim3(tiles * splits), dim3(kThreads), 0, s,
                       reinterpret_cast<const bf16*>(A.data_ptr()), A.stride(0),
                       reinterpret_cast<const bf16*>(B.data_ptr()), B.stride(0), M, N, K, rps, part,
                       bm, nullptr, nullptr);
  }
}

}  // namespace

void split_reduce_launch(const float* pp, int splits, int64_t n, at::Tensor& out, hipStream_t stream,
                         bool acc = false);
at::Tensor acc_target(const c10::optional<at::Tensor>& out, int64_t numel, at::ScalarType dtype,
                      const char* who);

namespace {

// C[N, K] = sum_m A[m, :]^T Bmapped[m, :]  -> out [N, K] (bf16 or fp32); with
// `acc` (a contiguous [N, K] gradient) the split reduce adds into it instead
at::Tensor run_tn(const at::Tensor& A, const at::Tensor& B, int M, int N, int K,
                  at::ScalarType out_dtype, const ConvMap& bmap, int kgran,
                  const float* bps = nullptr, const float* bpt = nullptr, at::Tensor acc = at::Tensor()) {
  auto stream = at::hip::getCurrentHIPStream();
  auto out = acc.defined() ? acc : at::empty({N, K}, A.options().dtype(out_dtype));
  if (M == 0) return acc.defined() ? out : out.zero_();
  // 128 x 256 output tiles (1 block/CU) halve the L2 re-reads of A (dy) for deep
  // implicit-GEMM weight gradients (K = taps * Cin, Cin % 256 == 0): g_tn_wide
  const bool wide = g_tn_wide && bps == nullptr && N >= 128 && K >= 256 && kgran % 256 == 0;
  // (256-row split-M tiles for N >= 256, K <= 128 measured slower and were
  // removed in round 6: profiles/README.md finding 58)
  const int bnt = N >= 128 ? 128 : 64;
  const int bkt = wide ? 256 : ((K >= 128 && kgran % 128 == 0) ? 128 : 64);
  const int tiles = ((N + bnt - 1) / bnt) * ((K + bkt - 1) / bkt);
  // ~4 blocks per CU, but keep the fp32 partial traffic well under the operand
  // traffic (the GEMM streams (N+K)*M bf16; partials cost 2 * splits*N*K*4 B).
  const int max_splits = std::max(1, (M + TN_BM - 1) / TN_BM);
  const int64_t operand_bytes = (int64_t)M * (N + K) * 2;
  const int64_t part_cap = std::max<int64_t>(operand_bytes / 4, 8 << 20);
  const int by_bytes = (int)std::max<int64_t>(1, part_cap / ((int64_t)N * K * 8));
  // at least ~2 blocks per CU even when that exceeds the byte budget (big N*K
  // with few tiles would otherwise leave most of the 256 CUs idle)
  const int fill = (512 + tiles - 1) / tiles, target = (1024 + tiles - 1) / tiles;
  int splits = std::min(max_splits, std::max({1, fill, std::min(by_bytes, target)}));
  int64_t rps = ((int64_t)M + splits - 1) / splits;
  rps = (rps + TN_BM - 1) / TN_BM * TN_BM;
  splits = (int)(((int64_t)M + rps - 1) / rps);
  auto part = at::empty({splits, N, K}, A.options().dtype(at::kFloat));
  float* pp = part.data_ptr<float>();
  if (bkt == 256) launch_tn<128, 256>(A, B, M, N, K, pp, splits, rps, bmap, bps, bpt, stream);
  else if (bnt == 128 && bkt == 128) launch_tn<128, 128>(A, B, M, N, K, pp, splits, rps, bmap, bps, bpt, stream);
  else if (bnt == 128) launch_tn<128, 64>(A, B, M, N, K, pp, splits, rps, bmap, bps, bpt, stream);
  else if (bkt == 128) launch_tn<64, 128>(A, B, M, N, K, pp, splits, rps, bmap, bps, bpt, stream);
  else launch_tn<64, 64>(A, B, M, N, K, pp, splits, rps, bmap, bps, bpt, stream);
  split_reduce_launch(pp, splits, (int64_t)N * K, out, stream, acc.defined());
  return out;
}

}  // namespace

// The gradient buffer a weight-gradient kernel accumulates into (pipeline
// micro-batch accumulation, ops/grad_accum.py): contiguous, the parameter's
// dtype, the gradient's element count.
at::Tensor acc_target(const c10::optional<at::Tensor>& out, int64_t numel, at::ScalarType dtype,
                      const char* who) {
  if (!out.has_value() || !out->defined()) return at::Tensor();
  TORCH_CHECK(out->is_cuda() && out->scalar_type() == dtype && out->numel() == numel &&
                  reinterpret_cast<uintptr_t>(out->data_ptr()) % 16 == 0 &&
                  (out->is_contiguous() || out->is_contiguous(at::MemoryFormat::ChannelsLast)),
              who, ": the accumulation target must be a 16-B aligned dense gradient of the output dtype and size");
  return *out;
}

// out[c] = sum over splits of part[s][c] (c < n, n % 4 == 0), bf16 or fp32 out
// (acc: out[c] += ..., one read-modify-write per element, no extra launch).
void split_reduce_launch(const float* pp, int splits, int64_t n, at::Tensor& out, hipStream_t stream, bool acc) {
  int sl = 1;  // split lanes per column: grow until >= 512 blocks or lanes cover the splits
  while (sl < 64 && sl < splits && (n / 4 + 256 / sl - 1) / (256 / sl) < 512) sl *= 2;
  const unsigned blocks = (unsigned)((n / 4 + 256 / sl - 1) / (256 / sl));
  if (out.scalar_type() == at::kBFloat16)
    hipLaunchKernelGGL((split_reduce_kernel<bf16>), dim3(blocks), dim3(256), 0, stream, pp, splits, n,
                       sl, reinterpret_cast<bf16*>(out.data_ptr()), (int)acc);
  else
    hipLaunchKernelGGL((split_reduce_kernel<float>), dim3(blocks), dim3(256), 0, stream, pp, splits, n,
                       sl, out.data_ptr<float>(), (int)acc);
}

// Weight gradient of a 1x1 conv: C[N, K] = A^T B with A [M, N], B [M, K] (bf16,
// row-major).  Output dtype bf16 or fp32.  b_map ([s, Ho, Wo, Hi, Wi]) reads
// B's logical row m from the strided physical row (stride-s 1x1 conv input).
at::Tensor gemm_tn(const at::Tensor& A, const at::Tensor& B, at::ScalarType out_dtype,
                   const std::vector<int64_t>& b_map, const c10::optional<at::Tensor>& pro_scale,
                   const c10::optional<at::Tensor>& pro_shift, bool a_mapped,
                   const c10::optional<at::Tensor>& out) {
  check_operand(A, "A");
  check_operand(B, "B");
  const RowMap rm = parse_map(b_map, "b_map");
  ConvMap cm;  // kc == 0: identity rows
  TORCH_CHECK(!a_mapped || rm.s != 1, "a_mapped needs a strided b_map");
  if (rm.s == 1) {
    TORCH_CHECK(A.size(0) == B.size(0), "A/B M mismatch");
  } else if (a_mapped) {  // Gram of a strided sample: A and B rows both through the map
    TORCH_CHECK(A.size(0) == B.size(0) && B.size(0) % ((int64_t)rm.hi * rm.wi) == 0,
                "a_mapped: A and B are the same physical rows");
    cm.kw = 1; cm.stride = rm.s; cm.pad = 0;
    cm.hi = rm.hi; cm.wi = rm.wi; cm.ho = rm.ho; cm.wo = rm.wo;
    cm.kc = (int)B.size(1);
    cm.amap = 1;
  } else {
    TORCH_CHECK(B.size(0) % ((int64_t)rm.hi * rm.wi) == 0 &&
                    A.size(0) == B.size(0) / ((int64_t)rm.hi * rm.wi) * rm.ho * rm.wo,
                "b_map does not match the A/B row counts");
    cm.kw = 1; cm.stride = rm.s; cm.pad = 0;
    cm.hi = rm.hi; cm.wi = rm.wi; cm.ho = rm.ho; cm.wo = rm.wo;
    cm.kc = (int)B.size(1);
  }
  const int M = cm.amap ? (int)(B.size(0) / ((int64_t)rm.hi * rm.wi) * rm.ho * rm.wo) : (int)A.size(0);
  const int N = (int)A.size(1), K = (int)B.size(1);
  TORCH_CHECK(N % 8 == 0 && K % 8 == 0, "N and K must be multiples of 8");
  const float* bps = nullptr;
  const float* bpt = nullptr;
  if (pro_scale.has_value() && pro_scale->defined()) {
    TORCH_CHECK(pro_shift.has_value() && pro_shift->defined() && pro_scale->numel() == K &&
                    pro_shift->numel() == K && pro_scale->scalar_type() == at::kFloat &&
                    pro_shift->scalar_type() == at::kFloat,
                "B prologue needs fp32 scale and shift of length K");
    bps = pro_scale->data_ptr<float>();
    bpt = pro_shift->data_ptr<float>();
  }
  return run_tn(A, B, M, N, K, out_dtype, cm, 128, bps, bpt, acc_target(out, (int64_t)N * K, out_dtype, "gemm_tn"));
}

// Weight gradient of an implicit-GEMM conv: dy [N*Ho*Wo, Cout] rows, x NHWC
// [N, Hi, Wi, Cin] -> dW [Cout, kh*kw*Cin] (channels_last weight memory).
at::Tensor conv_wgrad(const at::Tensor& dy, const at::Tensor& x, int64_t kh, int64_t kw,
                      int64_t stride, int64_t pad, int64_t ho, int64_t wo,
                      at::ScalarType out_dtype, int64_t kc, const c10::optional<at::Tensor>& out) {
  check_operand(dy, "dy");
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "x must be a channels_last bf16 GPU tensor");
  const int64_t nb = x.size(0), cin = x.size(1);
  const int64_t kcv = kc > 0 ? kc : cin;  // > cin: row taps over kc/cin consecutive pixels (conv_nt)
  if (kc > 0) {
    TORCH_CHECK(kcv % cin == 0 && stride == 1 && pad == 0 && (wo - 1) + (kw - 1) + kcv / cin - 1 < x.size(3) &&
                    (ho - 1) + (kh - 1) < x.size(2),
                "row-tap conv_wgrad: kc must be a multiple of Cin, stride 1, pad 0, taps inside the input");
  }
  TORCH_CHECK(kcv % 64 == 0, "conv_wgrad needs channels per tap % 64 == 0");
  TORCH_CHECK(dy.size(0) == nb * ho * wo, "dy rows must be N*Ho*Wo");
  TORCH_CHECK(dy.size(1) % 8 == 0, "output channels must be a multiple of 8");
  ConvMap cm;
  cm.kw = (int)kw; cm.stride = (int)stride; cm.pad = (int)pad;
  cm.hi = (int)x.size(2); cm.wi = (int)x.size(3); cm.ho = (int)ho; cm.wo = (int)wo;
  cm.kc = (int)kcv;
  const int M = (int)dy.size(0), N = (int)dy.size(1), K = (int)(kh * kw * kcv);
  // B rows are addressed through the map; ldb = Cin (pixel stride)
  auto xv = x.permute({0, 2, 3, 1}).reshape({-1, cin});
  return run_tn(dy, xv, M, N, K, out_dtype, cm, (int)(kcv % 128 == 0 ? 128 : 64), nullptr, nullptr,
                acc_target(out, (int64_t)N * K, out_dtype, "conv_wgrad"));
}

namespace {

template <bool CONV>
void dispatch_mode(const NtArgs& a, bool pro, int epi, int bm, hipStream_t s) {
  if (epi == EPI_STORE) {
    if (pro) dispatch_tile<true, EPI_STORE, CONV>(a, bm, s);
    else dispatch_tile<false, EPI_STORE, CONV>(a, bm, s);
  } else if (epi == EPI_MOMENTS) {
    if (pro) dispatch_tile<true, EPI_MOMENTS, CONV>(a, bm, s);
    else dispatch_tile<false, EPI_MOMENTS, CONV>(a, bm, s);
  } else if (nt_bnbwd(epi)) {
    TORCH_CHECK(!pro, "bnbwd epilogue has no prologue variant");
    if (epi == EPI_BNBWD_Y) dispatch_tile<false, EPI_BNBWD_Y, CONV>(a, bm, s);
    else if (epi == EPI_BNBWD_YO) dispatch_tile<false, EPI_BNBWD_YO, CONV>(a, bm, s);
    else dispatch_tile<false, EPI_BNBWD, CONV>(a, bm, s);
  } else {
    if (pro) dispatch_tile<true, EPI_AFFINE, CONV>(a, bm, s);
    else dispatch_tile<false, EPI_AFFINE, CONV>(a, bm, s);
  }
}

// Shared tail of gemm_nt / conv_nt: prologue / epilogue arguments, launch,
// moments reduction.  a.A/B/C, M/N/K and the maps are already set.
std::vector<at::Tensor> run_nt(NtArgs a, bool conv, const at::Tensor& like,
                               const c10::optional<at::Tensor>& pro_scale,
                               const c10::optional<at::Tensor>& pro_shift, const std::string& mode,
                               const c10::optional<at::Tensor>& epi_scale,
                               const c10::optional<at::Tensor>& epi_shift,
                               const c10::optional<at::Tensor>& residual, bool relu,
                               at::Tensor C) {
  auto stream = at::hip::getCurrentHIPStream();
  const bool pro = pro_scale.has_value() && pro_scale->defined();
  if (pro) {
    TORCH_CHECK(pro_shift.has_value() && pro_shift->defined(), "prologue needs scale and shift");
    TORCH_CHECK(pro_scale->scalar_type() == at::kFloat && pro_shift->scalar_type() == at::kFloat,
                "prologue coefficients must be fp32");
  }
  a.pro_s = pro ? pro_scale->data_ptr<float>() : nullptr;
  if (pro)
    TORCH_CHECK(reinterpret_cast<uintptr_t>(pro_scale->data_ptr()) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(pro_shift->data_ptr()) % 16 == 0,
                "prologue coefficients must be 16-B aligned");
  a.pro_t = pro ? pro_shift->data_ptr<float>() : nullptr;
  at::Tensor moments;
  if (a.M == 0) return {C, moments};
  const int bm = tile_m_for(a.N);
  const int tbm = tile_bm(a.N, bm);
  int epi = EPI_STORE;
  at::Tensor part;
  if (mode == "store") {
  } else if (mode == "moments" || mode == "bnbwd") {
    epi = mode == "moments" ? EPI_MOMENTS : EPI_BNBWD;
    TORCH_CHECK(epi != EPI_BNBWD || a.bx || a.bny, "bnbwd needs bn_x or bn_y (gemm_nt_bnbwd)");
    if (epi == EPI_BNBWD && a.bny) epi = a.bx ? EPI_BNBWD_Y : EPI_BNBWD_YO;
    if (nt_bnbwd(epi) && residual.has_value() && residual->defined()) {
      check_operand(*residual, "residual");
      const int64_t rrows = a.rmap.s == 1 ? a.M
                                          : (int64_t)a.M / ((int64_t)a.rmap.hi * a.rmap.wi) * a.rmap.ho * a.rmap.wo;
      TORCH_CHECK(residual->size(0) == rrows && residual->size(1) == a.N, "residual shape");
      a.R = reinterpret_cast<const bf16*>(residual->data_ptr());
      a.ldr = residual->stride(0);
    }
    const int mtiles = (a.M + tbm - 1) / tbm;
    part = at::empty({2, mtiles, a.N}, like.options().dtype(at::kFloat));
    a.part = part.data_ptr<float>();
    moments = at::empty({2 * (int64_t)a.N + 1}, like.options().dtype(at::kDouble));
    a.zsums = moments_zero_target(moments.data_ptr<double>(), mtiles);
  } else if (mode == "affine" || mode == "add") {
    epi = EPI_AFFINE;
    if (mode == "affine") {
      const bool hs = epi_scale.has_value() && epi_scale->defined();
      const bool ht = epi_shift.has_value() && epi_shift->defined();
      TORCH_CHECK(hs || ht, "affine epilogue needs scale and/or shift (missing = 1 / 0)");
      for (const auto* t : {&epi_scale, &epi_shift})
        if (t->has_value() && (*t)->defined())
          TORCH_CHECK((*t)->scalar_type() == at::kFloat && (*t)->is_contiguous() && (*t)->numel() == a.N &&
                          reinterpret_cast<uintptr_t>((*t)->data_ptr()) % 16 == 0,
                      "affine coefficients must be contiguous 16-B aligned fp32 [N]");
      a.epi_s = hs ? epi_scale->data_ptr<float>() : nullptr;
      a.epi_t = ht ? epi_shift->data_ptr<float>() : nullptr;
    } else {
      TORCH_CHECK(residual.has_value() && residual->defined(), "add epilogue needs a residual");
    }
    if (residual.has_value() && residual->defined()) {
      check_operand(*residual, "residual");
      TORCH_CHECK(residual->size(0) == a.M && residual->size(1) == a.N, "residual shape");
      a.R = reinterpret_cast<const bf16*>(residual->data_ptr());
      a.ldr = residual->stride(0);
    }
    a.epi_relu = relu;
  } else {
    TORCH_CHECK(false, "unknown epilogue mode ", mode);
  }
  if (conv) dispatch_mode<true>(a, pro, epi, bm, stream);
  else dispatch_mode<false>(a, pro, epi, bm, stream);
  if (epi == EPI_MOMENTS || nt_bnbwd(epi))
    bn_reduce_partials_launch(a.part, (a.M + tbm - 1) / tbm, a.N, moments.data_ptr<double>(),
                              (double)a.M, stream);
  return {C, moments};
}

}  // namespace

namespace {
// [A | A2] along K: A2 [rows(A), K2] row-major; the GEMM's K becomes K(A) + K2.
void set_second_source(NtArgs& a, const at::Tensor& A, const c10::optional<at::Tensor>& a2,
                       const std::vector<int64_t>& a2_map) {
  if (!(a2.has_value() && a2->defined())) return;
  check_operand(*a2, "a2");
  a.a2map = parse_map(a2_map, "a2_map");
  const RowMap& m = a.a2map;
  const int64_t rows = m.s == 1 ? a2->size(0) : a2->size(0) / ((int64_t)m.hi * m.wi) * m.ho * m.wo;
  TORCH_CHECK(m.s == 1 || a2->size(0) % ((int64_t)m.hi * m.wi) == 0, "a2_map does not match a2's rows");
  TORCH_CHECK(rows == a.M && a2->size(1) % 8 == 0, "a2 must be [GEMM rows (through a2_map), K2], K2 % 8 == 0");
  a.A2 = reinterpret_cast<const bf16*>(a2->data_ptr());
  a.lda2 = a2->stride(0);
  a.K1 = a.K;
  a.K += (int)a2->size(1);
}
}  // namespace

// C = prologue(A) @ B^T with an optional fused epilogue.  Returns (C, moments-or-undefined).
//   A [M, K] bf16, B [N, K] bf16 (both K-contiguous), K % 8 == 0, N % 8 == 0.
//   pro_scale/pro_shift [K] fp32: A' = relu(A*s + t)
//   mode "store" | "moments" (returns fp64 [2N+1] = (sum, sumsq, M)) | "affine"
//   (epi_scale/epi_shift [N], optional residual [M, N], relu flag) | "add"
//   (C = acc + residual).
//   a_map / c_map: [s, Ho, Wo, Hi, Wi] strided row maps for A reads / C writes.
//   a2: optional second A source, [A | a2] concatenated along K (B is [N, K + K2]).
std::vector<at::Tensor> gemm_nt(const at::Tensor& A, const at::Tensor& B,
                                const c10::optional<at::Tensor>& pro_scale,
                                const c10::optional<at::Tensor>& pro_shift, const std::string& mode,
                                const c10::optional<at::Tensor>& epi_scale,
                                const c10::optional<at::Tensor>& epi_shift,
                                const c10::optional<at::Tensor>& residual, bool relu,
                                const std::vector<int64_t>& a_map,
                                const std::vector<int64_t>& c_map,
                                const c10::optional<at::Tensor>& a2,
                                const std::vector<int64_t>& a2_map) {
  check_operand(A, "A");
  check_operand(B, "B");
  NtArgs a{};
  a.amap = parse_map(a_map, "a_map");
  a.cmap = parse_map(c_map, "c_map");
  TORCH_CHECK(a.cmap.s == 1 || !(residual.has_value() && residual->defined()),
              "a residual epilogue cannot be combined with a strided c_map");
  const RowMap& am = a.amap;
  const RowMap& cm = a.cmap;
  int64_t m64 = A.size(0);
  if (am.s != 1) {
    TORCH_CHECK(m64 % ((int64_t)am.hi * am.wi) == 0, "a_map does not match A's rows");
    m64 = m64 / ((int64_t)am.hi * am.wi) * am.ho * am.wo;
  }
  a.M = (int)m64;
  a.K = (int)A.size(1);
  a.N = (int)B.size(0);
  set_second_source(a, A, a2, a2_map);
  TORCH_CHECK(B.size(1) == a.K, "A/B K mismatch");
  TORCH_CHECK(a.K % 8 == 0 && a.N % 8 == 0, "K and N must be multiples of 8");
  TORCH_CHECK(!a.A2 || !(pro_scale.has_value() && pro_scale->defined()), "a2 has no prologue variant");
  if (pro_scale.has_value() && pro_scale->defined())
    TORCH_CHECK(pro_scale->numel() == a.K, "prologue coefficients must have K entries");
  at::Tensor C;
  if (cm.s == 1) {
    C = at::empty({a.M, a.N}, A.options());
  } else {
    // rows the strided scatter does not reach are exactly zero (dgrad of a strided 1x1 conv)
    TORCH_CHECK(a.M % ((int64_t)cm.ho * cm.wo) == 0, "c_map does not match the GEMM rows");
    C = at::zeros({(int64_t)a.M / ((int64_t)cm.ho * cm.wo) * cm.hi * cm.wi, a.N}, A.options());
  }
  a.A = reinterpret_cast<const bf16*>(A.data_ptr());
  a.lda = A.stride(0);
  a.B = reinterpret_cast<const bf16*>(B.data_ptr());
  a.ldb = B.stride(0);
  a.C = reinterpret_cast<bf16*>(C.data_ptr());
  a.ldc = C.stride(0);
  return run_nt(a, false, A, pro_scale, pro_shift, mode, epi_scale, epi_shift, residual, relu, C);
}

// Implicit-GEMM convolution on NHWC bf16 activations (kh x kw taps, any
// stride / padding), MFMA NT kernel with the tap gather in the A staging:
//   x    [N, Hi, Wi, Cin] (rows of Cin, channels_last memory)
//   wmat [Cout, kh*kw*Cin] (channels_last weight memory: [Cout][kh][kw][Cin])
//   -> y [N*Ho*Wo, Cout] (+ moments / affine epilogue like gemm_nt).
// transposed=true computes the data gradient of a conv with geometry
// (stride, pad): x is dy on the (hi, wi) grid, the output grid (ho, wo) is the
// conv input, wmat is [Cin][kh][kw][Cout] (weight permuted, not flipped).
// Cin % 64 == 0 (a K tile of 64 never straddles two taps).
std::vector<at::Tensor> conv_nt(const at::Tensor& x, const at::Tensor& wmat, int64_t kh,
                                int64_t kw, int64_t stride, int64_t pad, int64_t ho, int64_t wo,
                                bool transposed,
                                const c10::optional<at::Tensor>& pro_scale,
                                const c10::optional<at::Tensor>& pro_shift,
                                const std::string& mode,
                                const c10::optional<at::Tensor>& epi_scale,
                                const c10::optional<at::Tensor>& epi_shift,
                                const c10::optional<at::Tensor>& residual, bool relu,
                                int64_t kc) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4,
              "x must be a 4-D bf16 GPU tensor");
  TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast), "x must be channels_last");
  check_operand(wmat, "wmat");
  const int64_t nb = x.size(0), cin = x.size(1), hi = x.size(2), wi = x.size(3);
  // kc > cin: ROW TAPS -- tap (r, c) reads kc / cin CONSECUTIVE pixels starting at
  // (oh + r, ow + c) as one kc-channel operand (the pixels are adjacent in NHWC
  // memory, overlapping between neighbouring outputs).  Lets a few-channel
  // input (the ResNet stem after space-to-depth: 16 channels) run on the
  // 64-deep K tiles: a 4x4 kernel becomes 4 row taps of 64.
  const int64_t kcv = kc > 0 ? kc : cin;
  if (kc > 0) {
    TORCH_CHECK(!transposed && kcv % cin == 0 && stride == 1 && pad == 0 &&
                    (wo - 1) + (kw - 1) + kcv / cin - 1 < wi && (ho - 1) + (kh - 1) < hi,
                "row-tap conv_nt: kc must be a multiple of Cin, stride 1, pad 0, taps inside the input");
  }
  TORCH_CHECK(kcv % BK == 0, "conv_nt needs channels per tap % 64 == 0");
  TORCH_CHECK(wmat.size(1) == kh * kw * kcv, "wmat must be [Cout, kh*kw*kc]");
  TORCH_CHECK(wmat.size(0) % 8 == 0, "output channels must be a multiple of 8");
  TORCH_CHECK(ho > 0 && wo > 0 && stride >= 1 && pad >= 0, "bad conv geometry");
  if (pro_scale.has_value() && pro_scale->defined())
    TORCH_CHECK(pro_scale->numel() == cin, "prologue coefficients must have Cin entries");
  if (transposed && stride > 1 && g_phase_dgrad && mode == "store" &&
      !(pro_scale.has_value() && pro_scale->defined())) {
    TORCH_CHECK(kh * kw <= 16, "phase dgrad supports up to 16 taps");
    // dx [N*ho*wo, Cout'] written phase by phase: every row exactly once
    auto C = at::empty({nb * ho * wo, wmat.size(0)}, x.options());
    for (int py = 0; py < stride; ++py)
      for (int px = 0; px < stride; ++px) {
        const int64_t ha = (ho - py + stride - 1) / stride, wa = (wo - px + stride - 1) / stride;
        if (ha <= 0 || wa <= 0) continue;
        NtArgs a{};
        int nt = 0;
        for (int r = 0; r < kh; ++r)
          for (int c = 0; c < kw; ++c)
            if ((py + pad - r) % stride == 0 && (px + pad - c) % stride == 0) {
              a.cv.ptr[nt] = (int8_t)r;
              a.cv.ptc[nt] = (int8_t)c;
              ++nt;
            }
        if (nt == 0) {  // no tap reaches this phase: its dx rows are zero
          C.view({nb, ho, wo, -1}).slice(1, py, ho, stride).slice(2, px, wo, stride).zero_();
          continue;
        }
        a.cv.kw = (int)kw; a.cv.stride = (int)stride; a.cv.pad = (int)pad;
        a.cv.hi = (int)hi; a.cv.wi = (int)wi; a.cv.ho = (int)ha; a.cv.wo = (int)wa;
        a.cv.kc = (int)cin; a.cv.transposed = 2; a.cv.py = py; a.cv.px = px;
        a.cmap.s = (int)stride; a.cmap.ho = (int)ha; a.cmap.wo = (int)wa;
        a.cmap.hi = (int)ho; a.cmap.wi = (int)wo; a.cmap.oy = py; a.cmap.ox = px;
        a.M = (int)(nb * ha * wa);
        a.N = (int)wmat.size(0);
        a.K = nt * (int)cin;
        a.A = reinterpret_cast<const bf16*>(x.data_ptr());
        a.lda = cin;
        a.B = reinterpret_cast<const bf16*>(wmat.data_ptr());
        a.ldb = wmat.stride(0);
        a.C = reinterpret_cast<bf16*>(C.data_ptr());
        a.ldc = C.stride(0);
        run_nt(a, true, x, pro_scale, pro_shift, mode, epi_scale, epi_shift, residual, relu, C);
      }
    return {C, at::Tensor()};
  }
  NtArgs a{};
  a.cv.kw = (int)kw;
  a.cv.stride = (int)stride;
  a.cv.pad = (int)pad;
  a.cv.hi = (int)hi;
  a.cv.wi = (int)wi;
  a.cv.ho = (int)ho;
  a.cv.wo = (int)wo;
  a.cv.kc = (int)kcv;
  a.cv.transposed = transposed;
  TORCH_CHECK(nb * ho * wo < (1LL << 31), "too many output pixels");
  a.M = (int)(nb * ho * wo);
  a.N = (int)wmat.size(0);
  a.K = (int)(kh * kw * kcv);
  auto C = at::empty({a.M, a.N}, x.options());
  a.A = reinterpret_cast<const bf16*>(x.data_ptr());
  a.lda = cin;
  a.B = reinterpret_cast<const bf16*>(wmat.data_ptr());
  a.ldb = wmat.stride(0);
  a.C = reinterpret_cast<bf16*>(C.data_ptr());
  a.ldc = C.stride(0);
  return run_nt(a, true, x, pro_scale, pro_shift, mode, epi_scale, epi_shift, residual, relu, C);
}

// Data gradient of a 1x1 conv whose input is a training-mode BN(+residual)+ReLU
// output, fused with that BN's backward reductions (EPI_BNBWD):
//   G  = bf16(A @ B^T (+ residual))          A = dy [M, K], B = W^T [N, K]
//   dz = G * mask,  mask = y > 0 (bn_y given) or x*sc + sh > 0 with
//        sc = invstd * weight, sh = bias - mean * sc (weight / bias optional)
//   returns (dz [M, N], fp64 [2N+1] = (sum dz, sum dz*(x - mean), M))
CompactMap parse_compact(const std::vector<int64_t>& g, int64_t M) {
  CompactMap c;
  if (g.empty()) return c;
  TORCH_CHECK(g.size() == 5, "res_map must be [stride, Ho, Wo, Hi, Wi]");
  c.s = (int)g[0]; c.ho = (int)g[1]; c.wo = (int)g[2]; c.hi = (int)g[3]; c.wi = (int)g[4];
  TORCH_CHECK(c.s >= 1 && c.ho == (c.hi + c.s - 1) / c.s && c.wo == (c.wi + c.s - 1) / c.s &&
                  M % ((int64_t)c.hi * c.wi) == 0,
              "res_map does not describe a stride-s subsampling of the GEMM rows");
  return c;
}

std::vector<at::Tensor> gemm_nt_bnbwd(const at::Tensor& A, const at::Tensor& B,
                                      const c10::optional<at::Tensor>& residual,
                                      const c10::optional<at::Tensor>& bn_x,
                                      const c10::optional<at::Tensor>& bn_y,
                                      const c10::optional<at::Tensor>& mean,
                                      const c10::optional<at::Tensor>& invstd,
                                      const c10::optional<at::Tensor>& weight,
                                      const c10::optional<at::Tensor>& bias,
                                      const std::vector<int64_t>& res_map,
                                      const c10::optional<at::Tensor>& a2,
                                      const c10::optional<at::Tensor>& ebias,
                                      const std::vector<int64_t>& a2_map) {
  check_operand(A, "A");
  check_operand(B, "B");
  const bool has_x = bn_x.has_value() && bn_x->defined();
  const bool has_y = bn_y.has_value() && bn_y->defined();
  TORCH_CHECK(has_x || has_y, "bnbwd needs the BN input x and/or output y");
  NtArgs a{};
  a.rmap = parse_compact(res_map, A.size(0));
  a.M = (int)A.size(0);
  a.K = (int)A.size(1);
  a.N = (int)B.size(0);
  set_second_source(a, A, a2, a2_map);
  TORCH_CHECK(B.size(1) == a.K, "A/B K mismatch");
  TORCH_CHECK(a.K % 8 == 0 && a.N % 8 == 0, "K and N must be multiples of 8");
  auto f32vec = [&](const at::Tensor& t, const char* name) {
    TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous() && t.numel() == a.N &&
                    reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0,
                name, " must be a contiguous 16-B aligned fp32 [N] GPU tensor");
    return t.data_ptr<float>();
  };
  if (has_x) {
    check_operand(*bn_x, "bn_x");
    TORCH_CHECK(bn_x->size(0) == a.M && bn_x->size(1) == a.N, "bn_x must be [M, N]");
    a.bx = reinterpret_cast<const bf16*>(bn_x->data_ptr());
    a.ldbx = bn_x->stride(0);
    TORCH_CHECK(mean.has_value() && mean->defined(), "sum dz*(x-mean) needs the BN mean");
    a.bmean = f32vec(*mean, "mean");
  }
  if (ebias.has_value() && ebias->defined()) a.ebias = f32vec(*ebias, "ebias");
  if (has_y) {
    check_operand(*bn_y, "bn_y");
    TORCH_CHECK(bn_y->size(0) == a.M && bn_y->size(1) == a.N, "bn_y must be [M, N]");
    a.bny = reinterpret_cast<const bf16*>(bn_y->data_ptr());
    a.ldby = bn_y->stride(0);
  } else {
    TORCH_CHECK(invstd.has_value() && invstd->defined(), "mask from x needs the BN invstd");
    a.binv = f32vec(*invstd, "invstd");
    if (weight.has_value() && weight->defined()) a.bw = f32vec(*weight, "weight");
    if (bias.has_value() && bias->defined()) a.bb = f32vec(*bias, "bias");
  }
  auto C = at::empty({a.M, a.N}, A.options());
  a.A = reinterpret_cast<const bf16*>(A.data_ptr());
  a.lda = A.stride(0);
  a.B = reinterpret_cast<const bf16*>(B.data_ptr());
  a.ldb = B.stride(0);
  a.C = reinterpret_cast<bf16*>(C.data_ptr());
  a.ldc = C.stride(0);
  return run_nt(a, false, A, c10::nullopt, c10::nullopt, "bnbwd", c10::nullopt, c10::nullopt, residual,
                false, C);
}

void set_gemm_tile(int64_t t) { g_tile_override = (int)t; }
void set_phase_dgrad(bool on) { g_phase_dgrad = on; }
void set_tn_wide(bool on) { g_tn_wide = on; }

}  // namespace dmp
