// Large-tile MFMA bf16 GEMM for the transformer linears (ViT-B/16 qkv / proj /
// fc1 / fc2 in forward and data-gradient form), with fused epilogues.
//
//   C[M, N] = epi( A[M, K] * B[N, K]^T )        (both operands K-contiguous)
//
// Forward of nn.Linear: A = x [T, in], B = W [out, in].  Data gradient:
// A = dy [T, out], B = W^T [in, out] (a 4.7 MB transposed copy of W per step).
//
// Epilogues (what hipBLASLt + separate torch kernels would do in 2-3 passes):
//   XL_STORE     C = bf16(acc)
//   XL_BIAS      C = bf16(acc + b[n])
//   XL_BIAS_GELU Aux = bf16(acc + b[n]);  C = bf16(gelu(Aux))     (fc1 forward)
//   XL_DGELU     C = bf16(bf16(acc) * gelu'(Aux))                  (fc2 dgrad ->
//                the gradient at fc1's pre-activation: no GELU-backward pass)
//   XL_BIAS_RES  C = bf16(bf16(acc + b[n]) + R)                    (proj / fc2
//                forward + residual add)
// Rounding points match the unfused torch sequence (addmm -> bf16 -> gelu).
//
// Structure (cdna_hip_programming.md §5 "256² template" and T1-T5):
//   * 256 x BN tile (BN = 256 or 128), BK = 64, 512 threads = 8 waves as
//     2 (M) x 4 (N); each wave owns 128 x BN/4 outputs = 8 x BN/64 16x16
//     accumulators (v_mfma_f32_16x16x32_bf16);
//   * operands staged global -> LDS by global_load_lds_dwordx4 (no VGPR
//     round trip); the LDS image is lane-linear, so the bank swizzle is applied
//     to the per-lane SOURCE address and undone on the ds_read (rule 21);
//   * every K tile is split into two k32 halves living in their own LDS
//     regions ([A|B] x [k0|k1] x 2 buffers = 128 KB at BN = 256); one K tile is
//     4 phases (k-half x M-half of the wave tile, 16 / 8 MFMAs each), and each
//     phase issues the global->LDS copy of one region as soon as that region's
//     previous contents were consumed: the k0 halves of tile t+2 are issued
//     while tile t computes its k1 half, so ~5 phases of loads stay in flight
//     across the barriers (counted s_waitcnt vmcnt, raw s_barrier -- never
//     __syncthreads, whose fence would drain the DMA queue);
//   * one raw s_barrier per phase; the region written in phase p was last read
//     before the previous phase's barrier (WAR), and a region is read one phase
//     after the vmcnt that retired it (RAW);
//   * bijective XCD-aware block remap (T1); the N tiles of an M tile are
//     adjacent (they share the A panel in L2);
//   * epilogue restages the tile through LDS for 16-B row-contiguous stores.
#include <cstdlib>
#include <torch/extension.h>
#include <type_traits>
#include <ATen/hip/HIPContext.h>
#include "../common.h"

namespace dmp {
namespace {

using bf16 = __bf16;
constexpr int XBM = 256, XBK = 64, XTHREADS = 512;

enum XlEpi { XL_STORE = 0, XL_BIAS = 1, XL_BIAS_GELU = 2, XL_DGELU = 3, XL_BIAS_RES = 4,
             // conv epilogues (same semantics as gemm_bf16.hip's EPI_MOMENTS /
             // EPI_AFFINE "add" / EPI_BNBWD), for the wide 1x1 conv GEMMs
             XL_MOMENTS = 5, XL_ADD = 6, XL_BNBWD = 7,
             // C = act(acc * s[n] + t[n] (+ R)): conv + training-mode BN (+ residual)
             // + ReLU when the BN statistics were formed before the GEMM (ops/bn_fold.py)
             XL_AFFINE = 8,
             // XL_BNBWD with its operand set fixed at compile time (the runtime
             // flags cost the epilogue ~2x the VALU of the moments epilogue):
             // mask from y with x moments / mask from y, no x
             XL_BNBWD_Y = 9, XL_BNBWD_YO = 10 };
__host__ __device__ constexpr bool is_bnbwd(int e) { return e == XL_BNBWD || e == XL_BNBWD_Y || e == XL_BNBWD_YO; }

using gptr_t = const __attribute__((address_space(1))) void*;
using lptr_t = __attribute__((address_space(3))) void*;

__device__ __forceinline__ void glds16(const void* g, char* l) {
  __builtin_amdgcn_global_load_lds((gptr_t)g, (lptr_t)l, 16, 0, 0);
}

// Exact-GELU pieces for the epilogues: Phi(x) via erf(|x|/sqrt2) from
// Abramowitz-Stegun 7.1.26 (|error| <= 1.5e-7, far below the bf16 output's
// 2^-9 relative rounding) and phi(x) from the SAME exponential, since
// exp(-z^2) with z = x/sqrt2 is exp(-x^2/2).  ~12 VALU ops against erff's
// ~40: the epilogue runs after the MFMA loop at 1 block/CU, so its VALU time
// is not hidden (libm erff made the fused fc1 epilogue cost more than the
// separate GELU pass it replaces).
__device__ __forceinline__ void gelu_parts(float x, float& cdf, float& pdf) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.f));
  const float e = __expf(-z * z);
  const float poly =
      fmaf(fmaf(fmaf(fmaf(1.061405429f, t, -1.453152027f), t, 1.421413741f), t, -0.284496736f), t, 0.254829592f) * t;
  const float erf_abs = fmaf(-poly, e, 1.f);
  cdf = 0.5f + 0.5f * copysignf(erf_abs, x);
  pdf = 0.39894228040143268f * e;
}
__device__ __forceinline__ float gelu_f(float x) {
  float c, d;
  gelu_parts(x, c, d);
  return x * c;
}
__device__ __forceinline__ float gelu_grad_f(float x) {
  float c, d;
  gelu_parts(x, c, d);
  return fmaf(x, d, c);
}

// 16-B chunk swizzle of a k32 region (rows of 64 B = 4 chunks, 4 rows per
// 256-B bank row).  ds_read_b128 is serviced in four 16-lane groups
// {0-3,12-15,20-27}, {4-11,16-19,28-31} and their +32 images
// (MI355X_MICROARCH.md §LDS); an MFMA fragment read has lane l on row l & 15,
// chunk l >> 4, so each group holds rows {0-3,12-15} of one chunk and rows
// 4-11 of the neighbouring chunk.  XOR-ing the chunk with g(row >> 2) for
// g = {0, 2, 3, 1} gives every group 16 distinct bank slots (a plain
// XOR with row >> 2 leaves 2-way conflicts: rows 0-3 and 4-7 collide).
__device__ __forceinline__ int chunk_xor(int q) { return (0x78 >> (2 * (q & 3))) & 3; }

// Tile order: bijective XCD remap (consecutive logical ids share an XCD and
// run concurrently), then groups of GM M-tiles walked column by column, so
// the ~32 tiles resident on one XCD form a GM x 32/GM patch whose A and B
// panels are both reused from that XCD's L2.
__device__ __forceinline__ void tile_coords_id(int bid, int mtiles, int ntiles, int gm_max, int& mt, int& nt) {
  const int per_group = gm_max * ntiles;
  const int g = bid / per_group, r = bid - g * per_group;
  const int gm = min(gm_max, mtiles - g * gm_max);
  mt = g * gm_max + r % gm;
  nt = r / gm;
}
__device__ __forceinline__ void tile_coords(int nblocks, int mtiles, int ntiles, int gm_max,
                                            int& mt, int& nt) {
  const int bid = xcd_remap(blockIdx.x, nblocks);
  const int per_group = gm_max * ntiles;
  const int g = bid / per_group, r = bid - g * per_group;
  const int gm = min(gm_max, mtiles - g * gm_max);
  mt = g * gm_max + r % gm;
  nt = r / gm;
}

template <int N>
__device__ __forceinline__ void vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// s_waitcnt vmcnt(n) for a wave-uniform runtime n in {0, 2, .., MAX} (the
// immediate must be a constant): a chain of scalar compares, steady state first
template <int MAX>
__device__ __forceinline__ void vmcnt_upto(int n) {
  if constexpr (MAX <= 0) {
    vmcnt<0>();
  } else {
    if (n >= MAX) vmcnt<MAX>();
    else vmcnt_upto<MAX - 2>(n);
  }
}

__device__ __forceinline__ void barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Implicit-GEMM convolution view of the A operand (PIPE 7 only): GEMM row m
// is output pixel (n, oh, ow) of an NHWC input [N, Hi, Wi, cin]; K tile kt
// is channels c0..c0+63 of tap (tr, tc), K = taps * cin.  cin == 0: plain GEMM.
struct XlConv {
  int cin = 0, hi = 0, wi = 0, ho = 0, wo = 0, stride = 1, pad = 0, kw = 1;
};

// Output row map (XL_STORE only): GEMM row m = (n, oh, ow) of an ho x wo grid
// is written to row (n, s*oh + oy, s*ow + ox) of an hi x wi image -- one
// stride phase of a strided conv's data gradient.  s == 1: identity.
struct XlOutMap {
  int s = 1, ho = 1, wo = 1, hi = 1, wi = 1, oy = 0, ox = 0;
};
__device__ __forceinline__ int64_t xl_out_row(const XlOutMap& g, int row) {
  if (g.s == 1) return row;
  const int hw = g.ho * g.wo;
  const int n = row / hw, r = row - n * hw;
  const int oh = r / g.wo, ow = r - oh * g.wo;
  return ((int64_t)n * g.hi + oh * g.s + g.oy) * g.wi + ow * g.s + g.ox;
}

// 16-B reads of padding taps land here (LDS-DMA cannot write zeros itself).
__device__ __attribute__((aligned(16))) bf16 g_zero_row[128] = {};

struct XlArgs {
  const bf16* A; int64_t lda;
  const bf16* B; int64_t ldb;
  bf16* C; int64_t ldc;
  int M, N, K;
  const bf16* bias;             // [N] (XL_BIAS*)
  bf16* aux; int64_t ldaux;     // XL_BIAS_GELU: pre-activation out; XL_DGELU: pre-activation in
  const bf16* R; int64_t ldr;   // XL_BIAS_RES / XL_ADD / XL_BNBWD residual (optional for BNBWD)
  int group_m;                  // tile-order group height (M tiles)
  float* part;                  // XL_MOMENTS / XL_BNBWD partials [2][mtiles][N]
  double* zsums;                // moments target to zero (common.h) or null
  const bf16* bx; int64_t ldbx; // XL_BNBWD: BN input x [M, N]
  const bf16* bny; int64_t ldby;// XL_BNBWD: BN output y [M, N] (mask source) or null
  const float *bmean, *binv, *bw, *bb;  // mask affine as in gemm_bf16.hip EPI_BNBWD
  CompactMap rmap;              // XL_BNBWD residual in compact stride-s form
  XlConv cv;                    // implicit-GEMM conv gather of A (PIPE 7)
  XlOutMap omap;                // C row map (XL_STORE)
  // second A source (plain GEMM): K columns k >= K1 come from A2[row, k - K1]
  // (the [dz | a] operand of a BN-folded data gradient); K1 % 64 == 0
  const bf16* A2; int64_t lda2; int K1;
  XlOutMap a2m;                 // A2 rows through a strided map (x_s of a folded downsample)
  const float* ebias;           // XL_BNBWD: per-column constant added to the GEMM output
  const float *esc, *esh;       // XL_AFFINE coefficients (null: 1 / 0)
  int erelu;                    // XL_AFFINE ReLU
  // rows per tile of the PIPE 7 kernel (0 = 256): 192..240 trims the tile so
  // that an MFMA-bound grid fills whole 1-block/CU rounds (pick_bm)
  int bm;
  // diagnostics (set_gemm_xl_trace): per block [entry, operands landed, main
  // loop done, epilogue done] in 10-ns ticks, HW_ID, XCC_ID; null = off
  unsigned long long* tdbg;
};

__device__ __forceinline__ void xl_mark(const XlArgs& p, int k) {
  if (p.tdbg && threadIdx.x == 0) p.tdbg[(int64_t)blockIdx.x * 8 + k] = __builtin_amdgcn_s_memrealtime();
}

// Epilogue of the NT kernel (and of a split-K tail tile, gemm_xl_tail_epi):
// (acc [+ bias]) -> bf16 tile in LDS, then the row-contiguous pass with the
// fused operation; acc in the PIPE's register layout (7 / 8: transposed).
// PIPE 11 (gemm_xl_w4_kernel): 4 waves as 2 x 2, 128 x 128 outputs per wave,
// 256 threads in the row passes; every other PIPE: 8 waves as 2 x 4
__host__ __device__ constexpr int xl_waves(int pipe) { return pipe == 11 ? 4 : 8; }
template <int BN, int PIPE>
using XlAcc = f32x4[8][xl_waves(PIPE) == 4 ? BN / 32 : BN / 64];

// WMB (PIPE 11): 16-row blocks per wave actually computed (7: 224-row tile,
// wave row 1 starts at row 112; acc[7][*] unused).  WWN (PIPE 11): waves along
// N (1: four waves stacked along M over a BN = 128 tile)
template <int BN, int EPI, int PIPE, int LDS, int WMB = 8, int WWN = 2, typename ACC>
__device__ __forceinline__ void xl_epilogue(const XlArgs& p, ACC& acc, char* smem, int m0, int n0,
                                            int mt, int mtiles, int tbm = XBM) {
  constexpr int NW = xl_waves(PIPE), XTHREADS = NW * 64;
  constexpr int WTM = 16 * WMB, WTN = NW == 4 ? BN / WWN : BN / 4;
  constexpr int MI = WTM / 16, NI = WTN / 16;
  static_assert((WMB == 8 && WWN == 2) || PIPE == 11, "trimmed wave tiles: 4-wave kernel only");
  constexpr int CT_STRIDE = BN + 8;
  constexpr bool kMom = EPI == XL_MOMENTS || is_bnbwd(EPI) || EPI == XL_DGELU;
  // rows of this tile: [m0, min(M, m0 + tbm)); a trimmed tile's staged rows
  // past tbm belong to the next tile and are neither stored nor summed
  const int M = min(p.M, m0 + tbm), N = p.N;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = NW == 4 ? (WWN == 2 ? wave >> 1 : wave) : wave >> 2;
  const int wc = NW == 4 ? (WWN == 2 ? wave & 1 : 0) : wave & 3;
  (void)lane;
  // ---- batched epilogue operand loads (residual / BN input / BN output / aux).
  // Row passes of RPP rows; batch b covers passes [b PB, b PB + PB).  The
  // first batch goes out BEFORE the accumulator staging below and every later
  // batch one batch ahead of its use, so a whole tile's operand rows are in
  // flight through the epilogue instead of one batch at a time (finding 66:
  // the residual epilogue was ~10 us of an 18-20 us short-K tile, its two
  // batches each a full HBM round trip).
  constexpr int CV = BN / 8, RPP = XTHREADS / CV;
  const int cvi = tid % CV, rr0 = tid / CV;
  const int col = n0 + cvi * 8;
  constexpr bool kBatch = is_bnbwd(EPI) || EPI == XL_ADD || EPI == XL_AFFINE || EPI == XL_BIAS_RES ||
                          EPI == XL_DGELU;
  constexpr bool kL0 = kBatch;
  constexpr bool kL12 = is_bnbwd(EPI);
  constexpr bool kLx = EPI == XL_BNBWD || EPI == XL_BNBWD_Y, kLy = EPI == XL_BNBWD_Y || EPI == XL_BNBWD_YO;
  constexpr int NT = (kL0 ? 1 : 0) + (kLx ? 1 : 0) + (kLy ? 1 : 0);
  constexpr int NP = kBatch ? XBM / RPP : 0;
  constexpr int PB = NT >= 3 ? 2 : NT == 2 ? 4 : 8;  // two batches in flight: 2 PB NT 16-B loads per lane
  constexpr int NB = kBatch ? NP / PB : 1;
  // operand bases for branch-free loads: a missing operand reads a valid
  // dummy row (row 0 of C / of itself), its value is never used -- a
  // per-load branch would split every load into its own block, and the
  // compiler then waits for each one before the next (measured: the
  // forward affine epilogue kept exactly one load per lane in flight)
  const bf16* rsrc = EPI == XL_DGELU ? p.aux : p.R;  // GELU' reads the pre-activation
  const bf16* rbase = rsrc ? rsrc : p.C;
  const int64_t rld = rsrc ? (EPI == XL_DGELU ? p.ldaux : p.ldr) : 0;
  const bf16* xbase = p.bx ? p.bx : p.C;
  const int64_t xld = p.bx ? p.ldbx : 0;
  const bf16* ybase = p.bny ? p.bny : p.C;
  const int64_t yld = p.bny ? p.ldby : 0;
  // row pointers advance by a uniform RPP-row step (no per-row 64-bit
  // multiply); a row past M reads row 0 of the same operand instead
  // loads are issued by every lane (a load under a branch makes the compiler
  // drain the whole batch at the join): lanes past N read column N - 8
  const int coll = min(col, N - 8);
  const bf16* rrow = rbase + (int64_t)(m0 + rr0) * rld + coll;
  const int64_t rstep = (int64_t)RPP * rld;
  const bf16* xrow = xbase + (int64_t)(m0 + rr0) * xld + coll;
  const bf16* yrow = ybase + (int64_t)(m0 + rr0) * yld + coll;
  const int64_t xstep = (int64_t)RPP * xld, ystep = (int64_t)RPP * yld;
  bf16x8 L0[NB][PB], L1[NB][PB], L2[NB][PB];
  unsigned rok[NB];  // bit i: row pass b PB + i has a residual row (compact map)
  auto issue = [&](const int b) {
    rok[b] = 0;
#pragma unroll
    for (int i = 0; i < PB; ++i) {
      const int pass = b * PB + i;
      const int row_u = m0 + rr0 + pass * RPP;
      const int row = min(row_u, M - 1);
      if constexpr (kL0) {
        const bf16x8* rp;
        if constexpr (is_bnbwd(EPI)) {
          int64_t rr = p.R ? compact_row(p.rmap, row) : -1;
          rok[b] |= (rr >= 0 ? 1u : 0u) << i;
          rr = rr >= 0 ? rr : 0;
          rp = reinterpret_cast<const bf16x8*>(rbase + rr * rld + coll);
        } else {
          rp = reinterpret_cast<const bf16x8*>(row_u < M ? rrow + pass * rstep : rbase + coll);
        }
        L0[b][i] = *rp;
      }
      if constexpr (kL12) {
        if constexpr (kLx) L1[b][i] = *reinterpret_cast<const bf16x8*>(row_u < M ? xrow + pass * xstep : xbase + coll);
        if constexpr (kLy) L2[b][i] = *reinterpret_cast<const bf16x8*>(row_u < M ? yrow + pass * ystep : ybase + coll);
      }
    }
  };
  // BN-backward column constants, loaded ahead of everything else (branch-free:
  // an absent operand reads the zero row, a select picks the default)
  float bmu[8], bsc[8], bsh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) bmu[j] = bsc[j] = bsh[j] = 0.f;
  if constexpr (is_bnbwd(EPI)) {
    const float* zf0 = reinterpret_cast<const float*>(g_zero_row);
    const f32x8 mu = *reinterpret_cast<const f32x8*>(p.bmean ? p.bmean + coll : zf0);
    f32x8 iv = {}, ww = {}, bb = {};
    if constexpr (EPI == XL_BNBWD) {
      iv = *reinterpret_cast<const f32x8*>(p.binv ? p.binv + coll : zf0);
      ww = *reinterpret_cast<const f32x8*>(p.bw ? p.bw + coll : zf0);
      bb = *reinterpret_cast<const f32x8*>(p.bb ? p.bb + coll : zf0);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      bmu[j] = mu[j];
      if constexpr (EPI == XL_BNBWD) {
        bsc[j] = iv[j] * (p.bw ? ww[j] : 1.f);
        bsh[j] = bb[j] - bmu[j] * bsc[j];
      }
    }
  }
  bf16* ct = reinterpret_cast<bf16*>(smem);
  // per-column affine applied to the fp32 accumulator BEFORE the bf16 staging:
  // a bias / BN shift that nearly cancels acc (XL_BNBWD's folded-BN constant,
  // XL_AFFINE's -mean*scale) must not meet a bf16-rounded acc (finding 33)
  if constexpr (PIPE == 10 || PIPE == 11) {
    // transposed accumulators (see quad()): lane l holds row l & 15 and the 4
    // consecutive columns 4 (l >> 4) + e of each 16 x 16 block -> one 8-B LDS
    // write per block (a half-wave covers 16 rows x 16 B at a 528-B row pitch:
    // all 64 banks once) instead of four 2-B writes
    // the per-column coefficients first, then the first operand batch: a use
    // of a load waits for everything issued before it (in-order vmcnt), so
    // coefficients loaded after the batch would drain it before the staging
    // (branch-free as the batch: absent coefficients read the zero row,
    // columns past N read column N - 4, and selects pick the defaults)
    f32x4 s4a[NI], b4a[NI];
    const float* zf = reinterpret_cast<const float*>(g_zero_row);
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int colj = min(n0 + wc * WTN + j * 16 + (lane >> 4) * 4, N - 4);  // N % 8 == 0
      f32x4 s4 = {1.f, 1.f, 1.f, 1.f}, b4 = {0.f, 0.f, 0.f, 0.f};
      if constexpr (EPI == XL_BIAS || EPI == XL_BIAS_GELU || EPI == XL_BIAS_RES) {
#pragma unroll
        for (int e = 0; e < 4; ++e) b4[e] = (float)p.bias[colj + e];  // a bias view may be 2-B aligned only
      }
      if constexpr (is_bnbwd(EPI))
        b4 = *reinterpret_cast<const f32x4*>(p.ebias ? p.ebias + colj : zf);
      if constexpr (EPI == XL_AFFINE) {
        const f32x4 sl = *reinterpret_cast<const f32x4*>(p.esc ? p.esc + colj : zf);
        s4 = p.esc ? sl : s4;
        b4 = *reinterpret_cast<const f32x4*>(p.esh ? p.esh + colj : zf);
      }
      s4a[j] = s4;
      b4a[j] = b4;
    }
    __builtin_amdgcn_sched_barrier(0);  // keep the coefficient loads ahead of the batch
    // (4 waves: the 256 accumulators are still live here and the batch would
    // spill; it goes out after the staging instead)
    if constexpr (kBatch && NW == 8) issue(0);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int lc = wc * WTN + j * 16 + (lane >> 4) * 4;
      const f32x4 s4 = s4a[j], b4 = b4a[j];
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int row = wr * WTM + i * 16 + (lane & 15);
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaf(acc[i][j][e], s4[e], b4[e]);
        *reinterpret_cast<bf16x4*>(ct + row * CT_STRIDE + lc) = __builtin_convertvector(v, bf16x4);
      }
    }
    if constexpr (kBatch && NW == 4) issue(0);
  } else {
  float bv[NI], sv[NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int col = n0 + wc * WTN + j * 16 + (lane & 15);
    bv[j] = 0.f;
    sv[j] = 1.f;
    if constexpr (EPI == XL_BIAS || EPI == XL_BIAS_GELU || EPI == XL_BIAS_RES)
      bv[j] = col < N ? (float)p.bias[col] : 0.f;
    if constexpr (is_bnbwd(EPI))
      bv[j] = (col < N && p.ebias) ? p.ebias[col] : 0.f;
    if constexpr (EPI == XL_AFFINE) {
      sv[j] = (col < N && p.esc) ? p.esc[col] : 1.f;
      bv[j] = (col < N && p.esh) ? p.esh[col] : 0.f;
    }
  }
  if constexpr (kBatch) issue(0);
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int col = wc * WTN + j * 16 + (lane & 15);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = wr * WTM + i * 16 + (lane >> 4) * 4 + e;
        ct[row * CT_STRIDE + col] = (bf16)fmaf(acc[i][j][e], sv[j], bv[j]);
      }
    }
  }
  __syncthreads();
  float msum[8], msq[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { msum[j] = 0.f; msq[j] = 0.f; }
  if (col < N) {
    // Epilogue in batches of PB row passes (issued above / one batch ahead):
    // the loads must not sit behind the batch's stores -- C may alias them for
    // all the compiler knows, so a load-compute-store loop keeps ~2 loads per
    // lane in flight (measured 2.2-3.1 TB/s on the short-K conv epilogues at 1
    // block/CU, tools/epi_bench.py).  The load-free epilogues keep the
    // row-at-a-time loop below.
    bf16* const crow = p.C + (int64_t)(m0 + rr0) * p.ldc + col;
    const int64_t cstep = (int64_t)RPP * p.ldc;
    // XL_AFFINE without a residual still loads (a dummy row of C: branch-free
    // batch) and masks the bits to +0 instead of branching around the add
    const unsigned rmask = p.R ? 0xffffffffu : 0u;
    (void)rmask;
    if constexpr (kBatch) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      if (b + 1 < NB) issue(b + 1);
#pragma unroll
      for (int i = 0; i < PB; ++i) {
        const int lr = rr0 + (b * PB + i) * RPP;
        const int row = m0 + lr;
        if (row >= M) continue;
        bf16x8 v = *reinterpret_cast<const bf16x8*>(ct + lr * CT_STRIDE + cvi * 8);
        if constexpr (EPI == XL_MOMENTS) {
          const f32x8 f = __builtin_convertvector(v, f32x8);
#pragma unroll
          for (int j = 0; j < 8; ++j) { msum[j] += f[j]; msq[j] = fmaf(f[j], f[j], msq[j]); }
        } else if constexpr (EPI == XL_ADD || EPI == XL_BIAS_RES) {
          f32x8 f = __builtin_convertvector(v, f32x8);
          f += __builtin_convertvector(L0[b][i], f32x8);
          v = __builtin_convertvector(f, bf16x8);
        } else if constexpr (EPI == XL_AFFINE) {  // v = bf16(acc * s + t) (staged)
          f32x8 f = __builtin_convertvector(v, f32x8);
          u32x4 rb = __builtin_bit_cast(u32x4, L0[b][i]);
          rb &= rmask;
          f += __builtin_convertvector(__builtin_bit_cast(bf16x8, rb), f32x8);
          if (p.erelu) {
#pragma unroll
            for (int j = 0; j < 8; ++j) f[j] = fmaxf(f[j], 0.f);
          }
          v = __builtin_convertvector(f, bf16x8);
        } else if constexpr (is_bnbwd(EPI)) {
          f32x8 g = __builtin_convertvector(v, f32x8);  // ebias already in (staging)
          if (p.R) {  // the other branch's gradient: summed in fp32, rounded once (as XL_ADD)
            if ((rok[b] >> i) & 1u) g += __builtin_convertvector(L0[b][i], f32x8);
            v = __builtin_convertvector(g, bf16x8);
            g = __builtin_convertvector(v, f32x8);
          }
          // bx null: BN input never materialised (ops/bn_fold.py) -- mask from y, sum dz only.
          // XL_BNBWD keeps the operand set a runtime choice (the x2 kernel's
          // contract); _Y / _YO fix it: mask from y, with / without x moments
          constexpr bool kY = EPI != XL_BNBWD, kX = EPI != XL_BNBWD_YO;
          f32x8 xv = {}, yv = {};
          if constexpr (kLx) xv = __builtin_convertvector(L1[b][i], f32x8);
          if constexpr (kLy) yv = __builtin_convertvector(L2[b][i], f32x8);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            // (xl_conv_run maps an operand set with y to _Y / _YO: plain
            // XL_BNBWD here always has x and no y)
            bool on;
            if constexpr (kY) on = yv[j] > 0.f;
            else on = fmaf(xv[j], bsc[j], bsh[j]) > 0.f;
            const float dz = on ? g[j] : 0.f;
            g[j] = dz;
            msum[j] += dz;
            if constexpr (kX) msq[j] = fmaf(dz, xv[j] - bmu[j], msq[j]);
          }
          v = __builtin_convertvector(g, bf16x8);
        } else if constexpr (EPI == XL_BIAS_GELU) {
          *reinterpret_cast<bf16x8*>(p.aux + (int64_t)row * p.ldaux + col) = v;
          f32x8 f = __builtin_convertvector(v, f32x8);
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = gelu_f(f[j]);
          v = __builtin_convertvector(f, bf16x8);
        } else if constexpr (EPI == XL_DGELU) {
          f32x8 f = __builtin_convertvector(v, f32x8);
          const f32x8 x = __builtin_convertvector(L0[b][i], f32x8);
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] *= gelu_grad_f(x[j]);
          v = __builtin_convertvector(f, bf16x8);
          const f32x8 fv = __builtin_convertvector(v, f32x8);  // the stored dh, as a column sum reads it
#pragma unroll
          for (int j = 0; j < 8; ++j) msum[j] += fv[j];
        }
        static_assert(!kBatch || EPI != XL_STORE, "batched epilogues write C rows unmapped");
        bf16x8* cp = reinterpret_cast<bf16x8*>(crow + (b * PB + i) * cstep);
        *cp = v;
      }
    }
    }
    if constexpr (!kBatch) {
#pragma unroll 8
      for (int pr = 0; pr < XBM / RPP; ++pr) {
        const int lr = rr0 + pr * RPP;
        const int row = m0 + lr;
        if (row >= M) continue;
        bf16x8 v = *reinterpret_cast<const bf16x8*>(ct + lr * CT_STRIDE + cvi * 8);
        if constexpr (EPI == XL_MOMENTS) {
          const f32x8 f = __builtin_convertvector(v, f32x8);
#pragma unroll
          for (int j = 0; j < 8; ++j) { msum[j] += f[j]; msq[j] = fmaf(f[j], f[j], msq[j]); }
        } else if constexpr (EPI == XL_BIAS_GELU) {
          *reinterpret_cast<bf16x8*>(p.aux + (int64_t)row * p.ldaux + col) = v;
          f32x8 f = __builtin_convertvector(v, f32x8);
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = gelu_f(f[j]);
          v = __builtin_convertvector(f, bf16x8);
        }
        const int64_t orow = EPI == XL_STORE ? xl_out_row(p.omap, row) : (int64_t)row;
        bf16x8* cp = reinterpret_cast<bf16x8*>(p.C + orow * p.ldc + col);
        *cp = v;
      }
    }
  }
  if (kMom && (EPI != XL_DGELU || p.part)) {
    // fold the RPP row groups of each column through LDS: one partial per M tile
    static_assert(2 * RPP * BN * 4 <= LDS, "moments scratch exceeds LDS");
    __syncthreads();  // every thread finished reading the C tile
    float* red = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[(0 * RPP + rr0) * BN + cvi * 8 + j] = msum[j];
      red[(1 * RPP + rr0) * BN + cvi * 8 + j] = msq[j];
    }
    __syncthreads();
    for (int c = tid; c < BN; c += XTHREADS) {
      float s0 = 0.f, q0 = 0.f;
      for (int g = 0; g < RPP; ++g) {
        s0 += red[(0 * RPP + g) * BN + c];
        q0 += red[(1 * RPP + g) * BN + c];
      }
      if (n0 + c < N) {
        p.part[(int64_t)mt * N + n0 + c] = s0;
        p.part[(int64_t)(mtiles + mt) * N + n0 + c] = q0;
      }
    }
  }
}

template <int BN, int EPI, int PIPE>
__global__ __launch_bounds__(XTHREADS, 1) void gemm_xl_nt_kernel(const XlArgs p) {
  constexpr int WTM = 128, WTN = BN / 4;
  constexpr int MI = WTM / 16, NI = WTN / 16;       // 8 x (4 | 2) accumulators
  constexpr int RA = XBM * 64, RB = BN * 64;        // bytes of one k32 region
  constexpr int NA = RA / 1024 / 8, NB = RB / 1024 / 8;  // glds per wave per region
  constexpr int STAGE_LDS = 4 * RA + 4 * RB;
  constexpr int CT_STRIDE = BN + 8;
  constexpr int EPI_LDS = XBM * CT_STRIDE * 2;
  constexpr int LDS = STAGE_LDS > EPI_LDS ? STAGE_LDS : EPI_LDS;
  constexpr int W2 = 2 * (NA + NB);  // glds per wave per K tile
  static_assert(NA >= 1 && NB >= 1, "region smaller than one glds round");
  __shared__ __attribute__((aligned(16))) char smem[LDS];
  // XL_DGELU: column sums of the output (fc1's bias gradient) when p.part is set
  constexpr bool kMom = EPI == XL_MOMENTS || is_bnbwd(EPI) || EPI == XL_DGELU;
  if constexpr (kMom) zero_moments(p.zsums, 2 * p.N);

  const bf16* __restrict__ A = p.A;
  const bf16* __restrict__ B = p.B;
  const int64_t lda = p.lda, ldb = p.ldb;
  const int M = p.M, N = p.N, K = p.K;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int tbm = (PIPE == 10 && p.bm > 0) ? p.bm : XBM;  // rows per tile (pick_bm)
  const int mtiles = (M + tbm - 1) / tbm, ntiles = (N + BN - 1) / BN;
  int mt, nt;
  const int kt_begin = 0, kt_end = K / XBK;
  tile_coords(mtiles * ntiles, mtiles, ntiles, p.group_m, mt, nt);
  const int m0 = mt * tbm, n0 = nt * BN;
  const int ktiles = K / XBK;
  if (p.tdbg && threadIdx.x == 0) {
    p.tdbg[(int64_t)blockIdx.x * 8 + 0] = __builtin_amdgcn_s_memrealtime();
    p.tdbg[(int64_t)blockIdx.x * 8 + 4] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    p.tdbg[(int64_t)blockIdx.x * 8 + 5] = __builtin_amdgcn_s_getreg((31 << 11) | 20);
  }

  // ---- staging: lane L of a 1 KB glds instruction writes LDS bytes L*16..+16
  // of 16 rows x 64 B; the logical 16-B chunk it carries is the physical one
  // XOR swz(row) (row & 15 = L >> 2, so the XOR depends on L >> 4 only).
  const int srow = lane >> 2;
  const int schunk = (lane & 3) ^ chunk_xor(lane >> 4);
  const bf16* asrc[NA];
  const bf16* asrc2[NA];
  const bf16* bsrc[NB];
#pragma unroll
  for (int q = 0; q < NA; ++q) {
    const int r = (wave * NA + q) * 16 + srow;
    asrc[q] = A + (int64_t)min(m0 + r, M - 1) * lda + schunk * 8;
    asrc2[q] = p.A2 ? p.A2 + xl_out_row(p.a2m, min(m0 + r, M - 1)) * p.lda2 + schunk * 8 - p.K1 : nullptr;
  }
#pragma unroll
  for (int q = 0; q < NB; ++q) {
    const int r = (wave * NB + q) * 16 + srow;
    bsrc[q] = B + (int64_t)min(n0 + r, N - 1) * ldb + schunk * 8;
  }
  auto a_region = [&](int ks, int buf) { return smem + (buf * 2 + ks) * RA; };
  auto b_region = [&](int ks, int buf) { return smem + 4 * RA + (buf * 2 + ks) * RB; };
  auto stage_a = [&](int ks, int kt, int buf) {
    char* dst = a_region(ks, buf) + wave * NA * 1024;
    const int koff = kt * XBK + ks * 32;
    const bool second = p.A2 && koff >= p.K1;
#pragma unroll
    for (int q = 0; q < NA; ++q) glds16((second ? asrc2[q] : asrc[q]) + koff, dst + q * 1024);
  };
  auto stage_b = [&](int ks, int kt, int buf) {
    char* dst = b_region(ks, buf) + wave * NB * 1024;
    const int koff = kt * XBK + ks * 32;
#pragma unroll
    for (int q = 0; q < NB; ++q) glds16(bsrc[q] + koff, dst + q * 1024);
  };

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int lrow = lane & 15, lk = lane >> 4;
  // fragment byte offset of row r (multiple of 16 + lrow) in a k32 region
  const int frag_off = lrow * 64 + ((lk ^ chunk_xor(lrow >> 2)) << 4);
  bf16x8 fb[NI];

  auto phase = [&](int ks, int mh, int buf) {
    const char* ar = a_region(ks, buf) + (wr * WTM + mh * 64) * 64 + frag_off;
    bf16x8 fa[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) fa[i] = *reinterpret_cast<const bf16x8*>(ar + i * 16 * 64);
    if (mh == 0) {
      const char* br = b_region(ks, buf) + (wc * WTN) * 64 + frag_off;
#pragma unroll
      for (int j = 0; j < NI; ++j) fb[j] = *reinterpret_cast<const bf16x8*>(br + j * 16 * 64);
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j)
        acc[mh * 4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[mh * 4 + i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  if constexpr (PIPE == 0) {
  // ---- prologue: tile 0 (both halves) and tile 1's k0 half in flight ----
  stage_a(0, 0, 0);
  stage_b(0, 0, 0);
  stage_a(1, 0, 0);
  stage_b(1, 0, 0);
  if (ktiles > 1) {
    stage_a(0, 1, 1);
    stage_b(0, 1, 1);
    vmcnt<W2>();
  } else {
    vmcnt<NA + NB>();
  }
  barrier();

  for (int kt = 0; kt < ktiles; ++kt) {
    const int buf = kt & 1;
    const bool has1 = kt + 1 < ktiles, has2 = kt + 2 < ktiles;
    // phase 0: k0 half, M half 0; stage tile kt+1's A k1 half
    if (has1) stage_a(1, kt + 1, buf ^ 1);
    phase(0, 0, buf);
    barrier();
    // phase 1: k0, M half 1; stage tile kt+1's B k1; retire tile kt's k1 half
    if (has1) stage_b(1, kt + 1, buf ^ 1);
    phase(0, 1, buf);
    if (has1) vmcnt<W2>(); else vmcnt<0>();
    barrier();
    // phase 2: k1, M half 0; this tile's k0 regions are free: stage tile kt+2's A k0
    if (has2) stage_a(0, kt + 2, buf);
    phase(1, 0, buf);
    barrier();
    // phase 3: k1, M half 1; stage kt+2's B k0; retire tile kt+1's k0 half
    if (has2) stage_b(0, kt + 2, buf);
    phase(1, 1, buf);
    if (has2) vmcnt<W2>(); else if (has1) vmcnt<NA + NB>(); else vmcnt<0>();
    barrier();
  }
  } else if constexpr (PIPE == 10) {
  // ---- PIPE 7: ping-pong quadrant schedule (cdna_hip_programming.md §5 "256²
  // 8-phase template").  The two wave rows (wr) run one barrier apart: while
  // one group's 4 waves run a phase's 16 MFMAs, the other group (one wave on
  // each SIMD) issues that phase's ds_reads and LDS-DMA copies, so every SIMD
  // alternates a MFMA wave and a memory wave between consecutive barriers.
  // A K tile is 4 phases, one per quadrant (m half, n half) of the wave's
  // 128 x 64 outputs, in the order (0,0) (0,1) (1,1) (1,0) so that each phase
  // re-reads only one operand.  A tile's operands are staged as 4 units of
  // 16 KB (2 glds per wave): U0 = A rows of m half 0, U3 = m half 1, U1 = B
  // cols of n half 0, U2 = n half 1.  Phase r of tile t stages U3(t+1),
  // U1(t+1), U0(t+2), U2(t+2) (r = 0..3): every unit is written >= 2 barrier
  // slots after its previous contents were last read (WAR), and is retired by
  // the vmcnt(4) of a phase >= 2 before its first reader (RAW: the counted
  // wait -- never 0 in steady state -- then a barrier, then the ds_read).
  static_assert(BN == 256, "ping-pong schedule is written for 256 x 256 tiles");
  const int pks = wave >> 2;  // k32 half carried by this wave's two copies of a unit
  const bf16* pa[2][2];
  const bf16* pa2[2][2];
  const bf16* pb[2][2];
  int oa[2][2], ob[2][2];
#pragma unroll
  for (int v = 0; v < 2; ++v)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int j = (2 * wave + q) & 7;
      const int ba = (j & 3) + 8 * (j >> 2) + 4 * v, bb = (j & 1) + 4 * (j >> 1) + 2 * v;
      pa[v][q] = A + (int64_t)min(m0 + ba * 16 + srow, M - 1) * lda + schunk * 8 + pks * 32;
      pa2[v][q] = p.A2 ? p.A2 + xl_out_row(p.a2m, min(m0 + ba * 16 + srow, M - 1)) * p.lda2 + schunk * 8 + pks * 32 -
                             p.K1
                       : nullptr;
      pb[v][q] = B + (int64_t)min(n0 + bb * 16 + srow, N - 1) * ldb + schunk * 8 + pks * 32;
      oa[v][q] = ba * 1024;
      ob[v][q] = bb * 1024;
    }
  // conv gather: per staged A row, its top-left input pixel and coordinates
  const XlConv cv = p.cv;
  const bool gather = cv.cin > 0;
  const int loff = schunk * 8 + pks * 32;
  int gpix[2][2], gih[2][2], giw[2][2];
  if (gather) {
    const int hw = cv.ho * cv.wo;
#pragma unroll
    for (int v = 0; v < 2; ++v)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int j = (2 * wave + q) & 7;
        const int row = min(m0 + ((j & 3) + 8 * (j >> 2) + 4 * v) * 16 + srow, M - 1);
        const int n = row / hw, r = row - n * hw, oh = r / cv.wo, ow = r - oh * cv.wo;
        gih[v][q] = oh * cv.stride - cv.pad;
        giw[v][q] = ow * cv.stride - cv.pad;
        gpix[v][q] = (n * cv.hi + gih[v][q]) * cv.wi + giw[v][q];
      }
  }
  auto stage_unit = [&](auto u, int kt) {
    constexpr int U = decltype(u)::value;
    const int buf = kt & 1, koff = kt * XBK;
    if constexpr (U == 0 || U == 3) {
      if (gather) {  // tap (tr, tc), channels c0.. of every staged output pixel, or zeros
        const int cpt = cv.cin >> 6, tap = kt / cpt, c0 = (kt - tap * cpt) << 6;
        const int tr = tap / cv.kw, tc = tap - tr * cv.kw;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int ih = gih[U == 3][q] + tr, iw = giw[U == 3][q] + tc;
          const bool ok = (unsigned)ih < (unsigned)cv.hi && (unsigned)iw < (unsigned)cv.wi;
          const bf16* src = ok ? A + (int64_t)(gpix[U == 3][q] + tr * cv.wi + tc) * lda + c0 + loff
                               : g_zero_row + loff;
          glds16(src, a_region(pks, buf) + oa[U == 3][q]);
        }
        return;
      }
    }
    const bool second = p.A2 && koff >= p.K1;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      if constexpr (U == 0 || U == 3)
        glds16((second ? pa2[U == 3][q] : pa[U == 3][q]) + koff, a_region(pks, buf) + oa[U == 3][q]);
      else
        glds16(pb[U == 2][q] + koff, b_region(pks, buf) + ob[U == 2][q]);
    }
  };
  // PIPE 10 keeps both n halves of B in registers (qb[nq]): B half 0 is
  // read once per K tile instead of twice, so every unit has one reader phase
  // and its slot frees two phases earlier -- the copies are issued 4 phases
  // ahead of their readers instead of 2 (vmcnt(8): 64 KB in flight per wave
  // group instead of 32 KB)
  constexpr bool kDeep = true;  // (the round-4 schedule re-read B's n half 0: PIPE 7, removed)
  bf16x8 qa[2][4], qb[kDeep ? 2 : 1][2][2];
  auto read_a = [&](int mq, int buf) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        qa[ks][i] = *reinterpret_cast<const bf16x8*>(a_region(ks, buf) + (wr * WTM + mq * 64 + i * 16) * 64 + frag_off);
  };
  auto read_b = [&](int nq, int buf) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        qb[kDeep ? nq : 0][ks][j] =
            *reinterpret_cast<const bf16x8*>(b_region(ks, buf) + (wc * WTN + nq * 32 + j * 16) * 64 + frag_off);
  };
  // a trimmed tile (tbm < 256, >= 192): wave row 1's m-half-1 blocks past
  // row tbm are the next tile's rows -- their MFMAs are skipped (wave-uniform)
  const int ilim = wr ? ((tbm - 192) >> 4) : 4;
  auto quad = [&](auto mqc, auto nqc) {
    constexpr int MQ = decltype(mqc)::value, NQ = decltype(nqc)::value;
    barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    // operands swapped: acc holds C^T blocks (lane = output row, registers =
    // 4 consecutive output columns), so the epilogue stages 8-B row pieces
    if (MQ == 0 || ilim >= 4) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[MQ * 4 + i][NQ * 2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                qb[kDeep ? NQ : 0][ks][j], qa[ks][i], acc[MQ * 4 + i][NQ * 2 + j], 0, 0, 0);
    } else {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (i < ilim) {
#pragma unroll
            for (int j = 0; j < 2; ++j)
              acc[MQ * 4 + i][NQ * 2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                  qb[kDeep ? NQ : 0][ks][j], qa[ks][i], acc[MQ * 4 + i][NQ * 2 + j], 0, 0, 0);
          }
    }
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    barrier();
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  // K tiles [kt_begin, kt_end): the whole K, or one split of a tail tile
  // (kt_begin even, so K tile kt still lives in buffer kt & 1)
  // ---- PIPE 10 unit schedule.  Readers: U0, U1 of tile t in phase 0 (quad
  // (0,0)), U2 in phase 1, U3 in phase 2; phase 3 reads nothing.  Phase r of
  // tile t stages U2(t+1), U3(t+1), U0(t+2), U1(t+2): each is written >= 2
  // phases after its slot's previous reader (WAR) and retired by a vmcnt 4
  // phases after its issue, one phase before its reader (RAW).  The waits
  // leave the 4 youngest units (8 copies per wave) in flight; phase 2 has no
  // reader in the next phase and so no wait.
  stage_unit(I0{}, kt_begin);
  stage_unit(I1{}, kt_begin);
  stage_unit(I2{}, kt_begin);
  stage_unit(I3{}, kt_begin);
  if (kt_end - kt_begin > 1) {
    stage_unit(I0{}, kt_begin + 1);
    stage_unit(I1{}, kt_begin + 1);
    vmcnt<8>();
  } else {
    vmcnt<4>();
  }
  barrier();
  xl_mark(p, 1);
  if (wr == 1) barrier();  // the stagger: wave row 1 runs one barrier behind
  for (int kt = kt_begin; kt < kt_end; ++kt) {
    const int buf = kt & 1;
    const bool n1 = kt + 1 < kt_end, n2 = kt + 2 < kt_end;
    read_a(0, buf);
    read_b(0, buf);
    if (n1) { stage_unit(I2{}, kt + 1); vmcnt<8>(); } else { vmcnt<2>(); }
    quad(I0{}, I0{});
    read_b(1, buf);
    if (n1) { stage_unit(I3{}, kt + 1); vmcnt<8>(); } else { vmcnt<0>(); }
    quad(I0{}, I1{});
    read_a(1, buf);
    if (n2) stage_unit(I0{}, kt + 2);
    quad(I1{}, I1{});
    if (n2) { stage_unit(I1{}, kt + 2); vmcnt<8>(); } else if (n1) { vmcnt<4>(); } else { vmcnt<0>(); }
    quad(I1{}, I0{});
  }
  if (wr == 0) barrier();  // equal barrier counts before the epilogue
  barrier();
  xl_mark(p, 2);
  } else {
  // ---- PIPE 1: half-step ring.  Half-step s (K tile s/2, k32 half s%2) lives
  // in LDS region s%4.  During half-step s: stage region s%4 with the data of
  // half-step s+4 (its fragments were read in s-1 and retired before that
  // step's barrier), ds_read the fragments of s+1 into the other register set
  // (retired by the vmcnt at the end of s-1), run the 32 MFMAs of s.  One
  // barrier per half-step; three half-steps of copies in flight.
  const int S = 2 * ktiles;
  auto stage_h = [&](int h) {
    stage_a(h & 1, h >> 1, (h >> 1) & 1);
    stage_b(h & 1, h >> 1, (h >> 1) & 1);
  };
  bf16x8 xa[MI], xb[NI], ya[MI], yb[NI];
  auto read_frags = [&](bf16x8 (&fa)[MI], bf16x8 (&fbb)[NI], int h) {
    const char* ar = smem + (h & 3) * RA + (wr * WTM) * 64 + frag_off;
    const char* br = smem + 4 * RA + (h & 3) * RB + (wc * WTN) * 64 + frag_off;
#pragma unroll
    for (int j = 0; j < NI; ++j) fbb[j] = *reinterpret_cast<const bf16x8*>(br + j * 16 * 64);
#pragma unroll
    for (int i = 0; i < MI; ++i) fa[i] = *reinterpret_cast<const bf16x8*>(ar + i * 16 * 64);
  };
  auto mfmas = [&](const bf16x8 (&fa)[MI], const bf16x8 (&fbb)[NI]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fbb[j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  auto lgkm0 = [] { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); };
  // prologue: half-steps 0..3 in flight; retire 0, read it, retire 1
  stage_h(0);
  stage_h(1);
  if (S >= 4) {
    stage_h(2);
    stage_h(3);
    vmcnt<3 * (NA + NB)>();
  } else {
    vmcnt<NA + NB>();
  }
  barrier();
  read_frags(xa, xb, 0);
  if (S >= 4) vmcnt<2 * (NA + NB)>(); else vmcnt<0>();
  lgkm0();
  barrier();
  for (int s = 0; s < S; s += 2) {
    if (s + 4 < S) stage_h(s + 4);
    read_frags(ya, yb, s + 1);
    mfmas(xa, xb);
    if (s + 4 < S) vmcnt<2 * (NA + NB)>(); else vmcnt<0>();
    lgkm0();
    barrier();
    if (s + 5 < S) stage_h(s + 5);
    if (s + 2 < S) read_frags(xa, xb, s + 2);
    mfmas(ya, yb);
    if (s + 5 < S) vmcnt<2 * (NA + NB)>(); else vmcnt<0>();
    lgkm0();
    barrier();
  }
  }

  // ---- epilogue: (acc [+ bias]) -> bf16 tile in LDS, then row-contiguous pass ----
  // every operand copy has landed (the main loops end on vmcnt(0) in inline
  // asm, which the compiler cannot see): say so with a wait it does see, or it
  // drains the epilogue's first operand batch before its first LDS write to
  // order that write after the copies into LDS
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  xl_epilogue<BN, EPI, PIPE, LDS>(p, acc, smem, m0, n0, mt, mtiles, tbm);
  if (p.tdbg) {
    __syncthreads();
    xl_mark(p, 3);
  }
}

// ---- PIPE 11: 4-wave 256 x 256 kernel (cdna_hip_programming.md §5; profiles/
// README.md finding 69).  One wave per SIMD computes 128 x 128 outputs (64
// accumulators, all 256 AGPRs, tied in-place MFMAs: w4_mfma), so each
// fragment read from LDS feeds 8 MFMAs (128 KB of fragment reads per CU and K
// tile, against 224 KB for the 8-wave 128 x 64 wave tiles) and the only
// synchronisation is one barrier per K tile.  Every LDS-DMA instruction copies
// 8 rows x 128 B -- one whole K tile of 8 rows, 8 full cache lines -- into an
// [256 rows][128 B] image with 16-B chunk c of row r at c ^ ((r >> 1) & 7)
// (conflict-free fragment reads).  Copies of half-line pieces (16 rows x 64 B)
// cost the MFMA issue stream ~25 % at 8192^3; full lines, one per 4 MFMAs
// spread over the copy segment, brought it from 1.39 to 1.54 PF/s.
//   S1: k-half 0 MFMAs, reading k-half 1's fragments of tile t (one ds_read
//       per 4 MFMAs); vmcnt(0) + barrier: tile t + 1 has landed, buffer t & 1
//       is free;
//   S2: k-half 1 MFMAs, copying tile t + 2 into buffer t & 1 (one per 4
//       MFMAs) and reading k-half 0 of tile t + 1 (first half of the segment).
// Operand staging features: plain A / B, the second A source (A2 from column
// K1, a strided row map), the conv tap gather (cv; zero taps from g_zero_row).
__device__ __forceinline__ void w4_mfma(f32x4& c, const bf16x8& a, const bf16x8& b) {
  // tied dst == srcC in AGPRs: the builtin lets the register allocator pick an
  // untied dst for some accumulators and rotate all 256 through v_accvgpr
  // moves every K tile; "memory" pins the order of the interleaved LDS reads /
  // copies.  srcA/B come from ds_read results the compiler waits for; the
  // accumulate chain D -> C needs no wait states; reads of the accumulators
  // after the loop sit behind w4_drain().
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b) : "memory");
}
__device__ __forceinline__ void w4_drain() { asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory"); }
__device__ __forceinline__ int w4_swz(int c, int row) { return c ^ ((row >> 1) & 7); }

// SRC (compile-time, so the copy stream between the MFMAs has no branches):
// 0 = plain A, by buffer_load ... lds with one 32-bit lane offset per piece
// (operands < 2 GB); 1 = plain A with the second source A2 from column K1;
// 2 = conv tap gather (global_load_lds, zero taps read g_zero_row)
// MB: 16-row MFMA blocks per wave (8: 256-row tiles; 7: 224-row tiles, which
// fill the last 1-block/CU round of grids such as ViT's N = 768 GEMMs, 591 ->
// 678 tiles in the same three rounds of 7/8 the work each: pick_bm).
// WN: waves along N (2: 2 x 2 waves, 256-wide tiles; 1: the four waves stacked
// along M with 64 x 128 each, a 256 x 128 tile for N = 128 -- ResNet-50's
// layer-2 stride-2 3x3 forward, which a 256-wide tile would half waste).
// NBW: 16-column blocks per wave (8; 4 with WN = 1 gives a 256 x 64 tile: for
// ResNet-50 layer 1's N = 64 conv1 forward and conv3 data gradient + BN
// backward it measured slower than gemm_nt's 256 x 64 tile in-step, 112.48
// vs 111.23 ms, finding 78, so no launch uses it).
template <int EPI, int SRC, int MB = 8, int WN = 2, int NBW = 8>
__global__ __launch_bounds__(256, 1) void gemm_xl_w4_kernel(const XlArgs p) {
  static_assert((WN == 2 && (MB == 8 || MB == 7) && NBW == 8) || (WN == 1 && MB == 4 && (NBW == 8 || NBW == 4)),
                "4-wave tile shapes");
  constexpr int TBM = (4 / WN) * 16 * MB, TBN = 16 * NBW * WN;  // tile rows / columns
  constexpr int NRD = NBW + MB, NMF = NBW * MB;  // fragment reads / MFMAs per wave and k-half
  constexpr int OPB = 256 * 128, BUF = 2 * OPB;  // one operand's K tile, one buffer (A | B)
  constexpr int EPI_LDS = XBM * (256 + 8) * 2;
  constexpr int LDS = 2 * BUF > EPI_LDS ? 2 * BUF : EPI_LDS;
  __shared__ __attribute__((aligned(16))) char smem[LDS];
  constexpr bool kMom = EPI == XL_MOMENTS || is_bnbwd(EPI) || EPI == XL_DGELU;
  if constexpr (kMom) zero_moments(p.zsums, 2 * p.N);
  const int M = p.M, N = p.N, K = p.K;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = WN == 2 ? wave >> 1 : wave, wc = WN == 2 ? wave & 1 : 0;
  const int mtiles = (M + TBM - 1) / TBM, ntiles = (N + TBN - 1) / TBN;
  int mt, nt;
  tile_coords(mtiles * ntiles, mtiles, ntiles, p.group_m, mt, nt);
  const int m0 = mt * TBM, n0 = nt * TBN;
  const int ktiles = K / XBK;

  // (a 224-row tile still stages 256 A rows: the last 32 are the next tile's,
  // read but never multiplied)
  // copy c (0..15) of a K tile: operand c >> 3 (A, B), 8-row piece
  // 8 wave + (c & 7); lane L: row 8 piece + (L >> 3), stored chunk L & 7,
  // logical chunk w4_swz(L & 7, row)
  const int lrow8 = lane >> 3;
  const int64_t abytes = ((int64_t)(M - 1) * p.lda + K) * 2, bbytes = ((int64_t)(N - 1) * p.ldb + K) * 2;
  const auto rsa = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, (int)min(abytes, (int64_t)0x7fffffff),
                                                     0x00020000);
  const auto rsb = __builtin_amdgcn_make_buffer_rsrc((void*)p.B, (short)0, (int)min(bbytes, (int64_t)0x7fffffff),
                                                     0x00020000);
  uint32_t oa[8], ob[8];
  const bf16* pa2[8];
  const XlConv cv = p.cv;
  int gpix[8], gih[8], giw[8], lcq[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int row = (wave * 8 + q) * 8 + lrow8;
    const int lc = w4_swz(lane & 7, row) * 8;
    const int ra = min(m0 + row, M - 1);
    lcq[q] = lc;
    oa[q] = (uint32_t)(((int64_t)ra * p.lda + lc) * 2);
    ob[q] = (uint32_t)(((int64_t)min(n0 + row, N - 1) * p.ldb + lc) * 2);
    if constexpr (SRC == 1) pa2[q] = p.A2 + xl_out_row(p.a2m, ra) * p.lda2 + lc - p.K1;
    if constexpr (SRC == 2) {
      const int hw = cv.ho * cv.wo;
      const int n = ra / hw, r = ra - n * hw, oh = r / cv.wo, ow = r - oh * cv.wo;
      gih[q] = oh * cv.stride - cv.pad;
      giw[q] = ow * cv.stride - cv.pad;
      gpix[q] = (n * cv.hi + gih[q]) * cv.wi + giw[q];
    }
  }
  const int lcz = w4_swz(lane & 7, lrow8) * 8;  // zero-row chunk (any in-bounds 16 B)
  // B rows past a narrow tile (TBN < 256) are not copied: this wave's 64 B
  // rows are either all inside or all past it
  const bool cpb = wave * 64 < TBN;
  auto dma = [&](int kt, int buf, int c) {
    const int q = c & 7;
    char* dst = smem + buf * BUF + (c >> 3) * OPB + (wave * 8 + q) * 1024;
    const int koff = kt * XBK;
    if (c >= 8 && !cpb) return;
    if (c >= 8) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsb, (lptr_t)dst, 16, ob[q], koff * 2, 0, 0);
    } else if constexpr (SRC == 2) {  // tap (tr, tc), channels c0.. of this piece's pixels, or zeros
      const int cpt = cv.cin >> 6, tap = kt / cpt, c0 = (kt - tap * cpt) << 6;
      const int tr = tap / cv.kw, tcol = tap - tr * cv.kw;
      const int ih = gih[q] + tr, iw = giw[q] + tcol;
      const bool ok = (unsigned)ih < (unsigned)cv.hi && (unsigned)iw < (unsigned)cv.wi;
      glds16(ok ? p.A + (int64_t)(gpix[q] + tr * cv.wi + tcol) * p.lda + c0 + lcq[q] : g_zero_row + lcz, dst);
    } else if constexpr (SRC == 1) {
      if (koff >= p.K1) glds16(pa2[q] + koff, dst);
      else __builtin_amdgcn_raw_ptr_buffer_load_lds(rsa, (lptr_t)dst, 16, oa[q], koff * 2, 0, 0);
    } else {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsa, (lptr_t)dst, 16, oa[q], koff * 2, 0, 0);
    }
  };

  const int lrow = lane & 15, lk = lane >> 4;
  const int fo0 = lrow * 128 + (w4_swz(lk, lrow) << 4), fo1 = lrow * 128 + (w4_swz(4 + lk, lrow) << 4);
  const int aoff = wr * (16 * MB) * 128, boff = OPB + wc * 128 * 128;
  bf16x8 ra[2][MB], rb[2][NBW];
  // fragment read r (0..NRD-1) in the order the MFMAs consume them: A block 0,
  // B blocks 0..NBW-1, A blocks 1..MB-1
  auto rd = [&](auto hc, int buf, int r) {
    constexpr int H = decltype(hc)::value;
    const bool isb = r >= 1 && r <= NBW;
    const int blk = r == 0 ? 0 : (isb ? r - 1 : r - NBW);
    const char* base = smem + buf * BUF + (isb ? boff : aoff) + blk * 2048 + (H ? fo1 : fo0);
    if (isb) rb[H][blk] = *reinterpret_cast<const bf16x8*>(base);
    else ra[H][blk] = *reinterpret_cast<const bf16x8*>(base);
  };
  f32x4 acc[MB][NBW];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NBW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  // operands swapped: acc[i][j] holds the transposed 16 x 16 block (lane =
  // output row i*16 + (l & 15), registers = 4 consecutive output columns),
  // the layout xl_epilogue stages as 8-B row pieces
  auto iter = [&](auto st, auto rdn, int kt) {
    constexpr bool STAGE = decltype(st)::value, READ = decltype(rdn)::value;
    const int buf = kt & 1;
    // fragment read r after MFMA (r NMF) / NRD, copy c after MFMA (c NMF) / 16:
    // spread evenly (MB = 8: a read / copy per 4 MFMAs)
#pragma unroll
    for (int n = 0; n < NMF; ++n) {
      w4_mfma(acc[n / NBW][n % NBW], rb[0][n % NBW], ra[0][n / NBW]);
      // (closed form, no inner loop: every index must fold to a constant)
      const int r = (n * NRD + NMF - 1) / NMF;  // the read r with r NMF / NRD == n, if any
      if (r < NRD && r * NMF / NRD == n) rd(I1{}, buf, r);
    }
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    barrier();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int n = 0; n < NMF; ++n) {
      w4_mfma(acc[n / NBW][n % NBW], rb[1][n % NBW], ra[1][n / NBW]);
      if constexpr (STAGE) {
        const int c = (n * 16 + NMF - 1) / NMF;  // the copy c with c NMF / 16 == n, if any
        if (c < 16 && c * NMF / 16 == n) dma(kt + 2, buf, c);
      }
      if constexpr (READ)
        if ((n & 1) == 1 && (n >> 1) < NRD) rd(I0{}, buf ^ 1, n >> 1);
    }
  };
#pragma unroll
  for (int c = 0; c < 16; ++c) dma(0, 0, c);
  if (ktiles > 1) {
#pragma unroll
    for (int c = 0; c < 16; ++c) dma(1, 1, c);
    // tile 0 landed: one tile of this wave's copies (16, or 8 past a narrow B) in flight
    if (cpb) vmcnt<16>();
    else vmcnt<8>();
  } else {
    vmcnt<0>();
  }
  barrier();
  xl_mark(p, 1);
#pragma unroll
  for (int r = 0; r < NRD; ++r) rd(I0{}, 0, r);
  int kt = 0;
  for (; kt + 2 < ktiles; ++kt) iter(std::true_type{}, std::true_type{}, kt);
  if (kt + 1 < ktiles) iter(std::false_type{}, std::true_type{}, kt++);
  iter(std::false_type{}, std::false_type{}, kt);
  w4_drain();
  barrier();  // every wave is done with the operand buffers (the epilogue reuses the LDS)
  xl_mark(p, 2);
  // every copy has landed (the waits above are inline asm the compiler cannot
  // see): say so with a wait it does see (finding 66)
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  xl_epilogue<TBN, EPI, 11, LDS, MB, WN>(p, acc, smem, m0, n0, mt, mtiles, TBM);
  if (p.tdbg) {
    __syncthreads();
    xl_mark(p, 3);
  }
}

// ---------------------------------------------------------------------------
// Two-blocks-per-CU conv-epilogue GEMM for the SHORT-K 1x1 convolutions of
// ResNet-50 (K = 64..512 over M = 0.1-6.4 M rows, N = 256..2048) -- finding 43.
//
// With one 512-thread block per CU (gemm_xl_nt_kernel: 256x256 tile, 240
// VGPRs, 128-135 KB LDS), a CU alternates a compute phase (the main loop: no
// HBM traffic once the operands have landed) and a memory phase (the epilogue:
// residual / BN operand loads and the C stores), so HBM is busy only during
// the epilogue share of every tile: l3/l4 affine and BN-backward epilogues ran
// at 42-62 % of the HBM roofline, ~0.5 of it.  Here a 256 x 128 tile
// (8 waves as 2 x 4, 128 x 32 outputs = 64 accumulator VGPRs per wave), a
// single 48 KB operand buffer and NO LDS staging of C leave room for two
// blocks per CU (launch bounds: 4 waves per SIMD, <= 128 VGPRs; 2 x 48 KB LDS): one
// block's epilogue overlaps the other's main loop.
//
// The MFMA operands are swapped (B fragment first), so the accumulator holds
// C^T: lane l owns 4 consecutive output CHANNELS (n = 16 j + 4 (l >> 4) + e)
// of one pixel row (m = 16 i + (l & 15)), and every epilogue operand is one
// 8-byte load / store per lane; the 4 lane groups of a row cover 32 B, the
// two N fragments of a wave 128 B (one L2 line) of each row.  Rounding points
// and per-column affines are those of gemm_xl_nt_kernel (finding 33: the
// affine is applied to the fp32 accumulator before the bf16 rounding).
// ---------------------------------------------------------------------------
constexpr int X2_BM = 256, X2_BN = 128;

template <int EPI>
__global__ __launch_bounds__(XTHREADS, 4) void gemm_x2_kernel(const XlArgs p) {  // 4 waves per SIMD = 2 blocks per CU
  static_assert(EPI == XL_MOMENTS || EPI == XL_AFFINE || EPI == XL_BNBWD || EPI == XL_ADD || EPI == XL_STORE,
                "conv epilogues only");
  constexpr int RA = X2_BM * 64, RB = X2_BN * 64;   // one k32 half: 16 KB of A, 8 KB of B
  constexpr int NA = RA / 1024 / 8, NB = RB / 1024 / 8;  // glds per wave per half: 2, 1
  __shared__ __attribute__((aligned(16))) char smem[2 * RA + 2 * RB];
  constexpr bool kMom = EPI == XL_MOMENTS || EPI == XL_BNBWD;
  if constexpr (kMom) zero_moments(p.zsums, 2 * p.N);

  const int M = p.M, N = p.N, K = p.K;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int mtiles = (M + X2_BM - 1) / X2_BM, ntiles = N / X2_BN;
  int mt, nt;
  tile_coords(mtiles * ntiles, mtiles, ntiles, p.group_m, mt, nt);
  const int m0 = mt * X2_BM, n0 = nt * X2_BN;
  const int ktiles = K / XBK;

  // staging: glds lane L carries 16 B of row (L >> 2) of a 16-row x 64-B block,
  // logical chunk (L & 3) ^ chunk_xor(L >> 4) (the read undoes the swizzle)
  const int srow = lane >> 2;
  const int schunk = (lane & 3) ^ chunk_xor(lane >> 4);
  const bf16* asrc[NA];
  const bf16* asrc2[NA];
  const bf16* bsrc[NB];
#pragma unroll
  for (int q = 0; q < NA; ++q) {
    const int r = min(m0 + (wave * NA + q) * 16 + srow, M - 1);
    asrc[q] = p.A + (int64_t)r * p.lda + schunk * 8;
    asrc2[q] = p.A2 ? p.A2 + xl_out_row(p.a2m, r) * p.lda2 + schunk * 8 - p.K1 : nullptr;
  }
#pragma unroll
  for (int q = 0; q < NB; ++q) bsrc[q] = p.B + (int64_t)(n0 + (wave * NB + q) * 16 + srow) * p.ldb + schunk * 8;

  f32x4 acc[8][2];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int lrow = lane & 15, lk = lane >> 4;
  const int frag_off = lrow * 64 + ((lk ^ chunk_xor(lrow >> 2)) << 4);

  // two-stage LDS ring of k32 units (24 KB each: 256 x 32 A + 128 x 32 B):
  // unit u + 1's LDS-DMA is in flight while unit u's 16 MFMAs per wave run
  // (a single buffer waited on the full L2 / HBM latency every K tile: 32 x
  // ~1.5 us at K = 2048), and the second block on the CU overlaps the rest
  const int nk = ktiles * 2;
  auto issue = [&](int u) {
    const int koff = u * 32;
    const bool second = p.A2 && koff >= p.K1;
    char* da = smem + (u & 1) * RA + wave * NA * 1024;
    char* db = smem + 2 * RA + (u & 1) * RB + wave * NB * 1024;
#pragma unroll
    for (int q = 0; q < NA; ++q) glds16((second ? asrc2[q] : asrc[q]) + koff, da + q * 1024);
#pragma unroll
    for (int q = 0; q < NB; ++q) glds16(bsrc[q] + koff, db + q * 1024);
  };
  issue(0);
  for (int u = 0; u < nk; ++u) {
    if (u + 1 < nk) {
      issue(u + 1);
      vmcnt<NA + NB>();  // unit u landed, unit u + 1 still in flight
    } else {
      vmcnt<0>();
    }
    barrier();
    const char* ar = smem + (u & 1) * RA + (wr * 128) * 64 + frag_off;
    const char* br = smem + 2 * RA + (u & 1) * RB + (wc * 32) * 64 + frag_off;
    const bf16x8 b0 = *reinterpret_cast<const bf16x8*>(br);
    const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(br + 16 * 64);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      bf16x8 fa[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = *reinterpret_cast<const bf16x8*>(ar + (h * 4 + i) * 16 * 64);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        acc[h * 4 + i][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b0, fa[i], acc[h * 4 + i][0], 0, 0, 0);
        acc[h * 4 + i][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b1, fa[i], acc[h * 4 + i][1], 0, 0, 0);
      }
    }
    barrier();  // every wave read buffer u & 1 before unit u + 2 overwrites it
  }

  // ---- epilogue straight from the accumulators (C^T layout) ----
  // per-column constants of the block's 128 columns in LDS (the operand buffer
  // is free after the last barrier): few VGPRs, read where used
  float* cst = reinterpret_cast<float*>(smem + 4096);  // [5][128]: scale, shift/bias, mean, mask scale, mask shift
  if (tid < X2_BN) {
    const int col = n0 + tid;
    float c0 = 1.f, c1 = 0.f, c2 = 0.f, c3 = 0.f, c4 = 0.f;
    if constexpr (EPI == XL_AFFINE) {
      c0 = p.esc ? p.esc[col] : 1.f;
      c1 = p.esh ? p.esh[col] : 0.f;
    }
    if constexpr (EPI == XL_BNBWD) {
      c1 = p.ebias ? p.ebias[col] : 0.f;
      c2 = p.bmean ? p.bmean[col] : 0.f;
      if (!p.bny) {
        c3 = p.binv[col] * (p.bw ? p.bw[col] : 1.f);
        c4 = (p.bb ? p.bb[col] : 0.f) - c2 * c3;
      }
    }
    cst[0 * X2_BN + tid] = c0;
    cst[1 * X2_BN + tid] = c1;
    cst[2 * X2_BN + tid] = c2;
    cst[3 * X2_BN + tid] = c3;
    cst[4 * X2_BN + tid] = c4;
  }
  __syncthreads();
  const int lg = lane >> 4;
  float ms[2][4], mq[2][4];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) ms[j][e] = mq[j][e] = 0.f;
  constexpr bool kRes = EPI == XL_AFFINE || EPI == XL_BNBWD || EPI == XL_ADD;
  const bf16* rbase = p.R ? p.R : p.C;  // absent operands read a valid dummy row (branch-free loads)
  const int64_t rld = p.R ? p.ldr : 0;
  const bf16* xbase = p.bx ? p.bx : p.C;
  const int64_t xld = p.bx ? p.ldbx : 0;
  const bf16* ybase = p.bny ? p.bny : p.C;
  const int64_t yld = p.bny ? p.ldby : 0;
  // pixel fragments per batch: every operand load of a batch before its stores
  constexpr int PI = EPI == XL_BNBWD ? 1 : 2;
#pragma unroll
  for (int h = 0; h < 8 / PI; ++h) {
    bf16x4 l0[PI][2], l1[PI][2], l2[PI][2];
    unsigned rok = 0;
#pragma unroll
    for (int i = 0; i < PI; ++i) {
      const int row = min(m0 + wr * 128 + (h * PI + i) * 16 + lrow, M - 1);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = n0 + wc * 32 + j * 16 + 4 * lg;
        if constexpr (kRes) {
          int64_t rr = row;
          if constexpr (EPI == XL_BNBWD) {
            rr = p.R ? compact_row(p.rmap, row) : -1;
            rok |= (rr >= 0 ? 1u : 0u) << (2 * i + j);
            rr = rr >= 0 ? rr : 0;
          }
          l0[i][j] = *reinterpret_cast<const bf16x4*>(rbase + rr * rld + col);
        }
        if constexpr (EPI == XL_BNBWD) {
          l1[i][j] = *reinterpret_cast<const bf16x4*>(xbase + (int64_t)row * xld + col);
          l2[i][j] = *reinterpret_cast<const bf16x4*>(ybase + (int64_t)row * yld + col);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < PI; ++i) {
      const int row = m0 + wr * 128 + (h * PI + i) * 16 + lrow;
      const bool rin = row < M;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int cl = wc * 32 + j * 16 + 4 * lg;  // column within the block
        const f32x4 a = acc[h * PI + i][j];
        bf16x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = (bf16)fmaf(a[e], cst[cl + e], cst[X2_BN + cl + e]);  // staging rounding
        if constexpr (EPI == XL_MOMENTS) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float f = rin ? (float)v[e] : 0.f;
            ms[j][e] += f;
            mq[j][e] = fmaf(f, f, mq[j][e]);
          }
        } else if constexpr (EPI == XL_ADD) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = (bf16)((float)v[e] + (float)l0[i][j][e]);
        } else if constexpr (EPI == XL_AFFINE) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float f = (float)v[e];
            if (p.R) f += (float)l0[i][j][e];
            if (p.erelu) f = fmaxf(f, 0.f);
            v[e] = (bf16)f;
          }
        } else if constexpr (EPI == XL_BNBWD) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float g = (float)v[e];
            if (p.R) {
              if ((rok >> (2 * i + j)) & 1u) g += (float)l0[i][j][e];
              g = (float)(bf16)g;
            }
            const float xv = (float)l1[i][j][e], yv = (float)l2[i][j][e];
            const bool on = p.bny ? (yv > 0.f)
                                  : (fmaf(xv, cst[3 * X2_BN + cl + e], cst[4 * X2_BN + cl + e]) > 0.f);
            const float dz = (on && rin) ? g : 0.f;
            ms[j][e] += dz;
            if (p.bx) mq[j][e] = fmaf(dz, xv - cst[2 * X2_BN + cl + e], mq[j][e]);
            v[e] = (bf16)dz;
          }
        }
        if (rin) *reinterpret_cast<bf16x4*>(p.C + (int64_t)row * p.ldc + n0 + cl) = v;
      }
    }
  }
  if constexpr (kMom) {
    // per column: the 16 lanes of a lane group hold 16 different pixel rows
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) {
          ms[j][e] += __shfl_xor(ms[j][e], off, 64);
          mq[j][e] += __shfl_xor(mq[j][e], off, 64);
        }
    __syncthreads();  // the operand buffer is free: reuse it for the two wave rows' partials
    float* red = reinterpret_cast<float*>(smem);  // [2 stats][2 wr][128 cols]
    if (lrow == 0) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c = wc * 32 + j * 16 + 4 * lg + e;
          red[(0 * 2 + wr) * X2_BN + c] = ms[j][e];
          red[(1 * 2 + wr) * X2_BN + c] = mq[j][e];
        }
    }
    __syncthreads();
    for (int c = tid; c < X2_BN; c += XTHREADS) {
      p.part[(int64_t)mt * N + n0 + c] = red[(0 * 2 + 0) * X2_BN + c] + red[(0 * 2 + 1) * X2_BN + c];
      p.part[(int64_t)(mtiles + mt) * N + n0 + c] = red[(1 * 2 + 0) * X2_BN + c] + red[(1 * 2 + 1) * X2_BN + c];
    }
  }
}

// ---------------------------------------------------------------------------
// Weight-gradient GEMM on the ping-pong schedule:
//   part[split][n][k] = sum_{m in split} A[m, n] * B[m, k]
// (A = dy [M, N], B = x [M, K] or the implicit-GEMM tap gather of an NHWC
// input).  The reduction runs over the huge M = batch*H*W, split across
// blocks; a column reduce sums the fp32 partials.  256 (n) x 256 (k) output
// tile, 8 waves as 2 x 4 (128 x 64 each), 64 m per K tile.  MFMA operands
// need 8 consecutive m per lane: the LDS holds m-major tiles and fragments
// come from ds_read_b64_tr_b16 (transposing read).  Each operand tile of a
// stage is 8 planes of [64 m][32 cols] (64-B rows, 32-B chunk XOR row & 1),
// so every 16 KB staging unit is 4 whole planes: U0 / U3 = the n columns of
// the waves' m-halves 0 / 1, U1 / U2 = the k columns of their n-halves 0 / 1,
// with the same phase order, unit schedule and vmcnt counts as PIPE 7 of
// gemm_xl_nt_kernel.  LDS-DMA writes lane-linearly, so each lane fetches the
// logical 16 B that its physical slot holds under the swizzle.
// ---------------------------------------------------------------------------
struct TnPPArgs {
  const bf16* A; int64_t lda;
  const bf16* B; int64_t ldb;
  int M, N, K;
  int64_t rps;   // rows per split, a multiple of 64
  float* part;   // [splits][N][K]
  XlConv cv;     // cin > 0: B row m of a K tile = input pixel of its tap (K tile inside one tap)
  int gram = 0;  // 1: A = B = the gathered rows (Gram of a strided 1x1 sample; 4-wave kernel only)
};

// 32-B chunk XOR: row & 1 separates rows q, q+1 (one 256-B bank row holds 4
// rows); bit 3 separates rows r and r+8, which lanes l and l+16 of one
// ds_read_b64_tr_b16 half-wave read (they would otherwise share banks: 2x).
__device__ __forceinline__ int tn64_swz(int row) { return (row ^ (row >> 3)) & 1; }
__device__ __forceinline__ int tn64_off(int row, int col) {
  const int byte = col * 2;
  return row * 64 + ((((byte >> 5) ^ tn64_swz(row))) << 5) + (byte & 31);
}

__global__ __launch_bounds__(XTHREADS, 1) void gemm_tn_pp_kernel(const TnPPArgs p) {
  constexpr int PLANE = 64 * 64, OPER = 8 * PLANE;  // bytes
  __shared__ __attribute__((aligned(16))) char smem[4 * OPER];
  using v4i16 = short __attribute__((ext_vector_type(4)));
  using lds_v4 = __attribute__((address_space(3))) v4i16;
  const int M = p.M, N = p.N, K = p.K;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int ntiles = (N + 255) >> 8, ktiles = (K + 255) >> 8;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = bid % (ntiles * ktiles), split = bid / (ntiles * ktiles);
  const int n0 = (tile / ktiles) * 256, k0 = (tile % ktiles) * 256;
  const int64_t mb = (int64_t)split * p.rps;
  const int64_t me = min((int64_t)M, mb + p.rps);
  const int KT = (int)((me - mb + 63) >> 6);
  const XlConv cv = p.cv;
  const bool gather = cv.cin > 0;
  int tr = 0, tc = 0, kc0 = k0;
  if (gather) {
    const int tap = k0 / cv.cin;
    tr = tap / cv.kw;
    tc = tap - tr * cv.kw;
    kc0 = k0 - tap * cv.cin;
  }
  auto a_plane = [&](int buf, int pl) { return smem + buf * 2 * OPER + pl * PLANE; };
  auto b_plane = [&](int buf, int pl) { return smem + buf * 2 * OPER + OPER + pl * PLANE; };

  // staging roles: wave w writes blocks b = 2 (w & 1) + q (q = 0, 1) of the
  // unit's plane pi = w >> 1; lane -> physical row, 16-B slot
  const int pi = wave >> 1;
  int srow[2], scol[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int b = 2 * (wave & 1) + q;
    srow[q] = 16 * b + (lane >> 2);
    const int slot = lane & 3;
    scol[q] = ((((slot >> 1) ^ tn64_swz(srow[q]))) << 4) + (slot & 1) * 8;
  }
  auto stage_unit = [&](auto u, int kt) {
    constexpr int U = decltype(u)::value;
    const int buf = kt & 1;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int64_t m = mb + (int64_t)kt * 64 + srow[q];
      char* dst;
      const bf16* src = g_zero_row;
      if constexpr (U == 0 || U == 3) {
        const int pl = (U == 0 ? 0 : 2) + (pi & 1) + (pi >> 1) * 4;  // {0,1,4,5} / {2,3,6,7}
        const int col = n0 + pl * 32 + scol[q];
        dst = a_plane(buf, pl) + ((2 * (wave & 1) + q) << 10);
        if (m < me && col < N) src = p.A + m * p.lda + col;
      } else {
        const int pl = 2 * pi + (U == 2 ? 1 : 0);                     // {0,2,4,6} / {1,3,5,7}
        const int col = pl * 32 + scol[q];
        dst = b_plane(buf, pl) + ((2 * (wave & 1) + q) << 10);
        if (m < me && k0 + col < K) {
          if (!gather) {
            src = p.B + m * p.ldb + k0 + col;
          } else {
            const int hw = cv.ho * cv.wo;
            const int mi = (int)m, n = mi / hw, r = mi - n * hw, oh = r / cv.wo, ow = r - oh * cv.wo;
            const int ih = oh * cv.stride - cv.pad + tr, iw = ow * cv.stride - cv.pad + tc;
            if ((unsigned)ih < (unsigned)cv.hi && (unsigned)iw < (unsigned)cv.wi)
              src = p.B + ((int64_t)(n * cv.hi + ih) * cv.wi + iw) * p.ldb + kc0 + col;
          }
        }
      }
      glds16(src, dst);
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // tr-read lane roles (as gemm_tn_kernel): group g = lane >> 4 covers m rows
  // 8g..8g+7 of a k32 step; lane 4q+p of the group reads row q, cols 4p..4p+3
  const int g = lane >> 4, li = lane & 15, q4 = li >> 2, p4 = li & 3;
  bf16x8 qa[2][4], qb[2][2];
  auto tr_frag = [&](const char* plane, int ks, int col_in) {
    const int rb = ks * 32 + 8 * g + q4;
    v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(plane + tn64_off(rb, col_in)));
    v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(plane + tn64_off(rb + 4, col_in)));
    short __attribute__((ext_vector_type(8))) t8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, t8);
  };
  auto read_a = [&](int mq, int buf) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        qa[ks][i] = tr_frag(a_plane(buf, wr * 4 + mq * 2 + (i >> 1)), ks, (i & 1) * 16 + 4 * p4);
  };
  auto read_b = [&](int nq, int buf) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int j = 0; j < 2; ++j) qb[ks][j] = tr_frag(b_plane(buf, wc * 2 + nq), ks, j * 16 + 4 * p4);
  };
  auto quad = [&](auto mqc, auto nqc) {
    constexpr int MQ = decltype(mqc)::value, NQ = decltype(nqc)::value;
    barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[MQ * 4 + i][NQ * 2 + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa[ks][i], qb[ks][j], acc[MQ * 4 + i][NQ * 2 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    barrier();
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  if (KT > 0) {
    stage_unit(I0{}, 0);
    stage_unit(I2{}, 0);
    stage_unit(I3{}, 0);
    stage_unit(I1{}, 0);
    if (KT > 1) {
      stage_unit(I0{}, 1);
      stage_unit(I2{}, 1);
      vmcnt<4>();
    } else {
      vmcnt<0>();
    }
    barrier();
    if (wr == 1) barrier();
    for (int kt = 0; kt < KT; ++kt) {
      const int buf = kt & 1;
      const bool n1 = kt + 1 < KT, n2 = kt + 2 < KT;
      read_a(0, buf);
      read_b(0, buf);
      if (n1) { stage_unit(I3{}, kt + 1); vmcnt<4>(); } else { vmcnt<0>(); }
      quad(I0{}, I0{});
      read_b(1, buf);
      if (n1) { stage_unit(I1{}, kt + 1); vmcnt<4>(); } else { vmcnt<0>(); }
      quad(I0{}, I1{});
      read_a(1, buf);
      if (n2) { stage_unit(I0{}, kt + 2); vmcnt<4>(); } else { vmcnt<0>(); }
      quad(I1{}, I1{});
      read_b(0, buf);
      if (n2) { stage_unit(I2{}, kt + 2); vmcnt<4>(); } else { vmcnt<0>(); }
      quad(I1{}, I0{});
    }
    if (wr == 0) barrier();
  }
  float* out = p.part + (int64_t)split * N * K;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = k0 + wc * 64 + j * 16 + (lane & 15);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int n = n0 + wr * 128 + i * 16 + (lane >> 4) * 4 + e;
        if (n < N && k < K) out[(int64_t)n * K + k] = acc[i][j][e];
      }
    }
}

// ---- 4-wave weight-gradient kernel (the TN form of gemm_xl_w4_kernel;
// profiles/README.md finding 70).  Same output tile, M split and fp32
// partials as gemm_tn_pp_kernel, but: one wave per SIMD computing 128 (n) x
// 128 (k) outputs in 256 AGPRs (inline-asm MFMAs, w4_mfma); LDS-DMA pieces of
// 8 m-rows x 128 B (full cache lines; the ping-pong kernel's 16 x 64 B pieces
// half-use 16 lines each) into [64 m][64 cols] planes whose 16-B chunk c of
// row r sits at c ^ tnw_swz(r) (conflict-free ds_read_b64_tr_b16: the 8 rows a
// half-wave reads -- 4 rows of each of two 16-lane groups, 8 apart -- land on
// all 64 banks); one barrier per 64-deep K tile:
//   S1: the k32-half-0 MFMAs, reading half 1's fragments of tile t;
//       vmcnt(0) + barrier (tile t + 1 landed, buffer t & 1 free);
//   S2: the half-1 MFMAs, copying tile t + 2 into buffer t & 1 (one copy per
//       4 MFMAs) and reading half 0 of tile t + 1.
// SRC: 0 = plain B rows, 2 = the implicit-GEMM tap gather of an NHWC input,
// 3 = both operands the gathered rows (the Gram of a strided 1x1 sample).
__device__ __forceinline__ int tnw_swz(int row) { return (((row >> 1) & 1) << 1) | (((row >> 3) & 1) << 2); }

// Narrow tiles (SRC 0 only): TNN x TNK = 64 x 256 / 256 x 64 (the four
// waves along the wide side, 64 x 64 each) or 128 x 256 / 256 x 128 (2 x 2
// waves, 64 x 128 / 128 x 64 each) for outputs with a side of 64 or 128
// (ResNet-50 layers 1-2: a 256 x 256 tile multiplied 2-16x the useful MFMA
// work there); the copies of the operand planes past the tile are skipped.
template <int TNN, int TNK>
struct TnShape {
  static constexpr int WGN = TNN == 64 ? 1 : TNK == 64 ? 4 : 2;  // wave grid along n / k
  static constexpr int WGK = 4 / WGN;
  static constexpr int MB = TNN / 16 / WGN, NB = TNK / 16 / WGK;  // 16-blocks per wave along n / k
};

template <int SRC, int TNN = 256, int TNK = 256>
__global__ __launch_bounds__(256, 1) void gemm_tn_w4_kernel(const TnPPArgs p) {
  static_assert(SRC == 0 || (TNN == 256 && TNK == 256), "narrow TN tiles: plain operands only");
  constexpr int PLANE = 64 * 128, OPER = 4 * PLANE, BUF = 2 * OPER;  // bytes
  using SH = TnShape<TNN, TNK>;
  constexpr int WGK = SH::WGK, MB = SH::MB, NB = SH::NB;
  static_assert(MB * 16 * SH::WGN == TNN && NB * 16 * WGK == TNK && (MB == 4 || MB == 8) && (NB == 4 || NB == 8),
                "TN tile shape");
  constexpr int NMF = MB * NB, NRD = MB + NB;  // MFMAs / fragment reads per wave and k32 half
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];
  using v4i16 = short __attribute__((ext_vector_type(4)));
  using lds_v4 = __attribute__((address_space(3))) v4i16;
  const int M = p.M, N = p.N, K = p.K;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave / WGK, wc = wave % WGK;
  // this wave's operand planes inside the tile (64 columns each): copies of the others are skipped
  const bool cpa = wave * 64 < TNN, cpb = wave * 64 < TNK;
  const int ntiles = (N + TNN - 1) / TNN, ktiles = (K + TNK - 1) / TNK;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = bid % (ntiles * ktiles), split = bid / (ntiles * ktiles);
  const int n0 = (tile / ktiles) * TNN, k0 = (tile % ktiles) * TNK;
  const int64_t mb = (int64_t)split * p.rps;
  const int64_t me = min((int64_t)M, mb + p.rps);
  const int KT = (int)((me - mb + 63) >> 6);
  // SRC 2: the K tile (256 channels) lies inside one tap (Cin % 256 == 0)
  const XlConv cv = p.cv;
  int tr = 0, tc = 0, kc0 = k0;
  if constexpr (SRC >= 2) {
    const int tap = k0 / cv.cin;
    tr = tap / cv.kw;
    tc = tap - tr * cv.kw;
    kc0 = k0 - tap * cv.cin;
  }

  // copy c (0..15) of a K tile: operand c >> 3 (A = dy n columns, B = k
  // columns), plane `wave`, row group c & 7; lane L: row 8 (c & 7) + (L >> 3),
  // stored chunk L & 7, logical chunk (L & 7) ^ tnw_swz(row)
  const int prow = lane >> 3;
  const int lcol = wave * 64 + (((lane & 7) ^ tnw_swz(prow)) << 3);  // row & 15 = 8 (c & 1) + prow: bit 3 from c
  const int lcol8 = wave * 64 + (((lane & 7) ^ tnw_swz(8 + prow)) << 3);
  // buffer form (the global_load_lds form made the compiler drain every copy
  // before each k step's first ds_read): descriptors over THIS split's rows,
  // so a copy of a row past the split's end is out of range and lands as
  // zeros; columns past N / K read neighbouring bytes into outputs that are
  // never stored
  // The copies are inline asm: as compiler-visible LDS writes (either
  // builtin) they made it wait vmcnt(0) -- every copy in flight -- before
  // each transposing fragment read it cannot prove disjoint from them.  The
  // waits that order them (vmcnt, then the barrier) are explicit anyway.
  using i32x4 = int __attribute__((ext_vector_type(4)));
  const int64_t nrow = me - mb;
  auto desc = [&](const bf16* base, int64_t bytes) {
    const uint64_t a = reinterpret_cast<uint64_t>(base);
    i32x4 d;
    d[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
    d[1] = __builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32));  // stride 0
    d[2] = __builtin_amdgcn_readfirstlane((int)min(bytes, (int64_t)0x7fffffff));
    d[3] = 0x00020000;
    return d;
  };
  // SRC 2: B's descriptor spans the whole NHWC input (a padding tap's offset
  // is past its end: the copy lands zeros); every lane tracks the output pixel
  // (n, oh, ow) of each of its 8 staged rows, advanced by 64 pixels per K tile
  // (no per-copy division: the divisions made this form spill)
  // (based at the split's first image: offsets stay 32-bit for inputs > 2 GB)
  const int64_t img = (int64_t)cv.hi * cv.wi * p.ldb;  // elements per image
  const int nbase = SRC >= 2 ? (int)(mb / max(1, cv.ho * cv.wo)) : 0;
  const int64_t bbytes = SRC >= 2 ? ((me - 1) / max(1, cv.ho * cv.wo) - nbase + 1) * img * 2 : nrow * p.ldb * 2;
  // SRC 3 (the Gram x_s^T x_s of a strided sample): A IS B, both gathered
  const i32x4 rsb = desc(SRC >= 2 ? p.B + nbase * img : p.B + mb * p.ldb, bbytes),
              rsa = SRC == 3 ? rsb : desc(p.A + mb * p.lda, nrow * p.lda * 2);
  const uint32_t oa0 = (uint32_t)((prow * p.lda + n0 + lcol) * 2), oa8 = (uint32_t)((prow * p.lda + n0 + lcol8) * 2);
  const uint32_t ob0 = (uint32_t)((prow * p.ldb + k0 + lcol) * 2), ob8 = (uint32_t)((prow * p.ldb + k0 + lcol8) * 2);
  int gn[8], goh[8], gow[8];
  const int hw = cv.ho * cv.wo, adv_oh = SRC >= 2 ? 64 / max(1, cv.wo) : 0, adv_ow = SRC >= 2 ? 64 % max(1, cv.wo) : 0;
  if constexpr (SRC >= 2) {
#pragma unroll
    for (int rg = 0; rg < 8; ++rg) {
      const int mi = (int)min(mb + 8 * rg + prow, (int64_t)M - 1), n = mi / hw, r = mi - n * hw;
      gn[rg] = n - nbase;
      goh[rg] = r / cv.wo;
      gow[rg] = r - goh[rg] * cv.wo;
    }
  }
  // SRC 2: the 8 B row offsets of K tile kt, then advance every row by 64 pixels
  uint32_t bo[8];
  auto gather_rows = [&](int kt) __attribute__((always_inline)) {
#pragma unroll
    for (int rg = 0; rg < 8; ++rg) {
      const int ih = goh[rg] * cv.stride - cv.pad + tr, iw = gow[rg] * cv.stride - cv.pad + tc;
      const bool ok = kt * 64 + 8 * rg + prow < nrow && (unsigned)ih < (unsigned)cv.hi && (unsigned)iw < (unsigned)cv.wi;
      const int64_t pix = ((int64_t)gn[rg] * cv.hi + ih) * cv.wi + iw;
      bo[rg] = ok ? (uint32_t)((pix * p.ldb + kc0 + ((rg & 1) ? lcol8 : lcol)) * 2) : 0xfffffff0u;
      int ow = gow[rg] + adv_ow, oh = goh[rg] + adv_oh, n = gn[rg];
      if (ow >= cv.wo) { ow -= cv.wo; ++oh; }
#pragma unroll
      for (int w = 0; w < 3; ++w)  // adv_oh + 1 <= 3 ho (host-checked)
        if (oh >= cv.ho) { oh -= cv.ho; ++n; }
      gow[rg] = ow; goh[rg] = oh; gn[rg] = n;
    }
  };
  const uint32_t lds0 = (uint32_t)reinterpret_cast<uintptr_t>(smem);
  auto dma = [&](int kt, int buf, int c) __attribute__((always_inline)) {
    const int rg = c & 7;
    const bool odd = rg & 1;  // row bit 3
    const int ldst = __builtin_amdgcn_readfirstlane((int)(lds0 + buf * BUF + (c >> 3) * OPER + wave * PLANE + rg * 1024));
    uint32_t voff = c < 8 ? (odd ? oa8 : oa0) + (uint32_t)(8 * rg * p.lda * 2)
                          : (odd ? ob8 : ob0) + (uint32_t)(8 * rg * p.ldb * 2);
    int soff = __builtin_amdgcn_readfirstlane((int)(kt * 64 * (c < 8 ? p.lda : p.ldb) * 2));
    if constexpr (SRC == 2)
      if (c >= 8) {
        voff = bo[rg];
        soff = 0;
      }
    if constexpr (SRC == 3) {  // A's columns n0.. of the same gathered rows (a zero row stays zero)
      voff = c >= 8 || bo[rg] == 0xfffffff0u ? bo[rg] : bo[rg] + (uint32_t)((n0 - kc0) * 2);
      soff = 0;
    }
    unsigned keep;
    if ((c < 8 && !cpa) || (c >= 8 && !cpb)) return;  // a plane past a narrow tile
    if (c < 8)
      asm volatile("s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
                   "buffer_load_dwordx4 %2, %3, %4 offen lds\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep) : "s"(ldst), "v"(voff), "s"(rsa), "s"(soff) : "memory");
    else
      asm volatile("s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
                   "buffer_load_dwordx4 %2, %3, %4 offen lds\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep) : "s"(ldst), "v"(voff), "s"(rsb), "s"(soff) : "memory");
  };

  // tr-read lane roles (as gemm_tn_pp_kernel): group g = lane >> 4 covers m
  // rows 8g..8g+7 of a k32 step; lane 4q+p of the group reads row q (+4 for
  // the high half), cols 4p..4p+3 of the fragment's 16 columns
  const int g = lane >> 4, li = lane & 15, q4 = li >> 2, p4 = li & 3;
  auto tr_frag = [&](const char* plane, int h, int cin) __attribute__((always_inline)) {  // cin: column within the 64-col plane, % 16 == 0
    const int r0 = h * 32 + 8 * g + q4, r1 = r0 + 4;
    const int cb = (cin + 4 * p4) * 2;  // byte within the row
    const char* a0 = plane + r0 * 128 + ((((cb >> 4) ^ tnw_swz(r0))) << 4) + (cb & 15);
    const char* a1 = plane + r1 * 128 + ((((cb >> 4) ^ tnw_swz(r1))) << 4) + (cb & 15);
    v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)a0);
    v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)a1);
    short __attribute__((ext_vector_type(8))) t8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, t8);
  };
  bf16x8 ra[2][MB], rb[2][NB];
  // fragment read r (0..NRD-1) of k32 half H: A block (n) r == 0 ? 0 : r - NB, B blocks (k) 0..NB-1 for r = 1..NB
  auto rd = [&](auto hc, int buf, int r) __attribute__((always_inline)) {
    constexpr int H = decltype(hc)::value;
    const bool isb = r >= 1 && r <= NB;
    const int blk = r == 0 ? 0 : (isb ? r - 1 : r - NB);
    const int col = (isb ? wc * NB : wr * MB) * 16 + blk * 16;  // within the operand tile
    const char* plane = smem + buf * BUF + (isb ? OPER : 0) + (col >> 6) * PLANE;
    if (isb) rb[H][blk] = tr_frag(plane, H, col & 63);
    else ra[H][blk] = tr_frag(plane, H, col & 63);
  };
  f32x4 acc[MB][NB];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  // operands swapped: acc[i][j] holds the transposed 16 x 16 block: lane =
  // output row n (i), registers = 4 consecutive output columns k (j).
  // Read r follows MFMA (r NMF) / NRD, copy c MFMA (c NMF) / 16 (the 256 x 256
  // tile: one read / copy per 4 MFMAs); closed forms, so every index folds.
  auto iter = [&](auto st, auto rdn, int kt) __attribute__((always_inline)) {
    constexpr bool STAGE = decltype(st)::value, READ = decltype(rdn)::value;
    const int buf = kt & 1;
    if constexpr (SRC >= 2 && STAGE) gather_rows(kt + 2);
#pragma unroll
    for (int n = 0; n < NMF; ++n) {
      w4_mfma(acc[n / NB][n % NB], rb[0][n % NB], ra[0][n / NB]);
      const int r = (n * NRD + NMF - 1) / NMF;
      if (r < NRD && r * NMF / NRD == n) rd(I1{}, buf, r);
    }
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    barrier();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int n = 0; n < NMF; ++n) {
      w4_mfma(acc[n / NB][n % NB], rb[1][n % NB], ra[1][n / NB]);
      if constexpr (STAGE) {
        const int c = (n * 16 + NMF - 1) / NMF;
        if (c < 16 && c * NMF / 16 == n) dma(kt + 2, buf, c);
      }
      if constexpr (READ)
        if ((n & 1) == 1 && (n >> 1) < NRD) rd(I0{}, buf ^ 1, n >> 1);
    }
  };
  if (KT > 0) {
    if constexpr (SRC >= 2) gather_rows(0);
#pragma unroll
    for (int c = 0; c < 16; ++c) dma(0, 0, c);
    if (KT > 1) {
      if constexpr (SRC >= 2) gather_rows(1);
#pragma unroll
      for (int c = 0; c < 16; ++c) dma(1, 1, c);
      // tile 0 landed: at most one tile of this wave's copies (16, 8 or 0) in flight
      if (cpa && cpb) vmcnt<16>();
      else if (cpa || cpb) vmcnt<8>();
      else vmcnt<0>();
    } else {
      vmcnt<0>();
    }
    barrier();
#pragma unroll
    for (int r = 0; r < NRD; ++r) rd(I0{}, 0, r);
    int kt = 0;
    for (; kt + 2 < KT; ++kt) iter(std::true_type{}, std::true_type{}, kt);
    if (kt + 1 < KT) iter(std::false_type{}, std::true_type{}, kt++);
    iter(std::false_type{}, std::false_type{}, kt);
    w4_drain();
  }
  // fp32 partials: lane = row n, 16-B pieces of 4 consecutive k
  float* out = p.part + (int64_t)split * N * K;
  const int lrow = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int i = 0; i < MB; ++i) {
    const int n = n0 + wr * MB * 16 + i * 16 + lrow;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int k = k0 + wc * NB * 16 + j * 16 + lk * 4;
      if (n < N && k < K) *reinterpret_cast<f32x4*>(out + (int64_t)n * K + k) = acc[i][j];
    }
  }
}

int g_num_cus = 0;

// main loop of the 256 x 256 tiles: 11 = the 4-wave kernel (default), 10 =
// the 8-wave ping-pong quadrant schedule; 128-wide tiles run the half-step
// ring (1) or the round-1 two-buffer loop (0).  Measured and removed in round
// 6 (notes in profiles/README.md): the round-4 ping-pong that re-read B's n
// half 0 (7), its 10-slot LDS unit ring (8, slower: finding 43), the split-K
// tail (9, no faster: finding 54), the persistent form (6, slower: finding
// 66), timing-only ablations (2-5) and the non-temporal epilogue switch.
constexpr int kXlPipeDefault = 11;
int g_xl_pipe = [] {  // DMP_XL_PIPE=<n>: A/B of the main loop (10 = 8-wave ping-pong)
  const char* e = std::getenv("DMP_XL_PIPE");
  return e ? std::atoi(e) : kXlPipeDefault;
}();

// 256 x 256 launches: PIPE 11 (4 waves) or PIPE 10 (8-wave ping-pong)

int num_cus() {
  if (g_num_cus == 0) {
    int dev = 0;
    DMP_HIP_CHECK(hipGetDevice(&dev));
    DMP_HIP_CHECK(hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev));
  }
  return g_num_cus;
}

// Rows per tile of the PIPE 7 kernel.  One 256 x 256 block per CU makes a
// partly filled last round cost a full one (finding 54: layer-3 3x3s at batch
// 2048 are 1568 tiles = 6.1 rounds, ViT's N = 768 GEMMs 591 tiles = 2.3).
// An MFMA-bound GEMM (K >= 768) instead takes the tile height in
// {256, 240, .., 192} that minimises rounds x height: the skipped rows of a
// trimmed tile cost their staging only.  0 = auto, -1 = always 256, else forced (A/B).
int g_xl_bm = 0;

__host__ __device__ constexpr bool w4_epi(int e);

// 4-wave kernel (PIPE 11): 256- or 224-row tiles (MB = 8 / 7 blocks per
// wave), whichever needs fewer rounds x rows of 1-block/CU work: ViT's N = 768
// GEMMs 591 tiles (3 rounds x 256) -> 678 (3 x 224); ResNet-50 layer-3 3x3s
// 1568 (7 x 256) -> 1792 (7 x 224), layer-4 784 (4 x 256) -> 896 (4 x 224).
int pick_bm_w4(int64_t M, int64_t N) {
  if (N <= 128) return 256;  // the 256 x 128 tile (WN = 1) has 256 rows only
  if (g_xl_bm == 224 || g_xl_bm == 256) return g_xl_bm;
  if (g_xl_bm < 0) return 256;
  const int64_t cus = num_cus(), nt = (N + 255) / 256;
  auto cost = [&](int64_t bm) { return ((M + bm - 1) / bm * nt + cus - 1) / cus * bm; };
  // a 12.5 % cut (whole rounds of 7/8 the rows) only: a tile's fixed cost
  // (prologue, epilogue) does not shrink with its rows, and ViT's fc1 forward
  // (N = 3072, K = 768: 10 rounds x 256 vs 11 x 224) measured 0.330 vs 0.339 ms
  return cost(224) * 100 <= cost(256) * 90 ? 224 : 256;
}

// the heavy-epilogue GEMMs the 4-wave default leaves on PIPE 10 (folded-BN
// affine, BN backward) are short-K: their tile time is mostly the epilogue,
// which scales with the tile's rows, so trimmed tiles pay there too
// (set_gemm_xl_trim_heavy, A/B)
int g_xl_trim_heavy = 1;

int pick_bm(int64_t M, int64_t N, int64_t K, int epi) {
  if (g_xl_pipe == 11 && w4_epi(epi)) return pick_bm_w4(M, N);
  const bool heavy = g_xl_pipe == 11 && g_xl_trim_heavy;
  if (g_xl_pipe != 10 && !heavy) return 256;
  if (g_xl_bm > 0) return g_xl_bm;
  if (g_xl_bm < 0 || (K < 768 && !heavy)) return 256;
  const int64_t cus = num_cus(), nt = (N + 255) / 256;
  int best = 256;
  int64_t best_cost = ((M + 255) / 256 * nt + cus - 1) / cus * 256;
  for (int bm = 240; bm >= 192; bm -= 16) {
    const int64_t cost = ((M + bm - 1) / bm * nt + cus - 1) / cus * bm;
    if (cost * 100 < best_cost * 97) { best = bm; best_cost = cost; }
  }
  return best;
}

unsigned long long* g_xl_tdbg = nullptr;  // set_gemm_xl_trace

// Epilogues the 4-wave kernel takes.  The operand-heavy conv epilogues
// (folded-BN affine + residual, every BN-backward form) run on short-K 1x1
// GEMMs whose time is mostly epilogue, and with one wave per SIMD and half the
// threads per row pass their HBM round trips are less hidden: in the ResNet-50
// step XL_BNBWD_YO took 12.9 vs 10.8 ms and XL_AFFINE 10.4 vs 9.8 ms on the
// 4-wave kernel (profiles/README.md finding 69), so they keep the 8-wave
// ping-pong (PIPE 10).  XL_BNBWD's runtime operand flags would also spill
// accumulators behind the inline-asm MFMAs (tests/test_kernel_resources.py).
__host__ __device__ constexpr bool w4_epi(int e) { return e != XL_AFFINE && !is_bnbwd(e); }

// the 4-wave kernel addresses A (plain) and B through 32-bit buffer offsets
bool w4_ok(const XlArgs& a) {
  const int64_t lim = (int64_t)1 << 31;
  const bool bfit = ((int64_t)(a.N - 1) * a.ldb + a.K) * 2 < lim;
  const bool afit = a.cv.cin > 0 || ((int64_t)(a.M - 1) * a.lda + (a.A2 ? a.K1 : a.K)) * 2 < lim;
  return bfit && afit;
}

template <int EPI>
void launch_pp256(const XlArgs& a_in, int blocks, hipStream_t s) {
  XlArgs a = a_in;
  a.tdbg = g_xl_tdbg;
  // (XL_BNBWD with its runtime operand flags needs more registers than the
  // 4-wave epilogue has: the compiler spills accumulators right behind the
  // inline-asm MFMAs that write them -- read before the MFMA completes.  It
  // keeps the 8-wave kernel; tests/test_kernel_resources.py holds every
  // gemm_xl_w4_kernel instantiation to zero scratch.)
  if constexpr (w4_epi(EPI)) {
  if (g_xl_pipe == 11 && w4_ok(a)) {
    XlArgs w = a;
    // a.bm came from pick_bm (the moments partials are sized by it): 224 or 256
    w.bm = a.bm == 224 ? 224 : 256;
    if (w.N <= 128 && w.bm == 256) {  // 256 x 128 tiles, the four waves along M
      const int nblocks = (w.M + 255) / 256;
      if (w.cv.cin > 0)
        hipLaunchKernelGGL((gemm_xl_w4_kernel<EPI, 2, 4, 1>), dim3(nblocks), dim3(256), 0, s, w);
      else if (w.A2)
        hipLaunchKernelGGL((gemm_xl_w4_kernel<EPI, 1, 4, 1>), dim3(nblocks), dim3(256), 0, s, w);
      else
        hipLaunchKernelGGL((gemm_xl_w4_kernel<EPI, 0, 4, 1>), dim3(nblocks), dim3(256), 0, s, w);
      return;
    }
    const int wblocks = ((w.M + w.bm - 1) / w.bm) * ((w.N + 255) / 256);
    if (w.bm == 224) {
      if (w.cv.cin > 0)
        hipLaunchKernelGGL((gemm_xl_w4_kernel<EPI, 2, 7>), dim3(wblocks), dim3(256), 0, s, w);
      else if (w.A2)
        hipLaunchKernelGGL((gemm_xl_w4_kernel<EPI, 1, 7>), dim3(wblocks), dim3(256), 0, s, w);
      else
        hipLaunchKernelGGL((gemm_xl_w4_kernel<EPI, 0, 7>), dim3(wblocks), dim3(256), 0, s, w);
    } else if (w.cv.cin > 0) {
      hipLaunchKernelGGL((gemm_xl_w4_kernel<EPI, 2>), dim3(wblocks), dim3(256), 0, s, w);
    } else if (w.A2) {
      hipLaunchKernelGGL((gemm_xl_w4_kernel<EPI, 1>), dim3(wblocks), dim3(256), 0, s, w);
    } else {
      hipLaunchKernelGGL((gemm_xl_w4_kernel<EPI, 0>), dim3(wblocks), dim3(256), 0, s, w);
    }
    return;
  }
  }
  // PIPE 10, or an epilogue / operand the 4-wave kernel does not take
  hipLaunchKernelGGL((gemm_xl_nt_kernel<256, EPI, 10>), dim3(blocks), dim3(XTHREADS), 0, s, a);
}

template <int BN, int EPI>
void launch_xl(const XlArgs& a, hipStream_t s) {
  const int tbm = (BN == 256 && a.bm > 0) ? a.bm : XBM;
  const int blocks = ((a.M + tbm - 1) / tbm) * ((a.N + BN - 1) / BN);
  if constexpr (BN == 256) {
    if (g_xl_pipe >= 10) {
      launch_pp256<EPI>(a, blocks, s);
      return;
    }
  }
  if (g_xl_pipe == 0)
    hipLaunchKernelGGL((gemm_xl_nt_kernel<BN, EPI, 0>), dim3(blocks), dim3(XTHREADS), 0, s, a);
  else
    hipLaunchKernelGGL((gemm_xl_nt_kernel<BN, EPI, 1>), dim3(blocks), dim3(XTHREADS), 0, s, a);
}

// two-blocks-per-CU kernel (gemm_x2_kernel): 0 = off, 1 = where it measured
// faster than this kernel's 256 x 128 tile (N = 128 + 256 j: 1.14-1.59x on
// ResNet-50 l2 conv1 at batch 256, profiles/raw_r4/x2_bench_r4d.md; on
// N % 256 == 0 the 256 x 256 tile wins 0.76-1.08x), 2 = every conv-epilogue
// GEMM with N % 128 == 0 (A/B)
int g_xl_x2 = 1;


bool use_x2(const XlArgs& a) {
  if (g_xl_x2 == 0 || a.N % X2_BN != 0) return false;
  return g_xl_x2 == 2 || a.N % 256 != 0;
}

template <int EPI>
void launch_x2(const XlArgs& a, hipStream_t s) {
  const int blocks = ((a.M + X2_BM - 1) / X2_BM) * (a.N / X2_BN);
  hipLaunchKernelGGL((gemm_x2_kernel<EPI>), dim3(blocks), dim3(XTHREADS), 0, s, a);
}

template <int EPI>
void dispatch_bn(const XlArgs& a, int bn, hipStream_t s) {
  if constexpr (EPI == XL_MOMENTS || EPI == XL_AFFINE || is_bnbwd(EPI) || EPI == XL_ADD) {
    if (use_x2(a)) {
      launch_x2<is_bnbwd(EPI) ? (int)XL_BNBWD : EPI>(a, s);  // the x2 kernel keeps the runtime operand flags
      return;
    }
  }
  if constexpr (EPI >= XL_MOMENTS) {  // conv epilogues: ring kernel only (no persistent form)
    const int tbm = (bn == 256 && a.bm > 0) ? a.bm : XBM;
    const int blocks = ((a.M + tbm - 1) / tbm) * ((a.N + bn - 1) / bn);
    if (bn == 128)
      hipLaunchKernelGGL((gemm_xl_nt_kernel<128, EPI, 1>), dim3(blocks), dim3(XTHREADS), 0, s, a);
    else if (g_xl_pipe >= 10)
      launch_pp256<EPI>(a, blocks, s);
    else
      hipLaunchKernelGGL((gemm_xl_nt_kernel<256, EPI, 1>), dim3(blocks), dim3(XTHREADS), 0, s, a);
    return;
  }
  if (bn == 128) launch_xl<128, EPI>(a, s);
  else launch_xl<256, EPI>(a, s);
}

int g_xl_bn_override = 0;
int g_xl_group_m = 0;

// BN choice: 256-wide tiles unless that leaves the last round of a 1-block/CU
// grid mostly empty (N = 768: 3 column tiles -> 128-wide gives 2x the blocks).
int pick_bn(int M, int N) {
  if (g_xl_bn_override) return g_xl_bn_override;
  if (g_xl_pipe == 11) return 256;  // the 4-wave kernel has 256-wide tiles only
  const int cus = 256;
  auto eff = [&](int bn) {
    const double blocks = (double)((M + XBM - 1) / XBM) * ((N + bn - 1) / bn);
    const double rounds = std::ceil(blocks / cus);
    // useful work / (rounds x tile work); the 128-wide tile runs the ring
    // loop, ~12 % slower per FLOP than the 256-wide ring and ~25 % slower than
    // the 256-wide ping-pong loop (profiles/vit_gemm_backends.md)
    return blocks / (rounds * cus) * (bn == 256 ? 1.0 : (g_xl_pipe >= 10 ? 0.75 : 0.88));
  };
  return eff(128) > eff(256) ? 128 : 256;
}

void check_bf16_2d(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.dim() == 2, name,
              " must be a 2-D bf16 GPU tensor");
  TORCH_CHECK(t.stride(1) == 1 && t.stride(0) % 8 == 0, name, " rows must be contiguous and 16-B aligned");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-B aligned");
}

}  // namespace

// C = epi(A @ B^T).  mode: "store" | "bias" | "bias_gelu" | "dgelu" | "bias_res".
// Returns C ("bias_gelu": also fills aux with the pre-activation).
at::Tensor gemm_xl(const at::Tensor& A, const at::Tensor& B, const std::string& mode,
                   const c10::optional<at::Tensor>& bias, const c10::optional<at::Tensor>& aux,
                   const c10::optional<at::Tensor>& residual, const c10::optional<at::Tensor>& out) {
  check_bf16_2d(A, "A");
  check_bf16_2d(B, "B");
  const int64_t M = A.size(0), K = A.size(1), N = B.size(0);
  TORCH_CHECK(B.size(1) == K, "gemm_xl: A/B K mismatch");
  TORCH_CHECK(K % XBK == 0 && K >= XBK, "gemm_xl: K must be a positive multiple of 64");
  TORCH_CHECK(N % 8 == 0, "gemm_xl: N must be a multiple of 8");
  TORCH_CHECK(M > 0 && M < (1LL << 31) && N < (1LL << 31), "gemm_xl: size out of range");
  TORCH_CHECK(A.device() == B.device(), "gemm_xl: device mismatch");
  int epi;
  if (mode == "store") epi = XL_STORE;
  else if (mode == "bias") epi = XL_BIAS;
  else if (mode == "bias_gelu") epi = XL_BIAS_GELU;
  else if (mode == "dgelu") epi = XL_DGELU;
  else if (mode == "bias_res") epi = XL_BIAS_RES;
  else TORCH_CHECK(false, "gemm_xl: unknown mode ", mode);
  at::Tensor C;
  if (out) {
    C = *out;
    check_bf16_2d(C, "out");
    TORCH_CHECK(C.size(0) == M && C.size(1) == N, "gemm_xl: out shape");
  } else {
    C = at::empty({M, N}, A.options());
  }
  XlArgs a{};
  a.A = reinterpret_cast<const bf16*>(A.data_ptr());
  a.lda = A.stride(0);
  a.B = reinterpret_cast<const bf16*>(B.data_ptr());
  a.ldb = B.stride(0);
  a.C = reinterpret_cast<bf16*>(C.data_ptr());
  a.ldc = C.stride(0);
  a.M = (int)M; a.N = (int)N; a.K = (int)K;
  if (epi == XL_BIAS || epi == XL_BIAS_GELU || epi == XL_BIAS_RES) {
    TORCH_CHECK(bias && bias->scalar_type() == at::kBFloat16 && bias->numel() == N && bias->is_contiguous(),
                "gemm_xl: bias must be a contiguous bf16 [N]");
    a.bias = reinterpret_cast<const bf16*>(bias->data_ptr());
  }
  if (epi == XL_BIAS_GELU || epi == XL_DGELU) {
    TORCH_CHECK(aux.has_value(), "gemm_xl: mode needs aux");
    check_bf16_2d(*aux, "aux");
    TORCH_CHECK(aux->size(0) == M && aux->size(1) == N, "gemm_xl: aux shape");
    a.aux = reinterpret_cast<bf16*>(aux->data_ptr());
    a.ldaux = aux->stride(0);
  }
  if (epi == XL_BIAS_RES) {
    TORCH_CHECK(residual.has_value(), "gemm_xl: bias_res needs residual");
    check_bf16_2d(*residual, "residual");
    TORCH_CHECK(residual->size(0) == M && residual->size(1) == N, "gemm_xl: residual shape");
    a.R = reinterpret_cast<const bf16*>(residual->data_ptr());
    a.ldr = residual->stride(0);
  }
  const int bn = pick_bn((int)M, (int)N);
  a.group_m = g_xl_group_m > 0 ? g_xl_group_m : 4;
  a.bm = bn == 256 ? pick_bm(M, N, K, epi) : 256;
  hipStream_t s = at::hip::getCurrentHIPStream();
  switch (epi) {
    case XL_STORE: dispatch_bn<XL_STORE>(a, bn, s); break;
    case XL_BIAS: dispatch_bn<XL_BIAS>(a, bn, s); break;
    case XL_BIAS_GELU: dispatch_bn<XL_BIAS_GELU>(a, bn, s); break;
    case XL_DGELU: dispatch_bn<XL_DGELU>(a, bn, s); break;
    default: dispatch_bn<XL_BIAS_RES>(a, bn, s); break;
  }
  DMP_HIP_CHECK(hipGetLastError());
  return C;
}

// dh = bf16(bf16(A @ B^T) * gelu'(aux)) (fc2's data gradient through the GELU)
// and fc1's bias gradient sum_rows dh (fp32 [N]) from the same epilogue: the
// column sums leave as per-M-tile partials, no separate pass over dh.
std::vector<at::Tensor> gemm_xl_dgelu_bgrad(const at::Tensor& A, const at::Tensor& B, const at::Tensor& aux) {
  check_bf16_2d(A, "A");
  check_bf16_2d(B, "B");
  check_bf16_2d(aux, "aux");
  const int64_t M = A.size(0), K = A.size(1), N = B.size(0);
  TORCH_CHECK(B.size(1) == K && K % XBK == 0 && K >= XBK && N % 8 == 0, "gemm_xl_dgelu_bgrad: shapes");
  TORCH_CHECK(M > 0 && M < (1LL << 31), "gemm_xl_dgelu_bgrad: M out of range");
  TORCH_CHECK(aux.size(0) == M && aux.size(1) == N, "gemm_xl_dgelu_bgrad: aux shape");
  auto C = at::empty({M, N}, A.options());
  XlArgs a{};
  a.A = reinterpret_cast<const bf16*>(A.data_ptr()); a.lda = A.stride(0);
  a.B = reinterpret_cast<const bf16*>(B.data_ptr()); a.ldb = B.stride(0);
  a.C = reinterpret_cast<bf16*>(C.data_ptr()); a.ldc = C.stride(0);
  a.M = (int)M; a.N = (int)N; a.K = (int)K;
  a.aux = const_cast<bf16*>(reinterpret_cast<const bf16*>(aux.data_ptr())); a.ldaux = aux.stride(0);
  a.group_m = g_xl_group_m > 0 ? g_xl_group_m : 4;
  const int bn = pick_bn((int)M, (int)N);
  a.bm = bn == 256 ? pick_bm(M, N, K, XL_DGELU) : 256;
  const int mtiles = (int)((M + a.bm - 1) / a.bm);
  const bool fused = true;
  at::Tensor part;
  if (fused) {
    part = at::empty({2, mtiles, N}, A.options().dtype(at::kFloat));
    a.part = part.data_ptr<float>();
  }
  hipStream_t s = at::hip::getCurrentHIPStream();
  dispatch_bn<XL_DGELU>(a, bn, s);
  DMP_HIP_CHECK(hipGetLastError());
  auto bgrad = fused ? part[0].sum(0) : C.to(at::kFloat).sum(0);
  return {C, bgrad};
}

// bn_reduce_partials_launch: batchnorm.hip
void bn_reduce_partials_launch(const float* part, int rb, int C, double* sums, double count,
                               hipStream_t stream);

// Wide 1x1-conv GEMMs with the conv epilogues on the glds-ring kernel:
//   "moments": C = bf16(A @ B^T), returns fp64 [2N+1] (sum, sum^2, M) of C
//   "add"    : C = bf16(bf16(A @ B^T) + residual)
//   "bnbwd"  : C = dz = mask * bf16(A @ B^T (+ residual)), returns (sum dz, sum dz*(x-mean), M)
//              (same contract as gemm_nt_bnbwd)
namespace {

// Shared tail of gemm_xl_conv / conv_xl: epilogue operands, launch, moments reduce.
// `a` holds the operands and M, N, K; conv (a.cv.cin > 0) always runs the
// 256-wide ping-pong kernel (the only main loop with the gather).
std::vector<at::Tensor> xl_conv_run(XlArgs a, const at::Tensor& A, const std::string& mode,
                                    const c10::optional<at::Tensor>& residual,
                                    const c10::optional<at::Tensor>& bn_x,
                                    const c10::optional<at::Tensor>& bn_y,
                                    const c10::optional<at::Tensor>& mean,
                                    const c10::optional<at::Tensor>& invstd,
                                    const c10::optional<at::Tensor>& weight,
                                    const c10::optional<at::Tensor>& bias,
                                    const std::vector<int64_t>& res_map,
                                    const c10::optional<at::Tensor>& ebias = c10::nullopt,
                                    bool relu_flag = false) {
  const int64_t M = a.M, N = a.N;
  int epi;
  if (mode == "moments") epi = XL_MOMENTS;
  else if (mode == "add") epi = XL_ADD;
  else if (mode == "bnbwd") epi = XL_BNBWD;
  else if (mode == "affine") epi = XL_AFFINE;
  else if (mode == "store" && a.cv.cin > 0) epi = XL_STORE;
  else TORCH_CHECK(false, "gemm_xl_conv: unknown mode ", mode);
  auto C = at::empty({M, N}, A.options());
  a.C = reinterpret_cast<bf16*>(C.data_ptr()); a.ldc = C.stride(0);
  a.group_m = g_xl_group_m > 0 ? g_xl_group_m : 4;
  if (!res_map.empty()) {
    TORCH_CHECK(mode == "bnbwd" && res_map.size() == 5, "res_map: bnbwd only, [stride, Ho, Wo, Hi, Wi]");
    a.rmap.s = (int)res_map[0]; a.rmap.ho = (int)res_map[1]; a.rmap.wo = (int)res_map[2];
    a.rmap.hi = (int)res_map[3]; a.rmap.wi = (int)res_map[4];
    TORCH_CHECK(a.rmap.ho == (a.rmap.hi + a.rmap.s - 1) / a.rmap.s &&
                    a.rmap.wo == (a.rmap.wi + a.rmap.s - 1) / a.rmap.s && M % ((int64_t)a.rmap.hi * a.rmap.wi) == 0,
                "res_map does not describe a stride-s subsampling of the GEMM rows");
  }
  if (residual.has_value() && residual->defined()) {
    check_bf16_2d(*residual, "residual");
    const int64_t rrows = a.rmap.s == 1 ? M : M / ((int64_t)a.rmap.hi * a.rmap.wi) * a.rmap.ho * a.rmap.wo;
    TORCH_CHECK(residual->size(0) == rrows && residual->size(1) == N, "gemm_xl_conv: residual shape");
    a.R = reinterpret_cast<const bf16*>(residual->data_ptr());
    a.ldr = residual->stride(0);
  }
  TORCH_CHECK(epi != XL_ADD || a.R, "gemm_xl_conv: add needs a residual");
  auto f32vec = [&](const c10::optional<at::Tensor>& t, const char* name) {
    TORCH_CHECK(t.has_value() && t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous() &&
                    t->numel() == N && reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0,
                name, " must be a contiguous 16-B aligned fp32 [N] GPU tensor");
    return t->data_ptr<float>();
  };
  if (epi == XL_AFFINE) {
    // mean / invstd carry the affine scale / shift (either may be absent: 1 / 0)
    if (mean.has_value() && mean->defined()) a.esc = f32vec(mean, "scale");
    if (invstd.has_value() && invstd->defined()) a.esh = f32vec(invstd, "shift");
    a.erelu = relu_flag;
  }
  if (epi == XL_BNBWD) {
    const bool has_x = bn_x.has_value() && bn_x->defined();
    const bool has_y = bn_y.has_value() && bn_y->defined();
    epi = !has_y ? XL_BNBWD : has_x ? XL_BNBWD_Y : XL_BNBWD_YO;
    TORCH_CHECK(has_x || (bn_y.has_value() && bn_y->defined()), "bnbwd needs bn_x and/or bn_y");
    if (has_x) {
      check_bf16_2d(*bn_x, "bn_x");
      TORCH_CHECK(bn_x->size(0) == M && bn_x->size(1) == N, "bn_x shape");
      a.bx = reinterpret_cast<const bf16*>(bn_x->data_ptr()); a.ldbx = bn_x->stride(0);
      a.bmean = f32vec(mean, "mean");
    }
    if (ebias.has_value() && ebias->defined()) a.ebias = f32vec(ebias, "ebias");
    if (bn_y.has_value() && bn_y->defined()) {
      check_bf16_2d(*bn_y, "bn_y");
      TORCH_CHECK(bn_y->size(0) == M && bn_y->size(1) == N, "bn_y shape");
      a.bny = reinterpret_cast<const bf16*>(bn_y->data_ptr()); a.ldby = bn_y->stride(0);
    } else {
      a.binv = f32vec(invstd, "invstd");
      if (weight.has_value() && weight->defined()) a.bw = f32vec(weight, "weight");
      if (bias.has_value() && bias->defined()) a.bb = f32vec(bias, "bias");
    }
  }
  const bool conv = a.cv.cin > 0;
  const int bn = conv ? 256 : pick_bn((int)M, (int)N);
  // the two-blocks-per-CU route (dispatch_bn -> use_x2) keeps 256-row tiles
  const bool x2 = !conv && epi >= XL_MOMENTS && use_x2(a);
  a.bm = (bn == 256 && !x2) ? pick_bm(M, N, a.K, epi) : 256;
  at::Tensor sums, part;
  const int mtiles = (int)((M + a.bm - 1) / a.bm);
  const bool moments = epi == XL_MOMENTS || is_bnbwd(epi);
  if (moments) {
    part = at::empty({2, mtiles, N}, A.options().dtype(at::kFloat));
    sums = at::empty({2 * N + 1}, A.options().dtype(at::kDouble));
    a.part = part.data_ptr<float>();
    a.zsums = moments_zero_target(sums.data_ptr<double>(), mtiles);
  }
  hipStream_t s = at::hip::getCurrentHIPStream();
  if (conv) {
    const int blocks = mtiles * (int)((N + 255) / 256);
    switch (epi) {
      case XL_STORE: launch_pp256<XL_STORE>(a, blocks, s); break;
      case XL_MOMENTS: launch_pp256<XL_MOMENTS>(a, blocks, s); break;
      case XL_ADD: launch_pp256<XL_ADD>(a, blocks, s); break;
      case XL_BNBWD: launch_pp256<XL_BNBWD>(a, blocks, s); break;
      case XL_BNBWD_Y: launch_pp256<XL_BNBWD_Y>(a, blocks, s); break;
      case XL_BNBWD_YO: launch_pp256<XL_BNBWD_YO>(a, blocks, s); break;
      default: TORCH_CHECK(false, "conv_xl: mode ", mode, " has no implicit-GEMM variant");
    }
  } else {
    switch (epi) {
      case XL_MOMENTS: dispatch_bn<XL_MOMENTS>(a, bn, s); break;
      case XL_ADD: dispatch_bn<XL_ADD>(a, bn, s); break;
      case XL_AFFINE: dispatch_bn<XL_AFFINE>(a, bn, s); break;
      case XL_BNBWD_Y: dispatch_bn<XL_BNBWD_Y>(a, bn, s); break;
      case XL_BNBWD_YO: dispatch_bn<XL_BNBWD_YO>(a, bn, s); break;
      default: dispatch_bn<XL_BNBWD>(a, bn, s); break;
    }
  }
  DMP_HIP_CHECK(hipGetLastError());
  if (moments) bn_reduce_partials_launch(a.part, mtiles, (int)N, sums.data_ptr<double>(), (double)M, s);
  return {C, sums};
}

}  // namespace

std::vector<at::Tensor> gemm_xl_conv(const at::Tensor& A, const at::Tensor& B, const std::string& mode,
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
                                     const c10::optional<at::Tensor>& scale,
                                     const c10::optional<at::Tensor>& shift, bool relu,
                                     const std::vector<int64_t>& a2_map) {
  check_bf16_2d(A, "A");
  check_bf16_2d(B, "B");
  const int64_t M = A.size(0), K1 = A.size(1), N = B.size(0);
  int64_t K = K1;
  const bool two = a2.has_value() && a2->defined();
  XlOutMap a2m;
  if (two) {
    check_bf16_2d(*a2, "a2");
    int64_t rows = a2->size(0);
    if (!a2_map.empty()) {
      TORCH_CHECK(a2_map.size() == 5, "a2_map must be [stride, Ho, Wo, Hi, Wi]");
      a2m.s = (int)a2_map[0]; a2m.ho = (int)a2_map[1]; a2m.wo = (int)a2_map[2];
      a2m.hi = (int)a2_map[3]; a2m.wi = (int)a2_map[4];
      TORCH_CHECK(rows % ((int64_t)a2m.hi * a2m.wi) == 0, "a2_map does not match a2's rows");
      rows = rows / ((int64_t)a2m.hi * a2m.wi) * a2m.ho * a2m.wo;
    }
    TORCH_CHECK(rows == M && K1 % XBK == 0, "gemm_xl_conv: a2 must be [M (through a2_map), K2], K(A) % 64 == 0");
    K += a2->size(1);
  }
  TORCH_CHECK(B.size(1) == K && K % XBK == 0 && K >= XBK && N % 8 == 0, "gemm_xl_conv: bad shape");
  TORCH_CHECK(M > 0 && M < (1LL << 31), "gemm_xl_conv: M out of range");
  TORCH_CHECK(mode != "store", "gemm_xl_conv: use gemm_xl for a plain store");
  XlArgs a{};
  a.A = reinterpret_cast<const bf16*>(A.data_ptr()); a.lda = A.stride(0);
  a.B = reinterpret_cast<const bf16*>(B.data_ptr()); a.ldb = B.stride(0);
  a.M = (int)M; a.N = (int)N; a.K = (int)K;
  if (two) {
    a.A2 = reinterpret_cast<const bf16*>(a2->data_ptr()); a.lda2 = a2->stride(0); a.K1 = (int)K1;
    a.a2m = a2m;
  }
  if (mode == "affine")  // scale / shift travel in the mean / invstd slots of xl_conv_run
    return xl_conv_run(a, A, mode, residual, bn_x, bn_y, scale, shift, weight, bias, res_map, ebias, relu);
  return xl_conv_run(a, A, mode, residual, bn_x, bn_y, mean, invstd, weight, bias, res_map, ebias, relu);
}

// kh x kw convolution of an NHWC (channels-last) input as an implicit GEMM on
// the ping-pong kernel: C[N*Ho*Wo, Cout] = gather(x) @ wmat^T with wmat
// [Cout, kh*kw*Cin] (tap-major, channel-minor), padding taps read as zeros.
// mode "store" | "moments" | "add" | "bnbwd" (epilogues as gemm_xl_conv; the
// bnbwd / add operands are [N*Ho*Wo, Cout] row-major).  Returns (C, sums).
std::vector<at::Tensor> conv_xl(const at::Tensor& x, const at::Tensor& wmat, int64_t kh, int64_t kw,
                                int64_t stride, int64_t pad, int64_t ho, int64_t wo, const std::string& mode,
                                const c10::optional<at::Tensor>& residual,
                                const c10::optional<at::Tensor>& bn_x,
                                const c10::optional<at::Tensor>& bn_y,
                                const c10::optional<at::Tensor>& mean,
                                const c10::optional<at::Tensor>& invstd,
                                const c10::optional<at::Tensor>& weight,
                                const c10::optional<at::Tensor>& bias) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4, "conv_xl: x must be 4-D bf16 GPU");
  TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast), "conv_xl: x must be channels_last");
  check_bf16_2d(wmat, "wmat");
  const int64_t nb = x.size(0), cin = x.size(1), hi = x.size(2), wi = x.size(3);
  TORCH_CHECK(cin % 64 == 0, "conv_xl: Cin must be a multiple of 64");
  TORCH_CHECK(wmat.size(1) == kh * kw * cin && wmat.size(0) % 8 == 0, "conv_xl: wmat must be [Cout, kh*kw*Cin]");
  TORCH_CHECK(ho > 0 && wo > 0 && stride >= 1 && pad >= 0 && (ho - 1) * stride - pad + kh - 1 < hi + pad &&
                  (wo - 1) * stride - pad + kw - 1 < wi + pad, "conv_xl: bad geometry");
  TORCH_CHECK(nb * ho * wo < (1LL << 31) && nb * hi * wi < (1LL << 31), "conv_xl: too many pixels");
  TORCH_CHECK(x.device() == wmat.device(), "conv_xl: device mismatch");
  XlArgs a{};
  a.A = reinterpret_cast<const bf16*>(x.data_ptr()); a.lda = cin;
  a.B = reinterpret_cast<const bf16*>(wmat.data_ptr()); a.ldb = wmat.stride(0);
  a.M = (int)(nb * ho * wo); a.N = (int)wmat.size(0); a.K = (int)(kh * kw * cin);
  a.cv.cin = (int)cin; a.cv.hi = (int)hi; a.cv.wi = (int)wi; a.cv.ho = (int)ho; a.cv.wo = (int)wo;
  a.cv.stride = (int)stride; a.cv.pad = (int)pad; a.cv.kw = (int)kw;
  return xl_conv_run(a, x, mode, residual, bn_x, bn_y, mean, invstd, weight, bias, {});
}

// Data gradient of a 3x3 / stride-2 / pad-1 conv as four stride-phase
// implicit GEMMs on the ping-pong kernel (no zero-filled dx, no zero taps):
// dx[n, 2m + py, 2q + px, :] = sum over the taps (ky, kx) of phase (py, px) of
// dy[n, m + a(ky), q + a(kx), :] @ W[:, :, ky, kx], with a(1) = 0 for the even
// phase and a(2) = 0, a(0) = 1 for the odd one.  Each phase is a stride-1,
// pad-0 conv over dy with a 1x1 / 1x2 / 2x1 / 2x2 kernel (the gather's bounds
// check supplies the zero row / column past the edge), written through an
// output row map straight into its pixels of dx.  wph[2 py + px]:
// [Cin][taps_y][taps_x][Cout] flattened to [Cin, taps * Cout].
// dy: [N, Cout, Ho, Wo] channels_last; returns dx as [N*hi*wi, Cin].
at::Tensor conv_xl_dgrad_s2(const at::Tensor& dy, const std::vector<at::Tensor>& wph, int64_t hi, int64_t wi) {
  TORCH_CHECK(dy.is_cuda() && dy.scalar_type() == at::kBFloat16 && dy.dim() == 4 &&
                  dy.is_contiguous(at::MemoryFormat::ChannelsLast), "conv_xl_dgrad_s2: dy must be 4-D bf16 channels_last");
  TORCH_CHECK(wph.size() == 4, "conv_xl_dgrad_s2: four phase weight matrices");
  const int64_t nb = dy.size(0), cout = dy.size(1), ho = dy.size(2), wo = dy.size(3);
  TORCH_CHECK(cout % 64 == 0 && hi % 2 == 0 && wi % 2 == 0 && ho == hi / 2 && wo == wi / 2,
              "conv_xl_dgrad_s2: even input size, Ho = H / 2, Cout % 64 == 0");
  const int64_t cin = wph[0].size(0);
  TORCH_CHECK(cin % 256 == 0, "conv_xl_dgrad_s2: Cin must be a multiple of 256 (full 256-wide tiles)");
  TORCH_CHECK(nb * hi * wi < (1LL << 31), "conv_xl_dgrad_s2: too many pixels");
  auto dx = at::empty({nb * hi * wi, cin}, dy.options());
  hipStream_t s = at::hip::getCurrentHIPStream();
  for (int ph = 0; ph < 4; ++ph) {
    const int py = ph >> 1, px = ph & 1;
    const int ty = py ? 2 : 1, tx = px ? 2 : 1;
    const at::Tensor& w = wph[ph];
    check_bf16_2d(w, "wph");
    TORCH_CHECK(w.size(0) == cin && w.size(1) == ty * tx * cout && w.device() == dy.device(),
                "conv_xl_dgrad_s2: wph[", ph, "] must be [Cin, ", ty * tx, " * Cout]");
    XlArgs a{};
    a.A = reinterpret_cast<const bf16*>(dy.data_ptr()); a.lda = cout;
    a.B = reinterpret_cast<const bf16*>(w.data_ptr()); a.ldb = w.stride(0);
    a.C = reinterpret_cast<bf16*>(dx.data_ptr()); a.ldc = cin;
    a.M = (int)(nb * ho * wo); a.N = (int)cin; a.K = (int)(ty * tx * cout);
    a.group_m = g_xl_group_m > 0 ? g_xl_group_m : 4;
    a.cv.cin = (int)cout; a.cv.hi = (int)ho; a.cv.wi = (int)wo; a.cv.ho = (int)ho; a.cv.wo = (int)wo;
    a.cv.stride = 1; a.cv.pad = 0; a.cv.kw = tx;
    a.omap.s = 2; a.omap.ho = (int)ho; a.omap.wo = (int)wo; a.omap.hi = (int)hi; a.omap.wi = (int)wi;
    a.omap.oy = py; a.omap.ox = px;
    a.bm = pick_bm(a.M, a.N, a.K, XL_STORE);
    const int blocks = (int)((a.M + a.bm - 1) / a.bm) * (int)(cin / 256);
    launch_pp256<XL_STORE>(a, blocks, s);
  }
  DMP_HIP_CHECK(hipGetLastError());
  return dx;
}

void split_reduce_launch(const float* pp, int splits, int64_t n, at::Tensor& out, hipStream_t stream,
                         bool acc = false);
at::Tensor acc_target(const c10::optional<at::Tensor>& out, int64_t numel, at::ScalarType dtype,
                      const char* who);

namespace {

int g_tn_xl_rounds = 0;  // 0: auto; else rounds of 256 blocks (tools/tn_xl_bench.py sweeps)
int g_tn_narrow = 1;     // narrow TN tiles for sides of 64 / 128 (set_tn_narrow, A/B)

// rows per M split (a multiple of 64): one or two full rounds of 1-block/CU
// work, every split >= 16 K tiles
int64_t tn_rows_per_split(int M, int N, int K, int tnn = 256, int tnk = 256) {
  const int tiles = ((N + tnn - 1) / tnn) * ((K + tnk - 1) / tnk);
  const int mtl = (M + 63) / 64;
  int rounds = tiles >= 256 ? (tiles + 255) / 256 : (tiles * std::max(1, 256 / tiles) >= 192 ? 1 : 2);
  if (g_tn_xl_rounds > 0) rounds = g_tn_xl_rounds;
  const int splits = std::max(1, std::min(256 * rounds / tiles, mtl / 16));
  int64_t rps = ((int64_t)M + splits - 1) / splits;
  return (rps + 63) / 64 * 64;
}

// the gather form addresses the images one M split touches through 32-bit
// offsets from the split's first image (the kernel's descriptor base)
bool tn_w4_gather_fits(const TnPPArgs& a) {
  const int64_t hw = std::max(1, a.cv.ho * a.cv.wo);
  const int64_t imgs = std::min<int64_t>(a.M / hw + 1, a.rps / hw + 2);
  return (int64_t)a.cv.hi * a.cv.wi * imgs * a.ldb * 2 < ((int64_t)1 << 31) - 16;
}

at::Tensor run_tn_pp(TnPPArgs a, const at::Tensor& like, at::ScalarType out_dtype, at::Tensor acc = at::Tensor()) {
  const int M = a.M, N = a.N, K = a.K;
  auto out = acc.defined() ? acc : at::empty({N, K}, like.options().dtype(out_dtype));
  if (M == 0) return acc.defined() ? out : out.zero_();
  // plain operands on the 4-wave kernel: the narrowest tile that covers a
  // side of 64 / 128 (TnShape); the gather forms keep 256 x 256
  const bool plain_w4 = g_xl_pipe == 11 && a.cv.cin == 0;
  const int tnn = !plain_w4 || !g_tn_narrow ? 256 : N <= 64 ? 64 : K <= 64 ? 256 : N <= 128 ? 128 : 256;
  const int tnk = !plain_w4 || !g_tn_narrow || tnn != 256 ? 256 : K <= 64 ? 64 : K <= 128 ? 128 : 256;
  const int tiles = ((N + tnn - 1) / tnn) * ((K + tnk - 1) / tnk);
  const int64_t rps = tn_rows_per_split(M, N, K, tnn, tnk);
  const int splits = (int)(((int64_t)M + rps - 1) / rps);
  a.rps = rps;
  auto part = at::empty({splits, N, K}, like.options().dtype(at::kFloat));
  a.part = part.data_ptr<float>();
  hipStream_t s = at::hip::getCurrentHIPStream();
  // weight gradients on the 4-wave kernel (finding 70; DMP_XL_PIPE=10: the
  // ping-pong one), the tap gather included when its input fits 32-bit offsets
  const dim3 grid(tiles * splits);
  if (plain_w4 && tnn == 64)
    hipLaunchKernelGGL((gemm_tn_w4_kernel<0, 64, 256>), grid, dim3(256), 0, s, a);
  else if (plain_w4 && tnk == 64)
    hipLaunchKernelGGL((gemm_tn_w4_kernel<0, 256, 64>), grid, dim3(256), 0, s, a);
  else if (plain_w4 && tnn == 128)
    hipLaunchKernelGGL((gemm_tn_w4_kernel<0, 128, 256>), grid, dim3(256), 0, s, a);
  else if (plain_w4 && tnk == 128)
    hipLaunchKernelGGL((gemm_tn_w4_kernel<0, 256, 128>), grid, dim3(256), 0, s, a);
  else if (plain_w4)
    hipLaunchKernelGGL(gemm_tn_w4_kernel<0>, grid, dim3(256), 0, s, a);
  else if (a.gram)
    hipLaunchKernelGGL(gemm_tn_w4_kernel<3>, dim3(tiles * splits), dim3(256), 0, s, a);
  else if (g_xl_pipe == 11 && (64 / a.cv.wo + 1) <= 3 * a.cv.ho && tn_w4_gather_fits(a))
    hipLaunchKernelGGL(gemm_tn_w4_kernel<2>, dim3(tiles * splits), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(gemm_tn_pp_kernel, dim3(tiles * splits), dim3(XTHREADS), 0, s, a);
  DMP_HIP_CHECK(hipGetLastError());
  split_reduce_launch(a.part, splits, (int64_t)N * K, out, s, acc.defined());
  return out;
}

}  // namespace

// dW = A^T B on the ping-pong TN kernel: A [M, N], B [M, K] bf16 row-major.
at::Tensor gemm_tn_xl(const at::Tensor& A, const at::Tensor& B, at::ScalarType out_dtype,
                      const c10::optional<at::Tensor>& out) {
  check_bf16_2d(A, "A");
  check_bf16_2d(B, "B");
  TORCH_CHECK(A.size(0) == B.size(0), "gemm_tn_xl: M mismatch");
  TORCH_CHECK(A.size(1) % 8 == 0 && B.size(1) % 8 == 0, "gemm_tn_xl: N, K must be multiples of 8");
  TORCH_CHECK(A.size(0) < (1LL << 31), "gemm_tn_xl: M out of range");
  TORCH_CHECK(out_dtype == at::kFloat || out_dtype == at::kBFloat16, "gemm_tn_xl: fp32 or bf16 output");
  TnPPArgs a{};
  a.A = reinterpret_cast<const bf16*>(A.data_ptr()); a.lda = A.stride(0);
  a.B = reinterpret_cast<const bf16*>(B.data_ptr()); a.ldb = B.stride(0);
  a.M = (int)A.size(0); a.N = (int)A.size(1); a.K = (int)B.size(1);
  return run_tn_pp(a, A, out_dtype, acc_target(out, (int64_t)a.N * a.K, out_dtype, "gemm_tn_xl"));
}

// Gram G = x_s^T x_s (fp32 [Cin, Cin]) of the stride-s sample x[:, :, ::s, ::s]
// of an NHWC input, both operands gathered in place by the 4-wave TN kernel
// (the folded downsample BN's statistics, ops/bn_fold.py).  Cin % 256 == 0.
at::Tensor gram_strided_xl(const at::Tensor& x, int64_t stride, int64_t ho, int64_t wo) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast), "gram_strided_xl: x must be channels_last bf16");
  const int64_t nb = x.size(0), cin = x.size(1), hi = x.size(2), wi = x.size(3);
  TORCH_CHECK(cin % 256 == 0, "gram_strided_xl: Cin must be a multiple of 256");
  TORCH_CHECK(stride >= 1 && (ho - 1) * stride < hi && (wo - 1) * stride < wi, "gram_strided_xl: bad geometry");
  TORCH_CHECK(nb * ho * wo < (1LL << 31), "gram_strided_xl: too many pixels");
  TnPPArgs a{};
  a.A = a.B = reinterpret_cast<const bf16*>(x.data_ptr());
  a.lda = a.ldb = cin;
  a.M = (int)(nb * ho * wo); a.N = (int)cin; a.K = (int)cin;
  a.cv.cin = (int)cin; a.cv.hi = (int)hi; a.cv.wi = (int)wi; a.cv.ho = (int)ho; a.cv.wo = (int)wo;
  a.cv.stride = (int)stride; a.cv.pad = 0; a.cv.kw = 1;
  a.gram = 1;
  a.rps = tn_rows_per_split(a.M, a.N, a.K);
  TORCH_CHECK((64 / wo + 1) <= 3 * ho && tn_w4_gather_fits(a), "gram_strided_xl: geometry outside the 4-wave gather");
  return run_tn_pp(a, x, at::kFloat);
}

bool gram_strided_xl_supported(int64_t nb, int64_t cin, int64_t hi, int64_t wi, int64_t ho, int64_t wo) {
  if (cin % 256 != 0 || (64 / std::max<int64_t>(1, wo) + 1) > 3 * ho || nb * ho * wo >= (1LL << 31)) return false;
  TnPPArgs a{};
  a.M = (int)(nb * ho * wo); a.N = a.K = (int)cin; a.ldb = cin;
  a.cv.hi = (int)hi; a.cv.wi = (int)wi; a.cv.ho = (int)ho; a.cv.wo = (int)wo;
  a.rps = tn_rows_per_split(a.M, a.N, a.K);
  return tn_w4_gather_fits(a);
}

// Weight gradient of a kh x kw conv on the ping-pong TN kernel:
// dW[Cout, kh*kw*Cin] (tap-major) = dy^T @ im2col(x); dy [N*Ho*Wo, Cout]
// row-major, x NHWC (channels_last), Cin % 256 == 0 (a 256-wide K tile never
// straddles a tap).
at::Tensor conv_wgrad_xl(const at::Tensor& dy, const at::Tensor& x, int64_t kh, int64_t kw, int64_t stride,
                         int64_t pad, int64_t ho, int64_t wo, at::ScalarType out_dtype,
                         const c10::optional<at::Tensor>& out) {
  check_bf16_2d(dy, "dy");
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast), "conv_wgrad_xl: x must be channels_last bf16");
  const int64_t nb = x.size(0), cin = x.size(1), hi = x.size(2), wi = x.size(3);
  TORCH_CHECK(cin % 256 == 0, "conv_wgrad_xl: Cin must be a multiple of 256");
  TORCH_CHECK(dy.size(0) == nb * ho * wo && dy.size(1) % 8 == 0, "conv_wgrad_xl: dy must be [N*Ho*Wo, Cout]");
  TORCH_CHECK(nb * hi * wi < (1LL << 31) && dy.size(0) < (1LL << 31), "conv_wgrad_xl: too many pixels");
  TORCH_CHECK(out_dtype == at::kFloat || out_dtype == at::kBFloat16, "conv_wgrad_xl: fp32 or bf16 output");
  TnPPArgs a{};
  a.A = reinterpret_cast<const bf16*>(dy.data_ptr()); a.lda = dy.stride(0);
  a.B = reinterpret_cast<const bf16*>(x.data_ptr()); a.ldb = cin;
  a.M = (int)dy.size(0); a.N = (int)dy.size(1); a.K = (int)(kh * kw * cin);
  a.cv.cin = (int)cin; a.cv.hi = (int)hi; a.cv.wi = (int)wi; a.cv.ho = (int)ho; a.cv.wo = (int)wo;
  a.cv.stride = (int)stride; a.cv.pad = (int)pad; a.cv.kw = (int)kw;
  return run_tn_pp(a, dy, out_dtype, acc_target(out, (int64_t)a.N * a.K, out_dtype, "conv_wgrad_xl"));
}

void set_tn_xl_rounds(int r) { g_tn_xl_rounds = r; }
void set_tn_narrow(bool on) { g_tn_narrow = on ? 1 : 0; }
void set_gemm_xl_trim_heavy(bool on) { g_xl_trim_heavy = on ? 1 : 0; }

int get_gemm_xl_pipe() { return g_xl_pipe; }
void set_gemm_xl_x2(int mode) {
  TORCH_CHECK(mode >= 0 && mode <= 2, "x2 mode: 0 off, 1 short K, 2 always");
  g_xl_x2 = mode;
}
int get_gemm_xl_x2() { return g_xl_x2; }
// The trace buffer is held here (not just its pointer) so a tensor freed by
// the caller can never receive timestamps; tracing cannot be switched on
// while a stream is being captured (the pointer would be baked into the graph).
at::Tensor g_xl_tbuf;
void set_gemm_xl_trace(const c10::optional<at::Tensor>& buf) {
  if (!buf || !buf->defined()) {
    g_xl_tdbg = nullptr;
    g_xl_tbuf = at::Tensor();
    return;
  }
  TORCH_CHECK(buf->is_cuda() && buf->scalar_type() == at::kLong && buf->is_contiguous(),
              "trace buffer: contiguous int64 GPU tensor of 8 entries per block");
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  DMP_HIP_CHECK(hipStreamIsCapturing(at::hip::getCurrentHIPStream().stream(), &cs));
  TORCH_CHECK(cs == hipStreamCaptureStatusNone, "set_gemm_xl_trace: not while a stream is being captured");
  g_xl_tbuf = *buf;
  g_xl_tdbg = reinterpret_cast<unsigned long long*>(g_xl_tbuf.data_ptr());
}
void set_gemm_xl_bm(int bm) {
  TORCH_CHECK(bm == 0 || bm == -1 || (bm >= 192 && bm <= 256 && bm % 16 == 0),
              "bm: 0 (auto), -1 (always 256) or 192..256 in steps of 16");
  g_xl_bm = bm;
}
int get_gemm_xl_bm(int64_t M, int64_t N, int64_t K) { return pick_bm(M, N, K, XL_STORE); }

void set_gemm_xl_bn(int bn, int pipe, int group_m) {
  if (pipe < 0) pipe = kXlPipeDefault;
  TORCH_CHECK(group_m >= 0, "group_m must be >= 0 (0 = default)");
  g_xl_group_m = group_m;
  TORCH_CHECK(bn == 0 || bn == 128 || bn == 256, "bn must be 0 (auto), 128 or 256");
  TORCH_CHECK(pipe == 0 || pipe == 1 || pipe == 10 || pipe == 11,
              "pipe must be 0 / 1 (8-wave 256 x 128 / 256 x 256 ring kernels), 10 (8-wave ping-pong) or "
              "11 (4-wave, the default)");
  g_xl_bn_override = bn;
  g_xl_pipe = pipe;
}

}  // namespace dmp
