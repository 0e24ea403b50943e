// 4-wave 256 x 256 MFMA bf16 GEMM: one wave per SIMD, 128 x 128 outputs per
// wave (64 accumulators of 16 x 16 = 256 registers, AGPR-resident), memory
// instructions issued in the shadow of the MFMAs.
//
//   C[M, N] = A[M, K] * B[N, K]^T          (both operands K-contiguous)
//
// Why this shape (profiles/README.md finding 69): the 8-wave ping-pong kernel
// of gemm_xl.hip gives each wave a 128 x 64 tile, so a CU reads 224 KB of
// fragments from LDS per 64-deep K tile and every quarter-tile is a barrier
// hand-off between the two wave rows.  A 128 x 128 wave tile reads 128 KB per
// K tile (each fragment feeds 8 MFMAs instead of 4 or 8), and with one wave
// per SIMD the only synchronisation is one barrier per K tile; the LDS-DMA
// copies and fragment reads ride between MFMAs (1-2 MFMAs per memory
// instruction), as the vendor library's fastest gfx950 kernel does.
//
// K loop (tile t lives in LDS buffer t & 1; a buffer = A | B x two k32 halves,
// each half [256 rows][64 B] in the swizzled 16-row blocks of gemm_xl.hip):
//   S1: MFMAs of k-half 0 (fragments read during S2 of t - 1), while reading
//       k-half 1's fragments of tile t;  then lgkmcnt(0), vmcnt(0), barrier:
//       every wave is done with buffer t & 1 and tile t + 1 has landed.
//   S2: MFMAs of k-half 1, while copying tile t + 2 into buffer t & 1 and
//       reading k-half 0's fragments of tile t + 1 from the other buffer.
// A copy is issued one K tile (128 MFMAs per wave) before the barrier that
// retires it.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <type_traits>
#include "../common.h"

namespace dmp {
namespace {

using bf16 = __bf16;
using gptr_t = const __attribute__((address_space(1))) void*;
using lptr_t = __attribute__((address_space(3))) void*;

constexpr int W4_BM = 256, W4_BN = 256, W4_BK = 64, W4_THREADS = 256;
constexpr int W4_REGION = 256 * 64;           // one operand's k32 half: 16 KB

__device__ __forceinline__ void w4_glds(const void* g, char* l) {
  __builtin_amdgcn_global_load_lds((gptr_t)g, (lptr_t)l, 16, 0, 0);
}
__device__ __forceinline__ int w4_chunk_xor(int q) { return (0x78 >> (2 * (q & 3))) & 3; }
__device__ __forceinline__ void w4_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// MFMA with its accumulator pinned to AGPRs and tied (dst == srcC).  The
// builtin lets the register allocator pick an untied dst for some of the 64
// accumulators, and with all 256 AGPRs live it then rotates accumulators
// through v_accvgpr moves every K tile (~1.3 copies per MFMA, measured in the
// ISA).  The "memory" clobber also pins the program order of the fragment
// reads and LDS-DMA copies placed between the MFMAs (the interleave below).
// Hazards: srcA/B come from ds_read results (waited for by the compiler's
// lgkmcnt), the accumulate chain D -> C needs no wait states, and the reads
// of the accumulators after the loop sit behind w4_mfma_drain().
__device__ __forceinline__ void w4_mfma(f32x4& c, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b) : "memory");
}
__device__ __forceinline__ void w4_mfma_drain() { asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory"); }

struct W4Args {
  const bf16* A; int64_t lda;
  const bf16* B; int64_t ldb;
  bf16* C; int64_t ldc;
  int M, N, K;
  int group_m;
};

__device__ __forceinline__ void w4_tile(int nblocks, int mtiles, int ntiles, int gm_max, int& mt, int& nt) {
  const int bid = xcd_remap(blockIdx.x, nblocks);
  const int per_group = gm_max * ntiles;
  const int g = bid / per_group, r = bid - g * per_group;
  const int gm = min(gm_max, mtiles - g * gm_max);
  mt = g * gm_max + r % gm;
  nt = r / gm;
}

// NS = LDS slots of 32 KB (one k32 half-tile of A and B each): 4 (128 KB) or
// 5 (160 KB, one more half-tile of copies in flight)
// BUF: the copies as buffer_load ... lds (one 32-bit lane offset per block,
// the K offset in soffset) instead of global_load_lds (64-bit lane addresses).
// NOWAIT: timing-only ablation, no vmcnt in the loop (wrong results).
template <int NS, bool BUF, bool NOWAIT>
__global__ __launch_bounds__(W4_THREADS, 1) void gemm_w4_kernel(const W4Args p) {
  constexpr int SLOT = 2 * W4_REGION;
  __shared__ __attribute__((aligned(16))) char smem[NS * SLOT];
  const int M = p.M, N = p.N, K = p.K;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int mtiles = (M + W4_BM - 1) / W4_BM, ntiles = (N + W4_BN - 1) / W4_BN;
  int mt, nt;
  w4_tile(mtiles * ntiles, mtiles, ntiles, p.group_m, mt, nt);
  const int m0 = mt * W4_BM, n0 = nt * W4_BN;
  const int nh = K / 32;  // k32 half-tiles (even: K % 64 == 0)

  // staging: wave w copies 16-row blocks 4w .. 4w + 3 of A and of B per
  // half-tile (8 x 1 KB); lane L carries row L >> 2 of the block, logical
  // chunk (L & 3) ^ swz(row) (the fragment read undoes the XOR)
  const int srow = lane >> 2;
  const int schunk = (lane & 3) ^ w4_chunk_xor(lane >> 4);
  const bf16* ga[4];
  const bf16* gb[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int r = (wave * 4 + q) * 16 + srow;
    ga[q] = p.A + (int64_t)min(m0 + r, M - 1) * p.lda + schunk * 8;
    gb[q] = p.B + (int64_t)min(n0 + r, N - 1) * p.ldb + schunk * 8;
  }
  // LDS-DMA copy c (0..7) of half-tile j into its slot j % NS: A (c < 4) or B,
  // 16-row block 4 wave + (c & 3)
  // buffer form: descriptors from kernel arguments only (wave-uniform), lane
  // byte offsets of the same rows / chunks.  The K offset goes in soffset: an
  // immediate offset would also move the LDS destination.
  const int64_t abytes = ((int64_t)(M - 1) * p.lda + K) * 2, bbytes = ((int64_t)(N - 1) * p.ldb + K) * 2;
  const auto rsa = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, (int)min(abytes, (int64_t)0x7fffffff),
                                                     0x00020000);
  const auto rsb = __builtin_amdgcn_make_buffer_rsrc((void*)p.B, (short)0, (int)min(bbytes, (int64_t)0x7fffffff),
                                                     0x00020000);
  uint32_t oa[4], ob[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    oa[q] = (uint32_t)((ga[q] - p.A) * 2);
    ob[q] = (uint32_t)((gb[q] - p.B) * 2);
  }
  auto dma = [&](int j, int c) {
    const int q = c & 3;
    char* dst = smem + (j % NS) * SLOT + (c < 4 ? 0 : W4_REGION) + (wave * 4 + q) * 1024;
    if constexpr (BUF)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(c < 4 ? rsa : rsb, (lptr_t)dst, 16, c < 4 ? oa[q] : ob[q], j * 64, 0, 0);
    else
      w4_glds((c < 4 ? ga[q] : gb[q]) + j * 32, dst);
  };

  const int lrow = lane & 15, lk = lane >> 4;
  const int frag_off = lrow * 64 + ((lk ^ w4_chunk_xor(lrow >> 2)) << 4);
  const int aoff = (wr * 128) * 64 + frag_off, boff = W4_REGION + (wc * 128) * 64 + frag_off;
  bf16x8 ra[2][8], rb[2][8];
  // fragment read r (0..15) of half-tile j into register set P: A block r / 2 or B block r / 2
  auto rd = [&](auto pc, int j, int r) {
    constexpr int P = decltype(pc)::value;
    const char* base = smem + (j % NS) * SLOT + ((r & 1) ? boff : aoff) + (r >> 1) * 1024;
    if (r & 1) rb[P][r >> 1] = *reinterpret_cast<const bf16x8*>(base);
    else ra[P][r >> 1] = *reinterpret_cast<const bf16x8*>(base);
  };
  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Segment j (one k32 half-tile: 64 MFMAs per wave, register set j & 1):
  // the fragments of half-tile j + 1 are read into the other set (one
  // ds_read after every 4th MFMA), the copies of half-tile j + NS - 1 go into
  // the slot of half-tile j - 1 (one after every 8th MFMA: the CU's 32 copies
  // per segment stay spread over it instead of queueing on the address path
  // together, finding 69), then the wait retires half-tile j + 2 (read in
  // segment j + 1) and leaves the NS - 3 younger half-tiles in flight, and
  // the barrier publishes it and frees slot j for segment j + 1's copies.
  // WAR: slot (j - 1) % NS was last read in segment j - 2, before its barrier.
  // Operands swapped: acc[i][j] holds the transposed 16 x 16 block (lane =
  // output row i*16 + (l & 15), registers = 4 consecutive output columns).
  auto seg = [&](auto pc, auto steady, int j) {
    constexpr int P = decltype(pc)::value;
    constexpr bool STEADY = decltype(steady)::value;
    const bool do_rd = STEADY || j + 1 < nh, do_dma = STEADY || j + NS - 1 < nh;
#pragma unroll
    for (int n = 0; n < 64; ++n) {
      w4_mfma(acc[n >> 3][n & 7], rb[P][n & 7], ra[P][n >> 3]);
      if ((n & 3) == 0 && do_rd) rd(std::integral_constant<int, P ^ 1>{}, j + 1, n >> 2);
      if ((n & 7) == 2 && do_dma) dma(j + NS - 1, n >> 3);
    }
    if constexpr (NOWAIT) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    } else if constexpr (STEADY) {
      asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)" ::"n"(8 * (NS - 3)) : "memory");
    } else {
      const int out = min(NS - 3, max(0, min(j + NS - 1, nh - 1) - (j + 2)));
      if (out >= 2) asm volatile("s_waitcnt vmcnt(16)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
      else if (out == 1) asm volatile("s_waitcnt vmcnt(8)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
    }
    w4_barrier();
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;

  // prologue: half-tiles 0 .. NS - 2 in flight, 0 and 1 retired, 0 read
#pragma unroll
  for (int j = 0; j < NS - 1; ++j)
    if (j < nh)
#pragma unroll
      for (int c = 0; c < 8; ++c) dma(j, c);
  {
    const int out = min(NS - 3, max(0, nh - 2));
    if (out >= 2) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (out == 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  w4_barrier();
#pragma unroll
  for (int r = 0; r < 16; ++r) rd(I0{}, 0, r);
  int j = 0;
  for (; j + NS < nh; j += 2) {  // both segments issue their copies
    seg(I0{}, std::true_type{}, j);
    seg(I1{}, std::true_type{}, j + 1);
  }
  for (; j < nh; j += 2) {
    seg(I0{}, std::false_type{}, j);
    seg(I1{}, std::false_type{}, j + 1);
  }
  w4_mfma_drain();

  // prototype epilogue: 8-B row pieces straight from the transposed accumulators
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = m0 + wr * 128 + i * 16 + lrow;
    if (row >= M) continue;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int col = n0 + wc * 128 + j * 16 + lk * 4;
      if (col < N)
        *reinterpret_cast<bf16x4*>(p.C + (int64_t)row * p.ldc + col) = __builtin_convertvector(acc[i][j], bf16x4);
    }
  }
}

// Full-line form: every LDS-DMA instruction copies 8 rows x 128 B (one whole
// K tile of 8 rows: 8 cache lines, each used whole) instead of 16 rows x 64 B
// (16 lines, each half used, the other half fetched by a second
// instruction).  LDS image per operand and K tile: [256 rows][128 B], 16-B
// chunk c of row r stored at chunk c ^ ((r >> 1) & 7): the four 16-lane
// groups of a fragment ds_read_b128 (rows l & 15, chunks 4h + (l >> 4)) hit
// 16 distinct bank slots.  Two K-tile buffers (128 KB); per K tile:
//   S1: k-half 0 MFMAs while reading k-half 1's fragments of tile t;
//       vmcnt(0) (tile t + 1 landed), barrier (buffer t & 1 free);
//   S2: k-half 1 MFMAs while copying tile t + 2 into buffer t & 1 (one copy
//       per 4 MFMAs) and reading k-half 0 of tile t + 1.
__device__ __forceinline__ int w4l_chunk(int c, int row) { return c ^ ((row >> 1) & 7); }

// SPREAD: S2's copies one per 4 MFMAs over the whole segment (else one per 2
// MFMAs in its first half); the fragment reads go first in either case
template <bool SPREAD>
__global__ __launch_bounds__(W4_THREADS, 1) void gemm_w4l_kernel(const W4Args p) {
  constexpr int OPB = 256 * 128, BUF = 2 * OPB;  // one operand's K tile, one buffer
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];
  const int M = p.M, N = p.N, K = p.K;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int mtiles = (M + W4_BM - 1) / W4_BM, ntiles = (N + W4_BN - 1) / W4_BN;
  int mt, nt;
  w4_tile(mtiles * ntiles, mtiles, ntiles, p.group_m, mt, nt);
  const int m0 = mt * W4_BM, n0 = nt * W4_BN;
  const int ktiles = K / W4_BK;

  // copy c (0..15) of a K tile: operand c >> 3, 8-row piece 8 wave + (c & 7);
  // lane L: row 8 piece + (L >> 3), stored chunk L & 7, logical chunk swz
  const int64_t abytes = ((int64_t)(M - 1) * p.lda + K) * 2, bbytes = ((int64_t)(N - 1) * p.ldb + K) * 2;
  const auto rsa = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, (int)min(abytes, (int64_t)0x7fffffff),
                                                     0x00020000);
  const auto rsb = __builtin_amdgcn_make_buffer_rsrc((void*)p.B, (short)0, (int)min(bbytes, (int64_t)0x7fffffff),
                                                     0x00020000);
  uint32_t off[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    const int row = (wave * 8 + (c & 7)) * 8 + (lane >> 3);
    const int lc = w4l_chunk(lane & 7, row);
    off[c] = c < 8 ? (uint32_t)(((int64_t)min(m0 + row, M - 1) * p.lda + lc * 8) * 2)
                   : (uint32_t)(((int64_t)min(n0 + row, N - 1) * p.ldb + lc * 8) * 2);
  }
  auto dma = [&](int kt, int buf, int c) {
    char* dst = smem + buf * BUF + (c >> 3) * OPB + (wave * 8 + (c & 7)) * 1024;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(c < 8 ? rsa : rsb, (lptr_t)dst, 16, off[c], kt * 128, 0, 0);
  };

  const int lrow = lane & 15, lk = lane >> 4;
  // fragment byte offset within a 16-row block for k half h
  const int fo0 = lrow * 128 + (w4l_chunk(lk, lrow) << 4), fo1 = lrow * 128 + (w4l_chunk(4 + lk, lrow) << 4);
  const int aoff = wr * 128 * 128, boff = OPB + wc * 128 * 128;
  bf16x8 ra[2][8], rb[2][8];
  // read r (0..15) in the order the MFMAs consume them: A block 0, B blocks
  // 0..7, A blocks 1..7
  auto rd = [&](auto hc, int buf, int r) {
    constexpr int H = decltype(hc)::value;
    const bool isb = r >= 1 && r <= 8;
    const int blk = r == 0 ? 0 : (isb ? r - 1 : r - 8);
    const char* base = smem + buf * BUF + (isb ? boff : aoff) + blk * 2048 + (H ? fo1 : fo0);
    if (isb) rb[H][blk] = *reinterpret_cast<const bf16x8*>(base);
    else ra[H][blk] = *reinterpret_cast<const bf16x8*>(base);
  };
  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  auto iter = [&](auto st, auto rdn, int kt) {
    constexpr bool STAGE = decltype(st)::value, READ = decltype(rdn)::value;
    const int buf = kt & 1;
#pragma unroll
    for (int n = 0; n < 64; ++n) {
      w4_mfma(acc[n >> 3][n & 7], rb[0][n & 7], ra[0][n >> 3]);
      if ((n & 3) == 0) rd(I1{}, buf, n >> 2);
    }
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
    w4_barrier();
#pragma unroll
    for (int n = 0; n < 64; ++n) {
      w4_mfma(acc[n >> 3][n & 7], rb[1][n & 7], ra[1][n >> 3]);
      if constexpr (SPREAD) {
        if constexpr (STAGE)
          if ((n & 3) == 0) dma(kt + 2, buf, n >> 2);
        if constexpr (READ)
          if ((n & 1) == 1 && n < 32) rd(I0{}, buf ^ 1, n >> 1);
      } else {
        if constexpr (READ)
          if ((n & 1) == 0 && n < 32) rd(I0{}, buf ^ 1, n >> 1);
        if constexpr (STAGE)
          if ((n & 1) == 1 && n < 32) dma(kt + 2, buf, n >> 1);
      }
    }
  };
#pragma unroll
  for (int c = 0; c < 16; ++c) dma(0, 0, c);
  if (ktiles > 1) {
#pragma unroll
    for (int c = 0; c < 16; ++c) dma(1, 1, c);
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  w4_barrier();
#pragma unroll
  for (int r = 0; r < 16; ++r) rd(I0{}, 0, r);
  int kt = 0;
  for (; kt + 2 < ktiles; ++kt) iter(std::true_type{}, std::true_type{}, kt);
  if (kt + 1 < ktiles) iter(std::false_type{}, std::true_type{}, kt++);
  iter(std::false_type{}, std::false_type{}, kt);
  w4_mfma_drain();
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = m0 + wr * 128 + i * 16 + lrow;
    if (row >= M) continue;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int col = n0 + wc * 128 + j * 16 + lk * 4;
      if (col < N)
        *reinterpret_cast<bf16x4*>(p.C + (int64_t)row * p.ldc + col) = __builtin_convertvector(acc[i][j], bf16x4);
    }
  }
}

}  // namespace

at::Tensor gemm_w4(const at::Tensor& A, const at::Tensor& B, int64_t group_m, int64_t variant) {
  TORCH_CHECK(A.is_cuda() && B.is_cuda() && A.scalar_type() == at::kBFloat16 && B.scalar_type() == at::kBFloat16 &&
                  A.dim() == 2 && B.dim() == 2, "gemm_w4: A, B must be 2-D bf16 GPU tensors");
  TORCH_CHECK(A.stride(1) == 1 && B.stride(1) == 1 && A.stride(0) % 8 == 0 && B.stride(0) % 8 == 0,
              "gemm_w4: rows must be contiguous and 16-B aligned");
  const int64_t M = A.size(0), K = A.size(1), N = B.size(0);
  TORCH_CHECK(B.size(1) == K && K % 64 == 0 && K > 0 && N % 8 == 0 && M > 0 && M < (1LL << 31),
              "gemm_w4: shapes");
  auto C = at::empty({M, N}, A.options());
  W4Args a{};
  a.A = reinterpret_cast<const bf16*>(A.data_ptr()); a.lda = A.stride(0);
  a.B = reinterpret_cast<const bf16*>(B.data_ptr()); a.ldb = B.stride(0);
  a.C = reinterpret_cast<bf16*>(C.data_ptr()); a.ldc = C.stride(0);
  a.M = (int)M; a.N = (int)N; a.K = (int)K;
  a.group_m = group_m > 0 ? (int)group_m : 4;
  const int blocks = (int)(((M + W4_BM - 1) / W4_BM) * ((N + W4_BN - 1) / W4_BN));
  hipStream_t st = at::hip::getCurrentHIPStream();
  switch (variant) {
    case 4: hipLaunchKernelGGL((gemm_w4_kernel<4, false, false>), dim3(blocks), dim3(W4_THREADS), 0, st, a); break;
    case 5: hipLaunchKernelGGL((gemm_w4_kernel<5, false, false>), dim3(blocks), dim3(W4_THREADS), 0, st, a); break;
    case 14: hipLaunchKernelGGL((gemm_w4_kernel<4, true, false>), dim3(blocks), dim3(W4_THREADS), 0, st, a); break;
    case 15: hipLaunchKernelGGL((gemm_w4_kernel<5, true, false>), dim3(blocks), dim3(W4_THREADS), 0, st, a); break;
    case 104: hipLaunchKernelGGL((gemm_w4_kernel<4, false, true>), dim3(blocks), dim3(W4_THREADS), 0, st, a); break;
    case 20: hipLaunchKernelGGL(gemm_w4l_kernel<true>, dim3(blocks), dim3(W4_THREADS), 0, st, a); break;
    case 21: hipLaunchKernelGGL(gemm_w4l_kernel<false>, dim3(blocks), dim3(W4_THREADS), 0, st, a); break;
    default: TORCH_CHECK(false, "gemm_w4: variant must be 4, 5, 14, 15, 20, 21 or 104");
  }
  DMP_HIP_CHECK(hipGetLastError());
  return C;
}

}  // namespace dmp
