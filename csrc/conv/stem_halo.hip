// ResNet stem (7x7 / stride 2 / pad 3, 3 -> 64 channels at 224x224) as two
// persistent halo-tiled MFMA kernels on the space-to-depth image.
//
// ops/stem.py turns the conv into a 4x4 / stride-1 conv over the 2x2
// space-to-depth image s [N][115][115][16] (12 real channels + 4 zero, the
// zero padding already baked in), K = 16 taps x 16 channels = 256:
//     y[p][co] = sum_{kh,kw,c} s[p + (kh, kw)][c] * Wm[co][(kh*4 + kw)*16 + c].
// On the generic implicit GEMM (conv_nt / conv_wgrad, kc = 64 row taps) the
// forward ran at ~290 TF/s and the weight gradient at ~310 TF/s (2.9 + 2.7 ms
// per step at batch 2048, profiles/r50_ddp_bs2048_1gpu_v21.md): N = 64 output
// channels is the weak shape of a 128-wide GEMM tile, and every s pixel is
// gathered 16 times through L2.  Here a tile of output rows streams through
// LDS once:
//
// stem_fwd: the whole 64 x 256 weight matrix lives in VGPRs as MFMA B
//   fragments (128 registers, loaded once per persistent block); a tile is R = 4
//   output rows (448 pixels = 28 fragments of 16); its input slab -- 7 full s
//   rows, one contiguous 25.8 KB run of memory -- lands by LDS-DMA, double
//   buffered.  4 waves x 7 pixel fragments x 4 channel fragments, 8 k-steps
//   (2 taps each); every A fragment is one ds_read_b128 (16 consecutive pixels
//   x 8 channels; 32-B pixels keep each 16-lane group on 16 distinct bank
//   slots with no swizzle).  The output tile is restaged through LDS and
//   written with 16-B stores; MOM: per-channel (sum, sum^2) of the bf16 outputs
//   as the BN moments partial rows (gemm_bf16.hip's EPI_MOMENTS contract).
//
// stem_wgrad: the halo weight gradient of csrc/conv/wgrad3x3.hip for this
//   geometry: each block keeps a 64 x 256 fp32 dW partial in registers
//   (4 waves x 64 co x 4 taps), tiles of R = 2 output rows (224 pixels = 7
//   k-steps of 32) stream their dy rows and their 5-row s slab through LDS
//   (double buffered), both operands read with ds_read_b64_tr_b16; 8
//   consecutive 32-B s pixels per half-wave read = one bank row, so the s
//   image needs no swizzle and every tap offset rides in the instruction's
//   offset field.  Partials are summed in a fixed order (reproducible).
//
// Reference: the torchvision ResNet stem the reference's image models use
// (reference model_parallel.py:61 cudnn.benchmark).
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include "../common.h"

namespace dmp {

void bn_reduce_partials_launch(const float* part, int rb, int C, double* sums, double count,
                               hipStream_t stream);

namespace {

using bf16 = __bf16;
using lptr_t = __attribute__((address_space(3))) void*;
using v4i16 = short __attribute__((ext_vector_type(4)));
using lds_v4 = __attribute__((address_space(3))) v4i16;
using i16x8 = short __attribute__((ext_vector_type(8)));

constexpr int kWo = 112, kWs = 115, kC = 16, kCo = 64, kK = 256;
constexpr int kPixB = kC * 2;  // 32 B per s pixel

__device__ __attribute__((aligned(16))) uint32_t g_stem_zero[4];

// LDS-DMA from inline asm (see wgrad3x3.hip: the builtin makes hipcc drain
// every pending copy at the next LDS read / barrier)
__device__ __forceinline__ void glds16(const void* g, const char* lds) {
  const uint32_t l = (uint32_t)(uintptr_t)(lptr_t)lds;
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off"
               :: "s"(__builtin_amdgcn_readfirstlane(l)), "v"(g) : "memory", "m0");
}
template <int N>
__device__ __forceinline__ void vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Copy `bytes` contiguous bytes starting at src into LDS `dst` (this wave's
// pieces of a 1-KB-per-instruction lane-linear image); lanes past the end (or
// past the tensor) read the zero buffer.
template <int PIECES_PW, int NW>
__device__ __forceinline__ void slab_issue(const char* src, int64_t bytes, char* dst, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < PIECES_PW; ++i) {
    const int piece = wave + NW * i;
    const int64_t off = (int64_t)piece * 1024 + lane * 16;
    const void* g = off < bytes ? (const void*)(src + off) : (const void*)g_stem_zero;
    glds16(g, dst + piece * 1024);
  }
}

// ============================================================================
// forward
// ============================================================================
constexpr int FR = 4;                       // output rows per tile
constexpr int F_PIX = FR * kWo;             // 448
constexpr int F_FRAG = F_PIX / 16;          // 28
constexpr int F_FW = F_FRAG / 4;            // 7 per wave
constexpr int F_SLAB = (FR + 3) * kWs * kPixB;  // 25760 B
constexpr int F_PIECES = (F_SLAB + 1023) / 1024;  // 26
constexpr int F_PPW = (F_PIECES + 3) / 4;   // 7
constexpr int F_BUF = F_PPW * 4 * 1024;     // 28672
constexpr int F_STAGE = F_PIX * kCo * 2;    // 57344
constexpr int F_SMEM = 2 * F_BUF + F_STAGE + 2 * kCo * 4;
constexpr int F_KS = kK / 32;               // 8 k-steps (2 taps each)

// 16-B chunk swizzle of a staged pixel row: the epilogue writes 16 pixels x
// 16 B per half-wave (transposed accumulators), (p & 1) picks the 128-B half
// of a 256-B bank row and (p >> 1) & 7 the chunk: conflict-free
__device__ __forceinline__ int stage_key(int p) { return (p >> 1) & 7; }

template <bool MOM>
__global__ __launch_bounds__(256, 1) void stem_fwd_kernel(const bf16* __restrict__ s, const bf16* __restrict__ wm,
                                                          bf16* __restrict__ y, float* __restrict__ part,
                                                          double* zsums, int Hs, int Ho, int tiles,
                                                          int tiles_per_img, int64_t s_bytes) {
  __shared__ __attribute__((aligned(1024))) char smem[F_SMEM];
  bf16* ostage = reinterpret_cast<bf16*>(smem + 2 * F_BUF);
  float* mred = reinterpret_cast<float*>(smem + 2 * F_BUF + F_STAGE);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int l15 = lane & 15, lh = lane >> 4;
  if constexpr (MOM) {
    zero_moments(zsums, 2 * kCo);
    if (threadIdx.x < 2 * kCo) mred[threadIdx.x] = 0.f;
  }
  const int t_begin = (int)((int64_t)tiles * blockIdx.x / gridDim.x);
  const int t_end = (int)((int64_t)tiles * (blockIdx.x + 1) / gridDim.x);
  const int64_t img_bytes = (int64_t)Hs * kWs * kPixB;
  auto issue = [&](int t, char* buf) {
    const int n = t / tiles_per_img;
    const int r0 = (t - n * tiles_per_img) * FR;
    const int64_t start = n * img_bytes + (int64_t)r0 * kWs * kPixB;
    const int64_t avail = s_bytes - start;
    slab_issue<F_PPW, 4>(reinterpret_cast<const char*>(s) + start, avail < F_SLAB ? avail : F_SLAB, buf, wave, lane);
  };
  if (t_begin < t_end) issue(t_begin, smem);

  // weights -> B fragments: lane holds Wm[co = 16 nf + l15][k = 32 ks + 8 lh + j]
  bf16x8 bw[4][F_KS];
#pragma unroll
  for (int nf = 0; nf < 4; ++nf)
#pragma unroll
    for (int ks = 0; ks < F_KS; ++ks)
      bw[nf][ks] = *reinterpret_cast<const bf16x8*>(wm + (int64_t)(16 * nf + l15) * kK + 32 * ks + 8 * lh);
  // A fragment f of this wave: pixel 16 (7 wave + f) + l15 of the tile; lane
  // group lh reads tap (kh, 2 (ks & 1) + (lh >> 1)), channels 8 (lh & 1) ..
  int abase[F_FW];
#pragma unroll
  for (int f = 0; f < F_FW; ++f) {
    const int p = 16 * (F_FW * wave + f) + l15;
    const int oy = p / kWo, ox = p - oy * kWo;
    abase[f] = (oy * kWs + ox + (lh >> 1)) * kPixB + (lh & 1) * 16;
  }

  float s8[8], q8[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s8[j] = q8[j] = 0.f;
  int cur = 0;
  for (int t = t_begin; t < t_end; ++t) {
#pragma unroll
    for (int f = 0; f < F_FW; ++f) asm volatile("" : "+v"(abase[f]));
    vmcnt<0>();
    raw_barrier();
    if (t + 1 < t_end) issue(t + 1, smem + (cur ^ 1) * F_BUF);
    const char* hb = smem + cur * F_BUF;

    f32x4 acc[F_FW][4];
#pragma unroll
    for (int f = 0; f < F_FW; ++f)
#pragma unroll
      for (int nf = 0; nf < 4; ++nf) acc[f][nf] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 a[2][F_FW];
    auto load_step = [&](int ks, bf16x8 (&dst)[F_FW]) {
      const int kh = ks >> 1, kw0 = 2 * (ks & 1);
      const int o = (kh * kWs + kw0) * kPixB;
#pragma unroll
      for (int f = 0; f < F_FW; ++f) dst[f] = *reinterpret_cast<const bf16x8*>(hb + abase[f] + o);
    };
    load_step(0, a[0]);
#pragma unroll
    for (int ks = 0; ks < F_KS; ++ks) {
      if (ks + 1 < F_KS) load_step(ks + 1, a[(ks + 1) & 1]);
#pragma unroll
      for (int f = 0; f < F_FW; ++f)
#pragma unroll
        for (int nf = 0; nf < 4; ++nf)
          acc[f][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[nf][ks], a[ks & 1][f], acc[f][nf], 0, 0, 0);  // C^T
      if (ks + 1 < F_KS) {
#pragma unroll
        for (int f = 0; f < F_FW; ++f) {
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // MFMA
        }
        __builtin_amdgcn_sched_group_barrier(0x008, F_FW * 4 - 2 * F_FW, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // epilogue (transposed accumulators): pixel = 16 (F_FW wave + f) + l15,
    // channels 16 nf + 4 lh + i -> one 8-B LDS write per fragment
#pragma unroll
    for (int f = 0; f < F_FW; ++f)
#pragma unroll
      for (int nf = 0; nf < 4; ++nf) {
        const int p = 16 * (F_FW * wave + f) + l15;
        const int ch = (2 * nf + (lh >> 1)) ^ stage_key(p);
        *reinterpret_cast<bf16x4*>(ostage + p * kCo + ch * 8 + (lh & 1) * 4) =
            __builtin_convertvector(acc[f][nf], bf16x4);
      }
    __syncthreads();
    {
      const int n = t / tiles_per_img;
      const int r0 = (t - n * tiles_per_img) * FR;
      const int rows = min(FR, Ho - r0);
      const int chunks = rows * kWo * (kCo / 8);
      bf16* dst = y + (((int64_t)n * Ho + r0) * kWo) * kCo;
      for (int i = threadIdx.x; i < chunks; i += 256) {
        const int sp = i >> 3;
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(ostage + sp * kCo + (((i & 7) ^ stage_key(sp)) << 3));
        *reinterpret_cast<bf16x8*>(dst + (int64_t)i * 8) = v;
        if constexpr (MOM)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float fv = (float)v[j];
            s8[j] += fv;
            q8[j] = fmaf(fv, fv, q8[j]);
          }
      }
    }
    cur ^= 1;
    // the stage is rewritten only after the next tile's MFMA loop, behind the
    // next iteration's barrier
  }
  if constexpr (MOM) {
    // thread t always copied channels 8 (t % 8) .. +7
#pragma unroll
    for (int j = 0; j < 8; ++j) {
#pragma unroll
      for (int off = 8; off < 64; off <<= 1) {
        s8[j] += __shfl_xor(s8[j], off, 64);
        q8[j] += __shfl_xor(q8[j], off, 64);
      }
    }
    if (lane < 8)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        atomicAdd(&mred[8 * lane + j], s8[j]);
        atomicAdd(&mred[kCo + 8 * lane + j], q8[j]);
      }
    __syncthreads();
    if (threadIdx.x < 2 * kCo) {
      const int mo = threadIdx.x / kCo, ch = threadIdx.x % kCo;
      part[((int64_t)mo * gridDim.x + blockIdx.x) * kCo + ch] = mred[mo * kCo + ch];
    }
  }
}

// ============================================================================
// weight gradient
// ============================================================================
constexpr int WR = 2;                         // output rows per tile
constexpr int W_PIX = WR * kWo;               // 224 = 7 k-steps of 32
constexpr int W_KS = W_PIX / 32;
constexpr int W_DY_BYTES = W_PIX * kCo * 2;   // 28672 = 28 pieces
constexpr int W_DY_PPW = W_DY_BYTES / 1024 / 4;  // 7
constexpr int W_SLAB = (WR + 3) * kWs * kPixB;   // 18400
constexpr int W_S_PIECES = (W_SLAB + 1023) / 1024;  // 18
constexpr int W_S_PPW = (W_S_PIECES + 3) / 4;  // 5
constexpr int W_BUF = W_DY_BYTES + W_S_PPW * 4 * 1024;
constexpr int W_SMEM = 2 * W_BUF;

__device__ __forceinline__ int dy_key(int row) { return ((row >> 1) & 3) << 1; }

__global__ __launch_bounds__(256, 1) void stem_wgrad_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ s,
                                                            float* __restrict__ part, int Hs, int Ho, int tiles,
                                                            int tiles_per_img, int64_t s_bytes) {
  __shared__ __attribute__((aligned(1024))) char smem[W_SMEM];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int t_begin = (int)((int64_t)tiles * blockIdx.x / gridDim.x);
  const int t_end = (int)((int64_t)tiles * (blockIdx.x + 1) / gridDim.x);
  const int64_t img_bytes = (int64_t)Hs * kWs * kPixB;

  // dy DMA: piece (wave + 4 i) = dy rows 8 piece .. +7 (128 B each), chunk XOR key
  int dy_off[W_DY_PPW];
#pragma unroll
  for (int i = 0; i < W_DY_PPW; ++i) {
    const int piece = wave + 4 * i;
    const int row = piece * 8 + (lane >> 3);
    dy_off[i] = row * kCo + (((lane & 7) ^ dy_key(row)) * 8);
  }
  auto issue = [&](int t, char* buf) {
    const int n = t / tiles_per_img;
    const int r0 = (t - n * tiles_per_img) * WR;
    const int rows = min(WR, Ho - r0);
    const bf16* dyb = dy + (((int64_t)n * Ho + r0) * kWo) * kCo;
#pragma unroll
    for (int i = 0; i < W_DY_PPW; ++i) {
      const int piece = wave + 4 * i;
      const void* g = (piece * 8 + (lane >> 3)) < rows * kWo ? (const void*)(dyb + dy_off[i]) : (const void*)g_stem_zero;
      glds16(g, buf + piece * 1024);
    }
    const int64_t start = n * img_bytes + (int64_t)r0 * kWs * kPixB;
    const int64_t avail = s_bytes - start;
    slab_issue<W_S_PPW, 4>(reinterpret_cast<const char*>(s) + start, avail < W_SLAB ? avail : W_SLAB,
                           buf + W_DY_BYTES, wave, lane);
  };

  // tr-read geometry (wgrad3x3.hip): lane 16 g + 4 q + p; read r of k-step ks
  // addresses pixel 32 ks + 16 (g >> 1) + 8 r + 4 (g & 1) + q, columns 4 p .. +3
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int pin = 16 * (g >> 1) + 4 * (g & 1) + q;
  const int lofs = (p & 1) * 8 + (p >> 1) * 16;
  int a_base[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) a_base[i] = pin * 128 + (((2 * i) ^ dy_key(pin)) << 4) + lofs;
  // s rows (32 B, unswizzled): pixel pp at tap (kh, kw) -> slab pixel (oy + kh) * 115 + ox + kw
  int sb[W_KS][2];
#pragma unroll
  for (int ks = 0; ks < W_KS; ++ks)
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int pp = 32 * ks + 8 * r + pin;
      const int oy = pp / kWo, ox = pp - oy * kWo;
      sb[ks][r] = (oy * kWs + ox) * kPixB + p * 8 + W_DY_BYTES;
    }

  // wave w: all 64 co (4 A fragments) x taps 4 w .. 4 w + 3 (4 B fragments of 16 channels)
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto run = [&](auto wv_tag) {
    constexpr int WV = decltype(wv_tag)::value;
    if (t_begin < t_end) issue(t_begin, smem);
    int cur = 0;
    for (int t = t_begin; t < t_end; ++t) {
      int sbc[W_KS][2], abc[4];
#pragma unroll
      for (int ks = 0; ks < W_KS; ++ks) {
        asm volatile("" : "+v"(sb[ks][0]), "+v"(sb[ks][1]));
        sbc[ks][0] = sb[ks][0] + cur * W_BUF;
        sbc[ks][1] = sb[ks][1] + cur * W_BUF;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) abc[i] = a_base[i] + cur * W_BUF;
      vmcnt<0>();
      raw_barrier();
      if (t + 1 < t_end) issue(t + 1, smem + (cur ^ 1) * W_BUF);
      auto rd = [&](int addr) -> v4i16 {
        return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(smem + addr));
      };
      bf16x8 fa[2][4], fb[2][4];
      auto load_step = [&](auto ks_tag, bf16x8 (&da)[4], bf16x8 (&db)[4]) {
        constexpr int ks = decltype(ks_tag)::value;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const v4i16 lo = rd(abc[i] + (32 * ks) * 128);
          const v4i16 hi = rd(abc[i] + (32 * ks + 8) * 128);
          const i16x8 t8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          da[i] = __builtin_bit_cast(bf16x8, t8);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int tap = 4 * WV + j, kh = tap >> 2, kw = tap & 3;
          const int o = (kh * kWs + kw) * kPixB;
          const v4i16 lo = rd(sbc[ks][0] + o);
          const v4i16 hi = rd(sbc[ks][1] + o);
          const i16x8 t8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          db[j] = __builtin_bit_cast(bf16x8, t8);
        }
      };
      load_step(std::integral_constant<int, 0>{}, fa[0], fb[0]);
      auto step = [&](auto ks_tag) {
        constexpr int ks = decltype(ks_tag)::value;
        if constexpr (ks + 1 < W_KS)
          load_step(std::integral_constant<int, ks + 1>{}, fa[(ks + 1) & 1], fb[(ks + 1) & 1]);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[ks & 1][i], fb[ks & 1][j], acc[i][j], 0, 0, 0);
        if constexpr (ks + 1 < W_KS) {
#pragma unroll
          for (int u = 0; u < 16; ++u) {  // 16 reads over 16 MFMAs
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      };
      step(std::integral_constant<int, 0>{});
      step(std::integral_constant<int, 1>{});
      step(std::integral_constant<int, 2>{});
      step(std::integral_constant<int, 3>{});
      step(std::integral_constant<int, 4>{});
      step(std::integral_constant<int, 5>{});
      step(std::integral_constant<int, 6>{});
      static_assert(W_KS == 7, "unrolled k-steps");
      cur ^= 1;
    }
  };
  switch (wave) {
    case 0: run(std::integral_constant<int, 0>{}); break;
    case 1: run(std::integral_constant<int, 1>{}); break;
    case 2: run(std::integral_constant<int, 2>{}); break;
    default: run(std::integral_constant<int, 3>{}); break;
  }
  // partial [64 co][256]: row co = 16 i + 4 g + e, column = 64 wave + 16 j + (lane & 15)
  float* pb = part + (int64_t)blockIdx.x * (kCo * kK);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        pb[(16 * i + 4 * g + e) * kK + 64 * wave + 16 * j + (lane & 15)] = acc[i][j][e];
}

// out[e] = sum over nb partial rows (fixed order); block = 4 row groups x 64 x 4 columns
template <typename OT>
__global__ __launch_bounds__(256) void partial_sum_kernel(const float* __restrict__ part, int nb, int n,
                                                          OT* __restrict__ out) {
  const int grp = threadIdx.x >> 6, tl = threadIdx.x & 63;
  const int e0 = (blockIdx.x * 64 + tl) * 4;
  f32x4 acc[4] = {};
  if (e0 < n) {
    int b = grp;
    for (; b + 12 < nb; b += 16) {
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] += *reinterpret_cast<const f32x4*>(part + (int64_t)(b + 4 * u) * n + e0);
    }
    for (; b < nb; b += 4) acc[0] += *reinterpret_cast<const f32x4*>(part + (int64_t)b * n + e0);
  }
  __shared__ f32x4 red[256];
  red[threadIdx.x] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  __syncthreads();
  if (grp == 0 && e0 < n) {
    const f32x4 v = ((red[tl] + red[64 + tl]) + red[128 + tl]) + red[192 + tl];
#pragma unroll
    for (int u = 0; u < 4; ++u) out[e0 + u] = (OT)v[u];
  }
}

int num_cus() {
  int dev = 0, cus = 256;
  DMP_HIP_CHECK(hipGetDevice(&dev));
  DMP_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  return cus;
}

void check_s(const at::Tensor& s, int64_t ho) {
  TORCH_CHECK(s.is_cuda() && s.scalar_type() == at::kBFloat16 && s.dim() == 4 && s.size(1) == kC &&
                  s.size(3) == kWs && s.is_contiguous(at::MemoryFormat::ChannelsLast),
              "stem halo: s must be the [N, 16, Hs, 115] channels_last space-to-depth image");
  TORCH_CHECK(s.size(2) >= ho + 3, "stem halo: Hs >= Ho + 3");
}

}  // namespace

bool stem_halo_supported(int64_t hs, int64_t ws, int64_t ho, int64_t wo) {
  return ws == kWs && wo == kWo && hs >= ho + 3 && ho % FR == 0;
}

// y = stem conv of the s2d image s (ops/stem.py), wm: [64, 256] bf16.
// Returns (y [N*Ho*112, 64], moments fp64 [129] or empty).
std::vector<at::Tensor> stem_halo_fwd(const at::Tensor& s, const at::Tensor& wm, int64_t ho, bool moments) {
  check_s(s, ho);
  TORCH_CHECK(ho % FR == 0, "stem halo fwd: Ho % 4 == 0");
  TORCH_CHECK(wm.is_cuda() && wm.scalar_type() == at::kBFloat16 && wm.is_contiguous() && wm.size(0) == kCo &&
                  wm.size(1) == kK, "stem halo fwd: wm must be contiguous [64, 256] bf16");
  const int64_t n = s.size(0), hs = s.size(2);
  const int tpi = (int)(ho / FR);
  const int tiles = (int)(n * tpi);
  auto y = at::empty({n * ho * kWo, kCo}, s.options());
  auto stream = at::hip::getCurrentHIPStream();
  if (tiles == 0) return {y, at::zeros({moments ? 2 * kCo + 1 : 0}, s.options().dtype(at::kDouble))};
  const int grid = std::min(tiles, num_cus());
  const int64_t s_bytes = s.numel() * 2;
  at::Tensor mom;
  if (moments) {
    mom = at::empty({2 * kCo + 1}, s.options().dtype(at::kDouble));
    auto part = at::empty({2, grid, kCo}, s.options().dtype(at::kFloat));
    hipLaunchKernelGGL(stem_fwd_kernel<true>, dim3(grid), dim3(256), 0, stream,
                       reinterpret_cast<const bf16*>(s.data_ptr()), reinterpret_cast<const bf16*>(wm.data_ptr()),
                       reinterpret_cast<bf16*>(y.data_ptr()), part.data_ptr<float>(),
                       moments_zero_target(mom.data_ptr<double>(), grid), (int)hs, (int)ho, tiles, tpi, s_bytes);
    bn_reduce_partials_launch(part.data_ptr<float>(), grid, kCo, mom.data_ptr<double>(), (double)(n * ho * kWo),
                              stream);
  } else {
    mom = at::empty({0}, s.options().dtype(at::kDouble));
    hipLaunchKernelGGL(stem_fwd_kernel<false>, dim3(grid), dim3(256), 0, stream,
                       reinterpret_cast<const bf16*>(s.data_ptr()), reinterpret_cast<const bf16*>(wm.data_ptr()),
                       reinterpret_cast<bf16*>(y.data_ptr()), nullptr, nullptr, (int)hs, (int)ho, tiles, tpi,
                       s_bytes);
  }
  DMP_HIP_CHECK(hipGetLastError());
  return {y, mom};
}

// dWm [64, 256] (out_dtype) of the stem: dy [N*Ho*112, 64] bf16 rows, s the s2d image
at::Tensor stem_halo_wgrad(const at::Tensor& dy, const at::Tensor& s, int64_t ho, at::ScalarType out_dtype) {
  check_s(s, ho);
  const int64_t n = s.size(0), hs = s.size(2);
  TORCH_CHECK(dy.is_cuda() && dy.scalar_type() == at::kBFloat16 && dy.is_contiguous() && dy.dim() == 2 &&
                  dy.size(0) == n * ho * kWo && dy.size(1) == kCo,
              "stem halo wgrad: dy must be contiguous [N*Ho*112, 64] bf16");
  const int tpi = (int)((ho + WR - 1) / WR);
  const int tiles = (int)(n * tpi);
  auto out = at::empty({kCo, kK}, s.options().dtype(out_dtype));
  auto stream = at::hip::getCurrentHIPStream();
  if (tiles == 0) return out.zero_();
  const int grid = std::min(tiles, num_cus());
  auto part = at::empty({(int64_t)grid * kCo * kK}, s.options().dtype(at::kFloat));
  hipLaunchKernelGGL(stem_wgrad_kernel, dim3(grid), dim3(256), 0, stream,
                     reinterpret_cast<const bf16*>(dy.data_ptr()), reinterpret_cast<const bf16*>(s.data_ptr()),
                     part.data_ptr<float>(), (int)hs, (int)ho, tiles, tpi, (int64_t)s.numel() * 2);
  DMP_HIP_CHECK(hipGetLastError());
  const int nel = kCo * kK;
  if (out_dtype == at::kFloat)
    hipLaunchKernelGGL(partial_sum_kernel<float>, dim3(nel / 256), dim3(256), 0, stream, part.data_ptr<float>(),
                       grid, nel, out.data_ptr<float>());
  else {
    TORCH_CHECK(out_dtype == at::kBFloat16, "stem halo wgrad: fp32 or bf16 output");
    hipLaunchKernelGGL(partial_sum_kernel<bf16>, dim3(nel / 256), dim3(256), 0, stream, part.data_ptr<float>(),
                       grid, nel, reinterpret_cast<bf16*>(out.data_ptr()));
  }
  DMP_HIP_CHECK(hipGetLastError());
  return out;
}


// ---------------------------------------------------------------------------
// Tail of the folded stem weight gradient (ops/fused.py _StemBNReLUMaxPoolFn):
//   dW[o][(r*4 + q)*16 + c] = al[o] t_dz[o][k] + be[o] t_y[o][k] + cc[o] cols[k]
// with the BN-backward coefficients of output channel o
//   al = invstd w,  be = -al invstd^2 sum(dz (x - mean)) / cnt,
//   cc = -al sum(dz) / cnt - be mean
// and cols[(r, q, c)] = sum over oh < ho, ow < wo of img[oh + r][ow + q][c],
// img = the batch sum of the space-to-depth image.  One block: the 4 column
// window sums of every img row by a sliding window (fp64), then the 4 row
// windows of those -- the 16 x 16 rectangle sums the torch version formed from
// fp64 2-D prefix sums over ~20 small launches (~0.24 ms a step at any batch).
namespace {
constexpr int kFoldThreads = 256;

__global__ __launch_bounds__(1024) void stem_fold_finish_kernel(
    const float* __restrict__ img, int hs, int ws, int ho, int wo, const float* __restrict__ tdz,
    const float* __restrict__ ty, const double* __restrict__ sums, const double* __restrict__ cnt,
    const float* __restrict__ invstd, const float* __restrict__ w, const float* __restrict__ mean,
    float* __restrict__ out32, bf16* __restrict__ out16) {
  constexpr int CH = 16, NQ = 4, CO = kCo, KK = 256;
  extern __shared__ __attribute__((aligned(16))) char fold_smem[];
  double* rw = reinterpret_cast<double*>(fold_smem);  // [hs][NQ][CH] row-window sums
  __shared__ double cols[KK];
  __shared__ double coef[3][CO];
  const int tid = threadIdx.x;
  // phase 1: rw[h][q][c] = sum_{x = q}^{q + wo - 1} img[h][x][c]
  for (int hc = tid; hc < hs * CH; hc += blockDim.x) {
    const int h = hc / CH, c = hc - h * CH;
    const float* row = img + (int64_t)h * ws * CH + c;
    // four independent partial sums, 16 loads in flight: the single-block kernel
    // was a chain of wo dependent load round trips per (row, channel) item
    // (0.26 ms per step, round 6)
    double a[4] = {0.0, 0.0, 0.0, 0.0};
    int x = 0;
#pragma unroll 4
    for (; x + 4 <= wo; x += 4) {
#pragma unroll
      for (int u = 0; u < 4; ++u) a[u] += (double)row[(x + u) * CH];
    }
    for (; x < wo; ++x) a[0] += (double)row[x * CH];
    double s = (a[0] + a[1]) + (a[2] + a[3]);
    rw[(h * NQ + 0) * CH + c] = s;
    for (int q = 1; q < NQ; ++q) {
      s += (double)row[(q + wo - 1) * CH] - (double)row[(q - 1) * CH];
      rw[(h * NQ + q) * CH + c] = s;
    }
  }
  if (tid < CO) {
    const double n = cnt[0], is = (double)invstd[tid];
    const double al = is * (w ? (double)w[tid] : 1.0);
    const double be = -al * is * is * sums[CO + tid] / n;
    coef[0][tid] = al;
    coef[1][tid] = be;
    coef[2][tid] = -al * sums[tid] / n - be * (double)mean[tid];
  }
  __syncthreads();
  // phase 2: cols[(r*4 + q)*16 + c] = sum_{y = r}^{r + ho - 1} rw[y][q][c]
  if (tid < NQ * CH) {
    const int q = tid / CH, c = tid - q * CH;
    double a[4] = {0.0, 0.0, 0.0, 0.0};
    int y = 0;
#pragma unroll 2
    for (; y + 4 <= ho; y += 4) {
#pragma unroll
      for (int u = 0; u < 4; ++u) a[u] += rw[((y + u) * NQ + q) * CH + c];
    }
    for (; y < ho; ++y) a[0] += rw[(y * NQ + q) * CH + c];
    double s = (a[0] + a[1]) + (a[2] + a[3]);
    cols[(0 * NQ + q) * CH + c] = s;
    for (int r = 1; r < NQ; ++r) {
      s += rw[((r + ho - 1) * NQ + q) * CH + c] - rw[((r - 1) * NQ + q) * CH + c];
      cols[(r * NQ + q) * CH + c] = s;
    }
  }
  __syncthreads();
  // phase 3: the weight gradient
  for (int e = tid; e < CO * KK; e += blockDim.x) {
    const int o = e / KK, k = e - o * KK;
    const double v = coef[0][o] * (double)tdz[e] + coef[1][o] * (double)ty[e] + coef[2][o] * cols[k];
    if (out16) out16[e] = (bf16)(float)v;
    else out32[e] = (float)v;
  }
}
}  // namespace

at::Tensor stem_fold_finish(const at::Tensor& img, int64_t ho, int64_t wo, const at::Tensor& t_dz,
                            const at::Tensor& t_y, const at::Tensor& sums, const at::Tensor& cnt,
                            const at::Tensor& invstd, const c10::optional<at::Tensor>& weight, const at::Tensor& mean,
                            at::ScalarType out_dtype) {
  TORCH_CHECK(img.is_cuda() && img.scalar_type() == at::kFloat && img.dim() == 3 && img.size(2) == 16 &&
                  img.is_contiguous(), "stem_fold_finish: img must be contiguous fp32 [hs, ws, 16]");
  const int64_t hs = img.size(0), ws = img.size(1);
  TORCH_CHECK(ho >= 1 && wo >= 1 && ho + 3 <= hs && wo + 3 <= ws, "stem_fold_finish: window geometry");
  auto f32 = [&](const at::Tensor& t, int64_t n, const char* name) {
    TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous() && t.numel() == n &&
                    t.device() == img.device(), "stem_fold_finish: ", name, " must be contiguous fp32 [", n, "]");
    return t.data_ptr<float>();
  };
  const float* tdz = f32(t_dz, (int64_t)kCo * 256, "t_dz");
  const float* ty = f32(t_y, (int64_t)kCo * 256, "t_y");
  const float* is = f32(invstd, kCo, "invstd");
  const float* mu = f32(mean, kCo, "mean");
  const float* wp = nullptr;
  if (weight.has_value() && weight->defined()) wp = f32(*weight, kCo, "weight");
  TORCH_CHECK(sums.is_cuda() && sums.scalar_type() == at::kDouble && sums.is_contiguous() && sums.numel() >= 2 * kCo,
              "stem_fold_finish: sums must be fp64 [>= 2 * 64] (sum dz, sum dz (x - mean))");
  TORCH_CHECK(cnt.is_cuda() && cnt.scalar_type() == at::kDouble && cnt.numel() >= 1, "stem_fold_finish: cnt fp64");
  TORCH_CHECK(out_dtype == at::kFloat || out_dtype == at::kBFloat16, "stem_fold_finish: fp32 or bf16 output");
  auto out = at::empty({kCo, 256}, img.options().dtype(out_dtype));
  const size_t lds = (size_t)hs * 4 * 16 * sizeof(double);
  TORCH_CHECK(lds <= 96 * 1024, "stem_fold_finish: image too tall for the row-window buffer");
  hipStream_t st = at::hip::getCurrentHIPStream();
  hipLaunchKernelGGL(stem_fold_finish_kernel, dim3(1), dim3(1024), lds, st, img.data_ptr<float>(), (int)hs,
                     (int)ws, (int)ho, (int)wo, tdz, ty, sums.data_ptr<double>(), cnt.data_ptr<double>(), is, wp, mu,
                     out_dtype == at::kFloat ? out.data_ptr<float>() : nullptr,
                     out_dtype == at::kBFloat16 ? reinterpret_cast<bf16*>(out.data_ptr()) : nullptr);
  DMP_HIP_CHECK(hipGetLastError());
  return out;
}

}  // namespace dmp
