// 3x3 / stride-1 / pad-1 convolution for 64 -> 64 channels (ResNet-50 layer 1:
// 56x56, forward and data gradient) as a persistent, halo-tiled MFMA kernel.
//
// Why not the implicit GEMM: at Cin = Cout = 64 the tap-gather GEMMs
// (conv_nt, MIOpen's igemm) re-read every input pixel 9 times through L2 and
// run 3.7-4.6x over the conv's HBM floor (profiles/raw_r2/roofline_stem_l1.log:
// l1 conv2 fwd 0.51 ms, dgrad 0.62 ms at batch 1024 vs a 0.137 ms floor).
// Here each block keeps:
//   * the whole weight tensor in VGPRs, as MFMA B fragments: wave (wm, wn)
//     owns Cout [32 wn, 32 wn + 32) = 2 x 16 columns over the 18 k32 steps of
//     K = 9 taps x 64 channels (144 VGPRs, loaded once per persistent block);
//   * a (R+2) x (W+2)-pixel input halo in LDS (the zero padding included),
//     staged by global_load_lds_dwordx4 (LDS DMA, no VGPR round trip) and
//     double buffered: tile t+1's halo streams in while tile t multiplies;
//   * the R x W output pixels of a tile as one flat M range (R = 4, W = 56:
//     224 pixels = 14 row fragments of 16; wave row wm takes 7 of them), so
//     no MFMA row is padding.
// Every A fragment read is a ds_read_b128 of one halo pixel's 8 channels at
// tap offset (kh, kw); the 16-B chunk of a pixel is XOR-swizzled by a key of
// the pixel index (halo_key; applied to the DMA source address, undone on the read).
// Tiles are R full output rows of one image, so a tile's output is one
// contiguous 28 KB run of y: the epilogue restages it through LDS and writes
// it with 16-B row-contiguous stores.  Blocks take contiguous tile ranges
// (adjacent tiles share 2 halo rows in L2).  MOM: the block accumulates
// per-channel (sum, sum^2) of the bf16-rounded outputs over all its tiles and
// writes one partial row (gemm_bf16.hip's EPI_MOMENTS contract, reduced by
// bn_reduce_partials_launch).
//
// The data gradient of the same conv is this kernel over dy with the weights
// flipped and transposed (ops/conv_igemm.py), so one kernel serves both.
// Reference: the convolutions it replaces are torchvision ResNet-50's
// cuDNN/MIOpen 3x3s (reference model_parallel.py:61).
#include <cstdlib>
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include "../common.h"

namespace dmp {

void bn_reduce_partials_launch(const float* part, int rb, int C, double* sums, double count,
                               hipStream_t stream);

namespace {

using bf16 = __bf16;
using gptr_t = const __attribute__((address_space(1))) void*;
using lptr_t = __attribute__((address_space(3))) void*;

constexpr int C64 = 64;            // channels in and out
constexpr int KSTEPS = 9 * C64 / 32;  // 18 k32 steps

// 16 zero bytes the DMA reads for padding / out-of-image halo pixels
__device__ __attribute__((aligned(16))) uint32_t g_halo_zero[4];

template <int W, int R, int NW>
struct HaloGeo {
  static constexpr int NT = 64 * NW;                      // threads (NW waves: 2 M x NW/2 N)
  static constexpr int NFW = 8 / NW;                      // 16-channel output fragments per wave
  static constexpr int HW2 = W + 2;                       // halo row length (pixels)
  static constexpr int PIX = (R + 2) * HW2;               // halo pixels
  static constexpr int DMA_INSTR = (PIX * 8 + 63) / 64;   // 1 KB wave instructions per halo
  static constexpr int DMA_PER_WAVE = (DMA_INSTR + NW - 1) / NW;
  static constexpr int BUF_BYTES = DMA_PER_WAVE * NW * 1024;
  static constexpr int OUT_PIX = R * W;
  static constexpr int SMEM_BYTES = 2 * BUF_BYTES + OUT_PIX * 64 * 2 + 2 * 64 * 4;  // halo x2, stage, moments
  static constexpr int MFRAG = OUT_PIX / 16;              // row fragments per tile
  static constexpr int MF_WAVE = MFRAG / 2;               // per wave row
  static constexpr int STORES_PER_THREAD = OUT_PIX * 8 / NT;  // 16-B output chunks, full tile
  static constexpr bool STORES_EXACT = OUT_PIX * 8 % NT == 0;
  static_assert(NW == 4 || NW == 8, "4 waves (2 x 32 channels each) or 8 (1 x 16)");
  static_assert(OUT_PIX % 32 == 0, "R*W must split into 2 x 16-row fragments");
};

// 16-B chunk swizzle of halo pixel q (128 B = 8 chunks).  A fragment read has
// lane l on pixel q0 + (l & 15), chunk c0 + (l >> 4), and q0 takes every
// residue (the tap offsets kh * 58 + kw); ds_read_b128 is serviced in 16-lane
// groups {0-3,12-15,20-27}, {4-11,16-19,28-31} and their +32 images.  This
// period-8 table keeps every group on 16 distinct 16-B bank slots for all 16
// residues of q0 (exhaustive check; the (q >> 1) & 7 key of the GEMM tiles is
// conflict-free only for 4-aligned q0 and measured 17 % of the kernel in
// SQ_LDS_BANK_CONFLICT cycles).
constexpr uint32_t kHaloKeys = 0x31165572u;  // nibble i = key of residue i
__device__ __forceinline__ int halo_key(int q) { return (0x31165572u >> (4 * (q & 7))) & 7; }

// output stage [pixel][64 ch]: 16-B chunk swizzle by pixel (even values, so a
// channel pair of chunks stays adjacent)
// 16-B chunk swizzle of a staged pixel row: the epilogue writes 16 pixels x
// 16 B per half-wave (transposed accumulators), (p & 1) picks the 128-B half
// of a 256-B bank row and (p >> 1) & 7 the chunk: conflict-free
__device__ __forceinline__ int stage_key(int p) { return (p >> 1) & 7; }

// LDS-DMA from inline asm (see wgrad3x3.hip): with the builtin, hipcc cannot
// tell which LDS bytes a pending copy writes and drains it (vmcnt(0)) at the
// next LDS access / __syncthreads -- here the epilogue's stage barrier waited
// for the NEXT tile's halo every tile.  The explicit counted vmcnt + barrier
// at the top of each tile is the only ordering the copies need.
__device__ __forceinline__ void glds16(const void* g, char* lds) {
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

// The tile-invariant part of this lane's LDS-DMA slots: slot i of wave w is
// 16-B piece g = (11 w + i) * 64 + lane of the lane-linear halo image, i.e.
// halo pixel q = g / 8 and (swizzled) channel chunk c.  Packed per slot as
// (element offset from the tile's first output row) << 3 | halo row, plus a
// bitmask of the slots whose column is inside the image.
template <int W, int R, int NW>
struct HaloSlots {
  int pk[HaloGeo<W, R, NW>::DMA_PER_WAVE];
  uint32_t xok = 0;
};

template <int W, int R, int NW>
__device__ __forceinline__ HaloSlots<W, R, NW> halo_slots(int wave, int lane) {
  using G = HaloGeo<W, R, NW>;
  HaloSlots<W, R, NW> hs;
#pragma unroll
  for (int i = 0; i < G::DMA_PER_WAVE; ++i) {
    const int ins = wave * G::DMA_PER_WAVE + i;
    const int g = ins * 64 + lane;
    const int q = g >> 3;
    const int c = (g & 7) ^ halo_key(q);
    const int hy = q / G::HW2, hx = q - hy * G::HW2;
    const int ix = hx - 1;
    hs.pk[i] = (((hy - 1) * W + ix) * C64 + c * 8) * 8 + min(hy, 7);
    if (q < G::PIX && ins < G::DMA_INSTR && ix >= 0 && ix < W) hs.xok |= 1u << i;
  }
  return hs;
}

// Issue the LDS-DMA copies of tile `tile`'s halo into `buf` (this wave's share).
template <int W, int R, int NW>
__device__ __forceinline__ void halo_issue(const bf16* __restrict__ x, char* buf, int tile, int H,
                                           int tiles_per_img, int wave, int lane,
                                           const HaloSlots<W, R, NW>& hs) {
  using G = HaloGeo<W, R, NW>;
  const int n = tile / tiles_per_img;
  const int r0 = (tile - n * tiles_per_img) * R;
  const bf16* base = x + ((int64_t)n * H + r0) * W * C64;
  const int rlo = 1 - r0, rhi = H - r0 + 1;  // valid halo rows: rlo <= hy < rhi
#pragma unroll
  for (int i = 0; i < G::DMA_PER_WAVE; ++i) {
    const int ins = wave * G::DMA_PER_WAVE + i;
    const int hy = hs.pk[i] & 7;
    const bool ok = ((hs.xok >> i) & 1u) && hy >= rlo && hy < rhi;
    const void* src = ok ? (const void*)(base + (hs.pk[i] >> 3)) : (const void*)g_halo_zero;
    if (ins < G::DMA_INSTR)
      glds16(src, buf + ins * 1024);
  }
}

template <int W, int R, int NW, bool MOM>
__global__ __launch_bounds__(64 * NW, 1) void conv3x3_c64_kernel(
    const bf16* __restrict__ x, const bf16* __restrict__ wk, bf16* __restrict__ y, float* __restrict__ part,
    double* zsums, int H, int tiles, int tiles_per_img) {
  using G = HaloGeo<W, R, NW>;
  constexpr int NFW = G::NFW;
  // static LDS (no per-device hipFuncSetAttribute: one process may drive
  // several GPUs in DataParallel mode)
  __shared__ __attribute__((aligned(1024))) char smem[G::SMEM_BYTES];
  bf16* ostage = reinterpret_cast<bf16*>(smem + 2 * G::BUF_BYTES);  // [OUT_PIX][64]
  float* mred = reinterpret_cast<float*>(smem + 2 * G::BUF_BYTES + G::OUT_PIX * C64 * 2);  // [2][64]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int l15 = lane & 15, lh = lane >> 4;
  if constexpr (MOM) {
    zero_moments(zsums, 2 * C64);
    if (threadIdx.x < 2 * C64) mred[threadIdx.x] = 0.f;  // ordered by the first tile's barrier
  }

  // contiguous tile range of this block
  const int t_begin = (int)((int64_t)tiles * blockIdx.x / gridDim.x);
  const int t_end = (int)((int64_t)tiles * (blockIdx.x + 1) / gridDim.x);
  const HaloSlots<W, R, NW> hs = halo_slots<W, R, NW>(wave, lane);
  if (t_begin < t_end) halo_issue<W, R, NW>(x, smem, t_begin, H, tiles_per_img, wave, lane, hs);

  // weights -> B fragments: lane holds W[cout = 16 (NFW wn + nf) + l15][k = 32 s + 8 lh + j]
  bf16x8 bw[NFW][KSTEPS];
#pragma unroll
  for (int nf = 0; nf < NFW; ++nf) {
    const bf16* wrow = wk + (int64_t)(16 * (NFW * wn + nf) + l15) * (9 * C64) + 8 * lh;
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s) bw[nf][s] = *reinterpret_cast<const bf16x8*>(wrow + 32 * s);
  }
  // flat output pixel of each of this lane's A rows -> halo pixel at tap (0, 0)
  // Per fragment: the byte address of its tap-(0,0) halo pixel, and the
  // halo_key nibble table rotated to that pixel's residue with this lane's
  // chunk (lh) folded in, so a read at tap offset o costs one bit-field
  // extract (nibble o & 7) and one shift-add.  (Precomputing every (fragment,
  // k-step) offset instead -- the compiler's own choice -- holds 126 registers.)
  int qb[G::MF_WAVE];
  uint32_t kt[G::MF_WAVE];
#pragma unroll
  for (int f = 0; f < G::MF_WAVE; ++f) {
    const int p = (wm * G::MF_WAVE + f) * 16 + l15;
    const int oy = p / W, ox = p - oy * W;
    const int q = oy * G::HW2 + ox;
    qb[f] = q * 128;
    const uint32_t r = 4u * (uint32_t)(q & 7);
    const uint32_t rot = r == 0 ? kHaloKeys : (kHaloKeys >> r) | (kHaloKeys << (32u - r));
    kt[f] = rot ^ (0x11111111u * (uint32_t)lh);
  }

  // MOM: thread t always holds channels 8 (t % 8) .. +7 of the chunks it
  // copies out; its sums live across tiles and are reduced once at the end
  // (a per-tile cross-lane reduction measured +0.1 ms per launch)
  float s8[8], q8[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s8[j] = q8[j] = 0.f;
  int cur = 0;
  bool full_prev = false;  // previous tile issued exactly STORES_PER_THREAD stores
  for (int t = t_begin; t < t_end; ++t) {
    // opaque per tile: keeps the per-(fragment, tap) offsets from being
    // hoisted out of the tile loop into 126 live registers
#pragma unroll
    for (int f = 0; f < G::MF_WAVE; ++f) asm volatile("" : "+v"(kt[f]), "+v"(qb[f]));
    // this tile's halo landed.  VMEM ops retire in issue order (one VM_CNT for
    // loads, LDS-DMA and stores on CDNA), and the previous tile's stores were
    // issued after this halo's DMA: leaving them in flight overlaps their
    // write-back with this tile instead of draining it every tile
    if constexpr (G::STORES_EXACT) {
      if (full_prev) vmcnt<G::STORES_PER_THREAD>();
      else vmcnt<0>();
    } else {
      vmcnt<0>();
    }
    raw_barrier();     // ... for every wave; the other buffer is free again
    if (t + 1 < t_end) halo_issue<W, R, NW>(x, smem + (cur ^ 1) * G::BUF_BYTES, t + 1, H, tiles_per_img, wave, lane, hs);
    const char* hb = smem + cur * G::BUF_BYTES;

    f32x4 acc[G::MF_WAVE][NFW];
#pragma unroll
    for (int f = 0; f < G::MF_WAVE; ++f)
#pragma unroll
      for (int nf = 0; nf < NFW; ++nf) acc[f][nf] = f32x4{0.f, 0.f, 0.f, 0.f};

    // software pipeline over the 18 k-steps: step s+1's 7 fragment reads are
    // issued before step s's 14 MFMAs, so their LDS latency hides behind them
    // (one wave per SIMD: nothing else would).  The sched barrier keeps the
    // compiler from hoisting further (a third fragment set would spill).
    bf16x8 a[2][G::MF_WAVE];
    auto load_step = [&](int s, bf16x8 (&dst)[G::MF_WAVE]) {
      const int tap = s >> 1, kh = tap / 3, kw = tap - 3 * (tap / 3);
      const int o = kh * G::HW2 + kw;   // tap offset in halo pixels
#pragma unroll
      for (int f = 0; f < G::MF_WAVE; ++f) {
        // chunk = ((s & 1) * 4 + lh) ^ halo_key(q0 + o)
        const uint32_t ch = ((kt[f] >> (4 * (o & 7))) & 7u) ^ (uint32_t)((s & 1) * 4);
        dst[f] = *reinterpret_cast<const bf16x8*>(hb + qb[f] + o * 128 + (ch << 4));
      }
    };
    load_step(0, a[0]);
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s) {
      if (s + 1 < KSTEPS) load_step(s + 1, a[(s + 1) & 1]);
#pragma unroll
      for (int f = 0; f < G::MF_WAVE; ++f)
#pragma unroll
        for (int nf = 0; nf < NFW; ++nf)
          acc[f][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[nf][s], a[s & 1][f], acc[f][nf], 0, 0, 0);  // C^T
      // interleave: the next step's 7 ds_reads go one per MFMA over the first
      // half of this step, leaving 7 MFMAs (~112 cycles) for the last to land
      if (s + 1 < KSTEPS) {
#pragma unroll
        for (int f = 0; f < G::MF_WAVE; ++f) {
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
        }
        if constexpr (NFW > 1) __builtin_amdgcn_sched_group_barrier(0x008, G::MF_WAVE * (NFW - 1), 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }

    // epilogue (transposed accumulators): pixel (fragment row) = l15, channels
    // 16 (NFW wn + nf) + 4 lh + i -> one 8-B LDS write per fragment
#pragma unroll
    for (int f = 0; f < G::MF_WAVE; ++f)
#pragma unroll
      for (int nf = 0; nf < NFW; ++nf) {
        const int p = (wm * G::MF_WAVE + f) * 16 + l15;
        const int ch = (2 * (NFW * wn + nf) + (lh >> 1)) ^ stage_key(p);
        *reinterpret_cast<bf16x4*>(ostage + p * C64 + ch * 8 + (lh & 1) * 4) =
            __builtin_convertvector(acc[f][nf], bf16x4);
      }
    __syncthreads();
    // the tile = R whole output rows of one image = one contiguous run of y
    {
      const int n = t / tiles_per_img;
      const int r0 = (t - n * tiles_per_img) * R;
      const int rows = min(R, H - r0);
      const int chunks = rows * W * (C64 / 8);
      full_prev = chunks == G::STORES_PER_THREAD * G::NT;
      bf16* dst = y + (((int64_t)n * H + r0) * W) * C64;
      for (int i = threadIdx.x; i < chunks; i += G::NT) {
        const int sp = i >> 3;
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(ostage + sp * C64 + (((i & 7) ^ stage_key(sp)) << 3));
        *reinterpret_cast<bf16x8*>(dst + i * 8) = v;
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
    // the next iteration's barrier orders these LDS reads before the next tile's
    // stage writes (which come after its MFMA loop)
  }

  if constexpr (MOM) {
    // rows beyond H (a partial last tile) are never copied out, so they add
    // nothing to either moment
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
        atomicAdd(&mred[8 * lane + j], s8[j]);  // LDS atomics, 4 waves per address
        atomicAdd(&mred[C64 + 8 * lane + j], q8[j]);
      }
    __syncthreads();
    if (threadIdx.x < 2 * C64) {
      const int mo = threadIdx.x / C64, ch = threadIdx.x % C64;
      part[((int64_t)mo * gridDim.x + blockIdx.x) * C64 + ch] = mred[mo * C64 + ch];
    }
  }
}

template <int W, int R, int NW, bool MOM>
void launch_nw(const at::Tensor& x, const at::Tensor& wk, at::Tensor& y, float* part, double* zs, int H,
               int tiles, int tpi, int grid, hipStream_t stream) {
  using G = HaloGeo<W, R, NW>;
  static_assert(G::SMEM_BYTES <= 160 * 1024, "LDS budget");
  auto kern = conv3x3_c64_kernel<W, R, NW, MOM>;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(G::NT), 0, stream,
                     reinterpret_cast<const bf16*>(x.data_ptr()), reinterpret_cast<const bf16*>(wk.data_ptr()),
                     reinterpret_cast<bf16*>(y.data_ptr()), part, zs, H, tiles, tpi);
}

// 4 waves (1 per SIMD, 32 output channels and 144 weight VGPRs each); the
// 8-wave form (16 channels, 72 VGPRs) measured slower (profiles/README.md).
template <int W, int R, bool MOM>
void launch(const at::Tensor& x, const at::Tensor& wk, at::Tensor& y, float* part, double* zs, int H,
            int tiles, int tpi, int grid, hipStream_t stream) {
  launch_nw<W, R, 4, MOM>(x, wk, y, part, zs, H, tiles, tpi, grid, stream);
}

}  // namespace

// y = conv3x3(x, W), stride 1, pad 1, x: [N, 64, H, 56] bf16 channels_last,
// wmat: [64 cout][3][3][64 cin] flattened to [64, 576] bf16.  Returns
// (y as [N*H*W, 64], moments fp64 [129] or empty).
std::vector<at::Tensor> conv3x3_c64(const at::Tensor& x, const at::Tensor& wmat, bool moments) {
  constexpr int W = 56, R = 4;
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4, "conv3x3_c64: bf16 NCHW-shaped x");
  TORCH_CHECK(x.size(1) == C64 && x.size(3) == W && x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv3x3_c64: x must be [N, 64, H, 56] channels_last");
  TORCH_CHECK(wmat.scalar_type() == at::kBFloat16 && wmat.is_contiguous() && wmat.size(0) == C64 &&
                  wmat.size(1) == 9 * C64, "conv3x3_c64: wmat must be contiguous [64, 576] bf16");
  const int64_t n = x.size(0), H = x.size(2);
  const int tpi = (int)((H + R - 1) / R);
  const int64_t tiles64 = n * tpi;
  TORCH_CHECK(tiles64 < (1 << 30), "conv3x3_c64: too many tiles");
  const int tiles = (int)tiles64;
  auto y = at::empty({n * H * W, C64}, x.options());
  auto stream = at::hip::getCurrentHIPStream();
  at::Tensor mom;
  if (tiles == 0) return {y, at::zeros({moments ? 2 * C64 + 1 : 0}, x.options().dtype(at::kDouble))};
  int dev = 0, cus = 256;
  DMP_HIP_CHECK(hipGetDevice(&dev));
  DMP_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int grid = std::min(tiles, cus);
  if (moments) {
    mom = at::empty({2 * C64 + 1}, x.options().dtype(at::kDouble));
    auto part = at::empty({2, grid, C64}, x.options().dtype(at::kFloat));
    launch<W, R, true>(x, wmat, y, part.data_ptr<float>(), moments_zero_target(mom.data_ptr<double>(), grid),
                       (int)H, tiles, tpi, grid, stream);
    bn_reduce_partials_launch(part.data_ptr<float>(), grid, C64, mom.data_ptr<double>(),
                              (double)(n * H * W), stream);
  } else {
    mom = at::empty({0}, x.options().dtype(at::kDouble));
    launch<W, R, false>(x, wmat, y, nullptr, nullptr, (int)H, tiles, tpi, grid, stream);
  }
  DMP_HIP_CHECK(hipGetLastError());
  return {y, mom};
}

}  // namespace dmp
