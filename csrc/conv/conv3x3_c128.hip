// 3x3 / stride-1 / pad-1 convolution for 128 -> 128 channels on 28-wide maps
// (ResNet-50 layer 2: forward, and the data gradient as the same conv over
// flipped weights) as a persistent, halo-tiled MFMA kernel -- the C = 128
// sibling of conv3x3_halo.hip, which it follows except where noted.
//
// The weights of a 64 x 64 conv fit a 4-wave block's VGPRs (each wave 32 Cout
// x 576 K = 144 VGPRs); a 128 -> 128 conv has 4x the weights.  So:
//   * the grid is split in two halves, one per 64-channel Cout chunk: block
//     b < G/2 holds Cout 0..63, block b + G/2 Cout 64..127, and both walk the
//     same tile range at the same time on the same XCD (b and b + G/2 are
//     congruent mod 8), so each input halo is read from HBM once and from L2
//     once more;
//   * the K = 9 x 128 reduction is split between the wave pairs instead of
//     the output pixels: wave (wk, wn) holds W[32 wn .. +32][9 taps][64 wk ..
//     +64] (144 VGPRs) and multiplies all 112 pixels of the tile (7 row
//     fragments x 2 column fragments, 0.5 KB of LDS reads per MFMA -- the c64
//     kernel's ratio); the two K halves meet in LDS at the end of the tile
//     (each wave sends the fragments its partner finalises: 4 / 3 of 7);
//   * a halo pixel is 256 B = one whole LDS bank row, so the chunk swizzle is
//     2 (q & 7): a ds_read_b128 16-lane service group holds the lanes of one
//     lh parity at 8 consecutive pixels and of the other at the 8 after, and
//     the even / odd keys of those two sets can never collide (exhaustive
//     check over all 16 tap residues; the c64 table does not apply at this
//     stride).
// Tile = R = 4 full output rows of one image (112 px; 28 / 4 tiles per
// image), so its output chunk is one contiguous run of rows.  MOM: per-block
// (sum, sum^2) partials of the bf16 outputs, as conv3x3_halo.hip.
// Reference: these replace MIOpen's 3x3s of torchvision ResNet-50 layer 2
// (reference model_parallel.py:61, data_parallel.py:78).
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include "../common.h"

namespace dmp {

void bn_reduce_partials_launch(const float* part, int rb, int C, double* sums, double count,
                               hipStream_t stream);

namespace {

using bf16 = __bf16;
using lptr_t = __attribute__((address_space(3))) void*;

constexpr int CI = 128, CO = 128, CB = 64;   // channels in, out, out per block
constexpr int W = 28, R = 4;
constexpr int NT = 256;                      // 4 waves: wk = wave & 1, wn = wave >> 1
constexpr int HW2 = W + 2, PIX = (R + 2) * HW2;
constexpr int DMA_INSTR = PIX * (CI / 8) / 64;      // 1 KB wave instructions per halo (45)
constexpr int DMA_PER_WAVE = (DMA_INSTR + 3) / 4;   // 12
constexpr int BUF = DMA_PER_WAVE * 4 * 1024;
constexpr int OUT_PIX = R * W;                      // 112
constexpr int MF = OUT_PIX / 16;                    // 7 row fragments
constexpr int MF_LO = 4;                            // fragments finalised by wk = 0
constexpr int KSTEPS = 9 * 64 / 32;                 // k32 steps per K half
constexpr int SCR_OFF = 2 * BUF;                    // K-half exchange [2 wn][7 f][2 nf][64 lanes] x f32x4
constexpr int STAGE_OFF = SCR_OFF + 2 * MF * 2 * 1024;
constexpr int MRED_OFF = STAGE_OFF + OUT_PIX * CB * 2;
constexpr int SMEM = MRED_OFF + 2 * CB * 4;
static_assert(PIX * (CI / 8) % 64 == 0, "halo is a whole number of 1 KB DMA rounds");
static_assert(SMEM <= 160 * 1024, "LDS budget");

__device__ __attribute__((aligned(16))) uint32_t g_c128_zero[4];

__device__ __forceinline__ int hkey(int q) { return (q & 7) << 1; }
// output stage [pixel][64 ch] chunk swizzle (as conv3x3_halo.hip)
__device__ __forceinline__ int stage_key(int p) { return ((p >> 2) & 3) << 1; }

// LDS-DMA through inline asm (see wgrad3x3.hip: the builtin makes hipcc drain
// every pending copy at the next LDS access)
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

// Per DMA slot of this lane: (element offset from the tile's first output row
// of the logical 16-B chunk it carries) << 3 | halo row, and a bitmask of the
// slots whose column lies inside the image.
struct Slots {
  int pk[DMA_PER_WAVE];
  uint32_t xok = 0;
};

__device__ __forceinline__ Slots make_slots(int wave, int lane) {
  Slots s;
#pragma unroll
  for (int i = 0; i < DMA_PER_WAVE; ++i) {
    const int ins = wave * DMA_PER_WAVE + i;
    const int g = ins * 64 + lane;
    const int q = g >> 4;
    const int c = (g & 15) ^ hkey(q);
    const int hy = q / HW2, hx = q - hy * HW2, ix = hx - 1;
    s.pk[i] = (((hy - 1) * W + ix) * CI + c * 8) * 8 + min(hy, 7);
    if (q < PIX && ins < DMA_INSTR && ix >= 0 && ix < W) s.xok |= 1u << i;
  }
  return s;
}

__device__ __forceinline__ void halo_issue(const bf16* __restrict__ x, char* buf, int tile, int H, int tpi,
                                           int wave, const Slots& s) {
  const int n = tile / tpi;
  const int r0 = (tile - n * tpi) * R;
  const bf16* base = x + ((int64_t)n * H + r0) * W * CI;
  const int rlo = 1 - r0, rhi = H - r0 + 1;
#pragma unroll
  for (int i = 0; i < DMA_PER_WAVE; ++i) {
    const int ins = wave * DMA_PER_WAVE + i;
    const int hy = s.pk[i] & 7;
    const bool ok = ((s.xok >> i) & 1u) && hy >= rlo && hy < rhi;
    const void* src = ok ? (const void*)(base + (s.pk[i] >> 3)) : (const void*)g_c128_zero;
    if (ins < DMA_INSTR) glds16(src, buf + ins * 1024);
  }
}

template <bool MOM>
__global__ __launch_bounds__(NT, 1) void conv3x3_c128_kernel(
    const bf16* __restrict__ x, const bf16* __restrict__ wk, bf16* __restrict__ y, float* __restrict__ part,
    double* zsums, int H, int tiles) {
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];
  f32x4* scr = reinterpret_cast<f32x4*>(smem + SCR_OFF);
  bf16* ostage = reinterpret_cast<bf16*>(smem + STAGE_OFF);
  float* mred = reinterpret_cast<float*>(smem + MRED_OFF);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wkh = wave & 1, wn = wave >> 1;
  const int l15 = lane & 15, lh = lane >> 4;
  const int half = (int)gridDim.x >> 1;
  const int cb = (int)blockIdx.x >= half ? 1 : 0;      // Cout chunk
  const int rb = (int)blockIdx.x - cb * half;          // block within the chunk's half-grid
  const int tpi = H / R;
  if constexpr (MOM) {
    zero_moments(zsums, 2 * CO);
    if (threadIdx.x < 2 * CB) mred[threadIdx.x] = 0.f;
  }
  const int t_begin = (int)((int64_t)tiles * rb / half);
  const int t_end = (int)((int64_t)tiles * (rb + 1) / half);
  const Slots sl = make_slots(wave, lane);
  if (t_begin < t_end) halo_issue(x, smem, t_begin, H, tpi, wave, sl);

  // B fragments: lane holds W[cout = 64 cb + 32 wn + 16 nf + l15][tap][cin = 64 wkh + 32 (s & 1) + 8 lh + j]
  bf16x8 bw[2][KSTEPS];
#pragma unroll
  for (int nf = 0; nf < 2; ++nf) {
    const bf16* wrow = wk + (int64_t)(CB * cb + 32 * wn + 16 * nf + l15) * (9 * CI) + 64 * wkh + 8 * lh;
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s)
      bw[nf][s] = *reinterpret_cast<const bf16x8*>(wrow + (s >> 1) * CI + 32 * (s & 1));
  }
  // per fragment: byte offset of its tap-(0,0) halo pixel, and the 8 keys of
  // pixels q .. q+7 as a nibble table (read at tap offset o: nibble o & 7)
  int qb[MF];
  uint32_t kt[MF];
  const int lchunk = 8 * wkh + lh;  // logical 16-B chunk of k-step 0 (cin 64 wkh + 8 lh ..)
#pragma unroll
  for (int f = 0; f < MF; ++f) {
    const int p = f * 16 + l15;
    const int oy = p / W, ox = p - oy * W;
    const int q = oy * HW2 + ox;
    qb[f] = q * (CI * 2);
    uint32_t t = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) t |= (uint32_t)hkey(q + i) << (4 * i);
    kt[f] = t;
  }

  float s8[8], q8[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s8[j] = q8[j] = 0.f;
  int cur = 0;
  bool stored_prev = false;
  for (int t = t_begin; t < t_end; ++t) {
#pragma unroll
    for (int f = 0; f < MF; ++f) asm volatile("" : "+v"(kt[f]), "+v"(qb[f]));
    // this tile's halo landed: the previous tile's >= 3 stores per thread were
    // issued after it, so they may stay in flight
    if (stored_prev) vmcnt<3>();
    else vmcnt<0>();
    raw_barrier();
    if (t + 1 < t_end) halo_issue(x, smem + (cur ^ 1) * BUF, t + 1, H, tpi, wave, sl);
    const char* hb = smem + cur * BUF;

    f32x4 acc[MF][2];
#pragma unroll
    for (int f = 0; f < MF; ++f) acc[f][0] = acc[f][1] = f32x4{0.f, 0.f, 0.f, 0.f};

    bf16x8 a[2][MF];
    auto load_step = [&](int s, bf16x8 (&dst)[MF]) {
      const int tap = s >> 1, kh = tap / 3, kw = tap - 3 * (tap / 3);
      const int o = kh * HW2 + kw;
#pragma unroll
      for (int f = 0; f < MF; ++f) {
        // logical chunk 8 wkh + 4 (s & 1) + lh (folded into qb), XOR the pixel key
        const int key = (int)((kt[f] >> (4 * (o & 7))) & 15u);
        const int ch = (lchunk + 4 * (s & 1)) ^ key;
        dst[f] = *reinterpret_cast<const bf16x8*>(hb + qb[f] + o * (CI * 2) + (ch << 4));
      }
    };
    load_step(0, a[0]);
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s) {
      if (s + 1 < KSTEPS) load_step(s + 1, a[(s + 1) & 1]);
#pragma unroll
      for (int f = 0; f < MF; ++f)
#pragma unroll
        for (int nf = 0; nf < 2; ++nf)
          acc[f][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[s & 1][f], bw[nf][s], acc[f][nf], 0, 0, 0);
      if (s + 1 < KSTEPS) {
#pragma unroll
        for (int f = 0; f < MF; ++f) {
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
        }
        __builtin_amdgcn_sched_group_barrier(0x008, MF, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }

    // K-half exchange: wk = 0 finalises fragments 0..3, wk = 1 fragments 4..6
#pragma unroll
    for (int f = 0; f < MF; ++f) {
      const bool mine = (f < MF_LO) == (wkh == 0);
      if (!mine)
#pragma unroll
        for (int nf = 0; nf < 2; ++nf) scr[((wn * MF + f) * 2 + nf) * 64 + lane] = acc[f][nf];
    }
    __syncthreads();
#pragma unroll
    for (int f = 0; f < MF; ++f) {
      const bool mine = (f < MF_LO) == (wkh == 0);
      if (mine)
#pragma unroll
        for (int nf = 0; nf < 2; ++nf) {
          const f32x4 o = scr[((wn * MF + f) * 2 + nf) * 64 + lane];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int p = f * 16 + 4 * lh + i;
            const int ch = (4 * wn + 2 * nf + (l15 >> 3)) ^ stage_key(p);
            ostage[p * CB + ch * 8 + (l15 & 7)] = (bf16)(acc[f][nf][i] + o[i]);
          }
        }
    }
    __syncthreads();
    {
      const int n = t / tpi;
      const int r0 = (t - n * tpi) * R;
      bf16* dst = y + (((int64_t)n * H + r0) * W) * CO + CB * cb;
      for (int i = threadIdx.x; i < OUT_PIX * 8; i += NT) {
        const int sp = i >> 3;
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(ostage + sp * CB + (((i & 7) ^ stage_key(sp)) << 3));
        *reinterpret_cast<bf16x8*>(dst + (int64_t)sp * CO + (i & 7) * 8) = v;
        if constexpr (MOM)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float fv = (float)v[j];
            s8[j] += fv;
            q8[j] = fmaf(fv, fv, q8[j]);
          }
      }
    }
    stored_prev = true;
    cur ^= 1;
  }

  if constexpr (MOM) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int off = 8; off < 64; off <<= 1) {
        s8[j] += __shfl_xor(s8[j], off, 64);
        q8[j] += __shfl_xor(q8[j], off, 64);
      }
    if (lane < 8)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        atomicAdd(&mred[8 * lane + j], s8[j]);
        atomicAdd(&mred[CB + 8 * lane + j], q8[j]);
      }
    __syncthreads();
    if (threadIdx.x < 2 * CB) {
      const int mo = threadIdx.x / CB, ch = threadIdx.x % CB;
      part[((int64_t)mo * half + rb) * CO + CB * cb + ch] = mred[mo * CB + ch];
    }
  }
}

}  // namespace

bool conv3x3_c128_supported(int64_t c, int64_t h, int64_t w) {
  return c == CI && w == W && h > 0 && h % R == 0;
}

// y = conv3x3(x, W), stride 1, pad 1; x: [N, 128, H, 28] bf16 channels_last
// (H % 4 == 0), wmat: [128 cout][3][3][128 cin] flattened to [128, 1152].
// Returns (y as [N*H*W, 128], moments fp64 [257] or empty).
std::vector<at::Tensor> conv3x3_c128(const at::Tensor& x, const at::Tensor& wmat, bool moments) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4, "conv3x3_c128: bf16 NCHW-shaped x");
  TORCH_CHECK(conv3x3_c128_supported(x.size(1), x.size(2), x.size(3)) &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv3x3_c128: x must be [N, 128, H % 4 == 0, 28] channels_last");
  TORCH_CHECK(wmat.scalar_type() == at::kBFloat16 && wmat.is_contiguous() && wmat.size(0) == CO &&
                  wmat.size(1) == 9 * CI, "conv3x3_c128: wmat must be contiguous [128, 1152] bf16");
  const int64_t n = x.size(0), H = x.size(2);
  const int64_t tiles64 = n * (H / R);
  TORCH_CHECK(tiles64 < (1 << 30), "conv3x3_c128: too many tiles");
  const int tiles = (int)tiles64;
  auto y = at::empty({n * H * W, CO}, x.options());
  if (tiles == 0) return {y, at::zeros({moments ? 2 * CO + 1 : 0}, x.options().dtype(at::kDouble))};
  auto stream = at::hip::getCurrentHIPStream();
  int dev = 0, cus = 256;
  DMP_HIP_CHECK(hipGetDevice(&dev));
  DMP_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int half = std::max(1, std::min(tiles, cus / 2));
  const int grid = 2 * half;
  at::Tensor mom;
  if (moments) {
    mom = at::empty({2 * CO + 1}, x.options().dtype(at::kDouble));
    auto part = at::empty({2, half, CO}, x.options().dtype(at::kFloat));
    hipLaunchKernelGGL(conv3x3_c128_kernel<true>, dim3(grid), dim3(NT), 0, stream,
                       reinterpret_cast<const bf16*>(x.data_ptr()), reinterpret_cast<const bf16*>(wmat.data_ptr()),
                       reinterpret_cast<bf16*>(y.data_ptr()), part.data_ptr<float>(),
                       moments_zero_target(mom.data_ptr<double>(), half), (int)H, tiles);
    bn_reduce_partials_launch(part.data_ptr<float>(), half, CO, mom.data_ptr<double>(), (double)(n * H * W),
                              stream);
  } else {
    mom = at::empty({0}, x.options().dtype(at::kDouble));
    hipLaunchKernelGGL(conv3x3_c128_kernel<false>, dim3(grid), dim3(NT), 0, stream,
                       reinterpret_cast<const bf16*>(x.data_ptr()), reinterpret_cast<const bf16*>(wmat.data_ptr()),
                       reinterpret_cast<bf16*>(y.data_ptr()), nullptr, nullptr, (int)H, tiles);
  }
  DMP_HIP_CHECK(hipGetLastError());
  return {y, mom};
}

}  // namespace dmp
