// 3x3 convolutions with 128 -> 128 channels of ResNet-50 layer 2 as a
// persistent, halo-tiled MFMA kernel -- the C = 128 sibling of
// conv3x3_halo.hip, which it follows except where noted:
//   * stride 1 / pad 1 on 28-wide maps: the forward (+ BN moments) and the
//     data gradient (the same conv over flipped weights);
//   * the data gradient of the stride-2 block-0 conv (dy 28x28 -> dx 56x56)
//     as its four stride phases (PH): dx[2m + py, 2q + px] collects the taps
//     (ky, kx) of phase (py, px) -- 1, 2, 2 or 4 of the 9 -- from dy[m + a(ky),
//     q + a(kx)] (a(1) = 0 for the even phase, a(2) = 0 and a(0) = 1 for the
//     odd one).  One dy halo tile of 4 rows serves all four phases; each phase
//     is its own MFMA sweep and epilogue, written straight into its pixels of
//     dx: no zero-filled dx, no zero taps (MIOpen zero-fills dx, then runs
//     igemm_bwd).
//
// The weights of a 64 x 64 conv fit a 4-wave block's VGPRs (each wave 32 Cout
// x 576 K = 144 VGPRs); a 128 -> 128 conv has 4x the weights.  So:
//   * the grid is split in two halves, one per 64-channel output chunk: block
//     b < G/2 holds outputs 0..63, block b + G/2 outputs 64..127, and both walk
//     the same tile range at the same time on the same XCD (b and b + G/2 are
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
//     check over all 16 tap residues in tests/test_halo_layout.py; the c64
//     table does not apply at this stride).
// Tile = R = 4 full rows of one image (112 px; 28 / 4 tiles per image).
// MOM: per-block (sum, sum^2) partials of the bf16 outputs, as conv3x3_halo.hip.
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
constexpr int OUT_PIX = R * W;               // 112 pixels per tile (per phase)
constexpr int MF = OUT_PIX / 16;             // 7 row fragments
constexpr int MF_LO = 4;                     // fragments finalised by wk = 0
constexpr int KSTEPS = 9 * 64 / 32;          // k32 steps per K half (all 9 taps)

// PH = false: stride-1 conv, halo (R+2) x (W+2) starting one row / column
// before the tile; PH = true: stride-2 data gradient, dy halo (R+1) x (W+1)
// starting at the tile (the odd phases reach one row / column past it).
template <bool PH>
struct Geo {
  static constexpr int HR = PH ? R + 1 : R + 2, HC = PH ? W + 1 : W + 2;
  static constexpr int OFF = PH ? 0 : 1;  // halo (0, 0) = input (r0 - OFF, -OFF)
  static constexpr int PIX = HR * HC;
  static constexpr int DMA_INSTR = (PIX * (CI / 8) + 63) / 64;   // 1 KB wave instructions per halo
  static constexpr int DMA_PER_WAVE = (DMA_INSTR + 3) / 4;
  static constexpr int BUF = DMA_PER_WAVE * 4 * 1024;
  static constexpr int SCR_OFF = 2 * BUF;          // K-half exchange [2 wn][7 f][2 nf][64 lanes] x f32x4
  static constexpr int STAGE_OFF = SCR_OFF + 2 * MF * 2 * 1024;
  static constexpr int MRED_OFF = STAGE_OFF + OUT_PIX * CB * 2;
  static constexpr int SMEM = MRED_OFF + 2 * CB * 4;
  // stores per thread per tile: >= 3 per epilogue (896 16-B chunks / 256 threads)
  static constexpr int MIN_STORES = PH ? 12 : 3;
  static_assert(SMEM <= 160 * 1024, "LDS budget");
};

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

// Per DMA slot of this lane: (element offset from the tile's first input row
// of the logical 16-B chunk it carries) << 3 | halo row, and a bitmask of the
// slots whose column lies inside the image.
template <bool PH>
struct Slots {
  int pk[Geo<PH>::DMA_PER_WAVE];
  uint32_t xok = 0;
};

template <bool PH>
__device__ __forceinline__ Slots<PH> make_slots(int wave, int lane) {
  using G = Geo<PH>;
  Slots<PH> s;
#pragma unroll
  for (int i = 0; i < G::DMA_PER_WAVE; ++i) {
    const int ins = wave * G::DMA_PER_WAVE + i;
    const int g = ins * 64 + lane;
    const int q = g >> 4;
    const int c = (g & 15) ^ hkey(q);
    const int hy = q / G::HC, hx = q - hy * G::HC, ix = hx - G::OFF;
    s.pk[i] = (((hy - G::OFF) * W + ix) * CI + c * 8) * 8 + min(hy, 7);
    if (q < G::PIX && ins < G::DMA_INSTR && ix >= 0 && ix < W) s.xok |= 1u << i;
  }
  return s;
}

// H: input height (x for the stride-1 conv, dy for PH); tiles of R input rows.
template <bool PH>
__device__ __forceinline__ void halo_issue(const bf16* __restrict__ x, char* buf, int tile, int H, int tpi,
                                           int wave, const Slots<PH>& s) {
  using G = Geo<PH>;
  const int n = tile / tpi;
  const int r0 = (tile - n * tpi) * R;
  const bf16* base = x + ((int64_t)n * H + r0) * W * CI;
  const int rlo = G::OFF - r0, rhi = H - r0 + G::OFF;  // valid halo rows: rlo <= hy < rhi
#pragma unroll
  for (int i = 0; i < G::DMA_PER_WAVE; ++i) {
    const int ins = wave * G::DMA_PER_WAVE + i;
    const int hy = s.pk[i] & 7;
    const bool ok = ((s.xok >> i) & 1u) && hy >= rlo && hy < rhi;
    const void* src = ok ? (const void*)(base + (s.pk[i] >> 3)) : (const void*)g_c128_zero;
    if (ins < G::DMA_INSTR) glds16(src, buf + ins * 1024);
  }
}

// stride-phase tap tables: phase parity p, tap i -> kernel index / dy offset
__host__ __device__ constexpr int ph_k(int p, int i) { return p == 0 ? 1 : (i == 0 ? 2 : 0); }
__host__ __device__ constexpr int ph_a(int p, int i) { return p == 0 ? 0 : i; }

// One MFMA sweep over the k-steps of a phase (PH) or of the whole 3x3 (PY =
// PX = -1): step s -> tap (ky, kx), halo offset o, weight fragment index.
template <bool PH, int PY, int PX>
__device__ __forceinline__ void sweep(f32x4 (&acc)[MF][2], const bf16x8 (&bw)[2][KSTEPS], const char* hb,
                                      const int (&qb)[MF], const uint32_t (&kt)[MF], int lchunk) {
  using G = Geo<PH>;
  constexpr int NTY = PH ? (PY ? 2 : 1) : 3, NTX = PH ? (PX ? 2 : 1) : 3;
  constexpr int KS = 2 * NTY * NTX;
  bf16x8 a[2][MF];
  auto load_step = [&](int s, bf16x8 (&dst)[MF]) __attribute__((always_inline)) {
    const int t = s >> 1, ty = t / NTX, tx = t - ty * NTX;
    const int oy = PH ? ph_a(PY, ty) : ty, ox = PH ? ph_a(PX, tx) : tx;
    const int o = oy * G::HC + ox;
#pragma unroll
    for (int f = 0; f < MF; ++f) {
      const int key = (int)((kt[f] >> (4 * (o & 7))) & 15u);
      const int ch = (lchunk + 4 * (s & 1)) ^ key;
      dst[f] = *reinterpret_cast<const bf16x8*>(hb + qb[f] + o * (CI * 2) + (ch << 4));
    }
  };
  load_step(0, a[0]);
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    if (s + 1 < KS) load_step(s + 1, a[(s + 1) & 1]);
    const int t = s >> 1, ty = t / NTX, tx = t - ty * NTX;
    const int ky = PH ? ph_k(PY, ty) : ty, kx = PH ? ph_k(PX, tx) : tx;
    const int ws = (ky * 3 + kx) * 2 + (s & 1);
#pragma unroll
    for (int f = 0; f < MF; ++f)
#pragma unroll
      for (int nf = 0; nf < 2; ++nf)
        acc[f][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[s & 1][f], bw[nf][ws], acc[f][nf], 0, 0, 0);
    if (s + 1 < KS) {
#pragma unroll
      for (int f = 0; f < MF; ++f) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
      }
      __builtin_amdgcn_sched_group_barrier(0x008, MF, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// K-half exchange through LDS, bf16 rounding into the output stage; returns
// after the barrier that publishes the stage.
template <int F0, int F1>
__device__ __forceinline__ void send_frags(const f32x4 (&acc)[MF][2], f32x4* scr, int wn, int lane) {
#pragma unroll
  for (int f = F0; f < F1; ++f)
#pragma unroll
    for (int nf = 0; nf < 2; ++nf) scr[((wn * MF + f) * 2 + nf) * 64 + lane] = acc[f][nf];
}

template <int F0, int F1>
__device__ __forceinline__ void finish_frags(const f32x4 (&acc)[MF][2], const f32x4* scr, bf16* ostage, int wn,
                                             int lane, int l15, int lh) {
#pragma unroll
  for (int f = F0; f < F1; ++f)
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

// K-half exchange through LDS (wk = 0 finalises fragments 0..3, wk = 1
// fragments 4..6; the split is a wave-uniform branch over two statically
// indexed loops -- a runtime-selected fragment index would put acc in
// scratch), bf16 rounding into the output stage; returns after the barrier
// that publishes the stage.
__device__ __forceinline__ void exchange_to_stage(const f32x4 (&acc)[MF][2], f32x4* scr, bf16* ostage, int wkh,
                                                  int wn, int lane, int l15, int lh) {
  if (wkh == 0) send_frags<MF_LO, MF>(acc, scr, wn, lane);
  else send_frags<0, MF_LO>(acc, scr, wn, lane);
  __syncthreads();
  if (wkh == 0) finish_frags<0, MF_LO>(acc, scr, ostage, wn, lane, l15, lh);
  else finish_frags<MF_LO, MF>(acc, scr, ostage, wn, lane, l15, lh);
  __syncthreads();
}

// PH: x = dy [N, 28 (H), 28, 128], y = dx [N, 2H, 56, 128]; wk = W^T
// [dx ch][ky][kx][dy ch] (unflipped).  Otherwise x [N, H, 28, 128] -> y same.
template <bool MOM, bool PH>
__global__ __launch_bounds__(NT, 1) void conv3x3_c128_kernel(
    const bf16* __restrict__ x, const bf16* __restrict__ wk, bf16* __restrict__ y, float* __restrict__ part,
    double* zsums, int H, int tiles) {
  using G = Geo<PH>;
  __shared__ __attribute__((aligned(1024))) char smem[G::SMEM];
  f32x4* scr = reinterpret_cast<f32x4*>(smem + G::SCR_OFF);
  bf16* ostage = reinterpret_cast<bf16*>(smem + G::STAGE_OFF);
  float* mred = reinterpret_cast<float*>(smem + G::MRED_OFF);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wkh = wave & 1, wn = wave >> 1;
  const int l15 = lane & 15, lh = lane >> 4;
  const int half = (int)gridDim.x >> 1;
  const int cb = (int)blockIdx.x >= half ? 1 : 0;      // output-channel chunk
  const int rb = (int)blockIdx.x - cb * half;          // block within the chunk's half-grid
  const int tpi = H / R;
  if constexpr (MOM) {
    zero_moments(zsums, 2 * CO);
    if (threadIdx.x < 2 * CB) mred[threadIdx.x] = 0.f;
  }
  const int t_begin = (int)((int64_t)tiles * rb / half);
  const int t_end = (int)((int64_t)tiles * (rb + 1) / half);
  const Slots<PH> sl = make_slots<PH>(wave, lane);
  if (t_begin < t_end) halo_issue<PH>(x, smem, t_begin, H, tpi, wave, sl);

  // B fragments: lane holds W[out = 64 cb + 32 wn + 16 nf + l15][tap][in = 64 wkh + 32 (s & 1) + 8 lh + j]
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
  const int lchunk = 8 * wkh + lh;  // logical 16-B chunk of k-step 0 (channels 64 wk + 8 lh ..)
#pragma unroll
  for (int f = 0; f < MF; ++f) {
    const int p = f * 16 + l15;
    const int oy = p / W, ox = p - oy * W;
    const int q = oy * G::HC + ox;
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
    // this tile's halo landed: the previous tile's >= MIN_STORES stores per
    // thread were issued after it, so they may stay in flight
    if (stored_prev) vmcnt<G::MIN_STORES>();
    else vmcnt<0>();
    raw_barrier();
    if (t + 1 < t_end) halo_issue<PH>(x, smem + (cur ^ 1) * G::BUF, t + 1, H, tpi, wave, sl);
    const char* hb = smem + cur * G::BUF;
    const int n = t / tpi;
    const int r0 = (t - n * tpi) * R;

    // one epilogue: stage -> 16-B stores of this block's 64 channels per pixel
    auto store_stage = [&](int py, int px) __attribute__((always_inline)) {
      for (int i = threadIdx.x; i < OUT_PIX * 8; i += NT) {
        const int sp = i >> 3;
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(ostage + sp * CB + (((i & 7) ^ stage_key(sp)) << 3));
        int64_t pix;
        if constexpr (PH) {
          const int m = sp / W, q = sp - m * W;
          pix = ((int64_t)n * (2 * H) + 2 * (r0 + m) + py) * (2 * W) + 2 * q + px;
        } else {
          pix = ((int64_t)n * H + r0) * W + sp;
        }
        *reinterpret_cast<bf16x8*>(y + pix * CO + CB * cb + (i & 7) * 8) = v;
        if constexpr (MOM)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float fv = (float)v[j];
            s8[j] += fv;
            q8[j] = fmaf(fv, fv, q8[j]);
          }
      }
    };
    auto phase = [&](auto pyc, auto pxc) __attribute__((always_inline)) {
      constexpr int PY = decltype(pyc)::value, PX = decltype(pxc)::value;
      f32x4 acc[MF][2];
#pragma unroll
      for (int f = 0; f < MF; ++f) acc[f][0] = acc[f][1] = f32x4{0.f, 0.f, 0.f, 0.f};
      sweep<PH, PY, PX>(acc, bw, hb, qb, kt, lchunk);
      exchange_to_stage(acc, scr, ostage, wkh, wn, lane, l15, lh);
      store_stage(PY < 0 ? 0 : PY, PX < 0 ? 0 : PX);
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using IN = std::integral_constant<int, -1>;
    if constexpr (PH) {
      // the next phase's stage writes come after its MFMA sweep and the
      // exchange barrier, which every thread reaches only after finishing the
      // previous phase's store loop
      phase(I0{}, I0{});
      phase(I0{}, I1{});
      phase(I1{}, I0{});
      phase(I1{}, I1{});
    } else {
      phase(IN{}, IN{});
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

int grid_half(int tiles) {
  int dev = 0, cus = 256;
  DMP_HIP_CHECK(hipGetDevice(&dev));
  DMP_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  return std::max(1, std::min(tiles, cus / 2));
}

void check_wmat(const at::Tensor& wmat, const char* who) {
  TORCH_CHECK(wmat.scalar_type() == at::kBFloat16 && wmat.is_contiguous() && wmat.dim() == 2 &&
                  wmat.size(0) == CO && wmat.size(1) == 9 * CI, who, ": wmat must be contiguous [128, 1152] bf16");
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
  check_wmat(wmat, "conv3x3_c128");
  TORCH_CHECK(wmat.device() == x.device(), "conv3x3_c128: device mismatch");
  const int64_t n = x.size(0), H = x.size(2);
  const int64_t tiles64 = n * (H / R);
  TORCH_CHECK(tiles64 < (1 << 30), "conv3x3_c128: too many tiles");
  const int tiles = (int)tiles64;
  auto y = at::empty({n * H * W, CO}, x.options());
  if (tiles == 0) return {y, at::zeros({moments ? 2 * CO + 1 : 0}, x.options().dtype(at::kDouble))};
  auto stream = at::hip::getCurrentHIPStream();
  const int half = grid_half(tiles);
  const int grid = 2 * half;
  at::Tensor mom;
  if (moments) {
    mom = at::empty({2 * CO + 1}, x.options().dtype(at::kDouble));
    auto part = at::empty({2, half, CO}, x.options().dtype(at::kFloat));
    hipLaunchKernelGGL((conv3x3_c128_kernel<true, false>), dim3(grid), dim3(NT), 0, stream,
                       reinterpret_cast<const bf16*>(x.data_ptr()), reinterpret_cast<const bf16*>(wmat.data_ptr()),
                       reinterpret_cast<bf16*>(y.data_ptr()), part.data_ptr<float>(),
                       moments_zero_target(mom.data_ptr<double>(), half), (int)H, tiles);
    bn_reduce_partials_launch(part.data_ptr<float>(), half, CO, mom.data_ptr<double>(), (double)(n * H * W),
                              stream);
  } else {
    mom = at::empty({0}, x.options().dtype(at::kDouble));
    hipLaunchKernelGGL((conv3x3_c128_kernel<false, false>), dim3(grid), dim3(NT), 0, stream,
                       reinterpret_cast<const bf16*>(x.data_ptr()), reinterpret_cast<const bf16*>(wmat.data_ptr()),
                       reinterpret_cast<bf16*>(y.data_ptr()), nullptr, nullptr, (int)H, tiles);
  }
  DMP_HIP_CHECK(hipGetLastError());
  return {y, mom};
}

// Data gradient of a 3x3 / stride-2 / pad-1 128 -> 128 conv on a 2H x 56 input:
// dy [N, 128, H, 28] bf16 channels_last (H % 4 == 0), wt = W permuted to
// [cin][ky][kx][cout] (unflipped) flattened to [128, 1152].  Returns dx as
// [N*2H*56, 128].
at::Tensor conv3x3_c128_dgrad_s2(const at::Tensor& dy, const at::Tensor& wt) {
  TORCH_CHECK(dy.is_cuda() && dy.scalar_type() == at::kBFloat16 && dy.dim() == 4,
              "conv3x3_c128_dgrad_s2: bf16 NCHW-shaped dy");
  TORCH_CHECK(conv3x3_c128_supported(dy.size(1), dy.size(2), dy.size(3)) &&
                  dy.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv3x3_c128_dgrad_s2: dy must be [N, 128, H % 4 == 0, 28] channels_last");
  check_wmat(wt, "conv3x3_c128_dgrad_s2");
  TORCH_CHECK(wt.device() == dy.device(), "conv3x3_c128_dgrad_s2: device mismatch");
  const int64_t n = dy.size(0), H = dy.size(2);
  const int64_t tiles64 = n * (H / R);
  TORCH_CHECK(tiles64 < (1 << 30) && n * 4 * H * W < (1LL << 31), "conv3x3_c128_dgrad_s2: too large");
  const int tiles = (int)tiles64;
  auto dx = at::empty({n * 4 * H * W, CI}, dy.options());
  if (tiles == 0) return dx;
  auto stream = at::hip::getCurrentHIPStream();
  const int half = grid_half(tiles);
  hipLaunchKernelGGL((conv3x3_c128_kernel<false, true>), dim3(2 * half), dim3(NT), 0, stream,
                     reinterpret_cast<const bf16*>(dy.data_ptr()), reinterpret_cast<const bf16*>(wt.data_ptr()),
                     reinterpret_cast<bf16*>(dx.data_ptr()), nullptr, nullptr, (int)H, tiles);
  DMP_HIP_CHECK(hipGetLastError());
  return dx;
}

}  // namespace dmp
