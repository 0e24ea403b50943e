// Weight gradient of a 3x3 / stride-1 / pad-1 convolution (every stride-1 3x3
// of ResNet-50: 64 ch at 56x56, 128 at 28x28, 256 at 14x14, 512 at 7x7) as a
// persistent, halo-tiled MFMA kernel.
//
//   dW[co][kh][kw][ci] = sum over output pixels p of dy[p][co] * x[p + (kh-1, kw-1)][ci]
//
// The reduction runs over N*H*W pixels; the output is tiny.  The implicit-GEMM
// forms (our split-M TN kernel, MIOpen's igemm_wrw) gather the x operand nine
// times through L2 and ran at 0.35-0.64 ms per call at batch 1024 (3.4-4.7x the
// conv's floor, profiles/raw_r2/roofline_wgrad_xl.log).  Here every block
// owns one 64 (co) x 576 (9 taps x 64 ci) slice of dW in REGISTERS for its
// whole life and streams a contiguous range of pixel tiles through LDS:
//
//   * a tile is R output rows of one image (IMGS = 1) or IMGS whole small
//     images; its dy rows [P][64 co] and its zero-padded x halo
//     [(R+2) x (W+2) per image][64 ci] are staged by LDS-DMA
//     (global_load_lds_dwordx4), double buffered: tile t+1 lands while tile t
//     multiplies.  Both images keep whole 128-B pixel rows, 16-B chunks XOR-
//     swizzled by key(row) = 2 * ((row >> 1) & 3) (applied to the DMA source
//     address, undone on the read);
//   * 4 waves, one per SIMD; wave w owns all 64 co x columns [144 w, 144 w +
//     144) of the 576: 4 x 9 accumulator tiles of 16 x 16 (144 fp32 VGPRs);
//   * both MFMA operands (dy^T as A, the tapped x as B) need 8 consecutive
//     PIXELS per lane, i.e. a transpose of the pixel-major images: read with
//     ds_read_b64_tr_b16 (cdna_hip_programming.md T10).  The pixels of a
//     k-step are assigned to (lane group, element) so that each 32-lane half
//     reads 8 consecutive pixel rows (256 B = one bank row: conflict-free with
//     the key above for any 8 consecutive rows);
//   * each k-step (32 pixels) is 26 transposed reads and 36 MFMA 16x16x32 per
//     wave; the next k-step's reads are issued between the current MFMAs.
//
// Channel counts above 64 are cut into S = (C/64)^2 (co slice, ci slice)
// combos; the S blocks of one pixel range sit on one XCD (same L2: each dy / x
// slice is fetched from HBM once and re-read from L2).  Every block writes its
// 64 x 576 fp32 partial once; wgrad_reduce sums the partials of each combo in
// a fixed order (bitwise reproducible) straight into the bf16 [Cout][3][3][Cin]
// (channels-last) weight gradient.
// Reference: the convolutions whose weight gradients these are -- torchvision
// ResNet-50's cuDNN/MIOpen 3x3s (reference model_parallel.py:61).
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include "../common.h"
#include <type_traits>

namespace dmp {
namespace {

using bf16 = __bf16;
using gptr_t = const __attribute__((address_space(1))) void*;
using lptr_t = __attribute__((address_space(3))) void*;
using v4i16 = short __attribute__((ext_vector_type(4)));
using lds_v4 = __attribute__((address_space(3))) v4i16;
using i16x8 = short __attribute__((ext_vector_type(8)));

constexpr int kCh = 64;          // channels per slice (one 128-B LDS row per pixel)
constexpr int kWaves = 4;
constexpr int kCols = 9 * kCh;   // 576 output columns (tap, ci) per slice
constexpr int kWCols = kCols / kWaves;  // 144 per wave = 9 fragments of 16
constexpr int kNB = kWCols / 16;        // 9
constexpr int kMB = kCh / 16;           // 4 co fragments

__device__ __attribute__((aligned(16))) uint32_t g_wg_zero[4];

// Tile geometry for output width W, R output rows per tile, IMGS images per
// tile (small maps), stride S (1 or 2; pad 1), KS 32-pixel k-steps per tile.
// Halo of a tile = S*(R-1)+3 input rows x S*(W-1)+3 input columns per image;
// for S = 2 each halo row stores its even columns first, then the odd ones,
// so the pixels a tap reads for consecutive output columns stay consecutive
// rows of the LDS image (stride-1 reads, same bank analysis as S = 1).
template <int W, int R, int IMGS, int NW, int S, int KS>
struct WgGeo {
  static constexpr int HC = S * (W - 1) + 3;              // halo columns (LDS rows per halo row)
  static constexpr int HR = S * (R - 1) + 3;              // halo rows per image
  static constexpr int HIMG = HR * HC;                    // LDS rows per image
  static constexpr int HROWS = IMGS * HIMG;
  static constexpr int P = IMGS * R * W;                  // output pixels per full tile
  static constexpr int PALLOC = 32 * KS;
  static constexpr int DY_INSTR = (P + 7) / 8;            // 1-KB DMA pieces = 8 rows of 128 B
  static constexpr int H_INSTR = (HROWS + 7) / 8;
  static constexpr int DY_PW = (DY_INSTR + NW - 1) / NW;  // pieces per wave
  static constexpr int H_PW = (H_INSTR + NW - 1) / NW;
  static constexpr int DY_BYTES = PALLOC * 128;           // rows >= P stay zero (set once)
  static constexpr int BUF_BYTES = DY_BYTES + H_INSTR * 1024;
  static constexpr int SMEM = 2 * BUF_BYTES;
  static constexpr int MBW = kMB * kWaves / NW;           // co fragments per wave (4 or 2)
  // chunk-swizzle key index: the skewed index (conflict-free at row / image
  // crossings, see the hb / kt comment) where its parity matches the physical
  // row's, else the physical row itself
  static constexpr bool SKEW = S == 1 || (W % 2 == 0 && IMGS == 1);
  static_assert(P <= PALLOC && P > PALLOC - 32, "tile must fill its k-steps");
  static_assert(SMEM <= 160 * 1024, "LDS budget");
  static_assert(NW == 4 || NW == 8, "4 waves (64 co each) or 8 (32 co each, 2 per SIMD)");
  static_assert(S == 1 || S == 2, "stride 1 or 2");
  // LDS row of halo column hc inside a halo row
  static constexpr __device__ __host__ int pos(int hc) { return S == 1 ? hc : ((hc & 1) ? (HC + 1) / 2 + (hc >> 1) : hc >> 1); }
  // LDS row offset of tap (kh, kw) from the output pixel's tap-(0,0) row
  static constexpr __device__ __host__ int tap_off(int kh, int kw) { return kh * HC + pos(kw); }
  // key-index offset of tap (kh, kw) from the pixel's own key index
  static constexpr __device__ __host__ int key_off(int kh, int kw) {
    return !SKEW ? tap_off(kh, kw) : S == 1 ? kh * W + kw : (kh >> 1) * W + (kw >> 1) + (kh & 1) + (kw & 1);
  }
  // key index of halo row (img, hy, hc)
  static constexpr __device__ __host__ int key_of(int img, int hy, int hc) {
    return !SKEW ? img * HIMG + hy * HC + pos(hc)
                 : S == 1 ? img * (R * W) + hy * W + hc : (hy >> 1) * W + (hc >> 1) + (hy & 1) + (hc & 1);
  }
};

// step(integral_constant<int, 0>) ... step(integral_constant<int, N - 1>), in order
template <int I, int N, typename F>
__device__ __forceinline__ void static_for_impl(F& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for_impl<I + 1, N>(f);
  }
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F& f) {
  static_for_impl<0, N>(f);
}

__device__ __forceinline__ int wg_key(int row) { return ((row >> 1) & 3) << 1; }
// nibble i = wg_key(i) for row residues i = 0..7
constexpr uint32_t kKeyTab = 0x66442200u;

// LDS-DMA (global_load_lds_dwordx4) issued from inline asm: hipcc's waitcnt
// pass cannot tell which LDS bytes a pending builtin LDS-DMA writes, so it
// puts an s_waitcnt vmcnt(0) before the next ds_read -- i.e. every tile would
// wait for the NEXT tile's copy right after issuing it (measured: the first
// read of each tile).  Hidden in asm, the copies stay in flight across the
// whole tile; the explicit vmcnt(0) + barrier at the top of the next tile is
// the only (and sufficient) RAW ordering.  M0 = the wave's LDS destination.
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

struct WgArgs {
  const bf16* dy;  // [N*H*W][C] (channels-last), C = co channel stride
  const bf16* x;   // [N*H*W][C]
  float* part;     // [S][NB][64][576]
  int N, H, C;     // H = output rows; C = channels (in == out)
  int HI, WI;      // input rows / columns (stride 2: 2 H x 2 W)
  int S, NB;       // (co, ci) slice combos, blocks per combo
  int tiles, tiles_per_img;  // IMGS == 1: row tiles of R rows; IMGS > 1: image groups
};

// NW = 4: one wave per SIMD, wave w = all 64 co x columns [144 w, 144 w + 144).
// NW = 8: two waves per SIMD (<= 256 registers each); wave w: co half (w >> 2),
// the same 144 columns as wave (w & 3), so a SIMD's two waves can cover each
// other's LDS-read, DMA-issue and barrier stalls.
template <int W, int R, int IMGS, int NW, int S, int KS>
__global__ __launch_bounds__(64 * NW, 1) void wgrad3x3_kernel(WgArgs a) {
  using G = WgGeo<W, R, IMGS, NW, S, KS>;
  constexpr int MBW = G::MBW;
  __shared__ __attribute__((aligned(1024))) char smem[G::SMEM];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wc = wave & 3, wh = wave >> 2;

  // ---- block -> (slice combo, pixel-tile range); the S combos of a range share an XCD
  int combo, range;
  {
    const int b = blockIdx.x;
    if (a.S <= 32) {
      const int slot = b >> 3;
      combo = slot % a.S;
      range = (slot / a.S) * 8 + (b & 7);
    } else {
      combo = b % a.S;
      range = b / a.S;
    }
  }
  const int nsl = a.C / kCh;
  const int co0 = (combo / nsl) * kCh, ci0 = (combo % nsl) * kCh;
  const int t_begin = (int)((int64_t)a.tiles * range / a.NB);
  const int t_end = (int)((int64_t)a.tiles * (range + 1) / a.NB);
  const int HWp = a.H * W;              // output pixels per image
  const int HWi = a.HI * a.WI;          // input pixels per image

  // rows >= P of both dy buffers are never DMA'd: zero them once
  for (int i = G::P * 8 + threadIdx.x; i < G::PALLOC * 8; i += 64 * NW) {
    *reinterpret_cast<u32x4*>(smem + i * 16) = u32x4{0u, 0u, 0u, 0u};
    *reinterpret_cast<u32x4*>(smem + G::BUF_BYTES + i * 16) = u32x4{0u, 0u, 0u, 0u};
  }

  // ---- tile-invariant DMA slot tables (lane-linear LDS image, swizzled source)
  // dy: piece (wave + NW i) = rows 8 piece .. +7; this lane's row = 8 piece +
  // lane / 8, logical chunk = (lane & 7) ^ key(row)
  int dy_off[G::DY_PW];
  int dy_row[G::DY_PW];
#pragma unroll
  for (int i = 0; i < G::DY_PW; ++i) {
    const int piece = wave + NW * i;
    const int row = piece * 8 + (lane >> 3);
    const int c = (lane & 7) ^ wg_key(row);
    dy_row[i] = row;
    dy_off[i] = row * a.C + c * 8;
  }
  // halo: row -> (img, hy, hx); offset from the tile's (image, first output row)
  // origin, plus packed validity bits: hx in range (bit 0), hy (bits 1-5), img (6-8)
  int h_off[G::H_PW];
  int h_pk[G::H_PW];
#pragma unroll
  for (int i = 0; i < G::H_PW; ++i) {
    const int piece = wave + NW * i;
    const int row = piece * 8 + (lane >> 3);
    const int img = row / G::HIMG;
    const int rr = row - img * G::HIMG;
    const int hy = rr / G::HC, pr = rr - hy * G::HC;
    // LDS position pr -> halo column hc (S = 2: evens first, then odds)
    const int hc = S == 1 ? pr : (pr < (G::HC + 1) / 2 ? 2 * pr : 2 * (pr - (G::HC + 1) / 2) + 1);
    const int c = (lane & 7) ^ wg_key(G::key_of(img, hy, hc));
    const int ix = hc - 1;
    const bool xok = ix >= 0 && ix < a.WI && row < G::HROWS;
    h_off[i] = (img * HWi + (hy - 1) * a.WI + ix) * a.C + c * 8;
    h_pk[i] = (xok ? 1 : 0) | (hy << 1) | (img << 6);
  }

  auto issue = [&](int t, char* buf) {
    int n0, r0, valid_rows, valid_imgs;
    if constexpr (IMGS == 1) {
      n0 = t / a.tiles_per_img;
      r0 = (t - n0 * a.tiles_per_img) * R;
      valid_rows = min(R, a.H - r0);
      valid_imgs = 1;
    } else {
      n0 = t * IMGS;
      r0 = 0;
      valid_rows = R;
      valid_imgs = min(IMGS, a.N - n0);
    }
    const int64_t pix0 = (int64_t)n0 * HWp + (int64_t)r0 * W;
    const int pvalid = IMGS == 1 ? valid_rows * W : valid_imgs * R * W;
    const bf16* dyb = a.dy + pix0 * a.C + co0;
    // halo row hy of the tile = input row S*r0 - 1 + hy (h_off carries the -1)
    const bf16* xb = a.x + ((int64_t)n0 * HWi + (int64_t)(S * r0) * a.WI) * a.C + ci0;
#pragma unroll
    for (int i = 0; i < G::DY_PW; ++i) {
      const int piece = wave + NW * i;
      if (piece < G::DY_INSTR) {
        const void* src = dy_row[i] < pvalid ? (const void*)(dyb + dy_off[i]) : (const void*)g_wg_zero;
        glds16(src, buf + piece * 1024);
      }
    }
    char* hbuf = buf + G::DY_BYTES;
#pragma unroll
    for (int i = 0; i < G::H_PW; ++i) {
      const int piece = wave + NW * i;
      if (piece < G::H_INSTR) {
        const int pk = h_pk[i];
        const int hy = (pk >> 1) & 31, img = pk >> 6;
        const int iy = S * r0 - 1 + hy;
        const bool ok = (pk & 1) && iy >= 0 && iy < a.HI && img < valid_imgs;
        const void* src = ok ? (const void*)(xb + h_off[i]) : (const void*)g_wg_zero;
        glds16(src, hbuf + piece * 1024);
      }
    }
  };

  // ---- per-lane tr-read geometry.  Lane l = 16 g + 4 q + p; MFMA k index
  // 8 g + j (j = element) <-> k-step pixel 16 (g >> 1) + 8 (j >> 2) + 4 (g & 1) + (j & 3):
  // read r (= j >> 2) of lane l addresses pixel 32 ks + 16 (g >> 1) + 8 r + 4 (g & 1) + q,
  // channels 4 p .. 4 p + 3 of the fragment's 16.
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int pin = 16 * (g >> 1) + 4 * (g & 1) + q;  // + 32 ks + 8 r
  const int lofs = (p & 1) * 8 + (p >> 1) * 16;     // byte within the 32-B fragment span
  // B (halo) reads.  The halo row (img, hy, hx) keeps its chunks XOR-swizzled
  // by key(s), s = img*R*W + hy*W + hx -- a SKEWED index: output pixel pp at
  // tap (kh, kw) reads the row with s = pp + kh*W + kw, so the 8 consecutive
  // output pixels of a half-wave read always see 8 consecutive s, even where
  // they cross an output row or image (the physical halo row jumps by 2 there;
  // keyed by the physical row those reads were 2-way bank conflicts, ~10 % of
  // the l3 kernel).  s and the physical row have the same parity for every W,
  // so the read of a row pair stays on the two 128-B halves of a bank row.
  // Byte address of (row, chunk pair f) = row*128 + lofs + ((2f ^ key(s)) << 4);
  // key(s) depends on s & 7 only.  Per (k-step, r): hb = the tap-(0,0) row's
  // row*128 + lofs, and kt = the key table rotated to pp's residue, so the key
  // at tap offset (kh*W + kw) is one nibble of kt: per tap one bit-field
  // extract and one shift-or, per fragment one xor; the physical row offset
  // (kh*(W+2) + kw)*128 rides in the instruction's offset field.
  // Pixels past the tile's P (zero dy rows) are clamped onto a real halo row so
  // nothing non-finite is read.
  int hb[KS][2];
  uint32_t kt[KS][2];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int pp = min(32 * ks + 8 * r + pin, G::P - 1);
      const int img = pp / (R * W);
      const int rem = pp - img * (R * W);
      const int oy = rem / W, ox = rem - oy * W;
      const int row = img * G::HIMG + S * oy * G::HC + ox;  // tap (0, 0)
      hb[ks][r] = row * 128 + lofs + G::DY_BYTES;
      // key index at tap (0, 0): the skewed index is the pixel itself
      const int kidx = G::SKEW ? (S == 1 ? pp : oy * W + ox) : row;
      const uint32_t sh = 4u * (uint32_t)(kidx & 7);
      kt[ks][r] = sh == 0 ? kKeyTab : (kKeyTab >> sh) | (kKeyTab << (32u - sh));
    }
  // A (dy) reads: rows 32 ks + 8 r + pin have key(row) == key(pin) (the k-step
  // offsets only move bits >= 3): a_base[i] + a compile-time offset
  int a_base[MBW];
#pragma unroll
  for (int i = 0; i < MBW; ++i) a_base[i] = pin * 128 + (((2 * (MBW * wh + i)) ^ wg_key(pin)) << 4) + lofs;

  f32x4 acc[MBW][kNB];
#pragma unroll
  for (int i = 0; i < MBW; ++i)
#pragma unroll
    for (int j = 0; j < kNB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // each column group runs its own copy of the tile loop with its 9 fragments'
  // taps and channel groups as compile-time constants
  auto run = [&](auto wv_tag) {
    constexpr int WV = decltype(wv_tag)::value;
    if (t_begin < t_end) issue(t_begin, smem);
    int cur = 0;
    for (int t = t_begin; t < t_end; ++t) {
      int hbc[KS][2], abc[MBW];
      // opaque per tile: the per-(k-step, fragment) addresses are rebuilt inside
      // the loop instead of hoisted into ~130 live registers (they would spill)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        asm volatile("" : "+v"(hb[ks][0]), "+v"(hb[ks][1]), "+v"(kt[ks][0]), "+v"(kt[ks][1]));
        hbc[ks][0] = hb[ks][0] + cur * G::BUF_BYTES;
        hbc[ks][1] = hb[ks][1] + cur * G::BUF_BYTES;
      }
#pragma unroll
      for (int i = 0; i < MBW; ++i) abc[i] = a_base[i] + cur * G::BUF_BYTES;
      vmcnt<0>();     // this wave's pieces of tile t landed
      raw_barrier();  // ... every wave's; and everyone is done reading the other buffer
      if (t + 1 < t_end) issue(t + 1, smem + (cur ^ 1) * G::BUF_BYTES);

      bf16x8 fa[2][MBW], fb[2][kNB];
      auto rd = [&](int addr) -> v4i16 {
        return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(smem + addr));
      };
      auto load_step = [&](auto ks_tag, bf16x8 (&da)[MBW], bf16x8 (&db)[kNB]) {
        constexpr int ks = decltype(ks_tag)::value;
#pragma unroll
        for (int i = 0; i < MBW; ++i) {
          const v4i16 lo = rd(abc[i] + (32 * ks) * 128);
          const v4i16 hi = rd(abc[i] + (32 * ks + 8) * 128);
          const i16x8 t8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          da[i] = __builtin_bit_cast(bf16x8, t8);
        }
        int base[2][3];  // per r, per distinct tap of this column group (at most 3)
        constexpr int tap0 = (kWCols * WV) >> 6;
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
          for (int u = 0; u < 3; ++u) {
            const int tap = min(tap0 + u, 8);
            const int so = G::key_off(tap / 3, tap % 3);
            const uint32_t key = (kt[ks][r] >> (4 * (so & 7))) & 7u;
            base[r][u] = hbc[ks][r] | (int)(key << 4);
          }
#pragma unroll
        for (int j = 0; j < kNB; ++j) {
          const int col = kWCols * WV + 16 * j;
          const int tap = col >> 6, f = (col >> 4) & 3;
          const int o = G::tap_off(tap / 3, tap % 3);
          const v4i16 lo = rd((base[0][tap - tap0] ^ (f << 5)) + o * 128);
          const v4i16 hi = rd((base[1][tap - tap0] ^ (f << 5)) + o * 128);
          const i16x8 t8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          db[j] = __builtin_bit_cast(bf16x8, t8);
        }
      };
      load_step(std::integral_constant<int, 0>{}, fa[0], fb[0]);
      auto step = [&](auto ks_tag) {
        constexpr int ks = decltype(ks_tag)::value;
        constexpr int NRD = 2 * (MBW + kNB), NMF = MBW * kNB;
        if constexpr (ks + 1 < KS)
          load_step(std::integral_constant<int, ks + 1>{}, fa[(ks + 1) & 1], fb[(ks + 1) & 1]);
        // fragment-j-major order: the first MFMAs need A and B0 only, so the
        // waits on the next step's reads can be counted, not lgkmcnt(0)
#pragma unroll
        for (int j = 0; j < kNB; ++j)
#pragma unroll
          for (int i = 0; i < MBW; ++i)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[ks & 1][i], fb[ks & 1][j], acc[i][j], 0, 0, 0);
        if constexpr (ks + 1 < KS) {
          // the next step's reads spread over this step's MFMAs
          // (NW 4: 26 reads over 36 MFMAs; NW 8: 22 reads over 18, two per MFMA first)
          constexpr int PAIRS = NRD < NMF ? NRD : NMF;
          constexpr int DOUBLE = NRD > NMF ? NRD - NMF : 0;
#pragma unroll
          for (int u = 0; u < DOUBLE; ++u) {
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // DS read
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
          }
#pragma unroll
          for (int u = DOUBLE; u < PAIRS; ++u) {
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
          }
          if constexpr (NMF > PAIRS) __builtin_amdgcn_sched_group_barrier(0x008, NMF - PAIRS, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      };
      static_for<KS>(step);
      cur ^= 1;
    }
  };
  switch (wc) {
    case 0: run(std::integral_constant<int, 0>{}); break;
    case 1: run(std::integral_constant<int, 1>{}); break;
    case 2: run(std::integral_constant<int, 2>{}); break;
    default: run(std::integral_constant<int, 3>{}); break;
  }

  // ---- partial: D row = co (16 (MBW wh + i) + 4 g + e), column = 144 wc + 16 j + (lane & 15)
  float* pb = a.part + ((int64_t)combo * a.NB + range) * (int64_t)(kCh * kCols);
#pragma unroll
  for (int i = 0; i < MBW; ++i)
#pragma unroll
    for (int j = 0; j < kNB; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int co = 16 * (MBW * wh + i) + 4 * g + e;
        const int col = kWCols * wc + 16 * j + (lane & 15);
        pb[co * kCols + col] = acc[i][j][e];
      }
}

// out[co0 + co][tap][ci0 + ci] (bf16, [C][9][C]) = sum over the NB partials of
// the combo.  Block = 4 row groups x 64 threads x 4 consecutive columns.
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part, int NB, int C,
                                                           bf16* __restrict__ out) {
  constexpr int kElems = kCh * kCols;  // 36864 per combo
  const int combo = blockIdx.y;
  const int grp = threadIdx.x >> 6, tl = threadIdx.x & 63;
  const int e0 = (blockIdx.x * 64 + tl) * 4;  // 4 consecutive partial columns
  const float* src = part + (int64_t)combo * NB * kElems + e0;
  f32x4 s[4] = {};
  int b = grp;
  for (; b + 12 < NB; b += 16) {
#pragma unroll
    for (int u = 0; u < 4; ++u) s[u] += *reinterpret_cast<const f32x4*>(src + (int64_t)(b + 4 * u) * kElems);
  }
  for (; b < NB; b += 4) s[0] += *reinterpret_cast<const f32x4*>(src + (int64_t)b * kElems);
  f32x4 t = (s[0] + s[1]) + (s[2] + s[3]);
  __shared__ f32x4 red[256];
  red[threadIdx.x] = t;
  __syncthreads();
  if (grp == 0) {
    const f32x4 v = ((red[tl] + red[64 + tl]) + red[128 + tl]) + red[192 + tl];
    const int nsl = C / kCh;
    const int co0 = (combo / nsl) * kCh, ci0 = (combo % nsl) * kCh;
    const int co = e0 / kCols, col = e0 - co * kCols;  // 4 columns never cross a 64-ci row
    const int tap = col >> 6, ci = col & 63;
    bf16x4 o;
#pragma unroll
    for (int u = 0; u < 4; ++u) o[u] = (bf16)v[u];
    *reinterpret_cast<bf16x4*>(out + ((int64_t)(co0 + co) * 9 + tap) * C + ci0 + ci) = o;
  }
}

int g_wgrad_waves = 8;  // set_wgrad3x3_waves (A/B runs)

template <int W, int R, int IMGS, int S, int KS>
void launch(const WgArgs& a, int grid, hipStream_t stream) {
  // the 4-wave variant (A/B runs, set_wgrad3x3_waves) exists for stride 1 only
  if constexpr (S == 1) {
    if (g_wgrad_waves == 4) {
      hipLaunchKernelGGL((wgrad3x3_kernel<W, R, IMGS, 4, S, KS>), dim3(grid), dim3(256), 0, stream, a);
      return;
    }
  }
  hipLaunchKernelGGL((wgrad3x3_kernel<W, R, IMGS, 8, S, KS>), dim3(grid), dim3(512), 0, stream, a);
}

}  // namespace

void set_wgrad3x3_waves(int64_t nw) {
  TORCH_CHECK(nw == 4 || nw == 8, "wgrad3x3 waves: 4 or 8");
  g_wgrad_waves = (int)nw;
}

// (C, output H, output W, stride) of the 3x3 / pad-1 convs with a tile geometry
bool wgrad3x3_supported(int64_t C, int64_t H, int64_t W, int64_t stride) {
  if (stride == 1)
    return (C == 64 && W == 56) || (C == 128 && W == 28 && H % 7 == 0) || (C == 256 && W == 14 && H == 14) ||
           (C == 512 && W == 7 && H == 7);
  // stride 2 where the halo kernel is at least on par with MIOpen's igemm_wrw at
  // batch 2048 (profiles/raw_r3/wgrad_bench_s2.log): 128 ch 0.73 vs 0.87 ms,
  // 256 ch 0.69 vs 0.68; the 512-channel 7x7 one (49-pixel tiles) measured
  // 0.76 vs 0.66 and stays on MIOpen
  if (stride == 2) return (C == 128 && W == 28 && H % 2 == 0) || (C == 256 && W == 14 && H == 14);
  return false;
}

// dW of y = conv3x3(x, W, stride s, pad 1) for dy: [N, C, Ho, Wo], x: [N, C,
// s*Ho, s*Wo] bf16 channels_last (C in = C out).  Returns [C, C, 3, 3] bf16 in
// channels_last memory ([C][3][3][C]).
at::Tensor wgrad3x3(const at::Tensor& dy, const at::Tensor& x, int64_t stride) {
  TORCH_CHECK(dy.is_cuda() && x.is_cuda() && dy.scalar_type() == at::kBFloat16 &&
                  x.scalar_type() == at::kBFloat16 && dy.dim() == 4 && x.dim() == 4,
              "wgrad3x3: bf16 4-D GPU tensors");
  TORCH_CHECK(dy.is_contiguous(at::MemoryFormat::ChannelsLast) && x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "wgrad3x3: channels_last tensors");
  const int64_t N = dy.size(0), C = dy.size(1), H = dy.size(2), Wd = dy.size(3);
  TORCH_CHECK(x.size(0) == N && x.size(1) == C && x.size(2) == stride * H && x.size(3) == stride * Wd,
              "wgrad3x3: x must be [N, C, stride*Ho, stride*Wo] for dy [N, C, Ho, Wo]");
  TORCH_CHECK(wgrad3x3_supported(C, H, Wd, stride), "wgrad3x3: unsupported shape C=", C, " Ho=", H, " Wo=", Wd,
              " stride=", stride);
  auto out = at::empty({C, C, 3, 3}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto stream = at::hip::getCurrentHIPStream();
  const int S = (int)((C / kCh) * (C / kCh));
  int dev = 0, cus = 256;
  DMP_HIP_CHECK(hipGetDevice(&dev));
  DMP_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  // persistent grid: one block per CU, a multiple of 8 S (XCD grouping of the combos)
  int grid = S <= 32 ? std::max(8 * S, cus / (8 * S) * 8 * S) : std::max(S, cus / S * S);
  const int NB = grid / S;
  auto part = at::empty({(int64_t)grid * kCh * kCols}, x.options().dtype(at::kFloat));
  WgArgs a;
  a.dy = reinterpret_cast<const bf16*>(dy.data_ptr());
  a.x = reinterpret_cast<const bf16*>(x.data_ptr());
  a.part = part.data_ptr<float>();
  a.N = (int)N;
  a.H = (int)H;
  a.C = (int)C;
  a.HI = (int)x.size(2);
  a.WI = (int)x.size(3);
  a.S = S;
  a.NB = NB;
  // per-slot offsets are int32 relative to a tile origin; the origin is int64
  TORCH_CHECK(x.size(2) * x.size(3) * C * 4 < ((int64_t)1 << 31), "wgrad3x3: image too large");
  auto rows = [&](int R) {
    a.tiles_per_img = (int)((H + R - 1) / R);
    a.tiles = (int)(N * a.tiles_per_img);
  };
  auto imgs = [&](int I) {
    a.tiles_per_img = 1;
    a.tiles = (int)((N + I - 1) / I);
  };
  if (stride == 1) {
    if (C == 64) { rows(4); launch<56, 4, 1, 1, 7>(a, grid, stream); }
    else if (C == 128) { rows(7); launch<28, 7, 1, 1, 7>(a, grid, stream); }
    else if (C == 256) { rows(14); launch<14, 14, 1, 1, 7>(a, grid, stream); }
    else { imgs(4); launch<7, 7, 4, 1, 7>(a, grid, stream); }
  } else {
    // stride 2: the halo is ~4x the output tile, so tiles are shorter
    if (C == 128) { rows(2); launch<28, 2, 1, 2, 2>(a, grid, stream); }       // 56 px, 5 x 57 halo
    else if (C == 256) { rows(7); launch<14, 7, 1, 2, 4>(a, grid, stream); }  // 98 px, 15 x 29 halo
    else TORCH_CHECK(false, "wgrad3x3: no stride-2 tile for C=", C);
  }
  DMP_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(kCh * kCols / 256, S), dim3(256), 0, stream,
                     part.data_ptr<float>(), NB, (int)C, reinterpret_cast<bf16*>(out.data_ptr()));
  DMP_HIP_CHECK(hipGetLastError());
  return out;
}

}  // namespace dmp
