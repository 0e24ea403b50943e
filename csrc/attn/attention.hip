// Fused multi-head self-attention for ViT-sized sequences (S <= 256, head
// dim 64) on gfx950: forward and backward, reading the packed qkv GEMM output
// and writing the packed dqkv gradient directly.
//
// Why not the generic flash-attention kernels: at ViT-B/16's S = 197 the
// sequence fits one workgroup's LDS whole, and the generic path costs
//   * three layout copies per layer: q/k/v split + head permute before the
//     kernel, the output transpose after it, and a concatenation of dq/dk/dv
//     back into the qkv gradient (profiles/vit_b16_bs128_1gpu_v2.md: 2.6 ms
//     of a 37 ms step);
//   * flash kernels tiled for long sequences running at ~100-175 TF/s here.
// Layout contract (torchvision ViT): qkv[t, :] of token t = b*S + s holds
// [q | k | v], each [H, 64]; o[t, h*64 + d]; dqkv like qkv.
//
// One workgroup (4 waves) per (batch, head).  MFMA v_mfma_f32_16x16x32_bf16
// throughout, with every product arranged so that no register transposes are
// needed (cdna_hip_programming.md §5.5 T10/T12):
//   * a D tile (lane l holds rows 4*(l>>4)+e, column l&15) feeds the next MFMA
//     directly as the operand whose contraction index is D's ROW index, with
//     the k order pi = {4g..4g+3, 16+4g..16+4g+3} over two stacked D tiles;
//   * the matching other operand is read from LDS with ds_read_b64_tr_b16 in
//     the same pi order (row-major [token][64] image, no transposed copies);
//   * forward computes S^T = K Q^T so the softmax runs over a D tile's rows
//     and P^T feeds O^T = V^T P^T; the output lands 4 consecutive head dims
//     per lane (8-byte stores into o).
// Backward (one kernel, 2 workgroups/CU): D_i = rowsum(dO * O) and the saved base-2 logsumexp
// recompute P in-kernel; phase A (per 16-key block) accumulates dV^T = dO^T P
// and dK^T = Q^T dS over all queries, phase B (per 16-query tile)
// dQ^T = K^T dS^T over all keys -- no atomics, no dq/dkv kernel split.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include "../common.h"

namespace dmp {
namespace {

using bf16 = __bf16;
using v4i16 = short __attribute__((ext_vector_type(4)));
using lds_v4 = __attribute__((address_space(3))) v4i16;
constexpr int DH = 64;
constexpr int LROW = DH + 8;  // LDS row stride (bf16): 144 B, 16-B aligned rows, spreads banks
constexpr int kThreads = 256;
constexpr float kLog2e = 1.4426950408889634f;

__device__ __forceinline__ bf16x8 lds8(const bf16* base, int row, int col) {
  return *reinterpret_cast<const bf16x8*>(base + row * LROW + col);
}

// pi-ordered transposed read: lane (group g, index i) gets column col0 + i of
// rows rbase + 4g + {0..3} (elements 0-3) and rbase + 16 + 4g + {0..3} (4-7).
__device__ __forceinline__ bf16x8 lds_tr8(const bf16* base, int rbase, int col0, int lane) {
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const bf16* a = base + (rbase + 4 * g + q) * LROW + col0 + 4 * p;
  v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)a);
  v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(a + 16 * LROW));
  short __attribute__((ext_vector_type(8))) t = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, t);
}

// two stacked D tiles -> one pi-ordered MFMA operand
__device__ __forceinline__ bf16x8 pack_pi(const float (&a)[4], const float (&b)[4]) {
  f32x8 f = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_convertvector(f, bf16x8);
}

// v_exp_f32 / v_log_f32 / v_rcp_f32 directly: exp2f / log2f / 1/x expand to
// 4-5 VALU each for denormal range handling (a compare, two selects and a
// v_ldexp around the v_exp), which the softmax never needs -- its exp2
// arguments are <= 0 (a tiny result flushing to 0 is the right answer), l >= 1
__device__ __forceinline__ float ex2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ float lg2(float x) { return __builtin_amdgcn_logf(x); }
__device__ __forceinline__ float rcp(float x) { return __builtin_amdgcn_rcpf(x); }

__device__ __forceinline__ f32x4 mfma(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// rows [0, S) of two [S, 64] strided matrices into zero-padded [SP][LROW] LDS
// images.  Every global load of both images is issued before the first LDS
// store (SP*16/256 16-B loads in flight per lane instead of one): the staging
// is the latency-bound head of both kernels.
template <int SP, int NT = kThreads>
__device__ __forceinline__ void stage2(bf16* dst0, const bf16* src0, int64_t ld0, bf16* dst1,
                                       const bf16* src1, int64_t ld1, int S) {
  constexpr int PER = SP * (DH / 8);
  constexpr int IT = (PER + NT - 1) / NT;
  bf16x8 r0[IT], r1[IT];
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int v = threadIdx.x + i * NT;
    const int r = v >> 3, c = (v & 7) * 8;
    const bool ok = v < PER && r < S;
    r0[i] = ok ? *reinterpret_cast<const bf16x8*>(src0 + (int64_t)r * ld0 + c) : bf16x8{};
    r1[i] = ok ? *reinterpret_cast<const bf16x8*>(src1 + (int64_t)r * ld1 + c) : bf16x8{};
  }
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int v = threadIdx.x + i * NT;
    if (v < PER) {
      const int r = v >> 3, c = (v & 7) * 8;
      *reinterpret_cast<bf16x8*>(dst0 + r * LROW + c) = r0[i];
      *reinterpret_cast<bf16x8*>(dst1 + r * LROW + c) = r1[i];
    }
  }
}

__device__ __forceinline__ void store4(bf16* p, const f32x4& v, float s) {
  bf16x4 o = {(bf16)(v[0] * s), (bf16)(v[1] * s), (bf16)(v[2] * s), (bf16)(v[3] * s)};
  *reinterpret_cast<bf16x4*>(p) = o;
}

// QT query tiles per wave pass: every K fragment (ds_read_b128) and V
// fragment (ds_read_b64_tr_b16) read from LDS feeds QT MFMAs instead of one,
// halving the LDS read traffic per FLOP at QT = 2 (LDS bandwidth, not MFMA,
// bounds the QT = 1 loop: 448 LDS cycles vs 224 MFMA cycles per SIMD and
// 16-query tile); costs QT x the score registers (NKT x 4 each).
template <int SP, int NW = 4, int QT = 1>
__global__ __launch_bounds__(NW * 64, 2) void attn_fwd_kernel(const bf16* __restrict__ qkv, int64_t ld,
                                                            int S, int H, float scale,
                                                            bf16* __restrict__ o, int64_t ldo,
                                                            float* __restrict__ lse) {
  constexpr int NKT = SP / 16;
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * SP * LROW];
  bf16* Ks = smem;
  bf16* Vs = smem + SP * LROW;
  const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
  const int D = H * DH;
  const bf16* qb = qkv + (int64_t)b * S * ld + h * DH;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int nqt = (S + 15) / 16;
  // This wave's query groups (QT tiles each) are wave, wave + NW, ...: their Q
  // fragments are loaded up front, in flight together with the K / V staging,
  // instead of one dependent global load at the head of every group.
  constexpr int NGRP = (NKT + QT - 1) / QT;
  constexpr int MAXT = (NGRP + NW - 1) / NW;
  bf16x8 qf[MAXT][QT][2];
#pragma unroll
  for (int i = 0; i < MAXT; ++i)
#pragma unroll
    for (int u = 0; u < QT; ++u) {
      const int qc = min(((wave + NW * i) * QT + u) * 16 + li, S - 1);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        qf[i][u][ks] = *reinterpret_cast<const bf16x8*>(qb + (int64_t)qc * ld + ks * 32 + g * 8);
    }
  stage2<SP, NW * 64>(Ks, qb + D, ld, Vs, qb + 2 * D, ld, S);
  __syncthreads();
  const float sl2 = scale * kLog2e;
#pragma unroll
  for (int i = 0; i < MAXT; ++i) {
    const int grp = wave + NW * i;
    if (grp * QT >= nqt) break;
    f32x4 st[QT][NKT];
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      const bf16x8 k0 = lds8(Ks, kt * 16 + li, g * 8), k1 = lds8(Ks, kt * 16 + li, 32 + g * 8);
#pragma unroll
      for (int u = 0; u < QT; ++u) st[u][kt] = mfma(k1, qf[i][u][1], mfma(k0, qf[i][u][0], f32x4{0.f, 0.f, 0.f, 0.f}));
    }
    // padded keys -> -inf after the whole MFMA chain (a branch inside it would
    // split the block the scheduler hoists the LDS reads across)
    if (S < SP) {
      // opaque per group: hoisted out of the tile loop, the 4 * NKT lane masks
      // would live in (spilled) SGPR pairs
      int lim = S - 4 * g;
      asm volatile("" : "+v"(lim));
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt)
        if (kt * 16 + 16 > S) {  // uniform
#pragma unroll
          for (int u = 0; u < QT; ++u)
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (kt * 16 + e >= lim) st[u][kt][e] = -INFINITY;
        }
    }
    float mb[QT], l[QT];
#pragma unroll
    for (int u = 0; u < QT; ++u) {
      float m = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
        for (int e = 0; e < 4; ++e) m = fmaxf(m, st[u][kt][e]);
      m = fmaxf(m, __shfl_xor(m, 16, 64));
      m = fmaxf(m, __shfl_xor(m, 32, 64));
      mb[u] = m * sl2;
      float ls = 0.f;
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float p = ex2(st[u][kt][e] * sl2 - mb[u]);
          st[u][kt][e] = p;
          ls += p;
        }
      ls += __shfl_xor(ls, 16, 64);
      l[u] = ls + __shfl_xor(ls, 32, 64);
    }
    f32x4 acc[QT][4];
#pragma unroll
    for (int u = 0; u < QT; ++u)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[u][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kc = 0; kc < NKT / 2; ++kc) {
      bf16x8 pb[QT];
#pragma unroll
      for (int u = 0; u < QT; ++u) {
        float p0[4], p1[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) { p0[e] = st[u][2 * kc][e]; p1[e] = st[u][2 * kc + 1][e]; }
        pb[u] = pack_pi(p0, p1);
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const bf16x8 vf = lds_tr8(Vs, kc * 32, t * 16, lane);
#pragma unroll
        for (int u = 0; u < QT; ++u) acc[u][t] = mfma(vf, pb[u], acc[u][t]);
      }
    }
#pragma unroll
    for (int u = 0; u < QT; ++u) {
      const int q = (grp * QT + u) * 16 + li;
      if (q < S) {
        const float inv = rcp(l[u]);
        bf16* orow = o + ((int64_t)b * S + q) * ldo + h * DH;
#pragma unroll
        for (int t = 0; t < 4; ++t) store4(orow + t * 16 + 4 * g, acc[u][t], inv);
        if (g == 0) lse[(int64_t)bh * SP + q] = mb[u] + lg2(l[u]);  // base-2 logsumexp of the scaled scores
      }
    }
  }
}

// Persistent forward: a grid of 2 workgroups per CU walks the (batch, head)
// pairs; while head i computes, the K / V rows and this wave's Q fragments of
// head i + grid are already loading into registers (56 + 32 VGPRs), so the
// staging of the next head is hidden behind the current one's MFMAs instead
// of stalling a workgroup at its start (round 3: ~10 % of MFMA peak).
template <int SP>
__global__ __launch_bounds__(kThreads, 2) void attn_fwd_pp_kernel(const bf16* __restrict__ qkv, int64_t ld,
                                                                 int S, int H, float scale,
                                                                 bf16* __restrict__ o, int64_t ldo,
                                                                 float* __restrict__ lse, int nbh) {
  constexpr int NKT = SP / 16;
  constexpr int PER = SP * (DH / 8);
  constexpr int IT = (PER + kThreads - 1) / kThreads;
  constexpr int MAXT = (SP / 16 + 3) / 4;
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * SP * LROW];
  bf16* Ks = smem;
  bf16* Vs = smem + SP * LROW;
  const int D = H * DH;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int nqt = (S + 15) / 16;
  const float sl2 = scale * kLog2e;
  bf16x8 rk[IT], rv[IT], qn[MAXT][2];
  auto load = [&](int bh) {
    const int b = bh / H, h = bh - b * H;
    const bf16* qb = qkv + (int64_t)b * S * ld + h * DH;
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int v = threadIdx.x + i * kThreads;
      const int r = v >> 3, c = (v & 7) * 8;
      const bool ok = v < PER && r < S;
      rk[i] = ok ? *reinterpret_cast<const bf16x8*>(qb + (int64_t)r * ld + D + c) : bf16x8{};
      rv[i] = ok ? *reinterpret_cast<const bf16x8*>(qb + (int64_t)r * ld + 2 * D + c) : bf16x8{};
    }
#pragma unroll
    for (int i = 0; i < MAXT; ++i) {
      const int qc = min((wave + 4 * i) * 16 + li, S - 1);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) qn[i][ks] = *reinterpret_cast<const bf16x8*>(qb + (int64_t)qc * ld + ks * 32 + g * 8);
    }
  };
  int bh = blockIdx.x;
  if (bh >= nbh) return;
  load(bh);
  for (; bh < nbh; bh += gridDim.x) {
    __syncthreads();  // every wave finished reading the previous head's K / V
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int v = threadIdx.x + i * kThreads;
      if (v < PER) {
        const int r = v >> 3, c = (v & 7) * 8;
        *reinterpret_cast<bf16x8*>(Ks + r * LROW + c) = rk[i];
        *reinterpret_cast<bf16x8*>(Vs + r * LROW + c) = rv[i];
      }
    }
    bf16x8 qf[MAXT][2];
#pragma unroll
    for (int i = 0; i < MAXT; ++i) { qf[i][0] = qn[i][0]; qf[i][1] = qn[i][1]; }
    __syncthreads();
    if (bh + (int)gridDim.x < nbh) load(bh + gridDim.x);  // next head, in flight during this one
    const int b = bh / H, h = bh - b * H;
#pragma unroll
    for (int i = 0; i < MAXT; ++i) {
      const int qt = wave + 4 * i;
      if (qt >= nqt) break;
      const int q = qt * 16 + li;
      f32x4 st[NKT];
      float m = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt) {
        f32x4 a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) a = mfma(lds8(Ks, kt * 16 + li, ks * 32 + g * 8), qf[i][ks], a);
        st[kt] = a;
      }
      // padded keys -> -inf after the whole MFMA chain (a branch inside it would
      // split the block the scheduler hoists the LDS reads across)
      if (S < SP) {
        // opaque per tile: hoisted out of the head / tile loops, the 4 * NKT
        // lane masks would live in (spilled) SGPR pairs
        int lim = S - 4 * g;
        asm volatile("" : "+v"(lim));
#pragma unroll
        for (int kt = 0; kt < NKT; ++kt)
          if (kt * 16 + 16 > S) {  // uniform
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (kt * 16 + e >= lim) st[kt][e] = -INFINITY;
          }
      }
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
        for (int e = 0; e < 4; ++e) m = fmaxf(m, st[kt][e]);
      m = fmaxf(m, __shfl_xor(m, 16, 64));
      m = fmaxf(m, __shfl_xor(m, 32, 64));
      const float mb = m * sl2;
      float l = 0.f;
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float pv = ex2(st[kt][e] * sl2 - mb);
          st[kt][e] = pv;
          l += pv;
        }
      l += __shfl_xor(l, 16, 64);
      l += __shfl_xor(l, 32, 64);
      f32x4 acc[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < NKT / 2; ++kc) {
        float p0[4], p1[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) { p0[e] = st[2 * kc][e]; p1[e] = st[2 * kc + 1][e]; }
        const bf16x8 pb = pack_pi(p0, p1);
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[t] = mfma(lds_tr8(Vs, kc * 32, t * 16, lane), pb, acc[t]);
      }
      if (q < S) {
        const float inv = rcp(l);
        bf16* orow = o + ((int64_t)b * S + q) * ldo + h * DH;
#pragma unroll
        for (int t = 0; t < 4; ++t) store4(orow + t * 16 + 4 * g, acc[t], inv);
        if (g == 0) lse[(int64_t)bh * SP + q] = mb + lg2(l);
      }
    }
  }
}

// ---- backward building blocks (shared by the per-head and persistent kernels) ----
template <int SP>
struct BwdCtx {
  static constexpr int MAXT = (SP / 16 + 3) / 4;
  int S, D, lane, wave, g, li, nt;
  float scale, sl2;
};

// D_i = sum_d dO[i][d] * O[i][d] (fp32, O from global, dO from the LDS image)
// and the saved base-2 logsumexp, into LDS
template <int SP>
__device__ __forceinline__ void bwd_rowstats(const BwdCtx<SP>& c, const bf16* dOs, const bf16* o, int64_t ldo,
                                             const float* lse, int b, int h, int bh, float* lse_s, float* dd_s) {
  for (int r = threadIdx.x; r < SP; r += kThreads) {
    float acc = 0.f;
    if (r < c.S) {
      const bf16* orow = o + ((int64_t)b * c.S + r) * ldo + h * DH;
#pragma unroll
      for (int cc = 0; cc < DH; cc += 8) {
        const f32x8 x = __builtin_convertvector(*reinterpret_cast<const bf16x8*>(orow + cc), f32x8);
        const f32x8 y = __builtin_convertvector(lds8(dOs, r, cc), f32x8);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc = fmaf(x[j], y[j], acc);
      }
    }
    dd_s[r] = acc;
    lse_s[r] = r < c.S ? lse[(int64_t)bh * SP + r] : INFINITY;
  }
}

// phase A: per 16-key block, dV^T = dO^T P and dK^T = Q^T dS over all queries
template <int SP>
__device__ __forceinline__ void bwd_phase_a(const BwdCtx<SP>& c, const bf16* Qs, const bf16* dOs,
                                            const float* lse_s, const float* dd_s,
                                            const bf16* kg, const bf16* vg, int64_t ld, bf16* dq_base,
                                            int64_t lddq) {
  // K / V fragments of this wave's key blocks (wave, wave + 4, ...): block
  // i + 1's are loaded while block i computes (rolling one-ahead prefetch)
  bf16x8 kf[2], vf[2], kn[2], vn[2];
  auto frag = [&](int kb, bf16x8 (&f0)[2], bf16x8 (&f1)[2]) {
    const int r = min(kb * 16 + c.li, c.S - 1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      f0[ks] = *reinterpret_cast<const bf16x8*>(kg + (int64_t)r * ld + ks * 32 + c.g * 8);
      f1[ks] = *reinterpret_cast<const bf16x8*>(vg + (int64_t)r * ld + ks * 32 + c.g * 8);
    }
  };
  frag(c.wave, kf, vf);
#pragma unroll
  for (int i = 0; i < BwdCtx<SP>::MAXT; ++i) {
    const int kb = c.wave + 4 * i;
    if (kb >= c.nt) break;
    if (kb + 4 < c.nt) frag(kb + 4, kn, vn);
    const int key = kb * 16 + c.li;
    const bool kin = key < c.S;
    const float km = kin ? 1.f : 0.f;
    f32x4 dv[4], dk[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) { dv[t] = f32x4{0.f, 0.f, 0.f, 0.f}; dk[t] = dv[t]; }
#pragma unroll 1
    for (int qc = 0; qc < SP / 32; ++qc) {
      float pp[2][4], dss[2][4];
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        const int q0 = qc * 32 + hf * 16;
        f32x4 sv = {0.f, 0.f, 0.f, 0.f}, dp = sv;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          sv = mfma(lds8(Qs, q0 + c.li, ks * 32 + c.g * 8), kf[ks], sv);
          dp = mfma(lds8(dOs, q0 + c.li, ks * 32 + c.g * 8), vf[ks], dp);
        }
        // the 4 query rows of this lane: one 16-B LDS read per row constant
        const f32x4 ls = *reinterpret_cast<const f32x4*>(lse_s + q0 + 4 * c.g);
        const f32x4 dd = *reinterpret_cast<const f32x4*>(dd_s + q0 + 4 * c.g);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float pv = ex2(sv[e] * c.sl2 - ls[e]) * km;  // a multiply, not a branch around the exp
          pp[hf][e] = pv;
          dss[hf][e] = pv * (dp[e] - dd[e]);
        }
      }
      const bf16x8 pb = pack_pi(pp[0], pp[1]);
      const bf16x8 dsb = pack_pi(dss[0], dss[1]);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        dv[t] = mfma(lds_tr8(dOs, qc * 32, t * 16, c.lane), pb, dv[t]);
        dk[t] = mfma(lds_tr8(Qs, qc * 32, t * 16, c.lane), dsb, dk[t]);
      }
    }
    if (kin) {
      bf16* row = dq_base + (int64_t)key * lddq;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        store4(row + c.D + t * 16 + 4 * c.g, dk[t], c.scale);
        store4(row + 2 * c.D + t * 16 + 4 * c.g, dv[t], 1.f);
      }
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) { kf[ks] = kn[ks]; vf[ks] = vn[ks]; }
  }
}

// phase B: per 16-query tile, dQ^T = K^T dS^T over all keys
template <int SP>
__device__ __forceinline__ void bwd_phase_b(const BwdCtx<SP>& c, const bf16* Ks, const bf16* Vs,
                                            const float* lse_s, const float* dd_s,
                                            const bf16* qg, int64_t ldq, const bf16* dg, int64_t ldd,
                                            bf16* dq_base, int64_t lddq) {
  bf16x8 qf[2], dof[2], qn[2], dn[2];
  auto frag = [&](int qt, bf16x8 (&f0)[2], bf16x8 (&f1)[2]) {
    const int r = min(qt * 16 + c.li, c.S - 1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      f0[ks] = *reinterpret_cast<const bf16x8*>(qg + (int64_t)r * ldq + ks * 32 + c.g * 8);
      f1[ks] = *reinterpret_cast<const bf16x8*>(dg + (int64_t)r * ldd + ks * 32 + c.g * 8);
    }
  };
  frag(c.wave, qf, dof);
#pragma unroll
  for (int i = 0; i < BwdCtx<SP>::MAXT; ++i) {
    const int qt = c.wave + 4 * i;
    if (qt >= c.nt) break;
    if (qt + 4 < c.nt) frag(qt + 4, qn, dn);
    const int q = qt * 16 + c.li;
    const float lq = lse_s[q], dq_d = dd_s[q];
    f32x4 dq[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) dq[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int kc = 0; kc < SP / 32; ++kc) {
      float dss[2][4];
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        const int k0 = kc * 32 + hf * 16;
        f32x4 sv = {0.f, 0.f, 0.f, 0.f}, dp = sv;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          sv = mfma(lds8(Ks, k0 + c.li, ks * 32 + c.g * 8), qf[ks], sv);
          dp = mfma(lds8(Vs, k0 + c.li, ks * 32 + c.g * 8), dof[ks], dp);
        }
        // no key mask: a padded key's K and V rows are zero in LDS, so its dS
        // multiplies a zero K row into dQ; the clamp keeps that dS finite
        // (exp2 of a real key's argument is <= 0 already: lq is the row's
        // logsumexp)
#pragma unroll
        for (int e = 0; e < 4; ++e) dss[hf][e] = ex2(fminf(sv[e] * c.sl2 - lq, 0.f)) * (dp[e] - dq_d);
      }
      const bf16x8 dsb = pack_pi(dss[0], dss[1]);
#pragma unroll
      for (int t = 0; t < 4; ++t) dq[t] = mfma(lds_tr8(Ks, kc * 32, t * 16, c.lane), dsb, dq[t]);
    }
    if (q < c.S) {
      bf16* row = dq_base + (int64_t)q * lddq;
#pragma unroll
      for (int t = 0; t < 4; ++t) store4(row + t * 16 + 4 * c.g, dq[t], c.scale);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) { qf[ks] = qn[ks]; dof[ks] = dn[ks]; }
  }
}

template <int SP>
__device__ __forceinline__ BwdCtx<SP> bwd_ctx(int S, int H, float scale) {
  BwdCtx<SP> c;
  c.S = S;
  c.D = H * DH;
  c.lane = threadIdx.x & 63;
  c.wave = threadIdx.x >> 6;
  c.g = c.lane >> 4;
  c.li = c.lane & 15;
  c.nt = (S + 15) / 16;
  c.scale = scale;
  c.sl2 = scale * kLog2e;
  return c;
}

template <int SP>
__global__ __launch_bounds__(kThreads, 2) void attn_bwd_kernel(
    const bf16* __restrict__ qkv, int64_t ld, const bf16* __restrict__ dout, int64_t ldd,
    const bf16* __restrict__ o, int64_t ldo, const float* __restrict__ lse, int S, int H, float scale,
    bf16* __restrict__ dqkv, int64_t lddq) {
  // Two LDS images, reused: phase A holds Q and dO (K / V rows of the wave's
  // key block come straight from L2 into registers), phase B holds K and V
  // (Q / dO rows of the query tile from L2).  64 KB + 2 KB -> 2 workgroups/CU.
  __shared__ __attribute__((aligned(16))) char smem[2 * SP * LROW * 2 + 2 * SP * 4];
  bf16* X0 = reinterpret_cast<bf16*>(smem);
  bf16* X1 = X0 + SP * LROW;
  float* lse_s = reinterpret_cast<float*>(X1 + SP * LROW);
  float* dd_s = lse_s + SP;
  const BwdCtx<SP> c = bwd_ctx<SP>(S, H, scale);
  const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
  const bf16* qb = qkv + (int64_t)b * S * ld + h * DH;
  const bf16* db = dout + (int64_t)b * S * ldd + h * DH;
  bf16* dq_base = dqkv + (int64_t)b * S * lddq + h * DH;
  stage2<SP>(X0, qb, ld, X1, db, ldd, S);  // Q, dO
  __syncthreads();
  bwd_rowstats<SP>(c, X1, o, ldo, lse, b, h, bh, lse_s, dd_s);
  __syncthreads();
  bwd_phase_a<SP>(c, X0, X1, lse_s, dd_s, qb + c.D, qb + 2 * c.D, ld, dq_base, lddq);
  // phase B: K and V replace Q and dO in LDS
  __syncthreads();
  stage2<SP>(X0, qb + c.D, ld, X1, qb + 2 * c.D, ld, S);  // K, V
  __syncthreads();
  bwd_phase_b<SP>(c, X0, X1, lse_s, dd_s, qb, ld, db, ldd, dq_base, lddq);
}

// Persistent backward: 2 workgroups per CU walk the (batch, head) pairs; each
// phase's LDS image is loaded into registers during the previous phase (K / V
// of head i during its phase A, Q / dO of head i + grid during phase B of i),
// so no phase waits on an HBM round trip for its operands.
template <int SP>
__global__ __launch_bounds__(kThreads, 2) void attn_bwd_pp_kernel(
    const bf16* __restrict__ qkv, int64_t ld, const bf16* __restrict__ dout, int64_t ldd,
    const bf16* __restrict__ o, int64_t ldo, const float* __restrict__ lse, int S, int H, float scale,
    bf16* __restrict__ dqkv, int64_t lddq, int nbh) {
  __shared__ __attribute__((aligned(16))) char smem[2 * SP * LROW * 2 + 2 * SP * 4];
  bf16* X0 = reinterpret_cast<bf16*>(smem);
  bf16* X1 = X0 + SP * LROW;
  float* lse_s = reinterpret_cast<float*>(X1 + SP * LROW);
  float* dd_s = lse_s + SP;
  const BwdCtx<SP> c = bwd_ctx<SP>(S, H, scale);
  constexpr int PER = SP * (DH / 8);
  constexpr int IT = (PER + kThreads - 1) / kThreads;
  bf16x8 rA[IT], rB[IT];
  auto gload = [&](const bf16* s0, int64_t l0, const bf16* s1, int64_t l1) {
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int v = threadIdx.x + i * kThreads;
      const int r = v >> 3, cc = (v & 7) * 8;
      const bool ok = v < PER && r < S;
      rA[i] = ok ? *reinterpret_cast<const bf16x8*>(s0 + (int64_t)r * l0 + cc) : bf16x8{};
      rB[i] = ok ? *reinterpret_cast<const bf16x8*>(s1 + (int64_t)r * l1 + cc) : bf16x8{};
    }
  };
  auto lstore = [&] {
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int v = threadIdx.x + i * kThreads;
      if (v < PER) {
        const int r = v >> 3, cc = (v & 7) * 8;
        *reinterpret_cast<bf16x8*>(X0 + r * LROW + cc) = rA[i];
        *reinterpret_cast<bf16x8*>(X1 + r * LROW + cc) = rB[i];
      }
    }
  };
  int bh = blockIdx.x;
  if (bh >= nbh) return;
  {
    const int b = bh / H, h = bh - b * H;
    gload(qkv + (int64_t)b * S * ld + h * DH, ld, dout + (int64_t)b * S * ldd + h * DH, ldd);  // Q, dO
  }
  for (; bh < nbh; bh += gridDim.x) {
    const int b = bh / H, h = bh - b * H;
    const bf16* qb = qkv + (int64_t)b * S * ld + h * DH;
    const bf16* db = dout + (int64_t)b * S * ldd + h * DH;
    bf16* dq_base = dqkv + (int64_t)b * S * lddq + h * DH;
    __syncthreads();  // the previous head's phase B is done with X0 / X1 / lse_s / dd_s
    lstore();         // Q, dO
    __syncthreads();
    gload(qb + c.D, ld, qb + 2 * c.D, ld);  // K, V: in flight during phase A
    bwd_rowstats<SP>(c, X1, o, ldo, lse, b, h, bh, lse_s, dd_s);
    __syncthreads();
    bwd_phase_a<SP>(c, X0, X1, lse_s, dd_s, qb + c.D, qb + 2 * c.D, ld, dq_base, lddq);
    __syncthreads();  // phase A is done with Q / dO
    lstore();         // K, V
    __syncthreads();
    const int nb = bh + gridDim.x;
    if (nb < nbh) {  // the next head's Q, dO: in flight during phase B
      const int b2 = nb / H, h2 = nb - b2 * H;
      gload(qkv + (int64_t)b2 * S * ld + h2 * DH, ld, dout + (int64_t)b2 * S * ldd + h2 * DH, ldd);
    }
    bwd_phase_b<SP>(c, X0, X1, lse_s, dd_s, qb, ld, db, ldd, dq_base, lddq);
  }
}

int pad_seq(int64_t S) {
  const int sp = (int)((S + 31) / 32 * 32);
  return sp <= 64 ? 64 : sp <= 128 ? 128 : sp <= 160 ? 160 : sp <= 192 ? 192 : sp <= 224 ? 224 : 256;
}

void check_2d(const at::Tensor& t, const char* name, int64_t rows, int64_t min_cols) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.dim() == 2, name,
              " must be a 2-D bf16 GPU tensor");
  TORCH_CHECK(t.size(0) == rows && t.size(1) >= min_cols, name, " has the wrong shape");
  TORCH_CHECK(t.stride(1) == 1 && t.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0,
              name, " rows must be contiguous and 16-byte aligned");
}

#define DMP_ATTN_DISPATCH(SP_, ...)                                        \
  switch (SP_) {                                                           \
    case 64: { constexpr int SPC = 64; __VA_ARGS__; break; }               \
    case 128: { constexpr int SPC = 128; __VA_ARGS__; break; }             \
    case 160: { constexpr int SPC = 160; __VA_ARGS__; break; }             \
    case 192: { constexpr int SPC = 192; __VA_ARGS__; break; }             \
    case 224: { constexpr int SPC = 224; __VA_ARGS__; break; }             \
    default: { constexpr int SPC = 256; __VA_ARGS__; break; }              \
  }

}  // namespace

bool attention_supported(int64_t S, int64_t head_dim) { return head_dim == DH && S >= 1 && S <= 256; }

namespace {
// defaults measured at ViT-B/16 batch 256 (tools/attn_bench.py, profiles/raw_r4/attn_bench_r4e.log):
// forward 8-wave 0.081 ms vs 4-wave 0.090 / two-tile 0.084 / persistent 0.096;
// backward per-head 0.249-0.258 ms vs persistent 0.264-0.266
int g_attn_bwd_variant = 0;  // 0: one workgroup per (batch, head); 1: persistent with prefetch
int g_attn_fwd_variant = 2;  // 0: one 4-wave workgroup per (batch, head); 1: persistent with
                             // next-head prefetch; 2: one 8-wave workgroup per (batch, head);
                             // 3: as 0 with two query tiles per wave pass
int g_num_cus_attn = 0;
}  // namespace

void set_attention_variant(int fwd, int bwd) {
  TORCH_CHECK(fwd >= 0 && fwd <= 3, "attention forward variant: 0 (per head), 1 (persistent), 2 (per head, 8 waves), "
              "3 (per head, 2 query tiles per wave pass)");
  TORCH_CHECK(bwd >= 0 && bwd <= 1, "attention backward variant: 0 (per head), 1 (persistent)");
  g_attn_fwd_variant = fwd;
  g_attn_bwd_variant = bwd;
}

std::vector<int64_t> get_attention_variant() { return {g_attn_fwd_variant, g_attn_bwd_variant}; }

// qkv [B*S, >= 3*H*64] -> (o [B*S, H*64], lse [B*H, SP] fp32, base-2)
std::vector<at::Tensor> attention_forward(const at::Tensor& qkv, int64_t B, int64_t S, int64_t H, double scale) {
  TORCH_CHECK(attention_supported(S, DH), "attention: S must be in [1, 256]");
  check_2d(qkv, "qkv", B * S, 3 * H * DH);
  const int sp = pad_seq(S);
  auto o = at::empty({B * S, H * DH}, qkv.options());
  auto lse = at::empty({B * H, sp}, qkv.options().dtype(at::kFloat));
  hipStream_t st = at::hip::getCurrentHIPStream();
  if (g_attn_fwd_variant == 1) {
    if (g_num_cus_attn == 0) {
      int dev = 0;
      DMP_HIP_CHECK(hipGetDevice(&dev));
      DMP_HIP_CHECK(hipDeviceGetAttribute(&g_num_cus_attn, hipDeviceAttributeMultiprocessorCount, dev));
    }
    const int nbh = (int)(B * H);
    const int grid = std::min(nbh, 2 * g_num_cus_attn);  // 2 workgroups per CU (LDS, launch bounds)
    DMP_ATTN_DISPATCH(sp, hipLaunchKernelGGL((attn_fwd_pp_kernel<SPC>), dim3(grid), dim3(kThreads), 0, st,
                                             (const bf16*)qkv.data_ptr(), qkv.stride(0), (int)S, (int)H,
                                             (float)scale, (bf16*)o.data_ptr(), o.stride(0),
                                             lse.data_ptr<float>(), nbh));
  } else if (g_attn_fwd_variant == 3) {
    DMP_ATTN_DISPATCH(sp, hipLaunchKernelGGL((attn_fwd_kernel<SPC, 4, 2>), dim3(B * H), dim3(kThreads), 0, st,
                                             (const bf16*)qkv.data_ptr(), qkv.stride(0), (int)S, (int)H,
                                             (float)scale, (bf16*)o.data_ptr(), o.stride(0),
                                             lse.data_ptr<float>()));
  } else if (g_attn_fwd_variant == 2) {
    DMP_ATTN_DISPATCH(sp, hipLaunchKernelGGL((attn_fwd_kernel<SPC, 8>), dim3(B * H), dim3(512), 0, st,
                                             (const bf16*)qkv.data_ptr(), qkv.stride(0), (int)S, (int)H,
                                             (float)scale, (bf16*)o.data_ptr(), o.stride(0),
                                             lse.data_ptr<float>()));
  } else {
    DMP_ATTN_DISPATCH(sp, hipLaunchKernelGGL((attn_fwd_kernel<SPC>), dim3(B * H), dim3(kThreads), 0, st,
                                             (const bf16*)qkv.data_ptr(), qkv.stride(0), (int)S, (int)H,
                                             (float)scale, (bf16*)o.data_ptr(), o.stride(0),
                                             lse.data_ptr<float>()));
  }
  DMP_HIP_CHECK(hipGetLastError());
  return {o, lse};
}

at::Tensor attention_backward(const at::Tensor& dout, const at::Tensor& qkv, const at::Tensor& o,
                              const at::Tensor& lse, int64_t B, int64_t S, int64_t H, double scale) {
  TORCH_CHECK(attention_supported(S, DH), "attention: S must be in [1, 256]");
  check_2d(qkv, "qkv", B * S, 3 * H * DH);
  check_2d(dout, "dout", B * S, H * DH);
  check_2d(o, "o", B * S, H * DH);
  const int sp = pad_seq(S);
  TORCH_CHECK(lse.is_cuda() && lse.scalar_type() == at::kFloat && lse.is_contiguous() &&
                  lse.size(0) == B * H && lse.size(1) == sp, "attention: lse shape");
  auto dqkv = at::empty({B * S, 3 * H * DH}, qkv.options());
  hipStream_t st = at::hip::getCurrentHIPStream();
  if (g_attn_bwd_variant == 1) {
    if (g_num_cus_attn == 0) {
      int dev = 0;
      DMP_HIP_CHECK(hipGetDevice(&dev));
      DMP_HIP_CHECK(hipDeviceGetAttribute(&g_num_cus_attn, hipDeviceAttributeMultiprocessorCount, dev));
    }
    const int nbh = (int)(B * H);
    const int grid = std::min(nbh, 2 * g_num_cus_attn);
    DMP_ATTN_DISPATCH(sp, hipLaunchKernelGGL((attn_bwd_pp_kernel<SPC>), dim3(grid), dim3(kThreads), 0, st,
                                             (const bf16*)qkv.data_ptr(), qkv.stride(0),
                                             (const bf16*)dout.data_ptr(), dout.stride(0),
                                             (const bf16*)o.data_ptr(), o.stride(0), lse.data_ptr<float>(),
                                             (int)S, (int)H, (float)scale, (bf16*)dqkv.data_ptr(),
                                             dqkv.stride(0), nbh));
  } else {
    DMP_ATTN_DISPATCH(sp, hipLaunchKernelGGL((attn_bwd_kernel<SPC>), dim3(B * H), dim3(kThreads), 0, st,
                                             (const bf16*)qkv.data_ptr(), qkv.stride(0),
                                             (const bf16*)dout.data_ptr(), dout.stride(0),
                                             (const bf16*)o.data_ptr(), o.stride(0), lse.data_ptr<float>(),
                                             (int)S, (int)H, (float)scale, (bf16*)dqkv.data_ptr(),
                                             dqkv.stride(0)));
  }
  DMP_HIP_CHECK(hipGetLastError());
  return dqkv;
}

}  // namespace dmp
