// Shared device helpers for the gfx950 (MI355X / CDNA4) kernels of this package.
//
// Conventions used by every kernel here:
//   * wave64: lane = threadIdx.x & 63, never & 31.
//   * memory-bound kernels move 16 bytes per lane per access (bf16x8 / f32x4),
//     which is the coalescing sweet spot on CDNA4 (1 KiB per wave instruction).
//   * bf16 <-> f32 conversions use clang's native __bf16, which hipcc lowers to
//     v_cvt_pk_bf16_f32 / shifts on gfx950 (round-to-nearest-even).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dmp {

using f32x4 = float __attribute__((ext_vector_type(4)));
using f32x8 = float __attribute__((ext_vector_type(8)));
using bf16x8 = __bf16 __attribute__((ext_vector_type(8)));
using bf16x4 = __bf16 __attribute__((ext_vector_type(4)));
using u32x4 = uint32_t __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;

// ---- 16-byte vector of "VEC" elements of type T, converted to/from f32 ----
template <typename T> struct Vec16;

template <> struct Vec16<float> {
  static constexpr int N = 4;
  using raw = f32x4;
  __device__ __forceinline__ static void load(const float* p, float (&v)[4]) {
    f32x4 r = *reinterpret_cast<const f32x4*>(p);
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = r[i];
  }
  __device__ __forceinline__ static void store(float* p, const float (&v)[4]) {
    f32x4 r;
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = v[i];
    *reinterpret_cast<f32x4*>(p) = r;
  }
};

template <> struct Vec16<__bf16> {
  static constexpr int N = 8;
  using raw = bf16x8;
  __device__ __forceinline__ static void load(const __bf16* p, float (&v)[8]) {
    bf16x8 r = *reinterpret_cast<const bf16x8*>(p);
    f32x8 f = __builtin_convertvector(r, f32x8);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = f[i];
  }
  __device__ __forceinline__ static void store(__bf16* p, const float (&v)[8]) {
    f32x8 f;
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] = v[i];
    *reinterpret_cast<bf16x8*>(p) = __builtin_convertvector(f, bf16x8);
  }
};

// Streaming (non-temporal) 16-B accesses for tensors touched exactly once per
// pass and far larger than the 256 MB Infinity Cache (BN apply passes over
// 0.4-1.6 GB activations): the nt policy keeps them from evicting reused lines.
template <bool NT, typename T>
__device__ __forceinline__ void ld16(const T* p, float (&v)[Vec16<T>::N]) {
  if constexpr (NT) {
    using R = typename Vec16<T>::raw;
    const R r = __builtin_nontemporal_load(reinterpret_cast<const R*>(p));
    if constexpr (Vec16<T>::N == 8) {
      const f32x8 f = __builtin_convertvector(r, f32x8);
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = f[i];
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = r[i];
    }
  } else {
    Vec16<T>::load(p, v);
  }
}

template <bool NT, typename T>
__device__ __forceinline__ void st16(T* p, const float (&v)[Vec16<T>::N]) {
  if constexpr (NT) {
    using R = typename Vec16<T>::raw;
    R r;
    if constexpr (Vec16<T>::N == 8) {
      f32x8 f;
#pragma unroll
      for (int i = 0; i < 8; ++i) f[i] = v[i];
      r = __builtin_convertvector(f, bf16x8);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) r[i] = v[i];
    }
    __builtin_nontemporal_store(r, reinterpret_cast<R*>(p));
  } else {
    Vec16<T>::store(p, v);
  }
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// ---- BN moments plumbing shared by every producer of [2][rb][C] partials ----
// bn_reduce_partials_launch (batchnorm.hip) folds the partial rows in chunks of
// kBnRedRows; with more than one chunk it accumulates into sums with fp64
// atomics, so sums[0:2C] must be zero first.  The PRODUCER kernel zeroes it
// (block 0, before the reduce launch in stream order) -- no memset launch.
constexpr int kBnRedRows = 256;
inline double* moments_zero_target(double* sums, int rb) { return rb > kBnRedRows ? sums : nullptr; }
__device__ __forceinline__ void zero_moments(double* z, int n) {
  if (z != nullptr && blockIdx.x == 0 && blockIdx.y == 0)
    for (int i = threadIdx.x; i < n; i += blockDim.x) z[i] = 0.0;
}

// A stride-s "compact" residual: it holds the values of the full-resolution
// row m = (n*hi + h)*wi + w only at (h, w) = (s*a, s*b) -- the data gradient
// of a stride-s 1x1 conv (a ResNet downsample), which is zero everywhere
// else.  compact_row returns that row of the compact tensor, or -1 (zero).
struct CompactMap {
  int s = 1, ho = 1, wo = 1, hi = 1, wi = 1;
};
__device__ __forceinline__ int64_t compact_row(const CompactMap& c, int64_t m) {
  if (c.s == 1) return m;
  const int64_t hw = (int64_t)c.hi * c.wi;
  const int64_t n = m / hw;
  const int r = (int)(m - n * hw);
  const int h = r / c.wi, w = r - h * c.wi;
  if (h % c.s != 0 || w % c.s != 0) return -1;
  return (n * c.ho + h / c.s) * c.wo + w / c.s;
}

// Bijective XCD-aware remap of a 1-D block id (cdna_hip_programming.md §5.5 T1):
// consecutive logical tiles land on the same XCD (same L2).
__device__ __forceinline__ int xcd_remap(int bid, int nblocks) {
  const int nxcd = 8;
  if (nblocks < nxcd) return bid;
  int q = nblocks / nxcd, r = nblocks % nxcd;
  int xcd = bid % nxcd, idx = bid / nxcd;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

}  // namespace dmp

#include "check.h"
