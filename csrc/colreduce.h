// Deterministic second pass of the "per-block partial row" column reductions
// (LayerNorm dgamma/dbeta, Linear bias gradients): out[c] = sum_b part[b][c].
//
// The partial matrix is small (<= a few MB, L2-resident right after its
// producer) but tall (hundreds to ~1000 rows), so the pass is latency-bound:
// a block covers 8 columns x 32 row groups and every thread keeps 8
// independent loads in flight (an un-unrolled row loop measured 19-39 us per
// call, profiles/vit_b16_bs128_1gpu_v4.md).  Fixed summation order: bitwise
// reproducible run to run.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dmp {
namespace colreduce {

constexpr int kCols = 8, kGroups = 32, kThreads = kCols * kGroups, kInFlight = 8;

template <typename OT>
__global__ __launch_bounds__(kThreads) void partial_colsum_kernel(const float* __restrict__ part,
                                                                  int nb, int n,
                                                                  OT* __restrict__ out) {
  const int cl = threadIdx.x % kCols, g = threadIdx.x / kCols;
  const int c = blockIdx.x * kCols + cl;
  float acc[kInFlight];
#pragma unroll
  for (int u = 0; u < kInFlight; ++u) acc[u] = 0.f;
  if (c < n) {
    int b = g;
    for (; b + (kInFlight - 1) * kGroups < nb; b += kInFlight * kGroups) {
#pragma unroll
      for (int u = 0; u < kInFlight; ++u) acc[u] += part[(int64_t)(b + u * kGroups) * n + c];
    }
    for (; b < nb; b += kGroups) acc[0] += part[(int64_t)b * n + c];
  }
#pragma unroll
  for (int u = 1; u < kInFlight; ++u) acc[0] += acc[u];
  __shared__ float red[kThreads];
  red[threadIdx.x] = acc[0];
  __syncthreads();
  if (g == 0 && c < n) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < kGroups; ++q) t += red[q * kCols + cl];
    out[c] = (OT)t;
  }
}

template <typename OT>
inline void launch(const float* part, int nb, int n, OT* out, hipStream_t stream) {
  hipLaunchKernelGGL(partial_colsum_kernel<OT>, dim3((n + kCols - 1) / kCols), dim3(kThreads), 0,
                     stream, part, nb, n, out);
}

}  // namespace colreduce
}  // namespace dmp
