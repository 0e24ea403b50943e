// Linear-layer side passes for the ViT MLP / attention projections on gfx950:
// the bias gradient (column sum of dy over all tokens) and the GELU backward
// fused with it.
//
// Why (profiles/vit_b16_bs128_1gpu_v3.md): PyTorch-ROCm computes each
// nn.Linear bias gradient with a generic reduce kernel (52 calls, 1.77 ms per
// ViT-B/16 step, ~2.4 TB/s) and the GELU backward as a separate elementwise
// pass (12 calls, 1.04 ms) whose output the fc1 bias reduce then reads again.
// Here:
//   * colsum: dy [M, N] bf16 -> per-block fp32 partial rows -> one column
//     reduce launch; every wave streams whole rows with 8-row unrolled loads
//     in flight;
//   * gelu_bwd_colsum: dh = dy * gelu'(h) (exact erf GELU, as nn.GELU()) written
//     once, and its column sums (fc1's bias gradient) taken from registers.
// Block = 4 waves; blockIdx.x picks a window of 64*VW columns (lane -> VW
// consecutive columns), blockIdx.y a chunk of rows; the 4 waves interleave
// rows and fold through LDS into one partial row per block.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include "../colreduce.h"
#include "../common.h"

namespace dmp {
namespace {

constexpr int kThreads = 256;
constexpr int kUnroll = 8;

template <int VW> struct BVec;  // VW bf16 values <-> f32
template <> struct BVec<8> {
  using raw = bf16x8;
};
template <> struct BVec<4> {
  using raw = bf16x4;
};

template <int VW>
__device__ __forceinline__ void to_f32(const typename BVec<VW>::raw& r, float (&v)[VW]) {
#pragma unroll
  for (int i = 0; i < VW; ++i) v[i] = (float)r[i];
}

__device__ __forceinline__ float gelu_grad(float h) {
  // d/dh [0.5 h (1 + erf(h / sqrt2))] = 0.5 (1 + erf(h / sqrt2)) + h * phi(h)
  constexpr float kInvSqrt2 = 0.70710678118654752f, kInvSqrt2Pi = 0.39894228040143268f;
  return 0.5f * (1.f + erff(h * kInvSqrt2)) + h * kInvSqrt2Pi * __expf(-0.5f * h * h);
}

template <int VW, bool GELU>
__global__ __launch_bounds__(kThreads) void colsum_kernel(const __bf16* __restrict__ dy,
                                                          const __bf16* __restrict__ h,
                                                          __bf16* __restrict__ dh, int64_t M,
                                                          int N, int rows_per_block,
                                                          float* __restrict__ part) {
  using raw = typename BVec<VW>::raw;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int col = (blockIdx.x * 64 + lane) * VW;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_block;
  const int64_t r1 = r0 + rows_per_block < M ? r0 + rows_per_block : M;
  float acc[VW];
#pragma unroll
  for (int i = 0; i < VW; ++i) acc[i] = 0.f;
  if (col < N) {
    int64_t r = r0 + wid;
    for (; r + 4 * (kUnroll - 1) < r1; r += 4 * kUnroll) {
      raw a[kUnroll], b[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        a[u] = *reinterpret_cast<const raw*>(dy + (r + 4 * u) * N + col);
        if (GELU) b[u] = *reinterpret_cast<const raw*>(h + (r + 4 * u) * N + col);
      }
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        float g[VW];
        to_f32<VW>(a[u], g);
        if (GELU) {
          float hv[VW];
          to_f32<VW>(b[u], hv);
          raw o;
#pragma unroll
          for (int i = 0; i < VW; ++i) {
            g[i] *= gelu_grad(hv[i]);
            o[i] = (__bf16)g[i];
            g[i] = (float)o[i];  // sum what was stored: db == dh.sum(0) exactly
          }
          *reinterpret_cast<raw*>(dh + (r + 4 * u) * N + col) = o;
        }
#pragma unroll
        for (int i = 0; i < VW; ++i) acc[i] += g[i];
      }
    }
    for (; r < r1; r += 4) {
      float g[VW];
      to_f32<VW>(*reinterpret_cast<const raw*>(dy + r * N + col), g);
      if (GELU) {
        float hv[VW];
        to_f32<VW>(*reinterpret_cast<const raw*>(h + r * N + col), hv);
        raw o;
#pragma unroll
        for (int i = 0; i < VW; ++i) {
          g[i] *= gelu_grad(hv[i]);
          o[i] = (__bf16)g[i];
          g[i] = (float)o[i];
        }
        *reinterpret_cast<raw*>(dh + r * N + col) = o;
      }
#pragma unroll
      for (int i = 0; i < VW; ++i) acc[i] += g[i];
    }
  }
  __shared__ float red[kThreads / 64][64 * VW];
#pragma unroll
  for (int i = 0; i < VW; ++i) red[wid][lane * VW + i] = acc[i];
  __syncthreads();
  for (int e = threadIdx.x; e < 64 * VW; e += kThreads) {
    const int c = blockIdx.x * 64 * VW + e;
    if (c < N) {
      float s = 0.f;
#pragma unroll
      for (int q = 0; q < kThreads / 64; ++q) s += red[q][e];
      part[(int64_t)blockIdx.y * N + c] = s;
    }
  }
}


void launch_colsum(const at::Tensor& dy, const at::Tensor* h, at::Tensor* dh, at::Tensor& db) {
  const int64_t N = dy.size(-1), M = dy.numel() / N;
  const int VW = N % 512 == 0 ? 8 : 4;
  const int windows = (int)((N + 64 * VW - 1) / (64 * VW));
  // <= 256 row chunks (partial rows) per window, ~1024 blocks in total, at
  // least 4*kUnroll rows per block
  int chunks = (int)std::max<int64_t>(1, std::min<int64_t>(std::min(256, 1024 / windows), M / (4 * kUnroll)));
  const int rows_per_block = (int)((M + chunks - 1) / chunks);
  chunks = (int)((M + rows_per_block - 1) / rows_per_block);
  auto part = at::empty({chunks, N}, dy.options().dtype(at::kFloat));
  auto stream = at::hip::getCurrentHIPStream();
  const dim3 grid(windows, chunks);
  const __bf16* dyp = reinterpret_cast<const __bf16*>(dy.data_ptr());
  const __bf16* hp = h ? reinterpret_cast<const __bf16*>(h->data_ptr()) : nullptr;
  __bf16* dhp = dh ? reinterpret_cast<__bf16*>(dh->data_ptr()) : nullptr;
  if (M > 0) {
    if (VW == 8) {
      if (h) hipLaunchKernelGGL((colsum_kernel<8, true>), grid, dim3(kThreads), 0, stream, dyp, hp, dhp, M, (int)N, rows_per_block, part.data_ptr<float>());
      else hipLaunchKernelGGL((colsum_kernel<8, false>), grid, dim3(kThreads), 0, stream, dyp, hp, dhp, M, (int)N, rows_per_block, part.data_ptr<float>());
    } else {
      if (h) hipLaunchKernelGGL((colsum_kernel<4, true>), grid, dim3(kThreads), 0, stream, dyp, hp, dhp, M, (int)N, rows_per_block, part.data_ptr<float>());
      else hipLaunchKernelGGL((colsum_kernel<4, false>), grid, dim3(kThreads), 0, stream, dyp, hp, dhp, M, (int)N, rows_per_block, part.data_ptr<float>());
    }
  } else {
    part.zero_();
  }
  const int n = (int)N;
  if (db.scalar_type() == at::kBFloat16)
    colreduce::launch(part.data_ptr<float>(), chunks, n, reinterpret_cast<__bf16*>(db.data_ptr()), stream);
  else
    colreduce::launch(part.data_ptr<float>(), chunks, n, db.data_ptr<float>(), stream);
}

void check_2d(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.scalar_type() == at::kBFloat16, name,
              " must be a contiguous bf16 GPU tensor");
  TORCH_CHECK(t.dim() >= 1 && t.size(-1) % 256 == 0, name, ": last dim must be a multiple of 256");
}

}  // namespace

bool colsum_supported(int64_t N) { return N > 0 && N % 256 == 0; }

// Bias gradient: dy [..., N] bf16 -> sum over all leading dims, in out_dtype.
at::Tensor bias_grad(const at::Tensor& dy, at::ScalarType out_dtype) {
  check_2d(dy, "dy");
  auto db = at::empty({dy.size(-1)}, dy.options().dtype(out_dtype));
  launch_colsum(dy, nullptr, nullptr, db);
  return db;
}

// fc1 backward through GELU: returns (dh = dy * gelu'(h), db = dh.sum(leading dims)).
std::vector<at::Tensor> gelu_bwd_bias_grad(const at::Tensor& dy, const at::Tensor& h,
                                           at::ScalarType out_dtype) {
  check_2d(dy, "dy");
  check_2d(h, "h");
  TORCH_CHECK(dy.sizes() == h.sizes(), "dy / h shape mismatch");
  auto dh = at::empty_like(h);
  auto db = at::empty({dy.size(-1)}, dy.options().dtype(out_dtype));
  launch_colsum(dy, &h, &dh, db);
  return {dh, db};
}

}  // namespace dmp
