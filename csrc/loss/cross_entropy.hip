// Fused softmax cross-entropy (mean reduction, ignore_index) for [B, C] logits
// in bf16 or fp32 ("CrossEntropyLoss -> fused log-softmax +
// NLL"; reference criterion nn.CrossEntropyLoss at model_parallel.py:106,147,
// data_parallel.py:89).
//
// One wave64 per row: the row is streamed once for the max and once for the
// exp-sum (row length 10..1000 stays in L2 between the passes), the wave
// reduces with DPP shuffles, lane 0 writes (loss_i, lse_i).  The backward
// recomputes softmax from the saved lse and writes dlogits in the logits'
// dtype directly:  dx = (exp(x - lse) - onehot(t)) * g / n_valid  -- one pass,
// instead of cast + log_softmax + nll (+ their three backward kernels).
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include "../common.h"

namespace dmp {
namespace {

constexpr int kRowsPerBlock = 4;  // 4 waves, one row each

template <typename T>
__device__ __forceinline__ float ld(const T* p) { return (float)*p; }

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
  return v;
}

template <typename T>
__global__ __launch_bounds__(64 * kRowsPerBlock) void ce_fwd_kernel(
    const T* __restrict__ x, int64_t ldx, const int64_t* __restrict__ tgt, int B, int C,
    int64_t ignore_index, float* __restrict__ row_loss, float* __restrict__ lse_out,
    int* __restrict__ rank_out) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  if (row >= B) return;
  const T* xr = x + (int64_t)row * ldx;
  float m = -INFINITY;
  for (int c = lane; c < C; c += 64) m = fmaxf(m, ld(xr + c));
  m = wave_max(m);
  float s = 0.f;
  for (int c = lane; c < C; c += 64) s += __expf(ld(xr + c) - m);
  s = wave_sum(s);
  const int64_t t = tgt[row];
  if (rank_out) {
    // the target's rank: classes ahead of it in a stable descending sort
    // (greater logit, or equal logit at a lower index); top-k correct <=> rank < k
    const bool ok = t >= 0 && t < C;
    const float xt = ok ? ld(xr + t) : 0.f;
    int r = 0;
    for (int c = lane; c < C; c += 64) {
      const float v = ld(xr + c);
      r += (v > xt || (v == xt && c < t)) ? 1 : 0;
    }
    r = (int)wave_sum((float)r);
    if (lane == 0) rank_out[row] = ok ? r : C;
  }
  if (lane == 0) {
    const float lse = m + __logf(s);
    const bool valid = t != ignore_index;
    // a label outside [0, C) (class-count / dataset mismatch) must not read
    // past the row: it poisons the loss and this row's gradient with NaN
    // instead (F.cross_entropy raises; a device-side NaN is visible in the
    // very next loss.item() without a host sync here)
    const bool in_range = t >= 0 && t < C;
    row_loss[row] = !valid ? 0.f : in_range ? lse - ld(xr + t) : NAN;
    lse_out[row] = (valid && !in_range) ? NAN : lse;
  }
}

// loss = scale * sum(row_loss) / n_valid (also writes n_valid and scale for
// the backward); one block.  With ranks: also the top-1 / top-k (k = kmax)
// correct counts, and with acc (fp64 [3]) acc += (loss, top1, top-k) -- a
// pipeline micro-batch's statistics without a topk / sort / cast kernel chain.
__global__ __launch_bounds__(256) void ce_reduce_kernel(const float* __restrict__ row_loss,
                                                        const int64_t* __restrict__ tgt, int B,
                                                        int64_t ignore_index, float* __restrict__ out,
                                                        float scale, const int* __restrict__ rank,
                                                        int kmax, double* __restrict__ acc) {
  float s = 0.f, n = 0.f, c1 = 0.f, ck = 0.f;
  for (int i = threadIdx.x; i < B; i += 256) {
    s += row_loss[i];
    n += tgt[i] != ignore_index ? 1.f : 0.f;
    if (rank) {
      c1 += rank[i] < 1 ? 1.f : 0.f;
      ck += rank[i] < kmax ? 1.f : 0.f;
    }
  }
  s = wave_sum(s);
  n = wave_sum(n);
  c1 = wave_sum(c1);
  ck = wave_sum(ck);
  __shared__ float rs[4], rn[4], r1[4], rk[4];
  if ((threadIdx.x & 63) == 0) {
    rs[threadIdx.x >> 6] = s;
    rn[threadIdx.x >> 6] = n;
    r1[threadIdx.x >> 6] = c1;
    rk[threadIdx.x >> 6] = ck;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float S = rs[0] + rs[1] + rs[2] + rs[3], N = rn[0] + rn[1] + rn[2] + rn[3];
    const float L = N > 0.f ? S / N * scale : NAN;  // torch: mean over zero valid rows is nan
    out[0] = L;
    out[1] = N;
    out[2] = scale;
    if (acc) {
      acc[0] += (double)L;
      acc[1] += (double)(r1[0] + r1[1] + r1[2] + r1[3]);
      acc[2] += (double)(rk[0] + rk[1] + rk[2] + rk[3]);
    }
  }
}

template <typename T>
__global__ __launch_bounds__(64 * kRowsPerBlock) void ce_bwd_kernel(
    const T* __restrict__ x, int64_t ldx, const int64_t* __restrict__ tgt, const float* __restrict__ lse,
    const float* __restrict__ gout, const float* __restrict__ stats, int B, int C,
    int64_t ignore_index, T* __restrict__ dx) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  if (row >= B) return;
  const T* xr = x + (int64_t)row * ldx;
  T* dr = dx + (int64_t)row * C;
  const int64_t t = tgt[row];
  const float n = stats[1];
  const bool bad = t != ignore_index && (t < 0 || t >= C);  // NaN lse: gradient is NaN too
  const float scale = (t == ignore_index || n == 0.f) ? 0.f : bad ? NAN : gout[0] * stats[2] / n;
  const float l = lse[row];
  for (int c = lane; c < C; c += 64) {
    const float p = __expf(ld(xr + c) - l);
    dr[c] = (T)((p - (c == t ? 1.f : 0.f)) * scale);
  }
}

}  // namespace

// Returns (loss [1] fp32, lse [B] fp32, stats [3] fp32 = (loss, n_valid, scale)).
// loss = scale * mean cross-entropy.  acc (fp64 [3], optional): acc += (loss,
// top-1 correct, top-min(5, C) correct).
std::vector<at::Tensor> cross_entropy_fwd(const at::Tensor& x, const at::Tensor& target,
                                          int64_t ignore_index, double scale,
                                          const c10::optional<at::Tensor>& acc) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 2 && x.stride(1) == 1, "logits must be a row-major [B, C] GPU tensor");
  TORCH_CHECK(x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16, "logits must be fp32 or bf16");
  TORCH_CHECK(target.is_cuda() && target.scalar_type() == at::kLong && target.dim() == 1 &&
                  target.size(0) == x.size(0) && target.is_contiguous(),
              "target must be a contiguous int64 [B] GPU tensor");
  const int B = (int)x.size(0), C = (int)x.size(1);
  auto fo = x.options().dtype(at::kFloat);
  const bool want = acc.has_value() && acc->defined();
  if (want)
    TORCH_CHECK(acc->is_cuda() && acc->scalar_type() == at::kDouble && acc->numel() == 3 && acc->is_contiguous(),
                "cross_entropy_fwd: acc must be a contiguous fp64 [3] GPU tensor");
  auto row_loss = at::empty({B}, fo), lse = at::empty({B}, fo), stats = at::empty({3}, fo);
  at::Tensor rank;
  if (want) rank = at::empty({std::max(B, 1)}, x.options().dtype(at::kInt));
  int* rp = want ? rank.data_ptr<int>() : nullptr;
  auto stream = at::hip::getCurrentHIPStream();
  const int blocks = (B + kRowsPerBlock - 1) / kRowsPerBlock;
  if (B > 0) {
    if (x.scalar_type() == at::kFloat)
      hipLaunchKernelGGL(ce_fwd_kernel<float>, dim3(blocks), dim3(64 * kRowsPerBlock), 0, stream,
                         x.data_ptr<float>(), x.stride(0), target.data_ptr<int64_t>(), B, C, ignore_index,
                         row_loss.data_ptr<float>(), lse.data_ptr<float>(), rp);
    else
      hipLaunchKernelGGL(ce_fwd_kernel<__bf16>, dim3(blocks), dim3(64 * kRowsPerBlock), 0, stream,
                         reinterpret_cast<const __bf16*>(x.data_ptr()), x.stride(0),
                         target.data_ptr<int64_t>(), B, C, ignore_index, row_loss.data_ptr<float>(),
                         lse.data_ptr<float>(), rp);
  }
  hipLaunchKernelGGL(ce_reduce_kernel, dim3(1), dim3(256), 0, stream, row_loss.data_ptr<float>(),
                     target.data_ptr<int64_t>(), B, ignore_index, stats.data_ptr<float>(), (float)scale,
                     B > 0 ? rp : nullptr, std::min(5, C), want ? acc->data_ptr<double>() : nullptr);
  DMP_HIP_CHECK(hipGetLastError());
  return {stats.select(0, 0), lse, stats};  // 0-d view of the loss
}

at::Tensor cross_entropy_bwd(const at::Tensor& grad, const at::Tensor& x, const at::Tensor& target,
                             const at::Tensor& lse, const at::Tensor& stats, int64_t ignore_index) {
  const int B = (int)x.size(0), C = (int)x.size(1);
  auto g = grad.to(at::kFloat).contiguous();
  auto dx = at::empty({B, C}, x.options());
  if (B == 0) return dx;
  auto stream = at::hip::getCurrentHIPStream();
  const int blocks = (B + kRowsPerBlock - 1) / kRowsPerBlock;
  if (x.scalar_type() == at::kFloat)
    hipLaunchKernelGGL(ce_bwd_kernel<float>, dim3(blocks), dim3(64 * kRowsPerBlock), 0, stream,
                       x.data_ptr<float>(), x.stride(0), target.data_ptr<int64_t>(), lse.data_ptr<float>(),
                       g.data_ptr<float>(), stats.data_ptr<float>(), B, C, ignore_index, dx.data_ptr<float>());
  else
    hipLaunchKernelGGL(ce_bwd_kernel<__bf16>, dim3(blocks), dim3(64 * kRowsPerBlock), 0, stream,
                       reinterpret_cast<const __bf16*>(x.data_ptr()), x.stride(0), target.data_ptr<int64_t>(),
                       lse.data_ptr<float>(), g.data_ptr<float>(), stats.data_ptr<float>(), B, C,
                       ignore_index, reinterpret_cast<__bf16*>(dx.data_ptr()));
  DMP_HIP_CHECK(hipGetLastError());
  return dx;
}

}  // namespace dmp
