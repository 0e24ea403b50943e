// Single-launch SGD(momentum, weight decay, nesterov) over a FLAT parameter
// buffer: the whole model's parameters of one dtype live in one contiguous
// allocation laid out exactly like the DDP gradient buckets, so one kernel
// updates every parameter (ResNet-50: 25.6 M elements, ~1 launch instead of
// 161 per-tensor launches).  For bf16 models the kernel keeps fp32 master
// weights and momentum, reads the (already RCCL-averaged) bf16 gradient and
// writes the bf16 working copy back in the same pass -- no separate cast.
//
// Parity: the reference's optimizer is torch.optim.SGD(lr, momentum=0.9,
// weight_decay=1e-4) (model_parallel.py:105, data_parallel.py:90).
// Semantics match torch.optim.SGD exactly (first step seeds the buffer with
// the gradient, dampening applies from the second step on).
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include "../common.h"

namespace dmp {
namespace {

template <typename G, typename P, bool MASTER>
__global__ __launch_bounds__(256) void sgd_flat_kernel(
    float* __restrict__ master, float* __restrict__ mom, const G* __restrict__ grad,
    P* __restrict__ param, int64_t n, float lr, float wd, float momentum, float dampening,
    int nesterov, float grad_scale, int first_step) {
  // 8 elements per lane per iteration: bf16 grads/params = 16 B, fp32 = 2 x 16 B.
  const int64_t nvec = n / 8;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    const int64_t o = v * 8;
    float g[8], w[8], m[8];
    if constexpr (sizeof(G) == 2) {
      Vec16<__bf16>::load(reinterpret_cast<const __bf16*>(grad) + o, g);
    } else {
      float a[4], b[4];
      Vec16<float>::load(reinterpret_cast<const float*>(grad) + o, a);
      Vec16<float>::load(reinterpret_cast<const float*>(grad) + o + 4, b);
#pragma unroll
      for (int i = 0; i < 4; ++i) { g[i] = a[i]; g[4 + i] = b[i]; }
    }
    {
      float a[4], b[4];
      const float* wp = MASTER ? master : reinterpret_cast<const float*>(param);
      Vec16<float>::load(wp + o, a);
      Vec16<float>::load(wp + o + 4, b);
#pragma unroll
      for (int i = 0; i < 4; ++i) { w[i] = a[i]; w[4 + i] = b[i]; }
    }
    if (momentum != 0.f && !first_step) {
      float a[4], b[4];
      Vec16<float>::load(mom + o, a);
      Vec16<float>::load(mom + o + 4, b);
#pragma unroll
      for (int i = 0; i < 4; ++i) { m[i] = a[i]; m[4 + i] = b[i]; }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float d = fmaf(wd, w[i], g[i] * grad_scale);
      if (momentum != 0.f) {
        m[i] = first_step ? d : fmaf(momentum, m[i], (1.f - dampening) * d);
        d = nesterov ? fmaf(momentum, m[i], d) : m[i];
      }
      w[i] = fmaf(-lr, d, w[i]);
    }
    if (momentum != 0.f) {
      float a[4] = {m[0], m[1], m[2], m[3]}, b[4] = {m[4], m[5], m[6], m[7]};
      Vec16<float>::store(mom + o, a);
      Vec16<float>::store(mom + o + 4, b);
    }
    if (MASTER) {
      float a[4] = {w[0], w[1], w[2], w[3]}, b[4] = {w[4], w[5], w[6], w[7]};
      Vec16<float>::store(master + o, a);
      Vec16<float>::store(master + o + 4, b);
    }
    if constexpr (sizeof(P) == 2) {
      Vec16<__bf16>::store(reinterpret_cast<__bf16*>(param) + o, w);
    } else {
      float a[4] = {w[0], w[1], w[2], w[3]}, b[4] = {w[4], w[5], w[6], w[7]};
      Vec16<float>::store(reinterpret_cast<float*>(param) + o, a);
      Vec16<float>::store(reinterpret_cast<float*>(param) + o + 4, b);
    }
  }
}

}  // namespace

// master: fp32 flat (or undefined when `param` is fp32 and is its own master)
// mom:    fp32 flat momentum buffer (ignored when momentum == 0)
// grad:   flat gradient (bf16 or fp32), param: flat parameters (bf16 or fp32)
// numel must be a multiple of 8 (bucket layouts are padded to 16 B).
void sgd_flat_step(const c10::optional<at::Tensor>& master, const at::Tensor& mom,
                   const at::Tensor& grad, const at::Tensor& param, double lr, double wd,
                   double momentum, double dampening, bool nesterov, double grad_scale,
                   bool first_step) {
  const int64_t n = param.numel();
  TORCH_CHECK(grad.numel() == n, "grad/param size mismatch");
  TORCH_CHECK(n % 8 == 0, "flat buffers must be padded to a multiple of 8 elements");
  TORCH_CHECK(param.is_contiguous() && grad.is_contiguous(), "flat buffers must be contiguous");
  const bool has_master = master.has_value() && master->defined();
  TORCH_CHECK(has_master || param.scalar_type() == at::kFloat,
              "bf16 parameters need an fp32 master buffer");
  if (n == 0) return;
  auto stream = at::hip::getCurrentHIPStream();
  const int64_t nvec = n / 8;
  const int threads = 256;
  const int64_t blocks = std::min<int64_t>((nvec + threads - 1) / threads, 256 * 8);
  float* mp = has_master ? master->data_ptr<float>() : nullptr;
  float* mo = momentum != 0.0 ? mom.data_ptr<float>() : nullptr;
  auto launch = [&](auto gtag, auto ptag) {
    using G = decltype(gtag);
    using P = decltype(ptag);
    const G* gp = reinterpret_cast<const G*>(grad.data_ptr());
    P* pp = reinterpret_cast<P*>(param.data_ptr());
    if (has_master)
      hipLaunchKernelGGL((sgd_flat_kernel<G, P, true>), dim3(blocks), dim3(threads), 0, stream, mp,
                         mo, gp, pp, n, (float)lr, (float)wd, (float)momentum, (float)dampening,
                         (int)nesterov, (float)grad_scale, (int)first_step);
    else
      hipLaunchKernelGGL((sgd_flat_kernel<G, P, false>), dim3(blocks), dim3(threads), 0, stream, mp,
                         mo, gp, pp, n, (float)lr, (float)wd, (float)momentum, (float)dampening,
                         (int)nesterov, (float)grad_scale, (int)first_step);
  };
  const bool gb = grad.scalar_type() == at::kBFloat16, pb = param.scalar_type() == at::kBFloat16;
  if (gb && pb) launch(__bf16{}, __bf16{});
  else if (gb) launch(__bf16{}, float{});
  else if (pb) launch(float{}, __bf16{});
  else launch(float{}, float{});
}

}  // namespace dmp
