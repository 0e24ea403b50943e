// Channels-last (NHWC) max pooling for gfx950: the ResNet stem's 3x3/s2/p1
// pool (any k, s, p) without PyTorch's int64 index tensor.
//
// PyTorch's NHWC max_pool2d_with_indices writes an int64 argmax per output
// element (822 MB at ResNet-50 batch 256) and its backward scatters through
// it: 0.25 ms forward + 0.62 ms backward on MI355X (profiles/r50_*_v5.md).
// Here:
//   forward : one lane = one output pixel x one 16-B channel vector; the k*k
//             window is read as 16-B vectors (neighbouring lanes share input
//             lines in L2) and the winning tap per channel is stored as ONE
//             byte (k*k <= 255), 1/8 of the int64 index traffic.
//   backward: a GATHER per input pixel (no atomics, no zero-fill pass): the
//             <= ceil(k/s)^2 windows that contain it are enumerated, their
//             argmax bytes compared with the pixel's tap id, matching dy
//             summed -- every dx element written exactly once.
// Tie-breaking matches PyTorch (first maximum in window order; NaN wins).
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include "../common.h"

namespace dmp {
namespace {

struct PoolGeo {
  int N, C, H, W, Ho, Wo, k, s, p, cv;  // cv = C / VEC
};

template <typename T>
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                          uint8_t* __restrict__ idx, PoolGeo g,
                                                          int64_t total) {
  constexpr int VEC = Vec16<T>::N;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int cvi = (int)(i % g.cv);
  const int64_t pix = i / g.cv;
  const int ow = (int)(pix % g.Wo);
  const int64_t t = pix / g.Wo;
  const int oh = (int)(t % g.Ho);
  const int n = (int)(t / g.Ho);
  const int c0 = cvi * VEC;
  float m[VEC];
  uint8_t am[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) { m[j] = -INFINITY; am[j] = 0; }
  const int h0 = oh * g.s - g.p, w0 = ow * g.s - g.p;
  for (int a = 0; a < g.k; ++a) {
    const int ih = h0 + a;
    if (ih < 0 || ih >= g.H) continue;
    for (int b = 0; b < g.k; ++b) {
      const int iw = w0 + b;
      if (iw < 0 || iw >= g.W) continue;
      float v[VEC];
      Vec16<T>::load(x + (((int64_t)n * g.H + ih) * g.W + iw) * g.C + c0, v);
      const uint8_t tap = (uint8_t)(a * g.k + b);
#pragma unroll
      for (int j = 0; j < VEC; ++j)
        if (v[j] > m[j] || (v[j] != v[j] && m[j] == m[j])) { m[j] = v[j]; am[j] = tap; }
    }
  }
  Vec16<T>::store(y + pix * g.C + c0, m);
  uint8_t* ip = idx + pix * g.C + c0;
#pragma unroll
  for (int j = 0; j < VEC; ++j) ip[j] = am[j];
}

template <typename T>
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const T* __restrict__ dy,
                                                          const uint8_t* __restrict__ idx,
                                                          T* __restrict__ dx, PoolGeo g,
                                                          int64_t total) {
  constexpr int VEC = Vec16<T>::N;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int cvi = (int)(i % g.cv);
  const int64_t pix = i / g.cv;
  const int iw = (int)(pix % g.W);
  const int64_t t = pix / g.W;
  const int ih = (int)(t % g.H);
  const int n = (int)(t / g.H);
  const int c0 = cvi * VEC;
  float acc[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) acc[j] = 0.f;
  // windows oh with oh*s - p <= ih <= oh*s - p + k - 1
  const int oh_lo = max(0, (ih + g.p - g.k + g.s) / g.s), oh_hi = min(g.Ho - 1, (ih + g.p) / g.s);
  const int ow_lo = max(0, (iw + g.p - g.k + g.s) / g.s), ow_hi = min(g.Wo - 1, (iw + g.p) / g.s);
  for (int oh = oh_lo; oh <= oh_hi; ++oh) {
    const int a = ih - (oh * g.s - g.p);
    if (a < 0 || a >= g.k) continue;
    for (int ow = ow_lo; ow <= ow_hi; ++ow) {
      const int b = iw - (ow * g.s - g.p);
      if (b < 0 || b >= g.k) continue;
      const uint8_t tap = (uint8_t)(a * g.k + b);
      const int64_t o = (((int64_t)n * g.Ho + oh) * g.Wo + ow) * g.C + c0;
      uint8_t am[VEC];
      if constexpr (VEC == 8) {
        const uint64_t w = *reinterpret_cast<const uint64_t*>(idx + o);
#pragma unroll
        for (int j = 0; j < 8; ++j) am[j] = (uint8_t)(w >> (8 * j));
      } else {
        const uint32_t w = *reinterpret_cast<const uint32_t*>(idx + o);
#pragma unroll
        for (int j = 0; j < 4; ++j) am[j] = (uint8_t)(w >> (8 * j));
      }
      bool any = false;
#pragma unroll
      for (int j = 0; j < VEC; ++j) any |= am[j] == tap;
      if (!any) continue;
      float v[VEC];
      Vec16<T>::load(dy + o, v);
#pragma unroll
      for (int j = 0; j < VEC; ++j)
        if (am[j] == tap) acc[j] += v[j];
    }
  }
  Vec16<T>::store(dx + pix * g.C + c0, acc);
}

PoolGeo make_geo(const at::Tensor& x, int64_t k, int64_t s, int64_t p, int vec) {
  PoolGeo g;
  g.N = (int)x.size(0); g.C = (int)x.size(1); g.H = (int)x.size(2); g.W = (int)x.size(3);
  g.k = (int)k; g.s = (int)s; g.p = (int)p;
  g.Ho = (g.H + 2 * g.p - g.k) / g.s + 1;
  g.Wo = (g.W + 2 * g.p - g.k) / g.s + 1;
  g.cv = g.C / vec;
  return g;
}

void check_x(const at::Tensor& x, const char* name) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 4, name, " must be a 4-D GPU tensor");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kFloat,
              name, " must be bf16 or fp32");
  TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast), name, " must be channels_last");
  const int vec = x.scalar_type() == at::kBFloat16 ? 8 : 4;
  TORCH_CHECK(x.size(1) % vec == 0, name, ": channels must be a multiple of ", vec);
}

}  // namespace

// Returns (y, argmax-tap bytes [N, Ho, Wo, C] uint8).
std::vector<at::Tensor> maxpool2d_forward(const at::Tensor& x, int64_t k, int64_t s, int64_t p) {
  check_x(x, "x");
  TORCH_CHECK(k >= 1 && k * k <= 255 && s >= 1 && p >= 0 && 2 * p <= k, "unsupported pool geometry");
  const int vec = x.scalar_type() == at::kBFloat16 ? 8 : 4;
  PoolGeo g = make_geo(x, k, s, p, vec);
  TORCH_CHECK(g.Ho > 0 && g.Wo > 0, "pool output is empty");
  auto y = at::empty({g.N, g.C, g.Ho, g.Wo}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto idx = at::empty({(int64_t)g.N * g.Ho * g.Wo * g.C}, x.options().dtype(at::kByte));
  const int64_t total = (int64_t)g.N * g.Ho * g.Wo * g.cv;
  if (total == 0) return {y, idx};
  auto stream = at::hip::getCurrentHIPStream();
  const unsigned blocks = (unsigned)((total + 255) / 256);
  if (x.scalar_type() == at::kBFloat16)
    hipLaunchKernelGGL(maxpool_fwd_kernel<__bf16>, dim3(blocks), dim3(256), 0, stream,
                       reinterpret_cast<const __bf16*>(x.data_ptr()), reinterpret_cast<__bf16*>(y.data_ptr()),
                       idx.data_ptr<uint8_t>(), g, total);
  else
    hipLaunchKernelGGL(maxpool_fwd_kernel<float>, dim3(blocks), dim3(256), 0, stream,
                       x.data_ptr<float>(), y.data_ptr<float>(), idx.data_ptr<uint8_t>(), g, total);
  return {y, idx};
}

at::Tensor maxpool2d_backward(const at::Tensor& dy, const at::Tensor& idx, int64_t H, int64_t W,
                              int64_t k, int64_t s, int64_t p) {
  check_x(dy, "dy");
  const int vec = dy.scalar_type() == at::kBFloat16 ? 8 : 4;
  PoolGeo g;
  g.N = (int)dy.size(0); g.C = (int)dy.size(1); g.H = (int)H; g.W = (int)W;
  g.k = (int)k; g.s = (int)s; g.p = (int)p;
  g.Ho = (int)dy.size(2); g.Wo = (int)dy.size(3);
  g.cv = g.C / vec;
  TORCH_CHECK(g.Ho == (g.H + 2 * g.p - g.k) / g.s + 1 && g.Wo == (g.W + 2 * g.p - g.k) / g.s + 1,
              "dy does not match the pool geometry");
  TORCH_CHECK(idx.numel() == dy.numel() && idx.scalar_type() == at::kByte, "bad argmax tensor");
  auto dx = at::empty({g.N, g.C, g.H, g.W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int64_t total = (int64_t)g.N * g.H * g.W * g.cv;
  if (total == 0) return dx;
  auto stream = at::hip::getCurrentHIPStream();
  const unsigned blocks = (unsigned)((total + 255) / 256);
  if (dy.scalar_type() == at::kBFloat16)
    hipLaunchKernelGGL(maxpool_bwd_kernel<__bf16>, dim3(blocks), dim3(256), 0, stream,
                       reinterpret_cast<const __bf16*>(dy.data_ptr()), idx.data_ptr<uint8_t>(),
                       reinterpret_cast<__bf16*>(dx.data_ptr()), g, total);
  else
    hipLaunchKernelGGL(maxpool_bwd_kernel<float>, dim3(blocks), dim3(256), 0, stream,
                       dy.data_ptr<float>(), idx.data_ptr<uint8_t>(), dx.data_ptr<float>(), g, total);
  return dx;
}

}  // namespace dmp
