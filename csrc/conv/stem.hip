// ResNet stem (7x7 / stride 2 / pad 3 on 3 channels) re-cast for the MFMA
// implicit GEMM: space-to-depth by 2 turns it into a 4x4 / stride-1 / pad-0
// conv on 12 channels (padded to 16, so a pixel is 32 B and four adjacent
// pixels are one 64-channel "row tap" of conv_nt's kc override):
//   s[n, i, j, (dy*2 + dx)*3 + c] = x[n, 2i + dy - pad, 2j + dx - pad, c]   (0 outside)
//   y[n, oh, ow] = sum_{r, q < 4} s[n, oh + r, ow + q, :] . W'[r, q, :]
//   W'[r, q, (dy*2 + dx)*3 + c] = W[2r + dy, 2q + dx, c]   (0 for 2r+dy or 2q+dx = 7)
// With Cin = 3 MIOpen's direct / implicit-GEMM kernels run the 7x7 at ~140
// TF/s (profiles/conv_roofline_r2.md); the image itself needs no gradient.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include "../common.h"

namespace dmp {
namespace {

// one thread per output pixel: 2x2 input pixels x 3 channels -> 16 bf16 (2 x 16 B)
__global__ __launch_bounds__(256) void s2d_kernel(const __bf16* __restrict__ x, int64_t N, int H, int W,
                                                  int Hs, int Ws, int pad, __bf16* __restrict__ out) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = N * Hs * Ws;
  if (p >= total) return;
  const int j = (int)(p % Ws);
  const int64_t t = p / Ws;
  const int i = (int)(t % Hs);
  const int64_t n = t / Hs;
  float v[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) v[q] = 0.f;
#pragma unroll
  for (int dy = 0; dy < 2; ++dy) {
    const int h = 2 * i + dy - pad;
#pragma unroll
    for (int dx = 0; dx < 2; ++dx) {
      const int w = 2 * j + dx - pad;
      if ((unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W) {
        const __bf16* px = x + ((n * H + h) * W + w) * 3;
#pragma unroll
        for (int c = 0; c < 3; ++c) v[(dy * 2 + dx) * 3 + c] = (float)px[c];
      }
    }
  }
  __bf16* o = out + p * 16;
  float lo[8], hi[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) { lo[q] = v[q]; hi[q] = v[8 + q]; }
  Vec16<__bf16>::store(o, lo);
  Vec16<__bf16>::store(o + 8, hi);
}

// one thread per output pixel: copy C <= 16 channels, zero the rest / the border
__global__ __launch_bounds__(256) void pad16_kernel(const __bf16* __restrict__ x, int64_t N, int C, int H, int W,
                                                    int Hp, int Wp, int pad, __bf16* __restrict__ out) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = N * Hp * Wp;
  if (p >= total) return;
  const int j = (int)(p % Wp);
  const int64_t t = p / Wp;
  const int i = (int)(t % Hp);
  const int64_t n = t / Hp;
  float v[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) v[q] = 0.f;
  const int h = i - pad, w = j - pad;
  if ((unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W) {
    const __bf16* px = x + ((n * H + h) * W + w) * C;
    for (int c = 0; c < C; ++c) v[c] = (float)px[c];
  }
  __bf16* o = out + p * 16;
  float lo[8], hi[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) { lo[q] = v[q]; hi[q] = v[8 + q]; }
  Vec16<__bf16>::store(o, lo);
  Vec16<__bf16>::store(o + 8, hi);
}

}  // namespace

// x: [N, C <= 16, H, W] bf16 channels_last -> [N, 16, H + 2 pad, W + 2 pad + extra_w]
// zero-padded (channels and border): the input of a stride-1 few-channel conv run
// as 64-channel row taps (conv_nt kc=64 reads 4 adjacent 16-channel pixels).
at::Tensor pad_channels16(const at::Tensor& x, int64_t pad, int64_t extra_w) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4 && x.size(1) <= 16 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "pad_channels16 expects a channels_last bf16 [N, C<=16, H, W] GPU tensor");
  const int64_t N = x.size(0);
  const int C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  const int Hp = H + 2 * (int)pad, Wp = W + 2 * (int)pad + (int)extra_w;
  auto out = at::empty({N, 16, Hp, Wp}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int64_t total = N * Hp * Wp;
  if (total == 0) return out;
  hipLaunchKernelGGL(pad16_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     at::hip::getCurrentHIPStream(), reinterpret_cast<const __bf16*>(x.data_ptr()), N, C, H, W,
                     Hp, Wp, (int)pad, reinterpret_cast<__bf16*>(out.data_ptr()));
  DMP_HIP_CHECK(hipGetLastError());
  return out;
}

// x: [N, 3, H, W] bf16 channels_last -> [N, 16, Hs, Ws] bf16 channels_last,
// Hs = (H + 2 pad + 1) / 2 (the padded image is cut into 2x2 blocks).
at::Tensor space_to_depth2(const at::Tensor& x, int64_t pad, int64_t out_channels) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4 && x.size(1) == 3 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "space_to_depth2 expects a channels_last bf16 [N, 3, H, W] GPU tensor");
  TORCH_CHECK(out_channels == 16, "space_to_depth2 writes 16 channels (12 used)");
  const int64_t N = x.size(0);
  const int H = (int)x.size(2), W = (int)x.size(3);
  const int Hs = (H + 2 * (int)pad + 1) / 2, Ws = (W + 2 * (int)pad + 1) / 2;
  auto out = at::empty({N, 16, Hs, Ws}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int64_t total = N * Hs * Ws;
  if (total == 0) return out;
  hipLaunchKernelGGL(s2d_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     at::hip::getCurrentHIPStream(), reinterpret_cast<const __bf16*>(x.data_ptr()), N, H, W,
                     Hs, Ws, (int)pad, reinterpret_cast<__bf16*>(out.data_ptr()));
  DMP_HIP_CHECK(hipGetLastError());
  return out;
}

}  // namespace dmp
