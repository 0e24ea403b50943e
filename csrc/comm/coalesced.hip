// Coalesced multi-tensor movement for DataParallel / DDP on MI355X.
//
// Parity targets (reference Readme.md:28-68 describes the
// upstream scatter / broadcast_coalesced(10 MiB buckets) / reduce_add /
// gather path that nn.DataParallel runs every iteration):
//   * multi_copy:   ONE launch moves many (src, dst) byte ranges -- flatten a
//                   parameter list into a bucket, unflatten a bucket into
//                   replica tensors, or copy a peer GPU's bucket over xGMI
//                   (src pointer on the peer, kernel on the destination, so
//                   each of the 7 links is driven by its own GPU).
//   * reduce_add:   out = sum_k in_k for up to 16 inputs that may live on
//                   peer GPUs (xGMI reads), vectorised 16 B per lane.
//   * gather_rows:  LDS-staged gather of N [rows_i, cols] slabs into one
//                   output along dim 0 or along the inner dim (dim != 0),
//                   where the output rows are strided and a direct copy would
//                   be uncoalesced on one side.
#include <torch/extension.h>
#include <mutex>
#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPCachingAllocator.h>
#include "../common.h"

namespace dmp {
namespace {

constexpr int64_t kChunkBytes = 64 * 1024;

// The copy table travels in the kernel arguments (no pinned-memory upload, no
// H2D copy: one launch is self-contained, and safe inside hipGraph capture).
// Up to kMaxCopy tensors per launch; block b copies 64 KiB chunk b of the
// concatenated byte stream and finds its tensor by binary search over the
// chunk prefix (scalar loads from the argument segment).
constexpr int kMaxCopy = 96;
struct CopyTable {
  const uint8_t* src[kMaxCopy];
  uint8_t* dst[kMaxCopy];
  int64_t nbytes[kMaxCopy];
  int first_chunk[kMaxCopy + 1];
  int n;
};

__device__ __forceinline__ void copy_range(const uint8_t* src, uint8_t* dst, int64_t nbytes) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst) |
                      (uintptr_t)nbytes;
  if ((a & 15) == 0) {
    const u32x4* s = reinterpret_cast<const u32x4*>(src);
    u32x4* d = reinterpret_cast<u32x4*>(dst);
    const int64_t n = nbytes >> 4;
    int64_t i = threadIdx.x;
    // 4 x 16 B in flight per lane.
    for (; i + 3 * 256 < n; i += 4 * 256) {
      u32x4 v0 = s[i], v1 = s[i + 256], v2 = s[i + 512], v3 = s[i + 768];
      d[i] = v0; d[i + 256] = v1; d[i + 512] = v2; d[i + 768] = v3;
    }
    for (; i < n; i += 256) d[i] = s[i];
  } else if ((a & 3) == 0) {
    const uint32_t* s = reinterpret_cast<const uint32_t*>(src);
    uint32_t* d = reinterpret_cast<uint32_t*>(dst);
    for (int64_t i = threadIdx.x; i < (nbytes >> 2); i += 256) d[i] = s[i];
  } else if ((a & 1) == 0) {
    const uint16_t* s = reinterpret_cast<const uint16_t*>(src);
    uint16_t* d = reinterpret_cast<uint16_t*>(dst);
    for (int64_t i = threadIdx.x; i < (nbytes >> 1); i += 256) d[i] = s[i];
  } else {
    for (int64_t i = threadIdx.x; i < nbytes; i += 256) dst[i] = src[i];
  }
}

__global__ __launch_bounds__(256) void multi_copy_kernel(const CopyTable t) {
  const int cid = blockIdx.x;
  int lo = 0, hi = t.n - 1;  // last entry with first_chunk <= cid
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (t.first_chunk[mid] <= cid) lo = mid;
    else hi = mid - 1;
  }
  const int64_t off = (int64_t)(cid - t.first_chunk[lo]) * kChunkBytes;
  if (off >= t.nbytes[lo]) return;
  copy_range(t.src[lo] + off, t.dst[lo] + off, min(kChunkBytes, t.nbytes[lo] - off));
}

// ---- multi_transpose: many 2-byte [R, C] -> [C, R] transposes in one launch ----
// (the W^T operands of a step's 1x1-conv data gradients, ops/wt_cache.py).
// One 256-thread block per 64 x 64 tile through LDS: loads coalesced along
// the source rows, stores along the destination rows.
// Tap-wise form (taps T > 1): src [R, T*C], dst [C, T*R], tap t of src
// (columns t*C..) transposed into tap t' of dst, t' = T-1-t when flipped --
// a channels-last kh x kw conv weight [Cout][kh][kw][Cin] becomes the
// flipped [Cin][kh][kw][Cout] matrix of its data gradient (conv_igemm).
constexpr int kMaxT = 64, kTT = 64;
struct TransTable {
  const uint16_t* src[kMaxT];
  uint16_t* dst[kMaxT];
  int rows[kMaxT], cols[kMaxT], taps[kMaxT], flip[kMaxT];
  int first_tile[kMaxT + 1];
  int n;
};

__global__ __launch_bounds__(256) void multi_transpose_kernel(const TransTable t) {
  const int bid = blockIdx.x;
  int lo = 0, hi = t.n - 1;  // last entry with first_tile <= bid
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (t.first_tile[mid] <= bid) lo = mid;
    else hi = mid - 1;
  }
  const int R = t.rows[lo], Cc = t.cols[lo], T = t.taps[lo];
  const int ctiles = (Cc + kTT - 1) / kTT, rtiles = (R + kTT - 1) / kTT;
  const int local0 = bid - t.first_tile[lo], tap = local0 / (rtiles * ctiles), local = local0 - tap * rtiles * ctiles;
  const int r0 = (local / ctiles) * kTT, c0 = (local % ctiles) * kTT;
  const int dtap = t.flip[lo] ? T - 1 - tap : tap;
  __shared__ uint16_t tile[kTT][kTT + 2];
  const uint16_t* s = t.src[lo] + (int64_t)tap * Cc;  // row stride T*C
  uint16_t* d = t.dst[lo] + (int64_t)dtap * R;        // row stride T*R
  const int64_t sld = (int64_t)T * Cc, dld = (int64_t)T * R;
#pragma unroll 4
  for (int i = threadIdx.x; i < kTT * kTT; i += 256) {
    const int r = i / kTT, c = i % kTT;
    if (r0 + r < R && c0 + c < Cc) tile[r][c] = s[(int64_t)(r0 + r) * sld + c0 + c];
  }
  __syncthreads();
#pragma unroll 4
  for (int i = threadIdx.x; i < kTT * kTT; i += 256) {
    const int c = i / kTT, r = i % kTT;
    if (r0 + r < R && c0 + c < Cc) d[(int64_t)(c0 + c) * dld + r0 + r] = tile[r][c];
  }
}


// ---- multi_cast: many bf16 -> fp32 casts in one launch (the fp32 weights the
// BN-fold coefficient products read, refreshed once per optimizer step by
// ops/wt_cache.py instead of one cast kernel per folded layer per forward).
constexpr int kMaxCast = 64, kCastPerBlock = 256 * 8;
struct CastTable {
  const __bf16* src[kMaxCast];
  float* dst[kMaxCast];
  int64_t n[kMaxCast];
  int first_block[kMaxCast + 1];
  int count;
};

__global__ __launch_bounds__(256) void multi_cast_kernel(const CastTable t) {
  const int bid = blockIdx.x;
  int lo = 0, hi = t.count - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (t.first_block[mid] <= bid) lo = mid;
    else hi = mid - 1;
  }
  const int64_t base = (int64_t)(bid - t.first_block[lo]) * kCastPerBlock;
  const __bf16* s = t.src[lo];
  float* d = t.dst[lo];
  const int64_t n = t.n[lo];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int64_t i = base + (int64_t)k * 256 + threadIdx.x;
    if (i < n) d[i] = (float)s[i];
  }
}

constexpr int kMaxReduceInputs = 16;
struct PtrPack {
  const void* p[kMaxReduceInputs];
};

template <typename T>
__global__ __launch_bounds__(256) void reduce_add_kernel(PtrPack ins, int k, T* __restrict__ out,
                                                         int64_t n) {
  constexpr int VEC = Vec16<T>::N;
  const int64_t nvec = n / VEC;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    float acc[VEC];
    Vec16<T>::load(reinterpret_cast<const T*>(ins.p[0]) + v * VEC, acc);
    for (int j = 1; j < k; ++j) {
      float t[VEC];
      Vec16<T>::load(reinterpret_cast<const T*>(ins.p[j]) + v * VEC, t);
#pragma unroll
      for (int e = 0; e < VEC; ++e) acc[e] += t[e];
    }
    Vec16<T>::store(out + v * VEC, acc);
  }
  // scalar tail
  const int64_t tail0 = nvec * VEC;
  for (int64_t i = tail0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float acc = 0.f;
    for (int j = 0; j < k; ++j) acc += (float)reinterpret_cast<const T*>(ins.p[j])[i];
    out[i] = (T)acc;
  }
}

// LDS-staged row gather: output [R_total, Cout] (row-major, row stride ldo),
// input i is [R_i, C_i] contiguous placed at (row_off_i, col_off_i).  One block
// moves a 32-row x 256-byte tile: global -> LDS with 16-B loads along the
// input's rows, LDS -> global with 16-B stores along the output's rows.
struct SlabDesc {
  const uint8_t* src;
  int64_t rows;
  int64_t row_bytes;   // bytes per input row
  int64_t dst_row0;    // first output row
  int64_t dst_col0;    // byte offset inside an output row
  int64_t tiles_before;
  int64_t col_tiles;
};

constexpr int kTileRows = 32;
constexpr int kTileBytes = 256;

__global__ __launch_bounds__(256) void gather_slabs_kernel(const SlabDesc* __restrict__ slabs,
                                                           int nslabs, uint8_t* __restrict__ out,
                                                           int64_t out_row_bytes) {
  __shared__ __attribute__((aligned(16))) uint8_t tile[kTileRows][kTileBytes + 16];
  const int64_t t = blockIdx.x;
  int s = 0;
  while (s + 1 < nslabs && slabs[s + 1].tiles_before <= t) ++s;
  const SlabDesc d = slabs[s];
  const int64_t local = t - d.tiles_before;
  const int64_t rt = local / d.col_tiles, ct = local % d.col_tiles;
  const int64_t r0 = rt * kTileRows;
  const int64_t c0 = ct * kTileBytes;
  const int64_t cb = min<int64_t>(kTileBytes, d.row_bytes - c0);
  // 256 threads = 32 rows x 8 lanes of 16 B... use 4-byte granules for generality.
  const bool vec16 = ((reinterpret_cast<uintptr_t>(d.src) | d.row_bytes | c0 | cb) & 15) == 0;
  const int lane = threadIdx.x % 16, row = threadIdx.x / 16;  // 16 rows per pass
  for (int rr = row; rr < kTileRows; rr += 16) {
    const int64_t r = r0 + rr;
    if (r >= d.rows) break;
    const uint8_t* sp = d.src + r * d.row_bytes + c0;
    if (vec16) {
      if (lane * 16 < cb)
        *reinterpret_cast<u32x4*>(&tile[rr][lane * 16]) = *reinterpret_cast<const u32x4*>(sp + lane * 16);
    } else {
      for (int b = lane; b < cb; b += 16) tile[rr][b] = sp[b];
    }
  }
  __syncthreads();
  const bool ovec16 = ((out_row_bytes | (d.dst_col0 + c0) | cb) & 15) == 0 && vec16;
  for (int rr = row; rr < kTileRows; rr += 16) {
    const int64_t r = r0 + rr;
    if (r >= d.rows) break;
    uint8_t* dp = out + (d.dst_row0 + r) * out_row_bytes + d.dst_col0 + c0;
    if (ovec16) {
      if (lane * 16 < cb)
        *reinterpret_cast<u32x4*>(dp + lane * 16) = *reinterpret_cast<const u32x4*>(&tile[rr][lane * 16]);
    } else {
      for (int b = lane; b < cb; b += 16) dp[b] = tile[rr][b];
    }
  }
}

// Tables uploaded while a stream is being captured into a hipGraph: the graph's
// memcpy node re-reads the pinned source on every replay, so the source must
// outlive the graph (the caching host allocator would otherwise recycle it).
std::mutex g_graph_tables_mu;
std::vector<at::Tensor> g_graph_tables;

// Upload a POD table to the device through pinned memory on the current stream.
template <typename T>
at::Tensor upload_table(const std::vector<T>& host, const at::Device& dev) {
  const int64_t bytes = (int64_t)(host.size() * sizeof(T));
  auto pinned = at::empty({std::max<int64_t>(bytes, 1)},
                          at::TensorOptions().dtype(at::kByte).pinned_memory(true));
  std::memcpy(pinned.data_ptr(), host.data(), bytes);
  auto dev_table = pinned.to(dev, /*non_blocking=*/true);
  hipStreamCaptureStatus status = hipStreamCaptureStatusNone;
  DMP_HIP_CHECK(hipStreamIsCapturing(at::hip::getCurrentHIPStream(dev.index()).stream(), &status));
  if (status != hipStreamCaptureStatusNone) {
    std::lock_guard<std::mutex> lk(g_graph_tables_mu);
    g_graph_tables.push_back(pinned);
    g_graph_tables.push_back(dev_table);  // graph-pool memory: keep the address stable too
  }
  return dev_table;
}

}  // namespace

// dst[i] [C, R] = src[i] [R, C]^T for 2-byte (bf16 / fp16) matrices, in as few
// launches as the table size allows (one for up to 64 matrices).  taps[i]
// (optional): T > 1 transposes tap by tap (src [R, T*C] -> dst [C, T*R]),
// -T also reverses the tap order (the flipped weight of a conv data gradient).

// dst[i] (fp32) = src[i] (bf16), same element counts, in as few launches as the
// table allows (one for up to 64 tensors)
void multi_cast_bf16_f32(const std::vector<at::Tensor>& srcs, const std::vector<at::Tensor>& dsts) {
  TORCH_CHECK(srcs.size() == dsts.size(), "multi_cast: list length mismatch");
  if (srcs.empty()) return;
  const at::Device dev = dsts[0].device();
  auto stream = at::hip::getCurrentHIPStream(dev.index());
  CastTable t{};
  int blocks = 0;
  auto flush = [&]() {
    if (t.count == 0) return;
    t.first_block[t.count] = blocks;
    hipLaunchKernelGGL(multi_cast_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, t);
    DMP_HIP_CHECK(hipGetLastError());
    t = CastTable{};
    blocks = 0;
  };
  for (size_t i = 0; i < srcs.size(); ++i) {
    const auto& s = srcs[i];
    const auto& d = dsts[i];
    TORCH_CHECK(s.is_cuda() && s.device() == dev && d.device() == dev && s.is_contiguous() && d.is_contiguous() &&
                    s.scalar_type() == at::kBFloat16 && d.scalar_type() == at::kFloat && s.numel() == d.numel(),
                "multi_cast: contiguous bf16 -> fp32 pairs of equal size on one device");
    const int64_t n = s.numel();
    if (n == 0) continue;
    const int64_t nb = (n + kCastPerBlock - 1) / kCastPerBlock;
    TORCH_CHECK(nb < (1 << 30), "multi_cast: tensor too large");
    if (t.count == kMaxCast || blocks + nb >= (1LL << 31) - 1) flush();
    t.src[t.count] = reinterpret_cast<const __bf16*>(s.data_ptr());
    t.dst[t.count] = d.data_ptr<float>();
    t.n[t.count] = n;
    t.first_block[t.count] = blocks;
    blocks += (int)nb;
    ++t.count;
  }
  flush();
}

void multi_transpose(const std::vector<at::Tensor>& srcs, const std::vector<at::Tensor>& dsts,
                     const std::vector<int64_t>& taps) {
  TORCH_CHECK(srcs.size() == dsts.size(), "multi_transpose: list length mismatch");
  TORCH_CHECK(taps.empty() || taps.size() == srcs.size(), "multi_transpose: taps length mismatch");
  if (srcs.empty()) return;
  const at::Device dev = dsts[0].device();
  auto stream = at::hip::getCurrentHIPStream(dev.index());
  TransTable t{};
  int tiles = 0;
  auto flush = [&]() {
    if (t.n == 0) return;
    t.first_tile[t.n] = tiles;
    hipLaunchKernelGGL(multi_transpose_kernel, dim3((unsigned)tiles), dim3(256), 0, stream, t);
    DMP_HIP_CHECK(hipGetLastError());
    t = TransTable{};
    tiles = 0;
  };
  for (size_t i = 0; i < srcs.size(); ++i) {
    const auto& s = srcs[i];
    const auto& d = dsts[i];
    TORCH_CHECK(s.is_cuda() && d.device() == dev && s.device() == dev, "multi_transpose: one device");
    const int64_t tp = taps.empty() ? 1 : taps[i], T = tp < 0 ? -tp : tp;
    TORCH_CHECK(T >= 1 && T <= 64, "multi_transpose: 1..64 taps");
    TORCH_CHECK(s.dim() == 2 && d.dim() == 2 && s.is_contiguous() && d.is_contiguous() && s.element_size() == 2 &&
                    d.scalar_type() == s.scalar_type() && s.size(1) % T == 0 && d.size(0) == s.size(1) / T &&
                    d.size(1) == s.size(0) * T,
                "multi_transpose: contiguous 2-byte [R, T*C] -> [C, T*R] pairs");
    const int64_t R = s.size(0), C = s.size(1) / T;
    if (R == 0 || C == 0) continue;
    TORCH_CHECK(R < (1 << 30) && C < (1 << 30), "multi_transpose: matrix too large");
    const int64_t nt = T * ((R + kTT - 1) / kTT) * ((C + kTT - 1) / kTT);
    if (t.n == kMaxT || tiles + nt >= (1LL << 31) - 1) flush();
    t.src[t.n] = static_cast<const uint16_t*>(s.data_ptr());
    t.dst[t.n] = static_cast<uint16_t*>(d.data_ptr());
    t.rows[t.n] = (int)R;
    t.cols[t.n] = (int)C;
    t.taps[t.n] = (int)T;
    t.flip[t.n] = tp < 0 ? 1 : 0;
    t.first_tile[t.n] = tiles;
    tiles += (int)nt;
    ++t.n;
  }
  flush();
}

// Copy byte ranges src[i] -> dst[i] (contiguous tensors, equal nbytes) in one launch on
// the current stream of dst's device.  srcs may live on a peer device (xGMI read).
void multi_copy(const std::vector<at::Tensor>& srcs, const std::vector<at::Tensor>& dsts) {
  TORCH_CHECK(srcs.size() == dsts.size(), "multi_copy: list length mismatch");
  if (srcs.empty()) return;
  const at::Device dev = dsts[0].device();
  auto stream = at::hip::getCurrentHIPStream(dev.index());
  CopyTable t{};
  int chunks = 0;
  auto flush = [&]() {
    if (t.n == 0) return;
    t.first_chunk[t.n] = chunks;
    hipLaunchKernelGGL(multi_copy_kernel, dim3((unsigned)chunks), dim3(256), 0, stream, t);
    t = CopyTable{};
    chunks = 0;
  };
  for (size_t i = 0; i < srcs.size(); ++i) {
    const auto& s = srcs[i];
    const auto& d = dsts[i];
    // raw byte copy: both contiguous, or both dense with identical shape/strides
    // (e.g. channels_last grads into channels_last bucket views)
    TORCH_CHECK((s.is_contiguous() && d.is_contiguous()) ||
                    (s.is_non_overlapping_and_dense() && d.is_non_overlapping_and_dense() &&
                     s.sizes() == d.sizes() && s.strides() == d.strides()),
                "multi_copy needs contiguous tensors or dense ones with identical strides");
    const int64_t nb = s.numel() * s.element_size();
    TORCH_CHECK(nb == d.numel() * d.element_size(), "multi_copy: byte size mismatch at ", i);
    TORCH_CHECK(d.device() == dev, "multi_copy: all destinations must share one device");
    if (nb == 0) continue;
    const int64_t nchunk = (nb + kChunkBytes - 1) / kChunkBytes;
    TORCH_CHECK(nchunk < (1LL << 30), "multi_copy: tensor too large");
    if (t.n == kMaxCopy || chunks + nchunk >= (1LL << 31) - 1) flush();
    t.src[t.n] = static_cast<const uint8_t*>(s.data_ptr());
    t.dst[t.n] = static_cast<uint8_t*>(d.data_ptr());
    t.nbytes[t.n] = nb;
    t.first_chunk[t.n] = chunks;
    chunks += (int)nchunk;
    ++t.n;
  }
  flush();
}

// out = sum(inputs); inputs may live on peer devices (peer access must be enabled).
void reduce_add_into(const std::vector<at::Tensor>& inputs, at::Tensor& out) {
  TORCH_CHECK(!inputs.empty() && (int)inputs.size() <= kMaxReduceInputs,
              "reduce_add supports 1..16 inputs");
  TORCH_CHECK(out.is_contiguous(), "reduce_add output must be contiguous");
  PtrPack pk{};
  for (size_t i = 0; i < inputs.size(); ++i) {
    TORCH_CHECK(inputs[i].is_contiguous() && inputs[i].numel() == out.numel() &&
                    inputs[i].scalar_type() == out.scalar_type(),
                "reduce_add: inputs must be contiguous and match the output");
    pk.p[i] = inputs[i].data_ptr();
  }
  const int64_t n = out.numel();
  if (n == 0) return;
  auto stream = at::hip::getCurrentHIPStream(out.device().index());
  const int64_t blocks = std::min<int64_t>((n / 8 + 255) / 256 + 1, 256 * 8);
  if (out.scalar_type() == at::kBFloat16) {
    hipLaunchKernelGGL(reduce_add_kernel<__bf16>, dim3(blocks), dim3(256), 0, stream, pk,
                       (int)inputs.size(), reinterpret_cast<__bf16*>(out.data_ptr()), n);
  } else {
    TORCH_CHECK(out.scalar_type() == at::kFloat, "reduce_add supports float32/bfloat16");
    hipLaunchKernelGGL(reduce_add_kernel<float>, dim3(blocks), dim3(256), 0, stream, pk,
                       (int)inputs.size(), out.data_ptr<float>(), n);
  }
}

// Concatenate 2-D-viewable inputs along `dim` (0 = rows, 1 = inner) into `out`
// with the LDS-staged tile kernel.  Inputs are viewed as [rows_i, inner_i]
// (rows = product of dims before `dim` ... the Python layer does the view).
void gather_slabs(const std::vector<at::Tensor>& inputs, at::Tensor& out, bool along_inner) {
  TORCH_CHECK(out.is_contiguous() && out.dim() == 2, "gather_slabs: out must be contiguous 2-D");
  const int64_t es = out.element_size();
  const int64_t out_row_bytes = out.size(1) * es;
  std::vector<SlabDesc> descs;
  int64_t tiles = 0, row_off = 0, col_off = 0;
  for (const auto& t : inputs) {
    TORCH_CHECK(t.is_contiguous() && t.dim() == 2, "gather_slabs: inputs must be contiguous 2-D");
    SlabDesc d;
    d.src = static_cast<const uint8_t*>(t.data_ptr());
    d.rows = t.size(0);
    d.row_bytes = t.size(1) * es;
    d.dst_row0 = along_inner ? 0 : row_off;
    d.dst_col0 = along_inner ? col_off : 0;
    d.col_tiles = (d.row_bytes + kTileBytes - 1) / kTileBytes;
    d.tiles_before = tiles;
    const int64_t rt = (d.rows + kTileRows - 1) / kTileRows;
    if (d.rows > 0 && d.row_bytes > 0) {
      tiles += rt * d.col_tiles;
      descs.push_back(d);
    }
    row_off += t.size(0);
    col_off += d.row_bytes;
  }
  if (descs.empty()) return;
  auto table = upload_table(descs, out.device());
  auto stream = at::hip::getCurrentHIPStream(out.device().index());
  hipLaunchKernelGGL(gather_slabs_kernel, dim3((unsigned)tiles), dim3(256), 0, stream,
                     reinterpret_cast<const SlabDesc*>(table.data_ptr()), (int)descs.size(),
                     static_cast<uint8_t*>(out.data_ptr()), out_row_bytes);
}

// Enables every possible peer mapping among devices [0, num_devices) and
// returns direct[a][b] = "a kernel on device a may dereference device b's
// memory" (a == b is always direct).  Pairs without peer access are reported,
// not skipped silently: comm_ops routes them through a staged copy
// (hipMemcpyPeerAsync via torch's copy_) instead of a peer-pointer kernel.
std::vector<std::vector<bool>> enable_peer_access(int64_t num_devices) {
  std::vector<std::vector<bool>> direct(num_devices, std::vector<bool>(num_devices, false));
  int cur = 0;
  DMP_HIP_CHECK(hipGetDevice(&cur));
  for (int a = 0; a < num_devices; ++a) {
    DMP_HIP_CHECK(hipSetDevice(a));
    direct[a][a] = true;
    for (int b = 0; b < num_devices; ++b) {
      if (a == b) continue;
      int can = 0;
      DMP_HIP_CHECK(hipDeviceCanAccessPeer(&can, a, b));
      if (!can) continue;
      hipError_t e = hipDeviceEnablePeerAccess(b, 0);
      if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) {
        hipSetDevice(cur);
        TORCH_CHECK(false, "hipDeviceEnablePeerAccess(", a, "->", b, ") failed: ", hipGetErrorString(e));
      }
      (void)hipGetLastError();
      direct[a][b] = true;
    }
  }
  DMP_HIP_CHECK(hipSetDevice(cur));
  return direct;
}

}  // namespace dmp
