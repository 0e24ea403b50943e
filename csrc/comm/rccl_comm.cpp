#include "rccl_comm.h"

#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPCachingAllocator.h>
#include <c10/hip/HIPGuard.h>

#include "../check.h"

namespace dmp {

#define DMP_NCCL_CHECK(expr)                                                        \
  do {                                                                              \
    ncclResult_t _r = (expr);                                                       \
    TORCH_CHECK(_r == ncclSuccess, "RCCL error ", ncclGetErrorString(_r), " at ",   \
                __FILE__, ":", __LINE__);                                           \
  } while (0)

ncclDataType_t to_nccl_dtype(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return ncclFloat32;
    case at::kBFloat16: return ncclBfloat16;
    case at::kHalf: return ncclFloat16;
    case at::kDouble: return ncclFloat64;
    case at::kInt: return ncclInt32;
    case at::kLong: return ncclInt64;
    case at::kByte: return ncclUint8;
    case at::kChar: return ncclInt8;
    case at::kBool: return ncclUint8;
    default: TORCH_CHECK(false, "RCCL: unsupported dtype ", t.scalar_type());
  }
}

ncclRedOp_t to_nccl_op(const std::string& op) {
  if (op == "sum") return ncclSum;
  if (op == "avg") return ncclAvg;
  if (op == "max") return ncclMax;
  if (op == "min") return ncclMin;
  if (op == "prod") return ncclProd;
  TORCH_CHECK(false, "RCCL: unsupported reduce op ", op);
}

std::string RcclComm::new_unique_id() {
  ncclUniqueId id;
  DMP_NCCL_CHECK(ncclGetUniqueId(&id));
  return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}

RcclComm::RcclComm(const std::string& unique_id, int64_t nranks, int64_t rank, int64_t device,
                   bool high_priority)
    : nranks_(nranks),
      rank_(rank),
      device_(device),
      stream_(c10::hip::getStreamFromPool(high_priority, (c10::DeviceIndex)device)) {
  TORCH_CHECK(unique_id.size() == sizeof(ncclUniqueId), "bad ncclUniqueId length");
  c10::hip::HIPGuard guard((c10::DeviceIndex)device);
  ncclUniqueId id;
  std::memcpy(&id, unique_id.data(), sizeof(id));
  DMP_NCCL_CHECK(ncclCommInitRank(&comm_, (int)nranks, id, (int)rank));
  DMP_HIP_CHECK(hipEventCreateWithFlags(&ev_in_, hipEventDisableTiming));
  DMP_HIP_CHECK(hipEventCreateWithFlags(&ev_out_, hipEventDisableTiming));
}

RcclComm::~RcclComm() {
  if (comm_) {
    // Abort rather than Destroy: at interpreter exit peers may already be gone
    // and ncclCommDestroy would block on them.
    ncclCommAbort(comm_);
    comm_ = nullptr;
  }
  if (ev_in_) hipEventDestroy(ev_in_);
  if (ev_out_) hipEventDestroy(ev_out_);
}

hipStream_t RcclComm::st() const {
  return inline_ ? at::hip::getCurrentHIPStream((c10::DeviceIndex)device_).stream() : stream_.stream();
}

void RcclComm::sync_from_current() {
  if (inline_) return;
  auto cur = at::hip::getCurrentHIPStream((c10::DeviceIndex)device_);
  if (cur.stream() == stream_.stream()) return;
  DMP_HIP_CHECK(hipEventRecord(ev_in_, cur.stream()));
  DMP_HIP_CHECK(hipStreamWaitEvent(stream_.stream(), ev_in_, 0));
}

void RcclComm::record_usage(const at::Tensor& t) {
  if (!inline_ && t.defined() && t.is_cuda())
    c10::hip::HIPCachingAllocator::recordStream(t.storage().data_ptr(), stream_);
}

void RcclComm::all_reduce(at::Tensor& t, const std::string& op, bool on_current_stream) {
  std::lock_guard<std::mutex> lk(mu_);
  TORCH_CHECK(t.is_contiguous(), "all_reduce needs a contiguous tensor");
  c10::hip::HIPGuard guard((c10::DeviceIndex)device_);
  hipStream_t s;
  if (on_current_stream) {
    // a small collective whose result the very next kernel needs (SyncBN
    // moments): no side stream, no event pair, nothing to overlap anyway
    s = at::hip::getCurrentHIPStream((c10::DeviceIndex)device_).stream();
  } else {
    sync_from_current();
    record_usage(t);
    s = st();
  }
  DMP_NCCL_CHECK(ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), to_nccl_dtype(t),
                               to_nccl_op(op), comm_, s));
}

void RcclComm::all_reduce_coalesced(std::vector<at::Tensor>& ts, const std::string& op) {
  std::lock_guard<std::mutex> lk(mu_);
  c10::hip::HIPGuard guard((c10::DeviceIndex)device_);
  sync_from_current();
  DMP_NCCL_CHECK(ncclGroupStart());
  for (auto& t : ts) {
    TORCH_CHECK(t.is_contiguous(), "all_reduce needs contiguous tensors");
    record_usage(t);
    DMP_NCCL_CHECK(ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), to_nccl_dtype(t),
                                 to_nccl_op(op), comm_, st()));
  }
  DMP_NCCL_CHECK(ncclGroupEnd());
}

void RcclComm::broadcast(at::Tensor& t, int64_t root) {
  std::lock_guard<std::mutex> lk(mu_);
  c10::hip::HIPGuard guard((c10::DeviceIndex)device_);
  sync_from_current();
  record_usage(t);
  DMP_NCCL_CHECK(ncclBroadcast(t.data_ptr(), t.data_ptr(), t.numel(), to_nccl_dtype(t), (int)root,
                               comm_, st()));
}

void RcclComm::reduce(at::Tensor& t, int64_t root, const std::string& op) {
  std::lock_guard<std::mutex> lk(mu_);
  c10::hip::HIPGuard guard((c10::DeviceIndex)device_);
  sync_from_current();
  record_usage(t);
  DMP_NCCL_CHECK(ncclReduce(t.data_ptr(), t.data_ptr(), t.numel(), to_nccl_dtype(t),
                            to_nccl_op(op), (int)root, comm_, st()));
}

void RcclComm::all_gather(at::Tensor& out, const at::Tensor& in) {
  std::lock_guard<std::mutex> lk(mu_);
  TORCH_CHECK(out.numel() == in.numel() * nranks_, "all_gather: out must be nranks x in");
  c10::hip::HIPGuard guard((c10::DeviceIndex)device_);
  sync_from_current();
  record_usage(out);
  record_usage(in);
  DMP_NCCL_CHECK(ncclAllGather(in.data_ptr(), out.data_ptr(), in.numel(), to_nccl_dtype(in), comm_,
                               st()));
}

void RcclComm::reduce_scatter(at::Tensor& out, const at::Tensor& in, const std::string& op) {
  std::lock_guard<std::mutex> lk(mu_);
  TORCH_CHECK(in.numel() == out.numel() * nranks_, "reduce_scatter: in must be nranks x out");
  c10::hip::HIPGuard guard((c10::DeviceIndex)device_);
  sync_from_current();
  record_usage(out);
  record_usage(in);
  DMP_NCCL_CHECK(ncclReduceScatter(in.data_ptr(), out.data_ptr(), out.numel(), to_nccl_dtype(in),
                                   to_nccl_op(op), comm_, st()));
}

void RcclComm::all_to_all(at::Tensor& out, const at::Tensor& in) {
  std::lock_guard<std::mutex> lk(mu_);
  TORCH_CHECK(in.numel() == out.numel() && in.numel() % nranks_ == 0, "all_to_all: bad sizes");
  c10::hip::HIPGuard guard((c10::DeviceIndex)device_);
  sync_from_current();
  record_usage(out);
  record_usage(in);
  const size_t chunk = in.numel() / nranks_;
  const size_t bytes = chunk * in.element_size();
  auto dt = to_nccl_dtype(in);
  DMP_NCCL_CHECK(ncclGroupStart());
  for (int64_t p = 0; p < nranks_; ++p) {
    DMP_NCCL_CHECK(ncclSend(static_cast<const char*>(in.data_ptr()) + p * bytes, chunk, dt, (int)p,
                            comm_, st()));
    DMP_NCCL_CHECK(ncclRecv(static_cast<char*>(out.data_ptr()) + p * bytes, chunk, dt, (int)p,
                            comm_, st()));
  }
  DMP_NCCL_CHECK(ncclGroupEnd());
}

void RcclComm::send(const at::Tensor& t, int64_t peer) {
  std::lock_guard<std::mutex> lk(mu_);
  c10::hip::HIPGuard guard((c10::DeviceIndex)device_);
  sync_from_current();
  record_usage(t);
  DMP_NCCL_CHECK(ncclSend(t.data_ptr(), t.numel(), to_nccl_dtype(t), (int)peer, comm_,
                          st()));
}

void RcclComm::recv(at::Tensor& t, int64_t peer) {
  std::lock_guard<std::mutex> lk(mu_);
  c10::hip::HIPGuard guard((c10::DeviceIndex)device_);
  sync_from_current();
  record_usage(t);
  DMP_NCCL_CHECK(ncclRecv(t.data_ptr(), t.numel(), to_nccl_dtype(t), (int)peer, comm_,
                          st()));
}

void RcclComm::batch_p2p(std::vector<at::Tensor>& ts, const std::vector<int64_t>& peers,
                         const std::vector<bool>& is_send) {
  std::lock_guard<std::mutex> lk(mu_);
  TORCH_CHECK(ts.size() == peers.size() && ts.size() == is_send.size(), "batch_p2p: sizes");
  c10::hip::HIPGuard guard((c10::DeviceIndex)device_);
  sync_from_current();
  DMP_NCCL_CHECK(ncclGroupStart());
  for (size_t i = 0; i < ts.size(); ++i) {
    record_usage(ts[i]);
    if (is_send[i])
      DMP_NCCL_CHECK(ncclSend(ts[i].data_ptr(), ts[i].numel(), to_nccl_dtype(ts[i]), (int)peers[i],
                              comm_, st()));
    else
      DMP_NCCL_CHECK(ncclRecv(ts[i].data_ptr(), ts[i].numel(), to_nccl_dtype(ts[i]), (int)peers[i],
                              comm_, st()));
  }
  DMP_NCCL_CHECK(ncclGroupEnd());
}

void RcclComm::wait() {
  std::lock_guard<std::mutex> lk(mu_);
  c10::hip::HIPGuard guard((c10::DeviceIndex)device_);
  if (inline_) return;  // collectives already ran on the current stream
  auto cur = at::hip::getCurrentHIPStream((c10::DeviceIndex)device_);
  if (cur.stream() == stream_.stream()) return;
  DMP_HIP_CHECK(hipEventRecord(ev_out_, stream_.stream()));
  DMP_HIP_CHECK(hipStreamWaitEvent(cur.stream(), ev_out_, 0));
}

void RcclComm::synchronize() {
  c10::hip::HIPGuard guard((c10::DeviceIndex)device_);
  DMP_HIP_CHECK(hipStreamSynchronize(st()));
}

}  // namespace dmp
