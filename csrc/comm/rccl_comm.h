// Native RCCL communicator: one process per GPU, bootstrapped from an
// ncclUniqueId that the Python layer distributes through the torch.distributed
// store.  Collectives run on a dedicated (normal-priority) HIP stream per
// communicator so that gradient all-reduces overlap with backward kernels on
// the compute stream (xGMI transfers + RCCL kernels on their own queue).
//
// Reference parity: the reference moves activations with blocking
// dist.send/recv over NCCL (distributed_layers.py:11-13, 20-24, 42-60) and the
// README studies DDP's ring all-reduce per bucket (Readme.md:14,153-157).
// Here both are first-class native operations.
#pragma once

#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <rccl/rccl.h>

#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace dmp {

class RcclComm {
 public:
  RcclComm(const std::string& unique_id, int64_t nranks, int64_t rank, int64_t device,
           bool high_priority = false);
  ~RcclComm();

  static std::string new_unique_id();

  int64_t rank() const { return rank_; }
  int64_t size() const { return nranks_; }
  int64_t device() const { return device_; }

  // All ops: the comm stream first waits for the caller's current stream, then
  // enqueues the collective.  They return immediately (asynchronous).
  void all_reduce(at::Tensor& t, const std::string& op = "sum", bool on_current_stream = false);
  void all_reduce_coalesced(std::vector<at::Tensor>& ts, const std::string& op);
  void broadcast(at::Tensor& t, int64_t root);
  void reduce(at::Tensor& t, int64_t root, const std::string& op);
  void all_gather(at::Tensor& out, const at::Tensor& in);
  void reduce_scatter(at::Tensor& out, const at::Tensor& in, const std::string& op);
  void all_to_all(at::Tensor& out, const at::Tensor& in);
  void send(const at::Tensor& t, int64_t peer);
  void recv(at::Tensor& t, int64_t peer);
  // Batched point-to-point (ncclGroupStart/End): (tensor, peer, is_send).
  void batch_p2p(std::vector<at::Tensor>& ts, const std::vector<int64_t>& peers,
                 const std::vector<bool>& is_send);

  // Make the caller's current stream wait for all work enqueued so far.
  void wait();
  // Block the host until the comm stream is idle.
  void synchronize();
  // Raw stream handle (for event plumbing in the reducer).
  hipStream_t stream() const { return stream_.stream(); }
  c10::hip::HIPStream torch_stream() const { return stream_; }

  // Make the comm stream wait on the caller's current stream.
  void sync_from_current();
  // Inline mode: collectives run on the caller's current stream (no side
  // stream, no cross-stream events) -- no overlap with compute, no queue
  // interplay; chosen per process via DMP_COMM_INLINE (comm/rccl.py).
  void set_inline(bool v) { inline_ = v; }
  bool is_inline() const { return inline_; }
  void record_usage(const at::Tensor& t);

 private:
  ncclComm_t comm_ = nullptr;
  int64_t nranks_, rank_, device_;
  c10::hip::HIPStream stream_;
  bool inline_ = false;
  hipStream_t st() const;
  hipEvent_t ev_in_ = nullptr, ev_out_ = nullptr;
  std::mutex mu_;
};

ncclDataType_t to_nccl_dtype(const at::Tensor& t);
ncclRedOp_t to_nccl_op(const std::string& op);

}  // namespace dmp
