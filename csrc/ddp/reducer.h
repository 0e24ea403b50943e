// Native gradient Reducer for DistributedDataParallel.
//
// The reference studies upstream DDP's C++ Reducer in prose only
// (Readme.md:145-157: "Ring AllReduce is used, one time reduce one bucket.
// Parameters are separated into buckets"; "On each forward, it checks each
// variable is used or not").  This is an independent MI355X-first design:
//
//   * Gradients of one (dtype, device) group live in ONE flat allocation; the
//     buckets are contiguous slices of it, every parameter's .grad is a view
//     into it (gradient-as-bucket-view), so backward's AccumulateGrad writes
//     straight into the communication buffer and a flat fused optimizer can
//     step every parameter of the group in one kernel.
//   * Post-AccumulateGrad hooks are registered from C++ (no Python in the
//     backward path).  When the last gradient of a bucket lands, the bucket's
//     all-reduce is launched -- strictly in bucket order so every rank issues
//     identical RCCL calls -- on the backend's side stream.
//   * The backend is pluggable: native RCCL (ncclAvg on a dedicated HIP
//     stream) for MI355X, or a Python comm hook (gloo / any process group)
//     for CPU tests and custom compression hooks (upstream register_comm_hook).
//   * find_unused_parameters: a C++ walk of the autograd graph from the
//     forward outputs marks unreached parameters ready up front.
//   * The ready order of the first iteration is recorded so the Python layer
//     can rebuild buckets in true autograd order (rank 0's order, broadcast).
#pragma once

#include <torch/extension.h>
#include <torch/csrc/autograd/function.h>

#include <functional>
#include <memory>
#include <mutex>
#include <vector>

#include "../comm/rccl_comm.h"

namespace dmp {

class ReduceBackend {
 public:
  virtual ~ReduceBackend() = default;
  // Start an asynchronous AVERAGE all-reduce of `flat` (bucket `index`).
  virtual void launch(int64_t index, at::Tensor& flat) = 0;
  // Make results of every launched bucket visible to the caller's stream/host.
  virtual void wait_all() = 0;
};

class RcclReduceBackend : public ReduceBackend {
 public:
  // postscale: multiply the averaged bucket by this factor on the comm stream
  // (folds a loss-scale / accumulation divisor into the collective's tail).
  // debug_delay_cycles: spin the comm stream before the scale -- a test knob
  // that widens any missing comm-stream -> compute-stream ordering into a
  // visible wrong result (tests/test_gpu_ddp.py).
  // fp32_accum: a bf16 / fp16 bucket is averaged through an fp32 copy on the
  // comm stream (2x the bytes on the wire; the ring then rounds once, at the
  // end, instead of after every hop: tests/test_multirank_risks.py bounds both)
  explicit RcclReduceBackend(std::shared_ptr<RcclComm> comm, double postscale = 1.0,
                             int64_t debug_delay_cycles = 0, bool fp32_accum = false)
      : comm_(std::move(comm)), postscale_(postscale), delay_(debug_delay_cycles), fp32_(fp32_accum) {}
  ~RcclReduceBackend() override;
  void launch(int64_t, at::Tensor& flat) override;
  void wait_all() override;

  // Communication accounting (bench.py config.ddp_comm): with timing on, each
  // launch records an event on the launching stream (the bucket is ready) and
  // one on the collective's stream after it (done); wait_all() records the end
  // of backward and the point the compute stream may continue.  last_timing()
  // (host-synchronising) returns, for the last backward: per bucket the
  // ready -> done ms and the collective's own ms (from the later of its ready
  // point and the previous bucket's done: the comm stream is serial), then the
  // exposed tail ms (end of backward -> every bucket reduced).
  void set_timing(bool on) { timing_ = on; }
  std::vector<double> last_timing();

 private:
  std::shared_ptr<RcclComm> comm_;
  double postscale_;
  int64_t delay_;
  bool fp32_ = false;
  bool timing_ = false;
  int64_t launched_ = 0, last_n_ = 0;
  int device_ = -1;
  std::vector<hipEvent_t> ev_ready_, ev_done_;
  hipEvent_t ev_bwd_end_ = nullptr, ev_tail_ = nullptr;
};

// world_size == 1: the average over one rank is the identity, nothing to move.
class NullReduceBackend : public ReduceBackend {
 public:
  void launch(int64_t, at::Tensor&) override {}
  void wait_all() override {}
};

// hook(index, tensor) -> object with .wait(); the hook must leave the AVERAGED
// gradient in `tensor` once wait() returns.
class PyReduceBackend : public ReduceBackend {
 public:
  explicit PyReduceBackend(pybind11::object hook) : hook_(std::move(hook)) {}
  ~PyReduceBackend() override;
  void launch(int64_t index, at::Tensor& flat) override;
  void wait_all() override;

 private:
  pybind11::object hook_;
  std::vector<pybind11::object> pending_;
};

class Reducer {
 public:
  Reducer(std::vector<at::Tensor> params, std::vector<std::vector<int64_t>> buckets,
          std::shared_ptr<ReduceBackend> backend, bool find_unused);
  ~Reducer();

  // Arm the reducer for the next backward.  `outputs` are the forward outputs
  // (used only when find_unused is on).
  void prepare_for_backward(const std::vector<at::Tensor>& outputs);
  // Disarm without a backward (e.g. forward under no_sync, or eval).
  void disarm();

  // Replace the bucket assignment (same parameter set).  Existing gradient
  // values are carried over.
  void rebuild(const std::vector<std::vector<int64_t>>& buckets);

  std::vector<std::vector<int64_t>> buckets() const;
  std::vector<int64_t> ready_order() const { return ready_order_; }
  std::vector<at::Tensor> group_flats() const { return group_flats_; }
  // Per-parameter (group index, element offset within the group flat).
  std::vector<std::pair<int64_t, int64_t>> layout() const;
  std::vector<at::Tensor> grad_views() const { return views_; }
  std::vector<int64_t> unused_params() const { return last_unused_; }
  int64_t num_launched() const { return next_launch_; }
  void set_backend(std::shared_ptr<ReduceBackend> b) { backend_ = std::move(b); }
  // Point every .grad at its bucket view and zero the buckets (fast zero_grad).
  void zero_grad();
  bool steal_mode() const { return steal_mode_; }

 private:
  void build_layout(const std::vector<std::vector<int64_t>>& buckets);
  void on_grad_ready(int64_t idx);
  void mark_ready_locked(int64_t idx);
  void launch_ready_prefix_locked();
  void finalize();
  void install_views_locked(bool zero_undefined);

  struct Bucket {
    std::vector<int64_t> params;
    int64_t group = 0;
    int64_t offset = 0;  // element offset in the group flat
    int64_t numel = 0;
    int64_t pending = 0;
    at::Tensor flat;     // slice of the group flat
  };

  std::vector<at::Tensor> params_;
  std::vector<std::shared_ptr<torch::autograd::Node>> grad_accs_;
  std::vector<uintptr_t> hook_keys_;
  std::vector<at::Tensor> group_flats_;
  std::vector<Bucket> buckets_;
  std::vector<int64_t> param_bucket_;
  std::vector<int64_t> param_group_;
  std::vector<int64_t> param_offset_;
  std::vector<at::Tensor> views_;
  std::vector<char> ready_;
  std::vector<int64_t> ready_order_;
  std::vector<int64_t> last_unused_;
  std::shared_ptr<ReduceBackend> backend_;
  bool find_unused_;
  bool armed_ = false;
  bool callback_queued_ = false;
  bool record_order_ = true;
  int64_t next_launch_ = 0;
  // Steal mode (the common case: grads were zeroed or are None before the
  // backward): parameter grads start undefined, AccumulateGrad steals each new
  // gradient without a kernel, and a completed bucket is filled by ONE
  // coalesced copy launch -- instead of a zero-fill plus one in-place add per
  // parameter (161 add launches per ResNet-50 step).  Accumulate mode (grads
  // carry data, e.g. after no_sync) keeps the installed views.
  bool steal_mode_ = false;
  bool views_zeroed_ = true;      // views hold zeros (zero_grad) and nothing wrote since
  std::vector<at::Tensor> stolen_;
  void flush_bucket_locked(int64_t b);
  std::mutex mu_;
};

// Size-capped bucket assignment in reverse registration order (the usual
// autograd ready order): first bucket `first_cap` bytes, then `cap` bytes;
// buckets never mix (dtype, device) groups.
std::vector<std::vector<int64_t>> compute_bucket_assignment(const std::vector<at::Tensor>& params,
                                                            int64_t cap_bytes,
                                                            int64_t first_cap_bytes);

}  // namespace dmp
