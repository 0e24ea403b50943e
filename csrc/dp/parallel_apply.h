// Native DataParallel replica launcher (reference Readme.md:70-107
// studies upstream parallel_apply: one Python threading.Thread per replica,
// created on every forward, results in a dict under a lock, exceptions wrapped
// as ExceptionWrapper("in replica i on device d")).
//
// Here the replicas run on PERSISTENT C++ worker threads (one per extra
// replica, created once, parked on a condition variable between steps), so a
// forward costs no thread creation and no Python-level context managers.  The
// caller's thread-local state is propagated in C++: the caller's current HIP
// stream of each replica's device, grad mode and autocast (enabled + dtype).
// Replica 0 runs inline on the calling thread (it already owns device 0's
// stream); the caller releases the GIL while it waits for the others.  A
// replica's exception comes back as (type, "Caught <T> in replica i on device
// d.\nOriginal Traceback ...") for the Python layer to re-raise with the
// original exception type (upstream ExceptionWrapper.reraise semantics).
#pragma once

#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include <condition_variable>
#include <memory>
#include <mutex>
#include <optional>
#include <thread>
#include <vector>

namespace dmp {

class ParallelApply {
 public:
  ParallelApply() = default;
  ~ParallelApply();

  // modules[i](*inputs[i], **kwargs[i]) on devices[i] (-1 = CPU).  Returns one
  // (ok, value) tuple per replica; on failure value = (exc_type, message).
  // Not reentrant: a call made while another is in flight (a second Python
  // thread, or a DataParallel nested inside a replica) returns None at once and
  // the caller falls back to its own threads.
  // streams[i] (optional, raw hipStream_t handles; 0 = the caller's current
  // stream of devices[i]): replicas that share a device run on streams of
  // their own, so their kernels can overlap on the GPU (the Python layer
  // orders those streams after the caller's and joins them afterwards).
  pybind11::object apply(const pybind11::list& modules, const pybind11::list& inputs,
                       const pybind11::list& kwargs, const std::vector<int64_t>& devices,
                       const std::vector<int64_t>& streams = {});
  int64_t num_workers() const { return (int64_t)workers_.size(); }
  // Host-time breakdown of the last apply(): [apply wall ms, then per replica
  // (wall ms, ms waiting for the GIL before its module call started,
  // ms inside the module call)] -- the "threshing" of Readme.md:10 made
  // visible: replicas that serialise on the GIL show wall ~ sum of the calls.
  std::vector<double> last_times() const { return last_times_; }

 private:
  struct Job {
    pybind11::object fn, args, kwargs;
    int64_t index = 0;
    int64_t device = -1;
    std::optional<c10::hip::HIPStream> stream;
    bool grad_enabled = true;
    bool autocast = false;
    at::ScalarType autocast_dtype = at::kBFloat16;
    pybind11::object result;  // (ok, value)
    double wall_ms = 0, gil_wait_ms = 0, call_ms = 0;
  };
  struct Worker {
    std::thread thread;
    std::mutex mu;
    std::condition_variable cv;
    Job* job = nullptr;
    bool stop = false;
  };

  static void run_job(Job& job);       // never throws: errors become (False, ...)
  static void run_job_impl(Job& job);
  void worker_main(Worker* w);
  void ensure_workers(size_t n);

  std::mutex apply_mu_;  // held for the whole of one apply()
  std::vector<std::unique_ptr<Worker>> workers_;
  std::mutex done_mu_;
  std::condition_variable done_cv_;
  int64_t outstanding_ = 0;
  std::vector<double> last_times_;
};

}  // namespace dmp
