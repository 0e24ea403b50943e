#include "parallel_apply.h"

#include <ATen/autocast_mode.h>
#include <ATen/hip/HIPContext.h>
#include <c10/core/GradMode.h>
#include <c10/hip/HIPGuard.h>

#include <chrono>
#include <string>

#include "../trace.h"

namespace py = pybind11;

namespace dmp {

ParallelApply::~ParallelApply() {
  for (auto& w : workers_) {
    {
      std::lock_guard<std::mutex> lk(w->mu);
      w->stop = true;
    }
    w->cv.notify_one();
  }
  // joining may wait for a replica that needs the GIL: release it if we hold it
  const bool held = Py_IsInitialized() && PyGILState_Check();
  PyThreadState* ts = held ? PyEval_SaveThread() : nullptr;
  for (auto& w : workers_)
    if (w->thread.joinable()) w->thread.join();
  if (ts) PyEval_RestoreThread(ts);
}

void ParallelApply::ensure_workers(size_t n) {
  while (workers_.size() < n) {
    workers_.push_back(std::make_unique<Worker>());
    Worker* w = workers_.back().get();
    w->thread = std::thread([this, w] { worker_main(w); });
  }
}

namespace {
// restores the thread's autocast state however run_job_impl leaves
struct AutocastRestore {
  bool enabled = at::autocast::is_autocast_enabled(at::kCUDA);
  at::ScalarType dtype = at::autocast::get_autocast_dtype(at::kCUDA);
  ~AutocastRestore() {
    at::autocast::set_autocast_enabled(at::kCUDA, enabled);
    at::autocast::set_autocast_dtype(at::kCUDA, dtype);
  }
};
}  // namespace

// A C++ exception (c10::Error from the device guard, a pybind11 cast error)
// must not unwind through a worker thread or past apply() while other workers
// still read `jobs`: it becomes this replica's (False, (RuntimeError, msg)).
void ParallelApply::run_job(Job& job) {
  std::string err;
  try {
    run_job_impl(job);
  } catch (const std::exception& e) {
    err = e.what();
  } catch (...) {
    err = "unknown C++ exception";
  }
  if (err.empty()) return;
  py::gil_scoped_acquire gil;
  std::string dev = job.device >= 0 ? "cuda:" + std::to_string(job.device) : "cpu";
  std::string msg = "Caught RuntimeError in replica " + std::to_string(job.index) + " on device " + dev +
                    ".\n" + err;
  job.result = py::make_tuple(false, py::make_tuple(py::module_::import("builtins").attr("RuntimeError"), msg));
  job.fn = py::object();
  job.args = py::object();
  job.kwargs = py::object();
}

// Runs with the GIL NOT held; takes it only around the Python call.
namespace {
double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}
}  // namespace

void ParallelApply::run_job_impl(Job& job) {
  const auto t0 = std::chrono::steady_clock::now();
  char name[48];
  std::snprintf(name, sizeof(name), "dp.replica%lld", (long long)job.index);
  trace::Range range(name);
  std::optional<c10::hip::HIPGuard> dev_guard;
  if (job.device >= 0) {
    dev_guard.emplace((c10::DeviceIndex)job.device);
    if (job.stream) c10::hip::setCurrentHIPStream(*job.stream);
  }
  c10::AutoGradMode grad(job.grad_enabled);
  AutocastRestore ac_restore;
  at::autocast::set_autocast_enabled(at::kCUDA, job.autocast);
  at::autocast::set_autocast_dtype(at::kCUDA, job.autocast_dtype);
  {
    const auto tg = std::chrono::steady_clock::now();
    py::gil_scoped_acquire gil;
    job.gil_wait_ms = ms_since(tg);
    const auto tc = std::chrono::steady_clock::now();
    try {
      py::object out = job.fn(*job.args, **job.kwargs);
      job.call_ms = ms_since(tc);
      job.result = py::make_tuple(true, out);
    } catch (py::error_already_set& e) {
      std::string tb;
      try {
        py::object lines = py::module_::import("traceback")
                               .attr("format_exception")(e.type(), e.value(), e.trace());
        tb = py::str("").attr("join")(lines).cast<std::string>();
      } catch (...) {
        tb = e.what();
      }
      std::string dev = job.device >= 0 ? "cuda:" + std::to_string(job.device) : "cpu";
      std::string tname = py::str(e.type().attr("__name__")).cast<std::string>();
      std::string msg = "Caught " + tname + " in replica " + std::to_string(job.index) +
                        " on device " + dev + ".\nOriginal " + tb;
      job.result = py::make_tuple(false, py::make_tuple(e.type(), msg));
    }
    job.fn = py::object();
    job.args = py::object();
    job.kwargs = py::object();
  }
  job.wall_ms = ms_since(t0);
}

void ParallelApply::worker_main(Worker* w) {
  for (;;) {
    Job* job = nullptr;
    {
      std::unique_lock<std::mutex> lk(w->mu);
      w->cv.wait(lk, [w] { return w->stop || w->job != nullptr; });
      if (w->stop) return;
      job = w->job;
      w->job = nullptr;
    }
    run_job(*job);
    {
      std::lock_guard<std::mutex> lk(done_mu_);
      --outstanding_;
    }
    done_cv_.notify_all();
  }
}

py::object ParallelApply::apply(const py::list& modules, const py::list& inputs,
                                const py::list& kwargs, const std::vector<int64_t>& devices,
                                const std::vector<int64_t>& streams) {
  std::unique_lock<std::mutex> busy(apply_mu_, std::try_to_lock);
  if (!busy.owns_lock()) return py::none();  // re-entered: the caller uses its own threads
  const size_t n = py::len(modules);
  TORCH_CHECK(py::len(inputs) == n && py::len(kwargs) == n && devices.size() == n,
              "parallel_apply: modules, inputs, kwargs and devices must have the same length");
  TORCH_CHECK(streams.empty() || streams.size() == n, "parallel_apply: one stream handle per replica (or none)");
  if (n == 0) return py::list();
  // caller's thread-local state, captured here (GIL held, calling thread)
  const bool grad = c10::GradMode::is_enabled();
  const bool ac = at::autocast::is_autocast_enabled(at::kCUDA);
  const at::ScalarType ac_dtype = at::autocast::get_autocast_dtype(at::kCUDA);
  std::vector<Job> jobs(n);
  for (size_t i = 0; i < n; ++i) {
    Job& j = jobs[i];
    j.fn = modules[i];
    py::object a = inputs[i];
    j.args = py::isinstance<py::tuple>(a) ? a : (py::isinstance<py::list>(a) ? py::tuple(a) : py::make_tuple(a));
    j.kwargs = kwargs[i].is_none() ? py::dict() : py::object(kwargs[i]);
    j.index = (int64_t)i;
    j.device = devices[i];
    if (j.device >= 0) {
      const int64_t h = streams.empty() ? 0 : streams[i];
      j.stream = h ? c10::hip::getStreamFromExternal(reinterpret_cast<hipStream_t>(h), (c10::DeviceIndex)j.device)
                   : c10::hip::getCurrentHIPStream((c10::DeviceIndex)j.device);
    }
    j.grad_enabled = grad;
    j.autocast = ac;
    j.autocast_dtype = ac_dtype;
  }
  ensure_workers(n - 1);
  const auto t_apply = std::chrono::steady_clock::now();
  {
    py::gil_scoped_release nogil;
    {
      std::lock_guard<std::mutex> lk(done_mu_);
      outstanding_ = (int64_t)n - 1;
    }
    for (size_t i = 1; i < n; ++i) {
      Worker* w = workers_[i - 1].get();
      {
        std::lock_guard<std::mutex> lk(w->mu);
        w->job = &jobs[i];
      }
      w->cv.notify_one();
    }
    run_job(jobs[0]);  // replica 0 on the calling thread
    std::unique_lock<std::mutex> lk(done_mu_);
    done_cv_.wait(lk, [this] { return outstanding_ == 0; });
  }
  last_times_.assign(1, ms_since(t_apply));
  for (auto& j : jobs) {
    last_times_.push_back(j.wall_ms);
    last_times_.push_back(j.gil_wait_ms);
    last_times_.push_back(j.call_ms);
  }
  py::list out;
  for (auto& j : jobs) out.append(j.result);
  return out;
}

}  // namespace dmp
