#include "reducer.h"
#include "../trace.h"
#include "../check.h"

#include <ATen/hip/Sleep.h>
#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPGuard.h>

#include <torch/csrc/autograd/engine.h>
#include <torch/csrc/autograd/utils/lambda_post_hook.h>
#include <torch/csrc/autograd/variable.h>
#include <torch/csrc/autograd/grad_mode.h>

#include <algorithm>
#include <cstdio>
#include <map>
#include <unordered_set>

namespace dmp {

// coalesced.hip: one launch copying many dense tensors (same shapes/strides)
void multi_copy(const std::vector<at::Tensor>& srcs, const std::vector<at::Tensor>& dsts);


namespace py = pybind11;
using torch::autograd::Node;
using torch::autograd::variable_list;

// ---------------------------------------------------------------------------
// Python comm-hook backend
// ---------------------------------------------------------------------------
namespace {
hipEvent_t new_timing_event() {
  hipEvent_t e = nullptr;
  DMP_HIP_CHECK(hipEventCreate(&e));
  return e;
}
}  // namespace

RcclReduceBackend::~RcclReduceBackend() {
  if (device_ < 0) return;
  c10::hip::HIPGuard g(device_);
  for (auto e : ev_ready_) (void)hipEventDestroy(e);
  for (auto e : ev_done_) (void)hipEventDestroy(e);
  if (ev_bwd_end_) (void)hipEventDestroy(ev_bwd_end_);
  if (ev_tail_) (void)hipEventDestroy(ev_tail_);
}

void RcclReduceBackend::launch(int64_t index, at::Tensor& flat) {
  const int dev = flat.device().index();
  const hipStream_t caller = at::hip::getCurrentHIPStream(dev).stream();
  if (timing_) {
    c10::hip::HIPGuard g(dev);
    device_ = dev;
    while ((int64_t)ev_ready_.size() <= index) {
      ev_ready_.push_back(new_timing_event());
      ev_done_.push_back(new_timing_event());
    }
    DMP_HIP_CHECK(hipEventRecord(ev_ready_[index], caller));
  }
  if (fp32_ && (flat.scalar_type() == at::kBFloat16 || flat.scalar_type() == at::kHalf)) {
    // upcast, average and round back on the collective's stream (the copy is
    // allocated there, so the caching allocator keeps it until the copy-back)
    if (!comm_->is_inline()) comm_->sync_from_current();
    c10::hip::HIPStreamGuard guard(comm_->is_inline() ? at::hip::getCurrentHIPStream(dev) : comm_->torch_stream());
    at::Tensor wide = flat.to(at::kFloat);
    comm_->all_reduce(wide, "avg", /*on_current_stream=*/true);
    flat.copy_(wide);
  } else {
    comm_->all_reduce(flat, "avg");
  }
  // the tail runs on the stream the collective used, so wait_all() covers it
  const hipStream_t cs = comm_->is_inline() ? caller : comm_->stream();
  if (delay_ != 0 || postscale_ != 1.0) {
    c10::hip::HIPStreamGuard guard(comm_->is_inline() ? at::hip::getCurrentHIPStream(dev) : comm_->torch_stream());
    if (delay_ > 0) at::cuda::sleep(delay_);
    if (postscale_ != 1.0) flat.mul_(postscale_);
  }
  if (timing_) {
    DMP_HIP_CHECK(hipEventRecord(ev_done_[index], cs));
    launched_ = std::max(launched_, index + 1);
  }
}

void RcclReduceBackend::wait_all() {
  if (!timing_ || launched_ == 0) {
    comm_->wait();
    return;
  }
  c10::hip::HIPGuard g(device_);
  if (!ev_bwd_end_) {
    ev_bwd_end_ = new_timing_event();
    ev_tail_ = new_timing_event();
  }
  const hipStream_t cur = at::hip::getCurrentHIPStream(device_).stream();
  DMP_HIP_CHECK(hipEventRecord(ev_bwd_end_, cur));
  comm_->wait();
  DMP_HIP_CHECK(hipEventRecord(ev_tail_, cur));
  last_n_ = launched_;
  launched_ = 0;
}

std::vector<double> RcclReduceBackend::last_timing() {
  if (last_n_ == 0) return {};
  c10::hip::HIPGuard g(device_);
  DMP_HIP_CHECK(hipEventSynchronize(ev_tail_));
  auto ms = [](hipEvent_t a, hipEvent_t b) {
    float t = 0.f;
    DMP_HIP_CHECK(hipEventElapsedTime(&t, a, b));
    return (double)t;
  };
  std::vector<double> ready_done(last_n_), coll(last_n_);
  for (int64_t i = 0; i < last_n_; ++i) {
    ready_done[i] = ms(ev_ready_[i], ev_done_[i]);
    coll[i] = i == 0 ? ready_done[i] : std::min(ready_done[i], ms(ev_done_[i - 1], ev_done_[i]));
  }
  std::vector<double> out(ready_done);
  out.insert(out.end(), coll.begin(), coll.end());
  out.push_back(ms(ev_bwd_end_, ev_tail_));
  return out;
}

PyReduceBackend::~PyReduceBackend() {
  py::gil_scoped_acquire gil;
  pending_.clear();
  hook_ = py::object();
}

void PyReduceBackend::launch(int64_t index, at::Tensor& flat) {
  py::gil_scoped_acquire gil;
  pending_.push_back(hook_(index, flat));
}

void PyReduceBackend::wait_all() {
  py::gil_scoped_acquire gil;
  for (auto& h : pending_) {
    if (!h.is_none()) h.attr("wait")();
  }
  pending_.clear();
}

// ---------------------------------------------------------------------------
namespace {

constexpr int64_t kAlignElems = 8;  // 16 B for bf16, 32 B for fp32; matches the flat SGD vector

int64_t round_up(int64_t v, int64_t a) { return (v + a - 1) / a * a; }

struct GroupKey {
  at::ScalarType dtype;
  at::Device device;
  bool operator<(const GroupKey& o) const {
    if (dtype != o.dtype) return dtype < o.dtype;
    if (device.type() != o.device.type()) return device.type() < o.device.type();
    return device.index() < o.device.index();
  }
};

bool is_dense_non_overlapping(const at::Tensor& t) { return t.is_non_overlapping_and_dense(); }

}  // namespace

std::vector<std::vector<int64_t>> compute_bucket_assignment(const std::vector<at::Tensor>& params,
                                                            int64_t cap_bytes,
                                                            int64_t first_cap_bytes) {
  std::vector<std::vector<int64_t>> out;
  std::map<GroupKey, std::pair<std::vector<int64_t>, int64_t>> open;  // group -> (indices, bytes)
  bool first_emitted = false;
  for (int64_t i = (int64_t)params.size() - 1; i >= 0; --i) {
    const auto& p = params[i];
    GroupKey k{p.scalar_type(), p.device()};
    auto& slot = open[k];
    slot.first.push_back(i);
    slot.second += round_up(p.numel(), kAlignElems) * p.element_size();
    const int64_t limit = first_emitted ? cap_bytes : first_cap_bytes;
    if (slot.second >= limit) {
      out.push_back(std::move(slot.first));
      slot.first.clear();
      slot.second = 0;
      first_emitted = true;
    }
  }
  for (auto& kv : open)
    if (!kv.second.first.empty()) out.push_back(std::move(kv.second.first));
  return out;
}

// ---------------------------------------------------------------------------
Reducer::Reducer(std::vector<at::Tensor> params, std::vector<std::vector<int64_t>> buckets,
                 std::shared_ptr<ReduceBackend> backend, bool find_unused)
    : params_(std::move(params)), backend_(std::move(backend)), find_unused_(find_unused) {
  const int64_t n = (int64_t)params_.size();
  for (const auto& p : params_) {
    TORCH_CHECK(p.requires_grad(), "Reducer: every parameter must require grad");
    TORCH_CHECK(!p.is_sparse(), "Reducer: sparse parameters are not supported (SURVEY D10)");
    TORCH_CHECK(is_dense_non_overlapping(p), "Reducer: parameters must be dense");
  }
  ready_.assign(n, 0);
  build_layout(buckets);
  grad_accs_.resize(n);
  for (int64_t i = 0; i < n; ++i) {
    grad_accs_[i] = torch::autograd::impl::grad_accumulator(params_[i]);
    TORCH_CHECK(grad_accs_[i], "Reducer: parameter ", i, " is not a leaf");
    hook_keys_.push_back(grad_accs_[i]->add_post_hook(
        std::make_unique<torch::autograd::utils::LambdaPostHook>(
            [this, i](const variable_list& outputs, const variable_list&) {
              this->on_grad_ready(i);
              return outputs;
            })));
  }
}

Reducer::~Reducer() {
  // Remove our hooks: the accumulators may outlive the reducer.
  for (size_t i = 0; i < grad_accs_.size() && i < hook_keys_.size(); ++i)
    if (grad_accs_[i]) grad_accs_[i]->del_post_hook(hook_keys_[i]);
}

void Reducer::build_layout(const std::vector<std::vector<int64_t>>& buckets) {
  const int64_t n = (int64_t)params_.size();
  std::vector<char> seen(n, 0);
  for (const auto& b : buckets)
    for (int64_t i : b) {
      TORCH_CHECK(i >= 0 && i < n, "bucket index out of range");
      TORCH_CHECK(!seen[i], "parameter ", i, " assigned to two buckets");
      seen[i] = 1;
    }
  for (int64_t i = 0; i < n; ++i) TORCH_CHECK(seen[i], "parameter ", i, " has no bucket");

  std::map<GroupKey, int64_t> group_of;
  std::vector<int64_t> group_size;
  std::vector<GroupKey> group_keys;
  buckets_.clear();
  param_bucket_.assign(n, -1);
  param_group_.assign(n, -1);
  param_offset_.assign(n, 0);
  for (const auto& idxs : buckets) {
    if (idxs.empty()) continue;
    GroupKey k{params_[idxs[0]].scalar_type(), params_[idxs[0]].device()};
    auto it = group_of.find(k);
    int64_t g;
    if (it == group_of.end()) {
      g = (int64_t)group_keys.size();
      group_of[k] = g;
      group_keys.push_back(k);
      group_size.push_back(0);
    } else {
      g = it->second;
    }
    Bucket b;
    b.group = g;
    b.offset = group_size[g];
    for (int64_t i : idxs) {
      const auto& p = params_[i];
      TORCH_CHECK(p.scalar_type() == k.dtype && p.device() == k.device,
                  "a bucket must hold a single (dtype, device) group");
      param_bucket_[i] = (int64_t)buckets_.size();
      param_group_[i] = g;
      param_offset_[i] = group_size[g];
      group_size[g] += round_up(p.numel(), kAlignElems);
      b.params.push_back(i);
    }
    b.numel = group_size[g] - b.offset;
    buckets_.push_back(std::move(b));
  }
  std::vector<at::Tensor> old_views = views_;
  group_flats_.clear();
  for (size_t g = 0; g < group_keys.size(); ++g) {
    auto opts = at::TensorOptions().dtype(group_keys[g].dtype).device(group_keys[g].device);
    group_flats_.push_back(at::zeros({std::max<int64_t>(group_size[g], kAlignElems)}, opts));
  }
  for (auto& b : buckets_) b.flat = group_flats_[b.group].narrow(0, b.offset, b.numel);
  views_.assign(n, at::Tensor());
  torch::autograd::AutoGradMode no_grad(false);
  for (int64_t i = 0; i < n; ++i) {
    const auto& p = params_[i];
    views_[i] = group_flats_[param_group_[i]]
                    .narrow(0, param_offset_[i], p.numel())
                    .as_strided(p.sizes(), p.strides(), param_offset_[i]);
    // carry over existing gradients (rebuild)
    const auto& g = p.grad();
    if (g.defined()) {
      views_[i].copy_(g);
      p.mutable_grad() = views_[i];
    } else if (!old_views.empty() && old_views[i].defined()) {
      views_[i].copy_(old_views[i]);
    }
  }
}

void Reducer::rebuild(const std::vector<std::vector<int64_t>>& buckets) {
  std::lock_guard<std::mutex> lk(mu_);
  TORCH_CHECK(!armed_, "cannot rebuild buckets during backward");
  build_layout(buckets);
  record_order_ = false;
}

std::vector<std::vector<int64_t>> Reducer::buckets() const {
  std::vector<std::vector<int64_t>> out;
  for (const auto& b : buckets_) out.push_back(b.params);
  return out;
}

std::vector<std::pair<int64_t, int64_t>> Reducer::layout() const {
  std::vector<std::pair<int64_t, int64_t>> out;
  for (size_t i = 0; i < params_.size(); ++i) out.emplace_back(param_group_[i], param_offset_[i]);
  return out;
}

void Reducer::install_views_locked(bool zero_undefined) {
  torch::autograd::AutoGradMode no_grad(false);
  // Buckets whose every grad is undefined are zeroed with one fill.
  std::vector<char> bucket_all_undef(buckets_.size(), 1);
  for (size_t i = 0; i < params_.size(); ++i)
    if (params_[i].grad().defined()) bucket_all_undef[param_bucket_[i]] = 0;
  for (size_t b = 0; b < buckets_.size(); ++b)
    if (bucket_all_undef[b] && zero_undefined) buckets_[b].flat.zero_();
  for (size_t i = 0; i < params_.size(); ++i) {
    auto& p = params_[i];
    const auto& g = p.grad();
    if (!g.defined()) {
      if (zero_undefined && !bucket_all_undef[param_bucket_[i]]) views_[i].zero_();
      p.mutable_grad() = views_[i];
    } else if (!g.is_same(views_[i]) && g.data_ptr() != views_[i].data_ptr()) {
      views_[i].copy_(g);
      p.mutable_grad() = views_[i];
    }
  }
}

void Reducer::zero_grad() {
  std::lock_guard<std::mutex> lk(mu_);
  torch::autograd::AutoGradMode no_grad(false);
  for (auto& f : group_flats_) f.zero_();
  for (size_t i = 0; i < params_.size(); ++i) params_[i].mutable_grad() = views_[i];
  views_zeroed_ = true;
}

void Reducer::prepare_for_backward(const std::vector<at::Tensor>& outputs) {
  std::lock_guard<std::mutex> lk(mu_);
  // Steal mode iff no parameter carries gradient data the backward must add to.
  bool can_steal = true;
  for (size_t i = 0; i < params_.size() && can_steal; ++i) {
    const auto& g = params_[i].grad();
    if (g.defined() && !(views_zeroed_ && g.data_ptr() == views_[i].data_ptr())) can_steal = false;
  }
  steal_mode_ = can_steal;
  if (steal_mode_) {
    torch::autograd::AutoGradMode no_grad(false);
    for (auto& p : params_) p.mutable_grad() = at::Tensor();
    stolen_.assign(params_.size(), at::Tensor());
  } else {
    install_views_locked(/*zero_undefined=*/true);
  }
  views_zeroed_ = false;
  std::fill(ready_.begin(), ready_.end(), 0);
  for (auto& b : buckets_) b.pending = (int64_t)b.params.size();
  next_launch_ = 0;
  callback_queued_ = false;
  armed_ = true;
  if (record_order_) ready_order_.clear();
  last_unused_.clear();
  if (!find_unused_) return;

  // Walk the autograd graph from the outputs; any AccumulateGrad we do not
  // reach belongs to an unused parameter.
  std::unordered_set<Node*> seen;
  std::vector<Node*> stack;
  for (const auto& o : outputs) {
    if (!o.defined()) continue;
    auto fn = o.grad_fn();
    if (fn) {
      if (seen.insert(fn.get()).second) stack.push_back(fn.get());
    } else if (o.requires_grad()) {
      auto acc = torch::autograd::impl::try_get_grad_accumulator(o);
      if (acc && seen.insert(acc.get()).second) stack.push_back(acc.get());
    }
  }
  while (!stack.empty()) {
    Node* n = stack.back();
    stack.pop_back();
    for (const auto& e : n->next_edges()) {
      Node* m = e.function.get();
      if (m && seen.insert(m).second) stack.push_back(m);
    }
  }
  for (size_t i = 0; i < params_.size(); ++i) {
    if (!seen.count(grad_accs_[i].get())) last_unused_.push_back((int64_t)i);
  }
  // Unused parameters contribute zero gradients to their buckets.
  for (int64_t i : last_unused_) {
    views_[i].zero_();
    if (steal_mode_) params_[i].mutable_grad() = views_[i];
    mark_ready_locked(i);
  }
}

void Reducer::disarm() {
  std::lock_guard<std::mutex> lk(mu_);
  armed_ = false;
}

void Reducer::on_grad_ready(int64_t idx) {
  std::lock_guard<std::mutex> lk(mu_);
  views_zeroed_ = false;  // (also under no_sync: the views now hold data to accumulate into)
  if (!armed_) return;
  TORCH_CHECK(!ready_[idx], "Reducer: gradient of parameter ", idx,
              " became ready twice in one backward (reentrant backward or shared parameter "
              "used through an unused-parameter path?)");
  auto& p = params_[idx];
  const auto& g = p.grad();
  torch::autograd::AutoGradMode no_grad(false);
  if (g.defined() && g.data_ptr() != views_[idx].data_ptr()) {
    if (steal_mode_) {
      stolen_[idx] = g;  // copied into the bucket with its siblings in one launch
    } else {
      views_[idx].copy_(g);
      p.mutable_grad() = views_[idx];
    }
  }
  if (!callback_queued_) {
    callback_queued_ = true;
    torch::autograd::Engine::get_default_engine().queue_callback([this] { this->finalize(); });
  }
  mark_ready_locked(idx);
}

void Reducer::mark_ready_locked(int64_t idx) {
  ready_[idx] = 1;
  if (record_order_) ready_order_.push_back(idx);
  auto& b = buckets_[param_bucket_[idx]];
  b.pending -= 1;
  if (b.pending == 0) {
    if (steal_mode_) flush_bucket_locked(param_bucket_[idx]);
    launch_ready_prefix_locked();
  }
}

namespace {
bool same_dense_layout(const at::Tensor& a, const at::Tensor& b) {
  if (!a.is_cuda() || !b.is_cuda() || a.scalar_type() != b.scalar_type() || a.sizes() != b.sizes())
    return false;
  if (!a.is_non_overlapping_and_dense() || !b.is_non_overlapping_and_dense()) return false;
  for (int64_t d = 0; d < a.dim(); ++d)
    if (a.size(d) > 1 && a.stride(d) != b.stride(d)) return false;
  return true;
}
}  // namespace

void Reducer::flush_bucket_locked(int64_t bi) {
  std::vector<at::Tensor> srcs, dsts;
  for (int64_t i : buckets_[bi].params) {
    if (!stolen_[i].defined()) continue;
    srcs.push_back(stolen_[i]);
    dsts.push_back(views_[i]);
  }
  torch::autograd::AutoGradMode no_grad(false);
  // One coalesced launch for every pair with the same dense memory layout
  // (strides of size-1 dims do not matter: a [C,K,1,1] grad may carry either
  // contiguous or channels_last strides there); anything else copies alone.
  std::vector<at::Tensor> ms, md;
  for (size_t k = 0; k < srcs.size(); ++k) {
    if (same_dense_layout(srcs[k], dsts[k])) {
      ms.push_back(srcs[k]);
      md.push_back(dsts[k].as_strided(srcs[k].sizes(), srcs[k].strides()));
    } else {
      dsts[k].copy_(srcs[k]);
    }
  }
  if (!ms.empty()) multi_copy(ms, md);
  for (int64_t i : buckets_[bi].params) {
    stolen_[i] = at::Tensor();
    params_[i].mutable_grad() = views_[i];
  }
}

void Reducer::launch_ready_prefix_locked() {
  while (next_launch_ < (int64_t)buckets_.size() && buckets_[next_launch_].pending == 0) {
    char name[48];
    std::snprintf(name, sizeof(name), "ddp.bucket%lld.allreduce", (long long)next_launch_);
    trace::Range r(name);
    backend_->launch(next_launch_, buckets_[next_launch_].flat);
    ++next_launch_;
  }
}

void Reducer::finalize() {
  std::lock_guard<std::mutex> lk(mu_);
  if (!armed_) return;
  armed_ = false;
  if (next_launch_ != (int64_t)buckets_.size()) {
    std::string missing;
    int shown = 0;
    for (size_t i = 0; i < params_.size() && shown < 16; ++i)
      if (!ready_[i]) {
        missing += std::to_string(i) + " ";
        ++shown;
      }
    TORCH_CHECK(false,
                "DistributedDataParallel: backward finished but some parameters produced no "
                "gradient (indices: ", missing,
                "...). Pass find_unused_parameters=True if parts of the model are unused.");
  }
  {
    trace::Range r("ddp.wait_all");
    backend_->wait_all();
  }
  if (record_order_ && !ready_order_.empty()) record_order_ = false;
}

}  // namespace dmp
