#include "ps_core.h"

#include <algorithm>
#include <chrono>

#include "async_hyper.h"
#include "checkpoint.h"
#include "kernels/launchers.h"
#include "ops.h"

namespace psd {

// Timed waits use a system_clock deadline: libstdc++ then waits with pthread_cond_timedwait, which
// ThreadSanitizer intercepts (its steady_clock path, pthread_cond_clockwait, is invisible to the
// GCC 11 TSAN runtime and yields false "double lock" reports in tests/test_sanitizers.py).
static inline std::chrono::system_clock::time_point deadline(double seconds) {
  return std::chrono::system_clock::now() +
         std::chrono::duration_cast<std::chrono::system_clock::duration>(std::chrono::duration<double>(seconds));
}

namespace {
constexpr int64_t kAlign = 8;  // elements: keeps every tensor 16-B aligned inside the flat buffers
constexpr int kHistBins = 64;
int64_t round_up(int64_t x, int64_t a) { return (x + a - 1) / a * a; }
}  // namespace

PSCore::PSCore(PSConfig cfg, std::string device) : cfg_(std::move(cfg)), dev_(device), hist_(kHistBins, 0) {
  TORCH_CHECK(cfg_.total_workers >= 1, "psd: total_workers must be >= 1");
  dyn_ = at::zeros({8}, at::TensorOptions().dtype(at::kInt).device(dev_));
}

bool PSCore::initialized() const {
  std::lock_guard<std::mutex> g(mu_);
  return init_;
}

void PSCore::layout_locked(const std::vector<std::string>& names, const std::vector<std::vector<int64_t>>& shapes) {
  names_ = names;
  shapes_ = shapes;
  offsets_.clear();
  numels_.clear();
  int64_t off = 0;
  for (auto& s : shapes) {
    int64_t n = 1;
    for (int64_t d : s) n *= d;
    offsets_.push_back(off);
    numels_.push_back(n);
    off += round_up(std::max<int64_t>(n, 1), kAlign);
  }
  total_ = std::max<int64_t>(off, kAlign);
}

void PSCore::alloc_state_locked() {
  auto opt = at::TensorOptions().dtype(at::kFloat).device(dev_);
  master_ = at::zeros({total_}, opt);
  s1_ = (cfg_.opt_kind != OPT_SGD) ? at::zeros({total_}, opt) : at::Tensor();
  s2_ = (cfg_.opt_kind == OPT_ADAM || cfg_.opt_kind == OPT_ADAMW) ? at::zeros({total_}, opt) : at::Tensor();
  dyn_.zero_();
  slots_.clear();
  free_slots_.clear();
}

void PSCore::init_params(const std::vector<std::string>& names, const std::vector<std::vector<int64_t>>& shapes,
                         const std::vector<at::Tensor>& values) {
  TORCH_CHECK(names.size() == shapes.size() && names.size() == values.size(), "psd: init_params length mismatch");
  std::lock_guard<std::mutex> g(mu_);
  layout_locked(names, shapes);
  alloc_state_locked();
  for (size_t i = 0; i < values.size(); ++i) {
    TORCH_CHECK(values[i].numel() == numels_[i], "psd: init value size mismatch for ", names[i]);
    master_.narrow(0, offsets_[i], numels_[i]).copy_(values[i].reshape({-1}).to(at::kFloat));
  }
  iters_.clear();
  init_ = true;
  cv_.notify_all();
}

std::vector<std::string> PSCore::names() const {
  std::lock_guard<std::mutex> g(mu_);
  return names_;
}
std::vector<std::vector<int64_t>> PSCore::shapes() const {
  std::lock_guard<std::mutex> g(mu_);
  return shapes_;
}
std::vector<int64_t> PSCore::offsets() const {
  std::lock_guard<std::mutex> g(mu_);
  return offsets_;
}
int64_t PSCore::numel() const {
  std::lock_guard<std::mutex> g(mu_);
  return total_;
}

int32_t PSCore::take_slot_locked() {
  if (!free_slots_.empty()) {
    int32_t s = free_slots_.back();
    free_slots_.pop_back();
    return s;
  }
  slots_.push_back(at::zeros({total_}, at::TensorOptions().dtype(at::kFloat).device(dev_)));
  return (int32_t)slots_.size() - 1;
}

void PSCore::fill_slot_locked(at::Tensor& slot, const std::vector<std::string>& names, const std::vector<at::Tensor>& grads) {
  for (size_t i = 0; i < grads.size(); ++i) {
    slot.narrow(0, offsets_[i], numels_[i]).copy_(grads[i].reshape({-1}).to(at::kFloat), /*non_blocking=*/true);
  }
}

void PSCore::apply_locked(const std::vector<at::Tensor>& sources, double lr, double grad_scale, const AsyncHyper* ah) {
  std::vector<at::Tensor> srcs = sources;
  if (srcs.size() > (size_t)kMaxSources) {  // pre-reduce in groups of 16 (exact fp32 sums)
    at::Tensor acc = at::empty_like(srcs[0]);
    std::vector<at::Tensor> grp(srcs.begin(), srcs.begin() + kMaxSources);
    multi_reduce_(acc, grp, 1.0);
    for (size_t b = kMaxSources; b < srcs.size(); b += kMaxSources - 1) {
      std::vector<at::Tensor> g2{acc.clone()};
      for (size_t k = b; k < std::min(srcs.size(), b + kMaxSources - 1); ++k) g2.push_back(srcs[k]);
      multi_reduce_(acc, g2, 1.0);
    }
    srcs = {acc};
  }
  at::Tensor host = at::zeros({8}, at::kInt);
  float* hf = reinterpret_cast<float*>(host.data_ptr<int32_t>());
  // keep step/bias-corrections (written by optim_advance) and refresh lr / grad_scale
  at::Tensor cur = dyn_.to(at::kCPU);
  host.copy_(cur);
  hf[0] = (float)lr;
  hf[1] = (float)grad_scale;
  dyn_.copy_(host);
  // async pushes run with the per-push hyperparameters of async_hyper.h (one push = 1/W round)
  const double mom = ah ? ah->momentum : cfg_.momentum, wd = ah ? ah->weight_decay : cfg_.weight_decay;
  const double b1 = ah ? ah->beta1 : cfg_.beta1, b2 = ah ? ah->beta2 : cfg_.beta2;
  optim_advance_(dyn_, b1, b2);
  fused_apply_(master_, srcs, s1_.defined() ? c10::optional<at::Tensor>(s1_) : c10::nullopt,
               s2_.defined() ? c10::optional<at::Tensor>(s2_) : c10::nullopt, c10::nullopt, dyn_, cfg_.opt_kind,
               mom, cfg_.dampening, cfg_.nesterov, wd, b1, b2, cfg_.eps, false);
  ctr_["applies"] += 1;
}

void PSCore::trim_locked() {
  const int32_t lo = current_iteration_ - cfg_.window;
  for (auto it = iters_.begin(); it != iters_.end() && it->first < lo;) {
    for (auto& kv : it->second.slot_of) free_slots_.push_back(kv.second);
    it = iters_.erase(it);
  }
}

int32_t PSCore::min_clock_locked() const {
  if ((int32_t)clock_.size() < cfg_.total_workers) return 0;
  int32_t m = INT32_MAX;
  for (auto& kv : clock_) m = std::min(m, kv.second);
  return m == INT32_MAX ? 0 : m;
}

PushResult PSCore::push(int32_t wid, int32_t iteration, const std::vector<std::string>& names,
                        const std::vector<at::Tensor>& grads, int64_t pulled_version) {
  TORCH_CHECK(names.size() == grads.size(), "psd: push names/grads length mismatch");
  PushResult r;
  r.iteration = iteration;
  std::lock_guard<std::mutex> g(mu_);
  r.total_workers = cfg_.total_workers;
  ctr_["pushes"] += 1;
  const bool compat_first = !init_ && cfg_.reference_compat;
  if (!init_ && !compat_first) {
    r.message = "parameters not initialised";
    ctr_["rejected"] += 1;
    return r;
  }
  if (compat_first && names_.empty()) {
    std::vector<std::vector<int64_t>> shp;
    for (auto& t : grads) shp.push_back(t.sizes().vec());
    layout_locked(names, shp);
    alloc_state_locked();
  }
  // Validate layout: the reference silently skipped mismatching tensors (D10).
  if (names.size() != names_.size()) {
    r.message = "tensor count mismatch: got " + std::to_string(names.size()) + ", expected " + std::to_string(names_.size());
    ctr_["rejected"] += 1;
    return r;
  }
  for (size_t i = 0; i < names.size(); ++i) {
    if (names[i] != names_[i] || grads[i].numel() != numels_[i]) {
      r.message = "tensor mismatch at index " + std::to_string(i) + " (" + names[i] + ")";
      ctr_["rejected"] += 1;
      return r;
    }
  }

  if (cfg_.async_mode) {
    // apply-on-arrival is not idempotent: a client retry of a push the server already applied
    // (its deadline expired after the apply) must not apply the gradient twice
    auto ck = clock_.find(wid);
    if (ck != clock_.end() && iteration < ck->second) {
      ctr_["duplicates"] += 1;
      r.success = true;
      r.aggregation_complete = true;
      r.version = version_;
      r.message = "duplicate push ignored: iteration already applied";
      return r;
    }
    const int32_t s = take_slot_locked();
    fill_slot_locked(slots_[s], names, grads);
    int64_t base = pulled_version >= 0 ? pulled_version
                                       : (pulled_version_.count(wid) ? pulled_version_[wid] : version_);
    const int64_t stale = std::max<int64_t>(0, version_ - base);
    const AsyncHyper ah = async_hyper(cfg_.opt_kind, cfg_.total_workers, cfg_.momentum, cfg_.beta1, cfg_.beta2,
                                      cfg_.weight_decay);
    const double lr0 = cfg_.lr * ah.lr_factor;
    const double lr = cfg_.staleness_lr_scaling ? lr0 / (1.0 + (double)stale) : lr0;
    const double scale = cfg_.async_grad_scale > 0 ? cfg_.async_grad_scale : ah.grad_scale;
    apply_locked({slots_[s]}, lr, scale, &ah);
    free_slots_.push_back(s);
    ++version_;
    hist_[std::min<int64_t>(stale, kHistBins - 1)] += 1;
    clock_[wid] = std::max(clock_[wid], iteration + 1);
    current_iteration_ = std::max(current_iteration_, iteration);
    r.success = true;
    r.aggregation_complete = true;
    r.workers_received = 1;
    r.version = version_;
    r.staleness = stale;
    r.message = "applied";
    cv_.notify_all();
    return r;
  }

  if (iteration < current_iteration_ - cfg_.window) {
    r.message = "iteration " + std::to_string(iteration) + " is outside the retained window";
    ctr_["rejected"] += 1;
    return r;
  }
  current_iteration_ = std::max(current_iteration_, iteration);
  IterState& st = iters_[iteration];
  if (st.aggregated) {
    // Idempotent like the reference, but reported (D9).
    ctr_["late_dropped"] += 1;
    r.success = true;
    r.aggregation_complete = true;
    r.workers_received = (int32_t)st.slot_of.size();
    r.version = version_;
    r.message = "late push ignored: iteration already aggregated";
    return r;
  }
  auto it = st.slot_of.find(wid);
  int32_t s = it != st.slot_of.end() ? it->second : take_slot_locked();
  st.slot_of[wid] = s;
  fill_slot_locked(slots_[s], names, grads);
  const int32_t received = (int32_t)st.slot_of.size();
  r.success = true;
  r.workers_received = received;
  if (received >= cfg_.total_workers) {
    std::vector<at::Tensor> srcs;
    for (auto& kv : st.slot_of) srcs.push_back(slots_[kv.second]);
    if (compat_first) {
      // reference quirk: the first aggregate *becomes* the parameters
      multi_reduce_(master_, srcs, 1.0 / received);
      init_ = true;
    } else {
      apply_locked(srcs, cfg_.reference_compat ? 1.0 : cfg_.lr, 1.0 / received);
    }
    for (auto& kv : st.slot_of) free_slots_.push_back(kv.second);
    st.slot_of.clear();
    st.aggregated = true;
    r.workers_received = received;
    ++version_;
    hist_[0] += 1;
    r.aggregation_complete = true;
    r.message = "aggregated";
    trim_locked();
    cv_.notify_all();
  } else {
    r.message = "waiting for " + std::to_string(cfg_.total_workers - received) + " more worker(s)";
    // remember the received count after the slots were recycled
  }
  r.version = version_;
  return r;
}

std::tuple<bool, int32_t, int32_t> PSCore::sync_status(int32_t iteration) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = iters_.find(iteration);
  if (it == iters_.end()) return {false, 0, cfg_.total_workers};
  const int32_t recv = it->second.aggregated ? cfg_.total_workers : (int32_t)it->second.slot_of.size();
  return {it->second.aggregated, recv, cfg_.total_workers};
}

std::tuple<bool, int32_t, int64_t, at::Tensor> PSCore::pull(int32_t wid, int32_t iteration, double wait_s) {
  std::unique_lock<std::mutex> lk(mu_);
  if (!init_ && wait_s > 0) cv_.wait_until(lk, deadline(wait_s), [&] { return init_; });
  if (!init_) return {false, current_iteration_, version_, at::Tensor()};
  bool ready = true;
  if (cfg_.async_mode) {
    if (cfg_.staleness_bound >= 0) {
      auto ok = [&] { return iteration - min_clock_locked() <= cfg_.staleness_bound; };
      if (wait_s > 0) cv_.wait_until(lk, deadline(wait_s), ok);
      ready = ok();
      if (!ready) ctr_["bound_timeouts"] += 1;
    }
  } else {
    auto agg = [&] {
      auto it = iters_.find(iteration);
      return (it != iters_.end() && it->second.aggregated) || iteration < current_iteration_ - cfg_.window;
    };
    if (wait_s > 0) cv_.wait_until(lk, deadline(wait_s), agg);
    ready = agg();
  }
  pulled_version_[wid] = version_;
  ctr_["pulls"] += 1;
  at::Tensor out = master_.to(at::kCPU, /*non_blocking=*/false, /*copy=*/true);
  return {ready, current_iteration_, version_, out};
}

void PSCore::set_total_workers(int32_t n) {
  TORCH_CHECK(n >= 1, "psd: total_workers must be >= 1");
  std::lock_guard<std::mutex> g(mu_);
  cfg_.total_workers = n;
  ctr_["membership_changes"] += 1;
  // A pending sync iteration that already holds >= n pushes completes now (a worker left).
  for (auto& kv : iters_) {
    IterState& st = kv.second;
    if (!st.aggregated && (int32_t)st.slot_of.size() >= n && !st.slot_of.empty()) {
      std::vector<at::Tensor> srcs;
      for (auto& w : st.slot_of) srcs.push_back(slots_[w.second]);
      apply_locked(srcs, cfg_.reference_compat ? 1.0 : cfg_.lr, 1.0 / (double)st.slot_of.size());
      for (auto& w : st.slot_of) free_slots_.push_back(w.second);
      st.slot_of.clear();
      st.aggregated = true;
      ++version_;
      hist_[0] += 1;
    }
  }
  cv_.notify_all();
}

void PSCore::forget_worker(int32_t wid) {
  std::lock_guard<std::mutex> g(mu_);
  clock_.erase(wid);
  pulled_version_.erase(wid);
  cv_.notify_all();
}

int32_t PSCore::total_workers() const {
  std::lock_guard<std::mutex> g(mu_);
  return cfg_.total_workers;
}
int32_t PSCore::current_iteration() const {
  std::lock_guard<std::mutex> g(mu_);
  return current_iteration_;
}
int64_t PSCore::version() const {
  std::lock_guard<std::mutex> g(mu_);
  return version_;
}
std::vector<int64_t> PSCore::staleness_histogram() const {
  std::lock_guard<std::mutex> g(mu_);
  return hist_;
}
std::map<std::string, int64_t> PSCore::counters() const {
  std::lock_guard<std::mutex> g(mu_);
  return ctr_;
}

bool PSCore::save_reference(const std::string& path, int32_t epoch) {
  std::lock_guard<std::mutex> g(mu_);
  if (!init_) return false;
  at::Tensor m = master_.to(at::kCPU);
  std::vector<at::Tensor> ts;
  for (size_t i = 0; i < names_.size(); ++i) ts.push_back(m.narrow(0, offsets_[i], numels_[i]));
  save_reference_ckpt(path, epoch, current_iteration_, names_, shapes_, ts);
  return true;
}

std::tuple<bool, int32_t> PSCore::load_reference(const std::string& path) {
  auto [epoch, iteration, names, shapes, dtypes, data] = load_reference_ckpt(path);
  std::lock_guard<std::mutex> g(mu_);
  layout_locked(names, shapes);
  alloc_state_locked();
  for (size_t i = 0; i < data.size(); ++i) {
    TORCH_CHECK(data[i].numel() == numels_[i], "psd: checkpoint tensor ", names[i], " numel disagrees with its shape");
    master_.narrow(0, offsets_[i], numels_[i]).copy_(data[i]);
  }
  iters_.clear();  // D8: stale iteration states are not carried over a load
  current_iteration_ = iteration;
  init_ = true;
  cv_.notify_all();
  return {true, epoch};
}

std::vector<at::Tensor> PSCore::state_tensors() const {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<at::Tensor> out{master_.to(at::kCPU), dyn_.to(at::kCPU)};
  if (s1_.defined()) out.push_back(s1_.to(at::kCPU));
  if (s2_.defined()) out.push_back(s2_.to(at::kCPU));
  return out;
}

void PSCore::load_state_tensors(const std::vector<at::Tensor>& ts, int32_t iteration, int64_t version) {
  std::lock_guard<std::mutex> g(mu_);
  TORCH_CHECK(init_ || !names_.empty(), "psd: load_state_tensors needs a layout (init_params first)");
  TORCH_CHECK(ts.size() >= 2 && ts[0].numel() == total_, "psd: state tensor layout mismatch");
  if (!master_.defined()) alloc_state_locked();
  master_.copy_(ts[0]);
  dyn_.copy_(ts[1]);
  size_t k = 2;
  if (s1_.defined() && k < ts.size()) s1_.copy_(ts[k++]);
  if (s2_.defined() && k < ts.size()) s2_.copy_(ts[k++]);
  current_iteration_ = iteration;
  version_ = version;
  iters_.clear();
  init_ = true;
  cv_.notify_all();
}

}  // namespace psd
