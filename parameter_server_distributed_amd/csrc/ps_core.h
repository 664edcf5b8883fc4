// Parameter-server shard core: one flat fp32 master (host or HBM), optimizer state, per-worker
// gradient inboxes, sync barrier / async apply-on-arrival with bounded staleness, version counters
// and a staleness histogram.
//
// Reference parity: ParameterServerCore (include/parameter_server.h:17-54,
// src/parameter_server.cpp:18-188):
//   receive_gradients  -> PSCore::push    (barrier over the *live* worker count, bounded window of
//                                           iteration states instead of an unbounded map: D3, D4)
//   aggregate_gradients-> fused_apply     (HIP kernel on device shards, same math on host)
//   serve_parameters   -> PSCore::pull    (versioned; async mode enforces the staleness bound)
//   check_sync_status  -> PSCore::sync_status
//   save/load_checkpoint -> reference format + native format (checkpoint.h)
// Lock order: a single mutex guards bookkeeping and the apply (the reference used
// state_mutex_ -> params_mutex_; one lock removes the D7 races on current_iteration_).
#pragma once
#include <ATen/ATen.h>

#include <condition_variable>
#include <cstdint>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <tuple>
#include <unordered_map>
#include <vector>

namespace psd {

struct AsyncHyper;  // async_hyper.h

struct PSConfig {
  int32_t total_workers = 1;
  int32_t async_mode = 0;        // 0 = sync barrier (reference), 1 = async apply-on-arrival
  int32_t staleness_bound = -1;  // async: max clock lead over the slowest worker (-1: unbounded)
  int32_t window = 64;           // sync: iteration states retained
  int32_t opt_kind = 0;          // OptimKind
  double lr = 1.0;
  double momentum = 0.0, dampening = 0.0, weight_decay = 0.0;
  double beta1 = 0.9, beta2 = 0.999, eps = 1e-8;
  bool nesterov = false;
  bool reference_compat = false;  // first aggregate becomes the params (src/parameter_server.cpp:78-81)
  bool staleness_lr_scaling = false;  // async: lr / (1 + staleness)
  double async_grad_scale = 0.0;      // async: per-push scale (0 -> 1/total_workers)
  double pull_timeout_s = 30.0;       // async: max wait for the staleness bound
};

struct PushResult {
  bool success = false;
  std::string message;
  int32_t iteration = 0;
  bool aggregation_complete = false;
  int32_t workers_received = 0;
  int32_t total_workers = 0;
  int64_t version = 0;
  int64_t staleness = 0;
};

class PSCore {
 public:
  PSCore(PSConfig cfg, std::string device);

  bool initialized() const;
  void init_params(const std::vector<std::string>& names, const std::vector<std::vector<int64_t>>& shapes,
                   const std::vector<at::Tensor>& values);
  std::vector<std::string> names() const;
  std::vector<std::vector<int64_t>> shapes() const;
  std::vector<int64_t> offsets() const;
  int64_t numel() const;

  PushResult push(int32_t worker_id, int32_t iteration, const std::vector<std::string>& names,
                  const std::vector<at::Tensor>& grads, int64_t pulled_version);
  // returns (ready, iteration, version, flat fp32 params on CPU; empty if uninitialised).
  // wait_s > 0: sync mode blocks until `iteration` is aggregated, async mode until the staleness
  // bound admits the worker (at most wait_s seconds either way).
  std::tuple<bool, int32_t, int64_t, at::Tensor> pull(int32_t worker_id, int32_t iteration, double wait_s);
  // returns (ready, workers_received, total_workers)
  std::tuple<bool, int32_t, int32_t> sync_status(int32_t iteration) const;

  void set_total_workers(int32_t n);
  void forget_worker(int32_t worker_id);  // elastic leave: drop its SSP clock
  int32_t total_workers() const;
  int32_t current_iteration() const;
  int64_t version() const;
  std::vector<int64_t> staleness_histogram() const;
  std::map<std::string, int64_t> counters() const;

  bool save_reference(const std::string& path, int32_t epoch);
  // returns (ok, epoch); on success iteration states are cleared (fixes D8)
  std::tuple<bool, int32_t> load_reference(const std::string& path);
  // full state (master, optimizer state, dyn) for the native checkpoint
  std::vector<at::Tensor> state_tensors() const;
  void load_state_tensors(const std::vector<at::Tensor>& ts, int32_t iteration, int64_t version);

 private:
  struct IterState {
    std::map<int32_t, int32_t> slot_of;  // worker -> inbox slot
    bool aggregated = false;
  };

  PSConfig cfg_;
  at::Device dev_;
  mutable std::mutex mu_;
  std::condition_variable cv_;

  std::vector<std::string> names_;
  std::vector<std::vector<int64_t>> shapes_;
  std::vector<int64_t> offsets_, numels_;
  int64_t total_ = 0;
  bool init_ = false;
  at::Tensor master_, s1_, s2_, dyn_;
  std::vector<at::Tensor> slots_;
  std::vector<int32_t> free_slots_;

  std::map<int32_t, IterState> iters_;
  int32_t current_iteration_ = 0;
  int64_t version_ = 0;
  std::unordered_map<int32_t, int64_t> pulled_version_;
  std::unordered_map<int32_t, int32_t> clock_;
  std::vector<int64_t> hist_;
  std::map<std::string, int64_t> ctr_;

  void layout_locked(const std::vector<std::string>& names, const std::vector<std::vector<int64_t>>& shapes);
  void alloc_state_locked();
  int32_t take_slot_locked();
  void fill_slot_locked(at::Tensor& slot, const std::vector<std::string>& names, const std::vector<at::Tensor>& grads);
  void apply_locked(const std::vector<at::Tensor>& sources, double lr, double grad_scale,
                    const AsyncHyper* ah = nullptr);
  void trim_locked();
  int32_t min_clock_locked() const;
};

}  // namespace psd
