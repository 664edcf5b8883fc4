// Version counters + staleness histogram for the collective (RCCL) data plane.
// staleness of an applied gradient = shard version at apply - shard version the worker pulled
// (SURVEY.md §7.5.2). The reference has no versioning at all: pulls return "latest"
// (src/parameter_server.cpp:93-97).
#pragma once
#include <cstdint>
#include <map>
#include <mutex>
#include <utility>
#include <vector>

namespace psd {

class StalenessTracker {
 public:
  StalenessTracker(int num_shards, int bins) : versions_(num_shards, 0), hist_(bins, 0) {}

  void on_pull(int worker, int shard) {
    std::lock_guard<std::mutex> g(mu_);
    pulled_[{worker, shard}] = versions_.at(shard);
  }
  // returns the staleness recorded for this apply
  int64_t on_apply(int worker, int shard) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = pulled_.find({worker, shard});
    const int64_t base = it == pulled_.end() ? versions_.at(shard) : it->second;
    const int64_t s = versions_.at(shard) - base;
    hist_[s < (int64_t)hist_.size() ? s : hist_.size() - 1] += 1;
    versions_.at(shard) += 1;
    return s;
  }
  int64_t version(int shard) const {
    std::lock_guard<std::mutex> g(mu_);
    return versions_.at(shard);
  }
  std::vector<int64_t> histogram() const {
    std::lock_guard<std::mutex> g(mu_);
    return hist_;
  }
  // p in [0, 100]; -1 when empty
  int64_t percentile(double p) const {
    std::lock_guard<std::mutex> g(mu_);
    int64_t total = 0;
    for (auto c : hist_) total += c;
    if (total == 0) return -1;
    const double target = p / 100.0 * (double)total;
    int64_t acc = 0;
    for (size_t i = 0; i < hist_.size(); ++i) {
      acc += hist_[i];
      if ((double)acc >= target && acc > 0) return (int64_t)i;
    }
    return (int64_t)hist_.size() - 1;
  }
  void reset() {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& c : hist_) c = 0;
    pulled_.clear();
  }

 private:
  mutable std::mutex mu_;
  std::vector<int64_t> versions_;
  std::vector<int64_t> hist_;
  std::map<std::pair<int, int>, int64_t> pulled_;
};

}  // namespace psd
