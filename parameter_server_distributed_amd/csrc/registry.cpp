#include "registry.h"

#include <algorithm>
#include <chrono>

namespace psd {

// Timed waits use a system_clock deadline: libstdc++ then waits with pthread_cond_timedwait, which
// ThreadSanitizer intercepts (its steady_clock path, pthread_cond_clockwait, is invisible to the
// GCC 11 TSAN runtime and yields false "double lock" reports in tests/test_sanitizers.py).
static inline std::chrono::system_clock::time_point deadline(double seconds) {
  return std::chrono::system_clock::now() +
         std::chrono::duration_cast<std::chrono::system_clock::duration>(std::chrono::duration<double>(seconds));
}

static double mono_seconds() {
  using namespace std::chrono;
  return duration_cast<duration<double>>(steady_clock::now().time_since_epoch()).count();
}

Registry::Registry(std::string ps_host, int32_t ps_port) : ps_host_(std::move(ps_host)), ps_port_(ps_port) {}

double Registry::now_locked() const { return manual_clock_ ? manual_now_ : mono_seconds(); }

double Registry::now() const {
  std::lock_guard<std::mutex> g(mu_);
  return now_locked();
}

void Registry::use_manual_clock(double start) {
  std::lock_guard<std::mutex> g(mu_);
  manual_clock_ = true;
  manual_now_ = start;
}

void Registry::advance_clock(double dt) {
  std::lock_guard<std::mutex> g(mu_);
  manual_now_ += dt;
}

RegisterResult Registry::register_worker(int32_t id, const std::string& address, int32_t port,
                                         const std::string& hostname) {
  RegisterResult r;
  {
    std::lock_guard<std::mutex> g(mu_);
    const double t = now_locked();
    auto it = workers_.find(id);
    const bool fresh = it == workers_.end();
    WorkerEntry& e = workers_[id];
    e.worker_id = id;
    e.address = address.empty() ? "localhost" : address;
    e.port = port;
    e.hostname = hostname.empty() ? ("worker-" + std::to_string(id)) : hostname;
    e.last_heartbeat = t;
    if (fresh) {
      e.registered_at = t;
      ++epoch_;
      e.join_epoch = epoch_;
    }
    e.status = 0;
    r.success = true;
    r.message = fresh ? "registered" : "re-registered";
    r.ps_address = ps_host_ + ":" + std::to_string(ps_port_);
    r.total_workers = (int32_t)workers_.size();
    r.membership_epoch = epoch_;
  }
  cv_.notify_all();
  return r;
}

bool Registry::heartbeat(int32_t id, int32_t status) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = workers_.find(id);
  if (it == workers_.end()) return false;
  it->second.last_heartbeat = now_locked();
  it->second.status = status;
  return true;
}

bool Registry::deregister(int32_t id) {
  bool removed;
  {
    std::lock_guard<std::mutex> g(mu_);
    removed = workers_.erase(id) > 0;
    if (removed) ++epoch_;
  }
  if (removed) cv_.notify_all();
  return removed;
}

std::vector<WorkerEntry> Registry::list_workers() const {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<WorkerEntry> out;
  out.reserve(workers_.size());
  for (auto& kv : workers_) out.push_back(kv.second);
  std::sort(out.begin(), out.end(), [](const WorkerEntry& a, const WorkerEntry& b) { return a.worker_id < b.worker_id; });
  return out;
}

std::vector<int32_t> Registry::live_ids() const {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<int32_t> ids;
  for (auto& kv : workers_) ids.push_back(kv.first);
  std::sort(ids.begin(), ids.end());
  return ids;
}

std::tuple<std::string, int32_t> Registry::ps_address() const {
  std::lock_guard<std::mutex> g(mu_);
  return {ps_host_, ps_port_};
}

void Registry::set_ps_address(const std::string& host, int32_t port) {
  std::lock_guard<std::mutex> g(mu_);
  ps_host_ = host;
  ps_port_ = port;
}

std::vector<int32_t> Registry::remove_stale(double timeout_s) {
  std::vector<int32_t> removed;
  {
    std::lock_guard<std::mutex> g(mu_);
    const double t = now_locked();
    for (auto it = workers_.begin(); it != workers_.end();) {
      if (t - it->second.last_heartbeat > timeout_s) {
        removed.push_back(it->first);
        it = workers_.erase(it);
      } else {
        ++it;
      }
    }
    if (!removed.empty()) ++epoch_;
  }
  if (!removed.empty()) cv_.notify_all();
  std::sort(removed.begin(), removed.end());
  return removed;
}

int64_t Registry::membership_epoch() const {
  std::lock_guard<std::mutex> g(mu_);
  return epoch_;
}

int64_t Registry::wait_epoch_change(int64_t known, double timeout_s) {
  std::unique_lock<std::mutex> lk(mu_);
  cv_.wait_until(lk, deadline(timeout_s), [&] { return epoch_ != known; });
  return epoch_;
}

void Registry::set_shard(int32_t shard_id, const std::string& address, int32_t rank) {
  std::lock_guard<std::mutex> g(mu_);
  shards_[shard_id] = ShardInfo{shard_id, address, rank};
}

std::vector<ShardInfo> Registry::shards() const {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<ShardInfo> out;
  for (auto& kv : shards_) out.push_back(kv.second);
  return out;
}

void Registry::kv_set(const std::string& key, const std::string& value) {
  {
    std::lock_guard<std::mutex> g(mu_);
    kv_[key] = value;
  }
  cv_.notify_all();
}

std::tuple<bool, std::string> Registry::kv_get(const std::string& key, double timeout_s) {
  std::unique_lock<std::mutex> lk(mu_);
  cv_.wait_until(lk, deadline(timeout_s), [&] { return kv_.count(key) > 0; });
  auto it = kv_.find(key);
  if (it == kv_.end()) return {false, std::string()};
  return {true, it->second};
}

}  // namespace psd
