// Coordinator core: worker registry, heartbeat expiry, membership epochs, PS shard map and a small
// rendezvous key/value store (used to hand the RCCL unique id to every rank).
//
// Reference parity: CoordinatorCore (include/coordinator.h:10-38, src/coordinator.cpp:7-67):
//   register_worker (upsert by id, stamp heartbeat)      -> Registry::register_worker
//   update_heartbeat (false for unknown ids)             -> Registry::heartbeat
//   list_workers                                          -> Registry::list_workers (+status, +epoch)
//   get_parameter_server_address                          -> Registry::ps_address (host and port kept
//                                                            separate and consistent: fixes D1/D2)
//   remove_stale_workers(timeout)                         -> Registry::remove_stale
// Additions: membership epoch (bumped on every join/leave/expiry) so the PS barrier and the RCCL
// communicator follow live membership (fixes D3); an injectable clock for deterministic expiry
// tests; a PS shard map for 1..N shards.
#pragma once
#include <condition_variable>
#include <cstdint>
#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <unordered_map>
#include <vector>

namespace psd {

struct WorkerEntry {
  int32_t worker_id = 0;
  std::string address;
  int32_t port = 0;
  std::string hostname;
  int32_t status = 0;  // coordinator.WorkerStatus: IDLE/TRAINING/CHECKPOINTING/ERROR
  double last_heartbeat = 0.0;
  double registered_at = 0.0;
  int64_t join_epoch = 0;
};

struct RegisterResult {
  bool success = false;
  std::string message;
  std::string ps_address;  // "host:port"
  int32_t total_workers = 0;
  int64_t membership_epoch = 0;
};

struct ShardInfo {
  int32_t shard_id = 0;
  std::string address;
  int32_t rank = -1;  // data-plane rank owning the shard (-1: gRPC-only PS)
};

class Registry {
 public:
  Registry(std::string ps_host, int32_t ps_port);

  RegisterResult register_worker(int32_t id, const std::string& address, int32_t port, const std::string& hostname);
  bool heartbeat(int32_t id, int32_t status);
  bool deregister(int32_t id);
  std::vector<WorkerEntry> list_workers() const;
  std::vector<int32_t> live_ids() const;
  std::tuple<std::string, int32_t> ps_address() const;
  void set_ps_address(const std::string& host, int32_t port);
  std::vector<int32_t> remove_stale(double timeout_s);
  int64_t membership_epoch() const;
  // Blocks until the epoch differs from `known` or the timeout (seconds) elapses; returns the epoch.
  int64_t wait_epoch_change(int64_t known, double timeout_s);

  void set_shard(int32_t shard_id, const std::string& address, int32_t rank);
  std::vector<ShardInfo> shards() const;

  void kv_set(const std::string& key, const std::string& value);
  // Returns (found, value); waits up to timeout_s for the key to appear.
  std::tuple<bool, std::string> kv_get(const std::string& key, double timeout_s);

  // Clock: real monotonic seconds unless a manual clock is enabled (tests).
  void use_manual_clock(double start);
  void advance_clock(double dt);
  double now() const;

 private:
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::string ps_host_;
  int32_t ps_port_;
  std::unordered_map<int32_t, WorkerEntry> workers_;
  std::map<int32_t, ShardInfo> shards_;
  std::unordered_map<std::string, std::string> kv_;
  int64_t epoch_ = 0;
  bool manual_clock_ = false;
  double manual_now_ = 0.0;
  double now_locked() const;
};

}  // namespace psd
