// AsyncEngine (csrc/async_ps.cpp) under concurrency on host memory, for -fsanitize=thread and
// address,undefined (tests/test_sanitizers.py). Rank 0 is the only worker and owns 2 shards: its
// training thread pulls / pushes / commits while the engine thread applies each push on arrival
// (shared-memory rings, reader pins, version / clock atomics), and a monitor thread reads
// versions / clocks / histogram / counters.
#include <ATen/ATen.h>
#include <ATen/Parallel.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <thread>

#include "../async_ps.h"
#include "../kernels/launchers.h"

using namespace psd;

int main() {
  at::set_num_threads(1);
  const int64_t n = 4096, S = 1, steps = 300;
  const std::string shm = "/psd_tsan_" + std::to_string(getpid());
  AsyncEngine e(0, 1, {0, 0}, {0}, {0, n / 2}, {n / 2, n / 2}, (int)S, 4, shm, true, -1, 60.0, 4);
  e.attach_peer(0, e.local_desc());
  at::Tensor params = at::zeros({n});
  std::vector<at::Tensor> master, st1, dyn;
  for (int k = 0; k < 2; ++k) {
    master.push_back(at::zeros({n / 2}));
    st1.push_back(at::zeros({n / 2}));
    dyn.push_back(at::zeros({8}, at::kInt));
    reinterpret_cast<float*>(dyn.back().data_ptr<int32_t>())[0] = 0.01f;  // lr
    reinterpret_cast<float*>(dyn.back().data_ptr<int32_t>())[1] = 1.0f;   // grad scale
    e.set_shard_state(k, master[k], st1[k], c10::nullopt, dyn[k], OPT_MOMENTUM, 0.9, 0.0, false, 0.0, 0.9, 0.999,
                      1e-8);
    e.publish_initial(k);
  }
  e.enable_log(true);
  e.start();
  std::atomic<bool> stop{false};
  std::thread mon([&] {
    while (!stop.load()) {
      (void)e.version(0);
      (void)e.clocks(1);
      (void)e.histogram();
      (void)e.counters();
      (void)e.error();
      std::this_thread::yield();
    }
  });
  at::Tensor g = at::ones({n});
  for (int64_t t = 0; t < steps; ++t) {
    auto pulled = e.pull(t, params, 0);
    e.push(t, g, 0, n / 2, 0);
    e.push(t, g, n / 2, n, 0);
    e.commit(t, pulled, 0);
  }
  e.wait_all_applied(steps);
  stop.store(true);
  mon.join();
  e.stop();
  const auto log = e.apply_log();
  std::printf("ok async applies=%zu v0=%lld v1=%lld err='%s'\n", log.size(), (long long)e.version(0),
              (long long)e.version(1), e.error().c_str());
  if (e.version(0) != steps || e.version(1) != steps) return 1;
  e.close_peers();
  e.free_local();
  return (log.size() == (size_t)(2 * steps)) ? 0 : 1;
}
