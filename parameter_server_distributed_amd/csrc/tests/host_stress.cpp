// Host-side concurrency stress for the std-only native cores, built with -fsanitize=thread (and
// separately address,undefined) by tests/test_sanitizers.py. The reference had documented data races
// (unlocked `initialized_` / `current_iteration_`) and no sanitizer build at all.
//
// Exercised concurrently: Registry register / heartbeat / deregister / remove_stale / list / kv
// (rendezvous) / wait_epoch_change, and StalenessTracker on_pull / on_apply / histogram.
#include <atomic>
#include <cstdio>
#include <string>
#include <thread>
#include <vector>

#include "../registry.h"
#include "../staleness.h"

int main() {
  psd::Registry reg("ps-host", 50051);
  psd::StalenessTracker st(4, 64);
  std::atomic<bool> stop{false};
  std::vector<std::thread> ts;
  for (int w = 0; w < 8; ++w) {
    ts.emplace_back([&, w] {
      for (int i = 0; i < 500; ++i) {
        reg.register_worker(w, "10.0.0." + std::to_string(w), 7000 + w, "");
        reg.heartbeat(w, i & 1);
        if (i % 50 == 0) reg.deregister(w);
        st.on_pull(w, i % 4);
        st.on_apply(w, i % 4);
        if (i % 100 == 0) reg.kv_set("k" + std::to_string(w), std::string(128, char('a' + w)));
      }
    });
  }
  ts.emplace_back([&] {
    while (!stop.load()) {
      reg.remove_stale(1e9);
      auto l = reg.list_workers();
      (void)l;
      (void)st.histogram();
      (void)st.percentile(50.0);
      reg.wait_epoch_change(reg.membership_epoch(), 0.001);
    }
  });
  ts.emplace_back([&] {
    for (int i = 0; i < 200; ++i) {
      auto r = reg.kv_get("k3", 0.001);
      (void)r;
    }
  });
  for (int i = 0; i < 8; ++i) ts[i].join();  // workers
  ts[9].join();                               // kv reader
  stop.store(true);
  ts[8].join();                               // monitor
  int64_t total = 0;
  for (auto c : st.histogram()) total += c;
  std::printf("ok epochs=%lld applies=%lld\n", (long long)reg.membership_epoch(), (long long)total);
  return total == 8 * 500 ? 0 : 1;
}
