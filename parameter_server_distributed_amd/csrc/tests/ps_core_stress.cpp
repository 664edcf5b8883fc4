// PSCore (the C1 ParameterServerCore counterpart: mutex + condition variable + slot pool + version
// / SSP clocks) under concurrency, on CPU tensors, built with -fsanitize=thread and separately
// address,undefined by tests/test_sanitizers.py. The reference's D7 was exactly this kind of state
// (unlocked current_iteration_ read from the checkpoint thread, include/parameter_server.h:37).
//
// Concurrently: 4 workers push + pull (sync barrier mode, then async apply-on-arrival with an SSP
// bound), a monitor thread reads sync_status / counters / version / histogram / total_workers and
// writes reference-format checkpoints (the periodic-checkpoint thread of the PS service), and a
// membership thread calls set_total_workers / forget_worker.
#include <ATen/ATen.h>
#include <ATen/Parallel.h>

#include <atomic>
#include <cstdio>
#include <string>
#include <thread>
#include <unistd.h>
#include <vector>

#include "../kernels/launchers.h"
#include "../ps_core.h"

using namespace psd;

static int run(bool async_mode) {
  const int W = 4, N = 40;
  PSConfig c;
  c.total_workers = W;
  c.async_mode = async_mode ? 1 : 0;
  c.staleness_bound = async_mode ? 2 : -1;
  c.opt_kind = OPT_MOMENTUM;
  c.lr = 0.05;
  c.momentum = 0.9;
  PSCore ps(c, "cpu");
  std::vector<std::string> names{"w", "b"};
  std::vector<std::vector<int64_t>> shapes{{16, 8}, {8}};
  ps.init_params(names, shapes, {at::zeros({16, 8}), at::ones({8})});
  std::atomic<bool> stop{false};
  std::atomic<int> failures{0};
  std::vector<std::thread> ts;
  for (int w = 0; w < W; ++w) {
    ts.emplace_back([&, w] {
      for (int it = 0; it < N; ++it) {
        // sync: wait for the previous iteration's aggregate (the barrier); async: the SSP bound
        auto pr = ps.pull(w, async_mode ? it : it - 1, 10.0);
        if (!std::get<0>(pr) && (async_mode || it > 0)) failures++;
        std::vector<at::Tensor> g{at::full({16, 8}, 0.01f * (w + 1)), at::full({8}, 0.02f)};
        auto r = ps.push(w, it, names, g, std::get<2>(pr));
        if (!r.success) failures++;
      }
    });
  }
  ts.emplace_back([&] {  // monitor + periodic checkpoint
    // per-process path: the sanitizer variants of this binary run concurrently under pytest-xdist
    const std::string path = std::string("/tmp/psd_stress_") + (async_mode ? "a" : "s") + "_" +
                             std::to_string(static_cast<long>(getpid())) + ".ckpt";
    int k = 0;
    while (!stop.load()) {
      (void)ps.sync_status(ps.current_iteration());
      (void)ps.counters();
      (void)ps.version();
      (void)ps.staleness_histogram();
      (void)ps.total_workers();
      if (++k % 16 == 0) ps.save_reference(path, k);
      std::this_thread::yield();
    }
    std::remove(path.c_str());
  });
  ts.emplace_back([&] {  // membership churn that keeps the barrier size at W
    for (int i = 0; i < 200 && !stop.load(); ++i) {
      ps.set_total_workers(W);
      if (async_mode && i % 50 == 0) ps.forget_worker(W + 7);  // an id that never pushed
      std::this_thread::yield();
    }
  });
  for (int w = 0; w < W; ++w) ts[w].join();
  stop.store(true);
  ts[W].join();
  ts[W + 1].join();
  const int64_t want = async_mode ? (int64_t)W * N : N;
  std::printf("%s ok version=%lld failures=%d\n", async_mode ? "async" : "sync", (long long)ps.version(),
              failures.load());
  return (ps.version() == want && failures.load() == 0) ? 0 : 1;
}

int main() {
  at::set_num_threads(1);  // keep libtorch's (uninstrumented) OpenMP pool out of the picture
  int rc = run(false);
  rc |= run(true);
  std::printf("ok pscore\n");
  return rc;
}
