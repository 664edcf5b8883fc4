// Asynchronous parameter-server data plane: apply-on-arrival with bounded staleness (SSP) over
// xGMI peer memory, no collectives.
//
// The reference PS handles each worker's push as it arrives (src/parameter_server.cpp:18-75) but
// then waits for all `total_workers` before applying (:37) -- it has no asynchronous mode. Here
// every PS shard applies each worker's gradient the moment it lands, and a worker only waits when
// it would lead the slowest worker by more than S steps (stale-synchronous parallel).
//
// MI355X design (one process per GPU, one node, 7 xGMI links per GPU):
//   * Each shard owner allocates, in its own HBM, a gradient *inbox* (one slot ring of S+1 slices
//     per worker) and NB *publish* buffers (bf16 snapshots of its shard). Both are uncached
//     fine-grained memory exported with hipIpcGetMemHandle and mapped by every peer
//     (hipIpcOpenMemHandle + lazy peer access), so a peer's DMA write or read is coherent without
//     any cache maintenance on the owner.
//   * push: a worker DMA-copies its gradient slice straight into its inbox slot on the owner's GPU
//     (hipMemcpyAsync over the direct xGMI link to that peer), then posts a message to a
//     single-producer ring in a shared-memory control block once the copy has completed.
//   * apply: the owner's engine thread (C++, no GIL) polls the rings and gathers the arriving pushes
//     into rounds of K (any workers, in arrival order; set_round). A complete round launches the
//     fused gfx950 optimizer kernel on its PS stream: the K inbox slots summed in registers, scaled
//     by 1/K -> fp32 master / state -> bf16 written into a free publish buffer. When the kernel
//     completes the buffer becomes the shard's latest snapshot, the shard version advances by one,
//     the clock of every worker in the round advances, and each push's staleness (versions applied
//     since the snapshot its gradient was computed on) is recorded exactly. K = W is K-batch-async
//     SGD ("round" semantics: at SSP bound 0 the rounds are exactly the synchronous steps); K = 1
//     applies every push on arrival ("push" semantics).
//   * pull: a worker waits until every worker's clock at every shard is >= step - S (SSP), pins
//     the latest publish buffer (reader count), DMA-copies it into its working weights and
//     unpins when the copy completes.
// No GPU kernel ever waits on another process (no spinning collective kernels that could
// interlock through shared hardware queues); every host wait has a deadline and reports an
// error instead of hanging. Liveness: every engine thread stamps a heartbeat in the control block;
// a peer silent for PSD_ASYNC_DEAD_S (10 s) -- a killed or hung process -- sets the shared error,
// so every rank's SSP wait fails within seconds instead of at the 600 s deadline. With device = -1 the same protocol runs on host memory in POSIX
// shared memory (CPU CI, gloo plumbing config).
#pragma once
#include <ATen/ATen.h>

#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "kernels/launchers.h"

namespace psd {

struct AsyncCtl;  // shared-memory control block (async_ps.cpp)

class AsyncEngine {
 public:
  AsyncEngine(int rank, int world, std::vector<int> owners, std::vector<int> workers, std::vector<int64_t> shard_off,
              std::vector<int64_t> shard_len, int staleness, int nbuf, std::string shm_name, bool create, int device,
              double timeout_s, int elem_bytes = 2, bool mx = false);
  ~AsyncEngine();

  // -- memory exchange (collective through the caller's store) --
  std::string local_desc() const;                  // how peers map this rank's inbox/publish memory
  void attach_peer(int rank, const std::string& desc);

  // -- owner side --
  void set_shard_state(int shard, at::Tensor master, c10::optional<at::Tensor> state1, c10::optional<at::Tensor> state2,
                       at::Tensor dyn, int64_t kind, double momentum, double dampening, bool nesterov,
                       double weight_decay, double beta1, double beta2, double eps);
  // bf16(master) -> publish buffer 0 as the shard's snapshot `version` (blocking); with `clocks`
  // (one per worker) the SSP clocks are restored too (checkpoint resume)
  void publish_initial(int shard, int64_t version = 0, std::vector<int64_t> clocks = {});
  void set_round(int k);            // pushes per optimizer step (1..W); before start()
  // fixed schedule (before start(); needs K = W and nbuf >= S + 2): round r holds exactly every
  // worker's step-r push and a pull of step t takes exactly version max(t - S, base). The staleness
  // is then S for every gradient after the first S steps, independent of timing: the trajectory
  // is synchronous SGD with S-step-delayed gradients, bit-for-bit reproducible (tests, debugging).
  void set_fixed_schedule(bool on);
  void start();
  void stop();
  // teardown in two collective phases (barrier between): unmap the peers' memory, then free our
  // own -- explicitly, before interpreter exit tears the HIP runtime down
  void close_peers();
  void free_local();

  // -- worker side --
  std::vector<int64_t> pull(int64_t step, at::Tensor params_flat, int64_t stream);
  // MX engines: the e4m3 snapshot + E8M0 scales into (q_flat, sc_flat) instead of the bf16 one, and
  // dequantised into the bf16 working weights `out`
  std::vector<int64_t> pull_mx(int64_t step, at::Tensor q_flat, at::Tensor sc_flat, at::Tensor out, int64_t stream);
  // push / pull transport: true (GPU default) = one scatter / gather kernel per push / pull over
  // every owner's peer memory at once (kernels/xfer.hip); false = one hipMemcpyAsync per shard
  void set_xfer(bool kernel);
  std::string xfer_mode() const;
  // workgroups per segment of one scatter / gather launch (cap; default 48): the budget of CUs a
  // push may take from the backward pass running beside it (bench.py probes it at N > 1)
  void set_xfer_blocks(int cap);
  int xfer_blocks_cap() const { return xfer_cap_; }
  void push(int64_t step, const at::Tensor& grads_flat, int64_t lo, int64_t hi, int64_t stream);
  void commit(int64_t step, std::vector<int64_t> pulled, int64_t stream);
  void wait_applied(int64_t nsteps);  // this worker's pushes 0..nsteps-1 applied at every shard
  void wait_all_applied(int64_t nsteps);  // every worker's pushes 0..nsteps-1 applied at every shard

  // this rank's inbox slot of worker index wi at shard (owner side; start-up self-test)
  at::Tensor inbox_view(int shard, int wi, int slot) const;

  // -- introspection --
  std::vector<int64_t> histogram() const;  // staleness of the applies this process performed
  int64_t version(int shard) const;
  std::vector<int64_t> clocks(int shard) const;
  std::vector<int> my_shards() const { return my_shards_; }
  std::string memory_kind() const { return mem_kind_; }
  std::string error() const;
  // fail every rank's waits now (an external failure detector, e.g. the coordinator expired a peer)
  void inject_error(const std::string& msg);
  std::vector<int64_t> counters() const;  // applies, pushes posted, pulls, pull waits (us)
  // completed applies in order: (shard, worker rank, step, staleness, version after) -- for tests
  // and replay; recorded only after enable_log()
  void enable_log(bool on) { log_on_ = on; }
  std::vector<std::vector<int64_t>> apply_log() const;

 private:
  struct RoundItem {
    int wi, slot;
    int64_t step, pulled, staleness;
  };
  struct Pending {
    int shard, buf;
    std::vector<RoundItem> items;
    void* event;  // hipEvent_t (GPU)
  };
  struct Action {
    void* event;  // completion of the copies this action waits for (GPU), null = immediate
    std::function<void()> fn;
  };
  struct ShardState {
    at::Tensor master, s1, s2, dyn;
    OptimHyper hyper{};
    std::vector<at::Tensor> inbox;    // [workers * (S+1)] bf16 views
    std::vector<at::Tensor> publish;  // [nbuf] bf16 views
    std::vector<bool> busy;           // publish buffer is the target of an enqueued apply
    int64_t enq = 0;                  // applies enqueued (the version the next apply starts from)
    std::vector<RoundItem> round;     // pushes taken from the mailboxes, not yet applied
    std::vector<at::Tensor> acc;      // fp32 group sums (rounds of more than 16 pushes)
  };

  void quant_publish(ShardState& st, int shard, int buf, void* stream);
  int64_t slot_elems(int shard) const { return shard_len_[shard]; }
  int64_t region_bytes_for(int rank) const;
  int64_t pub_slot_bytes(int shard) const;
  int64_t shard_region_bytes(int shard) const;
  char* publish_q_ptr(int shard, int buf) const;
  char* publish_sc_ptr(int shard, int buf) const;
  std::vector<int64_t> pull_impl(int64_t step, char* dst, char* dst_sc, uint16_t* dst_bf16, int64_t stream);
  int64_t shard_base(int rank, int shard) const;  // byte offset of shard's region in rank's allocation
  char* inbox_ptr(int shard, int wi, int slot) const;
  char* publish_ptr(int shard, int buf) const;
  void apply_into(ShardState& st, const std::vector<at::Tensor>& g, int buf);
  int free_buf(int shard) const;
  bool claim_buf(int shard, int b);
  static bool done(void* event);
  void run();
  bool poll_once();
  void check_error() const;
  void check_peers(int64_t now_us);
  void fail(const std::string& msg);
  void copy(void* dst, const void* src, int64_t bytes, void* stream);
  void defer(void* stream, std::function<void()> fn);
  void post(int shard, int wi, int64_t step, int64_t pulled);
  int worker_index(int rank) const;

  int rank_, world_, S_, nbuf_, device_;
  int round_ = 1;
  bool fixed_ = false;
  bool xfer_kernel_ = false;  // set in the constructor: true on a GPU engine
  int xfer_cap_ = 48;         // set_xfer_blocks
  int apply_cap_ = 0;         // fused-apply workgroups (0: the launcher's 2048); see the constructor
  double timeout_s_;
  double dead_after_s_ = 10.0;  // a peer's engine silent this long is presumed dead (PSD_ASYNC_DEAD_S)
  int esz_;
  bool mx_ = false;  // MX fp8 publish: each publish slot also holds e4m3 + E8M0 scales of the snapshot
  std::vector<int> owners_, workers_, my_shards_;
  std::vector<int64_t> shard_off_, shard_len_;
  int my_wi_ = -1;
  std::string shm_name_;
  bool created_ = false;
  AsyncCtl* ctl_ = nullptr;
  size_t ctl_bytes_ = 0;
  std::string mem_kind_;

  // this rank's inbox/publish memory and the peers' mappings
  void* local_mem_ = nullptr;
  int64_t local_bytes_ = 0;
  std::string local_shm_;
  std::vector<char*> peer_base_;      // per rank: base pointer of its allocation in this process
  std::vector<bool> peer_ipc_;        // mapped through hipIpcOpenMemHandle (must be closed)
  std::vector<int64_t> peer_bytes_;

  std::vector<ShardState> shards_;  // indexed by shard id (only owned ones are populated)
  void* ps_stream_ = nullptr;       // hipStream_t of the apply kernels

  std::thread thr_;
  std::atomic<bool> stop_{false};
  bool running_ = false;
  std::deque<Pending> pending_;
  std::mutex act_mu_;
  std::deque<Action> actions_;
  std::vector<int64_t> hist_;
  bool log_on_ = false;
  std::vector<std::vector<int64_t>> log_;
  mutable std::mutex hist_mu_;
  std::atomic<int64_t> n_applies_{0}, n_posts_{0}, n_pulls_{0}, wait_us_{0};
};

}  // namespace psd
