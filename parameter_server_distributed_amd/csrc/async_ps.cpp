#include "async_ps.h"

#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <fcntl.h>
#include <hip/hip_runtime_api.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <sstream>

#include "kernels/launchers.h"
#include "kernels/launchers_xfer.h"
#include "ops.h"

namespace psd {

namespace {

constexpr uint64_t kMagic = 0x5053444153594e43ull;  // "PSDASYNC"
constexpr int kMaxShards = 64, kMaxWorkers = 64, kRing = 16, kMaxBuf = 8, kBins = 64, kMaxRanks = 128;
constexpr int64_t kHbLeft = -1;  // heartbeat slot of a rank whose engine stopped on purpose
constexpr int64_t kAlignBytes = 256;

struct Msg {
  int64_t step;
  int64_t pulled;  // shard version the gradient was computed on
};

struct alignas(64) Mailbox {  // single producer (worker wi) -> single consumer (owner of shard k)
  std::atomic<int64_t> head;
  char pad0[56];
  std::atomic<int64_t> tail;
  char pad1[56];
  Msg ring[kRing];
};

struct alignas(64) ShardCtl {
  std::atomic<int64_t> version;  // applies completed
  std::atomic<int32_t> latest;   // publish buffer holding `version`
  int32_t pad;
  std::atomic<int64_t> base_version;  // the version publish_initial published (fixed-schedule pulls)
  std::atomic<int64_t> buf_version[kMaxBuf];
  std::atomic<int32_t> readers[kMaxBuf];
  std::atomic<int64_t> clock[kMaxWorkers];  // pushes of worker wi applied at this shard
};

static_assert(std::atomic<int64_t>::is_always_lock_free, "cross-process atomics need lock-free int64");

}  // namespace

struct AsyncCtl {
  std::atomic<uint64_t> magic;
  std::atomic<int32_t> error;
  int32_t pad;
  char msg[512];
  // liveness: each rank's engine thread stamps its slot (steady-clock us, one clock for every
  // process of the node) every few ms; a peer silent for dead_after_s is presumed dead
  std::atomic<int64_t> hb_us[kMaxRanks];
  ShardCtl shard[kMaxShards];
  Mailbox mb[kMaxShards][kMaxWorkers];
};

namespace {

inline void hip_ok(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, "psd async: ", what, " failed: ", hipGetErrorString(e));
}

int64_t round_up(int64_t x, int64_t a) { return (x + a - 1) / a * a; }

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int64_t now_us() {
  return std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// Spin-wait backoff of the engine's host waits (SSP pulls, commit events, inbox flags): yields,
// then 20 us sleeps for the first ~1 s of a wait, 200 us after. (A wait the GPU ends -- a worker's
// pull for the next step waiting on this step's commit -- typically lasts 10-20 ms: with 200 us
// sleeps from ~20 ms on, it woke up to 200 us late, and the step boundary's GPU idle grew by that.)
void backoff(int& spins) {
  if (++spins < 64) {
    std::this_thread::yield();
  } else {
    std::this_thread::sleep_for(std::chrono::microseconds(spins < 50000 ? 20 : 200));
  }
}

void* map_shm(const std::string& name, size_t bytes, bool create) {
  int fd = shm_open(name.c_str(), create ? (O_CREAT | O_EXCL | O_RDWR) : O_RDWR, 0600);
  TORCH_CHECK(fd >= 0, "psd async: shm_open(", name, ") failed: ", std::strerror(errno));
  if (create) TORCH_CHECK(ftruncate(fd, (off_t)bytes) == 0, "psd async: ftruncate failed: ", std::strerror(errno));
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  TORCH_CHECK(p != MAP_FAILED, "psd async: mmap(", name, ") failed: ", std::strerror(errno));
  return p;
}

}  // namespace

namespace {
// utils/config.py FEATURES for the native side: PSD_FEATURES="name=0|1,..." (else the default)
bool psd_feature_on(const char* name, bool dflt) {
  const char* env = std::getenv("PSD_FEATURES");
  if (!env) return dflt;
  const std::string all(env), key(name);
  size_t pos = 0;
  while (pos <= all.size()) {
    const size_t end = std::min(all.find(',', pos), all.size());
    const std::string item = all.substr(pos, end - pos);
    const size_t eq = item.find('=');
    auto trim = [](std::string t) {
      const size_t a = t.find_first_not_of(" \t"), b = t.find_last_not_of(" \t");
      return a == std::string::npos ? std::string() : t.substr(a, b - a + 1);
    };
    if (trim(item.substr(0, eq)) == key) {
      const std::string v = eq == std::string::npos ? "1" : trim(item.substr(eq + 1));
      return !(v == "0" || v == "false" || v == "off" || v == "no");
    }
    pos = end + 1;
  }
  return dflt;
}
}  // namespace

AsyncEngine::AsyncEngine(int rank, int world, std::vector<int> owners, std::vector<int> workers,
                         std::vector<int64_t> shard_off, std::vector<int64_t> shard_len, int staleness, int nbuf,
                         std::string shm_name, bool create, int device, double timeout_s, int elem_bytes, bool mx)
    : rank_(rank),
      world_(world),
      S_(staleness),
      nbuf_(nbuf),
      device_(device),
      timeout_s_(timeout_s),
      esz_(elem_bytes),
      mx_(mx),
      owners_(std::move(owners)),
      workers_(std::move(workers)),
      shard_off_(std::move(shard_off)),
      shard_len_(std::move(shard_len)),
      shm_name_(std::move(shm_name)),
      hist_(kBins, 0) {
  const int P = (int)owners_.size(), W = (int)workers_.size();
  TORCH_CHECK(P >= 1 && P <= kMaxShards, "psd async: 1..", kMaxShards, " shards");
  TORCH_CHECK(W >= 1 && W <= kMaxWorkers, "psd async: 1..", kMaxWorkers, " workers");
  TORCH_CHECK(S_ >= 0 && S_ + 1 <= kRing, "psd async: staleness bound must be in [0, ", kRing - 1, "]");
  if (mx_) {
    TORCH_CHECK(device >= 0 && esz_ == 2, "psd async: the MX fp8 publish needs a GPU engine with bf16 weights");
    for (int k = 0; k < P; ++k)
      TORCH_CHECK(shard_off_[k] % 32 == 0 && shard_len_[k] % 32 == 0,
                  "psd async: MX shards must be 32-element aligned");
  }
  TORCH_CHECK(nbuf_ >= 2 && nbuf_ <= kMaxBuf, "psd async: 2..", kMaxBuf, " publish buffers");
  TORCH_CHECK(esz_ == 2 || esz_ == 4, "psd async: bf16 (2) or fp32 (4) elements");
  TORCH_CHECK(world_ >= 1 && world_ <= kMaxRanks, "psd async: 1..", kMaxRanks, " ranks");
  if (const char* e = getenv("PSD_ASYNC_DEAD_S")) dead_after_s_ = atof(e);
  TORCH_CHECK((int)shard_off_.size() == P && (int)shard_len_.size() == P, "psd async: shard ranges per owner");
  for (int k = 0; k < P; ++k) {
    TORCH_CHECK(owners_[k] >= 0 && owners_[k] < world_, "psd async: bad owner rank");
    if (owners_[k] == rank_) my_shards_.push_back(k);
  }
  my_wi_ = worker_index(rank_);

  // control block
  ctl_bytes_ = sizeof(AsyncCtl);
  if (create) {
    shm_unlink(shm_name_.c_str());
    ctl_ = static_cast<AsyncCtl*>(map_shm(shm_name_, ctl_bytes_, true));
    std::memset(static_cast<void*>(ctl_), 0, ctl_bytes_);
    ctl_->magic.store(kMagic);
    created_ = true;
  } else {
    ctl_ = static_cast<AsyncCtl*>(map_shm(shm_name_, ctl_bytes_, false));
    TORCH_CHECK(ctl_->magic.load() == kMagic, "psd async: control block ", shm_name_, " not initialised");
  }

  // this rank's inbox + publish memory
  local_bytes_ = region_bytes_for(rank_);
  peer_base_.assign(world_, nullptr);
  peer_ipc_.assign(world_, false);
  peer_bytes_.assign(world_, 0);
  if (local_bytes_ > 0) {
    if (device_ >= 0) {
      const c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device_));
      // uncached fine-grained: peers' DMA writes / reads are coherent without cache maintenance.
      // A world of one has no peer: plain device memory there (feature async_cached_local) -- the
      // pushes / pulls and the owner's apply then run at cached-HBM speed instead of the ~0.2 TB/s a
      // copy into uncached memory gets (BERT-base: 14 push copies of 16 MB, 74 us each)
      hipError_t e = hipErrorUnknown;
      if (world_ == 1 && psd_feature_on("async_cached_local", true)) {
        e = hipMalloc(&local_mem_, (size_t)local_bytes_);
        mem_kind_ = "device";
      }
      if (e != hipSuccess) {
        (void)hipGetLastError();
        e = hipExtMallocWithFlags(&local_mem_, (size_t)local_bytes_, hipDeviceMallocUncached);
        mem_kind_ = "uncached";
      }
      if (e != hipSuccess) {
        (void)hipGetLastError();
        e = hipExtMallocWithFlags(&local_mem_, (size_t)local_bytes_, hipDeviceMallocFinegrained);
        mem_kind_ = "finegrained";
      }
      hip_ok(e, "hipExtMallocWithFlags(inbox/publish)");
      hip_ok(hipMemset(local_mem_, 0, (size_t)local_bytes_), "hipMemset");
    } else {
      std::ostringstream nm;
      nm << shm_name_ << "_m" << rank_;
      local_shm_ = nm.str();
      shm_unlink(local_shm_.c_str());
      local_mem_ = map_shm(local_shm_, (size_t)local_bytes_, true);
      std::memset(local_mem_, 0, (size_t)local_bytes_);
      mem_kind_ = "host-shm";
    }
    peer_base_[rank_] = static_cast<char*>(local_mem_);
    peer_bytes_[rank_] = local_bytes_;
  }

  shards_.resize(P);
  const auto opt = at::TensorOptions()
                       .dtype(esz_ == 2 ? at::kBFloat16 : at::kFloat)
                       .device(device_ >= 0 ? c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device_)
                                            : c10::Device(c10::kCPU));
  for (int k : my_shards_) {
    ShardState& st = shards_[k];
    for (int wi = 0; wi < W; ++wi)
      for (int s = 0; s <= S_; ++s) st.inbox.push_back(at::from_blob(inbox_ptr(k, wi, s), {shard_len_[k]}, opt));
    for (int b = 0; b < nbuf_; ++b) st.publish.push_back(at::from_blob(publish_ptr(k, b), {shard_len_[k]}, opt));
    st.busy.assign(nbuf_, false);
  }
  if (device_ >= 0) {
    // With an SSP bound S >= 1 a round's apply has a whole worker step of slack (the pull that needs
    // it comes one step later), so it runs in the background: a normal-priority stream and at most
    // 2 workgroups per CU. A high-priority, 2048-workgroup apply took every CU slot for its ~0.85 ms
    // and held back the compute stream's next kernels (the gradient-zeroing fills waited up to
    // 215 us for a slot in a BERT-base kernel trace; step time neutral within the box spread in
    // plain runs, profiles/r6/boundary/README.md). At S = 0 the apply is on the critical path:
    // high priority, full grid.
    const bool bg = S_ >= 1 && psd_feature_on("async_apply_background", true);
    apply_cap_ = bg ? 512 : 0;
    ps_stream_ = c10::hip::getStreamFromPool(/*isHighPriority=*/!bg, (c10::DeviceIndex)device_).stream();
    xfer_kernel_ = true;
  }
}

AsyncEngine::~AsyncEngine() {
  try {
    stop();
  } catch (...) {
  }
  close_peers();
  free_local();
}

void AsyncEngine::close_peers() {
  for (int r = 0; r < world_; ++r) {
    if (r == rank_ || !peer_base_[r]) continue;
    if (peer_ipc_[r]) (void)hipIpcCloseMemHandle(peer_base_[r]);
    else munmap(peer_base_[r], (size_t)peer_bytes_[r]);
    peer_base_[r] = nullptr;
  }
}

void AsyncEngine::free_local() {
  // callers: stop() first, and every peer has closed its mapping (Python barrier in between)
  shards_.clear();
  if (local_mem_) {
    if (device_ >= 0) (void)hipFree(local_mem_);
    else {
      munmap(local_mem_, (size_t)local_bytes_);
      shm_unlink(local_shm_.c_str());
    }
    local_mem_ = nullptr;
    if (rank_ < (int)peer_base_.size()) peer_base_[rank_] = nullptr;
  }
  {
    std::lock_guard<std::mutex> g(act_mu_);
    for (auto& a : actions_)
      if (a.event) (void)hipEventDestroy(static_cast<hipEvent_t>(a.event));
    actions_.clear();
  }
  if (ctl_) {
    munmap(static_cast<void*>(ctl_), ctl_bytes_);
    if (created_) shm_unlink(shm_name_.c_str());
    ctl_ = nullptr;
  }
}

// ------------------------------------------------------------------ layout
int AsyncEngine::worker_index(int rank) const {
  for (size_t i = 0; i < workers_.size(); ++i)
    if (workers_[i] == rank) return (int)i;
  return -1;
}

// A shard's region: W * (S + 1) inbox slots, then nbuf publish slots; with MX a publish slot also
// holds the e4m3 copy of the snapshot and its E8M0 scales (one per 32 elements) after the bf16 one.
int64_t AsyncEngine::pub_slot_bytes(int shard) const {
  const int64_t sb = round_up(shard_len_[shard] * esz_, kAlignBytes);
  if (!mx_) return sb;
  return sb + round_up(shard_len_[shard], kAlignBytes) + round_up(shard_len_[shard] / 32, kAlignBytes);
}

int64_t AsyncEngine::shard_region_bytes(int shard) const {
  return (int64_t)workers_.size() * (S_ + 1) * round_up(shard_len_[shard] * esz_, kAlignBytes) +
         nbuf_ * pub_slot_bytes(shard);
}

int64_t AsyncEngine::region_bytes_for(int rank) const {
  int64_t b = 0;
  for (size_t k = 0; k < owners_.size(); ++k)
    if (owners_[k] == rank) b += shard_region_bytes((int)k);
  return b;
}

int64_t AsyncEngine::shard_base(int rank, int shard) const {
  int64_t b = 0;
  for (int k = 0; k < shard; ++k)
    if (owners_[k] == rank) b += shard_region_bytes(k);
  return b;
}

char* AsyncEngine::inbox_ptr(int shard, int wi, int slot) const {
  const int o = owners_[shard];
  TORCH_CHECK(peer_base_[o], "psd async: rank ", o, " memory not attached");
  const int64_t sb = round_up(shard_len_[shard] * esz_, kAlignBytes);
  return peer_base_[o] + shard_base(o, shard) + ((int64_t)wi * (S_ + 1) + slot) * sb;
}

char* AsyncEngine::publish_ptr(int shard, int buf) const {
  const int o = owners_[shard];
  TORCH_CHECK(peer_base_[o], "psd async: rank ", o, " memory not attached");
  const int64_t sb = round_up(shard_len_[shard] * esz_, kAlignBytes);
  return peer_base_[o] + shard_base(o, shard) + (int64_t)workers_.size() * (S_ + 1) * sb + buf * pub_slot_bytes(shard);
}

char* AsyncEngine::publish_q_ptr(int shard, int buf) const {
  return publish_ptr(shard, buf) + round_up(shard_len_[shard] * esz_, kAlignBytes);
}

char* AsyncEngine::publish_sc_ptr(int shard, int buf) const {
  return publish_q_ptr(shard, buf) + round_up(shard_len_[shard], kAlignBytes);
}

// the MX e4m3 copy (+ E8M0 scales) of the fp32 master into publish slot `buf` (kernels/fp8.hip)
void AsyncEngine::quant_publish(ShardState& st, int shard, int buf, void* stream) {
  hip_ok(launch_quant_mx(st.master.data_ptr(), DT_F32, shard_len_[shard], 0,
                         reinterpret_cast<uint8_t*>(publish_q_ptr(shard, buf)),
                         reinterpret_cast<uint8_t*>(publish_sc_ptr(shard, buf)), static_cast<hipStream_t>(stream)),
         "launch_quant_mx(publish)");
}

// ------------------------------------------------------------------ memory exchange
std::string AsyncEngine::local_desc() const {
  if (!local_mem_) return "N";
  if (device_ < 0) return "C" + local_shm_;
  hipIpcMemHandle_t h;
  hip_ok(hipIpcGetMemHandle(&h, local_mem_), "hipIpcGetMemHandle");
  std::string s = "G";
  s.append(reinterpret_cast<const char*>(&h), sizeof(h));
  return s;
}

void AsyncEngine::attach_peer(int rank, const std::string& desc) {
  TORCH_CHECK(rank >= 0 && rank < world_, "psd async: bad peer rank");
  if (rank == rank_ || desc.empty() || desc[0] == 'N') return;
  const int64_t bytes = region_bytes_for(rank);
  if (desc[0] == 'C') {
    peer_base_[rank] = static_cast<char*>(map_shm(desc.substr(1), (size_t)bytes, false));
  } else {
    TORCH_CHECK(desc[0] == 'G' && desc.size() == 1 + sizeof(hipIpcMemHandle_t), "psd async: bad descriptor");
    hipIpcMemHandle_t h;
    std::memcpy(&h, desc.data() + 1, sizeof(h));
    const c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device_));
    void* p = nullptr;
    hip_ok(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
    peer_base_[rank] = static_cast<char*>(p);
    peer_ipc_[rank] = true;
  }
  peer_bytes_[rank] = bytes;
}

// ------------------------------------------------------------------ owner side
void AsyncEngine::set_shard_state(int shard, at::Tensor master, c10::optional<at::Tensor> state1,
                                  c10::optional<at::Tensor> state2, at::Tensor dyn, int64_t kind, double momentum,
                                  double dampening, bool nesterov, double weight_decay, double beta1, double beta2,
                                  double eps) {
  TORCH_CHECK(shard >= 0 && shard < (int)owners_.size() && owners_[shard] == rank_, "psd async: shard ", shard,
              " is not owned by rank ", rank_);
  TORCH_CHECK(master.numel() == shard_len_[shard] && master.scalar_type() == at::kFloat && master.is_contiguous(),
              "psd async: master must be contiguous fp32 of the shard length");
  ShardState& st = shards_[shard];
  st.master = master;
  st.s1 = state1.has_value() ? *state1 : at::Tensor();
  st.s2 = state2.has_value() ? *state2 : at::Tensor();
  st.dyn = dyn;
  st.hyper.kind = (int32_t)kind;
  st.hyper.momentum = (float)momentum;
  st.hyper.dampening = (float)dampening;
  st.hyper.nesterov = nesterov;
  st.hyper.weight_decay = (float)weight_decay;
  st.hyper.beta1 = (float)beta1;
  st.hyper.beta2 = (float)beta2;
  st.hyper.eps = (float)eps;
}

void AsyncEngine::publish_initial(int shard, int64_t version, std::vector<int64_t> clocks) {
  ShardState& st = shards_[shard];
  TORCH_CHECK(st.master.defined(), "psd async: set_shard_state first");
  TORCH_CHECK(!running_, "psd async: publish_initial while the engine runs");
  TORCH_CHECK(version >= 0 && (clocks.empty() || clocks.size() == workers_.size()),
              "psd async: publish_initial takes a version >= 0 and one clock per worker");
  st.publish[0].copy_(st.master);
  if (mx_) quant_publish(st, shard, 0, c10::hip::getCurrentHIPStream((c10::DeviceIndex)device_).stream());
  if (device_ >= 0) hip_ok(hipDeviceSynchronize(), "hipDeviceSynchronize");
  ShardCtl& s = ctl_->shard[shard];
  for (int b = 1; b < nbuf_; ++b) s.buf_version[b].store(-1);
  s.buf_version[0].store(version);
  s.latest.store(0);
  s.version.store(version);
  s.base_version.store(version);
  for (size_t wi = 0; wi < clocks.size(); ++wi) s.clock[wi].store(clocks[wi]);
  st.enq = version;
  st.round.clear();
}

void AsyncEngine::set_round(int k) {
  TORCH_CHECK(!running_, "psd async: set_round while the engine runs");
  TORCH_CHECK(k >= 1 && k <= (int)workers_.size(), "psd async: round size must be in [1, W = ", workers_.size(),
              "], got ", k);
  round_ = k;
}

void AsyncEngine::set_fixed_schedule(bool on) {
  TORCH_CHECK(!running_, "psd async: set_fixed_schedule while the engine runs");
  TORCH_CHECK(!on || round_ == (int)workers_.size(), "psd async: the fixed schedule needs rounds of K = W pushes");
  TORCH_CHECK(!on || nbuf_ >= S_ + 2, "psd async: the fixed schedule keeps S + 1 versions: nbuf >= S + 2 (nbuf ",
              nbuf_, ", S ", S_, ")");
  fixed_ = on;
}

// The least recently published free buffer (not the latest, no enqueued apply, no reader): the
// fixed schedule's readers need the last S + 1 versions to stay until they are older than that.
int AsyncEngine::free_buf(int shard) const {
  const ShardState& st = shards_[shard];
  const ShardCtl& s = ctl_->shard[shard];
  const int latest = s.latest.load();
  int best = -1;
  int64_t best_v = 0;
  for (int b = 0; b < nbuf_; ++b) {
    if (b == latest || st.busy[b] || s.readers[b].load() != 0) continue;
    const int64_t v = s.buf_version[b].load();
    if (best < 0 || v < best_v) {
      best = b;
      best_v = v;
    }
  }
  return best;
}

// Claim free buffer b for an apply: invalidate its version, then re-check its reader count. A
// fixed-schedule reader pins (readers++) and then checks the version, so with these two
// sequentially consistent store -> load orders at least one side sees the other: the reader backs
// off, or the claim is dropped (the version is restored) and the round waits.
bool AsyncEngine::claim_buf(int shard, int b) {
  ShardCtl& s = ctl_->shard[shard];
  const int64_t v = s.buf_version[b].load();
  s.buf_version[b].store(-1);
  if (s.readers[b].load() != 0) {
    s.buf_version[b].store(v);
    return false;
  }
  return true;
}

void AsyncEngine::start() {
  if (running_) return;
  stop_.store(false);
  running_ = true;
  thr_ = std::thread([this] { run(); });
}

void AsyncEngine::stop() {
  if (!running_) return;
  stop_.store(true);
  thr_.join();
  running_ = false;
  if (ctl_) ctl_->hb_us[rank_].store(kHbLeft);  // stopped on purpose: not a dead peer
  // finish what is in flight (unpins / posts / applies) so the shared state is final and no
  // kernel or copy still touches the inbox / publish memory when it is freed
  for (int guard = 0; guard < 1000; ++guard) {
    if (device_ >= 0) {
      (void)hipStreamSynchronize(static_cast<hipStream_t>(ps_stream_));
      std::lock_guard<std::mutex> g(act_mu_);
      for (auto& a : actions_)
        if (a.event) (void)hipEventSynchronize(static_cast<hipEvent_t>(a.event));
    }
    if (!poll_once() && pending_.empty()) break;
  }
}

void AsyncEngine::run() {
  try {
    if (device_ >= 0) hip_ok(hipSetDevice(device_), "hipSetDevice");
    int spins = 0;
    int64_t last_check = now_us();
    while (!stop_.load()) {
      const int64_t t = now_us();
      ctl_->hb_us[rank_].store(t);
      if (dead_after_s_ > 0 && t - last_check > 100000) {  // peers' liveness, every 100 ms
        last_check = t;
        check_peers(t);
      }
      if (ctl_->error.load()) break;
      if (poll_once()) spins = 0;
      else backoff(spins);
    }
  } catch (const std::exception& e) {
    fail(std::string("engine thread (rank ") + std::to_string(rank_) + "): " + e.what());
  }
}

bool AsyncEngine::poll_once() {
  bool progress = false;
  // 1. worker-side deferred actions (unpin after a pull copy, post after push copies)
  for (;;) {
    Action a;
    {
      std::lock_guard<std::mutex> g(act_mu_);
      if (actions_.empty()) break;
      Action& f = actions_.front();
      if (!done(f.event)) break;
      a = std::move(f);
      actions_.pop_front();
    }
    a.fn();
    if (a.event) (void)hipEventDestroy(static_cast<hipEvent_t>(a.event));
    progress = true;
  }
  // 2. apply completions (one stream: in order)
  while (!pending_.empty()) {
    Pending& p = pending_.front();
    if (!done(p.event)) break;
    ShardCtl& s = ctl_->shard[p.shard];
    const int64_t v = s.version.load() + 1;
    s.buf_version[p.buf].store(v);
    s.latest.store(p.buf);
    s.version.store(v);
    for (const RoundItem& it : p.items) s.clock[it.wi].fetch_add(1);
    shards_[p.shard].busy[p.buf] = false;
    {
      std::lock_guard<std::mutex> g(hist_mu_);
      for (const RoundItem& it : p.items) {
        hist_[std::min<int64_t>(std::max<int64_t>(it.staleness, 0), kBins - 1)] += 1;
        if (log_on_) log_.push_back({p.shard, workers_[it.wi], it.step, it.staleness, v});
      }
    }
    n_applies_.fetch_add(1);
    if (p.event) (void)hipEventDestroy(static_cast<hipEvent_t>(p.event));
    pending_.pop_front();
    progress = true;
  }
  // 3. new pushes -> the shard's current round (one message per worker per pass: arrival order,
  //    no worker starved); a complete round is applied at once
  const int W = (int)workers_.size();
  for (int k : my_shards_) {
    ShardState& st = shards_[k];
    for (int wi = 0; wi < W; ++wi) {
      Mailbox& mb = ctl_->mb[k][wi];
      const int64_t t = mb.tail.load();
      if (t >= mb.head.load()) continue;
      // fixed schedule: round r takes exactly every worker's step-r push (a faster worker's next
      // push waits in its mailbox) -- the round composition no longer depends on arrival timing
      if (fixed_ && mb.ring[t % kRing].step != st.enq) continue;
      const bool completes = (int)st.round.size() + 1 >= round_;
      int buf = -1;
      if (completes) {
        buf = free_buf(k);
        if (buf >= 0 && !claim_buf(k, buf)) buf = -1;
        if (buf < 0) break;  // every snapshot is pinned or in flight: retry after completions
      }
      const Msg m = mb.ring[t % kRing];
      mb.tail.store(t + 1);
      st.round.push_back(RoundItem{wi, (int)(m.step % (S_ + 1)), m.step, m.pulled, 0});
      progress = true;
      if (!completes) continue;
      // sources in worker order: the fp32 sum inside the apply kernel is then independent of the
      // arrival order (bitwise-reproducible rounds at SSP bound 0)
      std::sort(st.round.begin(), st.round.end(),
                [](const RoundItem& x, const RoundItem& y) { return x.wi != y.wi ? x.wi < y.wi : x.step < y.step; });
      std::vector<at::Tensor> g;
      for (RoundItem& it : st.round) {
        it.staleness = st.enq - it.pulled;
        g.push_back(st.inbox[(size_t)it.wi * (S_ + 1) + it.slot]);
      }
      st.enq += 1;
      st.busy[buf] = true;
      hipEvent_t ev = nullptr;
      if (device_ >= 0) {
        c10::hip::HIPStreamGuard sg(c10::hip::getStreamFromExternal(static_cast<hipStream_t>(ps_stream_),
                                                                    (c10::DeviceIndex)device_));
        apply_into(st, g, buf);
        if (mx_) quant_publish(st, k, buf, ps_stream_);
        hip_ok(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate");
        hip_ok(hipEventRecord(ev, static_cast<hipStream_t>(ps_stream_)), "hipEventRecord");
      } else {
        apply_into(st, g, buf);
      }
      pending_.push_back(Pending{k, buf, std::move(st.round), ev});
      st.round.clear();
    }
  }
  return progress;
}

// One update: optimizer step counter, fused apply of the round's inbox slots (summed in registers,
// scaled by the dyn grad_scale = 1/K) onto the fp32 master, and the new snapshot written into
// publish buffer `buf` (bf16: by the apply kernel itself).
void AsyncEngine::apply_into(ShardState& st, const std::vector<at::Tensor>& g_in, int buf) {
  // a round of more than 16 pushes (the fused apply kernel's source limit): each group of 16
  // inbox slots (worker order) is summed into an fp32 workspace and the apply takes the group sums
  // (fixed order, so rounds stay bitwise reproducible). With K = W every round completes -- a
  // partial round stranded at W > 16 would hold a worker's clock back forever.
  std::vector<at::Tensor> g = g_in;
  if (g.size() > (size_t)kMaxSources) {
    const size_t ng = (g.size() + kMaxSources - 1) / kMaxSources;
    TORCH_CHECK(ng <= (size_t)kMaxSources, "psd async: at most 256 pushes per round");
    while (st.acc.size() < ng) st.acc.push_back(at::empty({st.master.numel()}, st.master.options().dtype(at::kFloat)));
    std::vector<at::Tensor> sums;
    for (size_t gi = 0; gi < ng; ++gi) {
      const size_t b = gi * kMaxSources, e = std::min(g.size(), b + kMaxSources);
      multi_reduce_(st.acc[gi], std::vector<at::Tensor>(g.begin() + b, g.begin() + e), 1.0);
      sums.push_back(st.acc[gi]);
    }
    g = std::move(sums);
  }
  optim_advance_(st.dyn, st.hyper.beta1, st.hyper.beta2);
  const bool bf16 = esz_ == 2;
  fused_apply_(st.master, g, st.s1.defined() ? c10::optional<at::Tensor>(st.s1) : c10::nullopt,
               st.s2.defined() ? c10::optional<at::Tensor>(st.s2) : c10::nullopt,
               bf16 ? c10::optional<at::Tensor>(st.publish[buf]) : c10::nullopt, st.dyn, st.hyper.kind,
               st.hyper.momentum, st.hyper.dampening, st.hyper.nesterov, st.hyper.weight_decay, st.hyper.beta1,
               st.hyper.beta2, st.hyper.eps, false, apply_cap_);
  if (!bf16) st.publish[buf].copy_(st.master);
}

bool AsyncEngine::done(void* event) {
  if (!event) return true;
  const hipError_t e = hipEventQuery(static_cast<hipEvent_t>(event));
  if (e == hipErrorNotReady) return false;
  hip_ok(e, "hipEventQuery");
  return true;
}

// ------------------------------------------------------------------ worker side
void AsyncEngine::copy(void* dst, const void* src, int64_t bytes, void* stream) {
  if (bytes <= 0) return;
  if (device_ >= 0) {
    hip_ok(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDefault, static_cast<hipStream_t>(stream)),
           "hipMemcpyAsync");
  } else {
    std::memcpy(dst, src, (size_t)bytes);
  }
}

void AsyncEngine::defer(void* stream, std::function<void()> fn) {
  if (device_ < 0 || !running_) {
    if (device_ >= 0) hip_ok(hipStreamSynchronize(static_cast<hipStream_t>(stream)), "hipStreamSynchronize");
    fn();
    return;
  }
  hipEvent_t ev = nullptr;
  hip_ok(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate");
  hip_ok(hipEventRecord(ev, static_cast<hipStream_t>(stream)), "hipEventRecord");
  std::lock_guard<std::mutex> g(act_mu_);
  actions_.push_back(Action{ev, std::move(fn)});
}

void AsyncEngine::post(int shard, int wi, int64_t step, int64_t pulled) {
  Mailbox& mb = ctl_->mb[shard][wi];
  const int64_t h = mb.head.load();
  if (h - mb.tail.load() >= kRing) {
    fail("mailbox overflow (shard " + std::to_string(shard) + ", worker " + std::to_string(wi) + ")");
    return;
  }
  mb.ring[h % kRing] = Msg{step, pulled};
  mb.head.store(h + 1);
  n_posts_.fetch_add(1);
}

void AsyncEngine::check_peers(int64_t t) {
  for (int r = 0; r < world_; ++r) {
    if (r == rank_) continue;
    const int64_t h = ctl_->hb_us[r].load();
    if (h <= 0) continue;  // not started yet, or stopped on purpose
    const double silent = (double)(t - h) * 1e-6;
    if (silent > dead_after_s_) {
      fail("rank " + std::to_string(r) + " presumed dead: its async engine has been silent for " +
           std::to_string((int)silent) + " s (PSD_ASYNC_DEAD_S=" + std::to_string((int)dead_after_s_) + ")");
      return;
    }
  }
}

void AsyncEngine::inject_error(const std::string& msg) { fail(msg); }

void AsyncEngine::check_error() const {
  if (ctl_->error.load()) TORCH_CHECK(false, "psd async: ", std::string(ctl_->msg));
}

void AsyncEngine::fail(const std::string& msg) {
  int32_t z = 0;
  if (ctl_->error.compare_exchange_strong(z, 1)) {
    std::strncpy(ctl_->msg, msg.c_str(), sizeof(ctl_->msg) - 1);
  }
}

std::vector<int64_t> AsyncEngine::pull(int64_t step, at::Tensor params_flat, int64_t stream) {
  TORCH_CHECK(params_flat.is_contiguous() && params_flat.element_size() == esz_, "psd async: working buffer dtype");
  return pull_impl(step, static_cast<char*>(params_flat.data_ptr()), nullptr, nullptr, stream);
}

// the MX e4m3 snapshot (1 byte / parameter + 1 / 32) instead of the bf16 one (kernels/fp8.hip scales),
// dequantised into the bf16 working weights `out` on the same stream
std::vector<int64_t> AsyncEngine::pull_mx(int64_t step, at::Tensor q_flat, at::Tensor sc_flat, at::Tensor out,
                                          int64_t stream) {
  TORCH_CHECK(mx_, "psd async: pull_mx on an engine without the MX publish");
  TORCH_CHECK(q_flat.is_contiguous() && q_flat.element_size() == 1 && sc_flat.is_contiguous() &&
                  sc_flat.element_size() == 1 && sc_flat.numel() * 32 == q_flat.numel(),
              "psd async: pull_mx buffers (1-byte q [n], 1-byte scales [n / 32])");
  TORCH_CHECK(out.is_contiguous() && out.scalar_type() == at::kBFloat16 && out.numel() == q_flat.numel(),
              "psd async: pull_mx output (bf16 [n])");
  return pull_impl(step, static_cast<char*>(q_flat.data_ptr()), static_cast<char*>(sc_flat.data_ptr()),
                   static_cast<uint16_t*>(out.data_ptr()), stream);
}

void AsyncEngine::set_xfer(bool kernel) {
  TORCH_CHECK(!kernel || device_ >= 0, "psd async: the scatter / gather kernels need a GPU engine");
  xfer_kernel_ = kernel;
}

void AsyncEngine::set_xfer_blocks(int cap) {
  TORCH_CHECK(cap >= 1 && cap <= 1024, "psd async: xfer workgroups per segment in [1, 1024]");
  xfer_cap_ = cap;
}

namespace {
// the scatter / gather kernels move 16-byte vectors: a segment with an unaligned end takes the copy
// path (hipMemcpyAsync accepts any alignment)
inline bool aligned16(const void* a, const void* b) {
  return ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b)) & 15) == 0;
}
}  // namespace

std::string AsyncEngine::xfer_mode() const {
  if (device_ < 0) return "host-memcpy";
  // "kernel": peer segments by the scatter / gather kernels, this rank's own by hipMemcpyAsync
  return xfer_kernel_ ? "kernel" : "hipMemcpyAsync";
}

std::vector<int64_t> AsyncEngine::pull_impl(int64_t step, char* dst, char* dst_sc, uint16_t* dst_bf16,
                                            int64_t stream) {
  TORCH_CHECK(my_wi_ >= 0, "psd async: rank ", rank_, " is not a worker");
  const double t0 = now_s();
  const int64_t need = step - S_;
  const int P = (int)owners_.size(), W = (int)workers_.size();
  if (need > 0) {
    for (int k = 0; k < P; ++k) {
      for (int wi = 0; wi < W; ++wi) {
        int spins = 0;
        while (ctl_->shard[k].clock[wi].load() < need) {
          check_error();
          if (now_s() - t0 > timeout_s_) {
            const std::string m = "pull of step " + std::to_string(step) + " on rank " + std::to_string(rank_) +
                                  " waited " + std::to_string(timeout_s_) + " s for worker " +
                                  std::to_string(workers_[wi]) + " at shard " + std::to_string(k) + " (clock " +
                                  std::to_string(ctl_->shard[k].clock[wi].load()) + " < " + std::to_string(need) + ")";
            fail(m);
            TORCH_CHECK(false, "psd async: ", m);
          }
          backoff(spins);
        }
      }
    }
  }
  wait_us_.fetch_add((int64_t)((now_s() - t0) * 1e6));
  std::vector<int64_t> pulled(P);
  std::vector<int> bufs(P, -1);
  for (int k = 0; k < P; ++k) {
    ShardCtl& s = ctl_->shard[k];
    int b = -1;
    if (fixed_) {
      // fixed schedule: exactly version max(step - S, base) -- the SSP bound's oldest admissible
      // snapshot, whatever the timing (deterministic staleness S). Pin, then check the version
      // (claim_buf's protocol); the owner keeps the last S + 1 versions (LRU reuse, nbuf >= S + 2)
      const int64_t want = std::max(step - (int64_t)S_, s.base_version.load());
      for (int bb = 0; bb < nbuf_ && b < 0; ++bb) {
        s.readers[bb].fetch_add(1);
        if (s.buf_version[bb].load() == want) b = bb;
        else s.readers[bb].fetch_sub(1);
      }
      if (b < 0) {
        for (int kk = 0; kk < k; ++kk) ctl_->shard[kk].readers[bufs[kk]].fetch_sub(1);
        const std::string m = "fixed-schedule pull of step " + std::to_string(step) + " on rank " +
                              std::to_string(rank_) + ": version " + std::to_string(want) + " of shard " +
                              std::to_string(k) + " is no longer published (latest " +
                              std::to_string(s.version.load()) + ")";
        fail(m);
        TORCH_CHECK(false, "psd async: ", m);
      }
    } else {
      for (;;) {  // pin the latest snapshot (re-check: the owner never writes the latest or a pinned one)
        b = s.latest.load();
        s.readers[b].fetch_add(1);
        if (s.latest.load() == b) break;
        s.readers[b].fetch_sub(1);
      }
    }
    pulled[k] = s.buf_version[b].load();
    bufs[k] = b;
  }
  void* sp = reinterpret_cast<void*>(stream);
  bool remote = false;  // any shard owned by another process (its peer-mapped memory)
  for (int k = 0; k < P; ++k) remote = remote || owners_[k] != rank_;
  // the gather kernel pays where it drives several peers' links at once; a pull of only this
  // rank's own shards is a local copy, which the copy engine does without taking CUs from the
  // compute stream (N = 1: ResNet-50 / BERT-base 0.2 % / 0.1 % faster with the copies)
  bool al = true;  // every segment 16-byte aligned (else the copy path)
  for (int k = 0; k < P && al; ++k) {
    if (dst_sc)
      al = aligned16(publish_q_ptr(k, bufs[k]), dst + shard_off_[k]) && aligned16(dst_bf16 + shard_off_[k], nullptr) &&
           shard_len_[k] % 32 == 0;
    else
      al = aligned16(publish_ptr(k, bufs[k]), dst + shard_off_[k] * esz_);
  }
  if (device_ >= 0 && xfer_kernel_ && remote && al) {
    const int cap = xfer_cap_;
    // every shard's snapshot in one gather launch: all owners' links at once (kernels/xfer.hip)
    const c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device_));
    if (dst_sc) {
      for (int k0 = 0; k0 < P; k0 += kMaxXferMxSeg) {
        XferMxList L{};
        int64_t mx = 0;
        for (int k = k0; k < std::min(P, k0 + kMaxXferMxSeg); ++k) {
          L.seg[L.count++] = XferMxSeg{reinterpret_cast<const uint8_t*>(publish_q_ptr(k, bufs[k])),
                                       reinterpret_cast<const uint8_t*>(publish_sc_ptr(k, bufs[k])),
                                       reinterpret_cast<uint8_t*>(dst + shard_off_[k]),
                                       reinterpret_cast<uint8_t*>(dst_sc + shard_off_[k] / 32),
                                       dst_bf16 + shard_off_[k], shard_len_[k]};
          mx = std::max(mx, shard_len_[k]);
        }
        L.blocks_per_seg = xfer_blocks(mx, cap);
        hip_ok(launch_xfer_mx(L, static_cast<hipStream_t>(sp)), "launch_xfer_mx(pull)");
      }
    } else {
      XferList L{};
      int64_t mx = 0;
      for (int k = 0; k < P; ++k) {
        L.seg[L.count++] = XferSeg{publish_ptr(k, bufs[k]), dst + shard_off_[k] * esz_, shard_len_[k] * esz_};
        mx = std::max(mx, shard_len_[k] * esz_);
      }
      L.blocks_per_seg = xfer_blocks(mx, cap);
      L.nt_load = 1;
      hip_ok(launch_xfer(L, static_cast<hipStream_t>(sp)), "launch_xfer(pull)");
    }
  } else {
    for (int k = 0; k < P; ++k) {
      const int b = bufs[k];
      if (dst_sc) {
        copy(dst + shard_off_[k], publish_q_ptr(k, b), shard_len_[k], sp);
        copy(dst_sc + shard_off_[k] / 32, publish_sc_ptr(k, b), shard_len_[k] / 32, sp);
      } else {
        copy(dst + shard_off_[k] * esz_, publish_ptr(k, b), shard_len_[k] * esz_, sp);
      }
    }
    if (dst_sc && dst_bf16)
      hip_ok(launch_dequant_mx(reinterpret_cast<const uint8_t*>(dst), reinterpret_cast<const uint8_t*>(dst_sc),
                               shard_off_[P - 1] + shard_len_[P - 1], dst_bf16, DT_BF16, static_cast<hipStream_t>(sp)),
             "launch_dequant_mx(pull)");
  }
  for (int k = 0; k < P; ++k) {
    std::atomic<int32_t>* rd = &ctl_->shard[k].readers[bufs[k]];
    defer(sp, [rd] { rd->fetch_sub(1); });
  }
  n_pulls_.fetch_add(1);
  return pulled;
}

void AsyncEngine::push(int64_t step, const at::Tensor& grads_flat, int64_t lo, int64_t hi, int64_t stream) {
  TORCH_CHECK(my_wi_ >= 0, "psd async: rank ", rank_, " is not a worker");
  TORCH_CHECK(grads_flat.is_contiguous() && grads_flat.element_size() == esz_, "psd async: gradient buffer dtype");
  check_error();
  const char* src = static_cast<const char*>(grads_flat.data_ptr());
  const int slot = (int)(step % (S_ + 1));
  bool remote = false, al = true;
  for (size_t k = 0; k < owners_.size(); ++k) {
    const int64_t a = std::max(lo, shard_off_[k]), b = std::min(hi, shard_off_[k] + shard_len_[k]);
    remote = remote || (a < b && owners_[k] != rank_);
    if (a < b) al = al && aligned16(src + a * esz_, inbox_ptr((int)k, my_wi_, slot) + (a - shard_off_[k]) * esz_);
  }
  if (device_ >= 0 && xfer_kernel_ && remote && al) {
    // the bucket's slice for every owner it overlaps in one scatter launch (kernels/xfer.hip); a
    // push into this rank's own inbox only is a local copy (see pull_impl; on the kernel it measured
    // no faster at N = 1, profiles/r6/ab_xfer_local.md)
    XferList L{};
    int64_t mx = 0;
    for (size_t k = 0; k < owners_.size(); ++k) {
      const int64_t a = std::max(lo, shard_off_[k]), b = std::min(hi, shard_off_[k] + shard_len_[k]);
      if (a >= b) continue;
      L.seg[L.count++] = XferSeg{src + a * esz_, inbox_ptr((int)k, my_wi_, slot) + (a - shard_off_[k]) * esz_,
                                 (b - a) * esz_};
      mx = std::max(mx, (b - a) * esz_);
    }
    L.blocks_per_seg = xfer_blocks(mx, xfer_cap_);
    L.nt_store = 1;
    const c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device_));
    hip_ok(launch_xfer(L, reinterpret_cast<hipStream_t>(stream)), "launch_xfer(push)");
    return;
  }
  for (size_t k = 0; k < owners_.size(); ++k) {
    const int64_t a = std::max(lo, shard_off_[k]), b = std::min(hi, shard_off_[k] + shard_len_[k]);
    if (a >= b) continue;
    copy(inbox_ptr((int)k, my_wi_, slot) + (a - shard_off_[k]) * esz_, src + a * esz_, (b - a) * esz_,
         reinterpret_cast<void*>(stream));
  }
}

void AsyncEngine::commit(int64_t step, std::vector<int64_t> pulled, int64_t stream) {
  TORCH_CHECK(my_wi_ >= 0, "psd async: rank ", rank_, " is not a worker");
  TORCH_CHECK(pulled.size() == owners_.size(), "psd async: one pulled version per shard");
  const int wi = my_wi_;
  const int P = (int)owners_.size();
  defer(reinterpret_cast<void*>(stream), [this, wi, P, step, pulled] {
    for (int k = 0; k < P; ++k) post(k, wi, step, pulled[k]);
  });
}

void AsyncEngine::wait_applied(int64_t nsteps) {
  TORCH_CHECK(my_wi_ >= 0, "psd async: rank ", rank_, " is not a worker");
  const double t0 = now_s();
  for (size_t k = 0; k < owners_.size(); ++k) {
    int spins = 0;
    while (ctl_->shard[k].clock[my_wi_].load() < nsteps) {
      check_error();
      TORCH_CHECK(now_s() - t0 <= timeout_s_, "psd async: rank ", rank_, " waited ", timeout_s_,
                  " s for its pushes to be applied at shard ", k);
      backoff(spins);
    }
  }
}

void AsyncEngine::wait_all_applied(int64_t nsteps) {
  const double t0 = now_s();
  for (size_t k = 0; k < owners_.size(); ++k) {
    for (size_t wi = 0; wi < workers_.size(); ++wi) {
      int spins = 0;
      while (ctl_->shard[k].clock[wi].load() < nsteps) {
        check_error();
        TORCH_CHECK(now_s() - t0 <= timeout_s_, "psd async: rank ", rank_, " waited ", timeout_s_,
                    " s for worker ", workers_[wi], " at shard ", k);
        backoff(spins);
      }
    }
  }
}

at::Tensor AsyncEngine::inbox_view(int shard, int wi, int slot) const {
  TORCH_CHECK(shard >= 0 && shard < (int)owners_.size() && owners_[shard] == rank_, "psd async: not my shard");
  TORCH_CHECK(wi >= 0 && wi < (int)workers_.size() && slot >= 0 && slot <= S_, "psd async: bad inbox index");
  return shards_[shard].inbox[(size_t)wi * (S_ + 1) + slot];
}

// ------------------------------------------------------------------ introspection
std::vector<int64_t> AsyncEngine::histogram() const {
  std::lock_guard<std::mutex> g(hist_mu_);
  return hist_;
}

int64_t AsyncEngine::version(int shard) const { return ctl_->shard[shard].version.load(); }

std::vector<int64_t> AsyncEngine::clocks(int shard) const {
  std::vector<int64_t> c(workers_.size());
  for (size_t wi = 0; wi < workers_.size(); ++wi) c[wi] = ctl_->shard[shard].clock[wi].load();
  return c;
}

std::vector<std::vector<int64_t>> AsyncEngine::apply_log() const {
  std::lock_guard<std::mutex> g(hist_mu_);
  return log_;
}

std::string AsyncEngine::error() const { return ctl_->error.load() ? std::string(ctl_->msg) : std::string(); }

std::vector<int64_t> AsyncEngine::counters() const {
  return {n_applies_.load(), n_posts_.load(), n_pulls_.load(), wait_us_.load()};
}

}  // namespace psd
