// Native RCCL communicator: the MI355X counterpart of the reference NCCLManager
// (include/nccl_manager.h:7-27, src/nccl_manager.cpp:11-121).
//
// Differences by design:
//   * one rank per GPU per process (the reference built N communicators in one process and issued
//     un-grouped collectives from one thread -- D6); the 128-byte unique id is bootstrapped through
//     the coordinator's key/value store instead of living in-process;
//   * every collective runs on an explicit HIP stream (default: the caller's current torch stream,
//     so push/pull can be placed on dedicated comm streams and overlapped with backward);
//   * the full PS data-plane set: reduce-scatter (push), all-gather (pull), reduce/broadcast for
//     PS shards fewer than workers, grouped send/recv for async/disjoint placements, all-reduce for
//     the reference's intra-worker average; abort() for elastic rebuilds.
#pragma once
#include <ATen/ATen.h>

#include <string>

namespace psd {

class RcclComm {
 public:
  static std::string unique_id();  // 128 raw bytes
  static int version();
  RcclComm(int rank, int world, const std::string& uid, int device);
  ~RcclComm();

  int rank() const { return rank_; }
  int world() const { return world_; }

  // stream = 0 -> current torch HIP stream of the tensor's device
  void all_reduce(at::Tensor t, const std::string& op, int64_t stream);
  void reduce_scatter(const at::Tensor& in, at::Tensor out, const std::string& op, int64_t stream);
  void all_gather(const at::Tensor& in, at::Tensor out, int64_t stream);
  void reduce(const at::Tensor& in, at::Tensor out, int root, const std::string& op, int64_t stream);
  void broadcast(at::Tensor t, int root, int64_t stream);
  void send(const at::Tensor& t, int peer, int64_t stream);
  void recv(at::Tensor t, int peer, int64_t stream);
  static void group_start();
  static void group_end();
  void abort();
  std::string async_error();

 private:
  void* comm_ = nullptr;  // ncclComm_t
  int rank_ = 0, world_ = 1, device_ = 0;
};

}  // namespace psd
