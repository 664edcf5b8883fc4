// Launch API of the async PS data plane's peer-memory scatter / gather kernels (xfer.hip).
#pragma once
#include <hip/hip_runtime_api.h>
#include <cstdint>

namespace psd {

constexpr int kMaxXferSeg = 64;  // one segment per PS shard (AsyncEngine: at most 64 shards)

// One contiguous byte range: src and dst 16-byte aligned (the tail of a length that is not a
// multiple of 16 is copied bytewise).
struct XferSeg {
  const void* src;
  void* dst;
  int64_t bytes;
};

// Every segment of the list in ONE launch, each on its own set of workgroups, so the copies into
// (push) or out of (pull) different peers' HBM run concurrently -- one xGMI link per peer -- where a
// sequence of hipMemcpyAsync calls on one stream drives one link at a time. Stores to peer memory
// are non-temporal (the owner's inbox / publish memory is uncached).
struct XferList {
  XferSeg seg[kMaxXferSeg];
  int32_t count;
  int32_t blocks_per_seg;
  int32_t nt_store;  // 1: destination is a peer's uncached memory (non-temporal stores)
  int32_t nt_load;   // 1: source is a peer's uncached memory (non-temporal loads)
};
hipError_t launch_xfer(const XferList& list, hipStream_t stream);

// MX pull: per shard, the owner's e4m3 snapshot (n bytes) + E8M0 scales (n / 32 bytes) into the
// worker's q / scale buffers AND dequantised into its bf16 working weights, in one pass over the
// peer memory (n % 32 == 0, every pointer 16-byte aligned except the scales).
struct XferMxSeg {
  const uint8_t* q_src;
  const uint8_t* sc_src;
  uint8_t* q_dst;
  uint8_t* sc_dst;
  uint16_t* bf16_dst;
  int64_t n;
};
constexpr int kMaxXferMxSeg = 32;
struct XferMxList {
  XferMxSeg seg[kMaxXferMxSeg];
  int32_t count;
  int32_t blocks_per_seg;
};
hipError_t launch_xfer_mx(const XferMxList& list, hipStream_t stream);

// blocks per segment for `bytes` (the largest segment of a launch): ~128 KiB per workgroup, at
// most `cap` (a local copy may take more CUs than one peer link can use)
inline int32_t xfer_blocks(int64_t bytes, int32_t cap) {
  int64_t b = (bytes + (128 << 10) - 1) >> 17;
  if (b < 1) b = 1;
  if (b > cap) b = cap;
  return (int32_t)b;
}

}  // namespace psd
