// Peer-memory scatter / gather of the asynchronous PS data plane (csrc/async_ps.cpp).
//
// A push of one gradient bucket touches every shard whose range it overlaps, and a pull touches
// every shard: one contiguous slice per owner GPU. Issued as a sequence of hipMemcpyAsync calls on
// one stream those slices cross the node one after another, so a worker drives ONE of its 7 xGMI
// links at a time (csrc/async_ps.cpp push / pull). Here every slice of a push or a pull
// is a segment of one launch, with its own group of workgroups: all owners' links carry data at
// once, on the stream the copies already used (no extra HIP stream: the process's 4 hardware queues
// are taken by compute, the engine's apply, push and pull).
//
// Layout: workgroup b serves segment b % count (so consecutive workgroups -- dispatched together --
// spread over the peers) and is the (b / count)-th of blocks_per_seg on it, grid-striding over the
// segment in 16-byte vectors, U vectors in flight per lane (loads first, then stores). Stores into a
// peer's uncached inbox / loads from its uncached publish buffer are non-temporal. Vector memory
// instructions only.
//
// The MX pull (xfer_mx_kernel) also dequantises: 16 e4m3 bytes per lane (half a 32-element block),
// the block's E8M0 byte, written to the worker's q / scale copies (the fp8 convolutions read them)
// and, dequantised, to its bf16 working weights -- the separate dequant_mx pass over the pulled
// copy is gone.
#include "common.h"
#include "launchers_xfer.h"
#include "mx_common.h"

namespace psd {

namespace {

template <bool NT>
__device__ __forceinline__ u32x4 ld16(const u32x4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT>
__device__ __forceinline__ void st16(u32x4* p, u32x4 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

}  // namespace

template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void xfer_kernel(XferList L) {
  const int s = (int)(blockIdx.x % (unsigned)L.count);
  const int j = (int)(blockIdx.x / (unsigned)L.count);
  const XferSeg g = L.seg[s];
  const int64_t n16 = g.bytes >> 4;
  const u32x4* __restrict__ src = static_cast<const u32x4*>(g.src);
  u32x4* __restrict__ dst = static_cast<u32x4*>(g.dst);
  const int64_t stride = (int64_t)L.blocks_per_seg * 256 * U;
  for (int64_t base = (int64_t)j * 256 * U + threadIdx.x; base < n16; base += stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (base + u * 256 < n16) v[u] = ld16<NTL>(src + base + u * 256);
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (base + u * 256 < n16) st16<NTS>(dst + base + u * 256, v[u]);
  }
  const int tail = (int)(g.bytes & 15);
  if (j == 0 && (int)threadIdx.x < tail) {
    const int64_t o = n16 * 16 + threadIdx.x;
    static_cast<uint8_t*>(g.dst)[o] = static_cast<const uint8_t*>(g.src)[o];
  }
  if constexpr (NTS) {
    // Stores into a peer's memory (push): a system-scope release per wave before the kernel ends,
    // so the commit event recorded behind this launch (async_ps.cpp defer -> post) can never be
    // observed by the owner ahead of the bytes, whatever scope the runtime gives the end-of-kernel
    // release (hipMemcpyAsync gave this ordering before). The counted wait is inline
    // asm so the compiler cannot drop it after the release (MI355X_MICROARCH.md, compiler hazard).
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

template <int U>
__global__ __launch_bounds__(256) void xfer_mx_kernel(XferMxList L) {
  const int s = (int)(blockIdx.x % (unsigned)L.count);
  const int j = (int)(blockIdx.x / (unsigned)L.count);
  const XferMxSeg g = L.seg[s];
  const int64_t n16 = g.n >> 4;  // 16-element items (two per 32-element block)
  const int64_t stride = (int64_t)L.blocks_per_seg * 256 * U;
  for (int64_t base = (int64_t)j * 256 * U + threadIdx.x; base < n16; base += stride) {
    u32x4 q[U];
    uint8_t sc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = base + u * 256;
      if (i < n16) {
        q[u] = ld16<true>(reinterpret_cast<const u32x4*>(g.q_src) + i);
        sc[u] = __builtin_nontemporal_load(g.sc_src + (i >> 1));
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = base + u * 256;
      if (i >= n16) continue;
      *(reinterpret_cast<u32x4*>(g.q_dst) + i) = q[u];
      if ((i & 1) == 0) g.sc_dst[i >> 1] = sc[u];
      const float scale = __uint_as_float((uint32_t)sc[u] << 23);  // 2^(eb - 127), as dequant_mx
      const uint32_t w[4] = {q[u].x, q[u].y, q[u].z, q[u].w};
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        float t[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          t[e] = e4m3_to_f32((uint8_t)(w[2 * h] >> (8 * e))) * scale;
          t[e + 4] = e4m3_to_f32((uint8_t)(w[2 * h + 1] >> (8 * e))) * scale;
        }
        store8_bf16(g.bf16_dst + i * 16 + h * 8, t);
      }
    }
  }
}

hipError_t launch_xfer(const XferList& L, hipStream_t st) {
  if (L.count <= 0) return hipSuccess;
  if (L.count > kMaxXferSeg || L.blocks_per_seg < 1) return hipErrorInvalidValue;
  for (int i = 0; i < L.count; ++i)
    if ((reinterpret_cast<uintptr_t>(L.seg[i].src) | reinterpret_cast<uintptr_t>(L.seg[i].dst)) & 15)
      return hipErrorInvalidValue;
  const dim3 grid((unsigned)(L.count * L.blocks_per_seg));
  if (L.nt_load && L.nt_store) hipLaunchKernelGGL((xfer_kernel<4, true, true>), grid, dim3(256), 0, st, L);
  else if (L.nt_load) hipLaunchKernelGGL((xfer_kernel<4, true, false>), grid, dim3(256), 0, st, L);
  else if (L.nt_store) hipLaunchKernelGGL((xfer_kernel<4, false, true>), grid, dim3(256), 0, st, L);
  else hipLaunchKernelGGL((xfer_kernel<4, false, false>), grid, dim3(256), 0, st, L);
  return hipGetLastError();
}

hipError_t launch_xfer_mx(const XferMxList& L, hipStream_t st) {
  if (L.count <= 0) return hipSuccess;
  if (L.count > kMaxXferMxSeg || L.blocks_per_seg < 1) return hipErrorInvalidValue;
  for (int i = 0; i < L.count; ++i) {
    const XferMxSeg& g = L.seg[i];
    if (g.n % 32 != 0 ||
        ((reinterpret_cast<uintptr_t>(g.q_src) | reinterpret_cast<uintptr_t>(g.q_dst) |
          reinterpret_cast<uintptr_t>(g.bf16_dst)) & 15))
      return hipErrorInvalidValue;
  }
  hipLaunchKernelGGL((xfer_mx_kernel<2>), dim3((unsigned)(L.count * L.blocks_per_seg)), dim3(256), 0, st, L);
  return hipGetLastError();
}

}  // namespace psd
