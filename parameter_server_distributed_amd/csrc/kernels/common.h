// Device helpers shared by the gfx950 kernels (wave64, 16-byte vector memory ops).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace psd {

constexpr int kWave = 64;  // CDNA wavefront: never 32

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf16_to_f32(uint16_t h) { return __uint_as_float(((uint32_t)h) << 16); }

// Round-to-nearest-even fp32 -> bf16, NaN preserved. A plain cast is one v_cvt_pk_bf16_f32 on
// gfx950 (two values per instruction when paired, pack_bf16x2_rne); the integer-arithmetic rounding
// this replaced cost ~5 VALU per value, which made the BN apply and stem pool passes issue-bound
// (SQ_WAIT_INST_ANY ~45 % of wave cycles in profiles/pmc_r1.md).
__device__ __forceinline__ uint16_t f32_to_bf16(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }

typedef __bf16 psd_bf16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack_bf16x2_rne(float lo, float hi) {
  const psd_bf16x2 v = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(uint32_t, v);
}

// ReLU with torch semantics: NaN propagates (relu(NaN) = NaN). fmaxf(x, 0) would return 0 for a
// NaN input and silently hide an upstream fault (a bad library GEMM once fed NaN into a BN whose
// fmaxf ReLU turned it into zeros: the step "trained" with NaN weights and a finite loss).
__device__ __forceinline__ float relu_nan(float x) { return x < 0.f ? 0.f : x; }

// 8 consecutive elements <-> registers, one 16-byte (bf16) or two 16-byte (fp32) loads per lane.
__device__ __forceinline__ void load8_f32(const float* p, float v[8]) {
  f32x4 a = *reinterpret_cast<const f32x4*>(p);
  f32x4 b = *reinterpret_cast<const f32x4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void store8_f32(float* p, const float v[8]) {
  *reinterpret_cast<f32x4*>(p) = f32x4{v[0], v[1], v[2], v[3]};
  *reinterpret_cast<f32x4*>(p + 4) = f32x4{v[4], v[5], v[6], v[7]};
}
// NT: nontemporal (streaming) load / store, for passes over tensors far larger than the 256 MB
// Infinity Cache whose bytes are touched once (the BN elementwise passes: +35-45 % bandwidth on
// 200-800 MB tensors, profiles/r6/elemt_variants.md)
template <bool NT = false>
__device__ __forceinline__ void load8_bf16(const uint16_t* p, float v[8]) {
  u32x4 w;
  if constexpr (NT) w = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  else w = *reinterpret_cast<const u32x4*>(p);
  uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(ws[i] << 16);
    v[2 * i + 1] = __uint_as_float(ws[i] & 0xffff0000u);
  }
}
template <bool NT = false>
__device__ __forceinline__ void store8_bf16(uint16_t* p, const float v[8]) {
  uint32_t ws[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) ws[i] = pack_bf16x2_rne(v[2 * i], v[2 * i + 1]);
  const u32x4 w{ws[0], ws[1], ws[2], ws[3]};
  if constexpr (NT) __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(p));
  else *reinterpret_cast<u32x4*>(p) = w;
}

// Item range of one lane in a per-channel elementwise pass over nvec 8-channel vectors (tpc = C/8
// vectors per pixel). span > 0, one-shot: block b owns items [b*span, (b+1)*span) and its lanes step
// by 256 (host: tpc | 256, so every item of a lane has channel group t % tpc). span == 0,
// grid-stride: items b*256 + t + k*gridDim*256 (host: that stride % tpc == 0). One-shot grids of
// 512-item blocks beat the 2048-block grid-stride loop by 30-45 % on large tensors
// (profiles/r6/elemt_variants.md).
struct ElemRange {
  int64_t v, stride, hi;
};
__device__ __forceinline__ ElemRange elem_range(int64_t nvec, int span) {
  if (span > 0) {
    const int64_t lo = (int64_t)blockIdx.x * span;
    const int64_t end = lo + span;
    return {lo + threadIdx.x, (int64_t)blockDim.x, end < nvec ? end : nvec};
  }
  return {(int64_t)blockIdx.x * blockDim.x + threadIdx.x, (int64_t)gridDim.x * blockDim.x, nvec};
}

// Division by a run-time-invariant divisor d >= 1 for 0 <= x < 2^31 (Granlund-Montgomery
// round-up form): q = (umulhi(x, m) + x) >> s, m and s computed once on the host. A 64-bit `/` or
// `%` is a ~100-instruction software sequence on the VALU; the grid-stride index maps of the stem's
// pool kernels did five of them per 16-byte item (1,365 VALU per wave-iteration, profiles/pmc_r1.md).
struct FastDiv {
  uint32_t d, m, s;
};
inline FastDiv make_fastdiv(uint32_t d) {
  uint32_t s = 0;
  while ((1ull << s) < d) ++s;
  const uint64_t m = ((uint64_t)1 << 32) * ((1ull << s) - d) / d + 1;
  return FastDiv{d, (uint32_t)m, s};
}
__device__ __forceinline__ uint32_t fdiv_q(uint32_t x, const FastDiv& f) { return (__umulhi(x, f.m) + x) >> f.s; }

// Grid size for a grid-stride streaming kernel: enough blocks to fill 256 CUs several times
// over, capped so that launch + tail cost stays small (guide G11: <= ~2048 blocks).
inline int stream_grid(int64_t work_items, int block) {
  int64_t g = (work_items + block - 1) / block;
  if (g < 1) g = 1;
  if (g > 2048) g = 2048;
  return (int)g;
}

// Counter-based dropout keep decision shared by the fused LayerNorm and attention kernels: one
// murmur3 finalizer per PAIR of elements (idx >> 1), each element taking 16 bits of it against the
// 16-bit threshold thresh32 >> 16 (keep probability resolution 2^-16). Forward and backward call it
// with the same (key, idx), so the backward regenerates the forward's mask. (Two finalizers per
// element before: the hash was ~a quarter of the LayerNorm passes' time.)
__device__ __forceinline__ uint32_t drop_mix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}
__device__ __forceinline__ uint32_t drop_pair_bits(uint32_t key, uint64_t idx) {
  const uint64_t pr = idx >> 1;
  return drop_mix32(key ^ (uint32_t)pr * 0x9e3779b9u ^ (uint32_t)(pr >> 32) * 0x7f4a7c15u);
}
__device__ __forceinline__ bool drop_keep(uint32_t key, uint64_t idx, uint32_t thresh32) {
  const uint32_t h = drop_pair_bits(key, idx);
  const uint32_t bits = (idx & 1) ? (h >> 16) : (h & 0xffffu);
  return bits >= (thresh32 >> 16);
}

}  // namespace psd
