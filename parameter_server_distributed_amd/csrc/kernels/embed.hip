// Embedding weight gradient for gfx950 (BERT's word embedding: 32768 tokens into a 30528 x 768
// table per step), deterministic without atomics.
//
// Why: PyTorch's dense embedding backward (sort, segment offsets, per-segment partial sums,
// sum_and_scatter) took ~0.35 ms per call at b256 x 128 tokens (profiles/bert_base_b256_r4
// kernel table). Here the ids are stable-sorted once (torch.sort, the stable merge sort) and the
// sorted positions are cut into segments: a segment starts where a run of equal ids starts or at
// a multiple of CH, so no wave sums more than CH rows however skewed the ids are (an MLM batch has
// thousands of [PAD] / [CLS] / [SEP] tokens: one wave walking a 10^4-row run serially took
// milliseconds). Two launches, both one wave per sorted position that starts a segment (every
// other wave exits at once):
//   pass 1  a segment that continues a run (starts at a multiple of CH inside it) sums its rows in
//           token order into an fp32 partial, slot = position / CH;
//   pass 2  a run's first segment sums its own rows, then adds the run's pass-1 partials in slot
//           order, and writes the bf16 table row.
// The summation order is fixed by the sort, so the gradient is bitwise reproducible. The table is
// zero-filled by the caller (rows with no token keep their zero gradient).
#include "common.h"
#include "launchers_embed.h"

namespace psd {

template <int NC>
__device__ __forceinline__ void embed_sum_rows(const int64_t* __restrict__ sorted, const int64_t* __restrict__ perm,
                                               const uint16_t* __restrict__ dy, int64_t i, int64_t end, int64_t id,
                                               int Hd, int lane, float (&acc)[NC][4]) {
  for (int64_t j = i; j < end && sorted[j] == id; ++j) {
    const uint16_t* row = dy + perm[j] * Hd + lane * 4;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const uint2 w = *reinterpret_cast<const uint2*>(row + c * 256);
      acc[c][0] += __uint_as_float(w.x << 16);
      acc[c][1] += __uint_as_float(w.x & 0xffff0000u);
      acc[c][2] += __uint_as_float(w.y << 16);
      acc[c][3] += __uint_as_float(w.y & 0xffff0000u);
    }
  }
}

template <int NC, bool PARTIAL>
__global__ __launch_bounds__(256) void embed_bwd_kernel(const int64_t* __restrict__ sorted, const int64_t* __restrict__ perm,
                                                        const uint16_t* __restrict__ dy, int64_t T, int Hd,
                                                        float* __restrict__ part, uint16_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= T) return;
  const int64_t id = sorted[i];
  const bool run_start = i == 0 || sorted[i - 1] != id;
  if (PARTIAL ? (run_start || (i % kEmbedChunk) != 0) : !run_start) return;
  float acc[NC][4];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[c][e] = 0.f;
  const int64_t seg_end = (i / kEmbedChunk + 1) * kEmbedChunk;
  embed_sum_rows<NC>(sorted, perm, dy, i, seg_end < T ? seg_end : T, id, Hd, lane, acc);
  if (PARTIAL) {
    float* p = part + (i / kEmbedChunk) * Hd + lane * 4;
#pragma unroll
    for (int c = 0; c < NC; ++c)
      *reinterpret_cast<float4*>(p + c * 256) = make_float4(acc[c][0], acc[c][1], acc[c][2], acc[c][3]);
    return;
  }
  for (int64_t s = seg_end; s < T && sorted[s] == id; s += kEmbedChunk) {
    const float* p = part + (s / kEmbedChunk) * Hd + lane * 4;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const float4 v = *reinterpret_cast<const float4*>(p + c * 256);
      acc[c][0] += v.x;
      acc[c][1] += v.y;
      acc[c][2] += v.z;
      acc[c][3] += v.w;
    }
  }
  uint16_t* o = out + id * Hd + lane * 4;
#pragma unroll
  for (int c = 0; c < NC; ++c)
    *reinterpret_cast<uint2*>(o + c * 256) =
        make_uint2(pack_bf16x2_rne(acc[c][0], acc[c][1]), pack_bf16x2_rne(acc[c][2], acc[c][3]));
}

template <int NC>
static void embed_launch(const int64_t* sorted, const int64_t* perm, const uint16_t* dy, int64_t T, int Hd,
                         float* part, uint16_t* out, hipStream_t st) {
  const dim3 grid((unsigned)((T + 3) / 4));
  if (T > kEmbedChunk)
    hipLaunchKernelGGL((embed_bwd_kernel<NC, true>), grid, dim3(256), 0, st, sorted, perm, dy, T, Hd, part, out);
  hipLaunchKernelGGL((embed_bwd_kernel<NC, false>), grid, dim3(256), 0, st, sorted, perm, dy, T, Hd, part, out);
}

hipError_t launch_embed_bwd(const int64_t* sorted, const int64_t* perm, const uint16_t* dy, int64_t T, int Hd,
                            float* part, uint16_t* out, hipStream_t st) {
  if (T <= 0) return hipSuccess;
  if (Hd % 256 != 0 || Hd > 256 * 8) return hipErrorInvalidValue;
  switch (Hd / 256) {
    case 1: embed_launch<1>(sorted, perm, dy, T, Hd, part, out, st); break;
    case 2: embed_launch<2>(sorted, perm, dy, T, Hd, part, out, st); break;
    case 3: embed_launch<3>(sorted, perm, dy, T, Hd, part, out, st); break;
    case 4: embed_launch<4>(sorted, perm, dy, T, Hd, part, out, st); break;
    default: embed_launch<8>(sorted, perm, dy, T, Hd, part, out, st); break;
  }
  return hipGetLastError();
}

}  // namespace psd
