// Embedding weight gradient for gfx950 (BERT's word embedding: 32768 tokens into a 30528 x 768
// table per step), deterministic without atomics.
//
// Why: PyTorch's dense embedding backward (sort, segment offsets, per-segment partial sums,
// sum_and_scatter) took ~0.35 ms per call at b256 x 128 tokens (profiles/bert_base_b256_r4
// kernel table). Here the ids are stable-sorted once (torch.sort, the stable merge sort) and one
// wave per sorted position i that STARTS a run of equal ids sums the run's dy rows in token order
// (fp32, 4 columns per lane per 256-column chunk) and writes the table row; every other wave exits
// at once. The table is zero-filled by the caller (rows with no token keep their zero gradient).
#include "common.h"
#include "launchers_embed.h"

namespace psd {

template <int NC>
__global__ __launch_bounds__(256) void embed_bwd_kernel(const int64_t* __restrict__ sorted, const int64_t* __restrict__ perm,
                                                        const uint16_t* __restrict__ dy, int64_t T, int Hd,
                                                        uint16_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= T) return;
  const int64_t id = sorted[i];
  if (i > 0 && sorted[i - 1] == id) return;  // not the first token of its run
  float acc[NC][4];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[c][e] = 0.f;
  for (int64_t j = i; j < T && sorted[j] == id; ++j) {
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
  uint16_t* o = out + id * Hd + lane * 4;
#pragma unroll
  for (int c = 0; c < NC; ++c)
    *reinterpret_cast<uint2*>(o + c * 256) =
        make_uint2(pack_bf16x2_rne(acc[c][0], acc[c][1]), pack_bf16x2_rne(acc[c][2], acc[c][3]));
}

hipError_t launch_embed_bwd(const int64_t* sorted, const int64_t* perm, const uint16_t* dy, int64_t T, int Hd,
                            uint16_t* out, hipStream_t st) {
  if (T <= 0) return hipSuccess;
  if (Hd % 256 != 0 || Hd > 256 * 8) return hipErrorInvalidValue;
  const dim3 grid((unsigned)((T + 3) / 4));
  switch (Hd / 256) {
    case 1: hipLaunchKernelGGL(embed_bwd_kernel<1>, grid, dim3(256), 0, st, sorted, perm, dy, T, Hd, out); break;
    case 2: hipLaunchKernelGGL(embed_bwd_kernel<2>, grid, dim3(256), 0, st, sorted, perm, dy, T, Hd, out); break;
    case 3: hipLaunchKernelGGL(embed_bwd_kernel<3>, grid, dim3(256), 0, st, sorted, perm, dy, T, Hd, out); break;
    case 4: hipLaunchKernelGGL(embed_bwd_kernel<4>, grid, dim3(256), 0, st, sorted, perm, dy, T, Hd, out); break;
    default: hipLaunchKernelGGL(embed_bwd_kernel<8>, grid, dim3(256), 0, st, sorted, perm, dy, T, Hd, out); break;
  }
  return hipGetLastError();
}

}  // namespace psd
