// Launch API of the embedding weight-gradient kernel (embed.hip).
#pragma once
#include <hip/hip_runtime_api.h>
#include <cstdint>

namespace psd {
// sorted positions summed by one wave at most (a longer run of equal ids is split into segments)
constexpr int kEmbedChunk = 64;
// out[sorted[i]] = sum of dy[perm[j]] over the run of equal sorted ids (ids stable-sorted, perm the
// sort permutation); out [V][Hd] bf16, zero-filled by the caller; Hd % 256 == 0, Hd <= 2048;
// part: fp32 scratch of ceil(T / kEmbedChunk) x Hd (the per-segment partial sums of long runs)
hipError_t launch_embed_bwd(const int64_t* sorted, const int64_t* perm, const uint16_t* dy, int64_t T, int Hd,
                            float* part, uint16_t* out, hipStream_t stream);
}  // namespace psd
