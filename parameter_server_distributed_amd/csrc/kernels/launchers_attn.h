#pragma once
#include <hip/hip_runtime_api.h>
#include <cstdint>

namespace psd {
// Fused short-sequence self-attention (kernels/attention.hip): packed qkv [B, S, 3, H, 64] in,
// o [B, S, H, 64] out; backward writes the packed dqkv.
struct AttnArgs {
  const uint16_t* qkv;    // [B, S, 3, H, 64] bf16
  uint16_t* o;            // fwd out / bwd in: [B, S, H, 64] bf16
  float* lse;             // fwd out / bwd in: [B, H, S] fp32 (natural-log row log-sum-exp)
  const uint16_t* dout;   // bwd in: [B, S, H, 64] bf16
  uint16_t* dqkv;         // bwd out: [B, S, 3, H, 64] bf16
  float* bpart;           // bwd out or null: [B][3*H*64] fp32 column sums of dqkv over each sequence
                          // (the QKV Linear's bias gradient, summed over B by the caller)
  const int64_t* step;    // device step counter mixed into the dropout hash (may be null)
  int32_t B, S, H;
  float scale;            // softmax scale (1/sqrt(64))
  uint32_t thresh;        // dropout: drop when hash < thresh (0: no dropout)
  float rescale;          // 1 / (1 - p)
  uint32_t seed;
};
bool attn_supported(int S, int head_dim);
hipError_t launch_attn_fwd(const AttnArgs& a, hipStream_t stream);
hipError_t launch_attn_bwd(const AttnArgs& a, hipStream_t stream);
}  // namespace psd
