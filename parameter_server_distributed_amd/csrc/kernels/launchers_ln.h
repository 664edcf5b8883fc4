#pragma once
#include <hip/hip_runtime_api.h>
#include <cstdint>

namespace psd {
// y = LayerNorm(x + dropout_p(h)) over rows of H (kernels/layernorm.hip) and its backward.
struct LnArgs {
  const uint16_t* x;      // fwd: residual input [rows, H] bf16
  const uint16_t* h;      // fwd: branch output (dropout applied) [rows, H] bf16
  const uint16_t* gamma;  // [H] bf16
  const uint16_t* beta;   // [H] bf16
  uint16_t* y;            // fwd out [rows, H]
  uint16_t* s;            // fwd out / bwd in: x + dropout(h), the LN input, bf16
  float* mean;            // [rows]
  float* rstd;            // [rows]
  const uint16_t* dy;     // bwd in
  uint16_t* dx;           // bwd out: gradient of x (= of s)
  uint16_t* dh;           // bwd out: gradient of h (dropout mask applied)
  uint16_t* dgamma;       // bwd out [H] bf16 (may be the PS gradient sink)
  uint16_t* dbeta;        // bwd out [H] bf16
  uint16_t* dhsum;        // bwd out [H] bf16 or null: column sums of dh (the branch Linear's bias gradient)
  float* part;            // bwd workspace [ln_bwd_blocks(rows)][3][H] fp32 ([2] without dhsum)
  const int64_t* step;    // device step counter mixed into the dropout hash (may be null)
  int64_t rows;
  int32_t H;
  float eps;
  float p;                // dropout probability (0: identity)
  uint32_t seed;          // per call site
};
// BERT's embedding tail y = dropout_p(LayerNorm(W[id] + P[row % S] + T[type])) (kernels/layernorm.hip)
// and its backward: dx (the gradient of the embedding sum, for the word table's sorted scatter),
// dgamma / dbeta and -- for <= 2 token types -- the type table's gradient, all from one pass.
struct EmbLnArgs {
  const int64_t* ids;     // [rows] word ids (outside [0, V): a zero row)
  const int64_t* types;   // [rows] token types (outside [0, NT): a zero row)
  const uint16_t* W;      // [V, H] word table
  const uint16_t* P;      // [>= S, H] position table (row = row index % S)
  const uint16_t* T;      // [NT, H] token-type table
  const uint16_t* gamma;  // [H]
  const uint16_t* beta;   // [H]
  uint16_t* y;            // fwd out [rows, H]
  float* mean;            // [rows]
  float* rstd;            // [rows]
  const uint16_t* dy;     // bwd in [rows, H]
  uint16_t* dx;           // bwd out [rows, H]: gradient of the embedding sum
  uint16_t* dgamma;       // bwd out [H]
  uint16_t* dbeta;        // bwd out [H]
  uint16_t* dT;           // bwd out [NT, H] (NT <= 2), or null
  float* part;            // bwd workspace [emb_ln_bwd_blocks(rows)][2 + NT][H]
  const int64_t* step;    // device step counter for the dropout hash (may be null)
  int64_t rows;
  int64_t V;
  int32_t S;
  int32_t NT;
  int32_t H;
  float eps;
  float p;
  uint32_t seed;
};
bool ln_supported(int H);
int ln_bwd_blocks(int64_t rows);
hipError_t launch_ln_fwd(const LnArgs& a, hipStream_t stream);
hipError_t launch_ln_bwd(const LnArgs& a, hipStream_t stream);
int emb_ln_bwd_blocks(int64_t rows);
hipError_t launch_emb_ln_fwd(const EmbLnArgs& a, hipStream_t stream);
hipError_t launch_emb_ln_bwd(const EmbLnArgs& a, hipStream_t stream);
}  // namespace psd
