// Launch API of the fused softmax cross-entropy (xent.hip).
#pragma once
#include <hip/hip_runtime_api.h>
#include <cstdint>

namespace psd {
// per row r of bf16 logits x [rows][ldx] (V valid columns): lse[r] and loss_row[r] = lse - x[label]
hipError_t launch_xent_fwd(const uint16_t* x, const int64_t* labels, int64_t rows, int64_t V, int64_t ldx, float* lse,
                           float* loss_row, hipStream_t stream);
// dx [rows][V] bf16 = (softmax(x) - onehot(label)) * *scale (rows with label < 0: 0)
hipError_t launch_xent_bwd(const uint16_t* x, const int64_t* labels, const float* lse, const float* scale, int64_t rows,
                           int64_t V, int64_t ldx, uint16_t* dx, hipStream_t stream);
}  // namespace psd
