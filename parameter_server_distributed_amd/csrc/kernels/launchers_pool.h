#pragma once
#include <hip/hip_runtime_api.h>
#include <cstdint>

namespace psd {
hipError_t launch_maxpool_fwd(const uint16_t* x, uint16_t* y, uint8_t* arg, int N, int H, int W, int C, int Ho, int Wo,
                              hipStream_t stream);
hipError_t launch_maxpool_bwd(const uint16_t* dy, const uint16_t* dy2, const uint8_t* arg, uint16_t* dx, int N, int H, int W, int C, int Ho,
                              int Wo, hipStream_t stream);
// global average pool over HW of NHWC bf16 [N, HW, C] <-> [N, C]
hipError_t launch_gap_fwd(const uint16_t* x, uint16_t* y, int N, int HW, int C, hipStream_t stream);
hipError_t launch_gap_bwd(const uint16_t* dy, uint16_t* dx, int N, int HW, int C, hipStream_t stream);
// y [N, H/2, W/2, C] = x[:, ::2, ::2, :] (NHWC bf16, C % 8 == 0, H and W even)
hipError_t launch_subsample2(const uint16_t* x, uint16_t* y, int N, int H, int W, int C, hipStream_t stream);
}  // namespace psd
