#pragma once
#include <hip/hip_runtime_api.h>
#include <cstdint>

namespace psd {
hipError_t launch_maxpool_fwd(const uint16_t* x, uint16_t* y, uint8_t* arg, int N, int H, int W, int C, int Ho, int Wo,
                              hipStream_t stream);
hipError_t launch_maxpool_bwd(const uint16_t* dy, const uint8_t* arg, uint16_t* dx, int N, int H, int W, int C, int Ho,
                              int Wo, hipStream_t stream);
}  // namespace psd
