#pragma once
#include <hip/hip_runtime_api.h>
#include <cstdint>

namespace psd {
// 7x7/s2/p3 3->64 NHWC bf16 stem convolution (kernels/stem.hip). wk = weights repacked as
// [64][192] (k = kh*24 + kw*3 + ci, zero elsewhere); part receives stem_conv_blocks() rows of
// [2][64] shifted BN partial sums (shift = running mean, may be null).
bool stem_conv_supported(int H, int W, int Ho, int Wo);
int stem_conv_blocks(int N, int Ho);
hipError_t launch_stem_conv(const uint16_t* x, const uint16_t* wk, uint16_t* y, const float* shift, float* part, int N,
                            int H, int W, int Ho, int Wo, hipStream_t stream);
// Weight gradient of the stem conv: dw = bf16 [64][7][7][3] (the channels_last [64,3,7,7] layout)
// from the image x and the conv-output gradient dy [N, Ho, Wo, 64]; part = stem_wgrad_blocks() x
// 192 x 64 fp32 workspace.
bool stem_wgrad_supported(int H, int W, int Ho, int Wo);
int stem_wgrad_blocks(int N, int Ho, int Wo);
hipError_t launch_stem_wgrad(const uint16_t* x, const uint16_t* dy, float* part, uint16_t* dw, int N, int H, int W,
                             int Ho, int Wo, hipStream_t stream);
}  // namespace psd
