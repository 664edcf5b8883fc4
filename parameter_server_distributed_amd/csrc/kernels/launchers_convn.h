// Launch API of the narrow-output implicit-GEMM convolution (convn.hip).
#pragma once
#include <hip/hip_runtime_api.h>
#include <cstdint>

namespace psd {

struct ConvnArgs {
  const void* x;       // NHWC bf16 input [Nb][H][W][C], C a power of two >= 64
  const void* w;       // bf16 [N][K] weights, K = R*S*C ordered (r, s, ci)
  void* y;             // bf16 [M][ldc] output, M = Nb*Ho*Wo
  float* part;         // optional: BN statistics partials [convn_stats_rows(M)][2][N] (needs shift)
  const float* shift;  // [N] fp32 shift k of the partial sums sum(y - k), sum((y - k)^2)
  uint32_t xbytes;     // bytes of x (< 2^32 - 256)
  uint32_t wbytes;     // bytes of w
  int M, N, K;
  int H, W, logC, Ho, Wo, R, S, stride, pad;
  int ldc;
  int variant;  // tile geometry (convn_variants(N) of them); -1: the default
  int nslot;    // set by the launcher
};

// output-channel tile of the kernel for N output channels (64, 128, 256 for N % 256 == 0), 0: unsupported
int convn_tile_n(int N);
// rows to allocate for the statistics partials of M output pixels (any variant)
int convn_stats_rows(int M);
// rows a launch with this variant writes (one per 64-pixel wave row of every tile)
int convn_part_rows(int M, int N, int variant);
int convn_variants(int N);
// hipErrorNotSupported outside the kernel's contract (nothing launched)
hipError_t launch_convn(const ConvnArgs& a, hipStream_t stream);

}  // namespace psd
