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
  // bwd-data with the producing BN's backward reduction in the epilogue (bwd 1 / 2, convn.hip);
  // part then receives sum g and sum g (x - mean) per channel
  int bwd;
  const uint16_t* bx;     // [M][N] the BN's input (its forward x)
  const float* bmean;     // [N] its saved mean
  const float* bss;       // bwd 1: [2N] its forward scale / shift (ReLU mask)
  const uint16_t* bdr;    // bwd 2: [M][N] the residual-branch gradient to add
  const uint8_t* bmbits;  // bwd 2: [M*N/8] the forward ReLU bit-mask
  // bwd 3 (dual tail relu(bn(x) + bnd(xd))): bnd's input, its saved mean and its partials
  const uint16_t* bxd;
  const float* bmean_d;
  float* part_d;
  // K-concatenated second operand (1x1 only): A(m, k) = x2[m][k - K1] for k >= K1, so
  // y = [x | x2] . w^T with w [N][K1 + C2] (the BN-backward fold of ops/bn.py: dgrad of a 1x1 conv
  // whose BN input gradient is never materialised)
  const void* x2;         // bf16 [M][C2], C2 = 1 << logC2 >= 64
  uint32_t x2bytes;
  int K1, logC2;
  const float* bias;      // optional fp32 [N] added to the output in the epilogue (before bwd / stats)
  // bwd 8 (a forward epilogue, despite the field name): y = relu(bf16(conv) * bss[c] + bss[N + c] +
  // ares) with its ReLU bit-mask into amask [M*N/8] -- the BN apply of a convolution output that is
  // never stored (ops/tail.py: statistics pass with y = nullptr, then this apply pass)
  const uint16_t* ares;
  uint8_t* amask;
  // stride-2 bwd-data phase launch (gathered variants): 0 = none, else 1 + (ph << 1 | pw); the M rows
  // of the Ho x Wo grid land at pixels (n, 2i + ph, 2j + pw) of a 2Ho x 2Wo output (convn.hip pix)
  int ophase;
};

// output-channel tile of the kernel for N output channels (64, 128, 256 for N % 256 == 0), 0: unsupported
int convn_tile_n(int N);
// rows to allocate for the statistics partials of M output pixels (any variant)
int convn_stats_rows(int M);
// rows a launch with this variant writes (one per 64-pixel wave row of every tile); HALO variants
// tile by output rows: _geo with the convolution's output height / width and kernel size
int convn_part_rows(int M, int N, int variant);
int convn_part_rows_geo(int M, int N, int variant, int Ho, int Wo, int R);
// variant v of an N-wide output is usable for this convolution (HALO: stride 1, R = S <= 3, pad
// R / 2, Wo + R - 1 <= 64, no second operand)
bool convn_variant_ok(int N, int v, int R, int S, int stride, int pad, int Wo, bool has_x2);
int convn_variants(int N);
// 0: gathered, 2: persistent HALO (convh_kernel: C = N = 64, 3x3 / stride 1 / pad 1,
// Wo <= 62, resident weights, double-buffered windows), 3: persistent 1x1 (convp / convpr),
// 4: the persistent 1x1 at two workgroups per CU; -1: no such variant
int convn_variant_kind(int N, int v);
// hipErrorNotSupported outside the kernel's contract (nothing launched)
hipError_t launch_convn(const ConvnArgs& a, hipStream_t stream);

}  // namespace psd
