// Launch API of the MFMA bf16 GEMM (gemm.hip).
#pragma once
#include <hip/hip_runtime_api.h>
#include <cstdint>

namespace psd {

struct GemmArgs {
  const void* A;     // bf16; a_kmajor ? [M][lda] : [K][lda]
  const void* B;     // bf16; b_kmajor ? [N][ldb] : [K][ldb]
  void* C;           // [M][ldc] bf16 (or fp32 if c_f32); split-K: fp32 slabs
  const void* bias;  // bf16 [N] or null
  void* aux;         // GELU pre-activation out [M][ldc] bf16 or null
  int M, N, K;
  int lda, ldb, ldc;
  int a_kmajor, b_kmajor;
  int act;           // 0 none, 1 relu, 2 gelu(tanh), 3 GELU backward (aux = pre in, part = colsum partials)
  int c_f32;
  int k_per_split;
  const float* a_scale;  // fp8 GEMM: dequant factors (device scalars), else unused
  const float* b_scale;
  // implicit-GEMM convolution (launch_conv_fwd): A = NHWC input [Nb][H][W][C], M = Nb*Ho*Wo output
  // pixels, K = R*S*C ordered (r, s, ci), C a power of two >= 64; B = weights [Cout][R][S][C]
  int cv_H, cv_W, cv_logC, cv_Ho, cv_Wo, cv_S, cv_stride, cv_pad;
  uint32_t cv_abytes;  // input tensor bytes
  int f8a;             // fp8 GEMMs: format of A (0 OCP e4m3, 1 OCP e5m2); B is always e4m3
  // MX fp8 (both set: block-scaled instead of a_scale / b_scale): E8M0 scale bytes per 32 contiguous
  // K-elements, A [M][K/32] (implicit-GEMM conv: of the input, [pixels][C/32]), B [N][K/32]
  const uint8_t* a_mx;
  const uint8_t* b_mx;
  // the consumer BatchNorm's batch statistics in the epilogue (single-split bf16 8-phase GEMMs, no
  // bias / activation): part [rows][2][N] fp32 shifted sums, shift [N] fp32; *rows_out <- rows
  float* part;
  const float* shift;
  int* rows_out;
};

hipError_t launch_gemm(const GemmArgs& g, hipStream_t stream);
// transposed store on 192 x 256 tiles: C [N][ldc] = (A . B^T)^T (+ bias[M])(act 0-2, aux), A [M][K] and
// B [N][K] K-major, M % 8 == 0, K % 64 == 0; hipErrorNotSupported outside that contract
hipError_t launch_gemm_ct(const GemmArgs& g, hipStream_t stream);
// C = (A_e4m3 . B_e4m3^T) * a_scale * b_scale (+bias)(act); A [M][K], B [N][K] fp8, K % 128 == 0
hipError_t launch_gemm_fp8(const GemmArgs& g, hipStream_t stream);
int gemm_splits(int M, int N, int K);
// split-K GEMMs with an N-major B: stage each B half as contiguous 128-column rows (whole 128-byte lines)
// instead of the quadrant-interleaved halves. Default off: no faster on the BERT weight gradients.
void gemm_set_bcontig(bool on);
// out[M][Cout] = conv(x, w) (NHWC, no bias / activation), on the persistent 8-phase kernel with A
// gathered from the input; hipErrorNotSupported when the shape is outside that kernel's contract
hipError_t launch_conv_fwd(const GemmArgs& g, hipStream_t stream);
// the same with x and w OCP e4m3 (C % 128 == 0), dequantised by *a_scale * *b_scale (bf16 out)
hipError_t launch_conv_fwd_fp8(const GemmArgs& g, hipStream_t stream);
// implicit-GEMM weight gradient: out [Cout][R*S*C] bf16 = dY^T . im2col(x) (A = dY [pixels][Cout],
// B = x NHWC, K = pixels % 64 == 0), split-K into slab [splits][Cout][R*S*C] fp32 + reduce;
// hipErrorNotSupported outside the kernel's contract
hipError_t launch_conv_wgrad(const GemmArgs& g, float* slab, int splits, void* out, hipStream_t stream);
// out = (accumulate ? out : 0) + scale * sum_s slab[s] over mn elements (bf16 or fp32 out). With
// `tree` (splitk_tree_floats(splits, mn) fp32 of workspace) many splits are summed in levels of 8
// first; the slab is then overwritten.
int64_t splitk_tree_floats(int splits, int64_t mn);
hipError_t launch_splitk_reduce(float* slab, int splits, int64_t mn, void* out, int out_bf16, int accumulate,
                                float scale, hipStream_t stream, float* tree = nullptr);
// split-K GEMM into fp32 slabs [splits][M][N], then out = (acc ? out : 0) + scale * sum(slabs)
hipError_t launch_gemm_splitk(const GemmArgs& g, float* slab, int splits, void* out, int out_bf16, int accumulate,
                              float scale, hipStream_t stream);
// out[n] (+)= sum_m x[m][n]; part is an fp32 [kColsumPartRows * N] scratch
constexpr int kColsumPartRows = 2048;
// pre/xo (optional): x is dy of a GELU(tanh) output; xo = bf16(dy * gelu'(pre)) is written and summed
// out[n] (+)= sum of the rows rows of part[rows][N] (the second pass of launch_colsum)
hipError_t launch_colsum_final(const float* part, int rows, int N, void* out, int out_bf16, int accumulate,
                               hipStream_t stream);
hipError_t launch_colsum(const uint16_t* x, int64_t M, int N, float* part, void* out, int out_bf16,
                         int accumulate, hipStream_t stream, const uint16_t* pre = nullptr, uint16_t* xo = nullptr);

}  // namespace psd
