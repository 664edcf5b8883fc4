// BN-backward fold for a 1x1 convolution followed by a BatchNorm (ResNet's conv3 -> bn3): the BN's
// input gradient  dy = A g + B y + C  (per channel c; g the masked upstream gradient, y = x W^T the
// conv output, kernels/bn.hip bn_bwd_finalize_kernel) is never materialised. Its two consumers are
// rewritten onto g and the conv input x, which the GEMMs read anyway:
//
//   dgrad  dx = dy W = [g | x] . [ (A o W)^T | W^T (B o W) ]^T + (C^T W)     (K = Cout + Cin)
//   wgrad  dW = dy^T x = A o (g^T x) + B o (W (x^T x)) + C (1^T x)
//
// kernels/convn.hip runs the dgrad with the K-concatenated operand and the bias, kernels/convw.hip the
// wgrad products g^T x, x^T x and 1^T x in one pass. This file holds the small per-step kernels
// around them: the folded dgrad weight and bias (prep) and the wgrad combination (combine). What the
// fold removes per bottleneck: the BN elementwise pass (read g and y, write dy: three full
// activations) -- ~1 ms per layer1 block at b1024 (profiles/resnet50_b1024_r3s3_kernels.md).
#include "common.h"
#include "launchers_bn.h"

namespace psd {

// one block per input channel j: w2[j][c] = A_c W[c][j] (c < Cout, row stride ldw), bw[c][j] = B_c W[c][j],
// bvec[j] = sum_c C_c W[c][j]
__global__ __launch_bounds__(256) void bnfold_prep_kernel(const uint16_t* __restrict__ W, const float* __restrict__ coef,
                                                          int Cout, int Wd, uint16_t* __restrict__ w2, int ldw,
                                                          uint16_t* __restrict__ bw, float* __restrict__ bvec) {
  __shared__ float red[256];
  const int j = blockIdx.x;
  float acc = 0.f;
  for (int c = threadIdx.x; c < Cout; c += blockDim.x) {
    const float w = bf16_to_f32(W[(int64_t)c * Wd + j]);
    w2[(int64_t)j * ldw + c] = f32_to_bf16(coef[c] * w);
    bw[(int64_t)c * Wd + j] = f32_to_bf16(coef[Cout + c] * w);
    acc = fmaf(coef[2 * Cout + c], w, acc);
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) bvec[j] = red[0];
}

// dW[c][i] = A_c P[c][i] + B_c sum_k W[c][k] G[k][i] + C_c s[i]  (G = P[Cout:Cout+Wd] = x^T x,
// s = P[Cout+Wd] = 1^T x). The W G product is a small fp32 GEMM on 32 x 32 output tiles, k in chunks
// of 32 staged through LDS (W transposed: a thread's 2 rows are one float2), 2 x 2 outputs per lane.
// The chunks are software-pipelined -- chunk k0 + 32's W and G loads are in registers before chunk
// k0's FMAs run -- and the tiles are small enough for several workgroups per CU: the 64 x 64 tile
// with a load -> sync -> compute chain per chunk ran 43 us per call on average, latency-bound (4 to
// 256 workgroups per launch; 0.65 ms per ResNet-50 step, profiles/r6/resnet50_b1024_r6f_kernels.md).
// The k order of every output's sum is unchanged (bitwise the same result).
constexpr int kCT = 32, kCK = 32;
__global__ __launch_bounds__(256) void bnfold_combine_kernel(const float* __restrict__ P, const uint16_t* __restrict__ W,
                                                             const float* __restrict__ coef, int Cout, int Wd,
                                                             uint16_t* __restrict__ out, int accumulate) {
  // W^T chunk ws[k][r], rows padded by 2 floats: the transposing stores (consecutive lanes =
  // consecutive k) spread over the banks instead of all hitting one; float2 reads stay aligned
  __shared__ __attribute__((aligned(16))) float ws[kCK][kCT + 2];
  __shared__ __attribute__((aligned(16))) float gs[kCK][kCT];  // G chunk: gs[k][i]
  const int r0 = blockIdx.x * kCT, i0 = blockIdx.y * kCT;
  const int tr = threadIdx.x >> 4, tc = threadIdx.x & 15;
  const float* G = P + (int64_t)Cout * Wd;
  const float* s = G + (int64_t)Wd * Wd;
  constexpr int kPer = kCK * kCT / 256;  // elements of each operand a lane stages per chunk (4)
  float wr[kPer], gr[kPer];
  auto load = [&](int k0) {
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int e = threadIdx.x + q * 256;
      const int r = e / kCK, k = e - r * kCK;  // consecutive lanes: consecutive k of one W row
      wr[q] = (r0 + r < Cout && k0 + k < Wd) ? bf16_to_f32(W[(int64_t)(r0 + r) * Wd + k0 + k]) : 0.f;
      const int kg = e / kCT, i = e - kg * kCT;
      gr[q] = (k0 + kg < Wd && i0 + i < Wd) ? G[(int64_t)(k0 + kg) * Wd + i0 + i] : 0.f;
    }
  };
  float t[2][2] = {{0.f, 0.f}, {0.f, 0.f}};
  load(0);
  for (int k0 = 0; k0 < Wd; k0 += kCK) {
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int e = threadIdx.x + q * 256;
      const int r = e / kCK, k = e - r * kCK;
      ws[k][r] = wr[q];
      const int kg = e / kCT, i = e - kg * kCT;
      gs[kg][i] = gr[q];
    }
    __syncthreads();
    if (k0 + kCK < Wd) load(k0 + kCK);  // next chunk in flight during this chunk's FMAs
#pragma unroll 8
    for (int k = 0; k < kCK; ++k) {
      const float2 wa = *reinterpret_cast<const float2*>(&ws[k][tr * 2]);
      const float2 gb = *reinterpret_cast<const float2*>(&gs[k][tc * 2]);
      t[0][0] = fmaf(wa.x, gb.x, t[0][0]);
      t[0][1] = fmaf(wa.x, gb.y, t[0][1]);
      t[1][0] = fmaf(wa.y, gb.x, t[1][0]);
      t[1][1] = fmaf(wa.y, gb.y, t[1][1]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const int c = r0 + tr * 2 + a;
    if (c >= Cout) break;
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int i = i0 + tc * 2 + b;
      if (i >= Wd) break;
      float v = coef[c] * P[(int64_t)c * Wd + i] + coef[Cout + c] * t[a][b] + coef[2 * Cout + c] * s[i];
      uint16_t* o = out + (int64_t)c * Wd + i;
      if (accumulate) v += bf16_to_f32(*o);
      *o = f32_to_bf16(v);
    }
  }
}

// sum_m g[m][c] y[m][c] for y = x W^T that was never stored (ops/tail.py): with P[:Cout] = g^T x
// from the fold wgrad, sum_m g y = sum_i W[c][i] P[c][i]. One wave per output channel, the row's
// bf16 weights and fp32 P entries in 8-wide lane chunks; writes the partial row (0, that sum) that
// completes the BN-backward partials of an epilogue that ran without the BN input (convn bwd modes
// 2 / 5 with bx null: sum g, -mean sum g).
__global__ __launch_bounds__(256) void bnfold_rowdot_kernel(const float* __restrict__ P, const uint16_t* __restrict__ W,
                                                            int Cout, int Wd, float* __restrict__ row) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= Cout) return;
  float acc = 0.f;
  for (int i = lane * 8; i < Wd; i += 64 * 8) {
    float w[8], p[8];
    load8_bf16(W + (int64_t)c * Wd + i, w);
    load8_f32(P + (int64_t)c * Wd + i, p);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc = fmaf(w[e], p[e], acc);
  }
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  if (lane == 0) {
    row[c] = 0.f;
    row[Cout + c] = acc;
  }
}

// Batch statistics of y = x W^T without forming y (ops/tail.py's statistics pass): with the Gram
// matrix G = x^T x and the column sums s = 1^T x (P from the Gram launch convw_gram_: rows [0, Wd) =
// G, row Wd = s), sum_m y_c = W_c . s and sum_m y_c^2 = W_c^T G W_c. Writes the shifted partial row
// (sum (y - k), sum (y - k)^2), k = shift (the running mean the finalize expects), the shift applied
// in fp64. A wave owns kGsCh output channels (their W rows staged in LDS as fp32, read as
// broadcasts) and streams G once for all of them: lane j holds u[c][j] = sum_i W[c][i] G[i][j].
constexpr int kGsCh = 4;

template <int JT>
__global__ __launch_bounds__(256) void bnfold_gram_stats_kernel(const float* __restrict__ P, const uint16_t* __restrict__ W,
                                                                const float* __restrict__ shift, int Cout, int Wd,
                                                                double M, float* __restrict__ row) {
  __shared__ float ws[4][kGsCh][JT * 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c0 = (blockIdx.x * 4 + wv) * kGsCh;
  if (c0 >= Cout) return;  // Cout % kGsCh == 0 (host): a live wave owns kGsCh real channels
#pragma unroll
  for (int k = 0; k < kGsCh; ++k)
#pragma unroll
    for (int t = 0; t < JT; ++t) ws[wv][k][t * 64 + lane] = bf16_to_f32(W[(int64_t)(c0 + k) * Wd + t * 64 + lane]);
  __builtin_amdgcn_wave_barrier();  // the wave reads back only its own rows
  const float* G = P;
  const float* cs = P + (int64_t)Wd * Wd;
  float u[kGsCh][JT];
#pragma unroll
  for (int k = 0; k < kGsCh; ++k)
#pragma unroll
    for (int t = 0; t < JT; ++t) u[k][t] = 0.f;
#pragma unroll 4
  for (int i = 0; i < Wd; ++i) {
    float g[JT];
#pragma unroll
    for (int t = 0; t < JT; ++t) g[t] = G[(int64_t)i * Wd + t * 64 + lane];
#pragma unroll
    for (int k = 0; k < kGsCh; ++k) {
      const float wk = ws[wv][k][i];
#pragma unroll
      for (int t = 0; t < JT; ++t) u[k][t] = fmaf(wk, g[t], u[k][t]);
    }
  }
#pragma unroll
  for (int k = 0; k < kGsCh; ++k) {
    double s1 = 0.0, s2 = 0.0;
#pragma unroll
    for (int t = 0; t < JT; ++t) {
      const double wj = (double)ws[wv][k][t * 64 + lane];
      s2 += wj * (double)u[k][t];
      s1 += wj * (double)cs[t * 64 + lane];
    }
    for (int off = 32; off > 0; off >>= 1) {
      s1 += __shfl_xor(s1, off, 64);
      s2 += __shfl_xor(s2, off, 64);
    }
    if (lane == 0) {
      const int c = c0 + k;
      const double kc = shift ? (double)shift[c] : 0.0;
      row[c] = (float)(s1 - M * kc);
      row[Cout + c] = (float)(s2 - 2.0 * kc * s1 + M * kc * kc);
    }
  }
}

// The dual tail's apply operands (ops/tail.py _DualTailFn): per output channel c the branch with the
// larger |BN scale| keeps its bf16 weights, the other's are scaled by the ratio of the scales (fp32
// product, one rounding); ss = [s_big | t3 + td]. One workgroup per 4 channels, one wave each.
__global__ __launch_bounds__(256) void bnfold_dual_weights_kernel(const uint16_t* __restrict__ W3,
                                                                  const uint16_t* __restrict__ Wd,
                                                                  const float* __restrict__ ss3,
                                                                  const float* __restrict__ ssd, int Cout, int C3, int Cd,
                                                                  uint16_t* __restrict__ wcat, float* __restrict__ ss) {
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (c >= Cout) return;
  const float s3 = ss3[c], sd = ssd[c];
  const bool big3 = fabsf(s3) >= fabsf(sd);
  const float sb = big3 ? s3 : sd;
  float r3 = big3 ? 1.f : (sb != 0.f ? s3 / sb : 0.f);
  float rd = big3 ? (sb != 0.f ? sd / sb : 0.f) : 1.f;
  if (sb == 0.f) r3 = rd = 0.f;
  const int K = C3 + Cd;
  for (int k = lane; k < K; k += 64) {
    const float v = k < C3 ? bf16_to_f32(W3[(int64_t)c * C3 + k]) * r3 : bf16_to_f32(Wd[(int64_t)c * Cd + k - C3]) * rd;
    wcat[(int64_t)c * K + k] = f32_to_bf16(v);
  }
  if (lane == 0) {
    ss[c] = sb;
    ss[Cout + c] = ss3[Cout + c] + ssd[Cout + c];
  }
}

hipError_t launch_bnfold_dual_weights(const uint16_t* W3, const uint16_t* Wd, const float* ss3, const float* ssd,
                                      int Cout, int C3, int Cd, uint16_t* wcat, float* ss, hipStream_t st) {
  if (Cout <= 0 || C3 <= 0 || Cd <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(bnfold_dual_weights_kernel, dim3((Cout + 3) / 4), dim3(256), 0, st, W3, Wd, ss3, ssd, Cout, C3, Cd,
                     wcat, ss);
  return hipGetLastError();
}

hipError_t launch_bnfold_gram_stats(const float* P, const uint16_t* W, const float* shift, int Cout, int Wd, int64_t M,
                                    float* row, hipStream_t st) {
  if (Cout <= 0 || Cout % kGsCh != 0 || M <= 0) return hipErrorInvalidValue;
  const dim3 grid((Cout / kGsCh + 3) / 4);
  if (Wd == 64) hipLaunchKernelGGL(bnfold_gram_stats_kernel<1>, grid, dim3(256), 0, st, P, W, shift, Cout, Wd, (double)M, row);
  else if (Wd == 128) hipLaunchKernelGGL(bnfold_gram_stats_kernel<2>, grid, dim3(256), 0, st, P, W, shift, Cout, Wd, (double)M, row);
  else if (Wd == 256) hipLaunchKernelGGL(bnfold_gram_stats_kernel<4>, grid, dim3(256), 0, st, P, W, shift, Cout, Wd, (double)M, row);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_bnfold_rowdot(const float* P, const uint16_t* W, int Cout, int Wd, float* row, hipStream_t st) {
  if (Cout <= 0 || Wd <= 0 || Wd % 8 != 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(bnfold_rowdot_kernel, dim3((Cout + 3) / 4), dim3(256), 0, st, P, W, Cout, Wd, row);
  return hipGetLastError();
}

hipError_t launch_bnfold_prep(const uint16_t* W, const float* coef, int Cout, int Wd, uint16_t* w2, int ldw,
                              uint16_t* bw, float* bvec, hipStream_t st) {
  if (Cout <= 0 || Wd <= 0 || ldw < Cout) return hipErrorInvalidValue;
  hipLaunchKernelGGL(bnfold_prep_kernel, dim3(Wd), dim3(256), 0, st, W, coef, Cout, Wd, w2, ldw, bw, bvec);
  return hipGetLastError();
}

hipError_t launch_bnfold_combine(const float* P, const uint16_t* W, const float* coef, int Cout, int Wd,
                                 uint16_t* out, int accumulate, hipStream_t st) {
  if (Cout <= 0 || Wd <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(bnfold_combine_kernel, dim3((Cout + kCT - 1) / kCT, (Wd + kCT - 1) / kCT), dim3(256), 0, st, P, W,
                     coef, Cout, Wd, out, accumulate);
  return hipGetLastError();
}

}  // namespace psd
