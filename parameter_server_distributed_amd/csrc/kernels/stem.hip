// ResNet stem convolution (7x7, stride 2, pad 3, 3 -> 64 channels, NHWC bf16) as an implicit GEMM
// on the gfx950 matrix cores, with the following BatchNorm's batch statistics reduced in the
// epilogue.
//
// Why: MIOpen's best stem kernel on the b1024 step (igemm_fwd_gtcx35 ... bt256x64x8) takes 1.4 ms
// (~170 TFLOP/s; Cin = 3 defeats its K tiling), and the BN statistics then re-read the 1.64 GB
// output (~0.33 ms). The GEMM is tiny (12.8M x 64 x 147): the pass is bound by the 1.64 GB output
// write (~0.3 ms at the measured 5.3 TB/s copy roof).
//
// GEMM view: C[m = (n, oh, ow)][co] = sum_k A[m][k] W[co][k], k = kh*24 + j, j = kw*3 + ci (< 21;
// j in 21..23 and kh = 7 carry zero weights), K = 192 = 6 k-blocks of v_mfma_f32_16x16x32_bf16.
// Because the stride is 2 and Cin = 3, the 21 (kw, ci) values of one kh are 21 CONTIGUOUS elements
// of the zero-padded input row, starting at element 6*ow: an A fragment (8 consecutive k of one
// row) is 8 contiguous bf16 in LDS -- no im2col anywhere.
//
// Work item = (image n, 4 output rows): its 13 input rows are staged in LDS (padded columns,
// zero rows outside the image), then each of the 4 waves computes 16-pixel x 64-channel tiles
// (Wo/16 per output row) with all 24 weight fragments held in VGPRs. The epilogue rounds to bf16
// (the BN statistics are taken on exactly the stored values, as the stand-alone reduce would),
// accumulates shifted sum / sum-of-squares per channel in registers, and writes the tile through a
// per-wave LDS stage as coalesced 16-byte rows. The grid is persistent (<= 1024 workgroups): each
// workgroup writes one partial-statistics row at the end, which the BN finalize kernel combines
// (deterministic, no atomics).
#include "common.h"
#include "launchers_stem.h"

namespace psd {

namespace {
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
constexpr int kStemRows = 4;      // output rows per work item
constexpr int kStemInRows = 13;   // 2 * (kStemRows - 1) + 7
constexpr int kStageLd = 72;      // bf16 per staged output pixel (64 + 8 pad: spreads LDS banks)
}  // namespace

__global__ __launch_bounds__(256) void stem_conv_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ wk,
                                                        uint16_t* __restrict__ y, const float* __restrict__ shift,
                                                        float* __restrict__ part, int N, int H, int W, int Ho, int Wo) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  const int RS = 6 * Wo + 24;  // patch row stride (elements): covers 6*(Wo-1) + 24
  uint16_t* patch = smem;      // [13][RS]
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  uint16_t* stage = smem + kStemInRows * RS + wv * 16 * kStageLd;  // per-wave [16 px][72]
  const int g = lane >> 4, m = lane & 15;

  // all 24 B fragments: B[k][co], k = kb*32 + 8g + 0..7, co = nb*16 + m  ->  wk[co][k..k+8]
  bf16x8 bfr[6][4];
#pragma unroll
  for (int kb = 0; kb < 6; ++kb)
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
      bfr[kb][nb] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(wk + (nb * 16 + m) * 192 + kb * 32 + 8 * g));
  float kshift[4], s1[4], s2[4];
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) {
    kshift[nb] = shift ? shift[nb * 16 + m] : 0.f;
    s1[nb] = s2[nb] = 0.f;
  }

  const int row_chunks = RS / 8;
  const int src_chunks = (3 * W) / 8;  // host: 3W % 8 == 0
  const int tiles_per_row = Wo / 16;
  const int items = N * (Ho / kStemRows);
  for (int it = blockIdx.x; it < items; it += gridDim.x) {
    const int n = it / (Ho / kStemRows);
    const int oh0 = (it % (Ho / kStemRows)) * kStemRows;
    const int ih0 = 2 * oh0 - 3;
    // stage the 13 input rows: patch element e of row r = x[n, ih0 + r, e/3 - 3, e%3] (0 outside).
    // Destination chunk c (8 elements) = source elements 8c-9 .. 8c-2 = last element of source
    // chunk c-2 followed by the first 7 of chunk c-1.
    for (int v = threadIdx.x; v < kStemInRows * row_chunks; v += blockDim.x) {
      const int r = v / row_chunks, c = v - r * row_chunks;
      const int ih = ih0 + r;
      u32x4 a = u32x4{0u, 0u, 0u, 0u}, b = u32x4{0u, 0u, 0u, 0u};
      if (ih >= 0 && ih < H) {
        const uint16_t* src = x + ((int64_t)n * H + ih) * W * 3;
        if (c - 2 >= 0 && c - 2 < src_chunks) a = *reinterpret_cast<const u32x4*>(src + (c - 2) * 8);
        if (c - 1 >= 0 && c - 1 < src_chunks) b = *reinterpret_cast<const u32x4*>(src + (c - 1) * 8);
      }
      // [a.h7, b.h0 .. b.h6] as four dwords
      u32x4 d;
      d.x = (a.w >> 16) | (b.x << 16);
      d.y = (b.x >> 16) | (b.y << 16);
      d.z = (b.y >> 16) | (b.z << 16);
      d.w = (b.z >> 16) | (b.w << 16);
      *reinterpret_cast<u32x4*>(patch + r * RS + c * 8) = d;
    }
    __syncthreads();
    for (int t = wv; t < kStemRows * tiles_per_row; t += 4) {
      const int ohl = t / tiles_per_row;
      const int ow0 = (t - ohl * tiles_per_row) * 16;
      f32x4 acc[4];
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) acc[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kb = 0; kb < 6; ++kb) {
        const int gi = kb * 4 + g;
        const int kh = gi / 3, j0 = (gi - kh * 3) * 8;
        u32x4 av = u32x4{0u, 0u, 0u, 0u};
        if (kh < 7) {  // 4-byte aligned: RS, 6*ow and j0 are even
          const uint32_t* p = reinterpret_cast<const uint32_t*>(patch + (2 * ohl + kh) * RS + 6 * (ow0 + m) + j0);
          av = u32x4{p[0], p[1], p[2], p[3]};
        }
        const bf16x8 a = __builtin_bit_cast(bf16x8, av);
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bfr[kb][nb], acc[nb], 0, 0, 0);
      }
      // epilogue: C[px = 4g + i][co = nb*16 + m]
#pragma unroll
      for (int nb = 0; nb < 4; ++nb)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint16_t h = f32_to_bf16(acc[nb][i]);
          const float d = bf16_to_f32(h) - kshift[nb];
          s1[nb] += d;
          s2[nb] = fmaf(d, d, s2[nb]);
          stage[(4 * g + i) * kStageLd + nb * 16 + m] = h;
        }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
      const int oh = oh0 + ohl;
#pragma unroll
      for (int hlf = 0; hlf < 2; ++hlf) {
        const int ch = lane + 64 * hlf;  // 128 chunks of 16 B: 16 px x 8
        const int px = ch >> 3, cp = ch & 7;
        const u32x4 v = *reinterpret_cast<const u32x4*>(stage + px * kStageLd + cp * 8);
        *reinterpret_cast<u32x4*>(y + (((int64_t)n * Ho + oh) * Wo + ow0 + px) * 64 + cp * 8) = v;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();  // the patch is rewritten by the next item
  }

  // partial statistics of this workgroup: lanes m (x 4 groups g) x 4 waves -> part[blockIdx][2][64]
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) {
    s1[nb] += __shfl_xor(s1[nb], 16);
    s1[nb] += __shfl_xor(s1[nb], 32);
    s2[nb] += __shfl_xor(s2[nb], 16);
    s2[nb] += __shfl_xor(s2[nb], 32);
  }
  float* red = reinterpret_cast<float*>(smem);  // [4 waves][2][64]
  if (g == 0) {
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      red[(wv * 2 + 0) * 64 + nb * 16 + m] = s1[nb];
      red[(wv * 2 + 1) * 64 + nb * 16 + m] = s2[nb];
    }
  }
  __syncthreads();
  if (threadIdx.x < 128) {
    const int which = threadIdx.x >> 6, c = threadIdx.x & 63;
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) s += red[(w * 2 + which) * 64 + c];
    part[(int64_t)blockIdx.x * 128 + which * 64 + c] = s;
  }
}

bool stem_conv_supported(int H, int W, int Ho, int Wo) {
  return Ho == H / 2 && Wo == W / 2 && H % 2 == 0 && W % 2 == 0 && Wo % 16 == 0 && Ho % kStemRows == 0 &&
         (3 * W) % 8 == 0;
}

int stem_conv_blocks(int N, int Ho) {
  const int items = N * (Ho / kStemRows);
  return items < 1024 ? (items < 1 ? 1 : items) : 1024;
}

hipError_t launch_stem_conv(const uint16_t* x, const uint16_t* wk, uint16_t* y, const float* shift, float* part, int N,
                            int H, int W, int Ho, int Wo, hipStream_t st) {
  if (!stem_conv_supported(H, W, Ho, Wo)) return hipErrorInvalidValue;
  const int RS = 6 * Wo + 24;
  const size_t lds = (size_t)(kStemInRows * RS + 4 * 16 * kStageLd) * 2;
  if (lds > 64 * 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL(stem_conv_kernel, dim3(stem_conv_blocks(N, Ho)), dim3(256), lds, st, x, wk, y, shift, part, N, H, W,
                     Ho, Wo);
  return hipGetLastError();
}

}  // namespace psd
