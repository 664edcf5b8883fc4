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

// Stage input rows ih0 .. ih0+rows-1 of image n as zero-padded patch rows of RS elements: element
// e of row r = x[n, ih0 + r, e/3 - 3, e%3] (0 outside the image). Destination chunk c (8 elements)
// = source elements 8c-9 .. 8c-2 = the last element of source chunk c-2 and the first 7 of c-1.
// Split into a register load (issued for the NEXT work item before the current one is computed, so
// the HBM latency hides behind the MFMA work) and the LDS store; a lane owns chunks tid + 256*i.
template <int IT>
__device__ __forceinline__ void patch_load(const uint16_t* __restrict__ x, int n, int ih0, int rows, int RS, int H, int W,
                                           u32x4 (&buf)[2 * IT]) {
  const int row_chunks = RS / 8;
  const int src_chunks = (3 * W) / 8;  // host: 3W % 8 == 0
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int v = threadIdx.x + i * 256;
    const int r = v / row_chunks, c = v - r * row_chunks;
    const int ih = ih0 + r;
    buf[2 * i] = buf[2 * i + 1] = u32x4{0u, 0u, 0u, 0u};
    if (r < rows && ih >= 0 && ih < H) {
      const uint16_t* src = x + ((int64_t)n * H + ih) * W * 3;
      if (c - 2 >= 0 && c - 2 < src_chunks) buf[2 * i] = *reinterpret_cast<const u32x4*>(src + (c - 2) * 8);
      if (c - 1 >= 0 && c - 1 < src_chunks) buf[2 * i + 1] = *reinterpret_cast<const u32x4*>(src + (c - 1) * 8);
    }
  }
}

template <int IT>
__device__ __forceinline__ void patch_store(uint16_t* patch, int rows, int RS, const u32x4 (&buf)[2 * IT]) {
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int v = threadIdx.x + i * 256;
    if (v >= rows * (RS / 8)) break;
    const u32x4 a = buf[2 * i], b = buf[2 * i + 1];
    u32x4 d;  // [a.h7, b.h0 .. b.h6]
    d.x = (a.w >> 16) | (b.x << 16);
    d.y = (b.x >> 16) | (b.y << 16);
    d.z = (b.y >> 16) | (b.z << 16);
    d.w = (b.z >> 16) | (b.w << 16);
    *reinterpret_cast<u32x4*>(patch + v * 8) = d;
  }
}

// register-staging capacity (chunks per lane) of the two kernels; the host checks the shapes fit
constexpr int kFwdPatchIt = 5;  // 13 rows x RS/8 chunks <= 1280  (Wo <= 128)
constexpr int kWgPatchIt = 4;   // 9 rows x RS/8 chunks <= 1024   (Wo <= 128)
constexpr int kWgDyIt = 8;      // 2*Wo pixels x 8 chunks <= 2048  (Wo <= 128)

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

  const int tiles_per_row = Wo / 16;
  const int per_img = Ho / kStemRows;
  const int items = N * per_img;
  u32x4 pbuf[2 * kFwdPatchIt];
  if (blockIdx.x < items)
    patch_load<kFwdPatchIt>(x, blockIdx.x / per_img, 2 * (blockIdx.x % per_img) * kStemRows - 3, kStemInRows, RS, H, W,
                            pbuf);
  for (int it = blockIdx.x; it < items; it += gridDim.x) {
    const int n = it / per_img;
    const int oh0 = (it % per_img) * kStemRows;
    patch_store<kFwdPatchIt>(patch, kStemInRows, RS, pbuf);
    __syncthreads();
    const int nx = it + gridDim.x;  // prefetch the next item's rows into registers
    if (nx < items)
      patch_load<kFwdPatchIt>(x, nx / per_img, 2 * (nx % per_img) * kStemRows - 3, kStemInRows, RS, H, W, pbuf);
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
         (3 * W) % 8 == 0 && kStemInRows * (6 * Wo + 24) / 8 <= 256 * kFwdPatchIt;
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

// ------------------------------------------------------------------ weight gradient
// dW[co][k] = sum_m dY[m][co] A[m][k] as C[k][co] += A^T[k][m] dY[m][co], a reduction over the
// 12.8M output pixels. Work item = (image n, 2 output rows): the 9 input rows go to LDS as in the
// forward, dY of the item's 2*Wo pixels is staged TRANSPOSED ([co][m], so a B fragment -- 8
// consecutive m of one channel -- is one 16-byte LDS read), and the A fragment (8 consecutive m of
// one k = (kh, kw*3+ci)) is gathered from the patch at stride 6 elements. The 11 live k-blocks of
// 16 (k < 176) are split over the 4 waves (3/3/3/2) x 4 channel blocks, so a wave keeps <= 12
// accumulators. Persistent grid: each workgroup writes its fp32 partial C, and stem_wgrad_reduce
// sums them into the bf16 [co][kh][kw][ci] (channels_last) gradient -- deterministic.
constexpr int kWgRows = 2;
constexpr int kWgInRows = 2 * (kWgRows - 1) + 7;
constexpr int kWgKBlocks = 11;  // k < 176 covers kh < 7 (k < 168)
// dT column swizzle: 8-element blocks XOR-ed by bits 3-4 of the channel (stays inside a 32-aligned
// pixel block, so any 32-multiple item width works; 16-byte fragment reads stay contiguous)
__device__ __forceinline__ int dt_swz(int c) { return ((c >> 3) & 3) << 3; }

__global__ __launch_bounds__(256) void stem_wgrad_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ dy,
                                                         float* __restrict__ part, int N, int H, int W, int Ho, int Wo) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  const int RS = 6 * Wo + 24;
  const int MI = kWgRows * Wo;      // pixels per item (host: % 32 == 0)
  const int DLD = MI + 8;           // dT row stride (elements): 16-byte aligned, spreads banks
  uint16_t* patch = smem;           // [9][RS]
  uint16_t* dT = smem + kWgInRows * RS;  // [64][DLD]
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int g = lane >> 4, i16 = lane & 15;
  const int kb0 = wv * 3, nkb = wv < 3 ? 3 : kWgKBlocks - 9;
  f32x4 acc[3][4];
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[a][c] = f32x4{0.f, 0.f, 0.f, 0.f};
  // this lane's A rows: k = (kb0 + a)*16 + i16 -> patch offset (kh*RS + j) (kh < 7 guaranteed for k < 176
  // except 168..175, which read the padding row 7*RS.. of a 9-row patch: rows 7, 8 exist, values unused)
  int koff[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const int k = (kb0 + a) * 16 + i16;
    const int kh = k / 24, j = k - kh * 24;
    koff[a] = kh * RS + j;
  }
  const int per_img = Ho / kWgRows;
  const int items = N * per_img;
  u32x4 pbuf[2 * kWgPatchIt], dbuf[kWgDyIt];
  // dY rows oh0 .. oh0+1 are contiguous: MI pixels x 64 channels; lane chunk v = (pixel v/8, channels 8*(v%8))
  auto dy_load = [&](int item) {
    const uint16_t* src = dy + ((int64_t)(item / per_img) * Ho + (item % per_img) * kWgRows) * Wo * 64;
#pragma unroll
    for (int i = 0; i < kWgDyIt; ++i) {
      const int v = threadIdx.x + i * 256;
      dbuf[i] = v < MI * 8 ? *reinterpret_cast<const u32x4*>(src + (int64_t)v * 8) : u32x4{0u, 0u, 0u, 0u};
    }
  };
  for (int it = blockIdx.x; it < items; it += gridDim.x) {
    // all loads of the item issued before any LDS store (one exposed HBM latency per item; a
    // register prefetch of the next item measured slower: it halves occupancy)
    patch_load<kWgPatchIt>(x, it / per_img, 2 * (it % per_img) * kWgRows - 3, kWgInRows, RS, H, W, pbuf);
    dy_load(it);
    patch_store<kWgPatchIt>(patch, kWgInRows, RS, pbuf);
#pragma unroll
    for (int i = 0; i < kWgDyIt; ++i) {  // transpose into dT[c][p ^ swz(c)]
      const int v = threadIdx.x + i * 256;
      if (v >= MI * 8) break;
      const int p = v >> 3, c0 = (v & 7) * 8;
      const int ps = p ^ dt_swz(c0);  // the 8 lanes of one pixel write 8 rows c0+.. : spread their banks
      const uint32_t ws[4] = {dbuf[i].x, dbuf[i].y, dbuf[i].z, dbuf[i].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        dT[(c0 + 2 * e) * DLD + ps] = (uint16_t)(ws[e] & 0xffffu);
        dT[(c0 + 2 * e + 1) * DLD + ps] = (uint16_t)(ws[e] >> 16);
      }
    }
    __syncthreads();
    for (int m0 = 0; m0 < MI; m0 += 32) {
      // B fragments: dY[m = m0 + 8g + t][co = cb*16 + i16]
      bf16x8 bfr[4];
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
        bfr[cb] = __builtin_bit_cast(
            bf16x8, *reinterpret_cast<const u32x4*>(dT + (cb * 16 + i16) * DLD + ((m0 + 8 * g) ^ dt_swz(cb * 16 + i16))));
      // A fragments: A[m][k] for 8 consecutive m (pixel p -> output row p / Wo, column p % Wo)
      // (an item is kWgRows = 2 output rows: the row of pixel p is a compare, not a division -- the
      // integer division by the runtime Wo made this loop VALU-bound, ~1,400 VALU per item per wave)
      static_assert(kWgRows == 2, "pixel -> output row below assumes two rows per item");
      int pofs[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const int p = m0 + 8 * g + t;
        const int ohl = p >= Wo ? 1 : 0, ow = p - ohl * Wo;
        pofs[t] = 2 * ohl * RS + 6 * ow;
      }
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        if (a >= nkb) break;
        uint32_t pk[4];
#pragma unroll
        for (int t = 0; t < 4; ++t)
          pk[t] = (uint32_t)patch[pofs[2 * t] + koff[a]] | ((uint32_t)patch[pofs[2 * t + 1] + koff[a]] << 16);
        const bf16x8 af = __builtin_bit_cast(bf16x8, u32x4{pk[0], pk[1], pk[2], pk[3]});
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) acc[a][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[cb], acc[a][cb], 0, 0, 0);
      }
    }
    __syncthreads();
  }
  // C[k = (kb0+a)*16 + 4g + i][co = cb*16 + i16] -> part[blk][k][co]
  float* dst = part + (int64_t)blockIdx.x * 192 * 64;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    if (a >= nkb) break;
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int i = 0; i < 4; ++i) dst[((kb0 + a) * 16 + 4 * g + i) * 64 + cb * 16 + i16] = acc[a][cb][i];
  }
}

// dW[co][kh][kw][ci] (bf16, channels_last [64,3,7,7]) = sum over blocks of part[blk][kh*24 + kw*3 + ci][co].
// One workgroup per r = kh*21 + kw*3 + ci: 4 lane groups split the blocks, 64 lanes the channels.
__global__ __launch_bounds__(256) void stem_wgrad_reduce_kernel(const float* __restrict__ part, int nblk,
                                                                uint16_t* __restrict__ dw) {
  const int r = blockIdx.x;
  const int kh = r / 21, j = r - kh * 21;
  const int k = kh * 24 + j;
  const int co = threadIdx.x & 63, q = threadIdx.x >> 6;
  float s0 = 0.f, s1 = 0.f;
  int b = q;
  for (; b + 4 < nblk; b += 8) {
    s0 += part[((int64_t)b * 192 + k) * 64 + co];
    s1 += part[((int64_t)(b + 4) * 192 + k) * 64 + co];
  }
  for (; b < nblk; b += 4) s0 += part[((int64_t)b * 192 + k) * 64 + co];
  __shared__ float red[4][64];
  red[q][co] = s0 + s1;
  __syncthreads();
  if (q == 0) dw[co * 147 + r] = f32_to_bf16((red[0][co] + red[1][co]) + (red[2][co] + red[3][co]));
}

bool stem_wgrad_supported(int H, int W, int Ho, int Wo) {
  return stem_conv_supported(H, W, Ho, Wo) && Ho % kWgRows == 0 && (kWgRows * Wo) % 32 == 0 &&
         kWgInRows * (6 * Wo + 24) / 8 <= 256 * kWgPatchIt && kWgRows * Wo * 8 <= 256 * kWgDyIt;
}

// (a grid capped at the resident workgroups -- 3 per CU by LDS -- measured slower: 1,013 vs 914 us,
// profiles/r5/resnet50_b1024_r5e_kernels.md vs r5d)
int stem_wgrad_blocks(int N, int Ho, int Wo) {
  (void)Wo;
  const int items = N * (Ho / kWgRows);
  return items < 1024 ? (items < 1 ? 1 : items) : 1024;
}

hipError_t launch_stem_wgrad(const uint16_t* x, const uint16_t* dy, float* part, uint16_t* dw, int N, int H, int W,
                             int Ho, int Wo, hipStream_t st) {
  if (!stem_wgrad_supported(H, W, Ho, Wo)) return hipErrorInvalidValue;
  const int RS = 6 * Wo + 24;
  const size_t lds = (size_t)(kWgInRows * RS + 64 * (kWgRows * Wo + 8)) * 2;
  if (lds > 64 * 1024) return hipErrorInvalidValue;
  const int nblk = stem_wgrad_blocks(N, Ho, Wo);
  hipLaunchKernelGGL(stem_wgrad_kernel, dim3(nblk), dim3(256), lds, st, x, dy, part, N, H, W, Ho, Wo);
  hipLaunchKernelGGL(stem_wgrad_reduce_kernel, dim3(147), dim3(256), 0, st, part, nblk, dw);
  return hipGetLastError();
}

}  // namespace psd
