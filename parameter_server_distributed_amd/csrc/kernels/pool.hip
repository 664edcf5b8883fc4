// NHWC bf16 3x3 / stride 2 / pad 1 max-pool (the ResNet stem), forward with a 1-byte argmax per
// element and a gather-form backward (no atomics: each input lane sums the <= 4 outputs whose
// window covers it and whose argmax points at it). Replaces PyTorch's max_pool2d NHWC kernels
// (260 us fwd + 610 us bwd per ResNet-50 b256 step in profiles/resnet50_r1_fusedbn_kernels.md).
#include "common.h"
#include "launchers_pool.h"
#include "pool_gather.h"

namespace psd {

__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                          uint8_t* __restrict__ arg, int N, int H, int W, int C,
                                                          int Ho, int Wo) {
  const int c8n = C >> 3;
  const int64_t total = (int64_t)N * Ho * Wo * c8n;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int c8 = (int)(t % c8n);
    int64_t r = t / c8n;
    const int wo = (int)(r % Wo);
    r /= Wo;
    const int ho = (int)(r % Ho);
    const int n = (int)(r / Ho);
    float best[8];
    uint8_t bi[8];
    maxpool3s2_max8(x, n, ho, wo, c8, H, W, C, [](float v, int) { return v; }, best, bi);
    store8_bf16(y + t * 8, best);
    store_argmax8(arg + t * 8, bi);
  }
}

// dy2 (optional, same shape as dy): a second consumer's gradient of the pool output (the
// downsample branch of the first bottleneck), summed here instead of by an autograd add kernel.
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ dy2,
                                                          const uint8_t* __restrict__ arg,
                                                          uint16_t* __restrict__ dx, int N, int H, int W, int C, int Ho,
                                                          int Wo) {
  const int c8n = C >> 3;
  const int64_t total = (int64_t)N * H * W * c8n;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int c8 = (int)(t % c8n);
    int64_t r = t / c8n;
    const int w = (int)(r % W);
    r /= W;
    const int h = (int)(r % H);
    const int n = (int)(r / H);
    float acc[8];
    maxpool3s2_grad8(dy, dy2, arg, n, h, w, c8, C, Ho, Wo, acc);
    store8_bf16(dx + t * 8, acc);
  }
}

hipError_t launch_maxpool_fwd(const uint16_t* x, uint16_t* y, uint8_t* arg, int N, int H, int W, int C, int Ho, int Wo,
                              hipStream_t st) {
  if (C % 8) return hipErrorInvalidValue;
  const int64_t total = (int64_t)N * Ho * Wo * (C / 8);
  hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(stream_grid(total, 256)), dim3(256), 0, st, x, y, arg, N, H, W, C, Ho, Wo);
  return hipGetLastError();
}

hipError_t launch_maxpool_bwd(const uint16_t* dy, const uint16_t* dy2, const uint8_t* arg, uint16_t* dx, int N, int H, int W, int C, int Ho,
                              int Wo, hipStream_t st) {
  if (C % 8) return hipErrorInvalidValue;
  const int64_t total = (int64_t)N * H * W * (C / 8);
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(stream_grid(total, 256)), dim3(256), 0, st, dy, dy2, arg, dx, N, H, W, C, Ho, Wo);
  return hipGetLastError();
}

// ------------------------------------------------------------------ global average pool
// NHWC [N, HW, C] -> [N, C] (the ResNet head). One lane per (n, 8 channels): HW 16-byte loads
// with stride C, fp32 sum. Backward writes dx[n, hw, :] = dy[n, :] / HW with 16-byte stores
// (PyTorch's channels_last expand kernel took ~400 us per b1024 step for the same 205 MB).
__global__ __launch_bounds__(256) void gap_fwd_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y, int N,
                                                      int HW, int C, float inv) {
  const int c8n = C >> 3;
  const int64_t total = (int64_t)N * c8n;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t n = t / c8n;
    const int c8 = (int)(t % c8n);
    const uint16_t* p = x + n * HW * C + c8 * 8;
    float a[8] = {0, 0, 0, 0, 0, 0, 0, 0}, b[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int i = 0;
    for (; i + 1 < HW; i += 2) {
      float v0[8], v1[8];
      load8_bf16(p + (int64_t)i * C, v0);
      load8_bf16(p + (int64_t)(i + 1) * C, v1);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        a[e] += v0[e];
        b[e] += v1[e];
      }
    }
    if (i < HW) {
      float v0[8];
      load8_bf16(p + (int64_t)i * C, v0);
#pragma unroll
      for (int e = 0; e < 8; ++e) a[e] += v0[e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) a[e] = (a[e] + b[e]) * inv;
    store8_bf16(y + t * 8, a);
  }
}

__global__ __launch_bounds__(256) void gap_bwd_kernel(const uint16_t* __restrict__ dy, uint16_t* __restrict__ dx, int N,
                                                      int HW, int C, float inv) {
  const int c8n = C >> 3;
  const int64_t total = (int64_t)N * HW * c8n;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int c8 = (int)(t % c8n);
    const int64_t n = t / ((int64_t)HW * c8n);
    float g[8];
    load8_bf16(dy + (n * c8n + c8) * 8, g);
#pragma unroll
    for (int e = 0; e < 8; ++e) g[e] *= inv;
    store8_bf16(dx + t * 8, g);
  }
}

hipError_t launch_gap_fwd(const uint16_t* x, uint16_t* y, int N, int HW, int C, hipStream_t st) {
  if (C % 8 || HW <= 0) return hipErrorInvalidValue;
  const int64_t total = (int64_t)N * (C / 8);
  hipLaunchKernelGGL(gap_fwd_kernel, dim3(stream_grid(total, 256)), dim3(256), 0, st, x, y, N, HW, C, 1.f / HW);
  return hipGetLastError();
}

hipError_t launch_gap_bwd(const uint16_t* dy, uint16_t* dx, int N, int HW, int C, hipStream_t st) {
  if (C % 8 || HW <= 0) return hipErrorInvalidValue;
  const int64_t total = (int64_t)N * HW * (C / 8);
  hipLaunchKernelGGL(gap_bwd_kernel, dim3(stream_grid(total, 256)), dim3(256), 0, st, dy, dx, N, HW, C, 1.f / HW);
  return hipGetLastError();
}


// stride-2 subsample of an NHWC bf16 tensor: y[n][ho][wo][:] = x[n][2 ho][2 wo][:] (the quarter-grid
// input of a stride-2 1x1 downsample convolution, ops/tail.py). 16-byte lanes; each output pixel's
// channels are one contiguous run in both tensors.
__global__ __launch_bounds__(256) void subsample2_kernel(const u32x4* __restrict__ x, u32x4* __restrict__ y, int64_t n16,
                                                         int C16, int Ho, int Wo, int H, int W) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
    const int64_t pix = i / C16;
    const int c = (int)(i - pix * C16);
    const int64_t n = pix / ((int64_t)Ho * Wo);
    const int rem = (int)(pix - n * Ho * Wo);
    const int ho = rem / Wo, wo = rem - ho * Wo;
    y[i] = __builtin_nontemporal_load(x + ((n * H + 2 * ho) * (int64_t)W + 2 * wo) * C16 + c);
  }
}

hipError_t launch_subsample2(const uint16_t* x, uint16_t* y, int N, int H, int W, int C, hipStream_t st) {
  if (C % 8 != 0 || H % 2 != 0 || W % 2 != 0) return hipErrorInvalidValue;
  const int Ho = H / 2, Wo = W / 2, C16 = C / 8;
  const int64_t n16 = (int64_t)N * Ho * Wo * C16;
  if (n16 <= 0) return hipSuccess;
  hipLaunchKernelGGL(subsample2_kernel, dim3(stream_grid(n16, 256)), dim3(256), 0, st,
                     reinterpret_cast<const u32x4*>(x), reinterpret_cast<u32x4*>(y), n16, C16, Ho, Wo, H, W);
  return hipGetLastError();
}

}  // namespace psd
