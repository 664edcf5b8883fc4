// FP8 (OCP e4m3fn -- gfx950 is OCP, NOT the MI300 fnuz encoding) quantisation helpers for the
// fp8-weights path (Wide-ResNet-101 / fp8 GEMMs): per-tensor amax on device, scale = 448/amax,
// saturating cast, and dequantisation. All stream-shaped: 8 elements per lane, grid-stride.
#include <hip/hip_fp8.h>
#include "common.h"
#include "launchers.h"
#include "mx_common.h"

namespace psd {

template <int DT>
__global__ __launch_bounds__(256) void amax_kernel(const void* __restrict__ x, int64_t n, float* amax) {
  float m = 0.f;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t nvec = n >> 3;  // 16-byte loads (bf16) / two 16-byte loads (fp32) per lane
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    float t[8];
    if (DT == DT_BF16) load8_bf16(static_cast<const uint16_t*>(x) + (v << 3), t);
    else load8_f32(static_cast<const float*>(x) + (v << 3), t);
#pragma unroll
    for (int e = 0; e < 8; ++e) m = fmaxf(m, fabsf(t[e]));
  }
  if (blockIdx.x == 0)
    for (int64_t i = (nvec << 3) + threadIdx.x; i < n; i += blockDim.x) {
      const float v = (DT == DT_BF16) ? bf16_to_f32(static_cast<const uint16_t*>(x)[i]) : static_cast<const float*>(x)[i];
      m = fmaxf(m, fabsf(v));
    }
  // wave64 butterfly, then one LDS slot per wave
  for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, kWave));
  __shared__ float red[4];
  const int wid = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  if (lane == 0) red[wid] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    float r = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    // non-negative floats order like their bit patterns: integer atomicMax is exact
    atomicMax(reinterpret_cast<unsigned int*>(amax), __float_as_uint(r));
  }
}

// ---- just-in-time per-tensor quantisation in two launches, no atomics and no zero-fill:
// amax_partial writes one max per block (16-byte loads, 4 in flight per lane); the quant kernel's
// blocks each reduce those <= kAmaxBlocks partials (4 KiB, L2-resident) before quantising. The first
// version (one 2-byte load per lane per iteration, a per-call atomic into a zeroed scalar) took
// 47 us per call and 11 % of the Wide-ResNet-101-2 fp8 step (profiles/wrn101_2_fp8_b512_r2_kernels.md).
constexpr int kAmaxBlocks = 1024;

__device__ __forceinline__ float block_max(float m) {
  for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, kWave));
  __shared__ float red[4];
  const int wid = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  if (lane == 0) red[wid] = m;
  __syncthreads();
  return fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

template <bool E5>
__device__ __forceinline__ uint8_t f32_to_f8_(float x) {
  return (uint8_t)__hip_cvt_float_to_fp8(x, __HIP_SATFINITE, E5 ? __HIP_E5M2 : __HIP_E4M3);
}

template <int DT>
__global__ __launch_bounds__(256) void amax_partial_kernel(const void* __restrict__ x, int64_t n, float* __restrict__ part) {
  float m = 0.f;
  const int64_t nvec = n >> 3;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  auto ld = [&](int64_t vi, float (&t)[8]) {
    if (DT == DT_BF16) load8_bf16(static_cast<const uint16_t*>(x) + (vi << 3), t);
    else load8_f32(static_cast<const float*>(x) + (vi << 3), t);
  };
  for (; v + 3 * stride < nvec; v += 4 * stride) {
    float t[4][8];
#pragma unroll
    for (int u = 0; u < 4; ++u) ld(v + u * stride, t[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int e = 0; e < 8; ++e) m = fmaxf(m, fabsf(t[u][e]));
  }
  for (; v < nvec; v += stride) {
    float t[8];
    ld(v, t);
#pragma unroll
    for (int e = 0; e < 8; ++e) m = fmaxf(m, fabsf(t[e]));
  }
  if (blockIdx.x == 0)
    for (int64_t i = (nvec << 3) + threadIdx.x; i < n; i += blockDim.x) {
      const float f = (DT == DT_BF16) ? bf16_to_f32(static_cast<const uint16_t*>(x)[i]) : static_cast<const float*>(x)[i];
      m = fmaxf(m, fabsf(f));
    }
  m = block_max(m);
  if (threadIdx.x == 0) part[blockIdx.x] = m;
}

template <int DT, bool E5>
__global__ __launch_bounds__(256) void quant_part_kernel(const void* __restrict__ x, int64_t n,
                                                         const float* __restrict__ part, int nparts, float fp8_max,
                                                         uint8_t* __restrict__ out, float* scale_inv) {
  float pm = 0.f;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) pm = fmaxf(pm, part[i]);
  const float a = fmaxf(block_max(pm), 1e-12f);
  const float scale = fp8_max / a;
  if (blockIdx.x == 0 && threadIdx.x == 0 && scale_inv) *scale_inv = a / fp8_max;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t nvec = n >> 3;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    const int64_t i = v << 3;
    float t[8];
    if (DT == DT_BF16) load8_bf16(static_cast<const uint16_t*>(x) + i, t);
    else load8_f32(static_cast<const float*>(x) + i, t);
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) lo |= (uint32_t)f32_to_f8_<E5>(t[e] * scale) << (8 * e);
#pragma unroll
    for (int e = 0; e < 4; ++e) hi |= (uint32_t)f32_to_f8_<E5>(t[4 + e] * scale) << (8 * e);
    *reinterpret_cast<uint2*>(out + i) = make_uint2(lo, hi);
  }
  if (blockIdx.x == 0)
    for (int64_t i = (nvec << 3) + threadIdx.x; i < n; i += blockDim.x) {
      const float f = (DT == DT_BF16) ? bf16_to_f32(static_cast<const uint16_t*>(x)[i]) : static_cast<const float*>(x)[i];
      out[i] = f32_to_f8_<E5>(f * scale);
    }
}

template <int DT>
static void launch_jit_t(const void* x, int64_t n, float* part, int nb, int gq, float fp8_max, uint8_t* out,
                         float* scale_inv, hipStream_t st, int e5m2) {
  hipLaunchKernelGGL(amax_partial_kernel<DT>, dim3((unsigned)nb), dim3(256), 0, st, x, n, part);
  if (e5m2)
    hipLaunchKernelGGL((quant_part_kernel<DT, true>), dim3(gq), dim3(256), 0, st, x, n, part, nb, fp8_max, out, scale_inv);
  else
    hipLaunchKernelGGL((quant_part_kernel<DT, false>), dim3(gq), dim3(256), 0, st, x, n, part, nb, fp8_max, out, scale_inv);
}

hipError_t launch_quant_fp8_jit(const void* x, int32_t dt, int64_t n, float* part, float fp8_max, uint8_t* out,
                                float* scale_inv, hipStream_t st, int e5m2) {
  if (n <= 0) return hipSuccess;
  if (dt != DT_BF16 && dt != DT_F32) return hipErrorInvalidValue;
  int64_t nb = ((n >> 3) + 256 * 8 - 1) / (256 * 8);  // >= 8 vectors per lane
  if (nb < 1) nb = 1;
  if (nb > kAmaxBlocks) nb = kAmaxBlocks;
  const int gq = stream_grid((n >> 3) > 0 ? (n >> 3) : 1, 256);
  if (dt == DT_BF16) launch_jit_t<DT_BF16>(x, n, part, (int)nb, gq, fp8_max, out, scale_inv, st, e5m2);
  else launch_jit_t<DT_F32>(x, n, part, (int)nb, gq, fp8_max, out, scale_inv, st, e5m2);
  return hipGetLastError();
}

// ---- delayed scaling (one read of x): quantise with the scale of the amax recorded by the previous
// call of the same tensor role (hist[0] * margin) and record this call's amax into hist[1] (integer
// atomicMax: non-negative floats order like their bit patterns); the roll kernel then moves
// hist[1] -> hist[0] and clears hist[1] for the next call. Values above the previous amax saturate.
template <int DT, bool E5>
__global__ __launch_bounds__(256) void quant_delayed_kernel(const void* __restrict__ x, int64_t n, float* hist,
                                                            float fp8_max, float margin, uint8_t* __restrict__ out,
                                                            float* __restrict__ scale_inv) {
  const float a = fmaxf(hist[0] * margin, 1e-12f);
  const float scale = fp8_max / a;
  if (blockIdx.x == 0 && threadIdx.x == 0) *scale_inv = a / fp8_max;
  float m = 0.f;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t nvec = n >> 3;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    const int64_t i = v << 3;
    float t[8];
    if (DT == DT_BF16) load8_bf16(static_cast<const uint16_t*>(x) + i, t);
    else load8_f32(static_cast<const float*>(x) + i, t);
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) m = fmaxf(m, fabsf(t[e]));
#pragma unroll
    for (int e = 0; e < 4; ++e) lo |= (uint32_t)f32_to_f8_<E5>(t[e] * scale) << (8 * e);
#pragma unroll
    for (int e = 0; e < 4; ++e) hi |= (uint32_t)f32_to_f8_<E5>(t[4 + e] * scale) << (8 * e);
    *reinterpret_cast<uint2*>(out + i) = make_uint2(lo, hi);
  }
  if (blockIdx.x == 0)
    for (int64_t i = (nvec << 3) + threadIdx.x; i < n; i += blockDim.x) {
      const float f = (DT == DT_BF16) ? bf16_to_f32(static_cast<const uint16_t*>(x)[i]) : static_cast<const float*>(x)[i];
      m = fmaxf(m, fabsf(f));
      out[i] = f32_to_f8_<E5>(f * scale);
    }
  m = block_max(m);
  if (threadIdx.x == 0) atomicMax(reinterpret_cast<unsigned int*>(hist + 1), __float_as_uint(m));
}

// Guard of the delayed path: when the recorded amax it scaled with was 0 or not finite (a tensor
// role that was all zeros on the previous step -- e.g. the dY of a zero-initialised bn3 -- or
// whose previous amax overflowed), every element would have saturated; re-quantise with this
// pass's own amax (hist[1], complete: same stream) instead. A valid history returns at once.
template <int DT, bool E5>
__global__ __launch_bounds__(256) void requant_unscaled_kernel(const void* __restrict__ x, int64_t n,
                                                               const float* hist, float fp8_max,
                                                               uint8_t* __restrict__ out, float* __restrict__ scale_inv) {
  const float h0 = hist[0];
  if (h0 > 0.f && h0 <= 3.0e38f) return;  // NaN fails the first test
  const float a = fmaxf(hist[1], 1e-12f);
  const float scale = fp8_max / a;
  if (blockIdx.x == 0 && threadIdx.x == 0) *scale_inv = a / fp8_max;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float f = (DT == DT_BF16) ? bf16_to_f32(static_cast<const uint16_t*>(x)[i]) : static_cast<const float*>(x)[i];
    out[i] = f32_to_f8_<E5>(f * scale);
  }
}

__global__ void amax_roll_kernel(float* hist) {
  hist[0] = hist[1];
  hist[1] = 0.f;
}

hipError_t launch_quant_fp8_delayed(const void* x, int32_t dt, int64_t n, float* hist, float fp8_max, float margin,
                                    uint8_t* out, float* scale_inv, hipStream_t st, int e5m2) {
  if (n <= 0) return hipSuccess;
  const int gq = stream_grid((n >> 3) > 0 ? (n >> 3) : 1, 256);
  if (dt == DT_BF16 && e5m2)
    hipLaunchKernelGGL((quant_delayed_kernel<DT_BF16, true>), dim3(gq), dim3(256), 0, st, x, n, hist, fp8_max, margin, out, scale_inv);
  else if (dt == DT_BF16)
    hipLaunchKernelGGL((quant_delayed_kernel<DT_BF16, false>), dim3(gq), dim3(256), 0, st, x, n, hist, fp8_max, margin, out, scale_inv);
  else if (dt == DT_F32 && e5m2)
    hipLaunchKernelGGL((quant_delayed_kernel<DT_F32, true>), dim3(gq), dim3(256), 0, st, x, n, hist, fp8_max, margin, out, scale_inv);
  else if (dt == DT_F32)
    hipLaunchKernelGGL((quant_delayed_kernel<DT_F32, false>), dim3(gq), dim3(256), 0, st, x, n, hist, fp8_max, margin, out, scale_inv);
  else return hipErrorInvalidValue;
  const int gr = stream_grid(n, 256) < 256 ? stream_grid(n, 256) : 256;
  if (dt == DT_BF16 && e5m2)
    hipLaunchKernelGGL((requant_unscaled_kernel<DT_BF16, true>), dim3(gr), dim3(256), 0, st, x, n, hist, fp8_max, out, scale_inv);
  else if (dt == DT_BF16)
    hipLaunchKernelGGL((requant_unscaled_kernel<DT_BF16, false>), dim3(gr), dim3(256), 0, st, x, n, hist, fp8_max, out, scale_inv);
  else if (e5m2)
    hipLaunchKernelGGL((requant_unscaled_kernel<DT_F32, true>), dim3(gr), dim3(256), 0, st, x, n, hist, fp8_max, out, scale_inv);
  else
    hipLaunchKernelGGL((requant_unscaled_kernel<DT_F32, false>), dim3(gr), dim3(256), 0, st, x, n, hist, fp8_max, out, scale_inv);
  hipLaunchKernelGGL(amax_roll_kernel, dim3(1), dim3(1), 0, st, hist);
  return hipGetLastError();
}

// E5: OCP e5m2 output (gradients), else e4m3
template <int DT, bool E5>
__global__ __launch_bounds__(256) void quant_kernel(const void* __restrict__ x, int64_t n, const float* amax,
                                                    float fp8_max, uint8_t* __restrict__ out, float* scale_inv) {
  const float a = fmaxf(*amax, 1e-12f);
  const float scale = fp8_max / a;
  if (blockIdx.x == 0 && threadIdx.x == 0 && scale_inv) *scale_inv = a / fp8_max;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t nvec = n >> 3;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    const int64_t i = v << 3;
    float t[8];
    if (DT == DT_BF16) load8_bf16(static_cast<const uint16_t*>(x) + i, t);
    else load8_f32(static_cast<const float*>(x) + i, t);
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) lo |= (uint32_t)f32_to_f8<E5>(t[e] * scale) << (8 * e);
#pragma unroll
    for (int e = 0; e < 4; ++e) hi |= (uint32_t)f32_to_f8<E5>(t[4 + e] * scale) << (8 * e);
    *reinterpret_cast<uint2*>(out + i) = make_uint2(lo, hi);
  }
  if (blockIdx.x == 0)
    for (int64_t i = (nvec << 3) + threadIdx.x; i < n; i += blockDim.x) {
      float v = (DT == DT_BF16) ? bf16_to_f32(static_cast<const uint16_t*>(x)[i]) : static_cast<const float*>(x)[i];
      out[i] = f32_to_f8<E5>(v * scale);
    }
}

template <int OD>
__global__ __launch_bounds__(256) void dequant_kernel(const uint8_t* __restrict__ x, int64_t n,
                                                      const float* scale_inv, void* __restrict__ out) {
  const float s = *scale_inv;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float v = e4m3_to_f32(x[i]) * s;
    if (OD == DT_BF16) static_cast<uint16_t*>(out)[i] = f32_to_bf16(v);
    else static_cast<float*>(out)[i] = v;
  }
}

hipError_t launch_amax(const void* x, int32_t dt, int64_t n, float* amax, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int grid = stream_grid((n >> 3) > 0 ? (n >> 3) : 1, 256);
  if (dt == DT_BF16) hipLaunchKernelGGL(amax_kernel<DT_BF16>, dim3(grid), dim3(256), 0, st, x, n, amax);
  else if (dt == DT_F32) hipLaunchKernelGGL(amax_kernel<DT_F32>, dim3(grid), dim3(256), 0, st, x, n, amax);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_quant_fp8(const void* x, int32_t dt, int64_t n, const float* amax, float fp8_max, uint8_t* out,
                            float* scale_inv, hipStream_t st, int e5m2) {
  if (n <= 0) return hipSuccess;
  const int grid = stream_grid((n >> 3) > 0 ? (n >> 3) : 1, 256);
  if (dt == DT_BF16 && e5m2)
    hipLaunchKernelGGL((quant_kernel<DT_BF16, true>), dim3(grid), dim3(256), 0, st, x, n, amax, fp8_max, out, scale_inv);
  else if (dt == DT_BF16)
    hipLaunchKernelGGL((quant_kernel<DT_BF16, false>), dim3(grid), dim3(256), 0, st, x, n, amax, fp8_max, out, scale_inv);
  else if (dt == DT_F32 && e5m2)
    hipLaunchKernelGGL((quant_kernel<DT_F32, true>), dim3(grid), dim3(256), 0, st, x, n, amax, fp8_max, out, scale_inv);
  else if (dt == DT_F32)
    hipLaunchKernelGGL((quant_kernel<DT_F32, false>), dim3(grid), dim3(256), 0, st, x, n, amax, fp8_max, out, scale_inv);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_dequant_fp8(const uint8_t* x, int64_t n, const float* scale_inv, void* out, int32_t od,
                              hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int grid = stream_grid(n, 256);
  if (od == DT_BF16) hipLaunchKernelGGL(dequant_kernel<DT_BF16>, dim3(grid), dim3(256), 0, st, x, n, scale_inv, out);
  else if (od == DT_F32) hipLaunchKernelGGL(dequant_kernel<DT_F32>, dim3(grid), dim3(256), 0, st, x, n, scale_inv, out);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

// ---- MX (OCP microscaling) fp8: one E8M0 scale per 32 consecutive elements ---------------------
// The format the block-scaled MFMA (v_mfma_scale_f32_16x16x128_f8f6f4) consumes: a lane's 32 K-values
// and the E8M0 byte 2^(s - 127) they share. Purely local -- no amax pass, no history, no device
// scalar -- so a PS owner quantises its slice of the flat weight buffer on its own (K-major weight
// rows of a multiple of 32 elements keep every block inside one GEMM row: tools/probes/mx_probe.hip
// pins the lane map), and an activation is quantised in the pass that produces it.
// Scale choice: the smallest power of two with amax * 2^-e <= fp8 max (no saturation in the block).

template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}

// 8 elements per lane, 4 lanes per 32-element block (n % 32 == 0; the grid stride is a multiple
// of 4 lanes, so a block's lanes are active together)
template <int DT, bool E5>
__global__ __launch_bounds__(256) void quant_mx_kernel(const void* __restrict__ x, int64_t n, uint8_t* __restrict__ q,
                                                       uint8_t* __restrict__ sc) {
  const int64_t nvec = n >> 3;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    float t[8];
    if (DT == DT_BF16) load8_bf16(static_cast<const uint16_t*>(x) + (v << 3), t);
    else load8_f32(static_cast<const float*>(x) + (v << 3), t);
    uint2 qb;
    const int eb = mx_quant8<E5>(t, qb);
    *reinterpret_cast<uint2*>(q + (v << 3)) = qb;
    if ((v & 3) == 0) sc[v >> 2] = (uint8_t)eb;
  }
}

template <int OD>
__global__ __launch_bounds__(256) void dequant_mx_kernel(const uint8_t* __restrict__ q, const uint8_t* __restrict__ sc,
                                                         int64_t n, void* __restrict__ out) {
  const int64_t nvec = n >> 3;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    const uint2 b = *reinterpret_cast<const uint2*>(q + (v << 3));
    const float s = __uint_as_float((uint32_t)sc[v >> 2] << 23);  // 2^(eb - 127) (eb 0: 0, exact enough)
    float t[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      t[e] = e4m3_to_f32((uint8_t)(b.x >> (8 * e))) * s;
      t[e + 4] = e4m3_to_f32((uint8_t)(b.y >> (8 * e))) * s;
    }
    if (OD == DT_BF16) store8_bf16(static_cast<uint16_t*>(out) + (v << 3), t);
    else store8_f32(static_cast<float*>(out) + (v << 3), t);
  }
}

hipError_t launch_quant_mx(const void* x, int32_t dt, int64_t n, int e5m2, uint8_t* q, uint8_t* scales, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (n % 32 != 0) return hipErrorInvalidValue;
  const int grid = stream_grid(n >> 3, 256);
#define PSD_QMX(D, E) hipLaunchKernelGGL((quant_mx_kernel<D, E>), dim3(grid), dim3(256), 0, st, x, n, q, scales)
  if (dt == DT_BF16) {
    if (e5m2) PSD_QMX(DT_BF16, true);
    else PSD_QMX(DT_BF16, false);
  } else if (dt == DT_F32) {
    if (e5m2) PSD_QMX(DT_F32, true);
    else PSD_QMX(DT_F32, false);
  } else {
    return hipErrorInvalidValue;
  }
#undef PSD_QMX
  return hipGetLastError();
}

hipError_t launch_dequant_mx(const uint8_t* q, const uint8_t* scales, int64_t n, void* out, int32_t od, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (n % 32 != 0) return hipErrorInvalidValue;
  const int grid = stream_grid(n >> 3, 256);
  if (od == DT_BF16) hipLaunchKernelGGL(dequant_mx_kernel<DT_BF16>, dim3(grid), dim3(256), 0, st, q, scales, n, out);
  else if (od == DT_F32) hipLaunchKernelGGL(dequant_mx_kernel<DT_F32>, dim3(grid), dim3(256), 0, st, q, scales, n, out);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace psd
