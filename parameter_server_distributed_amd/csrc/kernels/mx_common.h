// OCP fp8 conversions and MX (microscaling) block quantisation shared by the fp8 kernels
// (fp8.hip) and the kernels that write MX operands as a side output (bn.hip apply pass).
#pragma once
#include <hip/hip_fp8.h>

#include "common.h"

namespace psd {

__device__ __forceinline__ float e4m3_to_f32(uint8_t b) {
  const uint32_t s = b >> 7, e = (b >> 3) & 0xF, m = b & 7;
  float v;
  if (e == 0xF && m == 7) return __uint_as_float(0x7fc00000u);  // NaN (e4m3fn has no inf)
  if (e == 0) v = (float)m * 0.001953125f;                      // m/8 * 2^-6
  else v = __uint_as_float(((e + 120u) << 23) | (m << 20));     // (1+m/8) * 2^(e-7)
  return s ? -v : v;
}

__device__ __forceinline__ uint8_t f32_to_e4m3(float x) {
  return (uint8_t)__hip_cvt_float_to_fp8(x, __HIP_SATFINITE, __HIP_E4M3);
}
__device__ __forceinline__ uint8_t f32_to_e5m2(float x) {
  return (uint8_t)__hip_cvt_float_to_fp8(x, __HIP_SATFINITE, __HIP_E5M2);
}
template <bool E5>
__device__ __forceinline__ uint8_t f32_to_f8(float x) {
  if constexpr (E5) return f32_to_e5m2(x);
  else return f32_to_e4m3(x);
}

// E8M0 byte of a 32-element block with absolute maximum amax: the smallest power of two 2^e with
// amax * 2^-e <= fmax (e + 127; 127 for an all-zero or non-finite block)
__device__ __forceinline__ int mx_exp_byte(float amax, float fmax) {
  if (!(amax > 0.f) || !(amax < 3.0e38f)) return 127;  // zero / non-finite block: unit scale
  int p;
  const float m = frexpf(amax / fmax, &p);  // amax / fmax = m 2^p, m in [0.5, 1)
  int e = (m == 0.5f) ? p - 1 : p;
  e = e < -127 ? -127 : (e > 127 ? 127 : e);
  return e + 127;
}

template <int CTRL>
__device__ __forceinline__ float mx_dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}

// One lane's 8 consecutive elements of a 32-element block spread over a lane quad (lanes 4q..4q+3,
// in element order): the block's E8M0 byte (the same on the 4 lanes) and this lane's 8 fp8 bytes.
template <bool E5>
__device__ __forceinline__ int mx_quant8(const float (&t)[8], uint2& out) {
  const float fmax = E5 ? 57344.f : 448.f;
  float m = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) m = fmaxf(m, fabsf(t[e]));
  m = fmaxf(m, mx_dpp<0xB1>(m));  // quad_perm [1,0,3,2]
  m = fmaxf(m, mx_dpp<0x4E>(m));  // quad_perm [2,3,0,1]: the block's 4 lanes agree
  const int eb = mx_exp_byte(m, fmax);
  const float inv = __uint_as_float((uint32_t)(254 - eb) << 23);  // 2^(127 - eb)
  uint32_t lo = 0, hi = 0;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    lo |= (uint32_t)f32_to_f8<E5>(t[e] * inv) << (8 * e);
    hi |= (uint32_t)f32_to_f8<E5>(t[e + 4] * inv) << (8 * e);
  }
  out = make_uint2(lo, hi);
  return eb;
}

}  // namespace psd
