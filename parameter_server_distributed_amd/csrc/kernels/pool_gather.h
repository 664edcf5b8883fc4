// NHWC 3x3 / stride-2 / pad-1 max-pool window max and gather-form gradient, shared by the
// stand-alone pool kernels (pool.hip) and the stem's fused BN+ReLU+pool kernels (bn.hip).
#pragma once
#include "common.h"

namespace psd {

// best[8] / bi[8] = max and argmax (dh*3+dw) over the window of output (n, ho, wo) of f(x) for the
// 8 channels c8*8 .. +8, where f(v, j) transforms element j (identity for the plain pool; the
// stem applies BN scale/shift + ReLU on the fly). NaN propagates like torch.
// All 9 window loads are issued before any is used: coordinates are clamped into the image and
// out-of-image taps are skipped by a select afterwards. (A `continue` around a load makes hipcc
// branch around each load and wait for it before the next -- 9 dependent memory round trips per
// item, the latency that bound these passes at ~2.5 TB/s.)
template <typename F>
__device__ __forceinline__ void maxpool3s2_max8(const uint16_t* __restrict__ x, int n, int ho, int wo, int c8, int H, int W,
                                                int C, F f, float best[8], uint8_t bi[8]) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    best[e] = -INFINITY;
    bi[e] = 0;
  }
  u32x4 raw[9];
#pragma unroll
  for (int dh = 0; dh < 3; ++dh) {
    const int h = min(max(2 * ho - 1 + dh, 0), H - 1);
#pragma unroll
    for (int dw = 0; dw < 3; ++dw) {
      const int w = min(max(2 * wo - 1 + dw, 0), W - 1);
      raw[dh * 3 + dw] = *reinterpret_cast<const u32x4*>(x + (((int64_t)n * H + h) * W + w) * C + c8 * 8);
    }
  }
#pragma unroll
  for (int dh = 0; dh < 3; ++dh) {
    const int h = 2 * ho - 1 + dh;
#pragma unroll
    for (int dw = 0; dw < 3; ++dw) {
      const int w = 2 * wo - 1 + dw;
      const bool in = h >= 0 && h < H && w >= 0 && w < W;
      const u32x4 r = raw[dh * 3 + dw];
      const uint32_t ws[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float v = __uint_as_float((e & 1) ? (ws[e >> 1] & 0xffff0000u) : (ws[e >> 1] << 16));
        const float t = f(v, e);
        if (in && (t > best[e] || (t != t))) {
          best[e] = t;
          bi[e] = (uint8_t)(dh * 3 + dw);
        }
      }
    }
  }
}

__device__ __forceinline__ void store_argmax8(uint8_t* p, const uint8_t bi[8]) {
  const uint32_t lo = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((uint32_t)bi[3] << 24);
  const uint32_t hi = bi[4] | (bi[5] << 8) | (bi[6] << 16) | ((uint32_t)bi[7] << 24);
  *reinterpret_cast<uint2*>(p) = make_uint2(lo, hi);
}

// g[8] = d(pool)/d(x[n, h, w, c8*8 .. +8]): the sum of the <= 4 pooled gradients (gp, plus gp2 when
// given) whose 3x3 window covers (h, w) and whose stored argmax (1 byte per element, dh*3+dw)
// points at it.
__device__ __forceinline__ void maxpool3s2_grad8(const uint16_t* __restrict__ gp, const uint16_t* __restrict__ gp2,
                                                 const uint8_t* __restrict__ arg, int n, int h, int w, int c8, int C,
                                                 int Ho, int Wo, float g[8]) {
#pragma unroll
  for (int e = 0; e < 8; ++e) g[e] = 0.f;
  const int ho0 = h / 2, wo0 = w / 2;  // candidate outputs: ho in {ho0, ho0+1}, window rows 2ho-1..2ho+1
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const int ho = ho0 + a;
    const int dh = h - (2 * ho - 1);
    if (ho >= Ho || dh < 0 || dh > 2) continue;
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int wo = wo0 + b;
      const int dw = w - (2 * wo - 1);
      if (wo >= Wo || dw < 0 || dw > 2) continue;
      const int64_t o = (((int64_t)n * Ho + ho) * Wo + wo) * C + c8 * 8;
      const uint2 ai = *reinterpret_cast<const uint2*>(arg + o);
      float v[8];
      load8_bf16(gp + o, v);
      if (gp2) {
        float v2[8];
        load8_bf16(gp2 + o, v2);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += v2[e];
      }
      const uint8_t want = (uint8_t)(dh * 3 + dw);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const uint8_t ae = (uint8_t)(((e < 4 ? ai.x : ai.y) >> (8 * (e & 3))) & 0xff);
        if (ae == want) g[e] += v[e];
      }
    }
  }
}

// Pool gradient of the 2x2 input block (2k.., 2j..) for 8 channels: g[q][8], q = 2*(row parity) + col parity.
// The 4 pooled outputs' loads (gradient [+ second gradient] + argmax) are issued together with
// clamped indices; an output past the pooled map contributes nothing (select, not a branch).
__device__ __forceinline__ void pool_grad_block(const uint16_t* __restrict__ gp, const uint16_t* __restrict__ gp2,
                                                const uint8_t* __restrict__ arg, int n, int k, int j, int c8, int C,
                                                int Ho, int Wo, float g[4][8]) {
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int e = 0; e < 8; ++e) g[q][e] = 0.f;
  u32x4 rv[4], rv2[4];
  uint2 ra[4];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int ho = min(k + a, Ho - 1), wo = min(j + b, Wo - 1);
      const int64_t o = (((int64_t)n * Ho + ho) * Wo + wo) * C + c8 * 8;
      ra[2 * a + b] = *reinterpret_cast<const uint2*>(arg + o);
      rv[2 * a + b] = *reinterpret_cast<const u32x4*>(gp + o);
      if (gp2) rv2[2 * a + b] = *reinterpret_cast<const u32x4*>(gp2 + o);
    }
  // output (k + a, j + b) -> input (2k + pr, 2j + pc) through window offset (dh, dw) = (pr + 1 - 2a, pc + 1 - 2b)
#pragma unroll
  for (int a = 0; a < 2; ++a) {
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const bool in = k + a < Ho && j + b < Wo;
      const uint2 ai = ra[2 * a + b];
      float v[8];
      {
        const u32x4 r = rv[2 * a + b];
        const uint32_t ws[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = __uint_as_float((e & 1) ? (ws[e >> 1] & 0xffff0000u) : (ws[e >> 1] << 16));
      }
      if (gp2) {
        const u32x4 r = rv2[2 * a + b];
        const uint32_t ws[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
        for (int e = 0; e < 8; ++e)
          v[e] += __uint_as_float((e & 1) ? (ws[e >> 1] & 0xffff0000u) : (ws[e >> 1] << 16));
      }
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        const int dh = pr + 1 - 2 * a;
        if (dh < 0) continue;  // (compile-time: no load behind it)
#pragma unroll
        for (int pc = 0; pc < 2; ++pc) {
          const int dw = pc + 1 - 2 * b;
          if (dw < 0) continue;
          const uint8_t want = (uint8_t)(dh * 3 + dw);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const uint8_t ae = (uint8_t)(((e < 4 ? ai.x : ai.y) >> (8 * (e & 3))) & 0xff);
            if (in && ae == want) g[2 * pr + pc][e] += v[e];
          }
        }
      }
    }
  }
}

}  // namespace psd
