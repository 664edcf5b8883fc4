// Fused NHWC (channels_last) BatchNorm + residual add + ReLU, forward and backward, for gfx950.
//
// Why: rocprofv3 of the ResNet-50 training step (profiles/resnet50_r1_baseline_kernels.md) showed
// PyTorch's channels_last BN kernels at 66% of the step (collect_statistics 368 us and
// backward_reduce 400 us per layer on average, 53 layers), plus separate ReLU / ReLU-backward /
// residual-add kernels. These kernels are pure HBM streaming: the whole BN family of a ResNet-50
// step moves ~50 GB, i.e. ~9 ms at the measured 6 TB/s roof.
//
// Layout: x is [M, C] bf16 row-major (M = N*H*W), C % 8 == 0. One lane owns 8 consecutive channels
// (a 16-byte load); TPC = C/8 lanes cover a row and a 256-lane block covers RPI = 256/TPC rows
// per iteration (4 KiB contiguous), so every load instruction is fully coalesced.
//
// Forward (training):  reduce (shifted sum/sumsq per block) -> finalize (fp64 combine, running
//                      stats, scale/shift) -> apply y = act(x*scale + shift [+ r]).
// Backward:            reduce (sum dy', sum dy'(x-mean); writes dr = dy' for the residual branch)
//                      -> finalize (dgamma/dbeta straight into the parameter-gradient buffers,
//                      3 coefficients) -> elementwise dx = A dy' + B x + C.
// Block partials are combined by a separate finalize launch; a producer's many partial rows (one per
// convolution output tile) are summed and finalized in one ticketed launch (bn_fold_finalize_kernel:
// the agent-scope release / acquire hand-off, correct for any workgroup->XCD placement).
#include <hip/hip_fp8.h>
#include "common.h"
#include "mx_common.h"
#include "launchers_bn.h"
#include "pool_gather.h"

#include <cstdlib>
#include <mutex>

namespace psd {

namespace {

struct Map {
  int tpc, rpi, cg, r0;
  bool active;
};

__device__ __forceinline__ Map make_map(int C) {
  Map m;
  m.tpc = C >> 3;
  if (m.tpc >= 256) {
    m.rpi = 1;
    m.cg = blockIdx.y * 256 + threadIdx.x;
    m.r0 = 0;
    m.active = m.cg < m.tpc;
  } else {
    m.rpi = 256 / m.tpc;
    m.cg = threadIdx.x % m.tpc;
    m.r0 = threadIdx.x / m.tpc;
    m.active = m.r0 < m.rpi;
  }
  return m;
}

// Row visited at logical position r. With rev = 1 the reduce passes walk the rows back to front,
// meant to hit the tail the producing convolution wrote last in the 256 MB Infinity Cache (MALL)
// and leave the head cached for the front-to-back apply pass. Measured neutral at b1024 (the
// passes are HBM-bound at 5.4-6 TB/s either way), kept as an A/B switch.
__device__ __forceinline__ int64_t row_of(int64_t r, int64_t M, int rev) { return rev ? M - 1 - r : r; }

// Sum the per-lane partials (a[8], b[8]) of lanes sharing a channel group and write the block's
// partials to part[blockIdx.x][0|1][C].
__device__ __forceinline__ void block_partials(const Map& m, int C, const float a[8], const float b[8], float* part) {
  float* pa = part + (int64_t)blockIdx.x * 2 * C;
  float* pb = pa + C;
  if (m.tpc >= 256) {
    if (m.active) {
      store8_f32(pa + m.cg * 8, a);
      store8_f32(pb + m.cg * 8, b);
    }
    return;
  }
  __shared__ float red[2][256 * 8];  // [rows][C] flattened: rpi*C <= 256*8
  if (m.active) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[0][m.r0 * C + m.cg * 8 + j] = a[j];
      red[1][m.r0 * C + m.cg * 8 + j] = b[j];
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float sa = 0.f, sb = 0.f;
    for (int r = 0; r < m.rpi; ++r) {
      sa += red[0][r * C + c];
      sb += red[1][r * C + c];
    }
    pa[c] = sa;
    pb[c] = sb;
  }
}

// Finalize launches use one 256-lane block per 8 channels: lane (g, j) = (t >> 3, t & 7) sums the
// partial rows g, g+32, ... of channel c0+j (independent loads, no serial 2048-deep chain), then
// the 32 row groups are combined in LDS in fp64. Returns the totals in lanes t < 8.
constexpr int kFinCh = 8;
__device__ __forceinline__ bool sum_partials(const float* __restrict__ part, int nblk, int C, int c0, double& s,
                                             double& q) {
  const int j = threadIdx.x & 7, g = threadIdx.x >> 3;
  const int c = c0 + j;
  double a = 0.0, b = 0.0;
  if (c < C) {
    float fa[4] = {0.f, 0.f, 0.f, 0.f}, fb[4] = {0.f, 0.f, 0.f, 0.f};
    int r = g;
    for (; r + 96 < nblk; r += 128) {  // 4 fp32 accumulators, their 8 loads issued together
      float va[4], vb[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        va[u] = part[(int64_t)(r + 32 * u) * 2 * C + c];
        vb[u] = part[(int64_t)(r + 32 * u) * 2 * C + C + c];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        fa[u] += va[u];
        fb[u] += vb[u];
      }
    }
    for (int k = 0; r < nblk; r += 32, k = (k + 1) & 3) {
      fa[k] += part[(int64_t)r * 2 * C + c];
      fb[k] += part[(int64_t)r * 2 * C + C + c];
    }
    a = (double)fa[0] + fa[1] + fa[2] + fa[3];
    b = (double)fb[0] + fb[1] + fb[2] + fb[3];
  }
  __shared__ double red[2][32][kFinCh];
  red[0][g][j] = a;
  red[1][g][j] = b;
  __syncthreads();
  if (threadIdx.x < kFinCh) {
    s = 0.0;
    q = 0.0;
    for (int k = 0; k < 32; ++k) {
      s += red[0][k][threadIdx.x];
      q += red[1][k][threadIdx.x];
    }
    return c0 + (int)threadIdx.x < C;
  }
  return false;
}

}  // namespace

// ------------------------------------------------------------------ forward
__global__ __launch_bounds__(256) void bn_fwd_reduce_kernel(const uint16_t* __restrict__ x, int64_t M, int C,
                                                            const float* __restrict__ shift_k, float* __restrict__ part,
                                                            int rev) {
  const Map m = make_map(C);
  float a[8], b[8], k[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = b[j] = k[j] = 0.f;
  if (m.active) {
    if (shift_k) load8_f32(shift_k + m.cg * 8, k);
    const int64_t stride = (int64_t)gridDim.x * m.rpi;
    int64_t r = (int64_t)blockIdx.x * m.rpi + m.r0;
    for (; r + 3 * stride < M; r += 4 * stride) {  // 4 independent 16-B loads in flight per lane
      float v[4][8];
#pragma unroll
      for (int u = 0; u < 4; ++u) load8_bf16(x + row_of(r + u * stride, M, rev) * C + m.cg * 8, v[u]);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = v[u][j] - k[j];
          a[j] += d;
          b[j] = fmaf(d, d, b[j]);
        }
    }
    for (; r < M; r += stride) {
      float v0[8];
      load8_bf16(x + row_of(r, M, rev) * C + m.cg * 8, v0);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float d0 = v0[j] - k[j];
        a[j] += d0;
        b[j] = fmaf(d0, d0, b[j]);
      }
    }
  }
  block_partials(m, C, a, b, part);
}

// Forward finalize of channel c from its totals s = sum (x - k), q = sum (x - k)^2 (k = shift_k[c]):
// saved mean / invstd, scale / shift, running statistics. shift_k aliases running_mean (read, then
// updated by the same lane): no __restrict__ on either.
struct FinFwd {
  int64_t M;
  int C;
  const float* shift_k;
  const uint16_t* gamma;
  const uint16_t* beta;
  float* running_mean;
  float* running_var;
  float momentum, eps;
  float* save_mean;
  float* save_invstd;
  float* ss;
  int64_t* counter;
};

__device__ __forceinline__ void fin_fwd(const FinFwd& f, int c, double s, double q) {
  const double ms = s / (double)f.M;
  double var = q / (double)f.M - ms * ms;
  if (var < 0) var = 0;
  const float k = f.shift_k ? f.shift_k[c] : 0.f;
  const float mean = (float)(ms + (double)k);
  const float invstd = (float)(1.0 / sqrt(var + (double)f.eps));
  f.save_mean[c] = mean;
  f.save_invstd[c] = invstd;
  const float g = f.gamma ? bf16_to_f32(f.gamma[c]) : 1.f;
  const float bt = f.beta ? bf16_to_f32(f.beta[c]) : 0.f;
  const float scale = g * invstd;
  f.ss[c] = scale;
  f.ss[f.C + c] = bt - mean * scale;
  if (f.running_mean) f.running_mean[c] = (1.f - f.momentum) * f.running_mean[c] + f.momentum * mean;
  if (f.running_var) {
    const double unbiased = f.M > 1 ? var * (double)f.M / (double)(f.M - 1) : var;
    f.running_var[c] = (1.f - f.momentum) * f.running_var[c] + f.momentum * (float)unbiased;
  }
}

__global__ __launch_bounds__(256) void bn_fwd_finalize_kernel(const float* __restrict__ part, int nblk, FinFwd f) {
  const int c = blockIdx.x * kFinCh + threadIdx.x;
  if (blockIdx.x == 0 && threadIdx.x == 0 && f.counter) *f.counter += 1;
  double s, q;
  if (!sum_partials(part, nblk, f.C, blockIdx.x * kFinCh, s, q)) return;
  fin_fwd(f, c, s, q);
}

// MASK_OUT: also write the ReLU mask as one bit per element (one byte per 8-channel vector, so a
// wave stores 64 consecutive bytes): backward then reads 1/16 of the bytes y would cost.
// RSS: the residual is itself a raw BN input (the downsample branch's convolution output) whose
// scale/shift rss is applied here, so that BN's own apply pass (a full write + read of the
// residual) never runs.
// Q8 == 2: also write y as OCP e4m3 with MX block scales for an fp8 consumer convolution (one E8M0
// byte per 32 channels into q8mx: 4 lanes hold one block, the block maximum is a DPP quad
// reduction) -- the consumer's own quantise pass (a full read of y) never runs. (The per-tensor
// delayed-scaling form, Q8 == 1, measured no faster than the consumer quantising and was removed in
// round 6.)
// NT / span: streaming loads and stores, one-shot item ranges (common.h elem_range; host
// elem_launch)
template <bool RELU, bool RES, bool MASK_OUT, bool RSS = false, int Q8 = 0, bool NT = false>
__global__ __launch_bounds__(256) void bn_apply_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ res,
                                                       const float* __restrict__ ss, uint16_t* __restrict__ y,
                                                       uint8_t* __restrict__ mbits, int pack4, int64_t nvec, int C,
                                                       const float* __restrict__ rss = nullptr,
                                                       uint8_t* __restrict__ q8 = nullptr,
                                                       uint8_t* __restrict__ q8mx = nullptr, int span = 0) {
  static_assert(Q8 == 0 || Q8 == 2, "bn apply: fp8 side output is MX only");
  const int tpc = C >> 3;
  const ElemRange er = elem_range(nvec, span);
  const int64_t stride = er.stride, hi = er.hi;
  int64_t v = er.v;
  const int cg = (int)(v % tpc);
  float sc[8], sh[8], rsc[8], rsh[8];
  load8_f32(ss + cg * 8, sc);
  load8_f32(ss + C + cg * 8, sh);
  if (RSS) {
    load8_f32(rss + cg * 8, rsc);
    load8_f32(rss + C + cg * 8, rsh);
  }
  // two items in flight per lane (both items' loads issued before either is used: the streaming
  // passes sat at ~4.8 TB/s with one 16-byte load per lane outstanding)
  auto apply = [&](int64_t v, float (&t)[8], const float (&rr)[8]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float o = fmaf(t[j], sc[j], sh[j]);
      if (RSS) o += fmaf(rr[j], rsc[j], rsh[j]);
      else if (RES) o += rr[j];
      if (RELU) o = relu_nan(o);
      t[j] = o;
    }
    store8_bf16<NT>(y + v * 8, t);
    if (Q8 == 2) {  // MX: the stored (bf16-rounded) values, block scale from the lane quad
      float r[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] = bf16_to_f32(f32_to_bf16(t[j]));
      uint2 qb;
      const int eb = mx_quant8<false>(r, qb);
      *reinterpret_cast<uint2*>(q8 + v * 8) = qb;
      if ((v & 3) == 0) q8mx[v >> 2] = (uint8_t)eb;
    }
    if (MASK_OUT) {
      uint32_t bits = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) bits |= (t[j] > 0.f ? 1u : 0u) << j;
      if (pack4) {  // 4 lanes -> one dword store (host: nvec % 4 == 0, so a lane quad is all active)
        // lanes 1..3 of the quad via DPP quad_perm broadcasts (VALU; __shfl_down was an LDS
        // ds_bpermute per value)
        const uint32_t b1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)bits, 0x55, 0xF, 0xF, false);
        const uint32_t b2 = (uint32_t)__builtin_amdgcn_mov_dpp((int)bits, 0xAA, 0xF, 0xF, false);
        const uint32_t b3 = (uint32_t)__builtin_amdgcn_mov_dpp((int)bits, 0xFF, 0xF, 0xF, false);
        if ((threadIdx.x & 3) == 0)
          *reinterpret_cast<uint32_t*>(mbits + v) = bits | (b1 << 8) | (b2 << 16) | (b3 << 24);
      } else {
        mbits[v] = (uint8_t)bits;
      }
    }
  };
  for (; v + stride < hi; v += 2 * stride) {  // (lane quads stay together: nvec, stride, span % 4 == 0)
    float t0[8], t1[8], r0[8], r1[8];
    load8_bf16<NT>(x + v * 8, t0);
    load8_bf16<NT>(x + (v + stride) * 8, t1);
    if (RES) {
      load8_bf16<NT>(res + v * 8, r0);
      load8_bf16<NT>(res + (v + stride) * 8, r1);
    }
    apply(v, t0, r0);
    apply(v + stride, t1, r1);
  }
  for (; v < hi; v += stride) {
    float t[8], rr[8];
    load8_bf16<NT>(x + v * 8, t);
    if (RES) load8_bf16<NT>(res + v * 8, rr);
    apply(v, t, rr);
  }
}

// ------------------------------------------------------------------ backward
// ReLU mask source. kMaskY: y > 0 from the saved forward output (needed when a residual was added
// before the ReLU). kMaskX: x*scale + shift > 0 recomputed from the forward's fp32 scale/shift --
// the same fmaf the apply kernel rounded to y, so the mask is identical -- which saves one full
// [M, C] read in both backward passes (and keeps y out of the autograd context).
// kMaskBits: the 1-bit-per-element mask the forward apply wrote (residual BNs: 1/16 of y's bytes).
enum MaskSrc : int { kMaskNone = 0, kMaskY = 1, kMaskX = 2, kMaskBits = 3 };

// DUAL: also the reduction of a second BN that shares dy' (the downsample BN whose output was the
// residual: its upstream gradient is exactly dr): sum dy'(xd - mean_d) into part_d (sum dy' is common).
template <int MASK, bool RES_OUT, bool DUAL = false>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ dy2,
                                                            const uint16_t* __restrict__ y, const uint8_t* __restrict__ mbits,
                                                            const float* __restrict__ ssf,
                                                            const uint16_t* __restrict__ x, const float* __restrict__ mean,
                                                            uint16_t* __restrict__ dr, int64_t M, int C,
                                                            float* __restrict__ part, int rev,
                                                            const uint16_t* __restrict__ xd = nullptr,
                                                            const float* __restrict__ mean_d = nullptr,
                                                            float* __restrict__ part_d = nullptr) {
  const Map m = make_map(C);
  float a[8], b[8], bd[8], mu[8], mud[8], sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = b[j] = bd[j] = 0.f;
  if (m.active) {
    load8_f32(mean + m.cg * 8, mu);
    if (DUAL) load8_f32(mean_d + m.cg * 8, mud);
    if (MASK == kMaskX) {
      load8_f32(ssf + m.cg * 8, sc);
      load8_f32(ssf + C + m.cg * 8, sh);
    }
    const int64_t stride = (int64_t)gridDim.x * m.rpi;
    auto body = [&](int64_t off, const float* g0, const float* xv, const float* yv, uint32_t bits,
                    const float* xdv) {
      float g[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (MASK == kMaskY) g[j] = yv[j] > 0.f ? g0[j] : 0.f;
        else if (MASK == kMaskX) g[j] = fmaf(xv[j], sc[j], sh[j]) > 0.f ? g0[j] : 0.f;
        else if (MASK == kMaskBits) g[j] = ((bits >> j) & 1u) ? g0[j] : 0.f;
        else g[j] = g0[j];
      }
      if (RES_OUT) store8_bf16(dr + off, g);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        a[j] += g[j];
        b[j] = fmaf(g[j], xv[j] - mu[j], b[j]);
        if (DUAL) bd[j] = fmaf(g[j], xdv[j] - mud[j], bd[j]);
      }
    };
    int64_t r = (int64_t)blockIdx.x * m.rpi + m.r0;
    for (; r + stride < M; r += 2 * stride) {  // two rows (6 loads) in flight per lane
      const int64_t o0 = row_of(r, M, rev) * C + m.cg * 8, o1 = row_of(r + stride, M, rev) * C + m.cg * 8;
      float g0[8], g1[8], x0[8], x1[8], y0[8], y1[8];
      load8_bf16(dy + o0, g0);
      load8_bf16(dy + o1, g1);
      load8_bf16(x + o0, x0);
      load8_bf16(x + o1, x1);
      if (dy2) {  // residual-branch gradient folded in (replaces an autograd add kernel)
        float h0[8], h1[8];
        load8_bf16(dy2 + o0, h0);
        load8_bf16(dy2 + o1, h1);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          g0[j] += h0[j];
          g1[j] += h1[j];
        }
      }
      if (MASK == kMaskY) {
        load8_bf16(y + o0, y0);
        load8_bf16(y + o1, y1);
      }
      uint32_t b0 = 0, b1 = 0;
      if (MASK == kMaskBits) {  // one byte per 8-channel vector
        b0 = mbits[o0 >> 3];
        b1 = mbits[o1 >> 3];
      }
      float d0[8], d1[8];
      if (DUAL) {
        load8_bf16(xd + o0, d0);
        load8_bf16(xd + o1, d1);
      }
      body(o0, g0, x0, y0, b0, d0);
      body(o1, g1, x1, y1, b1, d1);
    }
    for (; r < M; r += stride) {
      const int64_t o0 = row_of(r, M, rev) * C + m.cg * 8;
      float g0[8], x0[8], y0[8];
      load8_bf16(dy + o0, g0);
      load8_bf16(x + o0, x0);
      if (dy2) {
        float h0[8];
        load8_bf16(dy2 + o0, h0);
#pragma unroll
        for (int j = 0; j < 8; ++j) g0[j] += h0[j];
      }
      if (MASK == kMaskY) load8_bf16(y + o0, y0);
      const uint32_t b0 = MASK == kMaskBits ? (uint32_t)mbits[o0 >> 3] : 0u;
      float d0[8];
      if (DUAL) load8_bf16(xd + o0, d0);
      body(o0, g0, x0, y0, b0, d0);
    }
  }
  block_partials(m, C, a, b, part);
  if (DUAL) {
    __syncthreads();  // block_partials' LDS staging is reused
    block_partials(m, C, a, bd, part_d);
  }
}

// Backward finalize of channel c from s1 = sum g, s2 = sum g (x - mean): dgamma / dbeta straight
// into the parameter-gradient buffers and the coefficients of dx = A g + B x + C.
struct FinBwd {
  int64_t M;
  int C;
  const uint16_t* gamma;
  const float* mean;
  const float* invstd;
  uint16_t* dgamma;
  uint16_t* dbeta;
  float* coef;
};

__device__ __forceinline__ void fin_bwd(const FinBwd& f, int c, double s1, double s2) {
  const float is = f.invstd[c];
  if (f.dgamma) f.dgamma[c] = f32_to_bf16((float)(s2 * is));
  if (f.dbeta) f.dbeta[c] = f32_to_bf16((float)s1);
  const float g = f.gamma ? bf16_to_f32(f.gamma[c]) : 1.f;
  const float k1 = g * is;
  const float k3 = (float)(s2 * (double)is * (double)is / (double)f.M);
  const float k2 = (float)(s1 / (double)f.M);
  f.coef[c] = k1;                                       // A
  f.coef[f.C + c] = -k1 * k3;                           // B
  f.coef[2 * f.C + c] = -k1 * k2 + k1 * k3 * f.mean[c];  // C
}

__global__ __launch_bounds__(256) void bn_bwd_finalize_kernel(const float* __restrict__ part, int nblk, FinBwd f) {
  const int c = blockIdx.x * kFinCh + threadIdx.x;
  double s1, s2;
  if (!sum_partials(part, nblk, f.C, blockIdx.x * kFinCh, s1, s2)) return;
  fin_bwd(f, c, s1, s2);
}

// The dual tail's second BN (the downsample branch) from the first one's sums: both see the same
// masked gradient g, so sum g is shared, and sum g (yd - mean_d) = r2 (= sum g yd, the downsample
// fold's rowdot row [0 | sum g yd]) - mean_d sum g. One pass over the partials for both BNs (the
// second used to get a cloned partials buffer with its own -mean_d sum g column, and a pass of its own).
__device__ __forceinline__ void fin_bwd_derived(const FinBwd& f2, const float* r2, int c, double s1) {
  fin_bwd(f2, c, s1 + (double)r2[c], (double)r2[f2.C + c] - (double)f2.mean[c] * s1);
}

__global__ __launch_bounds__(256) void bn_bwd_finalize_dual_kernel(const float* __restrict__ part, int nblk, FinBwd f,
                                                                   FinBwd f2, const float* __restrict__ r2) {
  const int c = blockIdx.x * kFinCh + threadIdx.x;
  double s1, s2;
  if (!sum_partials(part, nblk, f.C, blockIdx.x * kFinCh, s1, s2)) return;
  fin_bwd(f, c, s1, s2);
  fin_bwd_derived(f2, r2, c, s1);
}

// Many producer partial rows (a convolution epilogue writes one per output tile: ~50k for a b1024
// layer1 convolution) summed and finalized in ONE launch: block (f, cg) sums rows [f * chunk, ..)
// of the 32 channels of column group cg into a slab row ws[cg][f], then draws a ticket; the block
// that draws the last one sums the slab rows in a fixed order (deterministic) and runs the
// finalize. The hand-off is cdna_hip_programming.md's in-launch split-K recipe: writer stores ->
// vmcnt(0) -> barrier -> one agent-scope release -> vmcnt(0) -> relaxed agent-scope ticket; the
// reducer one agent-scope acquire before its loads. Replaces part_fold + finalize (two launches,
// ~12 + ~11 us each, 64 + 105 of them per ResNet-50 step).
constexpr int kFfCh = 32;    // channels per column group (64 floats per partial row: s and q)
constexpr int kFfMaxF = 256;  // slab rows per column group
template <bool BWD>
__global__ __launch_bounds__(256) void bn_fold_finalize_kernel(const float* __restrict__ part, int rows, int chunk,
                                                               float* __restrict__ ws, unsigned int* __restrict__ cnt,
                                                               FinFwd ff, FinBwd fb, FinBwd fb2,
                                                               const float* __restrict__ r2) {
  const int C = BWD ? fb.C : ff.C;
  const int f = blockIdx.x, cg = blockIdx.y, F = gridDim.x;
  // partial-row pass: 16 lanes x 16 bytes cover a row's 64 floats of this column group (32 sums,
  // then 32 sums of squares: column col = 4 q4 + e), 16 row groups; 4 independent 16-byte loads in
  // flight per lane (one float per lane per row left this fold at ~1 TB/s, 24 us per call)
  const int q4 = threadIdx.x & 15, rg = threadIdx.x >> 4;
  const int cq = cg * kFfCh + (q4 & 7) * 4;  // first of this lane's 4 channels (C % 8 == 0)
  const bool qok = cq < C;
  const int64_t qoff = (int64_t)(q4 >> 3) * C + cq;
  const int r0 = f * chunk, r1 = min(rows, r0 + chunk);
  f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0, a2 = a0, a3 = a0;
  if (qok) {
    int r = r0 + rg;
    for (; r + 48 < r1; r += 64) {
      a0 += *reinterpret_cast<const f32x4*>(part + (int64_t)r * 2 * C + qoff);
      a1 += *reinterpret_cast<const f32x4*>(part + (int64_t)(r + 16) * 2 * C + qoff);
      a2 += *reinterpret_cast<const f32x4*>(part + (int64_t)(r + 32) * 2 * C + qoff);
      a3 += *reinterpret_cast<const f32x4*>(part + (int64_t)(r + 48) * 2 * C + qoff);
    }
    for (; r < r1; r += 16) a0 += *reinterpret_cast<const f32x4*>(part + (int64_t)r * 2 * C + qoff);
  }
  __shared__ __attribute__((aligned(16))) float red[16][64];
  __shared__ double tot[4][64];
  __shared__ unsigned int ticket;
  *reinterpret_cast<f32x4*>(&red[rg][q4 * 4]) = (a0 + a1) + (a2 + a3);
  __syncthreads();
  const int col = threadIdx.x & 63, rq = threadIdx.x >> 6;
  const int c = cg * kFfCh + (col & 31);
  const bool cok = c < C;
  float* slab = ws + (int64_t)cg * kFfMaxF * 64;
  if (rq == 0) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += red[k][col];
    slab[f * 64 + col] = t;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ticket = __hip_atomic_fetch_add(&cnt[cg], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (ticket != (unsigned int)(F - 1)) return;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(&cnt[cg], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // reusable by the next launch
  }
  __syncthreads();
  // the reducing block: 8 independent slab loads in flight per lane (a one-load-per-iteration chain
  // over the 256 slab rows was most of this kernel's ~20 us)
  double t[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  int k = rq;
  for (; k + 28 < F; k += 32) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = slab[(k + 4 * u) * 64 + col];
#pragma unroll
    for (int u = 0; u < 8; ++u) t[u] += (double)v[u];
  }
  for (; k < F; k += 4) t[0] += (double)slab[k * 64 + col];
  tot[rq][col] = ((t[0] + t[1]) + (t[2] + t[3])) + ((t[4] + t[5]) + (t[6] + t[7]));
  __syncthreads();
  if (threadIdx.x < kFfCh && cok) {
    const int j = threadIdx.x;
    const double s = ((tot[0][j] + tot[1][j]) + tot[2][j]) + tot[3][j];
    const double q = ((tot[0][32 + j] + tot[1][32 + j]) + tot[2][32 + j]) + tot[3][32 + j];
    if (BWD) {
      fin_bwd(fb, c, s, q);
      if (fb2.coef) fin_bwd_derived(fb2, r2, c, s);  // (the dual tail's downsample BN)
    } else {
      fin_fwd(ff, c, s, q);
    }
  }
  if (!BWD && cg == 0 && threadIdx.x == 0 && ff.counter) *ff.counter += 1;
}

// per-device ticket counters of bn_fold_finalize_kernel: zero between launches (the reducing block
// resets its own); consecutive launches take disjoint slot ranges of the ring
static unsigned int* ff_counters(int need) {
  static std::mutex mu;
  const std::lock_guard<std::mutex> lock(mu);
  constexpr int kSlots = 1 << 16;
  static unsigned int* base[16] = {};
  static int next[16] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return nullptr;
  if (!base[dev]) {
    if (hipMalloc(&base[dev], kSlots * sizeof(unsigned int)) != hipSuccess) return nullptr;
    if (hipMemset(base[dev], 0, kSlots * sizeof(unsigned int)) != hipSuccess) return nullptr;
  }
  if (next[dev] + need > kSlots) next[dev] = 0;
  unsigned int* p = base[dev] + next[dev];
  next[dev] += (need + 63) & ~63;
  return p;
}

// fold + finalize of `rows` partial rows in one launch (ws: >= kFfMaxF * 64 * column groups floats)
template <bool BWD>
static hipError_t fold_finalize(const float* part, int rows, float* ws, const FinFwd& ff, const FinBwd& fb,
                                hipStream_t st, const FinBwd& fb2 = FinBwd{}, const float* r2 = nullptr) {
  const int C = BWD ? fb.C : ff.C;
  if (C % 8 != 0 || (reinterpret_cast<uintptr_t>(part) & 15)) return hipErrorInvalidValue;  // 16-byte row loads
  const int ncg = (C + kFfCh - 1) / kFfCh;
  // >= 256 rows per block: each block ends with an agent-scope release (its slab row must be visible
  // to the reducing block on any XCD), and at one block per 64 rows those fences, not the loads, set
  // the time (10-33 us per launch for 200-1600 blocks, profiles/r6/resnet50_b1024_r6i_kernels.md)
  int F = (rows + 255) / 256;
  F = F < 1 ? 1 : (F > kFfMaxF ? kFfMaxF : F);
  const int chunk = (rows + F - 1) / F;
  F = (rows + chunk - 1) / chunk;
  unsigned int* cnt = ff_counters(ncg);
  if (!cnt) return hipErrorOutOfMemory;
  hipLaunchKernelGGL((bn_fold_finalize_kernel<BWD>), dim3(F, ncg), dim3(256), 0, st, part, rows, chunk, ws, cnt, ff,
                     fb, fb2, r2);
  return hipGetLastError();
}

// MODE 0: dy' = dy; MODE 1: dy' = dy * (y > 0); MODE 2: dy' = g (already masked, = dr);
// MODE 3: dy' = dy * (x*scale + shift > 0) (mask recomputed, kMaskX)
// DQ: also write dx as MX e5m2 (one E8M0 byte per 32 channels) for the producing fp8 convolution's
// bwd-data, whose own quantise pass (a full read of dx) then never runs (ops/bn.py _dq8_args)
template <int MODE, bool DQ = false, bool NT = false>
__global__ __launch_bounds__(256) void bn_bwd_elemt_kernel(const uint16_t* __restrict__ g, const uint16_t* __restrict__ g2,
                                                           const uint16_t* __restrict__ y, const float* __restrict__ ssf,
                                                           const uint16_t* __restrict__ x, const float* __restrict__ coef,
                                                           uint16_t* __restrict__ dx, int64_t nvec, int C,
                                                           uint8_t* __restrict__ dq = nullptr,
                                                           uint8_t* __restrict__ dqmx = nullptr, int span = 0) {
  const int tpc = C >> 3;
  const ElemRange er = elem_range(nvec, span);
  const int64_t stride = er.stride, hi = er.hi;
  int64_t v = er.v;
  const int cg = (int)(v % tpc);
  float A[8], B[8], Cc[8], sc[8], sh[8];
  load8_f32(coef + cg * 8, A);
  load8_f32(coef + C + cg * 8, B);
  load8_f32(coef + 2 * C + cg * 8, Cc);
  if (MODE == 3) {
    load8_f32(ssf + cg * 8, sc);
    load8_f32(ssf + C + cg * 8, sh);
  }
  auto elemt = [&](int64_t v, float (&gv)[8], const float (&xv)[8], const float (&h)[8], const float (&yv)[8]) {
    if (MODE != 2 && g2) {
#pragma unroll
      for (int j = 0; j < 8; ++j) gv[j] += h[j];
    }
    if (MODE == 1) {
#pragma unroll
      for (int j = 0; j < 8; ++j) gv[j] = yv[j] > 0.f ? gv[j] : 0.f;
    }
    if (MODE == 3) {
#pragma unroll
      for (int j = 0; j < 8; ++j) gv[j] = fmaf(xv[j], sc[j], sh[j]) > 0.f ? gv[j] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) gv[j] = fmaf(A[j], gv[j], fmaf(B[j], xv[j], Cc[j]));
    store8_bf16<NT>(dx + v * 8, gv);
    if constexpr (DQ) {
#pragma unroll
      for (int j = 0; j < 8; ++j) gv[j] = bf16_to_f32(f32_to_bf16(gv[j]));  // the stored values
      uint2 qb;
      const int eb = mx_quant8<true>(gv, qb);
      *reinterpret_cast<uint2*>(dq + v * 8) = qb;
      if ((v & 3) == 0) dqmx[v >> 2] = (uint8_t)eb;
    }
  };
  // two items in flight per lane (all loads of both before either is used)
  for (; v + stride < hi; v += 2 * stride) {
    float g0[8], g1[8], x0[8], x1[8], h0[8], h1[8], y0[8], y1[8];
    load8_bf16<NT>(g + v * 8, g0);
    load8_bf16<NT>(g + (v + stride) * 8, g1);
    load8_bf16<NT>(x + v * 8, x0);
    load8_bf16<NT>(x + (v + stride) * 8, x1);
    if (MODE != 2 && g2) {
      load8_bf16<NT>(g2 + v * 8, h0);
      load8_bf16<NT>(g2 + (v + stride) * 8, h1);
    }
    if (MODE == 1) {
      load8_bf16<NT>(y + v * 8, y0);
      load8_bf16<NT>(y + (v + stride) * 8, y1);
    }
    elemt(v, g0, x0, h0, y0);
    elemt(v + stride, g1, x1, h1, y1);
  }
  for (; v < hi; v += stride) {
    float gv[8], xv[8], h[8], yv[8];
    load8_bf16<NT>(g + v * 8, gv);
    load8_bf16<NT>(x + v * 8, xv);
    if (MODE != 2 && g2) load8_bf16<NT>(g2 + v * 8, h);
    if (MODE == 1) load8_bf16<NT>(y + v * 8, yv);
    elemt(v, gv, xv, h, yv);
  }
}

// dual elementwise pass: dx = A g + B x + C and dxd = Ad g + Bd xd + Cd from one read of g (= dr)
// WDX false (the BN-backward fold of this BN's consumer convolution, ops/bn.py): only the downsample
// BN's input gradient is written; this BN's own is folded into its producer's backward GEMMs
template <bool WDX, bool NT = false>
__global__ __launch_bounds__(256) void bn_bwd_elemt_dual_kernel(const uint16_t* __restrict__ g, const uint16_t* __restrict__ x,
                                                                const float* __restrict__ coef, uint16_t* __restrict__ dx,
                                                                const uint16_t* __restrict__ xd,
                                                                const float* __restrict__ coef_d,
                                                                uint16_t* __restrict__ dxd, int64_t nvec, int C,
                                                                int span = 0) {
  const int tpc = C >> 3;
  const ElemRange er = elem_range(nvec, span);
  const int64_t stride = er.stride, hi = er.hi;
  int64_t v = er.v;
  const int cg = (int)(v % tpc);
  float A[8], B[8], Cc[8], Ad[8], Bd[8], Cd[8];
  load8_f32(coef + cg * 8, A);
  load8_f32(coef + C + cg * 8, B);
  load8_f32(coef + 2 * C + cg * 8, Cc);
  load8_f32(coef_d + cg * 8, Ad);
  load8_f32(coef_d + C + cg * 8, Bd);
  load8_f32(coef_d + 2 * C + cg * 8, Cd);
  auto dual = [&](int64_t v, const float (&gv)[8], const float (&dv)[8], const float (&xv)[8]) {
    float o[8];
    if constexpr (WDX) {
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = fmaf(A[j], gv[j], fmaf(B[j], xv[j], Cc[j]));
      store8_bf16<NT>(dx + v * 8, o);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = fmaf(Ad[j], gv[j], fmaf(Bd[j], dv[j], Cd[j]));
    store8_bf16<NT>(dxd + v * 8, o);
  };
  for (; v + stride < hi; v += 2 * stride) {  // two items in flight per lane
    float g0[8], g1[8], d0[8], d1[8], x0[8], x1[8];
    load8_bf16<NT>(g + v * 8, g0);
    load8_bf16<NT>(g + (v + stride) * 8, g1);
    load8_bf16<NT>(xd + v * 8, d0);
    load8_bf16<NT>(xd + (v + stride) * 8, d1);
    if constexpr (WDX) {
      load8_bf16<NT>(x + v * 8, x0);
      load8_bf16<NT>(x + (v + stride) * 8, x1);
    }
    dual(v, g0, d0, x0);
    dual(v + stride, g1, d1, x1);
  }
  for (; v < hi; v += stride) {
    float gv[8], dv[8], xv[8];
    load8_bf16<NT>(g + v * 8, gv);
    load8_bf16<NT>(xd + v * 8, dv);
    if constexpr (WDX) load8_bf16<NT>(x + v * 8, xv);
    dual(v, gv, dv, xv);
  }
}

// ------------------------------------------------------------------ stem: BN + ReLU + 3x3/s2 max-pool
// The stem BN's output feeds only the max-pool, so it is never materialised: the forward applies
// scale/shift + ReLU inside the pool window (rounded to bf16 first: bitwise the unfused result),
// and the backward recomputes the pool gradient from the pooled gradients + 1-byte argmax inside
// both BN backward passes. Per b1024 step this drops the 1.64 GB y write + read and the 1.64 GB
// pool-gradient write + two reads.
//
// Backward work item = one 2x2 input block (2k..2k+1, 2j..2j+1) x 8 channels: its gradient comes
// from the 4 pooled outputs (k..k+1, j..j+1) only (even rows / cols sit in one window, odd ones in
// two), so each pooled gradient is loaded once per block instead of once per covered input.
__global__ __launch_bounds__(256) void bn_relu_maxpool_kernel(const uint16_t* __restrict__ x, const float* __restrict__ ss,
                                                              uint16_t* __restrict__ y, uint8_t* __restrict__ arg, int N,
                                                              int H, int W, int C, int Ho, int Wo, FastDiv dc8,
                                                              FastDiv dwo, FastDiv dho) {
  // 32-bit item index (host: total < 2^31) split by fast division: (n, ho, wo, c8)
  const uint32_t total = (uint32_t)N * Ho * Wo * dc8.d;
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    const uint32_t r = fdiv_q(t, dc8);
    const int c8 = (int)(t - r * dc8.d);
    const uint32_t r2 = fdiv_q(r, dwo);
    const int wo = (int)(r - r2 * dwo.d);
    const uint32_t n = fdiv_q(r2, dho);
    const int ho = (int)(r2 - n * dho.d);
    float sc[8], sh[8];
    load8_f32(ss + c8 * 8, sc);
    load8_f32(ss + C + c8 * 8, sh);
    float best[8];
    uint8_t bi[8];
    maxpool3s2_max8(
        x, (int)n, ho, wo, c8, H, W, C,
        [&](float v, int e) { return bf16_to_f32(f32_to_bf16(relu_nan(fmaf(v, sc[e], sh[e])))); }, best, bi);
    store8_bf16(y + (int64_t)t * 8, best);
    store_argmax8(arg + (int64_t)t * 8, bi);
  }
}

// Blocks of the pool-fused backward: lane = (block item r0, channel group cg), rpi = 256 / (C/8)
// items per block iteration; items are (n, k, j) 2x2 input blocks.
__global__ __launch_bounds__(256) void bn_bwd_reduce_pool_kernel(const uint16_t* __restrict__ gp,
                                                                 const uint16_t* __restrict__ gp2,
                                                                 const uint8_t* __restrict__ arg,
                                                                 const float* __restrict__ ssf,
                                                                 const uint16_t* __restrict__ x,
                                                                 const float* __restrict__ mean, int N, int H, int W,
                                                                 int C, float* __restrict__ part, FastDiv dwo,
                                                                 FastDiv dho) {
  const Map m = make_map(C);
  const int Ho = H / 2, Wo = W / 2;
  float a[8], b[8], mu[8], sc[8], sh[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) a[e] = b[e] = 0.f;
  if (m.active) {
    load8_f32(mean + m.cg * 8, mu);
    load8_f32(ssf + m.cg * 8, sc);
    load8_f32(ssf + C + m.cg * 8, sh);
    const uint32_t items = (uint32_t)N * Ho * Wo;  // host: < 2^31
    const uint32_t stride = gridDim.x * m.rpi;
    for (uint32_t it = blockIdx.x * m.rpi + m.r0; it < items; it += stride) {
      const uint32_t q = fdiv_q(it, dwo);
      const int j = (int)(it - q * dwo.d);
      const uint32_t n = fdiv_q(q, dho);
      const int k = (int)(q - n * dho.d);
      float g[4][8];
      pool_grad_block(gp, gp2, arg, (int)n, k, j, m.cg, C, Ho, Wo, g);
#pragma unroll
      for (int pq = 0; pq < 4; ++pq) {
        const int h = 2 * k + (pq >> 1), w = 2 * j + (pq & 1);
        float xv[8];
        load8_bf16(x + (((int64_t)n * H + h) * W + w) * C + m.cg * 8, xv);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float gm = fmaf(xv[e], sc[e], sh[e]) > 0.f ? g[pq][e] : 0.f;
          a[e] += gm;
          b[e] = fmaf(gm, xv[e] - mu[e], b[e]);
        }
      }
    }
  }
  block_partials(m, C, a, b, part);
}

__global__ __launch_bounds__(256) void bn_bwd_elemt_pool_kernel(const uint16_t* __restrict__ gp,
                                                                const uint16_t* __restrict__ gp2,
                                                                const uint8_t* __restrict__ arg,
                                                                const float* __restrict__ ssf,
                                                                const uint16_t* __restrict__ x,
                                                                const float* __restrict__ coef,
                                                                uint16_t* __restrict__ dx, int N, int H, int W, int C,
                                                                FastDiv dc8, FastDiv dwo, FastDiv dho) {
  const int Ho = H / 2, Wo = W / 2;
  const uint32_t total = (uint32_t)N * Ho * Wo * dc8.d;  // host: < 2^31
  const uint32_t stride = gridDim.x * blockDim.x;        // host: stride % c8n == 0
  uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const int c8 = (int)(t - fdiv_q(t, dc8) * dc8.d);
  float A[8], B[8], Cc[8], sc[8], sh[8];
  load8_f32(coef + c8 * 8, A);
  load8_f32(coef + C + c8 * 8, B);
  load8_f32(coef + 2 * C + c8 * 8, Cc);
  load8_f32(ssf + c8 * 8, sc);
  load8_f32(ssf + C + c8 * 8, sh);
  for (; t < total; t += stride) {
    const uint32_t it = fdiv_q(t, dc8);
    const uint32_t q = fdiv_q(it, dwo);
    const int j = (int)(it - q * dwo.d);
    const uint32_t n = fdiv_q(q, dho);
    const int k = (int)(q - n * dho.d);
    float g[4][8];
    pool_grad_block(gp, gp2, arg, (int)n, k, j, c8, C, Ho, Wo, g);
#pragma unroll
    for (int pq = 0; pq < 4; ++pq) {
      const int h = 2 * k + (pq >> 1), w = 2 * j + (pq & 1);
      const int64_t off = (((int64_t)n * H + h) * W + w) * C + c8 * 8;
      float xv[8];
      load8_bf16<true>(x + off, xv);  // x and dx: touched once, streaming (1.6 GB at b1024)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float gm = fmaf(xv[e], sc[e], sh[e]) > 0.f ? g[pq][e] : 0.f;
        g[pq][e] = fmaf(A[e], gm, fmaf(B[e], xv[e], Cc[e]));
      }
      store8_bf16<true>(dx + off, g[pq]);
    }
  }
}

// ------------------------------------------------------------------ host launchers
static int gcd_i(int a, int b) { return b == 0 ? a : gcd_i(b, a % b); }

static void reduce_grid(int64_t M, int C, int& gx, int& gy) {
  const int tpc = C >> 3;
  int rpi;
  if (tpc >= 256) {
    gy = (tpc + 255) / 256;
    rpi = 1;
  } else {
    gy = 1;
    rpi = 256 / tpc;
  }
  // >= 16 rows per lane (4 loads in flight each), <= 512 partial rows: the finalize kernel then
  // sums at most 16 partials per lane instead of a 2048-deep dependent chain
  int64_t want = (M + (int64_t)rpi * 16 - 1) / ((int64_t)rpi * 16);
  int64_t cap = 512 / gy;
  if (cap < 1) cap = 1;
  gx = (int)(want < 1 ? 1 : (want > cap ? cap : want));
}

hipError_t launch_bn_reduce(const uint16_t* x, int64_t M, int C, const float* shift, float* part, hipStream_t st) {
  if (M <= 0 || C % 8 != 0) return hipErrorInvalidValue;
  int gx, gy;
  reduce_grid(M, C, gx, gy);
  hipLaunchKernelGGL(bn_fwd_reduce_kernel, dim3(gx, gy), dim3(256), 0, st, x, M, C, shift, part, 0);
  return hipGetLastError();
}

int bn_reduce_blocks(int64_t M, int C) {
  int gx, gy;
  reduce_grid(M, C, gx, gy);
  return gx;
}

static int elem_grid(int64_t nvec, int C) {
  const int tpc = C >> 3;
  int g = stream_grid(nvec, 256);
  const int mult = tpc / gcd_i(tpc, 256);  // (g*256) % tpc == 0  <=>  g % mult == 0
  g = ((g + mult - 1) / mult) * mult;
  return g;
}

// Launch shape of the per-channel elementwise passes (apply, backward elementwise, dual): one-shot
// 512-item blocks when C/8 divides 256 (common.h elem_range), else the grid-stride loop; streaming
// loads / stores for tensors above 128 MB, which cannot stay in the 256 MB Infinity Cache for their
// consumer anyway (below that the cached form measured faster: profiles/r6/elemt_variants.md).
struct ElemLaunch {
  int grid, span;
  bool nt;
};
static ElemLaunch elem_launch(int64_t nvec, int C) {
  const int tpc = C >> 3;
  const bool nt = nvec * 16 > (128LL << 20);
  if (tpc > 0 && 256 % tpc == 0) return {(int)((nvec + 511) / 512), 512, nt};
  return {elem_grid(nvec, C), 0, nt};
}

template <bool R, bool S, bool B, bool RS, int Q8>
static void apply_launch(const BnFwdArgs& a, const ElemLaunch& el, int64_t nvec, hipStream_t st) {
  const int pack4 = (int)(nvec % 4 == 0);
  if (el.nt)
    hipLaunchKernelGGL((bn_apply_kernel<R, S, B, RS, Q8, true>), dim3(el.grid), dim3(256), 0, st, a.x, a.res, a.ss,
                       a.y, a.mbits, pack4, nvec, a.C, a.res_ss, a.q8, a.q8mx, el.span);
  else
    hipLaunchKernelGGL((bn_apply_kernel<R, S, B, RS, Q8, false>), dim3(el.grid), dim3(256), 0, st, a.x, a.res, a.ss,
                       a.y, a.mbits, pack4, nvec, a.C, a.res_ss, a.q8, a.q8mx, el.span);
}

template <int MODE, bool DQ>
static void elemt_launch(const ElemLaunch& el, const uint16_t* g, const uint16_t* g2, const uint16_t* y,
                         const float* ssf, const uint16_t* x, const float* coef, uint16_t* dx, int64_t nvec, int C,
                         uint8_t* dq, uint8_t* dqmx, hipStream_t st) {
  if (el.nt)
    hipLaunchKernelGGL((bn_bwd_elemt_kernel<MODE, DQ, true>), dim3(el.grid), dim3(256), 0, st, g, g2, y, ssf, x, coef,
                       dx, nvec, C, dq, dqmx, el.span);
  else
    hipLaunchKernelGGL((bn_bwd_elemt_kernel<MODE, DQ, false>), dim3(el.grid), dim3(256), 0, st, g, g2, y, ssf, x, coef,
                       dx, nvec, C, dq, dqmx, el.span);
}

template <bool WDX>
static void dual_launch(const ElemLaunch& el, const uint16_t* g, const uint16_t* x, const float* coef, uint16_t* dx,
                        const uint16_t* xd, const float* coef_d, uint16_t* dxd, int64_t nvec, int C, hipStream_t st) {
  if (el.nt)
    hipLaunchKernelGGL((bn_bwd_elemt_dual_kernel<WDX, true>), dim3(el.grid), dim3(256), 0, st, g, x, coef, dx, xd,
                       coef_d, dxd, nvec, C, el.span);
  else
    hipLaunchKernelGGL((bn_bwd_elemt_dual_kernel<WDX, false>), dim3(el.grid), dim3(256), 0, st, g, x, coef, dx, xd,
                       coef_d, dxd, nvec, C, el.span);
}

hipError_t launch_bn_fwd(const BnFwdArgs& a, hipStream_t st) {
  if (a.M <= 0) return hipSuccess;
  if (a.C % 8 != 0) return hipErrorInvalidValue;
  int gx, gy;
  reduce_grid(a.M, a.C, gx, gy);
  if (a.training) {
    const FinFwd ff{a.M, a.C, a.running_mean, a.gamma, a.beta, a.running_mean, a.running_var, a.momentum, a.eps,
                    a.save_mean, a.save_invstd, a.ss, a.counter};
    if (a.part_ready > kFoldRows && a.fold_ws) {  // many producer partial rows (convolution epilogue)
      const hipError_t e = fold_finalize<false>(a.part, a.part_ready, a.fold_ws, ff, FinBwd{}, st);
      if (e != hipSuccess) return e;
    } else {
      if (a.part_ready > 0) {  // statistics already reduced by the producing kernel (stem conv epilogue)
        gx = a.part_ready;
      } else {
        hipLaunchKernelGGL(bn_fwd_reduce_kernel, dim3(gx, gy), dim3(256), 0, st, a.x, a.M, a.C, a.running_mean,
                           a.part, 0);
      }
      hipLaunchKernelGGL(bn_fwd_finalize_kernel, dim3((a.C + kFinCh - 1) / kFinCh), dim3(256), 0, st, a.part, gx, ff);
    }
    if (a.stats_only) return hipGetLastError();
  }
  if (a.pool_arg) {  // stem: y is the pooled output, the BN output is never written
    if (!a.relu || a.res || a.mbits || !bn_pool_supported(a.H, a.W, a.C) || (int64_t)a.N * a.H * a.W != a.M)
      return hipErrorInvalidValue;
    const int Ho = a.H / 2, Wo = a.W / 2;
    const int64_t total = (int64_t)a.N * Ho * Wo * (a.C / 8);
    if (total >= ((int64_t)1 << 31) - 2048 * 256) return hipErrorInvalidValue;  // 32-bit item indices
    // one item per lane (no grid-stride loop): like the elementwise passes, the one-shot grid
    // streams faster than 2048 looping workgroups (profiles/r6/elemt_variants.md)
    hipLaunchKernelGGL(bn_relu_maxpool_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, a.x, a.ss, a.y,
                       a.pool_arg, a.N, a.H, a.W, a.C, Ho, Wo, make_fastdiv((uint32_t)(a.C / 8)),
                       make_fastdiv((uint32_t)Wo), make_fastdiv((uint32_t)Ho));
    return hipGetLastError();
  }
  const int64_t nvec = a.M * (a.C / 8);
  const ElemLaunch el = elem_launch(nvec, a.C);
  if (a.q8 && a.q8mx) {  // MX fp8 side output (every lane quad = one 32-channel block)
    if (!a.relu || a.C % 32 != 0 || nvec % 4 != 0) return hipErrorInvalidValue;
    if (a.res_ss && a.res && a.mbits) apply_launch<true, true, true, true, 2>(a, el, nvec, st);
    else if (a.res && a.mbits && !a.res_ss) apply_launch<true, true, true, false, 2>(a, el, nvec, st);
    else if (!a.res && !a.mbits && !a.res_ss) apply_launch<true, false, false, false, 2>(a, el, nvec, st);
    else return hipErrorInvalidValue;
    return hipGetLastError();
  }
  if (a.q8) return hipErrorInvalidValue;  // the fp8 side output needs its MX scales
  if (a.res_ss) {  // residual = bn(res) applied on the fly (ReLU blocks only)
    if (!a.res || !a.relu) return hipErrorInvalidValue;
    if (a.mbits) apply_launch<true, true, true, true, 0>(a, el, nvec, st);
    else apply_launch<true, true, false, true, 0>(a, el, nvec, st);
    return hipGetLastError();
  }
  if (a.relu && a.res && a.mbits) apply_launch<true, true, true, false, 0>(a, el, nvec, st);
  else if (a.relu && a.mbits) apply_launch<true, false, true, false, 0>(a, el, nvec, st);
  else if (a.relu && a.res) apply_launch<true, true, false, false, 0>(a, el, nvec, st);
  else if (a.relu) apply_launch<true, false, false, false, 0>(a, el, nvec, st);
  else if (a.res) apply_launch<false, true, false, false, 0>(a, el, nvec, st);
  else apply_launch<false, false, false, false, 0>(a, el, nvec, st);
  return hipGetLastError();
}

bool bn_pool_supported(int H, int W, int C) {
  // 2x2 blocks of an even input; a block's lanes (C/8 channel groups) tile 256 lanes exactly
  return H > 0 && W > 0 && H % 2 == 0 && W % 2 == 0 && C % 8 == 0 && C / 8 <= 256 && 256 % (C / 8) == 0;
}

// More blocks than the plain reduce (<= 2048, not 512): a work item gathers 4 pooled gradients and
// 4 inputs, and at 512 blocks the pass ran at half the streaming bandwidth (latency-bound).
int bn_pool_reduce_blocks(int N, int H, int W, int C) {
  const int64_t items = (int64_t)N * (H / 2) * (W / 2);
  const int rpi = 256 / (C / 8);
  int64_t g = (items + (int64_t)rpi * 4 - 1) / ((int64_t)rpi * 4);
  return (int)(g < 1 ? 1 : (g > 2048 ? 2048 : g));
}

static hipError_t launch_bn_bwd_pool(const BnBwdArgs& a, hipStream_t st) {
  if (!a.relu || !a.ss || a.dr || a.dy2 || !bn_pool_supported(a.H, a.W, a.C) || (int64_t)a.N * a.H * a.W != a.M)
    return hipErrorInvalidValue;
  const int64_t total = (int64_t)a.N * (a.H / 2) * (a.W / 2) * (a.C / 8);
  if (total >= ((int64_t)1 << 31) - 2048 * 256) return hipErrorInvalidValue;  // 32-bit item indices
  const FastDiv dc8 = make_fastdiv((uint32_t)(a.C / 8)), dwo = make_fastdiv((uint32_t)(a.W / 2)),
                dho = make_fastdiv((uint32_t)(a.H / 2));
  const int gx = bn_pool_reduce_blocks(a.N, a.H, a.W, a.C), gy = 1;  // the caller sized part for this
  hipLaunchKernelGGL(bn_bwd_reduce_pool_kernel, dim3(gx, gy), dim3(256), 0, st, a.gpool, a.gpool2, a.pool_arg, a.ss, a.x,
                     a.save_mean, a.N, a.H, a.W, a.C, a.part, dwo, dho);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((a.C + kFinCh - 1) / kFinCh), dim3(256), 0, st, a.part, gx,
                     FinBwd{a.M, a.C, a.gamma, a.save_mean, a.save_invstd, a.dgamma, a.dbeta, a.coef});
  const int g = elem_grid(total, a.C);  // (a one-shot grid measured 4 % slower here, r6t)
  hipLaunchKernelGGL(bn_bwd_elemt_pool_kernel, dim3(g), dim3(256), 0, st, a.gpool, a.gpool2, a.pool_arg, a.ss, a.x,
                     a.coef, a.dx, a.N, a.H, a.W, a.C, dc8, dwo, dho);
  return hipGetLastError();
}

// finalize from `rows` producer-reduced partial rows (more than kFoldRows: summed and finalized in
// one ticketed launch, fold_ws its slab workspace)
static hipError_t finalize_pre(const float* part, int rows, float* fold_ws, int64_t M, int C, const uint16_t* gamma,
                               const float* mean, const float* invstd, uint16_t* dgamma, uint16_t* dbeta, float* coef,
                               hipStream_t st, const FinBwd& fb2 = FinBwd{}, const float* r2 = nullptr) {
  const FinBwd fb{M, C, gamma, mean, invstd, dgamma, dbeta, coef};
  if (rows > kFoldRows) return fold_finalize<true>(part, rows, fold_ws, FinFwd{}, fb, st, fb2, r2);
  if (fb2.coef)
    hipLaunchKernelGGL(bn_bwd_finalize_dual_kernel, dim3((C + kFinCh - 1) / kFinCh), dim3(256), 0, st, part, rows, fb,
                       fb2, r2);
  else
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + kFinCh - 1) / kFinCh), dim3(256), 0, st, part, rows, fb);
  return hipGetLastError();
}

// BN backward from a producer-reduced gradient (kernels/convn.hip bwd modes): g is already masked
// (and holds the residual-branch gradient), part holds `rows` rows of (sum g, sum g (x - mean)).
hipError_t launch_bn_bwd_pre(const uint16_t* g, const uint16_t* x, const uint16_t* gamma, const float* mean,
                             const float* invstd, const float* part, int rows, float* fold_ws, uint16_t* dgamma,
                             uint16_t* dbeta, float* coef, uint16_t* dx, int64_t M, int C, hipStream_t st, uint8_t* dq,
                             uint8_t* dqmx) {
  if (M <= 0) return hipSuccess;
  if (C % 8 != 0 || rows <= 0) return hipErrorInvalidValue;
  if (rows > kFoldRows && !fold_ws) return hipErrorInvalidValue;
  const hipError_t fe = finalize_pre(part, rows, fold_ws, M, C, gamma, mean, invstd, dgamma, dbeta, coef, st);
  if (fe != hipSuccess) return fe;
  if (!dx) return hipGetLastError();  // coefficients only (BN-backward fold)
  const int64_t nvec = M * (C / 8);
  if (dq) {
    if (!dqmx || C % 32 != 0) return hipErrorInvalidValue;
    elemt_launch<2, true>(elem_launch(nvec, C), g, nullptr, nullptr, nullptr, x, coef, dx, nvec, C, dq, dqmx, st);
  } else {
    elemt_launch<2, false>(elem_launch(nvec, C), g, nullptr, nullptr, nullptr, x, coef, dx, nvec, C, nullptr, nullptr,
                           st);
  }
  return hipGetLastError();
}

// dx = A g + B x + C per channel from finalized coefficients (the unfolded twin of the BN-backward
// fold: what the BN's own elementwise pass writes)
hipError_t launch_bn_elemt_coef(const uint16_t* g, const uint16_t* x, const float* coef, uint16_t* dx, int64_t M, int C,
                                hipStream_t st) {
  if (M <= 0) return hipSuccess;
  if (C % 8 != 0) return hipErrorInvalidValue;
  const int64_t nvec = M * (C / 8);
  elemt_launch<2, false>(elem_launch(nvec, C), g, nullptr, nullptr, nullptr, x, coef, dx, nvec, C, nullptr, nullptr, st);
  return hipGetLastError();
}



// Dual tail relu(bn(x) + bnd(xd)) backward from partials reduced in the consumer convolution's
// bwd-data epilogue (kernels/convn.hip bwd mode 3): finalize both BNs, then one elementwise pass (dx
// may be null: bn's input gradient folded into its producer, ops/conv.py _fold_backward).
hipError_t launch_bn_bwd_dual_pre(const BnDualPreArgs& a, hipStream_t st) {
  if (a.M <= 0) return hipSuccess;
  if (a.C % 8 != 0 || a.rows <= 0 || (a.rows > kFoldRows && (!a.fold_ws || (!a.fold_ws_d && !a.derive_d))))
    return hipErrorInvalidValue;
  hipError_t fe;
  if (a.derive_d) {  // part_d = the downsample fold's rowdot row: both BNs from one pass over part
    const FinBwd fb2{a.M, a.C, a.gamma_d, a.mean_d, a.invstd_d, a.dgamma_d, a.dbeta_d, a.coef_d};
    fe = finalize_pre(a.part, a.rows, a.fold_ws, a.M, a.C, a.gamma, a.mean, a.invstd, a.dgamma, a.dbeta, a.coef, st,
                      fb2, a.part_d);
  } else {
    fe = finalize_pre(a.part, a.rows, a.fold_ws, a.M, a.C, a.gamma, a.mean, a.invstd, a.dgamma, a.dbeta, a.coef, st);
    if (fe == hipSuccess)
      fe = finalize_pre(a.part_d, a.rows, a.fold_ws_d, a.M, a.C, a.gamma_d, a.mean_d, a.invstd_d, a.dgamma_d,
                        a.dbeta_d, a.coef_d, st);
  }
  if (fe != hipSuccess) return fe;
  if (!a.dx && !a.dxd) return hipSuccess;  // both BN input gradients folded into their convolutions
  if (!a.dxd) return hipErrorInvalidValue;
  const int64_t nvec = a.M * (a.C / 8);
  if (a.dx) dual_launch<true>(elem_launch(nvec, a.C), a.g, a.x, a.coef, a.dx, a.xd, a.coef_d, a.dxd, nvec, a.C, st);
  else dual_launch<false>(elem_launch(nvec, a.C), a.g, a.x, a.coef, a.dx, a.xd, a.coef_d, a.dxd, nvec, a.C, st);
  return hipGetLastError();
}

hipError_t launch_bn_bwd(const BnBwdArgs& a, hipStream_t st) {
  if (a.M <= 0) return hipSuccess;
  if (a.C % 8 != 0) return hipErrorInvalidValue;
  if (a.gpool) return launch_bn_bwd_pool(a, st);
  int gx, gy;
  reduce_grid(a.M, a.C, gx, gy);
  // ReLU mask: forward bit-mask, else y, else recomputed from x and the forward scale/shift
  const int mask = !a.relu ? kMaskNone : (a.mbits ? kMaskBits : (a.y ? kMaskY : kMaskX));
  if (mask == kMaskX && !a.ss) return hipErrorInvalidValue;
  if (mask == kMaskBits && !a.dr) return hipErrorInvalidValue;  // bits are kept for residual BNs only
  if (a.xd) {  // dual: this BN (bit-mask, dr out) + the downsample BN fed by dr
    if (mask != kMaskBits || !a.dxd || !a.coef_d || !a.part_d || !a.mean_d || !a.invstd_d)
      return hipErrorInvalidValue;
    hipLaunchKernelGGL((bn_bwd_reduce_kernel<kMaskBits, true, true>), dim3(gx, gy), dim3(256), 0, st, a.dy, a.dy2, a.y,
                       a.mbits, a.ss, a.x, a.save_mean, a.dr, a.M, a.C, a.part, 0, a.xd, a.mean_d, a.part_d);
    const dim3 fg((a.C + kFinCh - 1) / kFinCh);
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, fg, dim3(256), 0, st, a.part, gx,
                       FinBwd{a.M, a.C, a.gamma, a.save_mean, a.save_invstd, a.dgamma, a.dbeta, a.coef});
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, fg, dim3(256), 0, st, a.part_d, gx,
                       FinBwd{a.M, a.C, a.gamma_d, a.mean_d, a.invstd_d, a.dgamma_d, a.dbeta_d, a.coef_d});
    const int64_t nvec = a.M * (a.C / 8);
    if (a.dx) dual_launch<true>(elem_launch(nvec, a.C), a.dr, a.x, a.coef, a.dx, a.xd, a.coef_d, a.dxd, nvec, a.C, st);
    else dual_launch<false>(elem_launch(nvec, a.C), a.dr, a.x, a.coef, a.dx, a.xd, a.coef_d, a.dxd, nvec, a.C, st);
    return hipGetLastError();
  }
#define PSD_RED(K, O)                                                                                              \
  hipLaunchKernelGGL((bn_bwd_reduce_kernel<K, O>), dim3(gx, gy), dim3(256), 0, st, a.dy, a.dy2, a.y, a.mbits, a.ss, \
                     a.x, a.save_mean, a.dr, a.M, a.C, a.part, \
                     0)
  if (mask == kMaskBits) PSD_RED(kMaskBits, true);
  else if (mask == kMaskY && a.dr) PSD_RED(kMaskY, true);
  else if (mask == kMaskY) PSD_RED(kMaskY, false);
  else if (mask == kMaskX && a.dr) PSD_RED(kMaskX, true);
  else if (mask == kMaskX) PSD_RED(kMaskX, false);
  else if (a.dr) PSD_RED(kMaskNone, true);
  else PSD_RED(kMaskNone, false);
#undef PSD_RED
  if (a.reduce_only) return hipGetLastError();
  if (a.dq && (!a.dqmx || a.C % 32 != 0)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((a.C + kFinCh - 1) / kFinCh), dim3(256), 0, st, a.part, gx,
                     FinBwd{a.M, a.C, a.gamma, a.save_mean, a.save_invstd, a.dgamma, a.dbeta, a.coef});
  if (a.coef_only) return hipGetLastError();  // coefficients for the consumer's BN-backward fold
  const int64_t nvec = a.M * (a.C / 8);
  const ElemLaunch el = elem_launch(nvec, a.C);
#define PSD_EL(MODE, G, G2)                                                                          \
  if (a.dq) elemt_launch<MODE, true>(el, G, G2, a.y, a.ss, a.x, a.coef, a.dx, nvec, a.C, a.dq, a.dqmx, st); \
  else elemt_launch<MODE, false>(el, G, G2, a.y, a.ss, a.x, a.coef, a.dx, nvec, a.C, nullptr, nullptr, st)
  if (a.dr) PSD_EL(2, a.dr, nullptr);
  else if (mask == kMaskY) PSD_EL(1, a.dy, a.dy2);
  else if (mask == kMaskX) PSD_EL(3, a.dy, a.dy2);
  else PSD_EL(0, a.dy, a.dy2);
#undef PSD_EL
  return hipGetLastError();
}

}  // namespace psd
