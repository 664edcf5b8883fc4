// Fused transformer residual block tail for gfx950: y = LayerNorm(x + dropout(h)) forward and the
// matching backward (LN backward + dropout backward + the residual branch's gradient), bf16 in/out,
// fp32 statistics.
//
// Why: BERT-base's 24 post-attention / post-FFN sites ran this as 3 PyTorch kernels forward
// (dropout, add, layer_norm) and 4 backward (layer_norm_grad_input, two gamma/beta partial passes,
// masked_scale) -- ~2.9 ms of an 18 ms step (profiles/bert_base_b64_r1_tuned_kernels.md), each
// re-reading the [tokens, 768] activations. Here forward reads x and h once and writes y plus the
// bf16 sum s (the LN input backward needs); backward reads dy and s once and writes the residual
// gradient dx and the pre-dropout gradient dh.
//
// Layout: one wave (64 lanes) per row of H = 64*E elements, lane l owning columns [l*E, l*E + E)
// (8-byte loads/stores; E % 4 == 0: H = 768 -> E = 12). Row statistics by wave butterfly reductions.
// Dropout keeps element i with probability 1-p from a counter-based hash of (seed, step, i); the
// step is read from device memory (a counter the model bumps on the device every forward), so a
// replayed hipGraph draws new masks every step, and the backward regenerates the same mask.
// gamma/beta gradients: per-lane column partials across the rows a wave visits -> block partials
// [blk][2][H] -> deterministic finalize (fixed order).
#include "common.h"
#include "launchers_ln.h"

namespace psd {

namespace {

__device__ __forceinline__ uint32_t mix32(uint32_t h) {  // murmur3 finalizer
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}

// the lane's E keep flags (common.h drop_keep's mask: 16 bits of one hash per element pair; off is
// even -- a lane's E columns start at an even index -- so each pair's hash is computed once here)
template <int E>
__device__ __forceinline__ void keep_flags(uint32_t key, int64_t off, uint32_t thresh, bool (&kp)[E]) {
  const uint32_t t16 = thresh >> 16;
#pragma unroll
  for (int j = 0; j < E / 2; ++j) {
    const uint32_t hb = drop_pair_bits(key, (uint64_t)(off + 2 * j));
    kp[2 * j] = (hb & 0xffffu) >= t16;
    kp[2 * j + 1] = (hb >> 16) >= t16;
  }
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

template <int E>
__device__ __forceinline__ void load_e(const uint16_t* p, float v[E]) {
#pragma unroll
  for (int i = 0; i < E / 4; ++i) {
    const uint2 w = *reinterpret_cast<const uint2*>(p + 4 * i);
    v[4 * i + 0] = __uint_as_float(w.x << 16);
    v[4 * i + 1] = __uint_as_float(w.x & 0xffff0000u);
    v[4 * i + 2] = __uint_as_float(w.y << 16);
    v[4 * i + 3] = __uint_as_float(w.y & 0xffff0000u);
  }
}

template <int E>
__device__ __forceinline__ void store_e(uint16_t* p, const float v[E]) {
#pragma unroll
  for (int i = 0; i < E / 4; ++i)
    *reinterpret_cast<uint2*>(p + 4 * i) = make_uint2(pack_bf16x2_rne(v[4 * i], v[4 * i + 1]),
                                                      pack_bf16x2_rne(v[4 * i + 2], v[4 * i + 3]));
}

__device__ __forceinline__ uint32_t dropout_key(uint32_t seed, const int64_t* step) {
  return mix32(seed * 0x27d4eb2fu ^ (uint32_t)(step ? *step : 0) * 0x165667b1u);
}

}  // namespace

template <int E>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ h,
                                                     const uint16_t* __restrict__ gamma,
                                                     const uint16_t* __restrict__ beta, uint16_t* __restrict__ y,
                                                     uint16_t* __restrict__ s_out, float* __restrict__ mean_out,
                                                     float* __restrict__ rstd_out, int64_t rows, float eps,
                                                     uint32_t seed, const int64_t* __restrict__ step, uint32_t thresh,
                                                     float scale) {
  constexpr int H = 64 * E;
  const int lane = threadIdx.x & 63;
  const int c0 = lane * E;
  float g[E], b[E];
  load_e<E>(gamma + c0, g);
  load_e<E>(beta + c0, b);
  const uint32_t key = dropout_key(seed, step);
  const int64_t wstride = (int64_t)gridDim.x * (blockDim.x >> 6);
  // software-pipelined as the backward: the next row's x / h loads are issued before this row's
  // reductions (one row per wave in flight left the pass latency-bound)
  int64_t r = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  float nxv[E], nhv[E];
  if (r < rows) {
    load_e<E>(x + r * H + c0, nxv);
    load_e<E>(h + r * H + c0, nhv);
  }
  for (; r < rows; r += wstride) {
    const int64_t off = r * H + c0;
    float xv[E], hv[E];
#pragma unroll
    for (int i = 0; i < E; ++i) {
      xv[i] = nxv[i];
      hv[i] = nhv[i];
    }
    const int64_t rn = r + wstride;
    if (rn < rows) {
      load_e<E>(x + rn * H + c0, nxv);
      load_e<E>(h + rn * H + c0, nhv);
    }
    bool kp[E];
    if (thresh != 0u) keep_flags<E>(key, off, thresh, kp);
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < E; ++i) {
      const float d = (thresh == 0u || kp[i]) ? hv[i] * scale : 0.f;
      xv[i] = bf16_to_f32(f32_to_bf16(xv[i] + d));  // s, rounded as stored (the LN input)
      sum += xv[i];
    }
    const float mean = wave_sum(sum) * (1.f / H);
    float sq = 0.f;
#pragma unroll
    for (int i = 0; i < E; ++i) {
      const float d = xv[i] - mean;
      sq = fmaf(d, d, sq);
    }
    const float rstd = rsqrtf(wave_sum(sq) * (1.f / H) + eps);
    store_e<E>(s_out + off, xv);
#pragma unroll
    for (int i = 0; i < E; ++i) hv[i] = fmaf((xv[i] - mean) * rstd, g[i], b[i]);
    store_e<E>(y + off, hv);
    if (lane == 0) {
      mean_out[r] = mean;
      rstd_out[r] = rstd;
    }
  }
}

// HS: also the column sums of dh (the bias gradient of the Linear that produced h, which then skips
// its own column-sum pass: ops/layernorm.py): a third partial row per block
template <int E, bool HS>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ s,
                                                     const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
                                                     const uint16_t* __restrict__ gamma, uint16_t* __restrict__ dx,
                                                     uint16_t* __restrict__ dh, float* __restrict__ part, int64_t rows,
                                                     uint32_t seed, const int64_t* __restrict__ step, uint32_t thresh,
                                                     float scale) {
  constexpr int H = 64 * E;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c0 = lane * E;
  constexpr int NP = HS ? 3 : 2;
  float g[E], pg[E], pb[E], ph[E];
  load_e<E>(gamma + c0, g);
#pragma unroll
  for (int i = 0; i < E; ++i) pg[i] = pb[i] = ph[i] = 0.f;
  const uint32_t key = dropout_key(seed, step);
  const int64_t wstride = (int64_t)gridDim.x * (blockDim.x >> 6);
  // software-pipelined: the next row's dy / s / stats loads are issued before this row's two wave
  // reductions (one row per wave per iteration otherwise left the loads latency-bound, 2.9 TB/s)
  int64_t r = (int64_t)blockIdx.x * (blockDim.x >> 6) + wv;
  float ndv[E], nsv[E], nmean = 0.f, nrstd = 0.f;
  if (r < rows) {
    load_e<E>(dy + r * H + c0, ndv);
    load_e<E>(s + r * H + c0, nsv);
    nmean = mean_in[r];
    nrstd = rstd_in[r];
  }
  for (; r < rows; r += wstride) {
    const int64_t off = r * H + c0;
    float dv[E], sv[E];
#pragma unroll
    for (int i = 0; i < E; ++i) {
      dv[i] = ndv[i];
      sv[i] = nsv[i];
    }
    const float mean = nmean, rstd = nrstd;
    const int64_t rn = r + wstride;
    if (rn < rows) {
      load_e<E>(dy + rn * H + c0, ndv);
      load_e<E>(s + rn * H + c0, nsv);
      nmean = mean_in[rn];
      nrstd = rstd_in[rn];
    }
    float a = 0.f, bsum = 0.f;
#pragma unroll
    for (int i = 0; i < E; ++i) {
      sv[i] = (sv[i] - mean) * rstd;  // xhat
      pg[i] = fmaf(dv[i], sv[i], pg[i]);
      pb[i] += dv[i];
      dv[i] *= g[i];  // dxhat
      a += dv[i];
      bsum = fmaf(dv[i], sv[i], bsum);
    }
    a = wave_sum(a) * (1.f / H);
    bsum = wave_sum(bsum) * (1.f / H);
#pragma unroll
    for (int i = 0; i < E; ++i) dv[i] = rstd * (dv[i] - a - sv[i] * bsum);  // d s
    store_e<E>(dx + off, dv);
    bool kp[E];
    if (thresh != 0u) keep_flags<E>(key, off, thresh, kp);
#pragma unroll
    for (int i = 0; i < E; ++i) {
      dv[i] = (thresh == 0u || kp[i]) ? dv[i] * scale : 0.f;
      if constexpr (HS) ph[i] += dv[i];
    }
    store_e<E>(dh + off, dv);
  }
  // block partials of dgamma / dbeta (/ the dh column sums): [blk][NP][H], waves summed in a fixed order
  __shared__ float red[4][NP][H];
#pragma unroll
  for (int i = 0; i < E; ++i) {
    red[wv][0][c0 + i] = pg[i];
    red[wv][1][c0 + i] = pb[i];
    if constexpr (HS) red[wv][2][c0 + i] = ph[i];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < NP * H; c += blockDim.x) {
    const int which = c / H, col = c - which * H;
    part[((int64_t)blockIdx.x * NP + which) * H + col] =
        (red[0][which][col] + red[1][which][col]) + (red[2][which][col] + red[3][which][col]);
  }
}

// dgamma/dbeta[c] = sum over blocks of part[blk][which][c] -> bf16 (into the PS sink). Block =
// 32 outputs x 8 partial-row lanes, combined in a fixed order (deterministic); one lane per output
// walking all 256 partials was latency-bound at ~43 us.
__global__ __launch_bounds__(256) void ln_param_grad_kernel(const float* __restrict__ part, int nblk, int H, int NP,
                                                            uint16_t* __restrict__ dgamma, uint16_t* __restrict__ dbeta,
                                                            uint16_t* __restrict__ dhsum) {
  const int cl = threadIdx.x & 31, rl = threadIdx.x >> 5;
  const int t = blockIdx.x * 32 + cl;  // t = which * H + col
  float s0 = 0.f;
  if (t < NP * H) {
    const int which = t / H, col = t - which * H;
    float s4[4] = {0.f, 0.f, 0.f, 0.f};  // independent loads: nblk/32 round trips, not nblk/8
    int b = rl;
    for (; b + 24 < nblk; b += 32)
#pragma unroll
      for (int u = 0; u < 4; ++u) s4[u] += part[((int64_t)(b + 8 * u) * NP + which) * H + col];
    for (; b < nblk; b += 8) s4[0] += part[((int64_t)b * NP + which) * H + col];
    s0 = (s4[0] + s4[1]) + (s4[2] + s4[3]);
  }
  __shared__ float red[8][33];
  red[rl][cl] = s0;
  __syncthreads();
  if (rl != 0 || t >= NP * H) return;
#pragma unroll
  for (int r = 1; r < 8; ++r) s0 += red[r][cl];
  const int which = t / H, col = t - which * H;
  if (which == 0) dgamma[col] = f32_to_bf16(s0);
  else if (which == 1) dbeta[col] = f32_to_bf16(s0);
  else dhsum[(which - 2) * H + col] = f32_to_bf16(s0);  // the branch bias / the token-type rows
}

// ------------------------------------------------------------------ BERT embedding tail
// y = dropout(LayerNorm(W[id] + P[r % S] + T[type])): PyTorch ran it as three gathers, two adds, a
// layer_norm and a dropout forward (~0.22 ms of a BERT-base b256 step) and a dropout backward, the
// layer_norm backward (three kernels), the position table's broadcast-sum backward and the token-type
// one-hot GEMM backward (~0.26 ms; profiles/r6/bert_base_b256_r6d_kernels.md). Here one pass each way:
// forward gathers the three rows of each token straight from the tables (one wave per token row, the
// next row's gathers issued before this row's reductions) and writes y and the row statistics;
// backward re-gathers the rows (nothing but the statistics is saved: the embedding sum is recomputed
// exactly, in the same fp32 order), applies the dropout mask, runs the LN backward and writes the
// gradient of the embedding sum (the word table's sorted deterministic scatter and the position
// table's batch sum take it, ops/embedding.py) plus block partials of dgamma, dbeta and -- for the
// usual <= 2 token types -- each type row's gradient, finalized by ln_param_grad_kernel.
namespace {
template <int E>
struct EmbRows {
  float w[E], p[E], t[E];
  int ty;
};

// a row's ids, loaded one row ahead of its gathers (a gather right behind its own id load waits a
// full memory round trip before it can issue)
struct EmbIds {
  int64_t id, ty;
};
__device__ __forceinline__ EmbIds emb_ids(const EmbLnArgs& a, int64_t r) {
  EmbIds o{-1, -1};
  if (r < a.rows) {
    o.id = a.ids[r];
    o.ty = a.types ? a.types[r] : 0;
  }
  return o;
}

template <int E>
__device__ __forceinline__ void emb_fetch(const EmbLnArgs& a, int64_t r, EmbIds ids, int c0, EmbRows<E>& o) {
  constexpr int H = 64 * E;
  const int64_t id = ids.id;
  const int64_t ty = ids.ty;
  const int64_t s = r % a.S;
  o.ty = (ty >= 0 && ty < a.NT) ? (int)ty : -1;
  if (id >= 0 && id < a.V) {
    load_e<E>(a.W + id * H + c0, o.w);
  } else {
#pragma unroll
    for (int i = 0; i < E; ++i) o.w[i] = 0.f;
  }
  load_e<E>(a.P + s * H + c0, o.p);
  if (o.ty >= 0) {
    load_e<E>(a.T + (int64_t)o.ty * H + c0, o.t);
  } else {
#pragma unroll
    for (int i = 0; i < E; ++i) o.t[i] = 0.f;
  }
}
}  // namespace

template <int E>
__global__ __launch_bounds__(256) void emb_ln_fwd_kernel(EmbLnArgs a, uint32_t thresh, float scale) {
  constexpr int H = 64 * E;
  const int lane = threadIdx.x & 63;
  const int c0 = lane * E;
  float g[E], b[E];
  load_e<E>(a.gamma + c0, g);
  load_e<E>(a.beta + c0, b);
  const uint32_t key = dropout_key(a.seed, a.step);
  const int64_t wstride = (int64_t)gridDim.x * (blockDim.x >> 6);
  int64_t r = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  EmbRows<E> nx;
  if (r < a.rows) emb_fetch<E>(a, r, emb_ids(a, r), c0, nx);
  EmbIds nid = emb_ids(a, r + wstride);
  for (; r < a.rows; r += wstride) {
    const int64_t off = r * H + c0;
    float xv[E];
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < E; ++i) {
      xv[i] = (nx.w[i] + nx.p[i]) + nx.t[i];
      sum += xv[i];
    }
    const int64_t rn = r + wstride;
    if (rn < a.rows) {
      emb_fetch<E>(a, rn, nid, c0, nx);
      nid = emb_ids(a, rn + wstride);
    }
    const float mean = wave_sum(sum) * (1.f / H);
    float sq = 0.f;
#pragma unroll
    for (int i = 0; i < E; ++i) {
      const float d = xv[i] - mean;
      sq = fmaf(d, d, sq);
    }
    const float rstd = rsqrtf(wave_sum(sq) * (1.f / H) + a.eps);
    bool kp[E];
    if (thresh != 0u) keep_flags<E>(key, off, thresh, kp);
#pragma unroll
    for (int i = 0; i < E; ++i) {
      const float yv = fmaf((xv[i] - mean) * rstd, g[i], b[i]);
      xv[i] = (thresh == 0u) ? yv : (kp[i] ? yv * scale : 0.f);
    }
    store_e<E>(a.y + off, xv);
    if (lane == 0) {
      a.mean[r] = mean;
      a.rstd[r] = rstd;
    }
  }
}

template <int E, int NT>
__global__ __launch_bounds__(256) void emb_ln_bwd_kernel(EmbLnArgs a, uint32_t thresh, float scale) {
  constexpr int H = 64 * E;
  constexpr int NPART = 2 + NT;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c0 = lane * E;
  float g[E], pg[E], pb[E], pt[NT > 0 ? NT : 1][E];
  load_e<E>(a.gamma + c0, g);
#pragma unroll
  for (int i = 0; i < E; ++i) {
    pg[i] = pb[i] = 0.f;
#pragma unroll
    for (int k = 0; k < (NT > 0 ? NT : 1); ++k) pt[k][i] = 0.f;
  }
  const uint32_t key = dropout_key(a.seed, a.step);
  const int64_t wstride = (int64_t)gridDim.x * (blockDim.x >> 6);
  int64_t r = (int64_t)blockIdx.x * (blockDim.x >> 6) + wv;
  EmbRows<E> nx;
  float ndv[E], nmean = 0.f, nrstd = 0.f;
  EmbIds nid = emb_ids(a, r + wstride);
  if (r < a.rows) {
    emb_fetch<E>(a, r, emb_ids(a, r), c0, nx);
    load_e<E>(a.dy + r * H + c0, ndv);
    nmean = a.mean[r];
    nrstd = a.rstd[r];
  }
  for (; r < a.rows; r += wstride) {
    const int64_t off = r * H + c0;
    float xh[E], dv[E];
    const float mean = nmean, rstd = nrstd;
    const int ty = nx.ty;
#pragma unroll
    for (int i = 0; i < E; ++i) {
      xh[i] = ((nx.w[i] + nx.p[i]) + nx.t[i] - mean) * rstd;  // the forward's sum, same order
      dv[i] = ndv[i];
    }
    const int64_t rn = r + wstride;
    if (rn < a.rows) {
      emb_fetch<E>(a, rn, nid, c0, nx);
      nid = emb_ids(a, rn + wstride);
      load_e<E>(a.dy + rn * H + c0, ndv);
      nmean = a.mean[rn];
      nrstd = a.rstd[rn];
    }
    bool kp[E];
    if (thresh != 0u) keep_flags<E>(key, off, thresh, kp);
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < E; ++i) {
      if (thresh != 0u) dv[i] = kp[i] ? dv[i] * scale : 0.f;  // gradient at the LN output
      pg[i] = fmaf(dv[i], xh[i], pg[i]);
      pb[i] += dv[i];
      dv[i] *= g[i];
      s1 += dv[i];
      s2 = fmaf(dv[i], xh[i], s2);
    }
    s1 = wave_sum(s1) * (1.f / H);
    s2 = wave_sum(s2) * (1.f / H);
#pragma unroll
    for (int i = 0; i < E; ++i) dv[i] = rstd * (dv[i] - s1 - xh[i] * s2);
    store_e<E>(a.dx + off, dv);
    if constexpr (NT > 0) {
#pragma unroll
      for (int k = 0; k < NT; ++k)
        if (ty == k) {
#pragma unroll
          for (int i = 0; i < E; ++i) pt[k][i] += dv[i];
        }
    }
  }
  __shared__ float red[4][NPART][H];
#pragma unroll
  for (int i = 0; i < E; ++i) {
    red[wv][0][c0 + i] = pg[i];
    red[wv][1][c0 + i] = pb[i];
#pragma unroll
    for (int k = 0; k < NT; ++k) red[wv][2 + k][c0 + i] = pt[k][i];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < NPART * H; c += blockDim.x) {
    const int which = c / H, col = c - which * H;
    a.part[((int64_t)blockIdx.x * NPART + which) * H + col] =
        (red[0][which][col] + red[1][which][col]) + (red[2][which][col] + red[3][which][col]);
  }
}

int emb_ln_bwd_blocks(int64_t rows) {
  const int64_t want = (rows + 4 * 8 - 1) / (4 * 8);
  return (int)(want < 1 ? 1 : (want > 512 ? 512 : want));
}

int ln_bwd_blocks(int64_t rows) {
  const int64_t want = (rows + 4 * 8 - 1) / (4 * 8);  // >= 8 rows per wave, <= 2 blocks per CU
  return (int)(want < 1 ? 1 : (want > 512 ? 512 : want));
}

bool ln_supported(int H) { return H == 768 || H == 1024; }

static uint32_t keep_thresh(float p) {
  if (p <= 0.f) return 0u;
  const double t = (double)p * 4294967296.0;
  return t >= 4294967295.0 ? 4294967295u : (uint32_t)t;
}

hipError_t launch_ln_fwd(const LnArgs& a, hipStream_t st) {
  if (!ln_supported(a.H)) return hipErrorInvalidValue;
  const int64_t blocks64 = (a.rows + 3) / 4;
  const int blocks = (int)(blocks64 > 2048 ? 2048 : (blocks64 < 1 ? 1 : blocks64));
  const uint32_t th = keep_thresh(a.p);
  const float sc = a.p > 0.f ? 1.f / (1.f - a.p) : 1.f;
#define PSD_LNF(E)                                                                                                  \
  hipLaunchKernelGGL(ln_fwd_kernel<E>, dim3(blocks), dim3(256), 0, st, a.x, a.h, a.gamma, a.beta, a.y, a.s, a.mean, \
                     a.rstd, a.rows, a.eps, a.seed, a.step, th, sc)
  if (a.H == 768) PSD_LNF(12);
  else PSD_LNF(16);
#undef PSD_LNF
  return hipGetLastError();
}

hipError_t launch_ln_bwd(const LnArgs& a, hipStream_t st) {
  if (!ln_supported(a.H)) return hipErrorInvalidValue;
  const int blocks = ln_bwd_blocks(a.rows);
  const uint32_t th = keep_thresh(a.p);
  const float sc = a.p > 0.f ? 1.f / (1.f - a.p) : 1.f;
#define PSD_LNB(E, HS)                                                                                              \
  hipLaunchKernelGGL((ln_bwd_kernel<E, HS>), dim3(blocks), dim3(256), 0, st, a.dy, a.s, a.mean, a.rstd, a.gamma, \
                     a.dx, a.dh, a.part, a.rows, a.seed, a.step, th, sc)
  const bool hs = a.dhsum != nullptr;
  if (a.H == 768) {
    if (hs) PSD_LNB(12, true);
    else PSD_LNB(12, false);
  } else {
    if (hs) PSD_LNB(16, true);
    else PSD_LNB(16, false);
  }
#undef PSD_LNB
  const int np = hs ? 3 : 2;
  hipLaunchKernelGGL(ln_param_grad_kernel, dim3((np * a.H + 31) / 32), dim3(256), 0, st, a.part, blocks, a.H, np,
                     a.dgamma, a.dbeta, a.dhsum);
  return hipGetLastError();
}

hipError_t launch_emb_ln_fwd(const EmbLnArgs& a, hipStream_t st) {
  if (a.H != 768 || a.S <= 0 || a.NT < 0 || a.rows < 0) return hipErrorInvalidValue;
  if (a.rows == 0) return hipSuccess;
  // one row per wave up to 8192 workgroups: a gather waits on its id load, so the pass wants many
  // rows in flight (at the LayerNorm kernels' 2048-workgroup cap it ran at ~1.6 TB/s)
  const int64_t blocks64 = (a.rows + 3) / 4;
  const int blocks = (int)(blocks64 > 8192 ? 8192 : blocks64);
  const uint32_t th = keep_thresh(a.p);
  const float sc = a.p > 0.f ? 1.f / (1.f - a.p) : 1.f;
  hipLaunchKernelGGL(emb_ln_fwd_kernel<12>, dim3(blocks), dim3(256), 0, st, a, th, sc);
  return hipGetLastError();
}

hipError_t launch_emb_ln_bwd(const EmbLnArgs& a, hipStream_t st) {
  if (a.H != 768 || a.S <= 0 || a.NT < 0 || a.rows < 0) return hipErrorInvalidValue;
  const int nt = a.dT ? a.NT : 0;  // type-row gradients fused for NT <= 2 only
  if (nt > 2) return hipErrorInvalidValue;
  if (a.rows == 0) return hipSuccess;
  const int blocks = emb_ln_bwd_blocks(a.rows);
  const uint32_t th = keep_thresh(a.p);
  const float sc = a.p > 0.f ? 1.f / (1.f - a.p) : 1.f;
  if (nt == 0) hipLaunchKernelGGL((emb_ln_bwd_kernel<12, 0>), dim3(blocks), dim3(256), 0, st, a, th, sc);
  else if (nt == 1) hipLaunchKernelGGL((emb_ln_bwd_kernel<12, 1>), dim3(blocks), dim3(256), 0, st, a, th, sc);
  else hipLaunchKernelGGL((emb_ln_bwd_kernel<12, 2>), dim3(blocks), dim3(256), 0, st, a, th, sc);
  const int np = 2 + nt;
  hipLaunchKernelGGL(ln_param_grad_kernel, dim3((np * a.H + 31) / 32), dim3(256), 0, st, a.part, blocks, a.H, np,
                     a.dgamma, a.dbeta, a.dT);
  return hipGetLastError();
}

}  // namespace psd
