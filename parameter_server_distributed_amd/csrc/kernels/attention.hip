// Fused multi-head self-attention for short sequences (BERT pre-training, S <= 128, head dim 64) on
// gfx950, forward and backward, reading the packed QKV projection output [B, S, 3, H, 64] in place and
// writing O as [B, S, H, 64] (the output projection's input, no transpose) and dQKV in the packed
// layout (the QKV projection's dgrad input, no stack/cat).
//
// One workgroup per (batch, head), S/32 waves; the whole head (Q, K, V, dO: S x 64 bf16 each) lives
// in LDS and every product is a v_mfma_f32_32x32x16_bf16:
//   forward   S^T = K Q^T (keys x queries: the softmax reduction runs over a lane's own registers
//             plus one lane^32 exchange), P = softmax, dropout, then O = P V with P staged through
//             LDS; the row log-sum-exp is saved for backward.
//   backward  wave w owns key block w: S^T and dP^T = V dO^T recomputed, dS = P (dP - rowsum(dO.O)),
//             dV = Pd^T dO and dK = dS^T Q from transposed LDS reads (ds_read_b64_tr_b16); then
//             wave w owns query block w: dQ = dS K.
// Dropout keeps (b, h, q, key) from the same counter hash as the fused LayerNorm (seed, device step
// counter), so the mask is regenerated in backward and a replayed hipGraph draws fresh masks.
//
// Replaces what the reference's stub gradient (src/worker.cpp:316-329) stands in for: the model's
// real forward/backward; the attention is BERT's (BASELINE config 4).
#include <algorithm>

#include "common.h"
#include "launchers_attn.h"

namespace psd {

namespace {

typedef __bf16 abf16x8 __attribute__((ext_vector_type(8)));
typedef short as16x4 __attribute__((ext_vector_type(4)));
typedef float af32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) as16x4 alds_s16x4;

constexpr int D = 64;                 // head dim
constexpr int LDT = D + 8;            // Q/K/V/dO tile row stride (elements): 144 B

__device__ __forceinline__ uint32_t amix32(uint32_t h) {  // murmur3 finalizer (as layernorm.hip)
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}
// (common.h drop_keep: one hash per element pair, 16 bits each; fwd and bwd index elements alike)
// keep flags of the element pair (idx, idx + 1), idx even, from ONE hash -- drop_keep's mask bit for bit.
// (Calling drop_keep per element hashed every pair twice: dropout cost the forward 57 % of its
// time, 48.6 -> 76.2 us per BERT layer, tools/attn_bench.py.)
__device__ __forceinline__ void akeep2(uint32_t key, uint64_t idx, uint32_t thresh, bool& k0, bool& k1) {
  const uint32_t h = drop_pair_bits(key, idx);
  k0 = (h & 0xffffu) >= (thresh >> 16);
  k1 = (h >> 16) >= (thresh >> 16);
}
__device__ __forceinline__ uint32_t attn_key(uint32_t seed, const int64_t* step) {
  return amix32(seed * 0x27d4eb2fu ^ (uint32_t)(step ? *step : 0) * 0x165667b1u);
}

// A/B fragment whose 8 k-values are contiguous in LDS: lane -> row r0 + lane%32, k = k0 + 8*(lane/32) + e
__device__ __forceinline__ abf16x8 rowfrag(const uint8_t* base, int stride_b, int r0, int k0) {
  const int lane = threadIdx.x & 63;
  const u32x4 w = *reinterpret_cast<const u32x4*>(base + (r0 + (lane & 31)) * stride_b + (k0 + 8 * (lane >> 5)) * 2);
  return __builtin_bit_cast(abf16x8, w);
}
// Same fragment from a [k][col] tile (col contiguous): ds_read_b64_tr_b16 transposes within 16 lanes.
// lane -> col c0 + lane%32, k = k0 + 8*(lane/32) + e
__device__ __forceinline__ abf16x8 trfrag(const uint8_t* base, int stride_b, int k0, int c0) {
  const int lane = threadIdx.x & 63;
  const int G = lane >> 4, i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
  const int k = k0 + 8 * (G >> 1) + q;
  const int col = c0 + 16 * (G & 1) + 4 * p;
  const as16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((alds_s16x4*)(base + k * stride_b + col * 2));
  const as16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((alds_s16x4*)(base + (k + 4) * stride_b + col * 2));
  as16x4 both[2] = {lo, hi};
  return __builtin_bit_cast(abf16x8, both);
}

// trfrag with the key order of a 32x32 accumulator's rows: k-slot e of lane half hh is key
// kb + 8*(e/4) + 4*hh + e%4 -- exactly the keys acc_row(8*ks2 + e, hh) a lane holds in registers, so the
// softmax probabilities feed the P V MFMA as its B operand straight from the S^T accumulators
// (the k sum is order-free; A = V^T is read in the same permuted order)
__device__ __forceinline__ abf16x8 trfrag_accrows(const uint8_t* base, int stride_b, int kb, int c0) {
  const int lane = threadIdx.x & 63;
  const int G = lane >> 4, i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
  const int k = kb + 4 * (G >> 1) + q;
  const int col = c0 + 16 * (G & 1) + 4 * p;
  const as16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((alds_s16x4*)(base + k * stride_b + col * 2));
  const as16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((alds_s16x4*)(base + (k + 8) * stride_b + col * 2));
  as16x4 both[2] = {lo, hi};
  return __builtin_bit_cast(abf16x8, both);
}

__device__ __forceinline__ af32x16 mfma(abf16x8 a, abf16x8 b, af32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ af32x16 zero16() {
  af32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}
// accumulator element i of a 32x32 tile: row (i&3) + 8*(i>>2) + 4*(lane/32), col lane%32
__device__ __forceinline__ int acc_row(int i, int hh) { return (i & 3) + 8 * (i >> 2) + 4 * hh; }

// rows [0, S) of a [.., S, 3, H, 64] (or [.., S, H, 64]) tensor -> LDS tile [S][LDT]
__device__ __forceinline__ void stage_rows(uint8_t* lds, const uint16_t* src, int64_t row_stride, int S) {
  for (int c = threadIdx.x; c < S * 8; c += blockDim.x) {
    const int r = c >> 3, ch = c & 7;
    *reinterpret_cast<u32x4*>(lds + r * LDT * 2 + ch * 16) =
        *reinterpret_cast<const u32x4*>(src + (int64_t)r * row_stride + ch * 8);
  }
}

}  // namespace

static int attn_cus() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0)
      n = 256;
  }
  return n;
}

// Persistent (as many workgroups per CU as registers and the 36 KiB K + V image allow): the next
// (batch, head) item's K, V rows and this lane's Q fragments are loaded into registers while the
// current item is computed. The probabilities never leave registers (P V takes them as its B
// operand in accumulator-row key order) and O leaves in 8-B pieces.
template <int NW>
__global__ __launch_bounds__(64 * NW) void attn_fwd_kernel(AttnArgs a) {
  constexpr int S = 32 * NW;
  constexpr int NT = 64 * NW;
  constexpr int CH = S * 8 / NT;  // 16-B chunks per lane per tile (= 4)
  static_assert(CH * NT == S * 8, "chunking");
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* Ks = smem;
  uint8_t* Vs = Ks + S * LDT * 2;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hh = lane >> 5;
  const int HD = a.H * D;
  const int64_t qkv_rs = 3 * (int64_t)HD;
  const int nitems = a.B * a.H;
  const int q0 = 32 * w, q = q0 + (lane & 31);
  const float sl = a.scale * 1.4426950408889634f;
  const uint32_t key = attn_key(a.seed, a.step);
  const bool drop = a.thresh != 0u;

  u32x4 pk[CH], pv[CH], pq[4];
  auto fetch = [&](int bh) {
    const int b = bh / a.H, h = bh % a.H;
    const uint16_t* base = a.qkv + (int64_t)b * S * qkv_rs + h * D;
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int c = threadIdx.x + i * NT, r = c >> 3, ch = c & 7;
      pk[i] = *reinterpret_cast<const u32x4*>(base + HD + (int64_t)r * qkv_rs + ch * 8);
      pv[i] = *reinterpret_cast<const u32x4*>(base + 2 * HD + (int64_t)r * qkv_rs + ch * 8);
    }
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) pq[ks] = *reinterpret_cast<const u32x4*>(base + (int64_t)q * qkv_rs + 16 * ks + 8 * hh);
  };
  if ((int)blockIdx.x < nitems) fetch(blockIdx.x);

  for (int bh = blockIdx.x; bh < nitems; bh += gridDim.x) {
    const int b = bh / a.H, h = bh % a.H;
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int c = threadIdx.x + i * NT, r = c >> 3, ch = c & 7;
      *reinterpret_cast<u32x4*>(Ks + r * LDT * 2 + ch * 16) = pk[i];
      *reinterpret_cast<u32x4*>(Vs + r * LDT * 2 + ch * 16) = pv[i];
    }
    abf16x8 qf[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) qf[ks] = __builtin_bit_cast(abf16x8, pq[ks]);
    __syncthreads();
    if (bh + (int)gridDim.x < nitems) fetch(bh + gridDim.x);  // in flight during this item

    af32x16 sc[NW];  // S^T tiles: lane owns query q, keys 32j + acc_row(i)
#pragma unroll
    for (int j = 0; j < NW; ++j) {
      sc[j] = zero16();
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) sc[j] = mfma(rowfrag(Ks, LDT * 2, 32 * j, 16 * ks), qf[ks], sc[j]);
    }
    float m = -INFINITY;
#pragma unroll
    for (int j = 0; j < NW; ++j)
#pragma unroll
      for (int i = 0; i < 16; ++i) m = fmaxf(m, sc[j][i]);
    m = fmaxf(m, __shfl_xor(m, 32));
    float l = 0.f;
#pragma unroll
    for (int j = 0; j < NW; ++j)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        sc[j][i] = exp2f((sc[j][i] - m) * sl);
        l += sc[j][i];
      }
    l += __shfl_xor(l, 32);
    if (hh == 0) a.lse[(int64_t)bh * S + q] = m * a.scale + logf(l);
    const float inv = 1.f / l;
    const uint64_t rowidx = ((uint64_t)bh * S + q) * S;
    // O^T[d][q] = sum_key V^T[d][key] P^T[key][q]: B = this lane's probabilities (query q, keys in
    // accumulator-row order), A = V^T read in that order; no P round trip through LDS
    af32x16 ot[2] = {zero16(), zero16()};
#pragma unroll
    for (int j = 0; j < NW; ++j)
#pragma unroll
      for (int ks2 = 0; ks2 < 2; ++ks2) {
        float v[8];
        bool kp[8];
        if (drop) {  // elements e, e + 1 (e even) are keys kk, kk + 1 with kk even: one hash per pair
#pragma unroll
          for (int e = 0; e < 8; e += 2) akeep2(key, rowidx + 32 * j + acc_row(8 * ks2 + e, hh), a.thresh, kp[e], kp[e + 1]);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          v[e] = sc[j][8 * ks2 + e] * inv;
          if (drop) v[e] = kp[e] ? v[e] * a.rescale : 0.f;
        }
        const abf16x8 pb = __builtin_bit_cast(
            abf16x8, u32x4{pack_bf16x2_rne(v[0], v[1]), pack_bf16x2_rne(v[2], v[3]), pack_bf16x2_rne(v[4], v[5]),
                           pack_bf16x2_rne(v[6], v[7])});
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) ot[dt] = mfma(trfrag_accrows(Vs, LDT * 2, 32 * j + 16 * ks2, 32 * dt), pb, ot[dt]);
      }
    // lane: query q, d = 32 dt + acc_row(i): 4 consecutive d per 4 accumulators -> 8-B stores
    uint16_t* out = a.o + ((int64_t)b * S + q) * HD + h * D;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<uint2*>(out + 32 * dt + 8 * g + 4 * hh) =
            make_uint2(pack_bf16x2_rne(ot[dt][4 * g], ot[dt][4 * g + 1]), pack_bf16x2_rne(ot[dt][4 * g + 2], ot[dt][4 * g + 3]));
    __syncthreads();  // K, V of this item read by every wave before the next item's stores
  }
}

// 2*NW waves: the LDS image (Q, K, V, dO, Pd, dS: ~144 KiB at S = 128) allows one workgroup per
// CU, so a 32-row block is split between two waves (query blocks / head-dim halves) to keep two
// waves per SIMD: at one wave per SIMD (the first version) nothing hid the LDS and MFMA latencies
// and the kernel ran at 3.5x its HBM time (profiles/bert_base_b256_r2_kernels.md).
// Persistent: one workgroup per CU walks (batch, head) items; the next item's Q, K, V, dO, O rows
// and lse are loaded into registers (2 chunks of 16 B per tile per lane) while the current item is
// computed, so the HBM time of one item hides behind the MFMA/LDS work of the previous one (a
// workgroup per item loaded, synchronised and computed strictly in turn: 189 us per BERT layer,
// ~2 TB/s, profiles/bert_base_b256_r4 profile).
template <int NW>
__global__ __launch_bounds__(128 * NW) void attn_bwd_kernel(AttnArgs a) {
  constexpr int S = 32 * NW, LDP = S + 8;
  constexpr int NT = 128 * NW;
  constexpr int CH = S * 8 / NT;  // 16-B chunks per lane per tile (= 2)
  static_assert(CH * NT == S * 8, "chunking");
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* Qs = smem;
  uint8_t* Ks = Qs + S * LDT * 2;
  uint8_t* Vs = Ks + S * LDT * 2;
  uint8_t* dOs = Vs + S * LDT * 2;
  uint8_t* Pd = dOs + S * LDT * 2;  // dropped, rescaled probabilities [q][key]
  uint8_t* dS = Pd + S * LDP * 2;   // dS = P (dP - D) [q][key]
  float* lse_s = reinterpret_cast<float*>(dS + S * LDP * 2);
  float* D_s = lse_s + S;
  float* cs_s = D_s + S;  // [NW][3][64] per-key/query-block column sums of dq, dk, dv (bpart)

  const int lane = threadIdx.x & 63, hh = lane >> 5;
  const int w = threadIdx.x >> 7, sub = (threadIdx.x >> 6) & 1;  // 32-row block, half of its work
  const int HD = a.H * D;
  const int64_t qkv_rs = 3 * (int64_t)HD;
  const int nitems = a.B * a.H;
  const uint32_t key = attn_key(a.seed, a.step);
  const bool drop = a.thresh != 0u;
  const float sl = a.scale * 1.4426950408889634f;

  // register prefetch of one item: tile t (Q, K, V, dO, O) chunk i = row c >> 3, 16-B column c & 7
  u32x4 pf[5][CH];
  float plse = 0.f;
  auto fetch = [&](int bh) {
    const int b = bh / a.H, h = bh % a.H;
    const uint16_t* base = a.qkv + (int64_t)b * S * qkv_rs + h * D;
    const int64_t ob = (int64_t)b * S * HD + h * D;
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int c = threadIdx.x + i * NT, r = c >> 3, ch = c & 7;
#pragma unroll
      for (int t = 0; t < 3; ++t)
        pf[t][i] = *reinterpret_cast<const u32x4*>(base + t * HD + (int64_t)r * qkv_rs + ch * 8);
      pf[3][i] = *reinterpret_cast<const u32x4*>(a.dout + ob + (int64_t)r * HD + ch * 8);
      pf[4][i] = *reinterpret_cast<const u32x4*>(a.o + ob + (int64_t)r * HD + ch * 8);
    }
    if (threadIdx.x < S) plse = a.lse[(int64_t)bh * S + threadIdx.x];
  };
  if ((int)blockIdx.x < nitems) fetch(blockIdx.x);

  for (int bh = blockIdx.x; bh < nitems; bh += gridDim.x) {
    const int b = bh / a.H, h = bh % a.H;
    // the prefetched item -> LDS; D[q] = sum_d dO[q, d] O[q, d] (8 lanes per row)
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int c = threadIdx.x + i * NT, r = c >> 3, ch = c & 7;
      uint8_t* tiles[4] = {Qs, Ks, Vs, dOs};
#pragma unroll
      for (int t = 0; t < 4; ++t) *reinterpret_cast<u32x4*>(tiles[t] + r * LDT * 2 + ch * 16) = pf[t][i];
      const uint32_t xw[4] = {pf[3][i].x, pf[3][i].y, pf[3][i].z, pf[3][i].w};
      const uint32_t yw[4] = {pf[4][i].x, pf[4][i].y, pf[4][i].z, pf[4][i].w};
      float s = 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        s = fmaf(__uint_as_float(xw[e] << 16), __uint_as_float(yw[e] << 16), s);
        s = fmaf(__uint_as_float(xw[e] & 0xffff0000u), __uint_as_float(yw[e] & 0xffff0000u), s);
      }
      s += __shfl_xor(s, 1);
      s += __shfl_xor(s, 2);
      s += __shfl_xor(s, 4);
      if (ch == 0) D_s[r] = s;
    }
    if (threadIdx.x < S) lse_s[threadIdx.x] = plse;
    __syncthreads();
    if (bh + (int)gridDim.x < nitems) fetch(bh + gridDim.x);  // in flight during this item's phases

    // phase 1: waves (w, sub) own keys k0..k0+31; recompute S^T and dP^T against the query blocks
    // t = sub, sub + 2, ...
    const int k0 = 32 * w;
    abf16x8 kf[4], vf[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      kf[ks] = rowfrag(Ks, LDT * 2, k0, 16 * ks);
      vf[ks] = rowfrag(Vs, LDT * 2, k0, 16 * ks);
    }
#pragma unroll
    for (int t = sub; t < NW; t += 2) {
      af32x16 st = zero16(), dpt = zero16();
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        st = mfma(kf[ks], rowfrag(Qs, LDT * 2, 32 * t, 16 * ks), st);
        dpt = mfma(vf[ks], rowfrag(dOs, LDT * 2, 32 * t, 16 * ks), dpt);
      }
      const int q = 32 * t + (lane & 31);
      const float lse2 = lse_s[q] * 1.4426950408889634f, Dq = D_s[q];
      const uint64_t rowidx = ((uint64_t)bh * S + q) * S;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float pv[4], dv[4];
        bool kp[4];
        if (drop) {  // keys k0 + 8g + 4hh + e: pairs (0, 1), (2, 3) share one hash
          akeep2(key, rowidx + k0 + 8 * g + 4 * hh, a.thresh, kp[0], kp[1]);
          akeep2(key, rowidx + k0 + 8 * g + 4 * hh + 2, a.thresh, kp[2], kp[3]);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int i = 4 * g + e;
          const float p = exp2f(st[i] * sl - lse2);
          float pd = p, dp = dpt[i];
          if (drop) {
            pd = kp[e] ? p * a.rescale : 0.f;
            dp = kp[e] ? dp * a.rescale : 0.f;
          }
          pv[e] = pd;
          dv[e] = p * (dp - Dq);
        }
        const int off = q * LDP * 2 + (k0 + 8 * g + 4 * hh) * 2;
        *reinterpret_cast<uint2*>(Pd + off) = make_uint2(pack_bf16x2_rne(pv[0], pv[1]), pack_bf16x2_rne(pv[2], pv[3]));
        *reinterpret_cast<uint2*>(dS + off) = make_uint2(pack_bf16x2_rne(dv[0], dv[1]), pack_bf16x2_rne(dv[2], dv[3]));
      }
    }
    __syncthreads();

    // phase 2: dV[key, d] = sum_q Pd[q, key] dO[q, d];  dK = scale * sum_q dS[q, key] Q[q, d]
    // (wave (w, sub): keys of block w, head dims 32*sub..)
    uint16_t* dq_base = a.dqkv + (int64_t)b * S * qkv_rs + h * D;
    {
      const int dt = sub;
      af32x16 dv = zero16(), dk = zero16();
#pragma unroll
      for (int ks = 0; ks < S / 16; ++ks) {
        dv = mfma(trfrag(Pd, LDP * 2, 16 * ks, k0), trfrag(dOs, LDT * 2, 16 * ks, 32 * dt), dv);
        dk = mfma(trfrag(dS, LDP * 2, 16 * ks, k0), trfrag(Qs, LDT * 2, 16 * ks, 32 * dt), dk);
      }
      const int d = 32 * dt + (lane & 31);
      float sk = 0.f, sv = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int64_t r = (int64_t)(k0 + acc_row(i, hh)) * qkv_rs + d;
        dq_base[r + HD] = f32_to_bf16(dk[i] * a.scale);
        dq_base[r + 2 * HD] = f32_to_bf16(dv[i]);
        sk += dk[i];
        sv += dv[i];
      }
      if (a.bpart) {  // this wave's 32 keys: the two lane halves hold 16 rows each
        sk += __shfl_xor(sk, 32);
        sv += __shfl_xor(sv, 32);
        if (hh == 0) {
          cs_s[(w * 3 + 1) * 64 + d] = sk * a.scale;
          cs_s[(w * 3 + 2) * 64 + d] = sv;
        }
      }
    }
    // phase 3: waves (w, sub) own queries q0..q0+31, head dims 32*sub..: dQ = scale * dS K
    const int q0 = 32 * w;
    {
      const int dt = sub;
      af32x16 dq = zero16();
#pragma unroll
      for (int ks = 0; ks < S / 16; ++ks) dq = mfma(rowfrag(dS, LDP * 2, q0, 16 * ks), trfrag(Ks, LDT * 2, 16 * ks, 32 * dt), dq);
      const int d = 32 * dt + (lane & 31);
      float sq = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        dq_base[(int64_t)(q0 + acc_row(i, hh)) * qkv_rs + d] = f32_to_bf16(dq[i] * a.scale);
        sq += dq[i];
      }
      if (a.bpart) {
        sq += __shfl_xor(sq, 32);
        if (hh == 0) cs_s[(w * 3 + 0) * 64 + d] = sq * a.scale;
      }
    }
    if (a.bpart) {  // the item's column sums in a fixed order over the blocks -> bpart[b][t * HD + h * 64 + d]
      __syncthreads();
      if ((int)threadIdx.x < 3 * 64) {
        const int t = threadIdx.x >> 6, d = threadIdx.x & 63;
        float acc = 0.f;
#pragma unroll
        for (int ww = 0; ww < NW; ++ww) acc += cs_s[(ww * 3 + t) * 64 + d];
        a.bpart[(int64_t)b * 3 * HD + t * HD + h * D + d] = acc;
      }
    }
    __syncthreads();  // every read of this item's LDS done before the next item overwrites it
  }
}


bool attn_supported(int S, int head_dim) { return head_dim == D && S >= 32 && S <= 128 && S % 32 == 0; }

static int fwd_lds(int S) { return 2 * S * LDT * 2; }
static int bwd_lds(int S) { return 4 * S * LDT * 2 + 2 * S * (S + 8) * 2 + 2 * S * 4 + (S / 32) * 3 * 64 * 4; }

template <int NW>
static hipError_t launch_fwd_t(const AttnArgs& a, hipStream_t st) {
  const int lds = fwd_lds(32 * NW);
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_fwd_kernel<NW>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (e != hipSuccess) return e;
  // persistent: the resident workgroups per CU (registers / LDS), each walks items bh, bh + grid, ...
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(&attn_fwd_kernel<NW>), 64 * NW,
                                                   lds) != hipSuccess || per_cu < 1)
    per_cu = 1;
  const int grid = std::min(a.B * a.H, per_cu * attn_cus());
  hipLaunchKernelGGL(attn_fwd_kernel<NW>, dim3(grid), dim3(64 * NW), lds, st, a);
  return hipGetLastError();
}
template <int NW>
static hipError_t launch_bwd_t(const AttnArgs& a, hipStream_t st) {
  const int lds = bwd_lds(32 * NW);
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_bwd_kernel<NW>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (e != hipSuccess) return e;
  // persistent: one workgroup per CU (the LDS image admits one), each walks items bh, bh + grid, ...
  const int grid = std::min(a.B * a.H, attn_cus());
  hipLaunchKernelGGL(attn_bwd_kernel<NW>, dim3(grid), dim3(128 * NW), lds, st, a);
  return hipGetLastError();
}

hipError_t launch_attn_fwd(const AttnArgs& a, hipStream_t st) {
  if (!attn_supported(a.S, D)) return hipErrorInvalidValue;
  switch (a.S / 32) {
    case 1: return launch_fwd_t<1>(a, st);
    case 2: return launch_fwd_t<2>(a, st);
    case 3: return launch_fwd_t<3>(a, st);
    default: return launch_fwd_t<4>(a, st);
  }
}
hipError_t launch_attn_bwd(const AttnArgs& a, hipStream_t st) {
  if (!attn_supported(a.S, D)) return hipErrorInvalidValue;
  switch (a.S / 32) {
    case 1: return launch_bwd_t<1>(a, st);
    case 2: return launch_bwd_t<2>(a, st);
    case 3: return launch_bwd_t<3>(a, st);
    default: return launch_bwd_t<4>(a, st);
  }
}

}  // namespace psd
