// MFMA bf16 GEMM for gfx950: the worker's Linear / 1x1-conv forward and backward.
//
//   C[M,N] = sum_k A(m,k) * B(k,n)          bf16 in, fp32 accumulate (v_mfma_f32_32x32x16_bf16)
//
// Operand storage is a template choice, so all three GEMMs of a layer run without any transpose
// copies:
//   forward   Y  = X  . W^T   A = X  [M][K] (K-major)      B = W  [N][K] (K-major)      "NT"
//   dgrad     dX = dY . W     A = dY [M][K] (K-major)      B = W  [K][N] (N-major)      "NN"
//   wgrad     dW = dY^T . X   A = dY [K][M] (M-major)      B = X  [K][N] (N-major)      "TN", split-K
// K-major tiles are staged in LDS as [rows][64 k] (128-B rows, 16-B chunk XOR-swizzled by row>>1:
// ds_read_b128 fragment reads are bank-conflict-free). M/N-major tiles are staged as [64 k][rows]
// (k-rows, 64-B blocks XOR-swizzled by k&3) and read with the CDNA4 transpose read
// ds_read_b64_tr_b16 (two per fragment), so the MFMA always sees k-contiguous fragments.
//
// Workgroup = 256 lanes = 4 waves in a 2x2 grid; each wave owns TM x TN 32x32 MFMA tiles; BK = 64
// (4 MFMA k-steps per stage). Global -> registers -> LDS staging, double-buffered LDS, the next
// tile's global loads issued before the current tile's MFMAs (one barrier per K-stage).
// Blocks are remapped XCD-aware (bijective, cdna_hip_programming.md T1) so the blocks that share an
// A row-panel land on one XCD's L2.
//
// Epilogues: bf16 output with optional bias (bf16 [N]) and ReLU / GELU(tanh) (GELU also stores
// the pre-activation for backward); or fp32 split-K slabs reduced by gemm_splitk_reduce (which
// can write bf16 straight into the PS flat-gradient buffer).
#include "common.h"
#include "launchers_gemm.h"

#include <cstdlib>

namespace psd {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int BK = 64;

__device__ __forceinline__ int kmaj_off(int row, int kc) {  // byte offset in a [rows][64] tile
  return row * 128 + ((kc ^ ((row >> 1) & 7)) << 4);
}
template <int ROWS>
__device__ __forceinline__ int mnmaj_off(int k, int col) {  // byte offset in a [64][ROWS] tile
  constexpr int mask = ROWS >= 128 ? 3 : (ROWS >= 64 ? 1 : 0);
  return (k * ROWS + (col ^ ((k & mask) << 5))) * 2;
}

__device__ __forceinline__ float gelu_tanh(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  return 0.5f * x * (1.f + tanhf(k0 * (x + k1 * x * x * x)));
}

// Stage loader: each lane moves ROWS*8/256 16-byte chunks global -> registers.
template <int ROWS, bool KMAJ>
struct Stage {
  static constexpr int kChunks = ROWS * 8 / 256;
  u32x4 v[kChunks];

  // KMAJ: src is [ROWS-range rows][K] row-major (ld), tile rows r0.., k0..k0+63
  // !KMAJ: src is [K][ld] with rows contiguous; tile k0..k0+63, cols r0..r0+ROWS-1
  __device__ __forceinline__ void load(const uint16_t* __restrict__ src, int ld, int nrows, int K, int r0, int k0) {
#pragma unroll
    for (int i = 0; i < kChunks; ++i) {
      const int c = threadIdx.x + 256 * i;
      int row, kk;
      bool ok;
      const uint16_t* p;
      if (KMAJ) {
        row = c >> 3;
        kk = (c & 7) * 8;
        ok = (r0 + row < nrows) && (k0 + kk < K);
        p = src + (int64_t)(r0 + row) * ld + k0 + kk;
      } else {
        kk = c / (ROWS / 8);
        row = (c % (ROWS / 8)) * 8;
        ok = (k0 + kk < K) && (r0 + row < nrows);
        p = src + (int64_t)(k0 + kk) * ld + r0 + row;
      }
      v[i] = ok ? *reinterpret_cast<const u32x4*>(p) : u32x4{0u, 0u, 0u, 0u};
    }
  }
  __device__ __forceinline__ void store(uint8_t* lds) const {
#pragma unroll
    for (int i = 0; i < kChunks; ++i) {
      const int c = threadIdx.x + 256 * i;
      int off;
      if (KMAJ)
        off = kmaj_off(c >> 3, c & 7);
      else
        off = mnmaj_off<ROWS>(c / (ROWS / 8), (c % (ROWS / 8)) * 8);
      *reinterpret_cast<u32x4*>(lds + off) = v[i];
    }
  }
};

// Fragment of 32 rows x 16 k for k-step ks (0..3) starting at tile row r0 (lane-relative).
template <int ROWS, bool KMAJ>
__device__ __forceinline__ bf16x8 frag(const uint8_t* lds, int r0, int ks) {
  const int lane = threadIdx.x & 63;
  if (KMAJ) {
    const int row = r0 + (lane & 31);
    const int kc = ks * 2 + (lane >> 5);
    u32x4 w = *reinterpret_cast<const u32x4*>(lds + kmaj_off(row, kc));
    return __builtin_bit_cast(bf16x8, w);
  } else {
    const int G = lane >> 4, i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
    const int k = ks * 16 + 8 * (G >> 1) + q;
    const int col = r0 + 16 * (G & 1) + 4 * p;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + mnmaj_off<ROWS>(k, col)));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + mnmaj_off<ROWS>(k + 4, col)));
    s16x4 both[2] = {lo, hi};
    return __builtin_bit_cast(bf16x8, both);
  }
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  // bijective: blocks with equal bid%8 (one XCD under round-robin dispatch) get a contiguous range
  const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

}  // namespace

// MODE 0: bf16 C (+bias,+act); MODE 1: fp32 split-K slab (blockIdx.z = split)
template <int TM, int TN, bool AK, bool BKM, int MODE>
__global__ __launch_bounds__(256) void gemm_kernel(GemmArgs g) {
  constexpr int BM = 2 * TM * 32, BN = 2 * TN * 32;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  // LDS: [A buf0 | A buf1 | B buf0 | B buf1]
  auto As = [&](int b) { return smem + b * (BM * BK * 2); };
  auto Bs = [&](int b) { return smem + 2 * BM * BK * 2 + b * (BN * BK * 2); };

  const int tiles_n = (g.N + BN - 1) / BN;
  const int tiles_m = (g.M + BM - 1) / BM;
  const int nwg = tiles_m * tiles_n;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int tm = wg / tiles_n, tn = wg % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  int kbeg = 0, kend = g.K;
  if (MODE == 1) {
    kbeg = blockIdx.z * g.k_per_split;
    kend = min(g.K, kbeg + g.k_per_split);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  Stage<BM, AK> sa;
  Stage<BN, BKM> sb;
  const uint16_t* A = reinterpret_cast<const uint16_t*>(g.A);
  const uint16_t* B = reinterpret_cast<const uint16_t*>(g.B);
  const int nt = (kend - kbeg + BK - 1) / BK;
  if (nt > 0) {
    sa.load(A, g.lda, g.M, kend, m0, kbeg);
    sb.load(B, g.ldb, g.N, kend, n0, kbeg);
    sa.store(As(0));
    sb.store(Bs(0));
  }
  __syncthreads();
  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1;
    const bool more = t + 1 < nt;
    if (more) {
      sa.load(A, g.lda, g.M, kend, m0, kbeg + (t + 1) * BK);
      sb.load(B, g.ldb, g.N, kend, n0, kbeg + (t + 1) * BK);
    }
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = frag<BM, AK>(As(cur), wm * TM * 32 + i * 32, ks);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = frag<BN, BKM>(Bs(cur), wn * TN * 32 + j * 32, ks);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      sa.store(As(cur ^ 1));
      sb.store(Bs(cur ^ 1));
    }
    __syncthreads();
  }

  // epilogue: lane owns column n, rows (r&3) + 8*(r>>2) + 4*(lane>>5) of each 32x32 tile
  const int hl = lane >> 5, cl = lane & 31;
  if (MODE == 1) {  // fp32 split-K slab: 32 lanes store 128 contiguous bytes per row
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * TN * 32 + j * 32 + cl;
      if (n >= g.N) continue;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
          if (m < g.M) reinterpret_cast<float*>(g.C)[(int64_t)blockIdx.z * g.M * g.N + (int64_t)m * g.N + n] = acc[i][j][r];
        }
    }
    return;
  }
  if (g.c_f32) {  // fp32 C (tests / fp32 heads): direct 4-byte stores, full precision
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * TN * 32 + j * 32 + cl;
      if (n >= g.N) continue;
      const float bias = g.bias ? bf16_to_f32(reinterpret_cast<const uint16_t*>(g.bias)[n]) : 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
          if (m >= g.M) continue;
          float v = acc[i][j][r] + bias;
          if (g.act == 1) v = fmaxf(v, 0.f);
          else if (g.act == 2) v = gelu_tanh(v);
          reinterpret_cast<float*>(g.C)[(int64_t)m * g.ldc + n] = v;
        }
    }
    return;
  }
  // bf16 C: apply bias/act in registers, stage the BM x BN tile through LDS, then write whole
  // 16-byte row chunks (coalesced) instead of 2-byte per-lane scatters.
  constexpr int LDC = BN + 8;  // +16 B row pad
  uint16_t* cs = reinterpret_cast<uint16_t*>(smem);  // K-loop LDS is dead after the last barrier
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int nl = wn * TN * 32 + j * 32 + cl;
    const int n = n0 + nl;
    float bias = 0.f;
    if (g.bias && n < g.N) bias = bf16_to_f32(reinterpret_cast<const uint16_t*>(g.bias)[n]);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ml = wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
        float v = acc[i][j][r] + bias;
        if (g.act == 2 && g.aux && n < g.N && m0 + ml < g.M)
          reinterpret_cast<uint16_t*>(g.aux)[(int64_t)(m0 + ml) * g.ldc + n] = f32_to_bf16(v);
        if (g.act == 1) v = fmaxf(v, 0.f);
        else if (g.act == 2) v = gelu_tanh(v);
        cs[ml * LDC + nl] = f32_to_bf16(v);
      }
  }
  __syncthreads();
  constexpr int CPR = BN / 8;  // 16-byte chunks per tile row
  for (int c = threadIdx.x; c < BM * CPR; c += 256) {
    const int ml = c / CPR, nl = (c % CPR) * 8;
    const int m = m0 + ml, n = n0 + nl;
    if (m >= g.M || n >= g.N) continue;
    const u32x4 w = *reinterpret_cast<const u32x4*>(cs + ml * LDC + nl);
    uint16_t* o = reinterpret_cast<uint16_t*>(g.C) + (int64_t)m * g.ldc + n;
    if (n + 8 <= g.N && ((reinterpret_cast<uintptr_t>(o) & 15) == 0)) {
      *reinterpret_cast<u32x4*>(o) = w;
    } else {
      const uint16_t* src = cs + ml * LDC + nl;
      for (int e = 0; e < 8 && n + e < g.N; ++e) o[e] = src[e];
    }
  }
}

// ---------------------------------------------------------------------------------------------
// 256x256 tile, 8 waves (2 x 4), global_load_lds (LDS-DMA, 16 B/lane) staging, 2 LDS stages.
// Requirements: K % 64 == 0 (no K tail inside a stage); M/N edges clamp the source row (the
// garbage rows/cols are never stored). Per stage each lane issues 4 A + 4 B LDS-DMA loads; the
// next stage is issued before the current one's MFMAs and retired with a counted vmcnt(8) + raw
// s_barrier (a __syncthreads() would drain the in-flight DMA: cdna_hip_programming.md §5).
// The LDS image is lane-linear per 1 KiB DMA piece; the bank swizzle is applied to the per-lane
// SOURCE address and the same involution on the fragment read (rule 21).
namespace {
constexpr int kBig = 256;
constexpr int kBigStage = 2 * kBig * BK * 2;  // A + B bytes per stage (64 KiB)
constexpr int kBigLdc = kBig + 8;
constexpr int kBigLds = (2 * kBigStage > kBig * kBigLdc * 2) ? 2 * kBigStage : kBig * kBigLdc * 2;

template <bool KMAJ>
__device__ __forceinline__ void glds_stage(const uint16_t* __restrict__ src, int ld, int nrows, int r0, int k0,
                                           uint8_t* lds, int wid, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int piece = i * 8 + wid;  // 32 x 1 KiB pieces per 32 KiB operand tile
    const uint16_t* gp;
    if (KMAJ) {  // [256 rows][64 k], 128-B rows: a piece is 8 rows
      const int row = piece * 8 + (lane >> 3);
      const int kc = (lane & 7) ^ ((row >> 1) & 7);
      const int gr = min(r0 + row, nrows - 1);
      gp = src + (int64_t)gr * ld + k0 + kc * 8;
    } else {  // [64 k][256 cols], 512-B rows: a piece is 2 k-rows
      const int k = piece * 2 + (lane >> 5);
      const int col = ((lane & 31) * 8) ^ ((k & 3) << 5);
      const int gc = min(r0 + col, nrows - 8);
      gp = src + (int64_t)(k0 + k) * ld + gc;
    }
    __builtin_amdgcn_global_load_lds((const void*)gp, (__attribute__((address_space(3))) void*)(lds + piece * 1024), 16,
                                     0, 0);
  }
}
}  // namespace

// Epilogue of the 256x256 kernels: fp32 slab / fp32 C direct stores, or bf16 C (+bias, +act)
// staged through LDS and written as 16-byte row chunks.
template <int MODE>
__device__ __forceinline__ void big_epilogue(const GemmArgs& g, f32x16 (&acc)[4][2], int m0, int n0, int wm, int wn,
                                             int lane, uint8_t* smem) {
  const int hl = lane >> 5, cl = lane & 31;
  if (MODE == 1 || g.c_f32) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn * 64 + j * 32 + cl;
      if (n >= g.N) continue;
      const float bias = (MODE == 0 && g.bias) ? bf16_to_f32(reinterpret_cast<const uint16_t*>(g.bias)[n]) : 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm * 128 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
          if (m >= g.M) continue;
          if (MODE == 1) {
            reinterpret_cast<float*>(g.C)[(int64_t)blockIdx.z * g.M * g.N + (int64_t)m * g.N + n] = acc[i][j][r];
          } else {
            float v = acc[i][j][r] + bias;
            if (g.act == 1) v = fmaxf(v, 0.f);
            else if (g.act == 2) v = gelu_tanh(v);
            reinterpret_cast<float*>(g.C)[(int64_t)m * g.ldc + n] = v;
          }
        }
    }
    return;
  }
  uint16_t* cs = reinterpret_cast<uint16_t*>(smem);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int nl = wn * 64 + j * 32 + cl;
    const int n = n0 + nl;
    const float bias = (g.bias && n < g.N) ? bf16_to_f32(reinterpret_cast<const uint16_t*>(g.bias)[n]) : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ml = wm * 128 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
        float v = acc[i][j][r] + bias;
        if (g.act == 2 && g.aux && n < g.N && m0 + ml < g.M)
          reinterpret_cast<uint16_t*>(g.aux)[(int64_t)(m0 + ml) * g.ldc + n] = f32_to_bf16(v);
        if (g.act == 1) v = fmaxf(v, 0.f);
        else if (g.act == 2) v = gelu_tanh(v);
        cs[ml * kBigLdc + nl] = f32_to_bf16(v);
      }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < kBig * (kBig / 8); c += 512) {
    const int ml = c >> 5, nl = (c & 31) * 8;
    const int m = m0 + ml, n = n0 + nl;
    if (m >= g.M || n >= g.N) continue;
    uint16_t* o = reinterpret_cast<uint16_t*>(g.C) + (int64_t)m * g.ldc + n;
    const uint16_t* src = cs + ml * kBigLdc + nl;
    if (n + 8 <= g.N && ((reinterpret_cast<uintptr_t>(o) & 15) == 0))
      *reinterpret_cast<u32x4*>(o) = *reinterpret_cast<const u32x4*>(src);
    else
      for (int e = 0; e < 8 && n + e < g.N; ++e) o[e] = src[e];
  }
}

template <bool AK, bool BKM, int MODE>
__global__ __launch_bounds__(512) void gemm256_kernel(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tiles_n = (g.N + kBig - 1) / kBig;
  const int tiles_m = (g.M + kBig - 1) / kBig;
  const int wg = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int m0 = (wg / tiles_n) * kBig, n0 = (wg % tiles_n) * kBig;
  int kbeg = 0, kend = g.K;
  if (MODE == 1) {
    kbeg = blockIdx.z * g.k_per_split;
    kend = min(g.K, kbeg + g.k_per_split);
  }
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid >> 2, wn = wid & 3;  // wave tile: rows wm*128.., cols wn*64..
  const uint16_t* A = reinterpret_cast<const uint16_t*>(g.A);
  const uint16_t* B = reinterpret_cast<const uint16_t*>(g.B);

  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int nt = (kend - kbeg) / BK;
  if (nt > 0) {
    glds_stage<AK>(A, g.lda, g.M, m0, kbeg, smem, wid, lane);
    glds_stage<BKM>(B, g.ldb, g.N, n0, kbeg, smem + kBig * BK * 2, wid, lane);
  }
  for (int t = 0; t < nt; ++t) {
    uint8_t* cur = smem + (t & 1) * kBigStage;
    if (t + 1 < nt) {
      uint8_t* nxt = smem + ((t + 1) & 1) * kBigStage;
      glds_stage<AK>(A, g.lda, g.M, m0, kbeg + (t + 1) * BK, nxt, wid, lane);
      glds_stage<BKM>(B, g.ldb, g.N, n0, kbeg + (t + 1) * BK, nxt + kBig * BK * 2, wid, lane);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // stage t landed, stage t+1 in flight
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    const uint8_t* As = cur;
    const uint8_t* Bs = cur + kBig * BK * 2;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8 af[4], bfr[2];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = frag<kBig, AK>(As, wm * 128 + i * 32, ks);
#pragma unroll
      for (int j = 0; j < 2; ++j) bfr[j] = frag<kBig, BKM>(Bs, wn * 64 + j * 32, ks);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();  // every wave done reading `cur` before it is re-filled
  }

  big_epilogue<MODE>(g, acc, m0, n0, wm, wn, lane, smem);
}

// ---------------------------------------------------------------------------------------------
// 256x256 tile, ring-pipelined: the K loop runs over half-stages of 32 k (A 16 KiB + B 16 KiB),
// kept in a 4-slot LDS ring (128 KiB). Three half-stages are in flight ahead of the one being
// multiplied; one raw s_barrier per half-stage both publishes slot h (after this wave's counted
// vmcnt) and releases slot h-1 for the DMA of half-stage h+3. Per half-stage each wave issues 12
// (K-major) fragment reads and 16 v_mfma_f32_32x32x16_bf16, the MFMA cluster fenced with
// s_setprio (cdna_hip_programming.md T5). K-major half-stage image: [256 rows][32 k] (64-B rows,
// 16-B chunk XOR (row>>2)&3: conflict-free for the ds_read_b128 lane groups); M/N-major:
// [32 k][256] read with ds_read_b64_tr_b16 (same image as the 2-stage kernel, 32 k-rows).
namespace {
constexpr int kHalfK = 32;
constexpr int kHalfOp = kBig * kHalfK * 2;  // 16 KiB per operand per half-stage
constexpr int kHalfSlot = 2 * kHalfOp;      // A + B

__device__ __forceinline__ int kmaj32_off(int row, int c) { return row * 64 + ((c ^ ((row >> 2) & 3)) << 4); }

template <bool KMAJ>
__device__ __forceinline__ void glds_half(const uint16_t* __restrict__ src, int ld, int nrows, int r0, int k0,
                                          uint8_t* lds, int wid, int lane) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int piece = i * 8 + wid;  // 16 x 1 KiB pieces per operand half-stage
    const uint16_t* gp;
    if (KMAJ) {  // a piece is 16 rows x 64 B
      const int row = piece * 16 + (lane >> 2);
      const int c = (lane & 3) ^ ((row >> 2) & 3);
      const int gr = min(r0 + row, nrows - 1);
      gp = src + (int64_t)gr * ld + k0 + c * 8;
    } else {  // a piece is 2 k-rows x 512 B
      const int k = piece * 2 + (lane >> 5);
      const int col = ((lane & 31) * 8) ^ ((k & 3) << 5);
      const int gc = min(r0 + col, nrows - 8);
      gp = src + (int64_t)(k0 + k) * ld + gc;
    }
    __builtin_amdgcn_global_load_lds((const void*)gp, (__attribute__((address_space(3))) void*)(lds + piece * 1024), 16,
                                     0, 0);
  }
}

template <bool KMAJ>
__device__ __forceinline__ bf16x8 frag_half(const uint8_t* lds, int r0, int ks, int lane) {
  if (KMAJ) {
    const int row = r0 + (lane & 31);
    const u32x4 w = *reinterpret_cast<const u32x4*>(lds + kmaj32_off(row, ks * 2 + (lane >> 5)));
    return __builtin_bit_cast(bf16x8, w);
  } else {
    return frag<kBig, false>(lds, r0, ks);
  }
}
}  // namespace

template <bool AK, bool BKM, int MODE>
__global__ __launch_bounds__(512) void gemm256r_kernel(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tiles_n = (g.N + kBig - 1) / kBig;
  const int tiles_m = (g.M + kBig - 1) / kBig;
  const int wg = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int m0 = (wg / tiles_n) * kBig, n0 = (wg % tiles_n) * kBig;
  int kbeg = 0, kend = g.K;
  if (MODE == 1) {
    kbeg = blockIdx.z * g.k_per_split;
    kend = min(g.K, kbeg + g.k_per_split);
  }
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid >> 2, wn = wid & 3;
  const uint16_t* A = reinterpret_cast<const uint16_t*>(g.A);
  const uint16_t* B = reinterpret_cast<const uint16_t*>(g.B);

  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int nh = (kend - kbeg) / kHalfK;
  auto stage = [&](int h) {
    uint8_t* slot = smem + (h & 3) * kHalfSlot;
    glds_half<AK>(A, g.lda, g.M, m0, kbeg + h * kHalfK, slot, wid, lane);
    glds_half<BKM>(B, g.ldb, g.N, n0, kbeg + h * kHalfK, slot + kHalfOp, wid, lane);
  };
#pragma unroll
  for (int p = 0; p < 3; ++p)
    if (p < nh) stage(p);
  for (int h = 0; h < nh; ++h) {
    // half-stage h landed (this wave's DMA): leave min(2, nh-1-h) half-stages (4 DMA each) in flight
    const int ahead = nh - 1 - h;
    if (ahead >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave: slot h published, slot h-1 no longer read
    __builtin_amdgcn_sched_barrier(0);
    if (h + 3 < nh) stage(h + 3);
    const uint8_t* As = smem + (h & 3) * kHalfSlot;
    const uint8_t* Bs = As + kHalfOp;
    bf16x8 af[2][4], bfr[2][2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int j = 0; j < 2; ++j) bfr[ks][j] = frag_half<BKM>(Bs, wn * 64 + j * 32, ks, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i) af[ks][i] = frag_half<AK>(As, wm * 128 + i * 32, ks, lane);
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[ks][i], bfr[ks][j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
  }
  __builtin_amdgcn_s_barrier();  // the epilogue reuses the ring
  big_epilogue<MODE>(g, acc, m0, n0, wm, wn, lane, smem);
}

// out = (accumulate ? out : 0) + sum_s slab[s]   (M*N elements, 8 per lane)
template <bool OUT_BF16>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ slab, int splits, int64_t mn,
                                                            void* __restrict__ out, int accumulate, float scale) {
  const int64_t nvec = mn >> 3;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    float s[8];
    load8_f32(slab + v * 8, s);
    for (int k = 1; k < splits; ++k) {
      float t[8];
      load8_f32(slab + (int64_t)k * mn + v * 8, t);
#pragma unroll
      for (int e = 0; e < 8; ++e) s[e] += t[e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) s[e] *= scale;
    if (OUT_BF16) {
      uint16_t* o = reinterpret_cast<uint16_t*>(out) + v * 8;
      if (accumulate) {
        float t[8];
        load8_bf16(o, t);
#pragma unroll
        for (int e = 0; e < 8; ++e) s[e] += t[e];
      }
      store8_bf16(o, s);
    } else {
      float* o = reinterpret_cast<float*>(out) + v * 8;
      if (accumulate) {
        float t[8];
        load8_f32(o, t);
#pragma unroll
        for (int e = 0; e < 8; ++e) s[e] += t[e];
      }
      store8_f32(o, s);
    }
  }
  if (blockIdx.x == 0) {
    for (int64_t i = (nvec << 3) + threadIdx.x; i < mn; i += blockDim.x) {
      float s = 0.f;
      for (int k = 0; k < splits; ++k) s += slab[(int64_t)k * mn + i];
      s *= scale;
      if (OUT_BF16) {
        uint16_t* o = reinterpret_cast<uint16_t*>(out);
        o[i] = f32_to_bf16(s + (accumulate ? bf16_to_f32(o[i]) : 0.f));
      } else {
        float* o = reinterpret_cast<float*>(out);
        o[i] = s + (accumulate ? o[i] : 0.f);
      }
    }
  }
}

// column sums of a [M][N] bf16 matrix (bias gradient), deterministic two-pass: block partials
// (lane = 8 columns, 4 rows in flight) -> one finalize lane per column summing <= 64 partial rows.
constexpr int kColsumMaxBlocks = 512;  // partial rows (the caller's workspace is [512 * N] fp32)
__global__ __launch_bounds__(256) void colsum_partial_kernel(const uint16_t* __restrict__ x, int64_t M, int N,
                                                             float* __restrict__ part) {
  const int tpc = N >> 3;
  const int rpi = tpc >= 256 ? 1 : 256 / tpc;
  const int cg = tpc >= 256 ? blockIdx.y * 256 + threadIdx.x : threadIdx.x % tpc;
  const int r0 = tpc >= 256 ? 0 : threadIdx.x / tpc;
  const bool active = cg < tpc && r0 < rpi;
  float a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (active) {
    const int64_t stride = (int64_t)gridDim.x * rpi;
    int64_t r = (int64_t)blockIdx.x * rpi + r0;
    for (; r + 3 * stride < M; r += 4 * stride) {
      float t[4][8];
#pragma unroll
      for (int u = 0; u < 4; ++u) load8_bf16(x + (r + u * stride) * N + cg * 8, t[u]);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int e = 0; e < 8; ++e) a[e] += t[u][e];
    }
    for (; r < M; r += stride) {
      float t[8];
      load8_bf16(x + r * N + cg * 8, t);
#pragma unroll
      for (int e = 0; e < 8; ++e) a[e] += t[e];
    }
  }
  __shared__ float red[256 * 8];
  if (tpc >= 256) {
    if (active) store8_f32(part + (int64_t)blockIdx.x * N + cg * 8, a);
    return;
  }
  if (active)
#pragma unroll
    for (int e = 0; e < 8; ++e) red[r0 * N + cg * 8 + e] = a[e];
  __syncthreads();
  for (int c = threadIdx.x; c < N; c += 256) {
    float sum = 0.f;
    for (int rr = 0; rr < rpi; ++rr) sum += red[rr * N + c];
    part[(int64_t)blockIdx.x * N + c] = sum;
  }
}

// Deterministic second pass: block = 32 columns x 8 partial-row lanes; fixed summation order.
__global__ __launch_bounds__(256) void colsum_final_kernel(const float* __restrict__ part, int nblk, int N, void* out,
                                                           int out_bf16, int accumulate) {
  const int cl = threadIdx.x & 31, rl = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cl;
  float s = 0.f;
  if (c < N)
    for (int b = rl; b < nblk; b += 8) s += part[(int64_t)b * N + c];
  __shared__ float red[8][33];
  red[rl][cl] = s;
  __syncthreads();
  if (rl != 0 || c >= N) return;
#pragma unroll
  for (int r = 1; r < 8; ++r) s += red[r][cl];
  if (out_bf16) {
    uint16_t* o = reinterpret_cast<uint16_t*>(out);
    o[c] = f32_to_bf16(s + (accumulate ? bf16_to_f32(o[c]) : 0.f));
  } else {
    float* o = reinterpret_cast<float*>(out);
    o[c] = s + (accumulate ? o[c] : 0.f);
  }
}

__global__ void f32_to_bf16_kernel(const float* in, uint16_t* out, int n, int accumulate) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = f32_to_bf16(in[i] + (accumulate ? bf16_to_f32(out[i]) : 0.f));
}

// ------------------------------------------------------------------ host side
template <int TM, int TN, bool AK, bool BKM, int MODE>
static hipError_t launch_t(const GemmArgs& g, int splits, hipStream_t st) {
  constexpr int BM = 2 * TM * 32, BN = 2 * TN * 32;
  const int nwg = ((g.M + BM - 1) / BM) * ((g.N + BN - 1) / BN);
  const size_t lds = 2 * (size_t)(BM + BN) * BK * 2;
  hipLaunchKernelGGL((gemm_kernel<TM, TN, AK, BKM, MODE>), dim3(nwg, 1, splits), dim3(256), lds, st, g);
  return hipGetLastError();
}

static bool use_ring() {
  static const int v = [] {
    const char* e = getenv("PSD_GEMM_RING");
    return e ? atoi(e) : 1;
  }();
  return v != 0;
}

template <bool AK, bool BKM, int MODE>
static hipError_t launch_big(const GemmArgs& g, int splits, hipStream_t st) {
  const bool ring = use_ring();
  const void* fn = ring ? (const void*)gemm256r_kernel<AK, BKM, MODE> : (const void*)gemm256_kernel<AK, BKM, MODE>;
  static bool attr_set[2] = {false, false};  // per instantiation: set the >64 KiB LDS limit once
  if (!attr_set[ring]) {
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, kBigLds);
    if (e != hipSuccess) return e;
    attr_set[ring] = true;
  }
  const int nwg = ((g.M + kBig - 1) / kBig) * ((g.N + kBig - 1) / kBig);
  if (ring)
    hipLaunchKernelGGL((gemm256r_kernel<AK, BKM, MODE>), dim3(nwg, 1, splits), dim3(512), kBigLds, st, g);
  else
    hipLaunchKernelGGL((gemm256_kernel<AK, BKM, MODE>), dim3(nwg, 1, splits), dim3(512), kBigLds, st, g);
  return hipGetLastError();
}

static bool big_ok(const GemmArgs& g, int kseg) {
  // enough 256x256 tiles to fill the chip, no K tail inside a stage, MN-major operands 8-aligned
  const int64_t tiles = (int64_t)((g.M + 255) / 256) * ((g.N + 255) / 256);
  if (getenv("PSD_GEMM_SMALL_ONLY")) return false;
  // split-K (MODE 1) passes tiles * splits via k_per_split < K
  const int64_t waves = g.k_per_split > 0 ? tiles * ((g.K + g.k_per_split - 1) / g.k_per_split) : tiles;
  return g.M >= 256 && g.N >= 256 && kseg % 64 == 0 && waves >= 64 && g.K >= 256;
}

template <bool AK, bool BKM, int MODE>
static hipError_t launch_layout(const GemmArgs& g, int splits, hipStream_t st) {
  if (big_ok(g, MODE == 1 ? g.k_per_split : g.K) && (MODE == 1 || g.K % 64 == 0))
    return launch_big<AK, BKM, MODE>(g, splits, st);
  // tile choice: 128x128 by default, 128x64 / 64x128 for narrow operands (more tiles)
  if (g.N <= 64 && g.M > 64) return launch_t<2, 1, AK, BKM, MODE>(g, splits, st);
  if (g.M <= 64 && g.N > 64) return launch_t<1, 2, AK, BKM, MODE>(g, splits, st);
  if (g.M <= 64 && g.N <= 64) return launch_t<1, 1, AK, BKM, MODE>(g, splits, st);
  return launch_t<2, 2, AK, BKM, MODE>(g, splits, st);
}

hipError_t launch_gemm(const GemmArgs& g, hipStream_t st) {
  if (g.M <= 0 || g.N <= 0) return hipSuccess;
  if (g.a_kmajor && g.b_kmajor) return launch_layout<true, true, 0>(g, 1, st);
  if (g.a_kmajor && !g.b_kmajor) return launch_layout<true, false, 0>(g, 1, st);
  if (!g.a_kmajor && !g.b_kmajor) return launch_layout<false, false, 0>(g, 1, st);
  return launch_layout<false, true, 0>(g, 1, st);
}

int gemm_splits(int M, int N, int K) {
  if (M >= 256 && N >= 256 && K % 64 == 0 && K >= 4096) {  // 256x256 tiles, one workgroup per CU
    const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
    int s = (256 + tiles - 1) / tiles;
    const int kmax = K / 512;
    if (s > kmax) s = kmax;
    if (s > 64) s = 64;
    return s < 1 ? 1 : s;
  }
  const int BM = M <= 64 ? 64 : 128, BN = N <= 64 ? 64 : 128;
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  int s = (512 + tiles - 1) / tiles;      // ~2 workgroups per CU
  const int kmax = (K + 255) / 256;       // >= 256 k per split
  if (s > kmax) s = kmax;
  if (s > 64) s = 64;
  return s < 1 ? 1 : s;
}

hipError_t launch_gemm_splitk(const GemmArgs& g0, float* slab, int splits, void* out, int out_bf16, int accumulate,
                              float scale, hipStream_t st) {
  if (g0.M <= 0 || g0.N <= 0) return hipSuccess;
  GemmArgs g = g0;
  g.C = slab;
  int kps = (g.K + splits - 1) / splits;
  kps = (kps + BK - 1) / BK * BK;
  g.k_per_split = kps;
  const int eff = (g.K + kps - 1) / kps;  // splits that own a non-empty k-range
  hipError_t e;
  if (g.a_kmajor && g.b_kmajor) e = launch_layout<true, true, 1>(g, eff, st);
  else if (g.a_kmajor && !g.b_kmajor) e = launch_layout<true, false, 1>(g, eff, st);
  else if (!g.a_kmajor && !g.b_kmajor) e = launch_layout<false, false, 1>(g, eff, st);
  else e = launch_layout<false, true, 1>(g, eff, st);
  if (e != hipSuccess) return e;
  const int64_t mn = (int64_t)g.M * g.N;
  const int grid = stream_grid((mn >> 3) > 0 ? (mn >> 3) : 1, 256);
  if (out_bf16)
    hipLaunchKernelGGL(splitk_reduce_kernel<true>, dim3(grid), dim3(256), 0, st, slab, eff, mn, out, accumulate, scale);
  else
    hipLaunchKernelGGL(splitk_reduce_kernel<false>, dim3(grid), dim3(256), 0, st, slab, eff, mn, out, accumulate, scale);
  return hipGetLastError();
}

hipError_t launch_colsum(const uint16_t* x, int64_t M, int N, float* part, void* out, int out_bf16,
                         int accumulate, hipStream_t st) {
  if (N % 8 != 0) return hipErrorInvalidValue;
  const int tpc = N / 8;
  const int gy = tpc >= 256 ? (tpc + 255) / 256 : 1;
  const int rpi = tpc >= 256 ? 1 : 256 / tpc;
  // enough row-chunks to fill the chip (~1024 resident blocks over all column groups), each
  // thread summing >= 8 rows
  int64_t gx = (M + (int64_t)rpi * 8 - 1) / ((int64_t)rpi * 8);
  const int64_t want = (1024 + gy - 1) / gy;
  if (gx > want) gx = want;
  if (gx > kColsumMaxBlocks) gx = kColsumMaxBlocks;
  if (gx < 1) gx = 1;
  hipLaunchKernelGGL(colsum_partial_kernel, dim3((unsigned)gx, gy), dim3(256), 0, st, x, M, N, part);
  hipLaunchKernelGGL(colsum_final_kernel, dim3((N + 31) / 32), dim3(256), 0, st, part, (int)gx, N, out, out_bf16,
                     accumulate);
  return hipGetLastError();
}

}  // namespace psd
