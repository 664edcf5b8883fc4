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

#include <algorithm>
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

// GELU(tanh) = x * sigmoid(2u), u = sqrt(2/pi) (x + 0.044715 x^3): one v_exp_f32 + one v_rcp_f32
// (x -> -inf: exp -> inf, rcp -> 0, result -0 as the tanh form)
__device__ __forceinline__ float gelu_tanh(float x) {
  const float k0 = 2.f * 0.7978845608028654f, k1 = 2.f * 0.7978845608028654f * 0.044715f;
  const float e = __expf(-x * (k0 + k1 * x * x));
  return x * __builtin_amdgcn_rcpf(1.f + e);
}

// GELU(tanh) derivative: s = sigmoid(2u), d/dx [x s] = s + 2 x s (1 - s) u'(x)
__device__ __forceinline__ float gelu_tanh_grad(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float u = k0 * (x + k1 * x * x * x);
  const float sg = __builtin_amdgcn_rcpf(1.f + __expf(-2.f * u));
  return sg + 2.f * x * sg * (1.f - sg) * k0 * (1.f + 3.f * k1 * x * x);
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
          if (g.act == 1) v = relu_nan(v);
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
        if (g.act == 1) v = relu_nan(v);
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
namespace {
constexpr int kBig = 256;  // output tile width of the 8-phase kernel
}  // namespace

// ---------------------------------------------------------------------------------------------
// 256x256 tile, 8-phase ping-pong schedule (cdna_hip_programming.md §5 "256² 8-phase template",
// T2-T5), v_mfma_f32_16x16x32_bf16. 8 waves = 2 wave rows (wr) x 4 wave cols (wc); each wave owns
// 128x64 of C as four 64x32 quadrants (qm, qn). A K-tile (64 k) is four phases, one quadrant each:
//   phase 0: q(0,0)  reads B(qn0) then A(qm0)      stages A-half1 of tile t+1
//   phase 1: q(0,1)  reads B(qn1)                   stages B-half0 of tile t+2
//   phase 2: q(1,0)  reads A(qm1)  (B(qn0) kept)    stages A-half0 of tile t+2
//   phase 3: q(1,1)  no reads                       stages B-half1 of tile t+2, vmcnt(6)
// The LDS holds two K-tiles, each as four 16 KiB half-tiles: A-half h = the rows of quadrant row h
// of both wave rows, B-half h = the cols of quadrant col h of all four wave cols, so a half-tile is
// dead for the whole block as soon as its quadrant has been read. Every phase is
// {ds_reads, 2 LDS-DMA} -> s_barrier -> 16 MFMA (s_setprio 1) -> s_barrier, and wave row 1 runs one
// barrier behind wave row 0: the two waves sharing a SIMD alternate between reading and MFMA.
// RAW: a tile's last half is retired by the counted vmcnt(6) of the phase before its first read.
// WAR: a half is restaged >= 2 phases after its last read, or 1 phase after when an lgkmcnt before
// the reading phase's first barrier retired it (phase 0's lgkmcnt(8) retires the B(qn0) reads).
// Tiles past the end are staged from the last valid K offset (same count of DMA per phase, data
// never read), so the vmcnt bookkeeping is uniform.
namespace {
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int mn8_off(int k, int col) {  // M/N-major half image [64 k][128], 256-B rows
  const int f = (k & 3) | ((k >> 1) & 4);  // the 8 k-rows of one tr-read half-wave hit 8 distinct 32-B slots
  return k * 256 + ((col ^ (f << 4)) << 1);
}

// half-tile local row/col -> tile row/col (SEG = quadrant extent: 64 rows of A, 32 cols of B)
template <int SEG>
__device__ __forceinline__ int half_to_tile(int r, int h) {
  return (r / SEG) * (2 * SEG) + h * SEG + (r % SEG);
}

// Buffer-descriptor LDS-DMA staging: per piece the lane's byte offset = (scalar tile/k origin) +
// (per-lane part, loop-invariant); rows past the operand's end fall outside the descriptor's range
// and load zeros (only garbage rows/cols of C, never stored, depend on them), so no per-lane clamp.
typedef __amdgpu_buffer_rsrc_t rsrc_t;
__device__ __forceinline__ rsrc_t make_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
// per-lane byte offsets of one operand's pieces (piece i of half h), loop-invariant. VR: the valid
// rows (K-major) / columns (M/N-major) of a half image (BM = 192: 96 of its 128; the rest of the
// padded image is never read): the pieces / lanes past them get kMasked, an offset past every
// descriptor's range (operands < 2 GiB there), so their DMA writes zeros and moves no bytes
constexpr uint32_t kMasked = 0x80000000u;
// CONTIG (N-major B of the split-K GEMMs): half h holds tile columns [128 h, 128 h + 128) instead of
// quadrant column h of every wave column (four 32-column = 64-byte pieces per k-row), so each
// 256-byte LDS row is two whole 128-byte lines of the operand; the wave -> column map of the
// epilogue follows (ncol below)
template <bool KMAJ, int SEG, int ESZ, int PW, int VR = 128, bool CONTIG = false>
__device__ __forceinline__ void stage8_offsets(int ld, int wid, int lane, uint32_t (*vo)[PW]) {
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const int piece = i * 8 + wid;  // PW * 8 pieces of 1 KiB per half-tile
      if (KMAJ) {  // [128 rows][128 B of k]: a piece is 8 rows x 128 B
        const int row = piece * 8 + (lane >> 3);
        const int c = (lane & 7) ^ ((row >> 1) & 7);
        vo[h][i] = row < VR ? (uint32_t)half_to_tile<SEG>(row, h) * (uint32_t)ld * ESZ + c * 16 : kMasked;
      } else {  // [64 k][128 cols] bf16: a piece is 4 k-rows x 256 B
        const int k = piece * 4 + (lane >> 4);
        const int f = (k & 3) | ((k >> 1) & 4);
        const int col = ((lane & 15) * 8) ^ (f << 4);
        const int tc = CONTIG ? h * 128 + col : half_to_tile<SEG>(col, h);
        vo[h][i] = col < VR ? ((uint32_t)k * (uint32_t)ld + tc) * ESZ : kMasked;
      }
    }
}
template <bool KMAJ, int ESZ, int PW>
__device__ __forceinline__ void stage8(const void* base, uint32_t bytes, const uint32_t* vo, int ld, int r0, int k0,
                                       uint8_t* lds, int wid) {
  // scalar origin of the piece grid (bytes): K-major [rows][ld] at (r0, k0); M/N-major [k][ld] at (k0, r0);
  // readfirstlane keeps it a separate scalar term (not folded into a per-lane multiply)
  const uint32_t so = __builtin_amdgcn_readfirstlane(KMAJ ? ((uint32_t)r0 * (uint32_t)ld + (uint32_t)k0) * ESZ
                                                          : ((uint32_t)k0 * (uint32_t)ld + (uint32_t)r0) * ESZ);
  const rsrc_t src = make_rsrc(base, bytes);  // wave-uniform (kernel arguments)
#pragma unroll
  for (int i = 0; i < PW; ++i)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(src, (__attribute__((address_space(3))) void*)(lds + (i * 8 + wid) * 1024),
                                             16, vo[i] + so, 0, 0, 0);
}

// 16x16x32 fragment: lane holds row/col (rb*16 + lane&15), k = ks*32 + 8*(lane>>4) + 0..7
template <bool KMAJ>
__device__ __forceinline__ bf16x8 frag8(const uint8_t* lds, int rb, int ks, int lane) {
  if (KMAJ) {
    const int row = rb * 16 + (lane & 15);
    const u32x4 w = *reinterpret_cast<const u32x4*>(lds + kmaj_off(row, ks * 4 + (lane >> 4)));
    return __builtin_bit_cast(bf16x8, w);
  } else {
    const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
    const int k = ks * 32 + 8 * g + q;
    const int col = rb * 16 + 4 * p;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + mn8_off(k, col)));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + mn8_off(k + 4, col)));
    s16x4 both[2] = {lo, hi};
    return __builtin_bit_cast(bf16x8, both);
  }
}

typedef int i32x8 __attribute__((ext_vector_type(8)));
// fp8 (e4m3) 16x16x128 fragment: 32 bytes of one 128-B row = 16-B chunks (lane>>4) and 4+(lane>>4);
// A and B use the same k order, which is all the dot product needs
__device__ __forceinline__ i32x8 frag8_f8(const uint8_t* lds, int rb, int lane) {
  const int row = rb * 16 + (lane & 15);
  const u32x4 lo = *reinterpret_cast<const u32x4*>(lds + kmaj_off(row, lane >> 4));
  const u32x4 hi = *reinterpret_cast<const u32x4*>(lds + kmaj_off(row, 4 + (lane >> 4)));
  return i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
template <int N>
__device__ __forceinline__ void wait_lgkm() {
  static_assert(N >= 0, "lgkmcnt");
  if constexpr (N >= 15) asm volatile("s_waitcnt lgkmcnt(15)" ::: "memory");  // the counter saturates at 15
  else asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
}

template <int CTRL>
__device__ __forceinline__ float dpp_q(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
// 4x4 transpose inside a lane quad: in v[r] = C[row r][col L]; out w[c] = C[row L][col c]
__device__ __forceinline__ void quad_t4(const f32x4 v, int L, float (&w)[4]) {
  const bool o1 = L & 1, o2 = (L >> 1) & 1;
  const float r0 = dpp_q<0xB1>(o1 ? v[0] : v[1]);  // quad_perm [1,0,3,2]: partner L^1
  const float r1 = dpp_q<0xB1>(o1 ? v[2] : v[3]);
  const float a0 = o1 ? r0 : v[0], a1 = o1 ? v[1] : r0;  // row L&1,     cols (L&~1, L|1)
  const float b0 = o1 ? r1 : v[2], b1 = o1 ? v[3] : r1;  // row (L&1)+2, same cols
  const float q0 = dpp_q<0x4E>(o2 ? a0 : b0);            // quad_perm [2,3,0,1]: partner L^2
  const float q1 = dpp_q<0x4E>(o2 ? a1 : b1);
  w[0] = o2 ? q0 : a0;
  w[1] = o2 ? q1 : a1;
  w[2] = o2 ? b0 : q0;
  w[3] = o2 ? b1 : q1;
}
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  return (uint32_t)f32_to_bf16(lo) | ((uint32_t)f32_to_bf16(hi) << 16);
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

// lane-group sums for the statistics epilogue: x of lane ^ 16 / lane ^ 32 (the gfx950 half-row /
// half-wave swaps)
__device__ __forceinline__ float st_xor16(float x, int lane) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float((lane & 16) ? r[0] : r[1]);
}
__device__ __forceinline__ float st_xor32(float x, int lane) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float((lane & 32) ? r[0] : r[1]);
}

// grouped tile order inside one XCD's contiguous range: 4 tile-rows share each B panel
__device__ __forceinline__ void tile_of(int wg, int tiles_m, int tiles_n, int& tm, int& tn) {
  constexpr int G = 4;
  const int per = G * tiles_n;
  const int grp = wg / per;
  const int first = grp * G;
  const int gsz = min(G, tiles_m - first);
  const int r = wg - grp * per;
  tm = first + r % gsz;
  tn = r / gsz;
}
}  // namespace

#define PSD_SYNC_OPEN()                              \
  __builtin_amdgcn_s_barrier();                      \
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); \
  __builtin_amdgcn_sched_barrier(0);                 \
  __builtin_amdgcn_s_setprio(1);
#define PSD_SYNC_CLOSE()               \
  __builtin_amdgcn_s_setprio(0);       \
  __builtin_amdgcn_sched_barrier(0);   \
  __builtin_amdgcn_s_barrier();        \
  __builtin_amdgcn_sched_barrier(0);

// BM: 256 (8 waves x 128x64 of C) or 128 (8 waves x 64x64: twice the tiles for narrow problems).
// F8: A [M][K] and B [N][K] OCP e4m3 (K-major only), K-tile = 128, MX-scaled
// v_mfma_scale_f32_16x16x128_f8f6f4 with unit block scales (2x the bf16 MFMA rate); the per-tensor
// dequant factors *a_scale * *b_scale are applied in the epilogue.
//
// Persistent: a grid of G <= tiles workgroups (one per CU, LDS-limited), workgroup b owns the tiles
// v = b, b + G, b + 2G, ... (xcd_remap keeps v % 8 = the XCD, so each XCD walks a contiguous tile
// range). The K-tiles of consecutive output tiles form ONE stream: the two stages the 8-phase loop
// issues past the end of a tile are the next tile's first two K-tiles, so the LDS pipeline never
// drains between tiles. The epilogue therefore cannot stage C through the pipeline LDS (both buffers
// hold the next tile): each quad of lanes transposes its 4x4 C block in registers (quad_t4); fp32
// goes out as 16-byte row segments, bf16 through a per-wave 4 KiB LDS slot (whole 128-byte rows
// per store); the stores drain while the next tile's first phases run (retired by the first
// phase-3 vmcnt, in issue order).
// MX: the block-scaled fp8 form (per-32-K E8M0 scales of A rows and B columns): each K-tile's
// scales (BM x 4 B of A, 256 x 4 B of B) ride in SC bytes at the end of its buffer, staged by one
// extra 4-byte LDS-DMA per wave with the A-half0 pieces (so it is counted in VM like them).
// BM = 192 (IM = 3, 48-row quadrants) keeps the 256-row LDS geometry: each A half image is padded
// to 128 rows / columns (the last 32 masked at staging, never read), so the staging and the
// fragment reads are the BM = 256 ones and the LDS is 160 KiB. With CT (C^T stored) it is the
// 256 x 192 tile of Y = X W^T: 768-wide outputs make 4 x 128 = 512 tiles (2.0 rounds on 256 CUs)
// instead of 384 256-tiles (1.5 rounds, the last half idle).
template <int BM, bool MX = false>
struct P8 {
  static constexpr int IM = BM / 64;         // 16-row blocks per quadrant
  static constexpr int QA = BM / 4;          // quadrant rows
  static constexpr int VA = BM / 2;          // valid rows (K-major) / cols (M-major) of an A half image
  static constexpr int HA = (BM == 192 ? 128 : BM / 2) * 128;  // A half-tile bytes (BM 192: padded)
  static constexpr int HB = 128 * 128;       // B half-tile bytes
  static constexpr int PWA = HA / 8192;      // A DMA pieces per wave per half-tile
  static constexpr int VM = 4 + PWA + (MX ? 1 : 0);  // DMA in flight after phase 3 (three half-tiles)
  static constexpr int SC = MX ? 2048 : 0;   // scale bytes per buffer: A [BM][4] at 0, B [256][4] at 512
  static constexpr int BUF = 2 * HA + 2 * HB + SC;
  static constexpr int STG = 4096;           // per-wave epilogue staging (16 rows x 64 cols, C + aux)
  static constexpr int LDS = 2 * BUF + 8 * STG;
};

template <int ACT>
__device__ __forceinline__ float act_apply(float x) {
  if constexpr (ACT == 1) return relu_nan(x);
  else if constexpr (ACT == 2) return gelu_tanh(x);
  else return x;
}

// ACT: the epilogue activation as a template parameter (g.act must match): per-element branches made
// the unrolled epilogue several times larger, and at one output tile per ~10 K-tiles its instruction
// fetch, not its arithmetic, was the cost.
// GA: A is gathered as an implicit-GEMM convolution input (GemmArgs cv_*): each lane's A rows are
// output pixels whose (r, s)-shifted input pixel is computed per K-tile (one (r, s) per K-tile:
// C % 64 == 0); pixels outside the image get an offset past the descriptor, i.e. the zero padding.
// F8A: the A operand's fp8 format (0 e4m3, 1 e5m2: bwd-data of the fp8 convolutions takes e5m2 dY)
// ST: the consumer BatchNorm's batch statistics in the bf16 epilogue (g.part / g.shift): per output
// channel the shifted sums sum(y - shift) and sum((y - shift)^2) of the fp32 accumulators (before the
// bf16 rounding of the store: within 2^-9 per element of the stored tensor's; formed from the plain
// sums of the wave row, exact for |mean - shift| up to ~100 standard deviations) over each wave row's
// BM / 2 rows -> partial row (tile_m * 2 + wave row) of part [rows][2][N] (the layout of
// kernels/bn.hip bn_fwd_reduce_kernel), so the BN forward skips its statistics pass. The shift (the
// running mean) arrives by LDS-DMA with the bias, 4 B per lane.
// ACT 3 (GELU backward of the Linear that produced this GEMM's A-side input: C = dY W is d(gelu
// output)): the bf16 epilogue multiplies each stored element by gelu'(pre) (g.aux = the saved
// pre-activation, read 16 B per lane on the store side), stores g = bf16(C gelu'(pre)) and sums its
// columns per wave row -> g.part [rows][N] fp32 (the bias gradient's partials; one row per wave row
// of each 256 / 128-row tile). The separate GELU-backward + column-sum pass over C and pre is gone.
// GB: B is gathered as the im2col image of a convolution input for the weight gradient (MODE 1):
// dW[cout][(r, s, ci)] = sum over output pixels p of dY[p][cout] * x[pixel(p) + (r, s)][ci], A = dY
// M-major ([pixels][cout]), B = the gathered [pixels][R*S*C] N-major image (each lane's 16 bytes are
// 8 channels of one shifted input pixel; pixels outside the image load zeros).
// CT: the tile is stored transposed -- Y[n][m] = C[m][n], Y's row stride g.ldc -- with the bias per C
// row (g.bias [M]) and ACT 0 / 1 / 2 (+ aux): Y = X W^T + b with A = W [out][in], B = X [tokens][in].
// In the MFMA register layout a lane holds 4 consecutive C rows of one column = 4 contiguous Y
// elements, so the store needs no transpose (8-byte bf16 / 16-byte fp32 per lane and block).
template <int BM, bool AK, bool BKM, int MODE, bool F8 = false, int ACT = 0, bool GA = false, int F8A = 0,
          bool GB = false, bool MX = false, bool ST = false, bool CT = false, bool BC = false>
__global__ __launch_bounds__(512) void gemm8p_kernel(GemmArgs g) {
  static_assert(!BC || (MODE == 1 && !BKM), "contiguous B halves: split-K (fp32 epilogue) with an N-major B");
  static_assert(!CT || (MODE == 0 && !ST && !GA && !GB && !F8 && ACT <= 2 && AK && BKM),
                "transposed store: plain bf16 single-split GEMM of K-major operands");
  static_assert(BM != 192 || (!MX && !GA && !F8 && !ST && MODE == 0), "192-row tiles: plain bf16 GEMM");
  static_assert(!ST || (MODE == 0 && !GB && ACT == 0 && AK),
                "statistics epilogue: single split, bf16 out, no activation, K-major A (zero rows past M)");
  static_assert(!MX || (F8 && BM == 128 && MODE == 0), "MX: fp8, 128-row tiles (LDS), single split");
  static_assert(ACT != 3 || (MODE == 0 && !F8 && !GA && !GB && !ST), "GELU-backward epilogue: bf16 single-split GEMM");
  static_assert(!GB || (!AK && !BKM && MODE == 1 && !F8 && !GA), "implicit-GEMM wgrad: M-major dY, split-K");
  static_assert(!F8 || (AK && BKM), "fp8 GEMM takes K-major operands");
  static_assert(!GA || (AK && MODE == 0), "implicit-GEMM convolution: K-major A, single split");
  static_assert(BM == 256 || AK, "BM = 128 takes a K-major A");
  using P = P8<BM, MX>;
  constexpr int IM = P::IM;
  constexpr int KT = F8 ? 128 : BK;  // k per K-tile (128-B LDS rows either way)
  constexpr int ESZ = F8 ? 1 : 2;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tiles_n = (g.N + kBig - 1) / kBig;
  const int tiles_m = (g.M + BM - 1) / BM;
  const int ntiles = tiles_m * tiles_n;
  const int G = gridDim.x;
  const int ntl = (ntiles - (int)blockIdx.x + G - 1) / G;  // this workgroup's tiles (>= 1: G <= ntiles)
  auto origin = [&](int j, int& m0, int& n0) {
    int tm, tn;
    tile_of(xcd_remap(blockIdx.x + j * G, ntiles), tiles_m, tiles_n, tm, tn);
    m0 = tm * BM;
    n0 = tn * kBig;
  };
  int kbeg = 0, kend = g.K;
  if (MODE == 1) {
    kbeg = blockIdx.z * g.k_per_split;
    kend = min(g.K, kbeg + g.k_per_split);
  }
  // >= 2 whenever G < ntiles (host contract); GB: a partial last K-tile reads zeros past K (both
  // operands are range-checked), so K needs no multiple of 64
  const int nt = GB ? (kend - kbeg + KT - 1) / KT : (kend - kbeg) / KT;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid >> 2, wc = wid & 3;

  f32x4 acc[8 * IM];
#pragma unroll
  for (int i = 0; i < 8 * IM; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  int jt = 0, base = 0;  // current tile (local index) and its first K-tile in the stream
  int cm0, cn0, xm0, xn0;
  origin(0, cm0, cn0);
  xm0 = cm0;
  xn0 = cn0;
  if (ntl > 1) origin(1, xm0, xn0);
  auto half = [&](int u, int idx) {  // idx: 0/1 A-half, 2/3 B-half; u = K-tile index in the stream
    return smem + (u & 1) * P::BUF + (idx < 2 ? idx * P::HA : 2 * P::HA + (idx - 2) * P::HB);
  };
  // operand extents in bytes (host contract: < 2^32): K-major [rows][ld], M/N-major [K][ld]
  const uint32_t bytesA = AK ? ((uint32_t)(g.M - 1) * g.lda + g.K) * ESZ : ((uint32_t)(g.K - 1) * g.lda + g.M) * ESZ;
  const uint32_t bytesB = BKM ? ((uint32_t)(g.N - 1) * g.ldb + g.K) * ESZ : ((uint32_t)(g.K - 1) * g.ldb + g.N) * ESZ;
  uint32_t voA[2][P::PWA], voB[2][2];  // [half][piece]
  stage8_offsets<AK, P::QA, ESZ, P::PWA, P::VA>(g.lda, wid, lane, voA);
  stage8_offsets<BKM, 32, ESZ, 2, 128, BC>(g.ldb, wid, lane, voB);
  // GA: per (tile, half, piece) the window origin of the lane's output pixel: p0 = its top-left input
  // pixel index, hw = (h0 << 16) | (w0 & 0xffff) (h0 = -32768 for rows past M)
  int cp0[2][P::PWA], chw[2][P::PWA], np0[2][P::PWA], nhw[2][P::PWA];
  auto conv_rows = [&](int m0, int (&p0)[2][P::PWA], int (&hw)[2][P::PWA]) {
    const int howo = g.cv_Ho * g.cv_Wo;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < P::PWA; ++i) {
        const int row = (i * 8 + wid) * 8 + (lane >> 3);
        const int m = m0 + half_to_tile<P::QA>(row, h);
        const int n = m / howo, rem = m - n * howo;
        const int ho = rem / g.cv_Wo, wo = rem - ho * g.cv_Wo;
        const int h0 = ho * g.cv_stride - g.cv_pad, w0 = wo * g.cv_stride - g.cv_pad;
        p0[h][i] = (n * g.cv_H + h0) * g.cv_W + w0;
        hw[h][i] = m < g.M ? (int)(((uint32_t)h0 << 16) | ((uint32_t)w0 & 0xffffu)) : (int)0x80000000u;
      }
  };
  if constexpr (GA) {
    conv_rows(cm0, cp0, chw);
    conv_rows(xm0, np0, nhw);
  }
  auto stA = [&](int u, int m0, int k, int h, int n0s) {
    if constexpr (MX) {
      if (h == 0) {  // this K-tile's scales: waves 0-1 A rows, 2-5 B columns, 6-7 a dummy (zeros)
        uint8_t* sc = smem + (u & 1) * P::BUF + 2 * P::HA + 2 * P::HB;
        const uint32_t kblk = (uint32_t)g.K >> 5, kb = (uint32_t)k >> 5;
        const bool isA = wid < 2, isB = wid >= 2 && wid < 6;
        const uint32_t abytes = GA ? (g.cv_abytes >> 5) : (uint32_t)g.M * kblk;
        const rsrc_t src = isB ? make_rsrc(g.b_mx, (uint32_t)g.N * kblk) : make_rsrc(g.a_mx, abytes);
        uint32_t off = 0xFFFFFFF0u;  // past every range: zeros
        if (isA) {
          const int row = m0 + wid * 64 + lane;
          if constexpr (GA) {  // the row's gathered input pixel for this K-tile's (r, s): [pixels][C/32] scales
            if (row < g.M) {
              const int howo = g.cv_Ho * g.cv_Wo;
              const int n = row / howo, rem = row - n * howo;
              const int ho = rem / g.cv_Wo, wo = rem - ho * g.cv_Wo;
              const int rs = k >> g.cv_logC, ci0 = k & ((1 << g.cv_logC) - 1);
              const int r = rs / g.cv_S, s = rs - r * g.cv_S;
              const int hh = ho * g.cv_stride - g.cv_pad + r, ww = wo * g.cv_stride - g.cv_pad + s;
              if ((unsigned)hh < (unsigned)g.cv_H && (unsigned)ww < (unsigned)g.cv_W)
                off = ((uint32_t)((n * g.cv_H + hh) * g.cv_W + ww) << (g.cv_logC - 5)) + ((uint32_t)ci0 >> 5);
            }
          } else {
            if (row < g.M) off = (uint32_t)row * kblk + kb;
          }
        } else if (isB) {
          const int col = n0s + (wid - 2) * 64 + lane;
          if (col < g.N) off = (uint32_t)col * kblk + kb;
        }
        __builtin_amdgcn_raw_ptr_buffer_load_lds(src, (__attribute__((address_space(3))) void*)(sc + wid * 256), 4, off,
                                                 0, 0, 0);
      }
    }
    if constexpr (GA) {
      const bool cur = m0 == cm0;  // tiles with equal m0 share their A rows
      const int rs = k >> g.cv_logC, ci0 = k & ((1 << g.cv_logC) - 1);
      const int r = rs / g.cv_S, s = rs - r * g.cv_S;
      const rsrc_t src = make_rsrc(g.A, g.cv_abytes);
      uint8_t* lds = half(u, h);
#pragma unroll
      for (int i = 0; i < P::PWA; ++i) {
        const int row = (i * 8 + wid) * 8 + (lane >> 3);
        const int c = (lane & 7) ^ ((row >> 1) & 7);
        const int p0 = cur ? cp0[h][i] : np0[h][i], hw = cur ? chw[h][i] : nhw[h][i];
        const int hh = (hw >> 16) + r, ww = ((int)((uint32_t)hw << 16) >> 16) + s;
        const bool ok = (unsigned)hh < (unsigned)g.cv_H && (unsigned)ww < (unsigned)g.cv_W;
        const uint32_t off = ok ? ((uint32_t)((p0 + r * g.cv_W + s) << g.cv_logC) + ci0) * ESZ + c * 16 : 0xFFFFFFF0u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(src, (__attribute__((address_space(3))) void*)(lds + (i * 8 + wid) * 1024),
                                                 16, off, 0, 0, 0);
      }
    } else {
      stage8<AK, ESZ, P::PWA>(g.A, bytesA, voA[h], g.lda, m0, k, half(u, h), wid);
    }
  };
  auto stB = [&](int u, int n0, int k, int h) {
    if constexpr (GB) {
      const rsrc_t src = make_rsrc(g.B, g.cv_abytes);
      uint8_t* lds = half(u, 2 + h);
      const int howo = g.cv_Ho * g.cv_Wo;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int kk = (i * 8 + wid) * 4 + (lane >> 4);  // this lane's k-row (pixel) of the K-tile
        const int f = (kk & 3) | ((kk >> 1) & 4);
        const int col = ((lane & 15) * 8) ^ (f << 4);
        const int n = n0 + (BC ? h * 128 + col : half_to_tile<32>(col, h));  // (r, s, ci) column of dW
        const int rs = n >> g.cv_logC, ci = n & ((1 << g.cv_logC) - 1);
        const int r = rs / g.cv_S, sx = rs - r * g.cv_S;
        const int pix = k + kk;                           // output pixel
        const int img = pix / howo, rem = pix - img * howo;
        const int ho = rem / g.cv_Wo, wo = rem - ho * g.cv_Wo;
        const int hi = ho * g.cv_stride - g.cv_pad + r, wi = wo * g.cv_stride - g.cv_pad + sx;
        const bool ok = n < g.N && pix < g.K && (unsigned)hi < (unsigned)g.cv_H && (unsigned)wi < (unsigned)g.cv_W;
        const uint32_t off = ok ? ((uint32_t)(((img * g.cv_H + hi) * g.cv_W + wi) << g.cv_logC) + ci) * 2 : 0xFFFFFFF0u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(src, (__attribute__((address_space(3))) void*)(lds + (i * 8 + wid) * 1024),
                                                 16, off, 0, 0, 0);
      }
    } else {
      stage8<BKM, ESZ, 2>(g.B, bytesB, voB[h], g.ldb, n0, k, half(u, 2 + h), wid);
    }
  };
  if (nt > 0) {
    const int k1 = kbeg + min(1, nt - 1) * KT;  // nt = 1: a split of one K-tile re-stages it
    stB(0, cn0, kbeg, 0);
    stA(0, cm0, kbeg, 0, cn0);
    stB(0, cn0, kbeg, 1);
    stA(0, cm0, kbeg, 1, cn0);
    stB(1, cn0, k1, 0);
    stA(1, cm0, k1, 0, cn0);
    stB(1, cn0, k1, 1);
    wait_vm<P::VM>();  // tile 0 landed (this wave's DMA)
  }
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();  // wave row 1 runs one barrier behind
  __builtin_amdgcn_sched_barrier(0);

  // register subtiles: bf16 [row block][k-step] x 8 elements, or fp8 [row block] x 32 bytes
  bf16x8 a0[IM][2], a1[IM][2], b0[2][2], b1[2][2];
  i32x8 fa0[IM], fa1[IM], fb0[2], fb1[2];
  auto readA = [&](const uint8_t* h, bf16x8 (&a)[IM][2], i32x8 (&fa)[IM]) {
    if constexpr (F8) {
#pragma unroll
      for (int i = 0; i < IM; ++i) fa[i] = frag8_f8(h, wr * IM + i, lane);
    } else {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < IM; ++i) a[i][ks] = frag8<AK>(h, wr * IM + i, ks, lane);
    }
  };
  auto readB = [&](const uint8_t* h, bf16x8 (&b)[2][2], i32x8 (&fb)[2]) {
    if constexpr (F8) {
#pragma unroll
      for (int j = 0; j < 2; ++j) fb[j] = frag8_f8(h, wc * 2 + j, lane);
    } else {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int j = 0; j < 2; ++j) b[j][ks] = frag8<BKM>(h, wc * 2 + j, ks, lane);
    }
  };
  // one C quadrant x one K-tile: 8*IM bf16 MFMA (k-step outer: independent accumulators between
  // dependent issues) or 4*IM fp8 MX MFMA
  // MX: this lane's E8M0 scales of the current K-tile -- A [half][row block], B [half][col block];
  // lane (16 b + r) supplies block b (K bytes [32b, 32b+32)) of row / column r of its fragment
  // (tools/probes/mx_probe.hip)
  int sa[2][IM], sb[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int i = 0; i < IM; ++i) sa[h][i] = 127;
    sb[h][0] = sb[h][1] = 127;
  }
  auto readS = [&](int u) {
    if constexpr (MX) {
      const uint8_t* sc = smem + (u & 1) * P::BUF + 2 * P::HA + 2 * P::HB;
      const int b = lane >> 4, r = lane & 15;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int i = 0; i < IM; ++i) sa[h][i] = sc[half_to_tile<P::QA>((wr * IM + i) * 16 + r, h) * 4 + b];
#pragma unroll
        for (int j = 0; j < 2; ++j) sb[h][j] = sc[512 + half_to_tile<32>((wc * 2 + j) * 16 + r, h) * 4 + b];
      }
    }
  };
  auto quad = [&](int q, bf16x8 (&a)[IM][2], bf16x8 (&b)[2][2], i32x8 (&fa)[IM], i32x8 (&fb)[2]) {
    if constexpr (F8) {
#pragma unroll
      for (int i = 0; i < IM; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[(q * IM + i) * 2 + j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
              fa[i], fb[j], acc[(q * IM + i) * 2 + j], F8A, 0, 0, sa[q >> 1][i], 0, sb[q & 1][j]);
    } else {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < IM; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[(q * IM + i) * 2 + j] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][ks], b[j][ks], acc[(q * IM + i) * 2 + j], 0, 0, 0);
    }
  };
  // A reads of phase 0 (issued after the B reads): what may stay in flight at its lgkmcnt
  constexpr int kAReads = (AK ? 2 : 4) * IM;
  // epilogue geometry: 16x16 C layout, col = lane&15, row = 4*(lane>>4) + r; after quad_t4 every
  // lane owns 4 consecutive columns of one row
  const int cl = lane & 15, rq = (lane >> 4) * 4;
  const int L = cl & 3;
  auto mrow = [&](int qm, int i) { return wr * (BM / 2) + qm * P::QA + i * 16 + rq + L; };
  auto ncol = [&](int qn, int j) { return (BC ? qn * 128 + wc * 32 : wc * 64 + qn * 32) + j * 16 + (cl & ~3); };

  // VMEM stores of one tile's epilogue, per lane, in both output paths (exact: every store is
  // issued unconditionally, out-of-range rows/cols go to an offset outside the buffer descriptor)
  constexpr int kEpiStores = 8 * IM + (ST ? 8 : 0) + (CT ? 8 * IM : 0);  // CT: C and aux per block
  // One K-tile of the 8-phase schedule at stream index u (= base + t); (am1, ak1) is the A source
  // of K-tile u+1, (am2, bn2, ak2) the A/B sources of K-tile u+2. first: the K-tile right after an
  // epilogue, whose phase-0 DMA was issued before the epilogue's stores; its phase-3 wait leaves
  // those stores in flight (they are older than K-tile u+2's DMA only)
  auto kstep = [&](int u, int am1, int ak1, int am2, int bn2, int ak2, bool first) {
    // ---- phase 0: q(0,0)
    readS(u);  // (before the B reads: retired by the same lgkmcnt wait)
    readB(half(u, 2), b0, fb0);
    __builtin_amdgcn_sched_barrier(0);
    readA(half(u, 0), a0, fa0);
    if (!first) stA(u + 1, am1, ak1, 1, 0);
    wait_lgkm<kAReads>();  // retires every B(qn0) read (lgkmcnt saturates at 15)
    __builtin_amdgcn_sched_barrier(0);
    PSD_SYNC_OPEN()
    quad(0, a0, b0, fa0, fb0);
    PSD_SYNC_CLOSE()
    // ---- phase 1: q(0,1)
    readB(half(u, 3), b1, fb1);
    stB(u + 2, bn2, ak2, 0);
    __builtin_amdgcn_sched_barrier(0);
    PSD_SYNC_OPEN()
    quad(1, a0, b1, fa0, fb1);
    PSD_SYNC_CLOSE()
    // ---- phase 2: q(1,0)
    readA(half(u, 1), a1, fa1);
    stA(u + 2, am2, ak2, 0, bn2);
    __builtin_amdgcn_sched_barrier(0);
    PSD_SYNC_OPEN()
    quad(2, a1, b0, fa1, fb0);
    PSD_SYNC_CLOSE()
    // ---- phase 3: q(1,1)
    stB(u + 2, bn2, ak2, 1);
    if (first)
      wait_vm<P::VM + kEpiStores>();  // K-tile u+1 complete; the epilogue stores may still drain
    else
      wait_vm<P::VM>();  // K-tile u+1 complete (its A-half1 was staged in phase 0)
    __builtin_amdgcn_sched_barrier(0);
    PSD_SYNC_OPEN()
    quad(3, a1, b1, fa1, fb1);
    PSD_SYNC_CLOSE()
  };

  // output descriptors (host contract: extents < 2^32 bytes, N % 8 == 0, ldc % 8 == 0)
  constexpr uint32_t kOOB = 0xFFFFFFF0u;  // an offset past every descriptor's range: store dropped
  const bool f32out = MODE == 1 || g.c_f32;
  uint8_t* cbase = reinterpret_cast<uint8_t*>(g.C) + (MODE == 1 ? (int64_t)blockIdx.z * g.M * g.N * 4 : 0);
  const int ldo = MODE == 1 ? g.N : g.ldc;
  const uint32_t cbytes = CT ? ((uint32_t)(g.N - 1) * ldo + g.M) * (f32out ? 4 : 2)
                              : ((uint32_t)(g.M - 1) * ldo + g.N) * (f32out ? 4 : 2);
  const bool want_aux = MODE == 0 && ACT == 2 && g.aux;
  uint8_t* stg = smem + 2 * P::BUF + wid * P::STG;  // this wave's epilogue staging slot
  float fmul = 1.f;
  if constexpr (F8 && !MX) {
    fmul = *g.a_scale * *g.b_scale;
    asm volatile("" ::"v"(fmul));  // materialise now (a load left to the epilogue would drain the DMA there)
  }

  for (; jt < ntl; ++jt) {
    // bias of the wave's 64 columns -> the head of its (idle) staging slot by LDS-DMA, 4 B per lane
    // (columns past N load zeros); retired by the K loop's own counted waits (older than its DMA,
    // nt >= 2) and read back at the epilogue. A register load would make the compiler wait for it,
    // and with it every older store and DMA, right here.
    if (MODE == 0 && g.bias) {
      if constexpr (CT)  // the bias of the wave row's BM / 2 C rows (lanes past them: never read)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(make_rsrc(g.bias, (uint32_t)g.M * 2),
                                                 (__attribute__((address_space(3))) void*)stg, 4,
                                                 (uint32_t)(cm0 + wr * (BM / 2) + 2 * lane) * 2, 0, 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(make_rsrc(g.bias, (uint32_t)g.N * 2),
                                                 (__attribute__((address_space(3))) void*)stg, 4,
                                                 (uint32_t)(cn0 + wc * 64 + 2 * lane) * 2, 0, 0, 0);
    }
    if constexpr (ST)  // the statistics shift of the wave's 64 columns -> staging slot bytes 256..511
      __builtin_amdgcn_raw_ptr_buffer_load_lds(make_rsrc(g.shift, (uint32_t)g.N * 4),
                                               (__attribute__((address_space(3))) void*)(stg + 256), 4,
                                               (uint32_t)(cn0 + wc * 64 + lane) * 4, 0, 0, 0);
    // K-tiles nt, nt+1 of this tile's stream = the next tile's first two K-tiles (past the
    // workgroup's last tile: the last valid K-tile again, same DMA count, never read)
    const bool more = jt + 1 < ntl;
    const int sm0 = more ? xm0 : cm0, sn0 = more ? xn0 : cn0;
    const int sk0 = more ? kbeg : kbeg + max(nt - 1, 0) * KT;
    const int sk1 = more ? kbeg + min(1, nt - 1) * KT : sk0;
    for (int t = 0; t < nt; ++t) {  // uniform scalar selects, no branches in the K loop
      const int d1 = t + 1 - nt, d2 = t + 2 - nt;
      const int am1 = d1 >= 0 ? sm0 : cm0;
      const int ak1 = d1 >= 0 ? sk0 : kbeg + (t + 1) * KT;
      const int am2 = d2 >= 0 ? sm0 : cm0, bn2 = d2 >= 0 ? sn0 : cn0;
      const int ak2 = d2 > 0 ? sk1 : (d2 == 0 ? sk0 : kbeg + (t + 2) * KT);
      kstep(base + t, am1, ak1, am2, bn2, ak2, jt > 0 && t == 0);
    }
    // the next tile's first K-tile issues its phase-0 DMA (A-half1 of its K-tile 1) here, BEFORE
    // the stores below, so that its phase-3 wait can leave the stores in flight (nt >= 2 whenever
    // a workgroup has more than one tile)
    if (more) stA(base + nt + 1, xm0, kbeg + KT, 1, 0);

    // ---- epilogue of tile jt (no barrier: the pipeline LDS already holds the next tile)
    float bv[2][2] = {{0.f, 0.f}, {0.f, 0.f}};
    if (!CT && MODE == 0 && g.bias) {
#pragma unroll
      for (int qn = 0; qn < 2; ++qn)
#pragma unroll
        for (int j = 0; j < 2; ++j) bv[qn][j] = bf16_to_f32(reinterpret_cast<const uint16_t*>(stg)[qn * 32 + j * 16 + cl]);
    }
    if constexpr (F8 && !MX) {
#pragma unroll
      for (int i = 0; i < 8 * IM; ++i) acc[i] *= fmul;
    }
    const rsrc_t rc = make_rsrc(cbase, cbytes);
    if constexpr (CT) {
      // Y[n][m] = C[m][n]: per 16x16 block the lane's 4 accumulators are C rows rq..rq+3 of column
      // cl = 4 contiguous Y elements (g.M % 4 == 0: all valid or none); every store is issued (the
      // aux store against an empty descriptor when there is none), as the count kEpiStores assumes
      const bool has_bias = g.bias != nullptr;
      const rsrc_t ra = make_rsrc(want_aux ? g.aux : g.C, want_aux ? cbytes : 0u);
      const uint16_t* bst = reinterpret_cast<const uint16_t*>(stg);
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int i = 0; i < IM; ++i) {
          const int mloc = (q >> 1) * P::QA + i * 16 + rq;  // within the wave row's BM / 2 rows
          const int m = cm0 + wr * (BM / 2) + mloc;
          float b4[4] = {0.f, 0.f, 0.f, 0.f};
          if (has_bias) {
#pragma unroll
            for (int r = 0; r < 4; ++r) b4[r] = bf16_to_f32(bst[mloc + r]);
          }
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int n = cn0 + wc * 64 + (q & 1) * 32 + j * 16 + cl;
            const f32x4 a = acc[(q * IM + i) * 2 + j];
            float w[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) w[r] = a[r] + b4[r];
            const bool ok = m < g.M && n < g.N;
            if (f32out) {
              float o[4];
#pragma unroll
              for (int r = 0; r < 4; ++r) o[r] = act_apply<ACT>(w[r]);
              const uint32_t off = ok ? ((uint32_t)n * ldo + m) * 4 : kOOB;
              __builtin_amdgcn_raw_buffer_store_b128(
                  u32x4{__float_as_uint(o[0]), __float_as_uint(o[1]), __float_as_uint(o[2]), __float_as_uint(o[3])},
                  rc, off, 0, 0);
              __builtin_amdgcn_raw_buffer_store_b128(u32x4{0u, 0u, 0u, 0u}, ra, kOOB, 0, 0);
            } else {
              const uint32_t off = ok ? ((uint32_t)n * ldo + m) * 2 : kOOB;
              typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
              __builtin_amdgcn_raw_buffer_store_b64(u32x2_t{pack_bf16x2(w[0], w[1]), pack_bf16x2(w[2], w[3])}, ra,
                                                    want_aux ? off : kOOB, 0, 0);
              float o[4];
#pragma unroll
              for (int r = 0; r < 4; ++r) o[r] = act_apply<ACT>(w[r]);
              __builtin_amdgcn_raw_buffer_store_b64(u32x2_t{pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3])}, rc, off,
                                                    0, 0);
            }
          }
        }
    } else if (f32out) {  // fp32: 16-byte row segments straight from registers
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int n = cn0 + ncol(q & 1, j);
#pragma unroll
          for (int i = 0; i < IM; ++i) {
            float w[4];
            quad_t4(acc[(q * IM + i) * 2 + j] + bv[q & 1][j], L, w);
            const int m = cm0 + mrow(q >> 1, i);
#pragma unroll
            for (int e = 0; e < 4; ++e) w[e] = act_apply<ACT>(w[e]);
            const uint32_t off = (m < g.M && n < g.N) ? ((uint32_t)m * ldo + n) * 4 : kOOB;
            __builtin_amdgcn_raw_buffer_store_b128(
                u32x4{__float_as_uint(w[0]), __float_as_uint(w[1]), __float_as_uint(w[2]), __float_as_uint(w[3])},
                rc, off, 0, 0);
          }
        }
    } else {
      // bf16: each wave stages its 128x64 (BM 256) / 64x64 C block 16 rows at a time through its
      // own 4 KiB of LDS (no barrier: one wave's LDS ops complete in order), so the global stores
      // are 16-byte lanes covering whole 128-byte row segments. Staging image: [16 rows][128 B],
      // 8-byte column group g stored at g ^ 2*(row & 7) (conflict-spreading; keeps 16-byte pairs).
      // The GELU pre-activation (aux) goes through the second 2 KiB; without aux its stores are
      // issued against an empty descriptor (dropped) to keep the store count exact.
      const rsrc_t ra = make_rsrc(want_aux ? g.aux : g.C, want_aux ? cbytes : 0u);
      const int rrow = lane >> 3, c16 = lane & 7;  // read side: 8 rows x 8 16-byte chunks per pass
      // ST: per lane, the plain sums sum y and sum y^2 of its 4 columns (qn, j) over its rows, on the
      // fp32 accumulators before the transpose (column cl, 4 consecutive rows per block), as packed
      // fp32 pairs (2 v_pk_add + 2 v_pk_fma per 16x16 block: the epilogue is not overlapped with the
      // MFMA pipeline, so every instruction here is paid per tile); shifted once per wave row at the end
      // (rows past M need no mask: their A rows load as zeros -- K-major A past the descriptor, or the
      // implicit GEMM's out-of-image sentinel -- so their accumulators are exactly 0)
      f32x2 t1[2][2], t2[2][2];
      float shk[2][2];  // the shift of this lane's 4 columns (read before the staging overwrites it)
      float gs[8];      // ACT 3: column sums of g over the lane's stored rows (8 columns c16*8..+7)
      // ACT 3: the tile's pre-activation, every 16-B piece this lane stores, loaded up front (one
      // wait for all of them -- a load per store would wait on the pipeline's DMA in flight each time)
      u32x4 pv[2][IM][2];
      if constexpr (ACT == 3) {
#pragma unroll
        for (int e = 0; e < 8; ++e) gs[e] = 0.f;
        const int n = cn0 + wc * 64 + c16 * 8;
#pragma unroll
        for (int qm = 0; qm < 2; ++qm)
#pragma unroll
          for (int i = 0; i < IM; ++i)
#pragma unroll
            for (int k = 0; k < 2; ++k) {
              const int m = cm0 + wr * (BM / 2) + qm * P::QA + i * 16 + k * 8 + rrow;
              pv[qm][i][k] = u32x4{0u, 0u, 0u, 0u};
              if (m < g.M && n < g.N)
                pv[qm][i][k] = *reinterpret_cast<const u32x4*>(reinterpret_cast<const uint16_t*>(g.aux) + (int64_t)m * ldo + n);
            }
      }
      if constexpr (ST) {
#pragma unroll
        for (int qn = 0; qn < 2; ++qn)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            shk[qn][j] = reinterpret_cast<const float*>(stg + 256)[qn * 32 + j * 16 + cl];
            t1[qn][j] = t2[qn][j] = f32x2{0.f, 0.f};
          }
      }
#pragma unroll
      for (int qm = 0; qm < 2; ++qm)
#pragma unroll
        for (int i = 0; i < IM; ++i) {
          const int r = rq + L;  // this lane's row within the 16-row block (after quad_t4)
#pragma unroll
          for (int qn = 0; qn < 2; ++qn)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              if constexpr (ST) {
                const f32x4 a = acc[((qm * 2 + qn) * IM + i) * 2 + j];
                const f32x2 lo = __builtin_shufflevector(a, a, 0, 1), hi = __builtin_shufflevector(a, a, 2, 3);
                t1[qn][j] += lo + hi;
                t2[qn][j] = __builtin_elementwise_fma(lo, lo, t2[qn][j]);
                t2[qn][j] = __builtin_elementwise_fma(hi, hi, t2[qn][j]);
              }
              float w[4];
              quad_t4(acc[((qm * 2 + qn) * IM + i) * 2 + j] + bv[qn][j], L, w);
              const int gcol = (qn * 32 + j * 16 + (cl & ~3)) >> 2;  // 8-byte group 0..15
              const int off = r * 128 + ((gcol ^ ((r & 7) << 1)) << 3);
              // inline-asm LDS writes: a plain store would make the compiler wait for every
              // LDS-DMA in flight (it cannot tell this slot from the pipeline buffers)
              const uint32_t la = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)(stg + off);
              if (want_aux) {
                const uint64_t pa = (uint64_t)pack_bf16x2(w[0], w[1]) | ((uint64_t)pack_bf16x2(w[2], w[3]) << 32);
                asm volatile("ds_write_b64 %0, %1 offset:2048" ::"v"(la), "v"(pa) : "memory");
              }
#pragma unroll
              for (int e = 0; e < 4; ++e) w[e] = act_apply<ACT>(w[e]);
              const uint64_t pc = (uint64_t)pack_bf16x2(w[0], w[1]) | ((uint64_t)pack_bf16x2(w[2], w[3]) << 32);
              asm volatile("ds_write_b64 %0, %1" ::"v"(la), "v"(pc) : "memory");
            }
          const int mb = cm0 + wr * (BM / 2) + qm * P::QA + i * 16;
          const int n = cn0 + wc * 64 + c16 * 8;
#pragma unroll
          for (int k = 0; k < 2; ++k) {
            const int rr = k * 8 + rrow;
            const int off = rr * 128 + (((2 * c16) ^ ((rr & 7) << 1)) << 3);
            const int m = mb + rr;
            u32x4 v = *reinterpret_cast<const u32x4*>(stg + off);
            const u32x4 va = *reinterpret_cast<const u32x4*>(stg + 2048 + off);
            const uint32_t go = (m < g.M && n < g.N) ? ((uint32_t)m * ldo + n) * 2 : kOOB;
            if constexpr (ACT == 3) {
              const u32x4 p = pv[qm][i][k];
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const float g0 = bf16_to_f32(f32_to_bf16(bf16_to_f32((uint16_t)(v[e] & 0xFFFFu)) *
                                                         gelu_tanh_grad(bf16_to_f32((uint16_t)(p[e] & 0xFFFFu)))));
                const float g1 = bf16_to_f32(f32_to_bf16(bf16_to_f32((uint16_t)(v[e] >> 16)) *
                                                         gelu_tanh_grad(bf16_to_f32((uint16_t)(p[e] >> 16)))));
                gs[2 * e] += g0;
                gs[2 * e + 1] += g1;
                v[e] = pack_bf16x2(g0, g1);
              }
            }
            __builtin_amdgcn_raw_buffer_store_b128(v, rc, go, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b128(va, ra, go, 0, 0);
          }
        }
      if constexpr (ACT == 3) {
        // lanes with equal c16 (lane bits 0..2) hold the same 8 columns: sum over lane bits 3..5,
        // lanes 0..7 store the wave row's partial row (rows past M / columns past N summed zeros)
        const int prow = (cm0 / BM) * 2 + wr;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          gs[e] += __shfl_xor(gs[e], 8, 64);
          gs[e] += __shfl_xor(gs[e], 16, 64);
          gs[e] += __shfl_xor(gs[e], 32, 64);
        }
        const int n = cn0 + wc * 64 + c16 * 8;
        if (lane < 8 && n < g.N) {
          float* pp = g.part + (int64_t)prow * g.N + n;
          *reinterpret_cast<f32x4*>(pp) = f32x4{gs[0], gs[1], gs[2], gs[3]};
          *reinterpret_cast<f32x4*>(pp + 4) = f32x4{gs[4], gs[5], gs[6], gs[7]};
        }
      }
      if constexpr (ST) {
        // lanes with equal cl hold the same 4 columns: sum over lane bits 4..5, lanes 0..15 store
        const int prow = (cm0 / BM) * 2 + wr;
        const int prows = (g.M + BM - 1) / BM * 2;
        const rsrc_t rp = make_rsrc(g.part, (uint32_t)prows * 2u * (uint32_t)g.N * 4u);
        // the wave row's valid rows, then sum (y - k) = S1 - c k, sum (y - k)^2 = S2 - k (2 S1 - c k)
        const float cnt = (float)max(0, min(BM / 2, g.M - (cm0 + wr * (BM / 2))));
#pragma unroll
        for (int qn = 0; qn < 2; ++qn)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            float a1 = t1[qn][j][0] + t1[qn][j][1], a2 = t2[qn][j][0] + t2[qn][j][1];
            a1 += st_xor16(a1, lane);
            a2 += st_xor16(a2, lane);
            a1 += st_xor32(a1, lane);
            a2 += st_xor32(a2, lane);
            const float k = shk[qn][j];
            a2 = fmaf(-k, fmaf(-cnt, k, 2.f * a1), a2);
            a1 = fmaf(-cnt, k, a1);
            const int n = cn0 + wc * 64 + qn * 32 + j * 16 + cl;
            const bool mine = lane < 16 && n < g.N;
            const uint32_t o1 = mine ? ((uint32_t)prow * 2u * (uint32_t)g.N + (uint32_t)n) * 4u : kOOB;
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(a1), rp, o1, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(a2), rp, mine ? o1 + (uint32_t)g.N * 4u : kOOB, 0, 0);
          }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // staging reads retired: clean lgkm count
#pragma unroll
    for (int i = 0; i < 8 * IM; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    base += nt;
    cm0 = xm0;
    cn0 = xn0;
    if (jt + 2 < ntl) origin(jt + 2, xm0, xn0);
    if constexpr (GA) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < P::PWA; ++i) cp0[h][i] = np0[h][i], chw[h][i] = nhw[h][i];
      if (jt + 2 < ntl) conv_rows(xm0, np0, nhw);
    }
  }
  if (wr == 0) __builtin_amdgcn_s_barrier();  // re-align the two wave rows
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
#undef PSD_SYNC_OPEN
#undef PSD_SYNC_CLOSE

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
constexpr int kColsumMaxBlocks = kColsumPartRows;  // partial rows (the caller's workspace: [kColsumPartRows * N] fp32)

// Column partial sums of x[M, N] (bias gradients). GELU: x = bf16(dy * gelu'(pre)) is computed on
// the fly from dy and the saved pre-activation, written to xo, and summed as written (the GELU
// backward and the bias gradient of a GELU Linear in one pass over dy / pre).
template <bool GELU>
__global__ __launch_bounds__(256) void colsum_partial_kernel(const uint16_t* __restrict__ x, int64_t M, int N,
                                                             float* __restrict__ part,
                                                             const uint16_t* __restrict__ pre = nullptr,
                                                             uint16_t* __restrict__ xo = nullptr) {
  const int tpc = N >> 3;
  const int rpi = tpc >= 256 ? 1 : 256 / tpc;
  const int cg = tpc >= 256 ? blockIdx.y * 256 + threadIdx.x : threadIdx.x % tpc;
  const int r0 = tpc >= 256 ? 0 : threadIdx.x / tpc;
  const bool active = cg < tpc && r0 < rpi;
  float a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (active) {
    const int64_t stride = (int64_t)gridDim.x * rpi;
    int64_t r = (int64_t)blockIdx.x * rpi + r0;
    auto get = [&](int64_t row, float (&t)[8]) {
      load8_bf16(x + row * N + cg * 8, t);
      if constexpr (GELU) {
        float p[8];
        load8_bf16(pre + row * N + cg * 8, p);
#pragma unroll
        for (int e = 0; e < 8; ++e) t[e] = bf16_to_f32(f32_to_bf16(t[e] * gelu_tanh_grad(p[e])));
        store8_bf16(xo + row * N + cg * 8, t);
      }
    };
    for (; r + 3 * stride < M; r += 4 * stride) {
      float t[4][8];
#pragma unroll
      for (int u = 0; u < 4; ++u) get(r + u * stride, t[u]);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int e = 0; e < 8; ++e) a[e] += t[u][e];
    }
    for (; r < M; r += stride) {
      float t[8];
      get(r, t);
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

// Deterministic second pass: block = 8 columns x 128 partial-row lanes (1024 lanes), 4 independent
// accumulators per lane (a lane's loads are independent: ~nblk/512 round trips instead of a
// nblk/8-deep dependent chain), then the 128 lanes of a column are combined in LDS in a fixed order.
__global__ __launch_bounds__(1024) void colsum_final_kernel(const float* __restrict__ part, int nblk, int N, void* out,
                                                            int out_bf16, int accumulate) {
  const int cl = threadIdx.x & 7, rl = threadIdx.x >> 3;
  const int c = blockIdx.x * 8 + cl;
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  if (c < N) {
    int b = rl;
    for (; b + 384 < nblk; b += 512)
#pragma unroll
      for (int u = 0; u < 4; ++u) s[u] += part[(int64_t)(b + 128 * u) * N + c];
    for (; b < nblk; b += 128) s[0] += part[(int64_t)b * N + c];
  }
  __shared__ float red[128][9];
  __shared__ float red2[8][9];
  red[rl][cl] = (s[0] + s[1]) + (s[2] + s[3]);
  __syncthreads();
  if (rl < 8) {  // 8 x 8 lanes: each sums 16 of the 128 row lanes of one column
    float t = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) t += red[rl * 16 + r][cl];
    red2[rl][cl] = t;
  }
  __syncthreads();
  if (rl != 0 || c >= N) return;
  float t = red2[0][cl];
#pragma unroll
  for (int r = 1; r < 8; ++r) t += red2[r][cl];
  if (out_bf16) {
    uint16_t* o = reinterpret_cast<uint16_t*>(out);
    o[c] = f32_to_bf16(t + (accumulate ? bf16_to_f32(o[c]) : 0.f));
  } else {
    float* o = reinterpret_cast<float*>(out);
    o[c] = t + (accumulate ? o[c] : 0.f);
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

static int cu_count() {
  static const int n = [] {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      return 256;
    return cus;
  }();
  return n;
}

// workgroups of the persistent 8-phase grid: one per CU (the kernel's LDS allows no second)
static int persistent_grid() { return cu_count(); }

// contiguous B halves for the split-K GEMMs with an N-major B (weight gradients); g_bc: off for A/Bs
static bool g_bc = false;  // measured no faster on the BERT weight gradients (profiles/r6/gemm_probe_bert_r6b.md: TN vs TN0)
void gemm_set_bcontig(bool on) { g_bc = on; }

template <int BM, bool AK, bool BKM, int MODE, bool F8, int ACT, bool GA = false, int F8A = 0, bool GB = false,
          bool MX = false, bool ST = false, bool CT = false, bool BC = false>
static hipError_t launch_8p_act(const GemmArgs& g, int splits, hipStream_t st) {
  if constexpr (MODE == 1 && !BKM && !BC) {
    if (g_bc) return launch_8p_act<BM, AK, BKM, MODE, F8, ACT, GA, F8A, GB, MX, ST, CT, true>(g, splits, st);
  }
  if constexpr (ACT == 3) {  // GELU backward + bias-gradient partials (g.aux = pre, g.part = [rows][N])
    if (!g.part || !g.aux || g.c_f32 || g.bias || splits != 1) return hipErrorNotSupported;
    if (g.rows_out) *g.rows_out = (g.M + BM - 1) / BM * 2;
  } else if constexpr (!ST) {
    if (g.part) {  // the consumer BN's statistics in the epilogue
      if constexpr (MODE == 0 && !GB && ACT == 0 && AK && !CT && BM != 192) {
        if (g.c_f32 || g.bias || !g.shift || splits != 1) return hipErrorNotSupported;
        if (g.rows_out) *g.rows_out = (g.M + BM - 1) / BM * 2;
        return launch_8p_act<BM, AK, BKM, MODE, F8, ACT, GA, F8A, GB, MX, true>(g, splits, st);
      } else {
        return hipErrorNotSupported;
      }
    }
  }
  constexpr int lds = P8<BM, MX>::LDS;
  static bool attr_set = false;  // per instantiation: set the >64 KiB LDS limit once
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)gemm8p_kernel<BM, AK, BKM, MODE, F8, ACT, GA, F8A, GB, MX, ST, CT, BC>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const int nwg = ((g.M + BM - 1) / BM) * ((g.N + kBig - 1) / kBig);
  // persistent grid (one workgroup per CU) for the single-split GEMMs; the kernel needs >= 2
  // K-tiles per tile to run tiles back to back (big_ok guarantees K >= 256)
  constexpr int KT = F8 ? 128 : BK;
  int grid = nwg;
  if (MODE == 0 && splits == 1 && g.K / KT >= 2) grid = std::min(nwg, persistent_grid());
  hipLaunchKernelGGL((gemm8p_kernel<BM, AK, BKM, MODE, F8, ACT, GA, F8A, GB, MX, ST, CT, BC>), dim3(grid, 1, splits),
                     dim3(512), lds, st, g);
  return hipGetLastError();
}

template <int BM, bool AK, bool BKM, int MODE, bool F8 = false>
static hipError_t launch_8p(const GemmArgs& g, int splits, hipStream_t st) {
  if constexpr (MODE == 0) {
    if (g.act == 1) return launch_8p_act<BM, AK, BKM, MODE, F8, 1>(g, splits, st);
    if (g.act == 2) return launch_8p_act<BM, AK, BKM, MODE, F8, 2>(g, splits, st);
    if constexpr (!F8) {
      if (g.act == 3) return launch_8p_act<BM, AK, BKM, MODE, F8, 3>(g, splits, st);
    }
  }
  if (g.act == 3) return hipErrorNotSupported;
  return launch_8p_act<BM, AK, BKM, MODE, F8, 0>(g, splits, st);
}

// 8-phase tile height: a 128x256 tile costs ~0.55 of a 256x256 one, so narrow problems (few
// 256-tiles: wave quantisation over 256 CUs) take BM = 128 when that finishes in fewer rounds.
// (BM = 128 needs a K-major A: its M-major half image would be 64 columns wide)
static int pick_bm(int M, int N, int splits, bool a_kmajor = true) {
  if (!a_kmajor) return 256;
  const int64_t tn = (N + 255) / 256;
  const int64_t t256 = (int64_t)((M + 255) / 256) * tn * splits;
  const int64_t t128 = (int64_t)((M + 127) / 128) * tn * splits;
  const double c256 = (double)((t256 + 255) / 256);
  const double c128 = 0.55 * (double)((t128 + 255) / 256);
  return (M >= 128 && c128 < c256) ? 128 : 256;
}

template <bool AK, bool BKM, int MODE>
static hipError_t launch_big(const GemmArgs& g, int splits, hipStream_t st) {
  if constexpr (AK) {
    if (pick_bm(g.M, g.N, splits) == 128) return launch_8p<128, AK, BKM, MODE>(g, splits, st);
  }
  return launch_8p<256, AK, BKM, MODE>(g, splits, st);
}

// the 8-phase kernel addresses each operand through a buffer descriptor with 32-bit byte offsets
static bool fits_rsrc(const GemmArgs& g, int esz) {
  const int64_t a = g.a_kmajor ? (int64_t)(g.M - 1) * g.lda + g.K : (int64_t)(g.K - 1) * g.lda + g.M;
  const int64_t b = g.b_kmajor ? (int64_t)(g.N - 1) * g.ldb + g.K : (int64_t)(g.K - 1) * g.ldb + g.N;
  const int64_t c = (int64_t)(g.M - 1) * (g.k_per_split > 0 ? g.N : g.ldc) + g.N;  // C / one split-K slab
  return a * esz < (int64_t)1 << 32 && b * esz < (int64_t)1 << 32 && c * 4 < (int64_t)1 << 32;
}

static bool big_ok(const GemmArgs& g, int kseg) {
  // enough big tiles to fill the chip, no K tail inside a stage, MN-major operands 8-aligned
  if (!fits_rsrc(g, 2)) return false;
  // 8-phase epilogue: 16-byte stores of 8 bf16 / 4 fp32 columns, whole or dropped
  if (g.N % 8 != 0 || (g.k_per_split == 0 && g.ldc % 8 != 0)) return false;
  if (reinterpret_cast<uintptr_t>(g.bias) & 3) return false;  // bias: dword LDS-DMA
  const int splits = g.k_per_split > 0 ? (g.K + g.k_per_split - 1) / g.k_per_split : 1;
  // 8-phase: BM 128 or 256, BN 256
  const int bm = pick_bm(g.M, g.N, splits, g.a_kmajor);
  const int64_t tiles = (int64_t)((g.M + bm - 1) / bm) * ((g.N + 255) / 256) * splits;
  return g.M >= 128 && g.N >= 256 && kseg % 64 == 0 && tiles >= 64 && g.K >= 256;
}

template <bool AK, bool BKM, int MODE>
static hipError_t launch_layout(const GemmArgs& g, int splits, hipStream_t st) {
  // (the 8-phase K loop runs whole 64-k tiles: a K tail -- the last split's, in MODE 1 -- would be
  // dropped, and a K-major operand reads the next row past K, so K % 64 != 0 takes the 128-tile kernel)
  if (big_ok(g, MODE == 1 ? g.k_per_split : g.K) && g.K % 64 == 0) return launch_big<AK, BKM, MODE>(g, splits, st);
  if (g.part) return hipErrorNotSupported;  // statistics: the 8-phase epilogue only
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

// Y[N][M] (row stride g.ldc) = (A . B^T)^T (+ bias[M])(act) on 192 x 256 tiles (A rows x B rows):
// Y = X W^T + b with A = W [M = out][K], B = X [N = tokens][K], both K-major.
hipError_t launch_gemm_ct(const GemmArgs& g, hipStream_t st) {
  if (g.M <= 0 || g.N <= 0) return hipSuccess;
  const int64_t ab = ((int64_t)(g.M - 1) * g.lda + g.K) * 2, bb = ((int64_t)(g.N - 1) * g.ldb + g.K) * 2;
  const int64_t cb = ((int64_t)(g.N - 1) * g.ldc + g.M) * (g.c_f32 ? 4 : 2);
  const bool ok = g.a_kmajor && g.b_kmajor && g.M % 8 == 0 && g.ldc % 8 == 0 && g.K % 64 == 0 && g.K >= 128 &&
                  g.act >= 0 && g.act <= 2 && !g.part && !(g.aux && g.c_f32) && ab < ((int64_t)1 << 31) &&
                  bb < ((int64_t)1 << 32) && cb < ((int64_t)1 << 32) && !(reinterpret_cast<uintptr_t>(g.bias) & 3);
  if (!ok) return hipErrorNotSupported;
  if (g.act == 1) return launch_8p_act<192, true, true, 0, false, 1, false, 0, false, false, false, true>(g, 1, st);
  if (g.act == 2) return launch_8p_act<192, true, true, 0, false, 2, false, 0, false, false, false, true>(g, 1, st);
  return launch_8p_act<192, true, true, 0, false, 0, false, 0, false, false, false, true>(g, 1, st);
}

hipError_t launch_conv_fwd(const GemmArgs& g, hipStream_t st) {
  if (g.M <= 0 || g.N <= 0) return hipSuccess;
  const int C = 1 << g.cv_logC;
  const int64_t xbytes = (int64_t)g.cv_abytes;
  const bool ok = g.a_kmajor && g.b_kmajor && g.cv_logC >= 6 && g.K % C == 0 && g.K % 64 == 0 &&
                  g.M >= 128 && g.N >= 256 && g.N % 8 == 0 && g.ldc % 8 == 0 && !g.bias && g.act == 0 &&
                  (int64_t)(g.N - 1) * g.ldb + g.K < ((int64_t)1 << 31) && xbytes > 0 &&
                  (int64_t)(g.M - 1) * g.ldc + g.N < ((int64_t)1 << 31) && g.cv_S > 0 && g.cv_W < 32768 &&
                  g.cv_H < 32768;
  if (!ok) return hipErrorNotSupported;
  return pick_bm(g.M, g.N, 1) == 128 ? launch_8p_act<128, true, true, 0, false, 0, true>(g, 1, st)
                                     : launch_8p_act<256, true, true, 0, false, 0, true>(g, 1, st);
}

// fp8 implicit-GEMM forward: x and w OCP e4m3 (C % 128 == 0: one (r, s) per 128-wide K-tile),
// dequantised by *a_scale * *b_scale in the epilogue (bf16 out)
hipError_t launch_conv_fwd_fp8(const GemmArgs& g, hipStream_t st) {
  if (g.M <= 0 || g.N <= 0) return hipSuccess;
  const int C = 1 << g.cv_logC;
  const bool mx = g.a_mx && g.b_mx;
  const bool ok = g.a_kmajor && g.b_kmajor && g.cv_logC >= 7 && g.K % C == 0 && g.K % 128 == 0 && g.K >= 256 &&
                  g.M >= 128 && g.N >= 256 && g.N % 8 == 0 && g.ldc % 8 == 0 && !g.bias && g.act == 0 && !g.c_f32 &&
                  ((g.a_scale && g.b_scale) || (mx && g.ldb == g.K)) &&
                  (int64_t)(g.N - 1) * g.ldb + g.K < ((int64_t)1 << 31) &&
                  g.cv_abytes > 0 && (int64_t)(g.M - 1) * g.ldc + g.N < ((int64_t)1 << 31) && g.cv_S > 0 &&
                  g.cv_W < 32768 && g.cv_H < 32768;
  if (!ok) return hipErrorNotSupported;
  // 128-row tiles always: WRN-101-2 b512 A/B on two boxes, 3,443 vs 3,313 and 3,806 / 3,779 vs
  // 3,749 img/s against the bf16-calibrated pick_bm (the fp8 tile is LDS/DMA-bound, so the taller
  // tile's extra reuse buys less than its wave quantisation costs)
  if (mx)  // block-scaled: 128-row tiles (the scale staging needs the LDS a 256-row tile leaves no room for)
    return g.f8a == 1 ? launch_8p_act<128, true, true, 0, true, 0, true, 1, false, true>(g, 1, st)
                      : launch_8p_act<128, true, true, 0, true, 0, true, 0, false, true>(g, 1, st);
  if (g.f8a == 1) return launch_8p_act<128, true, true, 0, true, 0, true, 1>(g, 1, st);
  return launch_8p_act<128, true, true, 0, true, 0, true>(g, 1, st);
}

hipError_t launch_gemm_fp8(const GemmArgs& g, hipStream_t st) {
  if (g.M <= 0 || g.N <= 0) return hipSuccess;
  if (g.a_mx || g.b_mx) {  // block-scaled (MX): 128-row tiles
    if (!g.a_mx || !g.b_mx || g.K % 128 != 0 || !g.a_kmajor || !g.b_kmajor || g.lda != g.K || g.ldb != g.K ||
        !fits_rsrc(g, 1) || g.N % 8 != 0 || g.ldc % 8 != 0 || (reinterpret_cast<uintptr_t>(g.bias) & 3))
      return hipErrorInvalidValue;
    if (g.f8a == 1) {
      if (g.bias || g.act) return hipErrorInvalidValue;
      return launch_8p_act<128, true, true, 0, true, 0, false, 1, false, true>(g, 1, st);
    }
    if (g.act == 1) return launch_8p_act<128, true, true, 0, true, 1, false, 0, false, true>(g, 1, st);
    if (g.act == 2) return launch_8p_act<128, true, true, 0, true, 2, false, 0, false, true>(g, 1, st);
    return launch_8p_act<128, true, true, 0, true, 0, false, 0, false, true>(g, 1, st);
  }
  if (g.K % 128 != 0 || !g.a_kmajor || !g.b_kmajor || !g.a_scale || !g.b_scale || !fits_rsrc(g, 1) ||
      g.N % 8 != 0 || g.ldc % 8 != 0 || (reinterpret_cast<uintptr_t>(g.bias) & 3))
    return hipErrorInvalidValue;
  if (g.f8a == 1) {  // e5m2 A (fp8 bwd-data): no bias / activation
    if (g.bias || g.act) return hipErrorInvalidValue;
    return pick_bm(g.M, g.N, 1) == 128 ? launch_8p_act<128, true, true, 0, true, 0, false, 1>(g, 1, st)
                                       : launch_8p_act<256, true, true, 0, true, 0, false, 1>(g, 1, st);
  }
  return pick_bm(g.M, g.N, 1) == 128 ? launch_8p<128, true, true, 0, true>(g, 1, st)
                                     : launch_8p<256, true, true, 0, true>(g, 1, st);
}

// Implicit-GEMM convolution weight gradient: out[Cout][R*S*C] (bf16) = dY^T . im2col(x), split-K over
// the output pixels into fp32 slabs, then the deterministic slab reduce. g: A = dY [pixels][Cout]
// (lda = Cout), B = x (NHWC), M = Cout, N = R*S*C, K = pixels, cv_* the convolution geometry.
hipError_t launch_conv_wgrad(const GemmArgs& g0, float* slab, int splits, void* out, hipStream_t st) {
  if (g0.M <= 0 || g0.N <= 0) return hipSuccess;
  const bool ok = !g0.a_kmajor && !g0.b_kmajor && g0.cv_logC >= 3 && g0.N % (1 << g0.cv_logC) == 0 &&
                  g0.M >= 256 && g0.M % 8 == 0 && g0.N >= 256 && g0.N % 8 == 0 && g0.K >= 128 &&
                  g0.cv_abytes > 0 && g0.cv_S > 0 && g0.cv_W < 32768 && g0.cv_H < 32768 && splits >= 1 &&
                  (int64_t)(g0.K - 1) * g0.lda + g0.M < ((int64_t)1 << 31);
  if (!ok) return hipErrorNotSupported;
  GemmArgs g = g0;
  g.C = slab;
  int kps = (g.K + splits - 1) / splits;
  kps = (kps + 2 * BK - 1) / (2 * BK) * (2 * BK);  // >= 2 K-tiles per split, whole K-tiles
  g.k_per_split = kps;
  const int eff = (g.K + kps - 1) / kps;
  hipError_t e = launch_8p_act<256, false, false, 1, false, 0, false, 0, true>(g, eff, st);
  if (e != hipSuccess) return e;
  const int64_t mn = (int64_t)g.M * g.N;
  hipLaunchKernelGGL(splitk_reduce_kernel<true>, dim3(stream_grid((mn >> 3) > 0 ? (mn >> 3) : 1, 256)), dim3(256), 0, st,
                     slab, eff, mn, out, 0, 1.f);
  return hipGetLastError();
}

int gemm_splits(int M, int N, int K) {
  if (M >= 256 && N >= 256 && K % 64 == 0 && K >= 4096) {  // 256x256 tiles, one workgroup per CU
    // as many splits as fit ONE round of workgroups: rounding up (e.g. 36 tiles x 8 = 288 > 256
    // CUs) ran a second, almost empty round and doubled the BERT wgrad time
    const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
    int s = std::max(1, cu_count() / tiles);
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

// One level of a split-sum tree: out[c] = sum of in[s] for s in [G c, min(G c + G, splits)), mn
// (a multiple of 8) elements per slab, 8 per lane, the G loads of a lane independent. A serial loop
// over hundreds of splits in one lane (splitk_reduce_kernel) runs at the latency of dependent
// round trips when mn is small (a 64x64 weight gradient over 512 pixel splits: ~150 us); levels of
// G = 8 keep every lane's loads in flight together.
template <int G>
__global__ __launch_bounds__(256) void split_tree_kernel(const float* __restrict__ in, int splits, int64_t mn,
                                                         float* __restrict__ out) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= (mn >> 3)) return;
  const int c = blockIdx.y, s0 = c * G;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < G; ++k) {
    if (s0 + k < splits) {
      float t[8];
      load8_f32(in + (int64_t)(s0 + k) * mn + v * 8, t);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += t[e];
    }
  }
  store8_f32(out + (int64_t)c * mn + v * 8, acc);
}

// 8 < splits <= 8 * GPV in ONE launch: a workgroup = VPB = 256 / GPV 8-element vectors x GPV split
// groups; a lane sums its group's <= 8 slabs (independent loads, as a tree level), the groups'
// partials meet in LDS and 8 lanes per vector (one element each) sum them in a fixed group order
// (deterministic) and apply scale / accumulate / the output type. The tree of G = 8 levels plus the
// final pass took 2-3 launches of ~6-8 us each per weight gradient (~150 launches, ~1.2 ms per
// ResNet-50 step, profiles/r6/resnet50_b1024_r6j_kernels.md) for mostly small outputs.
template <bool OUT_BF16, int GPV>
__global__ __launch_bounds__(256) void split_reduce_lds_kernel(const float* __restrict__ slab, int splits, int64_t mn,
                                                               void* __restrict__ out, int accumulate, float scale) {
  constexpr int VPB = 256 / GPV;
  __shared__ float part[GPV][VPB * 8];
  const int v = threadIdx.x % VPB, gi = threadIdx.x / VPB;
  const int64_t nvec = mn >> 3;
  const int64_t vec = (int64_t)blockIdx.x * VPB + v;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (vec < nvec) {
    const int s0 = gi * 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (s0 + k < splits) {
        float t[8];
        load8_f32(slab + (int64_t)(s0 + k) * mn + vec * 8, t);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += t[e];
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) part[gi][v * 8 + e] = acc[e];
  __syncthreads();
  for (int q = threadIdx.x; q < VPB * 8; q += 256) {  // (VPB * 8 > 256 lanes for GPV < 8)
    const int vv = q >> 3, e = q & 7;
    const int64_t ov = (int64_t)blockIdx.x * VPB + vv;
    if (ov >= nvec) break;
    float sum = 0.f;
#pragma unroll 8
    for (int g = 0; g < GPV; ++g) sum += part[g][vv * 8 + e];
    sum *= scale;
    const int64_t i = ov * 8 + e;
    if (OUT_BF16) {
      uint16_t* o = reinterpret_cast<uint16_t*>(out);
      if (accumulate) sum += bf16_to_f32(o[i]);
      o[i] = f32_to_bf16(sum);
    } else {
      float* o = reinterpret_cast<float*>(out);
      if (accumulate) sum += o[i];
      o[i] = sum;
    }
  }
}

template <bool OUT_BF16>
static void launch_split_reduce_lds(const float* slab, int splits, int64_t mn, void* out, int accumulate, float scale,
                                    hipStream_t st) {
  const int groups = (splits + 7) / 8;  // 2 .. 64
  const int64_t nvec = mn >> 3;
#define PSD_SRL(G)                                                                                               \
  hipLaunchKernelGGL((split_reduce_lds_kernel<OUT_BF16, G>), dim3((unsigned)((nvec + 256 / G - 1) / (256 / G))), \
                     dim3(256), 0, st, slab, splits, mn, out, accumulate, scale)
  if (groups <= 2) PSD_SRL(2);
  else if (groups <= 4) PSD_SRL(4);
  else if (groups <= 8) PSD_SRL(8);
  else if (groups <= 16) PSD_SRL(16);
  else if (groups <= 32) PSD_SRL(32);
  else PSD_SRL(64);
#undef PSD_SRL
}

int64_t splitk_tree_floats(int splits, int64_t mn) { return ((int64_t)(splits + 7) / 8 + 1) * mn; }

// out (bf16 or fp32, [mn]) = (accumulate ? out : 0) + scale * sum over `splits` fp32 slabs of mn
// elements (the deterministic reduce of every split-K / split-pixel launch, e.g. convw.hip). With a
// tree workspace (splitk_tree_floats) and more than 8 splits, levels of 8 run first, ping-ponging
// between the workspace and the (consumed) slab.
hipError_t launch_splitk_reduce(float* slab, int splits, int64_t mn, void* out, int out_bf16, int accumulate,
                                float scale, hipStream_t st, float* tree) {
  if (mn <= 0) return hipSuccess;
  if (tree && mn % 8 == 0) {
    float* src = slab;
    float* dst = tree;
    while (splits > 512) {  // tree levels only above what one LDS-reduce launch takes
      const int chunks = (splits + 7) / 8;
      const dim3 grid((unsigned)(((mn >> 3) + 255) / 256), (unsigned)chunks);
      hipLaunchKernelGGL(split_tree_kernel<8>, grid, dim3(256), 0, st, src, splits, mn, dst);
      splits = chunks;
      float* t = src;
      src = dst;
      dst = t;
    }
    slab = src;
  }
  if (mn % 8 == 0 && splits > 8 && splits <= 512) {
    if (out_bf16) launch_split_reduce_lds<true>(slab, splits, mn, out, accumulate, scale, st);
    else launch_split_reduce_lds<false>(slab, splits, mn, out, accumulate, scale, st);
    return hipGetLastError();
  }
  const int grid = stream_grid((mn >> 3) > 0 ? (mn >> 3) : 1, 256);
  if (out_bf16)
    hipLaunchKernelGGL(splitk_reduce_kernel<true>, dim3(grid), dim3(256), 0, st, slab, splits, mn, out, accumulate, scale);
  else
    hipLaunchKernelGGL(splitk_reduce_kernel<false>, dim3(grid), dim3(256), 0, st, slab, splits, mn, out, accumulate,
                       scale);
  return hipGetLastError();
}

hipError_t launch_colsum_final(const float* part, int rows, int N, void* out, int out_bf16, int accumulate,
                               hipStream_t st) {
  if (N % 8 != 0 || rows <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(colsum_final_kernel, dim3((N + 7) / 8), dim3(1024), 0, st, part, rows, N, out, out_bf16,
                     accumulate);
  return hipGetLastError();
}

hipError_t launch_colsum(const uint16_t* x, int64_t M, int N, float* part, void* out, int out_bf16,
                         int accumulate, hipStream_t st, const uint16_t* pre, uint16_t* xo) {
  if (N % 8 != 0) return hipErrorInvalidValue;
  const int tpc = N / 8;
  const int gy = tpc >= 256 ? (tpc + 255) / 256 : 1;
  const int rpi = tpc >= 256 ? 1 : 256 / tpc;
  // A pure streaming pass: its bandwidth is set by the bytes in flight. At one 256-lane block per CU
  // (256 partial rows) the fused GELU-backward variant ran at half the HBM roof (260 us for a BERT
  // [32768, 3072] pass, rocprofv3 profiles/bert_base_b256_r2_kernels.md), so aim for ~8 blocks per CU
  // (each lane still sums >= 8 rows, 4 loads in flight); the finalize reads the partials with 32
  // independent lanes per column.
  const int64_t want = (int64_t)(8 * 256 + gy - 1) / gy;
  int64_t gx = (M + (int64_t)rpi * 8 - 1) / ((int64_t)rpi * 8);
  if (gx > want) gx = want;
  if (gx > kColsumMaxBlocks) gx = kColsumMaxBlocks;
  if (gx < 1) gx = 1;
  if (pre)
    hipLaunchKernelGGL(colsum_partial_kernel<true>, dim3((unsigned)gx, gy), dim3(256), 0, st, x, M, N, part, pre, xo);
  else
    hipLaunchKernelGGL(colsum_partial_kernel<false>, dim3((unsigned)gx, gy), dim3(256), 0, st, x, M, N, part,
                       nullptr, nullptr);
  hipLaunchKernelGGL(colsum_final_kernel, dim3((N + 7) / 8), dim3(1024), 0, st, part, (int)gx, N, out, out_bf16,
                     accumulate);
  return hipGetLastError();
}

}  // namespace psd
