// Narrow-output implicit-GEMM convolution for gfx950 (NHWC bf16), with the consumer BatchNorm's
// batch statistics reduced in the epilogue.
//
//   y[m][n] = sum_k A(m, k) * W[n][k]       m = output pixel (Nb*Ho*Wo), n = output channel,
//                                           k = (r, s, ci) with A(m, k) = x[pixel(m) + (r, s)][ci]
//
// Why a second conv kernel: the persistent 8-phase GEMM (gemm.hip) owns 256-wide output tiles, so
// the 64- and 128-channel convolutions of ResNet layer1/2 (and every short-K 1x1, K = 64/128,
// which the 8-phase kernel declines) ran on CK / MIOpen / hipBLASLt -- layer1's 3x3 at 2.7x its
// HBM time (435 us vs ~160 us, rocprofv3 of the b1024 step, profiles/) -- and a library output
// needs a separate BN statistics pass over the whole activation (bn_fwd_reduce: 4 ms of the step).
//
// Shape of the kernel (one output tile per workgroup, many workgroups per launch):
//   * tile = BM (128 / 256) output pixels x BN output channels (BN = 64, 128 or 256 = the whole
//     layer width for the narrow layers: the gathered input rows are staged once per pixel tile);
//   * (BM / 64) x (BN / WNT) waves, each owning 64 pixels x WNT channels of C on
//     v_mfma_f32_16x16x32_bf16;
//   * K-tile = 64 channels of one (r, s) (C % 64 == 0); A rows gathered straight into LDS by
//     buffer_load ... lds (16 B per lane, 8 channels of one shifted input pixel; pixels outside the
//     image fall outside the buffer range and load zeros = the padding), B = the weight rows;
//     K-major [rows][64] images, 16-B chunks XOR-swizzled by (row >> 1) & 7 on the SOURCE address
//     (the LDS-DMA image is lane-linear), read with ds_read_b128;
//   * NSLOT-deep LDS ring, NSLOT-1 K-tiles in flight, one raw s_barrier per K-tile: iteration t
//     waits for its own DMA of tile t with a counted vmcnt (the later tiles stay in flight), the
//     barrier publishes tile t and retires every wave's reads of tile t-1, whose slot then
//     receives tile t+NSLOT-1 (the ring is sized to min(NSLOT, K-tiles) at launch: a one-K-tile
//     1x1 convolution keeps several workgroups per CU);
//   * XCD-aware tile order (consecutive pixel tiles -- which share input rows through the 3x3
//     halo -- land on one XCD's L2);
//   * epilogue per wave, no block barrier: each 16-row block of the wave's C is transposed in
//     registers (quad_t4: 4 consecutive columns per lane), packed to bf16 and staged through the
//     wave's own 2 KiB of LDS, then stored as 16-byte lanes covering whole row segments; with
//     STATS, per output channel the shifted sums sum(y - k) and sum((y - k)^2) over the wave's
//     valid rows (y rounded to bf16 first: the statistics of the tensor that is stored), one
//     partial row per 64-pixel wave row in the layout of bn_fwd_reduce_kernel (bn.hip), so the BN
//     forward skips its reduce pass and goes straight to the finalize (kernel-start loads of the
//     shift: a load issued in the epilogue of a one-K-tile convolution is pure exposed latency).
// The same kernel runs a stride-1 bwd-data (conv of dY with the flipped, transposed weights) and
// a 1x1 bwd-data (dY . W as a 1x1 conv of dY with W^T).
//
// Gathering every K-tile's A rows re-reads each input pixel R*R times through L2 (layer1's 3x3:
// 9 x 0.41 GB per pass); the persistent HALO kernel below (convh_kernel) stages each input window
// once and reads the taps as shifted rows.
#include "common.h"
#include "launchers_convn.h"

namespace psd {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;

constexpr int kBM = 128;  // output pixels per tile
constexpr int kBK = 64;   // k per K-tile (one (r, s), 64 channels)
constexpr uint32_t kOOB = 0xFFFFFFF0u;  // past every descriptor's range: the load returns zeros

__device__ __forceinline__ rsrc_t make_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ int kmaj_off(int row, int kc) {  // byte offset in a [rows][64] bf16 tile
  return row * 128 + ((kc ^ ((row >> 1) & 7)) << 4);
}

// 16x16x32 fragment of row block rb, k-step ks: lane holds row rb*16 + (lane & 15), k 8*(lane>>4)..+7
__device__ __forceinline__ bf16x8 frag(const uint8_t* lds, int rb, int ks, int lane) {
  const int row = rb * 16 + (lane & 15);
  return __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(lds + kmaj_off(row, ks * 4 + (lane >> 4))));
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// wait until at most `ahead` K-tiles (DPSK loads each) of this wave are still in flight
template <int DPSK, int A>
__device__ __forceinline__ void wait_ahead(int ahead) {
  if constexpr (A <= 0) {
    wait_vm<0>();
  } else {
    if (ahead >= A) wait_vm<A * DPSK>();
    else wait_ahead<DPSK, A - 1>(ahead);
  }
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  // bijective: blocks with equal bid % 8 (one XCD under round-robin dispatch) get a contiguous range
  const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

// 4x4 transpose inside a lane quad: in v[r] = C[row r][col L]; out w[c] = C[row L][col c]
template <int CTRL>
__device__ __forceinline__ float dpp_q(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ void quad_t4(const f32x4 v, int L, float (&w)[4]) {
  const bool o1 = L & 1, o2 = (L >> 1) & 1;
  const float r0 = dpp_q<0xB1>(o1 ? v[0] : v[1]);  // quad_perm [1,0,3,2]: partner L^1
  const float r1 = dpp_q<0xB1>(o1 ? v[2] : v[3]);
  const float a0 = o1 ? r0 : v[0], a1 = o1 ? v[1] : r0;
  const float b0 = o1 ? r1 : v[2], b1 = o1 ? v[3] : r1;
  const float q0 = dpp_q<0x4E>(o2 ? a0 : b0);  // quad_perm [2,3,0,1]: partner L^2
  const float q1 = dpp_q<0x4E>(o2 ? a1 : b1);
  w[0] = o2 ? q0 : a0;
  w[1] = o2 ? q1 : a1;
  w[2] = o2 ? b0 : q0;
  w[3] = o2 ? b1 : q1;
}

// x[lane ^ 16] / x[lane ^ 32] through the gfx950 half-row / half-wave swaps (VALU, no LDS round
// trip: the statistics reduction of a one-K-tile convolution is on its critical path)
__device__ __forceinline__ float xor16(float x, int lane) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float((lane & 16) ? r[0] : r[1]);
}
__device__ __forceinline__ float xor32(float x, int lane) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float((lane & 32) ? r[0] : r[1]);
}

template <int N>
__device__ __forceinline__ float ror_row(float x) {  // x of lane (l + N) mod 16 within its 16-lane row
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0x120 + N, 0xF, 0xF, true));
}

// x / d for 0 <= x < 2^24 through the fp32 reciprocal (exact after one correction step: the
// product's error is below one unit there) -- the per-row integer divisions of an epilogue that
// maps output rows back to (n, h, w) cost ~40 instructions each
__device__ __forceinline__ int fdiv(int x, int d, float inv) {
  int q = (int)((float)x * inv);
  const int r = x - q * d;
  q += (r >= d ? 1 : 0) - (r < 0 ? 1 : 0);
  return q;
}

template <int BM, int BN, int WNT, int NSLOT>
struct Geo {
  static constexpr int WM = BM / 64;         // wave rows (64 output pixels each)
  static constexpr int NWC = BN / WNT;       // wave columns
  static constexpr int NW = WM * NWC;        // waves
  static constexpr int NT = 64 * NW;
  static constexpr int JN = WNT / 16;        // 16-column MFMA blocks per wave
  static constexpr int APW = (BM / 8) / NW;  // A DMA pieces (1 KiB = 8 rows) per wave per K-tile
  static constexpr int BPW = (BN / 8) / NW;  // B DMA pieces per wave per K-tile
  static constexpr int DPS = APW + BPW;      // DMA per wave per K-tile (the counted vmcnt)
  static constexpr int AB = BM * 128;        // A bytes per K-tile
  static constexpr int SLOT = AB + BN * 128;
  static constexpr int STG = 2048;           // per-wave epilogue staging (16 rows x <= 128 B)
  static_assert((BM / 8) % NW == 0 && (BN / 8) % NW == 0 && APW >= 1 && BPW >= 1, "DMA pieces per wave");
  static_assert(DPS * (NSLOT - 2) < 64, "vmcnt is 6 bits");  // (the LDS bound: convn_launch_t)
  static_assert(WNT == 32 || WNT == 64, "wave tile width");
};


}  // namespace

// Per-lane running sums of an epilogue's reductions: STATS in the C layout (this lane's column of
// each 16-column block, summed over its 16 rows), BWD over this lane's 8 channels. A one-tile kernel
// flushes them per tile; the persistent kernel keeps them across all its tiles and flushes once
// (one partial row per wave row per workgroup instead of per tile: no per-tile cross-lane reduction
// or store, and few enough rows that the BN finalize needs no fold pass).
template <int JN>
struct EpiSums {
  float s1[JN], s2[JN];
  float ga[8], gb[8], gd[8];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int j = 0; j < JN; ++j) s1[j] = s2[j] = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) ga[e] = gb[e] = gd[e] = 0.f;
  }
};

// Cross-lane reduction of the sums and the store of partial row `prow` (part / part_d layout
// [rows][2][N]).
template <int WNT, bool STATS, int BWD>
__device__ __forceinline__ void convn_flush(const ConvnArgs& a, EpiSums<WNT / 16>& es, int64_t prow, int wc, int lane,
                                            int n0) {
  constexpr int JN = WNT / 16;
  const int cl = lane & 15;
  if constexpr (STATS) {
#pragma unroll
    for (int j = 0; j < JN; ++j) {
      float s1 = es.s1[j], s2 = es.s2[j];
      s1 += xor16(s1, lane);
      s2 += xor16(s2, lane);
      s1 += xor32(s1, lane);
      s2 += xor32(s2, lane);
      if (lane < 16) {
        float* pr = a.part + prow * 2 * a.N;
        const int col = n0 + wc * WNT + j * 16 + cl;
        pr[col] = s1;
        pr[a.N + col] = s2;
      }
    }
  }
  if constexpr (BWD >= 1 && BWD <= 5) {
    constexpr int CPR = WNT * 2 / 16;  // 16-byte chunks per staged row
    const int my_col = n0 + wc * WNT + (lane % CPR) * 8;
    // lanes sharing this lane's channels: lane % CPR equal -> rotate-sum within the 16-lane row,
    // then across rows
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if constexpr (CPR == 4) {
        es.ga[e] += ror_row<4>(es.ga[e]);
        es.gb[e] += ror_row<4>(es.gb[e]);
      }
      es.ga[e] += ror_row<8>(es.ga[e]);
      es.gb[e] += ror_row<8>(es.gb[e]);
      es.ga[e] += xor16(es.ga[e], lane);
      es.gb[e] += xor16(es.gb[e], lane);
      es.ga[e] += xor32(es.ga[e], lane);
      es.gb[e] += xor32(es.gb[e], lane);
      if constexpr (BWD == 3) {
        if constexpr (CPR == 4) es.gd[e] += ror_row<4>(es.gd[e]);
        es.gd[e] += ror_row<8>(es.gd[e]);
        es.gd[e] += xor16(es.gd[e], lane);
        es.gd[e] += xor32(es.gd[e], lane);
      }
    }
    if (lane < CPR) {
      float* pr = a.part + prow * 2 * a.N;
      store8_f32(pr + my_col, es.ga);
      store8_f32(pr + a.N + my_col, es.gb);
      if constexpr (BWD == 3) {
        float* pd = a.part_d + prow * 2 * a.N;
        store8_f32(pd + my_col, es.ga);
        store8_f32(pd + a.N + my_col, es.gd);
      }
    }
  }
}

// The epilogue's per-row operands of one wave's 64 rows (the pixel index of each row this lane
// stores, and for the BN-backward modes the BN input x / residual gradient dr / ReLU bits / the dual
// tail's xd; for the apply mode the residual). epi_load issues the loads; a persistent kernel can
// issue them for its NEXT tile before that tile's MFMA loop (convh_kernel), so the loads' latency
// hides behind the taps instead of stalling the epilogue -- at one wave per SIMD nothing else does.
template <int WNT>
struct EpiOps {
  static constexpr int CPR = WNT * 2 / 16;
  static constexpr int PASSES = 16 * CPR / 64;
  int mm[4][PASSES];
  u32x4 exr[4][PASSES], rv4[4][PASSES], dv4[4][PASSES];
  uint32_t bt[4][PASSES];
};

template <int WNT, int BWD, typename Pix>
__device__ __forceinline__ void epi_load(const ConvnArgs& a, int wr, int wc, int lane, Pix pix, int n0, EpiOps<WNT>& o) {
  constexpr bool BRED = BWD >= 1 && BWD <= 5;
  constexpr bool APPLY = BWD == 8;
  constexpr int CPR = EpiOps<WNT>::CPR, PASSES = EpiOps<WNT>::PASSES;
  const int my_col = n0 + wc * WNT + (lane % CPR) * 8;
  const bool has_bx = !BRED || a.bx != nullptr;
  const bool fast_div = a.M < (1 << 24);
  float inv_hw = 0.f, inv_wo = 0.f;
  if constexpr (BWD == 5) {
    inv_hw = 1.f / (float)(a.Ho * a.Wo);
    inv_wo = 1.f / (float)a.Wo;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int ps = 0; ps < PASSES; ++ps) {
      const int c = ps * 64 + lane;
      const int rr = c / CPR;
      const int m = pix(wr * 64 + i * 16 + rr);
      o.mm[i][ps] = m;
      if constexpr (APPLY) {
        o.rv4[i][ps] = u32x4{0u, 0u, 0u, 0u};
        if (m >= 0 && a.ares) o.rv4[i][ps] = *reinterpret_cast<const u32x4*>(a.ares + (int64_t)m * a.N + my_col);
      }
      if constexpr (BRED) {
        o.exr[i][ps] = o.rv4[i][ps] = o.dv4[i][ps] = u32x4{0u, 0u, 0u, 0u};
        o.bt[i][ps] = 0u;
        if (m >= 0) {
          if (has_bx) o.exr[i][ps] = *reinterpret_cast<const u32x4*>(a.bx + (int64_t)m * a.N + my_col);
          if constexpr (BWD >= 2) {
            if constexpr (BWD == 5) {
              // residual-branch gradient of a stride-2 1x1 (downsample) convolution, on the quarter
              // grid: non-zero only at even (h, w) of this (Ho x Wo) output grid
              const int hw = a.Ho * a.Wo;
              const int n = fast_div ? fdiv(m, hw, inv_hw) : m / hw, rem = m - n * hw;
              const int h = fast_div ? fdiv(rem, a.Wo, inv_wo) : rem / a.Wo, w = rem - h * a.Wo;
              if (((h | w) & 1) == 0) {
                const int64_t q = ((int64_t)n * (a.Ho >> 1) + (h >> 1)) * (a.Wo >> 1) + (w >> 1);
                o.rv4[i][ps] = *reinterpret_cast<const u32x4*>(a.bdr + q * a.N + my_col);
              }
            } else {
              o.rv4[i][ps] = *reinterpret_cast<const u32x4*>(a.bdr + (int64_t)m * a.N + my_col);
            }
            o.bt[i][ps] = a.bmbits[((int64_t)m * a.N + my_col) >> 3];
          }
          if constexpr (BWD == 3) o.dv4[i][ps] = *reinterpret_cast<const u32x4*>(a.bxd + (int64_t)m * a.N + my_col);
        }
      }
    }
}

// Epilogue of one wave's 64 x WNT accumulator block (shared by the gathered kernel, the persistent
// HALO kernel and the persistent 1x1 kernel): per-wave, no barrier (``stg`` is this wave's own 2 KiB of LDS). C layout
// of a 16x16 block: col = lane & 15, row = 4 * (lane >> 4) + r. ``pix(p)``: output pixel of tile row
// p (-1: none). The reductions accumulate into ``es``; without DEFER they are flushed here to
// partial row (tm * WM + wr).
template <int BM, int BN, int WNT, bool STATS, int BWD, bool DEFER = false, bool PRE = false, typename Pix>
__device__ __forceinline__ void convn_epilogue(const ConvnArgs& a, f32x4 (&acc)[4][WNT / 16],
                                               const float (&kshift)[WNT / 16], int tm, int wr, int wc, int lane,
                                               uint8_t* stg, Pix pix, int n0, EpiSums<WNT / 16>& es,
                                               const EpiOps<WNT>* pre = nullptr) {
  constexpr int JN = WNT / 16;
  constexpr int WM = BM / 64;
  const int cl = lane & 15, rq = (lane >> 4) * 4;
  if (a.bias) {  // per-output-channel bias (the BN-backward fold's constant term)
#pragma unroll
    for (int j = 0; j < JN; ++j) {
      const float bv = a.bias[n0 + wc * WNT + j * 16 + cl];
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i][j] += f32x4{bv, bv, bv, bv};
    }
  }
  if constexpr (STATS) {
    // the statistics of the tensor the BN normalises: with a stored output, its bf16-rounded values
    // (what bn_apply reads; fp32 accumulators here put the chained-block gradients past the library
    // path's error level, tests/test_bnfold.py); in the statistics-only pass (a.y null: the recomputing
    // tail, ops/tail.py) the fp32 product, which the apply pass (mode 8) normalises before any
    // rounding -- the same values the tail's Gram statistics (sum y = W s, sum y^2 = W^T G W) describe,
    // so both statistics routes agree with the normalised tensor (tools/probes/tail_stats_probe.py:
    // normalising bf16(y) with the Gram moments of y moved the b8 test loss by 0.55 %). Packed fp32
    // pairs (v_pk_add / v_pk_fma): at two waves per SIMD the statistics-only pass was instruction-issue
    // bound (~460 VALU per wave-tile, profiles/convp_pmc_r4.md). A 16-row block whose last row is
    // valid is valid throughout (pix is monotone within a block): the wave-uniform test skips the
    // per-row masks there.
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    const bool rnd = a.y != nullptr;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bool full = pix(wr * 64 + i * 16 + 15) >= 0;
#pragma unroll
      for (int j = 0; j < JN; ++j) {
        const f32x2 k2 = {kshift[j], kshift[j]};
        f32x2 s1 = {0.f, 0.f}, s2 = {0.f, 0.f};
#pragma unroll
        for (int r = 0; r < 4; r += 2) {
          f32x2 d;
          if (rnd) {
            const uint32_t pk = pack_bf16x2_rne(acc[i][j][r], acc[i][j][r + 1]);
            d = f32x2{__uint_as_float(pk << 16), __uint_as_float(pk & 0xFFFF0000u)} - k2;
          } else {
            d = f32x2{acc[i][j][r], acc[i][j][r + 1]} - k2;
          }
          if (!full) {
            d[0] = pix(wr * 64 + i * 16 + rq + r) >= 0 ? d[0] : 0.f;
            d[1] = pix(wr * 64 + i * 16 + rq + r + 1) >= 0 ? d[1] : 0.f;
          }
          s1 += d;
          s2 = __builtin_elementwise_fma(d, d, s2);
        }
        es.s1[j] += s1[0] + s1[1];
        es.s2[j] += s2[0] + s2[1];
      }
    }
  }
  // reductions of the producing BN's backward (modes 1-5); mode 8 is the forward BN apply
  constexpr bool BRED = BWD >= 1 && BWD <= 5;
  constexpr bool APPLY = BWD == 8;
  if constexpr (STATS && !BRED && !APPLY) {
    if (a.y == nullptr) {  // statistics-only pass (the output is recomputed by an apply pass)
      if constexpr (!DEFER) convn_flush<WNT, STATS, BWD>(a, es, (int64_t)tm * WM + wr, wc, lane, n0);
      return;
    }
  }
  if constexpr (APPLY) {
    // mode 8: the BN affine on the fp32 product in the accumulator layout (column = this lane's
    // cl of block j), before the bf16 staging; the residual add + ReLU follow after the transpose
#pragma unroll
    for (int j = 0; j < JN; ++j) {
      const int col = n0 + wc * WNT + j * 16 + cl;
      const float sc = a.bss[col], sh = a.bss[a.N + col];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] = fmaf(acc[i][j][r], sc, sh);
    }
  }
  const int L = cl & 3;
  constexpr int RB = WNT * 2;       // staged row bytes (one 16-row block)
  constexpr int CPR = RB / 16;      // 16-byte chunks per staged row
  constexpr int PASSES = 16 * CPR / 64;
  uint16_t* y = reinterpret_cast<uint16_t*>(a.y);
  // BWD: this lane's 8 output channels are fixed (64 % CPR == 0): per-channel constants once
  const int my_c16 = lane % CPR;
  const int my_col = n0 + wc * WNT + my_c16 * 8;
  float bmu[8], bsc[8], bsh[8], bmd[8];
  if constexpr (BWD == 3) load8_f32(a.bmean_d + my_col, bmd);
  if constexpr (BRED) load8_f32(a.bmean + my_col, bmu);
  if constexpr (BWD == 1) {
    load8_f32(a.bss + my_col, bsc);
    load8_f32(a.bss + a.N + my_col, bsh);
  }
  // the epilogue operands of all this wave's rows (x, dr, mask bits, xd): issued here, before the
  // first is used -- the compiler cannot hoist them above the y stores (possible alias), and at one
  // workgroup per CU (LDS) the per-row load -> use latency was the epilogue's cost -- or (PRE) by
  // the caller before this tile's MFMA loop. (modes 2 / 3 / 5 without the BN input -- bx null: a BN
  // whose input was never stored, ops/tail.py -- take x as 0, so the second partial is -mean * sum g
  // and the caller adds sum g x itself)
  EpiOps<WNT> own;
  if constexpr (!PRE) epi_load<WNT, BWD>(a, wr, wc, lane, pix, n0, own);
  const EpiOps<WNT>& ops = PRE ? *pre : own;
  const auto& mm = ops.mm;
  const auto& exr = ops.exr;
  const auto& rv4 = ops.rv4;
  const auto& dv4 = ops.dv4;
  const auto& bt = ops.bt;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = rq + L;  // this lane's row within the 16-row block after quad_t4
#pragma unroll
    for (int j = 0; j < JN; ++j) {
      float w[4];
      quad_t4(acc[i][j], L, w);
      const int c8 = (j * 16 + (cl & ~3)) >> 2;  // 8-byte column group within the staged row
      const int off = r * RB + ((c8 ^ ((r & 7) << 1)) & (RB / 8 - 1)) * 8;
      const uint32_t lo = pack_bf16x2_rne(w[0], w[1]), hi = pack_bf16x2_rne(w[2], w[3]);
      *reinterpret_cast<uint64_t*>(stg + off) = (uint64_t)lo | ((uint64_t)hi << 32);
    }
    // one wave's LDS ops complete in order: the reads below see the writes above
#pragma unroll
    for (int ps = 0; ps < PASSES; ++ps) {
      const int c = ps * 64 + lane;
      const int rr = c / CPR, c16 = c % CPR;
      const int off = rr * RB + (((2 * c16) ^ ((rr & 7) << 1)) & (RB / 8 - 1)) * 8;
      u32x4 v = *reinterpret_cast<const u32x4*>(stg + off);
      const int m = mm[i][ps];
      if (m >= 0) {
        const int64_t go = (int64_t)m * a.ldc + n0 + wc * WNT + c16 * 8;
        if constexpr (APPLY) {
          // y = relu(bf16(acc * scale + shift) + residual) and its ReLU bit-mask: the convolution
          // output (never written) normalised in fp32 before its one rounding
          float d[8], rv[8];
          load8_bf16(reinterpret_cast<const uint16_t*>(&v), d);
          load8_bf16(reinterpret_cast<const uint16_t*>(&rv4[i][ps]), rv);
          uint32_t bits = 0;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float o = relu_nan(d[e] + rv[e]);
            d[e] = o;
            bits |= (o > 0.f ? 1u : 0u) << e;
          }
          uint32_t pk[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) pk[e] = pack_bf16x2_rne(d[2 * e], d[2 * e + 1]);
          v = u32x4{pk[0], pk[1], pk[2], pk[3]};
          a.amask[((int64_t)m * a.N + my_col) >> 3] = (uint8_t)bits;
        }
        if constexpr (BRED) {
          float d[8], xv[8];
          load8_bf16(reinterpret_cast<const uint16_t*>(&v), d);
          load8_bf16(reinterpret_cast<const uint16_t*>(&exr[i][ps]), xv);
          if constexpr (BWD >= 2) {
            float rv[8];
            load8_bf16(reinterpret_cast<const uint16_t*>(&rv4[i][ps]), rv);
            const uint32_t bits = bt[i][ps];
#pragma unroll
            for (int e = 0; e < 8; ++e) d[e] = ((bits >> e) & 1u) ? d[e] + rv[e] : 0.f;
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) d[e] = fmaf(xv[e], bsc[e], bsh[e]) > 0.f ? d[e] : 0.f;
          }
          uint32_t pk[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) pk[e] = pack_bf16x2_rne(d[2 * e], d[2 * e + 1]);
          v = u32x4{pk[0], pk[1], pk[2], pk[3]};
          float gq[8];  // the stored g
          load8_bf16(reinterpret_cast<const uint16_t*>(&v), gq);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            es.ga[e] += gq[e];
            es.gb[e] = fmaf(gq[e], xv[e] - bmu[e], es.gb[e]);
          }
          if constexpr (BWD == 3) {
            float dv[8];
            load8_bf16(reinterpret_cast<const uint16_t*>(&dv4[i][ps]), dv);
#pragma unroll
            for (int e = 0; e < 8; ++e) es.gd[e] = fmaf(gq[e], dv[e] - bmd[e], es.gd[e]);
          }
        }
        *reinterpret_cast<u32x4*>(y + go) = v;
      }
    }
  }
  if constexpr (!DEFER) convn_flush<WNT, STATS, BWD>(a, es, (int64_t)tm * WM + wr, wc, lane, n0);
}

// BWD (bwd-data of a convolution whose input came out of a BatchNorm + ReLU): the epilogue also runs
// that BN's backward reduction. 1: ReLU mask recomputed from the BN input x and the forward
// scale/shift (bn1 / bn2 of a bottleneck); 2: the output plus the handed-over residual-branch
// gradient dr, masked by the forward bit-mask (the previous block's bn3, whose output fed this
// convolution and the identity residual). The stored output is then g = mask (dX [+ dr]) -- the
// masked gradient the BN's elementwise pass consumes and, for 2, the residual gradient handed on --
// and the partials are sum g and sum g (x - mean) per channel (the layout of bn_bwd_reduce_kernel).
// 5: as 2 with dr the stride-2 downsample convolution's bwd-data on the quarter grid (added at even
// (h, w) only: the zero-filled full-size gradient is never written).
// 3: as 2 for a bottleneck tail relu(bn3(x) + bnd(xd)) (the downsample block's dual BN, whose
// upstream gradient g is shared): part_d also receives sum g and sum g (xd - mean_d) for bnd.
template <int BM, int BN, int WNT, int NSLOT, bool STATS, int BWD = 0>
__global__ __launch_bounds__(512) void convn_kernel(ConvnArgs a) {
  using G = Geo<BM, BN, WNT, NSLOT>;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tiles_m = gridDim.x;
  const int tm = xcd_remap(blockIdx.x, tiles_m);
  const int m0 = tm * BM, n0 = blockIdx.y * BN;
  constexpr int SLOTB = G::SLOT;  // ring slot bytes
  // output pixel of tile row p (-1: past M). A phase launch (ophase = 1 + (ph << 1 | pw): one of the
  // four output-parity classes of a stride-2 bwd-data, ops/conv.py _dgrad_s2_phases) computes row
  // m = (n, i, j) of the Ho x Wo phase grid and stores it at pixel (n, 2i + ph, 2j + pw) of the
  // 2Ho x 2Wo output (every epilogue operand -- y, the BN input bx -- is addressed by that pixel)
  const int oph = (a.ophase - 1) >> 1, opw = (a.ophase - 1) & 1;
  const float inv_ohw = 1.f / (float)(a.Ho * a.Wo), inv_owo = 1.f / (float)a.Wo;
  auto pix = [&](int p) -> int {
    const int m = m0 + p;
    if (m >= a.M) return -1;
    if (a.ophase == 0) return m;
    const int hw = a.Ho * a.Wo;
    const int n = fdiv(m, hw, inv_ohw), rem = m - n * hw;
    const int i = fdiv(rem, a.Wo, inv_owo), j = rem - i * a.Wo;
    return ((n * 2 * a.Ho + 2 * i + oph) * 2 * a.Wo) + 2 * j + opw;
  };
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid / G::NWC, wc = wid % G::NWC;
  const int cl = lane & 15, rq = (lane >> 4) * 4;

  // statistics shift of this lane's columns, loaded before any DMA is issued (its latency hides
  // behind the whole K loop)
  float kshift[G::JN];
#pragma unroll
  for (int j = 0; j < G::JN; ++j) kshift[j] = 0.f;
  if constexpr (STATS) {
#pragma unroll
    for (int j = 0; j < G::JN; ++j) kshift[j] = a.shift[n0 + wc * WNT + j * 16 + cl];
  }

  // this lane's A rows (one per DMA piece): window origin p0 = top-left input pixel index,
  // hw = (h0 << 16) | (w0 & 0xffff); rows past M get h0 = -32768 (never in the image)
  int p0[G::APW], hw[G::APW];
  {
    const int howo = a.Ho * a.Wo;
#pragma unroll
    for (int i = 0; i < G::APW; ++i) {
      const int row = (i * G::NW + wid) * 8 + (lane >> 3);
      const int m = m0 + row;
      const int n = m / howo, rem = m - n * howo;
      const int ho = rem / a.Wo, wo = rem - ho * a.Wo;
      const int h0 = ho * a.stride - a.pad, w0 = wo * a.stride - a.pad;
      p0[i] = (n * a.H + h0) * a.W + w0;
      hw[i] = m < a.M ? (int)(((uint32_t)h0 << 16) | ((uint32_t)w0 & 0xffffu)) : (int)0x80000000u;
    }
  }
  const rsrc_t xr = make_rsrc(a.x, a.xbytes);
  const rsrc_t x2r = make_rsrc(a.x2 ? a.x2 : a.x, a.x2 ? a.x2bytes : 0u);
  const rsrc_t wrs = make_rsrc(a.w, a.wbytes);
  const int cmask = (1 << a.logC) - 1;
  const int nslot = a.nslot;  // ring depth of this launch: min(NSLOT, K-tiles)

  auto stage = [&](int t) {
    uint8_t* slot = smem + (t % nslot) * SLOTB;
    const int k0 = t * kBK;
    if (k0 >= a.K1) {  // K-concatenated second operand (1x1: the row is the output pixel itself)
      const int c0 = k0 - a.K1;
#pragma unroll
      for (int i = 0; i < G::APW; ++i) {
        const int piece = i * G::NW + wid;
        const int row = piece * 8 + (lane >> 3);
        const int kc = (lane & 7) ^ ((row >> 1) & 7);
        const bool ok = hw[i] != (int)0x80000000u;
        const uint32_t off = ok ? ((((uint32_t)p0[i]) << a.logC2) + (uint32_t)(c0 + kc * 8)) * 2u : kOOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(x2r, (__attribute__((address_space(3))) void*)(slot + piece * 1024),
                                                 16, off, 0, 0, 0);
      }
    } else {
    const int rs = k0 >> a.logC, ci0 = k0 & cmask;
    const int r = rs / a.S, s = rs - r * a.S;
#pragma unroll
    for (int i = 0; i < G::APW; ++i) {
      const int piece = i * G::NW + wid;
      const int row = piece * 8 + (lane >> 3);
      const int kc = (lane & 7) ^ ((row >> 1) & 7);
      const int hh = (hw[i] >> 16) + r, ww = ((int)((uint32_t)hw[i] << 16) >> 16) + s;
      const bool ok = (unsigned)hh < (unsigned)a.H && (unsigned)ww < (unsigned)a.W;
      const uint32_t off = ok ? ((((uint32_t)(p0[i] + r * a.W + s)) << a.logC) + (uint32_t)(ci0 + kc * 8)) * 2u : kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (__attribute__((address_space(3))) void*)(slot + piece * 1024), 16,
                                               off, 0, 0, 0);
    }
    }
    // (the weight offsets are recomputed per K-tile: a per-lane offset array captured by this lambda
    // made hipcc's host pass silently drop the kernel's instantiation -- an undefined stub symbol)
#pragma unroll
    for (int i = 0; i < G::BPW; ++i) {
      const int piece = i * G::NW + wid;
      const int row = piece * 8 + (lane >> 3);
      const int kc = (lane & 7) ^ ((row >> 1) & 7);
      const uint32_t off = ((uint32_t)(n0 + row) * (uint32_t)a.K + (uint32_t)(k0 + kc * 8)) * 2u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs,
                                               (__attribute__((address_space(3))) void*)(slot + (SLOTB - BN * 128) +
                                                                                        piece * 1024),
                                               16, off, 0, 0, 0);
    }
  };

  f32x4 acc[4][G::JN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < G::JN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nt = a.K / kBK;
  const int D = nslot - 1 > 0 ? nslot - 1 : 1;  // K-tiles issued ahead
  for (int p = 0; p < D && p < nt; ++p) stage(p);
  constexpr int DPSK = G::DPS;  // this wave's DMA per K-tile
  for (int t = 0; t < nt; ++t) {
    // K-tile t landed (this wave's DMA): leave the (up to D-1) later K-tiles in flight
    wait_ahead<DPSK, NSLOT - 2>(min(nt - 1 - t, D - 1));
    __builtin_amdgcn_s_barrier();  // every wave: tile t published, tile t-1 no longer read
    __builtin_amdgcn_sched_barrier(0);
    if (t + D < nt) stage(t + D);
    const uint8_t* As = smem + (t % nslot) * SLOTB;
    const uint8_t* Bs = As + (SLOTB - BN * 128);
    // both k-steps' fragments are read before the first MFMA (one LDS latency per K-tile, not two:
    // at 1-2 waves per SIMD nothing else hides it)
    bf16x8 af[2][4], bf[2][G::JN];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int j = 0; j < G::JN; ++j) bf[ks][j] = frag(Bs, wc * G::JN + j, ks, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i) af[ks][i] = frag(As, wr * 4 + i, ks, lane);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < G::JN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks][i], bf[ks][j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }

  EpiSums<G::JN> es;
  es.zero();
  convn_epilogue<BM, BN, WNT, STATS, BWD>(a, acc, kshift, tm, wr, wc, lane,
                                          smem + a.nslot * SLOTB + wid * G::STG, pix,
                                          n0, es);
}


// ------------------------------------------------------------------ persistent 1x1 (stride 1)
// The 1x1 convolutions of the bottleneck ends (conv3 forward / statistics / BN-apply passes, conv1
// bwd-data with the producing BN's reduction) have K = 64..512 against M = 0.8-3.2M rows: a
// one-tile-per-workgroup launch of the kernel above is latency-bound there (the tail's
// statistics-only pass over layer1, 0.4 GB of input, took 500 us: every workgroup waits for its
// one DMA, computes 1-2 K-tiles and drains). Here a workgroup runs a contiguous run of 128-row
// tiles through the same ring of K-tile slots: the ring keeps streaming across tile boundaries, so
// the next tiles' A (and B) K-tiles land while this tile's MFMAs and epilogue run; the epilogue's
// reductions accumulate over the run (one partial row per wave row per workgroup). A [M][C] with
// row m the output pixel itself (and the K-concatenated x2 of the BN-backward fold).
template <int BN, int WNT, int NSLOT, bool STATS, int BWD>
__global__ __launch_bounds__(512) void convp_kernel(ConvnArgs a, int tiles_m) {
  constexpr int BM = 128;
  using G = Geo<BM, BN, WNT, NSLOT>;
  constexpr int SLOTB = G::SLOT;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int n0 = blockIdx.y * BN;
  const int gx = gridDim.x;
  const int bq = xcd_remap(blockIdx.x, gx);  // a contiguous run of tiles per workgroup, XCD-grouped
  const int t_begin = (int)(((int64_t)bq * tiles_m) / gx);
  const int t_end = (int)(((int64_t)(bq + 1) * tiles_m) / gx);
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid / G::NWC, wc = wid % G::NWC;
  const int cl = lane & 15;
  float kshift[G::JN];
#pragma unroll
  for (int j = 0; j < G::JN; ++j) kshift[j] = 0.f;
  if constexpr (STATS) {
#pragma unroll
    for (int j = 0; j < G::JN; ++j) kshift[j] = a.shift[n0 + wc * WNT + j * 16 + cl];
  }
  const rsrc_t xr = make_rsrc(a.x, a.xbytes);
  const rsrc_t x2r = make_rsrc(a.x2 ? a.x2 : a.x, a.x2 ? a.x2bytes : 0u);
  const rsrc_t wrs = make_rsrc(a.w, a.wbytes);
  const int nslot = a.nslot;
  const int nt = a.K / kBK;
  const int total = (t_end - t_begin) * nt;
  // K-tile T of the run: tile t_begin + T / nt, k-block T % nt
  auto stage = [&](int T) {
    uint8_t* slot = smem + (T % nslot) * SLOTB;
    const int tile = t_begin + T / nt;
    const int k0 = (T % nt) * kBK;
    const int m0 = tile * BM;
    const bool second = k0 >= a.K1;
    const int c0 = second ? k0 - a.K1 : k0;
    const int lc = second ? a.logC2 : a.logC;
#pragma unroll
    for (int i = 0; i < G::APW; ++i) {
      const int piece = i * G::NW + wid;
      const int row = piece * 8 + (lane >> 3);
      const int kc = (lane & 7) ^ ((row >> 1) & 7);
      const int m = m0 + row;
      const uint32_t off = m < a.M ? ((((uint32_t)m) << lc) + (uint32_t)(c0 + kc * 8)) * 2u : kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(second ? x2r : xr,
                                               (__attribute__((address_space(3))) void*)(slot + piece * 1024), 16, off,
                                               0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < G::BPW; ++i) {
      const int piece = i * G::NW + wid;
      const int row = piece * 8 + (lane >> 3);
      const int kc = (lane & 7) ^ ((row >> 1) & 7);
      const uint32_t off = ((uint32_t)(n0 + row) * (uint32_t)a.K + (uint32_t)(k0 + kc * 8)) * 2u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          wrs, (__attribute__((address_space(3))) void*)(slot + (SLOTB - BN * 128) + piece * 1024), 16, off, 0, 0, 0);
    }
  };
  f32x4 acc[4][G::JN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < G::JN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  EpiSums<G::JN> es;
  es.zero();
  uint8_t* stg = smem + nslot * SLOTB + wid * G::STG;
  const int D = nslot - 1;  // K-tiles issued ahead (nslot >= 2)
  for (int p = 0; p < D && p < total; ++p) stage(p);
  for (int T = 0; T < total; ++T) {
    wait_ahead<G::DPS, NSLOT - 2>(min(total - 1 - T, D - 1));
    __builtin_amdgcn_s_barrier();  // every wave: K-tile T published, K-tile T-1 no longer read
    __builtin_amdgcn_sched_barrier(0);
    if (T + D < total) stage(T + D);
    const uint8_t* As = smem + (T % nslot) * SLOTB;
    const uint8_t* Bs = As + (SLOTB - BN * 128);
    bf16x8 af[2][4], bf[2][G::JN];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int j = 0; j < G::JN; ++j) bf[ks][j] = frag(Bs, wc * G::JN + j, ks, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i) af[ks][i] = frag(As, wr * 4 + i, ks, lane);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < G::JN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks][i], bf[ks][j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    if (T % nt == nt - 1) {  // the tile's last K-tile: its epilogue (the ring keeps streaming underneath)
      const int tile = t_begin + T / nt;
      const int m0 = tile * BM;
      auto pix = [&](int p) -> int { return m0 + p < a.M ? m0 + p : -1; };
      convn_epilogue<BM, BN, WNT, STATS, BWD, true>(a, acc, kshift, tile, wr, wc, lane, stg, pix, n0, es);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < G::JN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      // (no drain: the epilogue's stores and loads also count in vmcnt, but loads return in issue
      // order, so "at most (D - 1) * DPS outstanding" above still means at most that many LOADS --
      // the K-tile DMA issued after K-tile T+1's -- are in flight: K-tile T+1 has landed. Stores
      // still pending only make that wait longer, never short. A full drain here cost the stats-only
      // pass its whole prefetch: 372 us vs ~100 for its 0.4 GB, profiles/resnet50_b1024_r4_kernels.md)
    }
  }
  convn_flush<WNT, STATS, BWD>(a, es, (int64_t)blockIdx.x * G::WM + wr, wc, lane, n0);
}

// Resident-B form (K <= 128 with the weight tile [BN][K] kept in LDS): the ring carries the A
// K-tiles only (16 KiB each), up to kPrMaxSlots deep. With K = 64 and BN = 256 the streamed form
// re-DMA'd the 32 KiB weight tile for every 16 KiB of input and kept 2 tiles in flight: the tail's
// statistics-only pass over layer1 ran at 1.4 TB/s of input (288 us, profiles/tail_passes_r4.md).
constexpr int kPrMaxSlots = 6;
template <int BN, int WNT, bool STATS, int BWD>
__global__ __launch_bounds__(512) void convpr_kernel(ConvnArgs a, int tiles_m) {
  constexpr int BM = 128;
  using G = Geo<BM, BN, WNT, 3>;
  constexpr int AB = BM * 128;  // one A K-tile
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int n0 = blockIdx.y * BN;
  const int gx = gridDim.x;
  const int bq = xcd_remap(blockIdx.x, gx);
  const int t_begin = (int)(((int64_t)bq * tiles_m) / gx);
  const int t_end = (int)(((int64_t)(bq + 1) * tiles_m) / gx);
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid / G::NWC, wc = wid % G::NWC;
  const int cl = lane & 15;
  float kshift[G::JN];
#pragma unroll
  for (int j = 0; j < G::JN; ++j) kshift[j] = 0.f;
  if constexpr (STATS) {
#pragma unroll
    for (int j = 0; j < G::JN; ++j) kshift[j] = a.shift[n0 + wc * WNT + j * 16 + cl];
  }
  const rsrc_t xr = make_rsrc(a.x, a.xbytes);
  const rsrc_t x2r = make_rsrc(a.x2 ? a.x2 : a.x, a.x2 ? a.x2bytes : 0u);
  const rsrc_t wrs = make_rsrc(a.w, a.wbytes);
  const int nslot = a.nslot;
  const int nt = a.K / kBK;
  uint8_t* bres = smem;                              // [nt][BN rows x 128 B] resident weights
  uint8_t* ring = smem + nt * BN * 128;              // nslot A K-tiles
  uint8_t* stg = ring + nslot * AB + wid * G::STG;   // this wave's epilogue staging
  // the weight tile of every K-tile, once (BN / 8 pieces of 1 KiB per K-tile over the waves)
  for (int pc = wid; pc < nt * (BN / 8); pc += G::NW) {
    const int kt = pc / (BN / 8), rp = pc - kt * (BN / 8);
    const int row = rp * 8 + (lane >> 3);
    const int kc = (lane & 7) ^ ((row >> 1) & 7);
    const uint32_t off = ((uint32_t)(n0 + row) * (uint32_t)a.K + (uint32_t)(kt * kBK + kc * 8)) * 2u;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (__attribute__((address_space(3))) void*)(bres + pc * 1024), 16, off, 0,
                                             0, 0);
  }
  wait_vm<0>();  // (the weights land before the ring's counted waits start)
  const int total = (t_end - t_begin) * nt;
  auto stage = [&](int T) {
    uint8_t* slot = ring + (T % nslot) * AB;
    const int tile = t_begin + T / nt;
    const int k0 = (T % nt) * kBK;
    const int m0 = tile * BM;
    const bool second = k0 >= a.K1;
    const int c0 = second ? k0 - a.K1 : k0;
    const int lc = second ? a.logC2 : a.logC;
#pragma unroll
    for (int i = 0; i < G::APW; ++i) {
      const int piece = i * G::NW + wid;
      const int row = piece * 8 + (lane >> 3);
      const int kc = (lane & 7) ^ ((row >> 1) & 7);
      const int m = m0 + row;
      const uint32_t off = m < a.M ? ((((uint32_t)m) << lc) + (uint32_t)(c0 + kc * 8)) * 2u : kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(second ? x2r : xr,
                                               (__attribute__((address_space(3))) void*)(slot + piece * 1024), 16, off,
                                               0, 0, 0);
    }
  };
  f32x4 acc[4][G::JN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < G::JN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  EpiSums<G::JN> es;
  es.zero();
  const int D = nslot - 1;
  for (int p = 0; p < D && p < total; ++p) stage(p);
  for (int T = 0; T < total; ++T) {
    // K-tile T landed: at most (D - 1) later K-tiles' A DMA in flight (loads return in issue order;
    // the epilogue's stores in the count only lengthen the wait)
    wait_ahead<G::APW, kPrMaxSlots - 2>(min(total - 1 - T, D - 1));
    __builtin_amdgcn_s_barrier();  // every wave: K-tile T published, K-tile T-1 no longer read
    __builtin_amdgcn_sched_barrier(0);
    if (T + D < total) stage(T + D);
    const uint8_t* As = ring + (T % nslot) * AB;
    const uint8_t* Bs = bres + (T % nt) * BN * 128;
    bf16x8 af[2][4], bf[2][G::JN];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int j = 0; j < G::JN; ++j) bf[ks][j] = frag(Bs, wc * G::JN + j, ks, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i) af[ks][i] = frag(As, wr * 4 + i, ks, lane);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < G::JN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks][i], bf[ks][j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    if (T % nt == nt - 1) {
      const int tile = t_begin + T / nt;
      const int m0 = tile * BM;
      auto pix = [&](int p) -> int { return m0 + p < a.M ? m0 + p : -1; };
      convn_epilogue<BM, BN, WNT, STATS, BWD, true>(a, acc, kshift, tile, wr, wc, lane, stg, pix, n0, es);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < G::JN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  convn_flush<WNT, STATS, BWD>(a, es, (int64_t)blockIdx.x * G::WM + wr, wc, lane, n0);
}

// ------------------------------------------------------------------ persistent HALO (layer1 3x3)
// The ResNet layer1 3x3 convolution (C = 64 -> N = 64, stride 1, pad 1, 56 x 56) and its bwd-data
// run at ~20 % of the MFMA rate on the gathered kernel above: every K-tile re-gathers 128 input
// rows through L2 -> LDS (9 per output pixel) and the per-CU fill rate (~46 GB/s, TD busy 67 %,
// profiles/convn_pmc_r4.md) bounds it; the plain HALO variant stages the window once per tile but
// waits for it before computing (one channel block: nothing to overlap it with).
// This kernel is persistent (one 256-thread workgroup per CU, a contiguous run of tiles each):
//   * the whole weight tensor (64 x 576 bf16 = 72 KiB, nine 64x64 tap images) is loaded into LDS
//     once per workgroup;
//   * tile = 2 output rows of one image x 64 slots (Wo <= 62 valid); its input window (4 rows x 64
//     slots x 64 channels = 32 KiB, zero outside the image by the out-of-range DMA) is double
//     buffered: tile i+1's window is DMA'd while tile i's nine taps run, one barrier per tile;
//   * 4 waves = 2 output rows x 2 x 32 channels, v_mfma_f32_16x16x32_bf16, A fragments read from the
//     window at row offset (r * 64 + s) (the tap shift), B fragments from the resident weights;
//   * the epilogue (statistics / bwd reductions / stores) is the shared one; the next window's DMA
//     is in flight underneath it.
// LDS image of the persistent kernel: [rows][64] bf16, 16-byte chunk c of row r at chunk
// c ^ (2 * ((r >> 1) & 3)). The taps read 16 consecutive rows from any start row (the tap shift s =
// 0..2 and the row offsets); with the gathered kernels' c ^ ((r >> 1) & 7) an odd start put two
// lanes of one ds_read_b128 lane group on one bank (SQ_LDS_BANK_CONFLICT 2.2e7 per launch,
// gpurun_out/convh pmc1); this one is conflict-free for every start row (exhaustive check over the
// four lane groups, both k-steps).
__device__ __forceinline__ int hx_swz(int row) { return ((row >> 1) & 3) << 1; }
__device__ __forceinline__ int hx_off(int row, int kc) { return row * 128 + ((kc ^ hx_swz(row)) << 4); }

constexpr int kHxWin = 4 * 64 * 128;          // window bytes (4 rows x 64 slots x 128 B)
constexpr int kHxW = 9 * 64 * 128;            // resident weights (9 taps x 64 rows x 128 B)
constexpr int kHxLds = kHxW + 2 * kHxWin + 4 * 2048 + 512;  // + 4 wave staging areas, + tap overrun

template <bool STATS, int BWD>
__global__ __launch_bounds__(256) void convh_kernel(ConvnArgs a, int ntiles) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* wlds = smem;
  auto winb = [&](int b) { return smem + kHxW + b * kHxWin; };
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid >> 1, wc = wid & 1;
  const int cl = lane & 15;
  const int tpi = (a.Ho + 1) >> 1;  // tiles per image
  // a contiguous run of tiles per workgroup: consecutive tiles share two window rows (L2 hits)
  const int t_begin = (int)(((int64_t)blockIdx.x * ntiles) / gridDim.x);
  const int t_end = (int)(((int64_t)(blockIdx.x + 1) * ntiles) / gridDim.x);
  if (t_begin >= t_end) return;
  float kshift[2] = {0.f, 0.f};
  if constexpr (STATS) {
#pragma unroll
    for (int j = 0; j < 2; ++j) kshift[j] = a.shift[wc * 32 + j * 16 + cl];
  }
  const rsrc_t xr = make_rsrc(a.x, a.xbytes);
  const rsrc_t wrs = make_rsrc(a.w, a.wbytes);
  // weights: tap t rows n = 0..63 of k = t*64 .. t*64+63, K-major swizzled images (72 pieces of 1 KiB)
  for (int pc = wid; pc < 72; pc += 4) {
    const int t = pc >> 3, row = (pc & 7) * 8 + (lane >> 3);
    const int kc = (lane & 7) ^ hx_swz(row);
    const uint32_t off = ((uint32_t)row * (uint32_t)a.K + (uint32_t)(t * 64 + kc * 8)) * 2u;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (__attribute__((address_space(3))) void*)(wlds + pc * 1024), 16, off,
                                             0, 0, 0);
  }
  // the input window of tile `tile` into buffer b: rows ho0-1 .. ho0+2, slots wi = -1 .. 62
  auto stage = [&](int tile, int b) {
    const int n = tile / tpi, ho0 = (tile - n * tpi) * 2;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int pc = i * 4 + wid;
      const int row = pc * 8 + (lane >> 3);
      const int jj = row >> 6, ws = row & 63;
      const int hi = ho0 - 1 + jj, wi = ws - 1;
      const int kc = (lane & 7) ^ hx_swz(row);
      const bool ok = (unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W;
      const uint32_t off = ok ? ((((uint32_t)((n * a.H + hi) * a.W + wi)) << 6) + (uint32_t)(kc * 8)) * 2u : kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (__attribute__((address_space(3))) void*)(winb(b) + pc * 1024), 16,
                                               off, 0, 0, 0);
    }
  };
  stage(t_begin, 0);
  wait_vm<0>();
  __syncthreads();
  uint8_t* stg = smem + kHxW + 2 * kHxWin + wid * 2048;
  EpiSums<2> es;  // this wave's reductions over all its tiles: one partial row per (workgroup, wave row)
  es.zero();
  // output pixel of row p of tile tl (2 output rows x 64 slots; -1 outside the image)
  auto pix_of = [&](int tl) {
    const int n = tl / tpi, ho0 = (tl - n * tpi) * 2;
    return [=](int p) -> int {
      const int j = p >> 6, wo = p & 63;
      return ((wo < a.Wo) & (ho0 + j < a.Ho)) ? (n * a.Ho + ho0 + j) * a.Wo + wo : -1;
    };
  };
  for (int tile = t_begin, it = 0; tile < t_end; ++tile, ++it) {
    const int b = it & 1;
    if (tile + 1 < t_end) stage(tile + 1, b ^ 1);  // lands under this tile's taps + epilogue
    const uint8_t* win = winb(b);
    f32x4 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // the 12 fragments of one tap (A: 4 row blocks, B: 2 column blocks, 2 k-steps each)
    auto load_tap = [&](int tap, bf16x8 (&af)[2][4], bf16x8 (&bf)[2][2]) {
      const int tr = tap / 3, ts = tap - tr * 3;
      const uint8_t* Bs = wlds + tap * 8192;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
          bf[ks][j] = __builtin_bit_cast(
              bf16x8, *reinterpret_cast<const u32x4*>(Bs + hx_off((wc * 2 + j) * 16 + (lane & 15), ks * 4 + (lane >> 4))));
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = (wr + tr) * 64 + i * 16 + (lane & 15) + ts;
          af[ks][i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(win + hx_off(row, ks * 4 + (lane >> 4))));
        }
      }
    };
    // software pipeline over the taps: tap t+1's fragments are read while tap t's 16 MFMAs run (one
    // wave per SIMD: nothing else hides the LDS latency; left to itself hipcc re-used 16 VGPRs and
    // waited on the LDS before every MFMA pair)
    bf16x8 fa[2][2][4], fb[2][2][2];
    load_tap(0, fa[0], fb[0]);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int cb = tap & 1;
      if (tap + 1 < 9) load_tap(tap + 1, fa[cb ^ 1], fb[cb ^ 1]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[cb][ks][i], fb[cb][ks][j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    // this wave's DMA of the next window landed (issued before the taps: nothing to wait for by
    // now) -- BEFORE the epilogue, so the drain never waits on the epilogue's own stores. (Loading the
    // epilogue operands one tile ahead, before the taps -- epi_load with PRE -- measured slower for
    // the mode-1 dgrad: 0.470 vs 0.445 ms, profiles/r5/resnet50_b1024_r5g_autotune.txt)
    wait_vm<0>();
    convn_epilogue<128, 64, 32, STATS, BWD, true>(a, acc, kshift, tile, wr, wc, lane, stg, pix_of(tile), 0, es);
    __syncthreads();  // every wave's: the next window is complete and this one no longer read
  }
  convn_flush<32, STATS, BWD>(a, es, (int64_t)blockIdx.x * 2 + wr, wc, lane, 0);
}

static bool convh_ok(const ConvnArgs& a) {
  return a.N == 64 && a.logC == 6 && a.R == 3 && a.S == 3 && a.stride == 1 && a.pad == 1 && a.H == a.Ho &&
         a.W == a.Wo && a.Wo + 2 <= 64 && !a.x2 && a.K == 576 && a.ldc == 64;
}

static int convh_grid(int ntiles) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || cus <= 0)
      cus = 256;
  }
  return ntiles < cus ? ntiles : cus;
}

template <bool STATS, int BWD>
static hipError_t convh_launch_t(const ConvnArgs& a, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    const hipError_t e =
        hipFuncSetAttribute((const void*)convh_kernel<STATS, BWD>, hipFuncAttributeMaxDynamicSharedMemorySize, kHxLds);
    if (e != hipSuccess) return e;
    attr = true;
  }
  const int ntiles = (a.M / (a.Ho * a.Wo)) * ((a.Ho + 1) / 2);
  hipLaunchKernelGGL((convh_kernel<STATS, BWD>), dim3(convh_grid(ntiles)), dim3(256), kHxLds, st, a, ntiles);
  return hipGetLastError();
}

static hipError_t convh_launch(const ConvnArgs& a, hipStream_t st) {
  if (a.bwd == 1) return convh_launch_t<false, 1>(a, st);
  if (a.bwd == 2) return convh_launch_t<false, 2>(a, st);
  if (a.bwd == 3) return convh_launch_t<false, 3>(a, st);
  if (a.bwd == 5) return convh_launch_t<false, 5>(a, st);
  return a.part ? convh_launch_t<true, 0>(a, st) : convh_launch_t<false, 0>(a, st);
}

// ------------------------------------------------------------------ persistent 1x1: host side
static int cu_count_cached() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || cus <= 0)
      cus = 256;
  }
  return cus;
}

// convp geometry per output-tile width: (WNT, waves, LDS bytes) -- NSLOT 3 ring
template <int BN>
struct P1Cfg;
template <>
struct P1Cfg<256> {
  static constexpr int WNT = 64;
};
template <>
struct P1Cfg<128> {
  static constexpr int WNT = 32;
};
template <>
struct P1Cfg<64> {
  static constexpr int WNT = 32;
};
constexpr int kP1Slots = 3;
template <int BN>
constexpr int p1_lds() {
  using G = Geo<128, BN, P1Cfg<BN>::WNT, kP1Slots>;
  return kP1Slots * G::SLOT + G::NW * G::STG;
}

// workgroups along M: one round of the whole grid (column tiles x this) over the CUs at the
// occupancy the LDS allows, never more than the M tiles
// workgroups along M: one workgroup per CU over the whole grid (column tiles x this), never more
// than the M tiles -- both forms run one 512-thread workgroup per CU (LDS), and the partial-row
// count (convn_part_rows) must not depend on which form the launch takes
static int convp_grid_x(int tiles_m, int tiles_n) {
  int g = cu_count_cached() / (tiles_n > 0 ? tiles_n : 1);
  if (g < 1) g = 1;
  return g < tiles_m ? g : tiles_m;
}

template <int BN, bool STATS, int BWD>
static hipError_t convp_launch_t(const ConvnArgs& a0, hipStream_t st, int grid_mul = 1) {
  constexpr int WNT = P1Cfg<BN>::WNT;
  using G = Geo<128, BN, WNT, kP1Slots>;
  constexpr int LDS = p1_lds<BN>();
  static_assert(LDS <= 160 * 1024, "LDS");
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)convp_kernel<BN, WNT, kP1Slots, STATS, BWD>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    if (e != hipSuccess) return e;
    attr = true;
  }
  ConvnArgs a = a0;
  a.nslot = kP1Slots;
  const int tiles_m = (a.M + 127) / 128, tiles_n = a.N / BN;
  int gx = convp_grid_x(tiles_m, tiles_n) * grid_mul;
  if (gx > tiles_m) gx = tiles_m;
  hipLaunchKernelGGL((convp_kernel<BN, WNT, kP1Slots, STATS, BWD>), dim3(gx, tiles_n), dim3(G::NT), LDS, st, a,
                     tiles_m);
  return hipGetLastError();
}

// resident-B LDS: weights nt * BN * 128 + ring slots x 16 KiB + staging; 0 when even 3 slots do
// not fit (then the streamed ring)
template <int BN>
static int pr_slots(int K) {
  using G = Geo<128, BN, P1Cfg<BN>::WNT, 3>;
  const int fixed = (K / kBK) * BN * 128 + G::NW * G::STG;
  int ns = (160 * 1024 - fixed) / (128 * 128);
  if (ns > kPrMaxSlots) ns = kPrMaxSlots;
  return ns >= 3 ? ns : 0;
}

template <int BN, bool STATS, int BWD>
static hipError_t convpr_launch_t(const ConvnArgs& a0, int ns, hipStream_t st, int grid_mul = 1) {
  constexpr int WNT = P1Cfg<BN>::WNT;
  using G = Geo<128, BN, WNT, 3>;
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)convpr_kernel<BN, WNT, STATS, BWD>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr = true;
  }
  ConvnArgs a = a0;
  a.nslot = ns;
  const int lds = (a.K / kBK) * BN * 128 + ns * 128 * 128 + G::NW * G::STG;
  const int tiles_m = (a.M + 127) / 128, tiles_n = a.N / BN;
  int gx = convp_grid_x(tiles_m, tiles_n) * grid_mul;
  if (gx > tiles_m) gx = tiles_m;
  hipLaunchKernelGGL((convpr_kernel<BN, WNT, STATS, BWD>), dim3(gx, tiles_n), dim3(G::NT), lds, st, a, tiles_m);
  return hipGetLastError();
}

template <int BN>
static hipError_t convpr_launch_s(const ConvnArgs& a, int ns, hipStream_t st, int gm = 1) {
  if (a.bwd == 1) return convpr_launch_t<BN, false, 1>(a, ns, st, gm);
  if (a.bwd == 2) return convpr_launch_t<BN, false, 2>(a, ns, st, gm);
  if (a.bwd == 3) return convpr_launch_t<BN, false, 3>(a, ns, st, gm);
  if (a.bwd == 5) return convpr_launch_t<BN, false, 5>(a, ns, st, gm);
  if (a.bwd == 8) return convpr_launch_t<BN, false, 8>(a, ns, st, gm);
  return a.part ? convpr_launch_t<BN, true, 0>(a, ns, st, gm) : convpr_launch_t<BN, false, 0>(a, ns, st, gm);
}

template <int BN>
static hipError_t convp_launch_s(const ConvnArgs& a, hipStream_t st, int gm = 1) {
  if (const int ns = pr_slots<BN>(a.K)) return convpr_launch_s<BN>(a, ns, st, gm);
  if (a.bwd == 1) return convp_launch_t<BN, false, 1>(a, st, gm);
  if (a.bwd == 2) return convp_launch_t<BN, false, 2>(a, st, gm);
  if (a.bwd == 3) return convp_launch_t<BN, false, 3>(a, st, gm);
  if (a.bwd == 5) return convp_launch_t<BN, false, 5>(a, st, gm);
  if (a.bwd == 8) return convp_launch_t<BN, false, 8>(a, st, gm);
  return a.part ? convp_launch_t<BN, true, 0>(a, st, gm) : convp_launch_t<BN, false, 0>(a, st, gm);
}

// The two-workgroup form of the resident-B 1x1 kernel (variant kind 3, "p2"): a two-slot ring
// (one A K-tile ahead) and twice the workgroups, two per CU when weights + ring + staging fit in
// half the LDS. The epilogue-heavy passes (a bwd-data with the BN reduction: dr / mask reads and
// the g stores per 128x256 tile against one 16 KiB A K-tile; the tail's apply pass) otherwise
// expose each tile's epilogue load latency at one workgroup per CU; the second workgroup's
// K-tile and epilogue run underneath. Shapes whose weights do not fit take the same grid on the
// single-workgroup ring (the partial-row count depends only on the grid).
template <int BN>
static hipError_t convp2_launch_s(const ConvnArgs& a, hipStream_t st) {
  using G = Geo<128, BN, P1Cfg<BN>::WNT, 3>;
  const int lds2 = (a.K / kBK) * BN * 128 + 2 * 128 * 128 + G::NW * G::STG;
  if (lds2 <= 80 * 1024) return convpr_launch_s<BN>(a, 2, st, 2);
  return convp_launch_s<BN>(a, st, 2);
}

static hipError_t convp2_launch(const ConvnArgs& a, int bn, hipStream_t st) {
  if (a.R != 1 || a.S != 1 || a.stride != 1 || a.pad != 0 || a.Ho != a.H || a.Wo != a.W) return hipErrorNotSupported;
  if (bn == 256) return convp2_launch_s<256>(a, st);
  if (bn == 128) return convp2_launch_s<128>(a, st);
  return convp2_launch_s<64>(a, st);
}

static hipError_t convp_launch(const ConvnArgs& a, int bn, hipStream_t st) {
  if (a.R != 1 || a.S != 1 || a.stride != 1 || a.pad != 0 || a.Ho != a.H || a.Wo != a.W) return hipErrorNotSupported;
  if (bn == 256) return convp_launch_s<256>(a, st);
  if (bn == 128) return convp_launch_s<128>(a, st);
  return convp_launch_s<64>(a, st);
}

// ------------------------------------------------------------------ host side
template <int BM, int BN, int WNT, int NSLOT, bool STATS, int BWD>
static hipError_t convn_launch_t(const ConvnArgs& a0, hipStream_t st) {
  using G = Geo<BM, BN, WNT, NSLOT>;
  constexpr int LDS_MAX = NSLOT * G::SLOT + G::NW * G::STG;
  static_assert(LDS_MAX <= 160 * 1024, "LDS");
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)convn_kernel<BM, BN, WNT, NSLOT, STATS, BWD>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    if (e != hipSuccess) return e;
    attr = true;
  }
  ConvnArgs a = a0;
  const int nt = a.K / kBK;
  a.nslot = nt < NSLOT ? (nt < 2 ? 1 : nt) : NSLOT;
  const int lds = a.nslot * G::SLOT + G::NW * G::STG;
  const int tiles_m = (a.M + BM - 1) / BM;
  hipLaunchKernelGGL((convn_kernel<BM, BN, WNT, NSLOT, STATS, BWD>), dim3(tiles_m, a.N / BN), dim3(G::NT), lds, st, a);
  return hipGetLastError();
}

template <int BM, int BN, int WNT, int NSLOT>
static hipError_t convn_launch_s(const ConvnArgs& a, hipStream_t st) {
  if (a.bwd == 1) return convn_launch_t<BM, BN, WNT, NSLOT, false, 1>(a, st);
  if (a.bwd == 2) return convn_launch_t<BM, BN, WNT, NSLOT, false, 2>(a, st);
  if (a.bwd == 3) return convn_launch_t<BM, BN, WNT, NSLOT, false, 3>(a, st);
  if (a.bwd == 5) return convn_launch_t<BM, BN, WNT, NSLOT, false, 5>(a, st);
  if (a.bwd == 8) return convn_launch_t<BM, BN, WNT, NSLOT, false, 8>(a, st);
  return a.part ? convn_launch_t<BM, BN, WNT, NSLOT, true, 0>(a, st)
                : convn_launch_t<BM, BN, WNT, NSLOT, false, 0>(a, st);
}

int convn_tile_n(int N) {
  if (N == 64) return 64;
  if (N == 128) return 128;
  if (N % 256 == 0) return 256;
  return 0;
}

// variants (tile geometry) per output width: the gathered ones (kind 0), then the persistent HALO
// variant (convh_kernel, kind 2) for the 64-wide outputs, then the persistent 1x1 variant
// (convp_kernel, kind 3) and its two-workgroups-per-CU form (kind 4). (The one-tile HALO variants -- kind 1 -- measured no faster than the
// gathered ones on the ResNet-50 shapes, profiles/convn_halo_r3.md, and were removed in round 5.)
static int plain_count(int bn) { return bn == 256 ? 3 : 4; }
static int persist_count(int bn) { return bn == 64 ? 1 : 0; }
static int p1_count(int bn) { return bn ? 2 : 0; }  // the persistent 1x1: one and two workgroups per CU
static int convn_variant_count(int bn) { return plain_count(bn) + persist_count(bn) + p1_count(bn); }
static bool is_persist(int bn, int v) { return v >= plain_count(bn) && v < plain_count(bn) + persist_count(bn); }
static bool is_p1(int bn, int v) { return v == plain_count(bn) + persist_count(bn); }
static bool is_p2(int bn, int v) { return v == plain_count(bn) + persist_count(bn) + 1; }

int convn_variant_kind(int N, int v) {
  const int bn = convn_tile_n(N);
  if (!bn || v < 0 || v >= convn_variant_count(bn)) return -1;
  return v < plain_count(bn) ? 0 : is_persist(bn, v) ? 2 : is_p1(bn, v) ? 3 : 4;
}

int convn_variants(int N) {
  const int bn = convn_tile_n(N);
  return bn ? convn_variant_count(bn) : 0;
}

static int default_variant(const ConvnArgs& a, int bn) {
  (void)a;
  (void)bn;
  return 0;
}

// BM of each variant (must match the dispatch in launch_convn)
static int variant_bm(int bn, int v) {
  if (is_persist(bn, v) || is_p1(bn, v) || is_p2(bn, v)) return 128;
  if (bn == 64) return (v == 2 || v == 3) ? 256 : 128;
  if (bn == 128) return v == 2 ? 256 : 128;
  return 128;
}

bool convn_variant_ok(int N, int v, int R, int S, int stride, int pad, int Wo, bool has_x2) {
  const int bn = convn_tile_n(N);
  if (!bn || v < 0 || v >= convn_variant_count(bn)) return false;
  if (v < plain_count(bn)) return true;
  if (is_p1(bn, v) || is_p2(bn, v)) return R == 1 && S == 1 && stride == 1 && pad == 0;
  // persistent HALO (C = 64 and H = Ho are checked at launch: the predicate has no C)
  return !has_x2 && N == 64 && R == 3 && S == 3 && stride == 1 && pad == 1 && Wo + 2 <= 64;
}

int convn_stats_rows(int M) { return 4 * ((M + 255) / 256) + 4; }  // >= (BM/64) * tiles for the gathered variants

int convn_part_rows_geo(int M, int N, int variant, int Ho, int Wo, int R) {
  const int bn = convn_tile_n(N);
  if (!bn) return 0;
  const int bm = variant_bm(bn, variant);
  if (is_persist(bn, variant)) {  // one row per (workgroup, wave row): convh_kernel's flush
    if (Ho <= 0 || Wo <= 0) return 0;
    return 2 * convh_grid((M / (Ho * Wo)) * ((Ho + 1) / 2));
  }
  if (is_p1(bn, variant)) return 2 * convp_grid_x((M + 127) / 128, N / bn);
  if (is_p2(bn, variant)) {
    const int t = (M + 127) / 128, g = 2 * convp_grid_x(t, N / bn);
    return 2 * (g < t ? g : t);
  }
  return (bm / 64) * ((M + bm - 1) / bm);
}

int convn_part_rows(int M, int N, int variant) { return convn_part_rows_geo(M, N, variant, 0, 0, 1); }

hipError_t launch_convn(const ConvnArgs& a_in, hipStream_t st) {
  if (a_in.M <= 0) return hipSuccess;
  ConvnArgs a = a_in;
  if (!a.x2) a.K1 = a.K;  // every K-tile from x
  const int bn = convn_tile_n(a.N);
  const int C = 1 << a.logC;
  const bool two = a.x2 != nullptr;
  const int K1 = two ? a.K1 : a.K;
  const bool ok = bn > 0 && a.logC >= 6 && a.K % kBK == 0 && K1 == a.R * a.S * C && a.ldc % 8 == 0 &&
                  (!two || (a.R == 1 && a.S == 1 && a.stride == 1 && a.pad == 0 && a.logC2 >= 6 && K1 % kBK == 0 &&
                            a.K == K1 + (1 << a.logC2) && a.x2bytes > 0 && a.x2bytes <= 0xFFFFFF00u)) &&
                  a.ldc >= a.N && a.H < 32768 && a.W < 32768 && a.xbytes > 0 && a.xbytes <= 0xFFFFFF00u &&
                  a.wbytes > 0 && a.variant < convn_variant_count(bn) &&
                  (a.y || (a.bwd == 0 && a.part)) &&
                  (a.bwd == 0 ? (!a.part || a.shift)
                   : a.bwd == 8 ? (!a.part && a.bss && a.amask && a.ldc == a.N && a.N % 8 == 0)
                              : (a.part && (a.bx || a.bwd >= 2) && a.bmean && a.ldc == a.N &&
                                 (a.bwd == 1 ? a.bss != nullptr
                                             : ((a.bwd == 2 || a.bwd == 3 || a.bwd == 5) && a.bdr && a.bmbits &&
                                                (a.bwd != 3 || (a.bxd && a.bmean_d && a.part_d)) &&
                                                (a.bwd != 5 || (a.Ho % 2 == 0 && a.Wo % 2 == 0))))));
  if (!ok) return hipErrorNotSupported;
  // phase launches (stride-2 bwd-data): the gathered variants only, stride 1 / pad 0 over dY, no
  // second operand, the plain or mode-1 epilogue; fdiv's exact range for the pixel map
  if (a.ophase != 0 &&
      (a.ophase > 4 || a.variant < 0 || a.variant >= plain_count(bn) || two || a.stride != 1 || a.pad != 0 ||
       (a.bwd != 0 && a.bwd != 1) || a.M >= (1 << 24) || a.R > 2 || a.S > 2 ||
       (int64_t)a.M * 4 * a.ldc * 2 > 0x7FFFFFFFll))
    return hipErrorNotSupported;
  const int v = a.variant >= 0 ? a.variant : default_variant(a, bn);
  if (is_p1(bn, v)) return convp_launch(a, bn, st);
  if (is_p2(bn, v)) return convp2_launch(a, bn, st);
  if (is_persist(bn, v)) {
    if (!convh_ok(a) || a.bwd == 8 || !a.y) return hipErrorNotSupported;
    return convh_launch(a, st);
  }
  switch (bn) {
    case 64:  // 4 waves of 64x32 (3 / 2 slots) | 4 waves of 64x64 (BM 256) | 8 waves of 64x32 (BM 256)
      if (v == 0) return convn_launch_s<128, 64, 32, 3>(a, st);
      if (v == 1) return convn_launch_s<128, 64, 32, 2>(a, st);
      if (v == 2) return convn_launch_s<256, 64, 64, 3>(a, st);
      return convn_launch_s<256, 64, 32, 3>(a, st);
    case 128:  // 8 waves of 64x32 (3 / 2 slots) | 4 waves of 64x64 | 8 waves of 64x64 (BM 256)
      if (v == 0) return convn_launch_s<128, 128, 32, 3>(a, st);
      if (v == 1) return convn_launch_s<128, 128, 64, 3>(a, st);
      if (v == 2) return convn_launch_s<256, 128, 64, 2>(a, st);
      return convn_launch_s<128, 128, 32, 2>(a, st);
    default:  // 8 waves of 64x64, 3 or 2 slots | 128-wide column tiles on a 2-slot ring (80 KiB: two
              // workgroups per CU; the 256-wide tile's 2- and 3-slot rings hold the CU alone)
      if (v == 0) return convn_launch_s<128, 256, 64, 3>(a, st);
      if (v == 1) return convn_launch_s<128, 256, 64, 2>(a, st);
      return convn_launch_s<128, 128, 32, 2>(a, st);
  }
}

}  // namespace psd
