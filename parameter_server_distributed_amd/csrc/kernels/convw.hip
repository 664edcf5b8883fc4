// Narrow implicit-GEMM convolution weight gradient for gfx950 (NHWC bf16), split over the output
// pixels.
//
//   dW[co][kk] = sum_m dY[m][co] * A(m, kk)      m = output pixel (Nb*Ho*Wo), kk = (r, s, ci),
//                                                A(m, kk) = x[pixel(m) * stride - pad + (r, s)][ci]
//
// Why its own kernel: the weight gradients of ResNet's 64/128-channel layers are pure HBM streams
// (layer1's 1x1 256->64: 2 GB of dY + x read for 0.1 TFLOP) that MIOpen's assembly kernels ran at
// about the copy roofline while the 256x256-tile split-K GEMM (gemm.hip) wasted 3/4 of its tile on
// a 64-row output (2-4x slower: profiles/resnet50_b1024_r3_bnbwd_twin_autotune.txt). Here the tile
// is the narrow output itself, so every dY and x element is read from HBM once:
//   * workgroup = 8 waves, output tile TCO (64 / 128 / 256 output channels) x TKK (64..256 columns
//     = 1..4 K-blocks of 64 channels of one (r, s)); a wave owns I x J 16x16 blocks of it on
//     v_mfma_f32_16x16x32_bf16 (the MFMA k = 32 output pixels);
//   * a stage = 64 output pixels: the dY rows [64 px][TCO] and, per K-block, the gathered input
//     rows [64 px][64 ch] are DMA'd straight into LDS (buffer_load ... lds, 16 B per lane; a pixel
//     outside the image or past M falls outside the buffer range and loads zeros = the padding) as
//     [64 px][64 ch] sub-images whose 16-B chunks are XOR-swizzled by row bits 1 and 3 on the SOURCE
//     address (the DMA image is lane-linear);
//   * both operands are pixel-major, so every MFMA fragment is read with the CDNA4 transpose read
//     ds_read_b64_tr_b16 (8 consecutive pixels of one channel per lane); with the swizzle the 8 rows
//     of a 32-lane half cover all 64 banks (conflict-free);
//   * NSLOT-deep stage ring, one raw s_barrier per stage and a counted vmcnt (the later stages stay
//     in flight), like convn.hip; every lane of a wave moves the same pixel row in all its pieces,
//     so the pixel -> (n, ho, wo) division runs once per lane per stage;
//   * grid = pixel splits x output tiles (XCD-aware order: the tiles of one split -- which share
//     their dY stage -- land on one XCD's L2), sized to one round of workgroups; each split writes
//     its fp32 partial tile to a slab, the deterministic slab reduce (gemm.hip) writes bf16 dW.
#include <algorithm>

#include "common.h"
#include "launchers_convw.h"
#include "launchers_gemm.h"

namespace psd {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __amdgpu_buffer_rsrc_t rsrc_t;

constexpr int kBP = 64;                  // output pixels per stage (two 32-deep MFMA k-steps)
constexpr int kSub = 64 * 128;           // one [64 px][64 ch] bf16 sub-image
constexpr uint32_t kOOB = 0xFFFFFFF0u;   // past every descriptor's range: the load returns zeros

__device__ __forceinline__ rsrc_t make_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

// 16-B chunk c of sub-image row r is stored at chunk c ^ swz(r). A ds_read_b64_tr_b16 fragment read
// touches, per 32-lane half, rows {q, q + 8} (q = 0..3, plus a multiple of 16) with one 32-B segment
// each; (r & 1, swz) is distinct on those 8 rows, so they cover the 8 segments of a 256-B bank row.
__device__ __forceinline__ int swz(int r) { return (((r >> 1) & 1) | (((r >> 3) & 1) << 1)) << 1; }

// v_mfma_f32_16x16x32_bf16 operand from a [64 px][64 ch] sub-image: lane -> channel cb*16 + (lane & 15),
// pixels ks*32 + 8*(lane >> 4) + 0..7 (the MFMA k). Transpose read: lane 4q+p of a 16-lane group
// addresses row q, channels 4p..4p+3; lane i receives channel i of the 4 rows.
__device__ __forceinline__ bf16x8 trfrag(const uint8_t* sub, int ks, int cb, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int r0 = ks * 32 + 8 * g + q, r1 = r0 + 4;
  const int c = 2 * cb + (p >> 1), b = (p & 1) * 8;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(sub + r0 * 128 + ((c ^ swz(r0)) << 4) + b));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(sub + r1 * 128 + ((c ^ swz(r1)) << 4) + b));
  const s16x4 both[2] = {lo, hi};
  return __builtin_bit_cast(bf16x8, both);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
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
  const float r0 = dpp_q<0xB1>(o1 ? v[0] : v[1]);
  const float r1 = dpp_q<0xB1>(o1 ? v[2] : v[3]);
  const float a0 = o1 ? r0 : v[0], a1 = o1 ? v[1] : r0;
  const float b0 = o1 ? r1 : v[2], b1 = o1 ? v[3] : r1;
  const float q0 = dpp_q<0x4E>(o2 ? a0 : b0);
  const float q1 = dpp_q<0x4E>(o2 ? a1 : b1);
  w[0] = o2 ? q0 : a0;
  w[1] = o2 ? q1 : a1;
  w[2] = o2 ? b0 : q0;
  w[3] = o2 ? b1 : q1;
}

template <int TCO, int TKK, int WR, int NSLOT, int NAR = -1>
struct WGeo {
  static constexpr int NW = 8;                // waves (one DMA piece = 8 pixel rows each)
  static constexpr int NT = 64 * NW;
  static constexpr int WC = NW / WR;          // wave columns
  static constexpr int I = TCO / 16 / WR;     // 16-row blocks per wave
  static constexpr int J = TKK / 16 / WC;     // 16-column blocks per wave
  // dY sub-images per stage: every row of the tile, or (NAR >= 0: a single-tile fold launch) only
  // the first NAR * 64 rows -- the rest are x rows (read from the B sub-images) and ones
  static constexpr int NA = NAR >= 0 ? NAR : TCO / 64;
  static constexpr int NB = TKK / 64;         // x sub-images (K-blocks) per stage
  static constexpr int DPS = NA + NB;         // DMA per wave per stage: one 1 KiB piece of each sub-image
  static constexpr int SLOT = DPS * kSub;
  static constexpr int LDS = NSLOT * SLOT;
  static_assert(I >= 1 && J >= 1 && I * 16 * WR == TCO && J * 16 * WC == TKK, "wave tiling");
  static_assert(I * J <= 16, "accumulators");
  static_assert(DPS * (NSLOT - 2) < 64 && NSLOT <= 5, "vmcnt is 6 bits");
  static_assert(LDS <= 160 * 1024, "LDS");
};

}  // namespace

template <int TCO, int TKK, int WR, int NSLOT, int NAR = -1>
__global__ __launch_bounds__(512) void convw_kernel(ConvwArgs a) {
  using G = WGeo<TCO, TKK, WR, NSLOT, NAR>;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tiles_co = a.Arows / TCO;
  const int ntile = tiles_co * (a.KK / TKK);
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = bid / ntile, tile = bid - split * ntile;
  const int co0 = (tile % tiles_co) * TCO, kk0 = (tile / tiles_co) * TKK;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid / G::WC, wc = wid % G::WC;
  const int prow = wid * 8 + (lane >> 3);       // this lane's pixel row in every piece it moves
  const int kc = (lane & 7) ^ swz(prow);        // the global 16-B chunk it moves into LDS chunk lane & 7
  const int howo = a.Ho * a.Wo;
  const int cmask = (1 << a.logC) - 1;
  const rsrc_t dyr = make_rsrc(a.dy, a.dybytes);
  const rsrc_t xr = make_rsrc(a.x, a.xbytes);
  // the (r, s, ci0) of each K-block are fixed for this workgroup's column tile: resolved once here,
  // not per stage (a runtime `/ S` per K-block and stage was a ~30-instruction VALU sequence)
  int kb_r[G::NB], kb_s[G::NB], kb_ci[G::NB];
#pragma unroll
  for (int b = 0; b < G::NB; ++b) {
    const int k0 = kk0 + b * 64;
    const int rs = k0 >> a.logC;
    kb_ci[b] = k0 & cmask;
    kb_r[b] = rs / a.S;
    kb_s[b] = rs - kb_r[b] * a.S;
  }
  const FastDiv dhw{(uint32_t)howo, a.howo_m, a.howo_s}, dwo{(uint32_t)a.Wo, a.wo_m, a.wo_s};

  const int total = (a.M + kBP - 1) / kBP;
  const int st0 = split * a.stages_per_split;
  const int nst = max(0, min(a.stages_per_split, total - st0));

  auto stage = [&](int t) {
    uint8_t* slot = smem + (t % NSLOT) * G::SLOT + wid * 1024;
    const int m = (st0 + t) * kBP + prow;
    const bool mv = m < a.M;
#pragma unroll
    for (int j = 0; j < G::NA; ++j) {
      // fold rows past dY are read from the x sub-images / constants: their DMA loads nothing (out of
      // range) but keeps every wave's per-stage count equal to DPS (the counted vmcnt)
      const bool dyrow = co0 + j * 64 < a.Cout;
      const uint32_t off = (mv && dyrow) ? ((uint32_t)m * (uint32_t)a.Cout + (uint32_t)(co0 + j * 64 + kc * 8)) * 2u : kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(dyr, (__attribute__((address_space(3))) void*)(slot + j * kSub), 16,
                                               off, 0, 0, 0);
    }
    // (n, ho, wo) of the pixel by multiply-high (m < 2^31): the per-stage integer divisions by the
    // runtime Ho*Wo and Wo were ~60 VALU per lane per stage
    const int n = (int)fdiv_q((uint32_t)m, dhw), rem = m - n * howo;
    const int ho = (int)fdiv_q((uint32_t)rem, dwo), wo = rem - ho * a.Wo;
    const int hb = ho * a.stride - a.pad, wb = wo * a.stride - a.pad;
#pragma unroll
    for (int b = 0; b < G::NB; ++b) {
      const int ci0 = kb_ci[b];
      const int r = kb_r[b], s = kb_s[b];
      const int hh = hb + r, ww = wb + s;
      const bool ok = mv && (unsigned)hh < (unsigned)a.H && (unsigned)ww < (unsigned)a.W;
      const uint32_t off =
          ok ? ((((uint32_t)((n * a.H + hh) * a.W + ww)) << a.logC) + (uint32_t)(ci0 + kc * 8)) * 2u : kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (__attribute__((address_space(3))) void*)(slot + (G::NA + b) * kSub),
                                               16, off, 0, 0, 0);
    }
  };

  f32x4 acc[G::I][G::J];
#pragma unroll
  for (int i = 0; i < G::I; ++i)
#pragma unroll
    for (int j = 0; j < G::J; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  constexpr int D = NSLOT - 1;  // stages issued ahead
  for (int p = 0; p < D && p < nst; ++p) stage(p);
  for (int t = 0; t < nst; ++t) {
    // stage t landed (this wave's DMA): leave the (up to D-1) later stages in flight
    const int ahead = min(nst - 1 - t, D - 1);
    if constexpr (D >= 4) {
      if (ahead >= 3) wait_vm<3 * G::DPS>();
      else if (ahead == 2) wait_vm<2 * G::DPS>();
      else if (ahead == 1) wait_vm<G::DPS>();
      else wait_vm<0>();
    } else if constexpr (D == 3) {
      if (ahead >= 2) wait_vm<2 * G::DPS>();
      else if (ahead == 1) wait_vm<G::DPS>();
      else wait_vm<0>();
    } else if constexpr (D == 2) {
      if (ahead >= 1) wait_vm<G::DPS>();
      else wait_vm<0>();
    } else {
      wait_vm<0>();
    }
    __builtin_amdgcn_s_barrier();  // every wave: stage t published, stage t-1 no longer read
    __builtin_amdgcn_sched_barrier(0);
    if (t + D < nst) stage(t + D);
    const uint8_t* sl = smem + (t % NSLOT) * G::SLOT;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[G::I], bf[G::J];
#pragma unroll
      for (int j = 0; j < G::J; ++j) {
        const int cbk = wc * G::J + j;  // 16-column block of the tile
        bf[j] = trfrag(sl + (G::NA + (cbk >> 2)) * kSub, ks, cbk & 3, lane);
      }
#pragma unroll
      for (int i = 0; i < G::I; ++i) {
        const int rb = wr * G::I + i;  // 16-row block of the tile
        const int gr = co0 + rb * 16;  // its first output row (wave-uniform source choice)
        if (gr < a.Cout) {
          af[i] = trfrag(sl + (rb >> 2) * kSub, ks, rb & 3, lane);
        } else if (gr < a.Cout + a.KK) {  // fold: x rows = the B sub-images of this (whole-KK) tile
          const int xb = (gr - a.Cout) >> 4;
          af[i] = trfrag(sl + (G::NA + (xb >> 2)) * kSub, ks, xb & 3, lane);
        } else {  // fold: ones rows -> column sums of x
          af[i] = bf16x8{(__bf16)1.f, (__bf16)1.f, (__bf16)1.f, (__bf16)1.f, (__bf16)1.f, (__bf16)1.f, (__bf16)1.f,
                         (__bf16)1.f};
        }
      }
#pragma unroll
      for (int i = 0; i < G::I; ++i)
#pragma unroll
        for (int j = 0; j < G::J; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  }

  // epilogue: this split's fp32 partial tile; a lane quad transposes each 16x16 block so a lane
  // stores 4 consecutive columns of one row (16 B)
  float* sl = a.slab + (int64_t)split * a.Arows * a.KK;
  const int L = lane & 3, rq = (lane >> 4) * 4, cq = (lane & 15) & ~3;
#pragma unroll
  for (int i = 0; i < G::I; ++i)
#pragma unroll
    for (int j = 0; j < G::J; ++j) {
      float w[4];
      quad_t4(acc[i][j], L, w);
      const int row = co0 + (wr * G::I + i) * 16 + rq + L;
      const int col = kk0 + (wc * G::J + j) * 16 + cq;
      *reinterpret_cast<f32x4*>(sl + (int64_t)row * a.KK + col) = f32x4{w[0], w[1], w[2], w[3]};
    }
}


// ------------------------------------------------------------------ persistent HALO (layer1 3x3)
// The weight gradient of the C = 64 -> N = 64 3x3 / stride 1 / pad 1 convolution (ResNet layer1
// conv2, 56 x 56): the tiled kernel above gathers the shifted input rows of every (r, s) K-block
// through L2 (9 x the input per pass) and re-reads dY once per column tile; MIOpen's igemm_wrw took
// 0.55 ms at b1024 (profiles/resnet50_b1024_r3_final_kernels.md). Here one workgroup per CU runs a
// contiguous run of output-row tiles (2 rows x 64 slots) and keeps the WHOLE 64 x 576 gradient of
// its run in registers (4 waves; wave w owns input channels 16w..16w+15 of all 9 taps and all 64
// output channels: 36 16x16 accumulators):
//   * per tile the dY rows ([128 slots][64 n], zero past Wo) and the input window (4 rows x 64 slots
//     x 64 channels, zero outside the image) are DMA'd once into LDS, double-buffered under the
//     previous tile's MFMA work -- 48 KiB per 128 output pixels instead of ~200;
//   * per 32-pixel k-step: 4 dY^T fragments (shared by the 9 taps) and 9 window fragments (the tap
//     shift is a row offset into the window), all with the transpose read ds_read_b64_tr_b16,
//     36 MFMAs;
//   * the workgroup's fp32 partial gradient goes to its slab row once at the end; the deterministic
//     slab reduce (gemm.hip) sums the workgroups and writes bf16 dW.
constexpr int kHwDy = 128 * 128;       // dY tile: 128 slots x 64 channels bf16
constexpr int kHwWin = 4 * 64 * 128;   // input window
// buffer = [window | dY]: the last k-step's taps read up to 2 rows past the 4-row window, i.e. the
// first rows of the SAME buffer's dY tile (staged by the same DMA: finite) -- those products meet dY
// rows of padding slots, which are 0. (dY first put the overrun into the other buffer, or past the
// end, where uninitialised LDS holding a NaN pattern made 0 x NaN = NaN in valid gradient entries.)
constexpr int kHwBuf = kHwDy + kHwWin;
constexpr int kHwLds = 2 * kHwBuf;

// transpose-read fragment of rows rbase + 8g + q (and + 4) of a pixel-major [rows][64 ch] image,
// channel block cb (lane -> channel cb*16 + (lane & 15))
__device__ __forceinline__ bf16x8 trfrag_rows(const uint8_t* img, int rbase, int cb, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int r0 = rbase + 8 * g + q, r1 = r0 + 4;
  const int c = 2 * cb + (p >> 1), b = (p & 1) * 8;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + r0 * 128 + ((c ^ swz(r0)) << 4) + b));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + r1 * 128 + ((c ^ swz(r1)) << 4) + b));
  const s16x4 both[2] = {lo, hi};
  return __builtin_bit_cast(bf16x8, both);
}

__global__ __launch_bounds__(256) void convhw_kernel(ConvwArgs a, int ntiles) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tpi = (a.Ho + 1) >> 1;
  const int t_begin = (int)(((int64_t)blockIdx.x * ntiles) / gridDim.x);
  const int t_end = (int)(((int64_t)(blockIdx.x + 1) * ntiles) / gridDim.x);
  const rsrc_t dyr = make_rsrc(a.dy, a.dybytes);
  const rsrc_t xr = make_rsrc(a.x, a.xbytes);
  auto buf = [&](int b) { return smem + b * kHwBuf; };
  // tile `tile` into buffer b: 16 dY pieces + 32 window pieces of 1 KiB (12 per wave)
  auto stage = [&](int tile, int b) {
    const int n = tile / tpi, ho0 = (tile - n * tpi) * 2;
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // dY: image rows = tile slots (row j, slot ws)
      const int pc = i * 4 + wid;
      const int row = pc * 8 + (lane >> 3);
      const int j = row >> 6, ws = row & 63;
      const int kc = (lane & 7) ^ swz(row);
      const bool ok = ws < a.Wo && ho0 + j < a.Ho;
      const uint32_t off = ok ? ((uint32_t)(((n * a.Ho + ho0 + j) * a.Wo + ws)) * 64u + (uint32_t)(kc * 8)) * 2u : kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(dyr, (__attribute__((address_space(3))) void*)(buf(b) + kHwWin + pc * 1024),
                                               16, off, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {  // window: rows ho0-1 .. ho0+2, slot ws = input column ws - 1
      const int pc = i * 4 + wid;
      const int row = pc * 8 + (lane >> 3);
      const int jj = row >> 6, ws = row & 63;
      const int hi = ho0 - 1 + jj, wi = ws - 1;
      const int kc = (lane & 7) ^ swz(row);
      const bool ok = (unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W;
      const uint32_t off = ok ? ((uint32_t)((n * a.H + hi) * a.W + wi) * 64u + (uint32_t)(kc * 8)) * 2u : kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (__attribute__((address_space(3))) void*)(buf(b) + pc * 1024), 16,
                                               off, 0, 0, 0);
    }
  };
  f32x4 acc[9][4];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) acc[t][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (t_begin < t_end) {
    stage(t_begin, 0);
    wait_vm<0>();
    __syncthreads();
  }
  for (int tile = t_begin, it = 0; tile < t_end; ++tile, ++it) {
    const int b = it & 1;
    if (tile + 1 < t_end) stage(tile + 1, b ^ 1);  // lands under this tile's MFMA work
    const uint8_t* win = buf(b);
    const uint8_t* dyi = buf(b) + kHwWin;
    // 4 k-steps of 32 output pixels (row j = ks / 2, slots (ks % 2) * 32 ..) x 9 taps = 36 steps of 4
    // MFMAs, software-pipelined: the window fragment of step s + 2 and the dY fragments of the next
    // k-step are read while step s's MFMAs run (one wave per SIMD: nothing else hides the LDS latency)
    auto wfrag = [&](int st) {
      const int ks = st / 9, t = st - ks * 9, r = t / 3, sx = t - r * 3;
      return trfrag_rows(win, ((ks >> 1) + r) * 64 + (ks & 1) * 32 + sx, wid, lane);
    };
    bf16x8 af[2][4], bw[3];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) af[0][nb] = trfrag_rows(dyi, 0, nb, lane);
    bw[0] = wfrag(0);
    bw[1] = wfrag(1);
#pragma unroll
    for (int st = 0; st < 36; ++st) {
      const int ks = st / 9, t = st - ks * 9;
      if (st + 2 < 36) bw[(st + 2) % 3] = wfrag(st + 2);
      if (t == 0 && ks + 1 < 4) {
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) af[(ks + 1) & 1][nb] = trfrag_rows(dyi, (ks + 1) * 32, nb, lane);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int nb = 0; nb < 4; ++nb)
        acc[t][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks & 1][nb], bw[st % 3], acc[t][nb], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    wait_vm<0>();     // this wave's DMA of the next tile landed
    __syncthreads();  // every wave's: the next tile is complete and this one no longer read
  }
  // this workgroup's partial gradient -> its slab: D[n][c] of 16x16 block (nb, wid) of tap t is
  // row n = nb*16 + 4*(lane >> 4) + i, column kk = t*64 + wid*16 + (lane & 15)
  float* sl = a.slab + (int64_t)blockIdx.x * 64 * 576;
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        sl[(nb * 16 + 4 * (lane >> 4) + i) * 576 + t * 64 + wid * 16 + (lane & 15)] = acc[t][nb][i];
}

// ------------------------------------------------------------------ host side
namespace {

struct Cfg {
  int tco, tkk, lds;
};

// tile variants per output-tile height (TCO): (TKK, WR, NSLOT) instantiated below
constexpr int kTkk64[] = {256, 192, 128, 64};
constexpr int kTkk128[] = {256, 192, 128, 64};
constexpr int kTkk256[] = {128, 64};

int tile_co(int Cout, bool fold = false) {
  if (Cout % 256 == 0) return 256;
  if (Cout == 128 || (fold && Cout % 128 == 0)) return 128;
  if (Cout == 64 || (fold && Cout % 64 == 0)) return 64;
  return 0;
}

// the v-th TKK that divides KK for this TCO (0 when there is none)
int pick_tkk(int tco, int KK, int v) {
  const int* list = tco == 64 ? kTkk64 : tco == 128 ? kTkk128 : kTkk256;
  const int n = tco == 256 ? 2 : 4;
  int k = 0;
  for (int i = 0; i < n; ++i)
    if (KK % list[i] == 0) {
      if (k == v) return list[i];
      ++k;
    }
  return 0;
}

// ring depth: as many stages as fit the 160 KiB LDS (<= 5; 4 for the 2-workgroup 64x64 tile) -- the
// kernel streams HBM, so its bandwidth is set by the stages in flight (3 -> 4 slots: +5-10 %)
constexpr int nslot_of(int tco, int tkk) {
  return (tco + tkk) <= 128 ? 4 : std::min(5, (160 * 1024) / ((tco + tkk) / 64 * kSub));
}
int lds_of(int tco, int tkk, bool two = false) {
  if (tco == 384) return (two ? 2 : 4) * (256 + 64) / 64 * kSub;  // the single-tile fold: 4 dY + 1 x sub-images
  return (two ? 2 : nslot_of(tco, tkk)) * (tco + tkk) / 64 * kSub;
}

int cu_count() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0)
      n = 256;
  }
  return n;
}

template <int TCO, int TKK, int WR, int NSLOT, int NAR = -1>
hipError_t launch_t(const ConvwArgs& a, int grid, hipStream_t st) {
  using G = WGeo<TCO, TKK, WR, NSLOT, NAR>;
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)convw_kernel<TCO, TKK, WR, NSLOT, NAR>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL((convw_kernel<TCO, TKK, WR, NSLOT, NAR>), dim3(grid), dim3(G::NT), G::LDS, st, a);
  return hipGetLastError();
}

}  // namespace

// tile shapes (TCO x TKK) for this launch: the ring as deep as the LDS allows (one workgroup per
// CU for the wider tiles), then (variant + count) the same shapes on a two-stage ring in half the
// LDS at two workgroups per CU -- the HBM-bound large-M shapes stall every wave of a lone workgroup
// at each stage's barrier; a second workgroup's stage runs underneath
static int tile_shapes(int Cout, int KK) {
  const int tco = tile_co(Cout);  // plain launches (fold launches have one fixed tile)
  if (!tco || KK <= 0 || KK % 64 != 0) return 0;
  int n = 0;
  while (pick_tkk(tco, KK, n)) ++n;
  return n;
}
static int tiled_variants(int Cout, int KK) { return 2 * tile_shapes(Cout, KK); }

// + the persistent HALO variant (convhw_kernel) for the 64 -> 64 3x3 shape (KK = 576)
int convw_variants(int Cout, int KK) { return tiled_variants(Cout, KK) + (Cout == 64 && KK == 576 ? 1 : 0); }

static bool is_persist_w(const ConvwArgs& a) {
  return !a.fold && a.Cout == 64 && a.KK == 576 && a.variant == tiled_variants(64, 576);
}
static bool persist_w_ok(const ConvwArgs& a) {
  return is_persist_w(a) && a.logC == 6 && a.S == 3 && a.stride == 1 && a.pad == 1 && a.H == a.Ho && a.W == a.Wo &&
         a.Wo + 2 <= 64 && !a.accumulate;
}
static int persist_w_tiles(const ConvwArgs& a) { return (a.M / (a.Ho * a.Wo)) * ((a.Ho + 1) / 2); }

// (tco, tkk) of a launch, 0 when unsupported; fold launches take the whole KK in one tile
static void tile_of(const ConvwArgs& a, int& tco, int& tkk) {
  const int rows = a.fold ? a.Arows : a.Cout;
  tco = tile_co(rows, a.fold != 0);
  tkk = 0;
  if (!tco) return;
  if (a.fold) {
    if (a.Cout == 256 && a.KK == 64 && a.Arows == 384) {  // one tile holds every row: dY read once
      tco = 384;
      tkk = 64;
      return;
    }
    for (int v = 0; pick_tkk(tco, a.KK, v); ++v)
      if (pick_tkk(tco, a.KK, v) == a.KK) tkk = a.KK;
    if (!tkk && tco > 64 && a.KK <= 256) {  // a narrower row tile admits a wider TKK
      tco = 64;
      for (int v = 0; pick_tkk(tco, a.KK, v); ++v)
        if (pick_tkk(tco, a.KK, v) == a.KK) tkk = a.KK;
    }
    return;
  }
  const int v = a.variant < 0 ? 0 : a.variant, ns = tile_shapes(a.Cout, a.KK);
  tkk = pick_tkk(tco, a.KK, ns > 0 ? v % ns : v);
}

// the two-stage-ring twin of a tile shape (fold / Gram launches: variant 1)
static bool two_stage(const ConvwArgs& a) {
  if (a.fold) return a.variant == 1;
  const int ns = tile_shapes(a.Cout, a.KK);
  return !a.fold && ns > 0 && a.variant >= ns && a.variant < 2 * ns;
}

bool convw_fold_ok(int Cout, int KK, int Arows) {
  ConvwArgs a{};
  a.Cout = Cout;
  a.KK = KK;
  a.Arows = Arows;
  a.fold = 1;
  int tco, tkk;
  tile_of(a, tco, tkk);
  return tkk == KK && tco > 0 && Arows % tco == 0 && Cout % 64 == 0 && KK >= 64 && (KK & (KK - 1)) == 0;
}

// Gram launch (fold == 2, 1x1, Cout = 0): A rows = [x (KK rows) | ones (the rest of Arows)], so
// out = fp32 [Arows][KK] holds x^T x and (row KK) the column sums of x from ONE read of x -- the
// stage carries no dY sub-images (NAR = 0), only the x sub-images both operands are read from.
// (tco, tkk, ring depth) per channel count; 0 when unsupported
static void gram_tile(int C, int& tco, int& tkk, int& nslot) {
  tco = tkk = nslot = 0;
  if (C == 64) tco = 128, tkk = 64, nslot = 5;
  else if (C == 128) tco = 256, tkk = 128, nslot = 5;
  else if (C == 256) tco = 128, tkk = 256, nslot = 4;
}

int convw_gram_rows(int C) {
  int tco, tkk, ns;
  gram_tile(C, tco, tkk, ns);
  return tco ? (C + 16 + tco - 1) / tco * tco : 0;
}

static void set_divs(ConvwArgs& a) {
  const FastDiv hw = make_fastdiv((uint32_t)std::max(1, a.Ho * a.Wo)), wo = make_fastdiv((uint32_t)std::max(1, a.Wo));
  a.howo_m = hw.m;
  a.howo_s = hw.s;
  a.wo_m = wo.m;
  a.wo_s = wo.s;
}

static ConvwPlan gram_plan(const ConvwArgs& a) {
  ConvwPlan p{0, 0};
  int tco, tkk, ns;
  gram_tile(a.KK, tco, tkk, ns);
  if (!tco || a.M <= 0 || a.Arows != convw_gram_rows(a.KK)) return p;
  const int ntile = a.Arows / tco;
  const int occ = std::max(1, std::min(2, (160 * 1024) / ((two_stage(a) ? 2 : ns) * tkk / 64 * kSub)));
  const int total = (a.M + kBP - 1) / kBP;
  int splits = std::max(1, (cu_count() * occ) / ntile);
  splits = std::min(splits, std::max(1, total / 4));
  const int sps = (total + splits - 1) / splits;
  p.splits = (total + sps - 1) / sps;
  const int64_t mn = (int64_t)a.Arows * a.KK;
  p.slab_floats = (int64_t)p.splits * mn + splitk_tree_floats(p.splits, mn);
  return p;
}

static hipError_t launch_gram(const ConvwArgs& a_in, hipStream_t st) {
  int tco, tkk, ns;
  gram_tile(a_in.KK, tco, tkk, ns);
  const bool ok = tco > 0 && a_in.Cout == 0 && a_in.KK == (1 << a_in.logC) && a_in.S == 1 && a_in.stride == 1 &&
                  a_in.pad == 0 && a_in.H == a_in.Ho && a_in.W == a_in.Wo && !a_in.accumulate &&
                  a_in.Arows == convw_gram_rows(a_in.KK) && a_in.xbytes > 0 && a_in.xbytes <= 0xFFFFFF00u &&
                  a_in.dybytes > 0 && (int64_t)a_in.M * a_in.KK * 2 <= (int64_t)a_in.xbytes && a_in.slab && a_in.out;
  if (!ok) return hipErrorNotSupported;
  ConvwArgs a = a_in;
  set_divs(a);
  const ConvwPlan p = gram_plan(a);
  if (p.splits <= 0) return hipErrorNotSupported;
  const int total = (a.M + kBP - 1) / kBP;
  a.splits = p.splits;
  a.stages_per_split = (total + p.splits - 1) / p.splits;
  const int grid = p.splits * (a.Arows / tco);
  hipError_t e;
  const bool two = two_stage(a);
  if (a.KK == 64) e = two ? launch_t<128, 64, 4, 2, 0>(a, grid, st) : launch_t<128, 64, 4, 5, 0>(a, grid, st);
  else if (a.KK == 128) e = two ? launch_t<256, 128, 4, 2, 0>(a, grid, st) : launch_t<256, 128, 4, 5, 0>(a, grid, st);
  else e = two ? launch_t<128, 256, 2, 2, 0>(a, grid, st) : launch_t<128, 256, 2, 4, 0>(a, grid, st);
  if (e != hipSuccess) return e;
  const int64_t mn = (int64_t)a.Arows * a.KK;
  return launch_splitk_reduce(a.slab, a.splits, mn, a.out, 0, 0, 1.f, st, a.slab + (int64_t)a.splits * mn);
}

ConvwPlan convw_plan(const ConvwArgs& a) {
  ConvwPlan p{0, 0};
  if (a.fold == 2) return gram_plan(a);
  if (is_persist_w(a)) {  // one slab per workgroup (one workgroup per CU)
    if (!persist_w_ok(a) || a.M <= 0) return p;
    p.splits = std::min(cu_count(), persist_w_tiles(a));
    const int64_t mn = 64 * 576;
    p.slab_floats = (int64_t)p.splits * mn + splitk_tree_floats(p.splits, mn);
    return p;
  }
  int tco, tkk;
  tile_of(a, tco, tkk);
  if (!tkk || a.M <= 0) return p;
  const int arows = a.fold ? a.Arows : a.Cout;
  const int ntile = (arows / tco) * (a.KK / tkk);
  const int occ = std::max(1, std::min(2, (160 * 1024) / lds_of(tco, tkk, two_stage(a))));
  const int total = (a.M + kBP - 1) / kBP;
  // one round of workgroups over the chip, >= 4 stages per split
  int splits = std::max(1, (cu_count() * occ) / ntile);
  splits = std::min(splits, std::max(1, total / 4));
  const int sps = (total + splits - 1) / splits;
  p.splits = (total + sps - 1) / sps;
  const int64_t mn = (int64_t)arows * a.KK;
  p.slab_floats = (int64_t)p.splits * mn + splitk_tree_floats(p.splits, mn);  // slabs + the reduce tree
  return p;
}

hipError_t launch_convw(const ConvwArgs& a_in, hipStream_t st) {
  if (a_in.M <= 0) return hipSuccess;
  if (a_in.fold == 2) return launch_gram(a_in, st);
  if (is_persist_w(a_in)) {
    if (!persist_w_ok(a_in) || !a_in.slab || !a_in.out || a_in.dybytes == 0 || a_in.xbytes == 0)
      return hipErrorNotSupported;
    static bool attr = false;
    if (!attr) {
      const hipError_t e = hipFuncSetAttribute((const void*)convhw_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               kHwLds);
      if (e != hipSuccess) return e;
      attr = true;
    }
    const ConvwPlan p = convw_plan(a_in);
    ConvwArgs a = a_in;
    a.splits = p.splits;
    hipLaunchKernelGGL(convhw_kernel, dim3(p.splits), dim3(256), kHwLds, st, a, persist_w_tiles(a));
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int64_t mn = 64 * 576;
    return launch_splitk_reduce(a.slab, a.splits, mn, a.out, 1, 0, 1.f, st, a.slab + (int64_t)a.splits * mn);
  }
  ConvwArgs a0 = a_in;
  if (!a0.fold) a0.Arows = a0.Cout;
  int tco, tkk;
  tile_of(a0, tco, tkk);
  const int C = 1 << a0.logC;
  const bool ok = tkk > 0 && a0.logC >= 6 &&
                  (!a0.fold || (a0.S == 1 && a0.KK == C && a0.stride == 1 && a0.pad == 0 && a0.Cout % 64 == 0 &&
                                a0.Arows > a0.Cout + a0.KK && a0.Arows % tco == 0 && tkk == a0.KK)) &&
                  a0.Cout % 64 == 0 && a0.KK % C == 0 && a0.KK / C == (a0.KK / C / a0.S) * a0.S && a0.S > 0 &&
                  a0.H < 32768 && a0.W < 32768 && a0.Ho > 0 && a0.Wo > 0 && a0.dybytes > 0 &&
                  a0.dybytes <= 0xFFFFFF00u && a0.xbytes > 0 && a0.xbytes <= 0xFFFFFF00u && a0.slab && a0.out &&
                  (int64_t)a0.M * a0.Cout * 2 <= (int64_t)a0.dybytes;
  if (!ok) return hipErrorNotSupported;
  ConvwArgs a = a0;
  set_divs(a);
  const ConvwPlan p = convw_plan(a);
  const int total = (a.M + kBP - 1) / kBP;
  a.splits = p.splits;
  a.stages_per_split = (total + p.splits - 1) / p.splits;
  const int grid = p.splits * (a.Arows / tco) * (a.KK / tkk);
  hipError_t e = hipErrorNotSupported;
#define PSD_CONVW(TCO_, TKK_, WR_)                                                                \
  (two_stage(a) ? launch_t<TCO_, TKK_, WR_, 2>(a, grid, st) : launch_t<TCO_, TKK_, WR_, nslot_of(TCO_, TKK_)>(a, grid, st))
  if (tco == 384) {
    e = two_stage(a) ? launch_t<384, 64, 8, 2, 4>(a, grid, st) : launch_t<384, 64, 8, 4, 4>(a, grid, st);
  } else if (tco == 64) {
    if (tkk == 256) e = PSD_CONVW(64, 256, 2);
    else if (tkk == 192) e = PSD_CONVW(64, 192, 2);
    else if (tkk == 128) e = PSD_CONVW(64, 128, 2);
    else e = PSD_CONVW(64, 64, 4);
  } else if (tco == 128) {
    if (tkk == 256) e = PSD_CONVW(128, 256, 2);
    else if (tkk == 192) e = PSD_CONVW(128, 192, 2);
    else if (tkk == 128) e = PSD_CONVW(128, 128, 2);
    else e = PSD_CONVW(128, 64, 4);
  } else {
    if (tkk == 128) e = PSD_CONVW(256, 128, 4);
    else e = PSD_CONVW(256, 64, 4);
  }
#undef PSD_CONVW
  if (e != hipSuccess) return e;
  const int64_t mn = (int64_t)a.Arows * a.KK;
  return launch_splitk_reduce(a.slab, a.splits, mn, a.out, a.fold ? 0 : 1, a.accumulate, 1.f, st,
                              a.slab + (int64_t)a.splits * mn);
}

}  // namespace psd
