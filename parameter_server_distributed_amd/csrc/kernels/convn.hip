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
//   * tile = 128 output pixels x BN output channels (BN = 64, 128 or 256 = the whole layer
//     width for the narrow layers: the gathered input rows are staged once per pixel tile);
//   * 2 x (BN / WNT) waves, each owning 64 x WNT of C on v_mfma_f32_16x16x32_bf16;
//   * K-tile = 64 channels of one (r, s) (C % 64 == 0); A rows gathered straight into LDS by
//     buffer_load ... lds (16 B per lane, 8 channels of one shifted input pixel; pixels outside the
//     image fall outside the buffer range and load zeros = the padding), B = the weight rows;
//     K-major [rows][64] images, 16-B chunks XOR-swizzled by (row >> 1) & 7 on the SOURCE address
//     (the LDS-DMA image is lane-linear), read with ds_read_b128;
//   * 3-slot LDS ring, two K-tiles in flight, one raw s_barrier per K-tile: iteration t waits for
//     its own DMA of tile t with a counted vmcnt (tile t+1 stays in flight), the barrier publishes
//     tile t and retires every wave's reads of tile t-1, whose slot then receives tile t+2;
//   * XCD-aware tile order (consecutive pixel tiles -- which share input rows through the 3x3
//     halo -- land on one XCD's L2);
//   * epilogue: bf16 C through LDS to 16-byte row stores; with STATS, per output channel the shifted
//     sums sum(y - k) and sum((y - k)^2) over the tile's valid rows (y rounded to bf16 first: the
//     statistics of the tensor that is stored), one partial row per (pixel tile, wave row) in the
//     layout of bn_fwd_reduce_kernel (bn.hip), so the BN forward skips its reduce pass and goes
//     straight to the finalize.
// The same kernel runs a stride-1 bwd-data (conv of dY with the flipped, transposed weights) and
// a 1x1 bwd-data (dY . W as a 1x1 conv of dY with W^T).
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

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  // bijective: blocks with equal bid % 8 (one XCD under round-robin dispatch) get a contiguous range
  const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

template <int BN, int WNT>
struct Geo {
  static constexpr int NWC = BN / WNT;       // wave columns
  static constexpr int NW = 2 * NWC;         // waves (2 wave rows of 64 pixels)
  static constexpr int NT = 64 * NW;
  static constexpr int JN = WNT / 16;        // 16-column MFMA blocks per wave
  static constexpr int APW = 16 / NW;        // A DMA pieces (1 KiB = 8 rows) per wave per K-tile
  static constexpr int BPW = (BN / 8) / NW;  // B DMA pieces per wave per K-tile
  static constexpr int DPS = APW + BPW;      // DMA per wave per K-tile (the counted vmcnt)
  static constexpr int AB = kBM * 128;       // A bytes per K-tile
  static constexpr int SLOT = AB + BN * 128;
  static constexpr int LDC = BN + 8;         // epilogue staging row (bf16 elements, +16 B)
  static constexpr int RING = 3 * SLOT;
  static constexpr int LDS = RING > kBM * LDC * 2 ? RING : kBM * LDC * 2;
  static_assert(16 % NW == 0 && (BN / 8) % NW == 0, "DMA pieces must divide over the waves");
  static_assert(LDS <= 160 * 1024, "LDS");
};

}  // namespace

template <int BN, int WNT, bool STATS>
__global__ __launch_bounds__(512) void convn_kernel(ConvnArgs a) {
  using G = Geo<BN, WNT>;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tiles_m = gridDim.x;
  const int tm = xcd_remap(blockIdx.x, tiles_m);
  const int m0 = tm * kBM, n0 = blockIdx.y * BN;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid / G::NWC, wc = wid % G::NWC;

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
  const rsrc_t wrs = make_rsrc(a.w, a.wbytes);
  const int cmask = (1 << a.logC) - 1;

  auto stage = [&](int t) {
    uint8_t* slot = smem + (t % 3) * G::SLOT;
    const int k0 = t * kBK;
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
    // (the weight offsets are recomputed per K-tile: a per-lane offset array captured by this lambda
    // made hipcc's host pass silently drop the kernel's instantiation -- an undefined stub symbol)
#pragma unroll
    for (int i = 0; i < G::BPW; ++i) {
      const int piece = i * G::NW + wid;
      const int row = piece * 8 + (lane >> 3);
      const int kc = (lane & 7) ^ ((row >> 1) & 7);
      const uint32_t off = ((uint32_t)(n0 + row) * (uint32_t)a.K + (uint32_t)(k0 + kc * 8)) * 2u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs,
                                               (__attribute__((address_space(3))) void*)(slot + G::AB + piece * 1024),
                                               16, off, 0, 0, 0);
    }
  };

  f32x4 acc[4][G::JN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < G::JN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nt = a.K / kBK;
  stage(0);
  if (nt > 1) stage(1);
  for (int t = 0; t < nt; ++t) {
    if (t + 1 < nt) wait_vm<G::DPS>();  // K-tile t landed (this wave's DMA), t+1 in flight
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();  // every wave: tile t published, tile t-1 no longer read
    __builtin_amdgcn_sched_barrier(0);
    if (t + 2 < nt) stage(t + 2);
    const uint8_t* As = smem + (t % 3) * G::SLOT;
    const uint8_t* Bs = As + G::AB;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[4], bf[G::JN];
#pragma unroll
      for (int j = 0; j < G::JN; ++j) bf[j] = frag(Bs, wc * G::JN + j, ks, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = frag(As, wr * 4 + i, ks, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < G::JN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  }

  // ---- epilogue: C layout col = lane & 15, row = 4 * (lane >> 4) + r
  __syncthreads();  // the ring is free (every DMA retired by the last vmcnt(0))
  uint16_t* cs = reinterpret_cast<uint16_t*>(smem);
  const int cl = lane & 15, rq = (lane >> 4) * 4;
#pragma unroll
  for (int j = 0; j < G::JN; ++j) {
    const int col = wc * WNT + j * 16 + cl;
    float s1 = 0.f, s2 = 0.f;
    float k = 0.f;
    if constexpr (STATS) k = a.shift[n0 + col];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wr * 64 + i * 16 + rq + r;
        const uint16_t hv = f32_to_bf16(acc[i][j][r]);
        cs[row * G::LDC + col] = hv;
        if constexpr (STATS) {
          if (m0 + row < a.M) {
            const float d = bf16_to_f32(hv) - k;
            s1 += d;
            s2 = fmaf(d, d, s2);
          }
        }
      }
    if constexpr (STATS) {
      s1 += __shfl_xor(s1, 16);
      s2 += __shfl_xor(s2, 16);
      s1 += __shfl_xor(s1, 32);
      s2 += __shfl_xor(s2, 32);
      if (lane < 16) {
        float* pr = a.part + ((int64_t)tm * 2 + wr) * 2 * a.N;
        pr[n0 + col] = s1;
        pr[a.N + n0 + col] = s2;
      }
    }
  }
  __syncthreads();
  constexpr int CPR = BN / 8;  // 16-byte chunks per tile row
  uint16_t* y = reinterpret_cast<uint16_t*>(a.y);
#pragma unroll 4
  for (int c = threadIdx.x; c < kBM * CPR; c += G::NT) {
    const int row = c / CPR, cc = (c % CPR) * 8;
    const int m = m0 + row;
    if (m < a.M)
      *reinterpret_cast<u32x4*>(y + (int64_t)m * a.ldc + n0 + cc) = *reinterpret_cast<const u32x4*>(cs + row * G::LDC + cc);
  }
}

// ------------------------------------------------------------------ host side
namespace {

template <int BN, int WNT, bool STATS>
hipError_t launch_t(const ConvnArgs& a, hipStream_t st) {
  using G = Geo<BN, WNT>;
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)convn_kernel<BN, WNT, STATS>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS);
    if (e != hipSuccess) return e;
    attr = true;
  }
  const int tiles_m = (a.M + kBM - 1) / kBM;
  hipLaunchKernelGGL((convn_kernel<BN, WNT, STATS>), dim3(tiles_m, a.N / BN), dim3(G::NT), G::LDS, st, a);
  return hipGetLastError();
}

template <int BN, int WNT>
hipError_t launch_s(const ConvnArgs& a, hipStream_t st) {
  return a.part ? launch_t<BN, WNT, true>(a, st) : launch_t<BN, WNT, false>(a, st);
}

}  // namespace

int convn_tile_n(int N) {
  if (N == 64) return 64;
  if (N == 128) return 128;
  if (N % 256 == 0) return 256;
  return 0;
}

int convn_stats_rows(int M) { return 2 * ((M + kBM - 1) / kBM); }

hipError_t launch_convn(const ConvnArgs& a, hipStream_t st) {
  if (a.M <= 0) return hipSuccess;
  const int bn = convn_tile_n(a.N);
  const int C = 1 << a.logC;
  const bool ok = bn > 0 && a.logC >= 6 && a.K % kBK == 0 && a.K == a.R * a.S * C && a.ldc % 8 == 0 &&
                  a.ldc >= a.N && a.H < 32768 && a.W < 32768 && a.xbytes > 0 && a.xbytes <= 0xFFFFFF00u &&
                  a.wbytes > 0 && (!a.part || a.shift);
  if (!ok) return hipErrorNotSupported;
  switch (bn) {
    case 64: return launch_s<64, 32>(a, st);
    case 128: return launch_s<128, 32>(a, st);
    default: return launch_s<256, 64>(a, st);
  }
}

}  // namespace psd
