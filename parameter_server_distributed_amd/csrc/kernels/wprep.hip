// Batched bwd-data weight preparation: every convolution's transposed / tap-flipped / stride-2-phase
// weight operand of one step in ONE launch. The bwd-data of a convolution runs as a convolution of dY
// with W'[ci][r'][s'][co] = W[co][r0 + r' sr][s0 + s' ss][ci] (1x1: the transpose W^T; stride-1 3x3:
// the tap flip r0 = R - 1, sr = -1; stride-2 3x3: the four output-parity phase subsets,
// ops/conv.py _s2_phase_weights). Built per convolution with torch ops that cost two launches each
// (flip + contiguous), ~56 launches / ~0.45 ms per ResNet-50 b1024 step
// (profiles/r5/resnet50_b1024_r5n_kernels.md); here one 64 x 64 LDS transpose per (job, tap, tile).
#include "common.h"
#include "launchers_wprep.h"

namespace psd {

namespace {

constexpr int kT = 64;  // co x ci tile

__global__ __launch_bounds__(256) void wprep_kernel(const WprepJob* __restrict__ jobs, int njobs) {
  __shared__ uint16_t t[kT][kT + 8];  // [co][ci], +8: 16-byte aligned rows, rotating banks
  // this block's job: the last one whose first tile is <= blockIdx.x (tile0 ascending)
  const int b = blockIdx.x;
  int lo = 0, hi = njobs - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (jobs[mid].tile0 <= b) lo = mid; else hi = mid - 1;
  }
  const WprepJob j = jobs[lo];
  const int tco = (j.co + kT - 1) / kT, tci = (j.ci + kT - 1) / kT;
  int rem = b - j.tile0;
  const int tc = rem % tci;
  rem /= tci;
  const int to = rem % tco;
  const int tap = rem / tco;  // (r', s') of the output
  const int rp = tap / j.Sp, sp = tap - rp * j.Sp;
  const int r = j.r0 + rp * j.sr, s = j.s0 + sp * j.ss;
  const int co0 = to * kT, ci0 = tc * kT;
  // load: 64 rows (co) x 8 chunks of 8 ci, 2 per thread (src [co][R][S][ci], ci contiguous)
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int q = threadIdx.x + k * 256;
    const int row = q >> 3, ch = q & 7;
    const int co = co0 + row, ci = ci0 + ch * 8;
    u32x4 v = u32x4{0u, 0u, 0u, 0u};
    if (co < j.co && ci < j.ci)
      v = *reinterpret_cast<const u32x4*>(j.src + (((int64_t)co * j.R + r) * j.S + s) * j.ci + ci);
    *reinterpret_cast<u32x4*>(&t[row][ch * 8]) = v;
  }
  __syncthreads();
  // store: 64 rows (ci) x 8 chunks of 8 co (dst [ci][Rp][Sp][co], co contiguous)
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int q = threadIdx.x + k * 256;
    const int row = q >> 3, ch = q & 7;
    const int ci = ci0 + row, co = co0 + ch * 8;
    if (ci < j.ci && co < j.co) {
      uint32_t pk[4];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        pk[e] = (uint32_t)t[ch * 8 + 2 * e][row] | ((uint32_t)t[ch * 8 + 2 * e + 1][row] << 16);
      *reinterpret_cast<u32x4*>(j.dst + (((int64_t)ci * j.Rp + rp) * j.Sp + sp) * j.co + co) =
          u32x4{pk[0], pk[1], pk[2], pk[3]};
    }
  }
}

}  // namespace

int wprep_tiles(int co, int ci, int Rp, int Sp) {
  return ((co + kT - 1) / kT) * ((ci + kT - 1) / kT) * Rp * Sp;
}

hipError_t launch_wprep(const WprepJob* jobs_dev, int njobs, int total_tiles, hipStream_t st) {
  if (njobs <= 0 || total_tiles <= 0) return hipSuccess;
  hipLaunchKernelGGL(wprep_kernel, dim3(total_tiles), dim3(256), 0, st, jobs_dev, njobs);
  return hipGetLastError();
}

}  // namespace psd
