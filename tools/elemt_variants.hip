// Launch-shape study for the BN elementwise backward pass dx = A g + B x + C (per channel, bf16,
// NHWC): the round-6 kernel (bn.hip bn_bwd_elemt_kernel<2>: <= 2048 workgroups, grid-stride loop,
// two items in flight per lane) against one-shot grids with I items per lane, with and without
// nontemporal loads / stores. Standalone: builds with hipcc, times with hip events.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I parameter_server_distributed_amd/csrc/kernels \
//         tools/elemt_variants.hip -o /tmp/elemt_variants && /tmp/elemt_variants
#include <cstdio>
#include <vector>

#include "common.h"

using namespace psd;

// the round-6 kernel's loop shape (MODE 2)
__global__ __launch_bounds__(256) void v_gridstride(const uint16_t* __restrict__ g, const uint16_t* __restrict__ x,
                                                    const float* __restrict__ coef, uint16_t* __restrict__ dx,
                                                    int64_t nvec, int C) {
  const int tpc = C >> 3;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int cg = (int)(v % tpc);
  float A[8], B[8], Cc[8];
  load8_f32(coef + cg * 8, A);
  load8_f32(coef + C + cg * 8, B);
  load8_f32(coef + 2 * C + cg * 8, Cc);
  auto el = [&](int64_t v, float (&gv)[8], const float (&xv)[8]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) gv[j] = fmaf(A[j], gv[j], fmaf(B[j], xv[j], Cc[j]));
    store8_bf16(dx + v * 8, gv);
  };
  for (; v + stride < nvec; v += 2 * stride) {
    float g0[8], g1[8], x0[8], x1[8];
    load8_bf16(g + v * 8, g0);
    load8_bf16(g + (v + stride) * 8, g1);
    load8_bf16(x + v * 8, x0);
    load8_bf16(x + (v + stride) * 8, x1);
    el(v, g0, x0);
    el(v + stride, g1, x1);
  }
  for (; v < nvec; v += stride) {
    float gv[8], xv[8];
    load8_bf16(g + v * 8, gv);
    load8_bf16(x + v * 8, xv);
    el(v, gv, xv);
  }
}

template <bool NT>
__device__ __forceinline__ u32x4 ld16(const uint16_t* p) {
  if (NT) return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return *reinterpret_cast<const u32x4*>(p);
}
template <bool NT>
__device__ __forceinline__ void st16(uint16_t* p, u32x4 w) {
  if (NT) __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(p));
  else *reinterpret_cast<u32x4*>(p) = w;
}
__device__ __forceinline__ void unpack(u32x4 w, float v[8]) {
  uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(ws[i] << 16);
    v[2 * i + 1] = __uint_as_float(ws[i] & 0xffff0000u);
  }
}

// one-shot: block b owns items [b*256*I, (b+1)*256*I); lane t takes t, t+256, ... (coalesced);
// tpc | 256 so a lane's channel group is t % tpc for every item
template <int I, bool NT>
__global__ __launch_bounds__(256) void v_oneshot(const uint16_t* __restrict__ g, const uint16_t* __restrict__ x,
                                                 const float* __restrict__ coef, uint16_t* __restrict__ dx,
                                                 int64_t nvec, int C) {
  const int tpc = C >> 3;
  const int cg = threadIdx.x & (tpc - 1);
  const int64_t base = (int64_t)blockIdx.x * 256 * I + threadIdx.x;
  float A[8], B[8], Cc[8];
  load8_f32(coef + cg * 8, A);
  load8_f32(coef + C + cg * 8, B);
  load8_f32(coef + 2 * C + cg * 8, Cc);
  u32x4 gw[I], xw[I];
#pragma unroll
  for (int k = 0; k < I; ++k) {
    const int64_t v = base + k * 256;
    if (v < nvec) {
      gw[k] = ld16<NT>(g + v * 8);
      xw[k] = ld16<NT>(x + v * 8);
    }
  }
#pragma unroll
  for (int k = 0; k < I; ++k) {
    const int64_t v = base + k * 256;
    if (v < nvec) {
      float gv[8], xv[8];
      unpack(gw[k], gv);
      unpack(xw[k], xv);
      uint32_t o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        o[j] = pack_bf16x2_rne(fmaf(A[2 * j], gv[2 * j], fmaf(B[2 * j], xv[2 * j], Cc[2 * j])),
                               fmaf(A[2 * j + 1], gv[2 * j + 1], fmaf(B[2 * j + 1], xv[2 * j + 1], Cc[2 * j + 1])));
      st16<NT>(dx + v * 8, u32x4{o[0], o[1], o[2], o[3]});
    }
  }
}

// grid-stride with G workgroups per CU-slot budget and I items in flight
template <int I, bool NT>
__global__ __launch_bounds__(256) void v_stride(const uint16_t* __restrict__ g, const uint16_t* __restrict__ x,
                                                const float* __restrict__ coef, uint16_t* __restrict__ dx,
                                                int64_t nvec, int C) {
  const int tpc = C >> 3;
  const int cg = threadIdx.x & (tpc - 1);
  float A[8], B[8], Cc[8];
  load8_f32(coef + cg * 8, A);
  load8_f32(coef + C + cg * 8, B);
  load8_f32(coef + 2 * C + cg * 8, Cc);
  for (int64_t base = (int64_t)blockIdx.x * 256 * I + threadIdx.x; base < nvec; base += (int64_t)gridDim.x * 256 * I) {
    u32x4 gw[I], xw[I];
#pragma unroll
    for (int k = 0; k < I; ++k) {
      const int64_t v = base + k * 256;
      if (v < nvec) {
        gw[k] = ld16<NT>(g + v * 8);
        xw[k] = ld16<NT>(x + v * 8);
      }
    }
#pragma unroll
    for (int k = 0; k < I; ++k) {
      const int64_t v = base + k * 256;
      if (v < nvec) {
        float gv[8], xv[8];
        unpack(gw[k], gv);
        unpack(xw[k], xv);
        uint32_t o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
          o[j] = pack_bf16x2_rne(fmaf(A[2 * j], gv[2 * j], fmaf(B[2 * j], xv[2 * j], Cc[2 * j])),
                                 fmaf(A[2 * j + 1], gv[2 * j + 1], fmaf(B[2 * j + 1], xv[2 * j + 1], Cc[2 * j + 1])));
        st16<NT>(dx + v * 8, u32x4{o[0], o[1], o[2], o[3]});
      }
    }
  }
}

#define CK(e)                                                               \
  do {                                                                      \
    hipError_t _e = (e);                                                    \
    if (_e != hipSuccess) {                                                 \
      printf("HIP error %s at %d\n", hipGetErrorString(_e), __LINE__);     \
      return 1;                                                             \
    }                                                                       \
  } while (0)

int main() {
  const int64_t shapes[][2] = {{3211264, 64}, {802816, 128}, {3211264, 128}, {200704, 256}, {802816, 256},
                               {50176, 512},  {200704, 512}};
  const int64_t maxe = 3211264LL * 128;
  uint16_t *g, *x, *d;
  float* coef;
  CK(hipMalloc(&g, maxe * 2));
  CK(hipMalloc(&x, maxe * 2));
  CK(hipMalloc(&d, maxe * 2));
  CK(hipMalloc(&coef, 3 * 4096 * 4));
  {
    std::vector<uint16_t> h(maxe);
    for (int64_t i = 0; i < maxe; ++i) h[i] = (uint16_t)(0x3f80 + (i * 7 % 64));
    CK(hipMemcpy(g, h.data(), maxe * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(x, h.data(), maxe * 2, hipMemcpyHostToDevice));
    std::vector<float> c(3 * 4096, 0.5f);
    CK(hipMemcpy(coef, c.data(), c.size() * 4, hipMemcpyHostToDevice));
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  printf("| shape | MB/tensor | variant | grid | us | TB/s |\n|---|---:|---|---:|---:|---:|\n");
  for (auto& s : shapes) {
    const int64_t M = s[0];
    const int C = (int)s[1];
    const int64_t nvec = M * C / 8;
    if ((C / 8) > 256 || 256 % (C / 8)) continue;
    auto run = [&](const char* name, int grid, auto launch) -> int {
      launch(grid);
      CK(hipDeviceSynchronize());
      const int it = 20;
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < it; ++i) launch(grid);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1e3 / it;
      printf("| %lld x %d | %.0f | %s | %d | %.1f | %.2f |\n", (long long)M, C, nvec * 16 / 1e6, name, grid, us,
             3.0 * nvec * 16 / us / 1e6);
      return 0;
    };
    auto oneshot_grid = [&](int I) { return (int)((nvec + 256LL * I - 1) / (256LL * I)); };
    run("gridstride (round 6)", 2048, [&](int gr) { v_gridstride<<<gr, 256>>>(g, x, coef, d, nvec, C); });
    run("oneshot I=1", oneshot_grid(1), [&](int gr) { v_oneshot<1, false><<<gr, 256>>>(g, x, coef, d, nvec, C); });
    run("oneshot I=2", oneshot_grid(2), [&](int gr) { v_oneshot<2, false><<<gr, 256>>>(g, x, coef, d, nvec, C); });
    run("oneshot I=4", oneshot_grid(4), [&](int gr) { v_oneshot<4, false><<<gr, 256>>>(g, x, coef, d, nvec, C); });
    run("oneshot I=2 nt", oneshot_grid(2), [&](int gr) { v_oneshot<2, true><<<gr, 256>>>(g, x, coef, d, nvec, C); });
    run("oneshot I=4 nt", oneshot_grid(4), [&](int gr) { v_oneshot<4, true><<<gr, 256>>>(g, x, coef, d, nvec, C); });
    for (int gr : {2048, 4096, 8192}) {
      run("stride I=2", gr, [&](int gg) { v_stride<2, false><<<gg, 256>>>(g, x, coef, d, nvec, C); });
      run("stride I=4", gr, [&](int gg) { v_stride<4, false><<<gg, 256>>>(g, x, coef, d, nvec, C); });
      run("stride I=4 nt", gr, [&](int gg) { v_stride<4, true><<<gg, 256>>>(g, x, coef, d, nvec, C); });
    }
    fflush(stdout);
  }
  return 0;
}
