// Fused parameter-server apply for gfx950: multi-source gradient reduce + optimizer update +
// bf16 shadow write, one HBM pass.
//
// Reference: ParameterServerCore::receive_gradients averages every worker's gradient
// (src/parameter_server.cpp:38-63) and aggregate_gradients applies `p -= g` with lr = 1
// (src/parameter_server.cpp:77-91) as two host loops over per-worker std::vector copies. Here the
// K gradient sources (K = 1 after an RCCL reduce-scatter; K = #workers for inbox/p2p pushes) are
// summed in registers, scaled by grad_scale (= 1/W), the update is applied to the fp32 master in
// HBM and the bf16 working copy that the all-gather publishes is written in the same pass.
//
// Regime: pure HBM streaming (SGD-momentum with bf16 grads: 20 B/element). Design rules applied
// (cdna_hip_programming.md G11/G13): 256-thread blocks (4 waves), 8 elements per lane per
// iteration via 16-byte vector loads, grid-stride loop with <= 2048 blocks. No LDS: there is no
// reuse to stage (T14 is null on streaming ops at high occupancy).
#include "common.h"
#include "launchers.h"

namespace psd {

template <int KIND>
__device__ __forceinline__ void opt_update(const OptimHyper& h, float lr, float bc1, float bc2_sqrt,
                                           bool first, float& p, float g, float& s1, float& s2) {
  if (h.maximize) g = -g;
  if (KIND == OPT_SGD) {
    if (h.weight_decay != 0.f) g = fmaf(h.weight_decay, p, g);
    p = fmaf(-lr, g, p);
  } else if (KIND == OPT_MOMENTUM) {
    if (h.weight_decay != 0.f) g = fmaf(h.weight_decay, p, g);
    float buf = first ? g : fmaf(h.momentum, s1, (1.f - h.dampening) * g);
    s1 = buf;
    float d = h.nesterov ? fmaf(h.momentum, buf, g) : buf;
    p = fmaf(-lr, d, p);
  } else {  // ADAM / ADAMW
    if (KIND == OPT_ADAMW) {
      p = p * (1.f - lr * h.weight_decay);
    } else if (h.weight_decay != 0.f) {
      g = fmaf(h.weight_decay, p, g);
    }
    float m = fmaf(h.beta1, s1, (1.f - h.beta1) * g);
    float v = fmaf(h.beta2, s2, (1.f - h.beta2) * g * g);
    s1 = m;
    s2 = v;
    float denom = __fsqrt_rn(v) / bc2_sqrt + h.eps;
    p = p - (lr / bc1) * (m / denom);
  }
}

template <int SRC_DT>
__device__ __forceinline__ void load_sources8(const SourceList& g, int64_t i, float scale, float out[8]) {
#pragma unroll
  for (int e = 0; e < 8; ++e) out[e] = 0.f;
  for (int k = 0; k < g.count; ++k) {
    float t[8];
    if (SRC_DT == DT_BF16)
      load8_bf16(static_cast<const uint16_t*>(g.ptr[k]) + i, t);
    else
      load8_f32(static_cast<const float*>(g.ptr[k]) + i, t);
#pragma unroll
    for (int e = 0; e < 8; ++e) out[e] += t[e];
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) out[e] *= scale;
}

template <int SRC_DT>
__device__ __forceinline__ float load_source1(const SourceList& g, int64_t i, float scale) {
  float acc = 0.f;
  for (int k = 0; k < g.count; ++k) {
    if (SRC_DT == DT_BF16)
      acc += bf16_to_f32(static_cast<const uint16_t*>(g.ptr[k])[i]);
    else
      acc += static_cast<const float*>(g.ptr[k])[i];
  }
  return acc * scale;
}

template <int KIND, int SRC_DT>
__global__ __launch_bounds__(256) void fused_apply_kernel(OptimHyper h, const OptimDyn* __restrict__ dyn,
                                                          float* __restrict__ master, SourceList g,
                                                          float* __restrict__ s1, float* __restrict__ s2,
                                                          uint16_t* __restrict__ shadow, int64_t n) {
  const float lr = dyn->lr;
  const float gs = dyn->grad_scale;
  const float bc1 = dyn->bc1;
  const float bc2s = sqrtf(dyn->bc2);
  const bool first = dyn->step <= 1;
  const bool has_state = (KIND != OPT_SGD);
  const bool two_state = (KIND == OPT_ADAM || KIND == OPT_ADAMW);

  const int64_t nvec = n >> 3;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    const int64_t i = v << 3;
    float gr[8], p[8], a[8], b[8];
    load_sources8<SRC_DT>(g, i, gs, gr);
    load8_f32(master + i, p);
    if (has_state) load8_f32(s1 + i, a);
    if (two_state) load8_f32(s2 + i, b);
#pragma unroll
    for (int e = 0; e < 8; ++e) opt_update<KIND>(h, lr, bc1, bc2s, first, p[e], gr[e], a[e], b[e]);
    store8_f32(master + i, p);
    if (has_state) store8_f32(s1 + i, a);
    if (two_state) store8_f32(s2 + i, b);
    if (shadow) store8_bf16(shadow + i, p);
  }
  // Tail (n % 8 elements): first block only.
  if (blockIdx.x == 0) {
    for (int64_t i = (nvec << 3) + threadIdx.x; i < n; i += blockDim.x) {
      float gr = load_source1<SRC_DT>(g, i, gs);
      float p = master[i];
      float a = has_state ? s1[i] : 0.f;
      float b = two_state ? s2[i] : 0.f;
      opt_update<KIND>(h, lr, bc1, bc2s, first, p, gr, a, b);
      master[i] = p;
      if (has_state) s1[i] = a;
      if (two_state) s2[i] = b;
      if (shadow) shadow[i] = f32_to_bf16(p);
    }
  }
}

__global__ void optim_advance_kernel(OptimDyn* dyn, float beta1, float beta2) {
  int step = dyn->step + 1;
  dyn->step = step;
  dyn->bc1 = 1.f - powf(beta1, (float)step);
  dyn->bc2 = 1.f - powf(beta2, (float)step);
}

template <int KIND>
static void dispatch_src(const OptimHyper& h, const OptimDyn* dyn, float* master, const SourceList& g,
                         float* s1, float* s2, uint16_t* shadow, int64_t n, hipStream_t st, int grid_cap) {
  const int block = 256;
  int grid = stream_grid((n >> 3) > 0 ? (n >> 3) : 1, block);
  if (grid_cap > 0 && grid > grid_cap) grid = grid_cap;
  if (g.dtype == DT_BF16)
    hipLaunchKernelGGL((fused_apply_kernel<KIND, DT_BF16>), dim3(grid), dim3(block), 0, st, h, dyn, master, g,
                       s1, s2, shadow, n);
  else
    hipLaunchKernelGGL((fused_apply_kernel<KIND, DT_F32>), dim3(grid), dim3(block), 0, st, h, dyn, master, g,
                       s1, s2, shadow, n);
}

hipError_t launch_fused_apply(const OptimHyper& h, const OptimDyn* dyn, float* master, const SourceList& g,
                              float* s1, float* s2, uint16_t* shadow, int64_t n, hipStream_t st, int grid_cap) {
  if (n <= 0) return hipSuccess;
  if (g.count < 1 || g.count > kMaxSources) return hipErrorInvalidValue;
  switch (h.kind) {
    case OPT_SGD: dispatch_src<OPT_SGD>(h, dyn, master, g, s1, s2, shadow, n, st, grid_cap); break;
    case OPT_MOMENTUM: dispatch_src<OPT_MOMENTUM>(h, dyn, master, g, s1, s2, shadow, n, st, grid_cap); break;
    case OPT_ADAM: dispatch_src<OPT_ADAM>(h, dyn, master, g, s1, s2, shadow, n, st, grid_cap); break;
    case OPT_ADAMW: dispatch_src<OPT_ADAMW>(h, dyn, master, g, s1, s2, shadow, n, st, grid_cap); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_optim_advance(OptimDyn* dyn, float beta1, float beta2, hipStream_t st) {
  hipLaunchKernelGGL(optim_advance_kernel, dim3(1), dim3(1), 0, st, dyn, beta1, beta2);
  return hipGetLastError();
}

}  // namespace psd
