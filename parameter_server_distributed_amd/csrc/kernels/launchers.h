// Host-side launch API for the CDNA4 (gfx950) kernels of the parameter-server runtime.
//
// Every launcher takes raw device pointers plus an explicit hipStream_t, never allocates, never
// synchronises and never calls hipMemcpy: all of them are legal inside hipGraph stream capture
// (the whole training step -- forward, backward, push/apply/pull -- is captured once and replayed).
//
// Reference parity:
//   fused optimizer      <- ParameterServerCore::aggregate_gradients `p -= g`   (src/parameter_server.cpp:77-91)
//   multi-source reduce  <- per-worker gradient average                        (src/parameter_server.cpp:38-63)
//   pack / cast          <- proto (de)serialisation loops                       (src/worker.cpp:40-66)
#pragma once
#include <hip/hip_runtime_api.h>
#include <cstdint>

namespace psd {

enum OptimKind : int32_t {
  OPT_SGD = 0,        // p -= lr * (g + wd p)
  OPT_MOMENTUM = 1,   // torch.optim.SGD(momentum, dampening, nesterov)
  OPT_ADAM = 2,       // torch.optim.Adam (L2 weight decay folded into g)
  OPT_ADAMW = 3,      // torch.optim.AdamW (decoupled weight decay)
};

enum DType : int32_t { DT_F32 = 0, DT_BF16 = 1, DT_F8E4M3 = 2 };

// Static hyper-parameters: passed by value, frozen into a captured graph (they never change
// during a run).
struct OptimHyper {
  int32_t kind;
  int32_t nesterov;
  int32_t maximize;
  int32_t _pad;
  float momentum;
  float dampening;
  float weight_decay;
  float beta1;
  float beta2;
  float eps;
};

// Per-step scalars: live in device memory so that graph replay sees the current values.
// `optim_advance` (a 1-thread kernel captured in front of the apply kernels) bumps `step` and
// recomputes the Adam bias corrections; `lr` / `grad_scale` are written by the host (pinned
// memcpy node) or left constant.
struct OptimDyn {
  float lr;
  float grad_scale;  // folds 1/W averaging (and staleness damping) into the apply
  float bc1;         // 1 - beta1^step
  float bc2;         // 1 - beta2^step
  int32_t step;      // number of applied updates (1-based once the first update is applied)
  int32_t _pad[3];
};
static_assert(sizeof(OptimDyn) == 32, "OptimDyn layout is shared with Python (8 x 4B)");

constexpr int kMaxSources = 16;

// Sum of up to kMaxSources gradient inboxes (same dtype), optionally fused with the optimizer.
struct SourceList {
  const void* ptr[kMaxSources];
  int32_t count;
  int32_t dtype;  // DType of every source
};

// master[i] (fp32) <- optimizer(master[i], grad = grad_scale * sum_k src_k[i], state1/2)
// shadow (bf16, optional) <- bf16(master[i]) in the same pass (the all-gather payload).
hipError_t launch_fused_apply(const OptimHyper& hyper, const OptimDyn* dyn, float* master,
                              const SourceList& grads, float* state1, float* state2,
                              uint16_t* shadow_bf16, int64_t n, hipStream_t stream, int grid_cap = 0);

// 1-thread kernel: dyn->step += 1; bias corrections for beta1/beta2.
hipError_t launch_optim_advance(OptimDyn* dyn, float beta1, float beta2, hipStream_t stream);

// out[i] = scale * sum_k src_k[i];  out dtype DT_F32 or DT_BF16.
hipError_t launch_multi_reduce(const SourceList& srcs, void* out, int32_t out_dtype, float scale,
                               int64_t n, hipStream_t stream);

// Segment table for pack/unpack: one entry per tensor.
struct PackSeg {
  const void* src;
  void* dst;
  int64_t numel;
};
// Casting gather/scatter of many tensors in one launch. `segs` lives in device memory,
// `chunk_seg`/`chunk_off` give, per 8K-element chunk, its segment and element offset.
hipError_t launch_pack_cast(const PackSeg* segs, const int32_t* chunk_seg, const int64_t* chunk_off,
                            int64_t n_chunks, int32_t src_dtype, int32_t dst_dtype,
                            hipStream_t stream);

// fp32/bf16 -> fp8 e4m3fn (OCP) with a per-tensor scale; amax is reduced on device.
hipError_t launch_amax(const void* x, int32_t dtype, int64_t n, float* amax_out, hipStream_t stream);
hipError_t launch_quant_fp8(const void* x, int32_t dtype, int64_t n, const float* amax,
                            float fp8_max, uint8_t* out, float* scale_inv_out, hipStream_t stream, int e5m2 = 0);
// just-in-time per-tensor quantisation (amax partials + quantise, two launches); part: >= 1024 floats
hipError_t launch_quant_fp8_jit(const void* x, int32_t dtype, int64_t n, float* part, float fp8_max, uint8_t* out,
                                float* scale_inv, hipStream_t stream, int e5m2);
// delayed-scaling quantisation: scale from hist[0] * margin (the previous call's amax), this call's
// amax recorded and rolled into hist[0] (hist: 2 device floats, hist[1] == 0 between calls)
hipError_t launch_quant_fp8_delayed(const void* x, int32_t dtype, int64_t n, float* hist, float fp8_max, float margin,
                                    uint8_t* out, float* scale_inv, hipStream_t stream, int e5m2);
hipError_t launch_dequant_fp8(const uint8_t* x, int64_t n, const float* scale_inv, void* out,
                              int32_t out_dtype, hipStream_t stream);
// MX fp8 (OCP microscaling): e4m3 / e5m2 payload + one E8M0 scale byte per 32 consecutive elements
// (n % 32 == 0; scales: n / 32 bytes)
hipError_t launch_quant_mx(const void* x, int32_t dtype, int64_t n, int e5m2, uint8_t* q, uint8_t* scales,
                           hipStream_t stream);
hipError_t launch_dequant_mx(const uint8_t* q, const uint8_t* scales, int64_t n, void* out, int32_t out_dtype,
                             hipStream_t stream);

}  // namespace psd
