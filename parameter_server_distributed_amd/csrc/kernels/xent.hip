// Fused softmax cross-entropy on bf16 logits [rows, V] for gfx950 (the MLM decoder's 4864 x 30528
// logits of a BERT-base b256 step; the ResNet classifier's 1024 x 1000).
//
// Why: F.cross_entropy(logits.float(), y) ran as a cast to fp32 (a 594 MB write), a log-softmax
// forward writing fp32 log-probs, and a backward reading them back and writing an fp32 gradient that
// autograd then cast to bf16: ~4 GB of HBM traffic and 0.8 ms of a 32 ms BERT step
// (profiles/bert_base_b256_r2s2_kernels.md). Here the forward reads the bf16 logits once (one
// workgroup per row: online max / sum-of-exp in fp32, then loss = lse - x[label]) and keeps only the
// row log-sum-exp; the backward reads them once more and writes the bf16 gradient
// (softmax - onehot) * dloss / rows directly. Labels < 0 (ignore_index -100) contribute nothing.
//
// Rows are reduced in a fixed order (per-lane strided partials, then a wave butterfly, then LDS):
// deterministic.
#include "common.h"
#include "launchers_xent.h"

namespace psd {

namespace {
constexpr int kXentThreads = 256;

__device__ __forceinline__ void online_merge(float& m, float& s, float m2, float s2) {
  const float mm = fmaxf(m, m2);
  if (mm == -INFINITY) return;  // both empty
  s = s * __expf(m - mm) + s2 * __expf(m2 - mm);
  m = mm;
}
}  // namespace

// one workgroup per row: lse[r] = log(sum exp(x)); loss_row[r] = lse - x[label] (0 for ignored rows)
__global__ __launch_bounds__(kXentThreads) void xent_fwd_kernel(const uint16_t* __restrict__ x, const int64_t* __restrict__ labels,
                                                                int64_t V, int64_t ldx, float* __restrict__ lse,
                                                                float* __restrict__ loss_row) {
  const int64_t r = blockIdx.x;
  const uint16_t* row = x + r * ldx;
  float m = -INFINITY, s = 0.f;
  const int64_t nvec = V >> 3;  // 16-byte loads (host: ldx % 8 == 0, 16-B aligned rows)
  for (int64_t v = threadIdx.x; v < nvec; v += kXentThreads) {
    float t[8];
    load8_bf16(row + (v << 3), t);
    float lm = t[0];
#pragma unroll
    for (int e = 1; e < 8; ++e) lm = fmaxf(lm, t[e]);
    float ls = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) ls += __expf(t[e] - lm);
    online_merge(m, s, lm, ls);
  }
  for (int64_t c = (nvec << 3) + threadIdx.x; c < V; c += kXentThreads) online_merge(m, s, bf16_to_f32(row[c]), 1.f);
  for (int off = 32; off > 0; off >>= 1) {
    const float m2 = __shfl_xor(m, off, kWave), s2 = __shfl_xor(s, off, kWave);
    online_merge(m, s, m2, s2);
  }
  __shared__ float wm[kXentThreads / kWave], ws[kXentThreads / kWave];
  const int wid = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  if (lane == 0) {
    wm[wid] = m;
    ws[wid] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = wm[0], S = ws[0];
    for (int w = 1; w < kXentThreads / kWave; ++w) online_merge(M, S, wm[w], ws[w]);
    const float l = M + __logf(S);
    lse[r] = l;
    const int64_t y = labels[r];
    loss_row[r] = (y >= 0 && y < V) ? l - bf16_to_f32(row[y]) : 0.f;
  }
}

// dx[r, c] = (exp(x - lse[r]) - [c == label]) * scale   (scale = dloss / count, device scalar)
__global__ __launch_bounds__(kXentThreads) void xent_bwd_kernel(const uint16_t* __restrict__ x, const int64_t* __restrict__ labels,
                                                                const float* __restrict__ lse, const float* __restrict__ scale,
                                                                int64_t V, int64_t ldx, uint16_t* __restrict__ dx) {
  const int64_t r = blockIdx.x;
  const int64_t y = labels[r];
  const float l = lse[r];
  const float g = (y >= 0 && y < V) ? *scale : 0.f;
  const uint16_t* row = x + r * ldx;
  uint16_t* out = dx + r * V;
  const int64_t nvec = V >> 3;
  for (int64_t v = threadIdx.x; v < nvec; v += kXentThreads) {
    float t[8];
    load8_bf16(row + (v << 3), t);
#pragma unroll
    for (int e = 0; e < 8; ++e) t[e] = (__expf(t[e] - l) - (((v << 3) + e) == y ? 1.f : 0.f)) * g;
    store8_bf16(out + (v << 3), t);
  }
  for (int64_t c = (nvec << 3) + threadIdx.x; c < V; c += kXentThreads)
    out[c] = f32_to_bf16((__expf(bf16_to_f32(row[c]) - l) - (c == y ? 1.f : 0.f)) * g);
}

hipError_t launch_xent_fwd(const uint16_t* x, const int64_t* labels, int64_t rows, int64_t V, int64_t ldx, float* lse,
                           float* loss_row, hipStream_t st) {
  if (rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(xent_fwd_kernel, dim3((unsigned)rows), dim3(kXentThreads), 0, st, x, labels, V, ldx, lse, loss_row);
  return hipGetLastError();
}

hipError_t launch_xent_bwd(const uint16_t* x, const int64_t* labels, const float* lse, const float* scale, int64_t rows,
                           int64_t V, int64_t ldx, uint16_t* dx, hipStream_t st) {
  if (rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(xent_bwd_kernel, dim3((unsigned)rows), dim3(kXentThreads), 0, st, x, labels, lse, scale, V, ldx, dx);
  return hipGetLastError();
}

}  // namespace psd
