// Tensor glue for the fused self-attention kernels (kernels/attention.hip).
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>

#include <cmath>
#include <vector>

#include "kernels/launchers_attn.h"
#include "kernels/launchers_gemm.h"

namespace psd {

namespace {
inline hipStream_t attn_stream(const at::Tensor& t) {
  return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}
void check_attn(const at::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.is_contiguous(), "psd attn: ", what,
              " must be a contiguous bf16 device tensor");
}
AttnArgs make_args(const at::Tensor& qkv, int64_t heads, double p, int64_t seed, const c10::optional<at::Tensor>& step) {
  TORCH_CHECK(qkv.dim() == 3 && heads > 0 && qkv.size(2) % (3 * heads) == 0, "psd attn: qkv must be [B, S, 3*H*Dh]");
  const int64_t dh = qkv.size(2) / (3 * heads);
  TORCH_CHECK(attn_supported((int)qkv.size(1), (int)dh), "psd attn: needs head dim 64 and S in {32, 64, 96, 128}");
  TORCH_CHECK(p >= 0.0 && p < 1.0, "psd attn: dropout p must be in [0, 1)");
  AttnArgs a{};
  a.qkv = reinterpret_cast<const uint16_t*>(qkv.data_ptr());
  a.B = (int32_t)qkv.size(0);
  a.S = (int32_t)qkv.size(1);
  a.H = (int32_t)heads;
  a.scale = (float)(1.0 / std::sqrt((double)dh));
  a.thresh = p > 0.0 ? (uint32_t)std::min(4294967295.0, std::floor(p * 4294967296.0)) : 0u;
  a.rescale = (float)(1.0 / (1.0 - p));
  a.seed = (uint32_t)seed;
  a.step = (step.has_value() && step->defined()) ? step->data_ptr<int64_t>() : nullptr;
  return a;
}
}  // namespace

std::vector<at::Tensor> attn_fwd(const at::Tensor& qkv, int64_t heads, double p, int64_t seed,
                                 c10::optional<at::Tensor> step) {
  check_attn(qkv, "qkv");
  const c10::DeviceGuard g(qkv.device());
  AttnArgs a = make_args(qkv, heads, p, seed, step);
  at::Tensor o = at::empty({qkv.size(0), qkv.size(1), qkv.size(2) / 3}, qkv.options());
  at::Tensor lse = at::empty({qkv.size(0), heads, qkv.size(1)}, qkv.options().dtype(at::kFloat));
  a.o = reinterpret_cast<uint16_t*>(o.data_ptr());
  a.lse = lse.data_ptr<float>();
  hipError_t e = launch_attn_fwd(a, attn_stream(qkv));
  TORCH_CHECK(e == hipSuccess, "psd attn fwd: ", hipGetErrorString(e));
  return {o, lse};
}

// bias_out (optional, [3*H*Dh] bf16/fp32): also the QKV Linear's bias gradient = the column sums of
// dqkv, from per-sequence partials the kernel writes + one deterministic column reduce
at::Tensor attn_bwd(const at::Tensor& dout_in, const at::Tensor& qkv, const at::Tensor& o, const at::Tensor& lse,
                    int64_t heads, double p, int64_t seed, c10::optional<at::Tensor> step,
                    c10::optional<at::Tensor> bias_out) {
  at::Tensor dout = dout_in.contiguous();
  check_attn(dout, "dout");
  check_attn(qkv, "qkv");
  check_attn(o, "o");
  const c10::DeviceGuard g(qkv.device());
  AttnArgs a = make_args(qkv, heads, p, seed, step);
  TORCH_CHECK(o.sizes() == dout.sizes() && o.size(0) == qkv.size(0) && o.size(1) == qkv.size(1) &&
                  o.size(2) * 3 == qkv.size(2),
              "psd attn bwd: o / dout must be [B, S, H*Dh]");
  TORCH_CHECK(lse.is_cuda() && lse.scalar_type() == at::kFloat && lse.is_contiguous() &&
                  lse.numel() == (int64_t)a.B * a.H * a.S,
              "psd attn bwd: lse must be fp32 [B, H, S]");
  at::Tensor dqkv = at::empty_like(qkv);
  a.o = reinterpret_cast<uint16_t*>(o.data_ptr());
  a.lse = lse.data_ptr<float>();
  a.dout = reinterpret_cast<const uint16_t*>(dout.data_ptr());
  a.dqkv = reinterpret_cast<uint16_t*>(dqkv.data_ptr());
  const bool bias = bias_out.has_value() && bias_out->defined();
  at::Tensor bpart;
  if (bias) {
    TORCH_CHECK(bias_out->is_cuda() && bias_out->is_contiguous() && bias_out->numel() == qkv.size(2) &&
                    (bias_out->scalar_type() == at::kBFloat16 || bias_out->scalar_type() == at::kFloat),
                "psd attn bwd: bias_out must be a contiguous [3*H*Dh] bf16/fp32 tensor");
    bpart = at::empty({(int64_t)a.B, qkv.size(2)}, qkv.options().dtype(at::kFloat));
    a.bpart = bpart.data_ptr<float>();
  }
  hipError_t e = launch_attn_bwd(a, attn_stream(qkv));
  TORCH_CHECK(e == hipSuccess, "psd attn bwd: ", hipGetErrorString(e));
  if (bias) {
    e = launch_colsum_final(a.bpart, a.B, (int)qkv.size(2), bias_out->data_ptr(),
                            bias_out->scalar_type() == at::kBFloat16, 0, attn_stream(qkv));
    TORCH_CHECK(e == hipSuccess, "psd attn bwd bias: ", hipGetErrorString(e));
  }
  return dqkv;
}

}  // namespace psd
