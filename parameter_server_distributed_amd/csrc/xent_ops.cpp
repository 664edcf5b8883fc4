// Tensor glue for the fused softmax cross-entropy (kernels/xent.hip).
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>

#include "kernels/launchers_xent.h"

namespace psd {

namespace {
inline hipStream_t stream_of(const at::Tensor& t) { return c10::hip::getCurrentHIPStream(t.device().index()).stream(); }
void check_logits(const at::Tensor& x, const at::Tensor& labels) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 2 && x.scalar_type() == at::kBFloat16 && x.stride(1) == 1 &&
                  x.stride(0) % 8 == 0 && (reinterpret_cast<uintptr_t>(x.data_ptr()) & 15) == 0,
              "psd xent: logits must be a 2-D bf16 device tensor with 16-B aligned rows");
  TORCH_CHECK(labels.is_cuda() && labels.dim() == 1 && labels.scalar_type() == at::kLong && labels.is_contiguous() &&
                  labels.size(0) == x.size(0),
              "psd xent: labels must be int64 [rows] on the device");
}
}  // namespace

// returns {loss_row [rows] fp32, lse [rows] fp32}
std::vector<at::Tensor> xent_fwd(const at::Tensor& x, const at::Tensor& labels) {
  check_logits(x, labels);
  const c10::DeviceGuard g(x.device());
  const int64_t rows = x.size(0), V = x.size(1);
  auto f32 = x.options().dtype(at::kFloat);
  at::Tensor lse = at::empty({rows}, f32), loss_row = at::empty({rows}, f32);
  hipError_t e = launch_xent_fwd(reinterpret_cast<const uint16_t*>(x.data_ptr()), labels.data_ptr<int64_t>(), rows, V,
                                 x.stride(0), lse.data_ptr<float>(), loss_row.data_ptr<float>(), stream_of(x));
  TORCH_CHECK(e == hipSuccess, "psd xent fwd: ", hipGetErrorString(e));
  return {loss_row, lse};
}

// dx [rows, V] bf16 = (softmax(x) - onehot) * scale; scale: fp32 device scalar
at::Tensor xent_bwd(const at::Tensor& x, const at::Tensor& labels, const at::Tensor& lse, const at::Tensor& scale) {
  check_logits(x, labels);
  TORCH_CHECK(lse.is_cuda() && lse.scalar_type() == at::kFloat && lse.numel() == x.size(0) && lse.is_contiguous(),
              "psd xent bwd: lse fp32 [rows]");
  TORCH_CHECK(scale.is_cuda() && scale.scalar_type() == at::kFloat && scale.numel() >= 1, "psd xent bwd: scale");
  const c10::DeviceGuard g(x.device());
  const int64_t rows = x.size(0), V = x.size(1);
  at::Tensor dx = at::empty({rows, V}, x.options());
  hipError_t e = launch_xent_bwd(reinterpret_cast<const uint16_t*>(x.data_ptr()), labels.data_ptr<int64_t>(),
                                 lse.data_ptr<float>(), scale.data_ptr<float>(), rows, V, x.stride(0),
                                 reinterpret_cast<uint16_t*>(dx.data_ptr()), stream_of(x));
  TORCH_CHECK(e == hipSuccess, "psd xent bwd: ", hipGetErrorString(e));
  return dx;
}

}  // namespace psd
