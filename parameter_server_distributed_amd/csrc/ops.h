#pragma once
#include <ATen/ATen.h>
#include <vector>

namespace psd {

void fused_apply_(at::Tensor master, const std::vector<at::Tensor>& grads, c10::optional<at::Tensor> state1,
                  c10::optional<at::Tensor> state2, c10::optional<at::Tensor> shadow, at::Tensor dyn, int64_t kind,
                  double momentum, double dampening, bool nesterov, double weight_decay, double beta1, double beta2,
                  double eps, bool maximize);
void optim_advance_(at::Tensor dyn, double beta1, double beta2);
void multi_reduce_(at::Tensor out, const std::vector<at::Tensor>& srcs, double scale);
void pack_cast_(const std::vector<at::Tensor>& srcs, const std::vector<at::Tensor>& dsts);
void amax_(const at::Tensor& x, at::Tensor amax_out);
void quant_fp8_(const at::Tensor& x, const at::Tensor& amax, double fp8_max, at::Tensor out, at::Tensor scale_inv);
void dequant_fp8_(const at::Tensor& x, const at::Tensor& scale_inv, at::Tensor out);

}  // namespace psd
