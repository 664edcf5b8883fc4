// Tensor glue for the embedding weight gradient (kernels/embed.hip).
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>

#include "kernels/launchers_embed.h"

namespace psd {

// out [V, Hd] bf16 (zero-filled by the caller) <- per-id sums of dy [T, Hd] bf16 rows; sorted / perm:
// torch.sort(ids, stable=True) of the flat int64 ids
void embed_bwd_(const at::Tensor& sorted, const at::Tensor& perm, const at::Tensor& dy, at::Tensor out) {
  TORCH_CHECK(sorted.is_cuda() && perm.is_cuda() && sorted.scalar_type() == at::kLong && perm.scalar_type() == at::kLong &&
                  sorted.dim() == 1 && perm.sizes() == sorted.sizes() && sorted.is_contiguous() && perm.is_contiguous(),
              "psd embed_bwd: sorted / perm must be contiguous int64 [T] device tensors");
  TORCH_CHECK(dy.is_cuda() && dy.dim() == 2 && dy.scalar_type() == at::kBFloat16 && dy.is_contiguous() &&
                  dy.size(0) == sorted.size(0) && dy.size(1) % 256 == 0 && dy.size(1) <= 2048,
              "psd embed_bwd: dy must be contiguous bf16 [T, Hd], Hd % 256 == 0, Hd <= 2048");
  TORCH_CHECK(out.is_cuda() && out.dim() == 2 && out.scalar_type() == at::kBFloat16 && out.is_contiguous() &&
                  out.size(1) == dy.size(1) && out.device() == dy.device(),
              "psd embed_bwd: out must be contiguous bf16 [V, Hd] on dy's device");
  const c10::DeviceGuard g(dy.device());
  const int64_t T = dy.size(0);
  at::Tensor part = at::empty({(T + kEmbedChunk - 1) / kEmbedChunk, dy.size(1)}, dy.options().dtype(at::kFloat));
  hipError_t e = launch_embed_bwd(sorted.data_ptr<int64_t>(), perm.data_ptr<int64_t>(),
                                  reinterpret_cast<const uint16_t*>(dy.data_ptr()), T, (int)dy.size(1),
                                  part.data_ptr<float>(), reinterpret_cast<uint16_t*>(out.data_ptr()),
                                  c10::hip::getCurrentHIPStream(dy.device().index()).stream());
  TORCH_CHECK(e == hipSuccess, "psd embed_bwd: ", hipGetErrorString(e));
}

}  // namespace psd
