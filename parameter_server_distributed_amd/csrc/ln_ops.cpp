// Tensor glue for the fused residual + dropout + LayerNorm kernels (kernels/layernorm.hip).
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>

#include <vector>

#include "kernels/launchers_ln.h"

namespace psd {

namespace {
inline hipStream_t ln_stream(const at::Tensor& t) { return c10::hip::getCurrentHIPStream(t.device().index()).stream(); }
inline const uint16_t* cu16(const at::Tensor& t) { return reinterpret_cast<const uint16_t*>(t.data_ptr()); }
inline uint16_t* u16(const at::Tensor& t) { return reinterpret_cast<uint16_t*>(t.data_ptr()); }
void check_bf16(const at::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.is_contiguous(), "psd ln: ", what,
              " must be a contiguous bf16 device tensor");
}
}  // namespace

std::vector<at::Tensor> ln_fwd(const at::Tensor& x, const at::Tensor& h, const at::Tensor& gamma, const at::Tensor& beta,
                               double eps, double p, int64_t seed, c10::optional<at::Tensor> step) {
  check_bf16(x, "x");
  check_bf16(h, "h");
  check_bf16(gamma, "gamma");
  check_bf16(beta, "beta");
  const int64_t H = x.size(-1);
  TORCH_CHECK(ln_supported((int)H) && h.sizes() == x.sizes() && gamma.numel() == H && beta.numel() == H,
              "psd ln fwd: shapes (H must be 768 or 1024)");
  const c10::DeviceGuard g(x.device());
  const int64_t rows = x.numel() / H;
  at::Tensor y = at::empty_like(x), s = at::empty_like(x);
  auto f32 = x.options().dtype(at::kFloat);
  at::Tensor mean = at::empty({rows}, f32), rstd = at::empty({rows}, f32);
  LnArgs a{};
  a.x = cu16(x);
  a.h = cu16(h);
  a.gamma = cu16(gamma);
  a.beta = cu16(beta);
  a.y = u16(y);
  a.s = u16(s);
  a.mean = mean.data_ptr<float>();
  a.rstd = rstd.data_ptr<float>();
  a.step = (step.has_value() && step->defined()) ? step->data_ptr<int64_t>() : nullptr;
  a.rows = rows;
  a.H = (int32_t)H;
  a.eps = (float)eps;
  a.p = (float)p;
  a.seed = (uint32_t)seed;
  hipError_t e = launch_ln_fwd(a, ln_stream(x));
  TORCH_CHECK(e == hipSuccess, "psd ln fwd: ", hipGetErrorString(e));
  return {y, s, mean, rstd};
}

std::vector<at::Tensor> ln_bwd(const at::Tensor& dy_in, const at::Tensor& s, const at::Tensor& mean,
                               const at::Tensor& rstd, const at::Tensor& gamma, double p, int64_t seed,
                               c10::optional<at::Tensor> step, c10::optional<at::Tensor> dgamma_out,
                               c10::optional<at::Tensor> dbeta_out, c10::optional<at::Tensor> dhsum_out) {
  at::Tensor dy = dy_in.contiguous();
  check_bf16(dy, "dy");
  check_bf16(s, "s");
  check_bf16(gamma, "gamma");
  const int64_t H = s.size(-1);
  TORCH_CHECK(ln_supported((int)H) && dy.sizes() == s.sizes() && gamma.numel() == H, "psd ln bwd: shapes");
  const c10::DeviceGuard g(s.device());
  const int64_t rows = s.numel() / H;
  TORCH_CHECK(mean.numel() == rows && rstd.numel() == rows, "psd ln bwd: statistics");
  at::Tensor dx = at::empty_like(s), dh = at::empty_like(s);
  at::Tensor dgamma = (dgamma_out.has_value() && dgamma_out->defined()) ? *dgamma_out : at::empty({H}, s.options());
  at::Tensor dbeta = (dbeta_out.has_value() && dbeta_out->defined()) ? *dbeta_out : at::empty({H}, s.options());
  check_bf16(dgamma, "dgamma");
  check_bf16(dbeta, "dbeta");
  const bool hs = dhsum_out.has_value() && dhsum_out->defined();
  if (hs) {
    check_bf16(*dhsum_out, "dhsum");
    TORCH_CHECK(dhsum_out->numel() == H, "psd ln bwd: dhsum must be [H]");
  }
  at::Tensor part = at::empty({(int64_t)ln_bwd_blocks(rows) * (hs ? 3 : 2) * H}, s.options().dtype(at::kFloat));
  LnArgs a{};
  a.dy = cu16(dy);
  a.s = u16(s);
  a.mean = mean.data_ptr<float>();
  a.rstd = rstd.data_ptr<float>();
  a.gamma = cu16(gamma);
  a.dx = u16(dx);
  a.dh = u16(dh);
  a.dgamma = u16(dgamma);
  a.dbeta = u16(dbeta);
  a.part = part.data_ptr<float>();
  a.dhsum = hs ? u16(*dhsum_out) : nullptr;
  a.step = (step.has_value() && step->defined()) ? step->data_ptr<int64_t>() : nullptr;
  a.rows = rows;
  a.H = (int32_t)H;
  a.p = (float)p;
  a.seed = (uint32_t)seed;
  hipError_t e = launch_ln_bwd(a, ln_stream(s));
  TORCH_CHECK(e == hipSuccess, "psd ln bwd: ", hipGetErrorString(e));
  return {dx, dh, dgamma, dbeta};
}

}  // namespace psd
