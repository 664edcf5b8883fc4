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

namespace {
EmbLnArgs emb_args(const at::Tensor& ids, const at::Tensor& types, const at::Tensor& W, const at::Tensor& P,
                   const at::Tensor& T, const at::Tensor& gamma, int64_t S, double p, int64_t seed,
                   const c10::optional<at::Tensor>& step) {
  TORCH_CHECK(ids.is_cuda() && ids.scalar_type() == at::kLong && ids.is_contiguous(), "psd emb ln: ids (int64)");
  TORCH_CHECK(types.is_cuda() && types.scalar_type() == at::kLong && types.is_contiguous() &&
                  types.numel() == ids.numel(),
              "psd emb ln: types (int64, like ids)");
  check_bf16(W, "word table");
  check_bf16(P, "position table");
  check_bf16(T, "type table");
  check_bf16(gamma, "gamma");
  const int64_t H = W.size(1);
  TORCH_CHECK(H == 768 && W.dim() == 2 && P.dim() == 2 && T.dim() == 2 && P.size(1) == H && T.size(1) == H &&
                  gamma.numel() == H,
              "psd emb ln: tables [*, 768]");
  TORCH_CHECK(S >= 1 && S <= P.size(0) && ids.numel() % S == 0, "psd emb ln: sequence length vs position table");
  TORCH_CHECK(T.size(0) >= 1, "psd emb ln: empty type table");
  EmbLnArgs a{};
  a.ids = ids.data_ptr<int64_t>();
  a.types = types.data_ptr<int64_t>();
  a.W = cu16(W);
  a.P = cu16(P);
  a.T = cu16(T);
  a.gamma = cu16(gamma);
  a.step = (step.has_value() && step->defined()) ? step->data_ptr<int64_t>() : nullptr;
  a.rows = ids.numel();
  a.V = W.size(0);
  a.S = (int32_t)S;
  a.NT = (int32_t)T.size(0);
  a.H = (int32_t)H;
  a.p = (float)p;
  a.seed = (uint32_t)seed;
  return a;
}
}  // namespace

std::vector<at::Tensor> emb_ln_fwd(const at::Tensor& ids, const at::Tensor& types, const at::Tensor& W,
                                   const at::Tensor& P, const at::Tensor& T, const at::Tensor& gamma,
                                   const at::Tensor& beta, int64_t S, double eps, double p, int64_t seed,
                                   c10::optional<at::Tensor> step) {
  EmbLnArgs a = emb_args(ids, types, W, P, T, gamma, S, p, seed, step);
  check_bf16(beta, "beta");
  TORCH_CHECK(beta.numel() == a.H, "psd emb ln: beta");
  const c10::DeviceGuard g(W.device());
  at::Tensor y = at::empty({a.rows, (int64_t)a.H}, W.options());
  auto f32 = W.options().dtype(at::kFloat);
  at::Tensor mean = at::empty({a.rows}, f32), rstd = at::empty({a.rows}, f32);
  a.beta = cu16(beta);
  a.y = u16(y);
  a.mean = mean.data_ptr<float>();
  a.rstd = rstd.data_ptr<float>();
  a.eps = (float)eps;
  hipError_t e = launch_emb_ln_fwd(a, ln_stream(W));
  TORCH_CHECK(e == hipSuccess, "psd emb ln fwd: ", hipGetErrorString(e));
  return {y, mean, rstd};
}

std::vector<at::Tensor> emb_ln_bwd(const at::Tensor& dy_in, const at::Tensor& ids, const at::Tensor& types,
                                   const at::Tensor& W, const at::Tensor& P, const at::Tensor& T,
                                   const at::Tensor& gamma, const at::Tensor& mean, const at::Tensor& rstd, int64_t S,
                                   double p, int64_t seed, c10::optional<at::Tensor> step,
                                   c10::optional<at::Tensor> dgamma_out, c10::optional<at::Tensor> dbeta_out,
                                   c10::optional<at::Tensor> dT_out) {
  EmbLnArgs a = emb_args(ids, types, W, P, T, gamma, S, p, seed, step);
  at::Tensor dy = dy_in.contiguous();
  check_bf16(dy, "dy");
  TORCH_CHECK(dy.numel() == a.rows * a.H && mean.numel() == a.rows && rstd.numel() == a.rows &&
                  mean.scalar_type() == at::kFloat && rstd.scalar_type() == at::kFloat,
              "psd emb ln bwd: shapes");
  const c10::DeviceGuard g(W.device());
  const int64_t H = a.H;
  at::Tensor dx = at::empty({a.rows, H}, W.options());
  at::Tensor dgamma = (dgamma_out.has_value() && dgamma_out->defined()) ? *dgamma_out : at::empty({H}, W.options());
  at::Tensor dbeta = (dbeta_out.has_value() && dbeta_out->defined()) ? *dbeta_out : at::empty({H}, W.options());
  check_bf16(dgamma, "dgamma");
  check_bf16(dbeta, "dbeta");
  TORCH_CHECK(dgamma.numel() == H && dbeta.numel() == H, "psd emb ln bwd: dgamma / dbeta");
  // the type table's gradient rides in the same pass for <= 2 types (else: none here, the caller sums)
  at::Tensor dT;
  if (a.NT <= 2) {
    dT = (dT_out.has_value() && dT_out->defined()) ? *dT_out : at::empty({(int64_t)a.NT, H}, W.options());
    check_bf16(dT, "dT");
    TORCH_CHECK(dT.numel() == a.NT * H, "psd emb ln bwd: dT");
  }
  const int nt = dT.defined() ? a.NT : 0;
  at::Tensor part = at::empty({(int64_t)emb_ln_bwd_blocks(a.rows) * (2 + nt) * H}, W.options().dtype(at::kFloat));
  a.dy = cu16(dy);
  a.mean = mean.data_ptr<float>();
  a.rstd = rstd.data_ptr<float>();
  a.dx = u16(dx);
  a.dgamma = u16(dgamma);
  a.dbeta = u16(dbeta);
  a.dT = dT.defined() ? u16(dT) : nullptr;
  a.part = part.data_ptr<float>();
  hipError_t e = launch_emb_ln_bwd(a, ln_stream(W));
  TORCH_CHECK(e == hipSuccess, "psd emb ln bwd: ", hipGetErrorString(e));
  return {dx, dgamma, dbeta, dT.defined() ? dT : at::Tensor()};
}

}  // namespace psd
