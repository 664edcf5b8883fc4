// Tensor glue for the fused NHWC BatchNorm kernels (kernels/bn.hip).
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>

#include <vector>

#include "kernels/launchers_bn.h"
#include "ops.h"
#include "kernels/launchers_stem.h"

namespace psd {

namespace {

inline hipStream_t stream_of(const at::Tensor& t) { return c10::hip::getCurrentHIPStream(t.device().index()).stream(); }

at::Tensor nhwc(const at::Tensor& t) {
  if (t.dim() == 4) return t.contiguous(at::MemoryFormat::ChannelsLast);
  return t.contiguous();
}

int64_t channels(const at::Tensor& t) { return t.dim() == 4 ? t.size(1) : t.size(-1); }

template <typename T>
T* opt_ptr(const c10::optional<at::Tensor>& t) {
  return (t.has_value() && t->defined()) ? reinterpret_cast<T*>(t->data_ptr()) : nullptr;
}

void check_vec(const c10::optional<at::Tensor>& t, int64_t C, at::ScalarType st, const char* name) {
  if (!t.has_value() || !t->defined()) return;
  TORCH_CHECK(t->numel() == C && t->scalar_type() == st && t->is_contiguous(), "psd bn: ", name, " must be [C] ",
              st);
}

}  // namespace

std::vector<at::Tensor> bn_fwd(const at::Tensor& x_in, c10::optional<at::Tensor> gamma, c10::optional<at::Tensor> beta,
                               c10::optional<at::Tensor> running_mean, c10::optional<at::Tensor> running_var,
                               c10::optional<at::Tensor> residual, bool relu, bool training, double momentum, double eps,
                               c10::optional<at::Tensor> counter, c10::optional<at::Tensor> ss_eval, bool mask_out,
                               c10::optional<at::Tensor> residual_ss, bool stats_only,
                               c10::optional<at::Tensor> q8_out, c10::optional<at::Tensor> part_in,
                               int64_t part_rows, c10::optional<at::Tensor> q8_mx) {
  TORCH_CHECK(x_in.is_cuda() && x_in.scalar_type() == at::kBFloat16, "psd bn: x must be a bf16 device tensor");
  const c10::DeviceGuard g(x_in.device());
  at::Tensor x = nhwc(x_in);
  const int64_t C = channels(x);
  TORCH_CHECK(C % 8 == 0, "psd bn: channels must be a multiple of 8, got ", C);
  const int64_t M = x.numel() / C;
  check_vec(gamma, C, at::kBFloat16, "gamma");
  check_vec(beta, C, at::kBFloat16, "beta");
  check_vec(running_mean, C, at::kFloat, "running_mean");
  check_vec(running_var, C, at::kFloat, "running_var");
  at::Tensor res;
  if (residual.has_value() && residual->defined()) {
    res = nhwc(*residual);
    TORCH_CHECK(res.sizes() == x.sizes() && res.scalar_type() == at::kBFloat16, "psd bn: residual shape/dtype");
  }
  auto f32 = x.options().dtype(at::kFloat);
  TORCH_CHECK(!stats_only || training, "psd bn: stats_only needs training mode");
  const bool rss = residual_ss.has_value() && residual_ss->defined();
  if (rss)
    TORCH_CHECK(res.defined() && relu && residual_ss->numel() == 2 * C && residual_ss->scalar_type() == at::kFloat &&
                    residual_ss->is_contiguous(),
                "psd bn: residual_ss [2C] fp32 needs a residual and ReLU");
  at::Tensor y = stats_only ? at::empty({0}, x.options()) : at::empty_like(x);
  at::Tensor mbits;
  if (relu && mask_out && !stats_only) mbits = at::empty({M * C / 8}, x.options().dtype(at::kByte));
  at::Tensor mean = at::empty({C}, f32), invstd = at::empty({C}, f32);
  at::Tensor ss;
  at::Tensor part, fold;
  const bool have_part = part_in.has_value() && part_in->defined();
  if (training) {
    ss = at::empty({2 * C}, f32);
    if (have_part) {  // statistics partials from the producing convolution's epilogue (kernels/convn.hip)
      TORCH_CHECK(part_rows > 0 && part_in->scalar_type() == at::kFloat && part_in->is_contiguous() &&
                      part_in->numel() >= part_rows * 2 * C && part_in->device() == x.device(),
                  "psd bn: part_in must be fp32 [part_rows, 2, C] on x's device");
      part = *part_in;
      if (part_rows > kFoldRows) fold = at::empty({(int64_t)kFoldRows * 2 * C}, f32);
    } else {
      part = at::empty({(int64_t)bn_reduce_blocks(M, (int)C) * 2 * C}, f32);
    }
  } else {
    TORCH_CHECK(ss_eval.has_value() && ss_eval->numel() == 2 * C, "psd bn: eval mode needs ss_eval [2C]");
    ss = ss_eval->contiguous();
  }
  BnFwdArgs a{};
  a.x = reinterpret_cast<const uint16_t*>(x.data_ptr());
  a.res = res.defined() ? reinterpret_cast<const uint16_t*>(res.data_ptr()) : nullptr;
  a.y = reinterpret_cast<uint16_t*>(y.data_ptr());
  a.mbits = mbits.defined() ? mbits.data_ptr<uint8_t>() : nullptr;
  a.gamma = opt_ptr<const uint16_t>(gamma);
  a.beta = opt_ptr<const uint16_t>(beta);
  a.running_mean = training ? opt_ptr<float>(running_mean) : nullptr;
  a.running_var = training ? opt_ptr<float>(running_var) : nullptr;
  a.save_mean = mean.data_ptr<float>();
  a.save_invstd = invstd.data_ptr<float>();
  a.ss = ss.data_ptr<float>();
  a.part = part.defined() ? part.data_ptr<float>() : nullptr;
  if (training && have_part) {
    a.part_ready = (int32_t)part_rows;
    a.fold_ws = fold.defined() ? fold.data_ptr<float>() : nullptr;
  }
  a.counter = training ? opt_ptr<int64_t>(counter) : nullptr;
  a.M = M;
  a.C = (int32_t)C;
  a.relu = relu;
  a.training = training;
  a.momentum = (float)momentum;
  a.eps = (float)eps;
  a.res_ss = rss ? residual_ss->data_ptr<float>() : nullptr;
  a.stats_only = stats_only;
  if (q8_out.has_value() && q8_out->defined()) {
    const at::Tensor& q = *q8_out;
    const bool laid = q.dim() == 4 ? q.is_contiguous(at::MemoryFormat::ChannelsLast) : q.is_contiguous();
    TORCH_CHECK(!stats_only && relu && q.scalar_type() == at::kFloat8_e4m3fn && q.sizes() == x.sizes() && laid &&
                    (reinterpret_cast<uintptr_t>(q.data_ptr()) & 7) == 0,
                "psd bn: q8_out must be an e4m3fn tensor laid out like x (ReLU BNs)");
    a.q8 = reinterpret_cast<uint8_t*>(q.data_ptr());
    // MX: E8M0 per 32 channels
    TORCH_CHECK(q8_mx.has_value() && q8_mx->defined() && q8_mx->scalar_type() == at::kByte && q8_mx->is_contiguous() &&
                    q8_mx->numel() * 32 == x.numel() && C % 32 == 0 && q8_mx->device() == x.device(),
                "psd bn: q8_out needs q8_mx uint8 [numel / 32] (channels % 32 == 0)");
    a.q8mx = q8_mx->data_ptr<uint8_t>();
  }
  hipError_t e = launch_bn_fwd(a, stream_of(x));
  TORCH_CHECK(e == hipSuccess, "psd bn fwd: ", hipGetErrorString(e));
  return {y, mean, invstd, ss, mbits};
}

at::Tensor bn_reduce_(const at::Tensor& x_in, const at::Tensor& shift) {
  TORCH_CHECK(x_in.is_cuda() && x_in.scalar_type() == at::kBFloat16, "psd bn_reduce: x must be a bf16 device tensor");
  const c10::DeviceGuard g(x_in.device());
  at::Tensor x = nhwc(x_in);
  const int64_t C = channels(x), M = x.numel() / C;
  TORCH_CHECK(C % 8 == 0 && shift.numel() == C && shift.scalar_type() == at::kFloat && shift.is_contiguous(),
              "psd bn_reduce: C % 8 == 0 and an fp32 [C] shift");
  at::Tensor part = at::empty({(int64_t)bn_reduce_blocks(M, (int)C), 2, C}, x.options().dtype(at::kFloat));
  const hipError_t e = launch_bn_reduce(reinterpret_cast<const uint16_t*>(x.data_ptr()), M, (int)C,
                                        shift.data_ptr<float>(), part.data_ptr<float>(), stream_of(x));
  TORCH_CHECK(e == hipSuccess, "psd bn_reduce: ", hipGetErrorString(e));
  return part;
}

namespace {
// optional MX e5m2 side output of a BN backward elementwise pass (dq like x, E8M0 scales [numel/32])
void set_dq(c10::optional<at::Tensor>& dq, c10::optional<at::Tensor>& dqmx, const at::Tensor& x, uint8_t*& q,
            uint8_t*& sc) {
  q = sc = nullptr;
  if (!(dq.has_value() && dq->defined())) return;
  const at::Tensor& t = *dq;
  const bool laid = t.dim() == 4 ? t.is_contiguous(at::MemoryFormat::ChannelsLast) : t.is_contiguous();
  TORCH_CHECK(t.scalar_type() == at::kFloat8_e5m2 && t.sizes() == x.sizes() && laid && dqmx.has_value() &&
                  dqmx->defined() && dqmx->scalar_type() == at::kByte && dqmx->is_contiguous() &&
                  dqmx->numel() * 32 == x.numel() && channels(x) % 32 == 0,
              "psd bn bwd: dq must be e5m2 laid out like x with uint8 [numel / 32] scales (channels % 32 == 0)");
  q = reinterpret_cast<uint8_t*>(t.data_ptr());
  sc = dqmx->data_ptr<uint8_t>();
}
}  // namespace

std::vector<at::Tensor> bn_bwd(const at::Tensor& dy_in, const at::Tensor& x_in, c10::optional<at::Tensor> y_in,
                               c10::optional<at::Tensor> gamma, const at::Tensor& save_mean,
                               const at::Tensor& save_invstd, bool relu, bool need_dr,
                               c10::optional<at::Tensor> dgamma_out, c10::optional<at::Tensor> dbeta_out,
                               c10::optional<at::Tensor> dy2_in, c10::optional<at::Tensor> ss_in,
                               c10::optional<at::Tensor> mbits_in, c10::optional<at::Tensor> dq,
                               c10::optional<at::Tensor> dqmx) {
  const c10::DeviceGuard g(x_in.device());
  at::Tensor x = nhwc(x_in), dy = nhwc(dy_in);
  at::Tensor dy2;
  if (dy2_in.has_value() && dy2_in->defined()) {
    dy2 = nhwc(*dy2_in);
    TORCH_CHECK(dy2.sizes() == x.sizes() && dy2.scalar_type() == at::kBFloat16, "psd bn bwd: dy2 shape/dtype");
  }
  const int64_t C = channels(x);
  const int64_t M = x.numel() / C;
  TORCH_CHECK(dy.sizes() == x.sizes() && dy.scalar_type() == at::kBFloat16, "psd bn bwd: dy shape/dtype");
  at::Tensor y, ss, mbits;
  if (relu) {
    // ReLU mask source: the forward bit-mask, the forward output y, or (no residual) x with the
    // forward scale/shift
    if (mbits_in.has_value() && mbits_in->defined()) {
      mbits = *mbits_in;
      TORCH_CHECK(need_dr, "psd bn bwd: the bit-mask path is for residual BNs");
      TORCH_CHECK(mbits.scalar_type() == at::kByte && mbits.is_contiguous() && mbits.numel() == M * C / 8,
                  "psd bn bwd: mbits must be uint8 [M*C/8]");
    } else if (y_in.has_value() && y_in->defined()) {
      y = nhwc(*y_in);
    } else {
      TORCH_CHECK(ss_in.has_value() && ss_in->defined(), "psd bn bwd: relu needs the forward output or scale/shift");
      TORCH_CHECK(!need_dr, "psd bn bwd: a residual ReLU mask needs the forward output");
      ss = ss_in->contiguous();
      TORCH_CHECK(ss.numel() == 2 * C && ss.scalar_type() == at::kFloat, "psd bn bwd: ss must be fp32 [2C]");
    }
  }
  auto f32 = x.options().dtype(at::kFloat);
  at::Tensor dx = at::empty_like(x);
  at::Tensor dr = need_dr ? at::empty_like(x) : at::Tensor();
  at::Tensor dgamma, dbeta;
  if (gamma.has_value() && gamma->defined()) {
    dgamma = (dgamma_out.has_value() && dgamma_out->defined()) ? *dgamma_out : at::empty({C}, x.options());
    dbeta = (dbeta_out.has_value() && dbeta_out->defined()) ? *dbeta_out : at::empty({C}, x.options());
    TORCH_CHECK(dgamma.numel() == C && dgamma.scalar_type() == at::kBFloat16 && dgamma.is_contiguous(),
                "psd bn bwd: dgamma buffer");
    TORCH_CHECK(dbeta.numel() == C && dbeta.scalar_type() == at::kBFloat16 && dbeta.is_contiguous(),
                "psd bn bwd: dbeta buffer");
  }
  at::Tensor coef = at::empty({3 * C}, f32);
  at::Tensor part = at::empty({(int64_t)bn_reduce_blocks(M, (int)C) * 2 * C}, f32);
  BnBwdArgs a{};
  a.dy = reinterpret_cast<const uint16_t*>(dy.data_ptr());
  a.dy2 = dy2.defined() ? reinterpret_cast<const uint16_t*>(dy2.data_ptr()) : nullptr;
  a.y = y.defined() ? reinterpret_cast<const uint16_t*>(y.data_ptr()) : nullptr;
  a.ss = ss.defined() ? ss.data_ptr<float>() : nullptr;
  a.mbits = mbits.defined() ? mbits.data_ptr<uint8_t>() : nullptr;
  a.x = reinterpret_cast<const uint16_t*>(x.data_ptr());
  a.gamma = opt_ptr<const uint16_t>(gamma);
  a.save_mean = save_mean.data_ptr<float>();
  a.save_invstd = save_invstd.data_ptr<float>();
  a.dx = reinterpret_cast<uint16_t*>(dx.data_ptr());
  a.dr = dr.defined() ? reinterpret_cast<uint16_t*>(dr.data_ptr()) : nullptr;
  a.dgamma = dgamma.defined() ? reinterpret_cast<uint16_t*>(dgamma.data_ptr()) : nullptr;
  a.dbeta = dbeta.defined() ? reinterpret_cast<uint16_t*>(dbeta.data_ptr()) : nullptr;
  a.coef = coef.data_ptr<float>();
  a.part = part.data_ptr<float>();
  a.M = M;
  a.C = (int32_t)C;
  a.relu = relu;
  set_dq(dq, dqmx, x, a.dq, a.dqmx);
  hipError_t e = launch_bn_bwd(a, stream_of(x));
  TORCH_CHECK(e == hipSuccess, "psd bn bwd: ", hipGetErrorString(e));
  return {dx, dr, dgamma, dbeta};
}

// The BN backward's reduction pass alone, as the BN would run it after a bwd-data convolution that
// does not fuse it: ReLU mask from x and ss (mbits absent), or the residual BN's bit-mask with the
// residual-branch gradient dy2 folded in and dr written. Autotune timing twin (ops/conv.py).
// Returns the partials.
at::Tensor bn_bwd_reduce_(const at::Tensor& dy_in, const at::Tensor& x_in, const at::Tensor& save_mean,
                          c10::optional<at::Tensor> ss_in, c10::optional<at::Tensor> dy2_in,
                          c10::optional<at::Tensor> mbits_in) {
  const c10::DeviceGuard g(x_in.device());
  at::Tensor x = nhwc(x_in), dy = nhwc(dy_in);
  const int64_t C = channels(x), M = x.numel() / C;
  TORCH_CHECK(dy.sizes() == x.sizes() && dy.scalar_type() == at::kBFloat16 && x.scalar_type() == at::kBFloat16 &&
                  C % 8 == 0 && save_mean.numel() == C,
              "psd bn_bwd_reduce: dy like x (bf16, C % 8 == 0), mean [C]");
  const bool bits = mbits_in.has_value() && mbits_in->defined();
  at::Tensor dy2, ss, mbits, dr;
  if (bits) {
    mbits = *mbits_in;
    TORCH_CHECK(mbits.scalar_type() == at::kByte && mbits.is_contiguous() && mbits.numel() == M * C / 8,
                "psd bn_bwd_reduce: mbits must be uint8 [M*C/8]");
    dr = at::empty_like(x);
  } else {
    TORCH_CHECK(ss_in.has_value() && ss_in->defined() && ss_in->numel() == 2 * C, "psd bn_bwd_reduce: ss [2C]");
    ss = ss_in->contiguous();
  }
  if (dy2_in.has_value() && dy2_in->defined()) {
    dy2 = nhwc(*dy2_in);
    TORCH_CHECK(dy2.sizes() == x.sizes() && dy2.scalar_type() == at::kBFloat16, "psd bn_bwd_reduce: dy2 like x");
  }
  at::Tensor part = at::empty({(int64_t)bn_reduce_blocks(M, (int)C), 2, C}, x.options().dtype(at::kFloat));
  BnBwdArgs a{};
  a.dy = reinterpret_cast<const uint16_t*>(dy.data_ptr());
  a.dy2 = dy2.defined() ? reinterpret_cast<const uint16_t*>(dy2.data_ptr()) : nullptr;
  a.ss = ss.defined() ? ss.data_ptr<float>() : nullptr;
  a.mbits = bits ? mbits.data_ptr<uint8_t>() : nullptr;
  a.x = reinterpret_cast<const uint16_t*>(x.data_ptr());
  a.save_mean = save_mean.data_ptr<float>();
  a.dr = dr.defined() ? reinterpret_cast<uint16_t*>(dr.data_ptr()) : nullptr;
  a.part = part.data_ptr<float>();
  a.M = M;
  a.C = (int32_t)C;
  a.relu = 1;
  a.reduce_only = 1;
  const hipError_t e = launch_bn_bwd(a, stream_of(x));
  TORCH_CHECK(e == hipSuccess, "psd bn_bwd_reduce: ", hipGetErrorString(e));
  return part;
}


// BN backward whose reduction the producing convolution's bwd-data epilogue already ran
// (kernels/convn.hip bwd modes): g = the masked gradient (for a residual BN also the residual-branch
// gradient), part = [rows, 2, C] partials. Returns {dx, dgamma, dbeta}.
std::vector<at::Tensor> bn_bwd_pre(const at::Tensor& g_in, const at::Tensor& x_in, c10::optional<at::Tensor> gamma,
                                   const at::Tensor& save_mean, const at::Tensor& save_invstd, const at::Tensor& part,
                                   int64_t rows, c10::optional<at::Tensor> dgamma_out,
                                   c10::optional<at::Tensor> dbeta_out, c10::optional<at::Tensor> dq,
                                   c10::optional<at::Tensor> dqmx) {
  const c10::DeviceGuard dg(x_in.device());
  at::Tensor x = nhwc(x_in), g = nhwc(g_in);
  const int64_t C = channels(x), M = x.numel() / C;
  TORCH_CHECK(g.sizes() == x.sizes() && g.scalar_type() == at::kBFloat16 && x.scalar_type() == at::kBFloat16,
              "psd bn_bwd_pre: g like x (bf16)");
  TORCH_CHECK(part.scalar_type() == at::kFloat && part.is_contiguous() && rows > 0 && part.numel() >= rows * 2 * C,
              "psd bn_bwd_pre: part must be fp32 [rows, 2, C]");
  auto f32 = x.options().dtype(at::kFloat);
  at::Tensor dx = at::empty_like(x);
  at::Tensor dgamma, dbeta;
  if (gamma.has_value() && gamma->defined()) {
    dgamma = (dgamma_out.has_value() && dgamma_out->defined()) ? *dgamma_out : at::empty({C}, x.options());
    dbeta = (dbeta_out.has_value() && dbeta_out->defined()) ? *dbeta_out : at::empty({C}, x.options());
  }
  at::Tensor coef = at::empty({3 * C}, f32);
  at::Tensor fold = rows > kFoldRows ? at::empty({(int64_t)kFoldRows * 2 * C}, f32) : at::Tensor();
  uint8_t *q8, *q8mx;
  set_dq(dq, dqmx, x, q8, q8mx);
  const hipError_t e = launch_bn_bwd_pre(
      reinterpret_cast<const uint16_t*>(g.data_ptr()), reinterpret_cast<const uint16_t*>(x.data_ptr()),
      opt_ptr<const uint16_t>(gamma), save_mean.data_ptr<float>(), save_invstd.data_ptr<float>(),
      part.data_ptr<float>(), (int)rows, fold.defined() ? fold.data_ptr<float>() : nullptr,
      dgamma.defined() ? reinterpret_cast<uint16_t*>(dgamma.data_ptr()) : nullptr,
      dbeta.defined() ? reinterpret_cast<uint16_t*>(dbeta.data_ptr()) : nullptr, coef.data_ptr<float>(),
      reinterpret_cast<uint16_t*>(dx.data_ptr()), M, (int)C, stream_of(x), q8, q8mx);
  TORCH_CHECK(e == hipSuccess, "psd bn_bwd_pre: ", hipGetErrorString(e));
  return {dx, dgamma, dbeta};
}

// relu(bn3(x) + bnd(xd)) backward (ops/bn.py _BNAddBNReluFn): bn3 through its forward bit-mask, and
// the downsample BN fed by the residual gradient dr, in one reduce and one elementwise pass.
// Returns {dx, dxd, dgamma, dbeta, dgamma_d, dbeta_d}.
std::vector<at::Tensor> bn_bwd_dual(const at::Tensor& dy_in, const at::Tensor& x_in, const at::Tensor& gamma,
                                    const at::Tensor& save_mean, const at::Tensor& save_invstd, const at::Tensor& mbits,
                                    c10::optional<at::Tensor> dy2_in, const at::Tensor& xd_in, const at::Tensor& gamma_d,
                                    const at::Tensor& mean_d, const at::Tensor& invstd_d,
                                    c10::optional<at::Tensor> dgamma_out, c10::optional<at::Tensor> dbeta_out,
                                    c10::optional<at::Tensor> dgamma_d_out, c10::optional<at::Tensor> dbeta_d_out,
                                    bool fold) {
  const c10::DeviceGuard g(x_in.device());
  at::Tensor x = nhwc(x_in), dy = nhwc(dy_in), xd = nhwc(xd_in);
  const int64_t C = channels(x);
  const int64_t M = x.numel() / C;
  TORCH_CHECK(C % 8 == 0 && dy.sizes() == x.sizes() && xd.sizes() == x.sizes() &&
                  dy.scalar_type() == at::kBFloat16 && xd.scalar_type() == at::kBFloat16,
              "psd bn bwd_dual: dy / xd like x (bf16)");
  at::Tensor dy2;
  if (dy2_in.has_value() && dy2_in->defined()) {
    dy2 = nhwc(*dy2_in);
    TORCH_CHECK(dy2.sizes() == x.sizes() && dy2.scalar_type() == at::kBFloat16, "psd bn bwd_dual: dy2 shape/dtype");
  }
  TORCH_CHECK(mbits.scalar_type() == at::kByte && mbits.is_contiguous() && mbits.numel() == M * C / 8,
              "psd bn bwd_dual: mbits must be uint8 [M*C/8]");
  for (const at::Tensor* t : {&save_mean, &save_invstd, &mean_d, &invstd_d})
    TORCH_CHECK(t->numel() == C && t->scalar_type() == at::kFloat && t->is_contiguous(), "psd bn bwd_dual: stats [C]");
  auto grad_buf = [&](const c10::optional<at::Tensor>& o) {
    at::Tensor t = (o.has_value() && o->defined()) ? *o : at::empty({C}, x.options());
    TORCH_CHECK(t.numel() == C && t.scalar_type() == at::kBFloat16 && t.is_contiguous(), "psd bn bwd_dual: grad buffer");
    return t;
  };
  at::Tensor dgamma = grad_buf(dgamma_out), dbeta = grad_buf(dbeta_out);
  at::Tensor dgamma_d = grad_buf(dgamma_d_out), dbeta_d = grad_buf(dbeta_d_out);
  auto f32 = x.options().dtype(at::kFloat);
  // fold: no dx (the consumer convolution folds it); its coefficients and dr (= g) are returned
  at::Tensor dx = fold ? at::Tensor() : at::empty_like(x), dxd = at::empty_like(x), dr = at::empty_like(x);
  at::Tensor coef = at::empty({3 * C}, f32), coef_d = at::empty({3 * C}, f32);
  const int64_t np = (int64_t)bn_reduce_blocks(M, (int)C) * 2 * C;
  at::Tensor part = at::empty({np}, f32), part_d = at::empty({np}, f32);
  BnBwdArgs a{};
  a.dy = reinterpret_cast<const uint16_t*>(dy.data_ptr());
  a.dy2 = dy2.defined() ? reinterpret_cast<const uint16_t*>(dy2.data_ptr()) : nullptr;
  a.mbits = mbits.data_ptr<uint8_t>();
  a.x = reinterpret_cast<const uint16_t*>(x.data_ptr());
  a.gamma = reinterpret_cast<const uint16_t*>(gamma.data_ptr());
  a.save_mean = save_mean.data_ptr<float>();
  a.save_invstd = save_invstd.data_ptr<float>();
  a.dx = fold ? nullptr : reinterpret_cast<uint16_t*>(dx.data_ptr());
  a.dr = reinterpret_cast<uint16_t*>(dr.data_ptr());
  a.dgamma = reinterpret_cast<uint16_t*>(dgamma.data_ptr());
  a.dbeta = reinterpret_cast<uint16_t*>(dbeta.data_ptr());
  a.coef = coef.data_ptr<float>();
  a.part = part.data_ptr<float>();
  a.M = M;
  a.C = (int32_t)C;
  a.relu = 1;
  a.xd = reinterpret_cast<const uint16_t*>(xd.data_ptr());
  a.gamma_d = reinterpret_cast<const uint16_t*>(gamma_d.data_ptr());
  a.mean_d = mean_d.data_ptr<float>();
  a.invstd_d = invstd_d.data_ptr<float>();
  a.dxd = reinterpret_cast<uint16_t*>(dxd.data_ptr());
  a.dgamma_d = reinterpret_cast<uint16_t*>(dgamma_d.data_ptr());
  a.dbeta_d = reinterpret_cast<uint16_t*>(dbeta_d.data_ptr());
  a.coef_d = coef_d.data_ptr<float>();
  a.part_d = part_d.data_ptr<float>();
  hipError_t e = launch_bn_bwd(a, stream_of(x));
  TORCH_CHECK(e == hipSuccess, "psd bn bwd_dual: ", hipGetErrorString(e));
  if (fold) return {dx, dxd, dgamma, dbeta, dgamma_d, dbeta_d, coef, dr};
  return {dx, dxd, dgamma, dbeta, dgamma_d, dbeta_d};
}

// BN backward without the elementwise pass (the BN-backward fold: the consumer convolution's dgrad /
// wgrad take g and these coefficients, kernels/bnfold.hip): returns {g, coef [3C] = (A, B, C) of
// dx = A g + B x + C, dgamma, dbeta}. With `part` the producer-reduced partials of an already masked
// g = dy (kernels/convn.hip bwd mode 2); else one reduction pass over dy (+ dy2) under the forward
// bit-mask that also writes g (the residual-branch gradient).
std::vector<at::Tensor> bn_bwd_coef(const at::Tensor& dy_in, const at::Tensor& x_in, const at::Tensor& gamma,
                                    const at::Tensor& save_mean, const at::Tensor& save_invstd,
                                    c10::optional<at::Tensor> mbits_in, c10::optional<at::Tensor> dy2_in,
                                    c10::optional<at::Tensor> part, int64_t rows, c10::optional<at::Tensor> dgamma_out,
                                    c10::optional<at::Tensor> dbeta_out) {
  const c10::DeviceGuard dg(x_in.device());
  at::Tensor x = nhwc(x_in), dy = nhwc(dy_in);
  const int64_t C = channels(x), M = x.numel() / C;
  TORCH_CHECK(C % 8 == 0 && dy.sizes() == x.sizes() && dy.scalar_type() == at::kBFloat16 &&
                  x.scalar_type() == at::kBFloat16,
              "psd bn_bwd_coef: dy like x (bf16)");
  for (const at::Tensor* t : {&save_mean, &save_invstd})
    TORCH_CHECK(t->numel() == C && t->scalar_type() == at::kFloat && t->is_contiguous(), "psd bn_bwd_coef: stats [C]");
  auto f32 = x.options().dtype(at::kFloat);
  auto grad_buf = [&](const c10::optional<at::Tensor>& o) {
    at::Tensor t = (o.has_value() && o->defined()) ? *o : at::empty({C}, x.options());
    TORCH_CHECK(t.numel() == C && t.scalar_type() == at::kBFloat16 && t.is_contiguous(), "psd bn_bwd_coef: grad buffer");
    return t;
  };
  at::Tensor dgamma = grad_buf(dgamma_out), dbeta = grad_buf(dbeta_out);
  at::Tensor coef = at::empty({3 * C}, f32);
  const uint16_t* gam = reinterpret_cast<const uint16_t*>(gamma.data_ptr());
  if (part.has_value() && part->defined()) {
    TORCH_CHECK(part->scalar_type() == at::kFloat && part->is_contiguous() && rows > 0 && part->numel() >= rows * 2 * C,
                "psd bn_bwd_coef: part must be fp32 [rows, 2, C]");
    at::Tensor fold = rows > kFoldRows ? at::empty({(int64_t)kFoldRows * 2 * C}, f32) : at::Tensor();
    const hipError_t e = launch_bn_bwd_pre(
        reinterpret_cast<const uint16_t*>(dy.data_ptr()), reinterpret_cast<const uint16_t*>(x.data_ptr()), gam,
        save_mean.data_ptr<float>(), save_invstd.data_ptr<float>(), part->data_ptr<float>(), (int)rows,
        fold.defined() ? fold.data_ptr<float>() : nullptr, reinterpret_cast<uint16_t*>(dgamma.data_ptr()),
        reinterpret_cast<uint16_t*>(dbeta.data_ptr()), coef.data_ptr<float>(), nullptr, M, (int)C, stream_of(x));
    TORCH_CHECK(e == hipSuccess, "psd bn_bwd_coef: ", hipGetErrorString(e));
    return {dy, coef, dgamma, dbeta};
  }
  TORCH_CHECK(mbits_in.has_value() && mbits_in->defined() && mbits_in->scalar_type() == at::kByte &&
                  mbits_in->is_contiguous() && mbits_in->numel() == M * C / 8,
              "psd bn_bwd_coef: without partials the forward bit-mask (uint8 [M*C/8]) is required");
  at::Tensor dy2;
  if (dy2_in.has_value() && dy2_in->defined()) {
    dy2 = nhwc(*dy2_in);
    TORCH_CHECK(dy2.sizes() == x.sizes() && dy2.scalar_type() == at::kBFloat16, "psd bn_bwd_coef: dy2 shape/dtype");
  }
  at::Tensor g = at::empty_like(x);
  at::Tensor pt = at::empty({(int64_t)bn_reduce_blocks(M, (int)C) * 2 * C}, f32);
  BnBwdArgs a{};
  a.dy = reinterpret_cast<const uint16_t*>(dy.data_ptr());
  a.dy2 = dy2.defined() ? reinterpret_cast<const uint16_t*>(dy2.data_ptr()) : nullptr;
  a.mbits = mbits_in->data_ptr<uint8_t>();
  a.x = reinterpret_cast<const uint16_t*>(x.data_ptr());
  a.gamma = gam;
  a.save_mean = save_mean.data_ptr<float>();
  a.save_invstd = save_invstd.data_ptr<float>();
  a.dr = reinterpret_cast<uint16_t*>(g.data_ptr());
  a.dgamma = reinterpret_cast<uint16_t*>(dgamma.data_ptr());
  a.dbeta = reinterpret_cast<uint16_t*>(dbeta.data_ptr());
  a.coef = coef.data_ptr<float>();
  a.part = pt.data_ptr<float>();
  a.M = M;
  a.C = (int32_t)C;
  a.relu = 1;
  a.coef_only = 1;
  const hipError_t e = launch_bn_bwd(a, stream_of(x));
  TORCH_CHECK(e == hipSuccess, "psd bn_bwd_coef: ", hipGetErrorString(e));
  return {g, coef, dgamma, dbeta};
}

// Stem BN + ReLU + 3x3/s2 max-pool (training forward): returns {y_pool, argmax, mean, invstd, ss}.
std::vector<at::Tensor> bn_pool_fwd(const at::Tensor& x_in, const at::Tensor& gamma, const at::Tensor& beta,
                                    const at::Tensor& running_mean, const at::Tensor& running_var, double momentum,
                                    double eps, c10::optional<at::Tensor> counter) {
  TORCH_CHECK(x_in.is_cuda() && x_in.scalar_type() == at::kBFloat16 && x_in.dim() == 4, "psd bn_pool: bf16 NCHW-shaped x");
  const c10::DeviceGuard g(x_in.device());
  at::Tensor x = nhwc(x_in);
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(bn_pool_supported((int)H, (int)W, (int)C), "psd bn_pool: unsupported shape ", x.sizes());
  const int64_t M = N * H * W;
  check_vec(gamma, C, at::kBFloat16, "gamma");
  check_vec(beta, C, at::kBFloat16, "beta");
  check_vec(running_mean, C, at::kFloat, "running_mean");
  check_vec(running_var, C, at::kFloat, "running_var");
  auto f32 = x.options().dtype(at::kFloat);
  const auto cl = x.options().memory_format(at::MemoryFormat::ChannelsLast);
  at::Tensor y = at::empty({N, C, H / 2, W / 2}, cl);
  at::Tensor arg = at::empty({N, C, H / 2, W / 2}, cl.dtype(at::kByte));
  at::Tensor mean = at::empty({C}, f32), invstd = at::empty({C}, f32), ss = at::empty({2 * C}, f32);
  at::Tensor part = at::empty({(int64_t)bn_reduce_blocks(M, (int)C) * 2 * C}, f32);
  BnFwdArgs a{};
  a.x = reinterpret_cast<const uint16_t*>(x.data_ptr());
  a.y = reinterpret_cast<uint16_t*>(y.data_ptr());
  a.gamma = reinterpret_cast<const uint16_t*>(gamma.data_ptr());
  a.beta = reinterpret_cast<const uint16_t*>(beta.data_ptr());
  a.running_mean = running_mean.data_ptr<float>();
  a.running_var = running_var.data_ptr<float>();
  a.save_mean = mean.data_ptr<float>();
  a.save_invstd = invstd.data_ptr<float>();
  a.ss = ss.data_ptr<float>();
  a.part = part.data_ptr<float>();
  a.counter = opt_ptr<int64_t>(counter);
  a.pool_arg = arg.data_ptr<uint8_t>();
  a.N = (int32_t)N;
  a.H = (int32_t)H;
  a.W = (int32_t)W;
  a.M = M;
  a.C = (int32_t)C;
  a.relu = 1;
  a.training = 1;
  a.momentum = (float)momentum;
  a.eps = (float)eps;
  hipError_t e = launch_bn_fwd(a, stream_of(x));
  TORCH_CHECK(e == hipSuccess, "psd bn_pool fwd: ", hipGetErrorString(e));
  return {y, arg, mean, invstd, ss};
}

// ResNet stem forward: conv 7x7/s2/p3 (3 -> 64, kernels/stem.hip, BN statistics reduced in its
// epilogue) -> BN finalize -> fused BN + ReLU + max-pool. Returns {y_pool, argmax, mean, invstd, ss,
// conv_out}; conv_out (the BN input) is kept for the backward.
std::vector<at::Tensor> stem_fwd(const at::Tensor& x_in, const at::Tensor& w, const at::Tensor& gamma,
                                 const at::Tensor& beta, const at::Tensor& running_mean, const at::Tensor& running_var,
                                 double momentum, double eps, c10::optional<at::Tensor> counter) {
  TORCH_CHECK(x_in.is_cuda() && x_in.scalar_type() == at::kBFloat16 && x_in.dim() == 4 && x_in.size(1) == 3,
              "psd stem: bf16 [N, 3, H, W] input");
  TORCH_CHECK(w.scalar_type() == at::kBFloat16 && w.sizes() == at::IntArrayRef({64, 3, 7, 7}), "psd stem: weight [64,3,7,7]");
  const c10::DeviceGuard g(x_in.device());
  at::Tensor x = x_in.contiguous(at::MemoryFormat::ChannelsLast);
  const int64_t N = x.size(0), H = x.size(2), W = x.size(3), Ho = H / 2, Wo = W / 2;
  TORCH_CHECK(stem_conv_supported((int)H, (int)W, (int)Ho, (int)Wo) && bn_pool_supported((int)Ho, (int)Wo, 64),
              "psd stem: unsupported input ", x.sizes());
  check_vec(gamma, 64, at::kBFloat16, "gamma");
  check_vec(beta, 64, at::kBFloat16, "beta");
  check_vec(running_mean, 64, at::kFloat, "running_mean");
  check_vec(running_var, 64, at::kFloat, "running_var");
  // [co][ci][kh][kw] -> [co][kh*24 + kw*3 + ci], zero for kw*3+ci >= 21 and the 8th kh block
  at::Tensor wk = at::constant_pad_nd(w.permute({0, 2, 3, 1}).reshape({64, 7, 21}), {0, 3, 0, 1}).reshape({64, 192})
                      .contiguous();
  const auto cl = x.options().memory_format(at::MemoryFormat::ChannelsLast);
  auto f32 = x.options().dtype(at::kFloat);
  at::Tensor conv = at::empty({N, 64, Ho, Wo}, cl);
  const int nblk = stem_conv_blocks((int)N, (int)Ho);
  at::Tensor part = at::empty({(int64_t)nblk * 128}, f32);
  hipStream_t st = stream_of(x);
  hipError_t e = launch_stem_conv(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                                  reinterpret_cast<const uint16_t*>(wk.data_ptr()),
                                  reinterpret_cast<uint16_t*>(conv.data_ptr()), running_mean.data_ptr<float>(),
                                  part.data_ptr<float>(), (int)N, (int)H, (int)W, (int)Ho, (int)Wo, st);
  TORCH_CHECK(e == hipSuccess, "psd stem conv: ", hipGetErrorString(e));
  at::Tensor y = at::empty({N, 64, Ho / 2, Wo / 2}, cl);
  at::Tensor arg = at::empty({N, 64, Ho / 2, Wo / 2}, cl.dtype(at::kByte));
  at::Tensor mean = at::empty({64}, f32), invstd = at::empty({64}, f32), ss = at::empty({128}, f32);
  BnFwdArgs a{};
  a.x = reinterpret_cast<const uint16_t*>(conv.data_ptr());
  a.y = reinterpret_cast<uint16_t*>(y.data_ptr());
  a.gamma = reinterpret_cast<const uint16_t*>(gamma.data_ptr());
  a.beta = reinterpret_cast<const uint16_t*>(beta.data_ptr());
  a.running_mean = running_mean.data_ptr<float>();
  a.running_var = running_var.data_ptr<float>();
  a.save_mean = mean.data_ptr<float>();
  a.save_invstd = invstd.data_ptr<float>();
  a.ss = ss.data_ptr<float>();
  a.part = part.data_ptr<float>();
  a.part_ready = nblk;
  a.counter = opt_ptr<int64_t>(counter);
  a.pool_arg = arg.data_ptr<uint8_t>();
  a.N = (int32_t)N;
  a.H = (int32_t)Ho;
  a.W = (int32_t)Wo;
  a.M = N * Ho * Wo;
  a.C = 64;
  a.relu = 1;
  a.training = 1;
  a.momentum = (float)momentum;
  a.eps = (float)eps;
  e = launch_bn_fwd(a, st);
  TORCH_CHECK(e == hipSuccess, "psd stem bn_pool: ", hipGetErrorString(e));
  return {y, arg, mean, invstd, ss, conv};
}

// Weight gradient of the stem conv (kernels/stem.hip): x [N, 3, H, W], dy [N, 64, H/2, W/2] (both
// channels_last bf16) -> dW [64, 3, 7, 7] bf16 channels_last.
at::Tensor stem_wgrad(const at::Tensor& x_in, const at::Tensor& dy_in) {
  TORCH_CHECK(x_in.is_cuda() && x_in.scalar_type() == at::kBFloat16 && x_in.dim() == 4 && x_in.size(1) == 3,
              "psd stem wgrad: bf16 [N, 3, H, W] input");
  const c10::DeviceGuard g(x_in.device());
  at::Tensor x = x_in.contiguous(at::MemoryFormat::ChannelsLast), dy = dy_in.contiguous(at::MemoryFormat::ChannelsLast);
  const int64_t N = x.size(0), H = x.size(2), W = x.size(3), Ho = H / 2, Wo = W / 2;
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && dy.sizes() == at::IntArrayRef({N, 64, Ho, Wo}), "psd stem wgrad: dy shape");
  TORCH_CHECK(stem_wgrad_supported((int)H, (int)W, (int)Ho, (int)Wo), "psd stem wgrad: unsupported input ", x.sizes());
  const int nblk = stem_wgrad_blocks((int)N, (int)Ho, (int)Wo);
  at::Tensor part = at::empty({(int64_t)nblk * 192 * 64}, x.options().dtype(at::kFloat));
  at::Tensor dw = at::empty({64, 3, 7, 7}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  hipError_t e = launch_stem_wgrad(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                                   reinterpret_cast<const uint16_t*>(dy.data_ptr()), part.data_ptr<float>(),
                                   reinterpret_cast<uint16_t*>(dw.data_ptr()), (int)N, (int)H, (int)W, (int)Ho, (int)Wo,
                                   stream_of(x));
  TORCH_CHECK(e == hipSuccess, "psd stem wgrad: ", hipGetErrorString(e));
  return dw;
}

// Backward of bn_pool_fwd: gpool (+ gpool2, a second consumer's gradient of the pooled output)
// -> {dx, dgamma, dbeta}; the pool gradient is recomputed inside the BN passes.
std::vector<at::Tensor> bn_pool_bwd(const at::Tensor& gpool_in, c10::optional<at::Tensor> gpool2_in, const at::Tensor& arg,
                                    const at::Tensor& x_in, const at::Tensor& gamma, const at::Tensor& save_mean,
                                    const at::Tensor& save_invstd, const at::Tensor& ss,
                                    c10::optional<at::Tensor> dgamma_out, c10::optional<at::Tensor> dbeta_out) {
  const c10::DeviceGuard g(x_in.device());
  at::Tensor x = nhwc(x_in), gp = nhwc(gpool_in);
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(bn_pool_supported((int)H, (int)W, (int)C), "psd bn_pool bwd: unsupported shape ", x.sizes());
  const std::vector<int64_t> ps{N, C, H / 2, W / 2};
  TORCH_CHECK(gp.sizes() == ps && gp.scalar_type() == at::kBFloat16, "psd bn_pool bwd: gpool shape/dtype");
  TORCH_CHECK(arg.sizes() == ps && arg.scalar_type() == at::kByte && arg.is_contiguous(at::MemoryFormat::ChannelsLast),
              "psd bn_pool bwd: argmax shape");
  TORCH_CHECK(ss.numel() == 2 * C && ss.scalar_type() == at::kFloat && ss.is_contiguous(), "psd bn_pool bwd: ss");
  at::Tensor gp2;
  if (gpool2_in.has_value() && gpool2_in->defined()) {
    gp2 = nhwc(*gpool2_in);
    TORCH_CHECK(gp2.sizes() == ps && gp2.scalar_type() == at::kBFloat16, "psd bn_pool bwd: gpool2 shape/dtype");
  }
  const int64_t M = N * H * W;
  auto f32 = x.options().dtype(at::kFloat);
  at::Tensor dx = at::empty_like(x);
  at::Tensor dgamma = (dgamma_out.has_value() && dgamma_out->defined()) ? *dgamma_out : at::empty({C}, x.options());
  at::Tensor dbeta = (dbeta_out.has_value() && dbeta_out->defined()) ? *dbeta_out : at::empty({C}, x.options());
  TORCH_CHECK(dgamma.numel() == C && dgamma.scalar_type() == at::kBFloat16 && dgamma.is_contiguous(), "psd bn_pool: dgamma");
  TORCH_CHECK(dbeta.numel() == C && dbeta.scalar_type() == at::kBFloat16 && dbeta.is_contiguous(), "psd bn_pool: dbeta");
  at::Tensor coef = at::empty({3 * C}, f32);
  at::Tensor part = at::empty({(int64_t)bn_pool_reduce_blocks((int)N, (int)H, (int)W, (int)C) * 2 * C}, f32);
  BnBwdArgs a{};
  a.gpool = reinterpret_cast<const uint16_t*>(gp.data_ptr());
  a.gpool2 = gp2.defined() ? reinterpret_cast<const uint16_t*>(gp2.data_ptr()) : nullptr;
  a.pool_arg = arg.data_ptr<uint8_t>();
  a.ss = ss.data_ptr<float>();
  a.x = reinterpret_cast<const uint16_t*>(x.data_ptr());
  a.gamma = reinterpret_cast<const uint16_t*>(gamma.data_ptr());
  a.save_mean = save_mean.data_ptr<float>();
  a.save_invstd = save_invstd.data_ptr<float>();
  a.dx = reinterpret_cast<uint16_t*>(dx.data_ptr());
  a.dgamma = reinterpret_cast<uint16_t*>(dgamma.data_ptr());
  a.dbeta = reinterpret_cast<uint16_t*>(dbeta.data_ptr());
  a.coef = coef.data_ptr<float>();
  a.part = part.data_ptr<float>();
  a.N = (int32_t)N;
  a.H = (int32_t)H;
  a.W = (int32_t)W;
  a.M = M;
  a.C = (int32_t)C;
  a.relu = 1;
  hipError_t e = launch_bn_bwd(a, stream_of(x));
  TORCH_CHECK(e == hipSuccess, "psd bn_pool bwd: ", hipGetErrorString(e));
  return {dx, dgamma, dbeta};
}

}  // namespace psd

// ---- NHWC 3x3/s2/p1 max-pool (kernels/pool.hip)
#include "kernels/launchers_pool.h"
namespace psd {
std::vector<at::Tensor> maxpool3s2_fwd(const at::Tensor& x_in) {
  TORCH_CHECK(x_in.is_cuda() && x_in.scalar_type() == at::kBFloat16 && x_in.dim() == 4, "psd maxpool: bf16 NCHW-shaped");
  const c10::DeviceGuard g(x_in.device());
  at::Tensor x = x_in.contiguous(at::MemoryFormat::ChannelsLast);
  const int N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int Ho = (H + 2 - 3) / 2 + 1, Wo = (W + 2 - 3) / 2 + 1;
  at::Tensor y = at::empty({N, C, Ho, Wo}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  at::Tensor arg = at::empty({N, C, Ho, Wo}, x.options().dtype(at::kByte).memory_format(at::MemoryFormat::ChannelsLast));
  hipError_t e = launch_maxpool_fwd(reinterpret_cast<const uint16_t*>(x.data_ptr()), reinterpret_cast<uint16_t*>(y.data_ptr()),
                                    arg.data_ptr<uint8_t>(), N, H, W, C, Ho, Wo, stream_of(x));
  TORCH_CHECK(e == hipSuccess, "psd maxpool fwd: ", hipGetErrorString(e));
  return {y, arg};
}
at::Tensor maxpool3s2_bwd(const at::Tensor& dy_in, const at::Tensor& arg, int64_t H, int64_t W,
                          const c10::optional<at::Tensor>& dy2_in) {
  const c10::DeviceGuard g(dy_in.device());
  at::Tensor dy = dy_in.contiguous(at::MemoryFormat::ChannelsLast);
  const int N = dy.size(0), C = dy.size(1), Ho = dy.size(2), Wo = dy.size(3);
  TORCH_CHECK(arg.is_contiguous(at::MemoryFormat::ChannelsLast) && arg.sizes() == dy.sizes(), "psd maxpool bwd: argmax shape");
  at::Tensor dy2;
  if (dy2_in.has_value() && dy2_in->defined()) {
    dy2 = dy2_in->contiguous(at::MemoryFormat::ChannelsLast);
    TORCH_CHECK(dy2.sizes() == dy.sizes() && dy2.scalar_type() == at::kBFloat16, "psd maxpool bwd: dy2 shape/dtype");
  }
  at::Tensor dx = at::empty({N, C, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  hipError_t e = launch_maxpool_bwd(reinterpret_cast<const uint16_t*>(dy.data_ptr()),
                                    dy2.defined() ? reinterpret_cast<const uint16_t*>(dy2.data_ptr()) : nullptr,
                                    arg.data_ptr<uint8_t>(),
                                    reinterpret_cast<uint16_t*>(dx.data_ptr()), N, (int)H, (int)W, C, Ho, Wo, stream_of(dy));
  TORCH_CHECK(e == hipSuccess, "psd maxpool bwd: ", hipGetErrorString(e));
  return dx;
}
}  // namespace psd

// ---- NHWC global average pool (kernels/pool.hip)
namespace psd {
at::Tensor gap_fwd(const at::Tensor& x_in) {
  TORCH_CHECK(x_in.is_cuda() && x_in.scalar_type() == at::kBFloat16 && x_in.dim() == 4 && x_in.size(1) % 8 == 0,
              "psd gap: bf16 NCHW-shaped, C % 8 == 0");
  const c10::DeviceGuard g(x_in.device());
  at::Tensor x = x_in.contiguous(at::MemoryFormat::ChannelsLast);
  const int N = x.size(0), C = x.size(1), HW = x.size(2) * x.size(3);
  at::Tensor y = at::empty({N, C}, x.options());
  hipError_t e = launch_gap_fwd(reinterpret_cast<const uint16_t*>(x.data_ptr()), reinterpret_cast<uint16_t*>(y.data_ptr()),
                                N, HW, C, stream_of(x));
  TORCH_CHECK(e == hipSuccess, "psd gap fwd: ", hipGetErrorString(e));
  return y;
}
at::Tensor gap_bwd(const at::Tensor& dy_in, int64_t H, int64_t W) {
  TORCH_CHECK(dy_in.is_cuda() && dy_in.scalar_type() == at::kBFloat16 && dy_in.dim() == 2 && dy_in.size(1) % 8 == 0,
              "psd gap bwd: bf16 [N, C], C % 8 == 0");
  const c10::DeviceGuard g(dy_in.device());
  at::Tensor dy = dy_in.contiguous();
  const int N = dy.size(0), C = dy.size(1);
  at::Tensor dx = at::empty({N, C, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  hipError_t e = launch_gap_bwd(reinterpret_cast<const uint16_t*>(dy.data_ptr()), reinterpret_cast<uint16_t*>(dx.data_ptr()),
                                N, (int)(H * W), C, stream_of(dy));
  TORCH_CHECK(e == hipSuccess, "psd gap bwd: ", hipGetErrorString(e));
  return dx;
}
at::Tensor subsample2(const at::Tensor& x) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast) && x.size(1) % 8 == 0 && x.size(2) % 2 == 0 &&
                  x.size(3) % 2 == 0,
              "psd subsample2: channels_last bf16 [N, C, H, W], C % 8 == 0, H and W even");
  const c10::DeviceGuard g(x.device());
  at::Tensor y = at::empty({x.size(0), x.size(1), x.size(2) / 2, x.size(3) / 2},
                           x.options().memory_format(at::MemoryFormat::ChannelsLast));
  hipError_t e = launch_subsample2(reinterpret_cast<const uint16_t*>(x.data_ptr()), reinterpret_cast<uint16_t*>(y.data_ptr()),
                                   (int)x.size(0), (int)x.size(2), (int)x.size(3), (int)x.size(1), stream_of(x));
  TORCH_CHECK(e == hipSuccess, "psd subsample2: ", hipGetErrorString(e));
  return y;
}
// ---- BN-backward fold of a 1x1 conv -> BN pair (kernels/bnfold.hip)

namespace {
at::Tensor fold_w2d(const at::Tensor& w) {
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kBFloat16 && (w.dim() == 2 || (w.dim() == 4 && w.size(2) == 1 &&
                                                                                   w.size(3) == 1)),
              "psd bnfold: w must be the bf16 [Cout, Cin(, 1, 1)] weight of a 1x1 convolution");
  return w.reshape({w.size(0), w.size(1)}).contiguous();
}
}  // namespace

// The folded dgrad operands: w2 [Cin, Cout + Cin] bf16 = [(A o W)^T | W^T (B o W)] and the bias
// bvec [Cin] fp32 = C^T W, so dgrad = [g | x] . w2^T + bvec (kernels/convn.hip with x2 = x).
std::vector<at::Tensor> bnfold_dgrad_weights(const at::Tensor& w_in, const at::Tensor& coef) {
  const c10::DeviceGuard dg(w_in.device());
  const at::Tensor w = fold_w2d(w_in);
  const int64_t Cout = w.size(0), Cin = w.size(1);
  TORCH_CHECK(coef.scalar_type() == at::kFloat && coef.is_contiguous() && coef.numel() == 3 * Cout &&
                  coef.device() == w.device(),
              "psd bnfold: coef must be fp32 [3 * Cout]");
  at::Tensor w2 = at::empty({Cin, Cout + Cin}, w.options());
  at::Tensor bw = at::empty({Cout, Cin}, w.options());
  at::Tensor bvec = at::empty({Cin}, w.options().dtype(at::kFloat));
  hipError_t e = launch_bnfold_prep(reinterpret_cast<const uint16_t*>(w.data_ptr()), coef.data_ptr<float>(), (int)Cout,
                                    (int)Cin, reinterpret_cast<uint16_t*>(w2.data_ptr()), (int)(Cout + Cin),
                                    reinterpret_cast<uint16_t*>(bw.data_ptr()), bvec.data_ptr<float>(), stream_of(w));
  TORCH_CHECK(e == hipSuccess, "psd bnfold prep: ", hipGetErrorString(e));
  // M = (B o W)^T W (Cin x Cin, symmetric) into the right block of w2 (the MFMA GEMM, TN layout)
  gemm_(bw, w, false, false, w2.narrow(1, Cout, Cin), c10::nullopt, 0, c10::nullopt, c10::nullopt, c10::nullopt);
  return {w2, bvec};
}

// dW = A o P[:Cout] + B o (W P[Cout:Cout+Cin]) + C P[Cout+Cin] (P = kernels/convw.hip fold output)
// into out (bf16 [Cout, Cin] view, += with accumulate)
void bnfold_combine(const at::Tensor& P, const at::Tensor& w_in, const at::Tensor& coef, at::Tensor out,
                    bool accumulate) {
  const c10::DeviceGuard dg(w_in.device());
  const at::Tensor w = fold_w2d(w_in);
  const int64_t Cout = w.size(0), Cin = w.size(1);
  TORCH_CHECK(P.scalar_type() == at::kFloat && P.is_contiguous() && P.dim() == 2 && P.size(1) == Cin &&
                  P.size(0) > Cout + Cin && P.device() == w.device(),
              "psd bnfold combine: P must be the fp32 convw fold result [rows, Cin]");
  TORCH_CHECK(coef.scalar_type() == at::kFloat && coef.is_contiguous() && coef.numel() == 3 * Cout,
              "psd bnfold combine: coef must be fp32 [3 * Cout]");
  TORCH_CHECK(out.scalar_type() == at::kBFloat16 && out.is_contiguous() && out.numel() == Cout * Cin &&
                  out.device() == w.device(),
              "psd bnfold combine: out must be a contiguous bf16 [Cout, Cin]");
  hipError_t e = launch_bnfold_combine(P.data_ptr<float>(), reinterpret_cast<const uint16_t*>(w.data_ptr()),
                                       coef.data_ptr<float>(), (int)Cout, (int)Cin,
                                       reinterpret_cast<uint16_t*>(out.data_ptr()), accumulate ? 1 : 0, stream_of(w));
  TORCH_CHECK(e == hipSuccess, "psd bnfold combine: ", hipGetErrorString(e));
}

// row [2, Cout] (a view into a partials buffer) = (0, sum_i W[c][i] P[c][i]): the sum g y of a BN
// whose input y = x W^T was never stored (ops/tail.py)
void bnfold_rowdot(const at::Tensor& P, const at::Tensor& w_in, at::Tensor row) {
  const c10::DeviceGuard dg(w_in.device());
  const at::Tensor w = fold_w2d(w_in);
  const int64_t Cout = w.size(0), Cin = w.size(1);
  TORCH_CHECK(P.scalar_type() == at::kFloat && P.is_contiguous() && P.dim() == 2 && P.size(1) == Cin &&
                  P.size(0) >= Cout && P.device() == w.device(),
              "psd bnfold rowdot: P must be the fp32 convw fold result [rows, Cin]");
  TORCH_CHECK(row.scalar_type() == at::kFloat && row.is_contiguous() && row.numel() == 2 * Cout &&
                  row.device() == w.device(),
              "psd bnfold rowdot: row must be a contiguous fp32 [2, Cout]");
  hipError_t e = launch_bnfold_rowdot(P.data_ptr<float>(), reinterpret_cast<const uint16_t*>(w.data_ptr()), (int)Cout,
                                      (int)Cin, row.data_ptr<float>(), stream_of(w));
  TORCH_CHECK(e == hipSuccess, "psd bnfold rowdot: ", hipGetErrorString(e));
}

// row [2, Cout] = the shifted batch statistics of y = x W^T from P = convw(x, x) in fold mode (the
// Gram matrix and column sums of x), without forming y (ops/tail.py)
void bnfold_gram_stats(const at::Tensor& P, const at::Tensor& w_in, const at::Tensor& shift, int64_t M, at::Tensor row) {
  const c10::DeviceGuard dg(w_in.device());
  const at::Tensor w = fold_w2d(w_in);
  const int64_t Cout = w.size(0), Cin = w.size(1);
  TORCH_CHECK(P.scalar_type() == at::kFloat && P.is_contiguous() && P.dim() == 2 && P.size(1) == Cin &&
                  P.size(0) > Cin && P.device() == w.device() && (Cin == 64 || Cin == 128 || Cin == 256) &&
                  Cout % 4 == 0,
              "psd bnfold gram stats: P must be the fp32 convw_gram_ result [rows > Cin, Cin], Cin 64/128/256, "
              "Cout % 4 == 0");
  TORCH_CHECK(shift.scalar_type() == at::kFloat && shift.numel() == Cout && shift.is_contiguous(),
              "psd bnfold gram stats: shift must be fp32 [Cout]");
  TORCH_CHECK(row.scalar_type() == at::kFloat && row.is_contiguous() && row.numel() == 2 * Cout,
              "psd bnfold gram stats: row must be a contiguous fp32 [2, Cout]");
  hipError_t e = launch_bnfold_gram_stats(P.data_ptr<float>(), reinterpret_cast<const uint16_t*>(w.data_ptr()),
                                          shift.data_ptr<float>(), (int)Cout, (int)Cin, M, row.data_ptr<float>(),
                                          stream_of(w));
  TORCH_CHECK(e == hipSuccess, "psd bnfold gram stats: ", hipGetErrorString(e));
}

// The dual tail's apply operands from both convolutions' weights and both BNs' scale/shift
// (kernels/bnfold.hip bnfold_dual_weights_kernel): {wcat [Cout, C3 + Cd] bf16, ss [2 Cout] fp32}
std::vector<at::Tensor> bnfold_dual_weights(const at::Tensor& w3_in, const at::Tensor& wd_in, const at::Tensor& ss3,
                                            const at::Tensor& ssd) {
  const c10::DeviceGuard dg(w3_in.device());
  const at::Tensor w3 = fold_w2d(w3_in), wd = fold_w2d(wd_in);
  const int64_t Cout = w3.size(0), C3 = w3.size(1), Cd = wd.size(1);
  TORCH_CHECK(wd.size(0) == Cout && w3.scalar_type() == at::kBFloat16 && wd.scalar_type() == at::kBFloat16,
              "psd bnfold dual weights: bf16 weights with one Cout");
  for (const at::Tensor* t : {&ss3, &ssd})
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous() && t->numel() == 2 * Cout && t->device() == w3.device(),
                "psd bnfold dual weights: ss must be fp32 [2 Cout]");
  at::Tensor wcat = at::empty({Cout, C3 + Cd}, w3.options());
  at::Tensor ss = at::empty({2 * Cout}, ss3.options());
  hipError_t e = launch_bnfold_dual_weights(reinterpret_cast<const uint16_t*>(w3.data_ptr()),
                                            reinterpret_cast<const uint16_t*>(wd.data_ptr()), ss3.data_ptr<float>(),
                                            ssd.data_ptr<float>(), (int)Cout, (int)C3, (int)Cd,
                                            reinterpret_cast<uint16_t*>(wcat.data_ptr()), ss.data_ptr<float>(),
                                            stream_of(w3));
  TORCH_CHECK(e == hipSuccess, "psd bnfold dual weights: ", hipGetErrorString(e));
  return {wcat, ss};
}

// Training-mode BN statistics from producer partials only (no activation is read): returns
// {mean, invstd, ss [2C]} and updates the running statistics, as bn_fwd with stats_only.
std::vector<at::Tensor> bn_finalize(const at::Tensor& part, int64_t rows, int64_t M, const at::Tensor& gamma,
                                    const at::Tensor& beta, at::Tensor running_mean, at::Tensor running_var,
                                    double momentum, double eps, c10::optional<at::Tensor> counter) {
  const c10::DeviceGuard dg(part.device());
  const int64_t C = running_mean.numel();
  check_vec(gamma, C, at::kBFloat16, "gamma");
  check_vec(beta, C, at::kBFloat16, "beta");
  check_vec(running_mean, C, at::kFloat, "running_mean");
  check_vec(running_var, C, at::kFloat, "running_var");
  TORCH_CHECK(C % 8 == 0 && M > 0 && rows > 0 && part.scalar_type() == at::kFloat && part.is_contiguous() &&
                  part.numel() >= rows * 2 * C && part.device() == running_mean.device(),
              "psd bn_finalize: part must be fp32 [rows, 2, C]");
  auto f32 = part.options();
  at::Tensor mean = at::empty({C}, f32), invstd = at::empty({C}, f32), ss = at::empty({2 * C}, f32);
  at::Tensor fold = rows > kFoldRows ? at::empty({(int64_t)kFoldRows * 2 * C}, f32) : at::Tensor();
  BnFwdArgs a{};
  a.gamma = opt_ptr<const uint16_t>(gamma);
  a.beta = opt_ptr<const uint16_t>(beta);
  a.running_mean = running_mean.data_ptr<float>();
  a.running_var = running_var.data_ptr<float>();
  a.save_mean = mean.data_ptr<float>();
  a.save_invstd = invstd.data_ptr<float>();
  a.ss = ss.data_ptr<float>();
  a.part = part.data_ptr<float>();
  a.part_ready = (int32_t)rows;
  a.fold_ws = fold.defined() ? fold.data_ptr<float>() : nullptr;
  a.counter = opt_ptr<int64_t>(counter);
  a.M = M;
  a.C = (int32_t)C;
  a.training = true;
  a.momentum = (float)momentum;
  a.eps = (float)eps;
  a.stats_only = true;
  const hipError_t e = launch_bn_fwd(a, stream_of(part));
  TORCH_CHECK(e == hipSuccess, "psd bn_finalize: ", hipGetErrorString(e));
  return {mean, invstd, ss};
}

at::Tensor bn_elemt_coef(const at::Tensor& g_in, const at::Tensor& x_in, const at::Tensor& coef) {
  const c10::DeviceGuard dg(x_in.device());
  at::Tensor x = nhwc(x_in), g = nhwc(g_in);
  const int64_t C = channels(x), M = x.numel() / C;
  TORCH_CHECK(g.sizes() == x.sizes() && g.scalar_type() == at::kBFloat16 && x.scalar_type() == at::kBFloat16 &&
                  coef.scalar_type() == at::kFloat && coef.numel() == 3 * C && coef.is_contiguous(),
              "psd bn_elemt_coef: g like x (bf16), coef fp32 [3C]");
  at::Tensor dx = at::empty_like(x);
  const hipError_t e = launch_bn_elemt_coef(reinterpret_cast<const uint16_t*>(g.data_ptr()),
                                            reinterpret_cast<const uint16_t*>(x.data_ptr()), coef.data_ptr<float>(),
                                            reinterpret_cast<uint16_t*>(dx.data_ptr()), M, (int)C, stream_of(x));
  TORCH_CHECK(e == hipSuccess, "psd bn_elemt_coef: ", hipGetErrorString(e));
  return dx;  // empty_like keeps the channels_last layout
}

// Dual tail backward from convn bwd-mode-3 partials: {dx (undefined with fold), dxd, dgamma, dbeta,
// dgamma_d, dbeta_d, coef} (kernels/bn.hip launch_bn_bwd_dual_pre)
std::vector<at::Tensor> bn_bwd_dual_pre(const at::Tensor& g_in, const at::Tensor& x_in, const at::Tensor& gamma,
                                        const at::Tensor& save_mean, const at::Tensor& save_invstd,
                                        const at::Tensor& part, const at::Tensor& part_d, int64_t rows,
                                        const at::Tensor& xd_in, const at::Tensor& gamma_d, const at::Tensor& mean_d,
                                        const at::Tensor& invstd_d, c10::optional<at::Tensor> dgamma_out,
                                        c10::optional<at::Tensor> dbeta_out, c10::optional<at::Tensor> dgamma_d_out,
                                        c10::optional<at::Tensor> dbeta_d_out, bool fold, bool fold_d, bool derive_d) {
  const c10::DeviceGuard dg(x_in.device());
  at::Tensor x = nhwc(x_in), g = nhwc(g_in), xd = nhwc(xd_in);
  const int64_t C = channels(x), M = x.numel() / C;
  TORCH_CHECK(C % 8 == 0 && g.sizes() == x.sizes() && xd.sizes() == x.sizes() && g.scalar_type() == at::kBFloat16 &&
                  x.scalar_type() == at::kBFloat16 && xd.scalar_type() == at::kBFloat16,
              "psd bn_bwd_dual_pre: g / xd like x (bf16)");
  for (const at::Tensor* t : {&save_mean, &save_invstd, &mean_d, &invstd_d})
    TORCH_CHECK(t->numel() == C && t->scalar_type() == at::kFloat && t->is_contiguous(), "psd bn_bwd_dual_pre: stats");
  for (const at::Tensor* t : {&part, &part_d})
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous() && rows > 0 &&
                    t->numel() >= (derive_d && t == &part_d ? 2 : rows * 2) * C,
                "psd bn_bwd_dual_pre: partials must be fp32 [rows, 2, C] (derive_d: part_d [2, C])");
  auto grad_buf = [&](const c10::optional<at::Tensor>& o) {
    at::Tensor t = (o.has_value() && o->defined()) ? *o : at::empty({C}, x.options());
    TORCH_CHECK(t.numel() == C && t.scalar_type() == at::kBFloat16 && t.is_contiguous(), "psd bn_bwd_dual_pre: grad buffer");
    return t;
  };
  at::Tensor dgamma = grad_buf(dgamma_out), dbeta = grad_buf(dbeta_out);
  at::Tensor dgamma_d = grad_buf(dgamma_d_out), dbeta_d = grad_buf(dbeta_d_out);
  auto f32 = x.options().dtype(at::kFloat);
  at::Tensor coef = at::empty({3 * C}, f32), coef_d = at::empty({3 * C}, f32);
  const bool many = rows > kFoldRows;
  at::Tensor fw = many ? at::empty({(int64_t)kFoldRows * 2 * C}, f32) : at::Tensor();
  at::Tensor fwd = many && !derive_d ? at::empty({(int64_t)kFoldRows * 2 * C}, f32) : at::Tensor();
  // fold / fold_d: the BN input gradient of bn3 / of the downsample BN is folded into its
  // convolution's backward (ops/conv.py _fold_backward): not written here
  TORCH_CHECK(!fold_d || fold, "psd bn_bwd_dual_pre: fold_d needs fold");
  at::Tensor dx = fold ? at::Tensor() : at::empty_like(x), dxd = fold_d ? at::Tensor() : at::empty_like(x);
  BnDualPreArgs a{};
  a.g = reinterpret_cast<const uint16_t*>(g.data_ptr());
  a.x = reinterpret_cast<const uint16_t*>(x.data_ptr());
  a.xd = reinterpret_cast<const uint16_t*>(xd.data_ptr());
  a.gamma = reinterpret_cast<const uint16_t*>(gamma.data_ptr());
  a.gamma_d = reinterpret_cast<const uint16_t*>(gamma_d.data_ptr());
  a.mean = save_mean.data_ptr<float>();
  a.invstd = save_invstd.data_ptr<float>();
  a.mean_d = mean_d.data_ptr<float>();
  a.invstd_d = invstd_d.data_ptr<float>();
  a.part = part.data_ptr<float>();
  a.part_d = part_d.data_ptr<float>();
  a.rows = (int)rows;
  a.fold_ws = many ? fw.data_ptr<float>() : nullptr;
  a.fold_ws_d = many && !derive_d ? fwd.data_ptr<float>() : nullptr;
  a.derive_d = derive_d ? 1 : 0;
  a.dgamma = reinterpret_cast<uint16_t*>(dgamma.data_ptr());
  a.dbeta = reinterpret_cast<uint16_t*>(dbeta.data_ptr());
  a.dgamma_d = reinterpret_cast<uint16_t*>(dgamma_d.data_ptr());
  a.dbeta_d = reinterpret_cast<uint16_t*>(dbeta_d.data_ptr());
  a.coef = coef.data_ptr<float>();
  a.coef_d = coef_d.data_ptr<float>();
  a.dx = fold ? nullptr : reinterpret_cast<uint16_t*>(dx.data_ptr());
  a.dxd = fold_d ? nullptr : reinterpret_cast<uint16_t*>(dxd.data_ptr());
  a.M = M;
  a.C = (int)C;
  const hipError_t e = launch_bn_bwd_dual_pre(a, stream_of(x));
  TORCH_CHECK(e == hipSuccess, "psd bn_bwd_dual_pre: ", hipGetErrorString(e));
  return {dx, dxd, dgamma, dbeta, dgamma_d, dbeta_d, coef, coef_d};
}

}  // namespace psd
