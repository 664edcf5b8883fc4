// Tensor-level entry points for the gfx950 kernels, with bit-compatible CPU implementations for the
// host-memory PS mode (reference parity: the reference PS keeps fp32 params in host memory,
// include/parameter_server.h:9-14) and for CPU-only CI.
//
// Device tensors dispatch to the HIP launchers on the caller's current HIP stream; nothing here
// allocates device memory on the apply path, so the calls are legal under hipGraph capture.
#include "ops.h"

#include <ATen/Parallel.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>

#include <cmath>
#include <cstring>

#include "kernels/launchers.h"
#include "kernels/launchers_xfer.h"

namespace psd {

namespace {

inline hipStream_t cur_stream(const at::Tensor& t) {
  return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

inline void hip_check(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, "psd: ", what, " failed: ", hipGetErrorString(e));
}

inline int32_t dt_of(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return DT_F32;
    case at::kBFloat16: return DT_BF16;
    case at::kFloat8_e4m3fn: return DT_F8E4M3;
    default: TORCH_CHECK(false, "psd: unsupported dtype ", t.scalar_type());
  }
}

inline void check_aligned(const at::Tensor& t, const char* name) {
  TORCH_CHECK((reinterpret_cast<uintptr_t>(t.data_ptr()) & 15u) == 0, "psd: ", name,
              " must be 16-byte aligned (flat buffers are carved at 8-element granularity)");
}

inline float bf16f(uint16_t h) {
  uint32_t u = ((uint32_t)h) << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}
inline uint16_t f2bf(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// Scalar optimizer step: identical operation order to the device kernel (optim.hip).
inline void cpu_update(const OptimHyper& h, float lr, float bc1, float bc2s, bool first, float& p, float g,
                       float& s1, float& s2) {
  if (h.maximize) g = -g;
  switch (h.kind) {
    case OPT_SGD:
      if (h.weight_decay != 0.f) g = std::fma(h.weight_decay, p, g);
      p = std::fma(-lr, g, p);
      break;
    case OPT_MOMENTUM: {
      if (h.weight_decay != 0.f) g = std::fma(h.weight_decay, p, g);
      float buf = first ? g : std::fma(h.momentum, s1, (1.f - h.dampening) * g);
      s1 = buf;
      float d = h.nesterov ? std::fma(h.momentum, buf, g) : buf;
      p = std::fma(-lr, d, p);
      break;
    }
    default: {
      if (h.kind == OPT_ADAMW) p = p * (1.f - lr * h.weight_decay);
      else if (h.weight_decay != 0.f) g = std::fma(h.weight_decay, p, g);
      float m = std::fma(h.beta1, s1, (1.f - h.beta1) * g);
      float v = std::fma(h.beta2, s2, (1.f - h.beta2) * g * g);
      s1 = m;
      s2 = v;
      float denom = std::sqrt(v) / bc2s + h.eps;
      p = p - (lr / bc1) * (m / denom);
    }
  }
}

OptimDyn* dyn_ptr(const at::Tensor& dyn) {
  TORCH_CHECK(dyn.scalar_type() == at::kInt && dyn.numel() == 8 && dyn.is_contiguous(),
              "psd: dyn must be a contiguous int32[8] tensor (OptimDyn)");
  return reinterpret_cast<OptimDyn*>(dyn.data_ptr());
}

SourceList make_sources(const std::vector<at::Tensor>& srcs, int64_t n, const at::Device& dev) {
  TORCH_CHECK(!srcs.empty() && (int)srcs.size() <= kMaxSources, "psd: 1..16 gradient sources required");
  SourceList s{};
  s.count = (int32_t)srcs.size();
  s.dtype = dt_of(srcs[0]);
  for (size_t k = 0; k < srcs.size(); ++k) {
    TORCH_CHECK(srcs[k].device() == dev, "psd: gradient source on wrong device");
    TORCH_CHECK(dt_of(srcs[k]) == s.dtype, "psd: gradient sources must share a dtype");
    TORCH_CHECK(srcs[k].is_contiguous() && srcs[k].numel() == n, "psd: gradient source shape mismatch");
    s.ptr[k] = srcs[k].data_ptr();
  }
  return s;
}

}  // namespace

void fused_apply_(at::Tensor master, const std::vector<at::Tensor>& grads, c10::optional<at::Tensor> state1,
                  c10::optional<at::Tensor> state2, c10::optional<at::Tensor> shadow, at::Tensor dyn, int64_t kind,
                  double momentum, double dampening, bool nesterov, double weight_decay, double beta1, double beta2,
                  double eps, bool maximize, int64_t grid_cap) {
  TORCH_CHECK(master.scalar_type() == at::kFloat && master.is_contiguous(), "psd: master must be contiguous fp32");
  const int64_t n = master.numel();
  OptimHyper h{};
  h.kind = (int32_t)kind;
  h.nesterov = nesterov;
  h.maximize = maximize;
  h.momentum = (float)momentum;
  h.dampening = (float)dampening;
  h.weight_decay = (float)weight_decay;
  h.beta1 = (float)beta1;
  h.beta2 = (float)beta2;
  h.eps = (float)eps;
  const bool need1 = kind != OPT_SGD, need2 = kind == OPT_ADAM || kind == OPT_ADAMW;
  float* s1 = nullptr;
  float* s2 = nullptr;
  if (need1) {
    TORCH_CHECK(state1.has_value() && state1->numel() == n && state1->scalar_type() == at::kFloat &&
                    state1->is_contiguous() && state1->device() == master.device(),
                "psd: optimizer needs fp32 state1 like master");
    s1 = state1->data_ptr<float>();
  }
  if (need2) {
    TORCH_CHECK(state2.has_value() && state2->numel() == n && state2->scalar_type() == at::kFloat &&
                    state2->is_contiguous() && state2->device() == master.device(),
                "psd: optimizer needs fp32 state2 like master");
    s2 = state2->data_ptr<float>();
  }
  uint16_t* sh = nullptr;
  if (shadow.has_value() && shadow->defined()) {
    TORCH_CHECK(shadow->scalar_type() == at::kBFloat16 && shadow->numel() == n && shadow->is_contiguous() &&
                    shadow->device() == master.device(),
                "psd: shadow must be contiguous bf16 like master");
    sh = reinterpret_cast<uint16_t*>(shadow->data_ptr());
  }
  SourceList src = make_sources(grads, n, master.device());
  TORCH_CHECK(dyn.device() == master.device(), "psd: dyn must live with master");

  if (master.is_cuda()) {
    const c10::DeviceGuard g(master.device());
    check_aligned(master, "master");
    if (s1) check_aligned(*state1, "state1");
    if (s2) check_aligned(*state2, "state2");
    if (sh) check_aligned(*shadow, "shadow");
    for (auto& t : grads) check_aligned(t, "grad");
    hip_check(launch_fused_apply(h, dyn_ptr(dyn), master.data_ptr<float>(), src, s1, s2, sh, n, cur_stream(master),
                                 (int)grid_cap),
              "fused_apply");
    return;
  }
  const OptimDyn d = *dyn_ptr(dyn);
  const float lr = d.lr, gs = d.grad_scale, bc1 = d.bc1, bc2s = std::sqrt(d.bc2);
  const bool first = d.step <= 1;
  float* p = master.data_ptr<float>();
  at::parallel_for(0, n, 1 << 14, [&](int64_t b, int64_t e) {
    for (int64_t i = b; i < e; ++i) {
      float g = 0.f;
      for (int k = 0; k < src.count; ++k)
        g += src.dtype == DT_BF16 ? bf16f(static_cast<const uint16_t*>(src.ptr[k])[i])
                                  : static_cast<const float*>(src.ptr[k])[i];
      g *= gs;
      float a = s1 ? s1[i] : 0.f, c = s2 ? s2[i] : 0.f;
      cpu_update(h, lr, bc1, bc2s, first, p[i], g, a, c);
      if (s1) s1[i] = a;
      if (s2) s2[i] = c;
      if (sh) sh[i] = f2bf(p[i]);
    }
  });
}

void optim_advance_(at::Tensor dyn, double beta1, double beta2) {
  OptimDyn* d = dyn_ptr(dyn);
  if (dyn.is_cuda()) {
    const c10::DeviceGuard g(dyn.device());
    hip_check(launch_optim_advance(d, (float)beta1, (float)beta2, cur_stream(dyn)), "optim_advance");
    return;
  }
  d->step += 1;
  d->bc1 = 1.f - std::pow((float)beta1, (float)d->step);
  d->bc2 = 1.f - std::pow((float)beta2, (float)d->step);
}

void multi_reduce_(at::Tensor out, const std::vector<at::Tensor>& srcs, double scale) {
  TORCH_CHECK(out.is_contiguous(), "psd: out must be contiguous");
  const int64_t n = out.numel();
  SourceList s = make_sources(srcs, n, out.device());
  const int32_t od = dt_of(out);
  TORCH_CHECK(od == DT_F32 || od == DT_BF16, "psd: reduce output must be fp32/bf16");
  if (out.is_cuda()) {
    const c10::DeviceGuard g(out.device());
    check_aligned(out, "out");
    for (auto& t : srcs) check_aligned(t, "src");
    hip_check(launch_multi_reduce(s, out.data_ptr(), od, (float)scale, n, cur_stream(out)), "multi_reduce");
    return;
  }
  at::parallel_for(0, n, 1 << 14, [&](int64_t b, int64_t e) {
    for (int64_t i = b; i < e; ++i) {
      float acc = 0.f;
      for (int k = 0; k < s.count; ++k)
        acc += s.dtype == DT_BF16 ? bf16f(static_cast<const uint16_t*>(s.ptr[k])[i])
                                  : static_cast<const float*>(s.ptr[k])[i];
      acc *= (float)scale;
      if (od == DT_BF16) static_cast<uint16_t*>(out.data_ptr())[i] = f2bf(acc);
      else static_cast<float*>(out.data_ptr())[i] = acc;
    }
  });
}

void xfer_(const std::vector<at::Tensor>& srcs, const std::vector<at::Tensor>& dsts, int64_t blocks_per_seg,
           bool nt_store) {
  TORCH_CHECK(srcs.size() == dsts.size() && !srcs.empty() && (int)srcs.size() <= kMaxXferSeg, "psd: xfer_ segments");
  XferList L{};
  for (size_t i = 0; i < srcs.size(); ++i) {
    const at::Tensor &a = srcs[i], &b = dsts[i];
    TORCH_CHECK(a.is_cuda() && b.is_cuda() && a.is_contiguous() && b.is_contiguous() && a.nbytes() == b.nbytes(),
                "psd: xfer_ takes contiguous device tensors of equal byte size");
    check_aligned(a, "xfer_ src");
    check_aligned(b, "xfer_ dst");
    L.seg[L.count++] = XferSeg{a.data_ptr(), b.data_ptr(), (int64_t)a.nbytes()};
  }
  L.blocks_per_seg = (int32_t)blocks_per_seg;
  L.nt_store = nt_store ? 1 : 0;
  const c10::DeviceGuard g(srcs[0].device());
  hip_check(launch_xfer(L, cur_stream(srcs[0])), "launch_xfer");
}

void pack_cast_(const std::vector<at::Tensor>& srcs, const std::vector<at::Tensor>& dsts) {
  TORCH_CHECK(srcs.size() == dsts.size(), "psd: pack_cast needs matching src/dst lists");
  if (srcs.empty()) return;
  const int32_t sd = dt_of(srcs[0]), dd = dt_of(dsts[0]);
  const auto dev = srcs[0].device();
  for (size_t i = 0; i < srcs.size(); ++i) {
    TORCH_CHECK(dt_of(srcs[i]) == sd && dt_of(dsts[i]) == dd, "psd: pack_cast dtypes must be uniform");
    TORCH_CHECK(srcs[i].numel() == dsts[i].numel(), "psd: pack_cast numel mismatch at ", i);
    TORCH_CHECK(srcs[i].is_contiguous() && dsts[i].is_contiguous(), "psd: pack_cast needs contiguous tensors");
    TORCH_CHECK(srcs[i].device() == dev && dsts[i].device() == dev, "psd: pack_cast device mismatch");
  }
  if (dev.is_cuda()) {
    constexpr int64_t kChunk = 8192;
    std::vector<PackSeg> segs(srcs.size());
    std::vector<int32_t> cseg;
    std::vector<int64_t> coff;
    for (size_t i = 0; i < srcs.size(); ++i) {
      segs[i] = PackSeg{srcs[i].data_ptr(), dsts[i].data_ptr(), srcs[i].numel()};
      for (int64_t o = 0; o < srcs[i].numel(); o += kChunk) {
        cseg.push_back((int32_t)i);
        coff.push_back(o);
      }
    }
    if (cseg.empty()) return;
    // one host staging tensor -> one H2D copy for the whole table
    const int64_t seg_bytes = (int64_t)(segs.size() * sizeof(PackSeg));
    const int64_t off_bytes = (int64_t)(coff.size() * sizeof(int64_t));
    const int64_t cs_bytes = (int64_t)(cseg.size() * sizeof(int32_t));
    const int64_t total = seg_bytes + off_bytes + cs_bytes;
    auto host = at::empty({total}, at::TensorOptions().dtype(at::kByte).pinned_memory(true));
    uint8_t* hp = host.data_ptr<uint8_t>();
    std::memcpy(hp, segs.data(), seg_bytes);
    std::memcpy(hp + seg_bytes, coff.data(), off_bytes);
    std::memcpy(hp + seg_bytes + off_bytes, cseg.data(), cs_bytes);
    const c10::DeviceGuard g(dev);
    auto table = at::empty({total}, at::TensorOptions().dtype(at::kByte).device(dev));
    table.copy_(host, /*non_blocking=*/true);
    uint8_t* tp = table.data_ptr<uint8_t>();
    hip_check(launch_pack_cast(reinterpret_cast<const PackSeg*>(tp), reinterpret_cast<const int32_t*>(tp + seg_bytes + off_bytes),
                               reinterpret_cast<const int64_t*>(tp + seg_bytes), (int64_t)cseg.size(), sd, dd,
                               cur_stream(srcs[0])),
              "pack_cast");
    return;
  }
  for (size_t t = 0; t < srcs.size(); ++t) {
    const int64_t n = srcs[t].numel();
    const void* sp = srcs[t].data_ptr();
    void* dp = dsts[t].data_ptr();
    at::parallel_for(0, n, 1 << 15, [&](int64_t b, int64_t e) {
      for (int64_t i = b; i < e; ++i) {
        float x = sd == DT_BF16 ? bf16f(static_cast<const uint16_t*>(sp)[i]) : static_cast<const float*>(sp)[i];
        if (dd == DT_BF16) static_cast<uint16_t*>(dp)[i] = f2bf(x);
        else static_cast<float*>(dp)[i] = x;
      }
    });
  }
}

void amax_(const at::Tensor& x, at::Tensor amax_out) {
  TORCH_CHECK(amax_out.scalar_type() == at::kFloat && amax_out.numel() >= 1, "psd: amax_out must be fp32[>=1]");
  TORCH_CHECK(x.is_contiguous(), "psd: amax input must be contiguous");
  if (x.is_cuda()) {
    const c10::DeviceGuard g(x.device());
    if (x.numel() >= 8) check_aligned(x, "x");  // 16-byte vector loads
    hip_check(launch_amax(x.data_ptr(), dt_of(x), x.numel(), amax_out.data_ptr<float>(), cur_stream(x)), "amax");
    return;
  }
  float m = amax_out.data_ptr<float>()[0];
  auto xf = x.to(at::kFloat);
  const float* p = xf.data_ptr<float>();
  for (int64_t i = 0; i < xf.numel(); ++i) m = std::max(m, std::fabs(p[i]));
  amax_out.data_ptr<float>()[0] = m;
}

void quant_fp8_(const at::Tensor& x, const at::Tensor& amax, double fp8_max, at::Tensor out, at::Tensor scale_inv) {
  const bool e5 = out.scalar_type() == at::kFloat8_e5m2;
  TORCH_CHECK((out.scalar_type() == at::kFloat8_e4m3fn || e5) && out.numel() == x.numel() && out.is_contiguous(),
              "psd: quant_fp8 out must be float8_e4m3fn or float8_e5m2 like x");
  TORCH_CHECK(x.is_contiguous(), "psd: quant_fp8 input must be contiguous");
  if (x.is_cuda()) {
    const c10::DeviceGuard g(x.device());
    if (x.numel() >= 8) {
      check_aligned(x, "x");
      TORCH_CHECK((reinterpret_cast<uintptr_t>(out.data_ptr()) & 7u) == 0, "psd: fp8 out must be 8-byte aligned");
    }
    hip_check(launch_quant_fp8(x.data_ptr(), dt_of(x), x.numel(), amax.data_ptr<float>(), (float)fp8_max,
                               reinterpret_cast<uint8_t*>(out.data_ptr()), scale_inv.data_ptr<float>(), cur_stream(x),
                               e5 ? 1 : 0),
              "quant_fp8");
    return;
  }
  const float a = std::max(amax.data_ptr<float>()[0], 1e-12f);
  const float scale = (float)fp8_max / a;
  scale_inv.data_ptr<float>()[0] = a / (float)fp8_max;
  out.copy_((x.to(at::kFloat) * scale).clamp(-fp8_max, fp8_max).to(out.scalar_type()));
}

// out = fp8(x * fp8_max / amax(x)), scale_inv = amax / fp8_max: amax found on the device in the same
// call (out e4m3fn or e5m2; fp8_max follows the format)
void quant_fp8_jit_(const at::Tensor& x, at::Tensor out, at::Tensor scale_inv) {
  const bool e5 = out.scalar_type() == at::kFloat8_e5m2;
  TORCH_CHECK((out.scalar_type() == at::kFloat8_e4m3fn || e5) && out.numel() == x.numel() && out.is_contiguous(),
              "psd: quant_fp8_jit out must be float8_e4m3fn or float8_e5m2 like x");
  TORCH_CHECK(x.is_contiguous() && x.is_cuda(), "psd: quant_fp8_jit input must be a contiguous device tensor");
  TORCH_CHECK(scale_inv.scalar_type() == at::kFloat && scale_inv.numel() >= 1, "psd: scale_inv fp32[>=1]");
  const c10::DeviceGuard g(x.device());
  if (x.numel() >= 8) {
    check_aligned(x, "x");
    TORCH_CHECK((reinterpret_cast<uintptr_t>(out.data_ptr()) & 7u) == 0, "psd: fp8 out must be 8-byte aligned");
  }
  at::Tensor part = at::empty({1024}, x.options().dtype(at::kFloat));
  hip_check(launch_quant_fp8_jit(x.data_ptr(), dt_of(x), x.numel(), part.data_ptr<float>(), e5 ? 57344.f : 448.f,
                                 reinterpret_cast<uint8_t*>(out.data_ptr()), scale_inv.data_ptr<float>(), cur_stream(x),
                                 e5 ? 1 : 0),
            "quant_fp8_jit");
}

// delayed scaling: out = fp8(x * fp8_max / (hist[0] * margin)); this call's amax -> hist[0] afterwards
void quant_fp8_delayed_(const at::Tensor& x, at::Tensor out, at::Tensor scale_inv, at::Tensor hist, double margin) {
  const bool e5 = out.scalar_type() == at::kFloat8_e5m2;
  TORCH_CHECK((out.scalar_type() == at::kFloat8_e4m3fn || e5) && out.numel() == x.numel() && out.is_contiguous(),
              "psd: quant_fp8_delayed out must be float8_e4m3fn or float8_e5m2 like x");
  TORCH_CHECK(x.is_contiguous() && x.is_cuda(), "psd: quant_fp8_delayed input must be a contiguous device tensor");
  TORCH_CHECK(scale_inv.scalar_type() == at::kFloat && scale_inv.numel() >= 1 && hist.scalar_type() == at::kFloat &&
                  hist.numel() >= 2 && hist.is_cuda() && hist.is_contiguous(),
              "psd: scale_inv fp32[>=1], hist fp32[2] device tensors");
  const c10::DeviceGuard g(x.device());
  if (x.numel() >= 8) {
    check_aligned(x, "x");
    TORCH_CHECK((reinterpret_cast<uintptr_t>(out.data_ptr()) & 7u) == 0, "psd: fp8 out must be 8-byte aligned");
  }
  hip_check(launch_quant_fp8_delayed(x.data_ptr(), dt_of(x), x.numel(), hist.data_ptr<float>(), e5 ? 57344.f : 448.f,
                                     (float)margin, reinterpret_cast<uint8_t*>(out.data_ptr()),
                                     scale_inv.data_ptr<float>(), cur_stream(x), e5 ? 1 : 0),
            "quant_fp8_delayed");
}

void dequant_fp8_(const at::Tensor& x, const at::Tensor& scale_inv, at::Tensor out) {
  TORCH_CHECK(x.scalar_type() == at::kFloat8_e4m3fn && out.numel() == x.numel(), "psd: dequant_fp8 shape/dtype");
  if (x.is_cuda()) {
    const c10::DeviceGuard g(x.device());
    hip_check(launch_dequant_fp8(reinterpret_cast<const uint8_t*>(x.data_ptr()), x.numel(), scale_inv.data_ptr<float>(),
                                 out.data_ptr(), dt_of(out), cur_stream(x)),
              "dequant_fp8");
    return;
  }
  out.copy_(x.to(at::kFloat) * scale_inv.data_ptr<float>()[0]);
}

// MX fp8: out = fp8(x / 2^(s - 127)) with one E8M0 byte s per 32 consecutive elements (scales)
void quant_mx_(const at::Tensor& x, at::Tensor out, at::Tensor scales) {
  const bool e5 = out.scalar_type() == at::kFloat8_e5m2;
  TORCH_CHECK((out.scalar_type() == at::kFloat8_e4m3fn || e5) && out.numel() == x.numel() && out.is_contiguous(),
              "psd: quant_mx out must be float8_e4m3fn or float8_e5m2 like x");
  TORCH_CHECK(x.is_contiguous() && x.is_cuda() && x.numel() % 32 == 0,
              "psd: quant_mx input must be a contiguous device tensor of a multiple of 32 elements");
  TORCH_CHECK(scales.scalar_type() == at::kByte && scales.is_contiguous() && scales.numel() == x.numel() / 32,
              "psd: quant_mx scales must be uint8 [numel / 32]");
  const c10::DeviceGuard g(x.device());
  if (x.numel() == 0) return;
  check_aligned(x, "x");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(out.data_ptr()) & 7u) == 0, "psd: fp8 out must be 8-byte aligned");
  hip_check(launch_quant_mx(x.data_ptr(), dt_of(x), x.numel(), e5 ? 1 : 0, reinterpret_cast<uint8_t*>(out.data_ptr()),
                            scales.data_ptr<uint8_t>(), cur_stream(x)),
            "quant_mx");
}

void dequant_mx_(const at::Tensor& q, const at::Tensor& scales, at::Tensor out) {
  TORCH_CHECK(q.scalar_type() == at::kFloat8_e4m3fn && q.is_contiguous() && q.is_cuda() && out.numel() == q.numel() &&
                  out.is_contiguous() && q.numel() % 32 == 0,
              "psd: dequant_mx q must be a contiguous e4m3fn device tensor (numel % 32 == 0), out like q");
  TORCH_CHECK(scales.scalar_type() == at::kByte && scales.is_contiguous() && scales.numel() == q.numel() / 32,
              "psd: dequant_mx scales must be uint8 [numel / 32]");
  const c10::DeviceGuard g(q.device());
  if (q.numel() == 0) return;
  TORCH_CHECK((reinterpret_cast<uintptr_t>(q.data_ptr()) & 7u) == 0, "psd: fp8 q must be 8-byte aligned");
  check_aligned(out, "out");
  hip_check(launch_dequant_mx(reinterpret_cast<const uint8_t*>(q.data_ptr()), scales.data_ptr<uint8_t>(), q.numel(),
                              out.data_ptr(), dt_of(out), cur_stream(q)),
            "dequant_mx");
}

}  // namespace psd
