// Tensor glue for the MFMA GEMM (kernels/gemm.hip).
#include <ATen/ATen.h>

#include <algorithm>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>

#include "kernels/launchers_convn.h"
#include "kernels/launchers_convw.h"
#include "kernels/launchers_gemm.h"

namespace psd {

namespace {
inline hipStream_t stream_of(const at::Tensor& t) { return c10::hip::getCurrentHIPStream(t.device().index()).stream(); }
void chk2d(const at::Tensor& t, const char* n) {
  TORCH_CHECK(t.is_cuda() && t.dim() == 2 && t.scalar_type() == at::kBFloat16 && t.stride(1) == 1 &&
                  t.stride(0) % 8 == 0 && (reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0,
              "psd gemm: ", n, " must be a 2-D bf16 device tensor, unit inner stride, 16-B aligned rows");
}
}  // namespace

int64_t gemm_stats_rows_(int64_t M) { return (M + 127) / 128 * 2; }

// the consumer BN's statistics partials in the 8-phase epilogue: part fp32 >= gemm_stats_rows(M) x 2 x N,
// shift fp32 [N] (the BN's running mean)
static void set_stats(GemmArgs& a, const c10::optional<at::Tensor>& part, const c10::optional<at::Tensor>& shift,
                      const at::Tensor& out, int* rows) {
  if (!part.has_value() || !part->defined()) return;
  const int64_t M = out.size(0), N = out.size(1);
  TORCH_CHECK(part->scalar_type() == at::kFloat && part->is_contiguous() && part->device() == out.device() &&
                  part->numel() >= gemm_stats_rows_(M) * 2 * N,
              "psd gemm: part must be fp32 contiguous with >= gemm_stats_rows(M) x 2 x N elements");
  TORCH_CHECK(shift.has_value() && shift->defined() && shift->scalar_type() == at::kFloat && shift->is_contiguous() &&
                  shift->numel() == N && shift->device() == out.device(),
              "psd gemm: statistics need shift fp32 [N]");
  TORCH_CHECK(out.scalar_type() == at::kBFloat16, "psd gemm: statistics need a bf16 output");
  a.part = part->data_ptr<float>();
  a.shift = shift->data_ptr<float>();
  a.rows_out = rows;
}

// out[M,N] = A op B (+bias)(act). A: a_kmajor ? [M,K] : [K,M]; B: b_kmajor ? [N,K] : [K,N]. With
// part/shift also the consumer BN's statistics partials: returns the partial rows written, 0 when the
// shape cannot carry them (nothing launched); 1 without statistics.
int64_t gemm_(const at::Tensor& A, const at::Tensor& B, bool a_kmajor, bool b_kmajor, at::Tensor out,
              c10::optional<at::Tensor> bias, int64_t act, c10::optional<at::Tensor> aux,
              c10::optional<at::Tensor> part, c10::optional<at::Tensor> shift) {
  chk2d(A, "A");
  chk2d(B, "B");
  const int64_t M = a_kmajor ? A.size(0) : A.size(1), K = a_kmajor ? A.size(1) : A.size(0);
  const int64_t N = b_kmajor ? B.size(0) : B.size(1), K2 = b_kmajor ? B.size(1) : B.size(0);
  TORCH_CHECK(K == K2, "psd gemm: K mismatch ", K, " vs ", K2);
  TORCH_CHECK(out.dim() == 2 && out.size(0) == M && out.size(1) == N && out.stride(1) == 1, "psd gemm: out shape");
  TORCH_CHECK(out.scalar_type() == at::kBFloat16 || out.scalar_type() == at::kFloat, "psd gemm: out dtype");
  TORCH_CHECK(K % 8 == 0 || !(a_kmajor && b_kmajor), "psd gemm: K must be a multiple of 8 for K-major operands");
  TORCH_CHECK(a_kmajor || M % 8 == 0, "psd gemm: M must be a multiple of 8 for an M-major A");
  TORCH_CHECK(b_kmajor || N % 8 == 0, "psd gemm: N must be a multiple of 8 for an N-major B");
  TORCH_CHECK(!(a_kmajor ^ b_kmajor) || K % 8 == 0, "psd gemm: K must be a multiple of 8");
  const c10::DeviceGuard g(A.device());
  GemmArgs a{};
  a.A = A.data_ptr();
  a.B = B.data_ptr();
  a.C = out.data_ptr();
  a.bias = (bias.has_value() && bias->defined()) ? bias->data_ptr() : nullptr;
  if (a.bias) TORCH_CHECK(bias->numel() == N && bias->scalar_type() == at::kBFloat16, "psd gemm: bias [N] bf16");
  a.aux = (aux.has_value() && aux->defined()) ? aux->data_ptr() : nullptr;
  a.M = (int)M;
  a.N = (int)N;
  a.K = (int)K;
  a.lda = (int)A.stride(0);
  a.ldb = (int)B.stride(0);
  a.ldc = (int)out.stride(0);
  a.a_kmajor = a_kmajor;
  a.b_kmajor = b_kmajor;
  a.act = (int)act;
  a.c_f32 = out.scalar_type() == at::kFloat;
  int rows = 0;
  set_stats(a, part, shift, out, &rows);
  hipError_t e = launch_gemm(a, stream_of(A));
  if (a.part && e == hipErrorNotSupported) return 0;
  TORCH_CHECK(e == hipSuccess, "psd gemm: ", hipGetErrorString(e));
  return a.part ? rows : 1;
}

bool gemm_ct_(const at::Tensor& A, const at::Tensor& B, at::Tensor out, c10::optional<at::Tensor> bias, int64_t act,
              c10::optional<at::Tensor> aux) {
  chk2d(A, "A");
  chk2d(B, "B");
  const int64_t M = A.size(0), K = A.size(1), N = B.size(0);
  TORCH_CHECK(B.size(1) == K, "psd gemm_ct: K mismatch ", K, " vs ", B.size(1));
  TORCH_CHECK(out.dim() == 2 && out.size(0) == N && out.size(1) == M && out.stride(1) == 1 &&
                  (out.scalar_type() == at::kBFloat16 || out.scalar_type() == at::kFloat),
              "psd gemm_ct: out must be [N, M] bf16 / fp32 with unit inner stride");
  TORCH_CHECK(act >= 0 && act <= 2, "psd gemm_ct: act 0-2");
  const bool has_aux = aux.has_value() && aux->defined();
  if (has_aux)
    TORCH_CHECK(aux->sizes() == out.sizes() && aux->strides() == out.strides() && aux->scalar_type() == at::kBFloat16,
                "psd gemm_ct: aux like out (bf16)");
  const bool has_bias = bias.has_value() && bias->defined();
  if (has_bias) TORCH_CHECK(bias->numel() == M && bias->scalar_type() == at::kBFloat16, "psd gemm_ct: bias [M] bf16");
  const c10::DeviceGuard g(A.device());
  GemmArgs a{};
  a.A = A.data_ptr();
  a.B = B.data_ptr();
  a.C = out.data_ptr();
  a.bias = has_bias ? bias->data_ptr() : nullptr;
  a.aux = has_aux ? aux->data_ptr() : nullptr;
  a.M = (int)M;
  a.N = (int)N;
  a.K = (int)K;
  a.lda = (int)A.stride(0);
  a.ldb = (int)B.stride(0);
  a.ldc = (int)out.stride(0);
  a.a_kmajor = 1;
  a.b_kmajor = 1;
  a.act = (int)act;
  a.c_f32 = out.scalar_type() == at::kFloat;
  hipError_t e = launch_gemm_ct(a, stream_of(A));
  if (e == hipErrorNotSupported) return false;
  TORCH_CHECK(e == hipSuccess, "psd gemm_ct: ", hipGetErrorString(e));
  return true;
}

// GELU-backward GEMM: out[M,N] = bf16(bf16(A op B) * gelu'(pre)) with the bias gradient
// db[N] (+)= colsum(out) from the epilogue's per-tile partials (kernels/gemm.hip ACT 3): the
// gradient of a GELU Linear's output computed by the next Linear's bwd-data GEMM goes straight to
// the pre-activation gradient. False (nothing launched) when the shape is not on the 8-phase kernel.
bool gemm_gelu_bwd_(const at::Tensor& A, const at::Tensor& B, bool a_kmajor, bool b_kmajor, const at::Tensor& pre,
                    at::Tensor out, at::Tensor db, bool accumulate) {
  chk2d(A, "A");
  chk2d(B, "B");
  chk2d(pre, "pre");
  const int64_t M = a_kmajor ? A.size(0) : A.size(1), K = a_kmajor ? A.size(1) : A.size(0);
  const int64_t N = b_kmajor ? B.size(0) : B.size(1), K2 = b_kmajor ? B.size(1) : B.size(0);
  TORCH_CHECK(K == K2, "psd gemm_gelu_bwd: K mismatch ", K, " vs ", K2);
  TORCH_CHECK(out.scalar_type() == at::kBFloat16 && out.is_contiguous() && out.dim() == 2 && out.size(0) == M &&
                  out.size(1) == N && pre.is_contiguous() && pre.sizes() == out.sizes(),
              "psd gemm_gelu_bwd: out and pre must be contiguous bf16 [M, N]");
  TORCH_CHECK(db.numel() == N && db.is_contiguous() &&
                  (db.scalar_type() == at::kBFloat16 || db.scalar_type() == at::kFloat),
              "psd gemm_gelu_bwd: db must be [N] bf16/fp32");
  if (N % 8 != 0 || K % 8 != 0 || (!a_kmajor && M % 8 != 0)) return false;
  const c10::DeviceGuard g(A.device());
  at::Tensor part = at::empty({gemm_stats_rows_(M) * N}, A.options().dtype(at::kFloat));
  GemmArgs a{};
  a.A = A.data_ptr();
  a.B = B.data_ptr();
  a.C = out.data_ptr();
  a.aux = const_cast<void*>(pre.data_ptr());
  a.M = (int)M;
  a.N = (int)N;
  a.K = (int)K;
  a.lda = (int)A.stride(0);
  a.ldb = (int)B.stride(0);
  a.ldc = (int)N;
  a.a_kmajor = a_kmajor;
  a.b_kmajor = b_kmajor;
  a.act = 3;
  a.part = part.data_ptr<float>();
  int rows = 0;
  a.rows_out = &rows;
  hipError_t e = launch_gemm(a, stream_of(A));
  if (e == hipErrorNotSupported) return false;
  TORCH_CHECK(e == hipSuccess, "psd gemm_gelu_bwd: ", hipGetErrorString(e));
  TORCH_CHECK(rows > 0 && rows <= gemm_stats_rows_(M), "psd gemm_gelu_bwd: partial rows ", rows);
  e = launch_colsum_final(part.data_ptr<float>(), rows, (int)N, db.data_ptr(), db.scalar_type() == at::kBFloat16,
                          accumulate, stream_of(A));
  TORCH_CHECK(e == hipSuccess, "psd gemm_gelu_bwd colsum: ", hipGetErrorString(e));
  return true;
}

// out[M,N] (+)= scale * (A op B) via split-K fp32 slabs (weight gradients: K = tokens).
void gemm_splitk_(const at::Tensor& A, const at::Tensor& B, bool a_kmajor, bool b_kmajor, at::Tensor out,
                  bool accumulate, double scale, int64_t splits) {
  chk2d(A, "A");
  chk2d(B, "B");
  const int64_t M = a_kmajor ? A.size(0) : A.size(1), K = a_kmajor ? A.size(1) : A.size(0);
  const int64_t N = b_kmajor ? B.size(0) : B.size(1), K2 = b_kmajor ? B.size(1) : B.size(0);
  TORCH_CHECK(K == K2, "psd gemm_splitk: K mismatch");
  TORCH_CHECK(out.is_contiguous() && out.numel() == M * N, "psd gemm_splitk: out must be contiguous [M,N]");
  TORCH_CHECK(a_kmajor || M % 8 == 0, "psd gemm_splitk: M % 8");
  TORCH_CHECK(b_kmajor || N % 8 == 0, "psd gemm_splitk: N % 8");
  const c10::DeviceGuard g(A.device());
  const int s = splits > 0 ? (int)splits : gemm_splits((int)M, (int)N, (int)K);
  if (s == 1 && !accumulate && scale == 1.0) {
    // one split (enough output tiles to fill the chip, e.g. the BERT MLM head's weight gradient:
    // 120 x 3 256-tiles): the single-split GEMM writes the output itself -- no fp32 slab
    // (94 MB written and read back there) and no reduce launch
    GemmArgs a{};
    a.A = A.data_ptr();
    a.B = B.data_ptr();
    a.C = out.data_ptr();
    a.M = (int)M;
    a.N = (int)N;
    a.K = (int)K;
    a.lda = (int)A.stride(0);
    a.ldb = (int)B.stride(0);
    a.ldc = (int)N;
    a.a_kmajor = a_kmajor;
    a.b_kmajor = b_kmajor;
    a.c_f32 = out.scalar_type() == at::kFloat;
    const hipError_t e = launch_gemm(a, stream_of(A));
    TORCH_CHECK(e == hipSuccess, "psd gemm_splitk (single split): ", hipGetErrorString(e));
    return;
  }
  at::Tensor slab = at::empty({(int64_t)s * M * N}, A.options().dtype(at::kFloat));
  GemmArgs a{};
  a.A = A.data_ptr();
  a.B = B.data_ptr();
  a.M = (int)M;
  a.N = (int)N;
  a.K = (int)K;
  a.lda = (int)A.stride(0);
  a.ldb = (int)B.stride(0);
  a.ldc = (int)N;
  a.a_kmajor = a_kmajor;
  a.b_kmajor = b_kmajor;
  hipError_t e = launch_gemm_splitk(a, slab.data_ptr<float>(), s, out.data_ptr(), out.scalar_type() == at::kBFloat16,
                                    accumulate, (float)scale, stream_of(A));
  TORCH_CHECK(e == hipSuccess, "psd gemm_splitk: ", hipGetErrorString(e));
}

// out[M,N] = (A_q . B_q^T) * a_scale * b_scale (+bias)(act): A [M,K], B [N,K] OCP e4m3fn, K % 128 == 0
int64_t gemm_fp8_(const at::Tensor& A, const at::Tensor& B, const at::Tensor& a_scale, const at::Tensor& b_scale,
                  at::Tensor out, c10::optional<at::Tensor> bias, int64_t act, c10::optional<at::Tensor> aux,
                  c10::optional<at::Tensor> part, c10::optional<at::Tensor> shift) {
  for (const at::Tensor* t : {&A, &B})
    TORCH_CHECK(t->is_cuda() && t->dim() == 2 && t->stride(1) == 1 && t->stride(0) % 16 == 0 &&
                    (reinterpret_cast<uintptr_t>(t->data_ptr()) & 15) == 0,
                "psd gemm_fp8: operands must be 2-D fp8 device tensors, unit inner stride, 16-B aligned rows");
  TORCH_CHECK((A.scalar_type() == at::kFloat8_e4m3fn || A.scalar_type() == at::kFloat8_e5m2) &&
                  B.scalar_type() == at::kFloat8_e4m3fn,
              "psd gemm_fp8: A e4m3fn or e5m2, B e4m3fn");
  const int64_t M = A.size(0), K = A.size(1), N = B.size(0);
  TORCH_CHECK(B.size(1) == K, "psd gemm_fp8: K mismatch");
  TORCH_CHECK(K % 128 == 0, "psd gemm_fp8: K must be a multiple of 128");
  // per-tensor (fp32 device scalars) or MX (uint8 E8M0 per 32 contiguous K: A [M, K/32], B [N, K/32])
  const bool mx = a_scale.scalar_type() == at::kByte;
  if (mx) {
    TORCH_CHECK(b_scale.scalar_type() == at::kByte && a_scale.is_cuda() && b_scale.is_cuda() &&
                    a_scale.is_contiguous() && b_scale.is_contiguous() && a_scale.numel() == M * (K / 32) &&
                    b_scale.numel() == N * (K / 32) && A.stride(0) == K && B.stride(0) == K,
                "psd gemm_fp8: MX scales must be uint8 [M, K/32] / [N, K/32] (contiguous operands)");
  } else {
    TORCH_CHECK(a_scale.scalar_type() == at::kFloat && b_scale.scalar_type() == at::kFloat && a_scale.numel() >= 1 &&
                    b_scale.numel() >= 1 && a_scale.is_cuda() && b_scale.is_cuda(),
                "psd gemm_fp8: scales must be fp32 device scalars (or MX uint8 block scales)");
  }
  TORCH_CHECK(out.dim() == 2 && out.size(0) == M && out.size(1) == N && out.stride(1) == 1, "psd gemm_fp8: out shape");
  TORCH_CHECK(out.scalar_type() == at::kBFloat16 || out.scalar_type() == at::kFloat, "psd gemm_fp8: out dtype");
  const c10::DeviceGuard g(A.device());
  GemmArgs a{};
  a.A = A.data_ptr();
  a.B = B.data_ptr();
  a.C = out.data_ptr();
  a.bias = (bias.has_value() && bias->defined()) ? bias->data_ptr() : nullptr;
  if (a.bias) TORCH_CHECK(bias->numel() == N && bias->scalar_type() == at::kBFloat16, "psd gemm_fp8: bias [N] bf16");
  a.aux = (aux.has_value() && aux->defined()) ? aux->data_ptr() : nullptr;
  a.M = (int)M;
  a.N = (int)N;
  a.K = (int)K;
  a.lda = (int)A.stride(0);
  a.ldb = (int)B.stride(0);
  a.ldc = (int)out.stride(0);
  a.a_kmajor = a.b_kmajor = 1;
  a.act = (int)act;
  a.c_f32 = out.scalar_type() == at::kFloat;
  if (mx) {
    a.a_mx = a_scale.data_ptr<uint8_t>();
    a.b_mx = b_scale.data_ptr<uint8_t>();
  } else {
    a.a_scale = a_scale.data_ptr<float>();
    a.b_scale = b_scale.data_ptr<float>();
  }
  a.f8a = A.scalar_type() == at::kFloat8_e5m2 ? 1 : 0;
  int rows = 0;
  set_stats(a, part, shift, out, &rows);
  hipError_t e = launch_gemm_fp8(a, stream_of(A));
  if (a.part && e == hipErrorNotSupported) return 0;
  TORCH_CHECK(e == hipSuccess, "psd gemm_fp8: ", hipGetErrorString(e));
  return a.part ? rows : 1;
}

// Implicit-GEMM NHWC convolution forward on the persistent 8-phase MFMA kernel (no bias/activation):
// x [Nb, C, H, W] channels_last, w2 [Cout, R*S*C] ((r, s, ci) order, i.e. an OHWI weight viewed
// 2-D), out [Nb*Ho*Wo, Cout] bf16 (an NHWC output's 2-D view). bf16 operands, or OCP e4m3 ones with
// per-tensor dequant scales (xs, ws: fp32 device scalars). Returns false (nothing launched) when the
// shape is outside the kernel's contract -- the caller falls back.
static int64_t conv_fwd_impl(const at::Tensor& x, const at::Tensor& w2, at::Tensor out, int64_t R, int64_t S,
                             int64_t stride, int64_t pad, const at::Tensor* xs, const at::Tensor* ws,
                             const c10::optional<at::Tensor>& part, const c10::optional<at::Tensor>& shift) {
  const bool f8 = xs != nullptr;
  const auto dt = f8 ? at::kFloat8_e4m3fn : at::kBFloat16;
  const bool x_e5 = f8 && x.scalar_type() == at::kFloat8_e5m2;  // bwd-data: e5m2 dY
  const int esz = f8 ? 1 : 2;
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 && (x.scalar_type() == dt || x_e5) &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "psd conv_fwd: x must be a channels_last ", f8 ? "e4m3fn / e5m2" : "bf16", " device tensor");
  TORCH_CHECK(w2.is_cuda() && w2.dim() == 2 && w2.scalar_type() == dt && w2.stride(1) == 1 &&
                  (w2.stride(0) * esz) % 16 == 0 && (reinterpret_cast<uintptr_t>(w2.data_ptr()) & 15) == 0,
              "psd conv_fwd: w2 must be a 2-D device tensor like x, unit inner stride, 16-B aligned rows");
  TORCH_CHECK(out.dim() == 2 && out.stride(1) == 1 && out.scalar_type() == at::kBFloat16, "psd conv_fwd: out");
  const bool mx = f8 && xs->scalar_type() == at::kByte;  // MX: E8M0 per 32 channels of x, per 32 K of w2
  if (mx) {
    TORCH_CHECK(ws->scalar_type() == at::kByte && xs->is_cuda() && ws->is_cuda() && xs->is_contiguous() &&
                    ws->is_contiguous() && xs->numel() == x.numel() / 32 && ws->numel() == w2.numel() / 32 &&
                    w2.stride(0) == w2.size(1),
                "psd conv_fwd_fp8: MX scales must be uint8 [pixels, C/32] / [Cout, K/32] (contiguous w2)");
  } else if (f8) {
    TORCH_CHECK(xs->scalar_type() == at::kFloat && ws->scalar_type() == at::kFloat && xs->is_cuda() && ws->is_cuda() &&
                    xs->numel() >= 1 && ws->numel() >= 1,
                "psd conv_fwd_fp8: scales must be fp32 device scalars (or MX uint8 block scales)");
  }
  const int64_t Nb = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int64_t Ho = (H + 2 * pad - R) / stride + 1, Wo = (W + 2 * pad - S) / stride + 1;
  const int64_t M = Nb * Ho * Wo, Cout = w2.size(0), K = R * S * C;
  TORCH_CHECK(w2.size(1) == K, "psd conv_fwd: w2 must be [Cout, R*S*C]");
  TORCH_CHECK(out.size(0) == M && out.size(1) == Cout, "psd conv_fwd: out must be [Nb*Ho*Wo, Cout]");
  const int64_t xbytes = x.numel() * esz;
  if ((C & (C - 1)) != 0 || C < (f8 ? 128 : 64) || xbytes >= ((int64_t)1 << 32) || M >= ((int64_t)1 << 31))
    return 0;
  int logc = 0;
  while ((1 << logc) < C) ++logc;
  const c10::DeviceGuard g(x.device());
  GemmArgs a{};
  a.A = x.data_ptr();
  a.B = w2.data_ptr();
  a.C = out.data_ptr();
  a.M = (int)M;
  a.N = (int)Cout;
  a.K = (int)K;
  a.lda = (int)K;
  a.ldb = (int)w2.stride(0);
  a.ldc = (int)out.stride(0);
  a.a_kmajor = a.b_kmajor = 1;
  a.cv_H = (int)H;
  a.cv_W = (int)W;
  a.cv_logC = logc;
  a.cv_Ho = (int)Ho;
  a.cv_Wo = (int)Wo;
  a.cv_S = (int)S;
  a.cv_stride = (int)stride;
  a.cv_pad = (int)pad;
  a.cv_abytes = (uint32_t)xbytes;
  if (mx) {
    a.a_mx = xs->data_ptr<uint8_t>();
    a.b_mx = ws->data_ptr<uint8_t>();
    a.f8a = x_e5 ? 1 : 0;
  } else if (f8) {
    a.a_scale = xs->data_ptr<float>();
    a.b_scale = ws->data_ptr<float>();
    a.f8a = x_e5 ? 1 : 0;
  }
  int rows = 0;
  set_stats(a, part, shift, out, &rows);
  hipError_t e = f8 ? launch_conv_fwd_fp8(a, stream_of(x)) : launch_conv_fwd(a, stream_of(x));
  if (e == hipErrorNotSupported) return 0;
  TORCH_CHECK(e == hipSuccess, "psd conv_fwd: ", hipGetErrorString(e));
  return a.part ? rows : 1;
}

int64_t convn_stats_rows_(int64_t M) { return convn_stats_rows((int)M); }
// partial rows a launch of this variant writes (allocate at least this many: HALO variants tile by rows)
int64_t convn_part_rows_(int64_t M, int64_t N, int64_t v, int64_t Ho, int64_t Wo, int64_t R) {
  return convn_part_rows_geo((int)M, (int)N, (int)v, (int)Ho, (int)Wo, (int)R);
}
bool convn_variant_ok_(int64_t N, int64_t v, int64_t R, int64_t S, int64_t stride, int64_t pad, int64_t Wo,
                       bool has_x2) {
  return convn_variant_ok((int)N, (int)v, (int)R, (int)S, (int)stride, (int)pad, (int)Wo, has_x2);
}
int64_t convn_variants_(int64_t N) { return convn_variants((int)N); }
int64_t convn_variant_kind_(int64_t N, int64_t v) { return convn_variant_kind((int)N, (int)v); }

namespace {
// K-concatenated second operand + epilogue bias of a convn launch (the BN-backward fold); returns the
// extra K (C2) or -1 when x2 is unusable. x2: channels_last bf16 [Nb, C2, H, W] like the input.
int64_t convn_x2(ConvnArgs& a, const at::Tensor& x, c10::optional<at::Tensor> x2, c10::optional<at::Tensor> bias,
                 int64_t N) {
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->numel() == N && bias->is_contiguous() &&
                    bias->device() == x.device(),
                "psd convn: bias must be fp32 [N] on the input's device");
    a.bias = bias->data_ptr<float>();
  }
  if (!(x2.has_value() && x2->defined())) return 0;
  TORCH_CHECK(x2->is_cuda() && x2->dim() == 4 && x2->scalar_type() == at::kBFloat16 &&
                  x2->is_contiguous(at::MemoryFormat::ChannelsLast) && x2->device() == x.device() &&
                  x2->size(0) == x.size(0) && x2->size(2) == x.size(2) && x2->size(3) == x.size(3),
              "psd convn: x2 must be a channels_last bf16 tensor with the input's N, H, W");
  const int64_t C2 = x2->size(1), bytes = x2->numel() * 2;
  if (C2 < 64 || (C2 & (C2 - 1)) != 0 || bytes > 0xFFFFFF00ll) return -1;
  int l = 0;
  while ((1 << l) < C2) ++l;
  a.x2 = x2->data_ptr();
  a.x2bytes = (uint32_t)bytes;
  a.logC2 = l;
  return C2;
}
}  // namespace

int64_t convn_(const at::Tensor& x, const at::Tensor& w2, at::Tensor out, int64_t R, int64_t S, int64_t stride,
               int64_t pad, c10::optional<at::Tensor> part, c10::optional<at::Tensor> shift, int64_t variant,
               c10::optional<at::Tensor> x2, c10::optional<at::Tensor> bias, bool no_store,
               c10::optional<at::Tensor> apply_ss, c10::optional<at::Tensor> apply_res,
               c10::optional<at::Tensor> apply_mask) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 && x.scalar_type() == at::kBFloat16 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "psd convn: x must be a channels_last bf16 device tensor");
  TORCH_CHECK(w2.is_cuda() && w2.dim() == 2 && w2.scalar_type() == at::kBFloat16 && w2.is_contiguous(),
              "psd convn: w2 must be a contiguous bf16 [Cout, R*S*C] device tensor");
  TORCH_CHECK(no_store || (out.is_cuda() && out.dim() == 2 && out.stride(1) == 1 && out.scalar_type() == at::kBFloat16 &&
                           (reinterpret_cast<uintptr_t>(out.data_ptr()) & 15) == 0),
              "psd convn: out must be a bf16 [M, Cout] device tensor, 16-B aligned");
  const bool apply = apply_ss.has_value() && apply_ss->defined();
  const int64_t Nb = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int64_t Ho = (H + 2 * pad - R) / stride + 1, Wo = (W + 2 * pad - S) / stride + 1;
  const int64_t M = Nb * Ho * Wo, Cout = w2.size(0), K1 = R * S * C;
  ConvnArgs a{};
  const int64_t C2 = convn_x2(a, x, x2, bias, Cout);
  if (C2 < 0) return 0;
  const int64_t K = K1 + C2;
  TORCH_CHECK(w2.size(1) == K, "psd convn: w2 must be [Cout, R*S*C (+ C2)]");
  TORCH_CHECK(no_store || (out.size(0) == M && out.size(1) == Cout), "psd convn: out must be [Nb*Ho*Wo, Cout]");
  const bool stats = part.has_value() && part->defined();
  TORCH_CHECK(!no_store || (stats && !apply), "psd convn: no_store is a statistics-only pass");
  if (apply) {
    TORCH_CHECK(!stats && apply_ss->scalar_type() == at::kFloat && apply_ss->numel() == 2 * Cout &&
                    apply_ss->is_contiguous() && apply_ss->device() == x.device(),
                "psd convn: apply_ss must be fp32 [2 Cout] (no statistics in an apply pass)");
    TORCH_CHECK(!(apply_res.has_value() && apply_res->defined()) ||
                    (apply_res->scalar_type() == at::kBFloat16 && apply_res->numel() == M * Cout &&
                     apply_res->device() == x.device() &&
                     (apply_res->dim() == 4 ? apply_res->is_contiguous(at::MemoryFormat::ChannelsLast)
                                            : apply_res->is_contiguous())),
                "psd convn: apply_res must be a bf16 [M, Cout] (or channels_last) residual, or None");
    TORCH_CHECK(apply_mask.has_value() && apply_mask->defined() && apply_mask->scalar_type() == at::kByte &&
                    apply_mask->numel() == M * Cout / 8 && apply_mask->is_contiguous(),
                "psd convn: apply_mask must be uint8 [M * Cout / 8]");
    TORCH_CHECK(out.stride(0) == Cout, "psd convn: the apply pass writes a dense [M, Cout] output");
  }
  if (stats) {
    TORCH_CHECK(shift.has_value() && shift->defined() && shift->numel() == Cout && shift->scalar_type() == at::kFloat &&
                    shift->is_contiguous() && shift->device() == x.device(),
                "psd convn: statistics need an fp32 [Cout] shift on x's device");
    TORCH_CHECK(part->scalar_type() == at::kFloat && part->is_contiguous() && part->device() == x.device() &&
                    part->numel() >= (int64_t)std::max(convn_stats_rows((int)M),
                                                       convn_part_rows_geo((int)M, (int)Cout,
                                                                           (int)std::max<int64_t>(variant, 0), (int)Ho,
                                                                           (int)Wo, (int)R)) * 2 * Cout,
                "psd convn: part must be fp32 [convn_part_rows(...), 2, Cout]");
  }
  const int64_t xbytes = x.numel() * 2, wbytes = w2.numel() * 2;
  if ((C & (C - 1)) != 0 || C < 64 || xbytes > 0xFFFFFF00ll || wbytes >= ((int64_t)1 << 32) ||
      M >= ((int64_t)1 << 31) - 256 || convn_tile_n((int)Cout) == 0 || (!no_store && out.stride(0) % 8 != 0) ||
      Ho <= 0 || Wo <= 0 || variant >= convn_variants((int)Cout))
    return 0;
  int logc = 0;
  while ((1 << logc) < C) ++logc;
  const c10::DeviceGuard g(x.device());
  a.K1 = (int)K1;
  a.x = x.data_ptr();
  a.w = w2.data_ptr();
  a.y = no_store ? nullptr : out.data_ptr();
  a.part = stats ? part->data_ptr<float>() : nullptr;
  a.shift = stats ? shift->data_ptr<float>() : nullptr;
  if (apply) {
    a.bwd = 8;
    a.bss = apply_ss->data_ptr<float>();
    a.ares = (apply_res.has_value() && apply_res->defined()) ? reinterpret_cast<const uint16_t*>(apply_res->data_ptr())
                                                             : nullptr;
    a.amask = apply_mask->data_ptr<uint8_t>();
  }
  a.xbytes = (uint32_t)xbytes;
  a.wbytes = (uint32_t)wbytes;
  a.M = (int)M;
  a.N = (int)Cout;
  a.K = (int)K;
  a.H = (int)H;
  a.W = (int)W;
  a.logC = logc;
  a.Ho = (int)Ho;
  a.Wo = (int)Wo;
  a.R = (int)R;
  a.S = (int)S;
  a.stride = (int)stride;
  a.pad = (int)pad;
  a.ldc = no_store ? (int)Cout : (int)out.stride(0);
  a.variant = (int)variant;
  const hipError_t e = launch_convn(a, c10::hip::getCurrentHIPStream(x.device().index()).stream());
  if (e == hipErrorNotSupported) return 0;
  TORCH_CHECK(e == hipSuccess, "psd convn: ", hipGetErrorString(e));
  return stats ? convn_part_rows_geo((int)M, (int)Cout, (int)std::max<int64_t>(variant, 0), (int)Ho, (int)Wo, (int)R)
               : 1;
}

// Stride-2 3x3 (pad 1) bwd-data as four phase launches of the gathered narrow kernel: output parity
// class (ph, pw) of dX[2i + ph][2j + pw] gathers dY rows {i, i + 1}^ph x columns {j, j + 1}^pw, i.e. a
// stride-1 / pad-0 convolution of dY with a (1 + ph) x (1 + pw) tap subset of the weights
// (wph[k], k = ph << 1 | pw, bf16 [Ci, (1 + ph)(1 + pw) Co], ordered (dr, ds, co): ops/conv.py
// _dgrad_s2_phases), written at its own pixels of the full-size dX (convn.hip ophase). 9 taps in
// all -- the forward's MACs, no zero-insertion, no zero-fill of dX (every pixel is in one class).
// Optional mode-1 epilogue (the producing BN + ReLU's backward reduction, bx = its input at dX's
// resolution): the four launches' partial rows are written one after another into part. Returns the
// partial rows written (1 without part), 0 when the kernel declines (nothing launched).
int64_t convn_dgrad_s2_(const at::Tensor& dy, const std::vector<at::Tensor>& wph, at::Tensor out, int64_t variant,
                        c10::optional<at::Tensor> part, c10::optional<at::Tensor> bx, c10::optional<at::Tensor> bmean,
                        c10::optional<at::Tensor> bss) {
  TORCH_CHECK(dy.is_cuda() && dy.dim() == 4 && dy.scalar_type() == at::kBFloat16 &&
                  dy.is_contiguous(at::MemoryFormat::ChannelsLast),
              "psd convn_dgrad_s2: dy must be a channels_last bf16 device tensor");
  TORCH_CHECK(wph.size() == 4, "psd convn_dgrad_s2: four phase weights");
  const int64_t Nb = dy.size(0), Co = dy.size(1), Ho = dy.size(2), Wo = dy.size(3);
  const int64_t Ci = wph[0].size(0), M = Nb * Ho * Wo;
  for (int k = 0; k < 4; ++k) {
    const int64_t taps = (1 + (k >> 1)) * (1 + (k & 1));
    TORCH_CHECK(wph[k].is_cuda() && wph[k].dim() == 2 && wph[k].scalar_type() == at::kBFloat16 &&
                    wph[k].is_contiguous() && wph[k].size(0) == Ci && wph[k].size(1) == taps * Co &&
                    wph[k].device() == dy.device(),
                "psd convn_dgrad_s2: wph[k] must be a contiguous bf16 [Ci, taps * Co] tensor");
  }
  TORCH_CHECK(out.dim() == 2 && out.is_contiguous() && out.scalar_type() == at::kBFloat16 && out.size(0) == 4 * M &&
                  out.size(1) == Ci && out.device() == dy.device(),
              "psd convn_dgrad_s2: out must be a contiguous bf16 [Nb * 2Ho * 2Wo, Ci] tensor");
  const bool fused = part.has_value() && part->defined();
  int64_t per = 0;
  if (fused) {
    TORCH_CHECK(bx.has_value() && bx->defined() && bx->scalar_type() == at::kBFloat16 && bx->numel() == 4 * M * Ci &&
                    bx->device() == dy.device() &&
                    (bx->dim() == 4 ? bx->is_contiguous(at::MemoryFormat::ChannelsLast) : bx->is_contiguous()),
                "psd convn_dgrad_s2: bx must be the BN input, bf16 like dX");
    TORCH_CHECK(bmean.has_value() && bmean->defined() && bmean->scalar_type() == at::kFloat && bmean->numel() == Ci &&
                    bmean->is_contiguous() && bss.has_value() && bss->defined() && bss->scalar_type() == at::kFloat &&
                    bss->numel() == 2 * Ci && bss->is_contiguous(),
                "psd convn_dgrad_s2: mode 1 needs the BN's fp32 mean [Ci] and scale/shift [2 Ci]");
    per = std::max(convn_stats_rows((int)M), convn_part_rows_geo((int)M, (int)Ci, (int)std::max<int64_t>(variant, 0),
                                                                  (int)Ho, (int)Wo, 2));
    TORCH_CHECK(part->scalar_type() == at::kFloat && part->is_contiguous() && part->device() == dy.device() &&
                    part->numel() >= 4 * per * 2 * Ci,
                "psd convn_dgrad_s2: part must be fp32 [4 * convn_dgrad_s2_rows(...), 2, Ci]");
  }
  const int64_t xbytes = dy.numel() * 2;
  if ((Co & (Co - 1)) != 0 || Co < 64 || xbytes > 0xFFFFFF00ll || convn_tile_n((int)Ci) == 0 || Ci % 8 != 0 ||
      variant < 0 || variant >= convn_variants((int)Ci) || convn_variant_kind((int)Ci, (int)variant) != 0 ||
      M >= (1 << 24))
    return 0;
  int logc = 0;
  while ((1 << logc) < Co) ++logc;
  const c10::DeviceGuard g(dy.device());
  const hipStream_t st = c10::hip::getCurrentHIPStream(dy.device().index()).stream();
  int64_t rows = 0;
  for (int k = 0; k < 4; ++k) {
    const int R = 1 + (k >> 1), S = 1 + (k & 1);
    ConvnArgs a{};
    a.K1 = R * S * (int)Co;
    a.x = dy.data_ptr();
    a.w = wph[k].data_ptr();
    a.y = out.data_ptr();
    a.xbytes = (uint32_t)xbytes;
    a.wbytes = (uint32_t)(wph[k].numel() * 2);
    a.M = (int)M;
    a.N = (int)Ci;
    a.K = a.K1;
    a.H = (int)Ho;
    a.W = (int)Wo;
    a.logC = logc;
    a.Ho = (int)Ho;
    a.Wo = (int)Wo;
    a.R = R;
    a.S = S;
    a.stride = 1;
    a.pad = 0;
    a.ldc = (int)Ci;
    a.variant = (int)variant;
    a.ophase = 1 + k;
    if (fused) {
      a.bwd = 1;
      a.part = part->data_ptr<float>() + rows * 2 * Ci;
      a.bx = reinterpret_cast<const uint16_t*>(bx->data_ptr());
      a.bmean = bmean->data_ptr<float>();
      a.bss = bss->data_ptr<float>();
    }
    const hipError_t e = launch_convn(a, st);
    if (e == hipErrorNotSupported) {
      TORCH_CHECK(k == 0, "psd convn_dgrad_s2: phase ", k, " declined after phase 0 ran");
      return 0;
    }
    TORCH_CHECK(e == hipSuccess, "psd convn_dgrad_s2: ", hipGetErrorString(e));
    if (fused) rows += convn_part_rows_geo((int)M, (int)Ci, (int)variant, (int)Ho, (int)Wo, R);
  }
  return fused ? rows : 1;
}

// partial rows to allocate for convn_dgrad_s2_ (all four phases) with this variant
int64_t convn_dgrad_s2_rows(int64_t Nb, int64_t Ho, int64_t Wo, int64_t Ci, int64_t variant) {
  const int M = (int)(Nb * Ho * Wo);
  return 4 * (int64_t)std::max(convn_stats_rows(M), convn_part_rows_geo(M, (int)Ci, (int)std::max<int64_t>(variant, 0),
                                                                         (int)Ho, (int)Wo, 2));
}

// bwd-data on the narrow kernel with the producing BN's backward reduction in the epilogue
// (kernels/convn.hip bwd modes): out = g = mask (conv(dy, w2) [+ dr]); part gets the partials.
// Returns the partial rows written, 0 when the kernel declines (nothing launched).
int64_t convn_bwd_(const at::Tensor& dy, const at::Tensor& w2, at::Tensor out, int64_t R, int64_t S, int64_t stride,
                   int64_t pad, at::Tensor part, int64_t variant, int64_t mode, c10::optional<at::Tensor> bx,
                   const at::Tensor& bmean, c10::optional<at::Tensor> bss, c10::optional<at::Tensor> bdr,
                   c10::optional<at::Tensor> bmbits, c10::optional<at::Tensor> x2, c10::optional<at::Tensor> bias,
                   c10::optional<at::Tensor> bxd, c10::optional<at::Tensor> bmean_d, c10::optional<at::Tensor> part_d) {
  TORCH_CHECK(dy.is_cuda() && dy.dim() == 4 && dy.scalar_type() == at::kBFloat16 &&
                  dy.is_contiguous(at::MemoryFormat::ChannelsLast),
              "psd convn_bwd: dy must be a channels_last bf16 device tensor");
  TORCH_CHECK(w2.is_cuda() && w2.dim() == 2 && w2.scalar_type() == at::kBFloat16 && w2.is_contiguous(),
              "psd convn_bwd: w2 must be a contiguous bf16 [N, R*S*C] tensor");
  TORCH_CHECK(out.dim() == 2 && out.is_contiguous() && out.scalar_type() == at::kBFloat16, "psd convn_bwd: out");
  TORCH_CHECK(mode == 1 || mode == 2 || mode == 3 || mode == 5,
              "psd convn_bwd: mode 1 (mask from x, ss), 2 (bit-mask + dr), 3 (2 + the dual tail's second BN) or 5 "
              "(2 with dr on the stride-2 quarter grid)");
  const int64_t Nb = dy.size(0), C = dy.size(1), H = dy.size(2), W = dy.size(3);
  const int64_t Ho = (H + 2 * pad - R) / stride + 1, Wo = (W + 2 * pad - S) / stride + 1;
  const int64_t M = Nb * Ho * Wo, N = w2.size(0), K1 = R * S * C;
  ConvnArgs a{};
  const int64_t C2 = convn_x2(a, dy, x2, bias, N);
  if (C2 < 0) return 0;
  const int64_t K = K1 + C2;
  TORCH_CHECK(w2.size(1) == K && out.size(0) == M && out.size(1) == N, "psd convn_bwd: shapes");
  auto like_out = [&](const at::Tensor& t, const char* what) {
    const at::Tensor u = t.dim() == 4 ? t.permute({0, 2, 3, 1}) : t;
    TORCH_CHECK(t.scalar_type() == at::kBFloat16 && t.numel() == M * N && t.device() == dy.device() &&
                    (t.dim() == 4 ? t.is_contiguous(at::MemoryFormat::ChannelsLast) : t.is_contiguous()),
                "psd convn_bwd: ", what, " must be a contiguous bf16 [M, N] (or channels_last) tensor");
    (void)u;
  };
  const bool has_bx = bx.has_value() && bx->defined();
  TORCH_CHECK(has_bx || mode == 2 || mode == 5, "psd convn_bwd: only modes 2 and 5 run without the BN input bx");
  if (has_bx) like_out(*bx, "bx");
  TORCH_CHECK(bmean.scalar_type() == at::kFloat && bmean.numel() == N && bmean.is_contiguous(), "psd convn_bwd: bmean");
  TORCH_CHECK(part.scalar_type() == at::kFloat && part.is_contiguous() &&
                  part.numel() >= (int64_t)std::max(convn_stats_rows((int)M),
                                                    convn_part_rows_geo((int)M, (int)N, (int)std::max<int64_t>(variant, 0),
                                                                        (int)Ho, (int)Wo, (int)R)) * 2 * N,
              "psd convn_bwd: part must be fp32 [convn_part_rows(...), 2, N]");
  if (mode == 1) {
    TORCH_CHECK(bss.has_value() && bss->defined() && bss->numel() == 2 * N && bss->scalar_type() == at::kFloat &&
                    bss->is_contiguous(),
                "psd convn_bwd: mode 1 needs ss fp32 [2N]");
  } else {
    if (mode == 3) {
      TORCH_CHECK(bxd.has_value() && bxd->defined() && bmean_d.has_value() && bmean_d->defined() &&
                      part_d.has_value() && part_d->defined(),
                  "psd convn_bwd: mode 3 needs bxd, bmean_d and part_d");
      like_out(*bxd, "bxd");
      TORCH_CHECK(bmean_d->scalar_type() == at::kFloat && bmean_d->numel() == N && bmean_d->is_contiguous(),
                  "psd convn_bwd: bmean_d");
      TORCH_CHECK(part_d->scalar_type() == at::kFloat && part_d->is_contiguous() && part_d->numel() >= part.numel(),
                  "psd convn_bwd: part_d like part");
    }
    TORCH_CHECK(bdr.has_value() && bdr->defined(), "psd convn_bwd: mode 2 needs dr");
    if (mode == 5) {
      TORCH_CHECK(bdr->scalar_type() == at::kBFloat16 && bdr->dim() == 4 && bdr->size(0) == Nb && bdr->size(1) == N &&
                      bdr->size(2) * 2 == Ho && bdr->size(3) * 2 == Wo &&
                      bdr->is_contiguous(at::MemoryFormat::ChannelsLast) && bdr->device() == dy.device(),
                  "psd convn_bwd: mode 5 dr must be channels_last bf16 [Nb, N, Ho/2, Wo/2]");
    } else {
      like_out(*bdr, "dr");
    }
    TORCH_CHECK(bmbits.has_value() && bmbits->defined() && bmbits->scalar_type() == at::kByte &&
                    bmbits->numel() == M * N / 8 && bmbits->is_contiguous(),
                "psd convn_bwd: mode 2 needs the uint8 [M*N/8] bit-mask");
  }
  const int64_t xbytes = dy.numel() * 2, wbytes = w2.numel() * 2;
  if ((C & (C - 1)) != 0 || C < 64 || xbytes > 0xFFFFFF00ll || wbytes >= ((int64_t)1 << 32) ||
      M >= ((int64_t)1 << 31) - 256 || convn_tile_n((int)N) == 0 || variant >= convn_variants((int)N) || N % 8 != 0)
    return 0;
  int logc = 0;
  while ((1 << logc) < C) ++logc;
  const c10::DeviceGuard g(dy.device());
  a.K1 = (int)K1;
  a.x = dy.data_ptr();
  a.w = w2.data_ptr();
  a.y = out.data_ptr();
  a.part = part.data_ptr<float>();
  a.xbytes = (uint32_t)xbytes;
  a.wbytes = (uint32_t)wbytes;
  a.M = (int)M;
  a.N = (int)N;
  a.K = (int)K;
  a.H = (int)H;
  a.W = (int)W;
  a.logC = logc;
  a.Ho = (int)Ho;
  a.Wo = (int)Wo;
  a.R = (int)R;
  a.S = (int)S;
  a.stride = (int)stride;
  a.pad = (int)pad;
  a.ldc = (int)N;
  a.variant = (int)variant;
  a.bwd = (int)mode;
  a.bx = has_bx ? reinterpret_cast<const uint16_t*>(bx->data_ptr()) : nullptr;
  a.bmean = bmean.data_ptr<float>();
  a.bss = mode == 1 ? bss->data_ptr<float>() : nullptr;
  a.bdr = mode >= 2 ? reinterpret_cast<const uint16_t*>(bdr->data_ptr()) : nullptr;
  a.bmbits = mode >= 2 ? bmbits->data_ptr<uint8_t>() : nullptr;
  if (mode == 3) {
    a.bxd = reinterpret_cast<const uint16_t*>(bxd->data_ptr());
    a.bmean_d = bmean_d->data_ptr<float>();
    a.part_d = part_d->data_ptr<float>();
  }
  const hipError_t e = launch_convn(a, c10::hip::getCurrentHIPStream(dy.device().index()).stream());
  if (e == hipErrorNotSupported) return 0;
  TORCH_CHECK(e == hipSuccess, "psd convn_bwd: ", hipGetErrorString(e));
  return convn_part_rows_geo((int)M, (int)N, (int)std::max<int64_t>(variant, 0), (int)Ho, (int)Wo, (int)R);
}

int64_t conv_fwd_(const at::Tensor& x, const at::Tensor& w2, at::Tensor out, int64_t R, int64_t S, int64_t stride,
                  int64_t pad, c10::optional<at::Tensor> part, c10::optional<at::Tensor> shift) {
  return conv_fwd_impl(x, w2, out, R, S, stride, pad, nullptr, nullptr, part, shift);
}

int64_t conv_fwd_fp8_(const at::Tensor& x, const at::Tensor& w2, const at::Tensor& x_scale, const at::Tensor& w_scale,
                      at::Tensor out, int64_t R, int64_t S, int64_t stride, int64_t pad, c10::optional<at::Tensor> part,
                      c10::optional<at::Tensor> shift) {
  return conv_fwd_impl(x, w2, out, R, S, stride, pad, &x_scale, &w_scale, part, shift);
}

// Implicit-GEMM convolution weight gradient: out [Cout, R*S*C] (an OHWI weight viewed 2-D, bf16) =
// dY^T . im2col(x), dY [Nb, Cout, Ho, Wo] and x [Nb, C, H, W] channels_last bf16; split-K over the
// output pixels (splits <= 0: about one round of workgroups). False (nothing launched) outside the
// kernel's contract.
bool conv_wgrad_(const at::Tensor& dy, const at::Tensor& x, at::Tensor out, int64_t R, int64_t S, int64_t stride,
                 int64_t pad, int64_t splits) {
  TORCH_CHECK(dy.is_cuda() && x.is_cuda() && dy.dim() == 4 && x.dim() == 4 && dy.scalar_type() == at::kBFloat16 &&
                  x.scalar_type() == at::kBFloat16 && dy.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "psd conv_wgrad: dy and x must be channels_last bf16 device tensors");
  const int64_t Nb = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int64_t Cout = dy.size(1), Ho = dy.size(2), Wo = dy.size(3);
  TORCH_CHECK(dy.size(0) == Nb && Ho == (H + 2 * pad - R) / stride + 1 && Wo == (W + 2 * pad - S) / stride + 1,
              "psd conv_wgrad: dy shape does not match the convolution");
  const int64_t N = R * S * C, K = Nb * Ho * Wo;
  TORCH_CHECK(out.dim() == 2 && out.size(0) == Cout && out.size(1) == N && out.is_contiguous() &&
                  out.scalar_type() == at::kBFloat16,
              "psd conv_wgrad: out must be a contiguous bf16 [Cout, R*S*C]");
  const int64_t xbytes = x.numel() * 2;
  if ((C & (C - 1)) != 0 || C < 8 || xbytes >= ((int64_t)1 << 32) || K >= ((int64_t)1 << 31) || K < 128) return false;
  int logc = 0;
  while ((1 << logc) < C) ++logc;
  const c10::DeviceGuard g(x.device());
  const int64_t tiles = ((Cout + 255) / 256) * ((N + 255) / 256);
  int64_t s = splits > 0 ? splits : std::max<int64_t>(1, 256 / tiles);
  s = std::min<int64_t>(s, std::max<int64_t>(1, K / 128));  // >= 2 K-tiles per split
  at::Tensor slab = at::empty({s * Cout * N}, x.options().dtype(at::kFloat));
  GemmArgs a{};
  a.A = dy.data_ptr();
  a.B = x.data_ptr();
  a.M = (int)Cout;
  a.N = (int)N;
  a.K = (int)K;
  a.lda = (int)Cout;
  a.ldb = (int)N;
  a.ldc = (int)N;
  a.a_kmajor = a.b_kmajor = 0;
  a.cv_H = (int)H;
  a.cv_W = (int)W;
  a.cv_logC = logc;
  a.cv_Ho = (int)Ho;
  a.cv_Wo = (int)Wo;
  a.cv_S = (int)S;
  a.cv_stride = (int)stride;
  a.cv_pad = (int)pad;
  a.cv_abytes = (uint32_t)xbytes;
  hipError_t e = launch_conv_wgrad(a, slab.data_ptr<float>(), (int)s, out.data_ptr(), stream_of(x));
  if (e == hipErrorNotSupported) return false;
  TORCH_CHECK(e == hipSuccess, "psd conv_wgrad: ", hipGetErrorString(e));
  return true;
}

// out[N] (+)= column sums of x[M,N] (bias gradient)
void colsum_(const at::Tensor& x, at::Tensor out, bool accumulate) {
  chk2d(x, "x");
  const int64_t M = x.size(0), N = x.size(1);
  TORCH_CHECK(N % 8 == 0 && x.is_contiguous(), "psd colsum: N % 8 and contiguous");
  TORCH_CHECK(out.numel() == N && out.is_contiguous(), "psd colsum: out [N]");
  const c10::DeviceGuard g(x.device());
  TORCH_CHECK(out.scalar_type() == at::kBFloat16 || out.scalar_type() == at::kFloat, "psd colsum: out dtype");
  at::Tensor part = at::empty({(int64_t)kColsumPartRows * N}, x.options().dtype(at::kFloat));
  hipError_t e = launch_colsum(reinterpret_cast<const uint16_t*>(x.data_ptr()), M, (int)N, part.data_ptr<float>(),
                               out.data_ptr(), out.scalar_type() == at::kBFloat16, accumulate, stream_of(x));
  TORCH_CHECK(e == hipSuccess, "psd colsum: ", hipGetErrorString(e));
}

// GELU(tanh) backward fused with the bias gradient: dx = bf16(dy * gelu'(pre)) and out[N] (+)= colsum(dx)
void gelu_bwd_colsum_(const at::Tensor& dy, const at::Tensor& pre, at::Tensor dx, at::Tensor out, bool accumulate) {
  chk2d(dy, "dy");
  chk2d(pre, "pre");
  chk2d(dx, "dx");
  const int64_t M = dy.size(0), N = dy.size(1);
  TORCH_CHECK(N % 8 == 0 && dy.is_contiguous() && pre.is_contiguous() && dx.is_contiguous() && pre.sizes() == dy.sizes() &&
                  dx.sizes() == dy.sizes(),
              "psd gelu_bwd_colsum: contiguous [M, N] tensors, N % 8");
  TORCH_CHECK(out.numel() == N && out.is_contiguous() &&
                  (out.scalar_type() == at::kBFloat16 || out.scalar_type() == at::kFloat),
              "psd gelu_bwd_colsum: out [N] bf16/fp32");
  const c10::DeviceGuard g(dy.device());
  at::Tensor part = at::empty({(int64_t)kColsumPartRows * N}, dy.options().dtype(at::kFloat));
  hipError_t e = launch_colsum(reinterpret_cast<const uint16_t*>(dy.data_ptr()), M, (int)N, part.data_ptr<float>(),
                               out.data_ptr(), out.scalar_type() == at::kBFloat16, accumulate, stream_of(dy),
                               reinterpret_cast<const uint16_t*>(pre.data_ptr()),
                               reinterpret_cast<uint16_t*>(dx.data_ptr()));
  TORCH_CHECK(e == hipSuccess, "psd gelu_bwd_colsum: ", hipGetErrorString(e));
}

// Narrow implicit-GEMM weight gradient (kernels/convw.hip): out[Cout][R*S*C] (bf16, the OHWI weight
// layout) = dY^T . im2col(x), or out += that with accumulate. Returns false when the kernel declines
// the shape (nothing launched).
int64_t convw_variants_(int64_t Cout, int64_t KK) { return convw_variants((int)Cout, (int)KK); }

// rows of a fold launch's fp32 result: [g^T x (Cout) | x^T x (Cin) | column sums of x (+ padding)]
// 0 when the fold launch is not supported for this shape
int64_t convw_fold_rows(int64_t Cout, int64_t Cin) {
  const int64_t rows = (Cout + Cin + 16 + 127) / 128 * 128;
  return convw_fold_ok((int)Cout, (int)Cin, (int)rows) ? rows : 0;
}

bool convw_(const at::Tensor& dy, const at::Tensor& x, at::Tensor out, int64_t R, int64_t S, int64_t stride,
            int64_t pad, int64_t variant, bool accumulate, bool fold) {
  TORCH_CHECK(dy.is_cuda() && x.is_cuda() && dy.dim() == 4 && x.dim() == 4 && dy.scalar_type() == at::kBFloat16 &&
                  x.scalar_type() == at::kBFloat16 && dy.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast) && dy.device() == x.device(),
              "psd convw: dy and x must be channels_last bf16 tensors on one device");
  const int64_t Nb = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int64_t Cout = dy.size(1), Ho = dy.size(2), Wo = dy.size(3);
  TORCH_CHECK(dy.size(0) == Nb && Ho == (H + 2 * pad - R) / stride + 1 && Wo == (W + 2 * pad - S) / stride + 1,
              "psd convw: dy shape does not match the convolution");
  const int64_t KK = R * S * C, M = Nb * Ho * Wo;
  const int64_t rows = fold ? convw_fold_rows(Cout, KK) : Cout;
  TORCH_CHECK(out.is_cuda() && out.device() == x.device() && out.dim() == 2 && out.size(0) == rows &&
                  out.size(1) == KK && out.is_contiguous() &&
                  out.scalar_type() == (fold ? at::kFloat : at::kBFloat16) &&
                  (reinterpret_cast<uintptr_t>(out.data_ptr()) & 15) == 0,
              "psd convw: out must be a contiguous [Cout, R*S*C] bf16 tensor (fold: fp32 [convw_fold_rows, C]) "
              "on x's device");
  if (fold && (R != 1 || S != 1 || stride != 1 || pad != 0 || accumulate)) return false;
  const int64_t xbytes = x.numel() * 2, dybytes = dy.numel() * 2;
  if ((C & (C - 1)) != 0 || C < 64 || xbytes > 0xFFFFFF00ll || dybytes > 0xFFFFFF00ll || M >= ((int64_t)1 << 31) ||
      (!fold && variant >= convw_variants((int)Cout, (int)KK)) || H >= 32768 || W >= 32768)
    return false;
  int logc = 0;
  while ((1 << logc) < C) ++logc;
  const c10::DeviceGuard g(x.device());
  ConvwArgs a{};
  a.dy = dy.data_ptr();
  a.x = x.data_ptr();
  a.out = out.data_ptr();
  a.dybytes = (uint32_t)dybytes;
  a.xbytes = (uint32_t)xbytes;
  a.M = (int)M;
  a.Cout = (int)Cout;
  a.KK = (int)KK;
  a.H = (int)H;
  a.W = (int)W;
  a.logC = logc;
  a.Ho = (int)Ho;
  a.Wo = (int)Wo;
  a.S = (int)S;
  a.stride = (int)stride;
  a.pad = (int)pad;
  a.variant = (int)variant;
  a.accumulate = accumulate ? 1 : 0;
  a.fold = fold ? 1 : 0;
  a.Arows = (int)rows;
  const ConvwPlan p = convw_plan(a);
  if (p.splits <= 0) return false;
  at::Tensor slab = at::empty({p.slab_floats}, x.options().dtype(at::kFloat));
  a.slab = slab.data_ptr<float>();
  const hipError_t e = launch_convw(a, stream_of(x));
  if (e == hipErrorNotSupported) return false;
  TORCH_CHECK(e == hipSuccess, "psd convw: ", hipGetErrorString(e));
  return true;
}

int64_t convw_gram_rows_(int64_t C) { return convw_gram_rows((int)C); }

// out = fp32 [convw_gram_rows(C), C]: rows [0, C) the Gram matrix x^T x of the [M, C] pixel rows of
// x, row C their column sums -- one read of x (the BN statistics of y = x W^T without forming y:
// ops/tail.py). False when the shape is unsupported.
bool convw_gram_(const at::Tensor& x, at::Tensor out, int64_t variant) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 && x.scalar_type() == at::kBFloat16 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "psd convw_gram: x must be a channels_last bf16 tensor");
  const int64_t Nb = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3), M = Nb * H * W;
  const int64_t rows = convw_gram_rows((int)C);
  TORCH_CHECK(out.is_cuda() && out.device() == x.device() && out.dim() == 2 && out.size(0) == rows &&
                  out.size(1) == C && out.is_contiguous() && out.scalar_type() == at::kFloat &&
                  (reinterpret_cast<uintptr_t>(out.data_ptr()) & 15) == 0,
              "psd convw_gram: out must be a contiguous fp32 [convw_gram_rows(C), C] tensor on x's device");
  const int64_t xbytes = x.numel() * 2;
  if (rows == 0 || xbytes > 0xFFFFFF00ll || M >= ((int64_t)1 << 31) || M == 0) return false;
  int logc = 0;
  while ((1 << logc) < C) ++logc;
  const c10::DeviceGuard g(x.device());
  ConvwArgs a{};
  a.dy = x.data_ptr();
  a.x = x.data_ptr();
  a.out = out.data_ptr();
  a.dybytes = (uint32_t)xbytes;
  a.xbytes = (uint32_t)xbytes;
  a.M = (int)M;
  a.Cout = 0;
  a.KK = (int)C;
  a.H = a.Ho = (int)H;
  a.W = a.Wo = (int)W;
  a.logC = logc;
  a.S = 1;
  a.stride = 1;
  a.pad = 0;
  a.fold = 2;
  a.variant = (int)variant;  // 1: the two-stage ring at two workgroups per CU
  a.Arows = (int)rows;
  const ConvwPlan p = convw_plan(a);
  if (p.splits <= 0) return false;
  at::Tensor slab = at::empty({p.slab_floats}, x.options().dtype(at::kFloat));
  a.slab = slab.data_ptr<float>();
  const hipError_t e = launch_convw(a, stream_of(x));
  if (e == hipErrorNotSupported) return false;
  TORCH_CHECK(e == hipSuccess, "psd convw_gram: ", hipGetErrorString(e));
  return true;
}

}  // namespace psd
