#pragma once
#include <ATen/ATen.h>
#include <tuple>
#include <vector>

namespace psd {

void fused_apply_(at::Tensor master, const std::vector<at::Tensor>& grads, c10::optional<at::Tensor> state1,
                  c10::optional<at::Tensor> state2, c10::optional<at::Tensor> shadow, at::Tensor dyn, int64_t kind,
                  double momentum, double dampening, bool nesterov, double weight_decay, double beta1, double beta2,
                  double eps, bool maximize, int64_t grid_cap = 0);
void optim_advance_(at::Tensor dyn, double beta1, double beta2);
void multi_reduce_(at::Tensor out, const std::vector<at::Tensor>& srcs, double scale);
void pack_cast_(const std::vector<at::Tensor>& srcs, const std::vector<at::Tensor>& dsts);
// the async plane's scatter kernel (kernels/xfer.hip) on explicit segments, on the current stream:
// dsts[i] <- srcs[i] bytewise, blocks_per_seg workgroups per segment (transport measurements)
void xfer_(const std::vector<at::Tensor>& srcs, const std::vector<at::Tensor>& dsts, int64_t blocks_per_seg,
           bool nt_store);
void amax_(const at::Tensor& x, at::Tensor amax_out);
void quant_fp8_(const at::Tensor& x, const at::Tensor& amax, double fp8_max, at::Tensor out, at::Tensor scale_inv);
void quant_fp8_jit_(const at::Tensor& x, at::Tensor out, at::Tensor scale_inv);
void quant_fp8_delayed_(const at::Tensor& x, at::Tensor out, at::Tensor scale_inv, at::Tensor hist, double margin);
void dequant_fp8_(const at::Tensor& x, const at::Tensor& scale_inv, at::Tensor out);
void quant_mx_(const at::Tensor& x, at::Tensor out, at::Tensor scales);
void dequant_mx_(const at::Tensor& q, const at::Tensor& scales, at::Tensor out);

std::vector<at::Tensor> bn_fwd(const at::Tensor& x, c10::optional<at::Tensor> gamma, c10::optional<at::Tensor> beta,
                               c10::optional<at::Tensor> running_mean, c10::optional<at::Tensor> running_var,
                               c10::optional<at::Tensor> residual, bool relu, bool training, double momentum, double eps,
                               c10::optional<at::Tensor> counter, c10::optional<at::Tensor> ss_eval,
                               bool mask_out, c10::optional<at::Tensor> residual_ss, bool stats_only,
                               c10::optional<at::Tensor> q8_out, c10::optional<at::Tensor> part_in,
                               int64_t part_rows, c10::optional<at::Tensor> q8_mx);
// statistics pass of the BN forward alone: shifted sums of x [M, C] into a fresh [rows, 2, C] fp32
at::Tensor bn_reduce_(const at::Tensor& x, const at::Tensor& shift);
at::Tensor bn_bwd_reduce_(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& save_mean,
                          c10::optional<at::Tensor> ss, c10::optional<at::Tensor> dy2,
                          c10::optional<at::Tensor> mbits);
std::vector<at::Tensor> bn_bwd_dual(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& gamma,
                                    const at::Tensor& save_mean, const at::Tensor& save_invstd, const at::Tensor& mbits,
                                    c10::optional<at::Tensor> dy2, const at::Tensor& xd, const at::Tensor& gamma_d,
                                    const at::Tensor& mean_d, const at::Tensor& invstd_d,
                                    c10::optional<at::Tensor> dgamma_out, c10::optional<at::Tensor> dbeta_out,
                                    c10::optional<at::Tensor> dgamma_d_out, c10::optional<at::Tensor> dbeta_d_out, bool fold);
at::Tensor bn_elemt_coef(const at::Tensor& g, const at::Tensor& x, const at::Tensor& coef);
std::vector<at::Tensor> bn_bwd_dual_pre(const at::Tensor& g, const at::Tensor& x, const at::Tensor& gamma,
                                        const at::Tensor& save_mean, const at::Tensor& save_invstd,
                                        const at::Tensor& part, const at::Tensor& part_d, int64_t rows,
                                        const at::Tensor& xd, const at::Tensor& gamma_d, const at::Tensor& mean_d,
                                        const at::Tensor& invstd_d, c10::optional<at::Tensor> dgamma_out,
                                        c10::optional<at::Tensor> dbeta_out, c10::optional<at::Tensor> dgamma_d_out,
                                        c10::optional<at::Tensor> dbeta_d_out, bool fold, bool fold_d, bool derive_d);
std::vector<at::Tensor> bnfold_dgrad_weights(const at::Tensor& w, const at::Tensor& coef);
void bnfold_combine(const at::Tensor& P, const at::Tensor& w, const at::Tensor& coef, at::Tensor out, bool accumulate);
void bnfold_rowdot(const at::Tensor& P, const at::Tensor& w, at::Tensor row);
void bnfold_gram_stats(const at::Tensor& P, const at::Tensor& w, const at::Tensor& shift, int64_t M, at::Tensor row);
std::vector<at::Tensor> bnfold_dual_weights(const at::Tensor& w3, const at::Tensor& wd, const at::Tensor& ss3,
                                            const at::Tensor& ssd);
std::vector<at::Tensor> bn_finalize(const at::Tensor& part, int64_t rows, int64_t M, const at::Tensor& gamma,
                                    const at::Tensor& beta, at::Tensor running_mean, at::Tensor running_var,
                                    double momentum, double eps, c10::optional<at::Tensor> counter);
std::vector<at::Tensor> bn_bwd_coef(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& gamma,
                                    const at::Tensor& save_mean, const at::Tensor& save_invstd,
                                    c10::optional<at::Tensor> mbits, c10::optional<at::Tensor> dy2,
                                    c10::optional<at::Tensor> part, int64_t rows, c10::optional<at::Tensor> dgamma_out,
                                    c10::optional<at::Tensor> dbeta_out);
std::vector<at::Tensor> bn_bwd(const at::Tensor& dy, const at::Tensor& x, c10::optional<at::Tensor> y,
                               c10::optional<at::Tensor> gamma, const at::Tensor& save_mean,
                               const at::Tensor& save_invstd, bool relu, bool need_dr,
                               c10::optional<at::Tensor> dgamma_out, c10::optional<at::Tensor> dbeta_out,
                               c10::optional<at::Tensor> dy2, c10::optional<at::Tensor> ss,
                               c10::optional<at::Tensor> mbits, c10::optional<at::Tensor> dq, c10::optional<at::Tensor> dqmx);

int64_t gemm_(const at::Tensor& A, const at::Tensor& B, bool a_kmajor, bool b_kmajor, at::Tensor out,
              c10::optional<at::Tensor> bias, int64_t act, c10::optional<at::Tensor> aux,
              c10::optional<at::Tensor> part, c10::optional<at::Tensor> shift);
// statistics partial rows to allocate for a gemm_ / gemm_fp8_ / conv_fwd_ with part (any tile height)
int64_t gemm_stats_rows_(int64_t M);
// out[N, M] = B A^T (+bias[M])(act 0-2, aux = pre-activation) on 192 x 256 tiles stored transposed
// (A [M, K], B [N, K] K-major: Y = X W^T + b with A = W, B = X); False when the shape is outside the
// kernel's contract (nothing launched)
bool gemm_ct_(const at::Tensor& A, const at::Tensor& B, at::Tensor out, c10::optional<at::Tensor> bias, int64_t act,
              c10::optional<at::Tensor> aux);
bool gemm_gelu_bwd_(const at::Tensor& A, const at::Tensor& B, bool a_kmajor, bool b_kmajor, const at::Tensor& pre,
                    at::Tensor out, at::Tensor db, bool accumulate);
void gemm_splitk_(const at::Tensor& A, const at::Tensor& B, bool a_kmajor, bool b_kmajor, at::Tensor out,
                  bool accumulate, double scale, int64_t splits);
void colsum_(const at::Tensor& x, at::Tensor out, bool accumulate);
void gelu_bwd_colsum_(const at::Tensor& dy, const at::Tensor& pre, at::Tensor dx, at::Tensor out, bool accumulate);
// narrow-output implicit-GEMM convolution (kernels/convn.hip): out [Nb*Ho*Wo, Cout] = conv(x, w2),
// w2 [Cout, R*S*C]; with part/shift also the consumer BN's shifted statistics partials (a buffer of
// convn_stats_rows(M) x 2 x Cout). Returns 0 (nothing launched) outside the kernel's contract, else
// the partial rows written (1 without statistics).
int64_t convn_part_rows_(int64_t M, int64_t N, int64_t v, int64_t Ho, int64_t Wo, int64_t R);
bool convn_variant_ok_(int64_t N, int64_t v, int64_t R, int64_t S, int64_t stride, int64_t pad, int64_t Wo, bool has_x2);
// no_store: statistics only (out unused); apply_ss / apply_res / apply_mask: the BN apply epilogue
// out = relu(bf16(conv) * ss[c] + ss[Cout + c] + res) + its ReLU bit-mask (bwd mode 8)
int64_t convn_(const at::Tensor& x, const at::Tensor& w2, at::Tensor out, int64_t R, int64_t S, int64_t stride,
               int64_t pad, c10::optional<at::Tensor> part, c10::optional<at::Tensor> shift, int64_t variant,
               c10::optional<at::Tensor> x2, c10::optional<at::Tensor> bias, bool no_store,
               c10::optional<at::Tensor> apply_ss, c10::optional<at::Tensor> apply_res,
               c10::optional<at::Tensor> apply_mask);
int64_t convn_stats_rows_(int64_t M);
int64_t convn_dgrad_s2_(const at::Tensor& dy, const std::vector<at::Tensor>& wph, at::Tensor out, int64_t variant,
                        c10::optional<at::Tensor> part, c10::optional<at::Tensor> bx, c10::optional<at::Tensor> bmean,
                        c10::optional<at::Tensor> bss);
int64_t convn_dgrad_s2_rows(int64_t Nb, int64_t Ho, int64_t Wo, int64_t Ci, int64_t variant);
int64_t convn_bwd_(const at::Tensor& dy, const at::Tensor& w2, at::Tensor out, int64_t R, int64_t S, int64_t stride,
                   int64_t pad, at::Tensor part, int64_t variant, int64_t mode, c10::optional<at::Tensor> bx,
                   const at::Tensor& bmean, c10::optional<at::Tensor> bss, c10::optional<at::Tensor> bdr,
                   c10::optional<at::Tensor> bmbits, c10::optional<at::Tensor> x2,
                   c10::optional<at::Tensor> bias, c10::optional<at::Tensor> bxd, c10::optional<at::Tensor> bmean_d,
                   c10::optional<at::Tensor> part_d);
std::vector<at::Tensor> bn_bwd_pre(const at::Tensor& g, const at::Tensor& x, c10::optional<at::Tensor> gamma,
                                   const at::Tensor& save_mean, const at::Tensor& save_invstd, const at::Tensor& part,
                                   int64_t rows, c10::optional<at::Tensor> dgamma_out,
                                   c10::optional<at::Tensor> dbeta_out, c10::optional<at::Tensor> dq,
                                   c10::optional<at::Tensor> dqmx);
int64_t convn_variants_(int64_t N);
int64_t convn_variant_kind_(int64_t N, int64_t v);
int64_t conv_fwd_(const at::Tensor& x, const at::Tensor& w2, at::Tensor out, int64_t R, int64_t S, int64_t stride,
                  int64_t pad, c10::optional<at::Tensor> part, c10::optional<at::Tensor> shift);
bool conv_wgrad_(const at::Tensor& dy, const at::Tensor& x, at::Tensor out, int64_t R, int64_t S, int64_t stride,
                 int64_t pad, int64_t splits);
bool convw_(const at::Tensor& dy, const at::Tensor& x, at::Tensor out, int64_t R, int64_t S, int64_t stride,
            int64_t pad, int64_t variant, bool accumulate, bool fold);
int64_t convw_fold_rows(int64_t Cout, int64_t Cin);
int64_t convw_gram_rows_(int64_t C);
bool convw_gram_(const at::Tensor& x, at::Tensor out, int64_t variant);
int64_t convw_variants_(int64_t Cout, int64_t KK);
int64_t conv_fwd_fp8_(const at::Tensor& x, const at::Tensor& w2, const at::Tensor& x_scale, const at::Tensor& w_scale,
                      at::Tensor out, int64_t R, int64_t S, int64_t stride, int64_t pad, c10::optional<at::Tensor> part,
                      c10::optional<at::Tensor> shift);
int64_t gemm_fp8_(const at::Tensor& A, const at::Tensor& B, const at::Tensor& a_scale, const at::Tensor& b_scale,
                  at::Tensor out, c10::optional<at::Tensor> bias, int64_t act, c10::optional<at::Tensor> aux,
                  c10::optional<at::Tensor> part, c10::optional<at::Tensor> shift);
std::vector<at::Tensor> maxpool3s2_fwd(const at::Tensor& x);
at::Tensor maxpool3s2_bwd(const at::Tensor& dy, const at::Tensor& arg, int64_t H, int64_t W,
                          const c10::optional<at::Tensor>& dy2);
at::Tensor gap_fwd(const at::Tensor& x);
std::vector<at::Tensor> bn_pool_fwd(const at::Tensor& x, const at::Tensor& gamma, const at::Tensor& beta,
                                    const at::Tensor& running_mean, const at::Tensor& running_var, double momentum,
                                    double eps, c10::optional<at::Tensor> counter);
std::vector<at::Tensor> stem_fwd(const at::Tensor& x, const at::Tensor& w, const at::Tensor& gamma, const at::Tensor& beta,
                                 const at::Tensor& running_mean, const at::Tensor& running_var, double momentum,
                                 double eps, c10::optional<at::Tensor> counter);
at::Tensor stem_wgrad(const at::Tensor& x, const at::Tensor& dy);
std::vector<at::Tensor> attn_fwd(const at::Tensor& qkv, int64_t heads, double p, int64_t seed,
                                 c10::optional<at::Tensor> step);
at::Tensor attn_bwd(const at::Tensor& dout, const at::Tensor& qkv, const at::Tensor& o, const at::Tensor& lse,
                    int64_t heads, double p, int64_t seed, c10::optional<at::Tensor> step,
                    c10::optional<at::Tensor> bias_out);
std::vector<at::Tensor> ln_fwd(const at::Tensor& x, const at::Tensor& h, const at::Tensor& gamma, const at::Tensor& beta,
                               double eps, double p, int64_t seed, c10::optional<at::Tensor> step);
std::vector<at::Tensor> ln_bwd(const at::Tensor& dy, const at::Tensor& s, const at::Tensor& mean, const at::Tensor& rstd,
                               const at::Tensor& gamma, double p, int64_t seed, c10::optional<at::Tensor> step,
                               c10::optional<at::Tensor> dgamma_out, c10::optional<at::Tensor> dbeta_out,
                               c10::optional<at::Tensor> dhsum_out);
std::vector<at::Tensor> emb_ln_fwd(const at::Tensor& ids, const at::Tensor& types, const at::Tensor& W,
                                   const at::Tensor& P, const at::Tensor& T, const at::Tensor& gamma,
                                   const at::Tensor& beta, int64_t S, double eps, double p, int64_t seed,
                                   c10::optional<at::Tensor> step);
std::vector<at::Tensor> emb_ln_bwd(const at::Tensor& dy, const at::Tensor& ids, const at::Tensor& types,
                                   const at::Tensor& W, const at::Tensor& P, const at::Tensor& T,
                                   const at::Tensor& gamma, const at::Tensor& mean, const at::Tensor& rstd, int64_t S,
                                   double p, int64_t seed, c10::optional<at::Tensor> step,
                                   c10::optional<at::Tensor> dgamma_out, c10::optional<at::Tensor> dbeta_out,
                                   c10::optional<at::Tensor> dT_out);
std::vector<at::Tensor> bn_pool_bwd(const at::Tensor& gpool, c10::optional<at::Tensor> gpool2, const at::Tensor& arg,
                                    const at::Tensor& x, const at::Tensor& gamma, const at::Tensor& save_mean,
                                    const at::Tensor& save_invstd, const at::Tensor& ss,
                                    c10::optional<at::Tensor> dgamma_out, c10::optional<at::Tensor> dbeta_out);
at::Tensor gap_bwd(const at::Tensor& dy, int64_t H, int64_t W);
at::Tensor subsample2(const at::Tensor& x);

// batched bwd-data weight preparation (wprep_ops.cpp)
std::tuple<at::Tensor, int64_t> wprep_table(const std::vector<at::Tensor>& srcs, const std::vector<at::Tensor>& dsts,
                                            const std::vector<int64_t>& geo);
void wprep_run(const at::Tensor& table, int64_t tiles);

// fused softmax cross-entropy on bf16 logits (xent_ops.cpp)
void embed_bwd_(const at::Tensor& sorted, const at::Tensor& perm, const at::Tensor& dy, at::Tensor out);
std::vector<at::Tensor> xent_fwd(const at::Tensor& x, const at::Tensor& labels);
at::Tensor xent_bwd(const at::Tensor& x, const at::Tensor& labels, const at::Tensor& lse, const at::Tensor& scale);

}  // namespace psd
