// Launch API of the fused NHWC BatchNorm(+residual)(+ReLU) kernels (bn.hip).
#pragma once
#include <hip/hip_runtime_api.h>
#include <cstdint>

namespace psd {

struct BnFwdArgs {
  const uint16_t* x;      // [M, C] bf16
  const uint16_t* res;    // optional residual [M, C] bf16
  uint16_t* y;            // [M, C] bf16
  uint8_t* mbits;         // optional: ReLU mask out, 1 bit per element ([M * C / 8] bytes)
  const uint16_t* gamma;  // [C] bf16 (optional)
  const uint16_t* beta;   // [C] bf16 (optional)
  float* running_mean;    // [C] fp32 (optional; also used as the variance shift)
  float* running_var;     // [C] fp32 (optional)
  float* save_mean;       // [C]
  float* save_invstd;     // [C]
  float* ss;              // [2C] scale, shift (inference: provided; training: produced)
  float* part;            // [bn_reduce_blocks * 2C] workspace
  int64_t* counter;       // num_batches_tracked (optional)
  int32_t part_ready;     // > 0: part already holds this many rows of partial sums (producer epilogue)
  float* fold_ws;         // [kFoldRows * 2C] workspace, needed when part_ready > kFoldRows
  const float* res_ss;    // optional [2C]: res is a raw BN input, added as res*res_ss[c] + res_ss[C+c]
  int32_t stats_only;     // training: statistics / running stats / scale-shift only, no apply pass
  uint8_t* q8;            // optional [M, C] e4m3 copy of y for an fp8 consumer (delayed scaling)
  uint8_t* q8mx;          // MX instead of per-tensor: [M * C / 32] E8M0 block scales of q8 (no history)
  uint8_t* pool_arg;      // stem fusion: y = maxpool3x3s2(relu(bn(x))) [N, H/2, W/2, C] + argmax (optional)
  int32_t N, H, W;        // x as [N, H, W, C] (pool fusion only)
  int64_t M;
  int32_t C;
  int32_t relu;
  int32_t training;
  float momentum;
  float eps;
};

struct BnBwdArgs {
  const uint16_t* dy;
  const uint16_t* dy2;    // optional second upstream gradient (residual-branch fusion): dy + dy2
  const uint16_t* y;      // forward output (ReLU mask); null: mask recomputed from x and ss
  const float* ss;        // [2C] forward scale/shift (needed when relu && !y && !mbits)
  const uint8_t* mbits;   // forward ReLU bit-mask (residual BNs; requires dr)
  const uint16_t* x;      // forward input
  const uint16_t* gamma;
  const float* save_mean;
  const float* save_invstd;
  uint16_t* dx;
  uint16_t* dr;           // optional: gradient of the residual input (= masked dy)
  uint16_t* dgamma;       // optional, bf16 [C]
  uint16_t* dbeta;        // optional, bf16 [C]
  float* coef;            // [3C] workspace
  float* part;            // [bn_reduce_blocks * 2C] workspace
  // stem fusion: dy = maxpool3x3s2 backward of gpool (+ gpool2) through pool_arg, computed on the
  // fly (never materialised); x is [N, H, W, C], H and W even; ReLU mask from x and ss
  const uint16_t* gpool;
  const uint16_t* gpool2;
  const uint8_t* pool_arg;
  int32_t N, H, W;
  int64_t M;
  int32_t C;
  int32_t relu;
  // dual (downsample blocks, ops/bn.py _BNAddBNReluFn): a second BN whose output was the residual,
  // input xd; its reduction rides on this one's reduce pass (same dr) and its dx on the same elemt
  // pass. Needs the bit-mask path with dr.
  const uint16_t* xd;
  const uint16_t* gamma_d;
  const float* mean_d;
  const float* invstd_d;
  uint16_t* dxd;
  uint16_t* dgamma_d;
  uint16_t* dbeta_d;
  float* coef_d;  // [3C]
  float* part_d;  // like part
  // the reduction pass alone (partials into part, dr when given): what a bwd-data convolution that
  // does not fuse it leaves to the BN (autotune timing twin, ops/conv.py _with_bn_bwd_reduce)
  int32_t reduce_only;
  // reduction + finalize only (coef, dgamma, dbeta; dr when given): the consumer convolution folds
  // the elementwise pass into its backward GEMMs (ops/bn.py, kernels/bnfold.hip)
  int32_t coef_only;
  // MX e5m2 copy of dx (+ E8M0 scales per 32 channels) for the producing fp8 convolution's bwd-data
  uint8_t* dq;
  uint8_t* dqmx;
};

// true when the fused stem BN+ReLU+max-pool kernels support this shape
bool bn_pool_supported(int H, int W, int C);
int bn_pool_reduce_blocks(int N, int H, int W, int C);  // partial rows of the pool-fused backward
int bn_reduce_blocks(int64_t M, int C);
// rows the finalize sums directly; more producer partial rows are folded into this many first
constexpr int kFoldRows = 512;
// the statistics pass alone (shifted sums into part [bn_reduce_blocks * 2C]): autotune timing
hipError_t launch_bn_reduce(const uint16_t* x, int64_t M, int C, const float* shift, float* part, hipStream_t st);
hipError_t launch_bn_fwd(const BnFwdArgs& a, hipStream_t stream);
hipError_t launch_bn_bwd(const BnBwdArgs& a, hipStream_t stream);
// backward from a producer-reduced, already-masked gradient g (convolution bwd-data epilogue):
// fold (> kFoldRows partial rows: fold_ws [kFoldRows * 2C]) + finalize + dx = A g + B x + C
hipError_t launch_bn_bwd_pre(const uint16_t* g, const uint16_t* x, const uint16_t* gamma, const float* mean,
                             const float* invstd, const float* part, int rows, float* fold_ws, uint16_t* dgamma,
                             uint16_t* dbeta, float* coef, uint16_t* dx, int64_t M, int C, hipStream_t stream,
                             uint8_t* dq = nullptr, uint8_t* dqmx = nullptr);

struct BnDualPreArgs {
  const uint16_t* g;      // masked upstream gradient (= the residual-branch gradient) [M, C]
  const uint16_t* x;      // bn's input
  const uint16_t* xd;     // bnd's input
  const uint16_t* gamma;
  const uint16_t* gamma_d;
  const float *mean, *invstd, *mean_d, *invstd_d;
  const float* part;      // [rows][2][C] sum g, sum g (x - mean)
  const float* part_d;    // [rows][2][C] sum g, sum g (xd - mean_d); derive_d: [2][C] = [0 | sum g yd]
  int rows;
  int derive_d;           // the downsample BN's sums from part's sum g and part_d's sum g yd
  float *fold_ws, *fold_ws_d;  // [kFoldRows * 2C] each when rows > kFoldRows
  uint16_t *dgamma, *dbeta, *dgamma_d, *dbeta_d;
  float *coef, *coef_d;   // [3C] each
  uint16_t* dx;           // optional (null: folded)
  uint16_t* dxd;
  int64_t M;
  int C;
};
hipError_t launch_bn_bwd_dual_pre(const BnDualPreArgs& a, hipStream_t stream);

// BN-backward fold (bnfold.hip); bn_elemt_coef (bn.hip): dx = A g + B x + C from finalized coefficients
hipError_t launch_bn_elemt_coef(const uint16_t* g, const uint16_t* x, const float* coef, uint16_t* dx, int64_t M, int C,
                                hipStream_t stream);
hipError_t launch_bnfold_gram_stats(const float* P, const uint16_t* W, const float* shift, int Cout, int Wd, int64_t M,
                                    float* row, hipStream_t st);
// dual tail apply operands: wcat [Cout, C3 + Cd] bf16 and ss [2 Cout] fp32 (ops/tail.py)
hipError_t launch_bnfold_dual_weights(const uint16_t* W3, const uint16_t* Wd, const float* ss3, const float* ssd,
                                      int Cout, int C3, int Cd, uint16_t* wcat, float* ss, hipStream_t st);
hipError_t launch_bnfold_rowdot(const float* P, const uint16_t* W, int Cout, int Wd, float* row, hipStream_t st);
hipError_t launch_bnfold_prep(const uint16_t* W, const float* coef, int Cout, int Wd, uint16_t* w2, int ldw,
                              uint16_t* bw, float* bvec, hipStream_t stream);
hipError_t launch_bnfold_combine(const float* P, const uint16_t* W, const float* coef, int Cout, int Wd,
                                 uint16_t* out, int accumulate, hipStream_t stream);

}  // namespace psd
