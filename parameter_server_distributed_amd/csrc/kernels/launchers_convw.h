// Launch API of the narrow implicit-GEMM convolution weight gradient (convw.hip).
#pragma once
#include <hip/hip_runtime_api.h>
#include <cstdint>

namespace psd {

struct ConvwArgs {
  const void* dy;      // bf16 [M][Cout] output gradient (NHWC rows), M = Nb*Ho*Wo
  const void* x;       // bf16 NHWC input [Nb][H][W][C], C a power of two >= 64
  float* slab;         // fp32 workspace of convw_plan().slab_floats: [splits][Cout][KK] partials + reduce tree
  void* out;           // bf16 [Cout][KK] result, KK = R*S*C ordered (r, s, ci) = the OHWI weight
  uint32_t dybytes;    // bytes of dy (< 2^32 - 256)
  uint32_t xbytes;     // bytes of x
  int M, Cout, KK;
  int H, W, logC, Ho, Wo, S, stride, pad;
  int variant;         // tile geometry, [0, convw_variants(Cout, KK)); -1: the default (0)
  int accumulate;      // out += result (bf16) instead of out = result
  // BN-backward fold (ops/bn.py): the A rows are [dY (Cout rows) | x (KK rows) | ones (the rest of
  // Arows)], so out = fp32 [Arows][KK] holds dY^T x, the Gram matrix x^T x and the column sums of x
  // (1x1 only, the whole KK in one tile). 0: plain (Arows = Cout, bf16 out). 2: the Gram launch
  // (Cout = 0, Arows = convw_gram_rows(KK)): x^T x and the column sums of x from one read of x
  int fold;
  int Arows;
  // set by the launcher
  int splits, stages_per_split;
  uint32_t howo_m, howo_s, wo_m, wo_s;  // round-up magic numbers of / (Ho*Wo) and / Wo (common.h FastDiv)
};

struct ConvwPlan {
  int splits;           // pixel splits (the grid is splits x output tiles)
  int64_t slab_floats;  // fp32 workspace the launch needs
};

// tile variants for Cout output channels and KK = R*S*C reduction columns (0: unsupported)
int convw_variants(int Cout, int KK);
// a fold launch (1x1, Cout dY rows, KK = Cin, Arows = convw_fold_rows) is supported
bool convw_fold_ok(int Cout, int KK, int Arows);
// rows of a Gram launch's fp32 result [x^T x (C rows) | column sums (row C) | padding]; 0: unsupported
int convw_gram_rows(int C);
// split plan of a launch (the caller allocates slab_floats fp32 for it)
ConvwPlan convw_plan(const ConvwArgs& a);
// hipErrorNotSupported outside the kernel's contract (nothing launched)
hipError_t launch_convw(const ConvwArgs& a, hipStream_t stream);

}  // namespace psd
