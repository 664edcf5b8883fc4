#!/usr/bin/env python3
"""MFMA GEMM probe: time the hand-written gfx950 GEMM (csrc/kernels/gemm.hip) against hipBLASLt
(torch.mm, TunableOp off) on a square reference and the BERT-base b256/s128 shapes, uniform random
[-1, 1) operands (zero-filled operands run ~19% faster on MI355X: MI355X_MICROARCH.md).

  python tools/gemm_probe.py [--shapes bert|square|all] [--it 20]          timing table (markdown)
  python tools/gemm_probe.py --pmc NTxMxNxK                                 5 launches of one GEMM (rocprofv3 --pmc)

Layouts: NT = X[M,K] . W[N,K]^T (forward), NN = dY[M,K] . W[K,N] (dgrad), TN = dY^T . X (wgrad,
split-K into the fp32 slab + reduce, as ops/linear.py runs it), CT = the NT product on the 192 x 256
transposed-store tile (gemm_ct_).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from parameter_server_distributed_amd import native  # noqa: E402

SQUARE = [("NT", 4096, 4096, 4096), ("NT", 8192, 8192, 8192), ("NN", 4096, 4096, 4096), ("TN", 4096, 4096, 4096)]
T = 256 * 128  # BERT-base tokens per step at the bench config
BERT = [("NT", T, 2304, 768), ("NT", T, 3072, 768), ("NT", T, 768, 3072), ("NT", T, 768, 768),
        ("NN", T, 768, 2304), ("NN", T, 768, 3072), ("NN", T, 3072, 768),
        ("TN", 2304, 768, T), ("TN", 3072, 768, T), ("TN", 768, 3072, T), ("TN", 768, 768, T),
        ("TN0", 2304, 768, T), ("TN0", 3072, 768, T), ("TN0", 768, 3072, T), ("TN0", 768, 768, T),
        ("CT", T, 2304, 768), ("CT", T, 768, 768), ("CT", T, 768, 3072), ("CT", T, 3072, 768)]


def rnd(*s):
    return (torch.rand(*s, device="cuda") * 2 - 1).to(torch.bfloat16)


def make(layout, M, N, K):
    """Operands and the two callables (ours, hipBLASLt) computing C[M, N]."""
    C = native()
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    if layout == "NT":
        a, b = rnd(M, K), rnd(N, K)
        return (lambda: C.gemm_(a, b, True, True, out)), (lambda: torch.mm(a, b.t(), out=out)), out, (a, b)
    if layout == "NN":
        a, b = rnd(M, K), rnd(K, N)
        return (lambda: C.gemm_(a, b, True, False, out)), (lambda: torch.mm(a, b, out=out)), out, (a, b)
    if layout == "CT":  # C[M, N] = X W^T on the 192 x 256 transposed-store tile (A = W [N, K], B = X [M, K])
        a, b = rnd(M, K), rnd(N, K)
        return (lambda: C.gemm_ct_(b, a, out)), (lambda: torch.mm(a, b.t(), out=out)), out, (a, b)
    # TN: C[M, N] = A^T B with A [K, M], B [K, N] (wgrad: M = out features, K = tokens); TN0: the same
    # with the B halves staged as contiguous 128-column rows (gemm_set_bcontig(True); default off)
    a, b = rnd(K, M), rnd(K, N)
    bc = layout == "TN0"

    def ours():
        C.gemm_set_bcontig(bc)
        C.gemm_splitk_(a, b, False, False, out, False, 1.0, 0)
        C.gemm_set_bcontig(False)

    return ours, (lambda: torch.mm(a.t(), b, out=out)), out, (a, b)


def t_us(fn, it):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="all", choices=["bert", "square", "all"])
    ap.add_argument("--it", type=int, default=20)
    ap.add_argument("--ksweep", default="", help="LAYOUTxMxN: time K = 256..4096 (per-tile fixed cost = intercept)")
    ap.add_argument("--pmc", default="", help="LAYOUTxMxNxK: launch ours 5x only (for rocprofv3 --pmc)")
    ap.add_argument("--lib", action="store_true", help="with --pmc: launch hipBLASLt instead of ours")
    a = ap.parse_args()
    import torch.cuda.tunable as tn

    tn.enable(False)
    if a.pmc:
        lay, M, N, K = a.pmc.split("x")
        ours, lib, _, _ = make(lay, int(M), int(N), int(K))
        for _ in range(5):
            (lib if a.lib else ours)()
        torch.cuda.synchronize()
        return
    shapes = {"bert": BERT, "square": SQUARE, "all": SQUARE + BERT}[a.shapes]
    if a.ksweep:
        lay, M, N = a.ksweep.split("x")
        shapes = [(lay, int(M), int(N), k) for k in (256, 512, 768, 1024, 1536, 2048, 3072, 4096)]
    print("| layout | M | N | K | ours us | TF/s | hipBLASLt us | TF/s | ours/lib | max rel err |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    for lay, M, N, K in shapes:
        ours, lib, out, _ = make(lay, M, N, K)
        lib()
        ref = out.float().clone()
        ours()
        err = float(((out.float() - ref).abs().max() / ref.abs().max()).item())
        to, tl = t_us(ours, a.it), t_us(lib, a.it)
        fl = 2.0 * M * N * K
        print(f"| {lay} | {M} | {N} | {K} | {to:.0f} | {fl / to / 1e6:.0f} | {tl:.0f} | {fl / tl / 1e6:.0f} | "
              f"{tl / to:.2f} | {err:.1e} |", flush=True)


if __name__ == "__main__":
    main()
