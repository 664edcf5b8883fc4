#!/usr/bin/env python3
"""A/B of the MFMA GEMM kernels on square and BERT-base shapes (uniform random operands): prints
one markdown row per (shape, layout) with us and TFLOP/s, plus the max error against an fp32
torch reference. Select the 256x256 kernel variant with PSD_GEMM_BIG=0/1/2 (one per process)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from parameter_server_distributed_amd import native  # noqa: E402

SHAPES = [("sq4096", 4096, 4096, 4096), ("sq8192", 8192, 8192, 8192),
          ("bert.qkv", 8192, 768, 2304), ("bert.o", 8192, 768, 768), ("bert.ffn1", 8192, 768, 3072),
          ("bert.ffn2", 8192, 3072, 768), ("bert512.ffn1", 65536, 768, 3072), ("bert512.ffn2", 65536, 3072, 768)]


def t_us(fn, it=20):
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
    ap.add_argument("--label", default=os.environ.get("PSD_GEMM_BIG", "2"))
    a = ap.parse_args()
    C = native()
    dev = torch.device("cuda")
    for name, M, K, N in SHAPES:
        g = torch.Generator(device=dev).manual_seed(0)
        X = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
        W = (torch.rand(N, K, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
        dY = (torch.rand(M, N, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
        Y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        dX = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
        dW = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * M * N * K
        runs = [("fwd NT", lambda: C.gemm_(X, W, True, True, Y), lambda: X.float() @ W.float().t(), Y),
                ("dgrad NN", lambda: C.gemm_(dY, W, True, False, dX), lambda: dY.float() @ W.float(), dX),
                ("wgrad TN", lambda: C.gemm_splitk_(dY, X, False, False, dW, False, 1.0, 0),
                 lambda: dY.float().t() @ X.float(), dW),
                ("blas fwd", lambda: torch.mm(X, W.t()), None, None)]
        if K % 128 == 0:
            from parameter_server_distributed_amd.ops import quantize_fp8

            Xq, sx = quantize_fp8(X)
            Wq, sw = quantize_fp8(W)
            runs.append(("fp8 fwd NT", lambda: C.gemm_fp8_(Xq, Wq, sx, sw, Y),
                         lambda: (Xq.float() * sx) @ (Wq.float() * sw).t(), Y))
        for lay, fn, ref, out in runs:
            us = t_us(fn)
            err = ""
            if ref is not None and M * N * K <= 8192 * 3072 * 768 * 4:
                fn()
                r = ref()
                err = f"{((out.float() - r).abs().max() / r.abs().max()).item():.2e}"
            print(f"| {a.label} | {name} | {M}x{K}x{N} | {lay} | {us:.1f} | {fl / us / 1e6:.0f} | {err} |", flush=True)
        del X, W, dY, Y, dX, dW
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
