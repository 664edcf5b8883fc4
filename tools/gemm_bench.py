#!/usr/bin/env python3
"""Time the MFMA GEMM (NT / NN / TN split-K) against hipBLASLt (torch.mm) and MIOpen 1x1 convs
on ResNet-50 1x1-conv shapes and a square 4096^3 reference. Markdown table out; "roof" is the HBM
time of one GEMM's compulsory traffic at 6 TB/s (these shapes are bandwidth-bound).

  python tools/gemm_bench.py [--batch 1024] [--benchmark 0]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from parameter_server_distributed_amd.utils import miopen as _m  # noqa: E402

_m.install()
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from parameter_server_distributed_amd import native  # noqa: E402


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
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--benchmark", type=int, default=0, help="MIOpen Find (1) or immediate mode (0)")
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = bool(a.benchmark)
    B = a.batch
    C = native()
    dev = torch.device("cuda")
    rows = []
    # (name, tokens M, cin, cout)
    shapes = [("sq4096", 4096, 4096, 4096), ("l1.c1", B * 3136, 256, 64), ("l1.c3", B * 3136, 64, 256),
              ("l2b0.c1", B * 3136, 256, 128),
              ("l2.c1", B * 784, 512, 128), ("l2.c3", B * 784, 128, 512), ("l3b0.c1", B * 784, 512, 256),
              ("l3.c1", B * 196, 1024, 256),
              ("l3.c3", B * 196, 256, 1024), ("l4b0.c1", B * 196, 1024, 512), ("l4.c1", B * 49, 2048, 512),
              ("l4.c3", B * 49, 512, 2048),
              ("bert.qkv", 65536, 768, 2304), ("bert.ffn1", 65536, 768, 3072), ("bert.ffn2", 65536, 3072, 768)]
    print(f"batch {B}, MIOpen {'Find' if a.benchmark else 'immediate mode'}\n")
    print("| shape | M | K(cin) | N(cout) | roof us | fwd ours us (TF) | fwd hipBLASLt | MIOpen fwd/dgrad/wgrad | dgrad ours "
          "| dgrad hipBLASLt | wgrad ours | wgrad hipBLASLt |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    for name, M, K, N in shapes:
        X = torch.randn(M, K, device=dev).to(torch.bfloat16)
        W = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
        dY = torch.randn(M, N, device=dev).to(torch.bfloat16)
        Y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        dX = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
        dW = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * M * N * K
        f_ours = t_us(lambda: C.gemm_(X, W, True, True, Y))
        f_blas = t_us(lambda: torch.mm(X, W.t()))
        d_ours = t_us(lambda: C.gemm_(dY, W, True, False, dX))
        d_blas = t_us(lambda: torch.mm(dY, W))
        w_ours = t_us(lambda: C.gemm_splitk_(dY, X, False, False, dW, False, 1.0, 0))
        w_blas = t_us(lambda: torch.mm(dY.t(), X))
        f_miop = ""
        if name.startswith("l"):
            hw = int(round((M / B) ** 0.5))
            x4 = X.view(B, hw, hw, K).permute(0, 3, 1, 2)
            w4 = W.view(N, K, 1, 1).contiguous(memory_format=torch.channels_last)
            g4 = dY.view(B, hw, hw, N).permute(0, 3, 1, 2)
            cb = torch.ops.aten.convolution_backward
            md = t_us(lambda: cb(g4, x4, w4, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1, [True, False, False]))
            mw = t_us(lambda: cb(g4, x4, w4, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1, [False, True, False]))
            f_miop = f"{t_us(lambda: F.conv2d(x4, w4)):.0f} / d {md:.0f} / w {mw:.0f}"
        tf = lambda us: f"{us:.0f} ({fl / us / 1e6:.0f})"  # noqa: E731
        roof = (M * K + M * N + N * K) * 2 / 6e12 * 1e6
        print(f"| {name} | {M} | {K} | {N} | {roof:.0f} | {tf(f_ours)} | {tf(f_blas)} | {f_miop} | {tf(d_ours)} | {tf(d_blas)} "
              f"| {tf(w_ours)} | {tf(w_blas)} |", flush=True)


if __name__ == "__main__":
    main()
