#!/usr/bin/env python3
"""Achieved HBM bandwidth of the fused BN kernels (csrc/kernels/bn.hip) on ResNet-50 b1024 NHWC
shapes, next to a plain device copy of the same tensor (the streaming roof on this box).

  python tools/bn_bench.py            -> markdown table (GB/s counts compulsory bytes only)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from parameter_server_distributed_amd import native  # noqa: E402


def t_us(fn, it=10):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / it * 1e3


def main():
    C = native()
    dev = torch.device("cuda")
    print("| shape (M x C) | MB | copy us (GB/s) | fwd reduce+apply us (GB/s) | fwd +res+mask us (GB/s) "
          "| bwd mask-x us (GB/s) | bwd res+bits+dy2 us (GB/s) |")
    print("|---|---:|---:|---:|---:|---:|---:|")
    for M, Ch in [(3211264, 256), (3211264, 64), (802816, 512), (802816, 128), (200704, 1024), (200704, 256),
                  (50176, 2048), (50176, 512)]:
        x = torch.randn(M, Ch, device=dev, dtype=torch.bfloat16)
        r = torch.randn_like(x)
        dy = torch.randn_like(x)
        dy2 = torch.randn_like(x)
        g = torch.ones(Ch, device=dev, dtype=torch.bfloat16)
        b = torch.zeros(Ch, device=dev, dtype=torch.bfloat16)
        rm = torch.zeros(Ch, device=dev)
        rv = torch.ones(Ch, device=dev)
        x4 = x.view(M, Ch)
        nb = x.numel() * 2
        out = torch.empty_like(x)
        tc = t_us(lambda: out.copy_(x))
        f1 = lambda: C.bn_fwd(x4, g, b, rm, rv, None, True, True, 0.1, 1e-5, None, None)  # noqa: E731
        f2 = lambda: C.bn_fwd(x4, g, b, rm, rv, r, True, True, 0.1, 1e-5, None, None, mask_out=True)  # noqa: E731
        t1, t2 = t_us(f1), t_us(f2)
        y, mean, invstd, ss, _ = f1()
        _, _, _, _, bits = f2()
        dg = torch.empty(Ch, device=dev, dtype=torch.bfloat16)
        db = torch.empty_like(dg)
        b1 = lambda: C.bn_bwd(dy, x4, None, g, mean, invstd, True, False, dg, db, None, ss, None)  # noqa: E731
        b2 = lambda: C.bn_bwd(dy, x4, None, g, mean, invstd, True, True, dg, db, dy2, None, bits)  # noqa: E731
        t3, t4 = t_us(b1), t_us(b2)
        gbs = lambda passes, t: f"{t:.0f} ({passes * nb / t / 1e3:.0f})"  # noqa: E731
        # compulsory passes: copy 2; fwd 3 (reduce x, apply x -> y); fwd+res 4 (+ r) + bits;
        # bwd mask-x 5 (reduce dy,x; elemt dy,x -> dx); bwd res 7 (reduce dy,dy2,x -> dr; elemt dr,x -> dx)
        print(f"| {M} x {Ch} | {nb / 1e6:.0f} | {gbs(2, tc)} | {gbs(3, t1)} | {gbs(4, t2)} | {gbs(5, t3)} | {gbs(7, t4)} |")
        del x, r, dy, dy2, out, y


if __name__ == "__main__":
    main()
