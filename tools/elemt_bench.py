#!/usr/bin/env python3
"""Achieved bandwidth of the BN elementwise backward pass alone (bn_bwd_elemt_kernel<2> via
bn_elemt_coef: read g and x, write dx) on the ResNet-50 b1024 shapes it runs on, next to torch's
add of two tensors of the same size (same bytes: two reads, one write).

  python tools/elemt_bench.py         -> markdown table (TB/s over the compulsory bytes)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from parameter_server_distributed_amd import native  # noqa: E402


def t_us(fn, it=20):
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
    print("| shape (M x C) | MB per tensor | torch add us (TB/s) | bn_elemt_coef us (TB/s) |")
    print("|---|---:|---:|---:|")
    for M, Ch in [(3211264, 64), (802816, 128), (3211264, 128), (200704, 256), (802816, 256), (50176, 512),
                  (200704, 512)]:
        g = torch.randn(M, Ch, device=dev, dtype=torch.bfloat16)
        x = torch.randn_like(g)
        out = torch.empty_like(g)
        coef = torch.randn(3 * Ch, device=dev)
        nb = g.numel() * 2
        ta = t_us(lambda: torch.add(g, x, out=out))
        te = t_us(lambda: C.bn_elemt_coef(g, x, coef))
        ref = (coef[:Ch] * g.float() + coef[Ch:2 * Ch] * x.float() + coef[2 * Ch:]).to(torch.bfloat16)
        got = C.bn_elemt_coef(g, x, coef)
        assert torch.allclose(got.float(), ref.float(), rtol=1e-2, atol=1e-2)
        tb = lambda t: 3 * nb / t / 1e6  # noqa: E731
        print(f"| {M} x {Ch} | {nb / 1e6:.0f} | {ta:.0f} ({tb(ta):.2f}) | {te:.0f} ({tb(te):.2f}) |", flush=True)
        del g, x, out, ref, got


if __name__ == "__main__":
    main()
