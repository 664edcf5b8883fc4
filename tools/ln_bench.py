#!/usr/bin/env python3
"""Time the fused residual-add + dropout + LayerNorm kernels (csrc/kernels/layernorm.hip) at the
BERT-base b256 x S128 shape (32,768 rows of 768): us per call and TB/s over the compulsory bytes
(forward: read x, h; write s, y. backward: read dy, s; write dx, dh).

  python tools/ln_bench.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from parameter_server_distributed_amd import native  # noqa: E402


def t_us(fn, it=50):
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
    R, H = 32768, 768
    x = torch.randn(R, H, device=dev).to(torch.bfloat16)
    h = torch.randn_like(x)
    dy = torch.randn_like(x)
    g = torch.ones(H, device=dev, dtype=torch.bfloat16)
    b = torch.zeros(H, device=dev, dtype=torch.bfloat16)
    step = torch.tensor([3], device=dev, dtype=torch.int64)
    nb = x.numel() * 2
    print("| p | fwd us | fwd TB/s | bwd us | bwd TB/s |")
    print("|---:|---:|---:|---:|---:|")
    for p in (0.0, 0.1):
        out = C.ln_fwd(x, h, g, b, 1e-12, p, 5, step)
        y, s, mean, rstd = out[0], out[1], out[2], out[3]
        tf = t_us(lambda: C.ln_fwd(x, h, g, b, 1e-12, p, 5, step))
        tb = t_us(lambda: C.ln_bwd(dy, s, mean, rstd, g, p, 5, step))
        print(f"| {p} | {tf:.1f} | {4 * nb / tf / 1e6:.2f} | {tb:.1f} | {4 * nb / tb / 1e6:.2f} |", flush=True)


if __name__ == "__main__":
    main()
