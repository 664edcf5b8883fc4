#!/usr/bin/env python3
"""Time the fused attention kernels (csrc/kernels/attention.hip) at BERT-base pre-training shape
(B 256, S 128, 12 heads of 64) with and without attention dropout: us per call, the compulsory HBM
bytes over that time, and the MFMA rate.

  python tools/attn_bench.py
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
    B, S, H, D = 256, 128, 12, 64
    qkv = (torch.randn(B, S, 3 * H * D, device=dev) * 0.5).to(torch.bfloat16)
    do = torch.randn(B, S, H * D, device=dev).to(torch.bfloat16)
    step = torch.tensor([3], device=dev, dtype=torch.int64)
    el = B * S * H * D * 2  # bytes of one [B, S, H, 64] bf16 tensor
    flop_f = 4 * B * H * S * S * D
    print("| p | fwd us | fwd TB/s | fwd TF/s | bwd us | bwd TB/s | bwd TF/s |")
    print("|---:|---:|---:|---:|---:|---:|---:|")
    for p in (0.0, 0.1):
        o, lse = C.attn_fwd(qkv, H, p, 7, step)
        tf = t_us(lambda: C.attn_fwd(qkv, H, p, 7, step))
        tb = t_us(lambda: C.attn_bwd(do, qkv, o, lse, H, p, 7, step, None))
        # fwd: read q, k, v; write o (+ lse). bwd: read q, k, v, o, dO; write dq, dk, dv
        print(f"| {p} | {tf:.1f} | {4 * el / tf / 1e6:.2f} | {flop_f / tf / 1e6:.0f} | {tb:.1f} | "
              f"{8 * el / tb / 1e6:.2f} | {2.5 * flop_f / tb / 1e6:.0f} |", flush=True)


if __name__ == "__main__":
    main()
