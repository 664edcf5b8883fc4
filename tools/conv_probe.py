#!/usr/bin/env python3
"""Time the implicit-GEMM NHWC convolution forward (native conv_fwd_) against MIOpen (F.conv2d,
channels_last bf16) on the ResNet-50 / Wide-ResNet-101-2 b1024 shapes it accepts (Cout >= 256)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from parameter_server_distributed_amd import native  # noqa: E402

B = int(os.environ.get("PROBE_BATCH", "1024"))
SHAPES = [  # name, C, H, Cout, R, stride
    ("r50 s3 conv2", 256, 14, 256, 3, 1), ("r50 s4 conv2", 512, 7, 512, 3, 1),
    ("r50 s3 conv2/s2", 256, 28, 256, 3, 2), ("r50 s4 conv2/s2", 512, 14, 512, 3, 2),
    ("r50 s2 down", 256, 56, 512, 1, 2), ("r50 s3 down", 512, 28, 1024, 1, 2), ("r50 s4 down", 1024, 14, 2048, 1, 2),
    ("wrn s2 conv2", 256, 28, 256, 3, 1), ("wrn s3 conv2", 512, 14, 512, 3, 1), ("wrn s4 conv2", 1024, 7, 1024, 3, 1),
]


def t_us(fn, it=10):
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
    print("| shape | Nb | C | HxW | Cout | RxR/s | ours us | TF/s | MIOpen us | TF/s | ours/MIOpen | max err |")
    print("|---|---:|---:|---:|---:|---|---:|---:|---:|---:|---:|---:|")
    for name, C, H, Cout, R, s in SHAPES:
        pad = R // 2
        x = (torch.rand(B, C, H, H, device="cuda") * 2 - 1).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        w = ((torch.rand(Cout, C, R, R, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        w2 = w.permute(0, 2, 3, 1).reshape(Cout, -1).contiguous()
        Ho = (H + 2 * pad - R) // s + 1
        out = torch.empty(B * Ho * Ho, Cout, device="cuda", dtype=torch.bfloat16)
        ours = lambda: native().conv_fwd_(x, w2, out, R, R, s, pad)  # noqa: E731
        lib = lambda: F.conv2d(x, w, stride=s, padding=pad)  # noqa: E731
        assert ours()
        ref = lib().permute(0, 2, 3, 1).reshape(-1, Cout).float()
        err = float(((out.float() - ref).abs().max() / ref.abs().max()).item())
        to, tl = t_us(ours), t_us(lib)
        fl = 2.0 * B * Ho * Ho * Cout * C * R * R
        print(f"| {name} | {B} | {C} | {H} | {Cout} | {R}x{R}/{s} | {to:.0f} | {fl / to / 1e6:.0f} | {tl:.0f} | "
              f"{fl / tl / 1e6:.0f} | {tl / to:.2f} | {err:.1e} |", flush=True)


if __name__ == "__main__":
    main()
