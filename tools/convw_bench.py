"""Time the narrow implicit-GEMM weight gradient (kernels/convw.hip) against MIOpen's bwd-weight and
the 256-tile split-K GEMM (gemm.hip) on the ResNet-50 b1024 shapes. Prints a markdown table; run on
the GPU box:

    python tools/convw_bench.py --batch 1024
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from parameter_server_distributed_amd import native  # noqa: E402
from parameter_server_distributed_amd.utils import miopen as _miopen  # noqa: E402
from tools.convn_bench import SHAPES, timeit  # noqa: E402

_miopen.install()

MORE = [
    ("l3.conv1 1x1 1024->256", 1024, 14, 256, 1, 1),
    ("l3.conv2 3x3/2 256->256", 256, 28, 256, 3, 2),
    ("l4.conv2 3x3 512->512", 512, 7, 512, 3, 1),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    C_ = native()
    conv_bwd = torch.ops.aten.convolution_backward
    print(f"batch {a.batch}; times in us (HBM bytes = x + dY once)\n")
    print("| shape | M | MB | MIOpen wgrad | gemm.hip igemm wgrad | convw per variant | best | GB/s | vs MIOpen |")
    print("|---|---:|---:|---:|---:|---|---:|---:|---:|")
    for name, C, H, Cout, R, stride in SHAPES + MORE:
        pad = R // 2
        cl = torch.channels_last
        x = torch.randn(a.batch, C, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
        w = torch.zeros(Cout, C, R, R, device=dev, dtype=torch.bfloat16).contiguous(memory_format=cl)
        Ho = (H + 2 * pad - R) // stride + 1
        dy = torch.randn(a.batch, Cout, Ho, Ho, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
        M = a.batch * Ho * Ho
        args = (None, [stride, stride], [pad, pad], [1, 1], False, [0, 0], 1)
        t_mi = timeit(lambda: conv_bwd(dy, x, w, *args, [False, True, False])[1], a.reps)
        o2 = torch.empty(Cout, R * R * C, device=dev, dtype=torch.bfloat16)
        t_ig = float("nan")
        if C_.conv_wgrad_(dy, x, o2, R, R, stride, pad):
            t_ig = timeit(lambda: C_.conv_wgrad_(dy, x, o2, R, R, stride, pad), a.reps)
        out = torch.empty(Cout, R * R * C, device=dev, dtype=torch.bfloat16)
        tv = {}
        for v in range(C_.convw_variants(Cout, R * R * C)):
            if C_.convw_(dy, x, out, R, R, stride, pad, variant=v):
                tv[v] = timeit(lambda: C_.convw_(dy, x, out, R, R, stride, pad, variant=v), a.reps)
        best = min(tv, key=tv.get) if tv else 0
        t_cw = tv[best] if tv else float("nan")
        if tv:
            C_.convw_(dy, x, out, R, R, stride, pad, variant=best)
            ref = conv_bwd(dy, x, w, *args, [False, True, False])[1].float().permute(0, 2, 3, 1).reshape(Cout, -1)
            err = float((out.float() - ref).norm() / ref.norm())
            assert err < 2e-2, (name, err)
        mb = (x.numel() + dy.numel()) * 2 / 1e6
        vs = " / ".join(f"{t:.0f}" for t in tv.values())
        print(f"| {name} | {M} | {mb:.0f} | {t_mi:.0f} | {t_ig:.0f} | {vs} | v{best} {t_cw:.0f} | {mb / t_cw * 1e3:.0f} | "
              f"{t_mi / t_cw:.2f}x |", flush=True)
        del x, w, dy, out, o2


if __name__ == "__main__":
    main()
