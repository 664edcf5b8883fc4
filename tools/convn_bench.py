"""Time the narrow-output implicit-GEMM convolution (kernels/convn.hip) against MIOpen / hipBLASLt
on the ResNet-50 b1024 layer1/layer2 shapes (forward, and bwd-data as conv(dY, W') where the
kernel takes it). Prints a markdown table; run on the GPU box:

    python tools/convn_bench.py --batch 1024
"""
from __future__ import annotations

import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from parameter_server_distributed_amd import native  # noqa: E402
from parameter_server_distributed_amd.utils import miopen as _miopen  # noqa: E402

_miopen.install()  # the bench's MIOpen setup: shipped find-db, immediate mode

SHAPES = [  # name, C, H, Cout, R, stride
    ("l1.conv1 1x1 64->64", 64, 56, 64, 1, 1),
    ("l1.conv1 1x1 256->64", 256, 56, 64, 1, 1),
    ("l1.conv2 3x3 64->64", 64, 56, 64, 3, 1),
    ("l1.conv3 1x1 64->256", 64, 56, 256, 1, 1),
    ("l2.conv1 1x1 256->128", 256, 56, 128, 1, 1),
    ("l2.conv2 3x3/2 128->128", 128, 56, 128, 3, 2),
    ("l2.conv1 1x1 512->128", 512, 28, 128, 1, 1),
    ("l2.conv2 3x3 128->128", 128, 28, 128, 3, 1),
    ("l2.conv3 1x1 128->512", 128, 28, 512, 1, 1),
    ("l2.ds 1x1/2 256->512", 256, 56, 512, 1, 2),
    ("l3.conv2 3x3 256->256", 256, 14, 256, 3, 1),
    ("l4.conv2 3x3 512->512", 512, 7, 512, 3, 1),
    ("l3.conv3 1x1 256->1024", 256, 14, 1024, 1, 1),
]


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.backends.cudnn.benchmark = False
    C_ = native()
    print(f"batch {a.batch}; times in us (HBM bytes = x + y once)\n")
    print("| shape | M | GFLOP | MB | miopen fwd | convn fwd per variant | best | convn+stats (best) | MIOpen+bn_reduce | TF/s | GB/s |")
    print("|---|---:|---:|---:|---:|---|---:|---:|---:|---:|---:|")
    for name, C, H, Cout, R, stride in SHAPES:
        pad = R // 2
        x = torch.randn(a.batch, C, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(Cout, C, R, R, device=dev) * 0.05).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        w2 = w.permute(0, 2, 3, 1).reshape(Cout, -1).contiguous()
        Ho = (H + 2 * pad - R) // stride + 1
        M = a.batch * Ho * Ho
        out = torch.empty(M, Cout, device=dev, dtype=torch.bfloat16)
        rows = C_.convn_stats_rows(M)
        part = torch.empty(rows, 2, Cout, device=dev)
        shift = torch.zeros(Cout, device=dev)
        t_mi = timeit(lambda: F.conv2d(x, w, stride=stride, padding=pad), a.reps)
        ok = C_.convn_(x, w2, out, R, R, stride, pad)
        tv = {}
        for v in range(C_.convn_variants(Cout) if ok else 0):
            if not C_.convn_variant_ok(Cout, v, R, R, stride, pad, Ho):
                continue
            tv[v] = timeit(lambda: C_.convn_(x, w2, out, R, R, stride, pad, variant=v), a.reps)
        best = min(tv, key=tv.get) if tv else 0
        t_cn = tv[best] if tv else float("nan")
        part = torch.empty(max(rows, C_.convn_part_rows(M, Cout, best, Ho, Ho, R)), 2, Cout, device=dev)
        t_cs = timeit(lambda: C_.convn_(x, w2, out, R, R, stride, pad, part=part, shift=shift, variant=best),
                      a.reps) if ok else float("nan")
        y = F.conv2d(x, w, stride=stride, padding=pad)
        t_red = timeit(lambda: C_.bn_reduce_(y, shift), a.reps)
        if ok:
            C_.convn_(x, w2, out, R, R, stride, pad, variant=best)
            ref = y.permute(0, 2, 3, 1).reshape(M, Cout).float()
            err = float((out.float() - ref).abs().max()) / max(float(ref.abs().max()), 1e-6)
            assert err < 2e-2, (name, err)
        gf = 2.0 * M * Cout * R * R * C / 1e9
        mb = (x.numel() + M * Cout) * 2 / 1e6
        vs = " / ".join(f"v{v}:{t:.0f}" for v, t in tv.items())
        print(f"| {name} | {M} | {gf:.0f} | {mb:.0f} | {t_mi:.0f} | {vs} | v{best} {t_cn:.0f} | {t_cs:.0f} | {t_mi + t_red:.0f} | "
              f"{gf / t_cn * 1e3:.0f} | {mb / t_cn * 1e3:.0f} |", flush=True)
        del x, w, w2, out, y, part


if __name__ == "__main__":
    main()
