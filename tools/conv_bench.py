#!/usr/bin/env python3
"""Per-shape timing of every ResNet-50 convolution (batch 256, NHWC bf16) on MI355X:
MIOpen (F.conv2d + autograd: fwd, bwd-data, bwd-weight) vs the GEMM formulation of the 1x1 convs
(torch.mm -> hipBLASLt on the [N*H*W, C] view). Prints a markdown table with TFLOP/s.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from parameter_server_distributed_amd.utils import miopen as _m  # noqa: E402

_m.install()
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def shapes(batch):
    out = []  # (name, cin, cout, k, stride, H_in, count)
    out.append(("stem7x7", 3, 64, 7, 2, 224, 1))
    H = 56
    cin = 64
    for li, (planes, blocks, stride) in enumerate([(64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)]):
        for b in range(blocks):
            s = stride if b == 0 else 1
            Hin = H
            Hout = H // s
            out.append((f"l{li+1}b{b}.c1", cin, planes, 1, 1, Hin, 1))
            out.append((f"l{li+1}b{b}.c2", planes, planes, 3, s, Hin, 1))
            out.append((f"l{li+1}b{b}.c3", planes, planes * 4, 1, 1, Hout, 1))
            if b == 0:
                out.append((f"l{li+1}b{b}.ds", cin, planes * 4, 1, s, Hin, 1))
            cin = planes * 4
            H = Hout
    # merge identical configs
    merged = {}
    for n, ci, co, k, s, h, c in out:
        key = (ci, co, k, s, h)
        if key in merged:
            merged[key][1] += 1
        else:
            merged[key] = [n, 1]
    return [(v[0], *k, v[1]) for k, v in merged.items()]


def timeit(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--benchmark", type=int, default=1)
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = bool(a.benchmark)
    dev = torch.device("cuda")
    B = a.batch
    tot = {"fwd": 0.0, "bwd": 0.0, "gemm": 0.0}
    print("| conv | cin | cout | k | s | H | n | fwd us | fwd TF | bwd(d+w) us | bwd TF | 1x1 GEMM fwd+bwd us |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    for name, ci, co, k, s, h, n in shapes(B):
        x = torch.randn(B, ci, h, h, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(co, ci, k, k, device=dev, dtype=torch.bfloat16) * 0.05).contiguous(
            memory_format=torch.channels_last)
        x.requires_grad_(True)
        w.requires_grad_(True)
        y = F.conv2d(x, w, stride=s, padding=k // 2)
        gy = torch.randn_like(y)
        ho = y.shape[2]
        flops = 2.0 * B * ho * ho * co * ci * k * k
        tf = timeit(lambda: F.conv2d(x, w, stride=s, padding=k // 2))

        def bwd():
            yy = F.conv2d(x, w, stride=s, padding=k // 2)
            torch.autograd.grad(yy, (x, w), gy)

        tb = timeit(bwd) - tf
        g = ""
        if k == 1 and s == 1:
            X = x.detach().permute(0, 2, 3, 1).reshape(-1, ci)
            W = w.detach().reshape(co, ci)
            GY = gy.permute(0, 2, 3, 1).reshape(-1, co)

            def gemm():
                torch.mm(X, W.t())
                torch.mm(GY, W)
                torch.mm(GY.t(), X)

            tg = timeit(gemm)
            g = f"{tg:.0f}"
            tot["gemm"] += tg * n
        else:
            tot["gemm"] += (tf + tb) * n
        tot["fwd"] += tf * n
        tot["bwd"] += tb * n
        print(f"| {name} | {ci} | {co} | {k} | {s} | {h} | {n} | {tf:.0f} | {flops / tf / 1e6:.0f} | {tb:.0f} | "
              f"{2 * flops / tb / 1e6:.0f} | {g} |", flush=True)
    print(f"\ntotal conv fwd {tot['fwd'] / 1e3:.2f} ms, bwd {tot['bwd'] / 1e3:.2f} ms; "
          f"with 1x1 as hipBLASLt GEMMs: {tot['gemm'] / 1e3:.2f} ms (fwd+bwd)")


if __name__ == "__main__":
    main()
