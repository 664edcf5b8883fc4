#!/usr/bin/env python3
"""fp8 vs bf16 training curves: a short Wide-ResNet (width_per_group 128, two blocks per stage,
fp8 compute on the bottleneck convolutions vs bf16) trained with SGD-momentum on a fixed synthetic
set of 8 batches (so the loss can fall by fitting it), same init, same batch order. Writes the two
loss curves as JSON (one line per 25 steps printed as progress).

  python tools/fp8_convergence.py --steps 300 --out gpurun_out/fp8_conv.json
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from parameter_server_distributed_amd.models import prepare  # noqa: E402
from parameter_server_distributed_amd.models.resnet import ResNet  # noqa: E402
from parameter_server_distributed_amd.ops.loss import cross_entropy  # noqa: E402


def run(fp8: bool, steps: int, batches, dev, lr: float):
    torch.manual_seed(0)
    m = prepare(ResNet((2, 2, 2, 2), num_classes=100, width_per_group=128, fp8=fp8), dev, torch.bfloat16,
                channels_last=True)
    for p in m.parameters():
        p.data = p.data.to(torch.bfloat16)
    m.train()
    # fp32 master weights + momentum in the optimizer (what the PS keeps), bf16 working copy
    master = [p.detach().float().clone() for p in m.parameters()]
    mom = [torch.zeros_like(t) for t in master]
    losses = []
    t0 = time.time()
    for t in range(steps):
        x, y = batches[t % len(batches)]
        loss = cross_entropy(m(x), y)
        for p in m.parameters():
            p.grad = None
        loss.backward()
        with torch.no_grad():
            for p, w, v in zip(m.parameters(), master, mom):
                v.mul_(0.9).add_(p.grad.float() + 5e-5 * w)
                w.add_(v, alpha=-lr)
                p.copy_(w)
        losses.append(float(loss))
        if (t + 1) % 25 == 0:
            print(f"{'fp8' if fp8 else 'bf16'} step {t + 1}: loss {losses[-1]:.4f} ({time.time() - t0:.1f} s)",
                  flush=True)
    return losses


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--lr", type=float, default=0.05)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(1)
    batches = [(torch.randn(a.batch, 3, 64, 64, generator=g).to(dev, torch.bfloat16).contiguous(
        memory_format=torch.channels_last), torch.randint(0, 100, (a.batch,), generator=g).to(dev)) for _ in range(8)]
    res = {"steps": a.steps, "batch": a.batch, "lr": a.lr, "model": "ResNet((2,2,2,2), width_per_group=128), 64x64",
           "bf16": run(False, a.steps, batches, dev, a.lr), "fp8": run(True, a.steps, batches, dev, a.lr)}
    last = lambda L: sum(L[-25:]) / 25  # noqa: E731
    res["final_avg25"] = {"bf16": last(res["bf16"]), "fp8": last(res["fp8"])}
    print(json.dumps(res["final_avg25"]))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f)


if __name__ == "__main__":
    main()
