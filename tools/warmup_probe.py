#!/usr/bin/env python3
"""Where does the first ResNet-50 training step spend its time? (MIOpen Find / kernel compile /
allocator). Times the first forward per convolution (synchronised hooks) and the first backward,
then a second step, and prints the slowest layers.

  python tools/warmup_probe.py [--batch 512] [--benchmark 1]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from parameter_server_distributed_amd.utils import miopen as _m  # noqa: E402

_m.install()
import torch  # noqa: E402

from parameter_server_distributed_amd import models  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--benchmark", type=int, default=1)
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = bool(a.benchmark)
    dev = torch.device("cuda", 0)
    t0 = time.perf_counter()
    spec = models.build("resnet50", dev, torch.bfloat16)
    for p in spec.model.parameters():
        p.data = p.data.to(torch.bfloat16)
    x, y = spec.make_batch(a.batch, dev)
    torch.cuda.synchronize()
    print(f"build {time.perf_counter() - t0:.1f} s", flush=True)
    times = []

    def pre(mod, inp):
        torch.cuda.synchronize()
        mod._t0 = time.perf_counter()

    def post(mod, inp, out):
        torch.cuda.synchronize()
        times.append((time.perf_counter() - mod._t0, mod._name, tuple(inp[0].shape)))

    hs = []
    for n, m in spec.model.named_modules():
        if isinstance(m, torch.nn.Conv2d):
            m._name = n
            hs += [m.register_forward_pre_hook(pre), m.register_forward_hook(post)]
    for step in range(2):
        times.clear()
        t0 = time.perf_counter()
        loss = spec.loss(spec.model(x), y)
        torch.cuda.synchronize()
        tf = time.perf_counter() - t0
        t1 = time.perf_counter()
        loss.backward()
        torch.cuda.synchronize()
        tb = time.perf_counter() - t1
        conv = sum(t for t, _, _ in times)
        print(f"step {step}: forward {tf:.2f} s (convs {conv:.2f} s), backward {tb:.2f} s", flush=True)
        for t, n, s in sorted(times, reverse=True)[:6]:
            print(f"   {t * 1e3:9.1f} ms  {n} {s}", flush=True)
        for p in spec.model.parameters():
            p.grad = None
    for h in hs:
        h.remove()


if __name__ == "__main__":
    main()
