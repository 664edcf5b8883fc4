#!/usr/bin/env python3
"""What the async plane's scatter kernel (kernels/xfer.hip) costs the backward pass it runs beside.

At N > 1 every gradient bucket is pushed by the scatter kernel on the push stream WHILE backward
keeps running on the compute stream, so its workgroups share the CUs with backward's kernels
(never measured). One MI355X cannot cross xGMI, so this measures the
CU-side cost on one device: ResNet-50 forward + backward (the framework's own kernels, batch B) on
the compute stream, alone and with a continuous stream of pushes of a ResNet-50-sized gradient
(split over `--owners` destination segments, like one bucket landing on several owners) on a side
stream, for several workgroup budgets per segment, and the same with hipMemcpyAsync (copy engines:
no CUs). Local HBM takes the pushes far faster than an xGMI link would, so the bytes moved per us
of backward -- and with them the interference -- are an upper bound on the N > 1 case.

  python tools/xfer_interference.py [--batch 256] [--owners 2] [--caps 8,16,32,48,96] [--json out.json]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from parameter_server_distributed_amd import models, native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--owners", type=int, default=2)
    ap.add_argument("--caps", default="8,16,32,48,96")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    C = native()
    torch.manual_seed(0)
    spec = models.build(a.model, dev, torch.bfloat16)
    for p in spec.model.parameters():  # bf16 working weights, as the PS planes give them
        p.data = p.data.to(torch.bfloat16)
    x, y = spec.make_batch(a.batch, dev, seed=0)
    n = sum(p.numel() for p in spec.model.parameters())
    seg = (n // a.owners + 63) // 64 * 64
    src = [torch.randn(seg, device=dev).to(torch.bfloat16) for _ in range(a.owners)]
    dst = [torch.empty_like(s) for s in src]
    side = torch.cuda.Stream(dev)

    def fwd_bwd():
        spec.model.zero_grad(set_to_none=True)
        spec.loss(spec.model(x), y).backward()

    def timed(fn, iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        e.synchronize()
        return s.elapsed_time(e) / iters

    for _ in range(3):  # autotune + warm
        fwd_bwd()
    torch.cuda.synchronize()
    base = min(timed(fwd_bwd, a.iters) for _ in range(2))

    def push(cap):
        if cap == "copy":
            for s_, d_ in zip(src, dst):
                d_.copy_(s_, non_blocking=True)
        else:
            C.xfer_(src, dst, int(cap))

    rows = []
    nbytes = sum(s.nbytes for s in src)
    for cap in ["copy"] + [int(c) for c in a.caps.split(",")]:
        with torch.cuda.stream(side):
            push(cap)
            side.synchronize()
            t_push = timed(lambda: push(cap), 10)  # alone
        # enough pushes queued to cover the whole measured compute window
        k = int(base * a.iters / max(t_push, 1e-3)) + 2
        torch.cuda.synchronize()
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(side):
            ev0.record()
            for _ in range(k):
                push(cap)
            ev1.record()
        t_comp = timed(fwd_bwd, a.iters)
        torch.cuda.synchronize()
        t_side = ev0.elapsed_time(ev1) / k
        rows.append({"cap": cap, "push_alone_ms": round(t_push, 4), "push_alone_GBps": round(nbytes / t_push / 1e6, 1),
                     "push_beside_ms": round(t_side, 4), "push_beside_GBps": round(nbytes / t_side / 1e6, 1),
                     "fwd_bwd_ms": round(t_comp, 3), "slowdown_pct": round((t_comp / base - 1) * 100, 2)})
        print(rows[-1], flush=True)
    out = {"model": a.model, "batch": a.batch, "owners": a.owners, "grad_MB": round(nbytes / 2**20, 1),
           "fwd_bwd_alone_ms": round(base, 3), "rows": rows,
           "note": "one MI355X: destinations are local HBM, not an xGMI peer; pushes run at HBM rate"}
    print("| push path | push alone GB/s | push beside bwd GB/s | fwd+bwd ms | slowdown |")
    print("|---|---:|---:|---:|---:|")
    print(f"| none | - | - | {base:.3f} | - |")
    for r in rows:
        name = "hipMemcpyAsync" if r["cap"] == "copy" else f"xfer kernel, {r['cap']} WG/segment"
        print(f"| {name} | {r['push_alone_GBps']} | {r['push_beside_GBps']} | {r['fwd_bwd_ms']} | {r['slowdown_pct']} % |")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
