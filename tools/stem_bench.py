#!/usr/bin/env python3
"""Time the ResNet stem's gfx950 passes at b1024 (kernels/stem.hip, bn.hip): the forward
(conv + BN statistics, fused BN + ReLU + max-pool) and the backward (pool-fused BN backward
writing dY, then the weight gradient). Prints a markdown table; run it under rocprofv3
--kernel-trace --stats for the per-kernel split (scripts/gpu_stem_bench.sh).

    python tools/stem_bench.py [--batch 1024]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from parameter_server_distributed_amd import native  # noqa: E402


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    C = native()
    dev = torch.device("cuda")
    cl = dict(memory_format=torch.channels_last)
    torch.manual_seed(0)
    N = a.batch
    x = torch.randn(N, 3, 224, 224, device=dev).to(torch.bfloat16).contiguous(**cl)
    w = (torch.randn(64, 3, 7, 7, device=dev) * 0.1).to(torch.bfloat16).contiguous(**cl)
    g = torch.empty(64, device=dev).uniform_(0.5, 1.5).to(torch.bfloat16)
    b = torch.empty(64, device=dev).uniform_(-0.5, 0.5).to(torch.bfloat16)
    rm, rv = torch.zeros(64, device=dev), torch.ones(64, device=dev)
    out = {}

    def fwd():
        out["f"] = C.stem_fwd(x, w, g, b, rm, rv, 0.1, 1e-5)

    t_fwd = timeit(fwd, a.reps)
    y, arg, mean, invstd, ss, conv = out["f"]
    gy = torch.randn_like(y)
    gy2 = torch.randn_like(y)

    def bwd2():
        dconv, dg, db = C.bn_pool_bwd(gy, gy2, arg, conv, g, mean, invstd, ss)
        out["b2"] = (C.stem_wgrad(x, dconv), dg, db)

    t_b2 = timeit(bwd2, a.reps)
    print(f"batch {N}; us per call (torch events)\n")
    print("| pass | us |\n|---|---:|")
    print(f"| forward: stem conv + BN stats + BN/ReLU/max-pool | {t_fwd:.0f} |")
    print(f"| backward (bn_pool_bwd writes dY, stem_wgrad) | {t_b2:.0f} |")


if __name__ == "__main__":
    main()
