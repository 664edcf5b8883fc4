#!/usr/bin/env python3
"""Layer1 3x3 (64 -> 64, 56 x 56, stride 1) at b1024 on the persistent HALO kernels
(kernels/convn.hip convh_kernel, kernels/convw.hip convhw_kernel) vs the gathered variants and
MIOpen: forward (plain / with the BN statistics epilogue), bwd-data (plain / mode-1 BN backward
epilogue) and the weight gradient. Prints a markdown table of per-call times (torch events); run
under rocprofv3 --kernel-trace --stats for per-kernel times, or --pmc for counters.

    python tools/convh_bench.py [--batch 1024] [--reps 5]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from parameter_server_distributed_amd import native  # noqa: E402
from parameter_server_distributed_amd.utils import miopen as _miopen  # noqa: E402

_miopen.install()


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
    C_ = native()
    dev = torch.device("cuda")
    cl = dict(memory_format=torch.channels_last)
    N, H = a.batch, 56
    M = N * H * H
    torch.manual_seed(0)
    x = torch.randn(N, 64, H, H, device=dev).to(torch.bfloat16).contiguous(**cl)
    dy = torch.randn(N, 64, H, H, device=dev).to(torch.bfloat16).contiguous(**cl)
    w = (torch.randn(64, 64, 3, 3, device=dev) * 0.05).to(torch.bfloat16).contiguous(**cl)
    w2 = w.permute(0, 2, 3, 1).reshape(64, -1).contiguous()
    wf = w.flip(2, 3).permute(1, 2, 3, 0).reshape(64, -1).contiguous()
    kinds = {v: C_.convn_variant_kind(64, v) for v in range(C_.convn_variants(64))}
    pv = [v for v, k in kinds.items() if k == 2][0]
    out = torch.empty(M, 64, device=dev, dtype=torch.bfloat16)
    shift = torch.zeros(64, device=dev)
    rows = lambda v: max(C_.convn_stats_rows(M), C_.convn_part_rows(M, 64, v, H, H, 3))  # noqa: E731
    bx = torch.randn(M, 64, device=dev).to(torch.bfloat16)
    mean = torch.zeros(64, device=dev)
    bss = torch.cat([torch.ones(64), torch.zeros(64)]).to(dev)
    res = []
    gf = 2.0 * M * 64 * 576 / 1e9
    t_mi = timeit(lambda: F.conv2d(x, w, padding=1), a.reps)
    res.append(("fwd MIOpen", t_mi))
    for v in (0, 3, pv):
        res.append((f"fwd psdn{v}", timeit(lambda: C_.convn_(x, w2, out, 3, 3, 1, 1, variant=v), a.reps)))
        part = torch.empty(rows(v), 2, 64, device=dev)
        res.append((f"fwd psdn{v} + stats", timeit(lambda: C_.convn_(x, w2, out, 3, 3, 1, 1, part=part, shift=shift,
                                                                       variant=v), a.reps)))
    for v in (0, pv):
        res.append((f"dgrad psdn{v}", timeit(lambda: C_.convn_(dy, wf, out, 3, 3, 1, 1, variant=v), a.reps)))
        part = torch.empty(rows(v), 2, 64, device=dev)
        res.append((f"dgrad psdnb{v} (mode 1)", timeit(lambda: C_.convn_bwd_(dy, wf, out, 3, 3, 1, 1, part, v, 1, bx,
                                                                             mean, bss=bss), a.reps)))
    wgt = torch.empty(64, 576, device=dev, dtype=torch.bfloat16)
    res.append(("wgrad MIOpen", timeit(lambda: torch.ops.aten.convolution_backward(
        dy, x, w, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False]), a.reps)))
    for v in range(C_.convw_variants(64, 576)):
        res.append((f"wgrad psdw{v}", timeit(lambda: C_.convw_(dy, x, wgt, 3, 3, 1, 1, variant=v), a.reps)))
    # correctness spot checks of the persistent kernels against the gathered ones
    C_.convn_(x, w2, out, 3, 3, 1, 1, variant=0)
    ref = out.clone()
    C_.convn_(x, w2, out, 3, 3, 1, 1, variant=pv)
    assert torch.equal(out, ref)
    C_.convw_(dy, x, wgt, 3, 3, 1, 1, variant=0)
    wref = wgt.float().clone()
    C_.convw_(dy, x, wgt, 3, 3, 1, 1, variant=C_.convw_variants(64, 576) - 1)
    err = float((wgt.float() - wref).norm() / wref.norm())
    assert err < 1e-2, err
    print(f"batch {N}, layer1 3x3 64->64 56x56: {gf:.0f} GFLOP per pass; us per call\n")
    print("| pass | us | TF/s |\n|---|---:|---:|")
    for name, t in res:
        print(f"| {name} | {t:.0f} | {gf / t * 1e3:.0f} |")
    print(f"\npersistent wgrad vs the tiled one: rel. L2 {err:.2e}")


if __name__ == "__main__":
    main()
