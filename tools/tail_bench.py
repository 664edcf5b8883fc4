#!/usr/bin/env python3
"""Time the narrow-conv 1x1 passes of the bottleneck tail (ops/tail.py) at ResNet-50 b1024 shapes on
every tile variant (gathered kinds 0 and the persistent 1x1 kind 3): the statistics-only pass, the
BN-apply pass, the plain forward with statistics, and the bwd-data mode-2 epilogue without the BN
input. Markdown table; "GB/s" counts the compulsory HBM bytes of the pass.

  python tools/tail_bench.py [--batch 1024]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from parameter_server_distributed_amd import native  # noqa: E402


def t_us(fn, it=10):
    for _ in range(2):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    a = ap.parse_args()
    C = native()
    dev = torch.device("cuda")
    B = a.batch
    print("| shape | pass | variant (kind) | us | GB/s |\n|---|---|---|---:|---:|")
    for name, hw, cin, cout in (("l1", 56, 64, 256), ("l2", 28, 128, 512), ("l3", 14, 256, 1024)):
        M = B * hw * hw
        x = torch.randn(B, cin, hw, hw, device=dev).relu().bfloat16().contiguous(memory_format=torch.channels_last)
        w = (torch.randn(cout, cin, device=dev) * 0.05).bfloat16()
        res = torch.randn(M, cout, device=dev).bfloat16()
        out = torch.empty(M, cout, device=dev, dtype=torch.bfloat16)
        mb = torch.empty(M * cout // 8, device=dev, dtype=torch.uint8)
        ss = torch.randn(2 * cout, device=dev)
        shift = torch.zeros(cout, device=dev)
        dy = torch.randn(B, cin, hw, hw, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
        wt = w.t().contiguous()  # [cin, cout]: dgrad of a cout -> cin 1x1 is this "conv" with N = cout
        wd = w  # dX[M, cout] = dY[M, cin] . w  -> narrow conv with w2 = w^T^T: [cout, cin]
        mean = torch.randn(cout, device=dev)
        bits = torch.randint(0, 255, (M * cout // 8,), device=dev, dtype=torch.uint8)
        dr = torch.randn(M, cout, device=dev).bfloat16()
        ain, aout = M * cin * 2, M * cout * 2
        ref = None
        if C.convw_gram_rows(cin) > 0:
            P = torch.empty(C.convw_gram_rows(cin), cin, device=dev)
            grow = torch.empty(2, cout, device=dev)
            us = t_us(lambda: C.convw_gram_(x, P))
            print(f"| {name} | Gram launch (x^T x, 1^T x) | - | {us:.0f} | {ain / us / 1e3:.0f} |")
            us = t_us(lambda: C.bnfold_gram_stats(P, w, shift, M, grow))
            print(f"| {name} | W^T G W per channel | - | {us:.0f} | - |")
        for v in range(C.convn_variants(cout)):
            kind = C.convn_variant_kind(cout, v)
            if kind not in (0, 3) or not C.convn_variant_ok(cout, v, 1, 1, 1, 0, hw):
                continue
            rows = max(C.convn_stats_rows(M), C.convn_part_rows(M, cout, v, hw, hw, 1)) + 1
            part = torch.empty(rows, 2, cout, device=dev)
            tag = f"{v} ({kind})"
            us = t_us(lambda: C.convn_(x, w, part, 1, 1, 1, 0, part=part, shift=shift, variant=v, no_store=True))
            print(f"| {name} | stats-only | {tag} | {us:.0f} | {ain / us / 1e3:.0f} |")
            us = t_us(lambda: C.convn_(x, w, out, 1, 1, 1, 0, variant=v, apply_ss=ss, apply_res=res, apply_mask=mb))
            print(f"| {name} | apply | {tag} | {us:.0f} | {(ain + 2 * aout + aout // 16) / us / 1e3:.0f} |")
            if ref is None:
                ref = out.clone()
            else:
                assert torch.equal(out, ref), f"{name} apply variant {v} differs from the first variant"
            us = t_us(lambda: C.convn_(x, w, out, 1, 1, 1, 0, part=part, shift=shift, variant=v))
            print(f"| {name} | fwd + stats | {tag} | {us:.0f} | {(ain + aout) / us / 1e3:.0f} |")
            us = t_us(lambda: C.convn_bwd_(dy, wd, out, 1, 1, 1, 0, part, v, 2, None, mean, bdr=dr, bmbits=bits))
            print(f"| {name} | dgrad mode 2 (no bx) | {tag} | {us:.0f} | {(ain + 2 * aout + aout // 16) / us / 1e3:.0f} |")
        del x, res, out, dr
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
