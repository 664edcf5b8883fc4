#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace into a per-training-step breakdown (markdown).

Step boundaries are the `optim_advance` marker kernel (one per PS step). The last `--steps`
complete steps are summarised: total kernel-busy ms per step and the top kernels by share.

  python tools/prof_summary.py <kernel_trace.csv[.gz]> --steps 10 --title "..." > out.md
"""
import argparse
import collections
import csv
import gzip
import re


def short(name: str) -> str:
    n = re.sub(r"\(.*", "", name.replace("(anonymous namespace)", "anon"))
    n = n.replace("void ", "")
    if len(n) > 110:
        n = n[:107] + "..."
    return n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--title", default="kernel breakdown")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--marker", default="optim_advance")
    a = ap.parse_args()
    op = gzip.open if a.trace.endswith(".gz") else open
    with op(a.trace, "rt") as f:
        rows = list(csv.DictReader(f))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    if len(marks) < a.steps + 1:
        raise SystemExit(f"only {len(marks)} markers found")
    lo, hi = marks[-(a.steps + 1)], marks[-1]
    win = rows[lo:hi]
    t0, t1 = int(win[0]["Start_Timestamp"]), int(win[-1]["Start_Timestamp"])
    agg = collections.defaultdict(lambda: [0, 0])
    busy = 0
    for r in win:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        busy += d
        agg[short(r["Kernel_Name"])][0] += d
        agg[short(r["Kernel_Name"])][1] += 1
    S = a.steps
    print(f"# {a.title}\n")
    print(f"- window: last {S} steps, wall {(t1 - t0) / 1e6 / S:.2f} ms/step, kernel-busy {busy / 1e6 / S:.2f} ms/step, "
          f"{len(win) / S:.0f} kernels/step\n")
    cats = collections.defaultdict(lambda: [0, 0])
    for n, (d, c) in agg.items():
        cats[category(n)][0] += d
        cats[category(n)][1] += c
    print("| category | share | calls/step | ms/step |\n|---|---:|---:|---:|")
    for n, (d, c) in sorted(cats.items(), key=lambda kv: -kv[1][0]):
        print(f"| {n} | {d / busy * 100:.1f}% | {c / S:.1f} | {d / 1e6 / S:.3f} |")
    print()
    print("| share | calls/step | avg us | ms/step | kernel |\n|---:|---:|---:|---:|---|")
    for n, (d, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[: a.top]:
        print(f"| {d / busy * 100:.1f}% | {c / S:.1f} | {d / c / 1e3:.1f} | {d / 1e6 / S:.3f} | `{n}` |")


CATEGORIES = [
    ("psd: batchnorm", r"psd::bn_"),
    ("psd: narrow conv (convn / convp / convpr / convh)", r"psd::conv(n|p|pr|h)_kernel"),
    ("psd: narrow conv wgrad (convw / convhw)", r"psd::convh?w_"),
    ("psd: gemm", r"psd::.*(gemm|colsum|splitk)"),
    ("psd: fp8 quantise / amax", r"psd::.*(quant|amax|requant)"),
    ("psd: optimizer / PS apply", r"psd::.*(fused_apply|optim|multi_reduce|pack_cast|f32_to_bf16)"),
    ("psd: other (pool, ...)", r"psd::"),
    ("MIOpen/CK conv fwd", r"conv_fwd|igemm_fwd|fwd_gtc"),
    ("MIOpen/CK conv bwd-data", r"bwd_data|igemm_bwd|bwd_gtc"),
    ("MIOpen/CK conv bwd-weight", r"wrw|bwd_weight"),
    ("CK batched GEMM (1x1 conv)", r"batched_gemm|gemm_xdl"),
    ("hipBLASLt GEMM (1x1 conv fwd/dgrad, fc)", r"^(Custom_)?Cijk_"),
    ("MIOpen tensor ops / fills", r"SubTensorOp|fillBuffer|Transpose|transpose"),
    ("HIP runtime copies", r"__amd_rocclr_copyBuffer"),
    ("torch elementwise / reduce", r"at::native"),
    ("RCCL", r"nccl|rccl"),
]


def category(name: str) -> str:
    for cat, pat in CATEGORIES:
        if re.search(pat, name):
            return cat
    return "other"


if __name__ == "__main__":
    main()
