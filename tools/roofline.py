#!/usr/bin/env python3
"""Per-kernel roofline table of a training step from rocprofv3 PMC passes over bench.py
(VERDICT r5 item 5): achieved TF/s (bf16 MFMA) and TB/s (HBM) per kernel vs the MI355X roofs, and
the dominant stall.

Inputs: the counter_collection.csv of each PMC pass (one run per counter group, the same pinned
autotune decisions in every run: PSD_AUTOTUNE_SAVE / PSD_AUTOTUNE_FILE) and the kernel trace of one
of them. Every pass is cut to its last ``--steps`` training steps (the ``optim_advance`` marker
kernel, one per PS step, as tools/prof_summary.py) and summed per kernel name, per step.

Derived (per kernel, per step):
* time: from the kernel trace window, ms/step;
* TF/s = SQ_INSTS_VALU_MFMA_MOPS_BF16 x 512 FLOP / time (one bf16 MFMA "MOP" = 512 FLOP: the
  v_mfma_f32_16x16x32_bf16 count of a GEMM of known size, profiles/gemm_pmc_r2.md);
* TB/s = (2 x FETCH_SIZE + WRITE_SIZE) KiB / time (gfx950 FETCH_SIZE tallies wide streaming reads
  at half their bytes: MI355X_MICROARCH.md);
* wait / issue-stall shares of wave cycles (SQ_WAIT_ANY, SQ_WAIT_INST_ANY over SQ_WAVE_CYCLES), LDS
  bank-conflict cycles over LDS-array cycles.

  python tools/roofline.py --trace run_kernel_trace.csv pass1.csv pass2.csv pass3.csv [--min-ms 1]
"""
import argparse
import collections
import csv
import gzip
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import category, short  # noqa: E402

PEAK_TF = 2500.0  # bf16 dense MFMA, MI355X
PEAK_TBS = 8.0    # HBM3E


def _rows(path):
    op = gzip.open if path.endswith(".gz") else open
    with op(path, "rt") as f:
        return list(csv.DictReader(f))


def _window(names_in_order, steps, marker):
    """Indices [lo, hi) of the last ``steps`` complete steps in a dispatch-ordered name list."""
    marks = [i for i, n in enumerate(names_in_order) if marker in n]
    if len(marks) < steps + 1:
        raise SystemExit(f"only {len(marks)} step markers ({marker}) found")
    return marks[-(steps + 1)], marks[-1]


def counters(path, steps, marker):
    """{kernel: {counter: per-step sum}} over the last ``steps`` steps of one PMC pass."""
    rows = _rows(path)
    disp = {}
    for r in rows:
        d = int(r["Dispatch_Id"])
        disp.setdefault(d, [r["Kernel_Name"], {}])[1][r["Counter_Name"]] = float(r["Counter_Value"] or 0)
    order = sorted(disp)
    lo, hi = _window([disp[d][0] for d in order], steps, marker)
    out = collections.defaultdict(lambda: collections.defaultdict(float))
    for d in order[lo:hi]:
        name, cs = disp[d]
        for c, v in cs.items():
            out[short(name)][c] += v / steps
    return out


def times(path, steps, marker):
    rows = sorted(_rows(path), key=lambda r: int(r["Start_Timestamp"]))
    lo, hi = _window([r["Kernel_Name"] for r in rows], steps, marker)
    t = collections.defaultdict(float)
    n = collections.defaultdict(int)
    for r in rows[lo:hi]:
        k = short(r["Kernel_Name"])
        t[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 / steps
        n[k] += 1
    wall = (int(rows[hi]["Start_Timestamp"]) - int(rows[lo]["Start_Timestamp"])) / 1e6 / steps
    return t, n, wall


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("passes", nargs="+")
    ap.add_argument("--trace", required=True)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--marker", default="optim_advance")
    ap.add_argument("--min-ms", type=float, default=1.0)
    ap.add_argument("--title", default="roofline")
    a = ap.parse_args()
    t, n, wall = times(a.trace, a.steps, a.marker)
    cs = collections.defaultdict(dict)
    for p in a.passes:
        for k, d in counters(p, a.steps, a.marker).items():
            cs[k].update(d)
    busy = sum(t.values())
    print(f"# {a.title}\n")
    print(f"- {a.steps} steps under rocprofv3 --pmc: wall {wall:.2f} ms/step, kernel-busy {busy:.2f} ms/step; "
          f"roofs {PEAK_TF:.0f} TF/s bf16 dense, {PEAK_TBS:.0f} TB/s HBM")
    print("- TF/s from SQ_INSTS_VALU_MFMA_MOPS_BF16 x 512; TB/s = (2 x FETCH_SIZE + WRITE_SIZE) / time; "
          "wait = SQ_WAIT_ANY / SQ_WAVE_CYCLES (parked on s_waitcnt / barrier), "
          "issue = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES, LDS-cf = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE\n")
    print("| kernel | category | calls/step | ms/step | TF/s | % bf16 peak | TB/s | % HBM | wait | issue | LDS-cf | bound |")
    print("|---|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|---|")
    for k in sorted(t, key=lambda k: -t[k]):
        if t[k] < a.min_ms:
            continue
        c = cs.get(k, {})
        sec = t[k] / 1e3
        tf = c.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0.0) * 512 / sec / 1e12 if sec else 0.0
        by = (2 * c.get("FETCH_SIZE", 0.0) + c.get("WRITE_SIZE", 0.0)) * 1024
        tbs = by / sec / 1e12 if sec else 0.0
        wc = c.get("SQ_WAVE_CYCLES", 0.0)
        wait = c.get("SQ_WAIT_ANY", 0.0) / wc if wc else float("nan")
        iss = c.get("SQ_WAIT_INST_ANY", 0.0) / wc if wc else float("nan")
        lds = c.get("SQ_LDS_IDX_ACTIVE", 0.0)
        cf = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / lds if lds else float("nan")
        fc, fb = tf / PEAK_TF, tbs / PEAK_TBS
        bound = "MFMA" if fc >= fb and fc > 0.3 else ("HBM" if fb > 0.5 else ("latency / sync" if wait > 0.5 else "issue"))
        print(f"| `{k[:80]}` | {category(k)} | {n[k] / a.steps:.0f} | {t[k]:.2f} | {tf:.0f} | {fc * 100:.0f} % | "
              f"{tbs:.2f} | {fb * 100:.0f} % | {wait:.2f} | {iss:.2f} | {cf:.3f} | {bound} |")


if __name__ == "__main__":
    main()
