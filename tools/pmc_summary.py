#!/usr/bin/env python3
"""Sum rocprofv3 --pmc counter_collection CSVs per (kernel, counter) over all dispatches and print
a markdown table plus the derived ratios used in profiles/gemm_pmc_r2.md.

  python tools/pmc_summary.py gpurun_out/gemm_TAG/pass*.csv [--kernel SUBSTR]
"""
import argparse
import collections
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csvs", nargs="+")
    ap.add_argument("--kernel", default="gemm8p", help="substring of the kernel name to keep")
    a = ap.parse_args()
    tot = collections.defaultdict(float)
    names = set()
    disp = collections.defaultdict(set)
    for f in a.csvs:
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "")
            if a.kernel not in k:
                continue
            names.add(re.sub(r"\(.*", "", k)[:90])
            c = r.get("Counter_Name")
            tot[c] += float(r.get("Counter_Value", 0) or 0)
            disp[c].add(r.get("Dispatch_Id"))
    print("kernels:", "; ".join(sorted(names)))
    print()
    print("| counter | sum over dispatches | dispatches |")
    print("|---|---:|---:|")
    for c in sorted(tot):
        print(f"| {c} | {tot[c]:.4g} | {len(disp[c])} |")
    g = lambda n: tot.get(n, 0.0)  # noqa: E731
    print()
    if g("SQ_WAVE_CYCLES"):
        print(f"- waiting (any) / wave cycles: {g('SQ_WAIT_ANY') / g('SQ_WAVE_CYCLES'):.3f}")
        print(f"- waiting on an instruction dependency (any) / wave cycles: {g('SQ_WAIT_INST_ANY') / g('SQ_WAVE_CYCLES'):.3f}")
        print(f"- issuing (active inst any) / wave cycles: {g('SQ_ACTIVE_INST_ANY') / g('SQ_WAVE_CYCLES'):.3f}")
    if g("SQ_LDS_IDX_ACTIVE"):
        print(f"- LDS bank conflict cycles / LDS active cycles: {g('SQ_LDS_BANK_CONFLICT') / g('SQ_LDS_IDX_ACTIVE'):.3f}")
    if g("SQ_WAVE_CYCLES") and g("SQ_WAIT_INST_LDS"):
        print(f"- waiting on LDS / wave cycles: {g('SQ_WAIT_INST_LDS') / g('SQ_WAVE_CYCLES'):.3f}")
    if g("GRBM_GUI_ACTIVE") and g("SQ_VALU_MFMA_BUSY_CYCLES"):
        print(f"- MFMA busy cycles / GPU-busy cycles (summed over units): "
              f"{g('SQ_VALU_MFMA_BUSY_CYCLES') / g('GRBM_GUI_ACTIVE'):.3g}")


if __name__ == "__main__":
    main()
