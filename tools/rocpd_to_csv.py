#!/usr/bin/env python3
"""rocprofv3's SQLite output (``run_results.db``, the default ``rocpd`` format) -> the
``kernel_trace.csv`` columns tools/prof_summary.py and tools/roofline.py read (Kernel_Name,
Start/End_Timestamp, Stream_Id, Queue_Id, Dispatch_Id, Grid/Workgroup sizes, register counts).

  python tools/rocpd_to_csv.py run_results.db kernel_trace.csv.gz
"""
import csv
import gzip
import sqlite3
import sys

COLS = [("Kernel_Name", "name"), ("Dispatch_Id", "dispatch_id"), ("Stream_Id", "stream_id"),
        ("Queue_Id", "queue_id"), ("Start_Timestamp", "start"), ("End_Timestamp", "end"),
        ("Grid_Size_X", "grid_x"), ("Grid_Size_Y", "grid_y"), ("Grid_Size_Z", "grid_z"),
        ("Workgroup_Size_X", "workgroup_x"), ("Workgroup_Size_Y", "workgroup_y"),
        ("Workgroup_Size_Z", "workgroup_z"), ("LDS_Block_Size", "lds_size"), ("Scratch_Size", "scratch_size"),
        ("VGPR_Count", "vgpr_count"), ("Accum_VGPR_Count", "accum_vgpr_count"), ("SGPR_Count", "sgpr_count")]


def main():
    src, dst = sys.argv[1], sys.argv[2]
    con = sqlite3.connect(src)
    q = "select " + ", ".join(c for _, c in COLS) + " from kernels order by start"
    op = gzip.open if dst.endswith(".gz") else open
    n = 0
    with op(dst, "wt", newline="") as f:
        w = csv.writer(f)
        w.writerow([h for h, _ in COLS])
        for row in con.execute(q):
            w.writerow(row)
            n += 1
    print(f"{n} kernel dispatches -> {dst}")


if __name__ == "__main__":
    main()
