#!/usr/bin/env python3
"""Copy one gpu_run.sh tag's results from gpurun_out/<tag>/ into profiles/<tag>/: the JSON / JSONL
results, pytest and smoke transcripts, and for every kernel trace (rocprofv3 --kernel-trace
directory) its per-kernel stats plus the last dispatches as a small CSV (the full traces stay
out of the tree).

    python scripts/collect_run.py <tag> [last_dispatches=80]
"""
import csv
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def tail(src, dst, n):
    rows = list(csv.DictReader(open(src)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    with open(dst, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "grid_x", "grid_y", "duration_us"])
        for r in rows[-n:]:
            w.writerow([r["Kernel_Name"][:80], r["Grid_Size_X"], r["Grid_Size_Y"],
                        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3])


def main():
    tag = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 80
    src = os.path.join(ROOT, "gpurun_out", tag)
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    for f in sorted(os.listdir(src)):
        p = os.path.join(src, f)
        if os.path.isfile(p) and (f.endswith((".json", ".jsonl")) or f.startswith(("pytest", "smoke"))):
            shutil.copy(p, os.path.join(dst, f))
        elif os.path.isdir(p):
            for g in os.listdir(p):
                if g.endswith("_kernel_stats.csv"):
                    shutil.copy(os.path.join(p, g), os.path.join(dst, f + "_kernel_stats.csv"))
                elif g.endswith("_kernel_trace.csv"):
                    tail(os.path.join(p, g), os.path.join(dst, f + "_last_dispatches.csv"), n)
    print(sorted(os.listdir(dst)))


if __name__ == "__main__":
    main()
