#!/usr/bin/env python3
"""Per-kernel sums of the query-path PMC passes (scripts/qprofile_pmc.sh <tag>): for the
interpreter's short runs (sieve_kernel, 256-row grids) and the guided generator, each counter
summed over dispatches, plus derived per-wave ratios.  Prints one JSON object.

    python scripts/summarize_qpmc.py <tag>
"""
import collections
import csv
import glob
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kind(name, grid):
    if "sieve_kernel" in name:  # first rounds (256 rows before round 5, 4096 since)
        g = int(grid)
        return "sieve_256" if g <= 256 else "sieve_4096" if g <= 4096 else "sieve_long"
    if "guided" in name:
        return "generate"
    return None


def main():
    tag = sys.argv[1]
    base = os.path.join(HERE, "gpurun_out", "qpmc_" + tag)
    sums = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in glob.glob(os.path.join(base, "*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = kind(r.get("Kernel_Name", ""), r.get("Grid_Size", r.get("Grid_Size_X", "0")))
            if k is None:
                continue
            sums[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[(k, r["Counter_Name"])].add(r.get("Dispatch_Id"))
    out = {}
    for k, c in sums.items():
        d = dict(c)
        d["dispatches"] = max(len(v) for (kk, _), v in disp.items() if kk == k)
        w = d.get("SQ_WAVES") or 0
        if w:
            for n in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_LDS",
                      "SQ_INSTS_BRANCH", "SQ_WAVE_CYCLES", "SQ_INSTS_VMEM_RD"):
                if n in d:
                    d[n + "_per_wave"] = d[n] / w
        if d.get("SQ_WAVE_CYCLES"):
            for n in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_SCA",
                      "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
                if n in d:
                    d[n + "_frac"] = d[n] / d["SQ_WAVE_CYCLES"]
        if d.get("SQC_DCACHE_REQ"):
            d["dcache_hit_rate"] = d.get("SQC_DCACHE_HITS", 0) / d["SQC_DCACHE_REQ"]
        out[k] = d
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
