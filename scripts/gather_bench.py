#!/usr/bin/env python3
"""The memory side of lane compaction, measured.

mh_microbench_gather on config 5's column shape (2^26 rows x 4 columns x 256 bits = 128 B per
row): the time to reload every survivor row's columns when 6.5 % of the rows survive the head
test (the measured survival rate, scripts/compaction_study.py), from the sieve's SoA layout and
from a row-major layout, against the streaming read of every row the kernel does today.  One
JSON line per (layout, survival rate).

    python scripts/gather_bench.py [log2_rows=26]
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

from mythril_amd import native  # noqa: E402

LAYOUTS = {0: "soa_gather", 1: "aos_gather", 2: "soa_stream"}


def main():
    log2_rows = int(sys.argv[1]) if len(sys.argv) > 1 else 26
    for layout in (2, 0, 1):
        for permille in ((1000,) if layout == 2 else (65, 200)):
            ms, gbps, n = native.microbench_gather(0, log2_rows, permille, layout, reps=5)
            rows = 1 << log2_rows
            rec = {"layout": LAYOUTS[layout], "rows": rows, "survivor_permille": permille,
                   "survivors": n if layout != 2 else rows, "ms": ms, "useful_GBps": gbps,
                   "ns_per_row": ms * 1e6 / (n if layout != 2 else rows)}
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
