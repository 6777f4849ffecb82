#!/usr/bin/env python3
"""Settles the integer VALU peak of SURVEY.md §8d on the box: mh_microbench_issue for every
instruction kind at 1, 2, 4 and 8 waves per SIMD.  Prints one JSON object:
  {kind: {waves: lane-ops/s}}, plus the derived cycles per wave64 instruction per SIMD at the
  nominal 2.4 GHz clock (cycles = 1024 SIMDs x 2.4e9 x 64 / rate).

    python scripts/valu_peak.py [kind names...] > profiles/<tag>/valu_peak.json
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mythril_amd import native  # noqa: E402


def main():
    ctx = native.Context(0)
    out = {"clock_ghz_nominal": 2.4, "simds": 1024, "kinds": {}}
    only = set(sys.argv[1:])
    for kind, name in enumerate(native.MB_KINDS):
        if only and name not in only:
            continue
        row = {}
        for waves in (1, 2, 4, 8):
            r = ctx.microbench(kind, waves)
            row[str(waves)] = {"lane_ops_per_s": r,
                               "cycles_per_wave_insn": 1024 * 2.4e9 * 64 / r}
        out["kinds"][name] = row
        print(name, {w: round(v["cycles_per_wave_insn"], 2) for w, v in row.items()},
              file=sys.stderr, flush=True)
    ctx.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
