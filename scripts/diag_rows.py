#!/usr/bin/env python3
"""Diagnostic: native code vs interpreter on config 5 as the row count grows (2^23..2^26), and
the C oracle on the first tapes where they differ.  One JSON line per size.

    python scripts/diag_rows.py [log2 sizes...]
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

from mythril_amd import native, synth  # noqa: E402
from mythril_amd.tape import TapeSet  # noqa: E402


def main():
    sizes = [int(x) for x in sys.argv[1:]] or [23, 24, 25, 26]
    from oracle import ctape

    ctx = native.Context(0)
    ts = synth.generate()
    seed = synth.load_spec()["assignment_seed"]
    ct = ctx.compile(ts)
    ct.jit()
    ref = ctx.compile(ts)
    for lg in sizes:
        rows = 1 << lg
        a = ctx.assignments(ts.n_vars, rows)
        a.generate(seed, 0)
        t0 = time.time()
        fh, hc = native.run(ctx, ct, a, mode=native.MODE_COUNT_ALL)
        t1 = time.time()
        fh0, hc0 = native.run(ctx, ref, a, mode=native.MODE_COUNT_ALL)
        t2 = time.time()
        bad = np.nonzero((hc != hc0) | (fh != fh0))[0]
        rec = {"rows": rows, "jit_s": t1 - t0, "interp_s": t2 - t1, "n_diff": int(len(bad)),
               "diff": []}
        for t in bad[:3]:
            sub = TapeSet(ts.var_names)
            sub.pool = ts.pool
            sub.tapes = [ts.tapes[int(t)]]
            cnt, first = ctape.count(sub, seed, 0, rows, threads=min(16, os.cpu_count() or 1),
                                     short_circuit=True)
            rec["diff"].append({"tape": int(t), "jit": [int(hc[t]), int(fh[t])],
                                "interp": [int(hc0[t]), int(fh0[t])],
                                "oracle": [int(cnt[0]), int(first[0])]})
        print(json.dumps(rec), flush=True)
        a.close()


if __name__ == "__main__":
    main()
