#!/usr/bin/env python3
"""Diagnostic: time mh_run on the config-5 tape set in both modes (first N tapes, 2^18 rows)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mythril_amd import native, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
modes = sys.argv[2].split(",") if len(sys.argv) > 2 else ["count", "first"]
ctx = native.Context(0)
ts = synth.generate(n)
t0 = time.time()
ct = ctx.compile(ts)
print("compile %.2fs fold=%s" % (time.time() - t0, "off" if os.environ.get("MH_NO_FOLD") else "on"),
      flush=True)
rows = int(os.environ.get("DIAG_ROWS", 1 << 18))
a = ctx.assignments(ts.n_vars, rows)
a.generate(synth.load_spec()["assignment_seed"], 0)
for m in modes:
    mode = native.MODE_COUNT_ALL if m == "count" else native.MODE_FIRST_HIT
    t0 = time.time()
    fh, hc = native.run(ctx, ct, a, mode=mode)
    print("%s %.3fs hits=%d" % (m, time.time() - t0, int((fh != native.NO_HIT).sum())), flush=True)
    out = os.environ.get("DIAG_OUT")
    if out:
        import numpy as np
        np.save("%s_%s.npy" % (out, m), np.stack([fh, hc]))
