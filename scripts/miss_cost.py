#!/usr/bin/env python3
"""What a sieve miss costs, per stage, on the device.

For the UNSAT variants of the largest LASER shapes (tests/laser_like.py hard_queries) and, for
reference, their SAT originals: Sieve.solve timed per stage (lower / guide / tapes / compile /
generate / run / download) with the default rounds, plus, per query tape set, what native code
would cost instead of the interpreter on the 2^16-row rounds: the mh_tapes_jit build (comgr
assembly + module load) and the device time of one 2^16-row FIRST_HIT run on each engine.
One JSON line per query.

    python scripts/miss_cost.py [reps]
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

from mythril_amd import native  # noqa: E402
from mythril_amd.sieve import Sieve  # noqa: E402
from tests.laser_like import hard_queries, queries, query_tapeset  # noqa: E402


def timed_run(ctx, ct, a, rows, reps):
    native.run(ctx, ct, a, mode=native.MODE_FIRST_HIT, row_count=rows)  # warm
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        native.run(ctx, ct, a, mode=native.MODE_FIRST_HIT, row_count=rows)
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    s = Sieve()
    ctx0, qs0 = queries()
    s.solve(ctx0.b, [c.node for c in qs0[0][1]])  # process warm-up (runtime, code objects)
    want = {"killbilly", "overflow", "k_storage"}
    todo = [("sat", n, cs, ctx0) for n, cs in qs0 if n in want]
    ctx1, qs1 = hard_queries()
    todo += [("unsat", n, cs, ctx1) for n, cs in qs1]
    for kind, name, cs, qctx in todo:
        rec = {"query": name, "kind": kind, "constraints": len(cs)}
        ms = []
        for _ in range(reps):
            before = dict(s.stats.stage_s)
            r0 = s.stats.rounds
            t0 = time.perf_counter()
            w = s.solve(qctx.b, [c.node for c in cs])
            ms.append((time.perf_counter() - t0) * 1e3)
            rec["hit"] = w is not None
            rec["rounds"] = s.stats.rounds - r0
            rec["stages_ms"] = {k: round((v - before.get(k, 0.0)) * 1e3, 3)
                                for k, v in s.stats.stage_s.items()
                                if v - before.get(k, 0.0) > 0}
        rec["ms_median"] = float(np.median(ms))
        rec["ms_all"] = [round(x, 3) for x in ms]
        # the same tape set on both engines over one 2^16-row round
        ts, schema, guide = query_tapeset(qctx.b, cs)
        rec["columns"] = ts.n_vars
        rec["tapes"] = len(ts.tapes)
        rows = s.rows
        a = s.ctx.assignments(max(ts.n_vars, 1), rows)
        a.generate_guided(s.seed, guide, global_base=0, count=rows)
        ref = s.ctx.compile(ts)
        rec["interp_run_ms"] = timed_run(s.ctx, ref, a, rows, reps)
        ct = s.ctx.compile(ts)
        t0 = time.perf_counter()
        info = ct.jit()
        rec["jit_build_ms"] = (time.perf_counter() - t0) * 1e3
        rec["jit_info"] = {k: info[k] for k in ("n_jitted", "n_groups", "n_modules", "max_vgpr",
                                                "code_bytes")}
        rec["jit_run_ms"] = timed_run(s.ctx, ct, a, rows, reps)
        f0, _ = native.run(s.ctx, ref, a, mode=native.MODE_FIRST_HIT, row_count=rows)
        f1, _ = native.run(s.ctx, ct, a, mode=native.MODE_FIRST_HIT, row_count=rows)
        rec["engines_agree"] = bool(np.array_equal(f0, f1))
        for x in (ref, ct, a):
            x.close()
        print(json.dumps(rec), flush=True)
    s.close()


if __name__ == "__main__":
    main()
