#!/usr/bin/env python3
"""Query latency against path length (DESIGN §6 length table).

For KillBilly, the transfer overflow and EtherThief grown to n constraints (tests/laser_paths.py:
the base shape plus the dispatcher fall-throughs, calldatasize guards, argument range checks,
SafeMath checks LASER adds along a path), on one Sieve, one JSON line per (shape, n):

* ``ms_laser`` — the path's last query timed after its parent prefixes were solved in LASER
  order (svm.py:257-262; each prefix keyed as frontend.get_model keys it), median of the last 8
  queries of the path, plus the mean over the whole path (``ms_laser_mean``);
* ``ms_cold`` — the full path on fresh terms, nothing solved (or compiled) before;
* ``ms_miss`` — the UNSAT variant's last query in LASER order (what an infeasible JUMPI branch
  pays before z3), and its interpreter time per round (``run`` stage / launches);
* the stages of the last LASER-order solve and the columns / tape nodes of the query.

SIEVE_HOST=python: the Python host stages instead of the native query compiler.

    python scripts/path_scaling.py [lengths=25,50,100,200,400]
"""
import gc
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

from mythril_amd.sieve import Sieve  # noqa: E402
from tests.laser_paths import grow  # noqa: E402


def laser_order(s, ctx, cs, timed_last=8):
    nodes = [c.node for c in cs]
    times, hits = [], []
    for k in range(1, len(nodes) + 1):
        gc.collect() if k > len(nodes) - timed_last else None
        t0 = time.perf_counter()
        w = s.solve(ctx.b, nodes[:k], key=tuple(nodes[:k]))
        times.append((time.perf_counter() - t0) * 1e3)
        hits.append(w is not None)
    return times, hits, w


def main():
    lengths = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "25,50,100,200,400").split(",")]
    s = Sieve(native_query=os.environ.get("SIEVE_HOST", "native") == "native")
    ctx, cs = grow("killbilly", 25)
    s.solve(ctx.b, [c.node for c in cs])  # warm-up: HIP runtime, code object loads
    for name in ("killbilly", "overflow", "ether_thief"):
        for n in lengths:
            rec = {"shape": name, "constraints": n}
            try:
                ctx, cs = grow(name, n)
                s.ctx.clear_cache()  # no code of the previous (shorter) path of this shape
                before = dict(s.stats.stage_s)
                r0 = s.stats.rounds
                times, hits, w = laser_order(s, ctx, cs)
                rec.update(hit=w is not None, prefix_hits=sum(hits),
                           ms_laser=float(np.median(times[-8:])),
                           ms_laser_mean=float(np.mean(times)),
                           ms_laser_max=float(np.max(times)),
                           launches_per_query=(s.stats.rounds - r0) / len(cs),
                           columns=len(w.schema.columns) if w else None)
                rec["stages_ms_per_query"] = {
                    k: round((v - before.get(k, 0.0)) * 1e3 / len(cs), 4)
                    for k, v in s.stats.stage_s.items() if v - before.get(k, 0.0) > 0}
                ctx, cs = grow(name, n)
                s.ctx.clear_cache()  # cold: nothing compiled before either
                gc.collect()
                t0 = time.perf_counter()
                wc = s.solve(ctx.b, [c.node for c in cs])
                rec.update(ms_cold=(time.perf_counter() - t0) * 1e3, hit_cold=wc is not None)
                ctx, cs = grow(name, n, unsat=True)
                nodes = [c.node for c in cs]
                for k in range(1, len(nodes)):
                    s.solve(ctx.b, nodes[:k], key=tuple(nodes[:k]))
                before = dict(s.stats.stage_s)
                r0 = s.stats.rounds
                gc.collect()
                t0 = time.perf_counter()
                wm = s.solve(ctx.b, nodes, key=tuple(nodes))
                rec.update(ms_miss=(time.perf_counter() - t0) * 1e3, miss=wm is None,
                           miss_launches=s.stats.rounds - r0)
                st = {k: (v - before.get(k, 0.0)) * 1e3 for k, v in s.stats.stage_s.items()
                      if v - before.get(k, 0.0) > 0}
                rec["miss_stages_ms"] = {k: round(v, 3) for k, v in st.items()}
                rec["miss_run_ms_per_launch"] = st.get("run", 0.0) / max(1, s.stats.rounds - r0)
            except Exception as e:  # noqa: BLE001 - the record shows it
                import traceback

                rec.update(error="%s: %s" % (type(e).__name__, e),
                           trace=traceback.format_exc().splitlines()[-4:])
            print(json.dumps(rec), flush=True)
    s.close()


if __name__ == "__main__":
    main()
