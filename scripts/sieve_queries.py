#!/usr/bin/env python3
"""Run the sieve on the LASER-shaped queries of tests/laser_like.py (the SAT shapes and the UNSAT
hard variants) and report, per query, two latencies (medians of SIEVE_QUERY_REPS, default 5):

* ``ms_incremental`` — the query as LASER issues it: every new state's ``is_possible`` extends
  its parent's path condition by one constraint (svm.py:257-262), so the parent prefixes
  cs[:1] .. cs[:-1] are solved first (untimed, with their keys, as frontend.get_model does) on
  fresh terms, then cs is timed (the ctx's compiled-tape cache cleared before the prefixes: it
  holds the parents' tapes, as in LASER, not an earlier repetition's);
* ``ms_cold`` — the same query on fresh terms with nothing solved before it (the first query
  that reads these calldata words / storage slots; compiled-tape cache cleared).

plus hit or miss, launches, per-stage milliseconds of the last timed incremental solve, and any
exception (the front end swallows them to fall back; this script shows them).  One JSON line
per query.  No query is ever timed twice on the same terms (get_model's lru_cache answers a
repeated query before the sieve sees it).  Each timed solve starts after a gc.collect(): every rep
rebuilds all the shapes on a fresh term context, and the collector's pause for that harness garbage
is not the query's.

SIEVE_HOST=python runs the host stages in Python (lower.py / buckets / local_tapeset) instead of
the native query compiler (csrc/query.cpp), for the A/B of DESIGN §6.

    python scripts/sieve_queries.py [rows_per_round]
"""
import gc
import json
import os
import sys
import time
import traceback

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

from mythril_amd.sieve import Sieve  # noqa: E402
from tests.laser_like import hard_queries, queries  # noqa: E402


def fresh(kind, name):
    """The named query built on a new term context (nothing memoised on its nodes)."""
    ctx, qs = (queries() if kind == "sat" else hard_queries())
    return ctx, dict(qs)[name]


def solve(s, ctx, cs, keyed=True):
    nodes = [c.node for c in cs]
    return s.solve(ctx.b, nodes, key=tuple(nodes) if keyed else None)


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 16
    reps = int(os.environ.get("SIEVE_QUERY_REPS", "5"))
    s = Sieve(rows=rows, native_query=os.environ.get("SIEVE_HOST", "native") == "native")
    ctx, qs = queries()
    # warm-up: the first query of a process pays the HIP runtime's lazy initialisation and the
    # code object load; LASER issues thousands of queries per process
    s.solve(ctx.b, [c.node for c in qs[0][1]])
    todo = [("sat", n) for n, _ in qs] + [("unsat", n) for n, _ in hard_queries()[1]]
    for kind, name in todo:
        rec = {"query": name, "kind": kind}
        try:
            inc, cold = [], []
            for _ in range(reps):
                # the ctx keeps compiled tapes by content: a repetition must not reuse the code of
                # the one before (the prefixes below refill it as LASER's parents would)
                s.ctx.clear_cache()
                qctx, cs = fresh(kind, name)
                for k in range(1, len(cs)):
                    solve(s, qctx, cs[:k])
                before = dict(s.stats.stage_s)
                r0 = s.stats.rounds
                gc.collect()  # the harness's own garbage (every rep rebuilds all the shapes)
                t0 = time.perf_counter()
                w = solve(s, qctx, cs)
                inc.append((time.perf_counter() - t0) * 1e3)
                stages = {k: round((v - before.get(k, 0.0)) * 1e3, 3)
                          for k, v in s.stats.stage_s.items() if v - before.get(k, 0.0) > 0}
                rounds = s.stats.rounds - r0
                qctx, cs = fresh(kind, name)
                s.ctx.clear_cache()
                gc.collect()
                t0 = time.perf_counter()
                wc = solve(s, qctx, cs)
                cold.append((time.perf_counter() - t0) * 1e3)
            rec.update(constraints=len(cs), hit=w is not None, hit_cold=wc is not None,
                       launches=rounds, index=getattr(w, "index", None),
                       columns=len(w.schema.columns) if w else None,
                       ms_incremental=float(np.median(inc)), ms_cold=float(np.median(cold)),
                       ms_incremental_all=[round(x, 3) for x in inc],
                       ms_cold_all=[round(x, 3) for x in cold], stages_ms=stages)
        except Exception as e:
            rec.update(error="%s: %s" % (type(e).__name__, e),
                       trace=traceback.format_exc().splitlines()[-4:])
        rec["extra"] = dict(s.stats.extra)
        print(json.dumps(rec), flush=True)
    st = s.stats
    print(json.dumps({"queries": st.queries, "hits": st.hits, "misses": st.misses,
                      "rounds": st.rounds, "host_s": st.host_s, "device_s": st.device_s}))
    s.close()


if __name__ == "__main__":
    main()
