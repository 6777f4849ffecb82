#!/usr/bin/env python3
"""Run the sieve on the LASER-shaped queries of tests/laser_like.py (the SAT shapes and the UNSAT
hard variants) and report, per query: hit or miss, launches, witness index, the median latency
of SIEVE_QUERY_REPS (5) solves, per-stage milliseconds of the last one, and any exception (the
front end swallows them to fall back; this script shows them).  One JSON line per query.

    python scripts/sieve_queries.py [rows_per_round]
"""
import json
import os
import sys
import time
import traceback

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

from mythril_amd.sieve import Sieve  # noqa: E402
from tests.laser_like import hard_queries, queries  # noqa: E402


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 16
    s = Sieve(rows=rows)
    ctx, qs = queries()
    # warm-up: the first query of a process pays the HIP runtime's lazy initialisation and the
    # code object load; LASER issues thousands of queries per process
    s.solve(ctx.b, [c.node for c in qs[0][1]])
    hctx, hqs = hard_queries()
    todo = [(ctx, n, cs) for n, cs in qs] + [(hctx, n, cs) for n, cs in hqs]
    reps = int(os.environ.get("SIEVE_QUERY_REPS", "5"))
    for qctx, name, cs in todo:
        # the median of `reps` solves (each a full query: lowering, guide, tapes, device)
        ms = []
        for _ in range(reps - 1):
            t0 = time.perf_counter()
            s.solve(qctx.b, [c.node for c in cs])
            ms.append((time.perf_counter() - t0) * 1e3)
        t0 = time.perf_counter()
        rec = {"query": name, "constraints": len(cs)}
        before = dict(s.stats.stage_s)
        try:
            w = s.solve(qctx.b, [c.node for c in cs])
            rec.update(hit=w is not None, rounds=getattr(w, "rounds", None),
                       index=getattr(w, "index", None),
                       columns=len(w.schema.columns) if w else None)
        except Exception as e:
            rec.update(error="%s: %s" % (type(e).__name__, e),
                       trace=traceback.format_exc().splitlines()[-4:])
        ms.append((time.perf_counter() - t0) * 1e3)
        rec["ms"] = sorted(ms)[len(ms) // 2]
        rec["ms_all"] = [round(x, 3) for x in ms]
        rec["extra"] = dict(s.stats.extra)
        rec["stages_ms"] = {k: round((v - before.get(k, 0.0)) * 1e3, 3)
                            for k, v in s.stats.stage_s.items() if v - before.get(k, 0.0) > 0}
        print(json.dumps(rec), flush=True)
    st = s.stats
    print(json.dumps({"queries": st.queries, "hits": st.hits, "misses": st.misses,
                      "rounds": st.rounds, "host_s": st.host_s, "device_s": st.device_s}))
    s.close()


if __name__ == "__main__":
    main()
