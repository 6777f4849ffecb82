#!/usr/bin/env python3
"""Query latency when both branches of every JUMPI are asked: LASER calls
is_possible on each state a JUMPI makes (svm.py:257-262) -- the path so far plus the condition,
then the path so far plus its negation -- and the next JUMPI extends one of them.  Here, for the
grown paths of tests/laser_paths.py, every constraint c_k is asked as P + c_k and then P + Not(c_k)
(P = c_1..c_{k-1}), and the walk continues from P + c_k, so the query compiler's incremental
path (a child of the last query) never applies to the sibling and to the walk's next query.  One
JSON line per (shape, n): per-query latency of the taken branch and of the sibling (median of
the last 8 of each), and the mean query-build (``lower``) stage over all queries, next to the
LASER-order figures of scripts/path_scaling.py for the same path.

    python scripts/jumpi_order.py [lengths=100,400]
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
from mythril_amd.smt import Not  # noqa: E402
from tests.laser_paths import grow  # noqa: E402


def main():
    lengths = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "100,400").split(",")]
    s = Sieve()
    ctx, cs = grow("killbilly", 25)
    s.solve(ctx.b, [c.node for c in cs])  # warm-up
    for name in ("ether_thief", "killbilly", "overflow"):
        for n in lengths:
            rec = {"shape": name, "constraints": n}
            ctx, cs = grow(name, n)
            s.ctx.clear_cache()
            nodes = [c.node for c in cs]
            neg = [Not(c).node for c in cs]
            taken, sib, hits = [], [], 0
            before = dict(s.stats.stage_s)
            for k in range(1, len(nodes) + 1):
                gc.collect() if k > len(nodes) - 8 else None
                t0 = time.perf_counter()
                w = s.solve(ctx.b, nodes[:k], key=tuple(nodes[:k]))
                t1 = time.perf_counter()
                s.solve(ctx.b, nodes[:k - 1] + [neg[k - 1]], key=tuple(nodes[:k - 1] + [neg[k - 1]]))
                t2 = time.perf_counter()
                taken.append((t1 - t0) * 1e3)
                sib.append((t2 - t1) * 1e3)
                hits += w is not None
            q = 2 * len(nodes)
            rec.update(ms_taken=float(np.median(taken[-8:])), ms_sibling=float(np.median(sib[-8:])),
                       ms_taken_mean=float(np.mean(taken)), ms_sibling_mean=float(np.mean(sib)),
                       taken_hits=hits)
            rec["stages_ms_per_query"] = {
                k: round((v - before.get(k, 0.0)) * 1e3 / q, 4)
                for k, v in s.stats.stage_s.items() if v - before.get(k, 0.0) > 0}
            print(json.dumps(rec), flush=True)
    s.close()


if __name__ == "__main__":
    main()
