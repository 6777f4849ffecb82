#!/usr/bin/env python3
"""Latency distribution of the sieve over a broad random query workload: random
conjunctions over free arrays, K arrays, stores, selects at constant and symbolic indices, a
tabled function, keccak with concrete pairs / bounds / its inverse and wide equalities
(tests/test_query_native._random_query), each asked in LASER order -- every prefix a query, the
parent solved first (svm.py:257-262) -- on one Sieve, as a long symbolic-execution run would.
Per query the outcome (hit, refuted, miss, host fallback for a definition, error) and the wall
time; one JSON line with counts and p50 / p90 / p99 / max per outcome.

    python scripts/random_workload.py [n_paths=300] [max_len=12] [passes=1]

With passes > 1 the same paths run again on fresh terms (the device-block pool and the runtime
warm), one JSON line per pass, each with its five slowest queries and their stages.
"""
import json
import os
import random
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

from mythril_amd.sieve import Sieve  # noqa: E402
from tests.test_query_native import _random_query  # noqa: E402


def one_pass(s, n_paths, max_len):
    times = {"hit": [], "refuted": [], "miss": [], "error": []}
    slow = []
    t_all = time.perf_counter()
    for seed in range(n_paths):
        rng = random.Random(seed)
        ctx, cs = _random_query(rng, 2 + seed % (max_len - 1))
        nodes = [c.node for c in cs]
        for k in range(1, len(nodes) + 1):
            r0 = s.stats.extra.get("refuted", 0)
            before = dict(s.stats.stage_s)
            t0 = time.perf_counter()
            try:
                w = s.solve(ctx.b, nodes[:k], key=tuple(nodes[:k]))
                dt = (time.perf_counter() - t0) * 1e3
                kind = ("hit" if w is not None else
                        "refuted" if s.stats.extra.get("refuted", 0) > r0 else "miss")
            except Exception:  # noqa: BLE001 - the front end falls back on any error
                dt, kind = (time.perf_counter() - t0) * 1e3, "error"
            times[kind].append(dt)
            stages = {n: round((v - before.get(n, 0.0)) * 1e3, 3)
                      for n, v in s.stats.stage_s.items() if v - before.get(n, 0.0) > 0}
            slow = sorted(slow + [(dt, seed, k, kind, stages)], reverse=True)[:5]
    out = {"paths": n_paths, "queries": sum(len(v) for v in times.values()),
           "wall_s": round(time.perf_counter() - t_all, 2),
           "host_python": s.stats.extra.get("host_python", 0)}
    for k, v in times.items():
        if v:
            a = np.array(v)
            out[k] = {"n": len(v), "p50": round(float(np.percentile(a, 50)), 3),
                      "p90": round(float(np.percentile(a, 90)), 3),
                      "p99": round(float(np.percentile(a, 99)), 3),
                      "max": round(float(a.max()), 3)}
        else:
            out[k] = {"n": 0}
    out["slowest"] = [{"ms": round(d, 3), "seed": sd, "prefix": k, "outcome": kd, "stages_ms": st}
                      for d, sd, k, kd, st in slow]
    return out


def main():
    n_paths = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    max_len = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    passes = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    s = Sieve()
    ctx, cs = _random_query(random.Random(12345), 4)  # warm-up: runtime, code objects
    s.solve(ctx.b, [c.node for c in cs])
    for p in range(passes):
        out = one_pass(s, n_paths, max_len)
        out["pass"] = p
        print(json.dumps(out), flush=True)
    s.close()


if __name__ == "__main__":
    main()
