#!/usr/bin/env python3
"""Where a definitions evaluation (Sieve.eval_terms) spends its time: the random workload's
queries that take the Python host stages for a definition (scripts/random_workload.py), each
asked twice on one Sieve; per piece of eval_terms (local tape set, compile, one-row buffer,
upload, device evaluation) the mean over the second asks, in ms.  One JSON line.

    python scripts/definitions_cost.py [n_paths=120]
"""
import json
import os
import random
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

from mythril_amd import native, sieve as sieve_mod  # noqa: E402
from mythril_amd.sieve import Sieve  # noqa: E402
from tests.test_query_native import _random_query  # noqa: E402

PIECES = {}


def _timed(name, fn):
    """fn timed when called inside eval_terms (eval_terms itself always) on the second asks."""
    def wrap(*a, **k):
        outer = name == "eval_terms"
        if outer:
            PIECES["_in"] = True
        t0 = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            if outer:
                PIECES["_in"] = False
            if PIECES.get("_on") and (outer or PIECES.get("_in")):
                PIECES.setdefault(name, []).append((time.perf_counter() - t0) * 1e3)
    return wrap


def main():
    n_paths = int(sys.argv[1]) if len(sys.argv) > 1 else 120
    s = Sieve()
    sieve_mod.local_tapeset = _timed("local_tapeset", sieve_mod.local_tapeset)
    s.compile = _timed("compile", s.compile)
    s.ctx.assignments = _timed("assignments", s.ctx.assignments)
    native.Assignments.upload = _timed("upload", native.Assignments.upload)
    native.eval_values = _timed("eval_values", native.eval_values)
    s.eval_terms = _timed("eval_terms", s.eval_terms)
    for rep in range(2):
        PIECES["_on"] = rep == 1
        for seed in range(n_paths):
            ctx, cs = _random_query(random.Random(seed), 2 + seed % 11)
            nodes = [c.node for c in cs]
            for k in range(1, len(nodes) + 1):
                s.solve(ctx.b, nodes[:k], key=tuple(nodes[:k]))
    PIECES.pop("_on")
    PIECES.pop("_in", None)
    n = len(PIECES.get("eval_terms", []))
    out = {"paths": n_paths, "evaluations": n}
    for name, v in PIECES.items():
        out[name] = {"calls": len(v), "mean_ms": round(sum(v) / max(1, len(v)), 4),
                     "total_ms": round(sum(v), 2)}
    print(json.dumps(out), flush=True)
    s.close()


if __name__ == "__main__":
    main()
