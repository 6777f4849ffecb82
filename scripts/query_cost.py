#!/usr/bin/env python3
"""Host-stage cost of one query: the native query compiler (mh_query_build behind
native.TermMirror, plus unpacking) against the Python stages it replaces (lower_query,
Sieve.bucket_roots, local_tapeset), host-only (no device).  DESIGN §6 host-stage table.

Per shape (tests/laser_like.py, grown paths of tests/laser_paths.py at 25..400 constraints):
``cold`` = the whole path as one query on fresh terms (nothing lowered before; the native
mirror's sync of the fresh nodes included), ``laser`` = the last query of the path after its
prefixes were built in LASER order (svm.py:257-262), median of the last 8.  One JSON line each.

    python scripts/query_cost.py [lengths=25,100,400]
"""
import gc
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

from mythril_amd import native  # noqa: E402
from mythril_amd.sieve import Sieve, local_tapeset, lower_query  # noqa: E402
from tests import laser_like  # noqa: E402
from tests.laser_paths import grow  # noqa: E402


def python_stages(b, roots):
    root, schema = lower_query(b, roots)
    cols = list(schema.columns) or ["__ground__"]
    groups = Sieve.bucket_roots(b, root)
    accs = [a for a, _ in groups]
    ts = local_tapeset(b, [root] + (accs if accs != [root] else []), cols)
    return ts


def native_stages(b, roots):
    return native.TermMirror.of(b).build(b, roots)


def timed(fn, b, roots):
    gc.collect()
    t0 = time.perf_counter()
    fn(b, roots)
    return (time.perf_counter() - t0) * 1e3


def measure(name, make):
    rec = {"query": name}
    for label, fn in (("python", python_stages), ("native", native_stages)):
        ctx, cs = make()
        nodes = [c.node for c in cs]
        rec["constraints"] = len(nodes)
        rec["%s_cold_ms" % label] = timed(fn, ctx.b, nodes)
        ctx, cs = make()
        nodes = [c.node for c in cs]
        ts = [timed(fn, ctx.b, nodes[:k]) for k in range(1, len(nodes) + 1)]
        rec["%s_laser_ms" % label] = float(np.median(ts[-8:]))
        rec["%s_laser_mean_ms" % label] = float(np.mean(ts))
    return rec


def main():
    lengths = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "25,100,400").split(",")]
    measure("warm-up", lambda: grow("killbilly", 25))
    for which in ("queries", "hard_queries"):
        _, qs = getattr(laser_like, which)()
        for i, (name, _) in enumerate(qs):
            def make(which=which, i=i):
                ctx, q = getattr(laser_like, which)()
                return ctx, q[i][1]
            print(json.dumps(measure(name, make)), flush=True)
    for shape in ("killbilly", "overflow", "ether_thief"):
        for n in lengths:
            print(json.dumps(measure("%s_%d" % (shape, n), lambda: grow(shape, n))), flush=True)


if __name__ == "__main__":
    main()
