#!/usr/bin/env python3
"""Query latency in the order LASER's default BFS asks queries.

For KillBilly, the transfer overflow and EtherThief grown to n constraints (tests/laser_paths.py),
the first `prefix` = n - levels constraints are asked in LASER order (one path), then `levels`
levels of a BFS over binary JUMPIs (tests/bfs_order.py: every open state asks both of its
branches back to back, svm.py:243-262; at most k states stay open, drawn at random so open paths
part at many depths; a state the compiler refutes is dropped, as LASER drops infeasible
states; cli.py:417-419).  One JSON line per (shape, n, k) with, over the BFS
queries: the query build (native query compiler, ``lower`` stage), the guide harvest, and --
with ``--solve`` on the GPU -- the whole ``Sieve.solve``, as mean / median / p90 ms, plus the
share of queries the compiler built from its state (``incremental``) and the guide session
reused.  k = 1 is the JUMPI order of scripts/jumpi_order.py (both branches, the walk goes on
from the first).  Host-only by default (no device: the compiler and harvester on this host).

    python scripts/bfs_order.py [--solve] [n=400] [levels=32] [ks=1,8,32]
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
from mythril_amd.smt import Not  # noqa: E402
from tests.bfs_order import bfs_queries  # noqa: E402
from tests.laser_paths import grow  # noqa: E402


def stats(xs):
    xs = np.asarray(xs, dtype=float)
    return {"mean": round(float(xs.mean()), 4), "p50": round(float(np.median(xs)), 4),
            "p90": round(float(np.percentile(xs, 90)), 4)}


def host_only(name, n, levels, k):
    ctx, cs = grow(name, n)
    nodes = [c.node for c in cs]
    negs = [Not(c).node for c in cs]
    m = native.TermMirror.of(ctx.b)
    sess = native.GuideSession()
    build, guide, inc, dropped = [], [], 0, set()
    prefix = n - levels
    for i, roots in enumerate(bfs_queries(nodes, negs, prefix, k, k, dropped)):
        t0 = time.perf_counter()
        cq = m.build(ctx.b, roots)
        t1 = time.perf_counter()
        if cq.flags & native.QUERY_REFUTED:  # infeasible: LASER drops the state
            dropped.add(tuple(roots))
        else:
            native.harvest_guide(cq.tapes[0], cq.consts, cq.widths, session=sess)
        t2 = time.perf_counter()
        if i >= prefix:
            build.append((t1 - t0) * 1e3)
            guide.append((t2 - t1) * 1e3)
            inc += bool(cq.flags & native.QUERY_INCREMENTAL)
    reused, fresh, _ = sess.stats()
    sess.close()
    return {"queries": len(build), "refuted": len(dropped), "build_ms": stats(build),
            "guide_ms": stats(guide), "incremental": round(inc / max(len(build), 1), 4),
            "guide_session_reused": reused, "guide_session_fresh": fresh}


def solve(s, name, n, levels, k):
    ctx, cs = grow(name, n)
    nodes = [c.node for c in cs]
    negs = [Not(c).node for c in cs]
    s.ctx.clear_cache()
    prefix = n - levels
    total, build, guide, hits, dropped = [], [], [], 0, set()
    for i, roots in enumerate(bfs_queries(nodes, negs, prefix, k, k, dropped)):
        before = dict(s.stats.stage_s)
        ref0 = s.stats.extra.get("refuted", 0)
        if i >= prefix and i % 16 == 0:
            gc.collect()
        t0 = time.perf_counter()
        w = s.solve(ctx.b, roots, key=tuple(roots))
        dt = (time.perf_counter() - t0) * 1e3
        if s.stats.extra.get("refuted", 0) > ref0:  # infeasible: LASER drops the state
            dropped.add(tuple(roots))
        if i >= prefix:
            st = {kk: (v - before.get(kk, 0.0)) * 1e3 for kk, v in s.stats.stage_s.items()}
            total.append(dt)
            build.append(st.get("lower", 0.0))
            guide.append(st.get("guide", 0.0))
            hits += w is not None
    return {"queries": len(total), "refuted": len(dropped), "solve_ms": stats(total),
            "build_ms": stats(build), "guide_ms": stats(guide), "hits": hits}


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    n = int(args[0]) if args else 400
    levels = int(args[1]) if len(args) > 1 else 32
    ks = [int(x) for x in (args[2] if len(args) > 2 else "1,8,32").split(",")]
    do_solve = "--solve" in sys.argv
    s = None
    if do_solve:
        from mythril_amd.sieve import Sieve

        s = Sieve()
        ctx, cs = grow("killbilly", 25)
        s.solve(ctx.b, [c.node for c in cs])  # warm-up
    for name in ("ether_thief", "killbilly", "overflow"):
        for k in ks:
            rec = {"shape": name, "constraints": n, "levels": levels, "k": k}
            rec.update(solve(s, name, n, levels, k) if do_solve else host_only(name, n, levels, k))
            print(json.dumps(rec), flush=True)
    if s is not None:
        s.close()


if __name__ == "__main__":
    main()
