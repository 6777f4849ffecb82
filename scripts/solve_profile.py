#!/usr/bin/env python3
"""Where a LASER-order query's wall time goes on the host: cProfile over the last queries of a
grown path (tests/laser_paths.py) solved in LASER order on one Sieve, after a warm-up pass.
Prints the stage times of Sieve.stats and the top functions by own and cumulative time.

    python scripts/solve_profile.py [shape=ether_thief] [n=400] [timed=40]
"""
import cProfile
import io
import json
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mythril_amd.sieve import Sieve  # noqa: E402
from tests.laser_paths import grow  # noqa: E402


def main():
    shape = sys.argv[1] if len(sys.argv) > 1 else "ether_thief"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 400
    timed = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    s = Sieve()
    ctx, cs = grow(shape, n)
    nodes = [c.node for c in cs]
    for k in range(1, len(nodes) - timed + 1):  # the parents, as LASER solved them
        s.solve(ctx.b, nodes[:k], key=tuple(nodes[:k]))
    before = dict(s.stats.stage_s)
    prof = cProfile.Profile()
    t0 = time.perf_counter()
    prof.enable()
    for k in range(len(nodes) - timed + 1, len(nodes) + 1):
        s.solve(ctx.b, nodes[:k], key=tuple(nodes[:k]))
    prof.disable()
    wall = (time.perf_counter() - t0) * 1e3 / timed
    stages = {k: round((v - before.get(k, 0.0)) * 1e3 / timed, 4)
              for k, v in s.stats.stage_s.items() if v - before.get(k, 0.0) > 0}
    print(json.dumps({"shape": shape, "constraints": n, "queries": timed,
                      "ms_per_query": round(wall, 4), "stages_ms_per_query": stages}))
    for key in ("tottime", "cumulative"):
        out = io.StringIO()
        pstats.Stats(prof, stream=out).sort_stats(key).print_stats(25)
        print(out.getvalue())
    s.close()


if __name__ == "__main__":
    main()
