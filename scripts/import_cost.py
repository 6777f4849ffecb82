#!/usr/bin/env python3
"""The product path's first stage, timed (DESIGN §6 import column).

Under the plugin every constraint reaches the sieve as z3's ``Solver.sexpr()`` text
(smtlib.Z3Importer; reference call site mythril/support/model.py:37-57).  Per LASER-shaped query
(tests/laser_like.py) and per grown path (tests/laser_paths.py, 25..400 constraints), in LASER
order (one new constraint per query, one importer for the whole path), this times the import of
each new constraint by the C++ reader (mh_smtlib_read + the host's new nodes, ``NativeReader``)
and by the Python reader it replaced (``Reader``), on z3-style text (tests/z3_style.py).  One
JSON line per query: constraints, text size, new host nodes, mean / max ms of both readers.

    python scripts/import_cost.py
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

from mythril_amd import smtlib  # noqa: E402
from tests.laser_like import hard_queries, queries  # noqa: E402
from tests.laser_paths import grow  # noqa: E402
from tests.z3_style import z3_sexpr  # noqa: E402


def measure(name, cs):
    texts = [z3_sexpr(c) for c in cs]
    nat, py = smtlib.NativeReader(), smtlib.Reader()
    tn, tp, new_nodes = [], [], []
    for t in texts:
        n0 = len(nat.b.nodes)
        t0 = time.perf_counter()
        nat.read(t, smtlib.Query(nat.ctx))
        t1 = time.perf_counter()
        q = smtlib.Query(py.ctx)
        for cmd in smtlib.read_sexps(t):
            py.command(cmd, q)
        t2 = time.perf_counter()
        tn.append((t1 - t0) * 1e3)
        tp.append((t2 - t1) * 1e3)
        new_nodes.append(len(nat.b.nodes) - n0)
    return {"query": name, "constraints": len(cs), "chars_max": max(len(t) for t in texts),
            "new_nodes_max": max(new_nodes), "new_nodes_mean": sum(new_nodes) / len(cs),
            "native_ms_mean": sum(tn) / len(tn), "native_ms_max": max(tn),
            "python_ms_mean": sum(tp) / len(tp), "python_ms_max": max(tp)}


def main():
    for make in (queries, hard_queries):
        _, qs = make()
        for name, cs in qs:
            measure(name, cs)  # warm-up (first calls of a process)
            print(json.dumps(measure(name, cs)), flush=True)
    for shape in ("killbilly", "overflow", "ether_thief"):
        for n in (25, 100, 400):
            _, cs = grow(shape, n)
            print(json.dumps(measure("%s_%d" % (shape, n), cs)), flush=True)


if __name__ == "__main__":
    main()
