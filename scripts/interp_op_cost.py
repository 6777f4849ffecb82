#!/usr/bin/env python3
"""Interpreter cost of a loaded-on-use column (D_LOADVAR, tape sets over 4 columns) against the
same tape over preloaded columns, and of another complex op, from HIP-event kernel time at a
query's 256-row round and at 2^16 rows.  One JSON line per case.

    python scripts/interp_op_cost.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

from mythril_amd import native, smt  # noqa: E402
from mythril_amd.smt import And, Not, symbol_factory as sf  # noqa: E402


def tapeset(n_cols, n_conj, kind):
    ctx = smt.Context()
    smt.set_context(ctx)
    xs = [sf.BitVecSym("x%d" % i, 8 if kind != "ovfl" else 256) for i in range(n_cols)]
    cs = []
    for i in range(n_conj):
        x = xs[i % n_cols]
        if kind == "eq":
            cs.append(x == sf.BitVecVal(i & 0xFF, 8))
        else:  # a complex op per conjunct: the overflow predicate
            cs.append(Not(smt.BVAddNoOverflow(x, sf.BitVecVal(i + 1, 256), False)))
    ctx.add_tape(And(*cs))
    return ctx.tapeset


def main():
    c = native.Context(0)
    c.enable_timing(True)
    for kind, n_cols, n_conj in (("eq", 4, 64), ("eq", 64, 64), ("eq", 64, 128), ("eq", 4, 128),
                                 ("ovfl", 4, 32), ("ovfl", 4, 64)):
        ts = tapeset(n_cols, n_conj, kind)
        ct = c.compile(ts)
        for rows in (256, 1 << 16):
            a = c.assignments(max(ts.n_vars, 1), rows)
            a.generate(7)
            native.run(c, ct, a, mode=native.MODE_COUNT_ALL)  # warm
            c.kernel_time()
            reps = 20
            for _ in range(reps):
                native.run(c, ct, a, mode=native.MODE_COUNT_ALL)
            ms, n = c.kernel_time()
            print(json.dumps({"kind": kind, "columns": n_cols, "conjuncts": n_conj, "rows": rows,
                              "kernel_us": round(ms / max(n, 1) * 1e3, 2), "launches": n,
                              "insns": int(ct.info()[0]["n_insns"]) if hasattr(ct, "info") else None}),
                  flush=True)
            a.close()
        ct.close()
    c.close()


if __name__ == "__main__":
    main()
