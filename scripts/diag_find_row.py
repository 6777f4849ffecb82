#!/usr/bin/env python3
"""Diagnostic: locate the 64-row chunk where the native code's count of one config-5 tape
differs from the C oracle (bisection over 64-aligned row ranges, the whole tape set jitted as
bench.py does), then dump that chunk's columns and both engines' per-row values.

    python scripts/diag_find_row.py TAPE LO HI OUT.npz
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

from mythril_amd import native, synth  # noqa: E402
from mythril_amd.tape import TapeSet  # noqa: E402


def main():
    tape, lo, hi, out = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    from oracle import ctape, smt_eval

    ctx = native.Context(0)
    ts = synth.generate()
    seed = synth.load_spec()["assignment_seed"]
    ct = ctx.compile(ts)
    ct.jit()
    a = ctx.assignments(ts.n_vars, hi)
    a.generate(seed, 0)
    sub = TapeSet(ts.var_names)
    sub.pool = ts.pool
    sub.tapes = [ts.tapes[tape]]
    th = min(16, os.cpu_count() or 1)

    def diff(r0, n):
        _, hc = native.run(ctx, ct, a, row_first=r0, row_count=n, mode=native.MODE_COUNT_ALL)
        cnt, _ = ctape.count(sub, seed, r0, n, threads=th, short_circuit=True)
        return int(hc[tape]) - int(cnt[0])

    r0, n = lo, hi - lo
    d = diff(r0, n)
    log = [{"range": [r0, n], "diff": d}]
    while n > 64 and d:
        half = (n // 2) // 64 * 64
        dl = diff(r0, half)
        if dl:
            n, d = half, dl
        else:
            r0, n, d = r0 + half, n - half, diff(r0 + half, n - half)
        log.append({"range": [r0, n], "diff": d})
    rec = {"tape": tape, "bisect": log}
    if d and n == 64:
        soa = a.download(r0, 64)[: ts.n_vars]
        truth = [int(smt_eval.evaluate(ts.tapes[tape].nodes, ts.pool.values,
                                        smt_eval.gen_assignment(seed, ts.n_vars, r0 + i)))
                 for i in range(64)]
        one = ctx.compile(sub)
        one.jit(values=True)
        jv = native.limbs_to_ints(one.jit_values(a, row_first=r0, row_count=64)[0])
        iv = native.limbs_to_ints(native.eval_values(ctx, ctx.compile(sub), 0, a, r0, 64))
        rec.update(chunk=r0, truth=truth, single_tape_jit=[int(x) for x in jv],
                   interp=[int(x) for x in iv],
                   single_tape_reproduces=[i for i in range(64) if jv[i] != truth[i]])
        np.savez(out, soa=soa, chunk=r0, tape=tape)
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
