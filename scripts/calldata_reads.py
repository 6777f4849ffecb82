#!/usr/bin/env python3
"""Latency of the reference's calldata loop over a sieve model.

SymbolicCalldata.concrete (calldata.py:234-245) reads a model one term at a time: the size, then
``model.eval(byte.raw, model_completion=True).as_long()`` per byte.  Driven through the printing
z3 stand-in (tests/test_model_z3_terms.py: z3's SMT-LIB text of each term, read by the importer),
on the GPU: per repetition a fresh query (front end reset), its witness, the 100-byte loop with
the batching of model.py (the size; then byte 0 with its 127 speculated siblings, one
``mh_eval_values_many`` launch each), the same loop again (memo hits), and the loop with
speculation off (model.SPECULATE = 0: one launch per byte -- round 5's cost model).  One JSON
line: launches and ms per loop, median over the repetitions.

    python scripts/calldata_reads.py [reps=9] [size=100] [--fake]

--fake runs on tests/fake_device.py (CPU: the launch counts, not the latency).
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

from mythril_amd import frontend, model, native  # noqa: E402
from mythril_amd.smtlib import Z3Importer  # noqa: E402
from tests.test_model_z3_terms import (RefExpr, calldata_query, concrete_calldata,  # noqa: E402
                                       printing_z3)


LAUNCHES = native.eval_launches


def one(size, speculate):
    frontend.reset()
    frontend.configure(to_terms=Z3Importer(), fallback=lambda *a: "fallback", rows=256)
    ref, cd, cs = calldata_query(size)
    m = frontend.get_model(tuple(RefExpr(c) for c in cs))
    assert isinstance(m, model.Model), m
    ctx = frontend.sieve().ctx
    model.SPECULATE = speculate
    try:
        l0 = LAUNCHES(ctx)
        t0 = time.perf_counter()
        got = concrete_calldata(m, cd)
        t1 = time.perf_counter()
        l1 = LAUNCHES(ctx)
        again = concrete_calldata(m, cd)
        t2 = time.perf_counter()
    finally:
        model.SPECULATE = 127
    assert got == again and len(got) == size and got[:4] == [0x9F, 0xA2, 0x99, 0xCC]
    return l1 - l0, (t1 - t0) * 1e3, (t2 - t1) * 1e3


def main():
    global LAUNCHES
    args = [int(a) for a in sys.argv[1:] if not a.startswith("--")]
    if "--fake" in sys.argv:
        import pytest

        from tests import fake_device

        fake_device.install(pytest.MonkeyPatch())
        LAUNCHES = lambda ctx: fake_device.LAUNCHES[0]  # noqa: E731
    reps = args[0] if args else 9
    size = args[1] if len(args) > 1 else 100
    sys.modules["z3"] = printing_z3()
    one(size, 127)  # warm-up (first import, compile caches)
    out = {"bytes": size, "reps": reps}
    for label, spec in (("batched", 127), ("per_term", 0)):
        runs = [one(size, spec) for _ in range(reps)]
        out[label] = {"launches": int(np.median([r[0] for r in runs])),
                      "first_loop_ms": round(float(np.median([r[1] for r in runs])), 3),
                      "memo_loop_ms": round(float(np.median([r[2] for r in runs])), 3)}
    frontend.reset()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
