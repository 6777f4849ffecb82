"""The round-5 mechanisms of the interpreter's asm core on long conjunctions,
against the C oracle (counts and first witnesses over generated rows) and the Python oracle (root
values on uploaded rows):

* short-circuit conjunctions (compile.cpp short_circuit, D_BANDZ): the newest conjunct first,
  waves leaving at the first AND false in every lane -- the newest conjunct false everywhere,
  false on about half the rows, true everywhere;
* instruction windows changed inside the core with the next window prefetched (tapes of up to
  ~3000 slots: streamed from global memory, dozens of windows), and left at complex ops
  (the overflow predicates, run by the C++ driver) in the middle of windows, so the driver reloads
  its lane-held window only when the core comes back in another one;
* the LOADVAR column prefetch (8 columns: 4 preloaded, the rest loaded in the core).
"""
import os
import random

import numpy as np
import pytest

from mythril_amd import native
from mythril_amd.tape import Op, TapeSet
from oracle import smt_eval
from tests.fuzz import assignment_soa, soa_row

pytestmark = pytest.mark.gpu

M64 = (1 << 64) - 1


def _conjunction(b, rng, xs, n, newest):
    """AND of n mostly-true conjuncts (two pass about half the rows) and then `newest`, built
    as LASER builds a path: ((c1 & c2) & c3) ..."""
    cs = []
    halves = set(rng.sample(range(n), 2))  # two conjuncts pass about half the rows
    for i in range(n):
        x, y = rng.sample(xs, 2)  # distinct: x ^ x would be 0
        r = 0.95 if i in halves else rng.random() * 0.9
        if r < 0.3:  # true unless a 256-bit value hits a constant
            c = b.op(Op.NOT, b.op(Op.EQ, b.op(Op.BVADD, x, y), b.const(rng.getrandbits(256), 256)))
        elif r < 0.45:  # an overflow predicate on masked operands: true, a complex op
            c = b.op(Op.BVADD_NOOVFL_U, b.op(Op.BVAND, x, b.const(M64, 256)),
                     b.op(Op.BVAND, y, b.const(M64, 256)))
        elif r < 0.6:  # a 64 x 64-bit product never overflows 256 bits: true, a complex op
            c = b.op(Op.BVMUL_NOOVFL_U, b.op(Op.BVAND, x, b.const(M64, 256)),
                     b.op(Op.BVAND, y, b.const(M64, 256)))
        elif r < 0.9:  # an unsigned bound almost every row meets
            c = b.op(Op.BVUGE, b.op(Op.BVXOR, x, y), b.const(rng.getrandbits(240), 256))
        else:  # about half the rows
            c = b.op(Op.BVULT, x, b.const(1 << 255, 256))
        cs.append(c)
    cs.append(newest)
    acc = cs[0]
    for c in cs[1:]:
        acc = b.op(Op.AND, acc, c)
    return acc


def _tapes(seed):
    rng = random.Random(seed)
    ts = TapeSet()
    b = ts.builder()
    xs = [b.var("x%d" % i) for i in range(8)]
    never = b.op(Op.EQ, xs[0], b.const(rng.getrandbits(256), 256))
    half = b.op(Op.BVULT, xs[1], b.const(1 << 255, 256))
    always = b.op(Op.NOT, b.op(Op.BVULT, xs[2], b.const(0, 256)))
    for n in (12, 60, 150, 300):
        for newest in (never, half, always):
            ts.add(b.finish(_conjunction(b, rng, xs, n, newest)))
    return ts


def test_long_conjunctions_against_the_oracle(gpu_ctx):
    from oracle import ctape

    ts = _tapes(9100)
    ct = gpu_ctx.compile(ts)
    info = ct.info()
    assert max(int(i["n_insns"]) for i in info) > 2048  # streamed tapes, many windows
    seed, rows = 0x51C0, 1 << 16
    a = gpu_ctx.assignments(ts.n_vars, rows)
    a.generate(seed, 0)
    cnt, first = ctape.count(ts, seed, 0, rows, threads=min(16, os.cpu_count() or 1))
    fh, hc = native.run(gpu_ctx, ct, a, mode=native.MODE_COUNT_ALL)
    assert np.array_equal(hc, cnt), "hit counts differ from the C oracle"
    assert np.array_equal(fh, first), "first hits differ from the C oracle"
    fh1, _ = native.run(gpu_ctx, ct, a, mode=native.MODE_FIRST_HIT)
    assert np.array_equal(fh1, first), "first-hit mode differs from the C oracle"
    # the "never" tapes have no hit; the others do (most conjuncts hold on most rows)
    assert all(int(hc[i]) == 0 for i in range(0, len(ts.tapes), 3))
    assert all(int(hc[i]) > 0 for i in range(len(ts.tapes)) if i % 3)
    # a short first round (a query's 4096 rows, one wave per SIMD)
    fh2, hc2 = native.run(gpu_ctx, ct, a, row_count=4096, mode=native.MODE_COUNT_ALL)
    c2, f2 = ctape.count(ts, seed, 0, 4096, threads=min(16, os.cpu_count() or 1))
    assert np.array_equal(hc2, c2) and np.array_equal(fh2, f2)


def test_long_conjunction_values(gpu_ctx):
    """Root values (the parity path: eval_values) equal the Python oracle's on uploaded rows --
    a wave that leaves at a false D_BANDZ reports 0 for its rows, which is the conjunction's
    value."""
    ts = _tapes(9101)
    soa = assignment_soa(random.Random(9102), ts.n_vars, 96)
    # rows 0..31 satisfy the half-probability conjuncts (x < 2^255 for every column)
    for r in range(32):
        for v in range(ts.n_vars):
            soa[v, 7, r] &= 0x7FFFFFFF
    ct = gpu_ctx.compile(ts)
    a = gpu_ctx.assignments(ts.n_vars, soa.shape[2])
    a.upload(soa)
    seen_true = 0
    for i, t in enumerate(ts.tapes):
        got = native.limbs_to_ints(native.eval_values(gpu_ctx, ct, i, a))
        for r in range(soa.shape[2]):
            want = int(smt_eval.evaluate(t.nodes, ts.pool.values, soa_row(soa, r)))
            assert got[r] == want, (i, r)
            seen_true += want
    assert seen_true > 0


def test_async_compile_equals_compile(gpu_ctx):
    """mh_tapes_compile_async on the context's worker thread gives the tape set mh_tapes_compile
    gives (the same per-tape summaries and results), a second pending compile is refused, and a
    context destroyed with an uncollected compile releases it."""
    ts = _tapes(9103)
    ct = gpu_ctx.compile(ts)
    pend = gpu_ctx.compile_async(ts)
    with pytest.raises(native.SieveError):
        gpu_ctx.compile_async(ts)  # one at a time per context
    ct2 = pend.wait()
    assert ct2.info() == ct.info()
    a = gpu_ctx.assignments(ts.n_vars, 4096)
    a.generate(0x77, 0)
    r1 = native.run(gpu_ctx, ct, a, mode=native.MODE_COUNT_ALL)
    r2 = native.run(gpu_ctx, ct2, a, mode=native.MODE_COUNT_ALL)
    assert all(np.array_equal(x, y) for x, y in zip(r1, r2))
    for c in (ct, ct2):
        c.close()
    a.close()
    ctx = native.Context(0)
    ctx.compile_async(ts)
    ctx.close()  # the pending compile is finished and dropped, the worker joined
