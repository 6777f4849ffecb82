"""The conjunct-parallel split of a long tape (compile.h split_conjunction, used by
mh_tapes_compile / mh_run_async for a query's short runs): the parts of a tape whose
root is a conjunction are self-contained tapes (operands before their users, a Bool root), every
conjunct lands in exactly one part in its order, and on every row the AND of the parts' values
equals the tape's (oracle/smt_eval.py) -- for config-5 tapes, random fuzz tapes and the
LASER-shaped queries' group tapes; each part also compiles for the interpreter (the host
emulator of tests/native/emu.cpp runs it, bit-exact with the oracle).  The device side (masks,
combine kernel) is checked in tests/test_gpu_parity.py."""
import ctypes as C
import random

import numpy as np
import pytest

from mythril_amd import native, synth
from mythril_amd.native import NODE_DTYPE
from mythril_amd.tape import ARITY, Op, TapeSet
from oracle import smt_eval
from tests.fuzz import TapeFuzzer, interesting

AND = int(Op.AND)


def split(emu, nodes, want):
    f = emu.lib.emu_split
    f.restype = C.c_int32
    f.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p, C.c_uint64, C.c_void_p]
    nodes = np.ascontiguousarray(nodes, dtype=NODE_DTYPE)
    cap = 4 * len(nodes) + 64
    out = np.zeros(cap, dtype=NODE_DTYPE)
    offs = np.zeros(want + 1, dtype=np.uint64)
    k = f(nodes.ctypes.data, len(nodes), want, out.ctypes.data, cap, offs.ctypes.data)
    assert k >= 0
    return [out[int(offs[i]):int(offs[i + 1])] for i in range(k)]


def conjuncts(nodes):
    out, st = [], [len(nodes) - 1]
    while st:
        u = st.pop()
        n = nodes[u]
        if int(n["op"]) == AND and int(n["width"]) == 0:
            st += [int(n["b"]), int(n["a"])]
        else:
            out.append(u)
    return out


def check(emu, nodes, consts, const_rows, n_vars, widths, rng, rows=24):
    """consts: the pool as ints (the oracle); const_rows: the same as [n, 8] u32 (the emulator)."""
    from mythril_amd.sieve import LocalPool
    from mythril_amd.tape import Tape

    nodes = np.ascontiguousarray(nodes, dtype=NODE_DTYPE)
    n_conj = len(conjuncts(nodes))
    vals = [[interesting(rng, w) for w in widths] for _ in range(rows)]
    soa = np.zeros((max(n_vars, 1), 8, rows), dtype=np.uint32)
    for r, row in enumerate(vals):
        for v, x in enumerate(row):
            for k in range(8):
                soa[v, k, r] = (x >> (32 * k)) & 0xFFFFFFFF
    whole = [bool(smt_eval.evaluate(nodes, consts, row)) for row in vals]
    for want in (2, 3, 8):
        parts = split(emu, nodes, want)
        if n_conj < 2:
            assert parts == []
            continue
        assert 2 <= len(parts) <= min(want, n_conj)
        assert sum(len(conjuncts(p)) for p in parts) == n_conj
        for p in parts:  # self-contained: operands before their users, a Bool root
            assert int(p[-1]["width"]) == 0
            for i, x in enumerate(p):
                k = ARITY[Op(int(x["op"]))]
                assert all(int(x[f]) < i for f in ("a", "b", "c")[:k])
        got = [all(bool(smt_eval.evaluate(p, consts, row)) for p in parts) for row in vals]
        assert got == whole
        # every part compiles for the interpreter and runs on its host emulator as the oracle says
        pts = TapeSet(["c%d" % i for i in range(n_vars)])
        pts.pool = LocalPool(const_rows)
        pts.tapes = [Tape(p) for p in parts]
        for i, p in enumerate(parts):
            ev, _ = emu.eval(pts, i, soa)
            assert [bool(x) for x in ev] == [bool(smt_eval.evaluate(p, consts, row))
                                             for row in vals]


def test_split_config5_tapes(emu):
    ts = synth.generate(60)
    rng = random.Random(5)
    for t in ts.tapes:
        check(emu, t.nodes, ts.pool.values, ts.pool.to_array(), ts.n_vars, [256] * ts.n_vars, rng)


@pytest.mark.parametrize("seed", range(6))
def test_split_fuzz_tapes(emu, seed):
    rng = random.Random(seed)
    ts = TapeSet()
    fz = TapeFuzzer(rng, ts, n_vars=3, max_depth=4)
    b = ts.builder()
    for _ in range(8):  # conjunctions of random Bool terms (the fuzzer's roots are single terms)
        root = fz.boolean(4)
        for _ in range(rng.randrange(1, 7)):
            root = fz.b.op(Op.AND, root, fz.boolean(4))
        ts.add(fz.b.finish(root))
    for t in ts.tapes:
        check(emu, t.nodes, ts.pool.values, ts.pool.to_array(), ts.n_vars, [256] * ts.n_vars, rng)


def test_split_laser_query_tapes(emu):
    from tests.laser_like import hard_queries, queries

    rng = random.Random(9)
    for make in (queries, hard_queries):
        ctx, qs = make()
        for _, cs in qs:
            cq = native.TermMirror.of(ctx.b).build(ctx.b, [c.node for c in cs])
            if cq.flags:
                continue
            consts = [int.from_bytes(np.ascontiguousarray(r, dtype="<u4").tobytes(), "little")
                      for r in cq.consts]
            widths = [int(w) for w in cq.widths]
            for tape in cq.tapes:
                check(emu, tape, consts, cq.consts, len(widths), widths, rng, rows=8)
