"""Host side of the sieve engine (mythril_amd/sieve.py), checked with the oracle and the
test-only host emulator of the device ISA (tests/native/emu.cpp, the product tape compiler).

* every LASER-shaped query of tests/laser_like.py compiles for the device (with
  rematerialisation where overlapping calldata words exceed the register file) and the compiled
  code agrees with the oracle on guided candidate rows;
* ``rematerialize`` preserves the value of a tape and lowers its register need.
"""
import numpy as np
import pytest

from mythril_amd.candidates import build_guide
from mythril_amd.lower import lower_query
from mythril_amd.sieve import local_tape, rematerialize
from mythril_amd.tape import Tape, TapeSet
from oracle import smt_eval as E
from oracle.guided_gen import generate_row
from tests.emu import EmuError
from tests.laser_like import queries


def _soa(rows, n_cols):
    soa = np.zeros((n_cols, 8, len(rows)), dtype=np.uint32)
    for j, row in enumerate(rows):
        for i, v in enumerate(row):
            for k in range(8):
                soa[i, k, j] = (v >> (32 * k)) & 0xFFFFFFFF
    return soa


@pytest.mark.parametrize("qi", range(len(queries()[1])))
def test_queries_compile_and_match_oracle(emu, qi):
    ctx, qs = queries()
    name, cs = qs[qi]
    root, schema = lower_query(ctx.b, [c.node for c in cs])
    cols = list(schema.columns)
    guide = build_guide(ctx.b, root, schema, cols).arrays()
    nodes = local_tape(ctx.b, root, cols)
    ts = TapeSet(cols)
    ts.pool = ctx.b.pool
    rows = [generate_row(11 + qi, r, guide) for r in range(96)]
    soa = _soa(rows, len(cols))
    got = None
    for size in (0, 8, 32, 256):  # the retry ladder of Sieve.compile
        ts.tapes[:] = [Tape(nodes if size == 0 else rematerialize(nodes, size))]
        try:
            got, nregs = emu.eval(ts, 0, soa)
            break
        except EmuError as e:
            assert "register pressure" in str(e), (name, str(e))
    assert got is not None, name
    for j, row in enumerate(rows):
        want = E.evaluate(nodes, ctx.b.pool.values, row)
        assert bool(got[j]) == bool(want), (name, j)
        # the rematerialised tape is the same function
        assert bool(E.evaluate(ts.tapes[0].nodes, ctx.b.pool.values, row)) == bool(want)


def test_rematerialize_removes_sharing_of_cheap_terms():
    ctx, qs = queries()
    cs = dict(qs)["address_arg"]
    root, _ = lower_query(ctx.b, [c.node for c in cs])
    nodes = local_tape(ctx.b, root, list(ctx.b.var_index))
    r = rematerialize(nodes, 8)
    # reachable part of r: every cheap node has one user
    from mythril_amd.tape import ARITY, Op

    n = len(r)
    reach = np.zeros(n, dtype=bool)
    reach[-1] = True
    uses = np.zeros(n, dtype=int)
    for i in range(n - 1, -1, -1):
        if not reach[i]:
            continue
        for x in [r["a"][i], r["b"][i], r["c"][i]][:ARITY[Op(int(r["op"][i]))]]:
            reach[x] = True
            uses[x] += 1
    shared_ites = [i for i in range(n) if reach[i] and int(r["op"][i]) == Op.ITE
                   and uses[i] > 1]
    assert not shared_ites


def test_buckets_split_variable_disjoint_conjuncts():
    from mythril_amd.sieve import Sieve

    ctx, qs = queries()
    sizes = {}
    for name, cs in qs:
        root, schema = lower_query(ctx.b, [c.node for c in cs])
        groups = Sieve.buckets(ctx.b, root)
        cols = [v for _, vs in groups for v in vs]
        assert len(cols) == len(set(cols)), name  # disjoint
        names = {ctx.b.var_index[c] for c in schema.columns}
        assert set(cols) == names, name  # every column of the query is in some group
        sizes[name] = sum(1 for _, vs in groups if vs)  # ground conjuncts form groups too
    assert sizes["selector"] == 2        # calldata bytes + size  |  sender in ACTORS
    assert sizes["owner_check"] == 1     # Storage[0] == sender ties them
    assert sizes["keccak_alias"] == 1


def test_hot_columns_are_loaded_once(emu):
    """A loaded-on-use column read by many operands (every calldata byte compares its index with
    calldatasize, calldata.py:48-54) is loaded once and held in a register by the interpreter's
    compiler (compile.cpp Lowering::hold_vars): fewer D_LOADVAR complex ops, same values."""
    import os

    from mythril_amd.sieve import local_tapeset

    ctx, qs = queries()
    cs = dict(qs)["overflow"]
    root, schema = lower_query(ctx.b, [c.node for c in cs])
    cols = list(schema.columns)
    ts = local_tapeset(ctx.b, [root], cols)
    guide = build_guide(ctx.b, root, schema, cols).arrays()
    rows = [generate_row(5, r, guide) for r in range(64)]
    soa = _soa(rows, len(cols))
    held, _ = emu.eval(ts, 0, soa)
    n_held = emu.n_slots(ts)
    os.environ["MH_NO_HOLD_VARS"] = "1"
    try:
        plain, _ = emu.eval(ts, 0, soa)
        n_plain = emu.n_slots(ts)
    finally:
        del os.environ["MH_NO_HOLD_VARS"]
    assert [bool(x) for x in held] == [bool(x) for x in plain]
    assert n_held < n_plain, (n_held, n_plain)


def test_root_conjunction_short_circuits(emu):
    """The interpreter's compiler flattens a query's root AND chain and emits every AND but the
    last as D_BANDZ (compile.cpp short_circuit): a wave whose lanes are all false there leaves
    the tape.  The emulator leaves at a false D_BANDZ per lane, so
    test_queries_compile_and_match_oracle checks that the root is then 0 for that row."""
    import os
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "mythril_amd", "csrc"))
    import gen_asm_core as G

    from mythril_amd.tape import Op

    ctx, qs = queries()
    seen = 0
    for name, cs in qs:
        root, schema = lower_query(ctx.b, [c.node for c in cs])
        cols = list(schema.columns)
        nodes = local_tape(ctx.b, root, cols)
        n_conj, stack = 0, [len(nodes) - 1]
        while stack:  # the root's AND chain (single-use ANDs) as the compiler sees it
            i = stack.pop()
            if int(nodes[i]["op"]) == int(Op.AND):
                stack += [int(nodes[i]["b"]), int(nodes[i]["a"])]
            else:
                n_conj += 1
        ts = TapeSet(cols)
        ts.pool = ctx.b.pool
        for size in (0, 8, 32, 256):
            ts.tapes[:] = [Tape(nodes if size == 0 else rematerialize(nodes, size))]
            try:
                w = emu.words(ts)
                break
            except EmuError as e:
                assert "register pressure" in str(e), (name, str(e))
        ops = [int(x) & 0xFF for x in w[1::2]]
        n_z = ops.count(G.OPNUM["BANDZ"])
        if n_conj < 2:
            assert n_z == 0, name
            continue
        seen += 1
        # conjuncts the fold or the lowering merged may be fewer than the source's
        assert 1 <= n_z <= n_conj - 1, (name, n_z, n_conj)
        last_and = max(i for i, o in enumerate(ops) if o in (G.OPNUM["BAND"], G.OPNUM["BANDZ"]))
        assert ops[last_and] == G.OPNUM["BAND"], name  # the last AND needs no test
    assert seen >= 5


def test_short_circuit_edge_shapes(emu):
    """Root conjunctions the short-circuit pass must keep exact: a conjunct twice, a chain AND
    also read inside a conjunct, a conjunct that is a shared sub-term of another, constant
    conjuncts, a lone conjunct, a non-Bool root -- the emulator leaves at a false D_BANDZ per
    lane and must still agree with the oracle on every row."""
    import random

    from mythril_amd.tape import Op
    from tests.fuzz import assignment_soa, soa_row

    ts = TapeSet()
    b = ts.builder()
    x, y, z = b.var("x"), b.var("y"), b.var("z")
    c1 = b.op(Op.BVULT, x, y)
    c2 = b.op(Op.NOT, b.op(Op.EQ, b.op(Op.BVADD, x, z), b.const(5, 256)))
    c3 = b.op(Op.BVUGT, z, b.const(1 << 200, 256))
    a12 = b.op(Op.AND, c1, c2)
    shapes = [
        b.op(Op.AND, c1, c1),                                   # the same conjunct twice
        b.op(Op.AND, a12, b.op(Op.NOT, a12)),                   # a chain AND read inside
        b.op(Op.AND, b.op(Op.AND, a12, c3), b.op(Op.OR, a12, c3)),
        b.op(Op.AND, b.op(Op.AND, c1, b.true()), c3),
        b.op(Op.AND, b.false(), c2),
        c3,                                                      # a lone conjunct
        b.op(Op.AND, b.op(Op.AND, b.op(Op.AND, c1, c2), c3), c2),
        b.op(Op.BVADD, x, y),                                    # not a Bool
    ]
    for s in shapes:
        ts.add(b.finish(s))
    soa = assignment_soa(random.Random(77), ts.n_vars, 64)
    for r in range(16):  # rows where x < y and z is large: the conjunctions can hold
        for k in range(8):
            soa[0, k, r], soa[1, k, r] = 0, 0xFFFFFFFF
        soa[2, 7, r] = 0xFFFFFFFF
    for i, t in enumerate(ts.tapes):
        got, _ = emu.eval(ts, i, soa)
        for r in range(soa.shape[2]):
            assert got[r] == int(E.evaluate(t.nodes, ts.pool.values, soa_row(soa, r))), (i, r)
