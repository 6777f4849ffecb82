"""mh_guide_harvest (mythril_amd/csrc/harvest.cpp) against the Python harvester it restates
(mythril_amd/candidates.py): the same guide arrays, bit for bit, for every LASER-shaped query of
tests/laser_like.py, asked in LASER order (each query extends its parent by one conjunct,
svm.py:257-262, so the Python side also answers from its builder-level memos) and with parent
witnesses.  Host-only: runs without a GPU."""
from __future__ import annotations

import hashlib

import numpy as np
import pytest

from mythril_amd import native
from mythril_amd.candidates import build_guide
from mythril_amd.lower import lower_query
from mythril_amd.sieve import local_tapeset

from . import laser_like

KEYS = ("width", "pool_off", "pool", "set_off", "set_prob", "alt_off", "entry_col", "entry_val")


def _lib_or_skip():
    try:
        native.load()
    except native.NativeUnavailable as e:  # pragma: no cover - build() makes it
        pytest.skip(str(e))


def _parent_of(cols, widths, salt: str):
    """A deterministic parent witness over some of the columns, plus one name the query does
    not read (the parent's own columns are not all the child's)."""
    out = {}
    for i, (c, w) in enumerate(zip(cols, widths)):
        h = int.from_bytes(hashlib.sha256(("%s/%s" % (salt, c)).encode()).digest(), "little")
        if h % 3:
            out[c] = h & ((1 << w) - 1) if h % 5 else 0
    out["__not_a_column__"] = 7
    return out


def _compare(b, roots, parent=None, parent_eval=False):
    root, schema = lower_query(b, roots)
    cols = list(schema.columns)
    if not cols:
        return 0
    widths = [schema.columns[c].width for c in cols]
    want = build_guide(b, root, schema, cols, parent, parent_eval=parent_eval).arrays()
    ts = local_tapeset(b, [root], cols)
    index = {c: i for i, c in enumerate(cols)}
    par = [(index[k], v) for k, v in (parent or {}).items() if k in index]
    got = native.harvest_guide(ts.tapes[0].nodes, ts.pool.to_array(), widths, par,
                               parent_eval=parent_eval)
    for k in KEYS:
        assert got[k].dtype == want[k].dtype, k
        assert got[k].shape == want[k].shape, (k, got[k].shape, want[k].shape)
        assert np.array_equal(got[k], want[k]), k
    return len(want["set_off"]) - 1


@pytest.mark.parametrize("which", ["queries", "hard_queries"])
def test_harvest_matches_python_laser_order(which):
    _lib_or_skip()
    ctx, qs = getattr(laser_like, which)()
    total = 0
    for name, cs in qs:
        for k in range(1, len(cs) + 1):  # LASER order: parent prefixes first
            total += _compare(ctx.b, [c.node for c in cs[:k]])
    assert total > 0


def test_harvest_matches_python_with_parents():
    _lib_or_skip()
    ctx, qs = laser_like.queries()
    for name, cs in qs:
        root, schema = lower_query(ctx.b, [c.node for c in cs])
        cols = list(schema.columns)
        widths = [schema.columns[c].width for c in cols]
        for salt in ("a", "b"):
            _compare(ctx.b, [c.node for c in cs], _parent_of(cols, widths, name + salt))
        # a parent that shares no column with the query adds no set
        _compare(ctx.b, [c.node for c in cs], {"__not_a_column__": 1})


def test_harvest_cold_builder():
    """Each query on a fresh builder (no memo from earlier queries on the Python side)."""
    _lib_or_skip()
    names = [n for n, _ in laser_like.queries()[1]]
    for name in names:
        ctx, qs = laser_like.queries()
        cs = dict(qs)[name]
        _compare(ctx.b, [c.node for c in cs])


def test_harvest_rejects_malformed():
    _lib_or_skip()
    from mythril_amd.tape import NODE_DTYPE, Op

    nodes = np.zeros(2, dtype=NODE_DTYPE)
    nodes[0] = (int(Op.VAR), 0, 8, 0, 0, 0, 0, 0)
    nodes[1] = (int(Op.EQ), 0, 0, 0, 1, 0, 0, 0)  # operand b refers to itself
    with pytest.raises(native.SieveError):
        native.harvest_guide(nodes, np.zeros((1, 8), np.uint32), [8])
    nodes[1] = (int(Op.CONST), 0, 8, 0, 0, 0, 5, 0)  # const index out of range
    with pytest.raises(native.SieveError):
        native.harvest_guide(nodes, np.zeros((1, 8), np.uint32), [8])
    with pytest.raises(native.SieveError):  # parent column out of range
        native.harvest_guide(nodes[:1], np.zeros((1, 8), np.uint32), [8], [(3, 1)])


def _random_query(rng, ctx):
    """A random path condition over a few scalars, a calldata array and the ops the harvest
    inverts (and some it does not), built with the term API."""
    from mythril_amd import smt
    from mythril_amd.smt import (And, Concat, Extract, If, Not, Or, UGE, ULE, ULT, UGT, URem,
                                 ZeroExt, symbol_factory as sf)

    V = lambda v, w: sf.BitVecVal(v, w)  # noqa: E731
    xs = [sf.BitVecSym("x%d" % i, w) for i, w in enumerate((256, 256, 160, 32, 8))]
    cd = laser_like.Calldata("f")
    consts = [0, 1, 2, 0xFF, 0x9FA299CC, laser_like.ATTACKER, (1 << 256) - 1, 1 << 255,
              rng.getrandbits(256), rng.getrandbits(64)]

    def word(depth=0):
        k = rng.randrange(12 if depth < 3 else 3)
        if k == 0:
            return rng.choice(xs[:2])
        if k == 1:
            return ZeroExt(96, xs[2])
        if k == 2:
            return cd.word(rng.choice((0, 4, 36)))
        a = word(depth + 1)
        c = V(rng.choice(consts), 256)
        if k == 3:
            return a + c
        if k == 4:
            return a - c if rng.random() < 0.5 else c - a
        if k == 5:
            return a ^ c
        if k == 6:
            return a * V(rng.choice((3, 5, 0x10001, 6)), 256)
        if k == 7:
            return ~a if rng.random() < 0.5 else -a
        if k == 8:
            return a & V((1 << rng.choice((8, 32, 160))) - 1, 256)
        if k == 9:
            return If(ULT(xs[3], V(rng.choice(consts) & 0xFFFFFFFF, 32)), a, word(depth + 1))
        if k == 10:
            return Concat(Extract(255, 128, a), Extract(127, 0, word(depth + 1)))
        return a + word(depth + 1)

    def cond(depth=0):
        k = rng.randrange(11 if depth < 2 else 7)
        a = word()
        if k == 0:
            return a == V(rng.choice(consts), 256)
        if k == 1:
            return Extract(255, 224, a) == V(rng.choice(consts) & 0xFFFFFFFF, 32)
        if k == 2:
            return rng.choice((ULT, ULE, UGT, UGE))(a, V(rng.choice(consts), 256))
        if k == 3:
            return rng.choice((a.__lt__, a.__gt__, a.__le__, a.__ge__))(V(rng.choice(consts), 256))
        if k == 4:
            return Extract(159, 0, a) == Extract(159, 0, word())
        if k == 5:
            return Not(smt.BVAddNoOverflow(a, word(), False))
        if k == 6:
            return smt.BVSubNoUnderflow(a, word(), False) if rng.random() < 0.5 else \
                Not(smt.BVMulNoOverflow(a, word(), False))
        if k == 7:
            return Or(cond(depth + 1), cond(depth + 1))
        if k == 8:
            return Not(cond(depth + 1))
        if k == 9:
            return And(cond(depth + 1), cond(depth + 1))
        return URem(a, V(rng.choice((7, 64, 1 << 32)), 256)) == V(0, 256)

    return [cond() for _ in range(rng.randrange(1, 5))]


def test_harvest_matches_python_random_queries():
    """Random query shapes (every inversion rule, Or / Not / And nesting, symbolic equalities,
    overflow predicates, wide and narrow columns), each also with a parent witness."""
    import random

    from mythril_amd import smt

    _lib_or_skip()
    rng = random.Random(20260417)
    compared = 0
    for i in range(120):
        ctx = smt.Context()
        smt.set_context(ctx)
        cs = _random_query(rng, ctx)
        try:
            root, schema = lower_query(ctx.b, [c.node for c in cs])
        except Exception:  # noqa: BLE001 - a shape the lowering refuses is not a harvest case
            continue
        cols = list(schema.columns)
        if not cols:
            continue
        widths = [schema.columns[c].width for c in cols]
        compared += _compare(ctx.b, [c.node for c in cs]) >= 0
        _compare(ctx.b, [c.node for c in cs], _parent_of(cols, widths, "r%d" % i))
    assert compared >= 100


def test_harvest_rejects_bad_layout_nodes():
    _lib_or_skip()
    from mythril_amd.tape import NODE_DTYPE, Op

    nodes = np.zeros(2, dtype=NODE_DTYPE)
    nodes[0] = (int(Op.VAR), 0, 8, 0, 0, 0, 0, 0)
    nodes[1] = (int(Op.ZEXT), 0, 16, 0, 0, 0, 5000, 0)  # extension beyond any width
    with pytest.raises(native.SieveError):
        native.harvest_guide(nodes, np.zeros((1, 8), np.uint32), [8])
    nodes[0] = (int(Op.TRUE), 0, 0, 0, 0, 0, 0, 0)
    nodes[1] = (int(Op.SEXT), 0, 8, 0, 0, 0, 8, 0)  # sign extension of a Bool
    with pytest.raises(native.SieveError):
        native.harvest_guide(nodes, np.zeros((1, 8), np.uint32), [8])


@pytest.mark.parametrize("name", ["killbilly", "overflow", "ether_thief"])
def test_harvest_matches_python_on_grown_paths(name):
    """Paths grown to 60 constraints (tests/laser_paths.py): several bounds on one term (the ABI
    decoder's calldatasize guards, argument range checks) give interval sets; LASER order, every
    prefix, plus the UNSAT variant at 120."""
    from .laser_paths import grow

    _lib_or_skip()
    ctx, cs = grow(name, 60)
    for k in range(1, len(cs) + 1):
        _compare(ctx.b, [c.node for c in cs[:k]])
    ctx, cs = grow(name, 120, unsat=True)
    _compare(ctx.b, [c.node for c in cs])


def test_interval_sets_propose_values_inside_every_bound():
    """Not(size < 68), size < 5000, Not(size < 4): the interval set's values lie in [68, 4999]
    (the single-bound sets alone propose 4, 5, 0 ... which break the other bounds)."""
    from mythril_amd.candidates import _interval_values
    from mythril_amd.smt import Not, ULT, symbol_factory as F

    from .laser_like import Calldata

    ctx, _ = laser_like.queries()
    cd = Calldata("9")
    cs = [Not(ULT(cd.size, F.BitVecVal(68, 256))), ULT(cd.size, F.BitVecVal(5000, 256)),
          Not(ULT(cd.size, F.BitVecVal(4, 256)))]
    root, schema = lower_query(ctx.b, [c.node for c in cs])
    cols = list(schema.columns)
    g = build_guide(ctx.b, root, schema, cols)
    last = g.sets[-1][1]
    vals = sorted(a["9_calldatasize"] for a in last)
    assert vals == sorted(_interval_values(68, 4999)) and all(68 <= v <= 4999 for v in vals)
    _compare(ctx.b, [c.node for c in cs])


def test_parent_eval_harvest_matches_python():
    """mh_guide_harvest_inc (the incremental round's guide: operands the parent witness fixes
    count as known) gives candidates.build_guide(parent_eval=True)'s arrays, on the LASER-shaped
    queries and on planted random paths with their planted models as parents -- and there it
    proposes alternatives the plain harvest cannot (x + y == k solved for x at y's parent value)."""
    _lib_or_skip()
    from tests.planted import planted_path

    ctx, qs = laser_like.queries()
    for name, cs in qs:
        root, schema = lower_query(ctx.b, [c.node for c in cs])
        cols = list(schema.columns)
        widths = [schema.columns[c].width for c in cols]
        _compare(ctx.b, [c.node for c in cs], _parent_of(cols, widths, name + "p"), True)
    more = 0
    for seed in range(6):
        pctx, pcs, m, _ = planted_path("random", seed, 12)
        nodes = [c.node for c in pcs]
        for k in range(2, len(nodes) + 1, 3):
            root, schema = lower_query(pctx.b, nodes[:k])
            parent = {c: v for c, v in m.vars.items() if c in schema.columns}
            a = _compare(pctx.b, nodes[:k], parent, True)
            more += a > _compare(pctx.b, nodes[:k], parent, False)
    assert more > 0


def test_parent_eval_solves_a_sum_for_one_side():
    from mythril_amd import smt
    from mythril_amd.smt import symbol_factory as sf

    _lib_or_skip()
    ctx = smt.set_context(smt.Context())
    x, y = sf.BitVecSym("x", 256), sf.BitVecSym("y", 256)
    c = x + y == sf.BitVecVal(1000, 256)
    root, schema = lower_query(ctx.b, [c.node])
    cols = list(schema.columns)
    plain = build_guide(ctx.b, root, schema, cols, {"y": 58}).arrays()
    inc = build_guide(ctx.b, root, schema, cols, {"y": 58}, parent_eval=True).arrays()
    vals = {int(v[0]) for v in inc["entry_val"]}
    assert 942 in vals and 942 not in {int(v[0]) for v in plain["entry_val"]}
    _compare(ctx.b, [c.node], {"y": 58}, True)
