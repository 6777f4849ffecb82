"""The native query compiler (mh_query_build, mythril_amd/csrc/query.cpp) against the Python stages
it replaces in Sieve.solve: lower_query (mythril_amd/lower.py), Sieve.buckets and local_tapeset
(mythril_amd/sieve.py).

For every query -- tests/laser_like.py in LASER order (svm.py:257-262: each query is its parent's
plus one constraint), the grown paths of tests/laser_paths.py and the reference's own cases
(tests/reference_cases.py) -- the two give the same columns (name, width, kind, symbol, key), the
same harvested tables (every array / function key, keccak bases and pairs), the same
column-disjoint groups and the SAME tapes once column and constant numbering are read by name and
value: node for node, operand for operand.  Host-only (no device); the library must be built.
"""
import numpy as np
import pytest

from mythril_amd import native
from mythril_amd.lower import LoweringUnsupported, lower_query
from mythril_amd.sieve import Sieve, eliminate_definitions, local_tapeset
from mythril_amd.tape import ARITY, Op
from tests import laser_like
from tests.laser_paths import grow
from tests.reference_cases import CASES


def canon(nodes, columns, consts):
    """A tape with VAR read as its column name and CONST as its value."""
    out = []
    for op, _, w, a, b, c, i0, i1 in nodes.tolist():
        k = ARITY[Op(op)]
        if op == Op.VAR:
            i0 = columns[i0]
        elif op == Op.CONST:
            i0 = consts[i0]
        out.append((op, w, a if k > 0 else 0, b if k > 1 else 0, c if k > 2 else 0, i0, i1))
    return out


def _values(rows):
    return native._ints(rows)


def python_stages(b, roots, keccak_reads=False):
    """The Python host stages of Sieve._host_python: lowering, definitions (solved for and
    substituted away, Sieve.solve_definitions), groups, the root tape."""
    root, schema = lower_query(b, roots, keccak_reads=keccak_reads)
    cols = list(schema.columns) or ["__ground__"]
    rest, defs = eliminate_definitions(b, Sieve.conjuncts(b, root), schema)
    if defs:
        root = rest[0] if rest else b.true()
        for x in rest[1:]:
            root = b.op(Op.AND, root, x)
    groups = Sieve.buckets(b, root)
    names = {b.var_index[c]: c for c in cols if c in b.var_index}
    ts = local_tapeset(b, [root], cols)
    return root, schema, cols, groups, names, ts, defs


def check_query(b, roots, label, keccak_reads=False):
    try:
        root, schema, cols, groups, names, ts, defs = python_stages(b, roots, keccak_reads)
    except LoweringUnsupported:
        with pytest.raises(native.Unsupported):
            native.TermMirror.of(b, keccak_reads).build(b, roots)
        return None
    cq = native.TermMirror.of(b, keccak_reads).build(b, roots)
    # columns
    got = {n: (w, k, s, key) for n, w, k, s, key in cq.columns}
    want = {c.name: (c.width, c.kind, c.symbol, c.key) for c in schema.columns.values()}
    if not want:
        want = {"__ground__": (1, "var", "__ground__", None)}
    assert got == want, label
    # tables
    tabs = {(k, n): items for k, n, items in cq.tables}
    for arr, cells in schema.cells.items():
        assert tabs.pop((native.TABLE_CELLS, arr)) == sorted(cells), (label, arr)
    for f, cells in schema.uf_cells.items():
        assert tabs.pop((native.TABLE_UF_CELLS, f)) == sorted(cells), (label, f)
    for f, km in schema.keccak.items():
        items = tabs.pop((native.TABLE_KECCAK, f))
        assert items[0] == km.base % (1 << 256), (label, f)
        assert dict(zip(items[1::2], items[2::2])) == km.pairs, (label, f)
    assert not tabs, (label, tabs)
    # groups (column sets, in order of their first conjunct)
    ncols = [c[0] for c in cq.columns]
    want_groups = [sorted(names[v] for v in vs) for _, vs in groups]
    got_groups = [sorted(ncols[i] for i in g) for g in cq.groups]
    assert got_groups == want_groups, label
    # the root tape, node for node
    assert canon(cq.tapes[0], ncols, _values(cq.consts)) == \
        canon(ts.tapes[0].nodes, cols, _values(ts.pool.to_array())), label
    # the group tapes
    if len(groups) > 1:
        accs = [acc for acc, _ in Sieve.bucket_roots(b, root)]
        gts = local_tapeset(b, accs, cols)
        assert len(cq.tapes) == 1 + len(accs), label
        pool = _values(gts.pool.to_array())
        for t, gt in zip(cq.tapes[1:], gts.tapes):
            assert canon(t, ncols, _values(cq.consts)) == canon(gt.nodes, cols, pool), label
    else:
        assert len(cq.tapes) == 1, label
    # definitions: the same symbols solved for, in the same order, by the same terms
    assert bool(cq.flags & native.QUERY_DEFINITIONS) == bool(defs), label
    assert [ncols[c] for c in cq.defs] == [c for c, _ in defs], label
    if defs:
        dts = local_tapeset(b, [t for _, t in defs], cols)
        pool = _values(dts.pool.to_array())
        for t, dt in zip(cq.def_tapes, dts.tapes):
            assert canon(t, ncols, _values(cq.consts)) == canon(dt.nodes, cols, pool), label
    return cq


@pytest.mark.parametrize("which", ["queries", "hard_queries"])
def test_laser_like_in_laser_order(which):
    ctx, qs = getattr(laser_like, which)()
    n = 0
    for name, cs in qs:
        nodes = [c.node for c in cs]
        for k in range(1, len(nodes) + 1):
            cq = check_query(ctx.b, nodes[:k], (name, k))
            if which == "queries" and name != "unsat_actor":  # SAT: never refuted
                assert not cq.flags & native.QUERY_REFUTED, (name, k)
            n += 1
    assert n > 20


@pytest.mark.parametrize("shape", ["killbilly", "overflow", "ether_thief"])
def test_grown_paths(shape):
    for n, unsat in ((25, False), (60, True)):
        ctx, cs = grow(shape, n, unsat=unsat)
        nodes = [c.node for c in cs]
        for k in (1, n // 3, n - 1, n):
            check_query(ctx.b, nodes[:k], (shape, n, k))


@pytest.mark.parametrize("case", CASES, ids=[c.name for c in CASES])
def test_reference_cases(case):
    ctx, cs = case.build()
    nodes = [c.node for c in cs if hasattr(c, "node")]
    cq = check_query(ctx.b, nodes, case.name)
    if case.expected == "sat" and cq is not None:
        assert not cq.flags & native.QUERY_REFUTED, case.name


def test_refutation():
    """MH_QUERY_REFUTED: syntactic contradictions are found, satisfiable neighbours are not."""
    from mythril_amd import smt
    from mythril_amd.smt import Not, ULE, ULT, UGT, symbol_factory

    ctx = smt.set_context(smt.Context())
    x = symbol_factory.BitVecSym("x", 256)
    y = symbol_factory.BitVecSym("y", 8)
    p = x + 1 == 7
    v = symbol_factory.BitVecVal

    def refuted(*cs):
        return bool(native.TermMirror.of(ctx.b).build(ctx.b, [c.node for c in cs]).flags
                    & native.QUERY_REFUTED)

    assert refuted(x == 1, x == 2)
    assert refuted(p, Not(p))
    assert refuted(x == 5, Not(x == 5))
    assert refuted(ULT(x, v(10, 256)), UGT(x, v(20, 256)))
    assert refuted(ULT(x, v(0, 256)))
    assert refuted(UGT(y, v(255, 8)))
    assert refuted(ULE(x, v(3, 256)), Not(ULT(x, v(4, 256))))
    assert refuted(ULE(v(4, 256), x), ULE(x, v(4, 256)), Not(x == 4))
    assert not refuted(x == 1, x + 0 == 1)
    assert not refuted(ULT(x, v(10, 256)), UGT(x, v(8, 256)))
    assert not refuted(ULE(x, v(4, 256)), ULE(v(4, 256), x))
    assert not refuted(p, x == 6)  # refuted by arithmetic, not syntax: the device decides
    assert not refuted(Not(x == 5), ULE(x, v(6, 256)))
    assert not refuted(y == 255, UGT(y, v(254, 8)))
    # the no-overflow predicates and term-term comparisons, decided by the operands' ranges
    from mythril_amd.smt import BVAddNoOverflow, BVMulNoOverflow, BVSubNoUnderflow

    z = symbol_factory.BitVecSym("z", 256)
    lim = v(1 << 128, 256)
    assert refuted(ULT(x, lim), ULT(z, lim), Not(BVAddNoOverflow(x, z, False)))
    assert not refuted(ULT(x, lim), Not(BVAddNoOverflow(x, z, False)))
    assert refuted(ULT(x, v(1 << 100, 256)), ULT(z, v(1 << 100, 256)),
                   Not(BVMulNoOverflow(x, z, False)))
    assert not refuted(ULT(x, v(1 << 200, 256)), ULT(z, v(1 << 100, 256)),
                       Not(BVMulNoOverflow(x, z, False)))
    assert refuted(ULT(x, v(5, 256)), UGT(z, v(9, 256)), Not(ULT(x, z)))
    assert not refuted(ULT(x, v(5, 256)), UGT(z, v(3, 256)), Not(ULT(x, z)))
    assert refuted(UGT(x, v(9, 256)), ULT(z, v(5, 256)), Not(BVSubNoUnderflow(x, z, False)))
    assert not refuted(UGT(x, v(2, 256)), ULT(z, v(5, 256)), Not(BVSubNoUnderflow(x, z, False)))


def test_unsat_shapes_refuted():
    """tests/laser_like.py hard_queries: KillBilly's third sender pinned to two actors, and the
    transfer overflow of two words below 2^128, are refuted without a device round (also on the
    grown paths); k_storage_unsat and ether_thief_unsat need more than syntax and ranges."""
    ctx, qs = laser_like.hard_queries()
    flags = {n: native.TermMirror.of(ctx.b).build(ctx.b, [c.node for c in cs]).flags
             for n, cs in qs}
    assert flags["killbilly_unsat"] & native.QUERY_REFUTED
    assert flags["overflow_unsat"] & native.QUERY_REFUTED
    assert not flags["ether_thief_unsat"] & native.QUERY_REFUTED
    for shape in ("killbilly", "overflow"):
        ctx, cs = grow(shape, 100, unsat=True)
        cq = native.TermMirror.of(ctx.b).build(ctx.b, [c.node for c in cs])
        assert cq.flags & native.QUERY_REFUTED, shape
        ctx, cs = grow(shape, 100)
        cq = native.TermMirror.of(ctx.b).build(ctx.b, [c.node for c in cs])
        assert not cq.flags & native.QUERY_REFUTED, shape


def test_empty_and_ground_queries():
    from mythril_amd import smt
    from mythril_amd.smt import symbol_factory

    ctx = smt.set_context(smt.Context())
    cq = check_query(ctx.b, [], "empty")
    assert [c[0] for c in cq.columns] == ["__ground__"]
    one = symbol_factory.BitVecVal(1, 256)
    check_query(ctx.b, [(one == one).node, (one != one).node], "ground")


def test_mirror_is_incremental():
    """A second query appends only the builder's new nodes; sizes match the builder."""
    from mythril_amd import smt
    from mythril_amd.smt import symbol_factory

    ctx = smt.set_context(smt.Context())
    x = symbol_factory.BitVecSym("x", 256)
    check_query(ctx.b, [(x == 3).node], "one")
    m = native.TermMirror.of(ctx.b)
    n1 = m.n[0]
    y = symbol_factory.BitVecSym("y", 256)
    check_query(ctx.b, [(x == 3).node, (y > x).node], "two")
    assert m.n[0] == len(ctx.b.nodes) > n1
    sizes = (native.C.c_uint64 * 5)()
    native._check(m.lib.mh_terms_sizes(m.h, sizes))
    assert list(sizes) == [len(ctx.b.nodes), len(ctx.b.pool.values), len(ctx.b.var_index),
                           len(ctx.b.symbols.array_names), len(ctx.b.symbols.function_names)]


def test_malformed_append_is_refused():
    m = native.TermMirror()
    bad = native.np.zeros(1, dtype=native.NODE_DTYPE)
    bad["op"] = int(Op.BVADD)
    bad["a"] = 5  # operand after the node itself
    with pytest.raises(native.SieveError):
        native._check(m.lib.mh_terms_append(m.h, bad.ctypes.data, 1, None, 0, None, 0, None, 0,
                                            None, 0))
    roots = native.np.zeros(1, dtype=native.np.uint32)
    with pytest.raises(native.SieveError):
        native._check(m.lib.mh_query_build(m.h, native._ptr(roots), 1,
                                           native.C.byref(native.C.c_void_p()),
                                           native.C.byref(native.QueryInfo())))
    m.close()


def test_rejected_append_changes_nothing():
    """A batch with a bad node after constants and good nodes leaves the store as it was (no
    constant lands twice when the batch is sent again), and the next good batch appends."""
    m = native.TermMirror()
    sizes = (native.C.c_uint64 * 5)()

    def store():
        native._check(m.lib.mh_terms_sizes(m.h, sizes))
        return list(sizes)

    consts = native.np.arange(16, dtype=native.np.uint32)  # two 256-bit constants
    batch = native.np.zeros(3, dtype=native.NODE_DTYPE)
    batch["op"] = [int(Op.CONST), int(Op.CONST), int(Op.BVADD)]
    batch["width"] = 256
    batch["imm0"] = [0, 1, 0]
    batch["a"], batch["b"] = [0, 0, 0], [0, 0, 1]
    bad = batch.copy()
    bad["a"][2] = 7  # operand outside the store
    with pytest.raises(native.SieveError):
        native._check(m.lib.mh_terms_append(m.h, bad.ctypes.data, 3, native._ptr(consts), 2,
                                            b"v\0", 1, None, 0, None, 0))
    assert store() == [0, 0, 0, 0, 0]
    bad2 = batch.copy()
    bad2["imm0"][1] = 2  # a constant index past this batch's constants
    with pytest.raises(native.SieveError):
        native._check(m.lib.mh_terms_append(m.h, bad2.ctypes.data, 3, native._ptr(consts), 2,
                                            None, 0, None, 0, None, 0))
    assert store() == [0, 0, 0, 0, 0]
    native._check(m.lib.mh_terms_append(m.h, batch.ctypes.data, 3, native._ptr(consts), 2,
                                        b"v\0", 1, None, 0, None, 0))
    assert store() == [3, 2, 1, 0, 0]
    m.close()


def test_refutation_is_sound_on_random_conjunctions():
    """Random conjunctions of comparisons, negations, ULE/UGE (Or forms) and the no-overflow
    predicates over three 4-bit symbols: every one MH_QUERY_REFUTED flags has no satisfying
    assignment (all 4096 enumerated with the oracle), and some are flagged."""
    import itertools
    import random

    from mythril_amd import smt
    from mythril_amd.smt import (And, BVAddNoOverflow, BVMulNoOverflow, BVSubNoUnderflow, Not,
                                 UGE, UGT, ULE, ULT, symbol_factory)
    from oracle import smt_eval as E

    rng = random.Random(77)
    flagged = 0
    for trial in range(150):
        ctx = smt.set_context(smt.Context())
        xs = [symbol_factory.BitVecSym(n, 4) for n in "xyz"]

        def term():
            return rng.choice(xs) if rng.random() < 0.8 else symbol_factory.BitVecVal(
                rng.randrange(16), 4)

        def atom():
            a, b = term(), term()
            k = rng.randrange(9)
            c = [lambda: a == b, lambda: ULT(a, b), lambda: UGT(a, b), lambda: ULE(a, b),
                 lambda: UGE(a, b), lambda: BVAddNoOverflow(a, b, False),
                 lambda: BVMulNoOverflow(a, b, False), lambda: BVSubNoUnderflow(a, b, False),
                 lambda: a == symbol_factory.BitVecVal(rng.randrange(16), 4)][k]()
            return Not(c) if rng.random() < 0.3 else c

        cs = [atom() for _ in range(rng.randrange(2, 6))]
        cs = [c for c in cs if not isinstance(c, bool)]
        if not cs:
            continue
        try:
            cq = native.TermMirror.of(ctx.b).build(ctx.b, [c.node for c in cs])
        except native.SieveError:
            continue
        if not cq.flags & native.QUERY_REFUTED:
            continue
        flagged += 1
        tape = ctx.b.finish(And(*cs).node)
        names = sorted(ctx.b.var_index, key=ctx.b.var_index.get)
        for vals in itertools.product(range(16), repeat=3):
            assign = [dict(zip("xyz", vals)).get(n, 0) for n in names]
            assert not E.evaluate(tape.nodes, ctx.b.pool.values, assign), (trial, vals)
    assert flagged >= 10


def _guide_equal(a, b):
    return a.keys() == b.keys() and all(np.array_equal(a[k], b[k]) for k in a)


@pytest.mark.parametrize("shape", ["killbilly", "overflow", "ether_thief"])
def test_guide_session_matches_fresh_harvest(shape):
    """mh_guide_harvest_with (a harvester kept across a path's queries) gives the arrays of
    mh_guide_harvest on every query of a grown path in LASER order, with and without a parent
    witness, and reuses its memo for the children that extend their parent's tape."""
    import random

    ctx, cs = grow(shape, 60)
    nodes = [c.node for c in cs]
    sess = native.GuideSession()
    rng = random.Random(5)
    m = native.TermMirror.of(ctx.b)
    for k in range(1, len(nodes) + 1):
        cq = m.build(ctx.b, nodes[:k])
        parent = [(c, rng.getrandbits(int(cq.widths[c]))) for c in range(len(cq.names))
                  if rng.random() < 0.3] if k % 2 else ()
        want = native.harvest_guide(cq.tapes[0], cq.consts, cq.widths, parent)
        got = native.harvest_guide(cq.tapes[0], cq.consts, cq.widths, parent, session=sess)
        assert _guide_equal(got, want), (shape, k)
    reused, fresh, _ = sess.stats()
    assert reused > len(nodes) // 2, (reused, fresh)
    sess.close()


def test_guide_session_laser_like():
    ctx, qs = laser_like.queries()
    sess = native.GuideSession()
    m = native.TermMirror.of(ctx.b)
    for name, cs in qs:
        nodes = [c.node for c in cs]
        for k in range(1, len(nodes) + 1):
            cq = m.build(ctx.b, nodes[:k])
            want = native.harvest_guide(cq.tapes[0], cq.consts, cq.widths)
            got = native.harvest_guide(cq.tapes[0], cq.consts, cq.widths, session=sess)
            assert _guide_equal(got, want), (name, k)
    sess.close()


@pytest.mark.parametrize("family", ["random", "laser"])
def test_guide_session_planted_paths(family):
    """The session's per-conjunct and per-(equality, constant) contributions (harvest.cpp
    Harvester::conj_done / eq_plan) replay exactly what a fresh harvest computes: planted paths
    (keccak manager conditions, stores, wide equalities) in LASER order, every prefix."""
    from tests.planted import planted_path

    for seed in range(3):
        ctx, cs, _, _ = planted_path(family, seed, 20)
        nodes = [c.node for c in cs]
        sess = native.GuideSession()
        m = native.TermMirror.of(ctx.b)
        for k in range(1, len(nodes) + 1):
            try:
                cq = m.build(ctx.b, nodes[:k])
            except native.Unsupported:
                continue
            if cq.flags & native.QUERY_REFUTED:
                continue
            want = native.harvest_guide(cq.tapes[0], cq.consts, cq.widths)
            got = native.harvest_guide(cq.tapes[0], cq.consts, cq.widths, session=sess)
            assert _guide_equal(got, want), (family, seed, k)
        sess.close()


def _random_query(rng, n):
    """n random constraints over free arrays, K arrays, store chains, selects at constant and
    symbolic indices, a tabled function, a keccak function with concrete pairs, bounds and its
    inverse, and a wide (512-bit) equality of concatenations."""
    from mythril_amd import smt
    from mythril_amd.smt import (K, Array, Concat, Function, If, Not, ULT, UGT,
                                 symbol_factory)

    ctx = smt.set_context(smt.Context())
    v = symbol_factory.BitVecVal
    xs = [symbol_factory.BitVecSym("x%d" % i, 256) for i in range(3)]
    arrs = [Array("A", 256, 256), Array("B", 256, 8)]
    kar = K(256, 256, 7)
    f = Function("f", 256, 256)
    kec = Function("keccak256_256", 256, 256)
    inv = Function("keccak256_256-1", 256, 256)
    keys = [v(k, 256) for k in (0, 1, 4, 36, 1 << 160)]

    def term(d=0):
        r = rng.random()
        if d > 2 or r < 0.25:
            return rng.choice(xs + keys)
        if r < 0.45:
            a = rng.choice(arrs + [kar])
            idx = rng.choice(keys) if rng.random() < 0.6 else term(d + 1)
            if a.range == 8:
                return smt.ZeroExt(248, a[idx])
            return a[idx]
        if r < 0.55:
            return f(rng.choice(keys) if rng.random() < 0.5 else term(d + 1))
        if r < 0.65:
            return kec(term(d + 1))
        if r < 0.7:
            return inv(kec(term(d + 1)))
        if r < 0.85:
            return term(d + 1) + term(d + 1)
        return If(ULT(term(d + 1), term(d + 1)), term(d + 1), term(d + 1))

    cs = []
    for _ in range(n):
        r = rng.random()
        if r < 0.1:  # a store into a free array, read back
            a = rng.choice(arrs[:1])
            a[rng.choice(keys)] = term(1)
            cs.append(a[term(2)] == term(2))
        elif r < 0.2:
            cs.append(kec(rng.choice(keys)) == v(rng.getrandbits(256), 256))
        elif r < 0.3:
            cs.append(UGT(kec(term(1)), v(rng.getrandbits(200) << 40, 256)))
        elif r < 0.38:
            cs.append(Concat(term(1), term(1)) == Concat(term(1), term(1)))
        elif r < 0.7:
            c = term() == term()
            cs.append(Not(c) if rng.random() < 0.3 else c)
        else:
            cs.append(ULT(term(), term()))
    return ctx, cs


@pytest.mark.parametrize("seed", range(40))
def test_random_queries_match_python_stages(seed):
    """Random queries over arrays, stores, K, a tabled function, keccak with pairs / bounds /
    inverse and wide equalities, built in LASER order (every prefix: extensions and afresh
    builds both happen): the native result equals the Python stages node for node."""
    import random

    rng = random.Random(seed)
    ctx, cs = _random_query(rng, 10)
    nodes = [c.node for c in cs if hasattr(c, "node")]
    for k in range(1, len(nodes) + 1):
        check_query(ctx.b, nodes[:k], (seed, k))


@pytest.mark.parametrize("seed", range(24))
def test_random_queries_in_jumpi_order(seed):
    """Both branches of every constraint, as LASER asks a JUMPI's two states (svm.py:257-262):
    the path with the condition, then with its negation, and the walk goes on from the first --
    so the second branch and the next query are not children of the last query and are built
    afresh, taking over the last query's lowering when the harvests agree (query.cpp
    QueryState::start).  Node for node the Python stages' result either way."""
    import random

    from mythril_amd.smt import Not

    rng = random.Random(seed)
    ctx, cs = _random_query(rng, 10)
    cs = [c for c in cs if hasattr(c, "node")]
    nodes = [c.node for c in cs]
    for k in range(1, len(nodes) + 1):
        check_query(ctx.b, nodes[:k], (seed, k, "taken"))
        check_query(ctx.b, nodes[:k - 1] + [Not(cs[k - 1]).node], (seed, k, "other"))


@pytest.mark.parametrize("shape", ["killbilly", "overflow", "ether_thief"])
def test_grown_paths_in_jumpi_order(shape):
    from mythril_amd.smt import Not

    ctx, cs = grow(shape, 40)
    nodes = [c.node for c in cs]
    for k in range(1, len(nodes) + 1):
        check_query(ctx.b, nodes[:k], (shape, k, "taken"))
        check_query(ctx.b, nodes[:k - 1] + [Not(cs[k - 1]).node], (shape, k, "other"))


def test_mirror_shared_by_threads():
    """Sieves of several threads over one builder take turns on its session: every result is the
    one a single thread gets."""
    import threading

    ctx, qs = laser_like.queries()
    want = {}
    for name, cs in qs:
        cq = native.TermMirror.of(ctx.b).build(ctx.b, [c.node for c in cs])
        want[name] = [t.tobytes() for t in cq.tapes]
    errors = []

    def work(seed):
        import random

        rng = random.Random(seed)
        for _ in range(30):
            name, cs = rng.choice(qs)
            cq = native.TermMirror.of(ctx.b).build(ctx.b, [c.node for c in cs])
            if [t.tobytes() for t in cq.tapes] != want[name]:
                errors.append(name)

    th = [threading.Thread(target=work, args=(i,)) for i in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors


def test_builder_packed_nodes_match_the_node_list():
    """TapeBuilder.node_bytes (the mh_node records TermMirror.sync hands over as they are) equals
    the builder's node tuples and flags, for nodes made by TapeBuilder._add and by the SMT-LIB
    reader's inlined merge (native.SmtlibSession._merge)."""
    import random

    from mythril_amd import smtlib
    from mythril_amd.native import NODE_DTYPE
    from tests.laser_like import queries
    from tests.z3_style import z3_sexpr

    ctx, qs = queries()
    nat = smtlib.NativeReader()
    for _, cs in qs[:6]:
        for c in cs:
            nat.read(z3_sexpr(c), smtlib.Query(nat.ctx))
    ctx2, _ = _random_query(random.Random(3), 9)
    for b in (ctx.b, nat.b, ctx2.b):
        got = np.frombuffer(bytes(b.node_bytes), dtype=NODE_DTYPE)
        assert len(got) == len(b.nodes)
        want = np.array([(n[0], f, n[1], n[2], n[3], n[4], n[5], n[6])
                         for n, f in zip(b.nodes, b.flags)], dtype=NODE_DTYPE)
        assert (got == want).all()


def test_definitions_are_solved_natively():
    """Definitions eliminated by the native compiler: a chain of them kept
    closed, a query that is nothing but definitions (TRUE root), the keccak_other_num shape, in
    LASER order -- each equal to the Python stages (check_query), and the defined column's tape
    evaluates, under a row satisfying the rest, to a value that satisfies the whole query."""
    from mythril_amd import smt
    from mythril_amd.smt import ULT, symbol_factory
    from oracle import smt_eval as E

    ctx = smt.set_context(smt.Context())
    v = symbol_factory.BitVecVal
    a, b_, c, d = (symbol_factory.BitVecSym(n, 256) for n in "abcd")
    cs = [b_ == a * v(3, 256) + v(1, 256),       # b := 3a + 1
          c == b_ + a,                            # c := b + a, closed: 4a + 1
          ULT(a, v(1000, 256)),
          d == c * c]                             # d := (4a + 1)^2
    nodes = [x.node for x in cs]
    seen_defs = []
    for k in range(1, len(nodes) + 1):
        cq = check_query(ctx.b, nodes[:k], ("chain", k))
        seen_defs.append(len(cq.defs))
    assert seen_defs == [1, 2, 2, 3]
    ncols = cq.names
    assert sorted(ncols[c] for c in cq.defs) == ["b", "c", "d"]
    # the remaining root reads only a; evaluate the definitions at a = 5
    row = [5 if n == "a" else 0 for n in ncols]
    consts = _values(cq.consts)
    got = {ncols[c]: E.evaluate(t, consts, row) for c, t in zip(cq.defs, cq.def_tapes)}
    assert got == {"b": 16, "c": 21, "d": 441}
    # nothing but definitions: the root is TRUE, one ground group
    cq = check_query(ctx.b, [nodes[0]], "one")
    assert cq.flags & native.QUERY_DEFINITIONS and len(cq.tapes) == 1
    assert int(cq.tapes[0]["op"][-1]) == int(Op.TRUE)


@pytest.mark.parametrize("shape,k,seed", [("killbilly", 4, 0), ("overflow", 8, 1),
                                          ("ether_thief", 4, 2), ("ether_thief", 8, 3)])
def test_grown_paths_in_bfs_order(shape, k, seed):
    """both branches of every JUMPI, the open states interleaved the way
    LASER's BFS pops them (cli.py:417-419, svm.py:243-262; tests/bfs_order.py).  The session's
    state is taken back to the common prefix of each query's roots and extended by the rest
    (query.cpp mh_query_build): node for node the Python stages' result in that order, and past
    the first queries every query is built from the state, none afresh."""
    from mythril_amd.smt import Not
    from tests.bfs_order import bfs_queries

    from mythril_amd.lower import Lowering

    ctx, cs = grow(shape, 30)
    nodes = [c.node for c in cs]
    negs = [Not(c).node for c in cs]
    last_fp, fresh, dropped = None, [], set()
    for i, roots in enumerate(bfs_queries(nodes, negs, 18, k, seed, dropped)):
        cq = check_query(ctx.b, roots, (shape, k, i))
        if cq is not None and cq.flags & native.QUERY_REFUTED:
            dropped.add(tuple(roots))
        fp = Lowering(ctx.b).collect(roots).fingerprint()
        if cq is not None and i > 0 and not cq.flags & native.QUERY_INCREMENTAL:
            fresh.append((i, fp != last_fp))
        last_fp = fp
    # afresh only where the query's harvest (constant keys, keccak pairs and bounds) is not the
    # last query's: the lowering depends on it
    assert all(changed for _, changed in fresh), fresh


@pytest.mark.parametrize("seed", range(8))
def test_random_queries_in_bfs_order(seed):
    """The same over random array / function / keccak conjunctions (a new constraint may change
    the harvest: that query is built afresh, still node for node the Python stages' result)."""
    import random

    from mythril_amd.smt import Not
    from tests.bfs_order import bfs_queries

    rng = random.Random(100 + seed)
    ctx, cs = _random_query(rng, 10)
    cs = [c for c in cs if hasattr(c, "node")]
    nodes = [c.node for c in cs]
    negs = [Not(c).node for c in cs]
    dropped = set()
    for i, roots in enumerate(bfs_queries(nodes, negs, 3, 4, seed, dropped)):
        cq = check_query(ctx.b, roots, (seed, i))
        if cq is not None and cq.flags & native.QUERY_REFUTED:
            dropped.add(tuple(roots))


@pytest.mark.parametrize("shape,k", [("killbilly", 4), ("ether_thief", 8), ("overflow", 4)])
def test_guide_session_in_bfs_order(shape, k):
    """The harvester session in BFS / JUMPI order: a tape that shares only a prefix with the
    last one (the other branch: the path's tape, then other nodes) keeps the memo of the prefix
    and gives the rest a new node generation (harvest.cpp Harvester::truncate) -- the arrays
    are those of a fresh harvest on every query, and most queries reuse the session."""
    import random

    from mythril_amd.smt import Not
    from tests.bfs_order import bfs_queries

    ctx, cs = grow(shape, 40)
    nodes = [c.node for c in cs]
    negs = [Not(c).node for c in cs]
    sess = native.GuideSession()
    rng = random.Random(7)
    m = native.TermMirror.of(ctx.b)
    n, dropped = 0, set()
    for i, roots in enumerate(bfs_queries(nodes, negs, 20, k, 3, dropped)):
        cq = m.build(ctx.b, roots)
        if cq.flags & native.QUERY_REFUTED:
            dropped.add(tuple(roots))
        parent = [(c, rng.getrandbits(int(cq.widths[c]))) for c in range(len(cq.names))
                  if rng.random() < 0.3] if i % 3 == 0 else ()
        want = native.harvest_guide(cq.tapes[0], cq.consts, cq.widths, parent)
        got = native.harvest_guide(cq.tapes[0], cq.consts, cq.widths, parent, session=sess)
        assert _guide_equal(got, want), (shape, k, i)
        n += 1
    reused, fresh, _ = sess.stats()
    assert reused >= 0.9 * n, (reused, fresh, n)
    sess.close()


@pytest.mark.parametrize("family", ["random", "laser"])
def test_guide_session_planted_paths_in_jumpi_order(family):
    """Planted paths (keccak conditions, stores, wide equalities) with both branches of every
    constraint asked: the session's arrays equal a fresh harvest's on every query."""
    from mythril_amd.smt import Not
    from tests.planted import planted_path

    for seed in range(3):
        ctx, cs, _, _ = planted_path(family, seed, 16)
        nodes = [c.node for c in cs]
        negs = [Not(c).node for c in cs]
        sess = native.GuideSession()
        m = native.TermMirror.of(ctx.b)
        for kk in range(1, len(nodes) + 1):
            for roots in (nodes[:kk], nodes[:kk - 1] + [negs[kk - 1]]):
                try:
                    cq = m.build(ctx.b, roots)
                except native.Unsupported:
                    continue
                if cq.flags & native.QUERY_REFUTED:
                    continue
                want = native.harvest_guide(cq.tapes[0], cq.consts, cq.widths)
                got = native.harvest_guide(cq.tapes[0], cq.consts, cq.widths, session=sess)
                assert _guide_equal(got, want), (family, seed, kk)
        sess.close()


@pytest.mark.parametrize("seed", range(24))
def test_keccak_reads_match_python_stages(seed):
    _kreads_parity(seed)


def _kreads_parity(seed):
    """The second-chance lowering (MH_TERMS_KECCAK_READS / lower_query(keccak_reads=True)): keccak
    applications as read columns with the injectivity and pair conjuncts -- node for node the
    Python stages' result, in LASER order and both branches of every constraint (JUMPI order),
    on a session of its own beside the default one (whose results are unchanged)."""
    import random

    from mythril_amd.smt import Not

    rng = random.Random(500 + seed)
    ctx, cs = _random_query(rng, 10)
    cs = [c for c in cs if hasattr(c, "node")]
    nodes = [c.node for c in cs]
    kreads = 0
    for k in range(1, len(nodes) + 1):
        cq = check_query(ctx.b, nodes[:k], (seed, k, "taken"), keccak_reads=True)
        kreads += cq is not None and any(c[2] == "kread" for c in cq.columns)
        check_query(ctx.b, nodes[:k], (seed, k, "default"))
        check_query(ctx.b, nodes[:k - 1] + [Not(cs[k - 1]).node], (seed, k, "other"),
                    keccak_reads=True)
    return kreads


def test_keccak_reads_are_made():
    """The random family does apply keccak at symbolic arguments (the parity above is not
    vacuous), and the LASER-shaped queries and grown paths match in that mode too."""
    assert sum(_kreads_parity(s) for s in range(6)) > 0
    ctx, qs = laser_like.queries()
    for name, cs in qs:
        nodes = [c.node for c in cs]
        for k in range(1, len(nodes) + 1):
            check_query(ctx.b, nodes[:k], (name, k), keccak_reads=True)
    for shape in ("killbilly", "overflow", "ether_thief"):
        ctx, cs = grow(shape, 25)
        nodes = [c.node for c in cs]
        for k in (1, 12, 25):
            check_query(ctx.b, nodes[:k], (shape, k), keccak_reads=True)


@pytest.mark.parametrize("seed", range(6))
def test_keccak_reads_in_bfs_order(seed):
    import random

    from mythril_amd.smt import Not
    from tests.bfs_order import bfs_queries

    rng = random.Random(700 + seed)
    ctx, cs = _random_query(rng, 10)
    cs = [c for c in cs if hasattr(c, "node")]
    nodes = [c.node for c in cs]
    negs = [Not(c).node for c in cs]
    dropped = set()
    for i, roots in enumerate(bfs_queries(nodes, negs, 3, 4, seed, dropped)):
        cq = check_query(ctx.b, roots, (seed, i), keccak_reads=True)
        if cq is not None and cq.flags & native.QUERY_REFUTED:
            dropped.add(tuple(roots))


@pytest.mark.parametrize("shape,k,seed", [("killbilly", 4, 0), ("ether_thief", 8, 3)])
def test_parent_len_splits_the_root_tape(shape, k, seed):
    """mh_query_info.parent_len: the root tape's first parent_len nodes are the tape of the query
    without its last root (linearised root by root), so the root is that prefix's root AND the
    newest root's conjuncts (sieve.newest_tape) -- on every row, in LASER, JUMPI and BFS order
    (random rows, the ORACLE evaluating all three tapes)."""
    import random

    from mythril_amd.sieve import newest_tape
    from mythril_amd.smt import Not
    from oracle import smt_eval as E
    from tests.bfs_order import bfs_queries

    ctx, cs = grow(shape, 30)
    nodes = [c.node for c in cs]
    negs = [Not(c).node for c in cs]
    m = native.TermMirror.of(ctx.b)
    rng = random.Random(seed)
    split = 0
    for roots in bfs_queries(nodes, negs, 18, k, seed, set()):
        cq = m.build(ctx.b, roots)
        if cq.flags & native.QUERY_DEFINITIONS or len(roots) < 2:
            assert cq.parent_len == 0
            continue
        t = cq.tapes[0]
        p = cq.parent_len
        assert 0 < p < len(t)
        ends = cq.root_ends
        assert len(ends) == len(roots) - 1 and ends[-1] == p and ends == sorted(ends)
        d = rng.randrange(1, len(roots))  # an ancestor's prefix splits the tape the same way
        anc = newest_tape(t, ends[d - 1])
        assert anc is not None
        inc = newest_tape(t, p)
        assert inc is not None
        hop = newest_tape(t, p, 1)  # plus the parent's conjuncts sharing a column: still implied
        assert hop is not None and len(hop) >= len(inc)
        split += 1
        consts = native._ints(cq.consts)
        for _ in range(4):
            row = [rng.getrandbits(int(w)) for w in cq.widths]
            whole = E.evaluate(t, consts, row)
            assert whole == (E.evaluate(t[:p], consts, row) and E.evaluate(inc, consts, row))
            assert not whole or E.evaluate(hop, consts, row)
            e = ends[d - 1]
            assert whole == (E.evaluate(t[:e], consts, row) and E.evaluate(anc, consts, row))
    assert split > 10
