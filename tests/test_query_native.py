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


def python_stages(b, roots):
    root, schema = lower_query(b, roots)
    cols = list(schema.columns) or ["__ground__"]
    groups = Sieve.buckets(b, root)
    names = {b.var_index[c]: c for c in cols if c in b.var_index}
    ts = local_tapeset(b, [root], cols)
    return root, schema, cols, groups, names, ts


def check_query(b, roots, label):
    try:
        root, schema, cols, groups, names, ts = python_stages(b, roots)
    except LoweringUnsupported:
        with pytest.raises(native.Unsupported):
            native.TermMirror.of(b).build(b, roots)
        return None
    cq = native.TermMirror.of(b).build(b, roots)
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
    # a query the Python stages would eliminate a definition in is flagged
    _, defs = eliminate_definitions(b, Sieve.conjuncts(b, root), schema)
    if defs:
        assert cq.flags & native.QUERY_DEFINITIONS, label
    return cq


@pytest.mark.parametrize("which", ["queries", "hard_queries"])
def test_laser_like_in_laser_order(which):
    ctx, qs = getattr(laser_like, which)()
    n = 0
    for name, cs in qs:
        nodes = [c.node for c in cs]
        for k in range(1, len(nodes) + 1):
            check_query(ctx.b, nodes[:k], (name, k))
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
    check_query(ctx.b, nodes, case.name)


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
