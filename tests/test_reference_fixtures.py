"""The reference's own solver-layer outcome tests (tests/reference_cases.py) on the CPU.

* every case lowers (no LoweringUnsupported: the sieve sees every one of them);
* ground cases (calldata / storage values after simplification): the lowered term, evaluated by
  the oracle, has the truth value the reference asserts;
* the sieve's first round restated on the host — guide (candidates.py), the guided rows
  (oracle/guided_gen.py), each variable-disjoint group (Sieve.buckets) evaluated by the oracle —
  finds a row for every SAT case the sieve answers, and that row is a model of the ORIGINAL query
  (oracle/term_eval.py); no row satisfies an UNSAT case; a SAT case with a ``fallback_reason``
  finds none (the GPU test asserts the fallback is asked);
* the DependenceMap partition and the expression-variable sets of independece_solver_test.py.
The same cases run through ``frontend.get_model`` on the GPU in tests/test_gpu_reference_fixtures.py.
"""
import pytest

from mythril_amd.candidates import build_guide
from mythril_amd.lower import lower_query, node_columns
from mythril_amd.sieve import Sieve, eliminate_definitions, local_tape
from mythril_amd.smt import And
from oracle import smt_eval as E
from oracle.guided_gen import generate_row
from oracle.term_eval import evaluate_term
from tests.reference_cases import (BY_NAME, CASES, DIVERGENT, KECCAK_MODULE, case_ids,
                                   dependence_map_case, expr_variables_case,
                                   shared_keccak_cases)
from tests.test_lowering import model_of


def holds_original(ctx, cs, schema, values) -> bool:
    names = [n for n, _ in sorted(ctx.b.var_index.items(), key=lambda kv: kv[1])]
    vars_, arrays, funcs = model_of(schema, values, ctx.b)
    tape = ctx.b.finish(And(*cs).node)
    return bool(evaluate_term(tape.nodes, ctx.b.pool.values, names, ctx.b.symbols.array_names,
                              ctx.b.symbols.function_names, vars_, arrays, funcs))


def host_first_round(ctx, cs, rows=256, seed=0x5EED5EED):
    """Sieve.solve's first launch restated on the host: per group the first guided row whose
    group conjunction holds; the witness (column -> value) or None."""
    b = ctx.b
    root, schema = lower_query(b, [c.node for c in cs])
    cols = list(schema.columns)
    if not cols:
        cols = ["__ground__"]
        b.var("__ground__", 1)
        from mythril_amd.lower import Column

        schema.columns["__ground__"] = Column("__ground__", 1, "var", "__ground__")
    rest, defs = eliminate_definitions(b, Sieve.conjuncts(b, root), schema)
    if defs:
        root = rest[0] if rest else b.true()
        for x in rest[1:]:
            root = _and(b, root, x)
    guide = build_guide(b, root, schema, cols).arrays()
    names = {b.var_index[c]: c for c in cols}
    groups = []
    for conj, vs in Sieve.buckets(b, root):
        acc = conj[0]
        for x in conj[1:]:
            acc = _and(b, acc, x)
        groups.append((local_tape(b, acc, cols), [names[v] for v in vs]))
    values, solved = {}, [False] * len(groups)
    for r in range(rows):
        row = generate_row(seed, r, guide)
        for g, (nodes, gcols) in enumerate(groups):
            if not solved[g] and E.evaluate(nodes, b.pool.values, row):
                solved[g] = True
                for c in gcols:
                    values[c] = row[cols.index(c)]
        if all(solved):
            for c in cols:
                values.setdefault(c, 0)
            full = [values[c] for c in cols]
            for c, t in defs:
                values[c] = E.evaluate(local_tape(b, t, cols), b.pool.values, full)
            return schema, values
    return schema, None


def _and(b, x, y):
    from mythril_amd.tape import Op

    return b.op(Op.AND, x, y)


def _check_host_outcome(case, ctx, cs):
    name = case.name
    schema, w = host_first_round(ctx, cs)
    if name in DIVERGENT:  # satisfiable as restated: a witness must be a model, a miss is fine
        assert w is None or holds_original(ctx, cs, schema, w), name
    elif case.expected == "unsat":
        assert w is None, (name, w)
    elif case.fallback_reason:
        assert w is None, (name, "the sieve now answers it: drop the fallback_reason")
    else:
        assert w is not None, name
        assert holds_original(ctx, cs, schema, w), name


@pytest.mark.parametrize("name", case_ids())
def test_reference_case_on_host(name):
    case = BY_NAME[name]
    ctx, cs = case.build()
    _check_host_outcome(case, ctx, cs)


def test_shared_manager_cases_on_host():
    """keccak_tests.py's cases over one shared manager, in file order (the reference's
    module-level manager): the same outcomes as with a fresh manager per case."""
    out = shared_keccak_cases()
    assert [c.name for c, _, _ in out] == KECCAK_MODULE
    for case, ctx, cs in out:
        _check_host_outcome(case, ctx, cs)


def _holds_under(ctx, cs, vars_, funcs):
    names = [n for n, _ in sorted(ctx.b.var_index.items(), key=lambda kv: kv[1])]
    tape = ctx.b.finish(And(*cs).node)
    fs = {f: (lambda x, t=t: t.get(x, 0)) for f, t in funcs.items()}
    return bool(evaluate_term(tape.nodes, ctx.b.pool.values, names, ctx.b.symbols.array_names,
                              ctx.b.symbols.function_names, vars_, {}, fs))


def test_divergent_cases_are_satisfiable():
    """Each DIVERGENT case: its model satisfies the restated query (the reference's own
    construction), in both variants, while the reference test asserts unsat."""
    shared = {c.name: (ctx, cs) for c, ctx, cs in shared_keccak_cases()}
    assert DIVERGENT
    for name, (why, vars_, funcs) in DIVERGENT.items():
        assert BY_NAME[name].expected == "unsat", name
        ctx, cs = BY_NAME[name].build()
        assert _holds_under(ctx, cs, vars_, funcs), (name, "fresh manager")
        ctx, cs = shared[name]
        assert _holds_under(ctx, cs, vars_, funcs), (name, "shared manager")


def test_ground_cases_have_the_reference_value():
    """The ground (variable-free) cases: the lowered query is a constant the oracle decides."""
    n = 0
    for case in CASES:
        ctx, cs = case.build()
        root, schema = lower_query(ctx.b, [c.node for c in cs])
        if schema.columns:
            continue
        nodes = ctx.b.finish(root).nodes
        assert bool(E.evaluate(nodes, ctx.b.pool.values, [])) == (case.expected == "sat"), \
            case.name
        n += 1
    assert n >= 18


def test_dependence_map_partition():
    """independece_solver_test.py:54-85 through Sieve.buckets (over the lowered columns)."""
    ctx, cs, want_vars, want_conds = dependence_map_case()
    b = ctx.b
    root, schema = lower_query(b, [c.node for c in cs])
    groups = Sieve.buckets(b, root)
    inv = {i: n for n, i in b.var_index.items()}
    got = {(frozenset(inv[v] for v in vs), frozenset(conj)) for conj, vs in groups}
    cnodes = [c.node for c in cs]
    want = {(frozenset(v), frozenset(cnodes[i] for i in idx))
            for v, idx in zip(want_vars, want_conds)}
    assert got == want


def test_expression_variables():
    """independece_solver_test.py:12-39: the symbols a term reads (node_columns)."""
    ctx, items = expr_variables_case()
    b = ctx.b
    inv = {i: n for n, i in b.var_index.items()}
    for term, want in items:
        got = node_columns(b, [term.node])[term.node]
        assert {inv[v] for v in got} == want


def test_model_accessors_on_host():
    """model_test.py: decls / __getitem__ / eval read the symbol's name (``x.raw.decl()``)."""
    BY_NAME["model_x_eq_2"].build()
    from mythril_amd.smt import symbol_factory
    from mythril_amd.tape import TapeError

    xs = symbol_factory.BitVecSym("x", 256)
    assert xs.raw is xs and xs.raw.decl() == "x"
    with pytest.raises(TapeError):
        (xs + 1).decl()
