"""The sieve front end on an MI355X: guided generator parity, witnesses of LASER-shaped queries,
Model.eval on the device.  Every witness is checked by the ORACLE: the original query (arrays,
keccak UFs, inverses) evaluated by oracle/term_eval.py under the model the witness row denotes.

Run on the GPU box:  python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
"""
import numpy as np
import pytest

from mythril_amd import frontend, native
from mythril_amd.candidates import build_guide
from mythril_amd.lower import lower_query
from mythril_amd.smt import And
from mythril_amd.support import SolverStatistics, UnsatError
from oracle.guided_gen import generate_row
from oracle.term_eval import evaluate_term
from tests.laser_like import queries
from tests.test_lowering import model_of

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _reset():
    frontend.reset()
    yield
    frontend.reset()


def _oracle_holds(ctx, cs, schema, values):
    names = [n for n, _ in sorted(ctx.b.var_index.items(), key=lambda kv: kv[1])]
    vars_, arrays, funcs = model_of(schema, values, ctx.b)
    tape = ctx.b.finish(And(*cs).node)
    return bool(evaluate_term(tape.nodes, ctx.b.pool.values, names, ctx.b.symbols.array_names,
                              ctx.b.symbols.function_names, vars_, arrays, funcs))


@pytest.mark.parametrize("qi", [0, 4, 5, 7, 9])
def test_guided_generator_matches_oracle(gpu_ctx, qi):
    ctx, qs = queries()
    _, cs = qs[qi]
    root, schema = lower_query(ctx.b, [c.node for c in cs])
    cols = list(schema.columns)
    arrays = build_guide(ctx.b, root, schema, cols).arrays()
    rows, seed, base = 512, 0xC0FFEE + qi, 1 << 20
    a = gpu_ctx.assignments(len(cols) + 3, rows)  # wider buffer: extra columns untouched
    a.generate(1, 0)
    before = a.download(0, rows)
    a.generate_guided(seed, arrays, global_base=base, first=0, count=rows)
    got = a.download(0, rows)
    assert np.array_equal(got[len(cols):], before[len(cols):])
    for r in list(range(0, rows, 37)) + [rows - 1]:
        want = generate_row(seed, base + r, arrays)
        for v, wv in enumerate(want):
            gv = sum(int(got[v, k, r]) << (32 * k) for k in range(8))
            assert gv == wv, (qi, r, cols[v])


def _random_guide(rng, n_cols, n_sets):
    """Guide arrays in mh_guide order with value and copy sets in random order (the generator's
    LDS form resolves the leading value-only sets, the rest run in memory)."""
    width = rng.choice([1, 8, 32, 160, 256], size=n_cols).astype(np.uint16)
    pool_n = rng.integers(0, 4, size=n_cols)
    pool_off = np.concatenate([[0], np.cumsum(pool_n)]).astype(np.uint32)
    pool = rng.integers(0, 1 << 32, size=(max(int(pool_off[-1]), 1), 8), dtype=np.uint64)
    set_off, alt_off, e_col, e_val, prob = [0], [0], [], [], []
    for j in range(n_sets):
        copy = rng.random() < 0.2
        for _ in range(int(rng.integers(1, 4))):
            for _ in range(int(rng.integers(1, 6))):
                c = int(rng.integers(0, n_cols))
                if copy:
                    src = int(rng.integers(0, n_cols))
                    nb = int(rng.integers(1, 65))
                    e_col.append(c | 0x80000000)
                    e_val.append([src, int(rng.integers(0, 192)), int(rng.integers(0, 192)), nb,
                                  0, 0, 0, 0])
                else:
                    e_col.append(c)
                    e_val.append(list(rng.integers(0, 1 << 32, size=8)))
            alt_off.append(len(e_col))
        set_off.append(len(alt_off) - 1)
        prob.append(int(rng.integers(0, 256)))
    return dict(width=width, pool_off=pool_off, pool=pool.astype(np.uint32),
                set_off=np.array(set_off, dtype=np.uint32),
                set_prob=np.array(prob or [0], dtype=np.uint8),
                alt_off=np.array(alt_off, dtype=np.uint32),
                entry_col=np.array(e_col or [0], dtype=np.uint32),
                entry_val=np.array(e_val or [[0] * 8], dtype=np.uint64).astype(np.uint32))


@pytest.mark.parametrize("n_cols,n_sets", [(7, 60), (150, 300), (200, 100)])
def test_guided_generator_random_guides(gpu_ctx, n_cols, n_sets):
    """Random guides (value and copy sets interleaved, up to 200 columns: past the LDS form's
    192) against oracle/guided_gen.py, bit for bit on sampled rows."""
    rng = np.random.default_rng(n_cols * 1000 + n_sets)
    arrays = _random_guide(rng, n_cols, n_sets)
    rows, seed, base = 200, 0xABCD + n_cols, 1 << 30
    a = gpu_ctx.assignments(n_cols, rows)
    a.generate_guided(seed, arrays, global_base=base, first=0, count=rows)
    got = a.download(0, rows)
    for r in list(range(0, rows, 23)) + [rows - 1]:
        want = generate_row(seed, base + r, arrays)
        for v, wv in enumerate(want):
            gv = sum(int(got[v, k, r]) << (32 * k) for k in range(8))
            assert gv == wv, (n_cols, r, v)


def test_guided_generator_rejects_malformed_guides(gpu_ctx):
    ctx, qs = queries()
    _, cs = qs[0]
    root, schema = lower_query(ctx.b, [c.node for c in cs])
    cols = list(schema.columns)
    arrays = build_guide(ctx.b, root, schema, cols).arrays()
    a = gpu_ctx.assignments(len(cols), 64)
    bad = dict(arrays, entry_col=arrays["entry_col"].copy())
    bad["entry_col"][0] = len(cols) + 5
    with pytest.raises(native.SieveError):
        a.generate_guided(1, bad)
    narrow = gpu_ctx.assignments(1, 64)
    with pytest.raises(native.SieveError):
        narrow.generate_guided(1, arrays)
    with pytest.raises(native.SieveError):
        a.generate_guided(1, arrays, first=60, count=10)


SAT_SHAPES = [n for n, _ in queries()[1] if not n.startswith("unsat")]


@pytest.mark.parametrize("name", SAT_SHAPES)
def test_sieve_witnesses_are_models(gpu_ctx, name):
    ctx, qs = queries()
    cs = dict(qs)[name]
    m = frontend.get_model(tuple(cs))  # no fallback: a miss would raise UnsatError
    assert _oracle_holds(ctx, cs, m.schema, m.values), name
    for c in cs:  # Model.eval on the device agrees
        assert m.eval(c, model_completion=True) is True, name


def test_unsat_query_goes_to_the_fallback(gpu_ctx):
    ctx, qs = queries()
    cs = dict(qs)["unsat_actor"]
    with pytest.raises(UnsatError):
        frontend.get_model(tuple(cs))
    frontend.configure(fallback=lambda *a: "z3 says")
    assert frontend.get_model(tuple(cs)) == "z3 says"
    assert SolverStatistics().sieve_misses >= 2


def test_model_eval_values(gpu_ctx):
    from tests.laser_like import Calldata

    ctx, qs = queries()
    cs = dict(qs)["selector_size"]
    m = frontend.get_model(tuple(cs))
    cd = Calldata("1")
    word = m.eval(cd.word(0), model_completion=True)
    assert word.as_long() >> 224 == 0x13AF4035
    size = m.eval(cd.size, model_completion=True)
    assert 36 <= size < 5000
    # a symbol outside the model: unevaluated without completion, 0 with it
    from mythril_amd.smt import symbol_factory

    y = symbol_factory.BitVecSym("not_in_query", 256)
    assert m.eval(y + 1) is not None and not isinstance(m.eval(y + 1), int)
    assert m.eval(y + 1, model_completion=True) == 1


def test_parent_witness_is_reused(gpu_ctx):
    ctx, qs = queries()
    cs = dict(qs)["selector_size"]
    s = frontend.sieve()
    frontend.get_model(tuple(cs[:2]))
    rounds_before = s.stats.rounds
    m = frontend.get_model(tuple(cs))
    assert s.stats.rounds - rounds_before == 1  # found in the first round
    assert _oracle_holds(ctx, cs, m.schema, m.values)


@pytest.mark.parametrize("name", SAT_SHAPES)
def test_solver_log_queries_on_gpu(gpu_ctx, name):
    """--solver-log ingestion: every LASER-shaped SAT query in the SMT-LIB2 form the reference's
    get_model writes (support/model.py:44-55, z3's sexpr()), read back by smtlib.parse and
    answered by the sieve on the GPU; each witness is a model of the PARSED query (oracle)."""
    from mythril_amd import smtlib

    ctx, qs = queries()
    cs = dict(qs)[name]
    try:
        text = smtlib.to_smtlib(cs)
    except smtlib.SmtlibError:
        pytest.skip("query holds a device-only op")
    q = smtlib.parse(text)
    m = frontend.get_model(tuple(q.constraints))
    assert _oracle_holds(q.ctx, q.constraints, m.schema, m.values), name


def test_z3_style_solver_log_on_gpu(gpu_ctx):
    """z3-printed text (let bindings, keccak UF and its inverse, distinct, =>, bvcomp,
    rotate_left, an objective) parsed and solved on the GPU; the witness checked by the oracle
    with the lowering's keccak interpretation."""
    from mythril_amd import smtlib
    from tests.test_smtlib import Z3_STYLE

    q = smtlib.parse(Z3_STYLE)
    m = frontend.get_model(tuple(q.constraints))
    assert _oracle_holds(q.ctx, q.constraints, m.schema, m.values)


@pytest.mark.parametrize("name", ["killbilly", "ether_thief", "overflow"])
def test_long_path_on_gpu(gpu_ctx, name):
    """A 200-constraint path (tests/laser_paths.py) through get_model in LASER order (every
    prefix first, keyed as the plugin keys it): the final witness is a model of the whole
    ORIGINAL path (oracle/term_eval.py), and the UNSAT variant goes to the fallback."""
    from tests.laser_paths import grow

    ctx, cs = grow(name, 200)
    s = frontend.sieve()
    for k in range(1, len(cs)):
        s.solve(ctx.b, [c.node for c in cs[:k]], key=tuple(c.node for c in cs[:k]))
    m = frontend.get_model(tuple(cs))
    assert _oracle_holds(ctx, cs, m.schema, m.values), name
    ctx, cs = grow(name, 200, unsat=True)
    frontend.configure(fallback=lambda *a: "z3")
    assert frontend.get_model(tuple(cs)) == "z3"


def test_native_and_python_host_stages_agree(gpu_ctx):
    """Sieve.solve with the native query compiler (csrc/query.cpp) and with the Python stages it
    replaced: the same hit or miss on every LASER-shaped query in LASER order, and every native
    witness is a model of the ORIGINAL query (oracle)."""
    from mythril_amd.sieve import Sieve
    from tests.laser_like import hard_queries

    for make in (queries, hard_queries):
        ctx, qs = make()
        ctx_py, qs_py = make()
        s_nat, s_py = Sieve(), Sieve(native_query=False)
        try:
            for (name, cs), (_, cs_py) in zip(qs, qs_py):
                for k in range(1, len(cs) + 1):
                    nodes = [c.node for c in cs[:k]]
                    w = s_nat.solve(ctx.b, nodes, key=tuple(nodes))
                    nodes_py = [c.node for c in cs_py[:k]]
                    w_py = s_py.solve(ctx_py.b, nodes_py, key=tuple(nodes_py))
                    assert (w is None) == (w_py is None), (name, k)
                    if w is not None:
                        assert _oracle_holds(ctx, cs[:k], w.schema, w.values), (name, k)
            assert s_nat.stats.hits > 10
        finally:
            s_nat.close()
            s_py.close()


def test_random_queries_native_witnesses_are_models(gpu_ctx):
    """Random queries over arrays, stores, K, a tabled function, keccak with pairs / bounds /
    inverse and wide equalities (tests/test_query_native.py _random_query), every prefix in
    LASER order through Sieve.solve with the native query compiler: every witness is a model of
    the ORIGINAL prefix (oracle/term_eval.py), and some prefixes are answered."""
    import random

    from mythril_amd.sieve import Sieve
    from tests.test_query_native import _random_query

    s = Sieve()
    hits = 0
    try:
        for seed in range(16):
            ctx, cs = _random_query(random.Random(seed), 8)
            cs = [c for c in cs if hasattr(c, "node")]
            for k in range(1, len(cs) + 1):
                nodes = [c.node for c in cs[:k]]
                try:
                    w = s.solve(ctx.b, nodes, key=tuple(nodes))
                except native.Unsupported:
                    continue
                if w is not None:
                    hits += 1
                    assert _oracle_holds(ctx, cs[:k], w.schema, w.values), (seed, k)
    finally:
        s.close()
    assert hits >= 16
