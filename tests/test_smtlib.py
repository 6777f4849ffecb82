"""SMT-LIB2 reader / writer (mythril_amd/smtlib.py): the --solver-log format and z3 import path.

Checked against the oracle: terms read from text evaluate (oracle/term_eval.py) exactly like the
same terms built through the mythril_amd.smt API, and ``parse(to_smtlib(query))`` preserves
every LASER-shaped query of tests/laser_like.py under random models.
"""
import random

import pytest

from mythril_amd import smt, smtlib
from mythril_amd.smt import And
from oracle.term_eval import evaluate_term
from tests.laser_like import queries

Z3_STYLE = """; what z3's Optimize.sexpr() prints for a dispatcher + actor query
(declare-fun |1_calldatasize| () (_ BitVec 256))
(declare-fun |1_calldata| () (Array (_ BitVec 256) (_ BitVec 8)))
(declare-fun sender_1 () (_ BitVec 256))
(declare-fun call_value1 () (_ BitVec 256))
(declare-fun keccak256_512 ((_ BitVec 512)) (_ BitVec 256))
(declare-fun keccak256_512-1 ((_ BitVec 256)) (_ BitVec 512))
(assert (let ((a!1 (concat (ite (bvsle |1_calldatasize| (_ bv0 256)) #x00
                                 (select |1_calldata| (_ bv0 256)))
                            (ite (bvsle |1_calldatasize| (_ bv1 256)) #x00
                                 (select |1_calldata| (_ bv1 256)))
                            (ite (bvsle |1_calldatasize| (_ bv2 256)) #x00
                                 (select |1_calldata| (_ bv2 256)))
                            (ite (bvsle |1_calldatasize| (_ bv3 256)) #x00
                                 (select |1_calldata| (_ bv3 256))))))
  (= a!1 #x9fa299cc)))
(assert (or (= sender_1 #x000000000000000000000000affeaffeaffeaffeaffeaffeaffeaffeaffeaffe)
            (= sender_1 #x000000000000000000000000deadbeefdeadbeefdeadbeefdeadbeefdeadbeef)
            (= sender_1 #x000000000000000000000000aaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaa)))
(assert (not (bvule call_value1 #b0000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000000)))
(assert (= ((_ extract 7 0) ((_ zero_extend 8) ((_ sign_extend 0) ((_ rotate_left 4) #xab)))) #xba))
(assert (distinct sender_1 call_value1 (bvnot call_value1)))
(assert (=> (bvult (bvcomp sender_1 sender_1) #b1) false))
(assert (= (keccak256_512-1 (keccak256_512 (concat sender_1 (_ bv1 256)))) (concat sender_1 (_ bv1 256))))
(minimize |1_calldatasize|)
(check-sat)
"""


def _names(ctx):
    return [n for n, _ in sorted(ctx.b.var_index.items(), key=lambda kv: kv[1])]


def _eval(ctx, terms, vars_, arrays, funcs):
    tape = ctx.b.finish(And(*terms).node)
    return bool(evaluate_term(tape.nodes, ctx.b.pool.values, _names(ctx),
                              ctx.b.symbols.array_names, ctx.b.symbols.function_names,
                              vars_, arrays, funcs))


def test_reads_z3_style_text():
    q = smtlib.parse(Z3_STYLE)
    assert len(q.constraints) == 7 and len(q.minimize) == 1 and not q.maximize
    inv = {}

    def f(x):
        y = (x * 0x9E3779B97F4A7C15) % (1 << 256)
        inv[y] = x
        return y

    funcs = {"keccak256_512": f, "keccak256_512-1": lambda y: inv.get(y, 0)}
    good = {"1_calldatasize": 4, "sender_1": 0xDEADBEEFDEADBEEFDEADBEEFDEADBEEFDEADBEEF,
            "call_value1": 5}
    arrays = {"1_calldata": ({0: 0x9F, 1: 0xA2, 2: 0x99, 3: 0xCC}, 0)}
    assert _eval(q.ctx, q.constraints, good, arrays, funcs)
    # calldatasize 3: the fourth byte reads 0 (ite), the selector check fails
    assert not _eval(q.ctx, q.constraints, dict(good, **{"1_calldatasize": 3}), arrays, funcs)
    assert not _eval(q.ctx, q.constraints, dict(good, sender_1=7), arrays, funcs)
    assert not _eval(q.ctx, q.constraints, dict(good, call_value1=0), arrays, funcs)


@pytest.mark.parametrize("qi", range(12))
def test_roundtrip_preserves_laser_queries(qi):
    ctx, qs = queries()
    name, cs = qs[qi]
    try:
        text = smtlib.to_smtlib(cs)
    except smtlib.SmtlibError:
        pytest.skip("query holds a device-only op")
    q = smtlib.parse(text)
    assert len(q.constraints) == len(cs)
    rng = random.Random(qi)
    arr_names = ctx.b.symbols.array_names
    for _ in range(40):
        vars_ = {n: rng.choice([0, 1, 4, 36, rng.getrandbits(256), rng.getrandbits(160)])
                 for n in ctx.b.var_index}
        vars_.update({n: rng.getrandbits(8) for n in ctx.b.var_index if "calldata[" in n})
        arrays = {a: ({k: rng.getrandbits(8) for k in range(40)}, rng.getrandbits(8))
                  for a in arr_names}
        funcs = {f: (lambda x, s=rng.getrandbits(64): (x * s + 64) % (1 << 256))
                 for f in ctx.b.symbols.function_names}
        want = _eval(ctx, cs, vars_, arrays, funcs)
        # Bool declarations become 1-bit variables compared with #b1: same values
        got = _eval(q.ctx, q.constraints, vars_, arrays, funcs)
        assert want == got, name


def test_unsupported_constructs_raise():
    base = "(declare-fun a () (Array (_ BitVec 8) (_ BitVec 8)))\n" \
           "(declare-fun b () (Array (_ BitVec 8) (_ BitVec 8)))\n"
    with pytest.raises(smtlib.SmtlibError):
        smtlib.parse(base + "(assert (= a b))")
    with pytest.raises(smtlib.SmtlibError):
        smtlib.parse("(assert (forall ((x (_ BitVec 8))) true))")
    with pytest.raises(smtlib.SmtlibError):
        smtlib.parse("(assert (= x #x01))")  # undeclared


def test_solver_log_written_by_front_end(tmp_path):
    from mythril_amd import frontend
    from mythril_amd.support import UnsatError, args

    ctx = smt.set_context(smt.Context())
    x = smt.symbol_factory.BitVecSym("x", 256)
    old = args.solver_log
    args.solver_log = str(tmp_path)
    frontend.configure(enabled=False)
    try:
        with pytest.raises(UnsatError):  # no sieve, no fallback: "unknown"
            frontend.get_model((x == 5,))
    finally:
        args.solver_log = old
        frontend.reset()
    files = list(tmp_path.glob("*.smt2"))
    assert len(files) == 1
    q = smtlib.parse(files[0].read_text())
    assert len(q.constraints) == 1


def test_deep_store_and_ite_chains_parse():
    """LASER terms nest thousands deep (a store per SSTORE, an ite per symbolic-index read);
    the reader must not recurse (round 1 hit Python's recursion limit near depth 1000)."""
    depth = 5000
    arr = "s0"
    text = ["(declare-fun s0 () (Array (_ BitVec 256) (_ BitVec 256)))",
            "(declare-fun k () (_ BitVec 256))"]
    t = arr
    for i in range(depth):
        t = "(store %s (_ bv%d 256) (_ bv%d 256))" % (t, i, i + 1)
    e = "(select %s k)" % t
    for i in range(depth):
        e = "(ite (= k (_ bv%d 256)) (bvadd %s (_ bv1 256)) k)" % (i, e)
    text.append("(assert (= %s (_ bv7 256)))" % e)
    q = smtlib.parse("\n".join(text))
    assert len(q.constraints) == 1
    # a deep let chain (z3's a!N bindings)
    lets = "(declare-fun x () (_ BitVec 8))\n(assert " + "".join(
        "(let ((a!%d (bvadd %s #x01))) " % (i, "x" if i == 0 else "a!%d" % (i - 1))
        for i in range(3000)) + "(= a!2999 #x00)" + ")" * 3000 + ")"
    q2 = smtlib.parse(lets)
    # x + 3000 == 0 (mod 256)  <=>  x == 256 - 3000 % 256
    want = (256 - 3000 % 256) % 256
    assert _eval(q2.ctx, q2.constraints, {"x": want}, {}, {})
    assert not _eval(q2.ctx, q2.constraints, {"x": want + 1}, {}, {})


class _FakeZ3Term:
    """A z3 AST stand-in: an id and the text z3's Solver.sexpr() would print for it."""

    _next = 0

    def __init__(self, text):
        _FakeZ3Term._next += 1
        self.id = _FakeZ3Term._next
        self.text = text

    def get_id(self):
        return self.id


def test_importer_memory_is_bounded():
    """A long run replays millions of is_possible queries: the importer's memo and term store
    must stay bounded (ADVICE: Z3Importer.memo / reader.ctx grew without bound)."""
    resets = []
    imp = smtlib.Z3Importer(max_memo=64, max_nodes=5000, sexpr_of=lambda raw: raw.text,
                            on_reset=lambda: resets.append(1))
    decl = "(declare-fun x () (_ BitVec 256))\n"
    peak = 0
    for i in range(2000):
        raw = _FakeZ3Term(decl + "(assert (bvult (bvmul x (_ bv%d 256)) (_ bv%d 256)))" % (i, i))
        ctx, terms = imp([raw])
        assert len(terms) == 1 and terms[0].ctx is ctx
        peak = max(peak, imp.n_nodes())
        assert len(imp.memo) <= 64
    assert resets and imp.resets == len(resets)
    assert peak <= 5000 + 10  # one query past the threshold at most
    # memo hit: the same AST object is not re-read
    raw = _FakeZ3Term(decl + "(assert (= x (_ bv1 256)))")
    n0 = imp([raw])[1][0].node
    before = imp.n_nodes()
    assert imp([raw])[1][0].node == n0 and imp.n_nodes() == before


def test_add_no_overflow_form_reads_back_as_the_predicate():
    """z3's printed BVAddNoOverflow(x, y, False) -- (= ((_ extract w w) (bvadd ((_ zero_extend 1)
    x) ((_ zero_extend 1) y))) #b0), either side order -- reads back as the one predicate, so the
    parsed query stays within 256 bits and lowers for the device."""
    from mythril_amd.lower import lower_query
    from mythril_amd.tape import Op

    ctx, qs = queries()
    cs = dict(qs)["overflow"]
    q = smtlib.parse(smtlib.to_smtlib(cs))
    tape = q.ctx.b.finish(And(*q.constraints).node)
    ops = {Op(int(o)) for o in tape.nodes["op"]}
    assert Op.BVADD_NOOVFL_U in ops and max(int(w) for w in tape.nodes["width"]) <= 256
    lower_query(q.ctx.b, [c.node for c in q.constraints])
    text = ("(declare-fun x () (_ BitVec 8))\n(declare-fun y () (_ BitVec 8))\n"
            "(assert (= #b0 ((_ extract 8 8) (bvadd ((_ zero_extend 1) x) "
            "((_ zero_extend 1) y)))))\n")
    q2 = smtlib.parse(text)
    t2 = q2.ctx.b.finish(q2.constraints[0].node)
    assert Op(int(t2.nodes["op"][-1])) == Op.BVADD_NOOVFL_U
