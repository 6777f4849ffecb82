"""The C++ SMT-LIB reader (mh_smtlib_read, smtlib.NativeReader) against the Python reader
(smtlib.Reader), on the CPU (the reader needs no device).

* every LASER-shaped query (tests/laser_like.py, SAT and UNSAT shapes) as z3 prints it
  (tests/z3_style.py: declarations + one assert per constraint, shared terms as lets), read
  constraint by constraint in LASER order into ONE session, gives the same terms as the Python
  reader (a canonical structural form: ops, widths, indices, symbol names, constant values);
* the --solver-log texts (to_smtlib: define-funs, objectives) and test_smtlib's hand-written
  z3-style text (keccak UF and its inverse, distinct, =>, bvcomp, rotate, repeat, objectives);
* a constraint already read hands the host no new node; a malformed text raises SmtlibError and
  leaves the session usable; the import is timed per new constraint (DESIGN §6's import column).
"""
import time

import pytest

from mythril_amd import native, smt, smtlib
from mythril_amd.tape import ARITY, Op
from tests.laser_like import hard_queries, queries
from tests.z3_style import z3_sexpr


def canon(b, root, memo=None):
    """A structural key of `root`: (op, width, symbol / value, imm, children)."""
    memo = {} if memo is None else memo
    var_names = {v: k for k, v in b.var_index.items()}
    stack = [root]
    while stack:
        n = stack[-1]
        if n in memo:
            stack.pop()
            continue
        op, w, a, bb, c, i0, i1 = b.nodes[n]
        kids = (a, bb, c)[:ARITY[Op(op)]]
        todo = [x for x in kids if x not in memo]
        if todo:
            stack += todo
            continue
        stack.pop()
        if op == Op.VAR:
            lab = ("var", var_names[i0])
        elif op == Op.CONST:
            lab = ("const", b.pool.values[i0])
        elif op == Op.ARRAY:
            lab = ("array", b.symbols.array_names[i0], i1)
        elif op == Op.UF:
            lab = ("uf", b.symbols.function_names[i0])
        else:
            lab = (i0, i1)
        memo[n] = hash((op, w, lab, tuple(memo[x] for x in kids)))
    return memo[root]


def _both(text, py_ctx=None, nat=None):
    q1 = smtlib.parse(text, py_ctx)
    if nat is None:
        nat = smtlib.NativeReader()
    q2 = smtlib.Query(nat.ctx)
    nat.read(text, q2)
    return q1, q2


def _same(q1, q2):
    assert len(q1.constraints) == len(q2.constraints)
    assert len(q1.minimize) == len(q2.minimize) and len(q1.maximize) == len(q2.maximize)
    for xs, ys in ((q1.constraints, q2.constraints), (q1.minimize, q2.minimize),
                   (q1.maximize, q2.maximize)):
        for x, y in zip(xs, ys):
            assert canon(x.ctx.b, x.node) == canon(y.ctx.b, y.node)


def _all_queries():
    out = []
    for make in (queries, hard_queries):
        _, qs = make()
        out += qs
    return out


@pytest.mark.parametrize("idx", range(len(_all_queries())))
def test_laser_order_matches_python_reader(idx):
    name, cs = _all_queries()[idx]
    texts = [z3_sexpr(c) for c in cs]
    py = smtlib.Reader()
    nat = smtlib.NativeReader()
    for t in texts:  # LASER order: one session, one new constraint at a time
        q1, q2 = smtlib.Query(py.ctx), smtlib.Query(nat.ctx)
        for cmd in smtlib.read_sexps(t):
            py.command(cmd, q1)
        nat.read(t, q2)
        _same(q1, q2)
    size = nat.session.size()
    q = smtlib.Query(nat.ctx)
    n_nodes = len(nat.b.nodes)
    nat.read(texts[-1], q)  # read again: nothing new reaches the host
    assert nat.session.size() == size and len(nat.b.nodes) == n_nodes, name


@pytest.mark.parametrize("idx", range(len(_all_queries())))
def test_solver_log_text_matches(idx):
    name, cs = _all_queries()[idx]
    try:
        text = smtlib.to_smtlib(cs, minimize=[], maximize=[])
    except smtlib.SmtlibError:
        pytest.skip("query holds a device-only op")
    _same(*_both(text))


def test_z3_style_text_matches():
    from tests.test_smtlib import Z3_STYLE

    _same(*_both(Z3_STYLE))


def test_literals_and_wide_constants():
    text = """(declare-fun x () (_ BitVec 256))
(declare-fun p () Bool)
(assert (= (concat x x) #x%s))
(assert (= ((_ extract 7 0) x) (_ bv200 8)))
(assert (=> p (bvult ((_ extract 15 0) x) #b0000000000000011)))
(assert (distinct ((_ extract 3 0) x) #x1 #x2 ((_ rotate_left 1) ((_ extract 3 0) x))))
(minimize ((_ extract 255 0) x))
""" % ("ab" * 64)
    _same(*_both(text))


def test_malformed_text_leaves_the_session_usable():
    nat = smtlib.NativeReader()
    size = nat.session.size()
    for bad in ("(assert (bvadd #x01 #x0001))", "(assert (= y #x01))", "(assert (and true",
                "(declare-fun f ((_ BitVec 8) (_ BitVec 8)) (_ BitVec 8))",
                "(assert #x01)"):
        with pytest.raises(smtlib.SmtlibError):
            nat.read(bad, smtlib.Query(nat.ctx))
        assert nat.session.size() == size
    q = smtlib.Query(nat.ctx)
    nat.read("(declare-fun y () (_ BitVec 8))\n(assert (= y #x01))", q)
    assert len(q.constraints) == 1


def test_import_cost_per_new_constraint():
    """DESIGN §6 import column: the C++ reader per new constraint in LASER order (the Python
    reader beside it).  The C++ parse is ~10 ns per character; what is left is the host builder's
    ~1.5 us per node the constraint adds (a fresh calldata word: 165-330 nodes)."""
    worst_nat, worst_py, sum_nat, sum_py = 0.0, 0.0, 0.0, 0.0
    for name, cs in _all_queries():
        texts = [z3_sexpr(c) for c in cs]
        py, nat = smtlib.Reader(), smtlib.NativeReader()
        for t in texts:
            t0 = time.perf_counter()
            q = smtlib.Query(py.ctx)
            for cmd in smtlib.read_sexps(t):
                py.command(cmd, q)
            t1 = time.perf_counter()
            nat.read(t, smtlib.Query(nat.ctx))
            t2 = time.perf_counter()
            worst_py = max(worst_py, t1 - t0)
            worst_nat = max(worst_nat, t2 - t1)
            sum_py += t1 - t0
            sum_nat += t2 - t1
    print("import per new constraint, worst: native %.3f ms, python %.3f ms"
          % (worst_nat * 1e3, worst_py * 1e3))
    # totals, not the worst single constraint: one scheduler hiccup on a loaded CI host must
    # not decide it
    assert sum_nat < sum_py / 2


def test_z3_importer_uses_the_native_reader():
    class Raw:
        def __init__(self, i, text):
            self.i, self.text = i, text

        def get_id(self):
            return self.i

    smt.set_context(smt.Context())
    _, qs = queries()
    cs = dict(qs)["killbilly"]
    raws = [Raw(i, z3_sexpr(c)) for i, c in enumerate(cs)]
    imp = smtlib.Z3Importer(sexpr_of=lambda r: r.text)
    assert isinstance(imp.reader, smtlib.NativeReader)
    ctx, terms = imp(raws)
    py = smtlib.Reader()
    for r, t in zip(raws, terms):
        q = smtlib.Query(py.ctx)
        for cmd in smtlib.read_sexps(r.text):
            py.command(cmd, q)
        assert canon(py.b, q.constraints[0].node) == canon(ctx.b, t.node)
    native.load()
