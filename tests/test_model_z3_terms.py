"""``Model`` read with reference (z3) terms, as the reference's callers read it.

Under the plugin a feasibility query arrives as z3 terms and the model that comes back is read
with z3 terms too:

* ``model.eval(self.size.raw, model_completion=True).as_long()`` then one
  ``model.eval(byte.raw, model_completion=True).as_long()`` per calldata byte
  (mythril/laser/ethereum/state/calldata.py:240-244);
* ``model.eval(tx.call_value.raw, model_completion=True)`` and
  ``model.eval(tx.caller.raw, model_completion=True)`` (mythril/analysis/solver.py:174-176);
* ``model.eval(val.raw)`` of a keccak application, ``.as_long()`` guarded by ``except
  AttributeError`` (keccak_function_manager.py:113) and of an inverse (analysis/solver.py:141);
* ``model[x.raw.decl()]`` and ``x.raw.decl() in model.decls()`` (tests/laser/smt/model_test.py).

z3 is absent, so a printing stand-in plays it: its terms are this package's terms of a separate
"reference-side" context, printed as z3 prints them (tests/z3_style.py: declarations, then an
``assert`` for a Bool or Optimize's ``minimize`` for a bit-vector).  Values are checked against
the ORACLE (oracle/term_eval.py) evaluating the reference-side term under the model the witness
denotes.  CPU: tests/fake_device.py stands in for the device; the GPU variant runs the same
through the real device (``-m gpu``).
"""
import itertools
import sys
import types

import pytest

from mythril_amd import frontend, smt
from mythril_amd.model import Model
from mythril_amd.smt import Concat, Not, ULT, symbol_factory
from mythril_amd.smtlib import Z3Importer
from oracle.term_eval import evaluate_term
from tests import fake_device
from tests.laser_like import ATTACKER, Calldata, KeccakManager, mapping_slot, selector_is, \
    sender_is_actor
from tests.test_lowering import model_of
from tests.z3_style import z3_sexpr

_ids = itertools.count(1)


class Z3Decl:
    def __init__(self, name):
        self._name = name

    def name(self):
        return self._name

    def __eq__(self, other):  # z3: structural equality of declarations
        return isinstance(other, Z3Decl) and other._name == self._name

    __hash__ = object.__hash__


class Z3Term:
    """A z3 ExprRef stand-in over a reference-side term."""

    def __init__(self, expr):
        self.expr = expr
        self._id = next(_ids)

    def get_id(self):
        return self._id

    def decl(self):
        return Z3Decl(self.expr.decl())


class RefExpr:
    """A reference laser/smt term: the z3 term is ``.raw``."""

    def __init__(self, expr):
        self.raw = Z3Term(expr)


def printing_z3():
    z3 = types.ModuleType("z3")
    z3.sat, z3.unsat, z3.unknown = "sat", "unsat", "unknown"
    z3.is_bool = lambda t: isinstance(t.expr, smt.Bool)

    class Solver:
        def __init__(self):
            self.assertions = []

        def add(self, *cs):
            self.assertions.extend(cs)

        def sexpr(self):
            assert len(self.assertions) == 1
            return z3_sexpr(self.assertions[0].expr)

    class Optimize(Solver):
        def __init__(self):
            super().__init__()
            self.objectives = []

        def minimize(self, t):
            self.objectives.append(t)

        def sexpr(self):
            assert not self.assertions and len(self.objectives) == 1
            return z3_sexpr(self.objectives[0].expr, head="minimize")

    z3.Solver, z3.Optimize = Solver, Optimize
    return z3


@pytest.fixture
def z3_world(monkeypatch):
    """The printing z3 stand-in installed, the front end importing through a Z3Importer."""
    monkeypatch.setitem(sys.modules, "z3", printing_z3())
    frontend.reset()
    imp = Z3Importer()
    frontend.configure(to_terms=imp, fallback=lambda *a: "fallback")
    yield imp
    frontend.reset()


def laser_query():
    """A transaction's query in the reference-side context: dispatcher, calldata size bounds,
    sender in ACTORS, a non-payable call, a mapping read (keccak of caller . slot 1)."""
    ref = smt.set_context(smt.Context())
    cd = Calldata("1")
    caller = symbol_factory.BitVecSym("sender_1", 256)
    value = symbol_factory.BitVecSym("call_value1", 256)
    km = KeccakManager()
    slot, cond = mapping_slot(km, caller, 1)
    storage = smt.Array("Storage", 256, 256)
    cs = [selector_is(cd, 0x9FA299CC), Not(ULT(cd.size, symbol_factory.BitVecVal(36, 256))),
          ULT(cd.size, symbol_factory.BitVecVal(40, 256)), sender_is_actor(caller),
          value == symbol_factory.BitVecVal(0, 256), cond,
          storage[slot] == symbol_factory.BitVecVal(1, 256)]
    return ref, cd, caller, value, km, slot, cs


def oracle_value(ref, expr, m):
    b = ref.b
    names = [n for n, _ in sorted(b.var_index.items(), key=lambda kv: kv[1])]
    vars_, arrays, funcs = model_of(m.schema, m.values, m.ctx.b)
    tape = b.finish(expr.node)
    return evaluate_term(tape.nodes, b.pool.values, names, b.symbols.array_names,
                         b.symbols.function_names, vars_, arrays, funcs)


def check_reference_reads(ref, cd, caller, value, km, slot, cs):
    m = frontend.get_model(tuple(RefExpr(c) for c in cs))
    assert isinstance(m, Model), m
    # calldata.py:240-244: the size, then every byte below it
    size = m.eval(RefExpr(cd.size).raw, model_completion=True).as_long()
    assert size == oracle_value(ref, cd.size, m) and 36 <= size < 40
    got = [m.eval(RefExpr(cd.load(i)).raw, model_completion=True).as_long()
           for i in range(size)]
    assert got == [oracle_value(ref, cd.load(i), m) for i in range(size)]
    assert got[:4] == [0x9F, 0xA2, 0x99, 0xCC]
    # analysis/solver.py:174-176
    assert m.eval(RefExpr(value).raw, model_completion=True).as_long() == 0
    c = m.eval(RefExpr(caller).raw, model_completion=True).as_long()
    assert c == oracle_value(ref, caller, m) and c in (0xAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFE,
                                                       ATTACKER,
                                                       0xAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAA)
    # model_test.py: the declaration of a reference symbol
    d = RefExpr(caller).raw.decl()
    assert d in m.decls() and m[d] == c and m[d].as_long() == c
    # keccak_function_manager.py:113: the keccak application, without completion
    h = m.eval(RefExpr(slot).raw)
    assert h.as_long() == oracle_value(ref, slot, m)
    # analysis/solver.py:141: the inverse of the hash -- the 512-bit input, two device slices
    f, inv = km.functions(512)
    x = m.eval(RefExpr(inv(slot)).raw)
    assert x.size() == 512 and x.as_long() == oracle_value(ref, inv(slot), m)
    assert x.as_long() == (c << 256) | 1
    # a 512-bit term built directly, and a 257-bit one
    wide = Concat(caller, cd.word(4))
    assert m.eval(RefExpr(wide).raw, model_completion=True).as_long() == \
        oracle_value(ref, wide, m)
    w257 = smt.ZeroExt(1, caller) + smt.ZeroExt(1, cd.word(4))
    assert m.eval(RefExpr(w257).raw, model_completion=True).as_long() == \
        oracle_value(ref, w257, m)
    # a symbol the query never mentions: unevaluated without completion, 0 with it
    y = symbol_factory.BitVecSym("retval_9", 256)
    t = RefExpr(y + symbol_factory.BitVecVal(1, 256)).raw
    assert m.eval(t) is t
    assert m.eval(t, model_completion=True) == 1
    assert m[Z3Decl("retval_9")] is None
    # a Bool term
    assert m.eval(RefExpr(cs[0]).raw) is True
    return m


def test_reference_reads_on_fake_device(monkeypatch, z3_world):
    fake_device.install(monkeypatch)
    frontend.configure(rows=256)
    check_reference_reads(*laser_query())


def test_model_survives_an_importer_reset(monkeypatch, z3_world):
    """The importer may start a new term context between queries (Z3Importer.reset): a model
    of an earlier query still reads reference terms, into its own context."""
    fake_device.install(monkeypatch)
    frontend.configure(rows=256)
    ref, cd, caller, value, km, slot, cs = laser_query()
    m = frontend.get_model(tuple(RefExpr(c) for c in cs))
    assert isinstance(m, Model)
    z3_world.reset()
    assert z3_world.ctx is not m.ctx
    c = m.eval(RefExpr(caller).raw, model_completion=True).as_long()
    assert c == oracle_value(ref, caller, m)


def test_model_interps_of_arrays_and_functions(monkeypatch, z3_world):
    fake_device.install(monkeypatch)
    frontend.configure(rows=256)
    ref, cd, caller, value, km, slot, cs = laser_query()
    m = frontend.get_model(tuple(RefExpr(c) for c in cs))
    names = {d.name() for d in m.decls()}
    assert {"sender_1", "call_value1", "1_calldatasize", "Storage", "keccak256_512"} <= names
    st = m[Z3Decl("Storage")].as_list()
    assert st[-1] == m.values.get("Storage[*]", 0)  # else value last, as z3's FuncInterp
    h = m.eval(RefExpr(slot).raw).as_long()
    assert dict((k, v) for k, v in st[:-1]).get(h, st[-1]) == 1  # Storage[slot] == 1 holds
    assert m[0] == m.decls()[0]


@pytest.mark.gpu
def test_reference_reads_on_gpu(gpu_ctx, z3_world):
    frontend.configure(rows=256)
    check_reference_reads(*laser_query())


def test_wide_terms_are_sliced_for_the_device():
    """Model.eval of a term wider than 256 bits: Slicer rewrites it as terms of its 256-bit slices
    (no device operation wider than 256 bits); their values, joined, equal the ORACLE's value of
    the wide term -- carries across slices, unaligned concatenation and extraction, extensions."""
    import random

    from mythril_amd.model import Slicer
    from mythril_amd.smt import Extract, SignExt, ZeroExt
    from oracle import smt_eval as E

    ctx = smt.set_context(smt.Context())
    b = ctx.b
    x, y = symbol_factory.BitVecSym("x", 256), symbol_factory.BitVecSym("y", 256)
    z = symbol_factory.BitVecSym("z", 40)
    terms = [ZeroExt(1, x) + ZeroExt(1, y), Concat(x, y), Concat(z, x, y),
             ZeroExt(256, x) - ZeroExt(256, y), Extract(300, 20, Concat(z, x, y)),
             SignExt(100, x) + Concat(Extract(59, 0, y), z, x), -(ZeroExt(8, x)),
             Concat(x, y) ^ Concat(y, x), smt.If(x == y, Concat(x, y), Concat(y, x)),
             SignExt(280, z) + ZeroExt(280, z)]
    names = [n for n, _ in sorted(b.var_index.items(), key=lambda kv: kv[1])]
    rng = random.Random(1)
    for t in terms:
        sl = Slicer(b).slices(t.node)
        assert all(b.width(s) <= 256 for s in sl)
        assert sum(b.width(s) for s in sl) == b.width(t.node)
        for _ in range(16):
            vals = {"x": rng.getrandbits(256), "y": rng.getrandbits(256), "z": rng.getrandbits(40)}
            if rng.random() < 0.25:
                vals["y"] = vals["x"]
            row = [vals[n] for n in names]
            want = E.evaluate(b.finish(t.node).nodes, b.pool.values, row)
            got = sum(E.evaluate(b.finish(s).nodes, b.pool.values, row) << (256 * i)
                      for i, s in enumerate(sl))
            assert got == want, t.node
    with pytest.raises(smt.TapeError if hasattr(smt, "TapeError") else Exception):
        Slicer(b).slices((ZeroExt(256, x) * ZeroExt(256, y)).node)


def calldata_query(size=100):
    """A transaction whose calldata size is pinned (0x64 bytes), its dispatcher and argument
    checks: the reference then reads the model byte by byte (calldata.py:234-245)."""
    ref = smt.set_context(smt.Context())
    cd = Calldata("1")
    caller = symbol_factory.BitVecSym("sender_1", 256)
    cs = [selector_is(cd, 0x9FA299CC), cd.size == symbol_factory.BitVecVal(size, 256),
          sender_is_actor(caller), ULT(cd.word(4), symbol_factory.BitVecVal(1 << 160, 256))]
    return ref, cd, cs


def concrete_calldata(m, cd):
    """SymbolicCalldata.concrete (calldata.py:234-245), term for term: the size, then one
    ``eval(_load(i).raw, model_completion=True).as_long()`` per byte."""
    n = m.eval(RefExpr(cd.size).raw, model_completion=True).as_long()
    return [m.eval(RefExpr(cd.load(i)).raw, model_completion=True).as_long() for i in range(n)]


def check_batched_calldata_reads(launches, size=100):
    """The reference's byte loop over a sieve model reads `size` bytes in at most two device
    launches (the size; then byte 0 with its speculated siblings), with the oracle's values."""
    import time

    from mythril_amd import native

    ref, cd, cs = calldata_query(size)
    m = frontend.get_model(tuple(RefExpr(c) for c in cs))
    assert isinstance(m, Model), m
    before = launches()
    t0 = time.perf_counter()
    got = concrete_calldata(m, cd)
    dt = time.perf_counter() - t0
    n_launch = launches() - before
    assert len(got) == size
    assert got == [oracle_value(ref, cd.load(i), m) for i in range(size)]
    assert got[:4] == [0x9F, 0xA2, 0x99, 0xCC]
    assert n_launch <= 2, n_launch
    # a second read of the same model is all memo hits
    before = launches()
    assert concrete_calldata(m, cd) == got and launches() == before
    return n_launch, dt


def test_calldata_loop_is_batched_on_fake_device(monkeypatch, z3_world):
    fake_device.install(monkeypatch)
    frontend.configure(rows=256)
    check_batched_calldata_reads(lambda: fake_device.LAUNCHES[0])


@pytest.mark.gpu
def test_calldata_loop_is_batched_on_gpu(gpu_ctx, z3_world):
    from mythril_amd import native

    frontend.configure(rows=256)
    n, dt = check_batched_calldata_reads(lambda: native.eval_launches(frontend.sieve().ctx))
    print("calldata.concrete: 100 bytes in %d launches, %.2f ms" % (n, 1e3 * dt))
