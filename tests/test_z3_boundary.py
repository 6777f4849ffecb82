"""The z3 side of the drop-in boundary, without z3: a recording stand-in of the z3 module.

z3 is absent here and on the GPU box, so the code that talks to it --
``plugin.z3_verifier`` (the re-verification every sieve witness must pass, support/model.py's
contract of SURVEY §8b), ``plugin.z3_log_writer`` (``--solver-log``, support/model.py:44-55) and
``SievePlugin.start`` wiring them into the front end -- runs here against a stub ``z3`` that
records every call.  The tests pin what those functions hand to z3: the constraints, the
witness as equalities on every scalar column and array cell, the solver timeout
``min(args.solver_timeout, what is left of get_model's budget)`` (support/model.py:26-31 and
laser/smt/solver/solver.py:47-64: ``set("timeout", ...)`` then ``check()``), and that ``unknown``
is a rejection that sends the query to the fallback and counts ``sieve_rejected``.  Whether z3
itself then answers sat is z3's business (parity unpinned here: no z3 to run).
"""
import sys
import types

import pytest

from mythril_amd import frontend, plugin, smt
from mythril_amd.lower import Column, Schema
from mythril_amd.support import SolverStatistics, args


class _Rec:
    """A z3 expression stand-in: records its construction."""

    def __init__(self, *what):
        self.what = what

    def __eq__(self, other):  # z3: builds an equality term
        return _Rec("==", self, other)

    __hash__ = object.__hash__

    def __repr__(self):
        return "Rec%r" % (self.what,)


def make_stub_z3(result="sat"):
    z3 = types.ModuleType("z3")
    z3.calls = []
    z3.sat, z3.unsat, z3.unknown = "sat", "unsat", "unknown"

    class Solver:
        def __init__(self):
            self.params, self.assertions = {}, []
            z3.calls.append(("Solver", self))

        def set(self, key, value):
            self.params[key] = value

        def add(self, *cs):
            for c in cs:
                self.assertions.extend(c if isinstance(c, list) else [c])

        def check(self):
            z3.calls.append(("check", self))
            return getattr(z3, result)

        def sexpr(self):
            return "(solver %d)" % len(self.assertions)

    class Optimize(Solver):
        def __init__(self):
            super().__init__()
            self.objectives = []

        def minimize(self, e):
            self.objectives.append(("min", e))

        def maximize(self, e):
            self.objectives.append(("max", e))

        def sexpr(self):
            return "(optimize %d asserts %d objectives)" % (len(self.assertions),
                                                            len(self.objectives))

    z3.Solver, z3.Optimize = Solver, Optimize
    z3.BitVec = lambda name, w: _Rec("BitVec", name, w)
    z3.BitVecVal = lambda v, w: _Rec("BitVecVal", v, w)
    z3.BitVecSort = lambda w: _Rec("BitVecSort", w)
    z3.Array = lambda name, d, r: _Rec("Array", name, d, r)
    z3.Select = lambda a, k: _Rec("Select", a, k)
    return z3


@pytest.fixture
def stub_z3(monkeypatch):
    z3 = make_stub_z3()
    monkeypatch.setitem(sys.modules, "z3", z3)
    frontend.reset()
    yield z3
    frontend.reset()


class RawBool:
    """A reference Bool (laser/smt/bool.py): the z3 term is ``.raw``."""

    def __init__(self, name):
        self.raw = _Rec("constraint", name)


def _model(values, schema, arrays=None):
    ctx = smt.Context()
    ctx.b.symbols.arrays.update(arrays or {})
    return types.SimpleNamespace(ctx=ctx, schema=schema, values=values)


def _schema():
    s = Schema()
    s.columns["sender_1"] = Column("sender_1", 256, "var", "sender_1")
    s.columns["1_calldatasize"] = Column("1_calldatasize", 256, "var", "1_calldatasize")
    cell = Column("Storage[0]", 256, "cell", "Storage")
    cell.key = 0
    s.columns["Storage[0]"] = cell
    s.columns["__ground__"] = Column("__ground__", 1, "var", "__ground__")
    return s


def test_verifier_pins_the_witness_and_the_timeout(stub_z3):
    """z3_verifier: the query's z3 terms (.raw) plus one equality per scalar column and per
    array cell of the witness; timeout = min(solver_timeout, timeout_ms); sat -> accepted."""
    old = args.solver_timeout
    args.solver_timeout = 10000
    try:
        m = _model({"sender_1": 0xAFFE, "1_calldatasize": 36, "Storage[0]": 7, "__ground__": 0},
                   _schema(), {"Storage": (0, 256, 256)})
        cs = [RawBool("c1"), RawBool("c2")]
        assert plugin.z3_verifier(cs, m, timeout_ms=2500.7) is True
        (_, solver), (_, checked) = stub_z3.calls
        assert checked is solver
        assert solver.params == {"timeout": 2500}
        a = solver.assertions
        assert [x.what for x in a[:2]] == [("constraint", "c1"), ("constraint", "c2")]
        eqs = {repr(x) for x in a[2:]}
        assert repr(_Rec("==", _Rec("BitVec", "sender_1", 256), 0xAFFE)) in eqs
        assert repr(_Rec("==", _Rec("BitVec", "1_calldatasize", 256), 36)) in eqs
        sel = _Rec("Select", _Rec("Array", "Storage", _Rec("BitVecSort", 256),
                                  _Rec("BitVecSort", 256)), _Rec("BitVecVal", 0, 256))
        assert repr(_Rec("==", sel, 7)) in eqs
        assert len(a) == 5  # the __ground__ column is not a symbol
        # no budget passed: the solver timeout itself; a larger budget is capped by it
        stub_z3.calls.clear()
        plugin.z3_verifier(cs, m)
        assert stub_z3.calls[0][1].params == {"timeout": 10000}
        stub_z3.calls.clear()
        plugin.z3_verifier(cs, m, timeout_ms=50000)
        assert stub_z3.calls[0][1].params == {"timeout": 10000}
    finally:
        args.solver_timeout = old


def test_verifier_rejects_unknown_and_a_spent_budget(stub_z3, monkeypatch):
    m = _model({"sender_1": 1}, Schema())
    monkeypatch.setattr(stub_z3.Solver, "check", lambda self: stub_z3.unknown)
    assert plugin.z3_verifier([RawBool("c")], m, timeout_ms=100) is False
    monkeypatch.setattr(stub_z3.Solver, "check", lambda self: stub_z3.unsat)
    assert plugin.z3_verifier([RawBool("c")], m, timeout_ms=100) is False
    # nothing left of the budget: rejected without a solver call
    stub_z3.calls.clear()
    assert plugin.z3_verifier([RawBool("c")], m, timeout_ms=0) is False
    assert not [c for c in stub_z3.calls if c[0] == "check"]


def test_log_writer_prints_the_optimize_problem(stub_z3):
    """--solver-log of reference terms: an Optimize holding the constraints and objectives,
    printed by sexpr() (support/model.py:37-55)."""
    x = types.SimpleNamespace(raw=_Rec("x"))
    text = plugin.z3_log_writer([RawBool("a"), RawBool("b")], (x,), ())
    assert text == "(optimize 2 asserts 1 objectives)"
    (_, opt), = stub_z3.calls
    assert [o[0] for o in opt.objectives] == ["min"]


class _FakeSieve:
    def __init__(self, witness):
        self.witness = witness
        self.witnesses = {}

    def solve(self, b, roots, key=None, budget_s=None):
        return self.witness


def test_plugin_start_wires_z3_and_unknown_goes_to_the_fallback(stub_z3, monkeypatch):
    """SievePlugin.start with z3 importable: the verifier, the log writer and the term importer
    are the z3 ones.  A witness z3 cannot confirm (unknown) is rejected: the query goes, as it
    came, to the reference's get_model, and sieve_rejected counts it."""
    from mythril_amd.sieve import Witness
    from mythril_amd.smtlib import Z3Importer

    calls = []

    def reference_get_model(constraints, minimize=(), maximize=(), enforce_execution_time=True):
        calls.append(constraints)
        return "z3 model"

    mod = types.SimpleNamespace(get_model=reference_get_model)
    p = plugin.SievePlugin(modules=[mod])
    p.start()
    try:
        assert frontend._config["verify"] is plugin.z3_verifier
        assert frontend._config["log_writer"] is plugin.z3_log_writer
        assert isinstance(frontend._config["to_terms"], Z3Importer)
        assert frontend._config["fallback"] is reference_get_model
        smt.set_context(smt.Context())
        x = smt.symbol_factory.BitVecSym("x", 256)
        schema = Schema()
        schema.columns["x"] = Column("x", 256, "var", "x")
        fake = _FakeSieve(Witness(schema, {"x": 3}, 0, 1))
        monkeypatch.setattr(frontend, "sieve", lambda: fake)
        monkeypatch.setattr(stub_z3.Solver, "check", lambda self: stub_z3.unknown)
        before = SolverStatistics().sieve_rejected
        c = x == 3
        assert mod.get_model((c,)) == "z3 model"
        assert calls == [(c,)]
        assert SolverStatistics().sieve_rejected == before + 1
        # z3 confirms: the sieve's model is returned, the reference is not asked
        monkeypatch.setattr(stub_z3.Solver, "check", lambda self: stub_z3.sat)
        m = mod.get_model((x == 3, x != 4))
        assert m != "z3 model" and m.values == {"x": 3}
        assert len(calls) == 1
    finally:
        p.stop()
    assert mod.get_model is reference_get_model


def test_verifier_without_a_timeout_parameter(monkeypatch):
    """A verifier written to the plain (constraints, model) -> bool contract is called without
    timeout_ms (it used to raise TypeError and reject every witness)."""
    from mythril_amd.sieve import Witness

    seen = []

    def verify(constraints, model):
        seen.append(model.values)
        return True

    smt.set_context(smt.Context())
    x = smt.symbol_factory.BitVecSym("x", 256)
    schema = Schema()
    schema.columns["x"] = Column("x", 256, "var", "x")
    monkeypatch.setattr(frontend, "sieve", lambda: _FakeSieve(Witness(schema, {"x": 9}, 0, 1)))
    frontend.reset()
    try:
        frontend.configure(fallback=lambda *a: "z3", verify=verify)
        m = frontend.get_model((x == 9,))
        assert m != "z3" and seen == [{"x": 9}]
    finally:
        frontend.reset()


def test_unusable_device_is_probed_once(monkeypatch):
    """No library or no device: the first query fails over to the fallback and the failure is
    remembered, so later queries neither import their terms nor probe the device again
    (ADVICE r02); reconfiguring the sieve probes again."""
    from mythril_amd import sieve as sieve_mod

    made = []

    class Broken:
        def __init__(self, **kw):
            made.append(kw)
            raise RuntimeError("no gfx950 device")

    monkeypatch.setattr(sieve_mod, "Sieve", Broken)
    imported = []
    frontend.reset()
    try:
        frontend.configure(fallback=lambda *a: "z3",
                           to_terms=lambda cs: imported.append(cs) or (None, []))
        for k in range(3):
            assert frontend.get_model((RawBool("c%d" % k),)) == "z3"
        assert len(made) == 1 and imported == []
        frontend.configure(rows=1 << 12)
        assert frontend.get_model((RawBool("again"),)) == "z3"
        assert len(made) == 2
    finally:
        frontend.reset()
