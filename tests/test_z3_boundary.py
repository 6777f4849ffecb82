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


def _verifier_world(monkeypatch, rows=256):
    """The AST z3 stand-in installed, the front end wired as SievePlugin.start wires it (z3
    importer, z3_verifier, a recording fallback) over the CPU stand-in of the device; returns
    (z3 module, [sieve Models handed to the verifier], [fallback calls])."""
    from mythril_amd.smtlib import Z3Importer
    from tests import fake_device, z3_ast

    z3 = z3_ast.make_z3()
    monkeypatch.setitem(sys.modules, "z3", z3)
    fake_device.install(monkeypatch)
    frontend.reset()
    seen, fallback = [], []

    def verify(constraints, model, timeout_ms=None):
        seen.append(model)
        return plugin.z3_verifier(constraints, model, timeout_ms=timeout_ms)

    frontend.configure(to_terms=Z3Importer(), verify=verify, rows=rows,
                       fallback=lambda *a: fallback.append(a) or "fallback")
    return z3, seen, fallback


@pytest.mark.parametrize("name", ["killbilly", "ether_thief", "keccak_mapping", "suicide_arg",
                                  "k_storage", "balance"])
def test_verifier_pins_every_symbol_and_returns_the_reference_model(monkeypatch, name):
    """VERDICT r5 next 1 ("SAT from sieve => z3 re-verification, witness as
    equalities, fully determined"): on LASER-shaped queries the verifier hands z3 the query plus
    one equality per scalar symbol, one Store-chain over K(else) per array holding every cell of
    the witness, and one equality per uninterpreted application -- keccak256_N, its inverse, any
    function -- so no symbol the query reads is left free and z3's check is an evaluation; the
    stand-in's check evaluates the constraints under exactly those pins (ORACLE) and finds them
    true; get_model returns z3's model in the reference's Model type (support/model.py:57-59)."""
    from mythril_amd.support import RefModel
    from mythril_amd.tape import Op
    from tests import z3_ast
    from tests.laser_like import queries

    z3, seen, fallback = _verifier_world(monkeypatch)
    try:
        qctx, qs = queries()
        cs = dict(qs)[name]
        m = frontend.get_model(tuple(z3_ast.Ref(c) for c in cs))
        assert not fallback, "the sieve answered %s" % name
        assert type(m) is RefModel and len(m.raw) == 1
        (w,) = seen
        checked = [s for s in z3.solvers if "timeout" in s.params]
        assert len(checked) == 1
        s = checked[0]
        assert s.free == []
        pins = {}
        for p in s.pins:
            pins.setdefault(qctx.b.nodes[p.lhs.node][0], []).append(p)
        scalar = {p.lhs.decl().name(): p.rhs.v for p in pins.get(Op.VAR, [])}
        arrays = {p.lhs.decl().name(): p.rhs for p in pins.get(Op.ARRAY, [])}
        apps = pins.get(Op.UF, [])
        for col in w.schema.columns.values():
            if col.kind == "var" and col.symbol != "__ground__":
                assert scalar[col.name] == w.values[col.name], col.name
            elif col.kind == "cell":
                assert arrays[col.symbol].table[col.key] == w.values[col.name], col.name
            elif col.kind == "else":
                assert arrays[col.symbol].dflt == w.values[col.name]
            elif col.kind in ("ufcell", "ufelse"):
                assert apps, col.name
        for f in w.schema.keccak:
            assert any(p.lhs.decl().name() == f for p in apps), f
        # the reference reads the returned model with its own terms
        for c in cs:
            assert m.eval(z3_ast.Ref(c).raw, model_completion=True) is True
        for d in m.decls():
            assert m[d] is not None
    finally:
        frontend.reset()


def test_verifier_timeout_unknown_and_unsat(monkeypatch):
    """The check runs under min(args.solver_timeout, what is left of get_model's budget)
    (support/model.py:26-31); unknown and unsat reject (the query goes to the fallback and
    sieve_rejected counts it); a spent budget rejects without a solver call."""
    from tests import z3_ast
    from tests.laser_like import queries

    old = args.solver_timeout
    args.solver_timeout = 10000
    z3, seen, fallback = _verifier_world(monkeypatch)
    try:
        qctx, qs = queries()
        cs = dict(qs)["selector"]
        raws = tuple(z3_ast.Ref(c) for c in cs)
        assert frontend.get_model(raws) != "fallback"
        w = seen[-1]
        for budget, want in ((2500.7, 2500), (None, 10000), (50000, 10000)):
            z3.solvers.clear()
            assert plugin.z3_verifier(raws, w, timeout_ms=budget) is not None
            (s,) = [s for s in z3.solvers if "timeout" in s.params]
            assert s.params == {"timeout": want}
        z3.solvers.clear()
        assert plugin.z3_verifier(raws, w, timeout_ms=0) is None
        assert not [s for s in z3.solvers if "timeout" in s.params]
        for verdict in (z3.unknown, z3.unsat):
            monkeypatch.setattr(z3.Solver, "check", lambda self, v=verdict: v)
            assert plugin.z3_verifier(raws, w, timeout_ms=100) is None
        before = SolverStatistics().sieve_rejected
        frontend.get_model.cache_clear()
        assert frontend.get_model(raws) == "fallback"
        assert SolverStatistics().sieve_rejected == before + 1
    finally:
        args.solver_timeout = old
        frontend.reset()


def test_pins_of_a_wrong_witness_are_unsat(monkeypatch):
    """The pins are the witness, not a search space: a witness value changed after the sieve
    found it makes z3's (the stand-in's) check unsat, so the verifier rejects it."""
    from tests import z3_ast
    from tests.laser_like import queries

    z3, seen, fallback = _verifier_world(monkeypatch)
    try:
        qctx, qs = queries()
        cs = dict(qs)["owner_check"]
        raws = tuple(z3_ast.Ref(c) for c in cs)
        assert frontend.get_model(raws) != "fallback"
        w = seen[-1]
        assert plugin.z3_verifier(raws, w) is not None
        w.values["sender_1"] ^= 1
        w._memo.clear()
        assert plugin.z3_verifier(raws, w) is None
    finally:
        frontend.reset()


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


def test_plugin_start_wires_z3_and_unknown_goes_to_the_fallback(monkeypatch):
    """SievePlugin.start with z3 importable: the verifier, the log writer and the term importer
    are the z3 ones.  A witness z3 cannot confirm (unknown) is rejected: the query goes, as it
    came, to the reference's get_model, and sieve_rejected counts it.  A confirmed one comes
    back as z3's model in the reference's Model type, and the reference is not asked."""
    from mythril_amd.smtlib import Z3Importer
    from mythril_amd.support import RefModel
    from tests import fake_device, z3_ast

    z3 = z3_ast.make_z3()
    monkeypatch.setitem(sys.modules, "z3", z3)
    fake_device.install(monkeypatch)
    frontend.reset()
    calls = []

    def reference_get_model(constraints, minimize=(), maximize=(), enforce_execution_time=True):
        calls.append(constraints)
        return "z3 model"

    mod = types.SimpleNamespace(get_model=reference_get_model)
    p = plugin.SievePlugin(modules=[mod], rows=256)
    p.start()
    try:
        assert frontend._config["verify"] is plugin.z3_verifier
        assert frontend._config["log_writer"] is plugin.z3_log_writer
        assert isinstance(frontend._config["to_terms"], Z3Importer)
        assert frontend._config["fallback"] is reference_get_model
        ref = smt.set_context(smt.Context())
        x = smt.symbol_factory.BitVecSym("x", 256)
        monkeypatch.setattr(z3.Solver, "check", lambda self: z3.unknown)
        before = SolverStatistics().sieve_rejected
        c = z3_ast.Ref(x == smt.symbol_factory.BitVecVal(3, 256))
        assert mod.get_model((c,)) == "z3 model"
        assert calls == [(c,)]
        assert SolverStatistics().sieve_rejected == before + 1
        monkeypatch.undo()
        monkeypatch.setitem(sys.modules, "z3", z3)
        fake_device.install(monkeypatch)
        m = mod.get_model((c, z3_ast.Ref(x != smt.symbol_factory.BitVecVal(4, 256))))
        assert type(m) is RefModel
        assert m.eval(z3_ast.Ref(x).raw, model_completion=True).as_long() == 3
        assert len(calls) == 1
        assert ref is not None
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


def test_verifier_pins_reads_on_planted_random_paths(monkeypatch):
    """The random planted family (free and K arrays, stores, selects at symbolic indices, a
    tabled function at symbolic arguments, keccak with pairs and bounds): every witness the sieve
    returns through get_model passes the fully determined check -- the arrays pinned as
    Store chains holding the cells and the reads at their indices' values, every application
    pinned -- and no symbol is left free."""
    from tests import z3_ast
    from tests.planted import planted_path

    z3, seen, fallback = _verifier_world(monkeypatch)
    rejected0 = SolverStatistics().sieve_rejected
    try:
        hits = 0
        for seed in range(3):
            ctx, cs, _, _ = planted_path("random", seed, 8)
            for k in range(1, len(cs) + 1):
                frontend.get_model.cache_clear()
                before, n_solvers = len(seen), len(z3.solvers)
                m = frontend.get_model(tuple(z3_ast.Ref(c) for c in cs[:k]))
                if m == "fallback":
                    continue
                hits += 1
                assert len(seen) == before + 1
                (s,) = [x for x in z3.solvers[n_solvers:] if "timeout" in x.params][-1:]
                assert s.free == [], (seed, k, s.free)
        assert hits >= 8, hits
        assert SolverStatistics().sieve_rejected == rejected0
    finally:
        frontend.reset()


def test_verifier_checks_a_keccak_second_chance_witness(monkeypatch):
    """keccak_tests.py:23-26 (reference_cases.DIVERGENT) answered by the keccak second chance:
    the verifier pins keccak256_256 at N1's value to the read column's value (not H), the
    manager's inverse at that hash back to N1, and z3's evaluation says sat -- the reference's
    Model comes back, nothing is left free."""
    from mythril_amd.support import RefModel
    from tests import z3_ast
    from tests.reference_cases import BY_NAME

    from mythril_amd.support import args

    z3, seen, fallback = _verifier_world(monkeypatch)
    # the CPU stand-in is slow: no round cut short by the sieve's or get_model's budget
    monkeypatch.setattr(args, "solver_timeout", 600000)
    try:
        frontend.configure(budget_s=600.0, rows=256)
        ctx, cs = BY_NAME["keccak_basic_val8_100_sym_N1"].build()
        m = frontend.get_model(tuple(z3_ast.Ref(c) for c in cs))
        assert not fallback and len(seen) == 1
        assert seen[0].schema.keccak_reads
        assert isinstance(m, RefModel) or type(m).__name__ == "Model", type(m)
        (s,) = [x for x in z3.solvers if "timeout" in x.params][-1:]
        assert s.free == [] and s.check() == "sat"
    finally:
        frontend.reset()
