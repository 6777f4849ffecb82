"""Host logic of the get_model front end and the plugin (no device needed).

``get_model`` must keep the reference's contract (mythril/support/model.py:15-62): Python
``False`` -> UnsatError, Python bools dropped, time budget -> UnsatError, objectives always go to
the fallback, results cached, UNSAT never cached.  The plugin must rebind and restore the three
import sites of SURVEY.md §3.2 from LASER's start/stop hooks (svm.py:578-643).
"""
import types

import pytest

from mythril_amd import frontend, plugin, smt
from mythril_amd.support import SolverStatistics, UnsatError, args, time_handler


@pytest.fixture(autouse=True)
def _reset():
    frontend.reset()
    yield
    frontend.reset()


def _x():
    smt.set_context(smt.Context())
    return smt.symbol_factory.BitVecSym("x", 256)


def test_python_false_is_unsat_and_bools_are_dropped():
    calls = []

    def fallback(cs, mn, mx, enf):
        calls.append(cs)
        return "model"

    frontend.configure(fallback=fallback, enabled=False)
    with pytest.raises(UnsatError):
        frontend.get_model((True, False))
    x = _x()
    assert frontend.get_model((True, x == 3)) == "model"
    assert len(calls[-1]) == 1  # the Python bool was dropped


def test_objectives_always_go_to_the_fallback():
    seen = []
    frontend.configure(fallback=lambda cs, mn, mx, enf: seen.append((mn, mx)) or "opt")
    x = _x()
    # the sieve is enabled, but minimize is set: it must not be consulted
    frontend._config["sieve_kwargs"] = {"device": 999}  # would fail loudly if it were built
    assert frontend.get_model((x == 3,), minimize=(x,)) == "opt"
    assert seen == [((x,), ())]


def test_sat_results_are_cached_unsat_are_not():
    n = {"calls": 0}

    def fallback(cs, mn, mx, enf):
        n["calls"] += 1
        if len(cs) > 1:
            raise UnsatError
        return "m"

    frontend.configure(fallback=fallback, enabled=False)
    x = _x()
    c1, c2 = x == 1, x == 2
    frontend.get_model((c1,))
    frontend.get_model((c1,))
    assert n["calls"] == 1
    for _ in range(2):
        with pytest.raises(UnsatError):
            frontend.get_model((c1, c2))
    assert n["calls"] == 3


def test_time_budget_exhausted_is_unsat():
    frontend.configure(fallback=lambda *a: "m", enabled=False)
    x = _x()
    old = (time_handler._start_time, time_handler._execution_time)
    time_handler.start_execution(0)  # no time left: min(timeout, remaining - 500) <= 0
    try:
        with pytest.raises(UnsatError):
            frontend.get_model((x == 9,))
        assert frontend.get_model((x == 9,), enforce_execution_time=False) == "m"
    finally:
        time_handler._start_time, time_handler._execution_time = old


def test_no_fallback_reports_unknown_as_unsat():
    frontend.configure(enabled=False)
    x = _x()
    with pytest.raises(UnsatError):
        frontend.get_model((x == 1,))


def test_sieve_failure_falls_back():
    # a device that cannot exist: the sieve errors, the fallback answers, the error is counted
    frontend.configure(fallback=lambda *a: "z3", device=12345)
    x = _x()
    before = SolverStatistics().sieve_errors
    assert frontend.get_model((x == 1,)) == "z3"
    assert SolverStatistics().sieve_errors == before + 1


def test_remembered_sieve_failure_raises_fresh_exceptions():
    """After a failed construction every query gets a NEW exception carrying the message (a
    re-raised saved exception would chain each query's frames, and their constraints, onto one
    traceback for the rest of the run)."""
    frontend.configure(fallback=lambda *a: "z3", device=12345)
    _x()
    with pytest.raises(Exception):
        frontend.sieve()
    seen = []
    for _ in range(3):
        with pytest.raises(frontend.SieveUnavailable) as ei:
            frontend.sieve()
        seen.append(ei.value)
    assert len({id(e) for e in seen}) == 3
    assert all(len(list(_tb(e))) < 4 for e in seen)
    x = smt.symbol_factory.BitVecSym("y", 256)
    assert frontend.get_model((x == 2,)) == "z3"


def _tb(e):
    tb = e.__traceback__
    while tb is not None:
        yield tb
        tb = tb.tb_next


class FakeLaser:
    """The hook registry of LaserEVM (svm.py:578-643)."""

    def __init__(self):
        self.hooks = {}

    def register_laser_hooks(self, hook_type, hook):
        self.hooks.setdefault(hook_type, []).append(hook)


def test_plugin_rebinds_and_restores_the_import_sites():
    orig = lambda *a, **k: "reference"  # noqa: E731
    mods = [types.SimpleNamespace(get_model=orig) for _ in range(3)]
    builder = plugin.SievePluginBuilder()
    assert builder.plugin_name == "constraint-sieve"
    assert builder.plugin_name != "dependency-pruner"
    assert hasattr(builder, "plugin_default_enabled")
    p = builder(modules=mods)
    laser = FakeLaser()
    p.initialize(laser)
    assert set(laser.hooks) == {"start_sym_exec", "stop_sym_exec"}
    for h in laser.hooks["start_sym_exec"]:
        h()
    assert all(m.get_model is frontend.get_model for m in mods)
    assert frontend._config["fallback"] is orig
    for h in laser.hooks["stop_sym_exec"]:
        h()
    assert all(m.get_model is orig for m in mods)
    assert frontend._config["fallback"] is None


def test_constraints_mirror_is_possible():
    """Constraints.is_possible (constraints.py:25-35) through the rebound name."""
    frontend.configure(fallback=lambda cs, *a: (_ for _ in ()).throw(UnsatError)
                       if len(cs) > 1 else "m", enabled=False)
    x = _x()

    def is_possible(cs):
        try:
            frontend.get_model(tuple(cs))
        except UnsatError:
            return False
        return True

    assert is_possible([x == 1])
    assert not is_possible([x == 1, x == 2])


# -- boundary defects of round 1 (VERDICT "What's weak" 7) -------------------------------------
def _stat_smt_query(func):
    """laser/smt/solver/solver_statistics.py:8-26 restated: the reference counts every z3
    check itself, on BaseSolver.check."""
    stats = SolverStatistics()

    def wrapper(*a, **k):
        if not stats.enabled:
            return func(*a, **k)
        stats.query_count += 1
        return func(*a, **k)
    return wrapper


def test_fallback_queries_are_counted_once():
    """The reference's get_model counts itself through stat_smt_query; the front end must not
    count the same query again (solver.py:47)."""
    stats = SolverStatistics()
    old = (stats.enabled, stats.query_count)
    stats.enabled = True
    stats.query_count = 0
    check = _stat_smt_query(lambda cs: "m")
    frontend.configure(fallback=lambda cs, mn, mx, enf: check(cs), enabled=False)
    try:
        x = _x()
        for k in range(5):
            frontend.get_model((x == k,))
        assert stats.query_count == 5
    finally:
        stats.enabled, stats.query_count = old


class ForeignBool:
    """A z3-backed reference Bool: no ``.ctx``, not an smt.Bool (z3 is absent here)."""

    def __init__(self, k):
        self.k = k

    def __hash__(self):
        return hash(("foreign", self.k))

    def __eq__(self, other):
        return isinstance(other, ForeignBool) and other.k == self.k


def test_solver_log_with_foreign_terms_does_not_escape(tmp_path):
    """--solver-log with reference terms: round 1 raised AttributeError out of get_model
    (smtlib.to_smtlib read items[0].ctx).  Now the query is answered and logged by the writer
    the plugin configures, or skipped when there is none."""
    old = args.solver_log
    args.solver_log = str(tmp_path / "log")
    try:
        frontend.configure(fallback=lambda *a: "z3")
        assert frontend.get_model((ForeignBool(1),)) == "z3"
        assert not (tmp_path / "log").exists() or not list((tmp_path / "log").iterdir())
        frontend.configure(log_writer=lambda cs, mn, mx: "(assert foreign)\n(check-sat)\n")
        assert frontend.get_model((ForeignBool(2),)) == "z3"
        files = list((tmp_path / "log").iterdir())
        assert len(files) == 1 and files[0].read_text().startswith("(assert foreign)")
        # the reference's own get_model as fallback writes its file itself: not written twice
        frontend.configure(fallback_logs=True)
        assert frontend.get_model((ForeignBool(3),)) == "z3"
        assert len(list((tmp_path / "log").iterdir())) == 1
    finally:
        args.solver_log = old


class _FakeSieve:
    def __init__(self, witness=None):
        self.budgets = []
        self.witness = witness
        self.witnesses = {}

    def solve(self, b, roots, key=None, budget_s=None):
        self.budgets.append(budget_s)
        return self.witness


def test_sieve_budget_follows_the_solver_timeout(monkeypatch):
    """The sieve runs inside get_model's own budget (support/model.py:26-31)."""
    fake = _FakeSieve()
    monkeypatch.setattr(frontend, "sieve", lambda: fake)
    old = args.solver_timeout
    args.solver_timeout = 1234
    try:
        frontend.configure(fallback=lambda *a: "z3")
        x = _x()
        assert frontend.get_model((x == 1,)) == "z3"
        assert fake.budgets == [pytest.approx(1.234)]
        t0 = (time_handler._start_time, time_handler._execution_time)
        time_handler.start_execution(1)  # 1000 ms left -> budget min(1234, 1000 - 500)
        try:
            assert frontend.get_model((x == 2,)) == "z3"
        finally:
            time_handler._start_time, time_handler._execution_time = t0
        assert fake.budgets[1] <= 0.5
    finally:
        args.solver_timeout = old


def test_verifier_gets_the_budget_and_errors_reject(monkeypatch):
    from mythril_amd.lower import Schema
    from mythril_amd.sieve import Witness

    fake = _FakeSieve(Witness(Schema(), {}, 0, 1))
    monkeypatch.setattr(frontend, "sieve", lambda: fake)
    seen = []

    def verify(cs, m, timeout_ms=None):
        seen.append(timeout_ms)
        return True

    old = args.solver_timeout
    args.solver_timeout = 2000
    try:
        frontend.configure(fallback=lambda *a: "z3", verify=verify)
        x = _x()
        m = frontend.get_model((x == 1,))
        assert m != "z3" and 0 < seen[0] <= 2000
        before = SolverStatistics().sieve_rejected

        def boom(cs, m, timeout_ms=None):
            raise RuntimeError("z3 exploded")

        frontend.configure(verify=boom)
        assert frontend.get_model((x == 5,)) == "z3"
        assert SolverStatistics().sieve_rejected == before + 1
    finally:
        args.solver_timeout = old


def test_plugin_is_default_enabled_and_env_switch(monkeypatch):
    """Only default-enabled entry-point plugins are loaded by the CLI (plugin/loader.py:73-80)."""
    assert plugin.SievePluginBuilder.plugin_default_enabled is True
    monkeypatch.setenv("MYTHRIL_AMD_SIEVE", "0")
    assert plugin.SievePluginBuilder().enabled is False
    monkeypatch.setenv("MYTHRIL_AMD_SIEVE", "1")
    assert plugin.SievePluginBuilder().enabled is True


def test_setup_declares_the_entry_point():
    """plugin/discovery.py:17-21: pkg_resources.iter_entry_points("mythril.plugins")."""
    import importlib
    import os
    import runpy

    import setuptools

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    captured = {}
    orig = setuptools.setup
    setuptools.setup = lambda **kw: captured.update(kw)
    try:
        runpy.run_path(os.path.join(root, "setup.py"), run_name="setup")
    finally:
        setuptools.setup = orig
    (line,) = captured["entry_points"]["mythril.plugins"]
    name, target = [x.strip() for x in line.split("=")]
    assert name == plugin.SievePluginBuilder.plugin_name
    mod, cls = target.split(":")
    assert getattr(importlib.import_module(mod), cls) is plugin.SievePluginBuilder
    assert "libmythril_hip.so" in captured["package_data"]["mythril_amd"]
