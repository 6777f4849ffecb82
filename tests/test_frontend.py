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
