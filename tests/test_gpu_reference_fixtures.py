"""The reference's own solver-layer outcome tests (tests/reference_cases.py) through
``frontend.get_model`` on an MI355X.

* UNSAT cases (keccak_tests.py, calldata_test.py, independece_solver_test.py, and the negated
  ground values of calldata/storage_test.py): the sieve returns no witness and the query goes to
  the fallback, unchanged (the fallback here records the call: z3 is absent on the box);
* SAT cases: the sieve returns a witness that the ORACLE accepts as a model of the original query
  (arrays, keccak UFs and inverses under the model the row denotes, oracle/term_eval.py); the
  fallback is never asked.  A SAT case the sieve cannot answer would carry a named
  ``fallback_reason`` in tests/reference_cases.py and must reach the fallback (none does);
* model_test.py: decls / ``model[x.raw.decl()]`` / ``model.eval(x.raw).as_long()``;
* calldata_test.py:28-39: ``model.eval(calldata.calldatasize)`` of an empty query is 7.

Run on the GPU box:  python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
"""
import pytest

from mythril_amd import frontend
from mythril_amd.model import Model
from mythril_amd.support import SolverStatistics
from tests.reference_cases import (BY_NAME, DIVERGENT, KECCAK_MODULE, ConcreteCalldata,
                                   case_ids, shared_keccak_cases)
from tests.test_reference_fixtures import holds_original

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _reset():
    frontend.reset()
    yield
    frontend.reset()


def _recording_fallback():
    calls = []

    def fallback(constraints, minimize, maximize, enforce_execution_time):
        calls.append(constraints)
        return "fallback"

    frontend.configure(fallback=fallback)
    return calls


def _check_outcome(case, ctx, cs):
    name = case.name
    calls = _recording_fallback()
    stats = SolverStatistics()
    misses = stats.sieve_misses
    m = frontend.get_model(tuple(cs))
    if name in DIVERGENT:
        # satisfiable as restated (the reference's assertion diverges from its code): the keccak
        # second chance answers it (round 6) with a model of the query
        assert isinstance(m, Model), (name, m)
        assert holds_original(ctx, cs, m.schema, m.values), name
    elif case.expected == "unsat" or case.fallback_reason:
        assert m == "fallback" and len(calls) == 1, name
        assert list(calls[0]) == list(cs)  # handed over unchanged
        assert stats.sieve_misses == misses + 1, name  # a miss, not an error / unsupported
    else:
        assert isinstance(m, Model) and not calls, name
        assert holds_original(ctx, cs, m.schema, m.values), name
        for c in cs:  # Model.eval on the device agrees with the witness
            assert m.eval(c, model_completion=True) is True, name
    return m


@pytest.mark.parametrize("name", case_ids())
def test_reference_outcome_on_gpu(gpu_ctx, name):
    case = BY_NAME[name]
    ctx, cs = case.build()
    _check_outcome(case, ctx, cs)


def test_reference_keccak_outcomes_with_a_shared_manager_on_gpu(gpu_ctx):
    """keccak_tests.py's cases in file order over ONE manager, as the reference's module-level
    keccak_function_manager serves them: concrete hashes of earlier cases join later cases'
    Or-chains.  Same outcomes as with a fresh manager."""
    out = shared_keccak_cases()
    assert [c.name for c, _, _ in out] == KECCAK_MODULE
    for case, ctx, cs in out:
        frontend.reset()
        _check_outcome(case, ctx, cs)


def test_keccak_other_num_defines_b(gpu_ctx):
    """keccak_tests.py:122-138: b == keccak(2 * keccak(a)) is answered by solving for b (a
    definition): the witness's b is the device's value of the keccak term under its a."""
    ctx, cs = BY_NAME["keccak_other_num"].build()
    s = frontend.sieve()
    before = s.stats.extra.get("definitions", 0)
    m = frontend.get_model(tuple(cs))
    assert isinstance(m, Model)
    assert s.stats.extra.get("definitions", 0) == before + 1
    assert holds_original(ctx, cs, m.schema, m.values)


def test_model_accessors(gpu_ctx):
    """model_test.py:5-56."""
    ctx, cs = BY_NAME["model_x_eq_2"].build()
    from mythril_amd.smt import symbol_factory

    x = symbol_factory.BitVecSym("x", 256)
    m = frontend.get_model(tuple(cs))
    assert isinstance(m, Model)
    assert x.raw.decl() in m.decls()
    assert 2 == m[x.raw.decl()]
    assert 2 == m.eval(x.raw).as_long()


def test_concrete_calldatasize_evaluates_to_7(gpu_ctx):
    """calldata_test.py:28-39: an empty query's model evaluates the concrete calldatasize to 7."""
    from mythril_amd import smt

    ctx = smt.Context()
    smt.set_context(ctx)
    calldata = ConcreteCalldata(0, [1, 4, 7, 3, 7, 2, 9])
    m = frontend.get_model(())
    assert isinstance(m, Model)
    assert m.eval(calldata.calldatasize.raw) == 7
    # and the concrete bytes read back through the K-store chain (calldata.py:118-147)
    assert [m.eval(calldata[i]) for i in range(7)] == [1, 4, 7, 3, 7, 2, 9]
    assert m.eval(calldata[100]) == 0
