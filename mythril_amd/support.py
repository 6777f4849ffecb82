"""The reference's solver-adjacent globals, reused when mythril is importable, mirrored if not.

* ``UnsatError``        mythril/exceptions.py:16-20
* ``args``              mythril/support/support_args.py:1-17 (solver_timeout 10000 ms, ...)
* ``time_handler``      mythril/laser/ethereum/time_handler.py:5-18
* ``RefModel``          mythril/laser/smt/model.py:6-59 (the Model get_model returns: a list of z3
                        ModelRefs), used for a z3-verified sieve witness
* ``SolverStatistics``  mythril/laser/smt/solver/solver_statistics.py:8-43, plus the sieve's own
                        counters (hits / misses / unsupported / errors / rejected, seconds), kept
                        beside z3's so wall-time splits stay comparable.

When the reference is importable its objects are used, so the front end reads the same
``args`` the CLI wrote (mythril_analyzer.py:72-78) and counts into the same statistics object.
"""
from __future__ import annotations

import time

try:  # the reference, when it runs around this module
    from mythril.exceptions import UnsatError  # type: ignore
    from mythril.laser.smt import Model as RefModel  # type: ignore
    from mythril.laser.ethereum.time_handler import time_handler  # type: ignore
    from mythril.laser.smt.solver.solver_statistics import \
        SolverStatistics as _RefStats  # type: ignore
    from mythril.support.support_args import args  # type: ignore

    HAVE_MYTHRIL = True
except Exception:  # z3 / mythril absent: standalone mirrors
    HAVE_MYTHRIL = False
    _RefStats = None

    class RefModel:  # type: ignore[no-redef]
        """laser/smt/model.py:6-59: wraps z3 ModelRefs; ``decls``, ``[item]`` and ``eval`` ask
        them in order (the last one answers ``eval`` when no earlier one declares the term)."""

        def __init__(self, models=None):
            self.raw = models or []

        def decls(self):
            result = []
            for internal_model in self.raw:
                result.extend(internal_model.decls())
            return result

        def __getitem__(self, item):
            for k, internal_model in enumerate(self.raw):
                try:
                    result = internal_model[item]
                    if result is not None:
                        return result
                except IndexError:
                    if k == len(self.raw) - 1:
                        raise
            return None

        def eval(self, expression, model_completion: bool = False):
            for k, internal_model in enumerate(self.raw):
                relevant = expression.decl() in list(internal_model.decls())
                if relevant or k == len(self.raw) - 1:
                    return internal_model.eval(expression, model_completion)
            return None

    class UnsatError(Exception):  # type: ignore[no-redef]
        """mythril/exceptions.py:16-20."""

    class _Args:
        """support_args.py:1-17."""

        def __init__(self):
            self.solver_timeout = 10000
            self.sparse_pruning = True
            self.unconstrained_storage = False
            self.parallel_solving = False
            self.call_depth_limit = 3
            self.iprof = True
            self.solver_log = None

    args = _Args()

    class _TimeHandler:
        """time_handler.py:5-18 (the reference's is a Singleton; so is this instance)."""

        def __init__(self):
            self._start_time = None
            self._execution_time = None

        def start_execution(self, execution_time):
            self._start_time = int(time.time() * 1000)
            self._execution_time = execution_time * 1000

        def time_remaining(self):
            if self._start_time is None:  # no analysis running: no execution budget
                return float("inf")
            return self._execution_time - (int(time.time() * 1000) - self._start_time)

    time_handler = _TimeHandler()

_SIEVE_FIELDS = ("sieve_hits", "sieve_misses", "sieve_unsupported", "sieve_errors",
                 "sieve_rejected")


class _Stats:
    """solver_statistics.py:8-43 plus sieve counters (a process-wide singleton)."""

    _inst = None

    def __new__(cls):
        if cls._inst is None:
            inst = object.__new__(cls)
            inst.enabled = False
            inst.query_count = 0
            inst.solver_time = 0.0
            cls._inst = inst
        return cls._inst

    def __repr__(self):
        return "Query count: {} \nSolver time: {}".format(self.query_count, self.solver_time)


def SolverStatistics():
    """The reference's SolverStatistics singleton (or the mirror), with sieve counters added."""
    s = _RefStats() if _RefStats is not None else _Stats()
    for f in _SIEVE_FIELDS:
        if not hasattr(s, f):
            setattr(s, f, 0)
    if not hasattr(s, "sieve_time"):
        s.sieve_time = 0.0
    return s
