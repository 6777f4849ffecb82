"""Solver front end: ``get_model`` with the reference's signature and semantics, sieve first.

Mirrors mythril/support/model.py:15-62 line for line in behaviour —

* ``lru_cache(maxsize=2**23)`` keyed on (constraints, minimize, maximize,
  enforce_execution_time); UNSAT raises, so it is never cached;
* time budget: ``min(args.solver_timeout, time_handler.time_remaining() - 500)``, and
  ``UnsatError`` when it is not positive (only with ``enforce_execution_time``);
* a Python ``False`` among the constraints raises ``UnsatError``; Python bools are dropped;
* ``args.solver_log``: the query is written as SMT-LIB2 to ``<dir>/<abs(hash(...))>.smt2``
  (smtlib.py prints this package's terms; foreign terms go through the configured
  ``log_writer``, z3's own ``Optimize.sexpr()`` under the plugin).  A query answered by the
  fallback is logged by the fallback itself (the reference's get_model writes the file), so no
  query is written twice and a writer error never escapes ``get_model``;
* sat -> a ``Model``; unknown / unsat -> ``UnsatError``
* ``SolverStatistics``: ``query_count`` / ``solver_time`` stay z3's own counters — the
  reference's ``stat_smt_query`` on ``BaseSolver.check`` (laser/smt/solver/solver.py:47)
  already counts every fallback query, so the front end adds only the ``sieve_*`` counters

— with one change: when there is nothing to optimise (``minimize == maximize == ()``, the
feasibility case of ``Constraints.is_possible`` and the detection modules), the
query first goes to the sieve (sieve.py).  A witness comes back as a sieve ``Model``, re-verified
by the configured verifier: under the plugin, z3 checks the query with every symbol pinned to the
witness (plugin.witness_pins) and the caller gets z3's model in the reference's ``Model``
(plugin.z3_verifier); with no verifier, the sieve ``Model`` itself.  A miss,
an unsupported term, a device error or a failed verification hands the query, unchanged, to the
fallback solver — the reference's own ``get_model`` when installed by the plugin.  With no
fallback configured a miss is reported the way the reference reports a z3 ``unknown``:
``UnsatError``.  Queries with objectives always go to the fallback (transaction sequences in
reports must stay z3 Optimize output, analysis/solver.py:48-96).
"""
from __future__ import annotations

import inspect
import logging
import threading
import time
from functools import lru_cache
from pathlib import Path
from typing import Callable, Optional

from .support import SolverStatistics, UnsatError, args, time_handler

log = logging.getLogger(__name__)

_tls = threading.local()
_config = {
    "fallback": None,   # callable(constraints, minimize, maximize, enforce_execution_time)
    "verify": None,     # callable(constraints, model[, timeout_ms=...]) -> verdict (z3 re-check):
                        # falsy rejects, True keeps the sieve Model, another object is the
                        # model returned instead (z3_verifier: the reference's Model); timeout_ms
                        # (what is left of get_model's budget) is passed only to a verifier that
                        # declares it (or **kwargs)
    "to_terms": None,   # callable(constraints) -> (smt.Context, [Bool]) for foreign terms
    "log_writer": None,  # callable(constraints, minimize, maximize) -> SMT-LIB2 text (foreign)
    "fallback_logs": False,  # the fallback writes --solver-log files itself (the reference's)
    "sieve_kwargs": {},
    "enabled": True,
}


class SieveUnavailable(RuntimeError):
    """This thread's sieve could not be created (no library, no gfx950 device); the message
    is the original failure's."""


def configure(*, fallback: Optional[Callable] = None, verify: Optional[Callable] = None,
              to_terms: Optional[Callable] = None, enabled: Optional[bool] = None,
              log_writer: Optional[Callable] = None, fallback_logs: Optional[bool] = None,
              **sieve_kwargs) -> None:
    """Set the fallback solver, the witness verifier, the term importer and sieve options."""
    if fallback is not None:
        _config["fallback"] = fallback
    if log_writer is not None:
        _config["log_writer"] = log_writer
    if fallback_logs is not None:
        _config["fallback_logs"] = fallback_logs
    if verify is not None:
        _config["verify"] = verify
    if to_terms is not None:
        _config["to_terms"] = to_terms
    if enabled is not None:
        _config["enabled"] = enabled
    if sieve_kwargs:
        _config["sieve_kwargs"] = dict(sieve_kwargs)
        close_sieve()
    get_model.cache_clear()


def _takes_timeout(fn) -> bool:
    try:
        ps = inspect.signature(fn).parameters.values()
    except (TypeError, ValueError):
        return False
    return any(p.name == "timeout_ms" or p.kind == p.VAR_KEYWORD for p in ps)


def _verify(verify, constraints, m, left):
    """The verifier's verdict: falsy rejects; True accepts the sieve's Model; any other object
    is the model to return instead (plugin.z3_verifier: the reference's Model of z3's check)."""
    if _takes_timeout(verify):
        return verify(constraints, m, timeout_ms=left)
    return verify(constraints, m)


def reset() -> None:
    """Back to defaults (tests, plugin stop)."""
    _config.update(fallback=None, verify=None, to_terms=None, log_writer=None,
                   fallback_logs=False, sieve_kwargs={}, enabled=True)
    close_sieve()
    get_model.cache_clear()


def sieve():
    """This thread's sieve (device context + buffers), created on first use.  A failure to
    create it (no library, no gfx950 device) is remembered: later queries go straight to the
    fallback without importing their terms or probing the device again, until the sieve is
    reconfigured (configure with sieve options, reset)."""
    s = getattr(_tls, "sieve", None)
    if s is None:
        failed = getattr(_tls, "sieve_failed", None)
        if failed is not None:
            # a fresh exception per query: re-raising one saved object would chain every
            # query's frames (and their constraints) onto its traceback
            raise SieveUnavailable(failed)
        from .sieve import Sieve

        try:
            s = _tls.sieve = Sieve(**_config["sieve_kwargs"])
        except Exception as e:
            _tls.sieve_failed = "%s: %s" % (type(e).__name__, e)
            log.warning("constraint sieve unavailable, every query goes to the fallback: %s", e)
            raise
    return s


def forget_witnesses() -> None:
    """Drop the sieve's parent-witness table (its keys are node ids of a term context the
    importer has just replaced)."""
    s = getattr(_tls, "sieve", None)
    if s is not None:
        s.witnesses.clear()


def close_sieve() -> None:
    s = getattr(_tls, "sieve", None)
    if s is not None:
        s.close()
        _tls.sieve = None
    _tls.sieve_failed = None


def _log_query(constraints, minimize, maximize) -> None:
    """support/model.py:44-55: one ``.smt2`` file per query, named by the hash of the query.
    This package's terms print through smtlib.to_smtlib; foreign (z3) terms through the
    configured ``log_writer``.  Never raises: a query that cannot be printed is skipped (the
    reference only logs what z3 can print, and a log must not change the answer)."""
    from . import smt

    try:
        if all(isinstance(c, smt.Bool) for c in constraints) and \
                all(isinstance(e, smt.BitVec) for e in tuple(minimize) + tuple(maximize)):
            from .smtlib import to_smtlib

            text = to_smtlib(constraints, minimize, maximize)
        elif _config["log_writer"] is not None:
            text = _config["log_writer"](constraints, minimize, maximize)
        else:
            log.debug("--solver-log: no writer for %s terms", type(constraints[0]).__name__)
            return
        Path(args.solver_log).mkdir(parents=True, exist_ok=True)
        key = tuple(list(constraints) + list(minimize) + list(maximize)
                    + [len(constraints), len(minimize), len(maximize)])
        with open(args.solver_log + "/%d.smt2" % abs(hash(key)), "w") as f:
            f.write(text)
    except Exception as e:  # noqa: BLE001 - logging is best effort
        log.debug("--solver-log write failed: %s", e)


def _terms(constraints):
    """(smt.Context, [Bool]) for the constraints: ours as they are, foreign ones imported."""
    from . import smt

    if all(isinstance(c, smt.Bool) for c in constraints):
        ctx = constraints[0].ctx if constraints else smt.context()
        if any(c.ctx is not ctx for c in constraints):
            raise ValueError("constraints from different term contexts")
        return ctx, list(constraints)
    conv = _config["to_terms"]
    if conv is None:
        raise TypeError("no importer for constraints of type %s"
                        % type(constraints[0]).__name__)
    return conv(constraints)


def sieve_model(constraints, timeout_ms: Optional[float] = None):
    """The sieve's answer for a feasibility query: a Model, or None (ask the fallback).
    ``timeout_ms`` is get_model's budget (support/model.py:26-31): the sieve's own rounds and the
    verifier both stop inside it."""
    from .model import Model

    stats = SolverStatistics()
    t0 = time.perf_counter()
    _tls.miss_key = None
    try:
        s = sieve()  # first: an unusable device skips the term import
        ctx, terms = _terms(constraints)
        key = tuple(t.node for t in terms)
        budget = None if timeout_ms is None else max(timeout_ms, 0.0) / 1000.0
        w = s.solve(ctx.b, [t.node for t in terms], key=key, budget_s=budget)
    except Exception as e:  # fail closed: any problem means "ask the fallback"
        from .lower import LoweringUnsupported
        from .native import Unsupported

        if isinstance(e, (LoweringUnsupported, Unsupported)):
            stats.sieve_unsupported += 1
        else:
            stats.sieve_errors += 1
            log.debug("sieve error: %s", e)
        return None
    if w is None:
        stats.sieve_misses += 1
        _tls.miss_key = key  # the fallback's model of this query is learnt (learn_from_fallback)
        _tls.miss_ctx = ctx
        return None
    conv = _config["to_terms"]  # reads reference terms for Model.eval / Model[decl]
    m = Model(s, ctx, w.schema, w.values, w.index,
              importer=conv if hasattr(conv, "term") else None)
    verify = _config["verify"]
    if verify is not None:
        left = None if timeout_ms is None else timeout_ms - 1000.0 * (time.perf_counter() - t0)
        try:
            ok = left is None or left > 0
            ok = ok and _verify(verify, constraints, m, left)
        except Exception as e:  # noqa: BLE001 - a failing verifier rejects
            log.debug("sieve witness verifier error: %s", e)
            ok = False
        if not ok:
            stats.sieve_rejected += 1
            return None
        if ok is not True:
            m = ok  # the verifier's own model (the reference's type)
    stats.sieve_hits += 1
    return m


@lru_cache(maxsize=2 ** 23)
def get_model(constraints, minimize=(), maximize=(), enforce_execution_time=True):
    """support/model.py:15-62 with the sieve in front of the solver (module docstring)."""
    timeout = args.solver_timeout
    if enforce_execution_time:
        timeout = min(timeout, time_handler.time_remaining() - 500)
        if timeout <= 0:
            raise UnsatError
    for constraint in constraints:
        if type(constraint) == bool and not constraint:
            raise UnsatError
    constraints = [c for c in constraints if type(c) != bool]
    stats = SolverStatistics()
    fallback = _config["fallback"]
    _tls.miss_key = None  # set by this call's sieve miss only
    if _config["enabled"] and not minimize and not maximize:
        t0 = time.perf_counter()
        m = sieve_model(constraints, timeout)
        if stats.enabled:
            stats.sieve_time += time.perf_counter() - t0
        if m is not None:
            if args.solver_log:
                _log_query(constraints, minimize, maximize)
            return m
    if args.solver_log and (fallback is None or not _config["fallback_logs"]):
        _log_query(constraints, minimize, maximize)
    if fallback is None:
        log.debug("sieve found no witness and no fallback solver is configured")
        raise UnsatError
    # the fallback (the reference's get_model) counts itself through stat_smt_query
    model = fallback(tuple(constraints), minimize, maximize, enforce_execution_time)
    learn_from_fallback(model)
    return model


def z3_column_reader(model, z3):
    """value_of(column) over a z3 model -- the reference's Model (laser/smt/model.py:12-59: its
    ``raw`` z3 ModelRefs) or a z3 ModelRef -- for Sieve.learn: a variable's value, an array cell
    ``Select(A, key)``, a function cell ``f(key)``, each evaluated with model completion; None
    for the else columns (any value completes a model) and for symbols the model does not
    declare.  ``value_of.value_at(column, index)`` reads a read column (``Select(A, i)``,
    ``f(i)``, keccak included) at its index term's value, which Sieve.learn computes."""
    models = list(getattr(model, "raw", None) or [model])
    decls = {}
    for zm in models:
        for d in zm.decls():
            decls.setdefault(d.name(), (zm, d))

    def at(col, key):
        hit = decls.get(col.symbol)
        if hit is None:
            return None
        zm, d = hit
        if col.kind == "var":
            v = zm.eval(d(), model_completion=True)
        elif col.kind in ("cell", "read"):
            v = zm.eval(z3.Select(d(), z3.BitVecVal(key, d.range().domain().size())),
                        model_completion=True)
        else:
            v = zm.eval(d(z3.BitVecVal(key, d.domain(0).size())), model_completion=True)
        return v.as_long() if z3.is_bv_value(v) else None

    def value_of(col):
        if col.kind not in ("var", "cell", "ufcell"):
            return None
        return at(col, col.key)

    def value_at(col, index):
        """A read column (an array's, a tabled function's or a keccak function's value at a
        symbolic index term) at that term's value ``index`` (Sieve.learn computes it)."""
        if col.kind not in ("read", "ufread", "kread"):
            return None
        return at(col, index)

    value_of.value_at = value_at
    return value_of


def learn_from_fallback(model) -> None:
    """The fallback's model of the query the sieve just missed becomes that query's witness in
    the sieve (Sieve.learn), so the query's children are generated around it.  Best effort: no
    z3, a model of another shape or any error leaves the sieve as it was."""
    key = getattr(_tls, "miss_key", None)
    _tls.miss_key = None
    s = getattr(_tls, "sieve", None)
    if key is None or s is None or model is None:
        return
    try:
        import z3

        reader = z3_column_reader(model, z3)
        s.learn(key, reader, ctx=getattr(_tls, "miss_ctx", None), value_at=reader.value_at)
    except Exception as e:  # noqa: BLE001 - learning never changes the answer
        log.debug("fallback model not learnt: %s", e)
