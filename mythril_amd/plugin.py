"""The sieve as a Mythril plugin (the drop-in boundary of SURVEY.md §8b).

``SievePluginBuilder`` is a ``MythrilLaserPlugin`` (mythril/plugin/interface.py:39-45): a
``MythrilPlugin`` and a LASER ``PluginBuilder`` (laser/plugin/builder.py:7-21) at once, found
through the setuptools entry point group ``mythril.plugins`` (plugin/discovery.py:17-21,57).  Its
``__call__`` returns a ``SievePlugin`` whose ``initialize(symbolic_vm)``
(laser/plugin/interface.py:4-23) registers two LASER hooks (svm.py:578-643):

* ``start_sym_exec``: configure the front end (fallback = the reference's own z3 ``get_model``,
  verifier = z3 re-check of the witness, importer = SMT-LIB import of z3 terms) and rebind
  ``get_model`` at the three import sites of SURVEY.md §3.2 —
  ``mythril.support.model``, ``mythril.analysis.solver`` (analysis/solver.py:6) and
  ``mythril.laser.ethereum.state.constraints`` (constraints.py:5);
* ``stop_sym_exec``: restore the three names and release the device.

The plugin never raises ``PluginSkipState`` / ``PluginSkipWorldState`` (laser/plugin/signals.py):
it changes how a feasibility query is answered, never which states exist.  Without the reference
importable (this container: no z3), the same classes are defined over minimal stand-ins of the
two base classes, so the hook logic is testable; ``install`` / ``uninstall`` then act on
whatever modules are passed.
"""
from __future__ import annotations

import importlib
import logging
from typing import Dict, List, Optional, Sequence

from . import frontend

log = logging.getLogger(__name__)

try:
    from mythril.laser.plugin.interface import LaserPlugin  # type: ignore
    from mythril.plugin.interface import MythrilLaserPlugin  # type: ignore
except Exception:  # standalone: stand-ins with the reference's attributes
    class LaserPlugin:  # type: ignore[no-redef]
        """laser/plugin/interface.py:4-23."""

        def initialize(self, symbolic_vm) -> None:
            raise NotImplementedError

    class MythrilLaserPlugin:  # type: ignore[no-redef]
        """plugin/interface.py:6-45 (MythrilPlugin + PluginBuilder)."""

        author = "Default Author"
        name = "Plugin Name"
        plugin_license = "All rights reserved."
        plugin_type = "Mythril Plugin"
        plugin_version = "0.0.1 "
        plugin_description = "This is an example plugin description"
        plugin_name = "Default Plugin Name"

        def __init__(self, **kwargs):
            self.enabled = True

        def __repr__(self):
            return "%s - %s - %s" % (type(self).__name__, self.plugin_version, self.author)

IMPORT_SITES = (
    "mythril.support.model",
    "mythril.analysis.solver",
    "mythril.laser.ethereum.state.constraints",
)


class Installation:
    """Rebinds ``get_model`` in a set of modules and remembers the originals."""

    def __init__(self):
        self.saved: Dict[int, tuple] = {}  # id(module) -> (module, original get_model)

    def install(self, modules: Sequence[object], replacement) -> None:
        for m in modules:
            if id(m) not in self.saved and hasattr(m, "get_model"):
                self.saved[id(m)] = (m, getattr(m, "get_model"))
                setattr(m, "get_model", replacement)

    def uninstall(self) -> None:
        for m, orig in self.saved.values():
            setattr(m, "get_model", orig)
        self.saved.clear()

    @property
    def original(self):
        """The first saved original (the reference's lru-cached z3 get_model)."""
        return next(iter(self.saved.values()), (None, None))[1]


def _reference_modules() -> List[object]:
    out = []
    for name in IMPORT_SITES:
        try:
            out.append(importlib.import_module(name))
        except Exception:
            pass
    return out


def z3_log_writer(constraints, minimize, maximize) -> str:
    """``--solver-log`` text of reference (z3-backed) terms exactly as support/model.py:37-55
    writes it: an ``Optimize`` with the constraints and objectives, printed by ``sexpr()``."""
    import z3

    s = z3.Optimize()
    for c in constraints:
        s.add(getattr(c, "raw", c))
    for e in minimize:
        s.minimize(getattr(e, "raw", e))
    for e in maximize:
        s.maximize(getattr(e, "raw", e))
    return s.sexpr()


def witness_pins(raws, model, z3) -> list:
    """Equalities that fix every uninterpreted symbol the query's z3 terms read to the sieve
    witness's interpretation, so that z3's check of the query under them is an evaluation, not
    a search ("witness as equalities, fully determined"):

    * a scalar symbol (bit-vector or Bool constant): its column's value -- a symbol the witness
      has no column for is one the lowered query does not read, and gets 0 (model completion);
    * an array symbol: ``A == Store(...Store(K(dom, else), k1, v1)..., kn, vn)``, the z3 form of
      the witness's table (its cells, its reads at their indices' values and its else value,
      lower.py; model.Model.table);
    * every application of an uninterpreted function -- keccak256_N, its inverse keccak256_N-1,
      any other ``Function`` -- at the argument it has in the query: ``f(t) == v``, v the
      witness's value of that application (``Model.eval_many``: one device batch for all).

    ``raws`` are z3 ``ExprRef``s.  Walks the DAG once by AST id."""
    scalars, arrays, apps = {}, {}, {}
    seen, stack = set(), list(raws)
    while stack:
        t = stack.pop()
        i = t.get_id()
        if i in seen:
            continue
        seen.add(i)
        if not z3.is_app(t):
            continue
        d = t.decl()
        if d.kind() == z3.Z3_OP_UNINTERPRETED:
            if d.arity() == 0:
                (arrays if z3.is_array(t) else scalars)[d.name()] = t
            else:
                apps[i] = t
        stack.extend(t.children())
    pins = []
    cols = model.schema.columns
    for name, t in sorted(scalars.items()):
        col = cols.get(name)
        v = model.values.get(name, 0) if col is not None and col.kind == "var" else 0
        pins.append(t == (z3.BoolVal(bool(v)) if z3.is_bool(t) else z3.BitVecVal(v, t.size())))
    for name, t in sorted(arrays.items()):
        srt = t.sort()
        dom, rng = srt.domain(), srt.range()
        got = model.table(name)
        tab, else_v = got if got is not None else ({}, 0)
        a = z3.K(dom, z3.BitVecVal(else_v, rng.size()))
        for key, v in sorted(tab.items()):
            a = z3.Store(a, z3.BitVecVal(key, dom.size()), z3.BitVecVal(v, rng.size()))
        pins.append(t == a)
    if apps:
        ordered = [apps[i] for i in sorted(apps)]
        for t, v in zip(ordered, model.eval_many(ordered, model_completion=True)):
            pins.append(t == (z3.BoolVal(bool(v)) if z3.is_bool(t)
                              else z3.BitVecVal(int(v), t.size())))
    return pins


def z3_verifier(constraints, model, timeout_ms=None):
    """Re-verify a sieve witness with z3 and return the reference's model.

    The constraints plus ``witness_pins`` (every scalar, array and function application fixed)
    must be SAT; the result is then what the reference's get_model returns,
    ``mythril.laser.smt.Model([solver.model()])`` (support/model.py:57-59, laser/smt/model.py:13-18;
    its mirror ``support.RefModel`` when the reference is not importable).  None rejects the
    witness: unsat, or ``unknown`` -- the check runs under get_model's own budget
    (``timeout_ms`` = what is left of ``min(args.solver_timeout, time_remaining - 500)``,
    support/model.py:26-31) -- and the query goes to the fallback unchanged."""
    import z3

    from .support import RefModel, args

    s = z3.Solver()
    budget = args.solver_timeout if timeout_ms is None else min(args.solver_timeout, timeout_ms)
    if budget <= 0:
        return None
    s.set("timeout", max(1, int(budget)))
    raws = [getattr(c, "raw", c) for c in constraints]
    s.add(raws)
    s.add(witness_pins(raws, model, z3))
    if s.check() != z3.sat:
        return None
    return RefModel([s.model()])


class SievePlugin(LaserPlugin):
    """LaserPlugin: installs the sieve front end for one symbolic execution."""

    def __init__(self, modules: Optional[Sequence[object]] = None, **sieve_kwargs):
        self.modules = modules
        self.sieve_kwargs = sieve_kwargs
        self.installation = Installation()

    def initialize(self, symbolic_vm) -> None:
        symbolic_vm.register_laser_hooks("start_sym_exec", self.start)
        symbolic_vm.register_laser_hooks("stop_sym_exec", self.stop)

    def start(self) -> None:
        modules = self.modules if self.modules is not None else _reference_modules()
        self.installation.install(modules, frontend.get_model)
        original = self.installation.original
        kwargs = dict(self.sieve_kwargs)
        conf = {}
        if original is not None:
            # the reference's get_model, unwrapped from its lru_cache (the front end has its
            # own); it writes its own --solver-log file and counts itself in SolverStatistics
            conf["fallback"] = getattr(original, "__wrapped__", original)
            conf["fallback_logs"] = True
        try:
            import z3  # noqa: F401

            from .smtlib import Z3Importer

            conf["verify"] = z3_verifier
            conf["log_writer"] = z3_log_writer
            conf["to_terms"] = Z3Importer(on_reset=frontend.forget_witnesses)
        except Exception:
            pass
        frontend.configure(**conf, **kwargs)
        log.info("constraint sieve installed at %d import sites", len(self.installation.saved))

    def stop(self) -> None:
        self.installation.uninstall()
        from .support import SolverStatistics

        s = SolverStatistics()
        log.info("constraint sieve: %d hits, %d misses, %d unsupported, %d errors, "
                 "%d rejected", s.sieve_hits, s.sieve_misses, s.sieve_unsupported,
                 s.sieve_errors, s.sieve_rejected)
        frontend.reset()


class SievePluginBuilder(MythrilLaserPlugin):
    """Entry point ``mythril.plugins``: constraint-sieve = mythril_amd.plugin:SievePluginBuilder.
    ``plugin_name`` is unique (not the ``dependency-pruner`` name the instruction profiler
    already takes, laser/plugin/plugins/instruction_profiler.py:35)."""

    name = "constraint-sieve"
    plugin_name = "constraint-sieve"
    author = "mythril_amd"
    plugin_license = "MIT"
    plugin_type = "Laser Plugin"
    plugin_version = "0.1.0"
    plugin_description = "MI355X constraint sieve: feasibility witnesses before z3"
    # the reference's CLI loads only default-enabled entry-point plugins
    # (plugin/loader.py:73-80, cli.py:39), so a drop-in must be default-enabled; the
    # environment variable MYTHRIL_AMD_SIEVE=0 turns it off without uninstalling
    plugin_default_enabled = True

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self.enabled = enabled_by_env()

    def __call__(self, *args, **kwargs) -> SievePlugin:
        return SievePlugin(**kwargs)


def enabled_by_env() -> bool:
    import os

    return os.environ.get("MYTHRIL_AMD_SIEVE", "1").strip().lower() not in ("0", "off", "false",
                                                                            "no")
