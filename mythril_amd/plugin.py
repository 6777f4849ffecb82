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


def z3_verifier(constraints, model, timeout_ms=None) -> bool:
    """Re-verify a sieve witness with z3: the constraints plus the witness as equalities on every
    scalar column must be SAT.  Runs only where z3 is importable.

    The check runs under get_model's own budget (``timeout_ms`` = what is left of
    ``min(args.solver_timeout, time_remaining - 500)``, support/model.py:26-31): array else-values
    and keccak / UF interpretations stay free, so the check is a real solver call, and ``unknown``
    (timeout) counts as a rejection — the query then goes to the fallback unchanged."""
    import z3  # noqa: F401

    from .support import args

    s = z3.Solver()
    budget = args.solver_timeout if timeout_ms is None else min(args.solver_timeout, timeout_ms)
    if budget <= 0:
        return False
    s.set("timeout", max(1, int(budget)))
    s.add([getattr(c, "raw", c) for c in constraints])
    arrays = model.ctx.b.symbols.arrays
    for col in model.schema.columns.values():
        v = model.values[col.name]
        if col.kind == "var" and col.symbol != "__ground__":
            s.add(z3.BitVec(col.symbol, col.width) == v)
        elif col.kind == "cell" and col.symbol in arrays:
            _, dom, rng = arrays[col.symbol]
            a = z3.Array(col.symbol, z3.BitVecSort(dom), z3.BitVecSort(rng))
            s.add(z3.Select(a, z3.BitVecVal(col.key, dom)) == v)
    return s.check() == z3.sat


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
