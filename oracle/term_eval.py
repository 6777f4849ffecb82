"""ORACLE (test infrastructure only — never imported by the product path).

Ground evaluation of a *term* (a tape that may still hold arrays, stores, selects and
uninterpreted-function applications) under an explicit z3-style model: what
``Model.eval(expr, model_completion=True)`` (mythril/laser/smt/model.py:45-59) computes for the
terms mythril.laser.smt builds with ``Array``/``K``/``Function`` (array.py:16-63,
function.py:7-25).

A model is
  vars:      {name: int}                                  missing names read 0 (completion)
  arrays:    {name: (table: {key: value}, else_value)}    missing arrays read 0 everywhere
  functions: {name: callable(int) -> int}                 missing functions return 0

Array values are (table, default) pairs: ``store`` copies the table, ``select`` looks the key up,
``K(v)`` is ({}, v) — the extensional semantics of the SMT-LIB array theory.  Bit-vector and
Bool nodes use oracle.smt_eval's rules (one restatement of each operator).
"""
from __future__ import annotations

from typing import Callable, Dict, Sequence, Tuple

try:
    from . import smt_eval as E
except ImportError:  # pragma: no cover
    import smt_eval as E  # type: ignore

# host-only op numbers (restated from mythril_amd/tape.py: ARRAY .. UF)
ARRAY, CONST_ARRAY, STORE, SELECT, UF = 80, 81, 82, 83, 84


def evaluate_term(nodes, consts: Sequence[int], var_names: Sequence[str],
                  array_names: Sequence[str], function_names: Sequence[str],
                  vars: Dict[str, int], arrays: Dict[str, Tuple[dict, int]],
                  functions: Dict[str, Callable[[int], int]]):
    assignment = [vars.get(n, 0) for n in var_names]

    def extra(op, nd, vals):
        w = int(nd["width"])
        a, b, c = int(nd["a"]), int(nd["b"]), int(nd["c"])
        i0 = int(nd["imm0"])
        if op == ARRAY:
            tab, dflt = arrays.get(array_names[i0], ({}, 0))
            return (dict(tab), dflt)
        if op == CONST_ARRAY:
            return ({}, vals[a])
        if op == STORE:
            tab, dflt = vals[a]
            tab = dict(tab)
            tab[vals[b]] = vals[c]
            return (tab, dflt)
        if op == SELECT:
            tab, dflt = vals[a]
            return tab.get(vals[b], dflt) & ((1 << w) - 1)
        if op == UF:
            f = functions.get(function_names[i0])
            return (f(vals[a]) if f is not None else 0) & ((1 << w) - 1)
        raise ValueError("unknown op %d" % op)

    return E.evaluate(nodes, consts, assignment, extra=extra)
