"""A z3 stand-in with an AST and a deciding solver (test infrastructure: z3 is absent here and on
the GPU box).

Its terms are this package's terms of a separate "reference-side" context, exposed through the
parts of z3's Python API the boundary code uses: ``ExprRef.get_id / children / decl / sort /
size / ==``, ``FuncDeclRef.kind / name / arity``, ``is_app / is_array / is_bool``,
``BitVecVal / BoolVal / K / Store``, and ``Solver`` / ``Optimize`` whose ``sexpr()`` prints one
term the way z3 does (tests/z3_style.py), so smtlib.Z3Importer reads them.

``Solver.check`` decides a query the way z3 does once every symbol is pinned: the assertions are
the constraints plus equalities ``symbol == value`` / ``array == Store(...K(...)...)`` /
``f(t) == value``; it records every uninterpreted symbol or application the constraints read
that no equality fixes (``free``) and answers ``unknown`` if there is one -- a check that would
be a search, not an evaluation -- else evaluates the constraints with the ORACLE
(oracle/term_eval.py) under the pinned interpretation: ``sat`` or ``unsat``.  ``model()`` is a
ModelRef of that interpretation.
"""
from __future__ import annotations

import types
from typing import Dict, List

from mythril_amd.tape import ARITY, BOOL, F_ARRAY, Op
from oracle.term_eval import evaluate_term
from tests.z3_style import z3_sexpr

Z3_OP_UNINTERPRETED = 2051
Z3_BOOL_SORT, Z3_BV_SORT, Z3_ARRAY_SORT = 1, 4, 5
_terms: Dict[tuple, "Term"] = {}


class Sort:
    def __init__(self, kind, size=0, dom=None, rng=None):
        self._kind, self._size, self._dom, self._rng = kind, size, dom, rng

    def kind(self):
        return self._kind

    def size(self):
        return self._size

    def domain(self):
        return self._dom

    def range(self):
        return self._rng


class FuncDecl:
    def __init__(self, name, kind, arity):
        self._name, self._kind, self._arity = name, kind, arity

    def name(self):
        return self._name

    def kind(self):
        return self._kind

    def arity(self):
        return self._arity

    def __eq__(self, other):
        return isinstance(other, FuncDecl) and other._name == self._name and \
            other._kind == self._kind

    def __hash__(self):
        return hash((self._name, self._kind))

    def __repr__(self):
        return self._name


class Val:
    """A numeral (BitVecVal / BoolVal): as_long(), size()."""

    def __init__(self, v, width):
        self.v, self.width = int(v), width

    def as_long(self):
        return self.v

    def size(self):
        return self.width

    def __eq__(self, other):
        return isinstance(other, Val) and (other.v, other.width) == (self.v, self.width)

    __hash__ = object.__hash__

    def __repr__(self):
        return "Val(%#x, %d)" % (self.v, self.width)


class ArrVal:
    """An array value built by K / Store: (table, else)."""

    def __init__(self, table, dflt):
        self.table, self.dflt = dict(table), dflt


class Eq:
    """``lhs == rhs`` with a term on the left: the boundary's pins (and any equality asserted)."""

    def __init__(self, lhs, rhs):
        self.lhs, self.rhs = lhs, rhs


class Term:
    """A z3 ExprRef stand-in over node `node` of the reference-side context `ctx`."""

    def __init__(self, ctx, node):
        self.ctx, self.node = ctx, node
        self.expr = types.SimpleNamespace(ctx=ctx, node=node)  # for z3_style.z3_sexpr

    @staticmethod
    def of(ctx, node) -> "Term":
        key = (id(ctx), node)
        t = _terms.get(key)
        if t is None:
            t = _terms[key] = Term(ctx, node)
        return t

    def _nd(self):
        return self.ctx.b.nodes[self.node]

    def get_id(self):
        return self.node

    def children(self) -> List["Term"]:
        op, _, a, bb, c = self._nd()[:5]
        return [Term.of(self.ctx, x) for x in (a, bb, c)[:ARITY[Op(op)]]]

    def decl(self) -> FuncDecl:
        b = self.ctx.b
        op, w, a, bb, c, i0, i1 = self._nd()
        op = Op(op)
        if op == Op.VAR:
            names = {v: k for k, v in b.var_index.items()}
            return FuncDecl(names[i0], Z3_OP_UNINTERPRETED, 0)
        if op == Op.ARRAY:
            return FuncDecl(b.symbols.array_names[i0], Z3_OP_UNINTERPRETED, 0)
        if op == Op.UF:
            return FuncDecl(b.symbols.function_names[i0], Z3_OP_UNINTERPRETED, 1)
        return FuncDecl(op.name, 256 + int(op), ARITY[op])

    def sort(self) -> Sort:
        b = self.ctx.b
        n = self.node
        if b.flags[n] & F_ARRAY:
            return Sort(Z3_ARRAY_SORT, 0, Sort(Z3_BV_SORT, b.nodes[n][6]),
                        Sort(Z3_BV_SORT, b.widths[n]))
        w = b.widths[n]
        return Sort(Z3_BOOL_SORT) if w == BOOL else Sort(Z3_BV_SORT, w)

    def size(self):
        return self.ctx.b.widths[self.node]

    def sexpr(self):
        return z3_sexpr(self.expr)

    def __eq__(self, other):
        return Eq(self, other)

    __hash__ = object.__hash__

    def __repr__(self):
        return "Term(%d)" % self.node


def make_z3():
    """A fresh stand-in module (installed with monkeypatch.setitem(sys.modules, "z3", ...))."""
    z3 = types.ModuleType("z3")
    z3.sat, z3.unsat, z3.unknown = "sat", "unsat", "unknown"
    z3.Z3_OP_UNINTERPRETED = Z3_OP_UNINTERPRETED
    z3.solvers = []
    z3.is_app = lambda t: isinstance(t, Term)
    z3.is_array = lambda t: isinstance(t, Term) and bool(t.ctx.b.flags[t.node] & F_ARRAY)
    z3.is_bool = lambda t: isinstance(t, Term) and t.ctx.b.widths[t.node] == BOOL
    z3.is_bv_value = lambda v: isinstance(v, Val) and v.width != BOOL
    z3.BitVecVal = lambda v, w: Val(v & ((1 << w) - 1), w)
    z3.BoolVal = lambda x: Val(1 if x else 0, BOOL)
    z3.BitVecSort = lambda w: Sort(Z3_BV_SORT, w)
    z3.K = lambda dom, v: ArrVal({}, v.v)
    z3.Store = lambda a, k, v: ArrVal({**a.table, k.v: v.v}, a.dflt)

    class ModelRef:
        def __init__(self, solver):
            self.s = solver

        def decls(self):
            s = self.s
            return ([FuncDecl(n, Z3_OP_UNINTERPRETED, 0) for n in s.vars] +
                    [FuncDecl(n, Z3_OP_UNINTERPRETED, 0) for n in s.arrays] +
                    [FuncDecl(n, Z3_OP_UNINTERPRETED, 1) for n in s.funcs])

        def __getitem__(self, d):
            name = d.name()
            if name in self.s.vars:
                return Val(self.s.vars[name], 0)
            if name in self.s.arrays:
                return self.s.arrays[name]
            return self.s.funcs.get(name)

        def eval(self, t, model_completion=False):
            v = self.s.evaluate(t)
            w = t.ctx.b.widths[t.node]
            return (v != 0) if w == BOOL else Val(v, w)

    class Solver:
        def __init__(self):
            self.params, self.assertions = {}, []
            self.free: List[str] = []
            self.vars, self.arrays, self.funcs = {}, {}, {}
            self.pins: List[Eq] = []
            z3.solvers.append(self)

        def set(self, key, value):
            self.params[key] = value

        def add(self, *cs):
            for c in cs:
                self.assertions.extend(c if isinstance(c, list) else [c])

        def sexpr(self):  # one term, printed as z3 prints it (the importer's use)
            (t,) = self.assertions
            return z3_sexpr(t.expr)

        def evaluate(self, t) -> int:
            b = t.ctx.b
            names = [n for n, _ in sorted(b.var_index.items(), key=lambda kv: kv[1])]
            arrays = {n: (a.table, a.dflt) for n, a in self.arrays.items()}
            funcs = {f: (lambda x, tab=tab: tab.get(x, 0)) for f, tab in self.funcs.items()}
            return evaluate_term(b.finish(t.node).nodes, b.pool.values, names,
                                 b.symbols.array_names, b.symbols.function_names, self.vars,
                                 arrays, funcs)

        def check(self):
            cons = [a for a in self.assertions if isinstance(a, Term)]
            self.pins = [a for a in self.assertions if isinstance(a, Eq)]
            if not cons:
                return z3.sat
            ctx = cons[0].ctx
            b = ctx.b
            app_pins = {}
            self.vars, self.arrays, self.funcs = {}, {}, {}
            for p in self.pins:
                t, v = p.lhs, p.rhs
                op = Op(b.nodes[t.node][0])
                if op == Op.VAR:
                    self.vars[t.decl().name()] = v.v
                elif op == Op.ARRAY:
                    self.arrays[t.decl().name()] = v
                elif op == Op.UF:
                    app_pins[t.node] = v.v
            # what the constraints read that no equality fixes
            free, seen, stack = [], set(), [c.node for c in cons]
            while stack:
                n = stack.pop()
                if n in seen:
                    continue
                seen.add(n)
                t = Term.of(ctx, n)
                op = Op(b.nodes[n][0])
                if op == Op.VAR and t.decl().name() not in self.vars:
                    free.append(t.decl().name())
                elif op == Op.ARRAY and t.decl().name() not in self.arrays:
                    free.append(t.decl().name())
                elif op == Op.UF and n not in app_pins:
                    free.append("%s(#%d)" % (t.decl().name(), n))
                stack.extend(c.node for c in t.children())
            self.free = sorted(set(free))
            if self.free:
                return z3.unknown
            # the functions at their pinned points, inner applications first (node ids are a
            # topological order of the DAG)
            for n in sorted(app_pins):
                t = Term.of(ctx, n)
                x = self.evaluate(t.children()[0])
                tab = self.funcs.setdefault(t.decl().name(), {})
                if tab.get(x, app_pins[n]) != app_pins[n]:
                    return z3.unsat  # two values for one point: not a function
                tab[x] = app_pins[n]
            return z3.sat if all(self.evaluate(c) for c in cons) else z3.unsat

        def model(self):
            return ModelRef(self)

    class Optimize(Solver):
        def __init__(self):
            super().__init__()
            self.objectives = []

        def minimize(self, t):
            self.objectives.append(t)

        def sexpr(self):
            assert not self.assertions and len(self.objectives) == 1
            return z3_sexpr(self.objectives[0].expr, head="minimize")

    z3.Solver, z3.Optimize = Solver, Optimize
    return z3


class Ref:
    """A reference laser/smt term (``.raw`` is the z3 term)."""

    def __init__(self, expr):
        self.raw = Term.of(expr.ctx, expr.node)
