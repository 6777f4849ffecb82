"""``Model`` for sieve witnesses (mirrors mythril/laser/smt/model.py:12-59).

A witness is one assignment row: a value per column of the query's schema (lower.py).  It
denotes a complete model — scalar symbols, array tables with an else-value, keccak functions as
concrete pairs plus the interval map — and ``eval`` evaluates any term under it ON THE DEVICE:
the term is lowered with the query's frozen schema (a constant key outside the table reads the
else-value, exactly what the model assigns it), compiled, and evaluated over the one witness row
(``mh_eval_values``, the parity path of the C-ABI, through ``Sieve.eval_terms``).

Under the plugin every term a reference caller holds is a z3 ``ExprRef`` (``x.raw``), and the
reference reads models as ``model.eval(x.raw, model_completion=True).as_long()``
(calldata.py:240-244, analysis/solver.py:174-176), ``model.eval(t.raw)`` (solver.py:141,
keccak_function_manager.py:113) and ``model[x.raw.decl()]`` (model_test.py:34).  Such a term is
imported through the front end's importer (smtlib.Z3Importer.term: z3's SMT-LIB text of the term,
read by the C++ session into the context the witness was found in) and evaluated the same way;
terms wider than 256 bits (512-bit keccak inputs, the 257-bit no-overflow sums) are evaluated as
256-bit slices.
"""
from __future__ import annotations

from typing import TYPE_CHECKING, List, Optional, Union

from .lower import Schema
from .tape import BOOL, Op

if TYPE_CHECKING:  # pragma: no cover
    from .sieve import Sieve
    from .smt import Context, Expression

SLICE = 256  # bits per device evaluation (mh_eval_values returns 8 limbs)


class BitVecValue(int):
    """An evaluated bit-vector: an int with z3's numeral accessors (``as_long``)."""

    def __new__(cls, value: int, size: int):
        obj = super().__new__(cls, value)
        obj._size = size
        return obj

    def as_long(self) -> int:
        return int(self)

    def size(self) -> int:
        return self._size

    def __repr__(self) -> str:
        return str(int(self))


class Decl:
    """A declaration the model interprets (z3 ``FuncDeclRef``): compares equal to another
    declaration, or a name, of the same symbol, so ``x.raw.decl() in model.decls()`` holds for a
    z3 declaration and for this package's (model_test.py:16-19)."""

    def __init__(self, name: str, kind: str):
        self._name = name
        self.kind = kind  # "var" | "array" | "function"

    def name(self) -> str:
        return self._name

    def arity(self) -> int:
        return 0 if self.kind == "var" else 1

    def __eq__(self, other) -> bool:
        return _decl_name(other) == self._name

    def __hash__(self) -> int:
        return hash(self._name)

    def __str__(self) -> str:
        return self._name

    __repr__ = __str__


class Interp:
    """The interpretation of an array or function symbol (z3 ``FuncInterp``): ``as_list()`` is
    ``[[key, value], ..., else_value]`` like z3's."""

    def __init__(self, entries, else_value: int):
        self.entries = list(entries)
        self.else_value = else_value

    def as_list(self) -> list:
        return [[k, v] for k, v in self.entries] + [self.else_value]

    def num_entries(self) -> int:
        return len(self.entries)

    def else_value_(self) -> int:
        return self.else_value


def _decl_name(d) -> Optional[str]:
    if isinstance(d, str):
        return d
    name = getattr(d, "name", None)
    if callable(name):
        return str(name())
    return None


class Model:
    """One witness of one query (the reference wraps a list of z3 models; a sieve model is one
    complete assignment, so ``raw`` holds one entry).  ``importer`` turns reference (z3) terms
    into terms of ``ctx`` (smtlib.Z3Importer; the front end passes its configured one)."""

    def __init__(self, sieve: "Sieve", ctx: "Context", schema: Schema, values: dict,
                 index: int = 0, importer=None):
        self.sieve = sieve
        self.ctx = ctx
        self.schema = schema
        self.values = dict(values)
        self.index = index
        self.importer = importer
        self._own_importer = None
        self.raw = [self]

    # -- declarations -------------------------------------------------------------------------
    def decls(self) -> List[Decl]:
        """The symbols this model interprets (model.py:19-25): scalar symbols, arrays, keccak
        functions."""
        out: List[Decl] = []
        seen = set()
        for c in self.schema.columns.values():
            if c.symbol in seen or c.symbol == "__ground__":
                continue
            seen.add(c.symbol)
            out.append(Decl(c.symbol, "var" if c.kind == "var" else
                            "function" if c.kind.startswith("uf") else "array"))
        for f in self.schema.keccak:
            if f not in seen:
                seen.add(f)
                out.append(Decl(f, "function"))
        return out

    def __getitem__(self, item):
        """model.py:34-51.  By index: the item-th declaration; by declaration (this package's,
        a z3 ``FuncDeclRef``, or a name): a scalar symbol's value (``BitVecValue``, a bool for a
        Bool symbol), an array's or function's ``Interp``; None when the model has no
        interpretation of it."""
        if isinstance(item, int):
            return self.decls()[item]
        name = _decl_name(item)
        if name is None:
            return None
        c = self.schema.columns.get(name)
        if c is not None and c.kind == "var":
            if name not in self.values:
                return None
            if c.width == 1 and self._bool_symbol(name):
                return bool(self.values[name])
            return BitVecValue(self.values[name], c.width)
        cells = self.schema.cells.get(name) or self.schema.uf_cells.get(name)
        els = [col for col in self.schema.columns.values()
               if col.symbol == name and col.kind in ("else", "ufelse")]
        if cells is not None or els:
            cells = cells or {}
            else_v = self.values.get(els[0].name, 0) if els else 0
            return Interp(sorted((k, self.values.get(cname, else_v))
                                 for k, cname in cells.items()), else_v)
        km = self.schema.keccak.get(name)
        if km is not None:
            return Interp(sorted(km.pairs.items()), 0)
        return None

    def _bool_symbol(self, name: str) -> bool:
        """A 1-bit column made by BoolSym (a Bool symbol: z3 gives True / False)."""
        return name in self.ctx.b.symbols.bool_vars

    # -- evaluation ---------------------------------------------------------------------------
    def _term(self, expression):
        """(node, foreign?) of `expression` in this model's context."""
        from . import smt

        if isinstance(expression, smt.Expression):
            if expression.ctx is not self.ctx:
                raise ValueError("the term belongs to another term context than the model")
            return expression.node, False
        imp = self.importer
        if imp is None or not hasattr(imp, "term"):
            raise TypeError("Model.eval of a %s term needs an importer (smtlib.Z3Importer)"
                            % type(expression).__name__)
        if getattr(imp, "ctx", None) is not self.ctx:
            # the importer has started a new context since this witness (Z3Importer.reset
            # between queries): read the term into the model's own context
            if self._own_importer is None:
                from .smtlib import Z3Importer

                self._own_importer = Z3Importer(self.ctx, term_sexpr_of=imp.term_sexpr_of)
            imp = self._own_importer
        return imp.term(expression).node, True

    def eval(self, expression: Union["Expression", object], model_completion: bool = False):
        """model.py:45-59: the value of `expression` (this package's term or a reference z3
        term) under this model.  Without model_completion, a term reading a symbol the model
        does not interpret is returned unevaluated, as given (z3 behaviour); with it, such
        symbols read 0."""
        from .lower import LoweringUnsupported

        b = self.ctx.b
        node, _ = self._term(expression)
        try:
            root, schema = lower_query_value(b, node, self.schema)
        except LoweringUnsupported:
            if not model_completion:  # e.g. a function the model does not interpret
                return expression
            raise
        fresh = [n for n, c in schema.columns.items()
                 if n not in self.values and c.kind == "var"]
        if fresh and not model_completion:
            return expression
        width = b.widths[node]
        columns = list(schema.columns) or ["__ground__"]
        if columns == ["__ground__"]:
            b.var("__ground__", 1)
        if width == BOOL or width <= SLICE:
            v = self.sieve.eval_terms(b, [root], columns, self.values)[0]
            return bool(v) if width == BOOL else BitVecValue(v, width)
        # wider than one device evaluation: 256-bit slices of the lowered term, low first
        roots = [b.op(Op.EXTRACT, root, imm0=min(lo + SLICE, width) - 1, imm1=lo)
                 for lo in range(0, width, SLICE)]
        parts = self.sieve.eval_terms(b, roots, columns, self.values)
        return BitVecValue(sum(int(p) << (SLICE * i) for i, p in enumerate(parts)), width)


def lower_query_value(b, node: int, frozen: Schema):
    """Lower one term (Bool or bit-vector) with a frozen schema; the schema copy gains plain
    variables the query did not mention (they read 0 under model completion)."""
    from copy import deepcopy

    from .lower import Lowering

    schema = deepcopy(frozen)
    L = Lowering(b, schema)
    return L.lower(node), schema
