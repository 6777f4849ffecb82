"""``Model`` for sieve witnesses (mirrors mythril/laser/smt/model.py:12-59).

A witness is one assignment row: a value per column of the query's schema (lower.py).  It
denotes a complete model — scalar symbols, array tables with an else-value, keccak functions as
concrete pairs plus the interval map — and ``eval`` evaluates any term under it ON THE DEVICE:
the term is lowered with the query's frozen schema (a constant key outside the table reads the
else-value, exactly what the model assigns it), compiled, and evaluated over the one witness row
(``mh_eval_values``, the parity path of the C-ABI, through ``Sieve.eval_terms``).
"""
from __future__ import annotations

from typing import TYPE_CHECKING, List, Optional, Union

from .lower import Schema
from .tape import BOOL, TapeError

if TYPE_CHECKING:  # pragma: no cover
    from .sieve import Sieve
    from .smt import Context, Expression


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


class Model:
    """One witness of one query (the reference wraps a list of z3 models; a sieve model is one
    complete assignment, so ``raw`` holds one entry)."""

    def __init__(self, sieve: "Sieve", ctx: "Context", schema: Schema, values: dict,
                 index: int = 0):
        self.sieve = sieve
        self.ctx = ctx
        self.schema = schema
        self.values = dict(values)
        self.index = index
        self.raw = [self]

    def decls(self) -> List[str]:
        """The symbols this model interprets (model.py:27-32)."""
        out = []
        for c in self.schema.columns.values():
            if c.symbol not in out:
                out.append(c.symbol)
        out += [f for f in self.schema.keccak if f not in out]
        return out

    def __getitem__(self, item: Union[int, str]):
        """By index: the item-th declaration; by name: the value of a scalar symbol."""
        if isinstance(item, int):
            return self.decls()[item]
        c = self.schema.columns.get(item)
        if c is None or c.kind != "var":
            return None
        return BitVecValue(self.values[item], c.width)

    def eval(self, expression: "Expression", model_completion: bool = False):
        """model.py:45-59: the value of `expression` under this model.  Without
        model_completion, a term reading a symbol the model does not interpret is returned
        unevaluated (z3 behaviour); with it, such symbols read 0."""
        b = self.ctx.b
        node = expression.node
        root, schema = lower_query_value(b, node, self.schema)
        fresh = [n for n, c in schema.columns.items()
                 if n not in self.values and c.kind == "var"]
        if fresh and not model_completion:
            return expression
        width = b.widths[node]
        if width > 256:
            raise TapeError("Model.eval of a %d-bit term (the parity path returns 256 bits)"
                            % width)
        columns = list(schema.columns) or ["__ground__"]
        if columns == ["__ground__"]:
            b.var("__ground__", 1)
        v = self.sieve.eval_terms(b, [root], columns, self.values)[0]
        if width == BOOL:
            return bool(v)
        return BitVecValue(v, width)


def lower_query_value(b, node: int, frozen: Schema):
    """Lower one term (Bool or bit-vector) with a frozen schema; the schema copy gains plain
    variables the query did not mention (they read 0 under model completion)."""
    from copy import deepcopy

    from .lower import Lowering

    schema = deepcopy(frozen)
    L = Lowering(b, schema)
    return L.lower(node), schema
