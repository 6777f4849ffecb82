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

from typing import TYPE_CHECKING, List, Optional, Sequence, Union

from .lower import Schema
from .tape import ARITY, BOOL, Op, TapeError

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
        self._memo: dict = {}      # (node, model_completion) -> value (eval_many)
        self._resident: dict = {}  # column tuple -> the witness row on the device

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
        got = self.table(name)
        km = self.schema.keccak.get(name)
        if km is not None:  # the stated pairs over its reads (keccak_reads: lower.py)
            tab = dict(got[0]) if got is not None else {}
            tab.update(km.pairs)
            return Interp(sorted(tab.items()), 0)
        if got is not None:
            return Interp(sorted(got[0].items()), got[1])
        return None

    def table(self, name: str):
        """({key: value}, else value) of array or tabled function `name` in this model, or None:
        its cells, then its reads -- each at its index term's value under the witness (one
        device batch), where no cell holds that key (lower.py: the read took the cell's branch
        there) -- over the else value (model.py:34-51 reads z3's FuncInterp the same way)."""
        from .lower import READ_KINDS

        sc = self.schema
        cells = sc.cells.get(name)
        if cells is None:
            cells = sc.uf_cells.get(name)
        cols = [c for c in sc.columns.values() if c.symbol == name]
        els = [c for c in cols if c.kind in ("else", "ufelse")]
        reads = sorted((c for c in cols if c.kind in READ_KINDS), key=lambda c: c.key)
        if cells is None and not els and not reads:
            return None
        cells = cells or {}
        else_v = self.values.get(els[0].name, 0) if els else 0
        tab = {k: self.values.get(cname, else_v) for k, cname in cells.items()}
        if reads:
            at = self._evaluate([c.key for c in reads], [], True)
            for c in reads:
                k = int(at[c.key])
                if k not in cells:
                    tab.setdefault(k, self.values.get(c.name, 0))
        return tab, else_v

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
        symbols read 0.  Values are memoised per term; see ``eval_many`` for the batching."""
        return self.eval_many([expression], model_completion)[0]

    def eval_many(self, expressions: Sequence[object], model_completion: bool = False) -> list:
        """The values of several terms: every term this model has not evaluated yet goes to the
        device in ONE batch (one compile, the witness row uploaded once per column set and kept,
        one ``mh_eval_values_many`` launch per register class).

        The reference reads models one term at a time in loops -- ``calldata.concrete`` asks
        ``eval(If(i < size, calldata[i], 0))`` for i = 0, 1, ... (calldata.py:234-245) -- so a
        lone term that reads an array at a constant index is evaluated together with the same
        term at the next ``SPECULATE`` indices (its constant index replaced; the terms are
        hash-consed, so the reference's next term imports to exactly that node and is then a
        memo hit).  A speculated term that cannot be evaluated is dropped silently."""
        mc = bool(model_completion)
        out: list = [None] * len(expressions)
        pending: "dict[int, list]" = {}
        for i, e in enumerate(expressions):
            node, _ = self._term(e)
            got = self._memo.get((node, mc))
            if got is not None:
                out[i] = e if got is _UNEVALUATED else got
            else:
                pending.setdefault(node, []).append(i)
        if pending:
            nodes = list(pending)
            extra = self._speculate(nodes[0]) if len(nodes) == 1 and SPECULATE else []
            vals = self._evaluate(nodes, extra, mc)
            for n, v in vals.items():
                self._memo[(n, mc)] = v
            for n, pos in pending.items():
                v = vals[n]
                for i in pos:
                    out[i] = expressions[i] if v is _UNEVALUATED else v
        return out

    def _evaluate(self, nodes: Sequence[int], extra: Sequence[int], mc: bool) -> dict:
        """{node: value or _UNEVALUATED} of `nodes` (requested: a lowering failure with model
        completion raises) and `extra` (speculated: failures are left out)."""
        from copy import deepcopy

        from .lower import Lowering, LoweringUnsupported, node_columns, var_names

        b = self.ctx.b
        schema = deepcopy(self.schema)
        L = Lowering(b, schema)
        res: dict = {}
        roots: "list[tuple[int, int]]" = []  # (node, lowered root)
        asked_set = set(nodes)
        for n in list(nodes) + [x for x in extra if x not in asked_set]:
            asked = n in asked_set
            try:
                roots.append((n, L.lower(n)))
            except LoweringUnsupported:
                if not asked:
                    continue
                if not mc:  # e.g. a function the model does not interpret
                    res[n] = _UNEVALUATED
                    continue
                raise
        names = var_names(b)
        cols = node_columns(b, [r for _, r in roots])
        todo: "list[tuple[int, int]]" = []
        for n, r in roots:
            if not mc and any(names[v] not in self.values and
                              schema.columns.get(names[v]) is not None and
                              schema.columns[names[v]].kind == "var" for v in cols[r]):
                if n in asked_set:
                    res[n] = _UNEVALUATED
                continue
            todo.append((n, r))
        if not todo:
            return res
        columns = list(schema.columns) or ["__ground__"]
        if columns == ["__ground__"]:
            b.var("__ground__", 1)
        flat: "list[int]" = []
        spans = []
        for n, r in todo:
            width = b.widths[n]
            if width == BOOL or width <= SLICE:
                spans.append((n, width, len(flat), 1))
                flat.append(r)
            else:
                # wider than the device's 256-bit operations: the lowered term rewritten as
                # terms of its 256-bit slices (Slicer), each evaluated on the device, low first
                sl = Slicer(b).slices(r)
                spans.append((n, width, len(flat), len(sl)))
                flat.extend(sl)
        vals = self.sieve.eval_terms(b, flat, columns, self.values, resident=self._resident)
        for n, width, at, k in spans:
            if width == BOOL:
                res[n] = bool(vals[at])
            elif k == 1:
                res[n] = BitVecValue(vals[at], width)
            else:
                res[n] = BitVecValue(sum(int(p) << (SLICE * i)
                                         for i, p in enumerate(vals[at:at + k])), width)
        return res

    def _speculate(self, node: int) -> "list[int]":
        """The same term at the next SPECULATE values of its one constant array index (none
        when the term reads no array at a constant index, reads several, or is large)."""
        b = self.ctx.b
        nodes = b.nodes
        idx, seen, stack = set(), set(), [node]
        while stack:
            x = stack.pop()
            if x in seen:
                continue
            seen.add(x)
            if len(seen) > SPECULATE_WALK:
                return []
            op, _, a, bb, c = nodes[x][:5]
            if op == Op.SELECT and nodes[bb][0] == Op.CONST:
                idx.add(bb)
            k = ARITY[Op(op)]
            if k:
                stack.extend((a, bb, c)[:k])
        if len(idx) != 1:
            return []
        c = idx.pop()
        v, w = b.const_value(c), b.widths[c]
        out = []
        for j in range(1, SPECULATE + 1):
            if v + j >> w:
                break
            out.append(_substitute(b, node, c, b.const(v + j, w)))
        return out


_UNEVALUATED = object()  # memo marker: returned as the expression itself (no interpretation)
SPECULATE = 127          # sibling terms evaluated with a lone array read at a constant index
SPECULATE_WALK = 4096    # ... only for terms of at most this many nodes


def _substitute(b, root: int, old: int, new: int) -> int:
    """`root` with node `old` replaced by `new` (same sort), rebuilt through the builder's
    hash-consing: the result is the node the same term written with `new` has."""
    from .tape import F_ARRAY

    nodes, flags = b.nodes, b.flags
    memo = {old: new}
    stack = [(root, False)]
    while stack:
        x, done = stack.pop()
        if x in memo:
            continue
        op, w, a, bb, c, i0, i1 = nodes[x]
        k = ARITY[Op(op)]
        kids = (a, bb, c)[:k]
        if not done:
            stack.append((x, True))
            stack.extend((y, False) for y in kids if y not in memo)
            continue
        new_kids = [memo.get(y, y) for y in kids]
        if new_kids == list(kids):
            memo[x] = x
            continue
        a2, b2, c2 = (new_kids + [a, bb, c][k:])[:3]
        memo[x] = b._add(Op(op), w, a2, b2, c2, i0, i1, flags=flags[x] & F_ARRAY)
    return memo[root]


def lower_query_value(b, node: int, frozen: Schema):
    """Lower one term (Bool or bit-vector) with a frozen schema; the schema copy gains plain
    variables the query did not mention (they read 0 under model completion)."""
    from copy import deepcopy

    from .lower import Lowering

    schema = deepcopy(frozen)
    L = Lowering(b, schema)
    return L.lower(node), schema


class Slicer:
    """A term wider than 256 bits as the list of its 256-bit slices (low first; the last one
    ``width % 256`` bits when that is not 0), each a term of at most 256 bits the device
    evaluates: concatenation, extraction, zero / sign extension, ITE and the bitwise ops split
    per slice; addition, subtraction and negation carry between slices through 256-bit
    compares.  Any other operator wider than 256 bits raises TapeError (Model.eval of such a
    term is not supported)."""

    def __init__(self, b):
        self.b = b
        self.memo = {}

    def _widths(self, w):
        return [min(SLICE, w - lo) for lo in range(0, w, SLICE)]

    def bits(self, sl, lo: int, hi: int) -> int:
        """A term of bits [lo, hi) (hi - lo <= 256) of the value whose slices are `sl`."""
        b = self.b
        parts = []  # high first, for CONCAT
        pos = lo
        while pos < hi:
            k = pos // SLICE
            top = min(hi, (k + 1) * SLICE)
            x = sl[k]
            a, z = pos - k * SLICE, top - k * SLICE  # bits [a, z) of slice k
            if a == 0 and z == b.width(x):
                parts.append(x)
            else:
                parts.append(b.op(Op.EXTRACT, x, imm0=z - 1, imm1=a))
            pos = top
        out = parts[0]
        for x in parts[1:]:
            out = b.op(Op.CONCAT, x, out)
        return out

    def _pack(self, pieces):
        """Slices of the concatenation of `pieces` [(term, width)] given low first."""
        b = self.b
        total = sum(w for _, w in pieces)
        # one list of <= 256-bit parts with their bit offsets, then regrouped into slices
        sl, offs = [], []
        pos = 0
        for t, w in pieces:
            for part, pw in zip(self.slices(t) if w > SLICE else [t], self._widths(w)):
                sl.append(part)
                offs.append((pos, pw))
                pos += pw
        out = []
        for lo in range(0, total, SLICE):
            hi = min(total, lo + SLICE)
            chunk = []
            for part, (o, pw) in zip(sl, offs):
                a, z = max(lo, o), min(hi, o + pw)
                if a < z:
                    chunk.append(part if (a, z) == (o, o + pw) else
                                 b.op(Op.EXTRACT, part, imm0=z - o - 1, imm1=a - o))
            acc = chunk[0]
            for x in chunk[1:]:
                acc = b.op(Op.CONCAT, x, acc)
            out.append(acc)
        return out

    def slices(self, n: int):
        got = self.memo.get(n)
        if got is not None:
            return got
        b = self.b
        w = b.width(n)
        if w <= SLICE:
            out = [n]
        else:
            op, _, a, bb, c, i0, i1 = b.nodes[n]
            op = Op(op)
            cv = b.const_value(n)
            if cv is not None:
                out = [b.const((cv >> lo) & ((1 << sw) - 1), sw)
                       for lo, sw in zip(range(0, w, SLICE), self._widths(w))]
            elif op == Op.CONCAT:  # a high, bb low
                out = self._pack([(bb, b.width(bb)), (a, b.width(a))])
            elif op == Op.ZEXT:
                out = self._pack([(a, b.width(a)), (b.const(0, i0), i0)] if i0 <= SLICE else
                                 [(a, b.width(a))] + [(b.const(0, sw), sw) for sw in
                                                      self._widths(i0)])
            elif op == Op.SEXT:
                wa = b.width(a)
                sign = b.op(Op.EQ, b.op(Op.EXTRACT, self.bits(self.slices(a), wa - 1, wa)
                                        if wa > SLICE else a, imm0=0, imm1=0)
                            if wa > SLICE else b.op(Op.EXTRACT, a, imm0=wa - 1, imm1=wa - 1),
                            b.const(1, 1))
                fill = [(b.op(Op.ITE, sign, b.const((1 << sw) - 1, sw), b.const(0, sw)), sw)
                        for sw in self._widths(i0)]
                out = self._pack([(a, wa)] + fill)
            elif op == Op.EXTRACT:
                src = self.slices(a)
                out = [self.bits(src, i1 + lo, i1 + lo + sw)
                       for lo, sw in zip(range(0, w, SLICE), self._widths(w))]
            elif op in (Op.BVAND, Op.BVOR, Op.BVXOR):
                out = [b.op(op, x, y) for x, y in zip(self.slices(a), self.slices(bb))]
            elif op == Op.BVNOT:
                out = [b.op(op, x) for x in self.slices(a)]
            elif op == Op.ITE:
                out = [b.op(Op.ITE, a, x, y) for x, y in zip(self.slices(bb), self.slices(c))]
            elif op in (Op.BVADD, Op.BVSUB, Op.BVNEG):
                xs = self.slices(a)
                ys = self.slices(bb) if op != Op.BVNEG else \
                    [b.const(0, sw) for sw in self._widths(w)]
                if op == Op.BVNEG:
                    xs, ys = ys, xs
                out = self._carry_chain(xs, ys, op == Op.BVADD)
            else:
                raise TapeError("Model.eval: %s wider than 256 bits (%d) is not supported"
                                % (op.name, w))
        self.memo[n] = out
        return out

    def _carry_chain(self, xs, ys, add: bool):
        """x + y (add) or x - y, slice by slice; the carry / borrow into slice k as a 0/1 term."""
        b = self.b
        out = []
        carry = None  # Bool node: a carry (borrow) into the current slice
        for x, y in zip(xs, ys):
            sw = b.width(x)
            one, zero = b.const(1, sw), b.const(0, sw)
            t = b.op(Op.BVADD if add else Op.BVSUB, x, y)
            c1 = b.op(Op.BVULT, t, x) if add else b.op(Op.BVULT, x, y)
            if carry is None:
                out.append(t)
                carry = c1
                continue
            cin = b.op(Op.ITE, carry, one, zero)
            s = b.op(Op.BVADD if add else Op.BVSUB, t, cin)
            c2 = b.op(Op.BVULT, s, t) if add else b.op(Op.BVULT, t, cin)
            out.append(s)
            carry = b.op(Op.OR, c1, c2)
        return out
