"""Lowering of arrays and uninterpreted functions into per-candidate tables.

LASER's path conditions read free arrays (``{tx}_calldata``, ``Storage``, ``balance``:
mythril/laser/ethereum/state/calldata.py:207-232, account.py:18-82, world_state.py:33-34) and
apply keccak uninterpreted functions (mythril/laser/ethereum/keccak_function_manager.py:59-149).
The device evaluates bit-vector terms only, so a query is lowered, once per ``get_model`` call,
into a term over scalar *columns* whose every assignment denotes one complete z3-style model:

* a free array ``A`` becomes a finite map over the constant keys the query reads (one *cell*
  column per key) plus one *read* column per symbolic index term the query reads it at
  (Ackermann's reduction, round 6): ``select(A, c)`` for a harvested constant ``c`` is cell
  ``A[c]``; ``select(A, i)`` for a symbolic ``i`` is ``ite(i == c1, A[c1], ... ite(i == ck, A[ck],
  A[@i]))``, and the query gains, after the constraint that first reads ``A[@j]``, one conjunct
  ``Or(Not(i == j), A[@i] == A[@j])`` per earlier read ``A[@i]`` (congruence), so two reads at
  unequal indices may differ.  A satisfying assignment is a model of the original query: ``A`` is
  ``Store(...Store(K(else), c1, v1)..., i_val, A[@i]_val ...)`` (the reads at their indices'
  values, where no cell is); ``store`` chains become ``ite`` over their keys and ``K(v)`` becomes
  ``v`` (array.py:16-63).  An index that lowers to a constant the harvest did not see
  (``select(A, select(K(7), i))``) is a read of its own, kept apart like any two reads.  A
  constant key outside the table in ``Model.eval`` of a term the query did not state reads the
  reads at equal indices, else the array's *else* value (0: no lowered query reads it).
* a keccak function ``keccak256_N`` becomes ``ite(x == c_i, k_i, H(x))`` over the concrete pairs
  ``keccak256_N(c_i) == k_i`` the query states (keccak_function_manager.py:92-97,145-148), with
  ``H(x) = base + ((keccak256(x) >> 139) << 6)``: a function of the argument (so congruence
  holds), injective up to keccak collisions in 117 bits (so the inverse condition
  ``keccak256_N-1(keccak256_N(x)) == x`` holds, lowered to ``x``), a multiple of 64, and inside
  ``[base, base + 2^123)``, where ``base`` is the greatest lower bound the query states on the
  function's values (``ULE(lo, f(x))`` of the manager's condition, ``UGT(f(x), c)``, ...),
  rounded up to a multiple of 64 — the interval of ``_create_condition`` (:121-149) is
  ``PART = (2^256-1) // 10^40 > 2^123 + 64`` wide, so the interval and ``mod 64`` conditions hold
  by construction.  The hash runs on the device's Keccak-f[1600].  The second-chance lowering
  (``keccak_reads``; Sieve.solve after a miss whose unsolved groups read H) gives every
  application at an argument no stated pair has a *kread* column instead of H, kept a function
  (congruence) and injective (``Or(i == j, Not(f[@i] == f[@j]))`` and ``Or(i == c, Not(f[@i] ==
  k))`` per stated pair): a path that pins a keccak value elsewhere than H has rows then.
* any other uninterpreted function is tabled like an array (cells over constant arguments, a
  read column per symbolic argument term with the same congruence conjuncts, function.py:7-25).

Anything else array- or function-sorted (array equality, ``ite`` over arrays, an inverse applied
to something other than its forward function) raises ``LoweringUnsupported``: the query goes to
z3 unchanged.
"""
from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

from .tape import ARITY, BOOL, F_ARRAY, F_HOST, Op, TapeBuilder, TapeError

def keccak_base(lower_bound: int) -> int:
    """The interval base of a keccak function's values: its greatest harvested lower bound,
    rounded up to a multiple of 64 (mod 2^256)."""
    return ((lower_bound + 63) & ~63) & ((1 << 256) - 1)


KECCAK_SHIFT = 139   # keep 117 bits of the hash ...
KECCAK_ALIGN = 6     # ... as multiples of 64: H - base < 2^123 < PART
ORDERED = {Op.BVULT, Op.BVULE, Op.BVUGT, Op.BVUGE, Op.BVSLT, Op.BVSLE, Op.BVSGT, Op.BVSGE}


class LoweringUnsupported(TapeError):
    """The query uses an array/function construct the sieve does not model: ask z3."""


@dataclass
class Column:
    """One scalar column of the candidate assignments of a query."""

    name: str             # VAR name in the tape set
    width: int
    kind: str             # "var" | "cell" | "else" | "ufcell" | "ufelse" | "read" | "ufread" |
                          # "kread"
    symbol: str           # variable / array / function name
    key: Optional[int] = None  # cells: the constant key; reads: the index term's node


READ_KINDS = ("read", "ufread", "kread")


def read_name(sym: str, index_node: int) -> str:
    """The column of the value `sym` (a free array or a tabled function) has at the symbolic
    index term `index_node` (the term as the query states it, before lowering)."""
    return "%s[@%d]" % (sym, index_node)


@dataclass
class KeccakMap:
    base: int                                            # aligned lower bound of the interval
    pairs: Dict[int, int] = field(default_factory=dict)  # concrete argument -> hash


@dataclass
class Schema:
    """What one query's columns mean: enough to rebuild a model from a witness row."""

    cells: Dict[str, Dict[int, str]] = field(default_factory=dict)   # array -> key -> column
    uf_cells: Dict[str, Dict[int, str]] = field(default_factory=dict)
    keccak: Dict[str, KeccakMap] = field(default_factory=dict)
    columns: Dict[str, Column] = field(default_factory=dict)         # column name -> Column
    # keccak applications as read columns (the second-chance lowering, Lowering keccak_reads)
    keccak_reads: bool = False


@dataclass
class Harvest:
    """What pass 1 reads off some constraints: constant keys per array / function, concrete
    keccak pairs and the greatest lower bound on each keccak function.  One per constraint, memoised on the builder, so a
    query that extends its parent (svm.py:257-262) only walks its new constraint."""

    cells: Dict[str, set] = field(default_factory=dict)
    uf_cells: Dict[str, set] = field(default_factory=dict)
    keccak: Dict[str, Dict[int, int]] = field(default_factory=dict)
    bounds: Dict[str, int] = field(default_factory=dict)

    def merge(self, o: "Harvest") -> None:
        for name, keys in o.cells.items():
            self.cells.setdefault(name, set()).update(keys)
        for name, keys in o.uf_cells.items():
            self.uf_cells.setdefault(name, set()).update(keys)
        for f, pairs in o.keccak.items():
            self.keccak.setdefault(f, {}).update(pairs)
        for f, v in o.bounds.items():
            self.bounds[f] = max(v, self.bounds.get(f, v))

    def fingerprint(self) -> tuple:
        """Everything the rewrite of pass 2 depends on: equal fingerprints lower every term to the
        same column-only term."""
        return (tuple(sorted((n, tuple(sorted(k))) for n, k in self.cells.items())),
                tuple(sorted((n, tuple(sorted(k))) for n, k in self.uf_cells.items())),
                tuple(sorted((f, tuple(sorted(p.items())), keccak_base(self.bounds.get(f, 0)))
                             for f, p in self.keccak.items())))


MEMO_LIMIT = 1 << 21  # entries of a builder-level memo before it is dropped (a long run's bound)


def _memo(b: TapeBuilder, name: str) -> dict:
    """A memo on the builder (its nodes are immutable and hash-consed), started afresh once it
    holds MEMO_LIMIT entries."""
    m = b.__dict__.get(name)
    if m is None or len(m) > MEMO_LIMIT:
        m = b.__dict__[name] = {}
    return m


def node_columns(b: TapeBuilder, roots: Iterable[int]) -> Dict[int, frozenset]:
    """The VAR indices under each of `roots` (memoised per root on the builder: nodes are
    immutable and hash-consed).  A walk stops at any node already in the memo, so a LASER query
    that extends its parent's (svm.py:257-262) only visits its new conjunct; the nodes between
    are not given sets of their own (a set per node cost more than the walk)."""
    cols: Dict[int, frozenset] = _memo(b, "_node_cols")
    nodes, var = b.nodes, Op.VAR
    for r in roots:
        if r in cols:
            continue
        vs, seen, st = set(), set(), [r]
        while st:
            n = st.pop()
            if n in seen:
                continue
            seen.add(n)
            got = cols.get(n)
            if got is not None:
                vs |= got
                continue
            op, _, a, bb, c, i0, _ = nodes[n]
            if op == var:
                vs.add(i0)
                continue
            k = ARITY[op]
            if k:
                st += (a, bb, c)[:k]
        cols[r] = frozenset(vs)
    return cols


def var_names(b: TapeBuilder) -> Dict[int, str]:
    """VAR index -> column name (cached; the builder's var_index only grows)."""
    got = b.__dict__.get("_var_names")
    if got is None or len(got) != len(b.var_index):
        got = b.__dict__["_var_names"] = {v: k for k, v in b.var_index.items()}
    return got


def cell_name(arr: str, key: int) -> str:
    return "%s[%#x]" % (arr, key)


def else_name(arr: str) -> str:
    return "%s[*]" % arr


def is_keccak(name: str) -> bool:
    return name.startswith("keccak256_") and not name.endswith("-1")


def _walk(b: TapeBuilder, roots: Iterable[int], host_only: bool = False) -> List[int]:
    """Every node reachable from roots (array chains included), children before parents; with
    ``host_only``, only the nodes that are or read host-only terms (F_HOST)."""
    order, seen = [], set()
    fl, nodes = b.flags, b.nodes
    want = F_HOST if host_only else -1  # flags & -1 is nonzero for every node but flags 0
    # a node is pushed as n (visit) and later as ~n (emit, after its operands)
    stack = [r for r in roots if not host_only or fl[r] & F_HOST]
    while stack:
        n = stack.pop()
        if n < 0:
            order.append(~n)
            continue
        if n in seen:
            continue
        seen.add(n)
        stack.append(~n)
        op, _, a, bb, c, _, _ = nodes[n]
        k = ARITY[op]
        if k == 0:
            continue
        if k > 2 and c not in seen and (not host_only or fl[c] & want):
            stack.append(c)
        if k > 1 and bb not in seen and (not host_only or fl[bb] & want):
            stack.append(bb)
        if a not in seen and (not host_only or fl[a] & want):
            stack.append(a)
    return order


_NEGATED = {Op.BVULT: Op.BVUGE, Op.BVULE: Op.BVUGT, Op.BVUGT: Op.BVULE, Op.BVUGE: Op.BVULT,
            Op.BVSLT: Op.BVSGE, Op.BVSLE: Op.BVSGT, Op.BVSGT: Op.BVSLE, Op.BVSGE: Op.BVSLT}


def _polarity(b: TapeBuilder, root: int) -> Dict[int, int]:
    """{node: 1 positive | 2 negative} of the host-only comparisons and equalities reached from
    Bool constraint `root` through AND / OR / NOT only (NOT flips); a node not in the map is
    read as positive (csrc/query.cpp polarity)."""
    nodes, fl = b.nodes, b.flags
    pol: Dict[int, int] = {}
    seen = set()
    st = [(root, 0)] if fl[root] & F_HOST else []
    while st:
        n, neg = st.pop()
        if (n, neg) in seen:
            continue
        seen.add((n, neg))
        op, _, a, bb = nodes[n][:4]
        if op in (Op.AND, Op.OR):
            st += [(x, neg) for x in (a, bb) if fl[x] & F_HOST]
        elif op == Op.NOT:
            if fl[a] & F_HOST:
                st.append((a, neg ^ 1))
        else:
            pol[n] = pol.get(n, 0) | (2 if neg else 1)
    return pol


def _arity(op: int) -> int:
    return ARITY[op]  # Op is an IntEnum: the int keys the table directly


class Lowering:
    """Harvest a query's constant keys, then rewrite its terms onto scalar columns.

    With ``frozen`` (the schema of a solved query) nothing is harvested: constant keys outside
    the schema read the else column, i.e. the value the model gives every other key — the
    behaviour ``Model.eval`` needs (mythril/laser/smt/model.py:45-59)."""

    def __init__(self, b: TapeBuilder, frozen: Optional[Schema] = None,
                 keccak_reads: bool = False):
        self.b = b
        self.frozen = frozen is not None
        self.schema = frozen if frozen is not None else Schema(keccak_reads=keccak_reads)
        self.keccak_reads = self.schema.keccak_reads
        self.memo: Dict[int, int] = {}
        self.sym = b.symbols
        # read column -> its lowered index term (the congruence conjuncts compare those)
        self.read_index: Dict[str, int] = {}
        # rewrites that read the harvest's tables (a table lookup at a symbolic key, a keccak
        # application) depend on the fingerprint; every other rewrite is the same under any
        # harvest that contains the node's own (a constant key is in it): those are kept on the
        # builder for every Lowering, so a query whose new constraint adds table keys (a fresh
        # calldata word) does not re-lower its parent's constraints
        self.dep: set = set()

    # -- pass 1: harvest ------------------------------------------------------------------
    def harvest(self, roots: Sequence[int]) -> None:
        if self.frozen:
            return
        self.apply_harvest(self.collect(roots))

    def collect(self, roots: Sequence[int]) -> "Harvest":
        """The constant keys, keccak pairs and keccak bounds the terms under `roots` state (root
        by root, as the native compiler harvests)."""
        h = Harvest()
        for r in roots:
            h.merge(self._collect_one(r))
        return h

    def _collect_one(self, root: int) -> "Harvest":
        b = self.b
        h = Harvest()
        pol = _polarity(b, root)
        # keys, keccak pairs and bounds all sit on host-only terms or their parents
        for n in _walk(b, [root], host_only=True):
            op, w, a, bb, c, i0, i1 = b.nodes[n]
            if (op == Op.EQ or op in ORDERED) and pol.get(n, 1) == 2:
                # reached only under an odd number of NOTs: the negated comparison states
                # (Not(UGT(f(x), c)) is an upper bound, not a lower one) -- a
                # disequality states no pair
                if op == Op.EQ:
                    continue
                op = _NEGATED[op]
            if op == Op.SELECT:
                base = self._array_base(a)
                if base is not None:
                    name = self.sym.array_names[b.nodes[base][5]]
                    key = b.const_value(bb)
                    cells = h.cells.setdefault(name, set())
                    if key is not None:
                        cells.add(key)
            elif op == Op.UF:
                fname = self.sym.function_names[i0]
                if is_keccak(fname):
                    h.keccak.setdefault(fname, {})
                elif not fname.endswith("-1"):
                    cells = h.uf_cells.setdefault(fname, set())
                    key = b.const_value(a)
                    if key is not None:
                        cells.add(key)
            elif op == Op.EQ or op in ORDERED:
                for x, y in ((a, bb), (bb, a)):
                    f = self._keccak_app(x)
                    kv = b.const_value(y)
                    if f is None or kv is None:
                        continue
                    if op == Op.EQ:
                        arg = b.const_value(b.nodes[x][2])
                        if arg is not None:  # keccak256_N(c) == k: a concrete pair
                            h.keccak.setdefault(f, {})[arg] = kv
                        continue
                    # a lower bound on the application (f > k, f >= k, k < f, k <= f); upper
                    # bounds and signed orders bound nothing here
                    lb = None
                    if x == a and op in (Op.BVUGT, Op.BVUGE):
                        lb = kv + (op == Op.BVUGT)
                    elif x == bb and op in (Op.BVULT, Op.BVULE):
                        lb = kv + (op == Op.BVULT)
                    if lb is not None:
                        h.bounds[f] = max(lb, h.bounds.get(f, lb))
        return h

    def apply_harvest(self, h: "Harvest") -> None:
        for name, keys in h.cells.items():
            cells = self.schema.cells.setdefault(name, {})
            for key in sorted(keys):
                cells.setdefault(key, cell_name(name, key))
        for name, keys in h.uf_cells.items():
            cells = self.schema.uf_cells.setdefault(name, {})
            for key in sorted(keys):
                cells.setdefault(key, cell_name(name, key))
        for f, pairs in h.keccak.items():
            km = self.schema.keccak.setdefault(f, KeccakMap(0))
            km.pairs.update(pairs)
            km.base = keccak_base(h.bounds.get(f, 0))

    def _keccak_app(self, n: int) -> Optional[str]:
        op, _, _, _, _, i0, _ = self.b.nodes[n]
        if op != Op.UF:
            return None
        name = self.sym.function_names[i0]
        return name if is_keccak(name) else None

    def _array_base(self, arr: int) -> Optional[int]:
        """The ARRAY node under a store chain, None for a K(...) base."""
        b = self.b
        while True:
            op = b.nodes[arr][0]
            if op == Op.STORE:
                arr = b.nodes[arr][2]
            elif op == Op.ARRAY:
                return arr
            elif op == Op.CONST_ARRAY:
                return None
            else:
                raise LoweringUnsupported("array term %s is not a store chain" % Op(op).name)

    # -- pass 2: rewrite -------------------------------------------------------------------
    def _column(self, name: str, width: int, kind: str, symbol: str,
                key: Optional[int] = None) -> int:
        if name not in self.schema.columns:
            # frozen (Model.eval): no new cells are ever made (constant keys outside the table
            # read the else column); a new else / variable column reads 0 (model completion)
            col = self.schema.columns[name] = Column(name, width, kind, symbol, key)
            if not self.frozen:  # a column's name fixes what it is, under every harvest
                self.b.__dict__.setdefault("_lower_columns", {}).setdefault(name, col)
        return self.b.var(name, width)

    def _deps(self, n: int) -> List[int]:
        b = self.b
        op, _, a, bb, c, i0, _ = b.nodes[n]
        if op == Op.SELECT:
            deps = [bb]
            arr = a
            while b.nodes[arr][0] == Op.STORE:
                deps += [b.nodes[arr][3], b.nodes[arr][4]]
                arr = b.nodes[arr][2]
            if b.nodes[arr][0] == Op.CONST_ARRAY:
                deps.append(b.nodes[arr][2])
            elif b.nodes[arr][0] != Op.ARRAY:
                raise LoweringUnsupported("array term %s is not a store chain"
                                          % Op(b.nodes[arr][0]).name)
            return deps
        if op == Op.UF:
            fname = self.sym.function_names[i0]
            if fname.endswith("-1"):
                inner = b.nodes[a]
                if inner[0] != Op.UF or self.sym.function_names[inner[5]] != fname[:-2]:
                    raise LoweringUnsupported("%s applied to something other than %s(...)"
                                              % (fname, fname[:-2]))
                return [inner[2]]
            return [a]
        if b.flags[n] & F_ARRAY:
            raise LoweringUnsupported("array-sorted term used as a value")
        k = _arity(op)
        for ch in (a, bb, c)[:k]:
            if b.flags[ch] & F_ARRAY:
                raise LoweringUnsupported("%s over arrays" % Op(op).name)
        return [a, bb, c][:k]

    def lower(self, root: int) -> int:
        """The column-only equivalent of node `root` (memoised across calls)."""
        memo = self.memo
        if root in memo:
            return memo[root]
        # a term that reads no host-only term lowers to itself (not with a frozen schema:
        # Model.eval registers every variable it meets, fresh ones read 0)
        fl = self.b.flags
        prune = not self.frozen
        if prune and not fl[root] & F_HOST:
            return root
        stable = _memo(self.b, "_stable_lower") if prune else {}
        dep = self.dep
        got = stable.get(root)
        if got is not None:
            memo[root] = got
            return got
        nodes, table_ops = self.b.nodes, (Op.SELECT, Op.UF)
        stack = [(root, None)]
        while stack:
            n, deps = stack.pop()
            if n in memo:
                continue
            if deps is None:  # first visit: operands first
                deps = self._deps(n)
                stack.append((n, deps))
                for d in deps:
                    if d in memo:
                        continue
                    if prune and not fl[d] & F_HOST:
                        memo[d] = d
                        continue
                    got = stable.get(d)
                    if got is not None:
                        memo[d] = got
                    else:
                        stack.append((d, None))
                continue
            low = memo[n] = self._rewrite(n)
            if (nodes[n][0] in table_ops and self._reads_tables(n)) or any(d in dep for d in deps):
                dep.add(n)
            elif prune:
                stable[n] = low
        return memo[root]

    def _reads_tables(self, n: int) -> bool:
        """Whether the rewrite of n itself depends on the harvest's tables (see __init__)."""
        b = self.b
        op, _, a, bb, _, i0, _ = b.nodes[n]
        if op == Op.SELECT:
            return self._array_base(a) is not None and b.const_value(bb) is None
        if op == Op.UF:
            fname = self.sym.function_names[i0]
            if is_keccak(fname):
                return True
            return not fname.endswith("-1") and b.const_value(a) is None
        return False

    def _rewrite(self, n: int) -> int:
        b, memo = self.b, self.memo
        op, w, a, bb, c, i0, i1 = b.nodes[n]
        if op == Op.VAR:
            name = self._var_name(i0)
            self._column(name, w, "var", name)
            return n
        if op == Op.SELECT:
            return self._select(a, memo[bb], bb)
        if op == Op.UF:
            return self._apply(n)
        k = _arity(op)
        if k == 0:
            return n
        args = [memo[x] for x in (a, bb, c)[:k]]
        if op == Op.EQ and b.widths[args[0]] > 256:
            return self.eq(args[0], args[1])
        if args == [a, bb, c][:k]:
            return n
        # the same op over operands of the same sorts (a lowered term keeps its width): the
        # node was checked when it was built, so it is hash-consed without re-checking
        args += [0] * (3 - k)
        return b._add(op, w, args[0], args[1], args[2], i0, i1)

    def _keccak_read(self, fname: str, km: "KeccakMap", x: int, a_orig: int) -> int:
        """The second-chance form of a keccak application (keccak_reads): the stated pairs'
        ite chain over a read column of its own, ``ite(x == c_i, k_i, f[@a])`` -- free, kept a
        function and injective by the conjuncts of ``congruence`` -- instead of the fixed
        H(x).  With a frozen schema (Model.eval) a term the query did not apply f to reads the
        reads at equal arguments, else H(x)."""
        b = self.b
        cx = b.const_value(x)
        if cx is not None and cx in km.pairs:  # a stated pair: its hash
            return b.const(km.pairs[cx], 256)
        rname = read_name(fname, a_orig)
        if cx is not None and (not self.frozen or rname in self.schema.columns):
            if not self.frozen:
                self.read_index.setdefault(rname, x)
            return self._column(rname, 256, "kread", fname, a_orig)  # no pair's argument
        if not self.frozen:
            acc = self._column(rname, 256, "kread", fname, a_orig)
            self.read_index.setdefault(rname, x)
        elif rname in self.schema.columns:
            acc = self._column(rname, 256, "kread", fname, a_orig)
        else:
            h = b.op(Op.KECCAK, x)
            h = b.op(Op.BVLSHR, h, b.const(KECCAK_SHIFT, 256))
            h = b.op(Op.BVSHL, h, b.const(KECCAK_ALIGN, 256))
            acc = b.op(Op.BVADD, h, b.const(km.base, 256)) if km.base else h
            reads = sorted((c for c in self.schema.columns.values()
                            if c.kind == "kread" and c.symbol == fname), key=lambda c: c.key)
            for c in reversed(reads):
                acc = b.op(Op.ITE, self.eq(x, self.lower(c.key)),
                           self._column(c.name, 256, "kread", fname, c.key), acc)
        for arg in sorted(km.pairs, reverse=True):
            acc = b.op(Op.ITE, self.eq(x, b.const(arg, b.widths[x])),
                       b.const(km.pairs[arg], 256), acc)
        return acc

    # -- wide equalities: the device compares at most 256 bits ---------------------------------
    def _pieces(self, n: int) -> List[int]:
        """Leaves of the CONCAT tree of n, most significant first (ZEXT = zeros ++ x)."""
        b = self.b
        out, stack = [], [n]
        while stack:
            x = stack.pop()
            op, w, a, bb, _, i0, _ = b.nodes[x]
            if op == Op.CONCAT:
                stack += [bb, a]
            elif op == Op.ZEXT:
                stack += [a, b.const(0, i0) if i0 <= 256 else self._zeros(i0)]
            elif w > 256 and b.const_value(x) is None:
                raise LoweringUnsupported("%d-bit %s operand of a wide equality"
                                          % (w, Op(op).name))
            else:
                out.append(x)
        return out

    def _zeros(self, w: int) -> int:
        return self.b.const(0, w)

    def _slice(self, piece: int, hi: int, lo: int) -> int:
        """Bits [lo, hi) of a <= 256-bit piece (constants sliced on the host)."""
        b = self.b
        w = b.widths[piece]
        if lo == 0 and hi == w:
            return piece
        cv = b.const_value(piece)
        if cv is not None:
            return b.const((cv >> lo) & ((1 << (hi - lo)) - 1), hi - lo)
        return b.op(Op.EXTRACT, piece, imm0=hi - 1, imm1=lo)

    def eq(self, x: int, y: int) -> int:
        """x == y for bit-vectors of any width: an AND of <= 256-bit equalities over the common
        refinement of the two sides' concat boundaries."""
        b = self.b
        w = b.widths[x]
        if w <= 256:
            return b.op(Op.EQ, x, y)
        sides = []
        for t in (x, y):
            pos, segs = w, []
            for p in self._pieces(t):
                pw = b.widths[p]
                segs.append((pos - pw, pos, p))
                pos -= pw
            sides.append(segs)
        cuts = sorted({lo for s in sides for lo, _, _ in s} | {w})
        acc = None
        for lo, hi in zip(cuts[:-1], cuts[1:]):
            parts = []
            for segs in sides:
                for plo, phi, p in segs:
                    if plo <= lo and hi <= phi:
                        parts.append(self._slice(p, hi - plo, lo - plo))
                        break
            e = b.op(Op.EQ, parts[0], parts[1])
            acc = e if acc is None else b.op(Op.AND, acc, e)
        return acc

    def _var_name(self, col: int) -> str:
        names = getattr(self, "_names", None)
        if names is None or len(names) != len(self.b.var_index):
            names = self._names = {v: k for k, v in self.b.var_index.items()}
        return names[col]

    def _select(self, arr: int, idx: int, idx_orig: int) -> int:
        b = self.b
        op = b.nodes[arr][0]
        if op == Op.STORE:
            key, val = self.memo[b.nodes[arr][3]], self.memo[b.nodes[arr][4]]
            rest = self._select(b.nodes[arr][2], idx, idx_orig)
            return b.op(Op.ITE, self.eq(idx, key), val, rest)
        if op == Op.CONST_ARRAY:
            return self.memo[b.nodes[arr][2]]
        name = self.sym.array_names[b.nodes[arr][5]]
        rng = b.widths[arr]
        return self._table(name, rng, idx, self.schema.cells.get(name, {}), "cell", "else",
                           "read", idx_orig)

    def _table(self, name: str, rng: int, idx: int, cells: Dict[int, str], kcell: str,
               kelse: str, kread: str, idx_orig: int) -> int:
        b = self.b
        key = b.const_value(idx)
        if key is not None and key in cells:
            return self._column(cells[key], rng, kcell, name, key)
        rname = read_name(name, idx_orig)
        if key is not None and (self.frozen and rname not in self.schema.columns):
            # Model.eval at a constant key outside the table: the reads, else the else value
            return self._fallback(name, rng, idx, kelse, kread)
        if key is not None:
            # an index that lowers to a constant no harvest saw (select(K(7), i) as a key): a
            # read of its own -- the else column would let a read at an equal index take another
            # value there (kept apart by congruence like any two reads)
            if not self.frozen:
                self.read_index.setdefault(rname, idx)
            return self._column(rname, rng, kread, name, idx_orig)
        if not self.frozen:
            acc = self._column(rname, rng, kread, name, idx_orig)
            self.read_index.setdefault(rname, idx)
        elif rname in self.schema.columns:  # Model.eval of a read the query made
            acc = self._column(rname, rng, kread, name, idx_orig)
        else:  # Model.eval at another index: the model's value there
            acc = self._fallback(name, rng, idx, kelse, kread)
        for ck in sorted(cells, reverse=True):
            cell = self._column(cells[ck], rng, kcell, name, ck)
            kn = b.const(ck, b.widths[idx])
            acc = b.op(Op.ITE, self.eq(idx, kn), cell, acc)
        return acc

    def _fallback(self, name: str, rng: int, idx: int, kelse: str, kread: str) -> int:
        """The value at an index no cell holds: the read whose index equals it, else the else
        column (with a frozen schema: the model's table; otherwise a query reads no such key)."""
        b = self.b
        acc = self._column(else_name(name), rng, kelse, name)
        if not self.frozen:
            return acc
        reads = sorted((c for c in self.schema.columns.values()
                        if c.kind == kread and c.symbol == name), key=lambda c: c.key)
        for c in reversed(reads):
            li = self.lower(c.key)
            acc = b.op(Op.ITE, self.eq(idx, li), self._column(c.name, rng, kread, name, c.key),
                       acc)
        return acc

    def _apply(self, n: int) -> int:
        b = self.b
        _, w, a, _, _, i0, _ = b.nodes[n]
        fname = self.sym.function_names[i0]
        if fname.endswith("-1"):
            return self.memo[b.nodes[a][2]]
        x = self.memo[a]
        if is_keccak(fname):
            km = self.schema.keccak.get(fname)
            if km is None:
                if not self.frozen:
                    raise LoweringUnsupported("keccak function %s not harvested" % fname)
                km = KeccakMap(0)
            if w != 256:
                raise LoweringUnsupported("keccak function %s has range %d" % (fname, w))
            if self.keccak_reads:
                return self._keccak_read(fname, km, x, a)
            h = b.op(Op.KECCAK, x)
            h = b.op(Op.BVLSHR, h, b.const(KECCAK_SHIFT, 256))
            h = b.op(Op.BVSHL, h, b.const(KECCAK_ALIGN, 256))
            acc = b.op(Op.BVADD, h, b.const(km.base, 256)) if km.base else h
            if w != 256:
                raise LoweringUnsupported("keccak function %s has range %d" % (fname, w))
            for arg in sorted(km.pairs, reverse=True):
                acc = b.op(Op.ITE, self.eq(x, b.const(arg, b.widths[x])),
                           b.const(km.pairs[arg], 256), acc)
            return acc
        cells = self.schema.uf_cells.get(fname, {})
        return self._table(fname, w, x, cells, "ufcell", "ufelse", "ufread", a)


MAX_LOWERINGS = 64  # pass-2 memos kept per builder, by harvest fingerprint (LRU)


def congruence(b: TapeBuilder, L: "Lowering", x: int, reads: list, seen: set) -> List[int]:
    """The conjuncts that keep the read columns functional (Ackermann's reduction): for every
    read column the lowered constraint `x` reads first in its query (directly or in the index
    term of a read it reads) -- ordered by (symbol, index term) -- and every read of the same
    symbol before it (`reads`, in the order the query introduced them; updated here),
    ``Or(Not(i == j), A[@i] == A[@j])``; keccak reads (the second-chance lowering) are also
    injective: ``Or(i == j, Not(f[@i] == f[@j]))`` after it, and ``Or(i == c,
    Not(f[@i] == k))`` for every stated pair (c, k) -- the lowering maps ``f-1(f(x))`` to ``x``.
    The native query compiler makes the same conjuncts in the same order (csrc/query.cpp
    congruence)."""
    names = var_names(b)
    cv = b.const_value
    found, work = {}, [x]
    while work:  # the reads under x, and under the index terms of those (A[B[i]])
        t = work.pop()
        for v in node_columns(b, [t])[t]:
            col = L.schema.columns.get(names[v])
            if col is not None and col.kind in READ_KINDS and col.name not in found:
                found[col.name] = col
                work.append(L.read_index[col.name])
    new = sorted((c for c in found.values() if c.name not in seen),
                 key=lambda c: (c.symbol, c.key))
    out = []
    for p in new:
        rp = b.var(p.name, p.width)
        for q in reads:
            if q.symbol == p.symbol and q.kind == p.kind:
                iq, ip = L.read_index[q.name], L.read_index[p.name]
                eqv = b.op(Op.EQ, b.var(q.name, q.width), rp)
                if p.kind == "kread" and cv(iq) is not None and cv(ip) is not None:
                    # two keccak reads at constant arguments: equal values, or unequal ones
                    out.append(eqv if cv(iq) == cv(ip) else b.op(Op.NOT, eqv))
                    continue
                same = L.eq(iq, ip)
                out.append(b.op(Op.OR, b.op(Op.NOT, same), eqv))
                if p.kind == "kread":  # injective too: Or(i == j, Not(f_i == f_j))
                    out.append(b.op(Op.OR, same, b.op(Op.NOT, eqv)))
        if p.kind == "kread":  # injective against the stated pairs too (the inverse reads them)
            km = L.schema.keccak[p.symbol]
            li = L.read_index[p.name]
            for arg in sorted(km.pairs):
                ne = b.op(Op.NOT, b.op(Op.EQ, rp, b.const(km.pairs[arg], 256)))
                # a constant argument is no pair's (those lower to the pair's hash)
                out.append(ne if cv(li) is not None else
                           b.op(Op.OR, L.eq(li, b.const(arg, b.widths[li])), ne))
        reads.append(p)
        seen.add(p.name)
    return out


def lower_query(b: TapeBuilder, roots: Sequence[int],
                frozen: Optional[Schema] = None, _fresh_prefix: bool = False,
                keccak_reads: bool = False) -> Tuple[int, Schema]:
    """Lower the conjunction of Bool `roots`: (root node of the column-only term, schema).

    Without ``frozen`` both passes are memoised on the builder: pass 1 per constraint
    (``Harvest``), pass 2 per harvest fingerprint (the rewrite of a node depends on nothing
    else), so a LASER query that adds one constraint to its parent's (svm.py:257-262) lowers only
    that constraint.  The schema's columns are the ones the lowered term reads, in VAR order.
    ``keccak_reads``: keccak applications as read columns (Lowering._keccak_read; the sieve's
    second chance for a query its first lowering missed)."""
    if frozen is not None:
        L = Lowering(b, frozen)
        low = [L.lower(r) for r in roots]
        schema = L.schema
    elif not _fresh_prefix and len(roots) > 1 and \
            _prefix_state(b, roots, keccak_reads) is not None:
        return _lower_extend(b, roots, keccak_reads)
    else:
        per_root: Dict[int, Harvest] = _memo(b, "_harvest_of")
        h = Harvest()
        for r in roots:
            got = per_root.get(r)
            if got is None:
                got = per_root[r] = Lowering(b).collect([r])
            h.merge(got)
        fp = h.fingerprint()
        lows = b.__dict__.setdefault("_lowerings", OrderedDict())
        L = lows.get((fp, keccak_reads))
        if L is None:
            L = lows[(fp, keccak_reads)] = Lowering(b, keccak_reads=keccak_reads)
            L.apply_harvest(h)
            if len(lows) > MAX_LOWERINGS:
                lows.popitem(last=False)
        else:
            lows.move_to_end((fp, keccak_reads))
        low, reads, seen = [], [], set()
        for r in roots:
            x = L.lower(r)
            low.append(x)
            low.extend(congruence(b, L, x, reads, seen))
        cols = node_columns(b, low)
        used = frozenset().union(*(cols[r] for r in low)) if low else frozenset()
        schema = _schema_of(b, L, used)
    for r in low:
        if b.widths[r] != BOOL:
            raise TapeError("constraints must be Bool")
    if not low:
        return b.true(), schema
    acc = low[0]
    for x in low[1:]:
        acc = b.op(Op.AND, acc, x)
    if frozen is None:
        _remember_prefix(b, roots, h, fp, L, low, used, acc, reads, seen, keccak_reads)
    return acc, schema


# -- LASER order: a query that extends its parent's roots by one constraint -------------------
PREFIX_STATES = 256  # lowered prefixes kept per builder


@dataclass
class _Prefix:
    harvest: Harvest
    fp: tuple
    lowering: "Lowering"
    low: List[int]
    used: frozenset
    acc: int
    reads: list = field(default_factory=list)   # read columns in introduction order
    seen: set = field(default_factory=set)


def _prefix_state(b: TapeBuilder, roots: Sequence[int], kr: bool = False) -> Optional[_Prefix]:
    cache = b.__dict__.get("_lower_prefixes")
    return None if cache is None else cache.get((kr, tuple(roots[:-1])))


def _remember_prefix(b, roots, h, fp, L, low, used, acc, reads, seen, kr=False) -> None:
    cache = b.__dict__.setdefault("_lower_prefixes", OrderedDict())
    cache[(kr, tuple(roots))] = _Prefix(h, fp, L, list(low), used, acc, list(reads), set(seen))
    while len(cache) > PREFIX_STATES:
        cache.popitem(last=False)


def _lower_extend(b: TapeBuilder, roots: Sequence[int], kr: bool = False
                  ) -> Tuple[int, "Schema"]:
    """lower_query of `roots` from the lowered state of ``roots[:-1]`` (svm.py:257-262: every new
    state's query is its parent's plus one constraint): the new constraint's harvest is merged
    into the parent's; an unchanged fingerprint keeps the parent's lowering and its lowered
    conjuncts, so only the new constraint is lowered and ANDed on.  The result is lower_query's
    from scratch (tests/test_lowering.py compares them)."""
    par = _prefix_state(b, roots, kr)
    new = roots[-1]
    per_root: Dict[int, Harvest] = _memo(b, "_harvest_of")
    hn = per_root.get(new)
    if hn is None:
        hn = per_root[new] = Lowering(b).collect([new])
    h = Harvest({k: set(v) for k, v in par.harvest.cells.items()},
                {k: set(v) for k, v in par.harvest.uf_cells.items()},
                {k: dict(v) for k, v in par.harvest.keccak.items()}, dict(par.harvest.bounds))
    h.merge(hn)
    fp = h.fingerprint()
    if fp != par.fp:  # new keys / keccak pairs: every constraint's rewrite may change
        return lower_query(b, list(roots[:-1]) + [new], _fresh_prefix=True, keccak_reads=kr)
    L = par.lowering
    x = L.lower(new)
    if b.widths[x] != BOOL:
        raise TapeError("constraints must be Bool")
    reads, seen = list(par.reads), set(par.seen)
    added = [x] + congruence(b, L, x, reads, seen)
    low = par.low + added
    used = par.used
    acc = par.acc
    for y in added:
        used = used | node_columns(b, [y])[y]
        acc = b._add(Op.AND, BOOL, acc, y)
    _remember_prefix(b, roots, h, fp, L, low, used, acc, reads, seen, kr)
    return acc, _schema_of(b, L, used)


def _schema_of(b: TapeBuilder, L: "Lowering", used: frozenset) -> "Schema":
    """The query's schema: the columns of the VARs its lowered term reads, in VAR order."""
    names = var_names(b)
    full = L.schema
    cols = {}
    for v in sorted(used):
        name = names[v]
        col = full.columns.get(name)
        if col is None:  # made by an earlier Lowering (a stable rewrite), else a plain
            # variable under a term the rewrite left as it was
            col = b.__dict__.get("_lower_columns", {}).get(name)
            if col is None:
                col = Column(name, b.symbols.var_widths[name], "var", name)
            full.columns[name] = col
        if col.kind != "var" and name in b.symbols.user_vars:
            # a declared symbol named like a cell: one column would stand for both (the native
            # compiler refuses the same, csrc/query.cpp QueryState::emit)
            raise LoweringUnsupported("variable %s is named like an array cell" % name)
        cols[name] = col
    return Schema(full.cells, full.uf_cells, full.keccak, cols, full.keccak_reads)
