"""Candidate generation for one query: what the sieve's assignment rows should try.

Uniform random 256-bit values almost never satisfy a path condition (a 4-byte selector check
alone has p = 2^-32, SURVEY.md §7 "hard parts"), so rows are drawn from a *guide* harvested from
the query's own terms:

* **sets of alternatives** — every conjunct of the path condition is inverted toward the
  columns it reads: ``t == K`` through ``concat`` / ``extract`` / ``zero_extend`` / ``ite`` /
  ``+ c`` / ``- c`` / ``xor c`` / ``* odd c`` / ``not`` gives partial assignments (column ->
  value) that make the conjunct true; ``Or`` gives alternatives (``sender`` in ACTORS,
  transaction/symbolic.py:22-67); ordered comparisons against constants give boundary values.
  An equality between two symbolic terms is tried with the query's constants of that width (an
  address argument equal to ``Extract(159, 0, sender)``).  The parent path condition's witness
  (the query minus its newest constraint, svm.py:257-262) is the first set;
* **per-column pools** — the values the inversions produced for that column, boundary values of
  comparisons, and 0, 1, 2^w - 1, 2^(w-1).

The device generator (``mh_assign_generate_guided``, restated in oracle/guided_gen.py) draws
each column from {small, uniform, pool} and then applies one alternative of each set with the
set's probability, from a counter-based RNG, so any row range regenerates independently.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .lower import Schema, var_names
from .tape import BOOL, Op, TapeBuilder

Alt = Dict[str, int]          # column name -> value
Copy = Tuple[str, str, int, int, int]  # (dst column, src column, dst_lo, src_lo, nbits)
MAX_ALTS = 16                 # alternatives kept per inversion
MAX_SETS = 1024
MAX_POOL = 64                 # values per column pool
MAX_EQ_CONSTS = 24            # constants tried against a symbolic-symbolic equality
PROB_DEFAULT = 208            # of 256: a set is applied to ~81 % of rows
PROB_PARENT = 192
COPY_FLAG = 0x80000000        # entry_col bit: the entry copies bits of another column
PROB_HINT = 64                # soft hints (conditions of ite branches)


def _mask(w: int) -> int:
    return (1 << w) - 1


def _interval_values(lo: int, hi: int) -> List[int]:
    """Values of [lo, hi] a guide proposes: both ends, the middle, lo + 1 (distinct, in order)."""
    out: List[int] = []
    for v in (lo, hi, lo + (hi - lo) // 2, lo + 1):
        if lo <= v <= hi and v not in out:
            out.append(v)
    return out


def _merge(xs: List[Alt], ys: List[Alt]) -> List[Alt]:
    if len(ys) == 1 and not ys[0]:
        return xs[:MAX_ALTS]
    if len(xs) == 1 and not xs[0]:
        return ys[:MAX_ALTS]
    if len(xs) == 1 and len(ys) == 1:  # the common case (bytes of one word): one pair
        x, y = xs[0], ys[0]
        if len(y) < len(x):
            x, y = y, x
        for k, v in x.items():
            if k in y and y[k] != v:
                return []
        z = dict(y)
        z.update(x)
        return [z]
    out = []
    for x in xs:
        for y in ys:
            if any(k in x and x[k] != v for k, v in y.items()):
                continue
            z = dict(x)
            z.update(y)
            out.append(z)
            if len(out) >= MAX_ALTS:
                return out
    return out


@dataclass
class Guide:
    """Host form of mh_guide (include/mythril_hip.h)."""

    columns: List[str]
    widths: List[int]
    pools: List[List[int]]
    sets: List[Tuple[int, List[Alt]]] = field(default_factory=list)  # (prob/256, alternatives)
    copy_sets: List[Tuple[int, List[List[Copy]]]] = field(default_factory=list)

    def arrays(self):
        """numpy arrays in mh_guide order."""
        col_index = {c: i for i, c in enumerate(self.columns)}
        width = np.array(self.widths, dtype=np.uint16)
        pool_off = np.zeros(len(self.columns) + 1, dtype=np.uint32)
        pool_vals: List[int] = []
        for i, p in enumerate(self.pools):
            pool_vals += p
            pool_off[i + 1] = len(pool_vals)
        n_sets = len(self.sets) + len(self.copy_sets)
        set_off = np.zeros(n_sets + 1, dtype=np.uint32)
        set_prob = np.zeros(max(n_sets, 1), dtype=np.uint8)
        alt_off: List[int] = [0]
        e_col: List[int] = []
        e_val: List[int] = []
        j = 0
        for prob, alts in self.sets:
            set_prob[j] = prob
            for alt in alts:  # an alternative's entries write distinct columns: any order
                for name, v in alt.items():
                    e_col.append(col_index[name])
                    e_val.append(v)
                alt_off.append(len(e_col))
            j += 1
            set_off[j] = len(alt_off) - 1
        for prob, alts in self.copy_sets:
            set_prob[j] = prob
            for alt in alts:
                for dst, src, dlo, slo, nb in alt:
                    e_col.append(col_index[dst] | COPY_FLAG)
                    e_val.append(col_index[src] | dlo << 32 | slo << 64 | nb << 96)
                alt_off.append(len(e_col))
            j += 1
            set_off[j] = len(alt_off) - 1
        return dict(
            width=width, pool_off=pool_off, pool=_limbs(pool_vals), set_off=set_off,
            set_prob=set_prob, alt_off=np.array(alt_off, dtype=np.uint32),
            entry_col=np.array(e_col or [0], dtype=np.uint32), entry_val=_limbs(e_val))


def _limbs(vals: Sequence[int]) -> np.ndarray:
    if not vals:
        return np.zeros((1, 8), dtype=np.uint32)
    buf = b"".join((v & ((1 << 256) - 1)).to_bytes(32, "little") for v in vals)
    return np.frombuffer(buf, dtype="<u4").reshape(len(vals), 8).astype(np.uint32)


MEMO_LIMIT = 1 << 20  # entries per builder-level memo before it is dropped


def _memo(b: TapeBuilder, name: str) -> dict:
    """A memo living on the builder: lowered nodes are immutable and hash-consed, so what is
    derived from a node alone holds for every later query that contains it (a LASER query
    extends its parent's, svm.py:257-262)."""
    m = b.__dict__.get(name)
    if m is None or len(m) > MEMO_LIMIT:
        m = b.__dict__[name] = {}
    return m


HINTS_PER_COLUMN = 2  # single-column hint sets kept per column and direction


def _prune_hints(hints: List[Tuple[int, List[Alt]]]) -> List[Tuple[int, List[Alt]]]:
    """Drop dominated single-column hints.  The conditions of a calldata word's byte reads,
    ``i < calldatasize`` for each byte index i (calldata.py:234-247), each give a boundary hint on
    the size; every one is implied by the largest index's.  Per column, the sets with the
    HINTS_PER_COLUMN largest and smallest values are kept (lower and upper bounds), in their
    order; hints over several columns are all kept."""
    by_col: Dict[str, List[int]] = {}
    for i, (_, alts) in enumerate(hints):
        cols = {c for a in alts for c in a}
        if len(cols) == 1 and all(len(a) == 1 for a in alts):
            by_col.setdefault(next(iter(cols)), []).append(i)
    drop = set()
    for c, idx in by_col.items():
        if len(idx) <= 2 * HINTS_PER_COLUMN:
            continue
        hi = sorted(idx, key=lambda i: -max(a[c] for a in hints[i][1]))[:HINTS_PER_COLUMN]
        lo = sorted(idx, key=lambda i: min(a[c] for a in hints[i][1]))[:HINTS_PER_COLUMN]
        drop.update(set(idx) - set(hi) - set(lo))
    return [h for i, h in enumerate(hints) if i not in drop]


class Harvester:
    def __init__(self, b: TapeBuilder, schema: Schema, columns: Sequence[str],
                 parent_eval: bool = False):
        self.b = b
        # parent_eval (mh_guide_harvest_inc): operands the parent witness fixes count as known
        # (_pick); set from harvest()'s parent, with a memo of this harvest's own
        self.parent_eval = parent_eval
        self._parent: Optional[Dict[str, int]] = None
        self._pv: Dict[int, Optional[int]] = {}
        self.schema = schema
        self.columns = list(columns)
        # every VAR under a lowered query is one of its columns
        self.col_of_var = var_names(b)
        self.pools: Dict[str, List[int]] = {c: [] for c in self.columns}
        self.sets: List[Tuple[int, List[Alt]]] = []
        # inversions by (node, value, mask) / (node, truth), with the hints each produced
        # (transitively), so a memo hit replays them exactly as a fresh inversion would
        self._inv_memo: Dict[tuple, tuple] = {} if parent_eval else _memo(b, "_guide_inv")
        self._cap: List[list] = []
        self._consts_by_width: Dict[int, List[int]] = {}
        self.hints: List[Tuple[int, List[Alt]]] = []
        self.copy_sets: List[List[List[Copy]]] = []
        self._hint_keys = set()

    def _pick(self, a: int, bb: int, a_first: bool = False) -> Optional[Tuple[int, int]]:
        """(the operand to solve for, the other side's value): a constant first (a before b
        with `a_first`, else b before a), then with ``parent_eval`` a side the parent witness
        fixes, b before a (csrc/harvest.cpp Harvester::pick)."""
        cv = self.b.const_value
        if a_first and cv(a) is not None:
            return bb, cv(a)
        if cv(bb) is not None:
            return a, cv(bb)
        if cv(a) is not None:
            return bb, cv(a)
        if self._parent is not None:
            pb = self._parent_value(bb)
            if pb is not None:
                return a, pb
            pa = self._parent_value(a)
            if pa is not None:
                return bb, pa
        return None

    def _parent_value(self, root: int) -> Optional[int]:
        """The value of term `root` under the parent witness, when every column it reads has
        a parent value and every op is a bit-layout or linear one; else None (memoised)."""
        b, memo = self.b, self._pv
        if root in memo:
            return memo[root]
        st = [(root, False)]
        un = (Op.BVNOT, Op.BVNEG, Op.ZEXT, Op.EXTRACT)
        bin_ = (Op.BVADD, Op.BVSUB, Op.BVXOR, Op.BVAND, Op.BVOR, Op.BVMUL, Op.CONCAT)
        while st:
            n, done = st.pop()
            if n in memo:
                continue
            op, w, a, bb, _, i0, i1 = b.nodes[n]
            c = b.const_value(n)
            if c is not None:
                memo[n] = c
                continue
            if op == Op.VAR:
                name = self.col_of_var.get(i0)
                v = self._parent.get(name) if name is not None else None
                memo[n] = None if v is None else v & _mask(w)
                continue
            if op not in un and op not in bin_:
                memo[n] = None
                continue
            if not done:
                st.append((n, True))
                st.append((a, False))
                if op in bin_:
                    st.append((bb, False))
                continue
            va = memo.get(a)
            vb = memo.get(bb) if op in bin_ else 0
            if va is None or vb is None:
                memo[n] = None
                continue
            m = _mask(w)
            if op == Op.BVNOT:
                v = ~va & m
            elif op == Op.BVNEG:
                v = -va & m
            elif op == Op.ZEXT:
                v = va
            elif op == Op.EXTRACT:
                v = (va >> i1) & m
            elif op == Op.BVADD:
                v = (va + vb) & m
            elif op == Op.BVSUB:
                v = (va - vb) & m
            elif op == Op.BVXOR:
                v = va ^ vb
            elif op == Op.BVAND:
                v = va & vb
            elif op == Op.BVOR:
                v = va | vb
            elif op == Op.BVMUL:
                v = (va * vb) & m
            else:  # CONCAT
                v = (va << b.widths[bb]) | vb
            memo[n] = v
        return memo[root]

    def _memoised(self, key: tuple, compute):
        got = self._inv_memo.get(key)
        if got is None:
            self._cap.append([])
            try:
                r = compute()
            finally:
                hints = self._cap.pop()
            self._inv_memo[key] = (r, tuple(hints))
            if self._cap:
                self._cap[-1].extend(hints)
            return r
        r, hints = got
        for h in hints:
            self._hint(h)
        return r

    # -- inversion -------------------------------------------------------------------------
    def invert_bits(self, n: int, value: int, mask: int, depth: int = 0) -> Optional[List[Alt]]:
        """Partial assignments making (term n) & mask == value & mask; None = don't know."""
        return self._memoised(
            (n, value, mask),
            lambda: self._invert_bits(n, value & mask, mask, depth) if depth < 64 else None)

    def _invert_bits(self, n: int, value: int, mask: int, depth: int) -> Optional[List[Alt]]:
        b = self.b
        op, w, a, bb, c, i0, i1 = b.nodes[n]
        full = mask == _mask(w)
        cv = b.const_value(n)
        if cv is not None:
            return [{}] if (cv & mask) == value else []
        if op == Op.VAR:
            name = self.col_of_var.get(i0)
            return None if name is None else [{name: value}]
        if op == Op.CONCAT:  # every leaf of the concat tree inverted on its own bit range
            acc: List[Alt] = [{}]
            for child, lo, wc in self._concat_leaves(n):
                m = (mask >> lo) & _mask(wc)
                if m == 0:
                    continue
                r = self.invert_bits(child, (value >> lo) & m, m, depth + 1)
                if r is None or r == [{}]:
                    continue
                acc = _merge(acc, r)
                if not acc:
                    return acc
            return acc
        if op == Op.EXTRACT:
            return self.invert_bits(a, value << i1, mask << i1, depth + 1)
        if op == Op.BVAND:  # x & m == value on `mask`: only the bits of m are free
            for x, m in ((a, b.const_value(bb)), (bb, b.const_value(a))):
                if m is not None:
                    if value & ~m & mask:
                        return []
                    return self.invert_bits(x, value & m, mask & m, depth + 1)
            return None
        if op in (Op.ZEXT, Op.SEXT):
            wa = b.widths[a]
            if op == Op.ZEXT and (value >> wa) != 0:
                return []
            return self.invert_bits(a, value & _mask(wa), mask & _mask(wa), depth + 1)
        if op == Op.ITE:
            # the branch's requirement is exact; the condition's is usually a range (calldata
            # bytes: `i < calldatasize`), so it is kept as a soft hint of its own, not merged
            out: List[Alt] = []
            for branch, truth in ((bb, True), (c, False)):
                r = self.invert_bits(branch, value, mask, depth + 1)
                if not r:
                    continue
                cond = self.invert_bool(a, truth, depth + 1)
                if cond and cond != [{}]:
                    self._hint(cond)
                out += r
            if len(out) > 1 and {} in out:
                # one branch already holds whatever the columns are (a calldata byte past
                # calldatasize reads 0): the other branch's assignments also satisfy the term,
                # and keeping the empty alternative beside them only multiplies the
                # combinations of every enclosing concat (up to MAX_ALTS each)
                out = [x for x in out if x]
            return out[:MAX_ALTS]
        if not full:
            return None
        m = _mask(w)
        if op in (Op.BVADD, Op.BVSUB, Op.BVXOR, Op.BVMUL):
            got = self._pick(a, bb)
            if got is None:
                return None
            x, k = got
            if op == Op.BVADD:
                t = value - k
            elif op == Op.BVSUB:
                t = value + k if x == a else k - value
            elif op == Op.BVXOR:
                t = value ^ k
            else:
                if k % 2 == 0:
                    return None
                t = value * pow(k, -1, 1 << w)
            return self.invert_bits(x, t & m, m, depth + 1)
        if op == Op.BVNOT:
            return self.invert_bits(a, ~value & m, m, depth + 1)
        if op == Op.BVNEG:
            return self.invert_bits(a, -value & m, m, depth + 1)
        return None

    def _concat_leaves(self, n: int) -> List[Tuple[int, int, int]]:
        """(leaf node, bit offset, width) of the maximal concat tree rooted at n, low bits first
        (memoised on the builder: nodes are immutable)."""
        b = self.b
        memo = b.__dict__.setdefault("_concat_leaves", {})
        got = memo.get(n)
        if got is None:
            got, stack = [], [(n, 0)]
            while stack:
                x, lo = stack.pop()
                node = b.nodes[x]
                if node[0] == Op.CONCAT:
                    stack.append((node[2], lo + b.widths[node[3]]))
                    stack.append((node[3], lo))
                else:
                    got.append((x, lo, b.widths[x]))
            memo[n] = got
        return got

    def invert_bool(self, n: int, truth: bool, depth: int = 0) -> Optional[List[Alt]]:
        """Partial assignments making Bool node n == truth; None = don't know."""
        if depth > 64:
            return None
        return self._memoised(("bool", n, truth), lambda: self._invert_bool(n, truth, depth))

    def _invert_bool(self, n: int, truth: bool, depth: int) -> Optional[List[Alt]]:
        b = self.b
        op, w, a, bb, c, i0, i1 = b.nodes[n]
        cv = b.const_value(n)
        if cv is not None:
            return [{}] if bool(cv) == truth else []
        if op == Op.NOT:
            return self.invert_bool(a, not truth, depth + 1)
        if op in (Op.AND, Op.OR):
            conj = (op == Op.AND) == truth
            x, y = self.invert_bool(a, truth, depth + 1), self.invert_bool(bb, truth, depth + 1)
            if conj:
                return _merge(x if x is not None else [{}], y if y is not None else [{}])
            out = (x or []) + (y or [])
            return out[:MAX_ALTS] if (x is not None or y is not None) else None
        if op == Op.EQ:
            if b.widths[a] == BOOL:
                return None
            got = self._pick(a, bb)
            if got is None:
                return None
            t, k = got
            if truth:
                return self.invert_bits(t, k, _mask(b.widths[t]))
            return [{}]  # t != K: almost every value satisfies it
        if op in (Op.BVADD_NOOVFL_U, Op.BVMUL_NOOVFL_U, Op.BVSUB_NOUDFL_U):
            wt = b.widths[a]
            if op == Op.BVSUB_NOUDFL_U:  # b <=u a
                pairs = [(0, 0), (1, 0)] if truth else [(0, 1), (1, 2)]
            elif truth:
                pairs = [(0, 0), (1, 1)]
            else:  # overflow: a = 2^w - 1 with b >= 2 (add: b >= 1)
                pairs = [(_mask(wt), 2), (_mask(wt), _mask(wt))]
            out = []
            for va, vb in pairs:
                ra = self.invert_bits(a, va, _mask(wt))
                rb = self.invert_bits(bb, vb, _mask(wt))
                if ra is None and rb is None:
                    continue
                out += _merge(ra if ra is not None else [{}], rb if rb is not None else [{}])
            return out[:MAX_ALTS] if out else None
        if op in (Op.BVULT, Op.BVULE, Op.BVUGT, Op.BVUGE, Op.BVSLT, Op.BVSLE, Op.BVSGT,
                  Op.BVSGE):
            got = self._pick(a, bb, a_first=True)
            if got is None:
                return None
            wt = b.widths[a]
            t, k = got
            out = []
            for v in self._boundary(Op(op), k, t == a, truth, wt):
                r = self.invert_bits(t, v, _mask(wt))
                if r:
                    out += r
            return out[:MAX_ALTS]
        return None

    @staticmethod
    def _boundary(op: Op, k: int, var_left: bool, truth: bool, w: int) -> List[int]:
        """Values of the symbolic side that make `op` come out `truth` near the constant k."""
        m = _mask(w)
        # normalise to "var < k" style: which side of k satisfies?
        less = op in (Op.BVULT, Op.BVULE, Op.BVSLT, Op.BVSLE)
        strict = op in (Op.BVULT, Op.BVUGT, Op.BVSLT, Op.BVSGT)
        want_below = less == var_left  # var < k (or <=) when the var is on the left of '<'
        if not truth:
            want_below, strict = not want_below, not strict
        if want_below:
            vals = [k - 1, k >> 1, 0] if strict else [k, k - 1, 0]
        else:
            vals = [k + 1, k + 2, (k << 1) + 1] if strict else [k, k + 1]
        return [v & m for v in vals]

    def segments(self, n: int, depth: int = 0) -> Optional[List[Tuple[int, int, str, int]]]:
        """Bits of term n that are bits of a column: [(lo, nbits, column, column_lo)], through
        concat / extract / zero_extend and the value branch of ite(c, x, const); None if the
        term computes."""
        if depth > 64:
            return None
        b = self.b
        op, w, a, bb, c, i0, i1 = b.nodes[n]
        if b.const_value(n) is not None:
            return []
        if op == Op.VAR:
            name = self.col_of_var.get(i0)
            return None if name is None else [(0, w, name, 0)]
        if op == Op.CONCAT:
            hi, lo = self.segments(a, depth + 1), self.segments(bb, depth + 1)
            if hi is None or lo is None:
                return None
            wb = b.widths[bb]
            return lo + [(x + wb, n_, col, cl) for x, n_, col, cl in hi]
        if op == Op.EXTRACT:
            inner = self.segments(a, depth + 1)
            if inner is None:
                return None
            out = []
            for x, n_, col, cl in inner:
                s0, s1 = max(x, i1), min(x + n_, i0 + 1)
                if s0 < s1:
                    out.append((s0 - i1, s1 - s0, col, cl + (s0 - x)))
            return out
        if op == Op.ZEXT:
            return self.segments(a, depth + 1)
        if op == Op.BVAND:  # x & (2^k - 1): the low k bits of x (ABI decoding of addresses)
            for x, m in ((a, b.const_value(bb)), (bb, b.const_value(a))):
                if m is not None and m & (m + 1) == 0:
                    inner = self.segments(x, depth + 1)
                    if inner is None:
                        return None
                    k = m.bit_length()
                    return [(lo, min(n_, k - lo), col, cl) for lo, n_, col, cl in inner
                            if lo < k]
            return None
        if op == Op.ITE:
            if b.const_value(c) is not None:
                return self.segments(bb, depth + 1)
            if b.const_value(bb) is not None:
                return self.segments(c, depth + 1)
        return None

    def copy_alternatives(self, x: int, y: int) -> List[List[Copy]]:
        """For x == y over column bits: copy y's bits into x's columns, or x's into y's."""
        sx, sy = self.segments(x), self.segments(y)
        if not sx or not sy:
            return []
        alts = []
        for dst_side, src_side in ((sx, sy), (sy, sx)):
            copies: List[Copy] = []
            for dlo, dn, dcol, dcl in dst_side:
                for slo, sn, scol, scl in src_side:
                    s0, s1 = max(dlo, slo), min(dlo + dn, slo + sn)
                    if s0 < s1 and dcol != scol:
                        copies.append((dcol, scol, dcl + (s0 - dlo), scl + (s0 - slo), s1 - s0))
            if copies:
                alts.append(copies[:256])
        return alts

    def _hint(self, alts: List[Alt]) -> None:
        if self._cap:
            self._cap[-1].append(alts)
        key = tuple(tuple(sorted(a.items())) for a in alts)
        if key not in self._hint_keys and len(self._hint_keys) < MAX_SETS // 4:
            self._hint_keys.add(key)
            self.hints.append((PROB_HINT, [a for a in alts if a][:MAX_ALTS]))

    # -- driver ----------------------------------------------------------------------------
    def _conjuncts(self, root: int) -> List[int]:
        out, stack = [], [root]
        while stack:
            n = stack.pop()
            op = self.b.nodes[n][0]
            if op == Op.AND:
                stack += [self.b.nodes[n][3], self.b.nodes[n][2]]
            else:
                out.append(n)
        return out

    def _consts_of_width(self, w: int) -> List[int]:
        got = self._consts_by_width.get(w)
        if got is None:
            vals = sorted({v & _mask(w) for v in self.query_consts},
                          key=lambda v: (-(v.bit_length() > 8), -v.bit_length(), v))
            got = self._consts_by_width[w] = vals[:MAX_EQ_CONSTS]
        return got

    def harvest(self, root: int, parent: Optional[Alt] = None) -> Guide:
        from .tape import ARITY

        b = self.b
        nodes, pool_values = b.nodes, b.pool.values
        conjuncts = self._conjuncts(root)
        consts_of = _memo(b, "_guide_consts")
        self.query_consts = qc = set()
        for conj in conjuncts:  # the constants of this query (the pool is shared by all queries)
            got = consts_of.get(conj)
            if got is None:
                got, seen, stack = set(), set(), [conj]
                while stack:
                    n = stack.pop()
                    if n in seen:
                        continue
                    seen.add(n)
                    node = nodes[n]
                    op = node[0]
                    if op == Op.CONST:
                        got.add(pool_values[node[5]])
                    k = ARITY[op]
                    if k:
                        stack += node[2:2 + k]
                got = consts_of[conj] = frozenset(got)
            qc |= got
        alt = {k: v for k, v in parent.items() if k in self.pools} if parent else {}
        if self.parent_eval:
            self._parent = alt
        if alt:
            self.sets.append((PROB_PARENT, [alt]))
        seen_eq = set()
        eq_pairs = _memo(b, "_guide_eq")
        for conj in conjuncts:
            alts = self.invert_bool(conj, True)
            if alts and alts != [{}]:
                self.sets.append((PROB_DEFAULT, [a for a in alts if a][:MAX_ALTS]))
            # symbolic == symbolic anywhere below this conjunct: try the query's constants
            for n in self._eq_nodes(conj):
                if n in seen_eq:
                    continue
                seen_eq.add(n)
                pair = eq_pairs.get(n)
                if pair is None:  # (x, y, copy alternatives) after peeling shared wrappers
                    _, _, x, y, _, _, _ = b.nodes[n]
                    if b.widths[x] == BOOL or b.const_value(x) is not None \
                            or b.const_value(y) is not None:
                        pair = ()
                    else:
                        x, y = self.strip_common(x, y)
                        # t == t (keccak inverse conditions after lowering): always true
                        pair = () if x == y else (x, y, self.copy_alternatives(x, y))
                    eq_pairs[n] = pair
                if not pair:
                    continue
                x, y, calts = pair
                w = b.widths[x]
                if calts:
                    if len(self.copy_sets) < MAX_SETS // 4:
                        self.copy_sets.append(calts)
                    continue
                for k in self._consts_of_width(w):
                    rx = self.invert_bits(x, k, _mask(w))
                    ry = self.invert_bits(y, k, _mask(w))
                    if rx and ry:
                        both = _merge(rx, ry)
                        if both and both != [{}]:
                            self.sets.append((PROB_DEFAULT // 2, both[:MAX_ALTS]))
                if len(self.sets) >= MAX_SETS:
                    break
            if len(self.sets) >= MAX_SETS:
                break
        # bounds on one term from several conjuncts (calldatasize guards of the ABI decoder,
        # argument range checks): values inside their intersection, last, so they override the
        # single-conjunct boundary values that satisfy one bound and break another
        for t, (lo, hi, n_bounds) in self._intervals(conjuncts).items():
            if n_bounds < 2 or lo > hi or len(self.sets) >= MAX_SETS:
                continue
            out: List[Alt] = []
            for v in _interval_values(lo, hi):
                r = self.invert_bits(t, v, _mask(b.widths[t]))
                if r:
                    out += [a for a in r if a]
            if out:
                self.sets.append((PROB_DEFAULT, out[:MAX_ALTS]))
        # hints first: the exact requirements of the conjuncts (later sets) override them
        hints = _prune_hints(self.hints)
        self.sets = self.sets[:1] + hints + self.sets[1:] if alt else hints + self.sets
        pools = self.pools
        for _, alts in self.sets:
            for alt in alts:
                for name, v in alt.items():
                    p = pools[name]
                    if len(p) < MAX_POOL and v not in p:
                        p.append(v)
        widths = [self.schema.columns[c].width for c in self.columns]
        for name, w in zip(self.columns, widths):
            p = self.pools[name]
            for v in (0, 1, _mask(w), 1 << (w - 1)):
                if v not in p and len(p) < MAX_POOL:
                    p.append(v)
        # copies go last (their sources are final by then); the two directions of one
        # equality are the two alternatives of one set
        copy_sets = [(PROB_DEFAULT, alts) for alts in self.copy_sets]
        return Guide(self.columns, widths, [self.pools[c] for c in self.columns],
                     self.sets[:MAX_SETS], copy_sets[:MAX_SETS // 4])

    def _bound_of(self, n: int) -> Optional[Tuple[int, int, int]]:
        """(term, lo, hi): conjunct n bounds a symbolic term to [lo, hi] (unsigned, inclusive)
        against a constant -- ULT / ULE / UGT / UGE either way round, their negations, and the
        Or(x < k, x == k) form of smt.ULE / smt.UGE; None otherwise."""
        b = self.b
        op, w, a, bb, c, i0, i1 = b.nodes[n]
        truth = True
        if op == Op.NOT:
            truth = False
            op, w, a, bb, c, i0, i1 = b.nodes[a]
        strict_ops = {Op.BVULT: (True, True), Op.BVULE: (True, False),
                      Op.BVUGT: (False, True), Op.BVUGE: (False, False)}
        if op == Op.OR:  # Or(cmp(x, k), x == k): the non-strict comparison
            l, r = b.nodes[a], b.nodes[bb]
            if r[0] != Op.EQ or l[0] not in (Op.BVULT, Op.BVUGT) or (l[2], l[3]) != (r[2], r[3]):
                return None
            op = Op.BVULE if l[0] == Op.BVULT else Op.BVUGE
            a, bb = l[2], l[3]
        if op not in strict_ops:
            return None
        ka, kb = b.const_value(a), b.const_value(bb)
        if (ka is None) == (kb is None):
            return None
        less, strict = strict_ops[op]
        t, k = (a, kb) if kb is not None else (bb, ka)
        if kb is None:  # k op t: flip to t op' k
            less = not less
        if not truth:  # not (t < k) == t >= k
            less, strict = not less, not strict
        m = _mask(b.widths[t])
        if less:
            lo, hi = 0, k - 1 if strict else k
        else:
            lo, hi = k + 1 if strict else k, m
        return t, lo, hi

    def _intervals(self, conjuncts: Sequence[int]) -> Dict[int, Tuple[int, int, int]]:
        """Per bounded term (first-seen order): the intersection of its bounds, and their count."""
        out: Dict[int, Tuple[int, int, int]] = {}
        for cj in conjuncts:
            got = self._bound_of(cj)
            if got is None:
                continue
            t, lo, hi = got
            if t in out:
                plo, phi, n = out[t]
                out[t] = (max(lo, plo), min(hi, phi), n + 1)
            else:
                out[t] = (lo, hi, 1)
        return out

    def _eq_nodes(self, root: int, limit: int = 4096) -> List[int]:
        """Equalities anywhere under a conjunct (also inside ite conditions of bit-vector terms:
        store-chain reads lower to ite(key == stored_key, ...))."""
        from .tape import ARITY

        memo = _memo(self.b, "_guide_eq_nodes")
        got = memo.get(root)
        if got is not None:
            return got
        out, seen, stack = [], set(), [root]
        b = self.b
        memo[root] = out
        while stack and len(seen) < limit:
            n = stack.pop()
            if n in seen:
                continue
            seen.add(n)
            node = b.nodes[n]
            op = node[0]
            if op == Op.EQ:
                out.append(n)
            k = ARITY[op]
            if k:
                stack += node[2:2 + k]
        return out

    def strip_common(self, x: int, y: int) -> Tuple[int, int]:
        """Peel wrappers both sides share (same op, same constant operand, or the same other
        concat half) so that f(x') == f(y') is tried as x' == y' — the keccak interval map
        H(x) = base + ((keccak(x) >> 139) << 6) of lower.py included (a heuristic for
        candidate generation only: the witness is checked on the device)."""
        b = self.b
        for _ in range(64):
            ox, oy = b.nodes[x], b.nodes[y]
            if ox[0] != oy[0] or ox[1] != oy[1]:
                break
            op = Op(ox[0])
            if op in (Op.KECCAK, Op.BVNOT, Op.BVNEG) or (op in (Op.ZEXT, Op.SEXT)
                                                          and ox[5] == oy[5]):
                x, y = ox[2], oy[2]
                continue
            if op in (Op.BVADD, Op.BVSUB, Op.BVXOR, Op.BVSHL, Op.BVLSHR, Op.BVMUL, Op.CONCAT):
                if ox[3] == oy[3] or (b.const_value(ox[3]) is not None
                                      and b.const_value(ox[3]) == b.const_value(oy[3])):
                    x, y = ox[2], oy[2]
                    continue
                if ox[2] == oy[2] or (b.const_value(ox[2]) is not None
                                      and b.const_value(ox[2]) == b.const_value(oy[2])):
                    x, y = ox[3], oy[3]
                    continue
            break
        return x, y


def build_guide(b: TapeBuilder, root: int, schema: Schema, columns: Sequence[str],
                parent: Optional[Alt] = None, parent_eval: bool = False) -> Guide:
    return Harvester(b, schema, columns, parent_eval).harvest(root, parent)
