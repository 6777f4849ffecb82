"""The sieve engine behind ``get_model``: one path condition -> a witness, or nothing.

For one query (the tuple of Bool constraints ``Constraints.is_possible`` hands to ``get_model``,
mythril/laser/ethereum/state/constraints.py:25-35, support/model.py:15-62):

1. lower arrays / keccak UFs onto scalar columns, split the conjuncts into column-disjoint groups
   and linearise the tapes -- in one native call (mh_query_build, csrc/query.cpp; the Python
   stages lower.py / buckets / local_tapeset are its reference and the definitions path);
   unsupported constructs -> the fallback, a self-contradicting query -> no device round;
2. harvest a candidate guide from the lowered term and the parent query's witness
   (mh_guide_harvest_with, harvest.cpp -- the algorithm of candidates.py, same arrays; the
   session reuses the inversions of the path's earlier queries); the guide stays in the library;
3. compile the group tapes over the query's own columns (mh_tapes_compile; tapes compiled
   before in this context, a LASER parent's unchanged groups, come from its cache);
4. two rounds at most, each ONE call (mh_query_round: guided generator, MH_MODE_FIRST_HIT run,
   and the witness rows, one host sync): ``first_rows`` guided rows, then, when a group is still
   unsolved, the remaining ``(max_rounds - 1) * rows`` rows over the unsolved groups' tapes;
5. on a hit, the witness (column name -> value) from the row that came back with the results.

Everything on the device path raises on failure; the caller (frontend.get_model) treats any
exception as "no answer from the sieve" and asks the fallback solver, so the reference's
behaviour is kept on every error (SURVEY.md §5 "fail closed").
"""
from __future__ import annotations

import os
import threading
import time
from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import native
from .lower import (Column, KeccakMap, LoweringUnsupported, Schema, cell_name, lower_query,
                    node_columns)
from .tape import NODE_DTYPE, Op, Tape, TapeBuilder, TapeError, TapeSet


@dataclass
class Witness:
    schema: Schema
    values: Dict[str, int]             # column name -> value
    index: int = 0                     # global candidate index that satisfied the query
    rounds: int = 0


@dataclass
class SieveStats:
    queries: int = 0
    hits: int = 0
    misses: int = 0
    unsupported: int = 0
    errors: int = 0
    rounds: int = 0
    rows: int = 0
    host_s: float = 0.0
    device_s: float = 0.0
    extra: Dict[str, int] = field(default_factory=dict)
    # seconds per stage: lower, guide, tapes, compile, generate, run, download
    stage_s: Dict[str, float] = field(default_factory=dict)

    def add(self, stage: str, dt: float) -> None:
        self.stage_s[stage] = self.stage_s.get(stage, 0.0) + dt


def local_tape(b: TapeBuilder, root: int, columns: Sequence[str]) -> np.ndarray:
    """The tape of `root` with VAR columns renumbered to the query's own column order."""
    tape = b.finish(root)
    nodes = tape.nodes.copy()
    local = {b.var_index[c]: i for i, c in enumerate(columns)}
    is_var = nodes["op"] == int(Op.VAR)
    if is_var.any():
        nodes["imm0"][is_var] = [local[int(x)] for x in nodes["imm0"][is_var]]
    return nodes


class LocalPool:
    """The constants one query's tapes read, renumbered 0..k-1 (the builder's pool holds every
    constant of the run: uploading it with each query would grow with the run)."""

    def __init__(self, rows: np.ndarray):
        self.rows = rows
        self.values = range(len(rows))

    def to_array(self) -> np.ndarray:
        return self.rows


def local_tapeset(b: TapeBuilder, roots: Sequence[int], columns: Sequence[str]) -> TapeSet:
    """One tape per root over the query's own columns (VAR renumbered to `columns` order) and
    its own constant pool (CONST renumbered to the constants the tapes read)."""
    ts = TapeSet(columns)
    tapes = [b.finish(r).nodes for r in roots]
    nodes = np.concatenate(tapes) if tapes else np.zeros(0, dtype=NODE_DTYPE)
    ops, imm0 = nodes["op"], nodes["imm0"].astype(np.int64)
    is_var = ops == int(Op.VAR)
    is_const = ops == int(Op.CONST)
    new0 = imm0.copy()
    if is_var.any():
        lut = np.full(len(b.var_index), -1, dtype=np.int64)
        vi = b.var_index
        for i, c in enumerate(columns):
            v = vi.get(c)  # a column no builder term reads (a native query's cell) maps nothing
            if v is not None:
                lut[v] = i
        new0[is_var] = lut[imm0[is_var]]
        if (new0[is_var] < 0).any():
            raise ValueError("a tape reads a variable outside the query's columns")
    used = np.unique(imm0[is_const])
    new0[is_const] = np.searchsorted(used, imm0[is_const])
    nodes = nodes.copy()
    nodes["imm0"] = new0.astype(nodes["imm0"].dtype)
    ts.pool = LocalPool(np.ascontiguousarray(b.pool.to_array()[used]) if len(used)
                        else np.zeros((1, 8), dtype=np.uint32))
    off = 0
    for t in tapes:
        ts.tapes.append(Tape(nodes[off:off + len(t)]))
        off += len(t)
    return ts


REFUTED = object()  # _host_native's answer for a query that contradicts itself


class NativeDefs(list):
    """The definitions the native query compiler eliminated (MH_QUERY_DEFINITIONS):
    [(column, tape of its defining term)] over the query's columns and constants ``consts``."""

    def __init__(self, items, consts):
        super().__init__(items)
        self.consts = consts


class NativeSchema(Schema):
    """The Schema of a query the native compiler built, decoded on first use: a witness's
    schema is read only when a model is evaluated (mythril/laser/smt/model.py:45-59, model.py
    here), LASER's is_possible never reads it (constraints.py:25-35)."""

    _FIELDS = ("cells", "uf_cells", "keccak", "columns")
    # one decode at a time, process-wide (a remembered witness may be read by several threads;
    # decodes are rare and short); not on the instance, so copies and pickles see only _cq
    _DECODE_LOCK = threading.Lock()

    def __init__(self, cq: "native.CompiledQuery", keccak_reads: bool = False):  # noqa: deferred
        self.__dict__["_cq"] = cq
        self.__dict__["keccak_reads"] = keccak_reads

    def __getattr__(self, name):
        if name not in self._FIELDS:
            raise AttributeError(name)
        # the compiled query is dropped only once the Schema is complete, so a decode that
        # raises leaves the next read to try again
        with NativeSchema._DECODE_LOCK:
            if name in self.__dict__:
                return self.__dict__[name]
            if "_cq" not in self.__dict__:
                raise AttributeError(name)
            self._decode(self.__dict__["_cq"])
            del self.__dict__["_cq"]
        return self.__dict__[name]

    def _decode(self, cq) -> None:
        cols = {n: Column(n, w, k, s, key) for n, w, k, s, key in cq.columns}
        cells: Dict[str, Dict[int, str]] = {}
        uf_cells: Dict[str, Dict[int, str]] = {}
        keccak: Dict[str, KeccakMap] = {}
        for kind, name_, items in cq.tables:
            if kind == native.TABLE_KECCAK:
                keccak[name_] = KeccakMap(items[0], dict(zip(items[1::2], items[2::2])))
            else:
                (cells if kind == native.TABLE_CELLS else uf_cells)[name_] = {
                    k: cell_name(name_, k) for k in items}
        Schema.__init__(self, cells, uf_cells, keccak, cols, self.__dict__["keccak_reads"])


def substitute(b: TapeBuilder, root: int, env: Dict[int, int]) -> int:
    """`root` with every VAR whose index is in `env` replaced by env's term (a rebuild of the
    nodes above the replaced ones; hash-consing shares everything else)."""
    nodes, out = b.nodes, {}
    st = [root]
    from .tape import ARITY

    while st:
        n = st[-1]
        if n in out:
            st.pop()
            continue
        op, w, a, bb, c, i0, i1 = nodes[n]
        if op == Op.VAR:
            out[n] = env.get(i0, n)
            st.pop()
            continue
        k = ARITY[Op(op)]
        kids = (a, bb, c)[:k]
        todo = [x for x in kids if x not in out]
        if todo:
            st += todo
            continue
        st.pop()
        new = tuple(out[x] for x in kids)
        out[n] = n if new == kids else b.op(Op(op), *new, imm0=i0, imm1=i1)
    return out[root]


def eliminate_definitions(b: TapeBuilder, conj: Sequence[int], schema: Schema
                          ) -> Tuple[List[int], List[Tuple[str, int]]]:
    """Solve-for-a-symbol on the lowered conjuncts: a conjunct ``v == t`` whose one side is a
    scalar symbol ``v`` and whose other side is a computed term ``t`` over other columns (not a
    constant, not a symbol: the guide already proposes those) defines ``v``.  The definition is
    dropped and ``v`` replaced by ``t`` in every other conjunct; the query is equisatisfiable, and
    a row satisfying the rest extends to a model with ``v = t(row)``.  This is what a query like
    ``b == keccak(2 * keccak(a))`` (tests/laser/keccak_tests.py:122-138) needs: no candidate row
    guesses a 256-bit hash, but every row of ``a`` determines ``b``.

    Returns (remaining conjuncts over the other columns, [(column, defining term)]) with every
    defining term over undefined columns only."""
    kinds = schema.columns
    var_col = {b.var_index[n]: n for n, c in kinds.items() if c.kind == "var"}
    nodes = b.nodes
    env: Dict[int, int] = {}
    defs: List[Tuple[str, int]] = []
    rest: List[int] = []
    for cn in conj:
        op, _, a, bb, _, _, _ = nodes[cn]
        done = False
        if op == Op.EQ:
            for vn, t in ((a, bb), (bb, a)):
                nv = nodes[vn]
                if nv[0] != Op.VAR or nv[5] not in var_col or nv[5] in env:
                    continue
                if nodes[t][0] in (Op.VAR, Op.CONST):
                    continue
                t2 = substitute(b, t, env) if env else t
                reads = node_columns(b, [t2])[t2]
                if not reads or nv[5] in reads:
                    continue
                one = {nv[5]: t2}
                for v in list(env):  # earlier definitions may read v: keep them closed
                    env[v] = substitute(b, env[v], one)
                env[nv[5]] = t2
                defs.append((var_col[nv[5]], nv[5]))
                done = True
                break
        if not done:
            rest.append(cn)
    if not env:
        return list(conj), []
    return ([substitute(b, cn, env) for cn in rest],
            [(col, env[idx]) for col, idx in defs])


def _may_define(b: TapeBuilder, root: int) -> bool:
    """Whether a conjunct of `root` has the shape of a definition (``v == t`` with a symbol on
    one side and a computed term on the other; eliminate_definitions decides), memoised per
    node on the builder: a child query's AND node answers from its parent's."""
    memo = b.__dict__.setdefault("_may_define", {})
    got = memo.get(root)
    if got is not None:
        return got
    nodes = b.nodes
    stack, order = [root], []
    while stack:  # the AND nodes not answered yet, parents after children
        n = stack.pop()
        if n in memo:
            continue
        order.append(n)
        if nodes[n][0] == Op.AND:
            stack += [x for x in (nodes[n][2], nodes[n][3]) if x not in memo]
    for n in reversed(order):
        op, _, a, bb = nodes[n][:4]
        if op == Op.AND:
            memo[n] = memo[a] or memo[bb]
        elif op == Op.EQ:
            ka, kb = nodes[a][0], nodes[bb][0]
            memo[n] = ((ka == Op.VAR and kb not in (Op.VAR, Op.CONST))
                       or (kb == Op.VAR and ka not in (Op.VAR, Op.CONST)))
        else:
            memo[n] = False
    return memo[root]


class _Group:
    __slots__ = ("first", "idx", "conj", "vars", "acc")

    def __init__(self, first, idx, conj, vars_, acc):
        self.first, self.idx, self.conj, self.vars, self.acc = first, idx, conj, vars_, acc


class _BucketState:
    """The variable-disjoint groups of an AND chain's conjuncts, extendable by more conjuncts.
    Groups are immutable (a child state shares its parent's)."""

    def __init__(self):
        self.n = 0
        self.groups: Dict[object, _Group] = {}
        self.var_group: Dict[int, object] = {}

    def copy(self) -> "_BucketState":
        st = _BucketState()
        st.n, st.groups, st.var_group = self.n, dict(self.groups), dict(self.var_group)
        return st

    def add(self, b: TapeBuilder, cn: int, vs: frozenset) -> None:
        i = self.n
        self.n += 1
        and_ = int(Op.AND)
        if not vs:  # a ground conjunct: its own group (one per node)
            key = ("ground", cn)
            g = self.groups.get(key)
            self.groups[key] = (_Group(i, (i,), (cn,), frozenset(), cn) if g is None else
                                _Group(g.first, g.idx + (i,), g.conj + (cn,), g.vars,
                                       b._add(and_, 0, g.acc, cn)))
            return
        gids = {self.var_group[v] for v in vs if v in self.var_group}
        if not gids:
            key = ("vars", i)
            self.groups[key] = _Group(i, (i,), (cn,), vs, cn)
        elif len(gids) == 1:
            key = next(iter(gids))
            g = self.groups[key]
            self.groups[key] = _Group(g.first, g.idx + (i,), g.conj + (cn,), g.vars | vs,
                                      b._add(and_, 0, g.acc, cn))
        else:  # the conjunct joins several groups: one group, conjuncts in path order
            members = [self.groups.pop(k) for k in gids]
            pairs = sorted([p for g in members for p in zip(g.idx, g.conj)] + [(i, cn)])
            acc = pairs[0][1]
            for _, x in pairs[1:]:
                acc = b._add(and_, 0, acc, x)
            vars_ = frozenset(vs).union(*[g.vars for g in members])
            key = ("vars", min(g.first for g in members))
            self.groups[key] = _Group(pairs[0][0], tuple(p[0] for p in pairs),
                                      tuple(p[1] for p in pairs), vars_, acc)
        for v in self.groups[key].vars:
            self.var_group[v] = key

    def ordered(self) -> List[_Group]:
        return sorted(self.groups.values(), key=lambda g: g.first)


BUCKET_STATES = 256  # states of recent AND roots kept per builder


def _bucket_state(b: TapeBuilder, root: int) -> _BucketState:
    """The grouping of `root`'s conjuncts, memoised per AND root on the builder: a query that
    extends its parent (svm.py:257-262, root = AND(parent, new)) adds only its new conjunct."""
    memo = b.__dict__.setdefault("_bucket_states", OrderedDict())
    got = memo.get(root)
    if got is not None:
        memo.move_to_end(root)
        return got
    node = b.nodes[root]
    base = memo.get(node[2]) if node[0] == Op.AND else None
    if base is not None:
        st = base.copy()
        new = Sieve.conjuncts(b, node[3])
    else:
        st = _BucketState()
        new = Sieve.conjuncts(b, root)
    cols = node_columns(b, new)
    for cn in new:
        st.add(b, cn, cols[cn])
    memo[root] = st
    while len(memo) > BUCKET_STATES:
        memo.popitem(last=False)
    return st


# ops whose recomputation is cheap enough to duplicate instead of keeping a value live
_HEAVY = {Op.BVMUL, Op.BVUDIV, Op.BVUREM, Op.BVSDIV, Op.BVSREM, Op.BVSMOD, Op.KECCAK,
          Op.EVM_EXP, Op.BVMUL_NOOVFL_U, Op.EVM_ADDMOD, Op.EVM_MULMOD}


def rematerialize(nodes: np.ndarray, max_size: int) -> np.ndarray:
    """Duplicate cheap shared sub-terms (at most `max_size` nodes, no multiply / divide /
    keccak) at every use instead of keeping their values live.  A path condition reads the same
    calldata bytes in several overlapping words (calldata.py:48-54: word(0) and word(4) share 28
    byte terms), which otherwise holds more values live than the device register file has; the
    copies cost a few cheap instructions each."""
    from .tape import ARITY

    n = len(nodes)
    ops = nodes["op"].astype(int)
    opnds = np.stack([nodes["a"], nodes["b"], nodes["c"]], axis=1).astype(int)
    ar = [ARITY[Op(o)] for o in ops]
    uses = np.zeros(n, dtype=int)
    size = np.zeros(n, dtype=int)
    cheap = np.zeros(n, dtype=bool)
    for i in range(n):
        kids = opnds[i, :ar[i]]
        for k in kids:
            uses[k] += 1
        size[i] = 1 + sum(int(size[k]) for k in kids)
        cheap[i] = (Op(ops[i]) not in _HEAVY and size[i] <= max_size
                    and all(cheap[k] for k in kids) and nodes["width"][i] <= 256)
    dup = cheap & (uses > 1)
    out: List[tuple] = []
    remap = {}

    def copy(k: int, deep: bool) -> int:
        # inside a duplicated sub-term every cheap node is copied too, so copies share nothing
        kids = [copy(int(x), True) if cheap[x] and (deep or dup[x]) else remap[int(x)]
                for x in opnds[k, :ar[k]]]
        rec = list(nodes[k].tolist())
        for j, x in enumerate(kids):
            rec[3 + j] = x
        out.append(tuple(rec))
        return len(out) - 1

    for i in range(n):
        if dup[i] and i != n - 1:
            continue
        remap[i] = copy(i, False)
    return np.array(out, dtype=nodes.dtype)


class Sieve:
    """A device context plus reusable buffers; one per thread (handles are not shared)."""

    def __init__(self, device: int = 0, rows: int = 1 << 16, max_rounds: int = 2,
                 seed: int = 0x5EED5EED, budget_s: float = 0.25, first_rows: Optional[int] = None,
                 native_query: bool = True, second_round: Optional[str] = None,
                 keccak_second_chance: Optional[bool] = None):
        self.ctx = native.Context(device)
        # host stages by the native query compiler (csrc/query.cpp); False: the Python stages
        # (lower.py, buckets, local_tapeset) it is checked against (tests/test_query_native.py)
        self.native_query = native_query
        # guide harvests that reuse the memo of the path's earlier queries (mh_harvester)
        self.guides = native.GuideSession()
        self.guides_kr: Optional[native.GuideSession] = None  # the second chance's (made on use)
        self.rows = rows
        # the harvested guide usually solves a LASER query in its first rows (round 1 found every
        # SAT witness of tests/laser_like.py within the first 16 rows): a small first round
        # answers those at a fraction of the latency, the full-size rounds follow.  4096 rows
        # (64 waves, one per SIMD of 64 CUs) take the 256-row round's time -- a short round is
        # latency-bound per wave -- and find in round 1 most of what round 2 found after 256
        # (planted random paths: 179 -> 60 round-2-only hits, profiles/r05g)
        if first_rows is None:  # SIEVE_FIRST_ROWS overrides the default (measurements)
            first_rows = int(os.environ.get("SIEVE_FIRST_ROWS", "4096"))
        self.first_rows = min(first_rows, rows)
        # a miss pays every round before z3 runs (an infeasible JUMPI branch, svm.py:257-262):
        # one 2^16-row round after the guided 256 keeps a miss near 1 ms of device time
        # (profiles/r03f: three such rounds took 1.6-2.3 ms) while no LASER-shaped SAT query
        # needed more than the first 256 rows
        self.max_rounds = max_rounds
        # when the rounds after the first run (SIEVE_ROUND2 overrides): "always"; "progress" --
        # only when the first round solved some of the query's groups but not all (a query
        # whose first round found nothing at all is left to the fallback at once); "never".
        # Default "progress": a first round that solves no group is almost always an UNSAT query
        # (EtherThief's UNSAT variant: 0.73 -> 0.45 ms, 400 constraints 2.48 -> 1.78 ms) and
        # the planted-SAT paths lose 2 of 2449 LASER-family answers (profiles/r05h)
        self.second_round = second_round or os.environ.get("SIEVE_ROUND2", "progress")
        if self.second_round not in ("always", "progress", "never"):
            raise ValueError("second_round must be always / progress / never")
        # a query the first lowering missed while an unsolved group read a keccak application
        # (fixed there at H(x), lower.py) is lowered again with keccak applications as read
        # columns (lower_query keccak_reads, MH_TERMS_KECCAK_READS) and given one more first
        # round: a path that pins keccak values elsewhere than H (VERDICT r5 missing 2; DESIGN
        # §6).  SIEVE_KECCAK2=0 turns it off (measurements)
        if keccak_second_chance is None:
            keccak_second_chance = os.environ.get("SIEVE_KECCAK2", "1") != "0"
        self.keccak_second_chance = keccak_second_chance
        # the second round of a query whose parent has a witness: the parent's witness under
        # the newest root's conjuncts (SIEVE_INCREMENTAL=0: the 2^16-row full-guide round)
        self.incremental_round = os.environ.get("SIEVE_INCREMENTAL", "1") != "0"
        # its rows: 16384 (256 one-wave workgroups, one per CU: a round's latency-bound cost
        # barely moves) answered 1.5 points more of the random family than 4096, LASER-shaped
        # latency unchanged (profiles/r06s)
        self.inc_rows = int(os.environ.get("SIEVE_INC_ROWS", "16384"))
        self.inc_hops = int(os.environ.get("SIEVE_INC_HOPS", "0"))  # newest_tape(hops)
        # its guide solving for one side of x op y == k with the other at the parent's value
        # (mh_guide_harvest_inc, SIEVE_INC_PEVAL=1): measured, not kept -- random recall 0.6686
        # -> 0.6625, learnt 0.9183 -> 0.9107 (profiles/r06v): its extra sets override the
        # parent's values in more rows than they complete
        self.inc_parent_eval = os.environ.get("SIEVE_INC_PEVAL", "0") == "1"
        # after the incremental round, the 2^16-row round of the full guide (SIEVE_ROUND3=1)
        self.round3 = os.environ.get("SIEVE_ROUND3", "0") == "1"
        # the last solve's rounds (diagnostics: scripts/planted_recall.py)
        self.last_rounds: Dict[str, int] = {}
        self.seed = seed
        self.budget_s = budget_s
        self.assign: Optional[native.Assignments] = None
        self.stats = SieveStats()
        self.witnesses: "OrderedDict[tuple, Dict[str, int]]" = OrderedDict()
        self.max_witnesses = 1 << 14
        # the last query this sieve missed after a device round, (key, schema): a model the
        # fallback then finds for it is learnt as its witness (learn)
        # (key, schema[, the keccak second chance's schema])
        self.last_miss: Optional[tuple] = None
        # the tape compile runs on the context's worker thread (mh_tapes_compile_async) while
        # this one harvests the guide: the harvest is host-only, both only read the query's
        # tapes, and the round needs both (SIEVE_OVERLAP=0: one after the other)
        self.overlap = os.environ.get("SIEVE_OVERLAP", "1") != "0"

    def close(self) -> None:
        if self.assign is not None:
            self.assign.close()
            self.assign = None
        self.guides.close()
        if self.guides_kr is not None:
            self.guides_kr.close()
        self.ctx.close()


    def _buffer(self, n_cols: int) -> native.Assignments:
        rows = max(self.first_rows, (self.max_rounds - 1) * self.rows)
        if self.assign is None or self.assign.n_vars < n_cols or self.assign.capacity < rows:
            if self.assign is not None:
                self.assign.close()
            cap = max(n_cols, 64)
            cap = 1 << (cap - 1).bit_length()
            self.assign = self.ctx.assignments(cap, rows)
        return self.assign

    def remember(self, key: tuple, w: Witness) -> None:
        self._store(key, w.values)

    def _store(self, key: tuple, values: Dict[str, int]) -> None:
        self.witnesses[key] = values
        self.witnesses.move_to_end(key)
        while len(self.witnesses) > self.max_witnesses:
            self.witnesses.popitem(last=False)

    def learn(self, key: tuple, value_of: Callable[[Column], Optional[int]], ctx=None,
              value_at: Optional[Callable[[Column, int], Optional[int]]] = None) -> int:
        """A model the fallback found for the query this sieve missed last (the same ``key``)
        becomes that query's remembered witness, so the query's LASER children are generated
        around it as around a witness of the sieve's own (svm.py:257-262: the children of a state
        z3 found feasible are asked next).  Without it one miss leaves every later query of the
        path without parent-guided rows.  ``value_of(column)`` is the model's value of a column
        (lower.Column: a variable, an array or function cell), None where the model does not fix
        it.  With the query's term context ``ctx`` and ``value_at(column, index)``, the read
        columns (arrays, functions and keccak at symbolic index terms) are learnt too: their index
        terms are evaluated on the device over what was learnt so far (a read inside an index term
        is learnt on the next pass).  Returns the number of columns learnt."""
        lm, self.last_miss = self.last_miss, None
        if not key or lm is None or lm[0] != key:
            return 0
        values: Dict[str, int] = {}
        # the columns of both lowerings the miss tried (the keccak second chance's reads too:
        # a child's second chance is then generated around the model's keccak values)
        for sc in lm[1:]:
            for name, col in sc.columns.items():
                if name in values:
                    continue
                try:
                    v = value_of(col)
                except Exception:  # noqa: BLE001 - a column the model cannot evaluate stays free
                    v = None
                if v is not None:
                    values[name] = int(v) & ((1 << col.width) - 1)
        if ctx is not None and value_at is not None:
            self._learn_reads(lm[1:], values, ctx, value_at)
        if values:
            self._store(key, values)
            self.stats.extra["learnt"] = self.stats.extra.get("learnt", 0) + 1
        return len(values)

    def _learn_reads(self, schemas, values: Dict[str, int], ctx, value_at) -> None:
        """Sieve.learn's read columns: each index term evaluated over the values learnt so far
        (Model._evaluate, one device batch per pass), the model's value there; three passes at
        most (a read whose index reads another read)."""
        from .lower import READ_KINDS
        from .model import Model

        for sc in schemas:
            reads = [c for c in sc.columns.values() if c.kind in READ_KINDS]
            for _ in range(3):
                todo = [c for c in reads if c.name not in values]
                if not todo:
                    break
                try:
                    at = Model(self, ctx, sc, dict(values), 0)._evaluate(
                        [c.key for c in todo], [], True)
                except Exception:  # noqa: BLE001 - learning is best effort
                    return
                got = 0
                for c in todo:
                    idx = at.get(c.key)
                    if not isinstance(idx, int):
                        continue
                    try:
                        v = value_at(c, idx)
                    except Exception:  # noqa: BLE001
                        v = None
                    if v is not None:
                        values[c.name] = int(v) & ((1 << c.width) - 1)
                        got += 1
                if not got:
                    break

    def compile(self, ts: TapeSet) -> native.CompiledTapes:
        """Compile a query's tapes; a tape that runs out of registers is retried with cheap
        sub-terms duplicated at their uses (rematerialize), widening what counts as cheap."""
        import re

        from .tape import Tape

        orig = [t.nodes for t in ts.tapes]
        level = [0] * len(orig)
        sizes = (0, 8, 32, 256)
        while True:
            try:
                return self.ctx.compile(ts)
            except native.Unsupported as e:
                m = re.search(r"tape (\d+): register pressure", str(e))
                if not m:
                    raise
                t = int(m.group(1))
                level[t] += 1
                if level[t] >= len(sizes):
                    raise
                ts.tapes[t] = Tape(rematerialize(orig[t], sizes[level[t]]))
                ts.flat = None  # the tapes no longer lie back to back
                k = "remat_%d" % sizes[level[t]]
                self.stats.extra[k] = self.stats.extra.get(k, 0) + 1

    @staticmethod
    def conjuncts(b: TapeBuilder, root: int) -> List[int]:
        """The leaves of `root`'s AND tree, left to right."""
        conj, stack = [], [root]
        while stack:
            n = stack.pop()
            if b.nodes[n][0] == Op.AND:
                stack += [b.nodes[n][3], b.nodes[n][2]]
            else:
                conj.append(n)
        return conj

    def solve_definitions(self, b: TapeBuilder, root: int, schema: Schema
                          ) -> Tuple[int, List[Tuple[str, int]]]:
        """`root` with its definitions eliminated (eliminate_definitions), and the definitions.
        A root whose conjuncts hold no candidate definition (memoised per AND node) is returned
        as it is without a walk over its conjuncts."""
        if not _may_define(b, root):
            return root, []
        conj = self.conjuncts(b, root)
        rest, defs = eliminate_definitions(b, conj, schema)
        if not defs:
            return root, []
        self.stats.extra["definitions"] = self.stats.extra.get("definitions", 0) + len(defs)
        if not rest:
            return b.true(), defs
        acc = rest[0]
        for x in rest[1:]:
            acc = b.op(Op.AND, acc, x)
        return acc, defs

    def eval_terms(self, b: TapeBuilder, terms: Sequence[int], columns: Sequence[str],
                   values: Dict[str, int], resident: Optional[dict] = None) -> List[int]:
        """The values of `terms` (bit-vector or Bool nodes over `columns`) under one assignment,
        evaluated on the device (mh_eval_values_many over a one-row buffer; `resident`, a dict
        the caller keeps, holds that buffer per column tuple across calls)."""
        return self.eval_tapeset(local_tapeset(b, terms, columns), columns, values, resident)

    def eval_definitions(self, b: TapeBuilder, defs, columns: Sequence[str],
                         values: Dict[str, int]) -> List[int]:
        """The defined columns' values under the witness row: the native compiler's definition
        tapes (NativeDefs), or the Python stages' terms."""
        if isinstance(defs, NativeDefs):
            ts = TapeSet(columns)
            ts.pool = LocalPool(defs.consts)
            ts.tapes = [Tape(t) for _, t in defs]
            return self.eval_tapeset(ts, columns, values)
        return self.eval_terms(b, [t for _, t in defs], columns, values)

    def eval_tapeset(self, ts: TapeSet, columns: Sequence[str], values: Dict[str, int],
                     resident: Optional[dict] = None) -> List[int]:
        """The root values of every tape of `ts` under one assignment of `columns`."""
        terms = ts.tapes
        ct = self.compile(ts)
        try:
            key = tuple(columns)
            assign = resident.get(key) if resident is not None else None
            if assign is None:
                assign = self.ctx.assignments(len(columns), 1)
                soa = np.zeros((len(columns), 8, 1), dtype=np.uint32)
                for i, c in enumerate(columns):
                    v = values.get(c, 0)
                    for k in range(8):
                        soa[i, k, 0] = (v >> (32 * k)) & 0xFFFFFFFF
                assign.upload(soa)
                if resident is not None:
                    resident[key] = assign
            try:
                # every root in one batch (mh_eval_values_many: one launch per register class)
                out = native.eval_values_many(self.ctx, ct, list(range(len(terms))), assign, 0)
                return [_limbs(out[i]) for i in range(len(terms))]
            finally:
                if resident is None:
                    assign.close()
        finally:
            ct.close()

    def _host_native(self, b: TapeBuilder, roots: Sequence[int], keccak_reads: bool = False):
        """The host stages by the native query compiler (mh_query_build: lowering, groups and
        tapes in one call, csrc/query.cpp); None for a query with a candidate definition (those
        take _host_python, whose eliminate_definitions solves for the symbol); REFUTED for a
        conjunction that contradicts itself syntactically (MH_QUERY_REFUTED: x == 1 and x == 2,
        p and not p, bounds with an empty range), which no row can satisfy."""
        t0 = time.perf_counter()
        st = self.stats
        try:
            cq = native.TermMirror.of(b, keccak_reads).build(b, roots)
        except native.Unsupported:
            # a shape the native compiler refuses (a variable named like an array cell, ...):
            # the Python stages it restates may still take it
            st.extra["native_unsupported"] = st.extra.get("native_unsupported", 0) + 1
            st.add("lower", time.perf_counter() - t0)
            return None
        st.add("lower", time.perf_counter() - t0)
        if cq.flags & native.QUERY_REFUTED:
            st.extra["refuted"] = st.extra.get("refuted", 0) + 1
            return REFUTED
        columns = cq.names
        defs = []
        if cq.flags & native.QUERY_DEFINITIONS:  # solved for the defined symbols natively
            st.extra["definitions"] = st.extra.get("definitions", 0) + len(cq.defs)
            defs = NativeDefs([(columns[c], t) for c, t in zip(cq.defs, cq.def_tapes)],
                              cq.consts)
        ts = TapeSet(columns)
        ts.pool = LocalPool(cq.consts)
        tapes = cq.tapes
        ts.tapes = [Tape(t) for t in (tapes if len(tapes) == 1 else tapes[1:])]
        # the group tapes already lie back to back (tapes 1.., or the one tape): no concatenation
        k = 0 if len(tapes) == 1 else 1
        off = np.asarray(cq.tape_off[k:], dtype=np.uint64)
        ts.flat = (cq.nodes[cq.tape_off[k]:cq.tape_off[-1]], off - off[0], cq.consts)
        if len(cq.groups) > 1:
            st.extra["bucketed"] = st.extra.get("bucketed", 0) + 1
        return (columns, cq.widths, NativeSchema(cq, keccak_reads), tapes[0], ts, cq.groups, defs,
                [] if defs else cq.root_ends)

    def _host_python(self, b: TapeBuilder, roots: Sequence[int], keccak_reads: bool = False):
        """The host stages in Python: lower_query, definitions, buckets, local tapes."""
        t0 = time.perf_counter()
        st = self.stats
        root, schema = lower_query(b, roots, keccak_reads=keccak_reads)
        t_l = time.perf_counter()
        st.add("lower", t_l - t0)
        columns = list(schema.columns)
        if not columns:  # ground query: one row decides it
            columns = ["__ground__"]
            b.var("__ground__", 1)
            from .lower import Column

            schema.columns["__ground__"] = Column("__ground__", 1, "var", "__ground__")
        root, defs = self.solve_definitions(b, root, schema)
        groups = self.bucket_roots(b, root)
        col_of = {b.var_index[c]: i for i, c in enumerate(columns)}
        group_cols = [[col_of[v] for v in vs] for _, vs in groups]
        accs = [acc for acc, _ in groups]
        # the guide is harvested natively from the root's tape: the one tape of a query whose
        # conjuncts share columns (the same AND chain), else an extra tape of the same tape set
        # (same constants), not compiled
        if accs == [root]:
            ts = local_tapeset(b, accs, columns)
            root_nodes = ts.tapes[0].nodes
        else:
            ts = local_tapeset(b, [root] + accs, columns)
            root_nodes = ts.tapes.pop(0).nodes
        if len(groups) > 1:
            st.extra["bucketed"] = st.extra.get("bucketed", 0) + 1
        st.add("tapes", time.perf_counter() - t_l)
        widths = [schema.columns[c].width for c in columns]
        return columns, widths, schema, root_nodes, ts, group_cols, defs, []

    @classmethod
    def buckets(cls, b: TapeBuilder, root: int) -> List[Tuple[List[int], set]]:
        """Variable-disjoint groups of the conjuncts of `root` (the DependenceMap of
        laser/smt/solver/independence_solver.py:38-83, over lowered columns): [(conjunct nodes,
        column var indices)], in order of each group's first conjunct.  Groups share no column,
        so each can take its witness from a different candidate row."""
        return [(list(g.conj), set(g.vars)) for g in _bucket_state(b, root).ordered()]

    @staticmethod
    def bucket_roots(b: TapeBuilder, root: int) -> List[Tuple[int, List[int]]]:
        """Per group of ``buckets``: (the AND of its conjuncts in order, its var indices)."""
        return [(g.acc, list(g.vars)) for g in _bucket_state(b, root).ordered()]

    def solve(self, b: TapeBuilder, roots: Sequence[int], key: Optional[tuple] = None,
              budget_s: Optional[float] = None) -> Optional[Witness]:
        """A witness of the conjunction of Bool nodes `roots` of builder `b`, or None.
        ``budget_s`` (get_model's remaining solver budget) caps this query's rounds below the
        sieve's own ``self.budget_s``; no round starts once it is spent.  A miss whose unsolved
        groups read a keccak application is tried once more with keccak applications as read
        columns (``keccak_second_chance``)."""
        t0 = time.perf_counter()
        budget = self.budget_s if budget_s is None else min(self.budget_s, budget_s)
        self.stats.queries += 1
        self.last_rounds = {}
        self.last_miss = None
        if budget <= 0:
            self.stats.misses += 1
            return None
        st = self.stats
        w, schema, kec = self._attempt(b, roots, key, budget, t0, False)
        schema2 = None
        if (w is None and kec and self.keccak_second_chance
                and time.perf_counter() - t0 < budget):
            st.extra["keccak2_tries"] = st.extra.get("keccak2_tries", 0) + 1
            first = self.last_rounds
            try:
                w, schema2, _ = self._attempt(b, roots, key, budget, t0, True,
                                              base_schema=schema)
            except (LoweringUnsupported, native.Unsupported):
                # a shape the second lowering cannot take (register pressure of its larger
                # tapes, ...): the first attempt's miss stands
                st.extra["keccak2_unsupported"] = st.extra.get("keccak2_unsupported", 0) + 1
                w = None
            self.last_rounds = dict(first, keccak2=int(w is not None))
            if w is not None:
                st.extra["keccak2_hits"] = st.extra.get("keccak2_hits", 0) + 1
        if w is None:
            self.stats.misses += 1
            if schema is not REFUTED and key:
                self.last_miss = ((key, schema) if schema2 is None or schema2 is REFUTED
                                  else (key, schema, schema2))
            return None
        if key:
            self.remember(key, w)
        self.stats.hits += 1
        return w

    def _guide_session(self, keccak_reads: bool) -> "native.GuideSession":
        """The harvester session of a lowering mode (each keeps its own path's memo)."""
        if not keccak_reads:
            return self.guides
        if self.guides_kr is None:
            self.guides_kr = native.GuideSession()
        return self.guides_kr

    # how far up a path Sieve._ancestor looks for a witness: 1, the parent.  Looking 8 up (past a
    # missed parent) answered 13 instead of 8 queries after a miss on the planted random family
    # (recall 0.651 either way) and took its misses from 1.32 to 2.24 ms (p50; profiles/r06l):
    # under the plugin a missed parent has the fallback's model learnt anyway
    ANCESTORS = int(os.environ.get("SIEVE_ANCESTORS", "1"))

    def _ancestor(self, key: Optional[tuple], root_ends: Sequence[int]):
        """(witness, root-tape nodes of its query) of the nearest of the query's last ANCESTORS
        prefixes that has a witness -- the parent, or past a missed parent the state above it
        (its children are then searched around the last model the path had) -- or (None, 0)."""
        if not key:
            return None, 0
        for j in range(len(key) - 1, max(len(key) - 1 - self.ANCESTORS, 0), -1):
            w = self.witnesses.get(key[:j])
            if w is not None:
                return w, (root_ends[j - 1] if j - 1 < len(root_ends) else 0)
        return None, 0

    def _parent_kreads(self, b: TapeBuilder, schema: Schema, base_schema: Schema,
                       parent: Dict[str, int]) -> Dict[str, int]:
        """The parent's witness with the keccak read columns of `schema` (the second chance's
        lowering) it lacks -- a witness of the default lowering has none -- at the values the
        default lowering gives those applications under it (the stated pair or H(x),
        `base_schema`; one device batch).  The incremental round's parent rows then satisfy
        the parent's keccak conjuncts too."""
        from copy import deepcopy

        from .lower import Lowering, LoweringUnsupported

        need = [c for c in schema.columns.values()
                if c.kind == "kread" and c.name not in parent]
        if not need:
            return parent
        try:
            sc = deepcopy(base_schema)
            L = Lowering(b, sc)
            terms = [L.lower(b.apply(c.symbol, b.widths[c.key], 256, c.key)) for c in need]
            vals = self.eval_terms(b, terms, list(sc.columns) or ["__ground__"], parent)
        except (LoweringUnsupported, native.Unsupported, TapeError):
            return parent
        out = dict(parent)
        for c, v in zip(need, vals):
            out[c.name] = v
        self.stats.extra["parent_kreads"] = self.stats.extra.get("parent_kreads", 0) + 1
        return out

    def _attempt(self, b: TapeBuilder, roots: Sequence[int], key: Optional[tuple],
                 budget: float, t0: float, keccak_reads: bool,
                 base_schema: Optional[Schema] = None):
        """One lowering of the query and its rounds: (witness or None, schema or REFUTED,
        whether a group left unsolved reads a keccak application).  ``base_schema``: the
        default lowering's schema, for the second chance's incremental round."""
        st = self.stats
        th = time.perf_counter()
        host = self._host_native(b, roots, keccak_reads) if self.native_query else None
        if host is REFUTED:  # no witness exists: no device round (the fallback still runs)
            self.stats.host_s += time.perf_counter() - th
            return None, REFUTED, False
        if host is None:
            host = self._host_python(b, roots, keccak_reads)
        columns, widths, schema, root_nodes, ts, group_cols, defs, root_ends = host
        t_t = time.perf_counter()
        pending = None
        try:  # from the compile's start: an error on this side still collects it
            if self.overlap and hasattr(self.ctx, "compile_async"):
                pending = self.ctx.compile_async(ts)
            col_index = {c: i for i, c in enumerate(columns)}
            parent, parent_len = self._ancestor(key, root_ends)
            guide = native.harvest_guide(
                root_nodes, ts.pool.to_array(), widths,
                [(col_index[k], v) for k, v in parent.items() if k in col_index] if parent else (),
                session=self._guide_session(keccak_reads), keep=True)  # kept for the rounds
        except BaseException:
            if pending is not None:  # the compile's tapes are not needed
                try:
                    pending.wait().close()
                except Exception:  # noqa: BLE001 - the harvest's error is the one to report
                    pass
            raise
        t1 = time.perf_counter()
        st.add("guide", t1 - t_t)
        self.stats.host_s += t1 - th
        try:
            ct = None
            if pending is not None:
                try:
                    ct = pending.wait()
                except native.Unsupported:  # register pressure: Sieve.compile's retries
                    ct = None
                if ct is not None:  # its own duration; the part the harvest did not hide
                    st.add("compile", ct.timing[1])
                    st.add("compile_wait", time.perf_counter() - t1)
            if ct is None:
                ct = self.compile(ts)
                st.add("compile", time.perf_counter() - t1)
        except BaseException:
            guide.close()
            raise
        t_c = time.perf_counter()
        round_guide = guide  # the incremental round's own guide replaces it (closed below)
        inc_guide = None
        ft, nt = getattr(ct, "timing", (0.0, 0.0))
        st.add("compile_flatten", ft)
        st.add("compile_native", nt)
        try:
            assign = self._buffer(len(columns))
            values: Dict[str, int] = {}
            solved = [False] * len(group_cols)
            first_index = None
            offset = (1 << 23) if keccak_reads else 0
            # the incremental round: the parent's witness under the newest root's conjuncts'
            # sets only (the parent's conjuncts hold there already), instead of the 2^16-row
            # round of the full guide -- a child whose own conjunct the full guide's rows keep
            # breaking while they break the parent's
            inc_ok = bool(parent) and parent_len > 0 and self.incremental_round
            launches = [self.first_rows]
            if self.max_rounds > 1:
                launches.append(min(self.inc_rows, self.rows) if inc_ok
                                else (self.max_rounds - 1) * self.rows)
            self.last_rounds = {"groups": len(group_cols), "r1_solved": 0, "rounds": 0}
            if keccak_reads and not inc_ok:  # the second chance: one first round
                launches = launches[:1]
            if inc_ok and self.round3 and self.max_rounds > 1 and not keccak_reads:
                launches.append((self.max_rounds - 1) * self.rows)  # then the full guide's
            for rnd, n in enumerate(launches):
                if rnd == 2:
                    round_guide = guide
                if rnd == 1:
                    k = sum(solved)
                    self.last_rounds["r1_solved"] = k
                    if self.second_round == "never" or (self.second_round == "progress"
                                                        and k == 0):
                        self.stats.extra["round2_skipped"] = \
                            self.stats.extra.get("round2_skipped", 0) + 1
                        break
                    if inc_ok:
                        ti = time.perf_counter()
                        inc = newest_tape(root_nodes, parent_len, self.inc_hops)
                        if inc is None:
                            break
                        pv = parent
                        if keccak_reads and base_schema is not None \
                                and base_schema is not REFUTED:
                            pv = self._parent_kreads(b, schema, base_schema, parent)
                        round_guide = inc_guide = native.harvest_guide(
                            inc, ts.pool.to_array(), widths,
                            [(col_index[k], v) for k, v in pv.items() if k in col_index],
                            keep=True, parent_eval=self.inc_parent_eval)
                        st.add("guide", time.perf_counter() - ti)
                        st.extra["inc_rounds"] = st.extra.get("inc_rounds", 0) + 1
                        self.last_rounds["incremental"] = 1
                self.last_rounds["rounds"] = rnd + 1
                base = (self.stats.queries << 24) + offset
                offset += n
                tb = time.perf_counter()
                # a later round runs only the tapes from the first to the last unsolved group
                g0 = solved.index(False)
                g1 = len(solved) - solved[::-1].index(False)
                # generator, run, and the first witnesses with their rows' columns in one call and
                # one copy back (mh_query_round)
                fh, _, wrows = native.query_round(self.ctx, ct, assign, round_guide, self.seed,
                                                  base, n, len(columns), tape_first=g0,
                                                  tape_count=g1 - g0,
                                                  mode=native.MODE_FIRST_HIT)
                tr = time.perf_counter()
                st.add("run", tr - tb)
                self.stats.rounds += 1
                self.stats.rows += n
                for i, hit in enumerate(fh.tolist()):
                    g = g0 + i
                    if solved[g] or hit == native.NO_HIT:
                        continue
                    # the row's columns as 32 little-endian bytes each
                    raw = np.ascontiguousarray(wrows[i], dtype="<u4").tobytes()
                    for c in group_cols[g]:
                        values[columns[c]] = int.from_bytes(raw[32 * c:32 * c + 32], "little")
                    solved[g] = True
                    first_index = hit if first_index is None else min(first_index, hit)
                if all(solved):
                    for c in columns:  # columns no conjunct reads: any value is a model
                        values.setdefault(c, 0)
                    if defs:  # defined symbols take their terms' values under the row
                        td = time.perf_counter()
                        got = self.eval_definitions(b, defs, columns, values)
                        for (c, _), v in zip(defs, got):
                            values[c] = v
                        st.add("definitions", time.perf_counter() - td)
                    if rnd and inc_ok:
                        st.extra["inc_hits"] = st.extra.get("inc_hits", 0) + 1
                    return Witness(schema, values, first_index, rnd + 1), schema, False
                if time.perf_counter() - t0 > budget:
                    break
            kec = any(not solved[g] and _reads_keccak(ts.tapes[g].nodes)
                      for g in range(len(solved)))
            return None, schema, kec
        finally:
            ct.close()
            guide.close()
            if inc_guide is not None:
                inc_guide.close()
            self.stats.device_s += time.perf_counter() - t1


def newest_tape(nodes: np.ndarray, parent_len: int, hops: int = 0) -> Optional[np.ndarray]:
    """The conjunction of the conjuncts a query's root tape adds to an ancestor's: the tape of
    ``AND(...AND(parent, c1)..., ck)`` lists the parent's root tape first (linearised root by
    root, query.cpp), ending in the parent's root at ``parent_len - 1``; the right operands of
    the AND chain above it are the new conjuncts (the newest constraint's lowering and its
    congruence conjuncts).  Their AND, re-linearised over the same columns and constants;
    None when there is none.  The guide harvested from it (the parent's witness under the newest
    conjuncts' sets only) is Sieve.solve's incremental round.  ``hops`` = 1 puts the parent's
    conjuncts that read a column a new conjunct reads in front of them (their sets re-satisfy
    what the new conjuncts' sets break; measured, SIEVE_INC_HOPS)."""
    n = len(nodes)
    if parent_len <= 0 or parent_len >= n:
        return None
    op, a, bb, cc = nodes["op"], nodes["a"], nodes["b"], nodes["c"]
    AND = int(Op.AND)
    # down the root's AND chain to the parent's root (the last prefix node): the right operands
    # on the way are the new conjuncts (a hash-consed one may be a node of the prefix), each
    # flattened into its AND leaves
    tops, x = [], n - 1
    while x >= parent_len and op[x] == AND:
        tops.append(int(bb[x]))
        x = int(a[x])
    if x != parent_len - 1 or not tops:
        return None
    leaves = []
    for top in reversed(tops):
        stack = [top]
        while stack:
            y = stack.pop()
            if op[y] == AND:
                stack += [int(bb[y]), int(a[y])]
            else:
                leaves.append(y)
    if hops:
        leaves = _column_neighbours(nodes, parent_len - 1, leaves) + leaves
    from .tape import ARITY

    ar = {int(o): ARITY[o] for o in Op}
    remap: Dict[int, int] = {}
    out: List[np.void] = []
    for leaf in leaves:
        st = [(leaf, False)]
        while st:
            x, done = st.pop()
            if x in remap:
                continue
            k = ar[int(op[x])]
            kids = (int(a[x]), int(bb[x]), int(cc[x]))[:k]
            if not done:
                st.append((x, True))
                st += [(y, False) for y in reversed(kids) if y not in remap]
                continue
            y = nodes[x].copy()
            for f, kid in zip(("a", "b", "c"), kids):
                y[f] = remap[kid]
            remap[x] = len(out)
            out.append(y)
    acc = remap[leaves[0]]
    for leaf in leaves[1:]:
        y = np.zeros((), dtype=nodes.dtype)
        y["op"], y["a"], y["b"] = AND, acc, remap[leaf]
        acc = len(out)
        out.append(y)
    return np.array(out, dtype=nodes.dtype)


def _column_neighbours(nodes: np.ndarray, parent_root: int, leaves: List[int]) -> List[int]:
    """The AND leaves under `parent_root` that read a column one of `leaves` reads."""
    op, a, bb, cc, i0 = nodes["op"], nodes["a"], nodes["b"], nodes["c"], nodes["imm0"]
    from .tape import ARITY

    ar = {int(o): ARITY[o] for o in Op}
    VAR, AND = int(Op.VAR), int(Op.AND)

    def cols(root: int) -> set:
        out, seen, st = set(), set(), [root]
        while st:
            x = st.pop()
            if x in seen:
                continue
            seen.add(x)
            o = int(op[x])
            if o == VAR:
                out.add(int(i0[x]))
                continue
            st += [int(y) for y in (a[x], bb[x], cc[x])[:ar[o]]]
        return out

    want = set()
    for leaf in leaves:
        want |= cols(leaf)
    pl, st = [], [parent_root]
    while st:
        y = st.pop()
        if int(op[y]) == AND:
            st += [int(bb[y]), int(a[y])]
        else:
            pl.append(y)
    return [y for y in pl if cols(y) & want]


def _reads_keccak(nodes) -> bool:
    """A tape applies keccak (the default lowering's H(x), lower.py)."""
    ops = nodes["op"] if isinstance(nodes, np.ndarray) else [n[0] for n in nodes]
    return bool(np.any(np.asarray(ops) == int(Op.KECCAK)))


def _limbs(col: np.ndarray) -> int:
    return sum(int(x) << (32 * k) for k, x in enumerate(col))
