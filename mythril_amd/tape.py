"""Tape IR: flattened z3 QF_BV / Bool terms as the sieve consumes them.

A *tape* is one path-constraint term (normally the conjunction handed to
``get_model``, mythril/support/model.py:15-62) flattened into a topologically
ordered node list; every node names its operands by tape-local index and the
last node is the root.  The node layout is ``mh_node`` of include/mythril_hip.h
(24 bytes).  Terms are hash-consed while a tape is built, so the DAG sharing z3
keeps (calldata concat chains, keccak conditions repeated across constraints) is
kept instead of being unrolled into a tree.

Sorts: ``width == 0`` is Bool, ``1..512`` a bit-vector.  The node kinds and the
reference construction that produces each one are tabulated in DESIGN.md
(§Tape IR) and in SURVEY.md §2.1.
"""
from __future__ import annotations

import enum
import struct
from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

BOOL = 0
MAX_WIDTH = 1088  # 136 bytes: one Keccak block
FINISH_CACHE = 256  # tapes of recent AND roots kept per builder (TapeBuilder.finish) ...
FINISH_CACHE_NODES = 1 << 20  # ... holding at most this many nodes in all (each entry keeps a
                              # node -> index map and the tape: a bound on memory, not entries)


class Op(enum.IntEnum):
    CONST = 0
    VAR = 1
    TRUE = 2
    FALSE = 3
    BVADD = 10
    BVSUB = 11
    BVMUL = 12
    BVUDIV = 13
    BVUREM = 14
    BVSDIV = 15
    BVSREM = 16
    BVSMOD = 17
    BVNEG = 18
    BVNOT = 19
    BVAND = 20
    BVOR = 21
    BVXOR = 22
    BVSHL = 23
    BVLSHR = 24
    BVASHR = 25
    EQ = 30
    BVULT = 31
    BVULE = 32
    BVUGT = 33
    BVUGE = 34
    BVSLT = 35
    BVSLE = 36
    BVSGT = 37
    BVSGE = 38
    AND = 40
    OR = 41
    XOR = 42
    NOT = 43
    ITE = 45
    EXTRACT = 50
    CONCAT = 51
    ZEXT = 52
    SEXT = 53
    KECCAK = 60
    BVADD_NOOVFL_U = 61
    BVMUL_NOOVFL_U = 62
    BVSUB_NOUDFL_U = 63
    EVM_EXP = 70
    EVM_SIGNEXTEND = 71
    EVM_BYTE = 72
    EVM_ADDMOD = 73   # (a + b) mod c, exact (imm0 = 1: c == 0 gives (a + b) mod 2^256, else 0)
    EVM_MULMOD = 74   # (a * b) mod c, exact (same zero rule)
    # host-only term kinds: built by the term layer (smt.py, smtlib.py) and removed by
    # lower.py before a tape reaches mh_tapes_compile (which rejects them)
    ARRAY = 80        # free array symbol: imm0 = array id, imm1 = domain width, width = range
    CONST_ARRAY = 81  # K(domain, v): a = default value node, imm1 = domain width
    STORE = 82        # store(a, b = key, c = value)
    SELECT = 83       # select(a = array, b = index) -> range-width bit-vector
    UF = 84           # uninterpreted function application: imm0 = function id, a = argument


NODE_DTYPE = np.dtype(
    [
        ("op", "u1"),
        ("flags", "u1"),
        ("width", "<u2"),
        ("a", "<u4"),
        ("b", "<u4"),
        ("c", "<u4"),
        ("imm0", "<u4"),
        ("imm1", "<u4"),
    ]
)
assert NODE_DTYPE.itemsize == 24
NODE_PACK = struct.Struct("<BBHIIIII").pack  # one NODE_DTYPE record

HOST_ONLY = {Op.ARRAY, Op.CONST_ARRAY, Op.STORE, Op.SELECT, Op.UF}
F_ARRAY = 1  # mh_node.flags bit of host-only array-sorted nodes (never sent to the device)
F_HOST = 2   # lowering rewrites the node: it is or reads a host-only term or an EQ over > 256 bits

# operand arity per op (number of node operands a, b, c used)
ARITY = {
    Op.CONST: 0, Op.VAR: 0, Op.TRUE: 0, Op.FALSE: 0,
    Op.BVNEG: 1, Op.BVNOT: 1, Op.NOT: 1, Op.EXTRACT: 1, Op.ZEXT: 1, Op.SEXT: 1, Op.KECCAK: 1,
    Op.ITE: 3, Op.EVM_ADDMOD: 3, Op.EVM_MULMOD: 3, Op.ARRAY: 0, Op.CONST_ARRAY: 1, Op.STORE: 3, Op.UF: 1,
}
for _op in Op:
    ARITY.setdefault(_op, 2)

BV_BINARY = {
    Op.BVADD, Op.BVSUB, Op.BVMUL, Op.BVUDIV, Op.BVUREM, Op.BVSDIV, Op.BVSREM, Op.BVSMOD,
    Op.BVAND, Op.BVOR, Op.BVXOR, Op.BVSHL, Op.BVLSHR, Op.BVASHR, Op.EVM_EXP,
    Op.EVM_SIGNEXTEND, Op.EVM_BYTE,
}
BV_COMPARE = {
    Op.BVULT, Op.BVULE, Op.BVUGT, Op.BVUGE, Op.BVSLT, Op.BVSLE, Op.BVSGT, Op.BVSGE,
    Op.BVADD_NOOVFL_U, Op.BVMUL_NOOVFL_U, Op.BVSUB_NOUDFL_U,
}
BOOL_BINARY = {Op.AND, Op.OR, Op.XOR}


class TapeError(ValueError):
    pass


@dataclass
class ConstPool:
    """Shared 256-bit constant pool of a tape set (8 little-endian u32 limbs per entry)."""

    values: List[int] = field(default_factory=list)
    index: Dict[int, int] = field(default_factory=dict)

    def add(self, value: int) -> int:
        if value < 0 or value >= 1 << 256:
            raise TapeError("constant pool entries are 256-bit: %r" % value)
        i = self.index.get(value)
        if i is None:
            i = len(self.values)
            self.values.append(value)
            self.index[value] = i
        return i

    def to_array(self) -> np.ndarray:
        """[n, 8] u32 limbs of every value (incremental: a pool shared by a process's queries
        only converts the values added since the last call)."""
        n = len(self.values)
        arr = self.__dict__.get("_arr")
        done = 0 if arr is None else self.__dict__["_arr_n"]
        if arr is None or arr.shape[0] < max(n, 1):
            grown = np.zeros((max(n, 1, 2 * done), 8), dtype=np.uint32)
            if arr is not None:
                grown[:done] = arr[:done]
            arr = self._arr = grown
        if n > done:
            buf = b"".join(v.to_bytes(32, "little") for v in self.values[done:n])
            arr[done:n] = np.frombuffer(buf, dtype="<u4").reshape(n - done, 8)
        self._arr_n = n
        return arr[:max(n, 1)]


class TapeBuilder:
    """Builds one tape; nodes are hash-consed (structurally equal terms share one node)."""

    def __init__(self, pool: ConstPool, var_index: Dict[str, int],
                 symbols: "Optional[Symbols]" = None):
        self.pool = pool
        self.var_index = var_index
        self.symbols = symbols if symbols is not None else Symbols()
        self.nodes: List[Tuple[int, int, int, int, int, int, int]] = []
        self.widths: List[int] = []
        self.flags: List[int] = []
        self._memo: Dict[tuple, int] = {}
        # the same nodes packed as the C-ABI's mh_node (24 bytes each, NODE_DTYPE), appended
        # alongside: native.TermMirror.sync hands a range of them to the library as they are
        self.node_bytes = bytearray()

    # -- node creation ------------------------------------------------------------------------
    def _add(self, op: Op, width: int, a=0, b=0, c=0, imm0=0, imm1=0, flags=0) -> int:
        key = (int(op), width, a, b, c, imm0, imm1)
        got = self._memo.get(key)
        if got is not None:
            return got
        k = ARITY[op]
        if op in HOST_ONLY or (op == Op.EQ and self.widths[a] > 256):
            flags |= F_HOST
        elif k:
            fl = self.flags
            flags |= (fl[a] | (fl[b] if k > 1 else 0) | (fl[c] if k > 2 else 0)) & F_HOST
        idx = len(self.nodes)
        self.nodes.append(key)
        self.widths.append(width)
        self.flags.append(flags)
        self.node_bytes += NODE_PACK(key[0], flags, width, a, b, c, imm0, imm1)
        self._memo[key] = idx
        return idx

    def width(self, n: int) -> int:
        return self.widths[n]

    def is_array(self, n: int) -> bool:
        return bool(self.flags[n] & F_ARRAY)

    def const_value(self, n: int) -> Optional[int]:
        """The value of a constant node, else None (memoised: nodes are immutable).  CONST / TRUE /
        FALSE, and the bit-layout ops CONCAT / EXTRACT / ZEXT / SEXT over constants, which z3's ``simplify`` folds before
        ``BitVec.symbolic`` / ``.value`` look (mythril/laser/smt/bitvec.py:44-60); arithmetic is
        not folded here."""
        cv = self.__dict__.setdefault("_cv", {})
        if n in cv:
            return cv[n]
        r = self._const_value(n)
        cv[n] = r
        return r

    def _const_value(self, n: int) -> Optional[int]:
        op, w, a, b, _, imm0, imm1 = self.nodes[n]
        if op == Op.CONST:
            return self.pool.values[imm0]
        if op == Op.TRUE:
            return 1
        if op == Op.FALSE:
            return 0
        if op == Op.CONCAT:
            hi, lo = self.const_value(a), self.const_value(b)
            if hi is None or lo is None:
                return None
            return (hi << self.widths[b]) | lo
        if op in (Op.EXTRACT, Op.ZEXT, Op.SEXT):
            x = self.const_value(a)
            if x is None:
                return None
            if op == Op.EXTRACT:
                return (x >> imm1) & ((1 << (imm0 - imm1 + 1)) - 1)
            if op == Op.SEXT and x >> (self.widths[a] - 1) & 1:
                return (x | (((1 << imm0) - 1) << self.widths[a]))
            return x
        return None

    # -- host-only term kinds (arrays, uninterpreted functions) -------------------------------
    def array(self, name: str, domain: int, value_range: int) -> int:
        """Free array symbol (mythril/laser/smt/array.py:35-47, z3.Array)."""
        aid = self.symbols.array_id(name, domain, value_range)
        return self._add(Op.ARRAY, value_range, imm0=aid, imm1=domain, flags=F_ARRAY)

    def const_array(self, domain: int, default: int) -> int:
        """K(domain, default) (array.py:50-63, z3.K); `default` is a bit-vector node."""
        if self.is_array(default) or self.widths[default] == BOOL:
            raise TapeError("K needs a bit-vector default")
        return self._add(Op.CONST_ARRAY, self.widths[default], a=default, imm1=domain,
                         flags=F_ARRAY)

    def store(self, arr: int, key: int, value: int) -> int:
        """z3.Store (array.py:27-32)."""
        dom, rng = self._array_sort(arr)
        if self.widths[key] != dom or self.widths[value] != rng:
            raise TapeError("store sort mismatch: key %d/%d, value %d/%d"
                            % (self.widths[key], dom, self.widths[value], rng))
        return self._add(Op.STORE, rng, a=arr, b=key, c=value, imm1=dom, flags=F_ARRAY)

    def select(self, arr: int, index: int) -> int:
        """z3.Select (array.py:19-25)."""
        dom, rng = self._array_sort(arr)
        if self.widths[index] != dom or self.is_array(index):
            raise TapeError("select index is %d bits, array domain %d"
                            % (self.widths[index], dom))
        return self._add(Op.SELECT, rng, a=arr, b=index)

    def apply(self, name: str, domain: int, value_range: int, arg: int) -> int:
        """Uninterpreted function application (mythril/laser/smt/function.py:7-25)."""
        if self.widths[arg] != domain or self.is_array(arg):
            raise TapeError("%s takes %d bits, got %d" % (name, domain, self.widths[arg]))
        fid = self.symbols.function_id(name, domain, value_range)
        return self._add(Op.UF, value_range, a=arg, imm0=fid)

    def _array_sort(self, arr: int) -> Tuple[int, int]:
        if not self.is_array(arr):
            raise TapeError("node %d is not an array" % arr)
        return self.nodes[arr][6], self.widths[arr]

    def const(self, value: int, width: int) -> int:
        """A constant; wider than 256 bits it is a CONCAT of pool entries (the pool is 256-bit)."""
        if not 1 <= width <= MAX_WIDTH:
            raise TapeError("constants are 1..%d bits wide: %d" % (MAX_WIDTH, width))
        value &= (1 << width) - 1
        if width > 256:
            lo = self.const(value & ((1 << 256) - 1), 256)
            return self.op(Op.CONCAT, self.const(value >> 256, width - 256), lo)
        return self._add(Op.CONST, width, imm0=self.pool.add(value))

    def var(self, name: str, width: int = 256) -> int:
        if not 1 <= width <= 256:
            raise TapeError("variables are 1..256 bits wide: %d" % width)
        self.symbols.check_var(name, width)
        if name not in self.var_index:
            self.var_index[name] = len(self.var_index)
        return self._add(Op.VAR, width, imm0=self.var_index[name])

    def user_var(self, name: str, width: int = 256) -> int:
        """var() for a symbol the terms declare (not a column lowering makes)."""
        n = self.var(name, width)
        self.symbols.user_vars.add(name)
        return n

    def true(self) -> int:
        return self._add(Op.TRUE, BOOL)

    def false(self) -> int:
        return self._add(Op.FALSE, BOOL)

    def op(self, op: Op, *args: int, imm0: int = 0, imm1: int = 0) -> int:
        if op.__class__ is not Op:
            op = Op(op)
        if op in HOST_ONLY:
            raise TapeError("%s is built with array()/const_array()/store()/select()/apply()"
                            % op.name)
        if any(self.flags[x] & F_ARRAY for x in args):
            raise TapeError("%s does not take array operands" % op.name)
        ws = [self.widths[x] for x in args]
        if len(args) != ARITY[op]:
            raise TapeError("%s takes %d operands" % (op.name, ARITY[op]))
        if op in BV_BINARY:
            if ws[0] == BOOL or ws[0] != ws[1]:
                raise TapeError("%s needs equal bit-vector widths, got %s" % (op.name, ws))
            w = ws[0]
        elif op in BV_COMPARE:
            if ws[0] == BOOL or ws[0] != ws[1]:
                raise TapeError("%s needs equal bit-vector widths, got %s" % (op.name, ws))
            w = BOOL
        elif op in (Op.BVNEG, Op.BVNOT):
            if ws[0] == BOOL:
                raise TapeError("%s needs a bit-vector" % op.name)
            w = ws[0]
        elif op == Op.EQ:
            if ws[0] != ws[1]:
                raise TapeError("EQ needs equal sorts, got %s" % ws)
            w = BOOL
        elif op in BOOL_BINARY or op == Op.NOT:
            if any(x != BOOL for x in ws):
                raise TapeError("%s needs Bool operands" % op.name)
            w = BOOL
        elif op == Op.ITE:
            if ws[0] != BOOL or ws[1] != ws[2]:
                raise TapeError("ITE needs (Bool, s, s), got %s" % ws)
            w = ws[1]
        elif op == Op.EXTRACT:
            hi, lo = imm0, imm1
            if ws[0] == BOOL or not (0 <= lo <= hi < ws[0]):
                raise TapeError("bad extract [%d:%d] of width %d" % (hi, lo, ws[0]))
            w = hi - lo + 1
        elif op == Op.CONCAT:
            if BOOL in ws:
                raise TapeError("CONCAT needs bit-vectors")
            w = ws[0] + ws[1]
        elif op in (Op.ZEXT, Op.SEXT):
            if ws[0] == BOOL:
                raise TapeError("%s needs a bit-vector" % op.name)
            w = ws[0] + imm0
        elif op == Op.KECCAK:
            if ws[0] == BOOL or ws[0] % 8:
                raise TapeError("KECCAK input must be a whole number of bytes, got %d" % ws[0])
            w = 256
        elif op in (Op.EVM_ADDMOD, Op.EVM_MULMOD):
            if ws != [256, 256, 256] or imm0 not in (0, 1):
                raise TapeError("%s needs three 256-bit words and imm0 0/1, got %s"
                                % (op.name, ws))
            w = 256
        else:
            raise TapeError("op %s is not built with op()" % op.name)
        if w > MAX_WIDTH:
            raise TapeError("width %d exceeds %d" % (w, MAX_WIDTH))
        a, b, c = (list(args) + [0, 0, 0])[:3]
        return self._add(op, w, a, b, c, imm0, imm1)

    def finish(self, root: int) -> "Tape":
        """Return the tape of the sub-DAG reachable from ``root`` (root last, topological).

        Post-order of AND(x, y) is x's post-order, then y's nodes not under x, then the AND; a
        path condition grows by one conjunct per LASER query (svm.py:257-262), so the tapes of
        recent roots are kept and a child query's tape extends its parent's."""
        cache = self.__dict__.setdefault("_finished", OrderedDict())
        got = cache.get(root)
        if got is not None:
            cache.move_to_end(root)
            return Tape(got[1])
        node = self.nodes[root]
        base = cache.get(node[2]) if node[0] == Op.AND else None
        if base is not None:
            remap = dict(base[0])
            start = [(node[3], False)]
        else:
            remap = {}
            start = [(root, False)]
        order: List[int] = []
        stack = start
        seen = set()
        while stack:
            n, done = stack.pop()
            if done:
                remap[n] = len(remap)
                order.append(n)
                continue
            if n in seen or n in remap:
                continue
            seen.add(n)
            stack.append((n, True))
            nd = self.nodes[n]
            for child in reversed(nd[2 : 2 + ARITY[nd[0]]]):
                if child not in seen and child not in remap:
                    stack.append((child, False))
        if base is not None and root not in remap:
            remap[root] = len(remap)
            order.append(root)
        rows = []
        flags = self.flags
        for old in order:
            op, w, a, b, c, i0, i1 = self.nodes[old]
            k = ARITY[op]
            rows.append((op, flags[old], w, remap[a] if k > 0 else 0, remap[b] if k > 1 else 0,
                         remap[c] if k > 2 else 0, i0, i1))
        arr = np.array(rows, dtype=NODE_DTYPE)
        if base is not None:
            arr = np.concatenate([base[1], arr])
        # every root is kept (a one-constraint query's root is its conjunct, the next query's
        # AND extends it)
        arr.flags.writeable = False  # shared with later tapes: callers copy to modify
        cache[root] = (remap, arr)
        held = self.__dict__.get("_finished_nodes", 0) + len(arr)
        while len(cache) > 1 and (len(cache) > FINISH_CACHE or held > FINISH_CACHE_NODES):
            held -= len(cache.popitem(last=False)[1][1])
        self._finished_nodes = held
        return Tape(arr)


class Symbols:
    """Declared arrays and uninterpreted functions of a tape set (name -> id and sort), plus the
    sorts of scalar variables, so one name always denotes one symbol of one sort (as in z3)."""

    def __init__(self):
        self.arrays: Dict[str, Tuple[int, int, int]] = {}     # name -> (id, domain, range)
        self.functions: Dict[str, Tuple[int, int, int]] = {}  # name -> (id, domain, range)
        self.array_names: List[str] = []
        self.function_names: List[str] = []
        self.var_widths: Dict[str, int] = {}
        # names of the scalar symbols terms declare (BitVecSym, the z3 import), as opposed to the
        # columns lowering makes (array cells "A[0x5]", else columns "A[*]"): a query holding both
        # under one name is refused (lower._schema_of), as the native compiler refuses it
        self.user_vars: set = set()
        self.bool_vars: set = set()  # ... of them Bool symbols (1-bit columns compared with 1)

    def array_id(self, name: str, domain: int, value_range: int) -> int:
        got = self.arrays.get(name)
        if got is None:
            got = self.arrays[name] = (len(self.array_names), domain, value_range)
            self.array_names.append(name)
        elif got[1:] != (domain, value_range):
            raise TapeError("array %r redeclared with another sort" % name)
        return got[0]

    def function_id(self, name: str, domain: int, value_range: int) -> int:
        got = self.functions.get(name)
        if got is None:
            got = self.functions[name] = (len(self.function_names), domain, value_range)
            self.function_names.append(name)
        elif got[1:] != (domain, value_range):
            raise TapeError("function %r redeclared with another sort" % name)
        return got[0]

    def check_var(self, name: str, width: int) -> None:
        got = self.var_widths.setdefault(name, width)
        if got != width:
            raise TapeError("variable %r is %d bits, used as %d" % (name, got, width))


@dataclass
class Tape:
    nodes: np.ndarray  # NODE_DTYPE, root last

    @property
    def root_width(self) -> int:
        return int(self.nodes[-1]["width"])

    def __len__(self) -> int:
        return len(self.nodes)


class TapeSet:
    """A batch of tapes sharing one constant pool and one assignment schema (variable columns)."""

    def __init__(self, var_names: Sequence[str] = ()):
        self.pool = ConstPool()
        self.var_index: Dict[str, int] = {}
        for n in var_names:
            self.var_index.setdefault(n, len(self.var_index))
        self.tapes: List[Tape] = []
        self.symbols = Symbols()
        # flatten()'s result when the tapes already lie back to back in one array (a native
        # query's, mythril_amd/sieve.py); whoever replaces a tape resets it
        self.flat: Optional[Tuple[np.ndarray, np.ndarray, np.ndarray]] = None

    def builder(self) -> TapeBuilder:
        return TapeBuilder(self.pool, self.var_index, self.symbols)

    def add(self, tape: Tape) -> int:
        host = [Op(int(o)).name for o in set(tape.nodes["op"].tolist()) if int(o) in HOST_ONLY]
        if host:
            raise TapeError("tape still holds host-only terms %s: lower it first "
                            "(mythril_amd.lower)" % sorted(host))
        self.tapes.append(tape)
        return len(self.tapes) - 1

    @property
    def n_vars(self) -> int:
        return len(self.var_index)

    @property
    def var_names(self) -> List[str]:
        return [n for n, _ in sorted(self.var_index.items(), key=lambda kv: kv[1])]

    def flatten(self) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """(nodes, tape_offsets[n+1] as u64, consts[n_consts, 8] as u32) for mh_tapes_compile."""
        if self.flat is not None:
            return self.flat
        offs = np.zeros(len(self.tapes) + 1, dtype=np.uint64)
        for i, t in enumerate(self.tapes):
            offs[i + 1] = offs[i] + len(t.nodes)
        nodes = (
            np.concatenate([t.nodes for t in self.tapes])
            if self.tapes
            else np.zeros(0, dtype=NODE_DTYPE)
        )
        return nodes, offs, self.pool.to_array()

    def save(self, path: str) -> None:
        nodes, offs, consts = self.flatten()
        np.savez_compressed(
            path,
            nodes=nodes.view(np.uint8),
            offsets=offs,
            consts=consts,
            var_names=np.array(self.var_names, dtype=object).astype(str),
        )

    @classmethod
    def load(cls, path: str) -> "TapeSet":
        z = np.load(path, allow_pickle=False)
        ts = cls([str(x) for x in z["var_names"]])
        consts = z["consts"]
        for row in consts:
            v = limbs_to_int(row)
            ts.pool.index.setdefault(v, len(ts.pool.values))
            ts.pool.values.append(v)
        nodes = z["nodes"].view(NODE_DTYPE)
        offs = z["offsets"]
        for i in range(len(offs) - 1):
            ts.tapes.append(Tape(nodes[int(offs[i]) : int(offs[i + 1])].copy()))
        return ts


def limbs_to_int(limbs: Sequence[int]) -> int:
    v = 0
    for k, x in enumerate(limbs):
        v |= int(x) << (32 * k)
    return v


def int_to_limbs(v: int, n: int = 8) -> List[int]:
    return [(v >> (32 * k)) & 0xFFFFFFFF for k in range(n)]
