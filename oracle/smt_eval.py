"""ORACLE (test infrastructure only — never imported by the product path).

Ground evaluation of a sieve tape under one candidate assignment, restated in plain Python
big-integer arithmetic.  This is the semantics the reference gets from z3's model evaluator,
``Model.eval(expr, model_completion=True)`` (mythril/laser/smt/model.py:45-59), for the terms
that mythril.laser.smt constructs:

  bvadd/bvsub/bvmul      BitVec.__add__/__sub__/__mul__        bitvec.py:63-94
  bvsdiv                 BitVec.__truediv__ (signed!)          bitvec.py:96-103
  bvudiv/bvurem/bvsrem   UDiv/URem/SRem                        bitvec_helper.py:131-161
  bvand/bvor/bvxor       BitVec.__and__/__or__/__xor__         bitvec.py:105-136
  bvslt/bvsgt/bvsle/bvsge BitVec.__lt__/__gt__/__le__/__ge__   bitvec.py:138-180
  bvult/bvugt            ULT/UGT; UGE/ULE = Or(UGT|ULT, =)     bitvec_helper.py:43-80
  =                      BitVec.__eq__ (zero-padded widths)    bitvec.py:16-22,183-216
  bvshl/bvashr/bvlshr    <<, >> (arithmetic), LShR             bitvec.py:218-243, bitvec_helper.py:21-23
  concat/extract         Concat/Extract                        bitvec_helper.py:83-128
  ite                    If                                    bitvec_helper.py:26-40
  and/or/xor/not         And/Or/Xor/Not                        bool.py:87-124
  *_no_overflow          BVAddNoOverflow/BVMulNoOverflow/BVSubNoUnderflow  bitvec_helper.py:178-227
  keccak                 find_concrete_keccak                  keccak_function_manager.py:43-57
  EVM_ADDMOD/MULMOD        yellow-paper ADDMOD/MULMOD, exact sum / product (evm_modop)
  EVM_EXP/SIGNEXTEND/BYTE  concrete branches of instructions.py:599-631 (pow mod 2^256),
                         :634-662 (SIGNEXTEND), :401-430 (BYTE)

Operator semantics follow SMT-LIB 2.6 QF_BV, which z3 implements: x bvudiv 0 = 2^w - 1,
x bvurem 0 = x, bvsdiv/bvsrem/bvsmod by the SMT-LIB sign rules, shifts by >= w give 0 (or the
sign fill for bvashr).  z3 is not installed in this container, so the
symbolic-divisor-by-zero rule and z3's BVAddNoOverflow/BVMulNoOverflow encodings are pinned to
SMT-LIB / z3's documented definitions only ("parity unpinned" for those cases).

Op numbers are restated here from include/mythril_hip.h (enum mh_op) so the oracle does not
import product code.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Union

try:  # package-relative when imported as oracle.smt_eval
    from .keccak import keccak256
except ImportError:  # pragma: no cover
    from keccak import keccak256  # type: ignore

# --- op numbers (include/mythril_hip.h, enum mh_op) ---------------------------------------------
CONST, VAR, TRUE, FALSE = 0, 1, 2, 3
BVADD, BVSUB, BVMUL, BVUDIV, BVUREM, BVSDIV, BVSREM, BVSMOD, BVNEG, BVNOT = range(10, 20)
BVAND, BVOR, BVXOR, BVSHL, BVLSHR, BVASHR = range(20, 26)
EQ, BVULT, BVULE, BVUGT, BVUGE, BVSLT, BVSLE, BVSGT, BVSGE = range(30, 39)
AND, OR, XOR, NOT = 40, 41, 42, 43
ITE = 45
EXTRACT, CONCAT, ZEXT, SEXT = 50, 51, 52, 53
KECCAK, BVADD_NOOVFL_U, BVMUL_NOOVFL_U, BVSUB_NOUDFL_U = 60, 61, 62, 63
EVM_EXP, EVM_SIGNEXTEND, EVM_BYTE, EVM_ADDMOD, EVM_MULMOD = 70, 71, 72, 73, 74


def _mask(w: int) -> int:
    return (1 << w) - 1


def _signed(x: int, w: int) -> int:
    return x - (1 << w) if x >> (w - 1) & 1 else x


def bvudiv(s: int, t: int, w: int) -> int:
    return _mask(w) if t == 0 else s // t


def bvurem(s: int, t: int, w: int) -> int:
    return s if t == 0 else s % t


def bvneg(x: int, w: int) -> int:
    return (-x) & _mask(w)


def bvsdiv(s: int, t: int, w: int) -> int:
    """SMT-LIB: bvsdiv defined through bvudiv on magnitudes, negating when signs differ."""
    ms, mt = s >> (w - 1) & 1, t >> (w - 1) & 1
    if not ms and not mt:
        return bvudiv(s, t, w)
    if ms and not mt:
        return bvneg(bvudiv(bvneg(s, w), t, w), w)
    if not ms and mt:
        return bvneg(bvudiv(s, bvneg(t, w), w), w)
    return bvudiv(bvneg(s, w), bvneg(t, w), w)


def bvsrem(s: int, t: int, w: int) -> int:
    """SMT-LIB: remainder takes the sign of the dividend."""
    ms, mt = s >> (w - 1) & 1, t >> (w - 1) & 1
    if not ms and not mt:
        return bvurem(s, t, w)
    if ms and not mt:
        return bvneg(bvurem(bvneg(s, w), t, w), w)
    if not ms and mt:
        return bvurem(s, bvneg(t, w), w)
    return bvneg(bvurem(bvneg(s, w), bvneg(t, w), w), w)


def bvsmod(s: int, t: int, w: int) -> int:
    """SMT-LIB: modulus takes the sign of the divisor."""
    ms, mt = s >> (w - 1) & 1, t >> (w - 1) & 1
    abs_s = bvneg(s, w) if ms else s
    abs_t = bvneg(t, w) if mt else t
    u = bvurem(abs_s, abs_t, w)
    if u == 0:
        return u
    if not ms and not mt:
        return u
    if ms and not mt:
        return (bvneg(u, w) + t) & _mask(w)
    if not ms and mt:
        return (u + t) & _mask(w)
    return bvneg(u, w)


def bvshl(s: int, t: int, w: int) -> int:
    return 0 if t >= w else (s << t) & _mask(w)


def bvlshr(s: int, t: int, w: int) -> int:
    return 0 if t >= w else s >> t


def bvashr(s: int, t: int, w: int) -> int:
    v = _signed(s, w)
    return (v >> min(t, w)) & _mask(w)


def evm_signextend(k: int, x: int, w: int) -> int:
    """instructions.py:634-662 (concrete k): k <= 31 extends from bit 8k+7, else x unchanged."""
    if k > 31:
        return x
    testbit = k * 8 + 7
    if testbit >= w:
        return x
    if x >> testbit & 1:
        return (x | (_mask(w) - ((1 << testbit) - 1))) & _mask(w)
    return x & ((1 << testbit) - 1) | (x & (1 << testbit))


def evm_modop(mul: bool, x: int, y: int, n: int, zero_low: bool) -> int:
    """Yellow-paper ADDMOD / MULMOD: (x + y) mod n, (x * y) mod n with the sum / product taken
    exactly (a 512-bit intermediate; instructions.py:569-596 states the same with z3 terms on
    concrete values).  n == 0 gives 0, or, with zero_low (mh_node.imm0 = 1), the low 256 bits of
    x op y -- extract[255:0](bvurem(zext x op zext y, zext n)), SMT-LIB's x % 0 = x."""
    u = x * y if mul else x + y
    if n == 0:
        return u & _mask(256) if zero_low else 0
    return u % n


def evm_byte(i: int, x: int, w: int) -> int:
    """instructions.py:401-430 (concrete index): byte i (0 = most significant) of a 256-bit word."""
    if i >= w // 8:
        return 0
    return (x >> (8 * (w // 8 - 1 - i))) & 0xFF


Value = Union[int, bool]


def evaluate(nodes, consts: Sequence[int], assignment: Sequence[int], all_values: bool = False,
             extra=None):
    """Evaluate one tape.

    nodes: structured array / sequence of records with fields op, width, a, b, c, imm0, imm1
    consts: the tape set's constant pool (Python ints)
    assignment: per-variable 256-bit values (Python ints), indexed by column
    Returns the root value (int for bit-vectors, bool for Bool); with all_values, every node's.
    extra(op, node, vals): value of an op this module does not know (oracle/term_eval.py uses it
    for arrays and uninterpreted functions).
    """
    vals: List[Value] = []
    for nd in nodes:
        op = int(nd["op"])
        w = int(nd["width"])
        a, b, c = int(nd["a"]), int(nd["b"]), int(nd["c"])
        i0, i1 = int(nd["imm0"]), int(nd["imm1"])
        if op == CONST:
            v: Value = consts[i0] & _mask(w)
        elif op == VAR:
            v = assignment[i0] & _mask(w)
        elif op == TRUE:
            v = True
        elif op == FALSE:
            v = False
        elif op in (BVADD, BVSUB, BVMUL, BVUDIV, BVUREM, BVSDIV, BVSREM, BVSMOD, BVAND, BVOR,
                    BVXOR, BVSHL, BVLSHR, BVASHR, EVM_EXP, EVM_SIGNEXTEND, EVM_BYTE):
            x, y = vals[a], vals[b]
            m = _mask(w)
            if op == BVADD:
                v = (x + y) & m
            elif op == BVSUB:
                v = (x - y) & m
            elif op == BVMUL:
                v = (x * y) & m
            elif op == BVUDIV:
                v = bvudiv(x, y, w)
            elif op == BVUREM:
                v = bvurem(x, y, w)
            elif op == BVSDIV:
                v = bvsdiv(x, y, w)
            elif op == BVSREM:
                v = bvsrem(x, y, w)
            elif op == BVSMOD:
                v = bvsmod(x, y, w)
            elif op == BVAND:
                v = x & y
            elif op == BVOR:
                v = x | y
            elif op == BVXOR:
                v = x ^ y
            elif op == BVSHL:
                v = bvshl(x, y, w)
            elif op == BVLSHR:
                v = bvlshr(x, y, w)
            elif op == BVASHR:
                v = bvashr(x, y, w)
            elif op == EVM_EXP:
                v = pow(x, y, 1 << w)
            elif op == EVM_SIGNEXTEND:
                v = evm_signextend(x, y, w)
            else:
                v = evm_byte(x, y, w)
        elif op in (EVM_ADDMOD, EVM_MULMOD):
            v = evm_modop(op == EVM_MULMOD, vals[a], vals[b], vals[c], i0 == 1)
        elif op == BVNEG:
            v = bvneg(vals[a], w)
        elif op == BVNOT:
            v = vals[a] ^ _mask(w)
        elif op == EQ:
            v = vals[a] == vals[b]
        elif op in (BVULT, BVULE, BVUGT, BVUGE, BVSLT, BVSLE, BVSGT, BVSGE, BVADD_NOOVFL_U,
                    BVMUL_NOOVFL_U, BVSUB_NOUDFL_U):
            wa = int(nodes[a]["width"])
            x, y = vals[a], vals[b]
            if op in (BVSLT, BVSLE, BVSGT, BVSGE):
                x, y = _signed(x, wa), _signed(y, wa)
            if op in (BVULT, BVSLT):
                v = x < y
            elif op in (BVULE, BVSLE):
                v = x <= y
            elif op in (BVUGT, BVSGT):
                v = x > y
            elif op in (BVUGE, BVSGE):
                v = x >= y
            elif op == BVADD_NOOVFL_U:
                v = x + y <= _mask(wa)
            elif op == BVMUL_NOOVFL_U:
                v = x * y <= _mask(wa)
            else:  # BVSUB_NOUDFL_U
                v = y <= x
        elif op == AND:
            v = bool(vals[a]) and bool(vals[b])
        elif op == OR:
            v = bool(vals[a]) or bool(vals[b])
        elif op == XOR:
            v = bool(vals[a]) != bool(vals[b])
        elif op == NOT:
            v = not vals[a]
        elif op == ITE:
            v = vals[b] if vals[a] else vals[c]
        elif op == EXTRACT:
            v = (vals[a] >> i1) & _mask(i0 - i1 + 1)
        elif op == CONCAT:
            wb = int(nodes[b]["width"])
            v = (vals[a] << wb) | vals[b]
        elif op == ZEXT:
            v = vals[a]
        elif op == SEXT:
            wa = int(nodes[a]["width"])
            v = _signed(vals[a], wa) & _mask(w)
        elif op == KECCAK:
            wa = int(nodes[a]["width"])
            v = int.from_bytes(keccak256(vals[a].to_bytes(wa // 8, "big")), "big")
        elif extra is not None:
            v = extra(op, nd, vals)
        else:
            raise ValueError("unknown op %d" % op)
        vals.append(v)
    return vals if all_values else vals[-1]


def as_limbs(v: Value, n: int = 8) -> List[int]:
    v = int(v)
    return [(v >> (32 * k)) & 0xFFFFFFFF for k in range(n)]


# --- counter-based assignment generator (restated from include/mythril_hip.h, mh_gen_limb) -----
_M64 = (1 << 64) - 1


def splitmix64(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & _M64
    z = x
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


def gen_limb(seed: int, var: int, index: int, limb: int) -> int:
    """One u32 limb of generated assignment ``index``, column ``var`` (see mh_gen_limb)."""
    h = splitmix64(seed ^ ((var * 8 + limb) * 0xD1B54A32D192ED03 & _M64))
    h = splitmix64(h ^ index)
    return h & 0xFFFFFFFF


def gen_word(seed: int, var: int, index: int) -> int:
    return sum(gen_limb(seed, var, index, k) << (32 * k) for k in range(8))


def gen_assignment(seed: int, n_vars: int, index: int) -> List[int]:
    return [gen_word(seed, v, index) for v in range(n_vars)]
