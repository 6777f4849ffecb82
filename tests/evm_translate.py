"""Straight-line EVM bytecode -> sieve tapes, following LASER's opcode lowering.

Test infrastructure: turns the reference's VMTests known-answer programs (tests/golden/vmtests.json)
into tapes so the oracle and the HIP kernel can be checked against official expected storage.

mode="laser": the terms LASER builds (mythril/laser/ethereum/instructions.py), including its
  quirks: DIV/SDIV/MOD/SMOD by a *concrete* zero push 0 (:480-566); ADDMOD/MULMOD are 256-bit
  URem chains (:569-596); NOT is (2^256-1) - x (:389-398); SIGNEXTEND/BYTE with a concrete index
  become and/or masks and concat/extract (:401-430,:634-662); comparisons push Bools that
  pop_bitvec turns into If(b, 1, 0) (util.py:67-88); ISZERO is If(x == 0, 1, 0) (:744-758);
  SHA3 of memory bytes is keccak of their Concat (:1010-1048).
mode="evm": the same programs through the EVM-word ops (EVM_EXP/EVM_SIGNEXTEND/EVM_BYTE) and
  ite-guarded division, to pin those device ops too.

Concreteness decisions LASER takes through z3 simplify (e.g. ``op1 == 0``) are taken here by
evaluating the sub-term with the oracle; the tapes themselves keep the full term.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

from mythril_amd import smt
from mythril_amd.smt import (BitVec, Bool, Concat, Extract, If, LShR, Not, SRem, UDiv, UGT,
                             ULT, URem, symbol_factory)
from oracle import smt_eval

TT256M1 = (1 << 256) - 1


class Unsupported(Exception):
    pass


class Translator:
    def __init__(self, mode: str = "laser"):
        assert mode in ("laser", "evm")
        self.mode = mode
        self.ctx = smt.set_context(smt.Context())

    # concrete value of a closed term (what z3 simplify would expose to LASER)
    def value(self, e) -> int:
        tape = self.ctx.b.finish(e.node)
        v = smt_eval.evaluate(tape.nodes, self.ctx.tapeset.pool.values, [])
        return int(v)

    def bv(self, x) -> BitVec:
        if isinstance(x, Bool):
            return If(x, symbol_factory.BitVecVal(1, 256), symbol_factory.BitVecVal(0, 256))
        return x

    def run(self, code: bytes) -> List[Tuple[BitVec, BitVec]]:
        """Execute; returns the SSTOREs as (key term, value term), in program order."""
        stack: List = []
        memory: Dict[int, BitVec] = {}
        stores = []
        BVV = symbol_factory.BitVecVal
        pc = 0

        def pop():
            if not stack:
                raise Unsupported("stack underflow")
            return stack.pop()

        def popbv():
            return self.bv(pop())

        while pc < len(code):
            op = code[pc]
            pc += 1
            if op == 0x00:
                break
            elif 0x60 <= op <= 0x7F:
                n = op - 0x5F
                stack.append(BVV(int.from_bytes(code[pc:pc + n].ljust(n, b"\0"), "big"), 256))
                pc += n
            elif 0x80 <= op <= 0x8F:
                k = op - 0x7F
                if len(stack) < k:
                    raise Unsupported("dup underflow")
                stack.append(stack[-k])
            elif 0x90 <= op <= 0x9F:
                k = op - 0x8F
                if len(stack) < k + 1:
                    raise Unsupported("swap underflow")
                stack[-1], stack[-1 - k] = stack[-1 - k], stack[-1]
            elif op == 0x50:
                pop()
            elif op == 0x01:
                stack.append(popbv() + popbv())
            elif op == 0x02:
                stack.append(popbv() * popbv())
            elif op == 0x03:
                stack.append(popbv() - popbv())
            elif op in (0x04, 0x05, 0x06, 0x07):
                a, b = popbv(), popbv()
                stack.append(self._div(op, a, b))
            elif op in (0x08, 0x09):
                a, b, n = popbv(), popbv(), popbv()
                if self.mode == "laser":
                    f = (lambda x, y: x + y) if op == 0x08 else (lambda x, y: x * y)
                    stack.append(URem(f(URem(a, n), URem(b, n)), n))
                else:  # EVM-exact: 512-bit intermediate, modulus 0 -> 0 (oracle-only width)
                    a5, b5, n5 = (smt.ZeroExt(256, x) for x in (a, b, n))
                    r = URem(a5 + b5 if op == 0x08 else a5 * b5, n5)
                    stack.append(If(n == 0, BVV(0, 256), Extract(255, 0, r)))
            elif op == 0x0A:
                base, exp = popbv(), popbv()
                stack.append(BitVec(self.ctx.b.op(smt.Op.EVM_EXP, base.node, exp.node),
                                    self.ctx))
            elif op == 0x0B:
                k, x = pop(), popbv()
                stack.append(self._signextend(self.bv(k), x))
            elif op == 0x10:
                stack.append(ULT(popbv(), popbv()))
            elif op == 0x11:
                stack.append(UGT(popbv(), popbv()))
            elif op == 0x12:
                stack.append(popbv() < popbv())
            elif op == 0x13:
                stack.append(popbv() > popbv())
            elif op == 0x14:
                a, b = self.bv(pop()), self.bv(pop())
                stack.append(a == b)
            elif op == 0x15:
                v = pop()
                e = Not(v) if isinstance(v, Bool) else v == 0
                stack.append(If(e, BVV(1, 256), BVV(0, 256)))
            elif op == 0x16:
                stack.append(self.bv(pop()) & self.bv(pop()))
            elif op == 0x17:
                stack.append(self.bv(pop()) | self.bv(pop()))
            elif op == 0x18:
                stack.append(popbv() ^ popbv())
            elif op == 0x19:
                stack.append(BVV(TT256M1, 256) - popbv())
            elif op == 0x1A:
                i, x = pop(), popbv()
                stack.append(self._byte(self.bv(i), x))
            elif op == 0x1B:
                shift, value = popbv(), popbv()
                stack.append(value << shift)
            elif op == 0x1C:
                shift, value = popbv(), popbv()
                stack.append(LShR(value, shift))
            elif op == 0x1D:
                shift, value = popbv(), popbv()
                stack.append(value >> shift)
            elif op == 0x20:
                off, ln = self.value(popbv()), self.value(popbv())
                if ln == 0:
                    # get_empty_keccak_hash (keccak_function_manager.py:74-81)
                    stack.append(BVV(0xC5D2460186F7233C927E7DB2DCC703C0E500B653CA82273B7BFAD8045D85A470, 256))
                    continue
                if off + ln > 1 << 16:
                    raise Unsupported("memory too large")
                data = [memory.get(off + i, BVV(0, 8)) for i in range(ln)]
                msg = Concat(data) if len(data) > 1 else data[0]
                stack.append(smt.Keccak256(msg))
            elif op == 0x51:
                off = self.value(popbv())
                if off > 1 << 16:
                    raise Unsupported("memory too large")
                stack.append(Concat([memory.get(off + i, BVV(0, 8)) for i in range(32)]))
            elif op == 0x52:
                off, v = self.value(popbv()), popbv()
                if off > 1 << 16:
                    raise Unsupported("memory too large")
                for i in range(32):
                    memory[off + i] = Extract(255 - 8 * i, 248 - 8 * i, v)
            elif op == 0x53:
                off, v = self.value(popbv()), popbv()
                if off > 1 << 16:
                    raise Unsupported("memory too large")
                memory[off] = Extract(7, 0, v)
            elif op == 0x55:
                key, val = popbv(), popbv()
                stores.append((key, val))
            else:
                raise Unsupported("opcode 0x%02x" % op)
        return stores

    def _div(self, op: int, a: BitVec, b: BitVec) -> BitVec:
        zero = symbol_factory.BitVecVal(0, 256)
        if self.mode == "laser":
            if self.value(b) == 0:  # `if op1 == 0` on a concrete term (instructions.py:490..565)
                return zero
            return {0x04: UDiv, 0x05: lambda x, y: x / y, 0x06: URem, 0x07: SRem}[op](a, b)
        f = {0x04: UDiv, 0x05: lambda x, y: x / y, 0x06: URem, 0x07: SRem}[op]
        return If(b == 0, zero, f(a, b))

    def _signextend(self, k: BitVec, x: BitVec) -> BitVec:
        if self.mode == "evm":
            return BitVec(self.ctx.b.op(smt.Op.EVM_SIGNEXTEND, k.node, x.node), self.ctx)
        s0 = self.value(k)
        if s0 > 31:
            return x
        testbit = s0 * 8 + 7
        if self.value(x) >> testbit & 1:  # not is_true((s1 & (1 << testbit)) == 0)
            return x | ((1 << 256) - (1 << testbit))
        return x & ((1 << testbit) - 1)

    def _byte(self, i: BitVec, x: BitVec) -> BitVec:
        if self.mode == "evm":
            return BitVec(self.ctx.b.op(smt.Op.EVM_BYTE, i.node, x.node), self.ctx)
        index = self.value(i)
        offset = (31 - index) * 8
        if offset >= 0:
            return Concat(symbol_factory.BitVecVal(0, 248), Extract(offset + 7, offset, x))
        return symbol_factory.BitVecVal(0, 256)


def vmtest_tapes(vec: dict, mode: str):
    """(tapeset, [(key_tape_index, value_tape_index)], expected_storage{int: int})."""
    tr = Translator(mode)
    stores = tr.run(bytes.fromhex(vec["code"]))
    pairs = []
    for key, val in stores:
        pairs.append((tr.ctx.add_tape(key), tr.ctx.add_tape(val)))
    expected = {int(k, 16): int(v, 16) for k, v in vec["post_storage"].items()}
    pre = {int(k, 16): int(v, 16) for k, v in vec["pre_storage"].items()}
    return tr.ctx.tapeset, pairs, expected, pre


def final_storage(pre: Dict[int, int], pairs, values) -> Dict[int, int]:
    """Apply SSTOREs (values[i] = evaluated tape i) and drop zero slots, as post-storage lists."""
    st = dict(pre)
    for kt, vt in pairs:
        st[int(values[kt])] = int(values[vt])
    return {k: v for k, v in st.items() if v != 0}


def lift_constants(ts, keep_exponents=False):
    """The same tapes with every constant leaf turned into an assignment column holding that
    constant (one row), so the compiler cannot fold them: the device evaluates every op of a
    VMTest on registers.  keep_exponents leaves the exponents of EVM_EXP constant (LASER only
    builds EXP over constants, instructions.py:599-631; the native code takes a constant
    exponent).  Returns (lifted tapeset, soa [n_cols, 8, 1] u32)."""
    import numpy as np

    from mythril_amd.tape import Op, Tape, TapeSet

    cols = {}
    out = TapeSet()
    for t in ts.tapes:
        nodes = t.nodes.copy()
        keep = set()
        if keep_exponents:
            keep = {int(n["b"]) for n in nodes if int(n["op"]) == int(Op.EVM_EXP)}
        for i in range(len(nodes)):
            if int(nodes[i]["op"]) == int(Op.CONST) and i not in keep:
                w = int(nodes[i]["width"])
                v = ts.pool.values[int(nodes[i]["imm0"])] & ((1 << w) - 1)
                name = "k%d_%x" % (w, v)
                if name not in cols:
                    cols[name] = v
                    out.var_index[name] = len(out.var_index)
                nodes[i]["op"] = int(Op.VAR)
                nodes[i]["imm0"] = out.var_index[name]
                nodes[i]["imm1"] = 0
        out.tapes.append(Tape(nodes))
    if keep_exponents:
        out.pool = ts.pool
    soa = np.zeros((max(out.n_vars, 1), 8, 1), dtype=np.uint32)
    for name, v in cols.items():
        c = out.var_index[name]
        for k in range(8):
            soa[c, k, 0] = (v >> (32 * k)) & 0xFFFFFFFF
    return out, soa


def vmtest_batch(vectors, mode: str, lifted: bool):
    """Every translatable vector's tapes in ONE tape set (one JIT build for the whole corpus):
    (tapeset, soa [n_cols, 8, 1], [(name, first tape, pairs, expected, pre)]).  Constants are
    re-pooled; lifted turns every constant leaf into a column (lift_constants) shared by value."""
    import numpy as np

    from mythril_amd.tape import Op, Tape, TapeSet

    out = TapeSet()
    index = []
    for vec in vectors:
        try:
            ts, pairs, expected, pre = vmtest_tapes(vec, mode)
        except Unsupported:
            continue
        index.append((vec["name"], len(out.tapes), pairs, expected, pre))
        for t in ts.tapes:
            nodes = t.nodes.copy()
            for i in range(len(nodes)):
                if int(nodes[i]["op"]) == int(Op.CONST):
                    nodes[i]["imm0"] = out.pool.add(ts.pool.values[int(nodes[i]["imm0"])])
                elif int(nodes[i]["op"]) == int(Op.VAR):
                    raise ValueError("VMTest tapes are concrete")
            out.tapes.append(Tape(nodes))
    if lifted:
        out, soa = lift_constants(out)
    else:
        soa = np.zeros((1, 8, 1), dtype=np.uint32)
    return out, soa, index

