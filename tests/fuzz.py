"""Random tape / assignment generators for parity tests (test infrastructure).

Tapes mix every op of the IR over widths 1..256 (plus Keccak over byte-aligned inputs up to
96 bytes) so the device lowering sees extract/concat/zext/sext chains, Bool plumbing and the
division family at odd widths.  Assignment values are biased toward the edges that matter
for bit-exactness: 0, 1, all-ones, sign boundaries, powers of two, short values.
"""
import random

import numpy as np

from mythril_amd.tape import BOOL, Op, TapeSet

WIDTHS = [1, 7, 8, 31, 32, 33, 64, 100, 128, 160, 200, 255, 256]


def interesting(rng: random.Random, w: int) -> int:
    m = (1 << w) - 1
    r = rng.random()
    if r < 0.08:
        return 0
    if r < 0.14:
        return 1
    if r < 0.22:
        return m
    if r < 0.30:
        return 1 << (w - 1)
    if r < 0.36:
        return (1 << (w - 1)) - 1
    if r < 0.46:
        return (1 << rng.randrange(w)) & m
    if r < 0.58:
        return rng.getrandbits(min(w, rng.choice([8, 16, 32, 40, 64, 96])))
    if r < 0.66:
        return (m - rng.getrandbits(min(w, 32))) & m
    return rng.getrandbits(w)


class TapeFuzzer:
    def __init__(self, rng: random.Random, ts: TapeSet, n_vars: int = 3, allow_keccak=True,
                 allow_evm=True, max_depth=4):
        self.rng = rng
        self.ts = ts
        self.b = ts.builder()
        self.vars = ["v%d" % i for i in range(n_vars)]
        for v in self.vars:
            self.b.var(v, 256)
        self.allow_keccak = allow_keccak
        self.allow_evm = allow_evm
        self.max_depth = max_depth

    def leaf(self, w):
        b, rng = self.b, self.rng
        if rng.random() < 0.6:
            v = self.b.var(rng.choice(self.vars), 256)
            if w == 256:
                return v
            lo = rng.randrange(0, 257 - w)
            return b.op(Op.EXTRACT, v, imm0=lo + w - 1, imm1=lo)
        return b.const(interesting(rng, w), w)

    def bv(self, w, depth):
        b, rng = self.b, self.rng
        if depth <= 0 or rng.random() < 0.2:
            return self.leaf(w)
        d = depth - 1
        choices = ["add", "sub", "mul", "div", "and", "or", "xor", "shl", "lshr", "ashr",
                   "shli", "neg", "not", "ite", "extract", "concat", "zext", "sext"]
        if w == 256 and self.allow_evm:
            choices += ["evm"]
        if w == 256 and self.allow_keccak:
            choices += ["keccak"]
        c = rng.choice(choices)
        if c in ("add", "sub", "mul", "and", "or", "xor"):
            op = {"add": Op.BVADD, "sub": Op.BVSUB, "mul": Op.BVMUL, "and": Op.BVAND,
                  "or": Op.BVOR, "xor": Op.BVXOR}[c]
            return b.op(op, self.bv(w, d), self.bv(w, d))
        if c == "div":
            op = rng.choice([Op.BVUDIV, Op.BVUREM, Op.BVSDIV, Op.BVSREM, Op.BVSMOD])
            return b.op(op, self.bv(w, d), self.bv(w, d))
        if c in ("shl", "lshr", "ashr"):
            op = {"shl": Op.BVSHL, "lshr": Op.BVLSHR, "ashr": Op.BVASHR}[c]
            amt = self.bv(w, d) if rng.random() < 0.5 else b.const(
                rng.choice([0, 1, w - 1, w, w + 1, rng.randrange(0, w + 3)]) & ((1 << w) - 1), w)
            return b.op(op, self.bv(w, d), amt)
        if c == "shli":
            op = rng.choice([Op.BVSHL, Op.BVLSHR, Op.BVASHR])
            return b.op(op, self.bv(w, d), b.const(rng.randrange(0, w + 2) & ((1 << w) - 1), w))
        if c == "neg":
            return b.op(Op.BVNEG, self.bv(w, d))
        if c == "not":
            return b.op(Op.BVNOT, self.bv(w, d))
        if c == "ite":
            return b.op(Op.ITE, self.boolean(d), self.bv(w, d), self.bv(w, d))
        if c == "extract":
            wa = rng.choice([x for x in WIDTHS if x >= w])
            lo = rng.randrange(0, wa - w + 1)
            return b.op(Op.EXTRACT, self.bv(wa, d), imm0=lo + w - 1, imm1=lo)
        if c == "concat":
            if w < 2:
                return self.leaf(w)
            wa = rng.randrange(1, w)
            return b.op(Op.CONCAT, self.bv(wa, d), self.bv(w - wa, d))
        if c in ("zext", "sext"):
            if w < 2:
                return self.leaf(w)
            wa = rng.randrange(1, w)
            return b.op(Op.ZEXT if c == "zext" else Op.SEXT, self.bv(wa, d), imm0=w - wa)
        if c == "evm":
            op = rng.choice([Op.EVM_SIGNEXTEND, Op.EVM_BYTE, Op.EVM_EXP, Op.EVM_ADDMOD,
                             Op.EVM_MULMOD])
            if op in (Op.EVM_ADDMOD, Op.EVM_MULMOD):
                n = self.bv(w, d) if rng.random() < 0.6 else b.const(
                    rng.choice([0, 1, 7, (1 << 255) + 3, (1 << 256) - 1, rng.getrandbits(100)]), 256)
                return b.op(op, self.bv(w, d), self.bv(w, d), n, imm0=rng.choice([0, 1]))
            if op == Op.EVM_EXP:
                e = b.const(rng.choice([0, 1, 2, 3, 255, 256, rng.getrandbits(16)]), 256)
                return b.op(op, self.bv(w, d), e if rng.random() < 0.7 else self.bv(w, d))
            k = b.const(rng.choice([0, 1, 15, 30, 31, 32, 33, 1 << 200]), 256)
            return b.op(op, k if rng.random() < 0.7 else self.bv(w, d), self.bv(w, d))
        # keccak of a byte-aligned input up to 96 bytes (pieces <= 256 bits each)
        nbytes = rng.choice([1, 4, 20, 32, 33, 64, 65, 96])
        parts, left = [], nbytes * 8
        while left:
            pw = min(left, rng.choice([8, 64, 160, 256]))
            parts.append(self.bv(pw, d))
            left -= pw
        x = parts[0]
        for p in parts[1:]:
            x = b.op(Op.CONCAT, x, p)
        return b.op(Op.KECCAK, x)

    def boolean(self, depth):
        b, rng = self.b, self.rng
        if depth <= 0:
            return b.true() if rng.random() < 0.5 else b.false()
        d = depth - 1
        c = rng.random()
        if c < 0.55:
            w = rng.choice(WIDTHS)
            op = rng.choice([Op.EQ, Op.BVULT, Op.BVULE, Op.BVUGT, Op.BVUGE, Op.BVSLT, Op.BVSLE,
                             Op.BVSGT, Op.BVSGE, Op.BVADD_NOOVFL_U, Op.BVMUL_NOOVFL_U,
                             Op.BVSUB_NOUDFL_U])
            return b.op(op, self.bv(w, d), self.bv(w, d))
        if c < 0.8:
            op = rng.choice([Op.AND, Op.OR, Op.XOR, Op.EQ])
            return b.op(op, self.boolean(d), self.boolean(d))
        if c < 0.9:
            return b.op(Op.NOT, self.boolean(d))
        return b.op(Op.ITE, self.boolean(d), self.boolean(d), self.boolean(d))

    def tape(self, root_bool=None):
        rb = self.rng.random() < 0.4 if root_bool is None else root_bool
        if rb:
            root = self.boolean(self.max_depth)
        else:
            root = self.bv(self.rng.choice(WIDTHS), self.max_depth)
        return self.ts.add(self.b.finish(root))


def assignment_soa(rng: random.Random, n_vars: int, rows: int) -> np.ndarray:
    soa = np.zeros((n_vars, 8, rows), dtype=np.uint32)
    for r in range(rows):
        for v in range(n_vars):
            x = interesting(rng, 256)
            for k in range(8):
                soa[v, k, r] = (x >> (32 * k)) & 0xFFFFFFFF
    return soa


def soa_row(soa: np.ndarray, r: int):
    out = []
    for v in range(soa.shape[0]):
        x = 0
        for k in range(8):
            x |= int(soa[v, k, r]) << (32 * k)
        out.append(x)
    return out
