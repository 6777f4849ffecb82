"""Tape compiler + device limb algorithms, checked on the host (test-only emulator) against the
oracle.  No GPU: tests/native/emu.cpp runs the compiled device code with the kernel's own
256-bit routines (mythril_amd/csrc/u256_ops.h)."""
import json
import os
import random

import numpy as np
import pytest

from mythril_amd.tape import Op, TapeSet
from oracle import smt_eval
from tests.emu import EmuError
from tests.evm_translate import Unsupported, final_storage, lift_constants, vmtest_tapes
from tests.fuzz import TapeFuzzer, assignment_soa, soa_row

HERE = os.path.dirname(os.path.abspath(__file__))
VMTESTS = json.load(open(os.path.join(HERE, "golden", "vmtests.json")))
LASER_DIVERGENT = {"addmodDivByZero", "addmodDivByZero1", "addmodDivByZero2", "mulmoddivByZero"}


def _as_int(v):
    return int(v)


@pytest.mark.parametrize("mode", ["laser", "evm"])
def test_vmtests_through_compiler(emu, mode):
    """Every straight-line VMTest: compiled device code == oracle == official post-storage."""
    checked = 0
    for vec in VMTESTS:
        try:
            ts, pairs, expected, pre = vmtest_tapes(vec, mode)
        except Unsupported:
            continue
        empty = np.zeros((max(ts.n_vars, 1), 8, 1), dtype=np.uint32)
        vals = []
        for i, t in enumerate(ts.tapes):
            want = smt_eval.evaluate(t.nodes, ts.pool.values, [])
            # the EVM-exact ADDMOD / MULMOD (z3's 512-bit form) compile to D_ADDMOD / D_MULMOD
            got, _ = emu.eval(ts, i, empty)
            assert got[0] == _as_int(want), (vec["name"], i)
            vals.append(got[0])
        if not (mode == "laser" and vec["name"] in LASER_DIVERGENT):
            assert final_storage(pre, pairs, vals) == expected, vec["name"]
        checked += 1
    assert checked >= 300


@pytest.mark.parametrize("mode", ["laser", "evm"])
def test_vmtests_lifted_through_compiler(emu, mode):
    """The VMTests with every constant lifted into an assignment column: nothing folds, every
    op runs as device code (the folded variant above checks the host folding)."""
    checked = 0
    for vec in VMTESTS:
        try:
            ts, pairs, expected, pre = vmtest_tapes(vec, mode)
        except Unsupported:
            continue
        lts, soa = lift_constants(ts)
        vals = []
        for i, t in enumerate(ts.tapes):
            want = int(smt_eval.evaluate(t.nodes, ts.pool.values, []))
            got, _ = emu.eval(lts, i, soa)
            assert got[0] == want, (vec["name"], i)
            vals.append(got[0])
        if not (mode == "laser" and vec["name"] in LASER_DIVERGENT):
            assert final_storage(pre, pairs, vals) == expected, vec["name"]
        checked += 1
    assert checked >= 300


def test_constant_folding(emu):
    """Constant-only subtrees fold on the host to the value the device computes; a select with
    a constant condition becomes its chosen operand; results match the oracle either way."""
    import random as _r

    rng = _r.Random(77)
    ts = TapeSet()
    b = ts.builder()
    x = b.var("x")
    k1 = b.const(rng.getrandbits(256), 256)
    k2 = b.const(rng.getrandbits(256), 256)
    kk = b.op(Op.BVMUL, b.op(Op.BVADD, k1, k2), b.op(Op.BVUDIV, k1, b.const(7, 256)))
    kx = b.op(Op.EXTRACT, kk, imm0=159, imm1=32)
    sel = b.op(Op.ITE, b.op(Op.BVULT, k1, k2), b.op(Op.BVXOR, x, kk), b.op(Op.BVSUB, x, kk))
    ts.add(b.finish(b.op(Op.BVADD, sel, b.op(Op.ZEXT, kx, imm0=128))))
    ts.add(b.finish(b.op(Op.AND, b.op(Op.BVULT, x, kk), b.op(Op.EQ, k1, k1))))
    soa = assignment_soa(rng, ts.n_vars, 16)
    for i, t in enumerate(ts.tapes):
        got, _ = emu.eval(ts, i, soa)
        for r in range(soa.shape[2]):
            assert got[r] == int(smt_eval.evaluate(t.nodes, ts.pool.values, soa_row(soa, r)))
    folded = emu.n_slots(ts)
    os.environ["MH_NO_FOLD"] = "1"
    try:
        unfolded = emu.n_slots(ts)
    finally:
        del os.environ["MH_NO_FOLD"]
    assert folded < unfolded, (folded, unfolded)


@pytest.mark.parametrize("seed", range(12))
def test_fuzz_tapes(emu, seed):
    rng = random.Random(1000 + seed)
    ts = TapeSet()
    fz = TapeFuzzer(rng, ts, n_vars=3, max_depth=4)
    for _ in range(12):
        fz.tape()
    soa = assignment_soa(rng, ts.n_vars, 24)
    unsupported = 0
    for i, t in enumerate(ts.tapes):
        try:
            got, nregs = emu.eval(ts, i, soa)
        except EmuError as e:
            assert e.code == -2, str(e)
            unsupported += 1
            continue
        for r in range(soa.shape[2]):
            want = smt_eval.evaluate(t.nodes, ts.pool.values, soa_row(soa, r))
            assert got[r] == int(want), (seed, i, r)
    assert unsupported <= 3


def test_division_edges(emu):
    """The division family on the edge values that decide bit-exactness."""
    rng = random.Random(7)
    for w in (8, 31, 64, 160, 255, 256):
        ts = TapeSet()
        b = ts.builder()
        x = b.op(Op.EXTRACT, b.var("x"), imm0=w - 1, imm1=0) if w < 256 else b.var("x")
        y = b.op(Op.EXTRACT, b.var("y"), imm0=w - 1, imm1=0) if w < 256 else b.var("y")
        for op in (Op.BVUDIV, Op.BVUREM, Op.BVSDIV, Op.BVSREM, Op.BVSMOD):
            ts.add(b.finish(b.op(op, x, y)))
        m = (1 << w) - 1
        vals = [0, 1, 2, 3, m, m - 1, 1 << (w - 1), (1 << (w - 1)) - 1, (1 << (w - 1)) + 1]
        vals += [rng.getrandbits(w) for _ in range(6)] + [rng.getrandbits(min(w, 33))
                                                          for _ in range(6)]
        pairs = [(a, c) for a in vals for c in vals]
        soa = np.zeros((2, 8, len(pairs)), dtype=np.uint32)
        for r, (a, c) in enumerate(pairs):
            for k in range(8):
                soa[0, k, r] = (a >> (32 * k)) & 0xFFFFFFFF
                soa[1, k, r] = (c >> (32 * k)) & 0xFFFFFFFF
        for i, t in enumerate(ts.tapes):
            got, _ = emu.eval(ts, i, soa)
            for r, (a, c) in enumerate(pairs):
                want = smt_eval.evaluate(t.nodes, ts.pool.values, [a, c])
                assert got[r] == want, (w, i, hex(a), hex(c))


def test_knuth_add_back_path(emu):
    """Operands that force the rare D6 add-back step of the long division."""
    # classic add-back trigger: u = 0x8000...0000 0000 0003 ..., v = 0x8000...0001 ...
    cases = [
        ((1 << 255) | 3, (1 << 128) | 1),
        ((0x7FFF800000000000 << 192) | 1, (0x800000000001 << 128) | 0xFFFFFFFF),
        ((1 << 256) - 1, (1 << 192) + 1),
        ((1 << 256) - 1, (1 << 224) + (1 << 223) + 1),
    ]
    rng = random.Random(11)
    for _ in range(40):
        v = (rng.getrandbits(32) | 0x80000000) << rng.choice([32, 64, 96, 128, 160, 192])
        v |= rng.getrandbits(32)
        cases.append((rng.getrandbits(256), v))
    ts = TapeSet()
    b = ts.builder()
    x, y = b.var("x"), b.var("y")
    ts.add(b.finish(b.op(Op.BVUDIV, x, y)))
    ts.add(b.finish(b.op(Op.BVUREM, x, y)))
    soa = np.zeros((2, 8, len(cases)), dtype=np.uint32)
    for r, (a, c) in enumerate(cases):
        for k in range(8):
            soa[0, k, r] = (a >> (32 * k)) & 0xFFFFFFFF
            soa[1, k, r] = (c >> (32 * k)) & 0xFFFFFFFF
    q, _ = emu.eval(ts, 0, soa)
    rem, _ = emu.eval(ts, 1, soa)
    for r, (a, c) in enumerate(cases):
        assert q[r] == a // c and rem[r] == a % c, (hex(a), hex(c))


def test_keccak_emulated_against_known_answers(emu):
    from oracle.keccak import keccak256

    ts = TapeSet()
    b = ts.builder()
    # keccak of a 32-byte word (mapping key), 64-byte (key ++ slot), 20-byte address
    x, y = b.var("x"), b.var("y")
    ts.add(b.finish(b.op(Op.KECCAK, x)))
    ts.add(b.finish(b.op(Op.KECCAK, b.op(Op.CONCAT, x, y))))
    ts.add(b.finish(b.op(Op.KECCAK, b.op(Op.EXTRACT, x, imm0=159, imm1=0))))
    rows = [(0, 0), (1, 2), ((1 << 256) - 1, 5), (0x1234 << 100, 1 << 255)]
    soa = np.zeros((2, 8, len(rows)), dtype=np.uint32)
    for r, (a, c) in enumerate(rows):
        for k in range(8):
            soa[0, k, r] = (a >> (32 * k)) & 0xFFFFFFFF
            soa[1, k, r] = (c >> (32 * k)) & 0xFFFFFFFF
    g0, _ = emu.eval(ts, 0, soa)
    g1, _ = emu.eval(ts, 1, soa)
    g2, _ = emu.eval(ts, 2, soa)
    for r, (a, c) in enumerate(rows):
        assert g0[r] == int.from_bytes(keccak256(a.to_bytes(32, "big")), "big")
        assert g1[r] == int.from_bytes(keccak256(a.to_bytes(32, "big") + c.to_bytes(32, "big")),
                                       "big")
        assert g2[r] == int.from_bytes(keccak256((a & ((1 << 160) - 1)).to_bytes(20, "big")),
                                       "big")
    # keccak(0^32) is the VMTests sha3 known answer (vmSha3Test sha3_memSizeQuadraticCost64_2)
    assert g0[0] == 0x290DECD9548B62A8D60345A988386FC84BA6BC95484008F6362F93160EF3E563


def test_register_pressure_reported(emu):
    ts = TapeSet()
    b = ts.builder()
    acc = b.var("x")
    for i in range(40):  # a deep left chain needs few registers
        acc = b.op(Op.BVADD, acc, b.const(i, 256))
    ts.add(b.finish(b.op(Op.BVULT, acc, b.var("y"))))
    soa = np.zeros((2, 8, 1), dtype=np.uint32)
    got, nregs = emu.eval(ts, 0, soa)
    assert nregs <= 5


def test_keccak_message_cuts(emu):
    """Keccak of messages of 1..96 bytes assembled from byte pieces of several widths: the
    compiler re-cuts them into left-aligned words with the pad byte in place (compile.cpp), the
    device absorbs whole words (exec.h keccak_words).  Checked against the oracle's Keccak-256."""
    from oracle.keccak import keccak256

    rng = random.Random(404)
    splits = [[1], [5], [20], [31], [32], [7, 26], [32, 1], [20, 32], [31, 31], [32, 32],
              [12, 32, 8], [32, 32, 1], [30, 3, 32], [32, 32, 31], [32, 32, 32], [8, 8, 8]]
    ts = TapeSet()
    b = ts.builder()
    xs = [b.var("x%d" % i) for i in range(3)]
    for parts in splits:
        node = None
        for i, nb in enumerate(parts):
            p = xs[i] if nb == 32 else b.op(Op.EXTRACT, xs[i], imm0=8 * nb - 1, imm1=0)
            node = p if node is None else b.op(Op.CONCAT, node, p)
        ts.add(b.finish(b.op(Op.KECCAK, node)))
    rows = [[rng.getrandbits(256) for _ in range(3)] for _ in range(6)] + [[0, 0, 0]]
    soa = np.zeros((3, 8, len(rows)), dtype=np.uint32)
    for r, vals in enumerate(rows):
        for v in range(3):
            for k in range(8):
                soa[v, k, r] = (vals[v] >> (32 * k)) & 0xFFFFFFFF
    for t, parts in enumerate(splits):
        got, _ = emu.eval(ts, t, soa)
        for r, vals in enumerate(rows):
            msg = b"".join((vals[i] & ((1 << (8 * nb)) - 1)).to_bytes(nb, "big")
                           for i, nb in enumerate(parts))
            assert got[r] == int.from_bytes(keccak256(msg), "big"), (parts, r)


@pytest.mark.parametrize("op", ["addmod", "mulmod"])
def test_evm_modops(emu, op):
    """EVM_ADDMOD / EVM_MULMOD (exact sum / product mod n) and z3's 512-bit form of them
    (rewritten by the compiler), both zero rules, on edge and random words; constants lifted
    into columns and folded."""
    rng = random.Random(3 if op == "addmod" else 4)
    m = (1 << 256) - 1
    edge = [0, 1, 2, 3, m, m - 1, 1 << 255, (1 << 255) - 1, 1 << 128, (1 << 224) + 5, 0xFFFFFFFF,
            1 << 32]
    rows = [[rng.choice(edge), rng.choice(edge), rng.choice(edge)] for _ in range(80)]
    rows += [[rng.getrandbits(rng.choice([8, 64, 200, 256])) for _ in range(3)] for _ in range(120)]
    rows += [[m, m, n] for n in (1, 2, 3, m, m - 1, 1 << 255, 0)]
    ts = TapeSet(["a", "b", "n"])
    b = ts.builder()
    a_, b_, n_ = (b.var(v, 256) for v in ("a", "b", "n"))
    kind = Op.EVM_ADDMOD if op == "addmod" else Op.EVM_MULMOD
    for zl in (0, 1):
        ts.add(b.finish(b.op(kind, a_, b_, n_, imm0=zl)))
    za, zb, zn = (b.op(Op.ZEXT, x, imm0=256) for x in (a_, b_, n_))
    wide = b.op(Op.BVADD if op == "addmod" else Op.BVMUL, za, zb)
    ts.add(b.finish(b.op(Op.EXTRACT, b.op(Op.BVUREM, wide, zn), imm0=255, imm1=0)))
    soa = np.zeros((3, 8, len(rows)), dtype=np.uint32)
    for r, vals in enumerate(rows):
        for v in range(3):
            for k in range(8):
                soa[v, k, r] = (vals[v] >> (32 * k)) & 0xFFFFFFFF
    for i, t in enumerate(ts.tapes):
        got, _ = emu.eval(ts, i, soa)
        for r, vals in enumerate(rows):
            want = int(smt_eval.evaluate(t.nodes, ts.pool.values, vals))
            u = vals[0] + vals[1] if op == "addmod" else vals[0] * vals[1]
            ref = u % vals[2] if vals[2] else (u & m if i else 0)
            assert want == ref and got[r] == want, (op, i, r)
