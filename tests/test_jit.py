"""The native-code JIT (mythril_amd/csrc/jit.cpp), checked on the host: the machine code it
emits for a tape runs on the test-only wave emulator (tests/native/jit_emu.cpp) and must give
the oracle's value on every row, bit for bit; whole tape sets assemble with comgr.  The GPU runs
the same code in tests/test_gpu_jit.py."""
import json
import os
import random

import numpy as np
import pytest

from mythril_amd import synth
from mythril_amd.tape import Op, TapeSet
from oracle import smt_eval
from tests.emu import (EmuError, jit_build, jit_eval, jit_module, set_short_circuit,
                       set_value_numbering)
from tests.evm_translate import Unsupported, final_storage, lift_constants, vmtest_tapes
from tests.fuzz import TapeFuzzer, assignment_soa, soa_row

HERE = os.path.dirname(os.path.abspath(__file__))
VMTESTS = json.load(open(os.path.join(HERE, "golden", "vmtests.json")))
EIP145 = json.load(open(os.path.join(HERE, "golden", "eip145.json")))
LASER_DIVERGENT = {"addmodDivByZero", "addmodDivByZero1", "addmodDivByZero2", "mulmoddivByZero"}


def soa_of(rows_vals, n_vars):
    soa = np.zeros((n_vars, 8, len(rows_vals)), dtype=np.uint32)
    for r, vals in enumerate(rows_vals):
        for v in range(n_vars):
            for k in range(8):
                soa[v, k, r] = (vals[v] >> (32 * k)) & 0xFFFFFFFF
    return soa


def check_tapes(emu, ts, soa, require_all=True, max_vgpr=128):
    jitted = 0
    for i, t in enumerate(ts.tapes):
        res = jit_eval(emu, ts, i, soa, max_vgpr)
        if not res.ok:
            assert not require_all, (i, res.why)
            continue
        jitted += 1
        for r in range(soa.shape[2]):
            want = int(smt_eval.evaluate(t.nodes, ts.pool.values, soa_row(soa, r)))
            assert res.values[r] == want, (i, r, hex(res.values[r]), hex(want))
    return jitted


@pytest.mark.parametrize("seed", range(8))
def test_fuzz_tapes_jit(emu, seed):
    """Random tapes over every op the JIT covers, narrow and wide, Bool and bit-vector roots."""
    rng = random.Random(9000 + seed)
    ts = TapeSet()
    fz = TapeFuzzer(rng, ts, n_vars=3, max_depth=4, allow_keccak=False)
    for _ in range(24):
        fz.tape()
    soa = assignment_soa(rng, ts.n_vars, 70)
    n = check_tapes(emu, ts, soa, require_all=False)
    assert n >= 12


@pytest.mark.parametrize("seed", range(4))
def test_fuzz_wide_schema_jit(emu, seed):
    """Random tapes over 7 columns (tape sets over 4 columns: the code loads each demanded limb
    from the SoA buffer instead of pinning the columns), every op including the EVM word ops,
    ADDMOD / MULMOD and the overflow predicates: all jitted (retried at 168 VGPRs like
    mh_tapes_jit), values equal to the oracle's on every row."""
    rng = random.Random(7100 + seed)
    ts = TapeSet()
    fz = TapeFuzzer(rng, ts, n_vars=7, max_depth=4, allow_keccak=seed % 2 == 1)
    for _ in range(16):
        fz.tape()
    soa = assignment_soa(rng, ts.n_vars, 70)
    for i, t in enumerate(ts.tapes):
        why, budget = jit_refusal(emu, ts, i, soa)
        assert why is None or "larger than 96 KB" in why, (i, why)
        if why:
            continue
        res = jit_run(emu, ts, i, soa, budget)
        for r in range(soa.shape[2]):
            want = int(smt_eval.evaluate(t.nodes, ts.pool.values, soa_row(soa, r)))
            assert res.values[r] == want, (i, r, hex(res.values[r]), hex(want))


def test_synthetic_tapes_jit(emu):
    """Config-5 tapes (the bench's), every one through the JIT, on generated rows."""
    ts = synth.generate(60)
    seed = synth.load_spec()["assignment_seed"]
    rows = [smt_eval.gen_assignment(seed, ts.n_vars, r) for r in range(100)]
    # plus edge rows: zeros, ones, all-ones, sign bits
    rows += [[0] * 4, [1] * 4, [(1 << 256) - 1] * 4, [1 << 255] * 4, [(1 << 255) - 1, 0, 1, 2]]
    n = check_tapes(emu, ts, soa_of(rows, ts.n_vars), require_all=False)
    assert n >= 55


def test_division_edges_jit(emu):
    rng = random.Random(8)
    for w in (8, 64, 160, 255, 256):
        ts = TapeSet()
        b = ts.builder()
        x = b.op(Op.EXTRACT, b.var("x"), imm0=w - 1, imm1=0) if w < 256 else b.var("x")
        y = b.op(Op.EXTRACT, b.var("y"), imm0=w - 1, imm1=0) if w < 256 else b.var("y")
        for op in (Op.BVUDIV, Op.BVUREM, Op.BVSDIV, Op.BVSREM, Op.BVSMOD):
            ts.add(b.finish(b.op(op, x, y)))
            ts.add(b.finish(b.op(op, x, b.const(rng.getrandbits(w) | 1, w))))
        m = (1 << w) - 1
        vals = [0, 1, 2, 3, m, m - 1, 1 << (w - 1), (1 << (w - 1)) - 1]
        vals += [rng.getrandbits(w) for _ in range(6)] + [rng.getrandbits(min(w, 40))
                                                          for _ in range(6)]
        pairs = [(p, q) for p in vals for q in vals]
        check_tapes(emu, ts, soa_of(pairs, 2))


def division_wave_rows(seed):
    """64-row waves shaped for the division subroutine's uniform paths: (a) every divisor
    >= 2^224 (the top-three-limb estimate), x above and below y; (b) the same with lanes whose
    small divisor exceeds x and lanes with y = 0, which sit outside the digit mask; (c) every
    divisor below 2^32 (the narrow path); (d) negative operands for the signed kinds."""
    rng = random.Random(seed)
    M = (1 << 256) - 1
    rows = []
    for _ in range(64):  # (a)
        y = rng.getrandbits(256) | (1 << (224 + rng.randrange(32)))
        x = rng.choice([rng.getrandbits(256), y + rng.getrandbits(200), y - 1, y, y * 3 & M,
                        rng.getrandbits(255)])
        rows.append([x & M, y])
    for i in range(64):  # (b)
        if i % 3 == 0:
            y = rng.getrandbits(256) | (1 << 255 >> rng.randrange(32))
            rows.append([(y + rng.getrandbits(100)) & M, y])
        elif i % 3 == 1:
            y = rng.getrandbits(rng.choice([8, 40, 100, 200])) + 2
            rows.append([rng.randrange(y), y])
        else:
            rows.append([rng.choice([0, 1, rng.getrandbits(256)]), 0])
    for _ in range(64):  # (c)
        rows.append([rng.getrandbits(256), rng.getrandbits(rng.choice([1, 8, 31, 32])) + 1])
    for _ in range(64):  # (d)
        y = rng.getrandbits(256) | (1 << 255)
        rows.append([rng.getrandbits(256), y if rng.random() < 0.5 else (-y) & M])
    for i in range(128):  # (e) x = q y + {-1, 0, 1}: quotient digits on an integer boundary
        y = rng.getrandbits(rng.choice([40, 100, 200, 230, 255]))  | 1
        q = rng.getrandbits(min(32, 256 - y.bit_length()) if i % 2 else 256 - y.bit_length())
        x = q * y + rng.choice([-1, 0, 0, 1])
        rows.append([x & M, y])
    return rows


def test_division_uniform_paths_jit(emu):
    ts = TapeSet()
    b = ts.builder()
    x, y = b.var("x"), b.var("y")
    for op in (Op.BVUDIV, Op.BVUREM, Op.BVSDIV, Op.BVSREM, Op.BVSMOD):
        ts.add(b.finish(b.op(op, x, y)))
        # a quotient and a remainder of one tape share a call site
        ts.add(b.finish(b.op(Op.BVXOR, b.op(op, x, y), b.op(Op.BVUREM, y, b.op(Op.BVADD, x,
                                                                              b.const(1, 256))))))
    for seed in range(3):
        check_tapes(emu, ts, soa_of(division_wave_rows(seed), 2))


def small_quotient_rows(seed):
    """64-row waves for the division's f32 small-quotient path (every lane that needs a digit
    has y >= 2^224 and an estimate below 2^10): x = q y + r with q up to 1023 and r at both
    ends of [0, y) -- the digit on an integer boundary, where the f32 estimate is one off and a
    correction must run -- plus a wave whose largest quotient reaches 2^10 (the f64 path), and
    waves mixing lanes with x < y and y = 0 (outside the digit mask)."""
    rng = random.Random(seed)
    M = (1 << 256) - 1
    rows = []
    for wave in range(6):
        for i in range(64):
            y = rng.getrandbits(256) | (1 << (224 + rng.randrange(32)))
            qmax = (1 << 10) - 1
            if wave == 5 and i == 0:  # the wave's largest estimate reaches 2^10
                y, qmax = rng.getrandbits(240) | (1 << 240), 1 << 10
            q = qmax if wave == 5 and i == 0 else rng.choice([1, 2, 3, 1023, rng.randrange(1, qmax + 1)])
            r = rng.choice([0, 1, 2, y - 1, y - 2, y - (y >> 20), y >> 20, rng.randrange(y)])
            x = q * y + r
            if x > M or wave == 4 and i % 4 == 0:
                x, y = (rng.randrange(y), y) if i % 8 else (rng.getrandbits(256), 0)
            rows.append([x & M, y])
    return rows


def mixed_top_limb_rows(seed):
    """64-row waves whose lanes alternate divisors with a nonzero top limb (y >= 2^224, the
    small-quotient estimate) and divisors below 2^224 (the long digit loop), x on integer
    boundaries of both (x = k y - 1, k y, k y + y - 1, quotients near 2^10)."""
    rng = random.Random(seed)
    M = (1 << 256) - 1
    rows = []
    for wave in range(4):
        for i in range(64):
            if i % 2:
                y = (1 << 224) + rng.choice([1, 2, rng.getrandbits(20), rng.getrandbits(224)])
                k = rng.choice([1, 2, 1022, 1023, 1024, rng.randrange(1, 1 << 10)])
            else:
                y = rng.getrandbits(rng.choice([32, 100, 200, 224])) | 1
                k = rng.getrandbits(rng.choice([10, 32, 256 - y.bit_length()]))
            x = k * y + rng.choice([-1, 0, y - 1])
            if x > M or x < 0:
                x = rng.randrange(y)
            rows.append([x, y])
    return rows


def test_division_small_quotient_jit(emu):
    ts = TapeSet()
    b = ts.builder()
    x, y = b.var("x"), b.var("y")
    for op in (Op.BVUDIV, Op.BVUREM, Op.BVSDIV, Op.BVSREM, Op.BVSMOD):
        ts.add(b.finish(b.op(op, x, y)))
    for seed in range(4):
        check_tapes(emu, ts, soa_of(small_quotient_rows(seed), 2))
        check_tapes(emu, ts, soa_of(mixed_top_limb_rows(seed), 2))


def test_keccak_message_cuts_jit(emu):
    """Keccak-256 in the native code (the mh_kec subroutine, absorb and byte swaps at the call
    site) for messages of 1..96 bytes cut from several pieces, plus constant pieces: every value
    equals the oracle's (which the reference's known answers pin, tests/test_oracle.py)."""
    rng = random.Random(405)
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
    # constant words mixed in (swapped on the host) and a hash feeding arithmetic
    k = b.const(0xAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFE, 256)
    ts.add(b.finish(b.op(Op.KECCAK, b.op(Op.CONCAT, xs[0], k))))
    ts.add(b.finish(b.op(Op.KECCAK, b.op(Op.CONCAT, k, xs[1]))))
    h = b.op(Op.KECCAK, b.op(Op.CONCAT, xs[0], xs[1]))
    ts.add(b.finish(b.op(Op.BVADD, b.op(Op.BVLSHR, h, b.const(139, 256)), xs[2])))
    rows = [[rng.getrandbits(256) for _ in range(3)] for _ in range(70)] + [[0, 0, 0]]
    assert check_tapes(emu, ts, soa_of(rows, 3)) == len(ts.tapes)


def test_keccak_variant_tapes_jit(emu):
    """SURVEY §8d's keccak variant (config 5 plus one keccak256 of 512 bits per tape)."""
    ts = synth.generate(24, keccak=True)
    soa = assignment_soa(random.Random(406), ts.n_vars, 64)
    assert check_tapes(emu, ts, soa, require_all=False) >= 22


def _kec_ops(emu):
    import collections

    ts = synth.generate(2, keccak=True)
    text, _, _ = jit_module(emu, ts, max_vgpr=168, assemble=False)
    kec = text[text.index("mh_kec:"):text.index(".Lmh_jit_end")]
    return collections.Counter(ln.split()[0] for ln in kec.splitlines()
                               if ln.strip() and not ln.strip().endswith(":")
                               and not ln.startswith("."))


def test_keccak_bitop3_rounds(emu):
    """gfx950's v_bitop3_b32 in the Keccak-f[1600] subroutine (the default): theta's parities as
    XOR3 pairs, D folded into the XOR3 that applies it, chi one op per half -- 120 bitop3 + 58
    alignbit per round (+ iota's xor); the values are pinned by the keccak tests above (emulator,
    which restates bitop3's truth-table semantics) and tests/test_gpu_jit.py (device)."""
    if os.environ.get("MH_JIT_KEC_BITOP3") == "0":
        pytest.skip("bitop3 rounds switched off")
    ops = _kec_ops(emu)
    assert ops["v_bitop3_b32"] == 24 * 120, ops
    assert ops["v_alignbit_b32"] == 24 * 58, ops
    assert ops["v_bfi_b32"] == 0 and ops["v_not_b32"] == 0, ops
    assert sum(ops.values()) <= 24 * 180 + 16, ops


def test_keccak_complement_plan():
    """MH_JIT_KEC_BITOP3=0: lane complementing in the Keccak-f[1600] subroutine, chi mostly as
    AND / OR + xor (2-cycle VALU) instead of xor + v_bfi (4-cycle), the same instruction count
    (the switch is read once per process: checked in a child)."""
    import subprocess
    import sys

    code = (
        "import json\n"
        "from tests.conftest import build_emulator\n"
        "from tests.emu import Emulator\n"
        "from tests.test_jit import _kec_ops\n"
        "print(json.dumps(_kec_ops(Emulator(build_emulator()))))\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", code], cwd=root, capture_output=True, text=True,
                         env=dict(os.environ, MH_JIT_KEC_BITOP3="0"), timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    ops = json.loads(out.stdout.strip().splitlines()[-1])
    get = lambda k: ops.get(k, 0)  # noqa: E731
    assert get("v_bfi_b32") <= 24 * 12, ops
    assert get("v_xnor_b32") <= 24 * 4, ops
    assert get("v_and_b32") + get("v_or_b32") >= 24 * 36, ops
    assert get("v_bitop3_b32") == 0, ops
    assert sum(ops.values()) <= 24 * 260 + 16, ops


def test_immediate_and_variable_shifts_jit(emu):
    rng = random.Random(31)
    ts = TapeSet()
    b = ts.builder()
    x, y = b.var("x"), b.var("y")
    s_sum = b.op(Op.BVADD, x, y)
    for s in list(range(1, 256, 7)) + [32, 64, 96, 128, 224, 255]:
        k = b.const(s, 256)
        for op in (Op.BVSHL, Op.BVLSHR, Op.BVASHR):
            ts.add(b.finish(b.op(op, x, k)))
            ts.add(b.finish(b.op(op, s_sum, k)))
    for op in (Op.BVSHL, Op.BVLSHR, Op.BVASHR):
        ts.add(b.finish(b.op(op, x, y)))
        ts.add(b.finish(b.op(op, x, b.op(Op.BVAND, y, b.const(0x1FF, 256)))))
    vals = [0, 1, (1 << 256) - 1, 1 << 255, (1 << 255) - 1] + [rng.getrandbits(256)
                                                               for _ in range(20)]
    amts = [0, 1, 31, 32, 33, 255, 256, 257, 1 << 200] + [rng.getrandbits(9) for _ in range(16)]
    rows = [[v, amts[(i * 7 + 3) % len(amts)]] for i, v in enumerate(vals * 2)]
    check_tapes(emu, ts, soa_of(rows, 2))


def test_mul_shapes_jit(emu):
    """Multiplication with constant / narrow operands (sparse product columns) and full 256."""
    rng = random.Random(77)
    ts = TapeSet()
    b = ts.builder()
    x, y = b.var("x"), b.var("y")
    consts = [1, 2, 0xFFFFFFFF, 1 << 32, (1 << 64) - 1, 1 << 255, (1 << 256) - 1,
              0xDEADBEEF << 96, rng.getrandbits(256)]
    for c in consts:
        ts.add(b.finish(b.op(Op.BVMUL, x, b.const(c, 256))))
    ts.add(b.finish(b.op(Op.BVMUL, x, y)))
    ts.add(b.finish(b.op(Op.BVMUL, x, x)))
    for w in (8, 32, 160):
        xe = b.op(Op.ZEXT, b.op(Op.EXTRACT, x, imm0=w - 1, imm1=0), imm0=256 - w)
        ye = b.op(Op.ZEXT, b.op(Op.EXTRACT, y, imm0=w - 1, imm1=0), imm0=256 - w)
        ts.add(b.finish(b.op(Op.BVMUL, xe, ye)))
        ts.add(b.finish(b.op(Op.BVMUL, xe, y)))
    vals = [0, 1, (1 << 256) - 1, 1 << 255] + [rng.getrandbits(256) for _ in range(20)]
    rows = [[v, vals[(i * 5 + 1) % len(vals)]] for i, v in enumerate(vals)]
    check_tapes(emu, ts, soa_of(rows, 2))


@pytest.mark.parametrize("op", ["shl", "shr", "sar"])
def test_eip145_jit(emu, op):
    """EIP-145 vectors (reference tests/instructions/*_test.py) through the JIT's code."""
    sop = {"shl": Op.BVSHL, "shr": Op.BVLSHR, "sar": Op.BVASHR}[op]
    ts = TapeSet()
    b = ts.builder()
    ts.add(b.finish(b.op(sop, b.var("value"), b.var("shift"))))
    rows = [[int(v["value"], 16), int(v["shift"], 16)] for v in EIP145[op]]
    res = jit_eval(emu, ts, 0, soa_of(rows, 2))
    assert res.ok
    assert res.values == [int(v["expected"], 16) for v in EIP145[op]]


# Why the native code may refuse a VMTest tape: none is expected (the tests below assert every
# tape is jitted); a refusal would have to name one of these.
JIT_REFUSALS = ()


def jit_refusal(emu, ts, i, soa):
    """(None, (max_vgpr, value numbering)) when tape i is jitted, else (the refusal text, None).
    As mh_tapes_jit: a tape over the 128-VGPR budget is retried at 168 (its own occupancy
    class), and one still over it, in a tape set whose columns load on use, with a load per use."""
    tries = [(128, 1), (168, 1)] + ([(168, 2)] if ts.n_vars > 4 else [])
    for budget, vn in tries:
        set_value_numbering(emu, vn)
        try:
            res = jit_eval(emu, ts, i, soa, budget)
        except EmuError as e:
            if "lowering:" not in str(e):
                raise
            return str(e), None
        finally:
            set_value_numbering(emu, 1)
        if res.ok:
            return None, (budget, vn)
        if "VGPR pressure" not in res.why:
            break
    return res.why, None


def jit_run(emu, ts, i, soa, how):
    """jit_eval at the (budget, value numbering) jit_refusal found."""
    set_value_numbering(emu, how[1])
    try:
        return jit_eval(emu, ts, i, soa, how[0])
    finally:
        set_value_numbering(emu, 1)


@pytest.mark.parametrize("mode", ["laser", "evm"])
@pytest.mark.parametrize("keep_exp", [False, True])
def test_vmtests_lifted_jit(emu, mode, keep_exp):
    """The reference's VMTests known answers with every constant lifted into a column (so no op
    folds on the host; keep_exp: EXP exponents stay constant): each op of each vector runs as
    JIT code, tape sets over 4 columns loading the limbs each use demands.  Every refusal is one
    of JIT_REFUSALS; the storage the jitted tapes produce is the vector's post-state whenever
    every tape of the vector is jitted."""
    checked, full, refused = 0, 0, {}
    for vec in VMTESTS:
        try:
            ts, pairs, expected, pre = vmtest_tapes(vec, mode)
        except Unsupported:
            continue
        lts, soa = lift_constants(ts, keep_exponents=keep_exp)
        vals, complete = [], True
        for i, t in enumerate(ts.tapes):
            why, budget = jit_refusal(emu, lts, i, soa)
            want = int(smt_eval.evaluate(t.nodes, ts.pool.values, []))
            if why is not None:
                assert any(r in why for r in JIT_REFUSALS), (vec["name"], i, why)
                refused.setdefault(why.split("(")[0].split(":")[-1].strip(), []).append(vec["name"])
                complete = False
                vals.append(want)
                continue
            got = jit_run(emu, lts, i, soa, budget).values[0]
            assert got == want, (vec["name"], i, hex(got), hex(want))
            vals.append(got)
            checked += 1
        if complete:
            full += 1
            if not (mode == "laser" and vec["name"] in LASER_DIVERGENT):
                assert final_storage(pre, pairs, vals) == expected, vec["name"]
    print("%s: %d tapes jitted, %d vectors fully native, refused: %s" % (
        mode, checked, full, {k: len(set(v)) for k, v in refused.items()}))
    assert not refused and checked >= 1350 and full >= 340


def test_module_assembles(emu):
    """A tape set's whole code object (count and values kernels) assembles and links with comgr
    for gfx950."""
    ts = synth.generate(120)
    for values in (False, True):
        text, nbytes, nj = jit_module(emu, ts, values=values)
        assert nj >= 110
        assert nbytes > 1000
        assert ".amdhsa_kernel mh_jit" in text


def test_occupancy_classes(emu, monkeypatch):
    """build_tapeset bins tapes by the VGPRs their code object needs: every jitted tape lands in
    exactly one code object, each object's VGPR count is within its class ceiling (so it runs at
    that class's waves per SIMD), tapes keep their order inside an object, and one class (the
    default, MH_JIT_CLASSES=0) gives the same tapes in objects at the single budget."""
    ts = synth.generate(300)
    monkeypatch.setenv("MH_JIT_CLASSES", "64,80,96")
    objs, where = jit_build(emu, ts)
    assert (where >= 0).sum() == 300
    ceilings = (64, 80, 96, 128)
    for i, (maxv, n) in enumerate(objs):
        assert n == (where == i).sum() and n > 0
        assert maxv <= 128
    # objects of a lower class really are smaller (more waves per SIMD)
    assert min(m for m, _ in objs) <= 80
    classes = sorted({min(c for c in ceilings if c >= m) for m, _ in objs})
    assert len(classes) >= 2, objs
    for i in range(len(objs)):
        ids = np.nonzero(where == i)[0]
        assert np.all(np.diff(ids) > 0)
    monkeypatch.setenv("MH_JIT_CLASSES", "0")
    objs1, where1 = jit_build(emu, ts)
    assert np.array_equal(where1 >= 0, where >= 0)
    assert len(objs1) <= 4


def test_jit_coverage_and_static_cost(emu):
    """How much of config 5 the JIT takes, and its static instruction counts (informational
    bounds: every tape fits the 128-VGPR budget; far fewer VALU per op than the interpreter)."""
    ts = synth.generate(200)
    soa = np.zeros((4, 8, 1), dtype=np.uint32)
    ok, valu, nodes = 0, 0, 0
    for i, t in enumerate(ts.tapes):
        r = jit_eval(emu, ts, i, soa)
        if r.ok:
            ok += 1
            valu += r.n_valu
            nodes += len(t.nodes)
    assert ok >= 195, ok
    print("jitted %d/200, %.1f static VALU per tape node" % (ok, valu / max(nodes, 1)))


def _hazards(text):
    """Pairs of adjacent instructions in the module text that break a manually inserted wait
    state of CDNA3/4 the JIT must honour: a VALU write of vN directly followed by
    v_readlane / v_readfirstlane of vN; v_rcp_f64 / v_rcp_f32 directly followed by a use of its result;
    a VALU write of an SGPR directly followed by a global_* instruction using that SGPR."""
    import re
    bad = []
    prev = None
    for ln in text.splitlines():
        ln = ln.strip()
        if not ln or ln.endswith(":") or ln.startswith("."):
            continue
        ins = ln.split()[0]
        if prev is not None and not ins.startswith("s_nop"):
            p_ins, p_ops = prev
            dst = p_ops[0] if p_ops else ""
            if ins in ("v_readlane_b32", "v_readfirstlane_b32") and p_ins.startswith("v_"):
                src = ln.split()[2].rstrip(",")
                if re.fullmatch(r"v\d+", dst) and dst == src:
                    bad.append((prev, ln))
            if p_ins in ("v_rcp_f64", "v_rcp_f32"):
                bad.append((prev, ln))
            if ins.startswith("global_") and p_ins.startswith("v_") and dst.startswith("s"):
                if dst.split("[")[0] in ln or dst in ln:
                    bad.append((prev, ln))
        if ins.startswith("s_nop"):
            prev = None
        else:
            ops = [x.strip(",") for x in ln.split()[1:]]
            prev = (ins, ops)
    return bad


def test_module_wait_states(emu):
    """The generated text honours the wait states above (the round-2 bring-up hit the first:
    a stale wave index read by v_readfirstlane right after the VALU that wrote it)."""
    ts = synth.generate(60)
    for values in (False, True):
        text, _, _ = jit_module(emu, ts, values=values, assemble=False)
        assert _hazards(text) == []


def test_short_circuit_jit(emu):
    """Short-circuit conjunctions (Options::short_circuit, on by default): config-5 tapes and
    LASER-like conjunctions give the same root value on every row as the full evaluation and
    the oracle, while executing far fewer VALU per wave; a partial last chunk (70 rows) whose
    only satisfying lanes lie past the end still counts nothing for them."""
    ts = synth.generate(40)
    seed = synth.load_spec()["assignment_seed"]
    rows = [smt_eval.gen_assignment(seed, ts.n_vars, r) for r in range(130)]
    soa = soa_of(rows, ts.n_vars)
    dyn = {}
    try:
        for sc in (False, True):
            set_short_circuit(emu, sc)
            vals, valu = [], 0
            for i in range(len(ts.tapes)):
                res = jit_eval(emu, ts, i, soa)
                assert res.ok, res.why
                vals.append(res.values)
                valu += res.dyn["valu"]
            dyn[sc] = (vals, valu)
    finally:
        set_short_circuit(emu, True)
    assert dyn[True][0] == dyn[False][0]
    assert dyn[True][1] < 0.6 * dyn[False][1], (dyn[True][1], dyn[False][1])
    for i, t in enumerate(ts.tapes[:10]):
        for r in range(0, len(rows), 7):
            assert dyn[True][0][i][r] == int(smt_eval.evaluate(t.nodes, ts.pool.values,
                                                                soa_row(soa, r)))
    # conjunctions whose conjuncts hold on some lanes only: x < 2^255, y == x & 0xff..,
    # z != 0, ite-guarded mul, with row 0 (copied into the unused lanes of the last chunk)
    # the only row satisfying the cheap conjunct
    ts2 = TapeSet(["x", "y", "z"])
    b = ts2.builder()
    x, y, z = (b.var(v, 256) for v in ("x", "y", "z"))
    c = lambda v: b.const(v, 256)
    eq = b.op(Op.EQ, y, c(12345))
    lt = b.op(Op.BVULT, x, c(1 << 255))
    nz = b.op(Op.NOT, b.op(Op.EQ, z, c(0)))
    mul = b.op(Op.BVUGT, b.op(Op.BVMUL, x, z), c(7))
    root = b.op(Op.AND, b.op(Op.AND, b.op(Op.AND, mul, nz), lt), eq)
    ts2.add(b.finish(root))
    rng = random.Random(77)
    rws = []
    for r in range(70):
        rws.append([rng.getrandbits(256 - (r % 3)), 12345 if r in (0, 5, 40) else rng.getrandbits(8),
                    rng.getrandbits(256) if r % 4 else 0])
    soa2 = soa_of(rws, 3)
    res = jit_eval(emu, ts2, 0, soa2)
    assert res.ok, res.why
    for r in range(70):
        want = int(smt_eval.evaluate(ts2.tapes[0].nodes, ts2.pool.values, soa_row(soa2, r)))
        assert res.values[r] == want, r
    assert res.values[0] == 1 or res.values[5] == 1 or res.values[40] == 1


def test_short_circuit_constant_conjuncts_jit(emu):
    """Conjunctions with constant conjuncts (a known-false one is scheduled first and ends every
    wave by an unconditional branch; a known-true one never tests) and a Bool-valued root that is
    not a conjunction: values equal the oracle's and the full evaluation's."""
    ts = TapeSet(["x", "y", "z"])
    b = ts.builder()
    x, y, z = (b.var(v, 256) for v in ("x", "y", "z"))
    lt = b.op(Op.BVULT, x, y)
    eq = b.op(Op.EQ, b.op(Op.BVAND, z, b.const(1, 256)), b.const(1, 256))
    mul = b.op(Op.BVUGT, b.op(Op.BVMUL, x, z), y)
    ts.add(b.finish(b.op(Op.AND, b.op(Op.AND, lt, b.false()), eq)))
    ts.add(b.finish(b.op(Op.AND, b.op(Op.AND, b.true(), lt), b.op(Op.AND, mul, eq))))
    ts.add(b.finish(b.op(Op.OR, lt, b.op(Op.AND, eq, mul))))
    ts.add(b.finish(b.op(Op.AND, lt, lt)))
    rng = random.Random(12)
    rows = [[rng.getrandbits(256) for _ in range(3)] for _ in range(130)]
    soa = soa_of(rows, 3)
    for sc in (True, False):
        set_short_circuit(emu, sc)
        try:
            assert check_tapes(emu, ts, soa) == len(ts.tapes)
        finally:
            set_short_circuit(emu, True)


def test_laser_query_tapes_jit(emu):
    """The sieve's tape sets for the LASER-shaped queries (tests/laser_like.py, SAT and the UNSAT
    hard variants; 1..109 columns, so most load their limbs on use) through the JIT's code on
    guided rows (oracle/guided_gen.py, the device generator's restatement): every tape jitted,
    values equal to the oracle's on every row."""
    from oracle.guided_gen import generate_row
    from tests.laser_like import hard_queries, queries, query_tapeset

    n = 0
    for maker in (queries, hard_queries):
        ctx, qs = maker()
        for name, cs in qs:
            ts, schema, guide = query_tapeset(ctx.b, cs)
            rows = [generate_row(0xC0FFEE, g, guide) for g in range(96)]
            soa = soa_of(rows, max(ts.n_vars, 1))
            for i, t in enumerate(ts.tapes):
                why, budget = jit_refusal(emu, ts, i, soa)
                assert why is None, (name, i, why)
                res = jit_run(emu, ts, i, soa, budget)
                for r in range(len(rows)):
                    want = int(smt_eval.evaluate(t.nodes, ts.pool.values, rows[r]))
                    assert res.values[r] == want, (name, i, r)
                n += 1
    assert n >= 30


@pytest.mark.parametrize("mode", ["laser", "evm"])
def test_vmtest_batch_jit(emu, mode):
    """The corpus as tests/test_gpu_native.py hands it to mh_tapes_jit: every vector's tapes in
    one tape set over the shared lifted columns (about 100, all loaded on use).  Every tape is
    jitted (with mh_tapes_jit's retries) and its value is the oracle's."""
    from tests.evm_translate import vmtest_batch

    ts, soa, index = vmtest_batch(VMTESTS, mode, True)
    row = soa_row(soa, 0)
    for i, t in enumerate(ts.tapes):
        why, how = jit_refusal(emu, ts, i, soa)
        assert why is None, (i, why)
        got = jit_run(emu, ts, i, soa, how).values[0]
        assert got == int(smt_eval.evaluate(t.nodes, ts.pool.values, row)), i


# 64-row chunks of config 5 where MI355X's native code once missed a hit (one Newton step on
# v_rcp_f64 left a digit estimate too far off for the division's skipped-correction test;
# scripts/diag_find_row.py located them at 2^24 and 2^25 rows): (tape, first row of the chunk)
DIV_REGRESSION_CHUNKS = ((2191, 10630848), (8720, 21484032))


def test_division_regression_chunks_jit(emu):
    ts = synth.generate()
    seed = synth.load_spec()["assignment_seed"]
    for tape, r0 in DIV_REGRESSION_CHUNKS:
        rows = [smt_eval.gen_assignment(seed, ts.n_vars, r0 + i) for i in range(64)]
        sub = TapeSet(ts.var_names)
        sub.pool = ts.pool
        sub.tapes = [ts.tapes[tape]]
        check_tapes(emu, sub, soa_of(rows, ts.n_vars))
