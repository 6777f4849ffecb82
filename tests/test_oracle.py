"""The oracle pinned against every known answer the reference's tests hold for this path
(SURVEY.md §8c), before it is trusted as the checker for the HIP path."""
import hashlib
import json
import os
import random

import pytest

from mythril_amd import smt
from mythril_amd.smt import (BVAddNoOverflow, BVMulNoOverflow, BVSubNoUnderflow, Concat,
                             Extract, If, LShR, SRem, UDiv, UGE, ULE, URem, symbol_factory)
from oracle import ctape, smt_eval
from oracle.keccak import keccak256, keccak256_int, sha3_256_fips
from tests.evm_translate import Unsupported, final_storage, vmtest_tapes

HERE = os.path.dirname(os.path.abspath(__file__))
VMTESTS = json.load(open(os.path.join(HERE, "golden", "vmtests.json")))
EIP145 = json.load(open(os.path.join(HERE, "golden", "eip145.json")))

# LASER lowers ADDMOD/MULMOD to 256-bit URem chains (instructions.py:569-596) with no guard for
# a zero modulus, and SMT-LIB defines x bvurem 0 = x: the VMTest expects 0, LASER's term gives
# (a + b) / (a * b).  The reference's own evm_test would disagree on these four as well.
LASER_DIVERGENT = {"addmodDivByZero": 5, "addmodDivByZero1": 1, "addmodDivByZero2": 1,
                   "mulmoddivByZero": 5}


# ---- Keccak-256 ------------------------------------------------------------------------------
@pytest.mark.parametrize("n", [0, 1, 31, 32, 64, 135, 136, 137, 200, 271, 272, 500])
def test_keccak_permutation_matches_hashlib_sha3(n):
    data = bytes((7 * i + 3) & 0xFF for i in range(n))
    assert sha3_256_fips(data) == hashlib.sha3_256(data).digest()


def test_keccak_known_answers():
    # keccak_function_manager.py:80 (get_empty_keccak_hash)
    assert int.from_bytes(keccak256(b""), "big") == \
        89477152217924674838424037953991966239322087453347756267410168184682657981552
    # VMTests vmSha3Test: sha3_1 (5 zero bytes), sha3_memSizeQuadraticCost64_2 (32 zero bytes)
    assert keccak256(bytes(5)).hex() == \
        "c41589e7559804ea4a2080dad19d876a024ccb05117835447d72ce08c1d020ec"
    assert keccak256(bytes(32)).hex() == \
        "290decd9548b62a8d60345a988386fc84ba6bc95484008f6362f93160ef3e563"
    # selectors: tests/cmd_line_test.py:27-29, README.md:73-75
    assert keccak256(b"setOwner(address)")[:4].hex() == "13af4035"
    assert keccak256(b"killerize(address)")[:4].hex() == "9fa299cc"
    assert keccak256(b"activatekillability()")[:4].hex() == "84057065"
    assert keccak256(b"commencekilling()")[:4].hex() == "7c11da20"
    assert keccak256_int(100, 32) == int.from_bytes(keccak256((100).to_bytes(32, "big")), "big")


# ---- VMTests (official Ethereum known answers, run by the reference through LASER) -----------
@pytest.mark.parametrize("mode", ["laser", "evm"])
def test_vmtests(mode):
    ok = 0
    for vec in VMTESTS:
        try:
            ts, pairs, expected, pre = vmtest_tapes(vec, mode)
        except Unsupported:
            assert vec["name"] == "sha3_bigOffset2"
            continue
        vals = [smt_eval.evaluate(t.nodes, ts.pool.values, []) for t in ts.tapes]
        got = final_storage(pre, pairs, vals)
        if mode == "laser" and vec["name"] in LASER_DIVERGENT:
            assert got == {0: LASER_DIVERGENT[vec["name"]]}
            assert expected == {}
            continue
        assert got == expected, vec["name"]
        ok += 1
    assert ok >= 337


def test_vmtests_c_oracle_agrees():
    for vec in VMTESTS[::3]:
        try:
            ts, pairs, expected, pre = vmtest_tapes(vec, "evm")
        except Unsupported:
            continue
        for i, t in enumerate(ts.tapes):
            assert ctape.evaluate(ts, i, []) == int(smt_eval.evaluate(t.nodes, ts.pool.values,
                                                                       [])), vec["name"]


# ---- EIP-145 shift vectors (tests/instructions/{shl,shr,sar}_test.py) -------------------------
@pytest.mark.parametrize("op", ["shl", "shr", "sar"])
def test_eip145(op):
    assert EIP145[op]
    for v in EIP145[op]:
        ctx = smt.set_context(smt.Context())
        value = symbol_factory.BitVecVal(int(v["value"], 16), 256)
        shift = symbol_factory.BitVecVal(int(v["shift"], 16), 256)
        # instructions.py:528-552: SHL value << shift, SHR LShR(value, shift), SAR value >> shift
        e = {"shl": lambda: value << shift, "shr": lambda: LShR(value, shift),
             "sar": lambda: value >> shift}[op]()
        t = ctx.tape(e)
        assert smt_eval.evaluate(t.nodes, ctx.tapeset.pool.values, []) == int(v["expected"], 16)


# ---- SMT-LIB semantics the reference's terms rely on -----------------------------------------
def _ev(expr):
    ctx = expr.ctx
    t = ctx.tape(expr)
    return smt_eval.evaluate(t.nodes, ctx.tapeset.pool.values, [])


def test_smtlib_division_rules():
    smt.set_context(smt.Context())
    B = lambda x, w=8: symbol_factory.BitVecVal(x & ((1 << w) - 1), w)  # noqa: E731
    assert _ev(UDiv(B(7), B(0))) == 0xFF  # bvudiv x 0 = all ones
    assert _ev(URem(B(7), B(0))) == 7     # bvurem x 0 = x
    assert _ev(B(-7) / B(2)) == (-3) & 0xFF  # bvsdiv truncates toward zero
    assert _ev(SRem(B(-7), B(2))) == (-1) & 0xFF  # sign of dividend
    assert _ev(smt.SMod(B(-7), B(2))) == 1        # sign of divisor
    assert _ev(smt.SMod(B(7), B(-2))) == (-1) & 0xFF
    assert _ev(B(-7) / B(0)) == 1          # -(all ones) for negative dividend
    assert _ev(B(7) / B(0)) == 0xFF
    assert _ev(SRem(B(-7), B(0))) == (-7) & 0xFF
    assert _ev(B(-128) / B(-1)) == 0x80   # overflow wraps


def test_laser_constructions():
    smt.set_context(smt.Context())
    a = symbol_factory.BitVecVal(5, 256)
    b = symbol_factory.BitVecVal(7, 256)
    assert _ev(UGE(b, a)) is True and _ev(ULE(b, a)) is False
    assert _ev(If(a == 5, 1, 2)) == 1
    assert _ev(Concat(symbol_factory.BitVecVal(1, 8), symbol_factory.BitVecVal(2, 8))) == 0x102
    assert _ev(Extract(7, 0, symbol_factory.BitVecVal(0x1234, 256))) == 0x34
    # mixed-width equality zero-pads (bitvec.py:16-22)
    assert _ev(symbol_factory.BitVecVal(3, 8) == symbol_factory.BitVecVal(3, 256)) is True
    m = (1 << 256) - 1
    assert _ev(BVAddNoOverflow(symbol_factory.BitVecVal(m, 256), 1, False)) is False
    assert _ev(BVAddNoOverflow(symbol_factory.BitVecVal(m - 1, 256), 1, False)) is True
    assert _ev(BVMulNoOverflow(symbol_factory.BitVecVal(1 << 128, 256), 1 << 128, False)) is False
    assert _ev(BVSubNoUnderflow(1, symbol_factory.BitVecVal(2, 256), False)) is False
    assert _ev(BVAddNoOverflow(symbol_factory.BitVecVal(1 << 254, 256), 1 << 254, True)) is False


def test_calldata_shape():
    """calldata.py:47-54,219-232: CALLDATALOAD is a Concat of 32 guarded byte reads."""
    ctx = smt.set_context(smt.Context())
    size = symbol_factory.BitVecSym("1_calldatasize", 256)
    byte_vars = [symbol_factory.BitVecSym("cd%d" % i, 8) for i in range(4)]
    word = Concat([If(smt.ULT(symbol_factory.BitVecVal(i, 256), size), byte_vars[i],
                      symbol_factory.BitVecVal(0, 8)) for i in range(4)])
    t = ctx.tape(word == 0x11223344)
    names = ctx.tapeset.var_names
    assign = [0] * len(names)
    assign[names.index("1_calldatasize")] = 4
    for i, v in enumerate([0x11, 0x22, 0x33, 0x44]):
        assign[names.index("cd%d" % i)] = v
    assert smt_eval.evaluate(t.nodes, ctx.tapeset.pool.values, assign) is True
    assign[names.index("1_calldatasize")] = 3
    assert smt_eval.evaluate(t.nodes, ctx.tapeset.pool.values, assign) is False


def test_c_oracle_matches_python_oracle_fuzz():
    from mythril_amd.tape import TapeSet
    from tests.fuzz import TapeFuzzer, interesting

    for seed in range(8):
        rng = random.Random(seed)
        ts = TapeSet()
        fz = TapeFuzzer(rng, ts, 3, max_depth=4)
        for _ in range(8):
            fz.tape()
        for i, t in enumerate(ts.tapes):
            for _ in range(6):
                a = [interesting(rng, 256) for _ in range(3)]
                assert ctape.evaluate(ts, i, a) == int(smt_eval.evaluate(t.nodes, ts.pool.values,
                                                                           a))


def test_generator_reproducible():
    from mythril_amd import synth

    a, b = synth.generate(20), synth.generate(20)
    for x, y in zip(a.tapes, b.tapes):
        assert (x.nodes == y.nodes).all()
    assert a.pool.values == b.pool.values
    sizes = [len(t.nodes) for t in a.tapes]
    assert min(sizes) >= 16


def test_c_oracle_short_circuit_counts():
    """ct_count_lazy (a Bool AND's second operand evaluated only when the first holds, the CPU
    baseline's evaluator) gives the eager evaluator's counts and first witnesses."""
    from mythril_amd import synth

    ts = synth.generate(60)
    seed = synth.load_spec()["assignment_seed"]
    eager = ctape.count(ts, seed, 0, 3000, threads=4)
    lazy = ctape.count(ts, seed, 0, 3000, threads=4, short_circuit=True)
    assert (eager[0] == lazy[0]).all() and (eager[1] == lazy[1]).all()
    assert eager[0].sum() > 0
