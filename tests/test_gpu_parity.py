"""HIP path (libmythril_hip on an MI355X) vs the CPU oracle.  Every check is bit-exact.

Run on the GPU box:  python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
"""
import json
import os
import random

import numpy as np
import pytest

from mythril_amd import native, synth
from mythril_amd.tape import Op, TapeSet
from oracle import smt_eval
from tests.evm_translate import Unsupported, final_storage, lift_constants, vmtest_tapes
from tests.fuzz import TapeFuzzer, assignment_soa, soa_row

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
VMTESTS = json.load(open(os.path.join(HERE, "golden", "vmtests.json")))
LASER_DIVERGENT = {"addmodDivByZero", "addmodDivByZero1", "addmodDivByZero2", "mulmoddivByZero"}


def upload(ctx, soa):
    a = ctx.assignments(soa.shape[0], soa.shape[2])
    a.upload(soa)
    return a


def test_library_and_device(gpu_ctx):
    assert native.version() == (0, 1, 0)
    assert native.device_count() >= 1


def test_generator_matches_oracle(gpu_ctx):
    seed, base, rows = 0xDEADBEEF, 12345, 1000
    a = gpu_ctx.assignments(4, rows)
    a.generate(seed, base)
    got = a.download(0, rows)
    for r in list(range(0, rows, 97)) + [rows - 1]:
        for v in range(4):
            for k in range(8):
                want = smt_eval.gen_limb(seed, v, base + r, k)
                assert int(got[v, k, r]) == want == native.gen_limb(seed, v, base + r, k)


@pytest.mark.parametrize("mode", ["laser", "evm"])
def test_vmtests_on_gpu(gpu_ctx, mode):
    """The reference's VMTests known answers, evaluated by the kernel."""
    checked = 0
    for vec in VMTESTS:
        try:
            ts, pairs, expected, pre = vmtest_tapes(vec, mode)
        except Unsupported:
            continue
        # EVM-exact ADDMOD / MULMOD arrive in z3's 512-bit form; the compiler rewrites them to
        # the device's D_ADDMOD / D_MULMOD
        ct = gpu_ctx.compile(ts)
        a = gpu_ctx.assignments(max(ts.n_vars, 1), 1)
        a.upload(np.zeros((max(ts.n_vars, 1), 8, 1), dtype=np.uint32))
        vals = []
        for i, t in enumerate(ts.tapes):
            got = native.limbs_to_ints(native.eval_values(gpu_ctx, ct, i, a))[0]
            want = int(smt_eval.evaluate(t.nodes, ts.pool.values, []))
            assert got == want, (vec["name"], i)
            vals.append(got)
        if not (mode == "laser" and vec["name"] in LASER_DIVERGENT):
            assert final_storage(pre, pairs, vals) == expected, vec["name"]
        checked += 1
    assert checked >= 300


@pytest.mark.parametrize("mode", ["laser", "evm"])
def test_vmtests_lifted_on_gpu(gpu_ctx, mode):
    """The VMTests known answers with every constant lifted into an assignment column, so no op
    folds on the host: the kernel's own handlers compute every operation of every vector."""
    checked = 0
    for vec in VMTESTS:
        try:
            ts, pairs, expected, pre = vmtest_tapes(vec, mode)
        except Unsupported:
            continue
        lts, soa = lift_constants(ts)
        ct = gpu_ctx.compile(lts)
        a = upload(gpu_ctx, soa)
        vals = []
        for i, t in enumerate(ts.tapes):
            got = native.limbs_to_ints(native.eval_values(gpu_ctx, ct, i, a))[0]
            want = int(smt_eval.evaluate(t.nodes, ts.pool.values, []))
            assert got == want, (vec["name"], i)
            vals.append(got)
        if not (mode == "laser" and vec["name"] in LASER_DIVERGENT):
            assert final_storage(pre, pairs, vals) == expected, vec["name"]
        checked += 1
    assert checked >= 300


@pytest.mark.parametrize("op", ["addmod", "mulmod"])
def test_evm_modops_on_gpu(gpu_ctx, op):
    """EVM_ADDMOD / EVM_MULMOD (exact sum / product mod n, both zero rules) and z3's 512-bit
    form of them, by the kernel on edge and random words, against the oracle."""
    rng = random.Random(30 if op == "addmod" else 31)
    m = (1 << 256) - 1
    edge = [0, 1, 2, 3, m, m - 1, 1 << 255, (1 << 255) - 1, 1 << 128, (1 << 224) + 5,
            0xFFFFFFFF, 1 << 32]
    rows = [[rng.choice(edge) for _ in range(3)] for _ in range(100)]
    rows += [[rng.getrandbits(rng.choice([8, 64, 200, 256])) for _ in range(3)] for _ in range(156)]
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
    ct = gpu_ctx.compile(ts)
    a = upload(gpu_ctx, soa)
    for i, t in enumerate(ts.tapes):
        got = native.limbs_to_ints(native.eval_values(gpu_ctx, ct, i, a))
        for r, vals in enumerate(rows):
            assert got[r] == int(smt_eval.evaluate(t.nodes, ts.pool.values, vals)), (op, i, r)


@pytest.mark.parametrize("seed", range(6))
def test_fuzz_tapes_on_gpu(gpu_ctx, seed):
    rng = random.Random(5000 + seed)
    ts = TapeSet()
    fz = TapeFuzzer(rng, ts, n_vars=3, max_depth=4)
    for _ in range(16):
        fz.tape()
    soa = assignment_soa(rng, ts.n_vars, 96)
    ct = gpu_ctx.compile(ts)
    a = upload(gpu_ctx, soa)
    for i, t in enumerate(ts.tapes):
        got = native.limbs_to_ints(native.eval_values(gpu_ctx, ct, i, a))
        for r in range(soa.shape[2]):
            want = int(smt_eval.evaluate(t.nodes, ts.pool.values, soa_row(soa, r)))
            assert got[r] == want, (seed, i, r)


def test_immediate_shifts_on_gpu(gpu_ctx):
    """Every constant amount 1..255 of bvshl / bvlshr, with the operand in a register (a column)
    and in the accumulator (a sum), result kept in X or written back (used twice): the
    limb-specialised shift bodies of the asm core against the oracle."""
    rng = random.Random(31)
    ts = TapeSet()
    b = ts.builder()
    x, y = b.var("x"), b.var("y")
    s_sum = b.op(Op.BVADD, x, y)
    for s in range(1, 256):
        k = b.const(s, 256)
        for op in (Op.BVSHL, Op.BVLSHR):
            ts.add(b.finish(b.op(op, x, k)))
            ts.add(b.finish(b.op(op, s_sum, k)))
            t = b.op(op, s_sum, k)
            ts.add(b.finish(b.op(Op.BVADD, b.op(Op.BVXOR, t, y), t)))
    vals = [0, 1, (1 << 256) - 1, 1 << 255, (1 << 255) - 1] + [rng.getrandbits(256)
                                                               for _ in range(27)]
    soa = np.zeros((2, 8, len(vals)), dtype=np.uint32)
    for r, v in enumerate(vals):
        w = vals[(r * 7 + 3) % len(vals)]
        for k in range(8):
            soa[0, k, r] = (v >> (32 * k)) & 0xFFFFFFFF
            soa[1, k, r] = (w >> (32 * k)) & 0xFFFFFFFF
    ct = gpu_ctx.compile(ts)
    a = upload(gpu_ctx, soa)
    for i, t in enumerate(ts.tapes):
        got = native.limbs_to_ints(native.eval_values(gpu_ctx, ct, i, a))
        for r in range(len(vals)):
            want = int(smt_eval.evaluate(t.nodes, ts.pool.values, soa_row(soa, r)))
            assert got[r] == want, (i, r)


def test_division_edges_on_gpu(gpu_ctx):
    rng = random.Random(8)
    for w in (8, 64, 160, 255, 256):
        ts = TapeSet()
        b = ts.builder()
        x = b.op(Op.EXTRACT, b.var("x"), imm0=w - 1, imm1=0) if w < 256 else b.var("x")
        y = b.op(Op.EXTRACT, b.var("y"), imm0=w - 1, imm1=0) if w < 256 else b.var("y")
        for op in (Op.BVUDIV, Op.BVUREM, Op.BVSDIV, Op.BVSREM, Op.BVSMOD):
            ts.add(b.finish(b.op(op, x, y)))
        m = (1 << w) - 1
        vals = [0, 1, 2, 3, m, m - 1, 1 << (w - 1), (1 << (w - 1)) - 1]
        vals += [rng.getrandbits(w) for _ in range(8)] + [rng.getrandbits(min(w, 40))
                                                          for _ in range(8)]
        pairs = [(p, q) for p in vals for q in vals]
        soa = np.zeros((2, 8, len(pairs)), dtype=np.uint32)
        for r, (p, q) in enumerate(pairs):
            for k in range(8):
                soa[0, k, r] = (p >> (32 * k)) & 0xFFFFFFFF
                soa[1, k, r] = (q >> (32 * k)) & 0xFFFFFFFF
        ct = gpu_ctx.compile(ts)
        a = upload(gpu_ctx, soa)
        for i, t in enumerate(ts.tapes):
            got = native.limbs_to_ints(native.eval_values(gpu_ctx, ct, i, a))
            for r, (p, q) in enumerate(pairs):
                assert got[r] == smt_eval.evaluate(t.nodes, ts.pool.values, [p, q]), (w, i, p, q)


def test_division_directed_rows_on_gpu(gpu_ctx):
    """The interpreter on the division vectors the native code is checked with
    (tests/test_gpu_jit.py::test_jit_division_digit_boundaries): divisors just above 2^224,
    quotients near 2^10 and on integer boundaries (x = k y - 1, k y, k y + y - 1), waves mixing
    divisors with and without a top limb, zero divisors -- bit-exact against the oracle."""
    from tests.test_jit import division_wave_rows, mixed_top_limb_rows, small_quotient_rows

    ts = TapeSet()
    b = ts.builder()
    x, y = b.var("x"), b.var("y")
    for op in (Op.BVUDIV, Op.BVUREM, Op.BVSDIV, Op.BVSREM, Op.BVSMOD):
        ts.add(b.finish(b.op(op, x, y)))
    ct = gpu_ctx.compile(ts)
    for seed in range(2):
        rows = division_wave_rows(seed) + small_quotient_rows(seed) + mixed_top_limb_rows(seed)
        soa = np.zeros((2, 8, len(rows)), dtype=np.uint32)
        for r, (p, q) in enumerate(rows):
            for k in range(8):
                soa[0, k, r] = (p >> (32 * k)) & 0xFFFFFFFF
                soa[1, k, r] = (q >> (32 * k)) & 0xFFFFFFFF
        a = upload(gpu_ctx, soa)
        for i, t in enumerate(ts.tapes):
            got = native.limbs_to_ints(native.eval_values(gpu_ctx, ct, i, a))
            for r, (p, q) in enumerate(rows):
                assert got[r] == smt_eval.evaluate(t.nodes, ts.pool.values, [p, q]), (seed, i, r)
        a.close()


def test_keccak_on_gpu(gpu_ctx):
    from oracle.keccak import keccak256

    ts = TapeSet()
    b = ts.builder()
    x, y = b.var("x"), b.var("y")
    ts.add(b.finish(b.op(Op.KECCAK, x)))
    ts.add(b.finish(b.op(Op.KECCAK, b.op(Op.CONCAT, x, y))))
    ts.add(b.finish(b.op(Op.KECCAK, b.op(Op.EXTRACT, x, imm0=159, imm1=0))))
    ts.add(b.finish(b.op(Op.KECCAK, b.op(Op.CONCAT, b.op(Op.CONCAT, x, y),
                                              b.op(Op.EXTRACT, y, imm0=7, imm1=0)))))
    rng = random.Random(3)
    rows = [(0, 0), (1, 2)] + [(rng.getrandbits(256), rng.getrandbits(256)) for _ in range(62)]
    soa = np.zeros((2, 8, len(rows)), dtype=np.uint32)
    for r, (p, q) in enumerate(rows):
        for k in range(8):
            soa[0, k, r] = (p >> (32 * k)) & 0xFFFFFFFF
            soa[1, k, r] = (q >> (32 * k)) & 0xFFFFFFFF
    ct = gpu_ctx.compile(ts)
    a = upload(gpu_ctx, soa)
    outs = [native.limbs_to_ints(native.eval_values(gpu_ctx, ct, i, a)) for i in range(4)]
    for r, (p, q) in enumerate(rows):
        pb, qb = p.to_bytes(32, "big"), q.to_bytes(32, "big")
        assert outs[0][r] == int.from_bytes(keccak256(pb), "big")
        assert outs[1][r] == int.from_bytes(keccak256(pb + qb), "big")
        assert outs[2][r] == int.from_bytes(keccak256(pb[12:]), "big")
        assert outs[3][r] == int.from_bytes(keccak256(pb + qb + qb[-1:]), "big")
    assert outs[0][0] == 0x290DECD9548B62A8D60345A988386FC84BA6BC95484008F6362F93160EF3E563


def _oracle_hits(ts, seed, rows, base=0):
    counts, first = [], []
    assigns = [smt_eval.gen_assignment(seed, ts.n_vars, base + r) for r in range(rows)]
    for t in ts.tapes:
        c, f = 0, native.NO_HIT
        for r in range(rows):
            if smt_eval.evaluate(t.nodes, ts.pool.values, assigns[r]):
                c += 1
                f = min(f, base + r)
        counts.append(c)
        first.append(f)
    return counts, first


def test_sieve_counts_and_witnesses(gpu_ctx):
    """Synthetic config-5 tapes: per-tape hit counts and first witnesses match the oracle."""
    ts = synth.generate(40)
    seed, rows, base = 0x5EED, 1536, 1000
    counts, first = _oracle_hits(ts, seed, rows, base)
    ct = gpu_ctx.compile(ts)
    a = gpu_ctx.assignments(ts.n_vars, rows)
    a.generate(seed, base)
    fh, hc = native.run(gpu_ctx, ct, a, index_base=base, mode=native.MODE_COUNT_ALL)
    assert [int(x) for x in hc] == counts
    assert [int(x) for x in fh] == first
    fh2, _ = native.run(gpu_ctx, ct, a, index_base=base, mode=native.MODE_FIRST_HIT)
    assert [int(x) for x in fh2] == first


def test_full_size_properties(gpu_ctx):
    """At bench scale (all 10^4 tapes, 2^18 rows): every reported witness satisfies its tape
    (oracle re-check), first-hit mode agrees with count mode, and shards recombine exactly."""
    ts = synth.generate()
    seed, rows = synth.load_spec()["assignment_seed"], 1 << 18
    ct = gpu_ctx.compile(ts)
    a = gpu_ctx.assignments(ts.n_vars, rows)
    a.generate(seed, 0)
    fh, hc = native.run(gpu_ctx, ct, a, mode=native.MODE_COUNT_ALL)
    fh1, _ = native.run(gpu_ctx, ct, a, mode=native.MODE_FIRST_HIT)
    assert np.array_equal(fh, fh1)
    assert int((hc > 0).sum()) == int((fh != native.NO_HIT).sum())
    # witness re-verification (the analogue of z3 re-checking a sieve model)
    hit_tapes = np.nonzero(fh != native.NO_HIT)[0]
    rng = random.Random(1)
    for t in rng.sample(list(hit_tapes), min(300, len(hit_tapes))):
        w = smt_eval.gen_assignment(seed, ts.n_vars, int(fh[t]))
        assert smt_eval.evaluate(ts.tapes[t].nodes, ts.pool.values, w), t
    # exact counts and first hits of a tape sample at full occupancy (1024 workgroups), by the
    # C oracle over every row: asm-core defects that only show with >= 2 waves per SIMD
    from mythril_amd.tape import TapeSet as _TS
    from oracle import ctape

    pick = sorted(rng.sample(range(len(ts.tapes)), 32))
    sub = _TS(ts.var_names)
    sub.pool = ts.pool
    sub.tapes = [ts.tapes[t] for t in pick]
    cnt, first = ctape.count(sub, seed, 0, rows, threads=min(16, os.cpu_count() or 1))
    assert np.array_equal(hc[pick], cnt), "hit counts differ from the C oracle"
    assert np.array_equal(fh[pick], first), "first hits differ from the C oracle"
    # a no-hit tape really has no witness in a sampled prefix
    for t in rng.sample([i for i in range(len(ts.tapes)) if fh[i] == native.NO_HIT],
                        min(20, int((fh == native.NO_HIT).sum()))):
        for r in range(64):
            w = smt_eval.gen_assignment(seed, ts.n_vars, r)
            assert not smt_eval.evaluate(ts.tapes[t].nodes, ts.pool.values, w)
    # sharding: 4 row shards (as 4 GPUs would see them) recombine to the full answer
    parts_f, parts_c = [], []
    for s in range(4):
        lo = s * rows // 4
        f, c = native.run(gpu_ctx, ct, a, row_first=lo, row_count=rows // 4,
                          mode=native.MODE_COUNT_ALL)
        parts_f.append(f)
        parts_c.append(c)
    assert np.array_equal(np.minimum.reduce(parts_f), fh)
    assert np.array_equal(np.sum(parts_c, axis=0), hc)


EIP145 = json.load(open(os.path.join(HERE, "golden", "eip145.json")))
_SHIFT_OP = {"shl": Op.BVSHL, "shr": Op.BVLSHR, "sar": Op.BVASHR}


@pytest.mark.parametrize("op", ["shl", "shr", "sar"])
def test_eip145_on_gpu(gpu_ctx, op):
    """The EIP-145 SHL/SHR/SAR vectors (tests/instructions/{shl,shr,sar}_test.py of the
    reference, instructions.py:528-552) through the kernel, three ways: folded on the host (both
    operands constant), value and shift both assignment columns (the per-lane variable-shift
    handlers), and value a column with the shift constant (the limb-specialised immediate
    shifts)."""
    vecs = EIP145[op]
    vals = [int(v["value"], 16) for v in vecs]
    shifts = [int(v["shift"], 16) for v in vecs]
    want = [int(v["expected"], 16) for v in vecs]
    # folded
    ts = TapeSet()
    b = ts.builder()
    for v, sh in zip(vals, shifts):
        ts.add(b.finish(b.op(_SHIFT_OP[op], b.const(v, 256), b.const(sh, 256))))
    ct = gpu_ctx.compile(ts)
    a = gpu_ctx.assignments(1, 1)
    a.upload(np.zeros((1, 8, 1), dtype=np.uint32))
    for i in range(len(vecs)):
        assert native.limbs_to_ints(native.eval_values(gpu_ctx, ct, i, a))[0] == want[i], (op, i)
    # lifted: one tape, one row per vector
    ts = TapeSet()
    b = ts.builder()
    ts.add(b.finish(b.op(_SHIFT_OP[op], b.var("value"), b.var("shift"))))
    soa = np.zeros((2, 8, len(vecs)), dtype=np.uint32)
    for r, (v, sh) in enumerate(zip(vals, shifts)):
        for k in range(8):
            soa[0, k, r] = (v >> (32 * k)) & 0xFFFFFFFF
            soa[1, k, r] = (sh >> (32 * k)) & 0xFFFFFFFF
    ct = gpu_ctx.compile(ts)
    a = upload(gpu_ctx, soa)
    assert native.limbs_to_ints(native.eval_values(gpu_ctx, ct, 0, a)) == want, op
    # shift constant, value a column: one tape per vector, evaluated on its own row
    ts = TapeSet()
    b = ts.builder()
    for sh in shifts:
        ts.add(b.finish(b.op(_SHIFT_OP[op], b.var("value"), b.const(sh, 256))))
    soa1 = np.ascontiguousarray(soa[:1])
    ct = gpu_ctx.compile(ts)
    a = upload(gpu_ctx, soa1)
    for i in range(len(vecs)):
        got = native.limbs_to_ints(native.eval_values(gpu_ctx, ct, i, a))
        assert got[i] == want[i], (op, i)


def test_bench_config_pinned(gpu_ctx):
    """bench.py's own workload at full size (all 10^4 config-5 tapes x 2^23 rows, one GPU's
    shard): exact per-tape counts and first hits of a 32-tape sample against the C oracle over
    all 2^23 rows, every reported witness of every tape re-checked by the oracle, first-hit mode
    equal to count mode, and the count of tapes with a witness recorded for the bench line."""
    from oracle import ctape

    ts = synth.generate()
    seed, rows = synth.load_spec()["assignment_seed"], 1 << 23
    ct = gpu_ctx.compile(ts)
    a = gpu_ctx.assignments(ts.n_vars, rows)
    a.generate(seed, 0)
    fh, hc = native.run(gpu_ctx, ct, a, mode=native.MODE_COUNT_ALL)
    fh1, _ = native.run(gpu_ctx, ct, a, mode=native.MODE_FIRST_HIT)
    assert np.array_equal(fh, fh1)
    hit = np.nonzero(fh != native.NO_HIT)[0]
    assert np.array_equal(hit, np.nonzero(hc > 0)[0])
    # every witness of every tape: the oracle evaluates that (tape, row) to true
    w_rows = [int(fh[t]) for t in hit]
    ok = ctape.eval_pairs(ts, seed, [int(t) for t in hit], w_rows)
    assert all(ok), [int(t) for t, g in zip(hit, ok) if not g][:10]
    rng = random.Random(23)
    pick = sorted(rng.sample(range(len(ts.tapes)), 32))
    sub = TapeSet(ts.var_names)
    sub.pool = ts.pool
    sub.tapes = [ts.tapes[t] for t in pick]
    cnt, first = ctape.count(sub, seed, 0, rows, threads=min(16, os.cpu_count() or 1))
    assert np.array_equal(hc[pick], cnt), "hit counts differ from the C oracle"
    assert np.array_equal(fh[pick], first), "first hits differ from the C oracle"
    print("bench config: %d tapes with a witness, %d total hits" % (len(hit), int(hc.sum())))


def test_microbench_issue(gpu_ctx):
    """mh_microbench_issue runs every kind and reports a plausible rate (below 2x the nominal
    2-cycle wave64 issue rate of 78.6 T lane-ops/s; the partial-EXEC kinds count 64 lanes per
    wave-instruction, so a SIMD that skipped inactive lane groups could report up to 4x)."""
    for kind in range(len(native.MB_KINDS)):
        r = gpu_ctx.microbench(kind, 4)
        bound = 4 if "exec" in native.MB_KINDS[kind] else 2
        assert 1e11 < r < bound * 78.7e12, (native.MB_KINDS[kind], r)


def test_unsupported_and_invalid(gpu_ctx):
    ts = TapeSet()
    b = ts.builder()
    x = b.op(Op.ZEXT, b.var("x"), imm0=256)  # 512-bit arithmetic: not on the device path
    ts.add(b.finish(b.op(Op.EQ, b.op(Op.BVADD, x, x), x)))
    with pytest.raises(native.Unsupported):
        gpu_ctx.compile(ts)
    ts2 = synth.generate(2)
    ct = gpu_ctx.compile(ts2)
    a = gpu_ctx.assignments(4, 16)
    with pytest.raises(native.SieveError):
        native.run(gpu_ctx, ct, a, row_first=10, row_count=10)


def test_keccak_variant_counts_on_gpu(gpu_ctx):
    """SURVEY §8d's keccak variant (one keccak256 of a 512-bit input per tape): exact per-tape
    counts and first hits against the C oracle, at a size that fills the chip."""
    from oracle import ctape

    ts = synth.generate(48, keccak=True)
    seed, rows = synth.load_spec()["assignment_seed"], 1 << 16
    ct = gpu_ctx.compile(ts)
    a = gpu_ctx.assignments(ts.n_vars, rows)
    a.generate(seed, 0)
    fh, hc = native.run(gpu_ctx, ct, a, mode=native.MODE_COUNT_ALL)
    cnt, first = ctape.count(ts, seed, 0, rows, threads=min(16, os.cpu_count() or 1))
    assert np.array_equal(hc, cnt)
    assert np.array_equal(fh, first)


def test_keccak_message_cuts_on_gpu(gpu_ctx):
    """Keccak of 1..96-byte messages cut from byte pieces of several widths, on the device."""
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
    rows = [[rng.getrandbits(256) for _ in range(3)] for _ in range(63)] + [[0, 0, 0]]
    soa = np.zeros((3, 8, len(rows)), dtype=np.uint32)
    for r, vals in enumerate(rows):
        for v in range(3):
            for k in range(8):
                soa[v, k, r] = (vals[v] >> (32 * k)) & 0xFFFFFFFF
    ct = gpu_ctx.compile(ts)
    a = upload(gpu_ctx, soa)
    for t, parts in enumerate(splits):
        got = native.limbs_to_ints(native.eval_values(gpu_ctx, ct, t, a))
        for r, vals in enumerate(rows):
            msg = b"".join((vals[i] & ((1 << (8 * nb)) - 1)).to_bytes(nb, "big")
                           for i, nb in enumerate(parts))
            assert got[r] == int.from_bytes(keccak256(msg), "big"), (parts, r)


def test_comm_library_path(gpu_ctx):
    """The library's RCCL exchange (mh_comm_init / mh_comm_allreduce_results) on a one-rank
    communicator: the all-reduce is the identity and the run's results are unchanged (the 8-GPU
    path is the same call with world = 8)."""
    import torch

    ts = synth.generate(16)
    seed, rows = synth.load_spec()["assignment_seed"], 4096
    ctx = native.Context(0)
    try:
        ctx.comm_init(native.comm_unique_id(), 0, 1)
        ct = ctx.compile(ts)
        a = ctx.assignments(ts.n_vars, rows)
        a.generate(seed, 0)
        fh0, hc0 = native.run(ctx, ct, a, mode=native.MODE_COUNT_ALL)
        fh = torch.empty(len(ts.tapes), dtype=torch.int64, device="cuda")
        hc = torch.empty(len(ts.tapes), dtype=torch.int64, device="cuda")
        native.results_reset(ctx, fh.data_ptr(), hc.data_ptr(), len(ts.tapes))
        native.run_async(ctx, ct, a, fh.data_ptr(), hc.data_ptr(), mode=native.MODE_COUNT_ALL)
        ctx.comm_allreduce(fh.data_ptr(), hc.data_ptr(), len(ts.tapes))
        ctx.synchronize()
        assert np.array_equal(fh.cpu().numpy().view(np.uint64), fh0)
        assert np.array_equal(hc.cpu().numpy().view(np.uint64), hc0)
        ctx.comm_destroy()
    finally:
        ctx.close()


def test_handles_outlive_their_context(gpu_ctx):
    """Tape sets and assignment buffers keep their context alive: destroying the context first
    and the children afterwards (Python's garbage collector picks any order) is safe, and the
    device pool of a context is reused by its next tape sets."""
    ts = synth.generate(8)
    ctx = native.Context(0)
    a = ctx.assignments(ts.n_vars, 1024)
    a.generate(1, 0)
    cts = [ctx.compile(ts) for _ in range(3)]
    fh, hc = native.run(ctx, cts[0], a, mode=native.MODE_COUNT_ALL)
    for ct in cts[1:]:
        ct.close()
    ct = ctx.compile(ts)  # a block from the pool
    fh2, hc2 = native.run(ctx, ct, a, mode=native.MODE_COUNT_ALL)
    assert np.array_equal(fh, fh2) and np.array_equal(hc, hc2)
    ctx.close()           # released, not freed: three children remain
    ct.close()
    cts[0].close()
    a.close()             # the last child frees the context


def test_wide_columns_full_occupancy(gpu_ctx):
    """Tapes over 24 columns: 20 beyond the 4 preloaded ones, read by D_LOADVAR, which the asm
    core of the complex-op variants runs itself (gen_asm_core.py run_lv: 8 global loads, no exit
    to the C++ driver).  At 2^20 rows (4096 workgroups, >= 2 waves per SIMD, where round 1's
    asm-core defects showed) every tape's hit count and first hit equal the C oracle's, and on a
    96-row upload every tape's value equals the Python oracle's."""
    from oracle import ctape

    rng = random.Random(7700)
    ts = TapeSet()
    fz = TapeFuzzer(rng, ts, n_vars=24, allow_keccak=False, max_depth=4)
    for _ in range(48):
        fz.tape(root_bool=True)
    ct = gpu_ctx.compile(ts)
    assert sum(1 for x in ct.info() if x["features"] & 8) >= 24  # F_CPLX: the run_lv variants
    seed, rows = 0x1D3A, 1 << 20
    a = gpu_ctx.assignments(ts.n_vars, rows)
    a.generate(seed, 0)
    fh, hc = native.run(gpu_ctx, ct, a, mode=native.MODE_COUNT_ALL)
    cnt, first = ctape.count(ts, seed, 0, rows, threads=min(16, os.cpu_count() or 1))
    assert np.array_equal(hc, cnt), "hit counts differ from the C oracle"
    assert np.array_equal(fh, first), "first hits differ from the C oracle"
    assert 0 < int((hc > 0).sum()) < len(ts.tapes) + 1
    ts2 = TapeSet()
    fz = TapeFuzzer(random.Random(7701), ts2, n_vars=24, allow_keccak=False, max_depth=4)
    for _ in range(24):
        fz.tape()
    soa = assignment_soa(random.Random(7702), ts2.n_vars, 96)
    ct2 = gpu_ctx.compile(ts2)
    a2 = upload(gpu_ctx, soa)
    for i, t in enumerate(ts2.tapes):
        got = native.limbs_to_ints(native.eval_values(gpu_ctx, ct2, i, a2))
        for r in range(soa.shape[2]):
            assert got[r] == int(smt_eval.evaluate(t.nodes, ts2.pool.values, soa_row(soa, r))), (i, r)


def test_capacity_above_2_30_rows(gpu_ctx):
    """A buffer of 2^30 + 64 rows per column (one column, 32 GiB): an asm-only tape runs over its
    last rows (64-bit column indexing) and matches the oracle; a complex-op tape (its core loads
    columns with a 32-bit limb-plane stride, run_lv) is refused with MH_E_UNSUPPORTED and a
    message, before anything is launched (the refusal is scoped to those variants)."""
    cap = (1 << 30) + 64
    ts = TapeSet(["x"])
    b = ts.builder()
    x = b.var("x", 256)
    ts.add(b.finish(b.op(Op.BVULT, b.op(Op.BVADD, x, b.const(3, 256)), b.const(1 << 255, 256))))
    ct = gpu_ctx.compile(ts)
    cx = TapeSet(["x"])
    bx = cx.builder()
    xx = bx.var("x", 256)
    cx.add(bx.finish(bx.op(Op.BVMUL_NOOVFL_U, xx, bx.const(3, 256))))
    ctc = gpu_ctx.compile(cx)
    a = gpu_ctx.assignments(1, cap)
    try:
        rows = 256
        first = cap - rows
        rng = random.Random(30)
        vals = [rng.getrandbits(256) for _ in range(rows)]
        soa = np.zeros((1, 8, rows), dtype=np.uint32)
        for r, v in enumerate(vals):
            for k in range(8):
                soa[0, k, r] = (v >> (32 * k)) & 0xFFFFFFFF
        a.upload(soa, first=first)
        fh, hc = native.run(gpu_ctx, ct, a, row_first=first, row_count=rows, index_base=0)
        want = [r for r, v in enumerate(vals)
                if smt_eval.evaluate(ts.tapes[0].nodes, ts.pool.values, [v])]
        assert int(hc[0]) == len(want)
        assert int(fh[0]) == (first + want[0] if want else native.NO_HIT)
        with pytest.raises(native.Unsupported, match="2\\^30 rows"):
            native.run(gpu_ctx, ctc, a, row_first=first, row_count=rows)
        with pytest.raises(native.Unsupported, match="2\\^30 rows"):
            native.eval_values(gpu_ctx, ctc, 0, a, first, rows)
    finally:
        a.close()
        ct.close()
        ctc.close()


def test_merged_short_run_matches_per_variant(gpu_ctx):
    """A short run over the whole tape set is one launch per register class, of the variant with
    every feature the class's tapes need (capi.cpp mh_run_async, MH_MERGE_ROWS); over a sub-range
    it is one launch per variant.  Both give the oracle's counts and first witnesses on a set
    mixing plain, division, keccak and EVM tapes (every register class the fuzzer reaches)."""
    rng = random.Random(4242)
    ts = TapeSet()
    fz = TapeFuzzer(rng, ts, n_vars=3, max_depth=4)
    for _ in range(24):
        fz.tape()
    b = ts.builder()
    x, y = b.var("v0"), b.var("v1")
    ts.add(b.finish(b.op(Op.EQ, b.op(Op.BVAND, b.op(Op.KECCAK, x), b.const(3, 256)),
                         b.const(1, 256))))
    ts.add(b.finish(b.op(Op.BVULT, b.op(Op.EVM_EXP, x, b.const(3, 256)), y)))
    ts.add(b.finish(b.op(Op.BVUGT, b.op(Op.BVUDIV, x, y), b.const(5, 256))))
    soa = assignment_soa(rng, ts.n_vars, 512)
    ct = gpu_ctx.compile(ts)
    a = upload(gpu_ctx, soa)
    want_counts, want_first = [], []
    for t in ts.tapes:
        hits = [r for r in range(soa.shape[2])
                if smt_eval.evaluate(t.nodes, ts.pool.values, soa_row(soa, r))]
        want_counts.append(len(hits))
        want_first.append(hits[0] if hits else native.NO_HIT)
    fh, hc = native.run(gpu_ctx, ct, a, mode=native.MODE_COUNT_ALL)  # merged
    assert [int(v) for v in hc] == want_counts
    assert [int(v) for v in fh] == want_first
    n = len(ts.tapes)
    fh2, hc2 = native.run(gpu_ctx, ct, a, tape_first=1, tape_count=n - 1,
                          mode=native.MODE_COUNT_ALL)  # per variant
    assert [int(v) for v in hc2] == want_counts[1:]
    assert [int(v) for v in fh2] == want_first[1:]
    variants = {(i["n_regs"], i["features"]) for i in ct.info()}
    assert len(variants) > 1


def test_compile_cache_reuses_identical_tapes(gpu_ctx):
    """mh_tapes_compile keeps compiled tapes by content per context: a LASER child's unchanged
    groups reuse their parent's words.  A set compiled twice, and a set where one tape changed and
    the others repeat, give the oracle's counts and the same tape info as a first compile."""
    rng = random.Random(77)
    ts = TapeSet()
    fz = TapeFuzzer(rng, ts, n_vars=3, max_depth=4)
    for _ in range(12):
        fz.tape()
    soa = assignment_soa(rng, ts.n_vars, 256)
    a = upload(gpu_ctx, soa)

    def oracle(tset):
        out = []
        for t in tset.tapes:
            out.append(sum(1 for r in range(soa.shape[2])
                           if smt_eval.evaluate(t.nodes, tset.pool.values, soa_row(soa, r))))
        return out

    want = oracle(ts)
    infos = []
    for _ in range(2):  # the second compile hits the cache for every tape
        ct = gpu_ctx.compile(ts)
        _, hc = native.run(gpu_ctx, ct, a, mode=native.MODE_COUNT_ALL)
        assert [int(v) for v in hc] == want
        infos.append(ct.info())
        ct.close()
    assert infos[0] == infos[1]
    fz.tape()  # one more tape: the first 12 repeat, the new one compiles
    ts.tapes[5], ts.tapes[-1] = ts.tapes[-1], ts.tapes[5]
    ct = gpu_ctx.compile(ts)
    _, hc = native.run(gpu_ctx, ct, a, mode=native.MODE_COUNT_ALL)
    assert [int(v) for v in hc] == oracle(ts)


def test_run_rows_returns_witness_columns(gpu_ctx):
    """mh_run_rows: each tape's first hit and the columns of that row in one copy, equal to
    mh_run's results and to mh_assign_download of the row; zero rows for tapes without a hit.
    The set spans several register classes, so the short run's launches overlap on the side
    streams (capi.cpp mh_run_async fan-out)."""
    rng = random.Random(9191)
    ts = TapeSet()
    fz = TapeFuzzer(rng, ts, n_vars=3, max_depth=4)
    for _ in range(16):
        fz.tape()
    b = ts.builder()
    x, y = b.var("v0"), b.var("v1")
    ts.add(b.finish(b.op(Op.BVUGT, b.op(Op.BVUDIV, x, y), b.const(5, 256))))
    ts.add(b.finish(b.op(Op.EQ, x, b.const(12345, 256))))  # no hit on random rows
    soa = assignment_soa(rng, ts.n_vars, 256)
    a = upload(gpu_ctx, soa)
    ct = gpu_ctx.compile(ts)
    base = 1 << 20
    fh, hc = native.run(gpu_ctx, ct, a, mode=native.MODE_FIRST_HIT, index_base=base)
    fh2, hc2, rows = native.run_rows(gpu_ctx, ct, a, ts.n_vars, mode=native.MODE_FIRST_HIT,
                                     index_base=base)
    assert fh.tolist() == fh2.tolist() and hc.tolist() == hc2.tolist()
    assert int(fh[-1]) == native.NO_HIT and not rows[-1].any()
    for t, h in enumerate(fh.tolist()):
        if h == native.NO_HIT:
            assert not rows[t].any()
            continue
        r = h - base
        assert smt_eval.evaluate(ts.tapes[t].nodes, ts.pool.values, soa_row(soa, r))
        assert (rows[t] == a.download(r, 1)[:, :, 0]).all()
    ct.close()


@pytest.mark.parametrize("rows", [256, 4096, 65536])
def test_conjunct_parallel_split_runs(gpu_ctx, rows):
    """A short run over a set whose long tapes are split into conjunct parts (MH_SPLIT_INSNS:
    the slots from which a tape is cut; mh_tapes_compile reads it per call) gives, per tape, the
    counts and first witnesses of the unsplit set -- whole set (merged launches on side streams,
    parts spread over grid y), a tape range that cuts through the split tapes, FIRST_HIT and
    COUNT_ALL -- and the oracle's on a tape sample."""
    rng = random.Random(rows)
    ts = TapeSet()
    fz = TapeFuzzer(rng, ts, n_vars=3, allow_keccak=rows <= 4096, max_depth=3)
    for _ in range(12):  # conjunctions of 2..8 random Bool terms
        root = fz.boolean(3)
        for _ in range(rng.randrange(1, 8)):
            root = fz.b.op(Op.AND, root, fz.boolean(3))
        ts.add(fz.b.finish(root))
    b = ts.builder()
    x, y = b.var("v0"), b.var("v1")
    # satisfiable by many rows: every part passes somewhere, the AND is what decides
    ts.add(b.finish(b.op(Op.AND, b.op(Op.BVULT, x, y), b.op(Op.BVUGT, x, b.const(5, 256)))))
    soa = assignment_soa(rng, ts.n_vars, rows)
    a = upload(gpu_ctx, soa)
    old = os.environ.get("MH_SPLIT_INSNS")
    try:
        os.environ["MH_SPLIT_INSNS"] = "0"
        whole = gpu_ctx.compile(ts)
        os.environ["MH_SPLIT_INSNS"] = "8"
        cut = gpu_ctx.compile(ts)
    finally:
        if old is None:
            os.environ.pop("MH_SPLIT_INSNS", None)
        else:
            os.environ["MH_SPLIT_INSNS"] = old
    n = len(ts.tapes)
    for mode in (native.MODE_FIRST_HIT, native.MODE_COUNT_ALL):
        for first, count in ((0, n), (3, n - 5), (n - 1, 1)):
            want = native.run(gpu_ctx, whole, a, tape_first=first, tape_count=count, mode=mode,
                              index_base=1000)
            got = native.run(gpu_ctx, cut, a, tape_first=first, tape_count=count, mode=mode,
                             index_base=1000)
            assert [int(v) for v in got[0]] == [int(v) for v in want[0]], (mode, first)
            if mode == native.MODE_COUNT_ALL:
                assert [int(v) for v in got[1]] == [int(v) for v in want[1]], (mode, first)
    fh, hc = native.run(gpu_ctx, cut, a, mode=native.MODE_COUNT_ALL, index_base=1000)
    for t in range(0, n, 4 if rows > 4096 else 1):  # the oracle on a sample of rows
        sample = range(0, rows, max(1, rows // 512))
        hits = [r for r in sample
                if smt_eval.evaluate(ts.tapes[t].nodes, ts.pool.values, soa_row(soa, r))]
        if rows <= 512:
            assert int(hc[t]) == len(hits)
            assert int(fh[t]) == (1000 + hits[0] if hits else native.NO_HIT)
        elif hits:
            assert int(fh[t]) <= 1000 + hits[0]
    whole.close()
    cut.close()


def test_query_round_equals_generate_then_run_rows(gpu_ctx):
    """mh_query_round (the guided generator, the run and the witness rows in one call, results
    reset by one kernel) gives what mh_assign_generate_guided followed by mh_run_rows gives, for
    every LASER-shaped query's first round: first witnesses, counts and witness rows."""
    from mythril_amd.sieve import Sieve
    from tests.laser_like import queries

    ctx, qs = queries()
    s = Sieve(rows=4096)
    try:
        for name, cs in qs:
            host = s._host_native(ctx.b, [c.node for c in cs])
            if host is None or not isinstance(host, tuple):
                continue
            columns, widths, _, root, ts = host[:5]
            guide = native.harvest_guide(root, ts.pool.to_array(), widths, keep=True)
            ct = s.compile(ts)
            a1 = s.ctx.assignments(len(columns), 256)
            a2 = s.ctx.assignments(len(columns), 256)
            base = 7 << 24
            for mode in (native.MODE_FIRST_HIT, native.MODE_COUNT_ALL):
                fh, hc, rows = native.query_round(s.ctx, ct, a1, guide, 99, base, 256,
                                                  len(columns), mode=mode)
                a2.generate_guided(99, guide.arrays(), global_base=base, count=256)
                fh2, hc2, rows2 = native.run_rows(s.ctx, ct, a2, len(columns), mode=mode,
                                                  index_base=base, row_count=256)
                assert fh.tolist() == fh2.tolist(), name
                assert (rows == rows2).all(), name
                if mode == native.MODE_COUNT_ALL:
                    assert hc.tolist() == hc2.tolist(), name
            ct.close()
            a1.close()
            a2.close()
            guide.close()
    finally:
        s.close()


def test_cpp_step_build_matches_oracle(gpu_ctx):
    """the C++ step() build of the interpreter (`make noasm`, MH_ASM_CORE=0) runs
    each short-circuit D_BANDZ and leaves a tape only when no lane's conjunction is left true,
    so its counts, first witnesses and a LASER query's witness equal the oracle's (the check runs
    in one child process with MYTHRIL_HIP_LIB naming that library: tests/noasm_check.py)."""
    import subprocess
    import sys

    root = os.path.dirname(HERE)
    lib = os.path.join(root, "mythril_amd", "libmythril_hip_noasm.so")
    assert os.path.exists(lib), "build it first: make -C mythril_amd/csrc noasm (build() does)"
    env = dict(os.environ, MYTHRIL_HIP_LIB=lib)
    r = subprocess.run([sys.executable, "-u", "-m", "tests.noasm_check"], cwd=root, env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "noasm ok" in r.stdout
