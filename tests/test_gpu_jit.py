"""The native-code path (mh_tapes_jit) on an MI355X against the oracle, bit for bit.

Run first on its own (a new code path): the smallest case, then values of random tapes, then
counts at the bench's scale against the interpreter and the C oracle."""
import os
import random

import numpy as np
import pytest

from mythril_amd import native, synth
from mythril_amd.tape import Op, TapeSet
from oracle import smt_eval
from tests.fuzz import TapeFuzzer, assignment_soa, soa_row

pytestmark = pytest.mark.gpu


def upload(ctx, soa):
    a = ctx.assignments(soa.shape[0], soa.shape[2])
    a.upload(soa)
    return a


def soa_of(rows_vals, n_vars):
    soa = np.zeros((n_vars, 8, len(rows_vals)), dtype=np.uint32)
    for r, vals in enumerate(rows_vals):
        for v in range(n_vars):
            for k in range(8):
                soa[v, k, r] = (vals[v] >> (32 * k)) & 0xFFFFFFFF
    return soa


def jit_values_match(ctx, ts, soa):
    ct = ctx.compile(ts)
    info = ct.jit(values=True)
    jitted = ct.jitted()
    a = upload(ctx, soa)
    vals = ct.jit_values(a)
    n = 0
    for i, t in enumerate(ts.tapes):
        if not jitted[i]:
            continue
        n += 1
        got = native.limbs_to_ints(vals[i])
        for r in range(soa.shape[2]):
            want = int(smt_eval.evaluate(t.nodes, ts.pool.values, soa_row(soa, r)))
            assert got[r] == want, (i, r, hex(got[r]), hex(want))
    ct.close()
    return n, info


def test_jit_smallest(gpu_ctx):
    """One tape, one 64-row chunk: x + y == c, values and counts."""
    ts = TapeSet()
    b = ts.builder()
    x, y = b.var("x"), b.var("y")
    ts.add(b.finish(b.op(Op.BVADD, x, y)))
    ts.add(b.finish(b.op(Op.EQ, b.op(Op.BVAND, b.op(Op.BVADD, x, y), b.const(3, 256)),
                         b.const(1, 256))))
    rng = random.Random(1)
    rows = [[rng.getrandbits(256), rng.getrandbits(256)] for _ in range(64)]
    n, info = jit_values_match(gpu_ctx, ts, soa_of(rows, 2))
    assert n == 2 and info["n_jitted"] == 2
    ct = gpu_ctx.compile(ts)
    ct.jit()
    a = upload(gpu_ctx, soa_of(rows, 2))
    fh, hc = native.run(gpu_ctx, ct, a, mode=native.MODE_COUNT_ALL)
    want = [r for r in range(64) if ((rows[r][0] + rows[r][1]) & 3) == 1]
    assert int(hc[1]) == len(want) and int(fh[1]) == (want[0] if want else native.NO_HIT)
    assert int(hc[0]) == sum(1 for r in rows if (r[0] + r[1]) % (1 << 256))


@pytest.mark.parametrize("seed", range(4))
def test_jit_fuzz_values(gpu_ctx, seed):
    rng = random.Random(9000 + seed)
    ts = TapeSet()
    fz = TapeFuzzer(rng, ts, n_vars=3, max_depth=4, allow_keccak=False)
    for _ in range(24):
        fz.tape()
    soa = assignment_soa(rng, ts.n_vars, 150)
    n, _ = jit_values_match(gpu_ctx, ts, soa)
    assert n >= 12


def test_jit_division_and_shift_edges(gpu_ctx):
    rng = random.Random(8)
    for w in (8, 160, 256):
        ts = TapeSet()
        b = ts.builder()
        x = b.op(Op.EXTRACT, b.var("x"), imm0=w - 1, imm1=0) if w < 256 else b.var("x")
        y = b.op(Op.EXTRACT, b.var("y"), imm0=w - 1, imm1=0) if w < 256 else b.var("y")
        for op in (Op.BVUDIV, Op.BVUREM, Op.BVSDIV, Op.BVSREM, Op.BVSMOD, Op.BVSHL, Op.BVLSHR,
                   Op.BVASHR, Op.BVMUL):
            ts.add(b.finish(b.op(op, x, y)))
            ts.add(b.finish(b.op(op, x, b.const(rng.getrandbits(w) | 1, w))))
        m = (1 << w) - 1
        vals = [0, 1, 2, 3, m, m - 1, 1 << (w - 1), (1 << (w - 1)) - 1]
        vals += [rng.getrandbits(w) for _ in range(6)] + [rng.getrandbits(min(w, 9))
                                                          for _ in range(6)]
        pairs = [[p, q] for p in vals for q in vals]
        n, _ = jit_values_match(gpu_ctx, ts, soa_of(pairs, 2))
        assert n == len(ts.tapes)


def test_jit_synthetic_values(gpu_ctx):
    """Config-5 tapes by the native code: root values on generated rows."""
    ts = synth.generate(64)
    seed = synth.load_spec()["assignment_seed"]
    rows = [smt_eval.gen_assignment(seed, ts.n_vars, r) for r in range(192)]
    n, _ = jit_values_match(gpu_ctx, ts, soa_of(rows, ts.n_vars))
    assert n == 64


def test_jit_division_digit_boundaries(gpu_ctx):
    """Quotient digits on an integer boundary (x = q y + {-1, 0, 1}) and the uniform paths of
    the division subroutine (tests/test_jit.py division_wave_rows), where the hardware's
    reciprocal decides whether a digit estimate lands one off and a correction must run."""
    from tests.test_jit import division_wave_rows, mixed_top_limb_rows, small_quotient_rows

    ts = TapeSet()
    b = ts.builder()
    x, y = b.var("x"), b.var("y")
    for op in (Op.BVUDIV, Op.BVUREM, Op.BVSDIV, Op.BVSREM, Op.BVSMOD):
        ts.add(b.finish(b.op(op, x, y)))
    for seed in range(4):
        for rows in (division_wave_rows(seed), small_quotient_rows(seed),
                     mixed_top_limb_rows(seed)):
            n, _ = jit_values_match(gpu_ctx, ts, soa_of(rows, 2))
            assert n == len(ts.tapes)


def test_jit_keccak_values(gpu_ctx):
    """Keccak-256 in the native code: messages of 1..96 bytes from several pieces (constant
    pieces swapped on the host) and the keccak variant's tapes, root values against the oracle."""
    rng = random.Random(405)
    splits = [[1], [20], [31], [32], [7, 26], [32, 1], [31, 31], [32, 32], [12, 32, 8],
              [32, 32, 31], [32, 32, 32]]
    ts = TapeSet()
    b = ts.builder()
    xs = [b.var("x%d" % i) for i in range(3)]
    for parts in splits:
        node = None
        for i, nb in enumerate(parts):
            p = xs[i] if nb == 32 else b.op(Op.EXTRACT, xs[i], imm0=8 * nb - 1, imm1=0)
            node = p if node is None else b.op(Op.CONCAT, node, p)
        ts.add(b.finish(b.op(Op.KECCAK, node)))
    k = b.const(0xAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFE, 256)
    ts.add(b.finish(b.op(Op.KECCAK, b.op(Op.CONCAT, k, xs[1]))))
    rows = [[rng.getrandbits(256) for _ in range(3)] for _ in range(130)] + [[0, 0, 0]]
    n, info = jit_values_match(gpu_ctx, ts, soa_of(rows, 3))
    assert n == len(ts.tapes)
    kv = synth.generate(32, keccak=True)
    seed = synth.load_spec()["assignment_seed"]
    rows = [smt_eval.gen_assignment(seed, kv.n_vars, r) for r in range(128)]
    n, _ = jit_values_match(gpu_ctx, kv, soa_of(rows, kv.n_vars))
    assert n >= 30


def test_jit_keccak_variant_counts(gpu_ctx):
    """The keccak variant through the native code: counts and first hits equal the
    interpreter's (its C++ Keccak) on 2^16 rows."""
    ts = synth.generate(160, keccak=True)
    seed, rows = synth.load_spec()["assignment_seed"], 1 << 16
    a = gpu_ctx.assignments(ts.n_vars, rows)
    a.generate(seed, 0)
    ref = gpu_ctx.compile(ts)
    fh0, hc0 = native.run(gpu_ctx, ref, a, mode=native.MODE_COUNT_ALL)
    ct = gpu_ctx.compile(ts)
    info = ct.jit()
    assert info["n_jitted"] >= 150
    fh, hc = native.run(gpu_ctx, ct, a, mode=native.MODE_COUNT_ALL)
    assert np.array_equal(hc, hc0) and np.array_equal(fh, fh0)


def test_jit_counts_match_interpreter_and_oracle(gpu_ctx):
    """Counts and first hits, native vs interpreter (same tape set, same rows) and vs the C
    oracle, at a size that fills the chip (several groups, many row blocks)."""
    from oracle import ctape

    ts = synth.generate(400)
    seed, rows = synth.load_spec()["assignment_seed"], 1 << 17
    a = gpu_ctx.assignments(ts.n_vars, rows)
    a.generate(seed, 0)
    ref = gpu_ctx.compile(ts)
    fh0, hc0 = native.run(gpu_ctx, ref, a, mode=native.MODE_COUNT_ALL)
    ct = gpu_ctx.compile(ts)
    info = ct.jit()
    assert info["n_jitted"] == 400 and info["n_groups"] >= 4
    fh, hc = native.run(gpu_ctx, ct, a, mode=native.MODE_COUNT_ALL)
    assert np.array_equal(hc, hc0)
    assert np.array_equal(fh, fh0)
    fh2, _ = native.run(gpu_ctx, ct, a, mode=native.MODE_FIRST_HIT)
    assert np.array_equal(fh2, fh0)
    # row sub-ranges with an index base (shards)
    f1, c1 = native.run(gpu_ctx, ct, a, row_first=1000, row_count=rows - 3000, index_base=7,
                        mode=native.MODE_COUNT_ALL)
    f0, c0 = native.run(gpu_ctx, ref, a, row_first=1000, row_count=rows - 3000, index_base=7,
                        mode=native.MODE_COUNT_ALL)
    assert np.array_equal(c1, c0) and np.array_equal(f1, f0)
    pick = list(range(0, 400, 13))
    sub = TapeSet(ts.var_names)
    sub.pool = ts.pool
    sub.tapes = [ts.tapes[t] for t in pick]
    cnt, first = ctape.count(sub, seed, 0, rows, threads=min(16, os.cpu_count() or 1))
    assert np.array_equal(hc[pick], cnt)
    assert np.array_equal(fh[pick], first)


def test_jit_bench_config_pinned(gpu_ctx):
    """bench.py's workload (10^4 tapes x 2^23 rows) through the native code: counts and first
    hits equal the interpreter's on every tape, and the C oracle's on a 32-tape sample."""
    from oracle import ctape

    ts = synth.generate()
    seed, rows = synth.load_spec()["assignment_seed"], 1 << 23
    a = gpu_ctx.assignments(ts.n_vars, rows)
    a.generate(seed, 0)
    ct = gpu_ctx.compile(ts)
    info = ct.jit()
    assert info["n_jitted"] >= 0.995 * len(ts.tapes)  # the rest run on the interpreter
    fh, hc = native.run(gpu_ctx, ct, a, mode=native.MODE_COUNT_ALL)
    ref = gpu_ctx.compile(ts)
    fh0, hc0 = native.run(gpu_ctx, ref, a, mode=native.MODE_COUNT_ALL)
    assert np.array_equal(hc, hc0) and np.array_equal(fh, fh0)
    rng = random.Random(23)
    pick = sorted(rng.sample(range(len(ts.tapes)), 32))
    sub = TapeSet(ts.var_names)
    sub.pool = ts.pool
    sub.tapes = [ts.tapes[t] for t in pick]
    cnt, first = ctape.count(sub, seed, 0, rows, threads=min(16, os.cpu_count() or 1))
    assert np.array_equal(hc[pick], cnt) and np.array_equal(fh[pick], first)
    print("jit: %s" % info)


def test_jit_short_circuit_matches_full_eval(gpu_ctx):
    """Short-circuit conjunctions (the default) against MH_JIT_FULL_EVAL on the same tapes and
    rows: identical counts and first hits in both modes, over partial row blocks too."""
    ts = synth.generate(1000)
    seed, rows = synth.load_spec()["assignment_seed"], (1 << 18) + 77
    a = gpu_ctx.assignments(ts.n_vars, rows)
    a.generate(seed, 0)
    sc = gpu_ctx.compile(ts)
    sc.jit()
    full = gpu_ctx.compile(ts)
    full.jit(short_circuit=False)
    for mode in (native.MODE_COUNT_ALL, native.MODE_FIRST_HIT):
        f1, c1 = native.run(gpu_ctx, sc, a, mode=mode)
        f0, c0 = native.run(gpu_ctx, full, a, mode=mode)
        assert np.array_equal(f1, f0)
        if mode == native.MODE_COUNT_ALL:
            assert np.array_equal(c1, c0) and int((c0 > 0).sum()) > 50
    f1, c1 = native.run(gpu_ctx, sc, a, row_first=333, row_count=rows - 1000, index_base=5,
                        mode=native.MODE_COUNT_ALL)
    f0, c0 = native.run(gpu_ctx, full, a, row_first=333, row_count=rows - 1000, index_base=5,
                        mode=native.MODE_COUNT_ALL)
    assert np.array_equal(c1, c0) and np.array_equal(f1, f0)


def test_code_id_equals_the_device_free_id(gpu_ctx):
    """CompiledTapes.code_id() (mh_tapes_jit_code_id, after a real build and load) is the id
    mh_jit_code_id computes on the host: bench.py's profile keys need no device to check."""
    ts = synth.generate(48)
    for sc in (True, False):
        ct = gpu_ctx.compile(ts)
        ct.jit(short_circuit=sc)
        assert ct.code_id() == native.jit_code_id(ts, short_circuit=sc)
        ct.close()
