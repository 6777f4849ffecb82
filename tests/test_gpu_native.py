"""The native code (mh_tapes_jit) on the reference's own vectors and on the product's query
shapes, on an MI355X, bit for bit against the oracle.

* the VMTests known answers (the reference's tests/laser/evm_testsuite corpus, as data in
  tests/golden/vmtests.json) and the EIP-145 SHL/SHR/SAR vectors (tests/instructions/*_test.py),
  in one JIT build per corpus: every tape must be jitted (a refusal fails the test with its
  reason), and the jitted values rebuild each vector's post-state storage;
* tape sets of more than 4 columns (the code loads the limbs each use demands) from the
  LASER-shaped queries of tests/laser_like.py over guided rows, native against the interpreter
  and the oracle;
* config 5 at its stated size, 10^4 tapes x 2^26 rows on one GPU.
"""
import json
import os
import random

import numpy as np
import pytest

from mythril_amd import native, synth
from mythril_amd.tape import Op, TapeSet
from oracle import smt_eval
from tests.evm_translate import final_storage, vmtest_batch
from tests.fuzz import TapeFuzzer, assignment_soa, soa_row

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
VMTESTS = json.load(open(os.path.join(HERE, "golden", "vmtests.json")))
EIP145 = json.load(open(os.path.join(HERE, "golden", "eip145.json")))
LASER_DIVERGENT = {"addmodDivByZero", "addmodDivByZero1", "addmodDivByZero2", "mulmoddivByZero"}


def upload(ctx, soa):
    a = ctx.assignments(soa.shape[0], soa.shape[2])
    a.upload(soa)
    return a


def jit_all(ct, values=True):
    """mh_tapes_jit, asserting every tape runs native (names the refused ones otherwise)."""
    info = ct.jit(values=values)
    jitted = ct.jitted()
    refused = [int(i) for i in np.nonzero(jitted == 0)[0]]
    assert not refused, "tapes left on the interpreter: %s" % refused[:20]
    return info


@pytest.mark.parametrize("lifted", [False, True])
@pytest.mark.parametrize("mode", ["laser", "evm"])
def test_native_vmtests(gpu_ctx, mode, lifted):
    """All translatable VMTests in one tape set through mh_tapes_jit(MH_JIT_VALUES) /
    mh_jit_eval_all: folded (constants only: the host folds, the code returns constants) and
    lifted (every constant a column, > 4 columns: nothing folds, every op runs on the device)."""
    ts, soa, index = vmtest_batch(VMTESTS, mode, lifted)
    assert len(index) >= 340
    ct = gpu_ctx.compile(ts)
    info = jit_all(ct)
    a = gpu_ctx.assignments(max(ts.n_vars, 1), 1)
    a.upload(soa if lifted else np.zeros((max(ts.n_vars, 1), 8, 1), dtype=np.uint32))
    vals = ct.jit_values(a)
    bounds = [i[1] for i in index] + [len(ts.tapes)]
    for j, (name, first, pairs, expected, pre) in enumerate(index):
        got = []
        for i in range(first, bounds[j + 1]):
            v = native.limbs_to_ints(vals[i])[0]
            nodes = ts.tapes[i].nodes
            want = int(smt_eval.evaluate(nodes, ts.pool.values, soa_row(soa, 0) if lifted else []))
            assert v == want, (name, i - first, hex(v), hex(want))
            got.append(v)
        if not (mode == "laser" and name in LASER_DIVERGENT):
            assert final_storage(pre, pairs, got) == expected, name
    print("%s lifted=%s: %d vectors, %d tapes, %d columns, jit %s" % (
        mode, lifted, len(index), len(ts.tapes), ts.n_vars, info))


_SHIFT_OP = {"shl": Op.BVSHL, "shr": Op.BVLSHR, "sar": Op.BVASHR}


@pytest.mark.parametrize("op", ["shl", "shr", "sar"])
def test_native_eip145(gpu_ctx, op):
    """EIP-145 vectors (reference tests/instructions/{shl,shr,sar}_test.py) by the native code:
    value and shift both columns (the LDS-window variable shift), and one tape per vector with a
    constant shift (register renaming + v_alignbit), each on its own row."""
    vecs = EIP145[op]
    vals = [int(v["value"], 16) for v in vecs]
    shifts = [int(v["shift"], 16) for v in vecs]
    want = [int(v["expected"], 16) for v in vecs]
    soa = np.zeros((2, 8, len(vecs)), dtype=np.uint32)
    for r, (v, sh) in enumerate(zip(vals, shifts)):
        for k in range(8):
            soa[0, k, r] = (v >> (32 * k)) & 0xFFFFFFFF
            soa[1, k, r] = (sh >> (32 * k)) & 0xFFFFFFFF
    ts = TapeSet()
    b = ts.builder()
    value, shift = b.var("value"), b.var("shift")
    ts.add(b.finish(b.op(_SHIFT_OP[op], value, shift)))
    for sh in shifts:
        ts.add(b.finish(b.op(_SHIFT_OP[op], value, b.const(sh, 256))))
    ct = gpu_ctx.compile(ts)
    jit_all(ct)
    out = ct.jit_values(upload(gpu_ctx, soa))
    assert native.limbs_to_ints(out[0]) == want, op
    for i in range(len(vecs)):
        assert native.limbs_to_ints(out[1 + i])[i] == want[i], (op, i)


@pytest.mark.parametrize("seed", range(3))
def test_native_wide_schema_fuzz(gpu_ctx, seed):
    """Random tapes over 7 columns with every op (EVM word ops, ADDMOD / MULMOD, EXP by a
    column, overflow predicates): native values equal the oracle's on every row."""
    rng = random.Random(7100 + seed)
    ts = TapeSet()
    fz = TapeFuzzer(rng, ts, n_vars=7, max_depth=4, allow_keccak=seed == 2)
    for _ in range(24):
        fz.tape()
    soa = assignment_soa(rng, ts.n_vars, 130)
    ct = gpu_ctx.compile(ts)
    ct.jit(values=True)
    jitted = ct.jitted()
    assert jitted.sum() >= len(ts.tapes) - 2  # a tape over 96 KB of code may stay interpreted
    vals = ct.jit_values(upload(gpu_ctx, soa))
    for i, t in enumerate(ts.tapes):
        if not jitted[i]:
            continue
        got = native.limbs_to_ints(vals[i])
        for r in range(soa.shape[2]):
            want = int(smt_eval.evaluate(t.nodes, ts.pool.values, soa_row(soa, r)))
            assert got[r] == want, (seed, i, r)


def test_native_laser_queries(gpu_ctx):
    """The sieve's tape sets for every LASER-shaped query (SAT and UNSAT, 1..109 columns) over
    2^16 guided rows: the native code's per-tape counts and first hits equal the interpreter's,
    and its root values equal the oracle's on a row sample."""
    from tests.laser_like import hard_queries, queries, query_tapeset

    rows = 1 << 16
    checked = 0
    for maker in (queries, hard_queries):
        ctx, qs = maker()
        for name, cs in qs:
            ts, schema, guide = query_tapeset(ctx.b, cs)
            a = gpu_ctx.assignments(max(ts.n_vars, 1), rows)
            a.generate_guided(0xC0FFEE, guide, global_base=0, count=rows)
            ref = gpu_ctx.compile(ts)
            fh0, hc0 = native.run(gpu_ctx, ref, a, mode=native.MODE_COUNT_ALL)
            ct = gpu_ctx.compile(ts)
            jit_all(ct)
            fh, hc = native.run(gpu_ctx, ct, a, mode=native.MODE_COUNT_ALL)
            assert np.array_equal(hc, hc0) and np.array_equal(fh, fh0), name
            ff, _ = native.run(gpu_ctx, ct, a, mode=native.MODE_FIRST_HIT)
            assert np.array_equal(ff, fh0), name
            if name.endswith("_unsat"):
                assert int(hc.sum()) == 0 or len(ts.tapes) > 1, name
            # values of a row sample (the hits first) against the oracle
            vct = gpu_ctx.compile(ts)
            vct.jit(values=True)
            sample = sorted({int(x) for x in fh if x != native.NO_HIT} | set(range(0, rows, 4099)))
            soa = a.download(0, rows)
            vals = vct.jit_values(a)
            for i, t in enumerate(ts.tapes):
                got = native.limbs_to_ints(vals[i][:, sample])
                for g, r in zip(got, sample):
                    assert g == int(smt_eval.evaluate(t.nodes, ts.pool.values,
                                                      soa_row(soa[: ts.n_vars], r))), (name, i, r)
            for x in (ref, ct, vct, a):
                x.close()
            checked += 1
    assert checked >= 15


@pytest.mark.timeout(900)
def test_native_config5_full_size(gpu_ctx):
    """Config 5 at its stated size on one GPU: 10^4 tapes x 2^26 rows (8 GiB of columns).  The
    native code's per-tape counts and first hits equal the interpreter's on every tape, and the
    C oracle's over every row on an 8-tape sample."""
    from oracle import ctape

    ts = synth.generate()
    seed, rows = synth.load_spec()["assignment_seed"], 1 << 26
    a = gpu_ctx.assignments(ts.n_vars, rows)
    a.generate(seed, 0)
    ct = gpu_ctx.compile(ts)
    info = ct.jit()
    assert info["n_jitted"] == len(ts.tapes)
    fh, hc = native.run(gpu_ctx, ct, a, mode=native.MODE_COUNT_ALL)
    ref = gpu_ctx.compile(ts)
    fh0, hc0 = native.run(gpu_ctx, ref, a, mode=native.MODE_COUNT_ALL)
    assert np.array_equal(hc, hc0) and np.array_equal(fh, fh0)
    rng = random.Random(26)
    pick = sorted(rng.sample(range(len(ts.tapes)), 8))
    sub = TapeSet(ts.var_names)
    sub.pool = ts.pool
    sub.tapes = [ts.tapes[t] for t in pick]
    cnt, first = ctape.count(sub, seed, 0, rows, threads=min(16, os.cpu_count() or 1),
                             short_circuit=True)
    assert np.array_equal(hc[pick], cnt) and np.array_equal(fh[pick], first)
    print("config 5 at 2^26 rows: %d tapes with a witness, %d hits" % (
        int((fh != native.NO_HIT).sum()), int(hc.sum())))
    for x in (ct, ref, a):
        x.close()


@pytest.mark.timeout(600)
def test_native_keccak_variant_2_20(gpu_ctx):
    """bench.py --variant keccak at its size (10^4 tapes, each with one keccak256 of a 512-bit
    input, keccak_function_manager.py:43-57) x 2^20 rows: the native code's per-tape counts and
    first hits equal the interpreter's on every tape, and the C oracle's over every row on an
    8-tape sample (every sampled tape reaches its keccak conjunct on some rows)."""
    from oracle import ctape

    ts = synth.generate(keccak=True)
    seed, rows = synth.load_spec()["assignment_seed"], 1 << 20
    a = gpu_ctx.assignments(ts.n_vars, rows)
    a.generate(seed, 0)
    ct = gpu_ctx.compile(ts)
    info = ct.jit()
    assert info["n_jitted"] == len(ts.tapes), info
    fh, hc = native.run(gpu_ctx, ct, a, mode=native.MODE_COUNT_ALL)
    ref = gpu_ctx.compile(ts)
    fh0, hc0 = native.run(gpu_ctx, ref, a, mode=native.MODE_COUNT_ALL)
    assert np.array_equal(hc, hc0) and np.array_equal(fh, fh0)
    rng = random.Random(20)
    pick = sorted(rng.sample(range(len(ts.tapes)), 8))
    sub = TapeSet(ts.var_names)
    sub.pool = ts.pool
    sub.tapes = [ts.tapes[t] for t in pick]
    cnt, first = ctape.count(sub, seed, 0, rows, threads=min(16, os.cpu_count() or 1),
                             short_circuit=True)
    assert np.array_equal(hc[pick], cnt) and np.array_equal(fh[pick], first)
    for x in (ct, ref, a):
        x.close()
