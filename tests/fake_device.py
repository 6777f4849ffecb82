"""A CPU stand-in for the device side of mythril_amd.native, for tests of Sieve.solve's host logic
without a GPU (test infrastructure only: the product path never imports this).

``install(monkeypatch)`` replaces native.Context, native.run, native.run_rows, native.query_round,
native.eval_values and native.eval_values_many with restatements on the oracle: the guided
generator (oracle/guided_gen.py, the restatement of mh_assign_generate_guided, pinned against the
device by tests/test_gpu_frontend.py) and the tape evaluator (oracle/smt_eval.py).  FIRST_HIT is the smallest satisfying row per tape.  Slow (Python
big-int evaluation): use small rounds, e.g. Sieve(rows=256).
"""
import numpy as np

from mythril_amd import native
from oracle import smt_eval as E
from oracle.guided_gen import generate_row


class FakeTapes:
    def __init__(self, ts):
        self.tapes = [t.nodes for t in ts.tapes]
        self.pool = native._ints(ts.pool.to_array())
        self.n_tapes = len(self.tapes)
        self.n_vars = ts.n_vars
        self.timing = (0.0, 0.0)

    def close(self):
        pass


class FakeAssign:
    def __init__(self, n_vars, capacity):
        self.n_vars, self.capacity = n_vars, capacity
        self.rows = {}

    def generate_guided(self, seed, arrays, global_base=0, first=0, count=None):
        count = self.capacity - first if count is None else count
        assert len(arrays["width"]) <= self.n_vars
        for r in range(count):
            self.rows[first + r] = generate_row(seed, global_base + first + r, arrays)

    def upload(self, soa, first=0):
        for r in range(soa.shape[2]):
            self.rows[first + r] = [sum(int(soa[v, k, r]) << (32 * k) for k in range(8))
                                    for v in range(soa.shape[0])]

    def download(self, first, count):
        out = np.zeros((self.n_vars, 8, count), dtype=np.uint32)
        for r in range(count):
            for v, x in enumerate(self.rows[first + r]):
                for k in range(8):
                    out[v, k, r] = (x >> (32 * k)) & 0xFFFFFFFF
        return out

    def close(self):
        pass


class FakeContext:
    def __init__(self, device=0):
        pass

    def close(self):
        pass

    def compile(self, ts):
        return FakeTapes(ts)

    def assignments(self, n_vars, capacity):
        return FakeAssign(n_vars, capacity)


def fake_run(ctx, tapes, assign, *, tape_first=0, tape_count=None, row_first=0, row_count=None,
             index_base=0, mode=native.MODE_COUNT_ALL):
    tc = tapes.n_tapes - tape_first if tape_count is None else tape_count
    rc = assign.capacity - row_first if row_count is None else row_count
    fh = np.full(max(tc, 1), native.NO_HIT, dtype=np.uint64)
    cnt = np.zeros(max(tc, 1), dtype=np.uint64)
    for t in range(tc):
        tape = tapes.tapes[tape_first + t]
        for r in range(row_first, row_first + rc):
            if E.evaluate(tape, tapes.pool, assign.rows[r]):
                if fh[t] == native.NO_HIT:
                    fh[t] = index_base + r
                cnt[t] += 1
                if mode == native.MODE_FIRST_HIT:
                    break
    return fh[:tc], cnt[:tc]


def fake_run_rows(ctx, tapes, assign, n_cols, *, tape_first=0, tape_count=None, row_first=0,
                  row_count=None, index_base=0, mode=native.MODE_FIRST_HIT):
    fh, cnt = fake_run(ctx, tapes, assign, tape_first=tape_first, tape_count=tape_count,
                       row_first=row_first, row_count=row_count, index_base=index_base, mode=mode)
    rows = np.zeros((len(fh), n_cols, 8), dtype=np.uint32)
    for i, h in enumerate(fh.tolist()):
        if h != native.NO_HIT:
            rows[i] = assign.download(h - index_base, 1)[:n_cols, :, 0]
    return fh, cnt, rows


def fake_query_round(ctx, tapes, assign, guide, seed, global_base, count, n_cols, *,
                     tape_first=0, tape_count=None, mode=native.MODE_FIRST_HIT):
    assign.generate_guided(seed, guide.arrays(), global_base=global_base, count=count)
    return fake_run_rows(ctx, tapes, assign, n_cols, tape_first=tape_first,
                         tape_count=tape_count, row_count=count, index_base=global_base,
                         mode=mode)


def fake_eval_values(ctx, tapes, tape, assign, row_first=0, row_count=None):
    rc = assign.capacity - row_first if row_count is None else row_count
    out = np.zeros((8, max(rc, 1)), dtype=np.uint32)
    for r in range(rc):
        v = int(E.evaluate(tapes.tapes[tape], tapes.pool, assign.rows[row_first + r]))
        for k in range(8):
            out[k, r] = (v >> (32 * k)) & 0xFFFFFFFF
    return out[:, :rc]


LAUNCHES = [0]  # batched evaluations (one per eval_values_many call: one variant stands in)


def fake_eval_values_many(ctx, tapes, ids, assign, row=0):
    LAUNCHES[0] += 1
    out = np.zeros((max(len(ids), 1), 8), dtype=np.uint32)
    for i, t in enumerate(ids):
        v = int(E.evaluate(tapes.tapes[t], tapes.pool, assign.rows[row]))
        for k in range(8):
            out[i, k] = (v >> (32 * k)) & 0xFFFFFFFF
    return out[:len(ids)]


def install(monkeypatch):
    monkeypatch.setattr(native, "Context", FakeContext)
    monkeypatch.setattr(native, "run", fake_run)
    monkeypatch.setattr(native, "run_rows", fake_run_rows)
    monkeypatch.setattr(native, "query_round", fake_query_round)
    monkeypatch.setattr(native, "eval_values", fake_eval_values)
    monkeypatch.setattr(native, "eval_values_many", fake_eval_values_many)
