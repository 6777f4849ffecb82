"""The N > 1 path on the CPU: world_size 2 over gloo.

Each rank evaluates its shard of candidate rows (mythril_amd.shard.shard_range: the
counter-based generator gives rank r the global rows [r*R, (r+1)*R)) — here with the ORACLE,
since the container has no GPU — and the product reduction (shard.allreduce_results: MIN of the
first witness, SUM of the counts) must reproduce the single-process answer over all 2R rows.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from mythril_amd import shard
from mythril_amd.tape import Op, TapeSet
from oracle import smt_eval

ROWS = 48
TAPES = 12
SEED = 0x5EED


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _tapes():
    """Tapes with satisfaction rates from ~1/2 down to 0 over the generated rows."""
    ts = TapeSet(["a", "b", "c", "d"])
    for t in range(TAPES):
        b = ts.builder()
        x, y = b.var("a"), b.var("b")
        if t % 3 == 0:
            root = b.op(Op.BVULT, x, y)
        elif t % 3 == 1:
            lo = b.op(Op.EXTRACT, x, imm0=2 + t // 3, imm1=0)  # p = 2^-(3 + t/3)
            root = b.op(Op.EQ, lo, b.const(t, 3 + t // 3))
        else:
            root = b.op(Op.EQ, b.op(Op.BVXOR, x, y), b.const(t, 256))  # never in 96 rows
        ts.add(b.finish(root))
    return ts


def _shard_results(ts, base, rows):
    fh = [-1] * len(ts.tapes)
    hc = [0] * len(ts.tapes)
    for r in range(rows):
        a = smt_eval.gen_assignment(SEED, ts.n_vars, base + r)
        for t, tape in enumerate(ts.tapes):
            if smt_eval.evaluate(tape.nodes, ts.pool.values, a):
                hc[t] += 1
                if fh[t] < 0:
                    fh[t] = base + r
    return fh, hc


def _worker(rank, world, port, out, strong=False):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ts = _tapes()
        if strong:  # bench.py --strong: ROWS * 2 + 1 rows in total, split unevenly
            base, rows = shard.strong_shard_range(rank, world, 2 * ROWS + 1)
        else:
            base, rows = shard.shard_range(rank, world, ROWS)
        fh, hc = _shard_results(ts, base, rows)
        fh_t = torch.tensor(fh, dtype=torch.int64)
        hc_t = torch.tensor(hc, dtype=torch.int64)
        shard.allreduce_results(fh_t, hc_t)
        out[rank] = (fh_t.tolist(), hc_t.tolist())
    finally:
        dist.destroy_process_group()


def test_two_rank_reduction_matches_single_process():
    world = 2
    port = _free_port()
    with mp.Manager() as mgr:
        out = mgr.dict()
        mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
        results = dict(out)
    ts = _tapes()
    want = _shard_results(ts, 0, ROWS * world)
    assert any(x >= ROWS for x in want[0])  # some first witnesses lie in rank 1's shard
    assert any(x < 0 for x in want[0]) and any(0 <= x < ROWS for x in want[0])
    assert results[0] == results[1]
    assert tuple(results[0][0]) == tuple(want[0])
    assert tuple(results[0][1]) == tuple(want[1])


def test_shard_range():
    assert shard.shard_range(0, 4, 100) == (0, 100)
    assert shard.shard_range(3, 4, 100) == (300, 100)
    with pytest.raises(ValueError):
        shard.shard_range(4, 4, 100)


def test_two_rank_strong_scaling_matches_single_process():
    """bench.py --strong: the TOTAL row count split over the ranks (uneven by one row) reduces
    to the single-process answer over the same rows."""
    world = 2
    port = _free_port()
    with mp.Manager() as mgr:
        out = mgr.dict()
        mp.spawn(_worker, args=(world, port, out, True), nprocs=world, join=True)
        results = dict(out)
    ts = _tapes()
    want = _shard_results(ts, 0, 2 * ROWS + 1)
    assert results[0] == results[1]
    assert tuple(results[0][0]) == tuple(want[0])
    assert tuple(results[0][1]) == tuple(want[1])


def test_strong_shard_range_partitions_the_rows():
    for total in (0, 1, 7, 1 << 26, (1 << 26) + 5):
        for world in (1, 2, 3, 8):
            parts = [shard.strong_shard_range(r, world, total) for r in range(world)]
            assert parts[0][0] == 0
            for (b0, n0), (b1, _) in zip(parts, parts[1:]):
                assert b0 + n0 == b1
            assert sum(n for _, n in parts) == total
            assert max(n for _, n in parts) - min(n for _, n in parts) <= 1
    with pytest.raises(ValueError):
        shard.strong_shard_range(2, 2, 10)


class _CommCtx:
    """A ctx whose mh_comm_init fails on the ranks in `fail` (the library cannot open RCCL)."""

    def __init__(self, rank, fail):
        self.rank, self.fail, self.calls = rank, fail, []

    def comm_init(self, uid, rank, world):
        self.calls.append((uid, rank, world))
        if rank in self.fail:
            raise RuntimeError("ncclCommInitRank: unhandled system error (stand-in)")


def _exchange_worker(rank, world, port, out, fail):
    import torch.distributed as dist

    from mythril_amd import native

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        native.comm_unique_id = lambda: b"uid-from-rank-0"  # rank 0 only asks
        ctx = _CommCtx(rank, fail)
        exchange, why = shard.setup_exchange(ctx, rank, world)
        out[rank] = (exchange, why, ctx.calls)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fail", [(), (1,), (0, 1)])
def test_exchange_fallback_is_reported(fail):
    """bench.py's result exchange (shard.setup_exchange, world 2 over gloo):
    every rank gets rank 0's communicator id; if any rank's mh_comm_init fails, EVERY rank falls
    back to torch.distributed's all-reduce and every rank holds the reason of each failing rank
    -- bench.py prints them in the JSON line (``exchange_fallback``), not only on stderr."""
    world = 2
    port = _free_port()
    with mp.Manager() as mgr:
        out = mgr.dict()
        mp.spawn(_exchange_worker, args=(world, port, out, fail), nprocs=world, join=True)
        res = dict(out)
    for r in range(world):
        exchange, why, calls = res[r]
        assert calls == [(b"uid-from-rank-0", r, world)]
        if fail:
            assert exchange == "torch"
            assert [w.split(":")[0] for w in why] == ["rank %d" % f for f in fail]
            assert all("ncclCommInitRank" in w for w in why)
        else:
            assert exchange == "library" and why == []
