#!/usr/bin/env python3
"""Two processes, one GPU: the N > 1 data path with kernel output.

Launched as `python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1
--master-port P tests/tools/shard_check.py [rows_per_rank]`.  Every rank builds the config-5 tape set
(first 256 tapes) on cuda:0, JIT-compiles it, generates ITS shard of candidate rows on the device
(shard.shard_range; here rank r sweeps shard world-1-r, so the first witnesses come from rank 1) and runs the native code over it; the
per-tape results are combined by shard.allreduce_results (MIN of first witnesses, SUM of counts)
over gloo -- the same reduction the library's RCCL exchange performs between GPUs.  Rank 0 then
runs the whole 2R-row range in one launch and checks that the reduced results are identical, and
checks every tape against the C oracle.  One JSON line on rank 0.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch
    import torch.distributed as dist

    from mythril_amd import native, shard, synth

    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 16
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    torch.cuda.set_device(0)
    spec = synth.load_spec()
    seed = spec["assignment_seed"]
    ts = synth.generate(256)
    ctx = native.Context(0)
    ct = ctx.compile(ts)
    info = ct.jit()
    # ranks sweep the shards in reverse (rank r takes shard world-1-r), so the global first
    # witnesses -- all in the lowest rows for these tapes -- come from rank 1 and the MIN has to
    # carry them across processes
    base, n = shard.shard_range(world - 1 - rank, world, rows)
    a = ctx.assignments(ts.n_vars, n)
    a.generate(seed, base)
    fh, hc = native.run(ctx, ct, a, index_base=base, mode=native.MODE_COUNT_ALL)
    fh_t = torch.tensor(fh.astype(np.int64))
    hc_t = torch.tensor(hc.astype(np.int64))
    shard.allreduce_results(fh_t, hc_t)
    if rank != 0:
        ctx.close()
        dist.destroy_process_group()
        return
    # the single-launch answer over all ranks' rows
    full = ctx.assignments(ts.n_vars, rows * world)
    full.generate(seed, 0)
    f1, h1 = native.run(ctx, ct, full, index_base=0, mode=native.MODE_COUNT_ALL)
    f1 = f1.astype(np.int64)
    h1 = h1.astype(np.int64)
    same = bool(np.array_equal(fh_t.numpy(), f1) and np.array_equal(hc_t.numpy(), h1))
    in_other = int(((f1 < rows) & (f1 != -1)).sum())  # swept by rank 1
    # the C oracle over the same rows (all cores)
    from oracle import ctape

    t0 = time.time()
    want_c, want_f = ctape.count(ts, seed, 0, rows * world, short_circuit=True)
    ok_oracle = bool(np.array_equal(want_c.astype(np.int64), h1) and
                     np.array_equal(want_f.astype(np.int64), f1))
    print(json.dumps({
        "check": "two-process shards on one GPU, gloo reduction of kernel results",
        "world": world, "rows_per_rank": rows, "tapes": len(ts.tapes),
        "jitted": info["n_jitted"], "reduced_equals_single_launch": same,
        "tapes_with_hits": int((h1 > 0).sum()),
        "first_witness_in_rank1_shard": in_other,
        "oracle_equal": ok_oracle,
        "oracle_s": round(time.time() - t0, 2)}), flush=True)
    ctx.close()
    dist.destroy_process_group()
    if not (same and ok_oracle and in_other > 0):
        sys.exit(1)


if __name__ == "__main__":
    main()
