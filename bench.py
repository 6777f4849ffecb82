#!/usr/bin/env python3
"""Sieve throughput on BASELINE.json config 5.

One step = every tape of the synthetic tape set (10^4 seeded random 256-bit constraint tapes,
mythril_amd/synth_spec.json) evaluated against this rank's shard of candidate assignments,
resident in HBM (config 5's 2^26 rows per GPU by default, 8 GiB of columns), in throughput mode:
every (tape, assignment) pair's Bool is decided (MH_MODE_COUNT_ALL), per-tape hit counts and
smallest witnesses are reduced in registers and flushed by atomics.  With N ranks the rows are sharded
(weak scaling) and the only exchange is one all-reduce (MIN of witness index, SUM of counts) of
2 x 8 B per tape over RCCL.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

`--gpus N` with N > 1 and no launcher around it (WORLD_SIZE unset) starts the second form itself,
as a child process before anything touches the GPU, and exits with its return code; rank 0's
JSON line reaches stdout unchanged.  Scaling is weak by default (every rank sweeps
--rows-per-gpu rows); `--strong` splits that many rows over the ranks.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

NOMINAL_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12  # u32 lane-ops/s: 256 CU x 4 SIMD32 x 2.4 GHz
PMC_SUMMARY = os.path.join(HERE, "profiles", "pmc_summary.json")
ALG_WORK = os.path.join(HERE, "profiles", "alg_work.json")
MIN_WORK = os.path.join(HERE, "profiles", "min_work.json")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(ts, seed, seconds: float):
    """Oracle port (oracle/tape_eval.c, OpenMP on all host cores) on a bounded sample, with the
    single-core figure of the same port beside it (SURVEY §8d CPU baseline (1))."""
    from oracle import ctape

    out = ctape.benchmark(ts, seed, seconds)
    one = ctape.benchmark(ts, seed, seconds / 2, threads=1)
    out["single_core"] = {"value": one["value"], "cores": 1, "sample": one["sample"]}
    return out


def launch_ranks(argv, n: int) -> int:
    """`bench.py --gpus N` run bare: one process per GPU through torch.distributed.run, started as
    a CHILD (never an exec: nothing has initialised the GPU yet, and the ranks must own it).
    stdout/stderr are inherited, so the driver reads rank 0's one JSON line as from a direct run."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(n), "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.abspath(__file__)] + list(argv)
    log("[launcher] %d ranks: %s" % (n, " ".join(cmd)))
    return subprocess.run(cmd).returncode


def launch_check(args) -> None:
    """--launch-check: the multi-rank plumbing without a GPU (gloo): every rank reports in and
    rank 0 prints one JSON line naming the ranks that ran.  Used by tests/test_bench_launch.py."""
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    if world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE %d" % (args.gpus, world))
    ranks = torch.zeros(world, dtype=torch.int64)
    ranks[rank] = rank + 1
    if world > 1:
        dist.all_reduce(ranks)
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world,
                          "ranks": [int(r) - 1 for r in ranks.tolist()],
                          "scaling": "strong" if args.strong else "weak"}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--tapes", type=int, default=None, help="default: spec n_tapes (10^4)")
    ap.add_argument("--rows-per-gpu", type=int, default=None,
                    help="default 2^26 (plain: config 5 on one GPU), 2^20 (keccak variant)")
    ap.add_argument("--variant", choices=["plain", "keccak"], default="plain",
                    help="keccak: SURVEY §8d's keccak variant (one keccak256 of a 512-bit "
                         "input per tape); the headline line is the plain config 5")
    ap.add_argument("--engine", choices=["jit", "interp"], default="jit",
                    help="jit: per-tape native gfx950 code (mh_tapes_jit), the interpreter only "
                         "for tapes the JIT does not cover; interp: the threaded-code interpreter")
    ap.add_argument("--max-vgpr", type=int, default=0, help="JIT register budget (0: default)")
    ap.add_argument("--full-eval", action="store_true",
                    help="jit: evaluate every conjunct of every row (MH_JIT_FULL_EVAL) instead of "
                         "leaving a tape once no row of the wave can satisfy it; same results")
    ap.add_argument("--no-companion", action="store_true",
                    help="skip the full-evaluation companion step (N=1, jit, short-circuit runs "
                         "time one full-evaluation step after the timed region and check that "
                         "its per-tape results are identical)")
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling: --rows-per-gpu is the TOTAL row count (config 5: "
                         "2^26 in total) split over the ranks, instead of every rank sweeping "
                         "that many (weak scaling, the default)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--launch-check", action="store_true",
                    help="check the rank launch only (gloo, no GPU): one JSON line with the ranks")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(sys.argv[1:], args.gpus))
    if args.launch_check:
        launch_check(args)
        return
    if args.rows_per_gpu is None:
        args.rows_per_gpu = 1 << 20 if args.variant == "keccak" else 1 << 26

    import torch
    import torch.distributed as dist

    from mythril_amd import native, shard, synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE %d" % (args.gpus, world))
    if world > 1:
        dist.init_process_group("nccl")
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    stream = torch.cuda.current_stream(dev)

    spec = synth.load_spec()
    t0 = time.time()
    ts = synth.generate(args.tapes, keccak=args.variant == "keccak")
    n_tapes = len(ts.tapes)
    ctx = native.Context(local_rank)
    ctx.set_stream(stream.cuda_stream)
    ct = ctx.compile(ts)
    info = ct.info()
    jit_info = None
    if args.engine == "jit":
        jit_info = ct.jit(max_vgpr=args.max_vgpr, short_circuit=not args.full_eval)
        log("[rank %d] jit: %s" % (rank, jit_info))
    # the code this run executes: a hash of the emitted module texts (jit) or of the library's
    # device code objects (interp) -- profiles of that code are keyed by it, host edits keep them
    build_id = ct.code_id() if args.engine == "jit" else native.interp_code_id()
    # SURVEY 8d's op table (mh_tape_info.alg_ops): informational, not a work count
    optable_per_row = sum(int(i["alg_ops"]) for i in info)
    if args.strong:
        index_base, rows = shard.strong_shard_range(rank, world, args.rows_per_gpu)
    else:
        index_base, rows = shard.shard_range(rank, world, args.rows_per_gpu)
    seed = spec["assignment_seed"]
    assign = ctx.assignments(ts.n_vars, rows)
    assign.generate(seed, index_base)
    fh = torch.empty(n_tapes, dtype=torch.int64, device=dev)
    hc = torch.empty(n_tapes, dtype=torch.int64, device=dev)
    exchange, exchange_fallback = None, []
    if world > 1:
        # the library's own RCCL communicator (mh_comm_init); if any rank cannot open it, every
        # rank uses torch.distributed's RCCL for the same MIN / SUM, and the JSON line names why
        exchange, exchange_fallback = shard.setup_exchange(ctx, rank, world, dev)
        log("[rank %d] result exchange: %s%s" % (rank, exchange, "".join(
            "\n  fallback: " + r for r in exchange_fallback)))
    torch.cuda.synchronize(dev)
    log("[rank %d] setup %.1fs: %d tapes, %d insns, %d rows, SURVEY op-table %.0f per row"
        % (rank, time.time() - t0, n_tapes, sum(i["n_insns"] for i in info), rows,
           optable_per_row))

    def step(timed: bool):
        native.results_reset(ctx, fh.data_ptr(), hc.data_ptr(), n_tapes)
        native.run_async(ctx, ct, assign, fh.data_ptr(), hc.data_ptr(), index_base=index_base,
                         mode=native.MODE_COUNT_ALL)
        if exchange == "library":  # the one exchange: MIN of first witnesses, SUM of counts
            ctx.comm_allreduce(fh.data_ptr(), hc.data_ptr(), n_tapes)
        elif exchange == "torch":
            shard.allreduce_results(fh, hc)

    for i in range(args.warmup):
        step(False)
        torch.cuda.synchronize(dev)
        log("[rank %d] warmup %d done" % (rank, i))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ctx.kernel_time()  # drop anything recorded so far
    ctx.enable_timing(True)  # HIP events on the library's own launch stream
    t_start = time.perf_counter()
    for i in range(args.steps):
        step(True)
        if rank == 0:
            torch.cuda.synchronize(dev)
            log("[rank 0] step %d done" % i)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    tot_ms, n_launch = ctx.kernel_time()
    ctx.enable_timing(False)
    kms = tot_ms / max(n_launch, 1)
    ms_per_step = elapsed * 1e3 / args.steps
    evals_per_step = n_tapes * (args.rows_per_gpu if args.strong else rows * world)
    value = evals_per_step / (ms_per_step / 1e3)
    hits = int((hc > 0).sum().item())

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    short_circuit = args.engine == "jit" and not args.full_eval
    companion = None
    if short_circuit and world == 1 and not args.no_companion:
        # the same step on native code without the short circuit: rate and identical results
        fh_sc, hc_sc = fh.clone(), hc.clone()
        ct_full = ctx.compile(ts)
        ct_full.jit(max_vgpr=args.max_vgpr, short_circuit=False)

        def step_full():
            native.results_reset(ctx, fh.data_ptr(), hc.data_ptr(), n_tapes)
            native.run_async(ctx, ct_full, assign, fh.data_ptr(), hc.data_ptr(),
                             index_base=index_base, mode=native.MODE_COUNT_ALL)

        step_full()
        torch.cuda.synchronize(dev)
        ctx.kernel_time()
        ctx.enable_timing(True)
        t1 = time.perf_counter()
        step_full()
        torch.cuda.synchronize(dev)
        full_s = time.perf_counter() - t1
        full_kms, full_n = ctx.kernel_time()
        ctx.enable_timing(False)
        companion = {
            "value": n_tapes * rows / full_s,
            "ms_per_step": full_s * 1e3,
            "kernel_ms": full_kms / max(full_n, 1),
            "results_identical": bool(torch.equal(fh, fh_sc) and torch.equal(hc, hc_sc)),
            "note": "one step of the same workload with MH_JIT_FULL_EVAL (every conjunct of "
                    "every row evaluated), timed after the headline steps",
        }
        log("[rank 0] full-eval companion: %s" % companion)
    try:
        peak_measured = ctx.microbench(0) / 1e12
    except Exception as e:  # pragma: no cover
        log("microbench failed: %s" % e)
        peak_measured = None
    traffic = valu_busy = exec_ops = None
    pmc_tag = None
    if os.path.exists(PMC_SUMMARY):  # the committed PMC profile of this workload and build
        for pmc in json.load(open(PMC_SUMMARY)).get("entries", []):
            if pmc.get("tapes") == n_tapes and pmc.get("rows_per_gpu") == rows and \
                    pmc.get("engine", "interp") == args.engine and \
                    pmc.get("variant", "plain") == args.variant and \
                    bool(pmc.get("short_circuit", False)) == short_circuit and \
                    pmc.get("codegen_id") == build_id:
                traffic = pmc.get("hbm_bytes_per_launch")
                valu_busy = pmc.get("valu_busy")
                exec_ops = pmc.get("exec_lane_ops_per_launch")
                pmc_tag = pmc.get("tag")
    exec_rate = (exec_ops / (kms / 1e3) / 1e12) if exec_ops else None
    # algorithmic work per evaluation of this build (scripts/alg_work.py): the lane-ops a
    # row-exact lazy evaluator needs with this code's per-op costs; neither mode can do less
    alg = None
    if os.path.exists(ALG_WORK) and args.engine == "jit" and n_tapes == spec["n_tapes"]:
        for e in json.load(open(ALG_WORK)).get("entries", []):
            if e.get("codegen_id") == build_id and e.get("variant") == args.variant:
                alg = e
    alg_per_eval = alg["alg_lane_ops_per_eval"] if alg else None
    alg_rate = (alg_per_eval * n_tapes * rows / (kms / 1e3) / 1e12) if alg else None
    # the code-independent minimum work per evaluation (scripts/min_work.py): the roofline's
    # algorithmic count; the code-priced count above is reported beside it as frac_codegen
    mw = None
    if os.path.exists(MIN_WORK) and n_tapes == spec["n_tapes"]:
        for e in json.load(open(MIN_WORK)).get("entries", []):
            if e.get("variant") == args.variant:
                mw = e
    min_per_eval = mw["min_lane_ops_per_eval"] if mw else None
    min_rate = (min_per_eval * n_tapes * rows / (kms / 1e3) / 1e12) if mw else None
    if companion is not None and mw:
        companion["roofline_achieved"] = min_per_eval * n_tapes * rows / (
            companion["kernel_ms"] / 1e3) / 1e12
        companion["roofline_frac"] = companion["roofline_achieved"] / NOMINAL_PEAK_TOPS
        if alg:
            companion["roofline_frac_codegen"] = alg_per_eval * n_tapes * rows / (
                companion["kernel_ms"] / 1e3) / 1e12 / NOMINAL_PEAK_TOPS
    line = {
        "metric": "constraint-evals/sec",
        "value": value,
        "unit": "evals/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong" if args.strong else "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (seeded config-5 tapes, counter-based PRNG assignments)",
        "config": {
            "workload": "synthetic config 5%s: %d random 256-bit constraint tapes x %d "
                        "assignments per GPU, throughput mode"
                        % (" (keccak variant: + one keccak256 of 512 bits per tape)"
                           if args.variant == "keccak" else "", n_tapes, rows),
            "variant": args.variant,
            "tapes": n_tapes,
            "rows_per_gpu": rows,
            "rows_total": args.rows_per_gpu if args.strong else rows * world,
            "vars": ts.n_vars,
            "mode": "count_all",
            "engine": args.engine,
            "short_circuit": short_circuit,
            "parallelism": "dp%d (row shards, all-reduce of per-tape results%s)"
                           % (world, "" if exchange is None else ", %s RCCL" % exchange),
        },
        "exchange": exchange,
        "exchange_fallback": "; ".join(exchange_fallback) or None,
        "per_gpu": value / world,
        "kernel_ms": kms,
        "tapes_with_witness": hits,
        "build": build_id,
        "jit": jit_info,
        "roofline": {
            "bound": "valu",
            "achieved": min_rate,
            "peak": NOMINAL_PEAK_TOPS,
            "unit": "T u32-ops/s",
            "frac": (min_rate / NOMINAL_PEAK_TOPS) if min_rate else None,
            "min_lane_ops_per_eval": min_per_eval,
            "min_profile": ("profiles/min_work.json (%d tapes x %d rows, code-independent op "
                            "table)" % (mw["tapes_sampled"], mw["rows"])) if mw else None,
            "achieved_codegen": alg_rate,
            "frac_codegen": (alg_rate / NOMINAL_PEAK_TOPS) if alg_rate else None,
            "traffic": traffic,
            "traffic_unit": "bytes per launch (PMC FETCH_SIZE + WRITE_SIZE, profiles/)",
            "alg_lane_ops_per_eval": alg_per_eval,
            "alg_profile": ("profiles/alg_work.json build %s (%d tapes x %d rows)"
                            % (build_id, alg["tapes_sampled"], alg["rows"])) if alg else None,
            "executed": exec_rate,
            "frac_executed": (exec_rate / NOMINAL_PEAK_TOPS) if exec_rate else None,
            "exec_lane_ops_per_eval": (exec_ops / (n_tapes * rows)) if exec_ops else None,
            "pmc_profile": pmc_tag,
            "valu_busy_pmc": valu_busy,
            "peak_measured_add_chain": peak_measured,
            "optable_ops_per_eval": optable_per_row / n_tapes,
            "note": "achieved = the code-independent minimum work per launch / this run's "
                    "kernel time: per (tape, row) the cheapest node set deciding the row's Bool "
                    "(lazy AND / OR / ITE, constants folded, demanded limbs) priced by a fixed "
                    "per-op table of minimum u32 lane-ops (min_lane_ops_per_eval, "
                    "scripts/min_work.py). achieved_codegen / frac_codegen = the same per "
                    "(tape, row) prefix in the emitted conjunct order at THIS code's per-op "
                    "cost (alg_lane_ops_per_eval, per build, scripts/alg_work.py on the host "
                    "emulator of the emitted code). Both <= executed, so frac <= frac_codegen "
                    "<= frac_executed <= 1. executed = PMC SQ_INSTS_VALU x 64 of the profile of "
                    "this build (pmc_profile; null when none) / kernel time; frac_executed / "
                    "frac = the lanes a wave keeps busy for rows already decided. peak = 256 CU "
                    "x 4 SIMD x 32 lanes x 2.4 GHz (a wave64 VALU op issues over 2 cycles). "
                    "optable_ops_per_eval prices SURVEY 8d's op table, which the native code "
                    "undercuts (DESIGN 5.1): informational, not a work count.",
        },
    }
    if companion is not None:
        line["full_eval"] = companion
    if world == 1 and not args.no_cpu_baseline:
        try:
            line["cpu_baseline"] = cpu_baseline(ts, seed, args.cpu_seconds)
        except Exception as e:  # pragma: no cover
            log("cpu baseline failed: %s" % e)
            line["cpu_baseline"] = None
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
