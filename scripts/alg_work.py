#!/usr/bin/env python3
"""Algorithmic work per evaluation of bench.py's workload, for roofline.achieved.

One evaluation = one (tape, row) pair decided.  Its algorithmic work is what a row-exact lazy
evaluator must execute with this code's per-op instruction costs: the tape's conjuncts in the
emitted (scheduled) order up to and including the first one that is false on that row (all of
them when the row satisfies the tape), each op at the VALU lane-ops the native code spends on
it -- demanded limbs only, constants folded, the division subroutine's executed instructions.
It is measured by running the very instruction lists the GPU runs on the host wave emulator
(tests/native/jit_emu.cpp) and weighting every executed VALU instruction by the fraction of the
wave's rows still undecided when it issues (``alive_valu``).  No evaluation mode can do less:
the short-circuit kernel executes these instructions plus the ones its wave-mates need (a wave
runs a conjunct while any of its 64 rows is alive), the full evaluation executes every
conjunct of every row.  So achieved = this count x evals / kernel time is <= the executed VALU
rate of either mode, and roofline.frac <= 1 for both.

The figures are per build (native.codegen_id()); bench.py reads profiles/alg_work.json only for
the build it runs.

    python scripts/alg_work.py [n_sample_tapes=10000] [rows=256] [--full] [--variant=keccak]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mythril_amd import native, synth  # noqa: E402
from oracle import smt_eval  # noqa: E402
from tests.conftest import build_emulator  # noqa: E402
from tests.emu import Emulator, jit_eval, set_short_circuit  # noqa: E402

OUT = os.path.join(ROOT, "profiles", "alg_work.json")


_W = {}


def _init(rows, full, variant="plain"):
    ts = synth.generate(None, keccak=variant == "keccak")
    seed = synth.load_spec()["assignment_seed"]
    soa = np.zeros((ts.n_vars, 8, rows), dtype=np.uint32)
    for r in range(rows):
        a = smt_eval.gen_assignment(seed, ts.n_vars, r)
        for v in range(ts.n_vars):
            for k in range(8):
                soa[v, k, r] = (a[v] >> (32 * k)) & 0xFFFFFFFF
    emu = Emulator(build_emulator())
    set_short_circuit(emu, not full)
    _W.update(ts=ts, soa=soa, emu=emu)


def _tape(t):
    ts, soa, emu = _W["ts"], _W["soa"], _W["emu"]
    res = jit_eval(emu, ts, t, soa)
    if not res.ok:  # over the 128-VGPR budget: built at 168 by mh_tapes_jit
        res = jit_eval(emu, ts, t, soa, 168)
    assert res.ok, (t, res.why)
    return res.dyn["valu"], res.dyn["alive_valu"]


def measure(picks, rows, full, procs, variant="plain"):
    import multiprocessing as mp

    with mp.get_context("fork").Pool(procs, initializer=_init,
                                     initargs=(rows, full, variant)) as pool:
        out = pool.map(_tape, picks, chunksize=16)
    return (sum(v for v, _ in out) / len(out), sum(a for _, a in out) / len(out))


def main():
    full = "--full" in sys.argv
    variant = next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--variant=")), "plain")
    argv = [a for a in sys.argv[1:] if not a.startswith("--")]
    n_pick = int(argv[0]) if argv else 10000
    rows = int(argv[1]) if len(argv) > 1 else 256
    procs = min(8, os.cpu_count() or 1)
    spec = synth.load_spec()
    n_tapes = spec["n_tapes"]
    stride = max(1, n_tapes // n_pick)
    picks = list(range(0, n_tapes, stride))[:n_pick]
    build_emulator()
    t0 = time.time()
    sc_valu, sc_alive = measure(picks, rows, False, procs, variant)
    entry = {
        "codegen_id": native.codegen_id("jit", variant),
        "variant": variant,
        "tapes_sampled": len(picks),
        "tape_stride": stride,
        "rows": rows,
        "assignment_seed": spec["assignment_seed"],
        "alg_lane_ops_per_eval": sc_alive,
        "exec_lane_ops_per_eval_sc": sc_valu,
        "lane_efficiency_sc": sc_alive / sc_valu,
    }
    if full:
        entry["exec_lane_ops_per_eval_full"] = measure(picks, rows, True, procs, variant)[0]
    entry["emulator_s"] = round(time.time() - t0, 1)
    entry["note"] = ("per (tape, row) evaluation, tapes x generated rows 0..rows-1, host wave "
                     "emulator over the emitted tape bodies (the kernel's per-chunk column loads "
                     "and hit bookkeeping excluded); alg = VALU weighted by the share of the "
                     "wave's rows still undecided (scripts/alg_work.py)")
    entries = []
    if os.path.exists(OUT):
        entries = [e for e in json.load(open(OUT)).get("entries", [])
                   if (e["codegen_id"], e["variant"]) != (entry["codegen_id"], entry["variant"])]
    entries.append(entry)
    json.dump({"entries": entries[-8:]}, open(OUT, "w"), indent=1)
    print(json.dumps(entry, indent=1))


if __name__ == "__main__":
    main()
