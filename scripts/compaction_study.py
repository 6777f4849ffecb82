#!/usr/bin/env python3
"""Compaction study for the headline kernel: how much executed VALU a survivor
queue would save, measured on the host wave emulator over the very instruction lists the GPU runs.

Per (tape, 64-row chunk) the emulator records the VALU executed up to each short-circuit test and
the live-lane mask after it (tests/native/jit_emu.cpp emu_jit_segments).  From those traces:

* ``current``: what the kernel executes (a segment runs when any lane of its wave is alive);
* ``compact@k``: the head (everything up to and including test k) runs per chunk as today; the
  rows alive after test k are queued and the rest of the tape runs on batches of 64 queued rows
  (a segment runs when any row of the batch is alive), a partial batch at the end of the row range;
* ``ideal``: every VALU weighted by the live lanes (the alg_work.py count).

    python scripts/compaction_study.py [n_tapes=400] [rows=4096]
"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mythril_amd import synth  # noqa: E402
from oracle import smt_eval  # noqa: E402
from tests.conftest import build_emulator  # noqa: E402
from tests.emu import Emulator, _jit_fn, jit_eval  # noqa: E402


def traces(emu, ts, t, soa):
    seg = _jit_fn(emu.lib, "emu_jit_segments", C.c_uint64, [C.c_void_p, C.c_uint64, C.c_int])
    seg(None, 0, 1)
    res = jit_eval(emu, ts, t, soa)
    if not res.ok:
        seg(None, 0, 1)
        res = jit_eval(emu, ts, t, soa, 168)
    n = seg(None, 0, 0)
    buf = np.zeros(4 * n, dtype=np.uint32)
    seg(buf.ctypes.data, n, 1)
    buf = buf.reshape(n, 4)
    chunks = []
    cur = []
    for c, v, lo, hi in buf.tolist():
        mask = lo | (hi << 32)
        if c & 0x80000000:
            chunks.append((cur, v))
            cur = []
        else:
            cur.append((v, mask))
    return chunks


def simulate(chunks, k):
    """VALU (wave instructions) of compaction after test k (1-based); k = 0: the current kernel."""
    total = 0
    queue = []  # (chunk index, lane)
    tails = []
    for ci, (tests, end) in enumerate(chunks):
        if k == 0 or len(tests) < k:
            # current behaviour: the chunk runs until its wave dies
            last = 0
            alive = True
            for v, mask in tests:
                last = v
                if mask == 0:
                    alive = False
                    break
            total += last if not alive else end
            continue
        v_head, m_head = tests[k - 1]
        total += v_head
        queue += [(ci, l) for l in range(64) if (m_head >> l) & 1]
        while len(queue) >= 64:
            tails.append(queue[:64])
            queue = queue[64:]
    if queue:
        tails.append(queue)
    for batch in tails:
        # the tail's segments: after test k, the later tests of the batch's chunks
        ci0 = batch[0][0]
        tests, end = chunks[ci0]
        v_prev = tests[k - 1][0]
        alive = set(batch)
        done_at = end
        for j in range(k, len(tests)):
            alive = {(c, l) for (c, l) in alive if (chunks[c][0][j][1] >> l) & 1}
            if not alive:
                done_at = tests[j][0]
                break
        total += done_at - v_prev
    return total


def simulate_pairs(chunks, k, merge_cost):
    """Pairwise merge in registers: heads (through test k) of two consecutive chunks; when their
    survivors fit one wave, the tail runs once on the merged lanes (plus merge_cost VALU)."""
    total = 0

    def tail_cost(rows):
        if not rows:
            return 0
        ci0 = rows[0][0]
        tests, end = chunks[ci0]
        v_prev = tests[k - 1][0]
        alive = set(rows)
        done_at = end
        for j in range(k, len(tests)):
            alive = {(c, l) for (c, l) in alive if (chunks[c][0][j][1] >> l) & 1}
            if not alive:
                done_at = tests[j][0]
                break
        return done_at - v_prev

    for ci in range(0, len(chunks) - 1, 2):
        pair = [ci, ci + 1]
        if any(len(chunks[c][0]) < k for c in pair):
            total += simulate([chunks[c] for c in pair], 0)
            continue
        surv = []
        for c in pair:
            tests, _ = chunks[c]
            total += tests[k - 1][0]
            surv.append([(c, l) for l in range(64) if (tests[k - 1][1] >> l) & 1])
        if len(surv[0]) + len(surv[1]) <= 64 and surv[0] and surv[1]:
            total += merge_cost + tail_cost(surv[0] + surv[1])
        else:
            total += tail_cost(surv[0]) + tail_cost(surv[1])
    return total


def main():
    n_t = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    rows = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    ts = synth.generate()
    seed = synth.load_spec()["assignment_seed"]
    soa = np.zeros((ts.n_vars, 8, rows), dtype=np.uint32)
    for r in range(rows):
        a = smt_eval.gen_assignment(seed, ts.n_vars, r)
        for v in range(ts.n_vars):
            for kk in range(8):
                soa[v, kk, r] = (a[v] >> (32 * kk)) & 0xFFFFFFFF
    emu = Emulator(build_emulator())
    stride = max(1, len(ts.tapes) // n_t)
    agg = {"current": 0, "compact@1": 0, "compact@2": 0, "ideal": 0.0, "chunks": 0}
    single = 0
    for t in range(0, len(ts.tapes), stride)[:n_t]:
        ch = traces(emu, ts, t, soa)
        agg["chunks"] += len(ch)
        agg["current"] += simulate(ch, 0)
        agg["compact@1"] += simulate(ch, 1)
        agg["compact@2"] += simulate(ch, 2)
        agg["pairs@1"] = agg.get("pairs@1", 0) + simulate_pairs(ch, 1, 40)
        qn = sum(bin(tests[0][1]).count("1") for tests, _ in ch if tests)
        agg["queued_rows"] = agg.get("queued_rows", 0) + qn
        agg["rows"] = agg.get("rows", 0) + 64 * len(ch)
        single += all(len(tests) == 0 for tests, _ in ch)
    agg["tapes"] = n_t
    agg["tapes_without_test"] = single
    for key in ("compact@1", "compact@2", "pairs@1"):
        agg[key + "_ratio"] = agg[key] / agg["current"]
    print(json.dumps(agg, indent=1))


if __name__ == "__main__":
    main()
