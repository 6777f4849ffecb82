#!/usr/bin/env python3
"""Per-op device cost on the MI355X, from HIP-event kernel time (mh_ctx_kernel_time).

(1) Tape sets made of one op kind (chains of 32 ops over the four synthetic variables) in
    throughput mode: prints cycles per (op x wave64) as `wave_cycles_per_op` assuming every SIMD
    of the chip busy at 2.4 GHz (so it includes interpreter overhead and latency not hidden).
(2) The config-5 synthetic tape set split by feature (tapes with / without the division family),
    to attribute the benchmark's time.
One JSON line per measurement."""
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

from mythril_amd import native, synth  # noqa: E402
from mythril_amd.tape import Op, TapeSet  # noqa: E402

ROWS = int(os.environ.get("ROWS", 1 << 21))
TAPES = 256
CHAIN = 32
SIMD_CYC = 1024 * 2.4e9  # SIMD-cycles per second, whole chip

KINDS = {
    "add": Op.BVADD, "sub": Op.BVSUB, "mul": Op.BVMUL, "and": Op.BVAND, "xor": Op.BVXOR,
    "udiv": Op.BVUDIV, "urem": Op.BVUREM, "sdiv": Op.BVSDIV, "srem": Op.BVSREM,
    "shl_var": Op.BVSHL, "lshr_var": Op.BVLSHR, "ult": Op.BVULT, "eq": Op.EQ,
}


def build(kind: str) -> TapeSet:
    ts = TapeSet(["a", "b", "c", "d"])
    for t in range(TAPES):
        b = ts.builder()
        vs = [b.var(n) for n in ("a", "b", "c", "d")]
        x = vs[t % 4]
        acc = None
        for i in range(CHAIN):
            y = vs[(t + i + 1) % 4]
            if kind in ("ult", "eq"):
                c = b.op(KINDS[kind], x, y)
                acc = c if acc is None else b.op(Op.AND, acc, c)
                x = b.op(Op.BVADD, x, b.const(i + 1, 256)) if i % 2 else y
            elif kind == "bnot":  # dispatch cost: one VALU op per instruction
                acc = b.op(Op.BVULT, x, y) if acc is None else b.op(Op.NOT, acc)
            elif kind == "shli":
                x = b.op(Op.BVSHL, x, b.const(1 + i % 200, 256))
            elif kind == "const_add":
                x = b.op(Op.BVADD, x, b.const((t * 977 + i) * 0x9E3779B97F4A7C15, 256))
            elif kind == "extract_concat":
                lo = b.op(Op.EXTRACT, x, imm0=127, imm1=0)
                hi = b.op(Op.EXTRACT, y, imm0=255, imm1=128)
                x = b.op(Op.CONCAT, lo, hi)
            elif kind == "ite":
                x = b.op(Op.ITE, b.op(Op.BVULT, x, y), y, x)
            elif kind in ("udiv_big", "urem_big"):
                # divisor with the top limb cleared: 2-digit quotients, x stays full width
                yy = b.op(Op.BVLSHR, y, b.const(32, 256))
                q = b.op(Op.BVUDIV if kind == "udiv_big" else Op.BVUREM, x, yy)
                x = b.op(Op.BVXOR, q, y)
            else:
                x = b.op(KINDS[kind], x, y)
        root = acc if acc is not None else b.op(Op.BVULT, x, vs[0])
        ts.add(b.finish(root))
    return ts


def timed_run(ctx, ct, a, rows, d_fh, d_hc, n):
    native.results_reset(ctx, d_fh.data_ptr(), d_hc.data_ptr(), n)
    native.run_async(ctx, ct, a, d_fh.data_ptr(), d_hc.data_ptr(), row_count=rows,
                     mode=native.MODE_COUNT_ALL)
    ctx.synchronize()
    ctx.kernel_time()
    ctx.enable_timing(True)
    native.run_async(ctx, ct, a, d_fh.data_ptr(), d_hc.data_ptr(), row_count=rows,
                     mode=native.MODE_COUNT_ALL)
    ms, _ = ctx.kernel_time()
    ctx.enable_timing(False)
    return ms


def main():
    import torch

    ctx = native.Context(0)
    a = ctx.assignments(4, ROWS)
    a.generate(12345, 0)
    d_fh = torch.empty(16384, dtype=torch.int64, device="cuda")
    d_hc = torch.empty(16384, dtype=torch.int64, device="cuda")
    waves = ROWS / 64
    kinds = ["bnot"] + list(KINDS) + ["shli", "const_add", "extract_concat", "ite", "udiv_big", "urem_big"]
    for kind in kinds:
        ts = build(kind)
        ct = ctx.compile(ts)
        info = ct.info()
        insns = sum(i["n_insns"] for i in info)
        ms = timed_run(ctx, ct, a, ROWS, d_fh, d_hc, len(ts.tapes))
        cyc = ms * 1e-3 * SIMD_CYC / (insns * waves)
        print(json.dumps({"op": kind, "device_insns": insns, "kernel_ms": round(ms, 3),
                          "wave_cycles_per_insn": round(cyc, 1)}), flush=True)
    # synthetic config-5 tapes split by feature
    ts = synth.generate(2000)
    ct = ctx.compile(ts)
    info = ct.info()
    feats = np.array([i["features"] for i in info])
    for name, sel in (("synth_nodiv", (feats & 1) == 0), ("synth_div", (feats & 1) != 0)):
        sub = TapeSet(ts.var_names)
        sub.pool = ts.pool
        for t, keep in zip(ts.tapes, sel):
            if keep:
                sub.tapes.append(t)
        cs = ctx.compile(sub)
        inf = cs.info()
        insns = sum(i["n_insns"] for i in inf)
        ms = timed_run(ctx, cs, a, ROWS // 4, d_fh, d_hc, len(sub.tapes))
        cyc = ms * 1e-3 * SIMD_CYC / (len(sub.tapes) * (ROWS // 4) / 64)
        print(json.dumps({"op": name, "tapes": len(sub.tapes), "device_insns": insns,
                          "kernel_ms": round(ms, 3), "wave_cycles_per_tape": round(cyc, 1),
                          "wave_cycles_per_insn": round(cyc * len(sub.tapes) / insns, 1),
                          "alg_ops_per_tape": sum(i["alg_ops"] for i in inf) / len(sub.tapes)}),
              flush=True)


if __name__ == "__main__":
    main()
