#!/usr/bin/env python3
"""Per-op device cost on the MI355X: tape sets made of one op kind (chains of 32 ops over the
four synthetic variables), timed in throughput mode.  Prints one JSON line per op kind:
ns per (op x 64-lane wave) and VALU-cycle equivalents, used to direct kernel work."""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

from mythril_amd import native  # noqa: E402
from mythril_amd.tape import Op, TapeSet  # noqa: E402

ROWS = int(os.environ.get("ROWS", 1 << 18))
TAPES = 64
CHAIN = 32

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
            else:
                x = b.op(KINDS[kind], x, y)
        root = acc if acc is not None else b.op(Op.BVULT, x, vs[0])
        ts.add(b.finish(root))
    return ts


def main():
    ctx = native.Context(0)
    a = ctx.assignments(4, ROWS)
    a.generate(12345, 0)
    kinds = list(KINDS) + ["shli", "const_add", "extract_concat", "ite"]
    for kind in kinds:
        ts = build(kind)
        ct = ctx.compile(ts)
        info = ct.info()
        insns = sum(i["n_insns"] for i in info)
        native.run(ctx, ct, a, row_count=1 << 14)  # warm-up
        t0 = time.perf_counter()
        native.run(ctx, ct, a)
        dt = time.perf_counter() - t0
        waves = ROWS / 64
        ns_per_insn_wave = dt * 1e9 / (insns * waves)
        # 1024 SIMDs issue one wave64 VALU op per 2 cycles at ~2.4 GHz
        cyc = ns_per_insn_wave * 1024 * 2.4 / 2
        print(json.dumps({"op": kind, "device_insns": insns, "seconds": round(dt, 4),
                          "valu_slots_per_insn": round(cyc, 1)}), flush=True)


if __name__ == "__main__":
    main()
