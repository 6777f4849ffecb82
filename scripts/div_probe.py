#!/usr/bin/env python3
"""Debug probe: device udiv/urem on chosen operand pairs (one row each) vs Python ints."""
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
import numpy as np  # noqa: E402

from mythril_amd import native  # noqa: E402
from mythril_amd.tape import Op, TapeSet  # noqa: E402

M = (1 << 256) - 1
PAIRS = [(M, 5), (M, 2), (M, 3), (M, 7), (M - 1, 5), (1 << 255, 5), ((1 << 224) - 1, 5),
         ((1 << 64) - 1, 5), (12345678901234567890, 5), (M, 0x100000001), (M, (1 << 200) + 1)]


def main():
    ctx = native.Context(0)
    for x, y in PAIRS:
        ts = TapeSet(["x", "y"])
        for op in (Op.BVUDIV, Op.BVUREM):
            for yconst in (False, True):
                b = ts.builder()
                yy = b.const(y, 256) if yconst else b.var("y")
                ts.add(b.finish(b.op(op, b.var("x"), yy)))
        ct = ctx.compile(ts)
        a = ctx.assignments(2, 1)
        soa = np.zeros((2, 8, 1), dtype=np.uint32)
        for k in range(8):
            soa[0, k, 0] = (x >> (32 * k)) & 0xFFFFFFFF
            soa[1, k, 0] = (y >> (32 * k)) & 0xFFFFFFFF
        a.upload(soa)
        res = [native.limbs_to_ints(native.eval_values(ctx, ct, i, a))[0] for i in range(4)]
        want = [x // y, x // y, x % y, x % y]
        ok = res == want
        print("OK " if ok else "BAD", hex(x), hex(y))
        if not ok:
            for r, w in zip(res, want):
                print("   got  %064x" % r)
                print("   want %064x" % w)


if __name__ == "__main__":
    main()
