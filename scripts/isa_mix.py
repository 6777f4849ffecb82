#!/usr/bin/env python3
"""Static instruction mix of the compiled config-5 tape set (test-only host emulator build):
per device opcode, how many instructions read their first operand from the accumulator
(a' = X) and skip the write-back (d' = X).  Guides which asm-core forms pay off."""
import ctypes as C
import os
import sys
from collections import Counter

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

from mythril_amd import synth  # noqa: E402
from mythril_amd.tape import NODE_DTYPE  # noqa: E402
from tests.conftest import build_emulator  # noqa: E402


def opnames():
    src = open(os.path.join(HERE, "mythril_amd", "csrc", "dev_isa.h")).read()
    body = src[src.index("enum mh_dop"):src.index("D_NUM_OPS")]
    body = "\n".join(line.split("//")[0] for line in body.splitlines())
    names, val = {}, -1
    import re
    for tok in re.findall(r"(D_[A-Z0-9_]+)\s*(?:=\s*([A-Z0-9_]+))?", body):
        name, v = tok
        if v:
            val = int(v) if v.isdigit() else names_rev[v]
        else:
            val += 1
        names[val] = name
        names_rev[name] = val
    return names


names_rev = {}


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    ts = synth.generate(n)
    lib = C.CDLL(build_emulator())
    f = lib.emu_compile_words
    f.restype = C.c_int32
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_uint32,
                  C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64), C.c_void_p, C.c_char_p, C.c_int]
    nodes, offs, consts = ts.flatten()
    nodes = np.ascontiguousarray(nodes, dtype=NODE_DTYPE)
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    consts = np.ascontiguousarray(consts, dtype=np.uint32)
    cap = 1 << 26
    out = np.zeros(cap, dtype=np.uint32)
    nw = C.c_uint64()
    nrx = np.zeros(len(ts.tapes), dtype=np.uint32)
    err = C.create_string_buffer(256)
    r = f(nodes.ctypes.data, offs.ctypes.data, len(ts.tapes), consts.ctypes.data,
          len(ts.pool.values), ts.n_vars, out.ctypes.data, C.c_uint64(cap), C.byref(nw),
          nrx.ctypes.data, err, 256)
    assert r == 0, err.value
    w = out[:nw.value].reshape(-1, 2)
    names = opnames()
    mix = Counter()
    pos = 0  # slot index within the current tape (windows are MH_WINDOW slots from its start)
    s = 0
    while s < len(w):
        w0, w1 = int(w[s][0]), int(w[s][1])
        op = w1 & 0xFF
        nm = names.get(op, str(op))
        if nm == "D_WINDOW":
            adv = (pos // 64 + 1) * 64 - pos
            s += adv
            pos += adv
            continue
        if nm == "D_END":
            s += 1
            pos = 0
            continue
        a, d = w0 & 0xFF, (w0 >> 16) & 0xFF
        mix[(nm, "aX" if a in (7, 9, 15) else "aR", "dX" if d in (7, 9, 15) else "dR")] += 1
        yc = nm.endswith(("_C", "_CX")) or nm in ("D_LOADC", "D_LOADC_X")
        n = 5 if (yc or (op >= names_rev["D_UADD_NOOVFL"] and w1 >> 31)) else 1
        s += n
        pos += n
    tot = sum(mix.values())
    for k, v in mix.most_common(40):
        print("%-12s %s %s %7d %5.1f%%" % (k[0], k[1], k[2], v, 100.0 * v / tot))
    print("total", tot)


if __name__ == "__main__":
    main()
