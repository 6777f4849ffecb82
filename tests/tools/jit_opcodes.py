#!/usr/bin/env python3
"""Executed VALU of the JIT's code on config-5 tapes by machine opcode (host wave emulator,
tests/native/jit_emu.cpp: the very instruction lists the GPU runs), per wave-evaluation, in the
tape bodies and in the division subroutine; e64 (VOP3-encoded) forms are counted with their op.
Round 6 uses it to price instruction-class substitutions.

    python tests/tools/jit_opcodes.py [n_tapes]
"""
import ctypes as C
import json
import os
import re
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from mythril_amd import synth  # noqa: E402
from oracle import smt_eval  # noqa: E402
from tests.conftest import build_emulator  # noqa: E402
from tests.emu import Emulator, jit_eval  # noqa: E402


def opcode_names():
    src = open(os.path.join(ROOT, "mythril_amd", "csrc", "jit.h")).read()
    body = src[src.index("enum Op : uint16_t"):]
    body = body[body.index("{") + 1:body.index("};")]
    body = re.sub(r"//[^\n]*", "", body)
    return [e.strip() for e in body.split(",") if e.strip()]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    emu = Emulator(build_emulator())
    ts = synth.generate(n)
    seed = synth.load_spec()["assignment_seed"]
    rows = 128
    soa = np.zeros((4, 8, rows), dtype=np.uint32)
    for r in range(rows):
        a = smt_eval.gen_assignment(seed, 4, r)
        for v in range(4):
            for k in range(8):
                soa[v, k, r] = (a[v] >> (32 * k)) & 0xFFFFFFFF
    f = emu.lib.emu_jit_opcode_valu
    f.restype = None
    f.argtypes = [C.POINTER(C.c_uint64), C.c_int]
    buf = (C.c_uint64 * 512)()
    f(buf, 1)
    m = 0
    for i in range(n):
        if jit_eval(emu, ts, i, soa).ok:
            m += 1
    f(buf, 1)
    names = opcode_names()
    chunks = m * (rows // 64)
    out = {"tapes": m, "body": {}, "div": {}}
    for d, key in ((0, "body"), (1, "div")):
        for i in range(256):
            if buf[256 * d + i]:
                out[key][names[i] if i < len(names) else str(i)] = round(buf[256 * d + i] / chunks, 3)
        out[key] = dict(sorted(out[key].items(), key=lambda kv: -kv[1]))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
