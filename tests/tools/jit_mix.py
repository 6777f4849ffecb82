#!/usr/bin/env python3
"""Executed instruction mix of the JIT's code on config-5 tapes, from the host wave emulator
(tests/native/jit_emu.cpp runs the very instruction lists the GPU runs, on the same generated
rows): VALU per wave-evaluation, split into 2-cycle and 4-cycle issue classes (the measured
issue costs of profiles/r02a/valu_peak.json) and into tape body vs the division subroutine.
With a measured evals/s it gives the cycle-weighted VALU issue busy of the native kernel.

    python tests/tools/jit_mix.py [n_tapes] [evals_per_s]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from mythril_amd import synth  # noqa: E402
from oracle import smt_eval  # noqa: E402
from tests.conftest import build_emulator  # noqa: E402
from tests.emu import Emulator, jit_eval  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    evals = float(sys.argv[2]) if len(sys.argv) > 2 else None
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
    tot = dict(valu=0, wide=0, salu=0, div_valu=0, div_wide=0, f64=0, alive_valu=0)
    import ctypes as C
    tagf = emu.lib.emu_jit_tag_valu
    tagf.restype = None
    tagf.argtypes = [C.POINTER(C.c_uint64), C.c_int]
    tags = (C.c_uint64 * 512)()
    tagf(tags, 1)
    m = 0
    for i in range(n):
        res = jit_eval(emu, ts, i, soa)
        if not res.ok:
            continue
        m += 1
        for k in tot:
            tot[k] += res.dyn[k]
    per = {k: v / m for k, v in tot.items()}
    tagf(tags, 1)
    chunks = m * (rows // 64)
    import re
    src = open(os.path.join(ROOT, "mythril_amd", "csrc", "dev_isa.h")).read()
    body = src[src.index("enum mh_dop"):]
    body = body[body.index("{") + 1:body.index("};")]
    body = re.sub(r"//[^\n]*", "", body)
    names, nxt = {}, 0
    for ent in [e.strip() for e in body.split(",") if e.strip()]:
        if "=" in ent:
            nm, val = [x.strip() for x in ent.split("=")]
            nxt = int(val, 0) if val[0].isdigit() else {v: k for k, v in names.items()}[val]
        else:
            nm = ent
        names[nxt] = nm
        nxt += 1
    by_op = {}
    for t in range(256):
        for base, suffix in ((0, ""), (256, "/div")):
            v = tags[base + t]
            if v:
                name = names.get(t, "other") if t != 255 else "other"
                by_op[name + suffix] = round(v / chunks, 2)
    by_op = dict(sorted(by_op.items(), key=lambda kv: -kv[1]))
    narrow = per["valu"] - per["wide"]
    # issue cycles per wave-evaluation at the measured costs (8 waves / SIMD,
    # profiles/r02e/valu_peak.json): 2-cycle class 2.56, VOP3 / carry / compare / shift 4.5,
    # f64 6.1 (counted inside the wide class)
    cyc = 2.56 * narrow + 4.5 * (per["wide"] - per["f64"]) + 6.1 * per["f64"]
    out = {"tapes": m, "per_wave_eval": per, "issue_cycles_per_wave_eval": cyc,
           "valu_lane_ops_per_eval": per["valu"], "valu_per_wave_eval_by_op": by_op}
    if evals:
        wave_evals = evals / 64.0
        out["issue_busy"] = wave_evals * cyc / (1024 * 2.4e9)
        out["exec_lane_ops_per_s"] = evals * per["valu"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
