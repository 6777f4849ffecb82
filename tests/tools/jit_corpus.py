#!/usr/bin/env python3
"""Write a corpus of tape sets for tests/native/jit_replay.cpp (test infrastructure): random
tapes of every IR op and width (tests/fuzz.py: division family, shifts, EVM ops, keccak,
extract / concat / extension chains; 3 columns held in registers and 24 loaded at use), the first
config-5 tapes (mythril_amd/synth.py, plain and keccak variants), each with edge-biased assignment
rows and the values the regular (unsanitized) emulator build gives for every tape: the
interpreter's lowering (emu_eval, csrc/compile.cpp) and the JIT's machine code (emu_jit_eval,
csrc/jit.cpp) on the host wave emulator.  The replay recomputes them under AddressSanitizer /
UBSan and must agree word for word (tests/test_host_sanitized.py).

Format (little-endian): u32 n_sets, then per set: u32 n_tapes, n_vars, n_consts, rows,
u64 offs[n_tapes + 1], mh_node nodes[offs[n_tapes]], u32 consts[n_consts][8],
u32 soa[n_vars][8][rows]; per tape: i32 interp_rc, u32 interp[8][rows], i32 jit_rc,
u32 jitted, u32 jit[8][rows].

    python tests/tools/jit_corpus.py OUT
"""
import ctypes as C
import os
import random
import struct
import sys

HERE = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

from mythril_amd import synth  # noqa: E402
from mythril_amd.native import NODE_DTYPE  # noqa: E402
from mythril_amd.tape import TapeSet  # noqa: E402
from tests.conftest import build_emulator  # noqa: E402
from tests.emu import _jit_fn  # noqa: E402
from tests.fuzz import TapeFuzzer, assignment_soa  # noqa: E402

ROWS = 64


def tapesets():
    for seed, n_vars, n in ((11, 3, 24), (12, 3, 24), (13, 24, 16), (14, 5, 24)):
        rng = random.Random(seed)
        ts = TapeSet()
        fz = TapeFuzzer(rng, ts, n_vars=n_vars, max_depth=4)
        for _ in range(n):
            fz.tape()
        yield ts, assignment_soa(rng, ts.n_vars, ROWS)
    for keccak in (False, True):
        ts = TapeSet()
        spec = synth.load_spec()
        for t in range(12):
            synth.gen_tape(ts, t, spec, keccak=keccak)
        yield ts, assignment_soa(random.Random(99), ts.n_vars, ROWS)


def main():
    lib = C.CDLL(build_emulator())
    args = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32,
            C.c_void_p, C.c_uint64, C.c_void_p]
    interp = _jit_fn(lib, "emu_eval", C.c_int32, args + [C.c_void_p, C.c_char_p, C.c_int])
    jit = _jit_fn(lib, "emu_jit_eval", C.c_int32,
                  args + [C.c_uint32, C.c_void_p, C.c_char_p, C.c_int])
    sets = list(tapesets())
    with open(sys.argv[1], "wb") as f:
        f.write(struct.pack("<I", len(sets)))
        for ts, soa in sets:
            nodes, offs, consts = ts.flatten()
            nodes = np.ascontiguousarray(nodes, dtype=NODE_DTYPE)
            offs = np.ascontiguousarray(offs, dtype=np.uint64)
            consts = np.ascontiguousarray(consts, dtype=np.uint32).reshape(-1, 8)
            soa = np.ascontiguousarray(soa, dtype=np.uint32)
            n_tapes, n_consts = len(ts.tapes), len(consts)
            f.write(struct.pack("<IIII", n_tapes, ts.n_vars, n_consts, ROWS))
            f.write(offs.tobytes() + nodes.tobytes() + consts.tobytes() + soa.tobytes())
            for t in range(n_tapes):
                out = np.zeros((8, ROWS), dtype=np.uint32)
                nregs = C.c_uint32()
                err = C.create_string_buffer(512)
                rc = interp(nodes.ctypes.data, offs.ctypes.data, n_tapes, consts.ctypes.data,
                            n_consts, ts.n_vars, t, soa.ctypes.data, ROWS, out.ctypes.data,
                            C.addressof(nregs), err, 512)
                f.write(struct.pack("<i", rc) + out.tobytes())
                out2 = np.zeros((8, ROWS), dtype=np.uint32)
                info = np.zeros(16, dtype=np.uint32)
                rc2 = jit(nodes.ctypes.data, offs.ctypes.data, n_tapes, consts.ctypes.data,
                          n_consts, ts.n_vars, t, soa.ctypes.data, ROWS, out2.ctypes.data, 128,
                          info.ctypes.data, err, 512)
                f.write(struct.pack("<iI", rc2, int(info[0])) + out2.tobytes())


if __name__ == "__main__":
    main()
