"""ctypes wrapper of the test-only host emulator (tests/native/emu.cpp)."""
import ctypes as C

import numpy as np

from mythril_amd.tape import NODE_DTYPE, TapeSet


class EmuError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("%d: %s" % (code, msg))
        self.code = code


class Emulator:
    def __init__(self, path):
        self.lib = C.CDLL(path)
        f = self.lib.emu_eval
        f.restype = C.c_int32
        f.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_uint32,
                      C.c_uint32, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_char_p,
                      C.c_int]

    def eval(self, ts: TapeSet, tape: int, soa: np.ndarray):
        """soa: [n_vars, 8, rows] u32.  Returns (list of root ints, n_regs)."""
        nodes, offs, consts = ts.flatten()
        nodes = np.ascontiguousarray(nodes, dtype=NODE_DTYPE)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        consts = np.ascontiguousarray(consts, dtype=np.uint32)
        rows = soa.shape[2] if soa.size else 1
        if soa.size == 0:
            soa = np.zeros((max(ts.n_vars, 1), 8, 1), dtype=np.uint32)
        soa = np.ascontiguousarray(soa, dtype=np.uint32)
        out = np.zeros((8, rows), dtype=np.uint32)
        nregs = C.c_uint32()
        err = C.create_string_buffer(512)
        r = self.lib.emu_eval(nodes.ctypes.data, offs.ctypes.data, len(ts.tapes),
                              consts.ctypes.data, len(ts.pool.values), ts.n_vars, tape,
                              soa.ctypes.data, rows, out.ctypes.data, C.byref(nregs), err, 512)
        if r != 0:
            raise EmuError(r, err.value.decode())
        vals = []
        for j in range(rows):
            v = 0
            for k in range(8):
                v |= int(out[k, j]) << (32 * k)
            vals.append(v)
        return vals, nregs.value

    def n_slots(self, ts: TapeSet) -> int:
        """Instruction slots the compiler emits for the whole tape set (emu_compile_words)."""
        f = self.lib.emu_compile_words
        f.restype = C.c_int32
        f.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_uint32,
                      C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64), C.c_void_p, C.c_char_p,
                      C.c_int]
        nodes, offs, consts = ts.flatten()
        nodes = np.ascontiguousarray(nodes, dtype=NODE_DTYPE)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        consts = np.ascontiguousarray(consts, dtype=np.uint32)
        cap = 1 << 20
        out = np.zeros(cap, dtype=np.uint32)
        nw = C.c_uint64()
        nrx = np.zeros(max(len(ts.tapes), 1), dtype=np.uint32)
        err = C.create_string_buffer(256)
        r = f(nodes.ctypes.data, offs.ctypes.data, len(ts.tapes), consts.ctypes.data,
              len(ts.pool.values), ts.n_vars, out.ctypes.data, C.c_uint64(cap), C.byref(nw),
              nrx.ctypes.data, err, 256)
        if r != 0:
            raise EmuError(r, err.value.decode())
        return int(nw.value) // 2
