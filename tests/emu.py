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
        return len(self.words(ts)) // 2

    def words(self, ts: TapeSet) -> np.ndarray:
        """The slot words (w0, w1 pairs) the compiler emits for the whole tape set."""
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
        return out[:int(nw.value)].copy()


class JitResult:
    def __init__(self, info, values, why):
        self.ok = bool(info[0])
        self.max_vgpr, self.n_valu, self.n_valu_wide, self.n_salu = (int(x) for x in info[1:5])
        self.calls_div, self.root_bool, self.code_bytes = bool(info[5]), bool(info[6]), int(info[7])
        self.values = values
        self.why = why
        # executed per 64-row chunk (wave): VALU, 4-cycle VALU, SALU, division VALU / 4-cycle
        self.dyn = dict(zip(("valu", "wide", "salu", "div_valu", "div_wide", "f64"),
                            (int(x) for x in info[8:14])))
        # VALU weighted by the fraction of lanes still satisfying the conjuncts tested so far:
        # what perfect lane compaction would execute
        self.dyn["alive_valu"] = int(info[14]) / 16.0


def _jit_fn(lib, name, restype, argtypes):
    f = getattr(lib, name)
    f.restype = restype
    f.argtypes = argtypes
    return f


def jit_eval(emu: "Emulator", ts: TapeSet, tape: int, soa: np.ndarray, max_vgpr: int = 128):
    """The JIT's machine code for one tape, run by the host wave emulator
    (tests/native/jit_emu.cpp) over rows of `soa` ([n_vars, 8, rows] u32).  Returns a
    JitResult whose .values are root ints per row (None when the tape is not jitted)."""
    f = _jit_fn(emu.lib, "emu_jit_eval", C.c_int32,
                [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_uint32,
                 C.c_uint32, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint32, C.c_void_p,
                 C.c_char_p, C.c_int])
    nodes, offs, consts = ts.flatten()
    nodes = np.ascontiguousarray(nodes, dtype=NODE_DTYPE)
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    consts = np.ascontiguousarray(consts, dtype=np.uint32)
    rows = soa.shape[2] if soa.size else 1
    if soa.size == 0:
        soa = np.zeros((max(ts.n_vars, 1), 8, 1), dtype=np.uint32)
    soa = np.ascontiguousarray(soa, dtype=np.uint32)
    out = np.zeros((8, rows), dtype=np.uint32)
    info = np.zeros(16, dtype=np.uint32)
    err = C.create_string_buffer(512)
    r = f(nodes.ctypes.data, offs.ctypes.data, len(ts.tapes), consts.ctypes.data,
          len(ts.pool.values), ts.n_vars, tape, soa.ctypes.data, rows, out.ctypes.data, max_vgpr,
          info.ctypes.data, err, 512)
    if r != 0:
        raise EmuError(r, err.value.decode())
    if not info[0]:
        return JitResult(info, None, err.value.decode())
    vals = [sum(int(out[k, j]) << (32 * k) for k in range(8)) for j in range(rows)]
    return JitResult(info, vals, "")


def set_short_circuit(emu: "Emulator", on: bool) -> None:
    """Options::short_circuit of the emulator's JIT builds (default on, like mh_tapes_jit)."""
    f = _jit_fn(emu.lib, "emu_jit_set_short_circuit", None, [C.c_int])
    f(int(on))


def set_value_numbering(emu: "Emulator", vn: int) -> None:
    """Value numbering of the emulator's lowering: 1 all (default), 2 all but the column loads
    (mh_tapes_jit's last retry under register pressure)."""
    f = _jit_fn(emu.lib, "emu_jit_set_vn", None, [C.c_int])
    f(int(vn))


def jit_module(emu: "Emulator", ts: TapeSet, values: bool = False, max_vgpr: int = 128,
               assemble: bool = True):
    """(module text, code object bytes, tapes jitted) for a whole tape set."""
    f = _jit_fn(emu.lib, "emu_jit_module", C.c_int64,
                [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_uint32,
                 C.c_uint32, C.c_uint32, C.c_int32, C.c_char_p, C.c_uint64,
                 C.POINTER(C.c_uint64), C.POINTER(C.c_uint32), C.c_char_p, C.c_int])
    nodes, offs, consts = ts.flatten()
    nodes = np.ascontiguousarray(nodes, dtype=NODE_DTYPE)
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    consts = np.ascontiguousarray(consts, dtype=np.uint32)
    cap = 64 << 20
    text = C.create_string_buffer(cap)
    hs = C.c_uint64()
    nj = C.c_uint32()
    err = C.create_string_buffer(8192)
    n = f(nodes.ctypes.data, offs.ctypes.data, len(ts.tapes), consts.ctypes.data,
          len(ts.pool.values), ts.n_vars, int(values), max_vgpr, int(assemble), text, cap,
          C.byref(hs), C.byref(nj), err, 8192)
    if n < 0:
        raise EmuError(int(n), err.value.decode())
    return text.value.decode(), int(hs.value), int(nj.value)


def jit_build(emu: "Emulator", ts: TapeSet, max_vgpr: int = 128, threads: int = 4):
    """build_tapeset as mh_tapes_jit runs it: ([(max_vgpr, n_tapes)] per code object, per-tape
    object index or -1)."""
    f = _jit_fn(emu.lib, "emu_jit_build", C.c_int32,
                [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_uint32,
                 C.c_uint32, C.c_uint32, C.c_void_p, C.c_uint32, C.c_void_p, C.c_char_p, C.c_int])
    nodes, offs, consts = ts.flatten()
    nodes = np.ascontiguousarray(nodes, dtype=NODE_DTYPE)
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    consts = np.ascontiguousarray(consts, dtype=np.uint32)
    objs = np.zeros(2 * 256, dtype=np.uint32)
    tape_obj = np.zeros(len(ts.tapes), dtype=np.int32)
    err = C.create_string_buffer(8192)
    n = f(nodes.ctypes.data, offs.ctypes.data, len(ts.tapes), consts.ctypes.data,
          len(ts.pool.values), ts.n_vars, max_vgpr, threads, objs.ctypes.data, 256,
          tape_obj.ctypes.data, err, 8192)
    if n < 0:
        raise EmuError(int(n), err.value.decode())
    return [(int(objs[2 * i]), int(objs[2 * i + 1])) for i in range(min(n, 256))], tape_obj
