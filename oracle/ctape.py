"""ORACLE (test infrastructure only): ctypes wrapper of oracle/tape_eval.c.

Built on first use with gcc (-O3 -fopenmp) into oracle/_build/ (git-ignored, travels to the GPU
box with the tree).  Used by tests/ for larger parity checks and by bench.py's cpu_baseline leg.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "tape_eval.c")
BUILD = os.path.join(HERE, "_build")
LIB = os.path.join(BUILD, "libctape.so")

_lib = None


def build() -> str:
    os.makedirs(BUILD, exist_ok=True)
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        subprocess.run(["gcc", "-O3", "-march=x86-64-v2", "-fopenmp", "-shared", "-fPIC", "-o",
                        LIB, SRC], check=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        _lib = C.CDLL(build())
        _lib.ct_eval.restype = C.c_int
        _lib.ct_eval.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint32, C.c_void_p,
                                 C.c_uint32, C.c_void_p]
        _lib.ct_count.restype = C.c_int
        _lib.ct_count.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32,
                                  C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint64, C.c_int,
                                  C.c_void_p, C.c_void_p]
        _lib.ct_count_lazy.restype = C.c_int
        _lib.ct_count_lazy.argtypes = _lib.ct_count.argtypes
        _lib.ct_max_threads.restype = C.c_int
    return _lib


def _flat(ts):
    nodes, offs, consts = ts.flatten()
    return (np.ascontiguousarray(nodes), np.ascontiguousarray(offs, dtype=np.uint64),
            np.ascontiguousarray(consts, dtype=np.uint32))


def evaluate(ts, tape: int, assignment) -> int:
    nodes = np.ascontiguousarray(ts.tapes[tape].nodes)
    consts = np.ascontiguousarray(ts.pool.to_array())
    a = np.zeros((max(ts.n_vars, 1), 8), dtype=np.uint32)
    for v, x in enumerate(assignment):
        for k in range(8):
            a[v, k] = (x >> (32 * k)) & 0xFFFFFFFF
    out = np.zeros(34, dtype=np.uint32)
    r = lib().ct_eval(nodes.ctypes.data, len(nodes), consts.ctypes.data, len(ts.pool.values),
                      a.ctypes.data, ts.n_vars, out.ctypes.data)
    if r != 0:
        raise ValueError("malformed tape")
    return sum(int(out[k]) << (32 * k) for k in range(34))


def count(ts, seed: int, row_first: int, rows: int, threads: int = 0, tapes=None,
          short_circuit: bool = False):
    """(hit_count[u64], first_hit[u64]) over generated rows, for tapes[:n] (default all).
    short_circuit: evaluate a Bool AND's second operand only when the first holds
    (ct_count_lazy; same results, less work)."""
    nodes, offs, consts = _flat(ts)
    n = len(ts.tapes) if tapes is None else tapes
    cnt = np.zeros(max(n, 1), dtype=np.uint64)
    first = np.zeros(max(n, 1), dtype=np.uint64)
    th = threads or lib().ct_max_threads()
    fn = lib().ct_count_lazy if short_circuit else lib().ct_count
    r = fn(nodes.ctypes.data, offs.ctypes.data, n, consts.ctypes.data,
                       len(ts.pool.values), ts.n_vars, seed, row_first, rows, th,
                       cnt.ctypes.data, first.ctypes.data)
    if r != 0:
        raise ValueError("malformed tape")
    return cnt[:n], first[:n]


def benchmark(ts, seed: int, seconds: float = 15.0, tapes: int = 100,
              short_circuit: bool = True, threads: int = 0):
    """Evals/s of this port on the host cores, on a bounded sample of the bench workload:
    the first `tapes` tapes over generated rows, rows grown until ~`seconds` of work.
    short_circuit: the lazy evaluator (the scalar counterpart of the device's short circuit).
    threads: 0 = every host thread OpenMP offers, 1 = the single-core figure."""
    th = threads or lib().ct_max_threads()
    tapes = min(tapes, len(ts.tapes))
    rows = 256
    while True:
        t0 = time.perf_counter()
        count(ts, seed, 0, rows, th, tapes, short_circuit=short_circuit)
        dt = time.perf_counter() - t0
        if dt >= seconds * 0.5 or rows >= 1 << 26:
            break
        rows = int(rows * min(64.0, max(2.0, seconds * 0.6 / max(dt, 1e-3))))
    return {
        "value": tapes * rows / dt,
        "unit": "evals/s",
        "cores": th,
        "kind": "port",
        "sample": "oracle/tape_eval.c (OpenMP, %d threads%s): first %d synthetic tapes x %d "
                  "generated rows, %.1f s" % (th, ", short-circuit ANDs" if short_circuit else "",
                                             tapes, rows, dt),
    }


def eval_pairs(ts, seed: int, tapes, rows):
    """[bool]: tape tapes[i] evaluated (C oracle) on generated row rows[i] — re-checks witness
    indices reported by the device."""
    from . import smt_eval

    out = []
    for t, r in zip(tapes, rows):
        out.append(evaluate(ts, int(t), smt_eval.gen_assignment(seed, ts.n_vars, int(r))) != 0)
    return out
