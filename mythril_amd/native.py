"""ctypes binding of libmythril_hip (include/mythril_hip.h).

The reference reaches its native solver (z3) in-process through ctypes as well
(z3-solver's ``z3core``); this module is the analogous binding for the sieve.  The
library is loaded from the package directory (built in-tree by ``__graft_entry__.build()``
or ``make -C mythril_amd/csrc``); a missing library raises ``NativeUnavailable`` — there is
no CPU fallback on the product path.

One HIP runtime per process: torch ships its own ``libamdhip64`` (same SONAME as ROCm's).  A
process that also uses torch on the GPU (bench.py, the GPU tests) imports torch and initialises
CUDA before this library loads, so both bind to torch's copy; the library's RCCL (mh_comm_*) is
ROCm's, opened with RTLD_DEEPBIND and bound to that same runtime.
"""
from __future__ import annotations

import ctypes as C
import os
from itertools import chain
from typing import List, Optional, Sequence, Tuple

import numpy as np

from .tape import NODE_DTYPE, TapeSet

LIB_NAME = "libmythril_hip.so"
LIB_PATH = os.environ.get("MYTHRIL_HIP_LIB") or os.path.join(
    os.path.dirname(os.path.abspath(__file__)), LIB_NAME)

MH_OK = 0
MH_E_INVALID = -1
MH_E_UNSUPPORTED = -2
MH_E_DEVICE = -3
MH_E_NOMEM = -4
MH_E_NODEVICE = -5

MODE_FIRST_HIT = 0
MODE_COUNT_ALL = 1
NO_HIT = 0xFFFFFFFFFFFFFFFF

# every symbol include/mythril_hip.h declares: name -> (restype, argtypes)
_u32p = C.POINTER(C.c_uint32)
_u64p = C.POINTER(C.c_uint64)
_vp = C.c_void_p
SIGNATURES = {
    "mh_version": (C.c_int32, [_u32p, _u32p, _u32p]),
    "mh_last_error": (C.c_char_p, []),
    "mh_device_count": (C.c_int32, [C.POINTER(C.c_int32)]),
    "mh_ctx_create": (C.c_int32, [C.c_int32, C.POINTER(_vp)]),
    "mh_ctx_destroy": (C.c_int32, [_vp]),
    "mh_ctx_set_stream": (C.c_int32, [_vp, _vp]),
    "mh_ctx_synchronize": (C.c_int32, [_vp]),
    "mh_ctx_clear_cache": (C.c_int32, [_vp]),
    "mh_tapes_compile": (C.c_int32, [_vp, _vp, _u64p, C.c_uint32, _u32p, C.c_uint32, C.c_uint32,
                                     C.POINTER(_vp)]),
    "mh_tapes_compile_async": (C.c_int32, [_vp, _vp, _u64p, C.c_uint32, _u32p, C.c_uint32,
                                           C.c_uint32]),
    "mh_tapes_compile_wait": (C.c_int32, [_vp, C.POINTER(C.c_void_p), C.POINTER(C.c_double)]),
    "mh_tapes_destroy": (C.c_int32, [_vp]),
    "mh_tapes_info": (C.c_int32, [_vp, _vp, C.c_uint32]),
    "mh_assign_create": (C.c_int32, [_vp, C.c_uint32, C.c_uint64, C.POINTER(_vp)]),
    "mh_assign_destroy": (C.c_int32, [_vp]),
    "mh_assign_upload": (C.c_int32, [_vp, _u32p, C.c_uint64, C.c_uint64]),
    "mh_assign_download": (C.c_int32, [_vp, _u32p, C.c_uint64, C.c_uint64]),
    "mh_assign_generate": (C.c_int32, [_vp, C.c_uint64, C.c_uint64]),
    "mh_gen_limb": (C.c_uint32, [C.c_uint64, C.c_uint32, C.c_uint64, C.c_uint32]),
    "mh_assign_generate_guided": (C.c_int32, [_vp, C.c_uint64, C.c_uint64, C.c_uint64,
                                              C.c_uint64, _vp]),
    "mh_results_reset": (C.c_int32, [_vp, _vp, _vp, C.c_uint32]),
    "mh_run": (C.c_int32, [_vp, _vp, C.c_uint32, C.c_uint32, _vp, C.c_uint64, C.c_uint64,
                           C.c_uint64, C.c_uint32, _u64p, _u64p]),
    "mh_run_rows": (C.c_int32, [_vp, _vp, C.c_uint32, C.c_uint32, _vp, C.c_uint64, C.c_uint64,
                                C.c_uint64, C.c_uint32, _u64p, _u64p, C.c_uint32, _u32p]),
    "mh_query_round": (C.c_int32, [_vp, _vp, _vp, _vp, C.c_uint64, C.c_uint64, C.c_uint64,
                                   C.c_uint32, C.c_uint32, C.c_uint32, _u64p, _u64p, C.c_uint32,
                                   _u32p]),
    "mh_run_async": (C.c_int32, [_vp, _vp, C.c_uint32, C.c_uint32, _vp, C.c_uint64, C.c_uint64,
                                 C.c_uint64, C.c_uint32, _vp, _vp]),
    "mh_eval_values": (C.c_int32, [_vp, _vp, C.c_uint32, _vp, C.c_uint64, C.c_uint64, _u32p]),
    "mh_microbench_valu": (C.c_int32, [_vp, C.c_uint32, C.POINTER(C.c_double)]),
    "mh_microbench_issue": (C.c_int32, [_vp, C.c_uint32, C.c_uint32, C.POINTER(C.c_double)]),
    "mh_microbench_gather": (C.c_int32, [C.c_int32, C.c_uint32, C.c_uint32, C.c_uint32,
                                         C.c_uint32, C.POINTER(C.c_double),
                                         C.POINTER(C.c_double), _u64p]),
    "mh_eval_values_many": (C.c_int32, [_vp, _vp, _u32p, C.c_uint32, _vp, C.c_uint64, _u32p]),
    "mh_ctx_eval_launches": (C.c_int32, [_vp, _u64p]),
    "mh_tapes_jit": (C.c_int32, [_vp, C.c_uint32, C.c_uint32]),
    "mh_tapes_jit_info": (C.c_int32, [_vp, _vp]),
    "mh_tapes_jit_code_id": (C.c_int32, [_vp, _u64p]),
    "mh_jit_code_id": (C.c_int32, [_vp, _u64p, C.c_uint32, _u32p, C.c_uint32, C.c_uint32,
                                   C.c_uint32, C.c_uint32, _u64p]),
    "mh_tapes_jitted": (C.c_int32, [_vp, C.POINTER(C.c_uint8), C.c_uint32]),
    "mh_jit_eval_all": (C.c_int32, [_vp, _vp, _vp, C.c_uint64, C.c_uint64, _u32p]),
    "mh_comm_unique_id": (C.c_int32, [_vp]),
    "mh_comm_init": (C.c_int32, [_vp, _vp, C.c_int32, C.c_int32]),
    "mh_comm_allreduce_results": (C.c_int32, [_vp, _vp, _vp, C.c_uint32]),
    "mh_comm_destroy": (C.c_int32, [_vp]),
    "mh_ctx_enable_timing": (C.c_int32, [_vp, C.c_int32]),
    "mh_ctx_kernel_time": (C.c_int32, [_vp, C.POINTER(C.c_double), _u64p]),
    "mh_guide_harvest": (C.c_int32, [_vp, C.c_uint32, _u32p, C.c_uint32, C.POINTER(C.c_uint16),
                                     C.c_uint32, _u32p, _u32p, C.c_uint32, C.POINTER(_vp), _vp]),
    "mh_guide_harvest_inc": (C.c_int32, [_vp, C.c_uint32, _u32p, C.c_uint32,
                                         C.POINTER(C.c_uint16), C.c_uint32, _u32p, _u32p,
                                         C.c_uint32, C.POINTER(_vp), _vp]),
    "mh_harvest_free": (C.c_int32, [_vp]),
    "mh_harvester_create": (C.c_int32, [C.POINTER(_vp)]),
    "mh_harvester_destroy": (C.c_int32, [_vp]),
    "mh_harvester_stats": (C.c_int32, [_vp, _u64p]),
    "mh_guide_harvest_with": (C.c_int32, [_vp, _vp, C.c_uint32, _u32p, C.c_uint32,
                                          C.POINTER(C.c_uint16), C.c_uint32, _u32p, _u32p,
                                          C.c_uint32, C.POINTER(_vp), _vp]),
    "mh_smtlib_create": (C.c_int32, [C.POINTER(_vp)]),
    "mh_smtlib_destroy": (C.c_int32, [_vp]),
    "mh_smtlib_read": (C.c_int32, [_vp, C.c_char_p, C.c_uint64, _vp]),
    "mh_smtlib_commit": (C.c_int32, [_vp, C.POINTER(C.c_int64), C.c_uint64]),
    "mh_smtlib_rollback": (C.c_int32, [_vp]),
    "mh_smtlib_size": (C.c_uint64, [_vp]),
    "mh_terms_create": (C.c_int32, [C.POINTER(_vp)]),
    "mh_terms_destroy": (C.c_int32, [_vp]),
    "mh_terms_set_options": (C.c_int32, [_vp, C.c_uint32]),
    "mh_terms_append": (C.c_int32, [_vp, _vp, C.c_uint64, _u32p, C.c_uint64, C.c_char_p,
                                    C.c_uint64, C.c_char_p, C.c_uint64, C.c_char_p, C.c_uint64]),
    "mh_terms_sizes": (C.c_int32, [_vp, _u64p]),
    "mh_query_build": (C.c_int32, [_vp, _u32p, C.c_uint32, C.POINTER(_vp), _vp]),
    "mh_query_free": (C.c_int32, [_vp]),
}

# mh_smt_record / mh_smt_result (include/mythril_hip.h)
SMT_RECORD_DTYPE = np.dtype([("op", "u1"), ("pad0", "u1"), ("pad1", "<u2"), ("width", "<u4"),
                             ("a", "<i8"), ("b", "<i8"), ("c", "<i8"), ("imm0", "<u4"),
                             ("imm1", "<u4"), ("name_off", "<u4"), ("name_len", "<u4"),
                             ("const_off", "<u4"), ("pad2", "<u4")])
SMT_RESULT_DTYPE = np.dtype([("kind", "<u4"), ("pad", "<u4"), ("node", "<i8")])
assert SMT_RECORD_DTYPE.itemsize == 56 and SMT_RESULT_DTYPE.itemsize == 16
SMT_ASSERT, SMT_MINIMIZE, SMT_MAXIMIZE = 0, 1, 2


class SmtBatch(C.Structure):
    _fields_ = [("records", _vp), ("n_records", C.c_uint64), ("const_limbs", _vp),
                ("names", _vp), ("results", _vp), ("n_results", C.c_uint64)]


# mh_microbench_issue kinds (include/mythril_hip.h)
MB_KINDS = ("add_co_chain", "mad_u64_u32", "add_u32", "xor_b32", "alignbit_b32", "cndmask_b32",
            "or3_b32", "readlane_b32", "mov_b32", "add_co_nocarryin", "sub_co_vcc_chain",
            "cndmask_e32_vcc", "cmp_eq_e32", "xor_literal", "lshlrev_b32", "add3_u32", "fma_f64",
            "xnor_b32", "and_b32", "or_b32", "not_b32", "xor_exec32", "alignbit_exec32",
            "xor_exec16", "xor_exec_alt", "dep_mad_u64_u32", "dep_add_u32", "dep_addc_vcc",
            "dep_mad_2chains", "dep_mad_carry", "dep_cmp_cndmask", "mix_mad_add", "mix_addc_xor",
            "mix_mad2_add2", "bitop3_b32", "mix_bitop3_alignbit", "cmp_lt_u64", "cmp_eq_u64",
            "lshl_add_u64", "mul_lo_u32", "mul_hi_u32", "mul_u32_u24", "sub_co_e64_sgpr",
            "cmp_lt_u32_e64", "lt256_via_u64")


class NativeUnavailable(RuntimeError):
    """libmythril_hip.so is missing or cannot be loaded."""


class SieveError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__("mythril_hip error %d: %s" % (code, msg))
        self.code = code


class Unsupported(SieveError):
    """The tape uses something the device path does not cover: fall back to z3."""


class TapeInfo(C.Structure):
    _fields_ = [
        ("n_nodes", C.c_uint32),
        ("n_insns", C.c_uint32),
        ("n_regs", C.c_uint32),
        ("features", C.c_uint32),
        ("alg_ops", C.c_uint64),
    ]


class JitInfo(C.Structure):
    """mh_jit_info (include/mythril_hip.h)."""

    _fields_ = [
        ("n_jitted", C.c_uint32),
        ("n_groups", C.c_uint32),
        ("n_modules", C.c_uint32),
        ("max_vgpr", C.c_uint32),
        ("code_bytes", C.c_uint64),
        ("valu_static", C.c_uint64),
        ("valu_wide_static", C.c_uint64),
        ("build_ms", C.c_double),
    ]


JIT_VALUES = 1
JIT_FULL_EVAL = 2


class Guide(C.Structure):
    """mh_guide (include/mythril_hip.h)."""

    _fields_ = [
        ("n_cols", C.c_uint32),
        ("col_width", C.POINTER(C.c_uint16)),
        ("pool_off", _u32p),
        ("pool", _u32p),
        ("n_sets", C.c_uint32),
        ("set_prob", C.POINTER(C.c_uint8)),
        ("set_off", _u32p),
        ("alt_off", _u32p),
        ("entry_col", _u32p),
        ("entry_val", _u32p),
    ]


_lib: Optional[C.CDLL] = None


def _limb_rows(vals) -> np.ndarray:
    """[n, 8] u32 limbs of 256-bit values."""
    buf = b"".join((int(v) & ((1 << 256) - 1)).to_bytes(32, "little") for v in vals)
    return np.frombuffer(buf, dtype="<u4").reshape(-1, 8).copy()


def _guide_arrays(g: "Guide") -> dict:
    """The arrays of an mh_guide the library owns, copied (one memcpy each)."""
    def arr(p, n, dt=np.uint32):
        dt = np.dtype(dt)
        return np.frombuffer(C.string_at(C.cast(p, C.c_void_p), n * dt.itemsize), dtype=dt)

    n_cols, n_sets = g.n_cols, g.n_sets
    pool_off = arr(g.pool_off, n_cols + 1)
    set_off = arr(g.set_off, n_sets + 1)
    alt_off = arr(g.alt_off, int(set_off[-1]) + 1)
    n_entries = max(int(alt_off[-1]), 1)
    return dict(
        width=arr(g.col_width, n_cols, np.uint16), pool_off=pool_off,
        pool=arr(g.pool, 8 * max(int(pool_off[-1]), 1)).reshape(-1, 8), set_off=set_off,
        set_prob=arr(g.set_prob, max(n_sets, 1), np.uint8), alt_off=alt_off,
        entry_col=arr(g.entry_col, n_entries), entry_val=arr(g.entry_val, 8 * n_entries).reshape(-1, 8))


class GuideHandle:
    """A harvested guide left in the library (mh_harvest): query_round hands its mh_guide to the
    generator as it is; arrays() copies it out (tests, the CPU stand-in of the device)."""

    def __init__(self, lib, h: C.c_void_p, g: "Guide"):
        self.lib, self.h, self.guide = lib, h, g

    def arrays(self) -> dict:
        return _guide_arrays(self.guide)

    def close(self) -> None:
        if self.h:
            self.lib.mh_harvest_free(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


def harvest_guide(nodes: np.ndarray, consts: np.ndarray, widths: Sequence[int],
                  parent: Sequence[Tuple[int, int]] = (), session: "Optional[GuideSession]" = None,
                  keep: bool = False, parent_eval: bool = False):
    """mh_guide_harvest: the guide of one lowered query tape (root last, VAR imm0 = column,
    CONST imm0 = row of `consts`), as the arrays candidates.Guide.arrays() gives -- the same
    values (tests/test_harvest.py).  `parent` = the parent witness as (column, value) pairs in
    the witness's order.  With `session` (a GuideSession) the harvest reuses the session's memo
    when the tape extends the last one (mh_guide_harvest_with; the same arrays).  keep=True
    returns a GuideHandle instead (the guide stays in the library for query_round).  Host-only:
    no device is touched."""
    lib = load()
    nodes = np.ascontiguousarray(nodes, dtype=NODE_DTYPE)
    consts = np.ascontiguousarray(consts, dtype=np.uint32).reshape(-1, 8)
    w = np.ascontiguousarray(widths, dtype=np.uint16)
    pc = np.ascontiguousarray([c for c, _ in parent], dtype=np.uint32)
    pv = _limb_rows([v for _, v in parent]) if len(parent) else np.zeros((1, 8), np.uint32)
    h = C.c_void_p()
    g = Guide()
    args = (nodes.ctypes.data, len(nodes), _ptr(consts), len(consts),
            w.ctypes.data_as(C.POINTER(C.c_uint16)), len(w), _ptr(pc), _ptr(pv), len(pc),
            C.byref(h), C.byref(g))
    if parent_eval:  # mh_guide_harvest_inc: operands the parent fixes count as known
        if session is not None:
            raise ValueError("parent_eval harvests are stateless")
        _check(lib.mh_guide_harvest_inc(*args))
    elif session is None:
        _check(lib.mh_guide_harvest(*args))
    else:
        _check(lib.mh_guide_harvest_with(session.h, *args))
    handle = GuideHandle(lib, h, g)
    if keep:
        return handle
    try:
        return handle.arrays()
    finally:
        handle.close()


class GuideSession:
    """An mh_harvester: guide harvests that reuse the memo of the path's earlier queries."""

    def __init__(self):
        self.lib = load()
        h = C.c_void_p()
        _check(self.lib.mh_harvester_create(C.byref(h)))
        self.h = h

    def stats(self) -> Tuple[int, int, int]:
        """(harvests that extended the last tape, harvests that started afresh, arena bytes)."""
        out = (C.c_uint64 * 3)()
        _check(self.lib.mh_harvester_stats(self.h, out))
        return int(out[0]), int(out[1]), int(out[2])

    def close(self) -> None:
        if self.h:
            self.lib.mh_harvester_destroy(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:
            pass


class SmtlibSession:
    """An SMT-LIB reader session (mh_smtlib): reads z3-printed text into a term builder,
    handing over only the nodes the builder does not have yet (include/mythril_hip.h)."""

    def __init__(self):
        self.lib = load()
        h = C.c_void_p()
        _check(self.lib.mh_smtlib_create(C.byref(h)))
        self.h = h

    def close(self) -> None:
        if self.h:
            self.lib.mh_smtlib_destroy(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:
            pass

    def size(self) -> int:
        return int(self.lib.mh_smtlib_size(self.h))

    def read(self, text: str, b) -> List[Tuple[int, int]]:
        """Parse `text` into builder `b`; [(SMT_ASSERT / MINIMIZE / MAXIMIZE, node)]."""
        data = text.encode()
        batch = SmtBatch()
        _check(self.lib.mh_smtlib_read(self.h, data, len(data), C.byref(batch)))
        n = int(batch.n_records)
        ids: List[int] = []
        if n:
            try:
                ids = self._merge(batch, n, b)
            except Exception:
                self.lib.mh_smtlib_rollback(self.h)
                raise
            arr = (C.c_int64 * n)(*ids)
            _check(self.lib.mh_smtlib_commit(self.h, arr, n))
        out = []
        nr = int(batch.n_results)
        if nr:
            res = np.frombuffer((C.c_char * (nr * 16)).from_address(batch.results),
                                dtype=SMT_RESULT_DTYPE)
            for kind, _, node in res.tolist():
                out.append((kind, node if node >= 0 else ids[-node - 1]))
        return out

    @staticmethod
    def _merge(batch, n: int, b) -> List[int]:
        """Build the batch's records in builder `b` (TapeBuilder._add's bookkeeping inlined for
        the plain ops: the reader checked their sorts with TapeBuilder.op's rules)."""
        from .tape import ARITY, F_HOST

        recs = np.frombuffer((C.c_char * (n * 56)).from_address(batch.records),
                             dtype=SMT_RECORD_DTYPE).tolist()
        nl = max((r[9] + r[10] for r in recs), default=0)
        names = C.string_at(batch.names, nl).decode() if nl else ""
        nc = max((r[11] + 8 for r in recs if r[0] == 0), default=0)
        cbuf = C.string_at(batch.const_limbs, 4 * nc) if nc else b""
        arity = _ARITY_BY_INT or _arity_table(ARITY)
        from .tape import NODE_PACK

        memo, nodes, widths, flags, packed = b._memo, b.nodes, b.widths, b.flags, b.node_bytes
        ids = [0] * n
        for k, (op, _, _, w, a, bb, c, i0, i1, noff, nlen, coff, _) in enumerate(recs):
            if a < 0:
                a = ids[-a - 1]
            if bb < 0:
                bb = ids[-bb - 1]
            if c < 0:
                c = ids[-c - 1]
            if 2 <= op < 80:  # plain ops (TRUE / FALSE included): TapeBuilder._add
                key = (op, w, a, bb, c, i0, i1)
                h = memo.get(key)
                if h is None:
                    ar = arity[op]
                    if op == 30 and widths[a] > 256:
                        f = F_HOST
                    elif ar:
                        f = (flags[a] | (flags[bb] if ar > 1 else 0)
                             | (flags[c] if ar > 2 else 0)) & F_HOST
                    else:
                        f = 0
                    h = len(nodes)
                    nodes.append(key)
                    widths.append(w)
                    flags.append(f)
                    packed += NODE_PACK(op, f, w, a, bb, c, i0, i1)
                    memo[key] = h
            elif op == 0:  # CONST (<= 256 bits; wider ones arrive as CONCATs)
                h = b.const(int.from_bytes(cbuf[4 * coff:4 * coff + 32], "little"), w)
            elif op == 1:
                h = b.user_var(names[noff:noff + nlen], w)
            elif op == 80:
                h = b.array(names[noff:noff + nlen], i1, w)
            elif op == 81:
                h = b.const_array(i1, a)
            elif op == 82:
                h = b.store(a, bb, c)
            elif op == 83:
                h = b.select(a, bb)
            else:
                h = b.apply(names[noff:noff + nlen], i1, w, a)
            ids[k] = h
        return ids


# mh_query_column / mh_query_table (include/mythril_hip.h)
QUERY_COLUMN_DTYPE = np.dtype([("name_off", "<u4"), ("name_len", "<u4"), ("symbol_off", "<u4"),
                               ("symbol_len", "<u4"), ("width", "<u4"), ("kind", "<u4"),
                               ("key_off", "<u4"), ("pad", "<u4")])
QUERY_TABLE_DTYPE = np.dtype([("kind", "<u4"), ("name_off", "<u4"), ("name_len", "<u4"),
                              ("limb_off", "<u4"), ("n_items", "<u4"), ("pad", "<u4")])
assert QUERY_COLUMN_DTYPE.itemsize == 32 and QUERY_TABLE_DTYPE.itemsize == 24
COLUMN_KINDS = ("var", "cell", "else", "ufcell", "ufelse", "read", "ufread", "kread")  # MH_COL_*
TERMS_KECCAK_READS = 1  # mh_terms_set_options
TABLE_CELLS, TABLE_UF_CELLS, TABLE_KECCAK = 0, 1, 2
QUERY_DEFINITIONS = 1
QUERY_REFUTED = 2
QUERY_INCREMENTAL = 4  # diagnostic: built from the session's state, not afresh
QUERY_KEY_LIMBS = 36


class QueryInfo(C.Structure):
    """mh_query_info (include/mythril_hip.h)."""

    _fields_ = [("nodes", _vp), ("tape_off", _u64p), ("consts", _u32p), ("columns", _vp),
                ("names", _vp), ("key_limbs", _u32p), ("group_cols", _u32p),
                ("group_off", _u32p), ("tables", _vp), ("table_limbs", _u32p),
                ("n_tapes", C.c_uint32), ("n_consts", C.c_uint32), ("n_columns", C.c_uint32),
                ("names_len", C.c_uint32), ("n_groups", C.c_uint32), ("n_tables", C.c_uint32),
                ("flags", C.c_uint32), ("n_keys", C.c_uint32), ("n_table_entries", C.c_uint32),
                ("n_defs", C.c_uint32), ("def_cols", _u32p), ("parent_len", C.c_uint32),
                ("root_ends", _u32p), ("n_root_ends", C.c_uint32)]


class CompiledQuery:
    """What mh_query_build returns, copied out of the library: the tapes (tape 0 the root; with
    several groups, tapes 1.. the groups'), the query constants, the column names and widths,
    each group's column indices and the flags; ``columns`` [(name, width, kind, symbol, key)] and
    ``tables`` [(kind, name, items)] are decoded on first use (a witness's schema is read only
    when a model is evaluated, mythril/laser/smt/model.py:45-59)."""

    __slots__ = ("tapes", "consts", "names", "widths", "groups", "flags", "nodes", "tape_off",
                 "defs", "def_tapes", "parent_len", "root_ends", "_raw", "_columns", "_tables")

    def __init__(self, info: QueryInfo):
        def raw(p, nbytes):
            return C.string_at(p, nbytes) if nbytes else b""

        nd = info.n_defs
        nt = info.n_tapes - nd  # the root and group tapes; the definitions' tapes follow
        off = np.frombuffer(raw(info.tape_off, 8 * (info.n_tapes + 1)),
                            dtype=np.uint64).tolist()
        nodes = np.frombuffer(raw(info.nodes, 24 * off[-1]), dtype=NODE_DTYPE)
        self.nodes, self.tape_off = nodes, off[:nt + 1]  # root and group tapes back to back
        self.tapes = [nodes[off[i]:off[i + 1]] for i in range(nt)]
        # MH_QUERY_DEFINITIONS: column index of each defined symbol, and the tape of its term
        self.defs = np.frombuffer(raw(info.def_cols, 4 * nd), dtype=np.uint32).tolist()
        self.def_tapes = [nodes[off[nt + i]:off[nt + i + 1]] for i in range(nd)]
        self.consts = np.frombuffer(raw(info.consts, 32 * info.n_consts),
                                    dtype=np.uint32).reshape(-1, 8)
        names = raw(info.names, info.names_len).decode()
        cols = np.frombuffer(raw(info.columns, 32 * info.n_columns), dtype=QUERY_COLUMN_DTYPE)
        no, nl = cols["name_off"].tolist(), cols["name_len"].tolist()
        self.names = [names[o:o + n] for o, n in zip(no, nl)]
        self.widths = cols["width"]
        ng = info.n_groups
        goff = np.frombuffer(raw(info.group_off, 4 * (ng + 1)), dtype=np.uint32).tolist()
        gcols = np.frombuffer(raw(info.group_cols, 4 * goff[-1]), dtype=np.uint32).tolist()
        self.groups = [gcols[goff[g]:goff[g + 1]] for g in range(ng)]
        self.flags = int(info.flags)
        self.parent_len = int(info.parent_len)  # root-tape nodes of the query minus its last root
        # root_ends[d - 1]: root-tape nodes of the query's first d roots
        self.root_ends = np.frombuffer(raw(info.root_ends, 4 * info.n_root_ends),
                                       dtype=np.uint32).tolist()
        kb = 4 * QUERY_KEY_LIMBS
        self._raw = (names, cols, raw(info.key_limbs, kb * info.n_keys),
                     raw(info.tables, 24 * info.n_tables),
                     raw(info.table_limbs, kb * info.n_table_entries))
        self._columns = self._tables = None

    @staticmethod
    def _ints(data: bytes) -> List[int]:
        k = 4 * QUERY_KEY_LIMBS
        return [int.from_bytes(data[i:i + k], "little") for i in range(0, len(data), k)]

    @property
    def columns(self) -> List[tuple]:
        if self._columns is None:
            names, cols, key_limbs, _, _ = self._raw
            keys = self._ints(key_limbs)
            self._columns = [(names[no:no + nl], w, COLUMN_KINDS[k], names[so:so + sl],
                              None if ko == 0xFFFFFFFF else keys[ko])
                             for no, nl, so, sl, w, k, ko, _ in cols.tolist()]
        return self._columns

    @property
    def tables(self) -> List[tuple]:
        if self._tables is None:
            names, _, _, tabs, limbs = self._raw
            vals = self._ints(limbs)
            self._tables = [
                (k, names[no:no + nl], vals[lo:lo + (2 * n + 1 if k == TABLE_KECCAK else n)])
                for k, no, nl, lo, n, _ in np.frombuffer(tabs, dtype=QUERY_TABLE_DTYPE).tolist()]
        return self._tables


def _ints(rows: np.ndarray) -> List[int]:
    """[n, k] u32 limbs -> n ints."""
    rows = np.ascontiguousarray(rows, dtype="<u4")
    data, k = rows.tobytes(), 4 * rows.shape[1]
    return [int.from_bytes(data[k * i:k * i + k], "little") for i in range(len(rows))]


class TermMirror:
    """An mh_terms session mirroring one TapeBuilder (tape.py): each sync hands the library the
    nodes, constants and names the builder made since the last one; build() compiles a query
    (mh_query_build).  One per builder and lowering mode, kept on it (``TermMirror.of``);
    ``keccak_reads``: keccak applications as read columns (MH_TERMS_KECCAK_READS, lower_query's
    keyword of that name)."""

    def __init__(self, keccak_reads: bool = False):
        import threading

        self.lib = load()
        h = C.c_void_p()
        _check(self.lib.mh_terms_create(C.byref(h)))
        self.h = h
        self.keccak_reads = keccak_reads
        if keccak_reads:
            _check(self.lib.mh_terms_set_options(h, TERMS_KECCAK_READS))
        self.n = [0, 0, 0, 0, 0]  # nodes, constants, variables, arrays, functions sent
        # one session per builder, used by one thread at a time (query.cpp keeps scratch and the
        # last query's state on it): sieves of several threads over one builder take turns
        self.lock = threading.Lock()

    @classmethod
    def of(cls, b, keccak_reads: bool = False) -> "TermMirror":
        attr = "_term_mirror_kr" if keccak_reads else "_term_mirror"
        m = b.__dict__.get(attr)
        if m is None:  # setdefault: two threads racing here end up with the same session
            m = b.__dict__.setdefault(attr, cls(keccak_reads))
        return m

    def close(self) -> None:
        if self.h:
            self.lib.mh_terms_destroy(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:
            pass

    def sync(self, b) -> None:
        n0, c0, v0, a0, f0 = self.n
        n1 = len(b.nodes)
        pool = b.pool
        c1 = len(pool.values)
        v1 = len(b.var_index)
        sym = b.symbols
        a1, f1 = len(sym.array_names), len(sym.function_names)
        if [n1, c1, v1, a1, f1] == self.n:
            return
        if n1 > n0:
            k = n1 - n0
            packed = getattr(b, "node_bytes", None)
            if packed is not None and len(packed) == 24 * n1:
                # the builder's packed mh_node records (the slice is a copy: nothing of the
                # builder's stays exported)
                nodes = np.frombuffer(bytes(packed[24 * n0:24 * n1]), dtype=NODE_DTYPE)
            else:
                rows = np.fromiter(chain.from_iterable(b.nodes[n0:n1]), np.int64, 7 * k).reshape(k, 7)
                nodes = np.empty(k, dtype=NODE_DTYPE)
                nodes["op"] = rows[:, 0]
                nodes["flags"] = np.fromiter(b.flags[n0:n1], np.uint8, k)
                nodes["width"] = rows[:, 1]
                for j, f in enumerate(("a", "b", "c", "imm0", "imm1")):
                    nodes[f] = rows[:, 2 + j]
        else:
            nodes = np.zeros(1, dtype=NODE_DTYPE)
        consts = (np.ascontiguousarray(pool.to_array()[c0:c1]) if c1 > c0
                  else np.zeros((1, 8), dtype=np.uint32))

        def names(seq) -> bytes:
            return b"".join(s.encode() + b"\0" for s in seq)

        vn = names(list(b.var_index)[v0:v1]) if v1 > v0 else b""
        an = names(sym.array_names[a0:a1]) if a1 > a0 else b""
        fn = names(sym.function_names[f0:f1]) if f1 > f0 else b""
        _check(self.lib.mh_terms_append(self.h, nodes.ctypes.data, n1 - n0, _ptr(consts), c1 - c0,
                                        vn, v1 - v0, an, a1 - a0, fn, f1 - f0))
        self.n = [n1, c1, v1, a1, f1]

    def build(self, b, roots: Sequence[int]) -> CompiledQuery:
        """mh_query_build of the conjunction of `roots` (after a sync with `b`)."""
        r = np.ascontiguousarray(roots, dtype=np.uint32)
        with self.lock:
            self.sync(b)
            h = C.c_void_p()
            info = QueryInfo()
            _check(self.lib.mh_query_build(self.h, _ptr(r), len(r), C.byref(h), C.byref(info)))
            try:
                return CompiledQuery(info)
            finally:
                self.lib.mh_query_free(h)


_ARITY_BY_INT: List[int] = []


def _arity_table(arity) -> List[int]:
    _ARITY_BY_INT[:] = [arity.get(o, 2) for o in range(256)]
    return _ARITY_BY_INT


def load(path: str = LIB_PATH) -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise NativeUnavailable(
            "%s not built; run `python -c 'import __graft_entry__ as g; g.build()'`" % path)
    try:
        lib = C.CDLL(path)
    except OSError as e:  # pragma: no cover - depends on the ROCm runtime
        raise NativeUnavailable("cannot load %s: %s" % (path, e)) from e
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _check(code: int) -> None:
    if code != MH_OK:
        msg = load().mh_last_error().decode(errors="replace")
        if code == MH_E_UNSUPPORTED:
            raise Unsupported(code, msg)
        raise SieveError(code, msg)


def _ptr(a: np.ndarray, t=C.c_uint32):
    return a.ctypes.data_as(C.POINTER(t))


def version() -> Tuple[int, int, int]:
    a, b, c = C.c_uint32(), C.c_uint32(), C.c_uint32()
    _check(load().mh_version(C.byref(a), C.byref(b), C.byref(c)))
    return a.value, b.value, c.value


def device_count() -> int:
    n = C.c_int32()
    _check(load().mh_device_count(C.byref(n)))
    return n.value


COMM_ID_BYTES = 128


def comm_unique_id() -> bytes:
    """A fresh RCCL unique id (rank 0 creates it; every rank passes it to Context.comm_init)."""
    buf = (C.c_uint8 * COMM_ID_BYTES)()
    _check(load().mh_comm_unique_id(C.cast(buf, C.c_void_p)))
    return bytes(buf)


_CODE_IDS = {}


def jit_code_id(tapeset: TapeSet, short_circuit: bool = True, max_vgpr: int = 0) -> str:
    """Identifier of the native code mh_tapes_jit would build for `tapeset` (mh_jit_code_id):
    a hash of the emitted module texts, computed on the host without a device or the assembler.
    Equal to CompiledTapes.code_id() after CompiledTapes.jit() with the same options."""
    nodes, offs, consts = tapeset.flatten()
    nodes = np.ascontiguousarray(nodes, dtype=NODE_DTYPE)
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    consts = np.ascontiguousarray(consts, dtype=np.uint32)
    out = C.c_uint64()
    _check(load().mh_jit_code_id(nodes.ctypes.data_as(C.c_void_p), _ptr(offs, C.c_uint64),
                                 len(tapeset.tapes), _ptr(consts), len(tapeset.pool.values),
                                 tapeset.n_vars, 0 if short_circuit else JIT_FULL_EVAL, max_vgpr,
                                 C.byref(out)))
    return "%016x" % out.value


def _elf_section(path: str, name: bytes) -> bytes:
    """The bytes of one section of a 64-bit little-endian ELF file."""
    import struct

    with open(path, "rb") as f:
        data = f.read()
    if data[:4] != b"\x7fELF" or data[4] != 2 or data[5] != 1:
        raise ValueError("%s: not a 64-bit little-endian ELF" % path)
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)

    def sh(i):  # (name offset, offset, size)
        b = shoff + i * shentsize
        nm, = struct.unpack_from("<I", data, b)
        off, size = struct.unpack_from("<QQ", data, b + 0x18)
        return nm, off, size

    _, stroff, _ = sh(shstrndx)
    for i in range(shnum):
        nm, off, size = sh(i)
        end = data.index(b"\0", stroff + nm)
        if data[stroff + nm:end] == name:
            return data[off:off + size]
    raise ValueError("%s: no section %r" % (path, name))


def interp_code_id() -> str:
    """Identifier of the interpreter's and the generator's device code: a hash of the code objects
    libmythril_hip.so embeds (its .hip_fatbin section: sieve_kernels.hip, generate.hip and the
    micro-benchmarks), so a host-only edit leaves it unchanged."""
    import hashlib

    return hashlib.sha256(_elf_section(LIB_PATH, b".hip_fatbin")).hexdigest()[:16]


def codegen_id(engine: str = "jit", variant: str = "plain", short_circuit: bool = True) -> str:
    """Identifier of the code one engine runs on bench.py's workload ("jit": the native code
    emitted for the config-5 tape set of `variant`, jit_code_id; "interp": the device code objects
    of the library, interp_code_id).  Profiles that price this code (profiles/pmc_summary.json,
    profiles/alg_work.json) record it, and bench.py uses a profile only for the code it runs."""
    key = (engine, variant, short_circuit)
    if key not in _CODE_IDS:
        if engine == "interp":
            _CODE_IDS[key] = interp_code_id()
        else:
            from . import synth

            ts = synth.generate(None, keccak=variant == "keccak")
            _CODE_IDS[key] = jit_code_id(ts, short_circuit=short_circuit)
    return _CODE_IDS[key]


def gen_limb(seed: int, var: int, index: int, limb: int) -> int:
    return int(load().mh_gen_limb(seed, var, index, limb))


class Context:
    """One GPU + one stream (mh_ctx)."""

    def __init__(self, device: int = 0):
        self.lib = load()
        h = C.c_void_p()
        _check(self.lib.mh_ctx_create(device, C.byref(h)))
        self.h = h
        self.device = device

    def set_stream(self, stream_ptr: Optional[int]) -> None:
        _check(self.lib.mh_ctx_set_stream(self.h, C.c_void_p(stream_ptr or 0)))

    def synchronize(self) -> None:
        _check(self.lib.mh_ctx_synchronize(self.h))

    def clear_cache(self) -> None:
        """Drop the compiled tapes mh_tapes_compile keeps by content (mh_ctx_clear_cache)."""
        _check(self.lib.mh_ctx_clear_cache(self.h))

    def close(self) -> None:
        if self.h:
            self.lib.mh_ctx_destroy(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def compile(self, tapeset: TapeSet) -> "CompiledTapes":
        return CompiledTapes(self, tapeset)

    def compile_async(self, tapeset: TapeSet) -> "PendingCompile":
        """mh_tapes_compile_async: the compile runs on the context's worker thread; the caller
        does host-only work meanwhile (no other call on this context) and then .wait()s."""
        return PendingCompile(self, tapeset)

    def assignments(self, n_vars: int, capacity: int) -> "Assignments":
        return Assignments(self, n_vars, capacity)

    def enable_timing(self, on: bool = True) -> None:
        _check(self.lib.mh_ctx_enable_timing(self.h, 1 if on else 0))

    def kernel_time(self) -> Tuple[float, int]:
        """(summed ms, launches) of the sieve launches timed since the last call."""
        ms, n = C.c_double(), C.c_uint64()
        _check(self.lib.mh_ctx_kernel_time(self.h, C.byref(ms), C.byref(n)))
        return ms.value, n.value

    def comm_init(self, unique_id: bytes, rank: int, world: int) -> None:
        """One RCCL communicator for this ctx (mh_comm_init)."""
        buf = (C.c_uint8 * COMM_ID_BYTES).from_buffer_copy(unique_id)
        _check(self.lib.mh_comm_init(self.h, C.cast(buf, C.c_void_p), rank, world))

    def comm_allreduce(self, d_first_hit: int, d_hit_count: int, n: int) -> None:
        """MIN of first witnesses, SUM of counts over the ranks, in place (device buffers)."""
        _check(self.lib.mh_comm_allreduce_results(self.h, C.c_void_p(d_first_hit),
                                                  C.c_void_p(d_hit_count), n))

    def comm_destroy(self) -> None:
        _check(self.lib.mh_comm_destroy(self.h))

    def microbench(self, kind: int, waves_per_simd: int = 8) -> float:
        """Sustained lane-ops/s of one instruction kind (mh_microbench_issue; MB_KINDS)."""
        v = C.c_double()
        _check(self.lib.mh_microbench_issue(self.h, kind, waves_per_simd, C.byref(v)))
        return v.value


def _compile_args(tapeset: TapeSet):
    nodes, offs, consts = tapeset.flatten()
    return (np.ascontiguousarray(nodes, dtype=NODE_DTYPE), np.ascontiguousarray(offs, dtype=np.uint64),
            np.ascontiguousarray(consts, dtype=np.uint32))


class PendingCompile:
    """A compile on the context's worker thread (Context.compile_async); its input arrays are
    held here until wait() returns the CompiledTapes."""

    def __init__(self, ctx: Context, tapeset: TapeSet):
        import time

        self.ctx, self.tapeset = ctx, tapeset
        t0 = time.perf_counter()
        args = _compile_args(tapeset)
        nodes, offs, consts = args
        self.t1 = time.perf_counter()
        self.flatten_s = self.t1 - t0
        _check(ctx.lib.mh_tapes_compile_async(
            ctx.h, nodes.ctypes.data_as(C.c_void_p), _ptr(offs, C.c_uint64), len(tapeset.tapes),
            _ptr(consts), len(tapeset.pool.values), tapeset.n_vars))
        # held from here on, and only once the compile is queued: a refused call (another
        # compile pending) leaves nothing for __del__ to collect -- it would take the other's
        self.args = args

    def wait(self) -> "CompiledTapes":
        import time

        h, secs = C.c_void_p(), C.c_double()
        try:
            _check(self.ctx.lib.mh_tapes_compile_wait(self.ctx.h, C.byref(h), C.byref(secs)))
        finally:
            self.args = None
        # timing: host flatten, the compile's own seconds on the worker (it overlapped the
        # caller's work; the wait itself is what the caller paid for it)
        self.wait_s = time.perf_counter() - self.t1
        return CompiledTapes(self.ctx, self.tapeset, _handle=h,
                             _timing=(self.flatten_s, secs.value))

    def __del__(self):  # dropped without wait(): collect the compile (the worker still reads the
        # input arrays this object holds) and free its tapes
        if getattr(self, "args", None) is not None and getattr(self.ctx, "h", None):
            try:
                self.wait().close()
            except Exception:  # noqa: BLE001 - interpreter shutdown, a failed compile
                pass


class CompiledTapes:
    """mh_tapeset: tapes lowered to device code, resident in HBM."""

    def __init__(self, ctx: Context, tapeset: TapeSet, _handle=None, _timing=None):
        import time

        self.ctx = ctx
        if _handle is not None:  # from PendingCompile.wait
            self.h = _handle
            self.timing = _timing
            self.n_tapes = len(tapeset.tapes)
            self.n_vars = tapeset.n_vars
            return
        t0 = time.perf_counter()
        nodes, offs, consts = _compile_args(tapeset)
        h = C.c_void_p()
        t1 = time.perf_counter()
        _check(ctx.lib.mh_tapes_compile(
            ctx.h, nodes.ctypes.data_as(C.c_void_p), _ptr(offs, C.c_uint64), len(tapeset.tapes),
            _ptr(consts), len(tapeset.pool.values), tapeset.n_vars, C.byref(h)))
        self.h = h
        # host flatten / native compile+upload seconds (per-stage latency reports)
        self.timing = (t1 - t0, time.perf_counter() - t1)
        self.n_tapes = len(tapeset.tapes)
        self.n_vars = tapeset.n_vars

    def jit(self, values: bool = False, max_vgpr: int = 0, short_circuit: bool = True) -> dict:
        """Compile the tapes the JIT covers to native gfx950 code (mh_tapes_jit); later runs
        over the whole set use it.  short_circuit=False evaluates every conjunct of every row
        (MH_JIT_FULL_EVAL; same results).  Returns mh_tapes_jit_info as a dict."""
        flags = (JIT_VALUES if values else 0) | (0 if short_circuit else JIT_FULL_EVAL)
        _check(self.ctx.lib.mh_tapes_jit(self.h, flags, max_vgpr))
        return self.jit_info()

    def code_id(self) -> str:
        """Identifier of the native code jit() built (mh_tapes_jit_code_id; see jit_code_id)."""
        out = C.c_uint64()
        _check(self.ctx.lib.mh_tapes_jit_code_id(self.h, C.byref(out)))
        return "%016x" % out.value

    def jit_info(self) -> dict:
        ji = JitInfo()
        _check(self.ctx.lib.mh_tapes_jit_info(self.h, C.byref(ji)))
        return {f: getattr(ji, f) for f, _ in JitInfo._fields_}

    def jitted(self) -> np.ndarray:
        out = np.zeros(max(self.n_tapes, 1), dtype=np.uint8)
        _check(self.ctx.lib.mh_tapes_jitted(self.h, out.ctypes.data_as(C.POINTER(C.c_uint8)),
                                            self.n_tapes))
        return out[: self.n_tapes]

    def jit_values(self, assign: "Assignments", row_first: int = 0,
                   row_count: Optional[int] = None) -> np.ndarray:
        """Root values of every jitted tape by the native code: u32 [n_tapes, 8, rows]."""
        rc = assign.capacity - row_first if row_count is None else row_count
        out = np.zeros((self.n_tapes, 8, max(rc, 1)), dtype=np.uint32)
        _check(self.ctx.lib.mh_jit_eval_all(self.ctx.h, self.h, assign.h, row_first, rc,
                                            _ptr(out)))
        return out[:, :, :rc]

    def info(self):
        arr = (TapeInfo * max(self.n_tapes, 1))()
        _check(self.ctx.lib.mh_tapes_info(self.h, C.cast(arr, C.c_void_p), self.n_tapes))
        return [dict(n_nodes=x.n_nodes, n_insns=x.n_insns, n_regs=x.n_regs,
                     features=x.features, alg_ops=x.alg_ops) for x in arr[: self.n_tapes]]

    def close(self) -> None:
        if self.h:
            self.ctx.lib.mh_tapes_destroy(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


class Assignments:
    """mh_assign: candidate assignments, SoA u32 limbs in HBM."""

    def __init__(self, ctx: Context, n_vars: int, capacity: int):
        self.ctx = ctx
        self.n_vars = n_vars
        self.capacity = capacity
        h = C.c_void_p()
        _check(ctx.lib.mh_assign_create(ctx.h, n_vars, capacity, C.byref(h)))
        self.h = h

    def upload(self, soa: np.ndarray, first: int = 0) -> None:
        """soa: u32 array shaped [n_vars, 8, count] (limb 0 least significant)."""
        soa = np.ascontiguousarray(soa, dtype=np.uint32)
        assert soa.shape[:2] == (self.n_vars, 8)
        _check(self.ctx.lib.mh_assign_upload(self.h, _ptr(soa), first, soa.shape[2]))

    def download(self, first: int, count: int) -> np.ndarray:
        out = np.zeros((self.n_vars, 8, count), dtype=np.uint32)
        _check(self.ctx.lib.mh_assign_download(self.h, _ptr(out), first, count))
        return out

    def generate(self, seed: int, global_base: int = 0) -> None:
        _check(self.ctx.lib.mh_assign_generate(self.h, seed, global_base))

    def generate_guided(self, seed: int, arrays: dict, global_base: int = 0, first: int = 0,
                        count: Optional[int] = None) -> None:
        """Rows [first, first+count) from a guide (mythril_amd.candidates.Guide.arrays())."""
        count = self.capacity - first if count is None else count
        a = {k: np.ascontiguousarray(v) for k, v in arrays.items()}
        n_cols = len(a["width"])
        n_sets = len(a["set_off"]) - 1
        g = Guide(n_cols, a["width"].ctypes.data_as(C.POINTER(C.c_uint16)), _ptr(a["pool_off"]),
                  _ptr(a["pool"]), n_sets, a["set_prob"].ctypes.data_as(C.POINTER(C.c_uint8)),
                  _ptr(a["set_off"]), _ptr(a["alt_off"]), _ptr(a["entry_col"]),
                  _ptr(a["entry_val"]))
        _check(self.ctx.lib.mh_assign_generate_guided(self.h, seed, global_base, first, count,
                                                      C.byref(g)))

    def close(self) -> None:
        if self.h:
            self.ctx.lib.mh_assign_destroy(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


def run(ctx: Context, tapes: CompiledTapes, assign: Assignments, *, tape_first: int = 0,
        tape_count: Optional[int] = None, row_first: int = 0, row_count: Optional[int] = None,
        index_base: int = 0, mode: int = MODE_COUNT_ALL):
    """Blocking run; returns (first_hit[u64], hit_count[u64]) per tape."""
    tc = tapes.n_tapes - tape_first if tape_count is None else tape_count
    rc = assign.capacity - row_first if row_count is None else row_count
    fh = np.zeros(max(tc, 1), dtype=np.uint64)
    hc = np.zeros(max(tc, 1), dtype=np.uint64)
    _check(ctx.lib.mh_run(ctx.h, tapes.h, tape_first, tc, assign.h, row_first, rc, index_base,
                          mode, _ptr(fh, C.c_uint64), _ptr(hc, C.c_uint64)))
    return fh[:tc], hc[:tc]


def run_rows(ctx: Context, tapes: CompiledTapes, assign: Assignments, n_cols: int, *,
             tape_first: int = 0, tape_count: Optional[int] = None, row_first: int = 0,
             row_count: Optional[int] = None, index_base: int = 0, mode: int = MODE_FIRST_HIT):
    """Blocking run plus each tape's witness row (mh_run_rows): (first_hit, hit_count,
    rows u32 [tape, column < n_cols, limb]; zero for a tape without a hit)."""
    tc = tapes.n_tapes - tape_first if tape_count is None else tape_count
    rc = assign.capacity - row_first if row_count is None else row_count
    fh = np.zeros(max(tc, 1), dtype=np.uint64)
    hc = np.zeros(max(tc, 1), dtype=np.uint64)
    rows = np.zeros((max(tc, 1), max(n_cols, 1), 8), dtype=np.uint32)
    _check(ctx.lib.mh_run_rows(ctx.h, tapes.h, tape_first, tc, assign.h, row_first, rc,
                               index_base, mode, _ptr(fh, C.c_uint64), _ptr(hc, C.c_uint64),
                               n_cols, _ptr(rows)))
    return fh[:tc], hc[:tc], rows[:tc, :n_cols]


def query_round(ctx: Context, tapes: CompiledTapes, assign: "Assignments", guide: GuideHandle,
                seed: int, global_base: int, count: int, n_cols: int, *, tape_first: int = 0,
                tape_count: Optional[int] = None, mode: int = MODE_FIRST_HIT):
    """One guided round (mh_query_round): rows [0, count) generated from `guide`, then
    run_rows over them with index_base = global_base.  Returns (first_hit, hit_count, rows)."""
    tc = tapes.n_tapes - tape_first if tape_count is None else tape_count
    fh = np.zeros(max(tc, 1), dtype=np.uint64)
    hc = np.zeros(max(tc, 1), dtype=np.uint64)
    rows = np.zeros((max(tc, 1), max(n_cols, 1), 8), dtype=np.uint32)
    _check(ctx.lib.mh_query_round(ctx.h, tapes.h, assign.h, C.byref(guide.guide), seed,
                                  global_base, count, tape_first, tc, mode, _ptr(fh, C.c_uint64),
                                  _ptr(hc, C.c_uint64), n_cols, _ptr(rows)))
    return fh[:tc], hc[:tc], rows[:tc, :n_cols]


def run_async(ctx: Context, tapes: CompiledTapes, assign: Assignments, d_first_hit: int,
              d_hit_count: int, *, tape_first: int = 0, tape_count: Optional[int] = None,
              row_first: int = 0, row_count: Optional[int] = None, index_base: int = 0,
              mode: int = MODE_COUNT_ALL) -> None:
    """Enqueue on the ctx stream; results accumulate into caller device buffers (u64)."""
    tc = tapes.n_tapes - tape_first if tape_count is None else tape_count
    rc = assign.capacity - row_first if row_count is None else row_count
    _check(ctx.lib.mh_run_async(ctx.h, tapes.h, tape_first, tc, assign.h, row_first, rc,
                                index_base, mode, C.c_void_p(d_first_hit),
                                C.c_void_p(d_hit_count)))


def results_reset(ctx: Context, d_first_hit: int, d_hit_count: int, n: int) -> None:
    _check(ctx.lib.mh_results_reset(ctx.h, C.c_void_p(d_first_hit), C.c_void_p(d_hit_count), n))


def eval_values(ctx: Context, tapes: CompiledTapes, tape: int, assign: Assignments,
                row_first: int = 0, row_count: Optional[int] = None) -> np.ndarray:
    """Root value of `tape` per row: u32 [8, rows] (limb-major)."""
    rc = assign.capacity - row_first if row_count is None else row_count
    out = np.zeros((8, max(rc, 1)), dtype=np.uint32)
    _check(ctx.lib.mh_eval_values(ctx.h, tapes.h, tape, assign.h, row_first, rc, _ptr(out)))
    return out[:, :rc]


def eval_values_many(ctx: Context, tapes: CompiledTapes, ids: Sequence[int], assign: Assignments,
                     row: int = 0) -> np.ndarray:
    """Root values of the tapes `ids` at one row (mh_eval_values_many): u32 [len(ids), 8]."""
    ids_a = np.ascontiguousarray(ids, dtype=np.uint32)
    out = np.zeros((max(len(ids_a), 1), 8), dtype=np.uint32)
    _check(ctx.lib.mh_eval_values_many(ctx.h, tapes.h, _ptr(ids_a), len(ids_a), assign.h, row,
                                       _ptr(out)))
    return out[:len(ids_a)]


def eval_launches(ctx: Context) -> int:
    """Kernel launches mh_eval_values_many has made on `ctx`."""
    v = C.c_uint64()
    _check(ctx.lib.mh_ctx_eval_launches(ctx.h, C.byref(v)))
    return int(v.value)


def limbs_to_ints(arr: np.ndarray) -> Sequence[int]:
    """[8, n] u32 limbs -> Python ints."""
    out = []
    for j in range(arr.shape[1]):
        v = 0
        for k in range(8):
            v |= int(arr[k, j]) << (32 * k)
        out.append(v)
    return out


def microbench_gather(device: int, log2_rows: int, permille: int, layout: int,
                      reps: int = 5) -> Tuple[float, float, int]:
    """mh_microbench_gather: (median ms per launch, useful GB/s, survivors)."""
    ms, gbps, n = C.c_double(), C.c_double(), C.c_uint64()
    _check(load().mh_microbench_gather(device, log2_rows, permille, layout, reps, C.byref(ms),
                                       C.byref(gbps), C.byref(n)))
    return ms.value, gbps.value, int(n.value)
