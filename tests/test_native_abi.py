"""The C-ABI library loads on a GPU-less host and exports every entry point include/mythril_hip.h
declares; host-only helpers agree with the oracle.  No device compute here."""
import ctypes as C
import os
import re

import pytest

from mythril_amd import native
from oracle import smt_eval

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include",
                      "mythril_hip.h")


def declared_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(
        r"^\s*(?:int32_t|uint32_t|uint64_t|const char\*)\s+(mh_\w+)\s*\(", text,
                                 re.M)))


def test_header_declares_the_abi():
    names = declared_functions()
    assert len(names) >= 20
    assert set(names) == set(native.SIGNATURES), set(names) ^ set(native.SIGNATURES)


def test_library_exports_every_symbol():
    lib = native.load()
    for name in declared_functions():
        assert hasattr(lib, name), name
        assert C.cast(getattr(lib, name), C.c_void_p).value


def test_noasm_library_is_current():
    """The C++ step() build (libmythril_hip_noasm.so, tests/noasm_check.py on the GPU) exports the
    same ABI: a stale copy failed the GPU suite once (r06w), so `make` now builds both."""
    path = os.path.join(os.path.dirname(os.path.abspath(native.__file__)),
                        "libmythril_hip_noasm.so")
    if not os.path.exists(path):
        pytest.skip("noasm library not built")
    lib = C.CDLL(path)
    for name in declared_functions():
        assert hasattr(lib, name), name


def test_version_and_errors_without_device():
    assert native.version() == (0, 1, 0)
    assert native.device_count() == 0 or native.device_count() >= 1
    lib = native.load()
    h = C.c_void_p()
    r = lib.mh_ctx_create(9999, C.byref(h))
    assert r == native.MH_E_NODEVICE
    assert b"device" in lib.mh_last_error()
    assert lib.mh_ctx_destroy(None) == native.MH_OK
    assert lib.mh_tapes_destroy(None) == native.MH_OK


def test_generator_restatement_matches_library():
    for seed, var, idx, limb in [(0, 0, 0, 0), (1, 2, 3, 4), (0xDEADBEEF, 3, 1 << 40, 7)]:
        assert native.gen_limb(seed, var, idx, limb) == smt_eval.gen_limb(seed, var, idx, limb)


def test_comm_argument_validation_without_device():
    """mh_comm_* (the library's RCCL exchange) refuse bad arguments with
    MH_E_INVALID before touching RCCL or a device, and never abort the process."""
    lib = native.load()
    uid = (C.c_uint8 * 128)()
    assert lib.mh_comm_init(None, uid, 0, 1) == native.MH_E_INVALID
    assert b"null" in lib.mh_last_error()
    assert lib.mh_comm_unique_id(None) == native.MH_E_INVALID
    assert lib.mh_comm_allreduce_results(None, None, None, 0) == native.MH_E_INVALID
    assert lib.mh_comm_destroy(None) == native.MH_E_INVALID


def test_comm_rank_world_checks(monkeypatch):
    """rank / world are checked before RCCL is opened (a ctx handle is needed to get that far:
    a fake, never dereferenced past the argument checks, stands in on a GPU-less host)."""
    lib = native.load()
    uid = (C.c_uint8 * 128)()
    fake = C.c_void_p(1)  # not a ctx: every call below must fail on its arguments first
    for rank, world in ((0, 0), (-1, 2), (2, 2), (5, 1)):
        assert lib.mh_comm_init(fake, uid, rank, world) == native.MH_E_INVALID, (rank, world)
        assert b"rank" in lib.mh_last_error()


def test_async_compile_argument_validation_without_device():
    """mh_tapes_compile_async / _wait refuse a null context and a wait with nothing pending."""
    lib = native.load()
    h = C.c_void_p()
    assert lib.mh_tapes_compile_async(None, None, None, 0, None, 0, 0) == native.MH_E_INVALID
    assert lib.mh_tapes_compile_wait(None, C.byref(h), None) == native.MH_E_INVALID
    assert b"null" in lib.mh_last_error()


def test_refused_async_compile_leaves_the_pending_one(monkeypatch):
    """A compile_async the library refuses (another compile pending on the ctx) must not collect
    the pending compile when its PendingCompile is dropped (it used to: __del__ waited on the
    ctx and took the other compile's result, r06b GPU suite)."""
    import gc
    import types

    from mythril_amd import synth

    waits = []
    lib = types.SimpleNamespace(
        mh_tapes_compile_async=lambda *a: native.MH_E_INVALID,
        mh_tapes_compile_wait=lambda *a: waits.append(a) or native.MH_OK)
    ctx = types.SimpleNamespace(lib=lib, h=C.c_void_p(1))
    with pytest.raises(native.SieveError):
        native.PendingCompile(ctx, synth.generate(2))
    gc.collect()
    assert waits == []
