"""Profiles are keyed to the emitted code, not to host sources.

bench.py finds the PMC profile and the algorithmic-work entry of the code it runs by
`CompiledTapes.code_id()` (a hash of the native module texts mh_tapes_jit emits) or, for the
interpreter, by a hash of the library's embedded device code objects.  Both are computed here
without a device (mh_jit_code_id, the ELF's .hip_fatbin section), and a host-only edit of capi.cpp
must leave both unchanged, so the committed profiles still resolve.  Host only.
"""
import os
import shutil
import subprocess
import sys

from mythril_amd import native, synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_jit_code_id_is_a_function_of_the_emitted_code():
    ts = synth.generate(40)
    a = native.jit_code_id(ts)
    assert a == native.jit_code_id(ts)  # deterministic (threaded emission)
    assert native.jit_code_id(ts, short_circuit=False) != a  # other code, other id
    assert native.jit_code_id(synth.generate(40, first=1)) != a


def test_code_id_rejects_bad_tapes():
    import numpy as np
    import pytest

    ts = synth.generate(2)
    nodes, offs, consts = ts.flatten()
    offs = np.ascontiguousarray(offs, dtype=np.uint64).copy()
    offs[1] = offs[0]  # an empty tape
    import ctypes as C

    out = C.c_uint64()
    nodes = np.ascontiguousarray(nodes, dtype=native.NODE_DTYPE)
    consts = np.ascontiguousarray(consts, dtype=np.uint32)
    with pytest.raises(native.SieveError):
        native._check(native.load().mh_jit_code_id(
            nodes.ctypes.data_as(C.c_void_p), native._ptr(offs, C.c_uint64), 2,
            native._ptr(consts), len(ts.pool.values), ts.n_vars, 0, 0, C.byref(out)))


_PROBE = ("import sys; sys.path.insert(0, %r); from mythril_amd import native; "
          "print(native.codegen_id('jit'), native.interp_code_id())")


def test_host_only_edit_keeps_the_profile_keys(tmp_path):
    """Rebuild the library with capi.cpp edited (a comment appended: host code only) and check
    that both code ids -- hence bench.py's pmc_profile / alg_work lookups -- are unchanged."""
    src = os.path.join(ROOT, "mythril_amd", "csrc")
    dst = tmp_path / "mythril_amd" / "csrc"
    shutil.copytree(src, dst, copy_function=shutil.copy2,
                    ignore=shutil.ignore_patterns("__pycache__"))
    (tmp_path / "include").mkdir()
    shutil.copy2(os.path.join(ROOT, "include", "mythril_hip.h"), tmp_path / "include")
    objs = os.path.join(ROOT, "build", "csrc")
    if os.path.isdir(objs):  # reuse the in-tree objects: only capi.o is rebuilt
        shutil.copytree(objs, tmp_path / "build" / "csrc", copy_function=shutil.copy2)
    with open(dst / "capi.cpp", "a") as f:
        f.write("\n// host-only edit (tests/test_code_id.py)\n")
    subprocess.run(["make", "-C", str(dst), "-j", "8"], check=True, capture_output=True,
                   timeout=1200)
    lib = tmp_path / "mythril_amd" / native.LIB_NAME
    assert lib.exists()
    env = dict(os.environ, MYTHRIL_HIP_LIB=str(lib))
    edited = subprocess.run([sys.executable, "-c", _PROBE % ROOT], env=env, check=True,
                            capture_output=True, text=True, timeout=600).stdout.split()
    assert edited == [native.codegen_id("jit"), native.interp_code_id()]
