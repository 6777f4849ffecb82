import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and the built HIP library")


EMU_DIR = os.path.join(ROOT, "tests", "native")
EMU_LIB = os.path.join(EMU_DIR, "libmh_emu.so")
CSRC = os.path.join(ROOT, "mythril_amd", "csrc")


def build_emulator() -> str:
    """Build the test-only host emulator (tests/native/emu.cpp + the tape compiler)."""
    srcs = [os.path.join(EMU_DIR, "emu.cpp"), os.path.join(EMU_DIR, "jit_emu.cpp"),
            os.path.join(CSRC, "compile.cpp"), os.path.join(CSRC, "jit.cpp"),
            os.path.join(CSRC, "jit_comgr.cpp")]
    deps = srcs + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    if os.path.exists(EMU_LIB) and all(os.path.getmtime(EMU_LIB) >= os.path.getmtime(d)
                                       for d in deps):
        return EMU_LIB
    cmd = ["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-I" + CSRC, "-I/opt/rocm/include",
           "-o", EMU_LIB] + srcs + ["-L/opt/rocm/lib", "-Wl,-rpath,/opt/rocm/lib",
                                    "-lamd_comgr"]
    subprocess.run(cmd, check=True, capture_output=True)
    return EMU_LIB


@pytest.fixture(scope="session")
def emu():
    from tests.emu import Emulator

    return Emulator(build_emulator())


@pytest.fixture(scope="session")
def gpu_ctx():
    # torch's HIP runtime first, as bench.py does: libmythril_hip then binds to the same
    # libamdhip64 (one runtime per process)
    try:
        import torch

        torch.cuda.init()
    except Exception:
        pass
    from mythril_amd import native

    if native.device_count() < 1:
        pytest.fail("no gfx950 device visible (GPU tests must run on an MI355X)")
    ctx = native.Context(0)
    yield ctx
    ctx.close()
