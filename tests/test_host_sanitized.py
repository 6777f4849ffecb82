"""The query path's host-only native code (csrc/query.cpp: the query compiler; csrc/harvest.cpp:
the guide harvester and its session; csrc/smtlib.cpp: the z3-text reader) under AddressSanitizer +
UBSan, on the calls the Python side really makes: tests/tools/host_record.py records them
(LASER-shaped queries and 60-constraint paths in LASER order, their UNSAT variants, 40 random
conjunctions over arrays / functions / keccak; every LASER-shaped query's z3 text read constraint
by constraint, and malformed texts), tests/native/host_replay.cpp replays them against a
sanitized build of the three files and reads every returned array end to end.  And the tape
compiler (compile.cpp) and the JIT (jit.cpp) on a corpus of tapes through the host emulators.
Host only: no device, no HIP runtime in the build.
"""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "mythril_amd", "csrc")
NATIVE = os.path.join(ROOT, "tests", "native")
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"]
ENV = dict(os.environ,
           # the runtime is linked in statically; a library the host environment preloads must
           # not make it refuse to start
           ASAN_OPTIONS="verify_asan_link_order=0:abort_on_error=0:exitcode=86",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=87")
needs_gxx = pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not installed")


def sanitized_build(srcs, exe, libs=()):
    """-O0 objects compiled in parallel (seconds, where -O1 takes minutes for jit.cpp), linked
    with the sanitizer runtimes."""
    inc = ["-I", CSRC, "-I", os.path.join(ROOT, "include"), "-I", "/opt/rocm/include"]
    objs, procs = [], []
    for i, src in enumerate(srcs):
        obj = "%s.%d.o" % (exe, i)
        objs.append(obj)
        procs.append(subprocess.Popen(["g++", "-std=c++17", "-O0", "-g1", "-fno-omit-frame-pointer"]
                                      + SAN + inc + ["-c", src, "-o", obj],
                                      stderr=subprocess.PIPE, text=True))
    for p in procs:
        _, err = p.communicate(timeout=900)
        assert p.returncode == 0, err[-3000:]
    subprocess.run(["g++"] + SAN + ["-static-libasan"] + objs + ["-o", exe] + list(libs),
                   check=True, timeout=300)


def replay(exe, data):
    r = subprocess.run([exe, data], capture_output=True, text=True, timeout=900, env=ENV)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr
    return dict(kv.split("=") for kv in r.stdout.split())


@needs_gxx
def test_query_compiler_and_harvester_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "host_replay")
    sanitized_build([os.path.join(CSRC, f) for f in ("query.cpp", "harvest.cpp", "smtlib.cpp")]
                    + [os.path.join(NATIVE, "host_replay.cpp")], exe)
    rec = str(tmp_path / "calls.bin")
    subprocess.run([sys.executable, os.path.join(ROOT, "tests", "tools", "host_record.py"), rec,
                    "40"], check=True, timeout=600, cwd=ROOT)
    stats = replay(exe, rec)
    assert int(stats["queries"]) > 500 and int(stats["guides"]) > 400


@needs_gxx
def test_tape_compiler_and_jit_under_asan_ubsan(tmp_path):
    """The interpreter lowering (compile.cpp) and the JIT (jit.cpp: SSA lowering, conjunct order,
    register allocation, emission, module text) on random tapes of every op and config-5 tapes,
    run by the host emulators (tests/native/emu.cpp, jit_emu.cpp): every output word equals the
    unsanitized build's (tests/tools/jit_corpus.py)."""
    corpus = str(tmp_path / "jit.bin")
    subprocess.run([sys.executable, os.path.join(ROOT, "tests", "tools", "jit_corpus.py"), corpus],
                   check=True, timeout=600, cwd=ROOT)
    exe = str(tmp_path / "jit_replay")
    sanitized_build([os.path.join(NATIVE, f) for f in ("emu.cpp", "jit_emu.cpp", "jit_replay.cpp")]
                    + [os.path.join(CSRC, f) for f in ("compile.cpp", "jit.cpp", "jit_comgr.cpp")],
                    exe, libs=["-L/opt/rocm/lib", "-Wl,-rpath,/opt/rocm/lib", "-lamd_comgr"])
    stats = replay(exe, corpus)
    assert int(stats["tapes"]) > 100 and int(stats["jitted"]) > 100
