"""The query path's host-only native code (csrc/query.cpp: the query compiler; csrc/harvest.cpp:
the guide harvester and its session; csrc/smtlib.cpp: the z3-text reader) under AddressSanitizer +
UBSan, on the calls the Python side really makes: tests/tools/host_record.py records them
(LASER-shaped queries and 60-constraint paths in LASER order, their UNSAT variants, 40 random
conjunctions over arrays / functions / keccak; every LASER-shaped query's z3 text read constraint
by constraint, and malformed texts), tests/native/host_replay.cpp replays them against a
sanitized build of the three files and reads every returned array end to end.  Host only: no device, no HIP runtime in the build.
"""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = [os.path.join(ROOT, "mythril_amd", "csrc", f)
       for f in ("query.cpp", "harvest.cpp", "smtlib.cpp")]


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not installed")
def test_query_compiler_and_harvester_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "host_replay")
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer",
                    "-static-libasan", "-I", os.path.join(ROOT, "include")] + SRC +
                   [os.path.join(ROOT, "tests", "native", "host_replay.cpp"), "-o", exe],
                   check=True, timeout=600)
    rec = str(tmp_path / "calls.bin")
    subprocess.run([sys.executable, os.path.join(ROOT, "tests", "tools", "host_record.py"), rec,
                    "40"], check=True, timeout=600, cwd=ROOT)
    env = dict(os.environ)
    # the runtime is linked in statically; a preloaded library of the host environment must not
    # make it refuse to start
    env["ASAN_OPTIONS"] = "verify_asan_link_order=0:abort_on_error=0:exitcode=86"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1:exitcode=87"
    r = subprocess.run([exe, rec], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr
    stats = dict(kv.split("=") for kv in r.stdout.split())
    assert int(stats["queries"]) > 500 and int(stats["guides"]) > 400
