"""The library's RCCL calls, checked against a recording stub librccl.

RCCL refuses two ranks on one GPU and this builder has no multi-GPU node, so the arguments of the
library's one exchange (capi.cpp mh_comm_*) are checked by pointing it at a stub (MH_RCCL_LIB):
a small C library, built here, that exports ncclGetUniqueId / ncclCommInitRank / ncclAllReduce /
ncclCommDestroy / ncclGetErrorString with RCCL's signatures (/opt/rocm/include/rccl/rccl.h) and
logs every call.  Each check runs in a child process (the library opens RCCL once per process).

* CPU: mh_comm_unique_id reaches the stub and returns its 128-byte id;
* GPU (a real ctx): mh_comm_init passes (world, the id, rank); mh_comm_allreduce_results issues
  exactly two in-place all-reduces on the ctx stream — first hits as ncclUint64 / ncclMin, counts
  as ncclUint64 / ncclSum, count = tapes — and mh_comm_destroy releases the communicator.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# rccl.h values (ncclDataType_t / ncclRedOp_t)
NCCL_UINT64, NCCL_SUM, NCCL_MIN = 5, 0, 3

STUB_C = r"""
#include <stdio.h>
#include <string.h>
typedef struct { char internal[128]; } ncclUniqueId;
typedef struct stub_comm { int nranks, rank; } *ncclComm_t;
static char g_log[16384];
static size_t g_len;
static struct stub_comm g_comm;
static void logf_(const char* s) {
    size_t n = strlen(s);
    if (g_len + n + 1 < sizeof g_log) { memcpy(g_log + g_len, s, n); g_len += n; g_log[g_len++] = '\n'; }
}
int ncclGetUniqueId(ncclUniqueId* id) {
    for (int i = 0; i < 128; ++i) id->internal[i] = (char)(i * 7 + 1);
    logf_("{\"call\": \"GetUniqueId\"}");
    return 0;
}
int ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank) {
    char b[256];
    unsigned sum = 0;
    for (int i = 0; i < 128; ++i) sum = sum * 31u + (unsigned char)id.internal[i];
    g_comm.nranks = nranks; g_comm.rank = rank;
    *comm = &g_comm;
    snprintf(b, sizeof b, "{\"call\": \"CommInitRank\", \"nranks\": %d, \"rank\": %d, \"id_hash\": %u, \"comm\": %lu}",
             nranks, rank, sum, (unsigned long)(size_t)*comm);
    logf_(b);
    return 0;
}
int ncclAllReduce(const void* send, void* recv, size_t count, int dtype, int op, ncclComm_t comm,
                  void* stream) {
    char b[320];
    snprintf(b, sizeof b, "{\"call\": \"AllReduce\", \"send\": %lu, \"recv\": %lu, \"count\": %lu, \"dtype\": %d, \"op\": %d, \"comm\": %lu, \"stream\": %lu}",
             (unsigned long)(size_t)send, (unsigned long)(size_t)recv, (unsigned long)count, dtype,
             op, (unsigned long)(size_t)comm, (unsigned long)(size_t)stream);
    logf_(b);
    return 0;
}
int ncclCommDestroy(ncclComm_t comm) {
    char b[128];
    snprintf(b, sizeof b, "{\"call\": \"CommDestroy\", \"comm\": %lu}", (unsigned long)(size_t)comm);
    logf_(b);
    return 0;
}
const char* ncclGetErrorString(int r) { (void)r; return "stub"; }
const char* stub_log(void) { g_log[g_len] = 0; return g_log; }
"""


def build_stub(tmp_path) -> str:
    src = tmp_path / "rccl_stub.c"
    src.write_text(STUB_C)
    out = tmp_path / "librccl_stub.so"
    subprocess.run(["gcc", "-O1", "-shared", "-fPIC", "-o", str(out), str(src)], check=True)
    return str(out)


def run_child(code: str, stub: str) -> list:
    env = dict(os.environ, MH_RCCL_LIB=stub, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    return [json.loads(x) for x in r.stdout.strip().splitlines() if x.startswith("{")]


CHILD_PRELUDE = """
import ctypes, os
from mythril_amd import native
stub = ctypes.CDLL(os.environ["MH_RCCL_LIB"])
stub.stub_log.restype = ctypes.c_char_p
def dump():
    print(stub.stub_log().decode(), flush=True)
"""


def test_unique_id_through_stub(tmp_path):
    stub = build_stub(tmp_path)
    calls = run_child(CHILD_PRELUDE + """
uid = native.comm_unique_id()
assert len(uid) == 128 and list(uid[:4]) == [1, 8, 15, 22], list(uid[:4])
dump()
""", stub)
    assert [c["call"] for c in calls] == ["GetUniqueId"]


@pytest.mark.gpu
def test_allreduce_arguments_through_stub(tmp_path):
    stub = build_stub(tmp_path)
    calls = run_child(CHILD_PRELUDE + """
import json
import torch
torch.cuda.init()
ctx = native.Context(0)
s = torch.cuda.Stream()
ctx.set_stream(s.cuda_stream)
uid = native.comm_unique_id()
ctx.comm_init(uid, 1, 2)
n = 37
fh = torch.zeros(n, dtype=torch.int64, device="cuda")
hc = torch.zeros(n, dtype=torch.int64, device="cuda")
ctx.comm_allreduce(fh.data_ptr(), hc.data_ptr(), n)
ctx.comm_destroy()
ctx.close()
print(json.dumps({"call": "expect", "fh": fh.data_ptr(), "hc": hc.data_ptr(), "n": n,
                  "stream": s.cuda_stream}), flush=True)
dump()
""", stub)
    want = calls[0]
    seq = [c for c in calls[1:]]
    assert [c["call"] for c in seq] == ["GetUniqueId", "CommInitRank", "AllReduce", "AllReduce",
                                        "CommDestroy"]
    init, red_min, red_sum, destroy = seq[1], seq[2], seq[3], seq[4]
    assert (init["nranks"], init["rank"]) == (2, 1)
    for red, ptr, op in ((red_min, want["fh"], NCCL_MIN), (red_sum, want["hc"], NCCL_SUM)):
        assert red["send"] == red["recv"] == ptr  # in place
        assert red["count"] == want["n"]
        assert red["dtype"] == NCCL_UINT64 and red["op"] == op
        assert red["comm"] == init["comm"]
        assert red["stream"] == want["stream"]  # the ctx stream, not the null stream
    assert destroy["comm"] == init["comm"]
