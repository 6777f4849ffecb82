"""The N > 1 data path with kernel output, re-runnable by the driver: two processes
on one GPU, started by torch.distributed.run before either touches the GPU, each running the
native code over its own shard of config-5 rows; the gloo MIN / SUM of their per-tape results
(shard.allreduce_results, the reduction the library's RCCL exchange performs between GPUs) must
equal one launch over both shards and the C oracle (tests/tools/shard_check.py).  RCCL refuses
two ranks on one device, so the library's own communicator with world > 1 runs only on the
driver's multi-GPU node; this checks the sharding and the reduction semantics with real kernels.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.timeout(400)
def test_two_process_shards_on_one_gpu():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "tools", "shard_check.py"), str(1 << 16)]
    env = dict(os.environ, OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "8"))
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=360)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0 and lines, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    rec = json.loads(lines[-1])
    print(rec)
    assert rec["reduced_equals_single_launch"] and rec["oracle_equal"]
    assert rec["first_witness_in_rank1_shard"] > 0 and rec["jitted"] == rec["tapes"]
