"""bench.py --gpus N launches N ranks by itself.

The driver runs `python bench.py --gpus N` for its scaling curve; without a launcher around it
bench.py must start one process per GPU (torch.distributed.run as a child) and relay rank 0's one
JSON line.  --launch-check runs that plumbing over gloo with no GPU work.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.pop("LOCAL_RANK", None)
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                       capture_output=True, text=True, timeout=240, cwd=ROOT)
    return p


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_n_launches_n_ranks_and_prints_one_line(n):
    p = _run(["--gpus", str(n), "--launch-check"])
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, p.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == n
    assert line["ranks"] == list(range(n))
    assert line["scaling"] == "weak"


def test_strong_flag_is_carried():
    p = _run(["--gpus", "2", "--launch-check", "--strong"])
    assert p.returncode == 0, p.stderr[-2000:]
    line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert line["scaling"] == "strong" and line["n_gpus"] == 2


def test_world_size_mismatch_is_refused():
    p = _run(["--gpus", "2", "--launch-check"], {"WORLD_SIZE": "1", "RANK": "0"})
    assert p.returncode != 0
    assert "WORLD_SIZE 1" in p.stderr


def test_single_gpu_runs_in_process():
    p = _run(["--gpus", "1", "--launch-check"])
    assert p.returncode == 0, p.stderr[-2000:]
    assert "[launcher]" not in p.stderr
    line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert line["ranks"] == [0]
