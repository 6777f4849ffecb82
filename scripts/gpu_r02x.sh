#!/bin/bash
# measured per-instruction costs in the conjunct order, hit bookkeeping only for chunks with
# hits: JIT GPU suite, default bench, round profile (plain + keccak variant)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02x
mkdir -p $O
stop() { case $1 in 124|134|137|139) echo "stop: exit $1"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_jit.py -x -v --timeout 300 --timeout-method thread > $O/pytest_jit.txt 2>&1
r=$?; echo "pytest: $r"; stop $r; [ $r -ne 0 ] && exit $r
timeout -k 10 300 python -u bench.py --cpu-seconds 8 > $O/bench_default.json 2> $O/bench_default.log
r=$?; echo "bench: $r"; stop $r; [ $r -ne 0 ] && exit $r
bash scripts/profile.sh r02x --no-companion && bash scripts/profile.sh r02x_keccak --variant keccak --no-companion
r=$?; echo "profile: $r"; exit $r
