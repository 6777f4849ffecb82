#!/bin/bash
# Short-circuit conjunctions: JIT GPU suite, default bench (with the full-eval companion), then
# the round profile of the short-circuit build (kernel trace + PMC passes)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02v
mkdir -p $O
stop() { case $1 in 124|134|137|139) echo "stop: exit $1"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_jit.py -x -v --timeout 300 --timeout-method thread > $O/pytest_jit.txt 2>&1
r=$?; echo "pytest: $r"; stop $r; [ $r -ne 0 ] && exit $r
timeout -k 10 300 python -u bench.py --cpu-seconds 8 > $O/bench_default.json 2> $O/bench_default.log
r=$?; echo "bench: $r"; stop $r; [ $r -ne 0 ] && exit $r
bash scripts/profile.sh r02v --no-companion
r=$?; echo "profile: $r"; exit $r
