#!/bin/bash
# round profile of the build with the uniform shortcuts: GPU JIT suite, default bench, keccak
# variant bench, kernel trace + PMC passes of both
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02at
mkdir -p $O
stop() { case $1 in 124|134|137|139) echo "stop: exit $1"; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_jit.py -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu_jit.txt 2>&1
r=$?; echo "pytest jit: $r"; stop $r; [ $r -ne 0 ] && exit $r
timeout -k 10 300 python -u bench.py --cpu-seconds 8 > $O/bench_default.json 2> $O/bench_default.log
r=$?; echo "bench: $r"; stop $r; [ $r -ne 0 ] && exit $r
timeout -k 10 300 python -u bench.py --variant keccak --cpu-seconds 8 > $O/bench_keccak.json 2> $O/bench_keccak.log
r=$?; echo "bench keccak: $r"; stop $r; [ $r -ne 0 ] && exit $r
bash scripts/profile.sh r02at --no-companion && bash scripts/profile.sh r02at_keccak --variant keccak --no-companion
r=$?; echo "profile: $r"; exit $r
