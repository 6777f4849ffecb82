#!/bin/bash
# keccak in the native code: GPU JIT suite, keccak-variant bench (jit), default bench
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02p
mkdir -p $O
stop() { case $1 in 124|134|137|139) echo "stop: exit $1"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_jit.py -x -v --timeout 300 --timeout-method thread > $O/pytest_jit.txt 2>&1
r=$?; echo "pytest: $r"; stop $r; [ $r -ne 0 ] && exit $r
timeout -k 10 300 python -u bench.py --variant keccak --no-cpu-baseline > $O/bench_keccak.json 2> $O/bench_keccak.log
r=$?; echo "bench keccak: $r"; stop $r
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.log
r=$?; echo "bench: $r"; exit $r
