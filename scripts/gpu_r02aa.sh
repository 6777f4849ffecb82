#!/bin/bash
# JIT GPU suite + default bench after the folding identities / value numbering
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02aa
mkdir -p $O
stop() { case $1 in 124|134|137|139) echo "stop: exit $1"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_jit.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1
r=$?; echo "pytest: $r"; stop $r; [ $r -ne 0 ] && exit $r
timeout -k 10 300 python -u bench.py --cpu-seconds 8 > $O/bench_default.json 2> $O/bench_default.log
r=$?; echo "bench: $r"; exit $r
