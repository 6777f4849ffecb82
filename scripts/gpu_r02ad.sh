#!/bin/bash
# occupancy classes: JIT GPU suite on the new build, then bench A/B over MH_JIT_CLASSES
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02ad
mkdir -p $O
stop() { case $1 in 124|134|137|139) echo "stop: exit $1"; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_jit.py -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu_jit.txt 2>&1
r=$?; echo "pytest jit: $r"; stop $r; [ $r -ne 0 ] && exit $r
for c in 0 64,80,96 72,80,96 80,96 64,80,96; do
  MH_JIT_CLASSES=$c timeout -k 10 200 python -u bench.py --steps 5 --no-companion --no-cpu-baseline > $O/bench_c${c//,/_}.json 2> $O/bench_c${c//,/_}.log
  r=$?; echo "bench classes=$c: $r"; stop $r; [ $r -ne 0 ] && exit $r
  python -c "import json,sys; d=json.load(open('$O/bench_c${c//,/_}.json')); print('$c', d['value'], d['kernel_ms'], d['jit']['n_modules'])"
done
exit 0
