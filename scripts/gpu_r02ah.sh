#!/bin/bash
# keccak lane complementing , theta chains interleaved and two-phase in-place chi: JIT GPU suite, keccak-variant bench A/B
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02ah
mkdir -p $O
stop() { case $1 in 124|134|137|139) echo "stop: exit $1"; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_jit.py -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu_jit.txt 2>&1
r=$?; echo "pytest jit: $r"; stop $r; [ $r -ne 0 ] && exit $r
for c in 1; do
  MH_JIT_KEC_COMPLEMENT=$c timeout -k 10 240 python -u bench.py --variant keccak --steps 5 --no-companion --no-cpu-baseline > $O/bench_keccak_c$c.json 2> $O/bench_keccak_c$c.log
  r=$?; echo "bench keccak complement=$c: $r"; stop $r; [ $r -ne 0 ] && exit $r
  python -c "import json; d=json.load(open('$O/bench_keccak_c$c.json')); print('$c', d['value'], d['kernel_ms'], d['tapes_with_witness'])"
done
exit 0
