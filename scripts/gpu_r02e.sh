#!/bin/bash
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02e
mkdir -p $O
T="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_jit.py > $O/jit_suite.txt 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_jit.json 2> $O/bench_jit.txt && \
timeout -k 10 300 python -u scripts/valu_peak.py > $O/valu_peak.json 2> $O/valu_peak.txt
