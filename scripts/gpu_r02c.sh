#!/bin/bash
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02c
mkdir -p $O
T="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_jit.py -k bench_config > $O/jit_bench_pin.txt 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_jit.json 2> $O/bench_jit.txt && \
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --engine interp --no-cpu-baseline > $O/bench_interp.json 2> $O/bench_interp.txt
