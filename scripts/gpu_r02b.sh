#!/bin/bash
# JIT bring-up: smallest JIT test alone first, then the JIT suite, then the interpreter suite,
# then bench both engines.  Every GPU step has its own time limit; the chain stops at the first
# failure.
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02b
mkdir -p $O
T="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
timeout -k 10 200 $T tests/test_gpu_jit.py -k smallest > $O/jit_smallest.txt 2>&1 && \
timeout -k 10 600 $T tests/test_gpu_jit.py > $O/jit_suite.txt 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_jit.json 2> $O/bench_jit.txt && \
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --engine interp --no-cpu-baseline > $O/bench_interp.json 2> $O/bench_interp.txt
