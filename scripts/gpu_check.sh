#!/bin/bash
# GPU-box check: parity tests, then a short bench, then a kernel-trace profile of the bench.
# Run via gpurun from the repo root:  gpurun -- bash scripts/gpu_check.sh [rows]
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
ROWS=${1:-1048576}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --rows-per-gpu $ROWS --cpu-seconds 8 > gpurun_out/bench_small.json 2> gpurun_out/bench_small.log && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --rows-per-gpu $ROWS --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/bench_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/bench_prof.log
