#!/bin/bash
# Quick GPU pass: parity tests + per-op costs + short bench + kernel-trace profile.
# gpurun -- bash scripts/gpu_quick.sh [rows]
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
ROWS=${1:-1048576}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u scripts/op_costs.py > gpurun_out/op_costs.jsonl 2> gpurun_out/op_costs.log && \
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --rows-per-gpu $ROWS --cpu-seconds 8 > gpurun_out/bench_small.json 2> gpurun_out/bench_small.log && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --rows-per-gpu $ROWS --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/bench_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/bench_prof.log
