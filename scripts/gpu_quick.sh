#!/bin/bash
# Quick GPU pass: parity tests + per-op costs + short bench.  gpurun -- bash scripts/gpu_quick.sh
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u scripts/op_costs.py > gpurun_out/op_costs.jsonl 2> gpurun_out/op_costs.log && \
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --rows-per-gpu 1048576 --no-cpu-baseline > gpurun_out/bench_small.json 2> gpurun_out/bench_small.log
