#!/bin/bash
# GPU-box quick pass: parity tests, smoke, then the default bench (one JSON line).
# Run via gpurun from the repo root:  gpurun -- bash scripts/gpu_quick.sh
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py --cpu-seconds 5 > gpurun_out/bench_default.json 2> gpurun_out/bench_default.log
