#!/bin/bash
# JIT profile (kernel trace + PMC passes) and the register-budget sweep.
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02d
mkdir -p $O
timeout -k 10 900 bash scripts/profile.sh r02d_jit && \
for v in 96 160; do
  timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --max-vgpr $v > $O/bench_vgpr$v.json 2> $O/bench_vgpr$v.txt || exit 1
done
