#!/bin/bash
# Full GPU-box pass: parity tests, bench, kernel-trace profile, PMC passes.
# Run via gpurun from the repo root:  gpurun -- bash scripts/gpu_all.sh [rows] [tag]
cd $GRAFT_REPO_ROOT
ROWS=${1:-1048576}
bash scripts/gpu_check.sh $ROWS && bash scripts/gpu_pmc.sh 262144
