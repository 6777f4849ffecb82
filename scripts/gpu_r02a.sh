#!/bin/bash
# Round-2 check: GPU suite (incl. EIP-145 and the bench-config pin), the VALU issue-rate sweep.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02a
O=gpurun_out/r02a
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python -u scripts/valu_peak.py > $O/valu_peak.json 2> $O/valu_peak.txt
