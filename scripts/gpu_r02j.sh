#!/bin/bash
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02j
mkdir -p $O
NCCL_DEBUG=WARN timeout -k 10 120 python -u scripts/diag_runtime.py torch_lazy > $O/torch_lazy.txt 2>&1
r=$?; echo "torch_lazy: $r"; exit 0
