#!/bin/bash
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02h
mkdir -p $O
python -c "import torch, os; print(torch.__file__); print([f for f in os.listdir(os.path.dirname(torch.__file__)+'/lib') if 'rccl' in f])" > $O/torch_rccl.txt 2>&1
NCCL_DEBUG=INFO timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k comm_library > $O/pytest_comm.txt 2>&1
timeout -k 10 300 python -u scripts/sieve_queries.py > $O/sieve_queries.jsonl 2> $O/sieve_queries.txt
