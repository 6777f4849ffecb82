#!/bin/bash
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02g
mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_parity.py -k "comm_library" > $O/pytest_comm.txt 2>&1 && \
timeout -k 10 300 python -u scripts/sieve_queries.py > $O/sieve_queries.jsonl 2> $O/sieve_queries.txt && \
timeout -k 10 300 python -u scripts/sieve_queries.py > $O/sieve_queries2.jsonl 2> $O/sieve_queries2.txt
