#!/bin/bash
# comm path through the library's own RCCL, smoke (interpreter + JIT), per-query latency
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02i
mkdir -p $O
stop() { case $1 in 124|134|137|139) echo "stop: exit $1"; exit $1;; esac; }
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k comm_library > $O/pytest_comm.txt 2>&1
r=$?; echo "comm: $r"; stop $r
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
r=$?; echo "smoke: $r"; stop $r
timeout -k 10 300 python -u scripts/sieve_queries.py > $O/sieve_queries.jsonl 2> $O/sieve_queries.txt
r=$?; echo "queries: $r"; exit $r
