#!/bin/bash
# per-query latency only
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02k
mkdir -p $O
MH_TRACE_COMPILE=1 timeout -k 10 300 python -u scripts/sieve_queries.py > $O/sieve_queries.jsonl 2> $O/sieve_queries.txt
r=$?; echo "queries: $r"; exit $r
