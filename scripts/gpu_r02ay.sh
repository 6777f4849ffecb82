#!/bin/bash
# per-query latency of the LASER-shaped queries on the current build
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02ay
mkdir -p $O
timeout -k 10 300 python -u scripts/sieve_queries.py > $O/sieve_queries.jsonl 2> $O/sieve_queries.log
r=$?; echo "queries: $r"; exit $r
