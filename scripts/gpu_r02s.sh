#!/bin/bash
# kernel trace of the per-query path (sieve_queries)
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r02s
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/sieve_queries.py > $O/sieve_queries.jsonl 2> $O/sieve_queries.txt
r=$?; echo "queries: $r"; exit $r
