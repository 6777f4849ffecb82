#!/bin/bash
# two processes on one GPU: shard results of the native code reduced over gloo vs one launch + C oracle
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02ae
mkdir -p $O
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 tests/tools/shard_check.py 65536 > $O/shard_check.json 2> $O/shard_check.log
r=$?; echo "shard_check: $r"; cat $O/shard_check.json; exit $r
