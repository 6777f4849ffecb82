#!/bin/bash
# round profile of the final build (plain and keccak variant), then the default bench
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02ax
mkdir -p $O
stop() { case $1 in 124|134|137|139) echo "stop: exit $1"; exit $1;; esac; }
bash scripts/profile.sh r02ax --no-companion && bash scripts/profile.sh r02ax_keccak --variant keccak --no-companion
r=$?; echo "profile: $r"; stop $r; [ $r -ne 0 ] && exit $r
timeout -k 10 300 python -u bench.py --variant keccak --cpu-seconds 8 > $O/bench_keccak.json 2> $O/bench_keccak.log
r=$?; echo "bench keccak: $r"; exit $r
