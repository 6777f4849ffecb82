#!/bin/bash
# A/B: number of code objects (launches per step) at 96 KB groups; keccak variant group size
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02y
mkdir -p $O
B="python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-companion"
run() {
  local tag=$1; shift
  E=$1; shift
  A="$@"
  env $E timeout -k 10 200 $B $A > $O/$tag.json 2> $O/$tag.log
  r=$?; echo "$tag: $r"
  case $r in 0) ;; *) exit $r;; esac
}
run t16 MH_JIT_THREADS=16
run t4 MH_JIT_THREADS=4
run t1 MH_JIT_THREADS=1
run k96 MH_JIT_GROUP_KB=96 --variant keccak
run k40 MH_JIT_GROUP_KB=40 --variant keccak
