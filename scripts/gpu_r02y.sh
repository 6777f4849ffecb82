#!/bin/bash
# A/B: VGPR budget (waves per SIMD) under the short circuit
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02y
mkdir -p $O
B="python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-companion"
run() {
  local tag=$1; shift
  timeout -k 10 200 $B "$@" > $O/$tag.json 2> $O/$tag.log
  r=$?; echo "$tag: $r"
  case $r in 0) ;; *) exit $r;; esac
}
run v96 --max-vgpr 96
run v128 --max-vgpr 128
run v104 --max-vgpr 104
run v168 --max-vgpr 168
