#!/bin/bash
# keccak variant: does occupancy matter?  all code objects padded to 168 VGPRs (3 waves/SIMD) and
# 256 (2 waves) vs the default (1/3 of the tapes at 4 waves, the rest at 3)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02ak
mkdir -p $O
stop() { case $1 in 124|134|137|139) echo "stop: exit $1"; exit $1;; esac; }
for p in 0 168 256; do
  MH_JIT_PAD_VGPR=$p timeout -k 10 240 python -u bench.py --variant keccak --steps 5 --no-companion --no-cpu-baseline > $O/bench_keccak_pad$p.json 2> $O/bench_keccak_pad$p.log
  r=$?; echo "bench keccak pad=$p: $r"; stop $r; [ $r -ne 0 ] && exit $r
  python -c "import json; d=json.load(open('$O/bench_keccak_pad$p.json')); print('$p', d['value'], d['kernel_ms'], d['jit']['max_vgpr'])"
done
exit 0
