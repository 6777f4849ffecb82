#!/bin/bash
# Round profile: kernel-trace + stats of the default bench, then PMC passes (one counter group
# per pass) over a shorter bench.  Run via gpurun from the repo root:
#   gpurun -- bash scripts/profile.sh <tag>
cd $GRAFT_REPO_ROOT
TAG=${1:-r01}
shift
EXTRA="$@"   # extra bench.py arguments (e.g. --engine interp)
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
B="python3 $GRAFT_REPO_ROOT/bench.py"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $B --steps 2 --warmup 1 --no-cpu-baseline $EXTRA > $OUT/bench_trace.json 2> $OUT/bench_trace.log || exit 1
pmc() {
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o $name -- $B --steps 1 --warmup 0 --no-cpu-baseline $EXTRA > $OUT/$name.out 2>&1
}
pmc sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU && \
pmc sq2 SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH GRBM_GUI_ACTIVE GRBM_COUNT && \
pmc tcc1 FETCH_SIZE && \
pmc tcc2 WRITE_SIZE
