#!/bin/bash
# Round profile: kernel-trace + stats of the bench, then PMC passes (one counter group per pass)
# over a one-step bench.  Run via gpurun from the repo root:
#   gpurun -- bash scripts/profile.sh <tag> [bench.py arguments, e.g. --full-eval]
# The companion full-evaluation step and the CPU baseline are off here, so every mh_jit launch
# counted belongs to the profiled mode.  Then: python scripts/summarize_profile.py <tag>
cd $GRAFT_REPO_ROOT
TAG=${1:-r01}
shift
EXTRA="$@"
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
B="python3 $GRAFT_REPO_ROOT/bench.py --no-companion --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $B --steps 2 --warmup 1 $EXTRA > $OUT/bench_trace.json 2> $OUT/bench_trace.log || exit 1
pmc() {
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o $name -- $B --steps 1 --warmup 0 $EXTRA > $OUT/$name.out 2>&1
}
pmc sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU && \
pmc sq2 SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH GRBM_GUI_ACTIVE GRBM_COUNT && \
pmc sq3 SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_WAIT_INST_LDS SQ_INSTS_VSKIPPED SQ_IFETCH SQ_IFETCH_LEVEL && \
pmc tcc1 FETCH_SIZE && \
pmc tcc2 WRITE_SIZE && \
pmc sqc1 SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE && \
pmc sqc2 SQC_TC_INST_REQ SQC_ICACHE_BUSY_CYCLES SQC_TC_STALL SQC_DCACHE_MISSES
