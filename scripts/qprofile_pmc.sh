#!/bin/bash
# PMC passes over one pass of the query harness (scripts/sieve_queries.py, SIEVE_QUERY_REPS=1):
# per-dispatch counters of the query-path kernels (interpreter rounds, guided generator), one
# counter group per pass.  Run via gpurun from the repo root:
#   gpurun -- bash scripts/qprofile_pmc.sh <tag>
# then: python scripts/summarize_qpmc.py <tag>
cd $GRAFT_REPO_ROOT
TAG=${1:?tag}
OUT=$GRAFT_REPO_ROOT/gpurun_out/qpmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp SIEVE_QUERY_REPS=1
cd /tmp
Q="python3 $GRAFT_REPO_ROOT/scripts/sieve_queries.py"
pmc() {
  local name=$1; shift
  timeout -s KILL 180 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o $name -- $Q > $OUT/$name.out 2>&1
}
pmc q1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH && \
pmc q2 SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC && \
pmc q3 SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_IFETCH SQ_IFETCH_LEVEL SQ_INSTS_VSKIPPED GRBM_GUI_ACTIVE GRBM_COUNT && \
pmc q4 SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_DCACHE_MISSES && \
pmc q5 SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_TC_DATA_READ_REQ SQC_TC_STALL
