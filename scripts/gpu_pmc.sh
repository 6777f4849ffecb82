#!/bin/bash
# PMC passes over a short bench run (one pass per counter group; gfx950 slot limits per pass:
# 8 SQ, 4 TCC (FETCH_SIZE uses 3, WRITE_SIZE 2), 2 GRBM).  Run via gpurun from the repo root.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
ROWS=${1:-262144}
export TMPDIR=/tmp
B="python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --rows-per-gpu $ROWS --no-cpu-baseline"
cd /tmp
rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/pmc/counters.txt 2>&1 || true
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc/$name -o $name -- $B > $GRAFT_REPO_ROOT/gpurun_out/pmc/$name.out 2>&1
}
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU && \
run sq2 SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE GRBM_COUNT && \
run tcc1 FETCH_SIZE GRBM_GUI_ACTIVE && \
run tcc2 WRITE_SIZE
