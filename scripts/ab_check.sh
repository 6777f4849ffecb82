#!/bin/bash
# A/B of two builds of libmythril_hip on the GPU box: exact results at full occupancy (all tapes
# of config 5 over DIAG_ROWS rows; counts and witnesses in count-all mode, witnesses in first-hit
# mode), then the default bench for each.
#   gpurun -- bash scripts/ab_check.sh build/ab/lib_a.so mythril_amd/libmythril_hip.so
cd $GRAFT_REPO_ROOT
A=${1:?lib A}; B=${2:?lib B}
OUT=gpurun_out/ab
mkdir -p $OUT
export DIAG_ROWS=${DIAG_ROWS:-1048576}
MYTHRIL_HIP_LIB=$PWD/$A DIAG_OUT=$OUT/a timeout -k 10 240 python -u scripts/diag_modes.py > $OUT/diag_a.log 2>&1 && \
MYTHRIL_HIP_LIB=$PWD/$B DIAG_OUT=$OUT/b timeout -k 10 240 python -u scripts/diag_modes.py > $OUT/diag_b.log 2>&1 && \
python -c "
import numpy as np, sys
for m in ('count', 'first'):
    a = np.load('$OUT/a_%s.npy' % m); b = np.load('$OUT/b_%s.npy' % m)
    if m == 'first':  # first-hit mode: witnesses exact; counts stop early, timing-dependent
        a, b = a[0], b[0]
    print(m, 'identical' if np.array_equal(a, b) else 'DIFFER (%d entries)' % int((a != b).sum()))
    if not np.array_equal(a, b): sys.exit(1)
" > $OUT/compare.log 2>&1 && \
MYTHRIL_HIP_LIB=$PWD/$A timeout -k 10 300 python -u bench.py --no-cpu-baseline $BENCH_ARGS > $OUT/bench_a.json 2> $OUT/bench_a.log && \
MYTHRIL_HIP_LIB=$PWD/$B timeout -k 10 300 python -u bench.py --no-cpu-baseline $BENCH_ARGS > $OUT/bench_b.json 2> $OUT/bench_b.log
