#!/bin/bash
# issue rates with partial EXEC masks (kinds 21-24) next to the full-mask kinds
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02aj
mkdir -p $O
timeout -k 10 180 python -u -c "
import json
from mythril_amd import native
ctx = native.Context(0)
out = {}
for k in [3, 4] + list(range(17, len(native.MB_KINDS))):
    out[native.MB_KINDS[k]] = {w: round(1024 * 2.4e9 * 64 / ctx.microbench(k, w), 3) for w in (2, 4, 8)}
print(json.dumps({'cycles_per_wave_insn': out}))
" > $O/valu_exec.json 2> $O/valu_exec.log
r=$?; echo "microbench: $r"; cat $O/valu_exec.json; [ $r -ne 0 ] && exit $r
timeout -k 10 180 python -u -m pytest tests/test_gpu_parity.py -k microbench -x -v --timeout 120 --timeout-method thread > $O/pytest_mb.txt 2>&1
r=$?; echo "pytest: $r"; tail -2 $O/pytest_mb.txt; exit $r
