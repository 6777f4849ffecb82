#!/bin/bash
# keccak lane complementing: JIT GPU suite, keccak-variant bench A/B, issue rates of
# xnor/and/or/not, and the two-process shard check
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02af
mkdir -p $O
stop() { case $1 in 124|134|137|139) echo "stop: exit $1"; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_jit.py -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu_jit.txt 2>&1
r=$?; echo "pytest jit: $r"; stop $r; [ $r -ne 0 ] && exit $r
for c in 1 0 1; do
  MH_JIT_KEC_COMPLEMENT=$c timeout -k 10 240 python -u bench.py --variant keccak --steps 5 --no-companion --no-cpu-baseline > $O/bench_keccak_c$c.json 2> $O/bench_keccak_c$c.log
  r=$?; echo "bench keccak complement=$c: $r"; stop $r; [ $r -ne 0 ] && exit $r
  python -c "import json; d=json.load(open('$O/bench_keccak_c$c.json')); print('$c', d['value'], d['kernel_ms'], d['tapes_with_witness'])"
done
timeout -k 10 120 python -u -c "
import json
from mythril_amd import native
ctx = native.Context(0)
out = {}
for k in range(17, len(native.MB_KINDS)):
    out[native.MB_KINDS[k]] = {w: 1024 * 2.4e9 * 64 / ctx.microbench(k, w) for w in (2, 4, 8)}
print(json.dumps({'cycles_per_wave_insn': out}))
" > $O/valu_kinds.json 2> $O/valu_kinds.log
r=$?; echo "microbench: $r"; cat $O/valu_kinds.json; stop $r; [ $r -ne 0 ] && exit $r
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 tests/tools/shard_check.py 65536 > $O/shard_check.json 2> $O/shard_check.log
r=$?; echo "shard_check: $r"; cat $O/shard_check.json; exit $r
