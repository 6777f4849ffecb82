#!/bin/bash
# full GPU suite + smoke + default bench, then the round profile of the plain workload and the
# keccak variant (kernel trace + PMC passes)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02ai
mkdir -p $O
stop() { case $1 in 124|134|137|139) echo "stop: exit $1"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
r=$?; echo "pytest: $r"; stop $r; [ $r -ne 0 ] && exit $r
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
r=$?; echo "smoke: $r"; stop $r; [ $r -ne 0 ] && exit $r
timeout -k 10 300 python -u bench.py --cpu-seconds 8 > $O/bench_default.json 2> $O/bench_default.log
r=$?; echo "bench: $r"; stop $r; [ $r -ne 0 ] && exit $r
timeout -k 10 300 python -u bench.py --variant keccak --cpu-seconds 8 > $O/bench_keccak.json 2> $O/bench_keccak.log
r=$?; echo "bench keccak: $r"; stop $r; [ $r -ne 0 ] && exit $r
bash scripts/profile.sh r02ai --no-companion && bash scripts/profile.sh r02ai_keccak --variant keccak --no-companion
r=$?; echo "profile: $r"; exit $r
