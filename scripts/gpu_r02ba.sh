#!/bin/bash
# final check of the round's build: full GPU suite, smoke, default bench
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02ba
mkdir -p $O
stop() { case $1 in 124|134|137|139) echo "stop: exit $1"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
r=$?; echo "pytest: $r"; tail -1 $O/pytest_gpu.txt; stop $r; [ $r -ne 0 ] && exit $r
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
r=$?; echo "smoke: $r"; stop $r; [ $r -ne 0 ] && exit $r
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.log
r=$?; echo "bench: $r"; cat $O/bench_default.json | head -c 600; exit $r
