#!/bin/bash
# full GPU suite, smoke, default bench (round-end rehearsal)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02n
mkdir -p $O
stop() { case $1 in 124|134|137|139) echo "stop: exit $1"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
r=$?; echo "pytest: $r"; stop $r
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
r=$?; echo "smoke: $r"; stop $r
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.log
r=$?; echo "bench: $r"; exit $r
