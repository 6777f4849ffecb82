#!/bin/bash
# JIT suite + handle-lifetime test, then the round profile (plain + keccak variant)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02r
mkdir -p $O
stop() { case $1 in 124|134|137|139) echo "stop: exit $1"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_jit.py tests/test_gpu_parity.py -k "jit or handles" -x -v --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1
r=$?; echo "pytest: $r"; stop $r; [ $r -ne 0 ] && exit $r
bash scripts/profile.sh r02r && bash scripts/profile.sh r02r_keccak --variant keccak
r=$?; echo "profile: $r"; exit $r
