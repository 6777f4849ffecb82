#!/bin/bash
# round profile of the current build: plain config 5 (JIT) and the keccak variant
cd $GRAFT_REPO_ROOT
bash scripts/profile.sh r02m && bash scripts/profile.sh r02m_keccak --variant keccak
