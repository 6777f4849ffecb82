#!/bin/bash
# round profile of the current build: plain config 5 and the keccak variant, both native code
cd $GRAFT_REPO_ROOT
bash scripts/profile.sh r02q && bash scripts/profile.sh r02q_keccak --variant keccak
