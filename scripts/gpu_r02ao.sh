#!/bin/bash
# round profile of the build with call-site signed abs and top-column carry pruning
cd $GRAFT_REPO_ROOT
bash scripts/profile.sh r02ao --no-companion
r=$?; echo "profile: $r"; exit $r
