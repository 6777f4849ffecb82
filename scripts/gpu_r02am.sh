#!/bin/bash
# profile of the full evaluation (no short circuit) for this build
cd $GRAFT_REPO_ROOT
bash scripts/profile.sh r02am_full --full-eval --no-companion
r=$?; echo "profile: $r"; exit $r
