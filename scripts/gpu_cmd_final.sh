cd $GRAFT_REPO_ROOT && bash scripts/gpu_run.sh r03r gpu smoke queries bench
