cd $GRAFT_REPO_ROOT && bash scripts/gpu_run.sh r03w gpu smoke queries profile bench
