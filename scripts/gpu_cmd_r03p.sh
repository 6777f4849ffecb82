cd $GRAFT_REPO_ROOT && bash scripts/gpu_run.sh r03p gpu smoke queries
