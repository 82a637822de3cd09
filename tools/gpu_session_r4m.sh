# round 4 session m: the final tree once more -- smoke, the whole GPU suite, the default bench
set -u
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_run.sh host smoke tests bench
