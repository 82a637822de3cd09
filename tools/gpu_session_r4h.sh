# round 4 session h: the final tree end to end -- smoke, the whole GPU suite,
# the headline bench, kernel-trace profiles of C2 and C4, C2's PMC bytes
set -u
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_run.sh host smoke tests bench prof || exit $?
PROF_CONFIG=c4 bash tools/gpu_run.sh prof || exit $?
bash tools/gpu_run.sh pmc
