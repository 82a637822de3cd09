# round 5 session t: PMC traffic (FETCH_SIZE / WRITE_SIZE passes) and
# rocprofv3 kernel stats for C2 and C4 on the final build (the copy kernel's
# change moved the device-code hash, so the earlier passes went stale)
set -u
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_run.sh pmc || exit $?
PMC_CONFIG=c4 bash tools/gpu_run.sh pmc pmcjson || exit $?
bash tools/gpu_run.sh prof || exit $?
PROF_CONFIG=c4 bash tools/gpu_run.sh prof || exit $?
