# round 4 session b: granule residency sweep, full GPU suite, small workers at 4 KiB,
# bench, rocprofv3 of C2 and C4 on the final tree
set -u
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_run.sh residency gran || exit $?
bash tools/gpu_run.sh tests || exit $?
SMALLW_ELEMS="1024" SMALLW_MODES="default sched ref" bash tools/gpu_run.sh smallw || exit $?
bash tools/gpu_run.sh bench prof || exit $?
PROF_CONFIG=c4 bash tools/gpu_run.sh prof
