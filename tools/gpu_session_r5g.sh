# round 5 session g: TSC cycles inside the fold vs the whole call (diagnostic shim build)
# (historical: the diagnostic shim builds under tools/diag_* that this session loaded were
# one-off variants of comp.cpp and are not kept; results: profiles/round5_host/isolate_*)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5g
mkdir -p $O
CPUS=$(python -c "import sys; sys.path.insert(0,'.'); import bench; c=bench.core_plan()[1]; c=c[1:]+c[:1]; print(','.join(map(str, c[:16])))")
for t in 1 8 16; do
    for mode in schedbf16 schedi16; do
        LD_LIBRARY_PATH=tools/diag_tsc SW_CPUS=$CPUS timeout -k 10 60 ./tools/small_workers $t 2048 $mode >> $O/sw.jsonl 2>> $O/diag.txt || exit $?
    done
done
