# round 5 session i: the MPI user op's 4 KiB call after the env snapshot and
# shard list were given whole cache lines, pinned and unpinned
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5i
mkdir -p $O
CPUS=$(python -c "import sys; sys.path.insert(0,'.'); import bench; c=bench.core_plan()[1]; c=c[1:]+c[:1]; print(','.join(map(str, c[:16])))")
for rep in 1 2; do
    for t in 1 8 16; do
        for mode in mpibf16 mpifp16 schedbf16 refbf16 reffp16; do
            SW_CPUS=$CPUS timeout -k 10 60 ./tools/small_workers $t 2048 $mode | sed "s/\"mode\": \"/\"mode\": \"pinned:/" >> $O/sw.jsonl 2>> $O/sw.err || exit $?
            timeout -k 10 60 ./tools/small_workers $t 2048 $mode >> $O/sw.jsonl 2>> $O/sw.err || exit $?
        done
    done
done
