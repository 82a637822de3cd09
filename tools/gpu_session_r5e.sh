# round 5 session e: diagnostic pairs for the 4 KiB bf16 call's growth
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5e
mkdir -p $O
CPUS=$(python -c "import sys; sys.path.insert(0,'.'); import bench; c=bench.core_plan()[1]; c=c[1:]+c[:1]; print(','.join(map(str, c[:16])))")
for rep in 1 2; do
    for t in 1 16; do
        for mode in foldi16 foldbf16 schedi16 schedbf16 schedi16+foldbf16 foldi16+foldbf16 schedi16x2; do
            SW_CPUS=$CPUS timeout -k 10 60 ./tools/small_workers $t 2048 $mode >> $O/sw.jsonl 2>> $O/sw.err || exit $?
        done
    done
done
