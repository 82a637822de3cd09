# round 5 session c: which part of the MPI user op's 4 KiB call grows with
# threads -- the fold alone (mi_host_reduce), the entry points around it, the
# reference's AVX-512 bodies -- pinned (node 0 cores, CPU 0 last) and unpinned
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5c
mkdir -p $O
CPUS=$(python -c "import sys; sys.path.insert(0,'.'); import bench; c=bench.core_plan()[1]; c=c[1:]+c[:1]; print(','.join(map(str, c[:16])))")
echo "cpus $CPUS" > $O/cpus.txt
for rep in 1 2; do
    for t in 1 8 16; do
        for mode in foldbf16 mpibf16 schedbf16 refbf16 foldfp16 mpifp16 reffp16; do
            timeout -k 10 60 ./tools/small_workers $t 2048 $mode >> $O/sw_unpinned.jsonl 2>> $O/sw.err || exit $?
            SW_CPUS=$CPUS timeout -k 10 60 ./tools/small_workers $t 2048 $mode >> $O/sw_pinned.jsonl 2>> $O/sw.err || exit $?
        done
        timeout -k 10 60 ./tools/small_workers $t 1024 sched >> $O/sw_unpinned.jsonl 2>> $O/sw.err || exit $?
        SW_CPUS=$CPUS timeout -k 10 60 ./tools/small_workers $t 1024 sched >> $O/sw_pinned.jsonl 2>> $O/sw.err || exit $?
    done
done
