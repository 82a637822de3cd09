# round 5 session b: the MPI user-op sweep with every thread pinned to its
# own physical core (round robin over node 0's CCDs, as bench.py's CPU sweep),
# the fp32 schedule path beside it; unpinned repeats at 4 KiB; then the bench
# (L3-ordered CPU sweep) and the same bench under rocprofv3 --kernel-trace --stats
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5b
mkdir -p $O
export TMPDIR=/tmp
CPUS=$(python -c "import sys; sys.path.insert(0,'.'); import bench; print(','.join(map(str, bench.core_plan()[1][:16])))")
echo "cpus $CPUS" > $O/cpus.txt
for n in 2048 32768 262144; do
    for t in 1 8 16; do
        for mode in mpibf16 refbf16 mpifp16 reffp16 bf16 fp16; do
            SW_CPUS=$CPUS timeout -k 10 60 ./tools/small_workers $t $n $mode >> $O/small_workers_mpiop_pinned.jsonl 2>> $O/sw.err || exit $?
        done
        SW_CPUS=$CPUS timeout -k 10 60 ./tools/small_workers $t $((n / 2)) sched >> $O/small_workers_mpiop_pinned.jsonl 2>> $O/sw.err || exit $?
        SW_CPUS=$CPUS timeout -k 10 60 ./tools/small_workers $t $((n / 2)) ref >> $O/small_workers_mpiop_pinned.jsonl 2>> $O/sw.err || exit $?
    done
done
for rep in 1 2; do
    for t in 1 8 16; do
        for mode in mpibf16 refbf16 mpifp16 reffp16; do
            timeout -k 10 60 ./tools/small_workers $t 2048 $mode >> $O/small_workers_mpiop_unpinned.jsonl 2>> $O/sw.err || exit $?
        done
    done
done
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python -u bench.py > $O/bench_under_rocprofv3.json 2> $O/rocprof.err
