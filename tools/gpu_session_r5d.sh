# round 5 session d: the 4 KiB call through ccl_comp_reduce under a host
# schedule for fp32 (4 and 8 KiB), int16, bf16 (avx512bf and avx512f flags)
# and fp16, pinned one thread per CCD: which dtypes grow with threads
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5d
mkdir -p $O
CPUS=$(python -c "import sys; sys.path.insert(0,'.'); import bench; c=bench.core_plan()[1]; c=c[1:]+c[:1]; print(','.join(map(str, c[:16])))")
for rep in 1 2; do
    for t in 1 8 16; do
        for mode in "sched 1024" "sched 2048" "schedi16 2048" "schedbf16 2048" "schedfp16 2048" "foldbf16 2048"; do
            set -- $mode
            SW_CPUS=$CPUS timeout -k 10 60 ./tools/small_workers $t $2 $1 >> $O/sw.jsonl 2>> $O/sw.err || exit $?
        done
        CCL_BF16=avx512f SW_CPUS=$CPUS timeout -k 10 60 ./tools/small_workers $t 2048 schedbf16 | sed 's/schedbf16/schedbf16-avx512f/' >> $O/sw.jsonl 2>> $O/sw.err || exit $?
        CCL_BF16=scalar SW_CPUS=$CPUS timeout -k 10 60 ./tools/small_workers $t 2048 schedbf16 | sed 's/schedbf16/schedbf16-scalar/' >> $O/sw.jsonl 2>> $O/sw.err || exit $?
    done
done
