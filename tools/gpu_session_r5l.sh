# round 5 session l: the small-host-chunk sweep with the harness's mode
# resolved outside the timed loop, and bench.py (memory plan vs measured)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5l
mkdir -p $O
for n in 2048 32768 262144; do
    for t in 1 8 16; do
        for mode in mpibf16 refbf16 bf16 mpifp16 reffp16 fp16; do
            timeout -k 10 60 ./tools/small_workers $t $n $mode >> $O/small_workers.jsonl 2>> $O/sw.err || exit $?
        done
        for mode in sched ref default copyhost memcpy; do
            timeout -k 10 60 ./tools/small_workers $t $((n / 2)) $mode >> $O/small_workers.jsonl 2>> $O/sw.err || exit $?
        done
    done
done
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
