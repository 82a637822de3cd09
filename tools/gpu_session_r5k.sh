# round 5 session k: the final tree's measurements
#  1. the small-host-chunk sweep after the snapshot fix (MPI user ops, the
#     schedule path, the reference's own code), 4/64/512 KiB x 1/8/16 threads
#  2. bench.py (default line)
#  3. the 8-rank rehearsal: python bench.py --gpus 8 on this one-GPU box
#     (VERDICT r4 item 4), wall time recorded
#  4. rocprofv3 --kernel-trace --stats of the C2 and C4 bench commands
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5k
mkdir -p $O
export TMPDIR=/tmp
for n in 2048 32768 262144; do
    for t in 1 8 16; do
        for mode in mpibf16 refbf16 bf16 mpifp16 reffp16 fp16; do
            timeout -k 10 60 ./tools/small_workers $t $n $mode >> $O/small_workers_after_fix.jsonl 2>> $O/sw.err || exit $?
        done
        for mode in sched ref default; do
            timeout -k 10 60 ./tools/small_workers $t $((n / 2)) $mode >> $O/small_workers_after_fix.jsonl 2>> $O/sw.err || exit $?
        done
    done
done
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
t0=$(date +%s.%N)
timeout -k 10 900 python -u bench.py --gpus 8 > $O/bench_gpus8_rehearsal.json 2> $O/bench_gpus8_rehearsal.err
rc=$?
t1=$(date +%s.%N)
echo "{\"rc\": $rc, \"wall_s\": $(python -c "print(round($t1 - $t0, 2))")}" > $O/bench_gpus8_wall.json
[ $rc -eq 0 ] || exit $rc
for pc in c2 c4; do
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/prof_$pc" -o bench -- \
        python3 "$GRAFT_REPO_ROOT/bench.py" --config $pc --steps 20 --warmup 5 --no-cpu-baseline --no-host-leg --no-config-legs \
        > "$GRAFT_REPO_ROOT/$O/prof_$pc.out" 2> "$GRAFT_REPO_ROOT/$O/prof_$pc.err") || exit $?
done
# 5. HBM bytes per launch of the C2 and C4 kernels: FETCH_SIZE and WRITE_SIZE
#    in separate --pmc passes (MI355X_MICROARCH.md, HBM / rocprofv3)
for pc in c2 c4; do
    for ctr in FETCH_SIZE WRITE_SIZE; do
        (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc $ctr --output-format csv -d "$GRAFT_REPO_ROOT/$O/pmc_$pc/pmc_$ctr" -o bench -- \
            python3 "$GRAFT_REPO_ROOT/bench.py" --config $pc --steps 5 --warmup 2 --no-cpu-baseline --no-host-leg --no-config-legs \
            > "$GRAFT_REPO_ROOT/$O/pmc_${pc}_$ctr.out" 2> "$GRAFT_REPO_ROOT/$O/pmc_${pc}_$ctr.err") || exit $?
    done
done
