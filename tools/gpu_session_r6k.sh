# round 6 session k: the 8- and 2-rank rehearsals of the final bench.py on
# the final build, wall time against the 600 s limit
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6k
mkdir -p $O
start=$(date +%s)
MI_BENCH_DETAIL=$O/bench_gpus8_detail.json timeout -k 10 700 python -u bench.py --gpus 8 \
    > $O/bench_gpus8_rehearsal.json 2> $O/bench_gpus8_rehearsal.err || exit $?
echo "wall_s $(( $(date +%s) - start ))" > $O/bench_gpus8_wall.txt
MI_BENCH_DETAIL=$O/bench_gpus2_detail.json timeout -k 10 400 python -u bench.py --gpus 2 \
    > $O/bench_gpus2_rehearsal.json 2> $O/bench_gpus2_rehearsal.err || exit $?
wc -lc $O/bench_gpus8_rehearsal.json $O/bench_gpus2_rehearsal.json >> $O/bench_gpus8_wall.txt
