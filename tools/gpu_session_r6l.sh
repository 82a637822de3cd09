# round 6 session l: the CPU baseline with the timing cores cleared of every
# other thread (this process's and the other ranks'): the default line, and
# the 8-rank rehearsal
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6l
mkdir -p $O
timeout -k 10 600 python -u bench.py --detail $O/bench_detail.json > $O/bench.json 2> $O/bench.err || exit $?
start=$(date +%s)
MI_BENCH_DETAIL=$O/bench_gpus8_detail.json timeout -k 10 700 python -u bench.py --gpus 8 \
    > $O/bench_gpus8_rehearsal.json 2> $O/bench_gpus8_rehearsal.err || exit $?
echo "wall_s $(( $(date +%s) - start ))" > $O/bench_gpus8_wall.txt
