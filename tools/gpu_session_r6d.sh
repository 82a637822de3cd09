# round 6 session d: the final tree end to end -- the GPU suite, smoke, the
# default bench line, and the 2- and 8-rank rehearsals of the final bench.py
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6d
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread \
    > $O/pytest_gpu.txt 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --detail $O/bench_detail.json > $O/bench.json 2> $O/bench.err || exit $?
MI_BENCH_DETAIL=$O/bench_gpus2_detail.json timeout -k 10 400 python -u bench.py --gpus 2 --steps 20 --warmup 5 \
    > $O/bench_gpus2_rehearsal.json 2> $O/bench_gpus2_rehearsal.err || exit $?
start=$(date +%s)
MI_BENCH_DETAIL=$O/bench_gpus8_detail.json timeout -k 10 700 python -u bench.py --gpus 8 \
    > $O/bench_gpus8_rehearsal.json 2> $O/bench_gpus8_rehearsal.err || exit $?
echo "wall_s $(( $(date +%s) - start ))" > $O/bench_gpus8_wall.txt
wc -c $O/bench.json $O/bench_gpus2_rehearsal.json $O/bench_gpus8_rehearsal.json >> $O/bench_gpus8_wall.txt
