# round 6 session e: the bench after routing everything but the JSON line
# off stdout: the default N = 1 line and the 2-rank self-launched line must
# each be exactly one line on stdout
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6e
mkdir -p $O
timeout -k 10 400 python -u bench.py --detail $O/bench_detail.json > $O/bench.json 2> $O/bench.err || exit $?
MI_BENCH_DETAIL=$O/bench_gpus2_detail.json timeout -k 10 400 python -u bench.py --gpus 2 --steps 20 --warmup 5 \
    --no-cpu-baseline > $O/bench_gpus2.json 2> $O/bench_gpus2.err || exit $?
wc -l $O/bench.json $O/bench_gpus2.json
