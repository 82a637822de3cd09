# round 6 session e: the 2-rank self-launched bench after moving native
# rendezvous notes off stdout (stdout must hold the one JSON line)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6e
mkdir -p $O
MI_BENCH_DETAIL=$O/bench_gpus2_detail.json timeout -k 10 400 python -u bench.py --gpus 2 --steps 20 --warmup 5 \
    --no-cpu-baseline > $O/bench_gpus2.json 2> $O/bench_gpus2.err || exit $?
wc -l $O/bench_gpus2.json
