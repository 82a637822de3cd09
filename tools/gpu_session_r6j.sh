# round 6 session j: the default bench line of the final build on another box
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6j_$(date +%s)
mkdir -p $O
timeout -k 10 600 python -u bench.py --detail $O/bench_detail.json > $O/bench.json 2> $O/bench.err || exit $?
