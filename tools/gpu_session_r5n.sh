# round 5 session n: the C5 size sweep (4 KiB - 1 GiB, fp32 sum / int32 max /
# int64 prod) on the final tree, and bench.py with the C1 leg under a host schedule
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5n
mkdir -p $O
timeout -k 10 600 python -u tools/size_sweep.py > $O/size_sweep.jsonl 2> $O/size_sweep.err || exit $?
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err
