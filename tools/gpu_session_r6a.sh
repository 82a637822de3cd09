# round 6 session a: the GPU suite (new: injected copy failures, the confined
# hand-off's device), then the full default bench with its compact line and
# the side file
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6a
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread \
    > $O/pytest_gpu.txt 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --detail $O/bench_detail.json > $O/bench.json 2> $O/bench.err || exit $?
wc -c $O/bench.json
