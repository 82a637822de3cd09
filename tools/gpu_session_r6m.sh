# round 6 session m: the final tree's GPU suite and smoke, as the driver runs them
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6m
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread \
    > $O/pytest_gpu.txt 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
