# round 6 session h: the final build (2-input kernel with buffer loads):
# PMC traffic and rocprofv3 of C2 / C4 on the new device code, the GPU suite,
# smoke and the default bench line
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6h
mkdir -p $O
bash tools/gpu_run.sh pmc || exit $?
PMC_CONFIG=c4 bash tools/gpu_run.sh pmc pmcjson || exit $?
bash tools/gpu_run.sh prof || exit $?
PROF_CONFIG=c4 bash tools/gpu_run.sh prof || exit $?
mkdir -p profiles/round6_run7 && cp gpurun_out/pmc.json profiles/round6_run7/pmc.json || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread \
    > $O/pytest_gpu.txt 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --detail $O/bench_detail.json > $O/bench.json 2> $O/bench.err || exit $?
