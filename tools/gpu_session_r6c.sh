# round 6 session c: the changed paths' GPU tests, smoke, then rocprofv3
# kernel stats and the PMC traffic passes of C2 and C4 for round 6's record
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6c
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_context_pool.py tests/test_gpu_copy_fault_injection.py \
    tests/test_gpu_pageable_align.py tests/test_gpu_registry.py -m gpu -v -p no:cacheprovider --timeout 120 \
    --timeout-method thread > $O/pytest_changed.txt 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
bash tools/gpu_run.sh pmc || exit $?
PMC_CONFIG=c4 bash tools/gpu_run.sh pmc pmcjson || exit $?
bash tools/gpu_run.sh prof || exit $?
PROF_CONFIG=c4 bash tools/gpu_run.sh prof || exit $?
