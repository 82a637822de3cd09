set -u
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_run.sh residency || exit $?
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu tests/test_gpu_registry.py tests/test_gpu_shim.py tests/test_gpu_dispatch.py -k "registry or cpp_caller or registered or pinned_registration or schedule or device_memory_is_refused or stream" > gpurun_out/pytest_sel.out 2>&1; rc=$?; echo "pytest_sel rc=$rc" >> gpurun_out/steps.log; [ $rc -le 1 ] || exit $rc
bash tools/gpu_run.sh smallw || exit $?
for T in 1 16; do MI_ROCTX=0 timeout -k 10 60 ./tools/small_workers $T 1024 sched >> gpurun_out/smallw.jsonl || exit $?; done
bash tools/gpu_run.sh bench
