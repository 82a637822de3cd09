# round 5 session s: ccl_comp_copy's streaming variant (sc1 nt stores,
# >= 64 MiB): its tests, the copy A/B, and the bench line's f3-copy leg
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_shim.py -m gpu -q -k "copy" -p no:cacheprovider --timeout 120 \
  --timeout-method thread > gpurun_out/s_tests.out 2>&1 || exit $?
timeout -k 10 240 python tools/copy_ab.py > gpurun_out/copy_ab_after.jsonl 2> gpurun_out/copy_ab_after.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-leg > gpurun_out/s_bench.json 2> gpurun_out/s_bench.err
