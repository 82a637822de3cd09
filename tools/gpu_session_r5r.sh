# round 5 session r: a confined caller's staged buckets on its worker
# (mi_reduce.hip sync_entry): the tests, then the host leg with the calling
# thread pinned to one core, hand-off on (default) and off, alternating
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_context_pool.py tests/test_gpu_pageable_align.py -m gpu -q \
  -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r_tests.out 2>&1 || exit $?
for i in 1 2; do
  for h in 1 0; do
    MI_BENCH_HOST_LEG_PIN=1 MI_REDUCE_CONFINED_HANDOFF=$h timeout -k 10 150 python bench.py --no-cpu-baseline \
      --no-config-legs > gpurun_out/h${h}_$i.json 2> gpurun_out/h${h}_$i.err || exit $?
  done
done
