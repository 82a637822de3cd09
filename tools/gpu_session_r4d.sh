# round 4 session d: placement spread of C2 and C4 over fresh allocations; new GPU tests
set -u
cd "$GRAFT_REPO_ROOT"
run() { local name=$1 t=$2; shift 2; echo "=== $name" >> gpurun_out/steps.log
        timeout -k 10 "$t" "$@" > "gpurun_out/$name.out" 2> "gpurun_out/$name.err"; local rc=$?
        echo "=== $name rc=$rc" >> gpurun_out/steps.log; [ $rc -le 1 ] || exit $rc; }
run placement_c2 300 python tools/placement_probe.py --inputs 2 --trials 16
run placement_c4 300 python tools/placement_probe.py --inputs 8 --trials 12
run pytest_registry 300 python -u -m pytest -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests/test_gpu_registry.py
