# round 6 session i: the streaming device copy with buffer loads (B) against
# the run-7 build (A), over fresh placements; the copy's GPU tests
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6i
mkdir -p $O
A=oneccl_amd/lib/ab_r7/libmi_reduce.so
B=oneccl_amd/lib/libmi_reduce.so
for lay in separate padded; do
    timeout -k 10 300 python -u tools/ab_c2.py $A $B --config copy --layout $lay --trials 10 --rounds 4 --launches 10 \
        > $O/ab_copy_$lay.jsonl 2> $O/ab_copy_$lay.err || exit $?
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_shim.py tests/test_gpu_pageable_align.py -m gpu -q -x -k "copy" \
    -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_copy.txt 2>&1 || exit $?
