# round 6 session g: the 2-input kernel with buffer loads (B) against the
# round-5 build with global loads (A, oneccl_amd/lib/ab_global/), over fresh
# placements, per config; then the GPU parity tests of the 2-input paths
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6g
mkdir -p $O
A=oneccl_amd/lib/ab_global/libmi_reduce.so
B=oneccl_amd/lib/libmi_reduce.so
for spec in "c2 separate" "c2 padded" "c3-bf16 separate" "c5-int64-prod separate" "c5-int32-max separate"; do
    set -- $spec
    timeout -k 10 300 python -u tools/ab_c2.py $A $B --config $1 --layout $2 --trials 10 --rounds 4 --launches 10 \
        > $O/ab_$1_$2.jsonl 2> $O/ab_$1_$2.err || exit $?
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ref_comp_vectors.py tests/test_gpu_ref_vectors.py \
    tests/test_gpu_nan.py tests/test_gpu_batch.py tests/test_gpu_fuzz.py -m gpu -q -x -p no:cacheprovider --timeout 300 \
    --timeout-method thread > $O/pytest_r2.txt 2>&1 || exit $?
