# round 4 session n: 256 MiB operands (C3's bucket) in one allocation at
# operand offsets 256 (contiguous), 1152 (the padded gap of 896 MiB) and
# 1920 MiB, and separate allocations
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for g in 0 896 1664 1152; do
    timeout -k 10 120 python tools/placement_probe.py --inputs 2 --bucket-mib 256 --trials 8 --launches 20 \
        --layout one --gap-mib $g > gpurun_out/b256_gap_$g.out 2> gpurun_out/b256_gap_$g.err || exit $?
done
timeout -k 10 120 python tools/placement_probe.py --inputs 2 --bucket-mib 256 --trials 12 --launches 20 \
    > gpurun_out/b256_separate.out 2> gpurun_out/b256_separate.err
