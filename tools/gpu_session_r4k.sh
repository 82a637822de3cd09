# round 4 session k: the operand gap on another box (C2) and for the 8-input fan-in
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for g in 0 128 896 1152 1920; do
    timeout -k 10 120 python tools/placement_probe.py --inputs 2 --trials 6 --launches 10 --layout one --gap-mib $g \
        > gpurun_out/k2_gap_$g.out 2> gpurun_out/k2_gap_$g.err || exit $?
done
timeout -k 10 150 python tools/placement_probe.py --inputs 2 --trials 12 --launches 10 \
    > gpurun_out/k2_separate.out 2> gpurun_out/k2_separate.err || exit $?
for g in 0 128 384 896; do
    timeout -k 10 200 python tools/placement_probe.py --inputs 8 --trials 4 --launches 10 --layout one --gap-mib $g \
        > gpurun_out/k8_gap_$g.out 2> gpurun_out/k8_gap_$g.err || exit $?
done
