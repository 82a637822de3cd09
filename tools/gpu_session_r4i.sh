# round 4 session i: C2 with both operands in one allocation at several gaps
# between them, against separate allocations, on one box
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for g in 0 2 64 256 512 1024; do
    timeout -k 10 150 python tools/placement_probe.py --inputs 2 --trials 8 --layout one --gap-mib $g \
        > gpurun_out/gap_$g.out 2> gpurun_out/gap_$g.err || exit $?
done
timeout -k 10 150 python tools/placement_probe.py --inputs 2 --trials 12 > gpurun_out/gap_sep.out 2> gpurun_out/gap_sep.err
