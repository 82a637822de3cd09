# round 4 session j: C2 in one allocation, the gap between the operands swept
# over 0-3 GiB in 128 MiB steps
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for g in $(seq 0 128 3072); do
    timeout -k 10 120 python tools/placement_probe.py --inputs 2 --trials 4 --launches 10 --layout one --gap-mib $g \
        > gpurun_out/gapsweep_$g.out 2> gpurun_out/gapsweep_$g.err || exit $?
done
