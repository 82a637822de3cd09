# round 4 session l: the final tree (smoke, GPU suite, bench, rocprofv3 of C2
# and C4, C2 PMC) and the padded layout's offset re-checked on this box
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
{ hostname; rocm-smi --showuniqueid 2>&1 | grep -i unique | head -2; } > gpurun_out/box.txt 2>&1
bash tools/gpu_run.sh host smoke tests bench prof || exit $?
PROF_CONFIG=c4 bash tools/gpu_run.sh prof || exit $?
bash tools/gpu_run.sh pmc || exit $?
for g in 0 896 1152 1920; do
    timeout -k 10 120 python tools/placement_probe.py --inputs 2 --trials 6 --launches 10 --layout one --gap-mib $g \
        > gpurun_out/k2_gap_$g.out 2> gpurun_out/k2_gap_$g.err || exit $?
done
timeout -k 10 150 python tools/placement_probe.py --inputs 2 --trials 10 --launches 10 \
    > gpurun_out/k2_separate.out 2> gpurun_out/k2_separate.err
