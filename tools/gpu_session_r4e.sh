# round 4 session e: does the operands' relative alignment set C2's slow mode?
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python tools/placement_probe.py --inputs 2 --trials 16 --offsets > gpurun_out/placement_offsets.out 2> gpurun_out/placement_offsets.err
