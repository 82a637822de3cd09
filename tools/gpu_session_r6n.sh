# round 6 session n: C5's size sweep (4 KiB - 1 GiB) on the final build
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6n
mkdir -p $O
timeout -k 10 600 python -u tools/size_sweep.py > $O/size_sweep.jsonl 2> $O/size_sweep.err || exit $?
