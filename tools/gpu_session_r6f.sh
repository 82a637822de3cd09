# round 6 session f: the 2-input kernel's load form (global vs buffer nt
# loads) and residency over fresh placements (tools/r2_load_ab.py)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6f
mkdir -p $O
timeout -k 10 400 python -u tools/r2_load_ab.py --trials 16 --launches 20 > $O/r2_load_ab.jsonl 2> $O/r2_load_ab.err || exit $?
