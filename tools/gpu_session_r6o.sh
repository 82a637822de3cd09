# round 6 session o: the resident-wave plan of the final build (2-input
# kernel with buffer loads) against its neighbours over fresh placements
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6o
mkdir -p $O
timeout -k 10 600 python -u tools/residency_ab.py --trials 12 --configs c2,c3-bf16,c3-fp16,c5-int32-max,c5-int64-prod \
    > $O/residency_ab.jsonl 2> $O/residency_ab.err || exit $?
