# round 6 session b: access patterns other than the fan-in's own, for the C4
# and C2 traffic (tools/c4_pattern_probe.py), then the 8-rank rehearsal of the
# final bench.py on this one GPU
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6b
mkdir -p $O
timeout -k 10 300 python -u tools/c4_pattern_probe.py --k 8 > $O/c4_patterns.jsonl 2> $O/c4_patterns.err || exit $?
timeout -k 10 300 python -u tools/c4_pattern_probe.py --k 2 --layouts padded,separate > $O/c2_patterns.jsonl \
    2> $O/c2_patterns.err || exit $?
start=$(date +%s)
MI_BENCH_DETAIL=$O/bench_gpus8_detail.json timeout -k 10 700 python -u bench.py --gpus 8 \
    > $O/bench_gpus8_rehearsal.json 2> $O/bench_gpus8_rehearsal.err || exit $?
echo "wall_s $(( $(date +%s) - start ))" > $O/bench_gpus8_wall.txt
wc -c $O/bench_gpus8_rehearsal.json >> $O/bench_gpus8_wall.txt
