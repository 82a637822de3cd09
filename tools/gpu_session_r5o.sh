# round 5 session o: the headline with 10 against 400 untimed warm-up launches,
# three processes each (profiles/round5_run11/warmup_ab.jsonl)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2 3; do
  for w in 10 400; do
    timeout -k 10 120 python bench.py --warmup $w --no-cpu-baseline --no-host-leg --no-config-legs > gpurun_out/w${w}_$i.json 2> gpurun_out/w${w}_$i.err || exit $?
  done
done
