# round 5 session p: the host-resident leg with its calling thread pinned to a
# GPU-local core (the default) against unpinned, three processes each,
# alternating (profiles/round5_run12/host_leg_pin_ab.jsonl)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2 3; do
  for pin in 1 0; do
    MI_BENCH_HOST_LEG_PIN=$pin timeout -k 10 150 python bench.py --no-cpu-baseline --no-config-legs \
      > gpurun_out/pin${pin}_$i.json 2> gpurun_out/pin${pin}_$i.err || exit $?
  done
done
