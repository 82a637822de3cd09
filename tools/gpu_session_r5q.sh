# round 5 session q: the host-resident leg's calling thread on core 0, on a
# core mid-node, on the node's last core, and unpinned (which core pays)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
nodecpus=$(cat /sys/devices/system/node/node0/cpulist)
echo "node0 cpus: $nodecpus" > gpurun_out/q_host.txt
nproc >> gpurun_out/q_host.txt
python - >> gpurun_out/q_host.txt <<'PY'
import os; a=sorted(os.sched_getaffinity(0)); print(len(a), a[:8], a[-8:])
PY
for i in 1 2; do
  for c in 0 8 31 unpinned; do
    if [ $c = unpinned ]; then envs="MI_BENCH_HOST_LEG_PIN=0"; else envs="MI_BENCH_HOST_LEG_CPU=$c"; fi
    env $envs timeout -k 10 150 python bench.py --no-cpu-baseline --no-config-legs \
      > gpurun_out/q${c}_$i.json 2> gpurun_out/q${c}_$i.err || exit $?
  done
done
