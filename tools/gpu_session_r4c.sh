# round 4 session c: ceiling with every probe flavour, the 2-rank rehearsal line
# (n_gpus counts devices), granule sweep with proper bf16 data, C1 with the host schedule
set -u
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_run.sh bench || exit $?
run() { local name=$1 t=$2; shift 2; echo "=== $name" >> gpurun_out/steps.log
        timeout -k 10 "$t" "$@" > "gpurun_out/$name.out" 2> "gpurun_out/$name.err"; local rc=$?
        echo "=== $name rc=$rc" >> gpurun_out/steps.log; [ $rc -le 1 ] || exit $rc; }
run dist2self 300 python bench.py --gpus 2 --steps 20 --warmup 5 --no-host-leg
SWEEP_ROUNDS=8 bash tools/gpu_run.sh gran || exit $?
run c1_sched 300 python tools/c1_allreduce.py --ranks 2 --iters 200 --sched
run c1_nosched 300 python tools/c1_allreduce.py --ranks 2 --iters 200
run c1_oracle 300 python tools/c1_allreduce.py --ranks 2 --iters 200 --reduce oracle
SMALLW_ELEMS="1024 16384" SMALLW_MODES="copy copyhost memcpy" bash tools/gpu_run.sh smallw || exit $?
bash tools/gpu_run.sh smoke tests
