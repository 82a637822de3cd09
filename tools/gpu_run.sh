#!/usr/bin/env bash
# GPU-box session script: every GPU step under its own timeout; stop at the
# first fault / abort / segfault / timeout (exit codes 124 134 137 139 or a
# signal), continue past ordinary test failures (pytest exit 1).
# Usage: tools/gpu_run.sh STEP [STEP ...]   steps: host tests sweep bench prof pmc benchall
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp

run() {  # run NAME TIMEOUT CMD...
    local name=$1 t=$2; shift 2
    echo "=== $name: $*" | tee -a "$OUT/steps.log"
    timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
    local rc=$?
    echo "=== $name rc=$rc" | tee -a "$OUT/steps.log"
    case $rc in
        0|1) return 0 ;;       # ok / test failures: keep going
        *) echo "STOP: $name exited $rc" | tee -a "$OUT/steps.log"; exit $rc ;;
    esac
}

for step in "$@"; do
    case $step in
        host)
            { nproc; lscpu; rocm-smi --showproductname --showmeminfo vram 2>&1 | head -40; } > "$OUT/host.txt" 2>&1 ;;
        tests)
            run pytest_gpu 1000 python -u -m pytest tests -m gpu -q --maxfail=50 -p no:cacheprovider --timeout 300 --timeout-method thread ;;
        tests_fast)
            run pytest_gpu 600 python -m pytest tests -m gpu -q --maxfail=50 -p no:cacheprovider -k "not full" ;;
        asan)
            run asan_build 600 python -m oneccl_amd.build --asan &&
            ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:quarantine_size_mb=0 run asan 300 ./tests/cpp/dropin_caller_asan &&
            run pytest_asan 300 python -m pytest tests/test_gpu_shim.py -m gpu -q -k asan -p no:cacheprovider ;;
        latency)
            run latency 300 ./tools/latency 2000 ;;
        smoke)
            run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
        sweep)
            run sweep 300 ./tools/reduce_sweep 1024 ${SWEEP_ROUNDS:-3} 10 ;;
        fansweep)
            run fansweep 300 ./tools/fan_sweep 1024 ${SWEEP_ROUNDS:-4} 8 ;;
        burst)
            run burst 300 ./tools/burst_sweep 1024 ${SWEEP_ROUNDS:-3} 6 ;;
        burstpmc)  # memory-side counters of every burst_sweep variant (tools/pmc_burst.py summarises)
            i=0
            for p in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_LEVEL_sum" \
                     "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_CYCLE_sum"; do
                d="$GRAFT_REPO_ROOT/$OUT/pmcburst_$i"
                (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc $p --output-format csv -d "$d" -o burst -- \
                    "$GRAFT_REPO_ROOT/tools/burst_sweep" 1024 1 2 > "$d.out" 2> "$d.err")
                rc=$?; echo "=== pmcburst $i rc=$rc" | tee -a "$OUT/steps.log"
                [ $rc -eq 0 ] || exit $rc
                i=$((i+1))
            done
            python tools/pmc_burst.py "$OUT/pmc_burst.json" "$OUT/pmcburst" > "$OUT/pmc_burst.out" 2>&1 ;;
        occpmc)  # memory-side counters: round 2's and the current launch of C2 (in place) and C4 (pmcset)
            for mode in ${OCCPMC_MODES:-pmcset}; do
                i=0
                for p in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_LEVEL_sum" \
                         "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_CYCLE_sum"; do
                    d="$GRAFT_REPO_ROOT/$OUT/occpmc_${mode}_$i"
                    (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc $p --output-format csv -d "$d" -o occ -- \
                        "$GRAFT_REPO_ROOT/tools/occupancy_sweep" 1024 2 4 $mode > "$d.out" 2> "$d.err")
                    rc=$?; echo "=== occpmc $mode $i rc=$rc" | tee -a "$OUT/steps.log"
                    [ $rc -eq 0 ] || exit $rc
                    i=$((i+1))
                done
                python tools/pmc_burst.py "$OUT/occpmc_$mode.json" "$OUT/occpmc_$mode" \
                    "rocprofv3 --pmc passes over tools/occupancy_sweep $mode (gpu_run.sh occpmc)" > "$OUT/occpmc_$mode.summary" 2>&1
            done ;;
        fanpipe)
            run fanpipe 300 ./tools/fan_sweep 1024 ${SWEEP_ROUNDS:-4} 8 pipe ;;
        ldsstage)  # inputs staged through LDS by LDS-DMA vs the library's register path (C2, C3, C4)
            run ldsstage 300 ./tools/lds_stage_sweep 1024 ${SWEEP_ROUNDS:-4} 8 ;;
        occ)  # block size x resident-wave cap (idle LDS) for the C2 / C3 / C4 kernels
            run occ 400 ./tools/occupancy_sweep 1024 ${SWEEP_ROUNDS:-6} 8 ${OCC_WHICH:-all} &&
            run occ_bf 300 ./tools/occupancy_sweep 1024 ${SWEEP_ROUNDS:-6} 8 c4bf ;;
        occr2)  # the 2-input kernel in place: block size and wave cap, per dtype
            run occr2 400 ./tools/occupancy_sweep 1024 ${SWEEP_ROUNDS:-10} 8 r2ab ;;
        occcopy)  # the copy and conversion kernels: block size and wave cap
            run occcopy 400 ./tools/occupancy_sweep 1024 ${SWEEP_ROUNDS:-10} 8 copyconv ;;
        fanu)  # the 8-input fan-in with 1, 2 or 4 vectors per lane, load order, wave cap
            run fanu 400 ./tools/occupancy_sweep 1024 ${SWEEP_ROUNDS:-6} 8 fanu ;;
        xcd)  # one-wave tiles handed to each XCD in runs of G consecutive tiles (C2 in place, C4)
            run xcd 400 ./tools/occupancy_sweep 1024 ${SWEEP_ROUNDS:-6} 8 xcd ;;
        ptrkind)  # pointer classification and small host reduces against concurrent threads
            run ptrkind 300 ./tools/pointer_kind_probe &&
            for T in 1 2 4 8 16; do
                run "small_workers_$T" 120 ./tools/small_workers $T 1024 &&
                run "small_workers_reg_$T" 120 ./tools/small_workers $T 1024 reg
            done ;;
        smallw)  # 4 KiB / 64 KiB / 512 KiB host chunks at T workers: drop-in (lookups, registry, host
                 # schedule) against the reference's own compiled CPU loop, one JSON line each
            for n in ${SMALLW_ELEMS:-1024 16384 131072}; do
                for T in 1 2 4 8 16; do
                    for mode in ${SMALLW_MODES:-default reg sched ref copy copyhost memcpy}; do
                        timeout -k 10 120 ./tools/small_workers $T $n $mode >> "$OUT/smallw.jsonl" 2>> "$OUT/smallw.err"
                        rc=$?
                        [ $rc -eq 0 ] || { echo "STOP: smallw $T $n $mode rc=$rc" | tee -a "$OUT/steps.log"; exit $rc; }
                    done
                done
                echo "=== smallw n=$n done" | tee -a "$OUT/steps.log"
            done ;;
        gran)  # the one-wave kernels at every residency whole LDS granules allow (C2, C3, C4, 6-input)
            run gran 400 ./tools/occupancy_sweep 1024 ${SWEEP_ROUNDS:-8} 8 gran ;;
        residency)  # resident one-wave workgroups per CU against the dynamic LDS each reserves
            run residency 120 ./tools/residency_probe 20 0 6826 6656 6144 7168 13653 13312 10240 16384 20480 27306 27136 ;;
        occk)  # the 64-lane fan-in over input count x wave cap
            run occk 400 ./tools/occupancy_sweep 1024 ${SWEEP_ROUNDS:-6} 6 fank ;;
        copysweep)
            run copysweep 300 ./tools/copy_sweep 1024 ${SWEEP_ROUNDS:-4} 8 ;;
        copyprof)  # per-kernel durations of every copy_sweep variant
            (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
                -d "$GRAFT_REPO_ROOT/$OUT/copyprof" -o copy -- "$GRAFT_REPO_ROOT/tools/copy_sweep" 1024 2 8 \
                > "$GRAFT_REPO_ROOT/$OUT/copyprof.out" 2> "$GRAFT_REPO_ROOT/$OUT/copyprof.err")
            rc=$?; echo "=== copyprof rc=$rc" | tee -a "$OUT/steps.log"
            [ $rc -eq 0 ] || exit $rc ;;
        copypmc)  # FETCH_SIZE / WRITE_SIZE of every copy_sweep variant (one launch round, 256 MiB)
            for ctr in FETCH_SIZE WRITE_SIZE; do
                (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv \
                    -d "$GRAFT_REPO_ROOT/$OUT/copypmc_$ctr" -o copy -- "$GRAFT_REPO_ROOT/tools/copy_sweep" 256 1 2 \
                    > "$GRAFT_REPO_ROOT/$OUT/copypmc_$ctr.out" 2> "$GRAFT_REPO_ROOT/$OUT/copypmc_$ctr.err")
                rc=$?; echo "=== copypmc $ctr rc=$rc" | tee -a "$OUT/steps.log"
                [ $rc -eq 0 ] || exit $rc
            done ;;
        fanskew)
            run fanskew 300 ./tools/fan_sweep 1024 ${SWEEP_ROUNDS:-4} 8 skew ;;
        fanlayout)
            run fanlayout 300 ./tools/fan_sweep 1024 ${SWEEP_ROUNDS:-4} 8 layout ;;
        policy)
            run policy 300 ./tools/policy_sweep 1024 5 10 ;;
        bench)
            run bench 600 python bench.py ;;
        bench3)  # run-to-run spread of the headline in one box
            for i in 1 2 3; do run "bench_rep$i" 300 python bench.py --no-cpu-baseline --no-host-leg; done ;;
        warm)
            run warm 300 python tools/warm_probe.py ;;
        c1)
            for P in 2 4; do
                for mode in dropin dropin-gpu oracle; do
                    run "c1_${mode}_p$P" 300 python tools/c1_allreduce.py --reduce $mode --ranks $P --iters 200 &&
                    run "c1_${mode}_p${P}_fused" 300 python tools/c1_allreduce.py --reduce $mode --ranks $P \
                        --iters 200 --fused
                done
            done ;;
        dispatch)
            run dispatch 600 python tools/dispatch_sweep.py --max-mib ${DISPATCH_MAX_MIB:-512} ;;
        adapt)  # the adaptive split followed over 12 calls per pointer kind
            run adapt 400 python tools/dispatch_sweep.py --adapt-trace --max-mib 256 --dtypes f32,bf16 \
                --shares 0.3,0.35,0.4,0.45,0.5,0.55 ;;
        workers)  # W concurrent worker threads through ccl_comp_reduce on host buckets, vs W oracle threads
            run workers 600 python tools/workers_sweep.py --segv-trace --workers ${WORKERS:-1,2,4,8,16} \
                --mib ${WORKERS_MIB:-8,64} --modes ${WORKERS_MODES:-oracle,host,split,default} &&
            run workers_pinned 600 python tools/workers_sweep.py --segv-trace --pinned --workers ${WORKERS:-1,2,4,8,16} \
                --mib ${WORKERS_MIB:-64} --modes ${WORKERS_MODES:-oracle,host,split,default} ;;
        exittests)  # process exit against thread teardown and un-waited asynchronous requests
            run pytest_exit 300 python -u -m pytest tests/test_gpu_shim.py -m gpu -q -k exit -p no:cacheprovider \
                --timeout 120 --timeout-method thread ;;
        dispatchtests)
            run pytest_dispatch 600 python -u -m pytest tests/test_gpu_dispatch.py tests/test_host_reduce.py -m "gpu or not gpu" \
                -q -p no:cacheprovider --timeout 120 --timeout-method thread ;;
        coop)  # the cooperative split above the crossover, shares swept
            run coop 600 python tools/dispatch_sweep.py --min-kib 16384 --max-mib 1024 --shares 0.2,0.3,0.4,0.5,0.6 ;;
        dist2)
            run dist2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
                --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo &&
            run dist2_strong 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
                --master-port 29534 bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo --scaling strong ;;
        dist2self)  # bench.py as its own launcher: --gpus 2 with no WORLD_SIZE (both ranks share the box's GPU)
            run dist2self 300 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline ;;  # nccl -> gloo on 1 GPU
        pmcjson)  # the PMC passes of `pmc` (and PMC_CONFIG=c4's) summarised into profiles-ready JSON
            specs="c2=$OUT:3221225472"
            [ -d "$OUT/pmc_c4" ] && specs="$specs c4=$OUT/pmc_c4:9663676416"
            python tools/pmc_traffic.py "$OUT/pmc.json" $specs > "$OUT/pmcjson.out" 2>&1 ;;
        ab)  # A/B of earlier kernel builds against the current one, same box (tools/ab_c2.py)
            for v in ${AB_VARIANTS:-old}; do
                run "ab_${v}_${AB_CONFIG:-c2}" 300 python tools/ab_c2.py tools/ab/$v/libmi_reduce.so \
                    oneccl_amd/lib/libmi_reduce.so --config ${AB_CONFIG:-c2} --rounds ${AB_ROUNDS:-10}
            done ;;
        sizes)
            run sizes 600 python tools/size_sweep.py ;;
        sizes_fp32)
            run sizes 300 python tools/size_sweep.py --configs fp32-sum ;;
        misalign)
            run misalign 300 python tools/misalign_probe.py ;;
        nanprobe)
            run nanprobe 300 python tools/nan_probe.py ;;
        soak)  # a longer seeded fuzz of the device and synchronous entries (FUZZ_CASES cases)
            MI_FUZZ_CASES=${FUZZ_CASES:-8000} run soak 900 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -q \
                -p no:cacheprovider --timeout 300 --timeout-method thread ;;
        benchall)
            for c in c3-bf16 c3-fp16 c4 c4-bf16acc c5-int32-max c5-int64-prod; do
                run "bench_$c" 300 python bench.py --config "$c" --no-cpu-baseline --no-host-leg
            done ;;
        prof)  # PROF_CONFIG=c4 etc. profiles another bench config
            pc=${PROF_CONFIG:-c2}; pd=prof; [ "$pc" = c2 ] || pd=prof_$pc
            (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
                -d "$GRAFT_REPO_ROOT/$OUT/$pd" -o bench -- \
                python3 "$GRAFT_REPO_ROOT/bench.py" --config "$pc" --steps 20 --warmup 5 --no-cpu-baseline --no-host-leg --no-config-legs \
                > "$GRAFT_REPO_ROOT/$OUT/$pd.out" 2> "$GRAFT_REPO_ROOT/$OUT/$pd.err")
            rc=$?; echo "=== $pd rc=$rc" | tee -a "$OUT/steps.log"
            [ $rc -eq 0 ] || exit $rc ;;
        proftrace)
            (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
                -d "$GRAFT_REPO_ROOT/$OUT/proftrace" -o policy -- "$GRAFT_REPO_ROOT/tools/policy_sweep" 1024 1 3 \
                > "$GRAFT_REPO_ROOT/$OUT/proftrace.out" 2> "$GRAFT_REPO_ROOT/$OUT/proftrace.err")
            rc=$?; echo "=== proftrace rc=$rc" | tee -a "$OUT/steps.log"
            [ $rc -eq 0 ] || exit $rc ;;
        pmc)  # PMC_CONFIG=c4 etc. counts another bench config (output under pmc_<config>/)
            pc=${PMC_CONFIG:-c2}; pdir=$OUT; [ "$pc" = c2 ] || pdir=$OUT/pmc_$pc
            mkdir -p "$pdir"
            for ctr in FETCH_SIZE WRITE_SIZE; do
                (cd /tmp && timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv \
                    -d "$GRAFT_REPO_ROOT/$pdir/pmc_$ctr" -o bench -- \
                    python3 "$GRAFT_REPO_ROOT/bench.py" --config "$pc" --steps 5 --warmup 2 --no-cpu-baseline \
                    --no-host-leg --no-config-legs > "$GRAFT_REPO_ROOT/$pdir/pmc_$ctr.out" 2> "$GRAFT_REPO_ROOT/$pdir/pmc_$ctr.err")
                rc=$?; echo "=== pmc $pc $ctr rc=$rc" | tee -a "$OUT/steps.log"
                [ $rc -eq 0 ] || exit $rc
            done ;;
        *) echo "unknown step $step"; exit 2 ;;
    esac
done
echo "=== all steps done" | tee -a "$OUT/steps.log"
