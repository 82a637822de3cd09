# round 5 session a: the new GPU tests (pinned-extent registry, unregister
# demotion, host-word check), the MPI user-op small-bucket sweep on the box's
# host cores, and one default bench run (mixed ceiling,
# c4-tmpbuf leg, pinned CPU sweep)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5a
mkdir -p $O
export TMPDIR=/tmp
{ nproc; lscpu; cat /sys/fs/cgroup/cpu.max; numactl -H 2>/dev/null | head -5; } > $O/host.txt 2>&1
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_registry.py tests/test_host_word_check.py tests/test_mpi_user_op.py > $O/pytest_new.log 2>&1 || exit $?
for n in 2048 32768 262144; do
    for t in 1 8 16; do
        for mode in mpibf16 bf16 refbf16 mpifp16 fp16 reffp16; do
            timeout -k 10 60 ./tools/small_workers $t $n $mode >> $O/small_workers_mpiop.jsonl 2>> $O/small_workers.err || exit $?
        done
    done
done
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
