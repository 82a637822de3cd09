# round 5 session f: the 4 KiB bf16 call under a host schedule with the
# (historical: the diagnostic shim builds under tools/diag_* that this session loaded were
# one-off variants of comp.cpp and are not kept; results: profiles/round5_host/isolate_*)
# product shim, a shim without the host-worker accounting (HostCall), and one
# with 128-byte accounting slots (tools/diag_*: diagnostic builds only)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5f
mkdir -p $O
CPUS=$(python -c "import sys; sys.path.insert(0,'.'); import bench; c=bench.core_plan()[1]; c=c[1:]+c[:1]; print(','.join(map(str, c[:16])))")
for rep in 1 2; do
    for t in 1 8 16; do
        for v in product nohc pad128; do
            for mode in schedbf16 mpibf16 schedi16; do
                if [ $v = product ]; then LLP=; else LLP=tools/diag_$v; fi
                LD_LIBRARY_PATH=$LLP SW_CPUS=$CPUS timeout -k 10 60 ./tools/small_workers $t 2048 $mode | sed "s/\"mode\": \"/\"mode\": \"$v:/" >> $O/sw.jsonl 2>> $O/sw.err || exit $?
            done
        done
    done
done
