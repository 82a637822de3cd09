# round 5 session h: the MPI user op's 4 KiB call with the host fold's AVX-512
# form (default) against its 8-lane AVX2 form (MI_HOST_ISA=avx2), pinned
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5h
mkdir -p $O
CPUS=$(python -c "import sys; sys.path.insert(0,'.'); import bench; c=bench.core_plan()[1]; c=c[1:]+c[:1]; print(','.join(map(str, c[:16])))")
for rep in 1 2; do
    for t in 1 8 16; do
        for isa in default avx2; do
            for mode in mpibf16 mpifp16 foldbf16 refbf16; do
                if [ $isa = default ]; then unset MI_HOST_ISA; else export MI_HOST_ISA=$isa; fi
                SW_CPUS=$CPUS timeout -k 10 60 ./tools/small_workers $t 2048 $mode | sed "s/\"mode\": \"/\"mode\": \"$isa:/" >> $O/sw.jsonl 2>> $O/sw.err || exit $?
            done
        done
    done
done
