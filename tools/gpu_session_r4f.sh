# round 4 session f: memory-path counters of C2 over fresh allocations (fast vs slow placement mode)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
i=0
for p in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum" \
         "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_RDREQ_GMI_CREDIT_STALL_sum TCC_EA0_RDREQ_IO_CREDIT_STALL_sum TCC_TAG_STALL_sum" \
         "TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE" \
         "TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_CYCLE_sum"; do
    d="$GRAFT_REPO_ROOT/gpurun_out/plpmc_$i"
    (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $p --output-format csv -d "$d" -o pl -- \
        python3 "$GRAFT_REPO_ROOT/tools/placement_probe.py" --inputs 2 --trials 12 --launches 8 > "$d.out" 2> "$d.err")
    rc=$?; echo "=== plpmc $i rc=$rc" >> gpurun_out/steps.log
    [ $rc -eq 0 ] || exit $rc
    i=$((i+1))
done
