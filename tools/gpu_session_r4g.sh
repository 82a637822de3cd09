# round 4 session g: one buffer or a pair? and per-channel L2 requests in each mode
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python tools/pair_probe.py --trials 5 > gpurun_out/pair_probe.out 2> gpurun_out/pair_probe.err || exit $?
d="$GRAFT_REPO_ROOT/gpurun_out/plpmc_inst"
(cd /tmp && timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ TCC_EA0_WRREQ --output-format csv -d "$d" -o pl -- \
    python3 "$GRAFT_REPO_ROOT/tools/placement_probe.py" --inputs 2 --trials 10 --launches 6 > "$d.out" 2> "$d.err")
