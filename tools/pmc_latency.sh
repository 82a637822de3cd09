#!/usr/bin/env bash
# PMC passes for the memory-side picture of the C2 (2-input) and C4 (8-input
# fan-in) kernels: EA read/write requests, requests in flight (Little's law:
# average latency = LEVEL / REQ cycles), DRAM credit stalls.  One counter set
# per rocprofv3 run, each under its own kill timer (the PMC rules of
# MI355X_MICROARCH.md / gpurun).  Output: gpurun_out/pmclat_<cfg>_<pass>/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
passes=(
  "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum"
  "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_LEVEL_sum"
  "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_CYCLE_sum"
)
for cfg in c2 c4; do
  i=0
  for p in "${passes[@]}"; do
    d="$GRAFT_REPO_ROOT/$OUT/pmclat_${cfg}_$i"
    (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $p --output-format csv -d "$d" -o bench -- \
        python3 "$GRAFT_REPO_ROOT/bench.py" --config "$cfg" --steps 5 --warmup 2 --no-cpu-baseline --no-host-leg \
        > "$d.out" 2> "$d.err")
    rc=$?
    echo "pmclat $cfg pass $i ($p) rc=$rc"
    [ $rc -eq 0 ] || exit $rc
    i=$((i+1))
  done
done
