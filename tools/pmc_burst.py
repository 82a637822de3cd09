#!/usr/bin/env python3
"""Summarise the PMC passes over tools/burst_sweep (gpu_run.sh step
`burstpmc`): per kernel variant — template instance and grid — the L2 -> memory
request counts, requests in flight, latency by Little's law and DRAM credit
stalls, with the same derivations as tools/pmc_latency.py (128-B read and 64-B
write requests; TCC_CYCLE summed over channels).  VERDICT r1 "next" #6 asked
for the burst experiment's result with these counters beside it.

  tools/pmc_burst.py OUT_JSON DIR_PREFIX [NOTE]  (DIR_PREFIX_0, _1, _2)

Also used for tools/occupancy_sweep (gpu_run.sh occpmc): variants are told
apart by template, grid and the LDS each workgroup reserves.
"""
from __future__ import annotations

import csv
import glob
import json
import re
import statistics
import sys
from collections import defaultdict


def short(name: str) -> str:
    m = re.match(r"void (\w+)<(.*)>\(", name)
    return f"{m.group(1)}<{m.group(2)}>" if m else name[:80]


def main() -> None:
    out, prefix = sys.argv[1], sys.argv[2]
    vals = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for i in range(3):
        path = glob.glob(f"{prefix}_{i}/*counter_collection.csv")[0]
        for r in csv.DictReader(open(path)):
            n = r["Kernel_Name"]
            if not any(k in n for k in ("burst_kernel", "reduce2_kernel", "fan_kernel", "copy_lean_kernel",
                                        "convert_kernel")):
                continue
            # the LDS a launch reserves tells apart tools/occupancy_sweep's wave caps
            key = (short(n), int(r["Grid_Size"]) // int(r["Workgroup_Size"]), int(r.get("LDS_Block_Size") or 0))
            vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    res = []
    for (kname, grid, lds), cs in sorted(vals.items()):
        m = {k: statistics.median(v) for k, v in cs.items()}
        need = ("TCC_EA0_RDREQ_sum", "TCC_EA0_WRREQ_sum", "TCC_CYCLE_sum", "TCC_EA0_RDREQ_LEVEL_sum",
                "TCC_EA0_WRREQ_LEVEL_sum", "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum",
                "TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum")
        if not all(k in m for k in need):
            continue
        rd, wr, cyc = m["TCC_EA0_RDREQ_sum"], m["TCC_EA0_WRREQ_sum"], m["TCC_CYCLE_sum"]
        res.append({
            "kernel": kname, "workgroups": grid, "lds_bytes_per_workgroup": lds,
            "launch_ms_median_under_pmc": round(statistics.median(dur[(kname, grid, lds)]), 4),
            "read_bytes": int(rd * 128), "write_bytes": int(wr * 64),
            "avg_read_latency_cycles": round(m["TCC_EA0_RDREQ_LEVEL_sum"] / rd, 1),
            "avg_write_latency_cycles": round(m["TCC_EA0_WRREQ_LEVEL_sum"] / wr, 1),
            "reads_in_flight_per_channel": round(m["TCC_EA0_RDREQ_LEVEL_sum"] / cyc, 1),
            "writes_in_flight_per_channel": round(m["TCC_EA0_WRREQ_LEVEL_sum"] / cyc, 1),
            "bytes_per_cycle_per_channel": round((128 * rd + 64 * wr) / cyc, 2),
            "read_dram_credit_stall_frac": round(m["TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum"] / cyc, 4),
            "write_dram_credit_stall_frac": round(m["TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum"] / cyc, 4),
        })
    note = sys.argv[3] if len(sys.argv) > 3 else (
        "One rocprofv3 --pmc pass per counter set over tools/burst_sweep 1024 MiB (gpu_run.sh burstpmc); "
        "medians over each variant's launches. Launches run slower under counter collection; the "
        "timed comparison is profiles/round2_burst/burst_sweep.jsonl.")
    doc = {"variants": res, "_note": note}
    with open(out, "w") as f:
        f.write(json.dumps(doc, indent=1) + "\n")
    for r in res:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
