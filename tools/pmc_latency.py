#!/usr/bin/env python3
"""Summarise tools/pmc_latency.sh: per launch of the reduce kernel, the L2
(TCC) -> memory (EA) request counts, requests in flight, DRAM credit stalls,
and what Little's law makes of them.

  reads per request      = 128 B (TCC_EA0_RDREQ counts 128-B requests here:
                           2 GiB of C2 reads = 16.78 M requests)
  writes per request     = 64 B
  avg read latency       = RDREQ_LEVEL / RDREQ            (TCC cycles)
  reads in flight / chan = RDREQ_LEVEL / TCC_CYCLE        (TCC_CYCLE is summed
                           over channels, so this is the per-channel mean)
  bytes / cycle / chan   = (128 RDREQ + 64 WRREQ) / TCC_CYCLE

  tools/pmc_latency.py OUT_JSON CFG=DIR_PREFIX ...   (DIR_PREFIX_0, _1, _2)
"""
from __future__ import annotations

import csv
import glob
import json
import statistics
import sys
from collections import defaultdict

NEEDLES = ("reduce2_kernel", "fan_kernel", "reduce_kernel")


def medians(prefix: str) -> tuple[dict, float]:
    vals, dur = defaultdict(list), []
    for i in range(3):
        path = glob.glob(f"{prefix}_{i}/*counter_collection.csv")[0]
        for r in csv.DictReader(open(path)):
            if any(n in r["Kernel_Name"] for n in NEEDLES):
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
                dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    return {k: statistics.median(v) for k, v in vals.items()}, statistics.median(dur)


def main() -> None:
    res = {}
    for spec in sys.argv[2:]:
        cfg, prefix = spec.split("=", 1)
        m, ms = medians(prefix)
        rd, wr, cyc = m["TCC_EA0_RDREQ_sum"], m["TCC_EA0_WRREQ_sum"], m["TCC_CYCLE_sum"]
        res[cfg] = {
            "counters_median_per_launch": m,
            "launch_ms_median_under_pmc": round(ms, 4),
            "read_bytes": int(rd * 128),
            "write_bytes": int(wr * 64),
            "avg_read_latency_cycles": round(m["TCC_EA0_RDREQ_LEVEL_sum"] / rd, 1),
            "avg_write_latency_cycles": round(m["TCC_EA0_WRREQ_LEVEL_sum"] / wr, 1),
            "reads_in_flight_per_channel": round(m["TCC_EA0_RDREQ_LEVEL_sum"] / cyc, 1),
            "writes_in_flight_per_channel": round(m["TCC_EA0_WRREQ_LEVEL_sum"] / cyc, 1),
            "read_bytes_per_cycle_per_channel": round(128 * rd / cyc, 2),
            "write_bytes_per_cycle_per_channel": round(64 * wr / cyc, 2),
            "bytes_per_cycle_per_channel": round((128 * rd + 64 * wr) / cyc, 2),
            "read_dram_credit_stall_frac": round(m["TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum"] / cyc, 4),
            "write_dram_credit_stall_frac": round(m["TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum"] / cyc, 4),
        }
    res["_note"] = ("One rocprofv3 --pmc pass per counter set (tools/pmc_latency.sh), bench.py --steps 5 "
                    "--warmup 2; medians over the reduce kernel's launches. Launch times run slower under "
                    "counter collection than in the bench line.")
    with open(sys.argv[1], "w") as f:
        f.write(json.dumps(res, indent=1) + "\n")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
