#!/usr/bin/env python3
"""HBM bytes per launch of the copy and conversion kernels from the two
`copypmc` passes of tools/gpu_run.sh (FETCH_SIZE, WRITE_SIZE over
`copy_sweep 256 1 2`), against their algorithmic bytes.  gfx950 correction as
in tools/pmc_traffic.py: reads = 2 x FETCH_SIZE KiB x 1024; writes = WRITE_SIZE
KiB x 1024.  Copy rows merge the aligned and src+4 launches.

  tools/pmc_copy.py OUT_JSON DIR   (DIR holds copypmc_FETCH_SIZE/ and copypmc_WRITE_SIZE/)
"""
from __future__ import annotations

import collections
import csv
import json
import statistics
import sys
from pathlib import Path

MIB = 256  # copy_sweep's buffer in the copypmc step


def load(d: Path, ctr: str) -> dict[str, list[float]]:
    out = collections.defaultdict(list)
    for r in csv.DictReader(open(next((d / f"copypmc_{ctr}").glob("*counter_collection.csv")))):
        out[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return out


def main() -> None:
    out, d = Path(sys.argv[1]), Path(sys.argv[2])
    fetch, write = load(d, "FETCH_SIZE"), load(d, "WRITE_SIZE")
    nbytes = MIB << 20
    res = {"buffer_MiB": MIB, "correction": "reads = 2 x FETCH_SIZE KiB x 1024 (gfx950), writes = WRITE_SIZE KiB x 1024",
           "kernels": {}}
    for name, fv in fetch.items():
        if "mi::" not in name:
            continue
        if "convert_kernel" in name:
            n = nbytes // 4  # elements: the fp32 side is the whole buffer
            narrowing = name.startswith("void mi::convert_kernel<float")
            rd, wr = (4 * n, 2 * n) if narrowing else (2 * n, 4 * n)
        else:
            rd = wr = nbytes
        f, w = statistics.median(fv), statistics.median(write.get(name, [0.0]))
        res["kernels"][name.split("(")[0].replace("void ", "")] = {
            "launches": len(fv), "read_ratio": round(2 * f * 1024 / rd, 4), "write_ratio": round(w * 1024 / wr, 4),
            "hbm_ratio": round((2 * f * 1024 + w * 1024) / (rd + wr), 4)}
    out.write_text(json.dumps(res, indent=1) + "\n")
    print(out.read_text())


if __name__ == "__main__":
    main()
