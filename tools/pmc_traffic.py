#!/usr/bin/env python3
"""Turn rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE in separate runs, as
/opt/skills/guides/MI355X_MICROARCH.md §HBM / rocprofv3 prescribes) into HBM
bytes per launch of the reduce kernel.

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE is in KiB and
reports exactly half the bytes of a wide coalesced streaming read (128-B
requests tallied at 64 B) -> x2; WRITE_SIZE (KiB) is exact for 16-B-per-lane
streaming stores.

  tools/pmc_traffic.py OUT_JSON CONFIG=DIR_WITH_pmc_FETCH_SIZE_AND_pmc_WRITE_SIZE[:ALGO_BYTES] ...
"""
from __future__ import annotations

import csv
import datetime
import json
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import bench  # noqa: E402  (kernel_identity: which device code a pass measured)


def kernel_values(path: Path, needles=("mi::reduce2_kernel", "mi::reduce_kernel", "mi::fan_kernel")) -> list[float]:
    # the library's own namespace: torch's at::native::reduce_kernel (the
    # parity check's chunked mismatch count) must not be taken for ours
    rows = list(csv.DictReader(open(path)))
    return [float(r["Counter_Value"]) for r in rows if any(n in r["Kernel_Name"] for n in needles)]


def main() -> None:
    out = Path(sys.argv[1])
    res = json.loads(out.read_text()) if out.exists() else {}
    for spec in sys.argv[2:]:
        cfg, rest = spec.split("=", 1)
        d, _, algo = rest.partition(":")
        d = Path(d)
        fetch = kernel_values(next((d / "pmc_FETCH_SIZE").glob("*counter_collection.csv")))
        write = kernel_values(next((d / "pmc_WRITE_SIZE").glob("*counter_collection.csv")))
        f_kib, w_kib = statistics.median(fetch), statistics.median(write)
        hbm = int(round((2 * f_kib + w_kib) * 1024))
        res[cfg] = {
            "hbm_bytes_per_launch": hbm,
            "fetch_size_kib_median": f_kib,
            "write_size_kib_median": w_kib,
            "launches": [len(fetch), len(write)],
            "correction": "hbm = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950: FETCH_SIZE counts half of a wide "
                          "coalesced stream; MI355X_MICROARCH.md §HBM)",
            "kernel_code": bench.kernel_identity(),
            "recorded_utc": datetime.datetime.now(datetime.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ"),
        }
        if algo:
            res[cfg]["algorithmic_bytes_per_launch"] = int(algo)
            res[cfg]["ratio_to_algorithmic"] = round(hbm / int(algo), 6)
    out.write_text(json.dumps(res, indent=1) + "\n")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
