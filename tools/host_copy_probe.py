#!/usr/bin/env python3
"""Host-to-host ccl_comp_copy on the calling thread's CPU: mi_host_copy with
nontemporal = 0 (a memcpy, the reference's `ccl::memcpy` path) against
nontemporal = 1 (streaming stores, the reference's memcpy_nontemporal path,
src/common/utils/memcpy.cpp:49-125).  GB/s = 2 x bytes / time (read + write),
best and median of --reps, modes interleaved per rep.

  python tools/host_copy_probe.py [--kib 256,4096,65536,524288] [--reps 20]
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    import numpy as np
    from oneccl_amd import _lib
    ap = argparse.ArgumentParser()
    ap.add_argument("--kib", default="256,4096,65536,524288")
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    hc = _lib.shim().mi_host_copy
    for kib in (int(x) for x in args.kib.split(",")):
        n = kib << 10
        src = np.full(n, 0x3F, np.uint8)
        dst = np.zeros(n, np.uint8)
        res = {0: [], 1: []}
        for rep in range(args.reps + 1):
            for nt in ((0, 1) if rep % 2 else (1, 0)):
                t0 = time.perf_counter()
                assert hc(dst.ctypes.data, src.ctypes.data, n, nt) == 0
                dt = time.perf_counter() - t0
                if rep:
                    res[nt].append(2 * n / dt / 1e9)
        for nt, r in res.items():
            print(json.dumps({"KiB": kib, "nontemporal": nt, "best_GBps": round(max(r), 1),
                              "median_GBps": round(statistics.median(r), 1)}), flush=True)


if __name__ == "__main__":
    main()
