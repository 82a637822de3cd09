#!/usr/bin/env python3
"""C5 (BASELINE.json configs[4]): bucket-size sweep 4 KiB .. 1 GiB, powers of 4,
for fp32 sum, int32 max and int64 prod.  Per size: device-resident kernel time
(hipEvent pair, mean of reps), the synchronous drop-in call on device buffers
(ccl_comp_reduce path: launch + stream sync, host wall), the host-resident
call on pinned and pageable buffers, and one CPU thread: the reference's own compiled
CCL_REDUCE (oracle/_ref) where built, else the oracle.
One JSON line per (config, size) on stdout.

  python tools/size_sweep.py [--max-mib 1024] [--reps 20]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

CONFIGS = [("fp32-sum", 9, 4, 0), ("int32-max", 4, 4, 3), ("int64-prod", 6, 8, 1)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--max-mib", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--configs", default="fp32-sum,int32-max,int64-prod")
    args = ap.parse_args()
    import numpy as np
    import torch

    import oracle
    from oneccl_amd import _lib
    m = _lib.mi()
    want = set(args.configs.split(","))
    sizes = []
    s = 4 << 10
    while s <= args.max_mib << 20:
        sizes.append(s)
        s *= 4
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream
    for name, dt, es, op in CONFIGS:
        if name not in want:
            continue
        for nbytes in sizes:
            n = nbytes // es
            tdt = {9: torch.float32, 4: torch.int32, 6: torch.int64}[dt]
            a = torch.ones(n, dtype=tdt, device="cuda")
            b = torch.ones(n, dtype=tdt, device="cuda")
            reps = args.reps if nbytes < (256 << 20) else max(5, args.reps // 4)
            for _ in range(3):
                _lib.check(m.mi_reduce(a.data_ptr(), b.data_ptr(), n, dt, op, 0, sh))
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(reps):
                m.mi_reduce(a.data_ptr(), b.data_ptr(), n, dt, op, 0, sh)
            e1.record(stream)
            torch.cuda.synchronize()
            kern_us = e0.elapsed_time(e1) * 1e3 / reps
            # synchronous drop-in path on device buffers, spin and blocking waits
            row = {"config": name, "bytes": nbytes, "elems": n, "kernel_us": round(kern_us, 2),
                   "kernel_GBps_3x": round(3 * nbytes / (kern_us * 1e-6) / 1e9, 1)}
            for mode, key in ((1, "sync_device_block_us"), (0, "sync_device_us")):
                m.mi_set_sync_mode(mode)
                t = []
                for _ in range(reps):
                    t0 = time.perf_counter()
                    m.mi_reduce_sync(a.data_ptr(), b.data_ptr(), n, dt, op, 0, -1)
                    t.append(time.perf_counter() - t0)
                row[key] = round(min(t) * 1e6, 2)
            if nbytes <= (256 << 20):
                ha = torch.ones(n, dtype=tdt).pin_memory()
                hb = torch.ones(n, dtype=tdt).pin_memory()
                pa = np.ones(n, oracle.NP_DTYPE[dt])
                pb = np.ones(n, oracle.NP_DTYPE[dt])
                for key, (x, y) in (("sync_pinned_us", (ha.data_ptr(), hb.data_ptr())),
                                    ("sync_pageable_us", (pa.ctypes.data, pb.ctypes.data))):
                    m.mi_reduce_sync(x, y, n, dt, op, 0, -1)
                    t = []
                    for _ in range(max(3, reps // 2)):
                        t0 = time.perf_counter()
                        m.mi_reduce_sync(x, y, n, dt, op, 0, -1)
                        t.append(time.perf_counter() - t0)
                    row[key] = round(min(t) * 1e6, 2)
                # one CPU thread: the reference's own compiled CCL_REDUCE where
                # oracle/_ref was built (it travels with the tree), else the oracle
                use_ref = oracle.ref_comp_available() and dt not in (8, 11)

                def cpu():
                    if use_ref:
                        oracle.ref_comp_reduce(pa, pb, dt, op)
                    else:
                        oracle.comp_reduce(pa, pb, dt, op)
                cpu()
                t = []
                for _ in range(max(3, reps // 2)):
                    t0 = time.perf_counter()
                    cpu()
                    t.append(time.perf_counter() - t0)
                row["cpu_1thread_us"] = round(min(t) * 1e6, 2)
                row["cpu_1thread_kind"] = "reference" if use_ref else "oracle"
            print(json.dumps(row), flush=True)
            del a, b
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
