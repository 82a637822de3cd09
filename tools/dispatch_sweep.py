#!/usr/bin/env python3
"""Crossover of the drop-in's dispatcher: for a
host-resident bucket, the calling thread's CPU (host_reduce.cpp) against the
GPU (staging / zero-copy), both through ccl_comp_reduce itself, next to the
CPU oracle on one thread (the reference's one-worker rate).  Sizes 4 KiB ..
--max-mib, powers of 2; pageable (posix_memalign-like numpy) and pinned
buffers.  One JSON line per (dtype, kind, size): best-of-reps microseconds.

  python tools/dispatch_sweep.py [--max-mib 512] [--dtypes f32,bf16]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

DT = {"f32": (9, 4), "bf16": (11, 2)}
KNOBS = ("CCL_COMP_HOST_MAX_BYTES", "CCL_COMP_HOST_MAX_PINNED_BYTES", "CCL_COMP_HOST_SHARE",
         "CCL_COMP_HOST_SHARE_PINNED")


def best_us(fn, reps):
    fn()
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        t.append(time.perf_counter() - t0)
    return round(min(t) * 1e6, 2), round(sorted(t)[len(t) // 2] * 1e6, 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--max-mib", type=int, default=512)
    ap.add_argument("--dtypes", default="f32,bf16")
    ap.add_argument("--kinds", default="pageable,pinned")
    ap.add_argument("--shares", default="0.3,0.45,0.6")
    ap.add_argument("--min-kib", type=int, default=4)
    args = ap.parse_args()
    import numpy as np
    import torch

    import oracle
    from oneccl_amd import comp
    sizes = []
    s = args.min_kib << 10
    while s <= args.max_mib << 20:
        sizes.append(s)
        s *= 2
    for dname in args.dtypes.split(","):
        dt, es = DT[dname]
        for kind in args.kinds.split(","):
            for nbytes in sizes:
                n = nbytes // es
                reps = 20 if nbytes <= (4 << 20) else (6 if nbytes <= (64 << 20) else 3)
                if kind == "pinned":
                    ta = torch.ones(nbytes, dtype=torch.uint8).pin_memory()
                    tb = torch.ones(nbytes, dtype=torch.uint8).pin_memory()
                    pa, pb = ta.data_ptr(), tb.data_ptr()
                    a = ta.numpy().view(oracle.NP_DTYPE[dt])
                    b = tb.numpy().view(oracle.NP_DTYPE[dt])
                else:
                    a = np.ones(n, oracle.NP_DTYPE[dt])
                    b = np.ones(n, oracle.NP_DTYPE[dt])
                    pa, pb = a.ctypes.data, b.ctypes.data
                row = {"dtype": dname, "kind": kind, "bytes": nbytes}
                modes = [("cpu", {"CCL_COMP_HOST_MAX_BYTES": str(1 << 40),
                                  "CCL_COMP_HOST_MAX_PINNED_BYTES": str(1 << 40)}),
                         ("gpu", {"CCL_COMP_HOST_MAX_BYTES": "0"}),
                         ("default", {})]
                if nbytes >= (32 << 20):  # the cooperative split (CPU head + GPU tail) at several shares
                    for sh in args.shares.split(","):
                        modes.append((f"coop{sh}", {"CCL_COMP_HOST_MAX_BYTES": str(1 << 20),
                                                    "CCL_COMP_HOST_MAX_PINNED_BYTES": str(1 << 20),
                                                    "CCL_COMP_HOST_SHARE": sh, "CCL_COMP_HOST_SHARE_PINNED": sh}))
                for mode, envs in modes:
                    for kk in KNOBS:
                        os.environ.pop(kk, None)
                    os.environ.update(envs)
                    comp.env_reload()
                    row[f"{mode}_us"], row[f"{mode}_median_us"] = best_us(
                        lambda: comp.comp_reduce(pa, n, pb, comp.datatype(dt), comp.reduction.sum), reps)
                row["oracle_1t_us"], _ = best_us(lambda: oracle.comp_reduce(a, b, dt, 0), reps)
                for mode, _ in modes:
                    row[f"{mode}_GiBps"] = round(nbytes / (row[f"{mode}_us"] * 1e-6) / 2**30, 2)
                print(json.dumps(row), flush=True)
    for kk in KNOBS:
        os.environ.pop(kk, None)


if __name__ == "__main__":
    main()
