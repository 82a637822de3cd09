#!/usr/bin/env python3
"""What slows the CPU head of the cooperative split on pinned buffers?  The
split done by hand through the C ABI (mi_reduce_start on the tail, then
mi_host_reduce on the head on this thread, then mi_wait), timing the head
alone, with the head in one call or in 8 MiB chunks, with and without an
mi_test poll between chunks, and the head alone with no GPU part running.
One JSON line per (kind, variant): best and median over reps.

  python tools/split_probe.py [--mib 256] [--share 0.5] [--reps 6]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=256)
    ap.add_argument("--share", type=float, default=0.5)
    ap.add_argument("--reps", type=int, default=6)
    args = ap.parse_args()
    import numpy as np
    import torch

    from oneccl_amd import _lib
    m, sh = _lib.mi(), _lib.shim()
    nbytes = args.mib << 20
    n = nbytes // 4
    s = int(n * args.share) // 256 * 256
    chunk = (8 << 20) // 4
    for kind in ("pinned", "pageable"):
        if kind == "pinned":
            ta = torch.full((nbytes,), 0x3F, dtype=torch.uint8).pin_memory()
            tb = torch.full((nbytes,), 0x3F, dtype=torch.uint8).pin_memory()
            pa, pb = ta.data_ptr(), tb.data_ptr()
        else:
            a = np.full(nbytes, 0x3F, np.uint8)
            b = np.full(nbytes, 0x3F, np.uint8)
            pa, pb = a.ctypes.data, b.ctypes.data

        def head(chunked, poll, req):
            step = chunk if chunked else s
            for i in range(0, s, step):
                c = min(step, s - i)
                arr = _lib.void_ptr_array([pb + 4 * i, pa + 4 * i])
                _lib.check(sh.mi_host_reduce(arr, 2, pb + 4 * i, c, 9, 0, 0))
                if poll and req is not None:
                    done = ctypes.c_int(0)
                    m.mi_test(req, ctypes.byref(done))

        variants = [("head alone, one call", False, False, False), ("head alone, 8 MiB chunks", True, False, False),
                    ("split, head one call", False, False, True), ("split, head chunked", True, False, True),
                    ("split, head chunked + mi_test polls", True, True, True)]
        for name, chunked, poll, split in variants:
            heads, totals = [], []
            for r in range(args.reps + 1):
                req = ctypes.c_void_p()
                t0 = time.perf_counter()
                if split:
                    gins = _lib.void_ptr_array([pb + 4 * s, pa + 4 * s])
                    _lib.check(m.mi_reduce_start(gins, 2, pb + 4 * s, n - s, 9, 0, 0, -1, ctypes.byref(req)))
                th = time.perf_counter()
                head(chunked, poll, req if split else None)
                t1 = time.perf_counter()
                if split:
                    _lib.check(m.mi_wait(req))
                    m.mi_request_free(req)
                t2 = time.perf_counter()
                if r:  # the first rep warms up
                    heads.append(t1 - th)
                    totals.append(t2 - t0)
            print(json.dumps({"kind": kind, "variant": name, "share": args.share, "bucket_MiB": args.mib,
                              "head_GiBps_best": round(s * 4 / min(heads) / 2**30, 2),
                              "head_GiBps_median": round(s * 4 / statistics.median(heads) / 2**30, 2),
                              "total_GiBps_best": round(nbytes / min(totals) / 2**30, 2)}), flush=True)


if __name__ == "__main__":
    main()
