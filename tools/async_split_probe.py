#!/usr/bin/env python3
"""Host buckets above the dispatcher's threshold through the asynchronous
entry (ccl_comp_reduce_start + wait) against the synchronous one.

  sync        ccl_comp_reduce: GPU tail + the calling thread's CPU head
  async       ccl_comp_reduce_start: GPU tail + a CPU head folded on the
              thread's staging worker (mi_reduce_split_start); start returns
  async-gpu   ccl_comp_reduce_start with CCL_COMP_HOST_SHARE*=0: the GPU
              alone (the asynchronous path before the split request)

For each: GiB/s of bucket (best and median of --reps, start to wait) and the
microseconds the caller spends inside start (what a schedule entry's start()
would block its worker for).  Buffers are 0x3F bytes (no denormals).

  python tools/async_split_probe.py [--mib 32,64,256,1024] [--reps 8] [--pin]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

MODES = {"sync": {}, "async": {}, "async-gpu": {"CCL_COMP_HOST_SHARE": "0", "CCL_COMP_HOST_SHARE_PINNED": "0"}}
KNOBS = ("CCL_COMP_HOST_SHARE", "CCL_COMP_HOST_SHARE_PINNED")


def buffers(kind, nbytes):
    import numpy as np
    import torch
    if kind == "pinned":
        a = torch.full((nbytes,), 0x3F, dtype=torch.uint8).pin_memory()
        b = torch.full((nbytes,), 0x3F, dtype=torch.uint8).pin_memory()
        return (a, b), a.data_ptr(), b.data_ptr(), lambda: b.fill_(0x3F)
    a = np.full(nbytes, 0x3F, np.uint8)
    b = np.full(nbytes, 0x3F, np.uint8)
    return (a, b), a.ctypes.data, b.ctypes.data, lambda: b.fill(0x3F)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", default="32,64,256,1024")
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--pin", action="store_true", help="after loading the library, pin this thread to one core "
                                                        "(a oneCCL worker under CCL_WORKER_AFFINITY)")
    args = ap.parse_args()
    from oneccl_amd import _lib, comp
    _lib.mi()
    _lib.shim()
    if args.pin:
        os.sched_setaffinity(0, {max(os.sched_getaffinity(0))})
    from concurrent.futures import ThreadPoolExecutor

    # one persistent thread per mode: a thread's adapted split share (and its
    # GPU-alone timing) lives in thread-local state that env_reload, called
    # from this thread to switch modes, leaves alone
    execs = {m: ThreadPoolExecutor(max_workers=1) for m in MODES}
    if args.pin:
        for ex in execs.values():
            ex.submit(os.sched_setaffinity, 0, {max(os.sched_getaffinity(0))}).result()

    def one(mode, pa, pb, n):
        t0 = time.perf_counter()
        if mode == "sync":
            comp.comp_reduce(pa, n, pb, comp.datatype.float32, comp.reduction.sum)
            t_start = time.perf_counter() - t0
        else:
            req = comp.comp_reduce_start(pa, n, pb, comp.datatype.float32, comp.reduction.sum)
            t_start = time.perf_counter() - t0
            req.wait()
            req.free()
        return time.perf_counter() - t0, t_start

    for mib in (int(x) for x in args.mib.split(",")):
        nbytes = mib << 20
        n = nbytes // 4
        for kind in ("pageable", "pinned"):
            keep, pa, pb, reset = buffers(kind, nbytes)
            res = {m: ([], []) for m in MODES}
            for rep in range(args.reps + 1):  # rep 0 warms every mode's staging and shares
                for j in range(len(MODES)):
                    mode = list(MODES)[(rep + j) % len(MODES)]
                    for k in KNOBS:
                        os.environ.pop(k, None)
                    os.environ.update(MODES[mode])
                    comp.env_reload()
                    reset()
                    dt, t_start = execs[mode].submit(one, mode, pa, pb, n).result()
                    if rep:
                        res[mode][0].append(nbytes / dt / 2**30)
                        res[mode][1].append(t_start * 1e6)
            for mode, (rates, starts) in res.items():
                print(json.dumps({"bucket_MiB": mib, "memory": kind, "mode": mode, "caller_pinned": args.pin,
                                  "best_GiBps": round(max(rates), 2), "median_GiBps": round(statistics.median(rates), 2),
                                  "caller_blocked_us_median": round(statistics.median(starts), 1)}), flush=True)
            del keep
    for ex in execs.values():
        ex.shutdown()
    for k in KNOBS:
        os.environ.pop(k, None)
    comp.env_reload()


if __name__ == "__main__":
    main()
