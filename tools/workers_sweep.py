#!/usr/bin/env python3
"""Host-resident buckets under W concurrent workers (SURVEY.md §8f rank 1:
"whether GPU offload ever wins over W CPU workers").  oneCCL runs each reduce
entry on one worker thread; with CCL_WORKER_COUNT=W the parallelizer gives
each worker its own part of a large collective, so W threads call
ccl_comp_reduce at once, each on its own host buffers
(src/exec/thread/worker.cpp:310-379, src/parallelizer/parallelizer.cpp:230-244).

For each W and per-worker bucket, W persistent threads (each first-touches
its own pageable buffers) run `--reps` rounds; a round starts on a barrier
and ends when every thread has returned.  Modes:
  oracle    each thread calls the CPU oracle (the reference's CCL_REDUCE loop)
  host      the drop-in with every host bucket on the calling thread's CPU
  gpu       the drop-in with every host bucket on the GPU
  default   the drop-in's dispatcher as shipped (CPU below the threshold,
            adaptive GPU + CPU split above it)
One JSON line per (W, bucket, mode): aggregate GiB/s (W x bucket / round time)
of every round, so the adaptive split's first rounds show, plus the best and
the median of the last half.  The inputs are 0x3F bytes (no denormals).

  python tools/workers_sweep.py [--workers 1,2,4,8,16] [--mib 8,64] [--reps 10]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import threading
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

KNOBS = ("CCL_COMP_HOST_MAX_BYTES", "CCL_COMP_HOST_MAX_PINNED_BYTES", "CCL_COMP_HOST_SHARE",
         "CCL_COMP_HOST_SHARE_PINNED", "CCL_COMP_HOST_SHARE_ADAPT")
MODES = {
    "oracle": None,
    "host": {"CCL_COMP_HOST_MAX_BYTES": str(1 << 40), "CCL_COMP_HOST_MAX_PINNED_BYTES": str(1 << 40)},
    "gpu": {"CCL_COMP_HOST_MAX_BYTES": "0"},
    "default": {},
}


def run_mode(mode, w, nbytes, reps, f32=9):
    import numpy as np

    import oracle
    from oneccl_amd import comp
    for k in KNOBS:
        os.environ.pop(k, None)
    if MODES[mode] is not None:
        os.environ.update(MODES[mode])
        comp.env_reload()
    n = nbytes // 4
    start, end = threading.Barrier(w + 1), threading.Barrier(w + 1)
    errors = []
    shares = [None] * w

    def worker(i):
        try:
            a = np.full(nbytes, 0x3F, np.uint8)  # first touch on this thread
            b = np.full(nbytes, 0x3F, np.uint8)
            fa, fb = a.view(np.float32), b.view(np.float32)
            pa, pb = a.ctypes.data, b.ctypes.data
            shim = None
            if mode != "oracle":
                from oneccl_amd import _lib
                shim = _lib.shim()
            for _ in range(reps):
                start.wait()
                if mode == "oracle":
                    oracle.comp_reduce(fa, fb, f32, 0)
                else:
                    comp.comp_reduce(pa, n, pb, comp.datatype(f32), comp.reduction.sum)
                end.wait()
                b[:] = 0x3F  # outside the round: keep values away from overflow
            if shim is not None:
                shares[i] = round(shim.mi_ccl_comp_split_share(0), 4)
        except Exception as e:  # noqa: BLE001 - reported in the JSON line
            errors.append(repr(e))
            start.abort()
            end.abort()

    ts = [threading.Thread(target=worker, args=(i,), daemon=True) for i in range(w)]
    for t in ts:
        t.start()
    rates = []
    try:
        for _ in range(reps):
            start.wait()
            t0 = time.perf_counter()
            end.wait()
            rates.append(w * nbytes / (time.perf_counter() - t0) / 2**30)
    except threading.BrokenBarrierError:
        pass
    for t in ts:
        t.join()
    for k in KNOBS:
        os.environ.pop(k, None)
    comp.env_reload()
    row = {"workers": w, "bucket_MiB_per_worker": nbytes >> 20, "mode": mode,
           "GiBps_per_round": [round(r, 2) for r in rates]}
    if rates:
        tail = rates[len(rates) // 2:]
        row.update(best_GiBps=round(max(rates), 2), steady_median_GiBps=round(statistics.median(tail), 2))
    if mode == "default":
        row["split_share_per_worker"] = shares
    if errors:
        row["errors"] = errors
    return row


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", default="1,2,4,8,16")
    ap.add_argument("--mib", default="8,64")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--modes", default="oracle,host,gpu,default")
    args = ap.parse_args()
    for mib in (int(x) for x in args.mib.split(",")):
        for w in (int(x) for x in args.workers.split(",")):
            for mode in args.modes.split(","):
                print(json.dumps(run_mode(mode, w, mib << 20, args.reps)), flush=True)


if __name__ == "__main__":
    main()
