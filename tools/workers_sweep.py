#!/usr/bin/env python3
"""Host-resident buckets under W concurrent workers (SURVEY.md §8f rank 1:
"whether GPU offload ever wins over W CPU workers").  oneCCL runs each reduce
entry on one worker thread; with CCL_WORKER_COUNT=W the parallelizer gives
each worker its own part of a large collective, so W threads call
ccl_comp_reduce at once, each on its own host buffers
(src/exec/thread/worker.cpp:310-379, src/parallelizer/parallelizer.cpp:230-244).

For each W and per-worker bucket, W persistent threads (each first-touches
its own buffers; `--pinned` also registers them with the GPU) run `--reps`
rounds of every mode.  A round starts on a barrier and ends when every thread
has returned.  The modes take turns round by round, in an order rotated each
rep, so a neighbour's load on the shared host falls on all of them alike.
Modes:
  oracle    each thread calls the CPU oracle (the reference's CCL_REDUCE loop)
  host      the drop-in with every host bucket on the calling thread's CPU
  gpu       the drop-in with every host bucket on the GPU
  split     the drop-in splitting every bucket above the threshold with the
            GPU whatever the number of workers (CCL_COMP_HOST_SPLIT_WORKERS=0)
  default   the drop-in's dispatcher as shipped
One JSON line per (W, bucket, mode): aggregate GiB/s (W x bucket / round
time) of every round, the best and the median of the second half, the
threads' adapted split shares, and the cgroup's CPU throttling and the
process's thread count over the mode's rounds.  The inputs are 0x3F bytes (no
denormals).

  python tools/workers_sweep.py [--workers 1,2,4,8,16] [--mib 8,64] [--reps 10] [--pinned] [--pin]
"""
from __future__ import annotations

import argparse
import faulthandler
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
         "CCL_COMP_HOST_SHARE_PINNED", "CCL_COMP_HOST_SHARE_ADAPT", "CCL_COMP_HOST_SPLIT_WORKERS",
         "CCL_COMP_HOST_SPLIT_WORKERS_PINNED")
MODES = {
    "oracle": {},
    "host": {"CCL_COMP_HOST_MAX_BYTES": str(1 << 40), "CCL_COMP_HOST_MAX_PINNED_BYTES": str(1 << 40)},
    "gpu": {"CCL_COMP_HOST_MAX_BYTES": "0"},
    "split": {"CCL_COMP_HOST_SPLIT_WORKERS": "0", "CCL_COMP_HOST_SPLIT_WORKERS_PINNED": "0"},
    "default": {},
}


def cpu_throttle():
    """(nr_throttled, throttled_usec) of this cgroup, or None."""
    try:
        kv = dict(line.split() for line in Path("/sys/fs/cgroup/cpu.stat").read_text().splitlines())
        return int(kv.get("nr_throttled", 0)), int(kv.get("throttled_usec", 0))
    except (OSError, ValueError):
        return None


def nthreads():
    for line in Path("/proc/self/status").read_text().splitlines():
        if line.startswith("Threads:"):
            return int(line.split()[1])
    return -1


def set_mode(mode):
    from oneccl_amd import comp
    for k in KNOBS:
        os.environ.pop(k, None)
    os.environ.update(MODES[mode])
    comp.env_reload()


def run_point(modes, w, nbytes, reps, pinned, pin=None, f32=9):
    import numpy as np

    import oracle
    from oneccl_amd import _lib, comp
    n = nbytes // 4
    start, end = threading.Barrier(w + 1), threading.Barrier(w + 1)
    cur = {"mode": None}
    errors = []
    shares = [None] * w

    def worker(i):
        try:
            if pin:  # one core per worker, as oneCCL pins its workers (CCL_WORKER_AFFINITY)
                os.sched_setaffinity(0, {pin[i % len(pin)]})
            a = np.full(nbytes, 0x3F, np.uint8)  # first touch on this thread
            b = np.full(nbytes, 0x3F, np.uint8)
            fa, fb = a.view(np.float32), b.view(np.float32)
            pa, pb = a.ctypes.data, b.ctypes.data
            m = _lib.mi()
            if pinned:
                _lib.check(m.mi_host_register(pa, nbytes))
                _lib.check(m.mi_host_register(pb, nbytes))
            try:
                for _ in range(reps * len(modes)):
                    start.wait()
                    if cur["mode"] == "oracle":
                        oracle.comp_reduce(fa, fb, f32, 0)
                    else:
                        comp.comp_reduce(pa, n, pb, comp.datatype(f32), comp.reduction.sum)
                    end.wait()
                    b[:] = 0x3F  # outside the round: keep values away from overflow
                shares[i] = round(_lib.shim().mi_ccl_comp_split_share(1 if pinned else 0), 4)
            finally:
                if pinned:
                    m.mi_host_unregister(pa)
                    m.mi_host_unregister(pb)
        except Exception as e:  # noqa: BLE001 - reported in the JSON line
            errors.append(repr(e))
            start.abort()
            end.abort()

    ts = [threading.Thread(target=worker, args=(i,), daemon=True) for i in range(w)]
    for t in ts:
        t.start()
    rates = {m: [] for m in modes}
    thr = {m: [0, 0] for m in modes}
    workers_seen = {m: [] for m in modes}
    maxthreads = 0
    try:
        for r in range(reps):
            for j in range(len(modes)):
                mode = modes[(r + j) % len(modes)]
                set_mode(mode)
                cur["mode"] = mode
                t_before = cpu_throttle()
                start.wait()
                t0 = time.perf_counter()
                end.wait()
                dt = time.perf_counter() - t0
                workers_seen[mode].append(_lib.shim().mi_ccl_comp_host_workers())
                t_after = cpu_throttle()
                if t_before and t_after:
                    thr[mode][0] += t_after[0] - t_before[0]
                    thr[mode][1] += t_after[1] - t_before[1]
                maxthreads = max(maxthreads, nthreads())
                rates[mode].append(w * nbytes / dt / 2**30)
    except threading.BrokenBarrierError:
        pass
    for t in ts:
        t.join()
    set_mode("default")
    rows = []
    for mode in modes:
        rs = rates[mode]
        row = {"workers": w, "bucket_MiB_per_worker": nbytes >> 20, "memory": "pinned" if pinned else "pageable",
               "mode": mode, "workers_pinned_to_cores": bool(pin), "GiBps_per_round": [round(x, 2) for x in rs]}
        if rs:
            tail = rs[len(rs) // 2:]
            row.update(best_GiBps=round(max(rs), 2), steady_median_GiBps=round(statistics.median(tail), 2))
        if mode != "oracle":
            row["host_workers_seen"] = sorted(set(workers_seen[mode]))
        row["cgroup_throttled"] = {"periods": thr[mode][0], "usec": thr[mode][1]}
        row["max_process_threads"] = maxthreads
        if errors:
            row["errors"] = errors
        rows.append(row)
    rows.append({"workers": w, "bucket_MiB_per_worker": nbytes >> 20, "memory": "pinned" if pinned else "pageable",
                 "split_share_per_worker": shares})
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", default="1,2,4,8,16")
    ap.add_argument("--mib", default="8,64")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--modes", default="oracle,host,split,default")
    ap.add_argument("--pinned", action="store_true", help="register each thread's buffers with the GPU")
    ap.add_argument("--segv-trace", action="store_true", help="native backtrace on SIGSEGV (tools/libsegv_trace.so)")
    ap.add_argument("--pin", action="store_true", help="pin each worker thread to its own core, as oneCCL does")
    args = ap.parse_args()
    if args.segv_trace:  # before faulthandler, which restores it when Python finalizes
        import ctypes
        ctypes.CDLL(str(ROOT / "tools" / "libsegv_trace.so"))
    faulthandler.enable()
    modes = args.modes.split(",")
    print(json.dumps({"host": {"cpus_allowed": len(os.sched_getaffinity(0)), "cpu.max": _read("/sys/fs/cgroup/cpu.max"),
                               "nproc": os.cpu_count()}}), flush=True)
    for mib in (int(x) for x in args.mib.split(",")):
        for w in (int(x) for x in args.workers.split(",")):
            pin = sorted(os.sched_getaffinity(0))[::-1] if args.pin else None  # oneCCL takes the last cores
            for row in run_point(modes, w, mib << 20, args.reps, args.pinned, pin):
                print(json.dumps(row), flush=True)
    print(json.dumps({"done": True}), flush=True)


def _read(p):
    try:
        return Path(p).read_text().strip()
    except OSError:
        return None


if __name__ == "__main__":
    main()
