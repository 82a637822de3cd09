#!/usr/bin/env python3
"""How much of a device-resident reduce's time is where its buffers land?

The same kernel on the same box measured 0.471 ms per 1 GiB fp32 2-input
reduce on the occupancy sweep's buffers and 0.487 ms on bench.py's
(profiles/round4_run3/), and round 3 saw the 8-input fan-in move 1.51-1.59 ms
with its buffers' placement (tools/c4_placement_probe.py).  The kernel cannot
see physical addresses, so this probe measures the spread itself: `trials`
times, it frees everything, allocates a random pad (0-3 GiB in 2 MiB steps)
and K fresh 1 GiB inputs, and times 20 in-place launches of the library's
reduce (mi_reduce for K = 2, mi_reduce_multi otherwise) between HIP events.
One JSON line per trial, then a summary line.

  python tools/placement_probe.py [--inputs 2] [--trials 12] [--seed 1] [--offsets] [--layout L]
--layout: `separate` (default) one allocation per input; `one` all K inputs
consecutive slices of one allocation; `nreduce` the accumulator alone and the
other K - 1 inputs in one allocation, as oneCCL's nreduce lays out the peers'
chunks in its tmp buffer (allreduce.cpp:333-394).
--gap-mib G (layouts one / nreduce): G MiB between consecutive slices.
--bucket-mib B: each input B MiB of fp32 (default 1024).
--offsets (2 inputs): in each trial `in` is allocated 2 MiB larger and the
same launch is timed with `in` shifted by 0, 4 KiB, 64 KiB and 1 MiB from its
start, so the two operands' relative alignment changes while their pages do
not.
"""
from __future__ import annotations

import argparse
import json
import random
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--inputs", type=int, default=2)
    ap.add_argument("--trials", type=int, default=12)
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--offsets", action="store_true")
    ap.add_argument("--layout", choices=("separate", "one", "nreduce"), default="separate")
    ap.add_argument("--gap-mib", type=int, default=0)
    ap.add_argument("--bucket-mib", type=int, default=1024, help="bytes per input (fp32)")
    a = ap.parse_args()
    import torch

    from oneccl_amd import _lib
    m = _lib.mi()
    s = torch.cuda.current_stream()
    n = (a.bucket_mib << 20) // 4
    nb = n * 4
    k = a.inputs
    rng = random.Random(a.seed)
    meds = []
    if a.offsets:
        return offsets_mode(a, m, s, n, rng)
    for trial in range(a.trials):
        torch.cuda.empty_cache()
        pad_mib = 2 * rng.randrange(0, 1536)
        pad = torch.empty(pad_mib << 18, dtype=torch.float32, device="cuda") if pad_mib else None
        if a.layout == "separate":
            ins = [torch.empty(n, dtype=torch.float32, device="cuda").uniform_(-1, 1) for _ in range(k)]
        else:
            first = 0 if a.layout == "one" else 1
            ins = [torch.empty(n, dtype=torch.float32, device="cuda").uniform_(-1, 1)] if first else []
            stride = n + (a.gap_mib << 18)
            slab = torch.empty((k - first) * stride, dtype=torch.float32, device="cuda").uniform_(-1, 1)
            ins += [slab[j * stride:j * stride + n] for j in range(k - first)]
            del slab
        arr = _lib.void_ptr_array([t.data_ptr() for t in ins])

        def launch():
            if k == 2:
                return m.mi_reduce(ins[1].data_ptr(), ins[0].data_ptr(), n, 9, 0, 0, s.cuda_stream)
            return m.mi_reduce_multi(arr, k, ins[0].data_ptr(), n, 9, 0, 0, s.cuda_stream)

        for _ in range(3):
            _lib.check(launch())
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.launches):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            _lib.check(launch())
            e1.record(s)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        med = ts[len(ts) // 2]
        meds.append(med)
        print(json.dumps({"trial": trial, "inputs": k, "layout": a.layout, "gap_MiB": a.gap_mib, "pad_MiB": pad_mib, "median_ms": round(med, 5),
                          "best_ms": round(ts[0], 5), "TBps_median": round((k + 1) * nb / med / 1e9, 3),
                          "addr_GiB": [round(t.data_ptr() / 2**30, 3) for t in ins]}), flush=True)
        del ins, arr, pad
    print(json.dumps({"summary": True, "inputs": k, "layout": a.layout, "gap_MiB": a.gap_mib, "trials": a.trials, "min_ms": round(min(meds), 5),
                      "median_ms": round(statistics.median(meds), 5), "max_ms": round(max(meds), 5),
                      "spread": round(max(meds) / min(meds) - 1, 4),
                      "frac_of_8TBps_best": round((k + 1) * nb / (min(meds) / 1e3) / 1e12 / 8.0, 4),
                      "frac_of_8TBps_worst": round((k + 1) * nb / (max(meds) / 1e3) / 1e12 / 8.0, 4)}),
          flush=True)


def offsets_mode(a, m, s, n, rng):
    import torch

    from oneccl_amd import _lib
    offs = [0, 4096, 65536, 1 << 20]
    rows = []
    for trial in range(a.trials):
        torch.cuda.empty_cache()
        pad_mib = 2 * rng.randrange(0, 1536)
        pad = torch.empty(pad_mib << 18, dtype=torch.float32, device="cuda") if pad_mib else None
        acc = torch.empty(n, dtype=torch.float32, device="cuda").uniform_(-1, 1)
        inb = torch.empty(n + (2 << 20) // 4, dtype=torch.float32, device="cuda").uniform_(-1, 1)
        res = {}
        for off in offs:
            pin = inb.data_ptr() + off

            def launch():
                return m.mi_reduce(pin, acc.data_ptr(), n, 9, 0, 0, s.cuda_stream)

            for _ in range(3):
                _lib.check(launch())
            torch.cuda.synchronize()
            ts = []
            for _ in range(a.launches):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                _lib.check(launch())
                e1.record(s)
                e1.synchronize()
                ts.append(e0.elapsed_time(e1))
            ts.sort()
            res[off] = round(ts[len(ts) // 2], 5)
        rows.append(res)
        print(json.dumps({"trial": trial, "pad_MiB": pad_mib, "median_ms_by_in_offset": res,
                          "addr_GiB": [round(acc.data_ptr() / 2**30, 3), round(inb.data_ptr() / 2**30, 3)]}),
              flush=True)
        del acc, inb, pad
    print(json.dumps({"summary": True, "mode": "offsets", "trials": a.trials,
                      "median_ms_by_in_offset": {o: round(statistics.median(r[o] for r in rows), 5) for o in offs},
                      "max_ms_by_in_offset": {o: max(r[o] for r in rows) for o in offs}}), flush=True)


if __name__ == "__main__":
    main()
