#!/usr/bin/env python3
"""The library's resident-wave plan against its neighbours, per bench config,
over fresh allocations.

Round 3 chose the one-wave kernels' caps from single-placement sweeps; round 4
found that C2 runs in placement modes (tools/pair_probe.py) and that the
granule sweep and the per-pair sweep disagree by about 1 % on which residency
is best.  Here each trial frees everything, allocates a random pad and fresh
inputs of every config, and times the library's own launch (mi_reduce /
mi_reduce_multi, in place as bench.py runs it) at each residency through
mi_set_residency, the residencies rotated between trials so no one is always
first.  One JSON line per trial x config, then per config the median over
trials of each residency's time relative to the plan's.

  python tools/residency_ab.py [--trials 8] [--configs c2,c3-bf16,...] [--launches 10]
"""
from __future__ import annotations

import argparse
import json
import random
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

WAVES = {2: [16, 18, 21, 25, 32], 8: [8, 9, 10, 12, 14]}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=8)
    ap.add_argument("--configs", default="c2,c3-bf16,c3-fp16,c5-int32-max,c5-int64-prod,c4")
    ap.add_argument("--launches", type=int, default=10)
    ap.add_argument("--seed", type=int, default=5)
    a = ap.parse_args()
    import ctypes

    import torch

    import bench
    from oneccl_amd import _lib
    m = _lib.mi()
    s = torch.cuda.current_stream()
    sh = s.cuda_stream
    rng = random.Random(a.seed)
    names = a.configs.split(",")
    plan = {}
    for name in names:
        k = bench.CONFIGS[name][4]
        w = ctypes.c_int()
        _lib.check(m.mi_get_residency(-1, k, ctypes.byref(w), None))
        plan[name] = w.value
    rel = {name: {w: [] for w in WAVES[bench.CONFIGS[name][4]]} for name in names}
    for trial in range(a.trials):
        torch.cuda.empty_cache()
        pad_mib = 2 * rng.randrange(0, 1536)
        pad = torch.empty(pad_mib << 18, dtype=torch.float32, device="cuda") if pad_mib else None
        for name in names:
            _, dt, es, op, k, bucket, flags = bench.CONFIGS[name]
            n = bucket // es
            ins = [torch.empty(n, dtype=bench.torch_dtype(dt), device="cuda") for _ in range(k)]
            for i, t in enumerate(ins):
                bench.fill(t, 1000 * trial + i)
            arr = _lib.void_ptr_array([t.data_ptr() for t in ins])

            def launch():
                if k == 2:
                    return m.mi_reduce(ins[1].data_ptr(), ins[0].data_ptr(), n, dt, op, flags, sh)
                return m.mi_reduce_multi(arr, k, ins[0].data_ptr(), n, dt, op, flags, sh)

            ws = WAVES[k]
            r = trial % len(ws)
            order = ws[r:] + ws[:r]
            ms = {}
            try:
                for w in order:
                    _lib.check(m.mi_set_residency(k, w))
                    for _ in range(2):
                        _lib.check(launch())
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(s)
                    for _ in range(a.launches):
                        launch()
                    e1.record(s)
                    e1.synchronize()
                    ms[w] = round(e0.elapsed_time(e1) / a.launches, 5)
            finally:
                _lib.check(m.mi_set_residency(k, 0))
            for w in ws:
                rel[name][w].append(ms[w] / ms[plan[name]])
            print(json.dumps({"trial": trial, "config": name, "pad_MiB": pad_mib, "plan_waves": plan[name],
                              "ms_by_waves": {str(w): ms[w] for w in ws}, "order": order}), flush=True)
            del ins, arr
        del pad
    for name in names:
        print(json.dumps({"summary": True, "config": name, "trials": a.trials, "plan_waves": plan[name],
                          "median_time_vs_plan": {str(w): round(statistics.median(v), 4)
                                                  for w, v in rel[name].items()},
                          "best_waves_by_median": min(rel[name], key=lambda w: statistics.median(rel[name][w]))}),
              flush=True)


if __name__ == "__main__":
    main()
