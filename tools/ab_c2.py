#!/usr/bin/env python3
"""A/B of two builds of libmi_reduce.so on the same box, same buffers,
interleaved rounds: the C2 headline launch (2-input fp32 sum, 1 GiB) or any
bench config's 2-input / K-input launch.  Box-to-box spread (~5 %) hides
kernel changes of a few percent; this does not.

  python tools/ab_c2.py LIB_A LIB_B [--config c2] [--rounds 8] [--launches 20]

Prints one JSON line per (round, lib) and a summary line: mean / min launch
time and the B/A ratio.  Measurement tool only (not product, not a test)."""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("lib_a")
    p.add_argument("lib_b")
    p.add_argument("--config", default="c2")
    p.add_argument("--rounds", type=int, default=8)
    p.add_argument("--launches", type=int, default=20)
    p.add_argument("--trials", type=int, default=1,
                   help="fresh operands (after a random pad) per trial: the A/B over placements")
    p.add_argument("--layout", default="separate", choices=["separate", "padded", "one"])
    a = p.parse_args()
    import torch

    import bench
    # "copy": ccl_comp_copy's device kernel (mi_copy), 1 GiB from ins[1] to ins[0]
    desc, dt, es, op, k, bucket, flags = bench.CONFIGS["c2" if a.config == "copy" else a.config]
    n = bucket // es
    libs = {}
    for name, path in (("A", a.lib_a), ("B", a.lib_b)):
        L = ctypes.CDLL(str(Path(path).resolve()), mode=os.RTLD_LOCAL)
        L.mi_reduce.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                ctypes.c_uint, ctypes.c_void_p]
        L.mi_reduce_multi.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                      ctypes.c_int, ctypes.c_int, ctypes.c_uint, ctypes.c_void_p]
        L.mi_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
        libs[name] = L
    import random
    rng = random.Random(17)
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream
    res = {"A": [], "B": []}
    ratios = []
    for trial in range(a.trials):
        torch.cuda.empty_cache()
        pad_mib = 2 * rng.randrange(0, 1536) if a.trials > 1 else 0
        pad = torch.empty(pad_mib << 18, dtype=torch.float32, device="cuda") if pad_mib else None
        ins = bench.alloc_inputs(k, n, bench.torch_dtype(dt), a.layout)
        tr = one_trial(a, libs, ins, k, n, es, dt, op, flags, sh, stream, trial)
        for name in ("A", "B"):
            res[name] += tr[name]
        ratios.append(statistics.mean(tr["B"]) / statistics.mean(tr["A"]))
        del ins, pad
    algo = (2 if a.config == "copy" else k + 1) * n * es
    out = {"config": a.config, "layout": a.layout, "trials": a.trials, "lib_a": a.lib_a, "lib_b": a.lib_b,
           "launches_per_round": a.launches}
    for name in ("A", "B"):
        out[name] = {"mean_ms": round(statistics.mean(res[name]), 5), "min_ms": round(min(res[name]), 5),
                     "frac_of_8TBps_at_mean": round(algo / (statistics.mean(res[name]) / 1e3) / 8e12, 4)}
    out["B_over_A_mean_time"] = round(statistics.mean(res["B"]) / statistics.mean(res["A"]), 4)
    out["B_over_A_per_trial"] = {"median": round(statistics.median(ratios), 4), "min": round(min(ratios), 4),
                                 "max": round(max(ratios), 4)}
    print(json.dumps(out), flush=True)


def one_trial(a, libs, ins, k, n, es, dt, op, flags, sh, stream, trial):
    import torch

    import bench
    for j, t in enumerate(ins):
        bench.fill(t, 0xAB + j)
    arr = (ctypes.c_void_p * k)(*[t.data_ptr() for t in ins])

    def launch(L):
        if a.config == "copy":
            return L.mi_copy(ins[1].data_ptr(), ins[0].data_ptr(), n * es, 0, sh)
        if k == 2:
            return L.mi_reduce(ins[1].data_ptr(), ins[0].data_ptr(), n, dt, op, flags, sh)
        return L.mi_reduce_multi(arr, k, ins[0].data_ptr(), n, dt, op, flags, sh)

    for L in libs.values():  # warm both
        for _ in range(3):
            assert launch(L) == 0
    torch.cuda.synchronize()
    res = {"A": [], "B": []}
    for r in range(a.rounds):
        order = ("A", "B") if r % 2 == 0 else ("B", "A")
        for name in order:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(a.launches):
                assert launch(libs[name]) == 0
            e1.record(stream)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.launches
            res[name].append(ms)
            print(json.dumps({"trial": trial, "round": r, "lib": name, "avg_launch_ms": round(ms, 5)}), flush=True)
    return res


if __name__ == "__main__":
    main()
