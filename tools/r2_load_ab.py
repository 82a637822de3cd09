#!/usr/bin/env python3
"""The 2-input kernel's load form over fresh placements: the library's
reduce2_kernel (global nt loads, sc1 nt stores) against the same fold with
buffer nt loads (tools/ceiling_probe.hip mic_sum2_buffer), each at a few
one-wave residencies, and the mixed probe beside them.

Why: in round 6 the mixed probe (buffer loads, no arithmetic) ran 0.5-0.9 %
faster than the kernel on the same buffers, and in separate allocations the
kernel sat at 0.98 of it.  Each trial frees everything, allocates a random
pad and fresh operands in two layouts (separate allocations, the bench's
padded pair), and times every variant (order rotated per trial).  One JSON
line per trial x layout, then per layout the median over trials of each
variant's time relative to the library's plan.  The buffer fold's result is
checked bit for bit against torch (fp32 add) once per trial.

  python tools/r2_load_ab.py [--trials 10] [--launches 10]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import random
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=10)
    ap.add_argument("--launches", type=int, default=10)
    ap.add_argument("--seed", type=int, default=11)
    a = ap.parse_args()
    import torch

    import bench
    from oneccl_amd import _lib
    m = _lib.mi()
    L = ctypes.CDLL(str(ROOT / bench.CEILING_LIB))
    L.mic_sum2_buffer.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_void_p, ctypes.c_void_p]
    L.mic_mixed_streams.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_void_p,
                                    ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    s = torch.cuda.current_stream()
    sh = s.cuda_stream
    n = (1 << 30) // 4
    nb = n * 4
    plan = ctypes.c_int()
    _lib.check(m.mi_get_residency(-1, 2, ctypes.byref(plan), None))
    sink = torch.zeros(64, dtype=torch.int32, device="cuda")
    rng = random.Random(a.seed)
    variants = [f"lib w{w}" for w in (18, 21, 25)] + [f"buf w{w} f{f}" for w in (18, 21, 25) for f in (2, 1)] + \
               ["mixed w21 f2", "mixed w25 f2"]
    rel = {lay: {v: [] for v in variants} for lay in ("separate", "padded")}
    for trial in range(a.trials):
        torch.cuda.empty_cache()
        pad_mib = 2 * rng.randrange(0, 1536)
        pad = torch.empty(pad_mib << 18, dtype=torch.float32, device="cuda") if pad_mib else None
        for lay in ("separate", "padded"):
            ins = bench.alloc_inputs(2, n, torch.float32, lay)
            for j in range(2):
                bench.fill(ins[j], 0x77 + 13 * trial + j)
            io, x = ins[0], ins[1]
            arr = _lib.void_ptr_array([io.data_ptr(), x.data_ptr()])

            def launch(v):
                kind, w = v.split()[0], int(v.split()[1][1:])
                if kind == "lib":
                    return m.mi_reduce(x.data_ptr(), io.data_ptr(), n, 9, 0, 0, sh)
                f = int(v.split()[2][1:])
                if kind == "buf":
                    return L.mic_sum2_buffer(x.data_ptr(), io.data_ptr(), nb, w, f, sink.data_ptr(), sh)
                return L.mic_mixed_streams(arr, 2, io.data_ptr(), nb, 64, w, f, sh)

            order = variants[:]
            rng.shuffle(order)
            ms = {}
            for v in order:
                if v.startswith("lib"):
                    _lib.check(m.mi_set_residency(2, int(v.split()[1][1:])))
                for _ in range(2):
                    if launch(v):
                        raise SystemExit(f"launch refused: {v}")
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(a.launches):
                    launch(v)
                e1.record(s)
                torch.cuda.synchronize()
                ms[v] = e0.elapsed_time(e1) / a.launches
            _lib.check(m.mi_set_residency(2, 0))
            # the buffer fold's bits against torch's fp32 add, once
            bench.fill(io, 0x99 + trial)
            bench.fill(x, 0x9A + trial)
            exp = io + x
            torch.cuda.synchronize()
            _lib.check(L.mic_sum2_buffer(x.data_ptr(), io.data_ptr(), nb, plan.value, 2, sink.data_ptr(), sh))
            torch.cuda.synchronize()
            mism = bench.count_mismatches(io, exp)
            del exp
            base = ms[f"lib w{plan.value}"]
            for v in variants:
                rel[lay][v].append(ms[v] / base)
            print(json.dumps({"trial": trial, "layout": lay, "pad_MiB": pad_mib, "plan_waves": plan.value,
                              "ms": {v: round(ms[v], 5) for v in variants}, "buffer_fold_mismatches": mism}),
                  flush=True)
            del ins, io, x, arr
            torch.cuda.empty_cache()
        del pad
    for lay, d in rel.items():
        print(json.dumps({"summary": True, "layout": lay, "trials": a.trials, "plan": f"lib w{plan.value}",
                          "median_time_vs_plan": {v: round(statistics.median(r), 4) for v, r in d.items()},
                          "best_time_vs_plan": {v: round(min(r), 4) for v, r in d.items()},
                          "worst_time_vs_plan": {v: round(max(r), 4) for v, r in d.items()}}), flush=True)


if __name__ == "__main__":
    main()
