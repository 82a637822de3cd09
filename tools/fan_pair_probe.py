#!/usr/bin/env python3
"""Does one pair of inputs set the 8-input fan-in's placement mode, as one
pair sets the 2-input reduce's (tools/pair_probe.py --streams)?

Per trial: a random pad, eight fresh 1 GiB fp32 inputs (separate
allocations, or one allocation with --layout one), then
  fan_ms    the library's 8-input fan-in in place (mi_reduce_multi);
  read8_ms  the eight read together with no arithmetic (libmi_ceiling.so);
  read2_ms  every unordered pair of them read together.
One JSON line per trial.

  python tools/fan_pair_probe.py [--trials 8] [--layout separate|one]
"""
from __future__ import annotations

import argparse
import ctypes
import itertools
import json
import random
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=8)
    ap.add_argument("--launches", type=int, default=10)
    ap.add_argument("--layout", choices=("separate", "one"), default="separate")
    ap.add_argument("--seed", type=int, default=9)
    a = ap.parse_args()
    import torch

    import bench
    from oneccl_amd import _lib
    m = _lib.mi()
    L = ctypes.CDLL(str(ROOT / "oneccl_amd" / "lib" / "libmi_ceiling.so"))
    L.mic_read_streams.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_size_t, ctypes.c_int,
                                   ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    s = torch.cuda.current_stream()
    sh = s.cuda_stream
    k, n = 8, (1 << 30) // 4
    nb = n * 4
    sink = torch.zeros(1024, dtype=torch.int32, device="cuda")
    rng = random.Random(a.seed)

    def timed(fn):
        for _ in range(2):
            _lib.check(fn())
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(a.launches):
            fn()
        e1.record(s)
        torch.cuda.synchronize()
        return round(e0.elapsed_time(e1) / a.launches, 5)

    for trial in range(a.trials):
        torch.cuda.empty_cache()
        pad_mib = 2 * rng.randrange(0, 1536)
        pad = torch.empty(pad_mib << 18, dtype=torch.float32, device="cuda") if pad_mib else None
        ins = bench.alloc_inputs(k, n, torch.float32, a.layout)
        for j, t in enumerate(ins):
            t.uniform_(-1, 1)
        arr = _lib.void_ptr_array([t.data_ptr() for t in ins])
        fan = timed(lambda: m.mi_reduce_multi(arr, k, ins[0].data_ptr(), n, 9, 0, 0, sh))
        read8 = timed(lambda: L.mic_read_streams(arr, k, nb, 64, 0, 0, sink.data_ptr(), sh))
        read2 = {}
        for i, j in itertools.combinations(range(k), 2):
            pa = _lib.void_ptr_array([ins[i].data_ptr(), ins[j].data_ptr()])
            read2[f"{i}{j}"] = timed(lambda: L.mic_read_streams(pa, 2, nb, 64, 0, 0, sink.data_ptr(), sh))
        lo = min(read2.values())
        print(json.dumps({"trial": trial, "layout": a.layout, "pad_MiB": pad_mib, "fan_ms": fan, "read8_ms": read8,
                          "read2_min_ms": lo, "read2_max_ms": max(read2.values()),
                          "slow_pairs": sorted(p for p, v in read2.items() if v > lo * 1.04),
                          "read2_ms": read2}), flush=True)
        del ins, arr, pad


if __name__ == "__main__":
    main()
