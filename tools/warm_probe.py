#!/usr/bin/env python3
"""Per-launch kernel time of the C2 reduce over a long run, to see whether the
first launches after idle run slower (clock / power-state ramp) and how many
warm-up launches the bench needs.

  python tools/warm_probe.py [--steps 400] [--idle 1.0]
Prints one JSON line per phase: per-decile mean kernel ms.
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=400)
    p.add_argument("--idle", type=float, default=1.0)
    args = p.parse_args()
    import torch

    from oneccl_amd import _lib
    m = _lib.mi()
    n = (1 << 30) // 4
    a = torch.empty(n, device="cuda").uniform_(-1, 1)
    b = torch.empty(n, device="cuda").uniform_(-1, 1)
    s = torch.cuda.current_stream()
    sh = s.cuda_stream
    for phase in ("cold", "after_idle", "after_idle_2"):
        torch.cuda.synchronize()
        if phase != "cold":
            time.sleep(args.idle)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
        for i in range(args.steps):
            ev[i][0].record(s)
            _lib.check(m.mi_reduce(a.data_ptr(), b.data_ptr(), n, 9, 0, 0, sh))
            ev[i][1].record(s)
        torch.cuda.synchronize()
        ms = [x.elapsed_time(y) for x, y in ev]
        groups = [ms[i:i + 10] for i in range(0, min(len(ms), 100), 10)]
        dec = max(1, len(ms) // 10)
        print(json.dumps({"phase": phase, "first10": [round(v, 4) for v in ms[:10]],
                          "per10_first100": [round(statistics.mean(g), 4) for g in groups],
                          "per_decile": [round(statistics.mean(ms[i:i + dec]), 4) for i in range(0, len(ms), dec)],
                          "median": round(statistics.median(ms), 4), "min": round(min(ms), 4)}), flush=True)


if __name__ == "__main__":
    main()
