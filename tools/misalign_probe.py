#!/usr/bin/env python3
"""Rate of mi_reduce when the operands' misalignments (mod 16 bytes) differ —
the shape of oneCCL ring chunks whose element counts are not multiples of
16 / element size (allreduce.cpp:346-366 offsets = idx * elem_count * size).
Times the 2-input and the 8-input fan-in on 256 MiB buckets for several
(in, inout) byte offsets and prints one JSON line per case.

  python tools/misalign_probe.py [--mib 256] [--reps 20]
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--mib", type=int, default=256)
    p.add_argument("--reps", type=int, default=20)
    args = p.parse_args()
    import torch

    from oneccl_amd import _lib
    m = _lib.mi()
    s = torch.cuda.current_stream()
    sh = s.cuda_stream
    nbytes = args.mib << 20
    cases = []
    for dt, es, name in ((9, 4, "f32"), (11, 2, "bf16"), (0, 1, "int8")):
        for offs in ((0, 0), (es, es), (es, 0), (0, es), (3 * es, es)):
            if offs[0] % 16 == offs[1] % 16 == 0 or offs[0] == offs[1]:
                kinds = "common"
            else:
                kinds = "differ"
            cases.append((dt, es, name, 2, offs, kinds))
        cases.append((dt, es, name, 8, (es,) + (0,) * 7 + (0,), "differ"))
        cases.append((dt, es, name, 8, (0,) * 9, "common"))
    for dt, es, name, k, offs, kinds in cases:
        n = nbytes // es - 64
        bufs = [torch.empty(nbytes + 64, dtype=torch.uint8, device="cuda") for _ in range(k + (0 if k == 2 else 1))]
        for b in bufs:
            b.random_(0, 64)
        if k == 2:
            pin, pio = bufs[0].data_ptr() + offs[0], bufs[1].data_ptr() + offs[1]

            def step():
                return m.mi_reduce(pin, pio, n, dt, 0, 0, sh)
        else:
            ptrs = [bufs[i].data_ptr() + offs[i] for i in range(k)]
            arr = _lib.void_ptr_array(ptrs)
            pout = bufs[k].data_ptr() + offs[k]

            def step():
                return m.mi_reduce_multi(arr, k, pout, n, dt, 0, 0, sh)
        for _ in range(3):
            _lib.check(step())
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.reps)]
        for a, b in ev:
            a.record(s)
            _lib.check(step())
            b.record(s)
        torch.cuda.synchronize()
        ms = statistics.median([a.elapsed_time(b) for a, b in ev])
        tbs = (k + 1) * n * es / (ms / 1e3) / 1e12
        print(json.dumps({"dtype": name, "inputs": k, "byte_offsets": list(offs), "alignment": kinds,
                          "median_ms": round(ms, 4), "TB_s": round(tbs, 3)}), flush=True)
        del bufs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
