#!/usr/bin/env python3
"""Does the 8-input fan-in's rate depend on where its buffers sit?

bench.py's `--config c4` (buffers allocated first in a fresh process) timed
1.57 ms per launch while the same launch in its config legs (allocated after
other legs freed theirs) took 1.47 ms.  Here one process allocates the
eight 1 GiB inputs several ways and times 20 launches of each layout
(mi_reduce_multi, in place into input 0, HIP events), printing the buffer
addresses too.  Usage: python tools/c4_placement_probe.py
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main() -> None:
    import torch

    from oneccl_amd import _lib
    m = _lib.mi()
    s = torch.cuda.current_stream()
    n = (1 << 30) // 4

    def run(ins, label, launches=20):
        arr = _lib.void_ptr_array([t.data_ptr() for t in ins])
        for _ in range(3):
            _lib.check(m.mi_reduce_multi(arr, 8, ins[0].data_ptr(), n, 9, 0, 0, s.cuda_stream))
        torch.cuda.synchronize()
        ts = []
        for _ in range(launches):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            _lib.check(m.mi_reduce_multi(arr, 8, ins[0].data_ptr(), n, 9, 0, 0, s.cuda_stream))
            e1.record(s)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        print(json.dumps({"layout": label, "median_ms": round(ts[len(ts) // 2], 5), "best_ms": round(ts[0], 5),
                          "addr_GiB": [round(t.data_ptr() / 2**30, 3) for t in ins]}), flush=True)

    def fresh(pad_gib=0):
        pad = torch.empty(pad_gib << 28, dtype=torch.float32, device="cuda") if pad_gib else None
        ins = [torch.empty(n, dtype=torch.float32, device="cuda").uniform_(-1, 1) for _ in range(8)]
        return ins, pad

    ins, _ = fresh()
    run(ins, "first allocation in the process")
    run(ins, "same buffers again")
    del ins
    torch.cuda.empty_cache()
    ins, _ = fresh()
    run(ins, "reallocated after empty_cache")
    del ins
    torch.cuda.empty_cache()
    ins, pad = fresh(3)
    run(ins, "after a 3 GiB pad")
    del ins, pad
    torch.cuda.empty_cache()
    big = torch.empty(8 * n, dtype=torch.float32, device="cuda").uniform_(-1, 1)
    run([big[j * n:(j + 1) * n] for j in range(8)], "one 8 GiB allocation, inputs contiguous")
    del big
    torch.cuda.empty_cache()
    # inputs interleaved with 1 GiB holes
    hold = []
    ins = []
    for j in range(8):
        ins.append(torch.empty(n, dtype=torch.float32, device="cuda").uniform_(-1, 1))
        hold.append(torch.empty(n, dtype=torch.float32, device="cuda"))
    run(ins, "inputs with a 1 GiB allocation between each")
    del ins, hold
    torch.cuda.empty_cache()
    ins, _ = fresh()
    run(ins, "reallocated again")


if __name__ == "__main__":
    main()
