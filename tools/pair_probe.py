#!/usr/bin/env python3
"""Is C2's slow placement mode a property of one buffer or of a pair?

tools/placement_probe.py found the 1 GiB fp32 in-place reduce bimodal over
fresh allocations (0.473-0.480 ms or 0.508-0.511 ms) and independent of the
operands' relative offset.  Here, per trial, four fresh 1 GiB buffers are
allocated; each is read alone and written alone by the memory-only probes
(libmi_ceiling.so, best flavour), and every ordered pair is reduced in place
(acc, in) with mi_reduce.  One JSON line per trial.

--streams: per ordered pair also the reduce's traffic without its arithmetic,
so that the slow mode can be pinned on one interaction: both buffers read at
once (`read2`), `in` copied onto `acc` by the library's copy kernel (`copy`:
read one, write the other), and `acc` rewritten from itself (`self`: the
in-place read-modify-write of one buffer, mi_copy with src == dst).

--slab: the buffers are consecutive 1 GiB slices of one allocation, not
allocations of their own.

  python tools/pair_probe.py [--trials 4] [--buffers 4] [--streams] [--slab]
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
    ap.add_argument("--trials", type=int, default=4)
    ap.add_argument("--buffers", type=int, default=4)
    ap.add_argument("--launches", type=int, default=10)
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--streams", action="store_true")
    ap.add_argument("--slab", action="store_true")
    a = ap.parse_args()
    import torch

    from oneccl_amd import _lib
    m = _lib.mi()
    L = ctypes.CDLL(str(ROOT / "oneccl_amd" / "lib" / "libmi_ceiling.so"))
    L.mic_read_streams.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_size_t, ctypes.c_int,
                                   ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    L.mic_write_stream.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_void_p]
    s = torch.cuda.current_stream()
    sh = s.cuda_stream
    n = (1 << 30) // 4
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
        if a.slab:
            slab = torch.empty(a.buffers * n, dtype=torch.float32, device="cuda").uniform_(-1, 1)
            bufs = [slab[i * n:(i + 1) * n] for i in range(a.buffers)]
        else:
            bufs = [torch.empty(n, dtype=torch.float32, device="cuda").uniform_(-1, 1) for _ in range(a.buffers)]
        read1, write1 = {}, {}
        for i, b in enumerate(bufs):
            arr = _lib.void_ptr_array([b.data_ptr()])
            read1[i] = timed(lambda: L.mic_read_streams(arr, 1, nb, 64, 0, 0, sink.data_ptr(), sh))
            write1[i] = timed(lambda: L.mic_write_stream(b.data_ptr(), nb, 256, 0, 2, sh))
            b.uniform_(-1, 1)
        pairs = {}
        for i, j in itertools.permutations(range(a.buffers), 2):
            acc, inp = bufs[i], bufs[j]
            pairs[f"{i}{j}"] = timed(lambda: m.mi_reduce(inp.data_ptr(), acc.data_ptr(), n, 9, 0, 0, sh))
        row = {"trial": trial, "slab": a.slab, "pad_MiB": pad_mib, "read_1stream_ms": read1, "write_ms": write1,
               "reduce_ms_acc_in": pairs, "addr_GiB": [round(b.data_ptr() / 2**30, 3) for b in bufs]}
        if a.streams:
            read2, copy, self_ = {}, {}, {}
            for i, j in itertools.permutations(range(a.buffers), 2):
                acc, inp = bufs[i], bufs[j]
                arr = _lib.void_ptr_array([acc.data_ptr(), inp.data_ptr()])
                read2[f"{i}{j}"] = timed(lambda: L.mic_read_streams(arr, 2, nb, 64, 0, 0, sink.data_ptr(), sh))
                copy[f"{i}{j}"] = timed(lambda: m.mi_copy(inp.data_ptr(), acc.data_ptr(), nb, 1, sh))
            for i, b in enumerate(bufs):
                self_[i] = timed(lambda: m.mi_copy(b.data_ptr(), b.data_ptr(), nb, 1, sh))
            row.update({"read2_ms_acc_in": read2, "copy_ms_in_to_acc": copy, "self_copy_ms": self_})
        print(json.dumps(row), flush=True)
        del bufs, pad
        if a.slab:
            del slab


if __name__ == "__main__":
    main()
