"""A/B of ccl_comp_copy's device kernel (mi_copy: copy_lean_kernel, nt loads,
plain or nt stores, no residency cap) against the one-wave memory-only copy of
tools/ceiling_probe.hip (mic_mixed_streams with K = 1: buffer nt loads, nt or
sc1 nt stores, residency capped by reserved LDS) on the same 1 GiB buffers,
interleaved over rounds in one process.  One JSON line per variant.
  python tools/copy_ab.py [--mib 1024] [--rounds 6] [--launches 20]"""
from __future__ import annotations

import argparse
import ctypes
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    import torch

    from oneccl_amd import _lib
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=1024)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--launches", type=int, default=20)
    a = ap.parse_args()
    nbytes = a.mib << 20
    m = _lib.mi()
    L = ctypes.CDLL(str(ROOT / "oneccl_amd" / "lib" / "libmi_ceiling.so"))
    L.mic_mixed_streams.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                    ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    src = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    dst = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    src.random_(0, 256)
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream
    arr = _lib.void_ptr_array([src.data_ptr()])
    variants = {"mi_copy (library, plain stores)": lambda: m.mi_copy(src.data_ptr(), dst.data_ptr(), nbytes, 0, sh),
                "mi_copy (library, nt stores)": lambda: m.mi_copy(src.data_ptr(), dst.data_ptr(), nbytes, 1, sh)}
    fl_name = {0: "global nt loads + nt stores", 1: "buffer nt loads + nt stores", 2: "buffer nt loads + sc1 nt stores"}
    for fl in (0, 1, 2):
        for w in (0, 16, 21, 25, 32):
            variants[f"one-wave copy, {fl_name[fl]}, {w or 'no'} cap"] = (
                lambda fl=fl, w=w: L.mic_mixed_streams(arr, 1, dst.data_ptr(), nbytes, 64, w, fl, sh))
    times = {k: [] for k in variants}
    for _ in range(a.rounds):
        for name, f in variants.items():
            assert f() == 0, name
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(a.launches):
                f()
            e1.record(stream)
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / a.launches)
    assert torch.equal(src, dst)
    for name, t in times.items():
        med = statistics.median(t)
        print(json.dumps({"variant": name, "bytes": nbytes, "median_ms": round(med, 5), "best_ms": round(min(t), 5),
                          "median_TBps": round(2 * nbytes / (med / 1e3) / 1e12, 3),
                          "frac_of_8TBps": round(2 * nbytes / (med / 1e3) / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()
