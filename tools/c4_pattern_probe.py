#!/usr/bin/env python3
"""Access patterns other than the fan-in's own, for the same traffic
(VERDICT r5 item 3).  On one set of buffers, in one process, interleaved
over rounds:

  kernel       the library's fan_kernel through mi_reduce_multi (the real reduce)
  mixed        tools/ceiling_probe.hip mic_mixed_streams: the kernel's own
               pattern (each lane loads its vector of all K inputs and stores
               one), no arithmetic, at the library's block and residency cap
  burst-lds    mic_burst_streams: each workgroup reads a run of T tiles of all
               K inputs, parks the outputs in LDS, then writes the T tiles back
               to back (write bursts of T x block x 16 bytes)
  burst-reg    the same with the outputs parked in registers (T <= 4), at a
               few one-wave residency caps

Prints one JSON line per (layout, variant): best and median time per launch
and the rate of (K + 1) x bytes.  Measurement infrastructure, not product.

  python tools/c4_pattern_probe.py [--k 8] [--gib 1] [--rounds 3] [--launches 10]
"""
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
    p = argparse.ArgumentParser()
    p.add_argument("--k", type=int, default=8)
    p.add_argument("--gib", type=float, default=1.0)
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--launches", type=int, default=10)
    p.add_argument("--layouts", default="one,tmpbuf")
    args = p.parse_args()
    import torch

    import bench
    from oneccl_amd import _lib
    m = _lib.mi()
    L = ctypes.CDLL(str(ROOT / bench.CEILING_LIB))
    L.mic_mixed_streams.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                    ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    L.mic_burst_streams.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                    ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_void_p]
    k = args.k
    n = int(args.gib * (1 << 30)) // 4
    nb = n * 4
    waves = ctypes.c_int(0)
    _lib.check(m.mi_get_residency(-1, k, ctypes.byref(waves), None), "mi_get_residency")
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream
    lib_flavor = 2 if k == 2 else 1  # the library's stores: sc1 nt (2-input), nt (fan-in)

    variants = [("kernel", None), ("mixed", (64, waves.value, lib_flavor))]
    for fl in (1, 2):
        for block in (64, 256, 1024):
            for t in (2, 4, 8, 16, 32):
                if t * block * 16 <= 160 * 1024:
                    variants.append((f"burst-lds b{block} t{t} f{fl}", ("lds", block, t, 0, fl)))
        for t in (1, 2, 4):
            for w in (0, waves.value, 16):
                variants.append((f"burst-reg b64 t{t} w{w} f{fl}", ("reg", 64, t, w, fl)))

    for layout in args.layouts.split(","):
        if layout == "tmpbuf":
            ins = bench.alloc_tmpbuf(k, n, torch.float32)
        else:
            ins = bench.alloc_inputs(k, n, torch.float32, layout)
        for j in range(k):
            bench.fill(ins[j], 0x51 + j)
        arr = _lib.void_ptr_array([t.data_ptr() for t in ins])
        out = ins[0].data_ptr()

        def launch(spec):
            if spec is None:
                return m.mi_reduce_multi(arr, k, out, n, 9, 0, 0, sh) if k > 2 else \
                    m.mi_reduce(ins[1].data_ptr(), out, n, 9, 0, 0, sh)
            if len(spec) == 3:
                b, w, fl = spec
                return L.mic_mixed_streams(arr, k, out, nb, b, w, fl, sh)
            mode, b, t, w, fl = spec
            return L.mic_burst_streams(arr, k, out, nb, b, t, 1 if mode == "lds" else 0, w, fl, sh)

        times = {name: [] for name, _ in variants}
        bad = set()
        for r in range(args.rounds):
            for name, spec in variants:
                if name in bad:
                    continue
                if launch(spec):
                    bad.add(name)
                    continue
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(args.launches):
                    launch(spec)
                e1.record(stream)
                torch.cuda.synchronize()
                times[name].append(e0.elapsed_time(e1) / args.launches)
            print(f"round {r} done", file=sys.stderr, flush=True)
        algo = (k + 1) * nb
        ref = min(times["mixed"]) if times["mixed"] else None
        for name, _ in variants:
            tt = times[name]
            if not tt:
                print(json.dumps({"layout": layout, "variant": name, "error": "launch refused"}), flush=True)
                continue
            rec = {"layout": layout, "k": k, "bytes_per_stream": nb, "variant": name,
                   "best_ms": round(min(tt), 5), "median_ms": round(statistics.median(tt), 5),
                   "TBps_best": round(algo / (min(tt) / 1e3) / 1e12, 3),
                   "frac_of_spec": round(algo / (min(tt) / 1e3) / 8e12, 4)}
            if ref:
                rec["vs_mixed"] = round(ref / min(tt), 4)
            print(json.dumps(rec), flush=True)
        del ins, arr
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
