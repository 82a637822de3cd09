#!/usr/bin/env python3
"""Crossover of the drop-in's dispatcher: for a
host-resident bucket, the calling thread's CPU (host_reduce.cpp) against the
GPU (staging / zero-copy), both through ccl_comp_reduce itself, next to the
CPU oracle on one thread (the reference's one-worker rate).  Sizes 4 KiB ..
--max-mib, powers of 2; pageable (posix_memalign-like numpy) and pinned
buffers.  One JSON line per (dtype, kind, size): best-of-reps microseconds.

  python tools/dispatch_sweep.py [--max-mib 512] [--dtypes f32,bf16]
  python tools/dispatch_sweep.py --recommend [--min-kib 4 --max-mib 1024]
  python tools/dispatch_sweep.py --adapt-trace [--max-mib 256]

--adapt-trace follows the adaptive split (no CCL_COMP_HOST_SHARE* set): for
one bucket of --max-mib per pointer kind, 12 consecutive ccl_comp_reduce
calls on one thread, each line the share it ran with, the share it left and
its GiB/s.

--recommend ends with the dispatcher settings these measurements imply for
this host (one JSON line, and `export` lines on stderr): per pointer kind,
the largest bucket up to which the calling thread's CPU beats the GPU, and
the CPU share of the cooperative split that moved the most bytes above it.
The defaults in oneccl_amd/csrc/comp.cpp came from this sweep on the MI355X
box's EPYC 9575F; another host can run it once and export the result.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

DT = {"f32": (9, 4), "bf16": (11, 2)}
KNOBS = ("CCL_COMP_HOST_MAX_BYTES", "CCL_COMP_HOST_MAX_PINNED_BYTES", "CCL_COMP_HOST_SHARE",
         "CCL_COMP_HOST_SHARE_PINNED")


def best_us(fn, reps):
    fn()
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        t.append(time.perf_counter() - t0)
    return round(min(t) * 1e6, 2), round(sorted(t)[len(t) // 2] * 1e6, 2)


def recommend(rows):
    """Dispatcher settings from sweep rows (dicts as printed by main()):
    {kind: {"host_max_bytes": B, "share": S}} for each pointer kind seen."""
    out = {}
    for kind in sorted({r["kind"] for r in rows}):
        rs = sorted((r for r in rows if r["kind"] == kind), key=lambda r: r["bytes"])
        host_max = 0
        for r in rs:  # the CPU path must beat the GPU alone and every split at every size up to it
            alt = min([r["gpu_us"]] + [v for k, v in r.items() if k.startswith("coop") and k.endswith("_us")
                                       and not k.endswith("median_us")])
            if r["cpu_us"] <= alt:
                host_max = r["bytes"]
            else:
                break
        shares = sorted({float(k[4:-6]) for r in rs for k in r if k.startswith("coop") and k.endswith("_GiBps")})
        best, best_rate = None, 0.0
        for sh in shares:
            rates = [r[f"coop{sh:g}_GiBps"] for r in rs if f"coop{sh:g}_GiBps" in r and r["bytes"] > host_max]
            if rates and sum(rates) / len(rates) > best_rate:
                best, best_rate = sh, sum(rates) / len(rates)
        out[kind] = {"host_max_bytes": host_max, "share": best, "split_mean_GiBps": round(best_rate, 2)}
    return out


def adapt_trace(args):
    import numpy as np
    import torch

    from oneccl_amd import _lib, comp
    shim = _lib.shim()
    for kk in KNOBS:
        os.environ.pop(kk, None)
    nbytes = args.max_mib << 20
    for dname in args.dtypes.split(","):
        dt, es = DT[dname]
        n = nbytes // es
        for kind in args.kinds.split(","):
            comp.env_reload()
            if kind == "pinned":
                ta = torch.full((nbytes,), 0x3F, dtype=torch.uint8).pin_memory()
                tb = torch.full((nbytes,), 0x3F, dtype=torch.uint8).pin_memory()
                pa, pb = ta.data_ptr(), tb.data_ptr()
            else:
                a = np.full(nbytes, 0x3F, np.uint8)
                b = np.full(nbytes, 0x3F, np.uint8)
                pa, pb = a.ctypes.data, b.ctypes.data
            for i in range(12):
                before = shim.mi_ccl_comp_split_share(1 if kind == "pinned" else 0)
                t0 = time.perf_counter()
                comp.comp_reduce(pa, n, pb, comp.datatype(dt), comp.reduction.sum)
                dt_s = time.perf_counter() - t0
                print(json.dumps({"dtype": dname, "kind": kind, "bytes": nbytes, "call": i,
                                  "share_in": round(before, 4),
                                  "share_out": round(shim.mi_ccl_comp_split_share(1 if kind == "pinned" else 0), 4),
                                  "GiBps": round(nbytes / dt_s / 2**30, 2)}), flush=True)
                if kind != "pinned":
                    b[:] = 0x3F  # keep the values away from overflow and denormals
                else:
                    tb.fill_(0x3F)
            # the same buffers at fixed shares: where the adapted share should have landed
            env = "CCL_COMP_HOST_SHARE_PINNED" if kind == "pinned" else "CCL_COMP_HOST_SHARE"
            fixed = {}
            for sh in args.shares.split(","):
                os.environ[env] = sh
                comp.env_reload()
                best = float("inf")
                for i in range(4):
                    t0 = time.perf_counter()
                    comp.comp_reduce(pa, n, pb, comp.datatype(dt), comp.reduction.sum)
                    if i:
                        best = min(best, time.perf_counter() - t0)
                    if kind != "pinned":
                        b[:] = 0x3F
                    else:
                        tb.fill_(0x3F)
                fixed[sh] = round(nbytes / best / 2**30, 2)
            os.environ.pop(env, None)
            comp.env_reload()
            print(json.dumps({"dtype": dname, "kind": kind, "bytes": nbytes, "fixed_share_GiBps": fixed}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--max-mib", type=int, default=512)
    ap.add_argument("--dtypes", default="f32,bf16")
    ap.add_argument("--kinds", default="pageable,pinned")
    ap.add_argument("--shares", default="0.3,0.45,0.6")
    ap.add_argument("--min-kib", type=int, default=4)
    ap.add_argument("--recommend", action="store_true", help="end with the dispatcher settings for this host")
    ap.add_argument("--adapt-trace", action="store_true", help="follow the adaptive split over 12 calls")
    args = ap.parse_args()
    if args.adapt_trace:
        return adapt_trace(args)
    rows = []
    import numpy as np
    import torch

    import oracle
    from oneccl_amd import comp
    sizes = []
    s = args.min_kib << 10
    while s <= args.max_mib << 20:
        sizes.append(s)
        s *= 2
    for dname in args.dtypes.split(","):
        dt, es = DT[dname]
        for kind in args.kinds.split(","):
            for nbytes in sizes:
                n = nbytes // es
                reps = 20 if nbytes <= (4 << 20) else (6 if nbytes <= (64 << 20) else 3)
                if kind == "pinned":
                    ta = torch.ones(nbytes, dtype=torch.uint8).pin_memory()
                    tb = torch.ones(nbytes, dtype=torch.uint8).pin_memory()
                    pa, pb = ta.data_ptr(), tb.data_ptr()
                    a = ta.numpy().view(oracle.NP_DTYPE[dt])
                    b = tb.numpy().view(oracle.NP_DTYPE[dt])
                else:
                    a = np.ones(n, oracle.NP_DTYPE[dt])
                    b = np.ones(n, oracle.NP_DTYPE[dt])
                    pa, pb = a.ctypes.data, b.ctypes.data
                row = {"dtype": dname, "kind": kind, "bytes": nbytes}
                modes = [("cpu", {"CCL_COMP_HOST_MAX_BYTES": str(1 << 40),
                                  "CCL_COMP_HOST_MAX_PINNED_BYTES": str(1 << 40)}),
                         ("gpu", {"CCL_COMP_HOST_MAX_BYTES": "0"}),
                         ("default", {})]
                if nbytes >= (32 << 20):  # the cooperative split (CPU head + GPU tail) at several shares
                    for sh in args.shares.split(","):
                        modes.append((f"coop{sh}", {"CCL_COMP_HOST_MAX_BYTES": str(1 << 20),
                                                    "CCL_COMP_HOST_MAX_PINNED_BYTES": str(1 << 20),
                                                    "CCL_COMP_HOST_SHARE": sh, "CCL_COMP_HOST_SHARE_PINNED": sh}))
                for mode, envs in modes:
                    for kk in KNOBS:
                        os.environ.pop(kk, None)
                    os.environ.update(envs)
                    comp.env_reload()
                    row[f"{mode}_us"], row[f"{mode}_median_us"] = best_us(
                        lambda: comp.comp_reduce(pa, n, pb, comp.datatype(dt), comp.reduction.sum), reps)
                row["oracle_1t_us"], _ = best_us(lambda: oracle.comp_reduce(a, b, dt, 0), reps)
                for mode, _ in modes:
                    row[f"{mode}_GiBps"] = round(nbytes / (row[f"{mode}_us"] * 1e-6) / 2**30, 2)
                rows.append(row)
                print(json.dumps(row), flush=True)
    for kk in KNOBS:
        os.environ.pop(kk, None)
    if args.recommend:
        rec = recommend([r for r in rows if r["dtype"] == args.dtypes.split(",")[0]])
        print(json.dumps({"recommend": rec}), flush=True)
        env = {"pageable": ("CCL_COMP_HOST_MAX_BYTES", "CCL_COMP_HOST_SHARE"),
               "pinned": ("CCL_COMP_HOST_MAX_PINNED_BYTES", "CCL_COMP_HOST_SHARE_PINNED")}
        for kind, r in rec.items():
            print(f"export {env[kind][0]}={r['host_max_bytes']}", file=sys.stderr)
            if r["share"] is not None:
                print(f"export {env[kind][1]}={r['share']:g}", file=sys.stderr)


if __name__ == "__main__":
    main()
