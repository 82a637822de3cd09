#!/usr/bin/env python3
"""The dispatcher's CPU side against the reference's own compiled code, one
thread, on this host (run it on the GPU box: the deployment CPU).

For host buckets up to CCL_COMP_HOST_MAX_BYTES the drop-in reduces on the
calling thread (oneccl_amd/csrc/host_reduce.cpp).  This times that path,
entered through ccl_comp_reduce of the drop-in, beside the reference's own
compiled code on the same buffers and the same core:
  float32 / float64 / int32 sum : ccl_comp_reduce_regular (CCL_REDUCE,
                                  oracle/_ref/libref_ccl_comp.so)
  bf16 (avx512bf) / fp16 (avx512f) sum : the reference's AVX-512 bodies
                                  (oracle/_ref/libref_comp.so)
and checks that both give the same bits.  Measurement tool only.

  python tools/host_vs_ref.py [--kib 512,4096,16384] [--reps 50]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--kib", default="512,4096,16384")
    p.add_argument("--reps", type=int, default=50)
    a = p.parse_args()
    import numpy as np

    import oracle
    from oneccl_amd import _lib, comp
    os.environ.setdefault("CCL_FP16", "avx512f")  # libref_comp.so holds the f16c / avx512f bodies
    shim = _lib.shim()
    comp.env_reload()
    os.sched_setaffinity(0, {min(os.sched_getaffinity(0))})  # one core for both
    avx = ctypes.CDLL(str(ROOT / "oracle" / "_ref" / "libref_comp.so"))
    for f in ("ref_bf16_reduce", "ref_fp16_reduce"):
        getattr(avx, f).argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    b_impl, f_impl = comp.impl_types()
    rng = np.random.default_rng(1)
    for kib in (int(x) for x in a.kib.split(",")):
        nbytes = kib << 10
        for name, dt in (("float32", 9), ("float64", 10), ("int32", 4), ("bfloat16", 11), ("float16", 8)):
            es = 2 if dt in (8, 11) else (8 if dt == 10 else 4)
            n = nbytes // es
            if dt in (9, 10):
                x = rng.standard_normal(n).astype(np.float32 if dt == 9 else np.float64)
                y = rng.standard_normal(n).astype(x.dtype)
            elif dt == 4:
                x = rng.integers(-1000, 1000, n).astype(np.int32)
                y = rng.integers(-1000, 1000, n).astype(np.int32)
            else:
                f = rng.standard_normal(n).astype(np.float32)
                x = oracle.f32_to_bf16(f, True) if dt == 11 else oracle.f32_to_fp16(f)
                y = oracle.f32_to_bf16(f[::-1].copy(), True) if dt == 11 else oracle.f32_to_fp16(f[::-1].copy())

            def ours(bb):
                _lib.check_shim(shim.mi_ccl_comp_reduce(x.ctypes.data, n, bb.ctypes.data, None, dt, 0),
                                "ccl_comp_reduce")

            flags = comp.reference_flags(comp.datatype(dt), b_impl, f_impl)
            ins = _lib.void_ptr_array([0, x.ctypes.data])

            def host_only(bb):  # the same fold without the entry point's dispatch
                ins[0] = bb.ctypes.data
                assert shim.mi_host_reduce(ins, 2, bb.ctypes.data, n, dt, 0, flags) == 0

            def ref(bb):
                if dt == 11:
                    assert avx.ref_bf16_reduce(int(b_impl), 0, x.ctypes.data, bb.ctypes.data, n) == 0
                elif dt == 8:
                    assert avx.ref_fp16_reduce(int(f_impl), 0, x.ctypes.data, bb.ctypes.data, n) == 0
                else:
                    oracle.ref_comp_reduce(x, bb, dt, 0)

            bo, br = y.copy(), y.copy()
            ours(bo)
            ref(br)
            same = bool(np.array_equal(bo.view(np.uint8), br.view(np.uint8)))
            row = {"dtype": name, "bytes": nbytes, "same_bits": same, "impl": {"bf16": int(b_impl), "fp16": int(f_impl)}}
            for key, fn in (("dropin_GiBps", ours), ("host_fold_GiBps", host_only), ("reference_GiBps", ref)):
                bb = y.copy()
                ts = []
                for _ in range(a.reps):
                    t0 = time.perf_counter()
                    fn(bb)
                    ts.append(time.perf_counter() - t0)
                row[key] = round(nbytes / (1 << 30) / statistics.median(ts), 2)
            row["ratio"] = round(row["dropin_GiBps"] / row["reference_GiBps"], 3)
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
