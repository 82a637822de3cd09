#!/usr/bin/env python3
"""TEST INFRASTRUCTURE ONLY.  The reference's own avx512fp16 fp16 reduce
(oracle/_ref/libref_fp16native.so, `make -C oracle ref`) against the oracle's
avx512fp16 model on every (in, inout) pair of fp16 bit patterns, each op:
65536 calls of 65536 elements per op (in fixed, inout all patterns).  Needs a
CPU with AVX512_FP16.  Writes oracle/FP16_NATIVE_REF_CHECK.json.

  python oracle/fp16_native_ref_check.py [--stride S]   (S > 1: every S-th `in` only)
"""
from __future__ import annotations

import argparse
import ctypes
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    import oracle
    ap = argparse.ArgumentParser()
    ap.add_argument("--stride", type=int, default=1)
    ap.add_argument("--out", default=str(ROOT / "oracle" / "FP16_NATIVE_REF_CHECK.json"))
    args = ap.parse_args()
    ref = ctypes.CDLL(str(ROOT / "oracle" / "_ref" / "libref_fp16native.so"))
    ref.ref_fp16native_reduce.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    if not ref.ref_fp16native_supported():
        print(json.dumps({"skipped": True, "reason": "no AVX512_FP16"}))
        return 2
    allv = np.arange(65536, dtype=np.uint16)
    names = {0: "sum", 1: "prod", 2: "min", 3: "max"}
    bad = {}
    t0 = time.time()
    for op, name in names.items():
        bad[name] = 0
        for a in range(0, 65536, args.stride):
            inn = np.full(65536, a, np.uint16)
            r = allv.copy()
            assert ref.ref_fp16native_reduce(inn.ctypes.data, r.ctypes.data, 65536, op) == 0
            o = allv.copy()
            oracle.comp_reduce(inn, o, 8, op, oracle.BF16_AVX512BF, oracle.FP16_AVX512FP16)
            bad[name] += int(np.count_nonzero(r != o))
    cpu = next((l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")), "?")
    res = {"pairs_per_op": (65536 // args.stride + (65536 % args.stride > 0)) * 65536, "stride": args.stride,
           "mismatches": bad, "seconds": round(time.time() - t0, 1), "cpu": cpu,
           "producer": "oracle/_ref/libref_fp16native.so (reference src/comp/fp16/fp16_intrisics.{hpp,cpp}, "
                       "CCL_FP16_AVX512FP16_COMPILER, clang++)",
           "model": "oracle/comp_oracle.c orc_comp_reduce, fp16 impl avx512fp16"}
    if args.stride == 1:
        Path(args.out).write_text(json.dumps(res, indent=1) + "\n")
    print(json.dumps(res))
    return 0 if not any(bad.values()) else 1


if __name__ == "__main__":
    sys.exit(main())
