#!/usr/bin/env python3
"""Generate tests/golden/ref_vectors_fp16native.npz: golden vectors produced by
the REFERENCE'S OWN avx512fp16 fp16 reduce (native half-precision math,
src/comp/fp16/fp16_intrisics.cpp:23-41, fp16_intrisics.hpp:150-176) through
oracle/_ref/libref_fp16native.so (`make -C oracle ref`: ROCm's clang++ over the
reference sources where they lie, see oracle/ref_fp16native.cpp).  Needs
/root/reference and a CPU with AVX512_FP16 (this container); the committed
.npz is what the CPU and GPU tests read.

Cases: 2-input, ops sum/prod/min/max, counts N (a 13-element masked tail of
the 32-wide body), 32, 31, 1; chained 8-input fan-ins (7 calls) for sum and
max.  Inputs: make_ref_vectors.py's fp16 generator (16 x 16 special values —
signalling and quiet NaNs of both signs among them — then random bits, wide
exponents and near-ties), so the signalling-NaN `inout` rows that separate
this impl from f16c / avx512f are present.
"""
from __future__ import annotations

import ctypes
import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path.insert(0, str(HERE))
from make_ref_vectors import FP16_SPECIALS, K_FAN, N, OPS, _inputs  # noqa: E402

OUT = HERE / "ref_vectors_fp16native.npz"
REF_SO = ROOT / "oracle" / "_ref" / "libref_fp16native.so"
COUNTS = [N, 32, 31, 1]


def _lib():
    L = ctypes.CDLL(str(REF_SO))
    L.ref_fp16native_reduce.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    L.ref_fp16native_reduce.restype = ctypes.c_int
    L.ref_fp16native_supported.restype = ctypes.c_int
    return L


def generate() -> dict[str, np.ndarray]:
    L = _lib()
    if not L.ref_fp16native_supported():
        raise SystemExit("this CPU lacks AVX512_FP16: the reference's avx512fp16 code cannot run")
    arrs: dict[str, np.ndarray] = {}
    cases = []
    a, b = _inputs(FP16_SPECIALS, True, seed=0xF16)
    arrs["fp16_in"], arrs["fp16_inout"] = a, b
    for op, oname in OPS.items():
        for count in COUNTS:
            out = b.copy()
            assert L.ref_fp16native_reduce(a.ctypes.data, out.ctypes.data, count, op) == 0
            key = f"fp16_avx512fp16_{oname}_n{count}"
            arrs[key] = out
            cases.append({"key": key, "kind": "fp16", "impl": 4, "op": op, "count": count})
    fan = np.stack([_inputs(FP16_SPECIALS, True, seed=0xFA0 + j + 100)[0] for j in range(K_FAN)])
    arrs["fan_fp16"] = fan
    for op in (0, 3):
        acc = fan[0].copy()
        for j in range(1, K_FAN):
            assert L.ref_fp16native_reduce(fan[j].ctypes.data, acc.ctypes.data, N, op) == 0
        key = f"fan_fp16_avx512fp16_{OPS[op]}"
        arrs[key] = acc
        cases.append({"key": key, "kind": "fan_fp16", "impl": 4, "op": op, "count": N, "k": K_FAN})
    meta = {"generator": "tests/golden/make_ref_vectors_fp16native.py",
            "producer": "oracle/_ref/libref_fp16native.so = oracle/ref_fp16native.cpp + reference "
                        "src/comp/fp16/fp16_intrisics.{hpp,cpp} with CCL_FP16_AVX512FP16_COMPILER (clang++)",
            "n": N, "k_fan": K_FAN, "cases": cases}
    arrs["meta"] = np.array(json.dumps(meta))
    return arrs


if __name__ == "__main__":
    arrs = generate()
    np.savez_compressed(OUT, **arrs)
    print(f"wrote {OUT} ({len(json.loads(str(arrs['meta']))['cases'])} cases)")
