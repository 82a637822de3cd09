#!/usr/bin/env python3
"""Generate tests/golden/ref_vectors.npz: bit-level golden vectors produced by
the REFERENCE'S OWN bf16/fp16 reduce code (oracle/_ref/libref_comp.so, built
by `make -C oracle ref` from /root/reference/src/comp/{bf16,fp16}/*_intrisics.*;
see oracle/ref_harness.cpp).  Runs only where /root/reference is present (this
container); the committed .npz is what the CPU and GPU tests read.

Cases (all element-wise, inout updated in place, the reference's masked tails
included):
  bf16 2-input:  impl avx512f (truncation) and avx512bf (VCVTNEPS2BF16), ops
                 sum/prod/min/max, counts N (odd 16-tail), 16, 15, 1
                 (bf16_intrisics.hpp:78-114)
  fp16 2-input:  impl f16c (8-wide, memcpy tail) and avx512f (16-wide, masked
                 tail), same ops and counts (fp16_intrisics.hpp:95-148,179-196)
  chained fan-in: 8 inputs folded by 7 calls (the reference's chained
                 ccl_comp_reduce, comp.cpp:236-245) per impl for sum and max
  conversions:   16-element fp32 -> bf16 stores of both AVX-512 impls and the
                 bf16 -> fp32 load (bf16_intrisics.hpp:62-76)
Inputs: the cross product of 16 special values per type (±0, ±1, ±inf, quiet
and signalling NaNs of both signs, denormals, smallest normal, largest finite,
1+ulp), then seeded random bit patterns, wide-exponent values and values near 1
(rounding ties of the sum).
"""
from __future__ import annotations

import ctypes
import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
OUT = HERE / "ref_vectors.npz"
REF_SO = ROOT / "oracle" / "_ref" / "libref_comp.so"

N = 2061  # 128 full 16-wide vectors + a 13-element masked tail (f16c: 257 x 8 + 5)
COUNTS = [N, 16, 15, 1]
OPS = {0: "sum", 1: "prod", 2: "min", 3: "max"}
BF16_IMPLS = {1: "avx512f", 2: "avx512bf"}  # ccl_bf16_impl_type
FP16_IMPLS = {2: "f16c", 3: "avx512f"}  # ccl_fp16_impl_type
K_FAN = 8

BF16_SPECIALS = [0x0000, 0x8000, 0x3F80, 0xBF80, 0x7F80, 0xFF80, 0x7FC0, 0x7F81,
                 0xFFC1, 0x0001, 0x8001, 0x007F, 0x0080, 0x7F7F, 0xFF7F, 0x3F81]
FP16_SPECIALS = [0x0000, 0x8000, 0x3C00, 0xBC00, 0x7C00, 0xFC00, 0x7E00, 0x7C01,
                 0xFE01, 0x0001, 0x8001, 0x03FF, 0x0400, 0x7BFF, 0xFBFF, 0x3C01]


def _inputs(specials: list[int], fp16: bool, seed: int, n: int = N) -> tuple[np.ndarray, np.ndarray]:
    """(in, inout): special cross product first, then three random thirds."""
    rng = np.random.default_rng(seed)
    s = np.array(specials, np.uint16)
    a = np.repeat(s, len(s))
    b = np.tile(s, len(s))
    rest = n - a.size

    def rand_part(m):
        third = m // 3
        bits = rng.integers(0, 1 << 16, third, dtype=np.uint32).astype(np.uint16)
        if fp16:
            wide = (rng.standard_normal(third) * 2.0 ** rng.integers(-24, 16, third)).clip(-65504, 65504)
            wide = wide.astype(np.float16).view(np.uint16)
            near = (1.0 + rng.integers(0, 2048, m - 2 * third) * 2.0 ** -11).astype(np.float16).view(np.uint16)
        else:
            f = (rng.standard_normal(third) * 2.0 ** rng.integers(-130, 127, third)).astype(np.float32)
            wide = (f.view(np.uint32) >> 16).astype(np.uint16)
            near = ((np.float32(1.0) + rng.integers(0, 256, m - 2 * third).astype(np.float32) * np.float32(2.0 ** -8))
                    .astype(np.float32).view(np.uint32) >> 16).astype(np.uint16)
        p = np.concatenate([bits, wide, near])
        rng.shuffle(p)
        return p

    return np.concatenate([a, rand_part(rest)]), np.concatenate([b, rand_part(rest)])


def _conv_inputs(seed: int) -> np.ndarray:
    """fp32 values for the 16-element stores: rounding ties and near-ties in
    both parities, denormals, NaN payloads, infinities, then random bits."""
    rng = np.random.default_rng(seed)
    hand = []
    for hi in (0x3F80, 0x3F81, 0xBF80, 0x7F7F, 0x0080, 0x0000, 0x8000, 0x7F80, 0x0001):
        for lo in (0x0000, 0x0001, 0x7FFF, 0x8000, 0x8001, 0xFFFF, 0x4000, 0xC000):
            hand.append((hi << 16) | lo)
    hand += [0x7FC00000, 0xFFC00000, 0x7F800001, 0xFF800001, 0x7FBFFFFF, 0x7FFFFFFF, 0x007FFFFF, 0x807FFFFF,
             0x00000001, 0x80000001, 0x00400000, 0x7F7FFFFF, 0xFF7FFFFF, 0x7F7F8000, 0x7F7F7FFF]
    hand = np.array(hand, np.uint32)
    rnd = rng.integers(0, 1 << 32, 4096 - hand.size, dtype=np.uint64).astype(np.uint32)
    return np.concatenate([hand, rnd]).view(np.float32)


def _lib():
    L = ctypes.CDLL(str(REF_SO))
    for f in ("ref_bf16_reduce", "ref_fp16_reduce"):
        getattr(L, f).argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        getattr(L, f).restype = ctypes.c_int
    L.ref_fp32_to_bf16.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    L.ref_bf16_to_fp32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    return L


def generate() -> dict[str, np.ndarray]:
    L = _lib()
    arrs: dict[str, np.ndarray] = {}
    cases = []
    for kind, impls, specials, fn in (("bf16", BF16_IMPLS, BF16_SPECIALS, L.ref_bf16_reduce),
                                      ("fp16", FP16_IMPLS, FP16_SPECIALS, L.ref_fp16_reduce)):
        a, b = _inputs(specials, kind == "fp16", seed=0xB16 if kind == "bf16" else 0xF16)
        arrs[f"{kind}_in"], arrs[f"{kind}_inout"] = a, b
        for impl, iname in impls.items():
            for op, oname in OPS.items():
                for count in COUNTS:
                    out = b.copy()
                    assert fn(impl, op, a.ctypes.data, out.ctypes.data, count) == 0
                    key = f"{kind}_{iname}_{oname}_n{count}"
                    arrs[key] = out
                    cases.append({"key": key, "kind": kind, "impl": impl, "op": op, "count": count})
        fan = np.stack([_inputs(specials, kind == "fp16", seed=0xFA0 + j + (0 if kind == "bf16" else 100))[0]
                        for j in range(K_FAN)])
        arrs[f"fan_{kind}"] = fan
        for impl, iname in impls.items():
            for op in (0, 3):
                acc = fan[0].copy()
                for j in range(1, K_FAN):
                    assert fn(impl, op, fan[j].ctypes.data, acc.ctypes.data, N) == 0
                key = f"fan_{kind}_{iname}_{OPS[op]}"
                arrs[key] = acc
                cases.append({"key": key, "kind": f"fan_{kind}", "impl": impl, "op": op, "count": N, "k": K_FAN})
    f = _conv_inputs(0xC0)
    arrs["cvt_f32"] = f
    for impl, iname in BF16_IMPLS.items():
        o = np.empty(f.size, np.uint16)
        assert L.ref_fp32_to_bf16(impl, f.ctypes.data, o.ctypes.data, f.size) == 0
        arrs[f"cvt_bf16_{iname}"] = o
        cases.append({"key": f"cvt_bf16_{iname}", "kind": "cvt", "impl": impl, "count": int(f.size)})
    src = np.random.default_rng(0x10AD).integers(0, 1 << 16, 1024, dtype=np.uint32).astype(np.uint16)
    src[:len(BF16_SPECIALS)] = BF16_SPECIALS
    dst = np.empty(src.size, np.float32)
    assert L.ref_bf16_to_fp32(src.ctypes.data, dst.ctypes.data, src.size) == 0
    arrs["load_bf16"], arrs["load_f32"] = src, dst
    cases.append({"key": "load_f32", "kind": "load", "count": int(src.size)})
    meta = {"generator": "tests/golden/make_ref_vectors.py",
            "producer": "oracle/_ref/libref_comp.so = oracle/ref_harness.cpp + reference "
                        "src/comp/bf16/bf16_intrisics.{hpp,cpp}, src/comp/fp16/fp16_intrisics.{hpp,cpp}",
            "n": N, "k_fan": K_FAN, "cases": cases}
    arrs["meta"] = np.array(json.dumps(meta))
    return arrs


def main() -> int:
    if not REF_SO.exists():
        print(f"{REF_SO} missing: run `make -C oracle ref` (needs /root/reference)", file=sys.stderr)
        return 1
    arrs = generate()
    np.savez_compressed(OUT, **arrs)
    print(f"wrote {len(json.loads(str(arrs['meta']))['cases'])} cases to {OUT} ({OUT.stat().st_size} bytes)")
    return 0


if __name__ == "__main__":
    sys.exit(main())
