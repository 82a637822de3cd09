#!/usr/bin/env python3
"""Generate tests/golden/ref_comp_vectors.npz: golden vectors produced by the
REFERENCE'S OWN compiled src/comp code (oracle/_ref/libref_ccl_comp.so, built
by `make -C oracle refcomp` from /root/reference/src/comp/comp.cpp, bf16.cpp,
... with the reference's Release flags; see oracle/ref_comp_harness.cpp).
Runs only where /root/reference is present (this container); the committed
.npz is what the CPU and GPU tests read.

Cases:
  reduce   ccl_comp_reduce_regular -> CCL_REDUCE (comp.cpp:31-58, 76-121) for
           the ten non-LP types int8..uint64, float32, float64 x sum/prod/min/
           max; whether *out_count was written is recorded too
  reduce1  the same for float32/float64 one element per call over the 256
           special pairs (the compiled loop's scalar path)
  bf16s    the scalar bf16 impl, ccl_bf16_reduce_scalar_impl (bf16.cpp:63-85:
           fp32 math, truncation to bf16, std::min/max operand order)
  batch    ccl_comp_batch_reduce, storage-precision chain (comp.cpp:236-245):
           5 inputs at unaligned offsets of one buffer, int32/int64/float32/
           float64 x four ops
  keep     ccl_comp_batch_reduce's keep-precision mode (comp.cpp:214-234) for
           the avx512f and avx512bf impls x four ops, composed from the
           reference's compiled parts (the function itself reads
           global_data::get()): its AVX-512 array-conversion bodies
           (oracle/_ref/libref_comp.so) and CCL_REDUCE(float)
Inputs: the cross product of 16 special values per type first (integers:
0, +-1, extremes, values whose sums and products wrap; floating point: +-0,
+-1, +-inf, quiet NaNs with payloads of both signs, a signalling NaN,
denormals, the largest finite, 1 + ulp), then seeded random values of three
kinds (any bits, wide exponents, near 1).
"""
from __future__ import annotations

import ctypes
import json
import os
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
OUT = HERE / "ref_comp_vectors.npz"
REF_SO = ROOT / "oracle" / "_ref" / "libref_ccl_comp.so"

N = 1031  # 256 special pairs + random; odd, so vector loops have a scalar tail
OPS = {0: "sum", 1: "prod", 2: "min", 3: "max"}
TYPES = {0: np.int8, 1: np.uint8, 2: np.int16, 3: np.uint16, 4: np.int32, 5: np.uint32, 6: np.int64,
         7: np.uint64, 9: np.float32, 10: np.float64}
BATCH_TYPES = (4, 6, 9, 10)
K_BATCH = 5
SENTINEL = 0xFFFFFFFFFFFFFFFF

F32_SPECIALS = [0x00000000, 0x80000000, 0x3F800000, 0xBF800000, 0x7F800000, 0xFF800000, 0x7FC00000, 0x7FC00123,
                0xFFC00456, 0x7F800001, 0x00000001, 0x807FFFFF, 0x00800000, 0x7F7FFFFF, 0xFF7FFFFF, 0x3F800001]
F64_SPECIALS = [0x0000000000000000, 0x8000000000000000, 0x3FF0000000000000, 0xBFF0000000000000,
                0x7FF0000000000000, 0xFFF0000000000000, 0x7FF8000000000000, 0x7FF8000000000123,
                0xFFF8000000000456, 0x7FF0000000000001, 0x0000000000000001, 0x800FFFFFFFFFFFFF,
                0x0010000000000000, 0x7FEFFFFFFFFFFFFF, 0xFFEFFFFFFFFFFFFF, 0x3FF0000000000001]
BF16_SPECIALS = [0x0000, 0x8000, 0x3F80, 0xBF80, 0x7F80, 0xFF80, 0x7FC0, 0x7F81,
                 0xFFC1, 0x0001, 0x8001, 0x007F, 0x0080, 0x7F7F, 0xFF7F, 0x3F81]


def _int_specials(t) -> list[int]:
    info = np.iinfo(t)
    v = [0, 1, info.max, info.min, info.max - 1, info.min + 1, 2, 3, info.max // 2, info.max // 2 + 1, 100, 127,
         255 % (info.max + 1), 1 << (info.bits // 2), (1 << (info.bits // 2)) + 1, info.max // 3]
    if info.min < 0:
        v[7], v[10] = -1, -100
    return v


def _specials(dt: int) -> np.ndarray:
    t = TYPES.get(dt)
    if dt == 9:
        return np.array(F32_SPECIALS, np.uint32).view(np.float32)
    if dt == 10:
        return np.array(F64_SPECIALS, np.uint64).view(np.float64)
    if dt == 11:
        return np.array(BF16_SPECIALS, np.uint16)
    bits = np.iinfo(t).bits
    return np.array([x % (1 << bits) for x in _int_specials(t)], dtype=np.uint64).astype(
        {8: np.uint8, 16: np.uint16, 32: np.uint32, 64: np.uint64}[bits]).view(t)


def _random(dt: int, m: int, rng) -> np.ndarray:
    third = m // 3
    if dt == 11:
        bits = rng.integers(0, 1 << 16, third, dtype=np.uint32).astype(np.uint16)
        f = (rng.standard_normal(third) * 2.0 ** rng.integers(-130, 127, third)).astype(np.float32)
        wide = (f.view(np.uint32) >> 16).astype(np.uint16)
        near = ((np.float32(1.0) + rng.integers(0, 256, m - 2 * third).astype(np.float32) * np.float32(2.0 ** -8))
                .astype(np.float32).view(np.uint32) >> 16).astype(np.uint16)
        p = np.concatenate([bits, wide, near])
    elif dt in (9, 10):
        ft, it, eb = (np.float32, np.uint32, 126) if dt == 9 else (np.float64, np.uint64, 1020)
        bits = rng.integers(0, np.iinfo(it).max, third, dtype=it, endpoint=True).view(ft)
        wide = (rng.standard_normal(third) * 2.0 ** rng.integers(-eb, eb, third)).astype(ft)
        near = (1.0 + rng.integers(0, 1 << 12, m - 2 * third) * 2.0 ** -23).astype(ft)
        p = np.concatenate([bits, wide, near])
    else:
        t = TYPES[dt]
        info = np.iinfo(t)
        bits = rng.integers(info.min, info.max, third, dtype=t, endpoint=True)
        small = rng.integers(-3 if info.min < 0 else 0, 4, third).astype(t)
        mid = rng.integers(max(info.min, -1000), min(info.max, 1000), m - 2 * third, endpoint=True).astype(t)
        p = np.concatenate([bits, small, mid])
    rng.shuffle(p)
    return p


def _pair(dt: int, seed: int, n: int = N) -> tuple[np.ndarray, np.ndarray]:
    rng = np.random.default_rng(seed)
    s = _specials(dt)
    a, b = np.repeat(s, s.size), np.tile(s, s.size)
    rest = n - a.size
    return np.concatenate([a, _random(dt, rest, rng)]), np.concatenate([b, _random(dt, rest, rng)])


def _lib():
    L = ctypes.CDLL(str(REF_SO), mode=os.RTLD_LAZY)  # global_data::get/env stay unbound (never called)
    L.ref_ccl_comp_reduce_regular.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_int, ctypes.c_size_t, ctypes.c_int]
    L.ref_ccl_bf16_reduce_scalar.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    L.ref_ccl_comp_batch_reduce.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t,
                                            ctypes.c_int]
    L.ref_ccl_comp_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    return L


REF_AVX_SO = ROOT / "oracle" / "_ref" / "libref_comp.so"


def _lib_avx():
    A = ctypes.CDLL(str(REF_AVX_SO))
    A.ref_fp32_to_bf16.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    A.ref_bf16_to_fp32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    return A


def _bf16_to_f32_arrays(A, src: np.ndarray) -> np.ndarray:
    """ccl_convert_bf16_to_fp32_arrays for a non-scalar impl (bf16.cpp:152-169):
    16-element loads, the reference's own body, then the scalar tail (<< 16)."""
    src = np.ascontiguousarray(src)
    out = np.empty(src.size, np.float32)
    lim = src.size // 16 * 16
    if lim:
        assert A.ref_bf16_to_fp32(src.ctypes.data, out.ctypes.data, lim) == 0
    out.view(np.uint32)[lim:] = src[lim:].astype(np.uint32) << 16
    return out


def _f32_to_bf16_arrays(A, src: np.ndarray, impl: int) -> np.ndarray:
    """ccl_convert_fp32_to_bf16_arrays for a non-scalar impl (bf16.cpp:130-150):
    16-element stores of the impl (avx512f truncation, avx512bf
    VCVTNEPS2BF16), the reference's own bodies, then the scalar tail
    (truncation)."""
    out = np.empty(src.size, np.uint16)
    lim = src.size // 16 * 16
    if lim:
        assert A.ref_fp32_to_bf16(impl, src.ctypes.data, out.ctypes.data, lim) == 0
    out[lim:] = (src[lim:].view(np.uint32) >> 16).astype(np.uint16)
    return out


def batch_offsets(n: int) -> list[int]:
    """Element offsets of the K inputs in one buffer: gaps that leave every
    input at a different alignment (offsets[0] names inout, never read)."""
    return [0, n + 1, 2 * n + 7, 3 * n + 10, 4 * n + 29]


def generate() -> dict[str, np.ndarray]:
    L = _lib()
    arrs: dict[str, np.ndarray] = {}
    cases = []
    for dt, t in TYPES.items():
        a, b = _pair(dt, seed=0xC0 + dt)
        arrs[f"reduce_{dt}_in"], arrs[f"reduce_{dt}_inout"] = a, b
        for op, oname in OPS.items():
            out = b.copy()
            oc = ctypes.c_size_t(SENTINEL)
            assert L.ref_ccl_comp_reduce_regular(a.ctypes.data, a.size, out.ctypes.data, ctypes.byref(oc), dt,
                                                 a.itemsize, op) == 0
            key = f"reduce_{dt}_{oname}"
            arrs[key] = out
            cases.append({"key": key, "kind": "reduce", "dtype": dt, "op": op, "count": int(a.size),
                          "out_count_written": oc.value != SENTINEL})
    # one element per call over the floating-point special pairs: the
    # compiled loop's scalar path (the vector body above may order operands
    # differently; here it does not)
    for dt in (9, 10):
        s = _specials(dt)
        a, b = np.repeat(s, s.size), np.tile(s, s.size)
        arrs[f"reduce1_{dt}_in"], arrs[f"reduce1_{dt}_inout"] = a, b
        for op, oname in OPS.items():
            out = b.copy()
            for i in range(a.size):
                assert L.ref_ccl_comp_reduce_regular(a[i:].ctypes.data, 1, out[i:].ctypes.data, None, dt, a.itemsize,
                                                     op) == 0
            key = f"reduce1_{dt}_{oname}"
            arrs[key] = out
            cases.append({"key": key, "kind": "reduce1", "dtype": dt, "op": op, "count": 1, "calls": int(a.size)})
    a, b = _pair(11, seed=0xB5)
    arrs["bf16s_in"], arrs["bf16s_inout"] = a, b
    for op, oname in OPS.items():
        out = b.copy()
        assert L.ref_ccl_bf16_reduce_scalar(a.ctypes.data, out.ctypes.data, a.size, op) == 0
        arrs[f"bf16s_{oname}"] = out
        cases.append({"key": f"bf16s_{oname}", "kind": "bf16s", "dtype": 11, "op": op, "count": int(a.size)})
    offs = batch_offsets(N)
    for dt in BATCH_TYPES:
        # the inputs are slices of one tmp buffer, as nreduce's
        buf = np.concatenate([_pair(dt, seed=0xBB + 16 * dt + j)[0] for j in range(K_BATCH + 1)])
        buf = buf[:offs[-1] + N].copy()
        inout = _pair(dt, seed=0xBC + dt)[1]
        arrs[f"batch_{dt}_buf"], arrs[f"batch_{dt}_inout"] = buf, inout
        o = (ctypes.c_size_t * len(offs))(*offs)
        for op, oname in OPS.items():
            out = inout.copy()
            oc = ctypes.c_size_t(SENTINEL)
            assert L.ref_ccl_comp_batch_reduce(buf.ctypes.data, o, len(offs), N, out.ctypes.data, ctypes.byref(oc),
                                               dt, buf.itemsize, op) == 0
            key = f"batch_{dt}_{oname}"
            arrs[key] = out
            cases.append({"key": key, "kind": "batch", "dtype": dt, "op": op, "count": N, "offsets": offs,
                          "out_count_written": oc.value != SENTINEL})
    # keep-precision batch reduce (comp.cpp:214-234), composed from the
    # reference's own compiled parts: its array conversions' 16-element
    # AVX-512 bodies (libref_comp.so, bf16_intrisics.hpp:62-76) with the
    # arrays' scalar tails (bf16.cpp:130-169), and CCL_REDUCE(float) on the fp32
    # scratch (libref_ccl_comp.so).  The whole function calls
    # global_data::get() for its float32 datatype, so it is not called itself.
    A = _lib_avx()
    for impl, iname in ((1, "avx512f"), (2, "avx512bf")):
        rng = np.random.default_rng(0x4B + impl)
        buf = np.concatenate([_pair(11, seed=0x4C + 16 * impl + j)[0] for j in range(K_BATCH + 1)])
        buf = buf[:offs[-1] + N].copy()
        inout = _pair(11, seed=0x4D + impl)[1]
        arrs[f"kp_{impl}_buf"], arrs[f"kp_{impl}_inout"] = buf, inout
        for op, oname in OPS.items():
            acc = _bf16_to_f32_arrays(A, inout)
            for o in offs[1:]:
                tmp = _bf16_to_f32_arrays(A, buf[o:o + N])
                assert L.ref_ccl_comp_reduce_regular(tmp.ctypes.data, N, acc.ctypes.data, None, 9, 4, op) == 0
            out = _f32_to_bf16_arrays(A, acc, impl)
            key = f"kp_{impl}_{oname}"
            arrs[key] = out
            cases.append({"key": key, "kind": "keep", "dtype": 11, "impl": impl, "op": op, "count": N,
                          "offsets": offs})
        del rng
    meta = {"generator": "tests/golden/make_ref_comp_vectors.py",
            "producer": "oracle/_ref/libref_ccl_comp.so = oracle/ref_comp_harness.cpp + reference src/comp/comp.cpp, "
                        "bf16/bf16.cpp, bf16/bf16_intrisics.cpp, fp16/fp16.cpp, fp16/fp16_intrisics.cpp, "
                        "common/log/log.cpp, common/utils/{spinlock,yield,memcpy}.cpp, common/datatype/datatype.cpp "
                        "(g++ -std=gnu++11 -O3 -DNDEBUG -fvisibility=internal, ITT off)",
            "n": N, "k_batch": K_BATCH, "cases": cases}
    arrs["meta"] = np.array(json.dumps(meta))
    return arrs


def main() -> int:
    if not REF_SO.exists():
        print(f"{REF_SO} missing: run `make -C oracle refcomp` (needs /root/reference)", file=sys.stderr)
        return 1
    arrs = generate()
    np.savez_compressed(OUT, **arrs)
    print(f"wrote {len(json.loads(str(arrs['meta']))['cases'])} cases to {OUT} ({OUT.stat().st_size} bytes)")
    return 0


if __name__ == "__main__":
    sys.exit(main())
