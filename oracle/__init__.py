"""TEST INFRASTRUCTURE ONLY — Python bindings of the CPU oracle
(oracle/comp_oracle.c, a restatement of oneCCL src/comp).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package, and only as the checker / the timed CPU baseline.  The
product (oneccl_amd) never imports it.
"""
from __future__ import annotations

import ctypes
import subprocess
from ctypes import POINTER, c_float, c_int, c_size_t, c_uint16, c_void_p
from pathlib import Path

import numpy as np

ODIR = Path(__file__).resolve().parent
LIB = ODIR / "lib" / "libcomp_oracle.so"

# ccl::datatype ids (include/oneapi/ccl/types.hpp:52-69) -> numpy storage
NP_DTYPE = {0: np.int8, 1: np.uint8, 2: np.int16, 3: np.uint16, 4: np.int32, 5: np.uint32,
            6: np.int64, 7: np.uint64, 8: np.uint16, 9: np.float32, 10: np.float64, 11: np.uint16}
BF16_SCALAR, BF16_AVX512F, BF16_AVX512BF = 0, 1, 2
FP16_NO_COMPILER, FP16_NO_HW, FP16_F16C, FP16_AVX512F, FP16_AVX512FP16 = 0, 1, 2, 3, 4

_lib = None


def build() -> None:
    subprocess.run(["make", "-C", str(ODIR), "-j4"], check=True, capture_output=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        L = ctypes.CDLL(str(LIB))
        L.orc_comp_reduce.argtypes = [c_void_p, c_size_t, c_void_p, POINTER(c_size_t), c_int, c_int, c_int, c_int]
        L.orc_comp_reduce_mt.argtypes = [c_void_p, c_size_t, c_void_p, c_int, c_int, c_int, c_int, c_int]
        L.orc_comp_batch_reduce.argtypes = [c_void_p, POINTER(c_size_t), c_size_t, c_size_t, c_void_p,
                                            POINTER(c_size_t), c_int, c_int, c_int, POINTER(c_float),
                                            POINTER(c_float), c_int, c_int]
        L.orc_convert_fp32_to_bf16_arrays.argtypes = [c_void_p, c_void_p, c_size_t, c_int]
        L.orc_convert_bf16_to_fp32_arrays.argtypes = [c_void_p, c_void_p, c_size_t]
        L.orc_convert_fp32_to_fp16_arrays.argtypes = [c_void_p, c_void_p, c_size_t]
        L.orc_convert_fp16_to_fp32_arrays.argtypes = [c_void_p, c_void_p, c_size_t]
        L.orc_bf16_to_fp32.argtypes = [c_uint16]
        L.orc_bf16_to_fp32.restype = c_float
        L.orc_fp32_to_bf16_trunc.argtypes = [c_float]
        L.orc_fp32_to_bf16_trunc.restype = c_uint16
        L.orc_fp32_to_bf16_rne.argtypes = [c_float]
        L.orc_fp32_to_bf16_rne.restype = c_uint16
        L.orc_fp16_to_fp32.argtypes = [c_uint16]
        L.orc_fp16_to_fp32.restype = c_float
        L.orc_fp32_to_fp16_rne.argtypes = [c_float]
        L.orc_fp32_to_fp16_rne.restype = c_uint16
        L.orc_lp_fanin_acc_fp32.argtypes = [POINTER(c_void_p), c_int, c_void_p, c_size_t, c_int, c_int, c_int, c_int]
        for f in ("orc_comp_reduce", "orc_comp_reduce_mt", "orc_comp_batch_reduce", "orc_lp_fanin_acc_fp32"):
            getattr(L, f).restype = c_int
        _lib = L
    return _lib


def _ptr(a: np.ndarray) -> int:
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data


def comp_reduce(in_buf: np.ndarray, inout_buf: np.ndarray, dtype: int, op: int,
                bf16_impl: int = BF16_AVX512BF, fp16_impl: int = FP16_AVX512F) -> int | None:
    """ccl_comp_reduce_regular on host arrays; inout_buf updated in place.
    Returns out_count (None when the reference leaves it untouched)."""
    assert in_buf.size == inout_buf.size
    oc = c_size_t(0xFFFFFFFFFFFFFFFF)
    rc = lib().orc_comp_reduce(_ptr(in_buf), in_buf.size, _ptr(inout_buf), ctypes.byref(oc), dtype, op,
                               bf16_impl, fp16_impl)
    if rc:
        raise ValueError("oracle rejected dtype/op")
    return None if oc.value == 0xFFFFFFFFFFFFFFFF else oc.value


def comp_reduce_mt(in_buf, inout_buf, dtype, op, nthreads, bf16_impl=BF16_AVX512BF, fp16_impl=FP16_AVX512F):
    rc = lib().orc_comp_reduce_mt(_ptr(in_buf), in_buf.size, _ptr(inout_buf), dtype, op, bf16_impl,
                                  fp16_impl, nthreads)
    if rc:
        raise ValueError("oracle rejected dtype/op")


def batch_reduce(in_buf: np.ndarray, offsets, count: int, inout_buf: np.ndarray, dtype: int, op: int,
                 keep_precision: int, bf16_impl: int = BF16_AVX512BF, fp16_impl: int = FP16_AVX512F):
    offs = (c_size_t * len(offsets))(*offsets)
    tmp = np.zeros(max(count, 1), np.float32)
    acc = np.zeros(max(count, 1), np.float32)
    oc = c_size_t(0xFFFFFFFFFFFFFFFF)
    rc = lib().orc_comp_batch_reduce(_ptr(in_buf), offs, len(offsets), count, _ptr(inout_buf), ctypes.byref(oc),
                                     dtype, op, keep_precision,
                                     tmp.ctypes.data_as(POINTER(c_float)), acc.ctypes.data_as(POINTER(c_float)),
                                     bf16_impl, fp16_impl)
    if rc:
        raise ValueError("oracle rejected dtype/op")
    return None if oc.value == 0xFFFFFFFFFFFFFFFF else oc.value


def fanin(inputs: list[np.ndarray], dtype: int, op: int, bf16_impl: int = BF16_AVX512BF,
          fp16_impl: int = FP16_AVX512F) -> np.ndarray:
    """Left fold acc = in0; acc = op(in_j, acc): the chained ccl_comp_reduce calls."""
    acc = inputs[0].copy()
    for x in inputs[1:]:
        comp_reduce(x, acc, dtype, op, bf16_impl, fp16_impl)
    return acc


def lp_fanin_acc_fp32(inputs: list[np.ndarray], dtype: int, op: int, bf16_rne: bool,
                      minmax_inout_first: bool) -> np.ndarray:
    out = np.empty_like(inputs[0])
    arr = (c_void_p * len(inputs))(*[_ptr(x) for x in inputs])
    rc = lib().orc_lp_fanin_acc_fp32(arr, len(inputs), _ptr(out), out.size, dtype, op, int(bf16_rne),
                                     int(minmax_inout_first))
    if rc:
        raise ValueError("oracle rejected dtype/op")
    return out


def f32_to_bf16(x: np.ndarray, rne: bool) -> np.ndarray:
    """Vectorised restatement of the oracle's scalar conversions (checked
    against them in tests/test_oracle.py)."""
    u = np.ascontiguousarray(x, np.float32).view(np.uint32)
    if not rne:
        return (u >> 16).astype(np.uint16)
    r = ((u + np.uint32(0x7FFF) + ((u >> 16) & np.uint32(1))) >> 16).astype(np.uint32)
    nan = (u & np.uint32(0x7FFFFFFF)) > np.uint32(0x7F800000)
    r = np.where(nan, (u >> 16) | np.uint32(0x40), r)
    den = (u & np.uint32(0x7F800000)) == 0
    r = np.where(den, (u >> 16) & np.uint32(0x8000), r)
    return r.astype(np.uint16)


def bf16_to_f32(b: np.ndarray) -> np.ndarray:
    return (b.astype(np.uint32) << 16).view(np.float32)


def f32_to_fp16(x: np.ndarray) -> np.ndarray:
    """VCVTPS2PH imm8=0 over an array (the oracle's scalar restatement, in C)."""
    src = np.ascontiguousarray(x, np.float32)
    out = np.empty(src.shape, np.uint16)
    lib().orc_convert_fp32_to_fp16_arrays(src.ctypes.data, out.ctypes.data, src.size)
    return out


def fp16_to_f32(h: np.ndarray) -> np.ndarray:
    """VCVTPH2PS over an array (C restatement: quiets a signalling NaN, which
    numpy's own half -> float conversion does not)."""
    src = np.ascontiguousarray(h).view(np.uint16)
    out = np.empty(src.shape, np.float32)
    lib().orc_convert_fp16_to_fp32_arrays(src.ctypes.data, out.ctypes.data, src.size)
    return out


# ---- the reference's own compiled CCL_REDUCE (oracle/_ref, built here) ----
# oracle/_ref/libref_ccl_comp.so = oracle/ref_comp_harness.cpp over the
# reference's src/comp/comp.cpp & co. with its Release flags (Makefile target
# refcomp).  Built in the container (needs /root/reference); the built library
# travels to the GPU box, where bench.py's cpu_baseline leg times it.
REF_COMP_SO = ODIR / "_ref" / "libref_ccl_comp.so"
_ref_comp = None


def ref_comp_available() -> bool:
    return REF_COMP_SO.exists()


def ref_comp_lib() -> ctypes.CDLL:
    """Loaded RTLD_LAZY: ccl::global_data::get/env stay unbound and are never
    called on the paths used (see the harness)."""
    global _ref_comp
    if _ref_comp is None:
        import os
        L = ctypes.CDLL(str(REF_COMP_SO), mode=os.RTLD_LAZY)
        L.ref_ccl_comp_reduce_regular.argtypes = [c_void_p, c_size_t, c_void_p, c_void_p, c_int, c_size_t, c_int]
        L.ref_ccl_comp_reduce_regular.restype = c_int
        _ref_comp = L
    return _ref_comp


def ref_comp_reduce(in_buf: np.ndarray, inout_buf: np.ndarray, dtype: int, op: int, nthreads: int = 1,
                    pool=None) -> None:
    """The reference's ccl_comp_reduce_regular on host arrays (non-LP types),
    the element range split over `nthreads` threads (ctypes drops the GIL),
    as CCL_WORKER_COUNT workers would each reduce their chunk."""
    L = ref_comp_lib()
    n, es = in_buf.size, in_buf.itemsize
    if nthreads <= 1:
        assert L.ref_ccl_comp_reduce_regular(in_buf.ctypes.data, n, inout_buf.ctypes.data, None, dtype, es, op) == 0
        return
    per = (n + nthreads - 1) // nthreads
    parts = [(i * per, min(n, (i + 1) * per)) for i in range(nthreads) if i * per < n]

    def one(se):
        s, e = se
        return L.ref_ccl_comp_reduce_regular(in_buf.ctypes.data + s * es, e - s, inout_buf.ctypes.data + s * es,
                                             None, dtype, es, op)

    if pool is None:
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(nthreads) as ex:
            assert all(rc == 0 for rc in ex.map(one, parts))
    else:
        assert all(rc == 0 for rc in pool.map(one, parts))
