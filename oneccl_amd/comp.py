"""Host-side Python mirror of oneCCL's local-reduction interface, over the HIP
C ABI (include/mi_reduce.h).

Names and argument meaning follow the reference:
  reduction / datatype          include/oneapi/ccl/types.hpp:41-69
  comp_reduce(in, inout, ...)   ccl_comp_reduce, src/comp/comp.cpp:123-200
  comp_batch_reduce(...)        ccl_comp_batch_reduce, src/comp/comp.cpp:202-249
  comp_copy(...)                ccl_comp_copy, src/comp/comp.cpp:60-74
  reduction_to_str(op)          ccl_reduction_to_str, src/comp/comp.cpp:251-260
The device entry points (`reduce`, `reduce_out`, `reduce_multi`) take torch
CUDA(HIP) tensors and launch asynchronously on a stream; `comp_*` go through
the drop-in C++ shim (libccl_comp_hip.so) and are synchronous with host or
device buffers, exactly as src/sched calls src/comp.
"""
from __future__ import annotations

import ctypes
from enum import IntEnum
from typing import Optional, Sequence

from . import _lib
from ._lib import check, check_shim, mi, shim, void_ptr_array


class reduction(IntEnum):
    sum = 0
    prod = 1
    min = 2
    max = 3
    custom = 4


class datatype(IntEnum):
    int8 = 0
    uint8 = 1
    int16 = 2
    uint16 = 3
    int32 = 4
    uint32 = 5
    int64 = 6
    uint64 = 7
    float16 = 8
    float32 = 9
    float64 = 10
    bfloat16 = 11


class bf16_impl(IntEnum):  # ccl_bf16_impl_type, src/comp/bf16/bf16_utils.hpp:26
    scalar = 0
    avx512f = 1
    avx512bf = 2


class fp16_impl(IntEnum):  # ccl_fp16_impl_type, src/comp/fp16/fp16_utils.hpp:26-32
    no_compiler_support = 0
    no_hardware_support = 1
    f16c = 2
    avx512f = 3
    avx512fp16 = 4


# semantic variant flags (include/mi_reduce.h)
F_MINMAX_INOUT_FIRST = 0x1
F_BF16_RNE = 0x2
F_ACC_FP32 = 0x4
F_BF16_TAIL_TRUNC16 = 0x8
F_FP16_NATIVE_MINMAX = 0x10

DTYPE_SIZE = {datatype.int8: 1, datatype.uint8: 1, datatype.int16: 2, datatype.uint16: 2, datatype.int32: 4,
              datatype.uint32: 4, datatype.int64: 8, datatype.uint64: 8, datatype.float16: 2,
              datatype.float32: 4, datatype.float64: 8, datatype.bfloat16: 2}


def bf16_flags(impl: bf16_impl) -> int:
    """Bit-level behaviour of the reference's bf16 reduce for an impl type
    (bf16.cpp:63-110, bf16_intrisics.hpp:62-147)."""
    impl = bf16_impl(impl)
    if impl == bf16_impl.scalar:
        return 0
    if impl == bf16_impl.avx512f:
        return F_MINMAX_INOUT_FIRST
    return F_MINMAX_INOUT_FIRST | F_BF16_RNE


def fp16_flags(impl: fp16_impl = fp16_impl.avx512f) -> int:
    """f16c / avx512f / avx512fp16: MINPS order, RNE (fp16_intrisics.hpp:204-248)."""
    return F_MINMAX_INOUT_FIRST


def reference_flags(dtype: datatype, bf16: bf16_impl = bf16_impl.avx512bf,
                    fp16: fp16_impl = fp16_impl.avx512f) -> int:
    """The flags under which the kernels reproduce ccl_comp_reduce for `dtype`."""
    if dtype == datatype.bfloat16:
        return bf16_flags(bf16)
    if dtype == datatype.float16:
        return fp16_flags(fp16)
    return 0


def _torch_ccl_dtype(t) -> datatype:
    import torch
    table = {torch.int8: datatype.int8, torch.uint8: datatype.uint8, torch.int16: datatype.int16,
             torch.int32: datatype.int32, torch.int64: datatype.int64, torch.float16: datatype.float16,
             torch.float32: datatype.float32, torch.float64: datatype.float64, torch.bfloat16: datatype.bfloat16}
    for name, dt in (("uint16", datatype.uint16), ("uint32", datatype.uint32), ("uint64", datatype.uint64)):
        if hasattr(torch, name):
            table[getattr(torch, name)] = dt
    if t.dtype not in table:
        raise TypeError(f"no ccl datatype for {t.dtype}")
    return table[t.dtype]


def _stream_handle(stream) -> int:
    import torch
    if stream is None:
        stream = torch.cuda.current_stream()
    return int(stream.cuda_stream) if hasattr(stream, "cuda_stream") else int(stream)


def _dev_args(tensors, dtype):
    t0 = tensors[0]
    dt = datatype(dtype) if dtype is not None else _torch_ccl_dtype(t0)
    esize = DTYPE_SIZE[dt]
    for t in tensors:
        if not t.is_cuda:
            raise ValueError("device entry points take device tensors (use comp_reduce for host buffers)")
        if not t.is_contiguous():
            raise ValueError("tensors must be contiguous")
        if t.numel() * t.element_size() != t0.numel() * t0.element_size():
            raise ValueError("all operands must have the same byte size")
    nbytes = t0.numel() * t0.element_size()
    if nbytes % esize:
        raise ValueError("byte size is not a multiple of the datatype size")
    return dt, nbytes // esize


def reduce(in_t, inout_t, op: reduction = reduction.sum, flags: Optional[int] = None,
           dtype: Optional[datatype] = None, stream=None) -> None:
    """inout = op(in, inout) on device tensors, asynchronously on `stream`."""
    dt, count = _dev_args([in_t, inout_t], dtype)
    f = reference_flags(dt) if flags is None else flags
    check(mi().mi_reduce(in_t.data_ptr(), inout_t.data_ptr(), count, int(dt), int(op), f, _stream_handle(stream)),
          "mi_reduce")


def reduce_out(in1, in2, out, op: reduction = reduction.sum, flags: Optional[int] = None,
               dtype: Optional[datatype] = None, stream=None) -> None:
    """out = op(in1 [in role], in2 [inout role]) on device tensors."""
    dt, count = _dev_args([in1, in2, out], dtype)
    f = reference_flags(dt) if flags is None else flags
    check(mi().mi_reduce_out(in1.data_ptr(), in2.data_ptr(), out.data_ptr(), count, int(dt), int(op), f,
                             _stream_handle(stream)), "mi_reduce_out")


def reduce_multi(inputs: Sequence, out, op: reduction = reduction.sum, flags: Optional[int] = None,
                 dtype: Optional[datatype] = None, stream=None) -> None:
    """out = left fold over inputs (acc = inputs[0]; acc = op(inputs[j], acc))."""
    dt, count = _dev_args(list(inputs) + [out], dtype)
    f = reference_flags(dt) if flags is None else flags
    arr = void_ptr_array([t.data_ptr() for t in inputs])
    check(mi().mi_reduce_multi(arr, len(inputs), out.data_ptr(), count, int(dt), int(op), f,
                               _stream_handle(stream)), "mi_reduce_multi")


# ---- the drop-in shim (synchronous, host or device pointers) ------------

def comp_reduce(in_ptr: int, count: int, inout_ptr: int, dtype: datatype, op: reduction) -> Optional[int]:
    """ccl_comp_reduce(nullptr, in, count, inout, &out_count, dtype, op, nullptr).
    Returns out_count if the reference would have written it (bf16/fp16)."""
    oc = ctypes.c_size_t(0xFFFFFFFFFFFFFFFF)
    check_shim(shim().mi_ccl_comp_reduce(in_ptr, count, inout_ptr, ctypes.byref(oc), int(dtype), int(op)),
               "ccl_comp_reduce")
    return None if oc.value == 0xFFFFFFFFFFFFFFFF else oc.value


def comp_batch_reduce(in_ptr: int, offsets: Sequence[int], count: int, inout_ptr: int, dtype: datatype,
                      op: reduction, bf16_keep_precision_mode: int = 0) -> Optional[int]:
    offs = (ctypes.c_size_t * len(offsets))(*offsets)
    oc = ctypes.c_size_t(0xFFFFFFFFFFFFFFFF)
    check_shim(shim().mi_ccl_comp_batch_reduce(in_ptr, offs, len(offsets), count, inout_ptr, ctypes.byref(oc),
                                               int(dtype), int(op), int(bf16_keep_precision_mode)),
               "ccl_comp_batch_reduce")
    return None if oc.value == 0xFFFFFFFFFFFFFFFF else oc.value


class comp_request:
    """An in-flight ccl_comp_reduce_start (include/mi_ccl_comp_async.hpp).
    `out_count` is what the reference would have written (bf16/fp16) or None."""

    def __init__(self, handle: int, out_count: Optional[int], keep=None):
        self._h = handle
        self.out_count = out_count
        self._keep = keep  # a ctypes callback must outlive the call

    def test(self) -> bool:
        done = ctypes.c_int(0)
        check_shim(shim().mi_ccl_comp_request_test(self._h, ctypes.byref(done)), "ccl_comp_request_test")
        return bool(done.value)

    def wait(self) -> None:
        check_shim(shim().mi_ccl_comp_request_wait(self._h), "ccl_comp_request_wait")

    def free(self) -> None:
        if self._h is not None:
            h, self._h = self._h, None
            check_shim(shim().mi_ccl_comp_request_free(h), "ccl_comp_request_free")


def comp_reduce_start(in_ptr: int, count: int, inout_ptr: int, dtype: datatype, op: reduction,
                      fn=None) -> comp_request:
    """ccl_comp_reduce_start: issue the reduce, return a request to poll
    (the async form a schedule entry's start()/update() pair would use)."""
    oc = ctypes.c_size_t(0xFFFFFFFFFFFFFFFF)
    h = ctypes.c_void_p()
    cb = _lib.MI_CCL_REDUCTION_FN(fn) if fn is not None else _lib.MI_CCL_REDUCTION_FN()
    check_shim(shim().mi_ccl_comp_reduce_start(in_ptr, count, inout_ptr, ctypes.byref(oc), int(dtype), int(op), cb,
                                               ctypes.byref(h)), "ccl_comp_reduce_start")
    return comp_request(h.value, None if oc.value == 0xFFFFFFFFFFFFFFFF else oc.value, cb)


def comp_batch_reduce_start(in_ptr: int, offsets: Sequence[int], count: int, inout_ptr: int, dtype: datatype,
                            op: reduction, bf16_keep_precision_mode: int = 0) -> comp_request:
    """ccl_comp_batch_reduce_start: the fused K-input fold as one request."""
    offs = (ctypes.c_size_t * len(offsets))(*offsets)
    oc = ctypes.c_size_t(0xFFFFFFFFFFFFFFFF)
    h = ctypes.c_void_p()
    check_shim(shim().mi_ccl_comp_batch_reduce_start(in_ptr, offs, len(offsets), count, inout_ptr, ctypes.byref(oc),
                                                     int(dtype), int(op), int(bf16_keep_precision_mode),
                                                     ctypes.byref(h)), "ccl_comp_batch_reduce_start")
    return comp_request(h.value, None if oc.value == 0xFFFFFFFFFFFFFFFF else oc.value)


def comp_copy(in_ptr: int, out_ptr: int, nbytes: int, use_nontemporal: bool = False) -> None:
    check_shim(shim().mi_ccl_comp_copy(in_ptr, out_ptr, nbytes, int(use_nontemporal)), "ccl_comp_copy")


def reduction_to_str(op: int) -> str:
    return shim().mi_ccl_reduction_to_str(int(op)).decode()


def impl_types() -> tuple[bf16_impl, fp16_impl]:
    b, f = ctypes.c_int(), ctypes.c_int()
    check_shim(shim().mi_ccl_impl_types(ctypes.byref(b), ctypes.byref(f)), "impl_types")
    return bf16_impl(b.value), fp16_impl(f.value)


def env_reload() -> None:
    """Re-read CCL_BF16 / CCL_FP16 / CCL_COMP_HIP_DEVICE."""
    check_shim(shim().mi_ccl_env_reload(), "env_reload")


def shard_range(count: int, rank: int, world: int, align: int = 256) -> tuple[int, int]:
    b, e = ctypes.c_size_t(), ctypes.c_size_t()
    check(mi().mi_shard_range(count, rank, world, align, ctypes.byref(b), ctypes.byref(e)), "mi_shard_range")
    return b.value, e.value


__all__ = ["reduction", "datatype", "bf16_impl", "fp16_impl", "reduce", "reduce_out", "reduce_multi",
           "comp_reduce", "comp_reduce_start", "comp_batch_reduce_start", "comp_request", "comp_batch_reduce", "comp_copy", "reduction_to_str", "impl_types", "env_reload",
           "shard_range", "bf16_flags", "fp16_flags", "reference_flags", "F_MINMAX_INOUT_FIRST", "F_BF16_RNE",
           "F_ACC_FP32", "F_BF16_TAIL_TRUNC16", "DTYPE_SIZE", "_lib"]
