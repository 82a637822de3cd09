"""ctypes bindings for the native libraries.

The product path is libmi_reduce.so (HIP, include/mi_reduce.h) and the drop-in
shim libccl_comp_hip.so (include/mi_ccl_comp.h).  Loading fails loudly if a
library is missing: there is no CPU fallback anywhere in the product.
"""
from __future__ import annotations

import ctypes
from ctypes import POINTER, c_char_p, c_double, c_int, c_long, c_size_t, c_uint, c_void_p
from pathlib import Path

PKG = Path(__file__).resolve().parent
LIB_DIR = PKG / "lib"

_mi = None
_shim = None


class MiReduceError(RuntimeError):
    pass


def _load(name: str) -> ctypes.CDLL:
    path = LIB_DIR / name
    if not path.exists():
        raise MiReduceError(
            f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(hipcc --offload-arch=gfx950). The product has no CPU fallback.")
    return ctypes.CDLL(str(path), mode=ctypes.RTLD_GLOBAL)


class MiReduceDesc(ctypes.Structure):
    """mi_reduce_desc_t (include/mi_reduce.h)."""
    _fields_ = [("in_", c_void_p), ("inout", c_void_p), ("count", c_size_t)]


# (name, restype, argtypes) — mirrors include/mi_reduce.h
MI_API = [
    ("mi_reduce", c_int, [c_void_p, c_void_p, c_size_t, c_int, c_int, c_uint, c_void_p]),
    ("mi_reduce_out", c_int, [c_void_p, c_void_p, c_void_p, c_size_t, c_int, c_int, c_uint, c_void_p]),
    ("mi_reduce_multi", c_int, [POINTER(c_void_p), c_int, c_void_p, c_size_t, c_int, c_int, c_uint, c_void_p]),
    ("mi_reduce_batch", c_int, [POINTER(MiReduceDesc), c_int, c_int, c_int, c_uint, c_void_p]),
    ("mi_reduce_sync", c_int, [c_void_p, c_void_p, c_size_t, c_int, c_int, c_uint, c_int]),
    ("mi_reduce_multi_sync", c_int, [POINTER(c_void_p), c_int, c_void_p, c_size_t, c_int, c_int, c_uint, c_int]),
    ("mi_convert", c_int, [c_void_p, c_int, c_void_p, c_int, c_size_t, c_uint, c_void_p]),
    ("mi_convert_sync", c_int, [c_void_p, c_int, c_void_p, c_int, c_size_t, c_uint, c_int]),
    ("mi_reduce_start", c_int, [POINTER(c_void_p), c_int, c_void_p, c_size_t, c_int, c_int, c_uint, c_int,
                                POINTER(c_void_p)]),
    ("mi_reduce_start_timed", c_int, [POINTER(c_void_p), c_int, c_void_p, c_size_t, c_int, c_int, c_uint, c_int,
                                      POINTER(c_void_p)]),
    ("mi_request_run_time", c_int, [c_void_p, POINTER(c_double)]),
    ("mi_reduce_split_start", c_int, [POINTER(c_void_p), c_int, c_void_p, c_size_t, c_int, c_int, c_uint, c_int,
                                      c_size_t, c_void_p, POINTER(c_void_p)]),
    ("mi_request_split_times", c_int, [c_void_p, POINTER(c_double), POINTER(c_double)]),
    ("mi_test", c_int, [c_void_p, POINTER(c_int)]),
    ("mi_thread_sync", c_int, []),
    ("mi_wait", c_int, [c_void_p]),
    ("mi_request_free", c_int, [c_void_p]),
    ("mi_reduce_sharded", c_int, [c_int, POINTER(c_int), POINTER(c_void_p), c_int, POINTER(c_void_p),
                                  POINTER(c_size_t), c_int, c_int, c_uint]),
    ("mi_reduce_multi_sync_sharded", c_int, [POINTER(c_void_p), c_int, c_void_p, c_size_t, c_int, c_int, c_uint,
                                             c_int, POINTER(c_int)]),
    ("mi_copy_sync", c_int, [c_void_p, c_void_p, c_size_t, c_int, c_int]),
    ("mi_copy", c_int, [c_void_p, c_void_p, c_size_t, c_int, c_void_p]),
    ("mi_shard_range", c_int, [c_size_t, c_int, c_int, c_size_t, POINTER(c_size_t), POINTER(c_size_t)]),
    ("mi_pointer_kind", c_int, [c_void_p, POINTER(c_int)]),
    ("mi_pointer_kind_range", c_int, [c_void_p, c_size_t, POINTER(c_int)]),
    ("mi_host_declare", c_int, [c_void_p, c_size_t]),
    ("mi_host_undeclare", c_int, [c_void_p]),
    ("mi_host_declared_kind", c_int, [c_void_p, c_size_t]),
    ("mi_pointer_lookups", c_size_t, []),
    ("mi_test_hold_exit_guard", c_int, [c_int]),
    ("mi_test_fail_copy", c_int, [c_long]),
    ("mi_test_staged_device", c_int, []),
    ("mi_test_copy_error", c_int, [c_void_p, c_size_t, c_size_t, c_int, c_int]),
    ("mi_host_register", c_int, [c_void_p, c_size_t]),
    ("mi_host_unregister", c_int, [c_void_p]),
    ("mi_reduction_to_str", c_char_p, [c_int]),
    ("mi_dtype_size", c_size_t, [c_int]),
    ("mi_last_error", c_char_p, []),
    ("mi_version", c_int, []),
    ("mi_device_count", c_int, []),
    ("mi_get_launch_config", c_int, [POINTER(c_int), POINTER(c_int), POINTER(c_int)]),
    ("mi_get_residency", c_int, [c_int, c_int, POINTER(c_int), POINTER(c_uint)]),
    ("mi_set_max_blocks", c_int, [c_int]),
    ("mi_set_residency", c_int, [c_int, c_int]),
    ("mi_set_host_mode", c_int, [c_int]),
    ("mi_set_sync_mode", c_int, [c_int]),
    ("mi_set_unaligned_vectors", c_int, [c_int]),
    ("mi_helper_cpu_count", c_int, []),
    ("mi_context_stats", c_int, [POINTER(c_size_t), POINTER(c_size_t)]),
    ("mi_release_pooled_contexts", c_int, []),
]

# mirrors include/mi_ccl_comp.h
MI_CCL_REDUCTION_FN = ctypes.CFUNCTYPE(None, c_void_p, c_size_t, c_void_p, POINTER(c_size_t), c_int, c_void_p)
SHIM_API = [
    ("mi_ccl_comp_reduce", c_int, [c_void_p, c_size_t, c_void_p, POINTER(c_size_t), c_int, c_int]),
    ("mi_ccl_comp_reduce_custom", c_int, [c_void_p, c_size_t, c_void_p, POINTER(c_size_t), c_int, MI_CCL_REDUCTION_FN]),
    ("mi_ccl_comp_batch_reduce", c_int, [c_void_p, POINTER(c_size_t), c_size_t, c_size_t, c_void_p,
                                         POINTER(c_size_t), c_int, c_int, c_int]),
    ("mi_ccl_comp_batch_reduce_custom", c_int, [c_void_p, POINTER(c_size_t), c_size_t, c_size_t, c_void_p,
                                                POINTER(c_size_t), c_int, c_int, MI_CCL_REDUCTION_FN]),
    ("mi_ccl_comp_copy", c_int, [c_void_p, c_void_p, c_size_t, c_int]),
    ("mi_ccl_comp_copy_host", c_int, [c_void_p, c_void_p, c_size_t, c_int]),
    ("mi_ccl_bf16_reduce", c_int, [c_void_p, c_size_t, c_void_p, POINTER(c_size_t), c_int]),
    ("mi_ccl_fp16_reduce", c_int, [c_void_p, c_size_t, c_void_p, POINTER(c_size_t), c_int]),
    ("mi_ccl_bf16_reduce_host", c_int, [c_void_p, c_size_t, c_void_p, POINTER(c_size_t), c_int]),
    ("mi_ccl_fp16_reduce_host", c_int, [c_void_p, c_size_t, c_void_p, POINTER(c_size_t), c_int]),
    ("mi_ccl_convert_fp32_to_bf16_arrays", c_int, [c_void_p, c_void_p, c_size_t]),
    ("mi_ccl_convert_bf16_to_fp32_arrays", c_int, [c_void_p, c_void_p, c_size_t]),
    ("mi_ccl_convert_fp32_to_fp16", c_int, [c_void_p, c_void_p]),
    ("mi_ccl_convert_fp16_to_fp32", c_int, [c_void_p, c_void_p]),
    ("mi_ccl_comp_reduce_start", c_int, [c_void_p, c_size_t, c_void_p, POINTER(c_size_t), c_int, c_int,
                                         MI_CCL_REDUCTION_FN, POINTER(c_void_p)]),
    ("mi_ccl_comp_batch_reduce_start", c_int, [c_void_p, POINTER(c_size_t), c_size_t, c_size_t, c_void_p,
                                               POINTER(c_size_t), c_int, c_int, c_int, POINTER(c_void_p)]),
    ("mi_ccl_comp_request_test", c_int, [c_void_p, POINTER(c_int)]),
    ("mi_ccl_comp_request_wait", c_int, [c_void_p]),
    ("mi_ccl_comp_request_free", c_int, [c_void_p]),
    ("mi_ccl_reduction_to_str", c_char_p, [c_int]),
    ("mi_ccl_env_reload", c_int, []),
    ("mi_ccl_comp_split_share", c_double, [c_int]),
    ("mi_ccl_comp_host_workers", c_int, []),
    ("mi_ccl_comp_split_gpu_rate", c_double, [c_int, POINTER(c_uint)]),
    ("mi_ccl_comp_split_take_gpu_alone", c_int, [c_int]),
    ("mi_ccl_comp_split_feed", c_int, [c_int, c_size_t, c_size_t, c_double, c_double]),
    ("mi_ccl_comp_host_max", c_int, [POINTER(c_size_t), POINTER(c_size_t), POINTER(c_double), POINTER(c_double)]),
    ("mi_ccl_comp_register_host_buffer", c_int, [c_void_p, c_size_t]),
    ("mi_ccl_comp_unregister_host_buffer", c_int, [c_void_p]),
    ("mi_ccl_comp_pointer_lookups", c_size_t, []),
    ("mi_ccl_comp_shim_sched", c_int, [c_int]),
    ("mi_ccl_impl_types", c_int, [POINTER(c_int), POINTER(c_int)]),
    ("mi_ccl_comp_device", c_int, []),
    ("mi_ccl_last_error", c_char_p, []),
]


# mirrors include/mi_host_reduce.h (exported by libccl_comp_hip.so)
HOST_API = [
    ("mi_host_supported", c_int, []),
    ("mi_host_reduce", c_int, [POINTER(c_void_p), c_int, c_void_p, c_size_t, c_int, c_int, c_uint]),
    ("mi_host_convert", c_int, [c_void_p, c_int, c_void_p, c_int, c_size_t, c_uint]),
    ("mi_host_copy", c_int, [c_void_p, c_void_p, c_size_t, c_int]),
]


def _bind(lib: ctypes.CDLL, api) -> ctypes.CDLL:
    for name, res, args in api:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def mi() -> ctypes.CDLL:
    """libmi_reduce.so with typed signatures."""
    global _mi
    if _mi is None:
        _mi = _bind(_load("libmi_reduce.so"), MI_API)
    return _mi


def shim() -> ctypes.CDLL:
    """libccl_comp_hip.so (the drop-in src/comp) with typed signatures."""
    global _shim
    if _shim is None:
        mi()
        _shim = _bind(_bind(_load("libccl_comp_hip.so"), SHIM_API), HOST_API)
    return _shim


def check(rc: int, what: str = "mi_reduce") -> None:
    if rc != 0:
        raise MiReduceError(f"{what} failed ({rc}): {mi().mi_last_error().decode()}")


def check_shim(rc: int, what: str = "ccl_comp") -> None:
    if rc != 0:
        raise MiReduceError(f"{what} failed ({rc}): {shim().mi_ccl_last_error().decode()}")


def void_ptr_array(ptrs) -> ctypes.Array:
    arr = (c_void_p * len(ptrs))()
    for i, p in enumerate(ptrs):
        arr[i] = p
    return arr


def desc_array(triples) -> ctypes.Array:
    """[(in_ptr, inout_ptr, count), ...] -> mi_reduce_desc_t[]."""
    arr = (MiReduceDesc * max(len(triples), 1))()
    for i, (a, b, n) in enumerate(triples):
        arr[i] = MiReduceDesc(a, b, n)
    return arr


def lib_paths() -> list[str]:
    return [str(LIB_DIR / "libmi_reduce.so"), str(LIB_DIR / "libccl_comp_hip.so")]


__all__ = ["mi", "shim", "check", "check_shim", "void_ptr_array", "MiReduceError", "MI_CCL_REDUCTION_FN",
           "MI_API", "SHIM_API", "HOST_API", "lib_paths"]
