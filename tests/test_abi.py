"""CPU-side checks of the boundary: the libraries load without a GPU, export
every symbol the public headers declare, and the pure-host functions behave
(no device compute here)."""
from __future__ import annotations

import ctypes
import re
import subprocess
from pathlib import Path

import pytest

from oneccl_amd import _lib

ROOT = Path(__file__).resolve().parent.parent


def _declared(header: str) -> list[str]:
    text = (ROOT / "include" / header).read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return re.findall(r"^\s*(?:const\s+)?[a-z_]+\s*\**\s+(mi_[a-z0-9_]+)\s*\(", text, flags=re.M)


def _exported(lib: str) -> set[str]:
    out = subprocess.run(["nm", "-D", "--defined-only", str(ROOT / "oneccl_amd" / "lib" / lib)],
                         check=True, capture_output=True, text=True).stdout
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


@pytest.mark.parametrize("header,lib", [("mi_reduce.h", "libmi_reduce.so"), ("mi_ccl_comp.h", "libccl_comp_hip.so"),
                                        ("mi_host_reduce.h", "libccl_comp_hip.so")])
def test_every_declared_symbol_is_exported(header, lib):
    decl = _declared(header)
    assert len(decl) >= 3
    missing = set(decl) - _exported(lib)
    assert not missing, f"{lib} lacks {sorted(missing)}"


def test_python_binding_covers_header():
    assert {n for n, _, _ in _lib.MI_API} == set(_declared("mi_reduce.h"))
    assert {n for n, _, _ in _lib.SHIM_API} == set(_declared("mi_ccl_comp.h"))
    assert {n for n, _, _ in _lib.HOST_API} == set(_declared("mi_host_reduce.h"))


def test_shim_exports_onecll_mangled_entry_points():
    """The drop-in exports oneCCL's own C++ symbols (src/comp/comp.hpp:23-51)."""
    out = subprocess.run(["nm", "-DC", "--defined-only", str(ROOT / "oneccl_amd/lib/libccl_comp_hip.so")],
                         check=True, capture_output=True, text=True).stdout
    want = [
        "ccl_comp_reduce(ccl_sched*, void const*, unsigned long, void*, unsigned long*, ccl_datatype const&, "
        "ccl::v1::reduction, void (*)(void const*, unsigned long, void*, unsigned long*, ccl::v1::datatype, "
        "ccl::v1::fn_context const*), ccl::v1::fn_context const*)",
        "ccl_comp_copy(void const*, void*, unsigned long, bool)",
        "ccl_reduction_to_str(ccl::v1::reduction)",
        "ccl_bf16_reduce(void const*, unsigned long, void*, unsigned long*, ccl::v1::reduction)",
        "ccl_fp16_reduce(void const*, unsigned long, void*, unsigned long*, ccl::v1::reduction)",
        "ccl_comp_batch_reduce(void const*, std::vector<unsigned long, std::allocator<unsigned long> > const&, "
        "unsigned long, void*, unsigned long*, ccl_datatype const&, ccl::v1::reduction, void (*)(void const*, "
        "unsigned long, void*, unsigned long*, ccl::v1::datatype, ccl::v1::fn_context const*), "
        "ccl::v1::fn_context const*, int, float*, float*)",
    ]
    for w in want:
        assert w in out, w


def test_shim_exports_async_entry_points():
    """The asynchronous form declared in include/mi_ccl_comp_async.hpp."""
    out = subprocess.run(["nm", "-DC", "--defined-only", str(ROOT / "oneccl_amd/lib/libccl_comp_hip.so")],
                         check=True, capture_output=True, text=True).stdout
    for w in ["ccl_comp_reduce_start(ccl_sched*, void const*, unsigned long, void*, unsigned long*, ccl_datatype const&, "
              "ccl::v1::reduction, void (*)(void const*, unsigned long, void*, unsigned long*, ccl::v1::datatype, "
              "ccl::v1::fn_context const*), ccl::v1::fn_context const*, ccl_comp_request**)",
              "ccl_comp_request_test(ccl_comp_request*)", "ccl_comp_request_wait(ccl_comp_request*)",
              "ccl_comp_request_free(ccl_comp_request*)"]:
        assert w in out, w


def test_shim_exports_mpi_user_op_host_entries():
    """The MPI user ops' host-word entries (include/mi_ccl_lp_host.hpp,
    integration/0002), with ccl_bf16_reduce's signature."""
    out = subprocess.run(["nm", "-DC", "--defined-only", str(ROOT / "oneccl_amd/lib/libccl_comp_hip.so")],
                         check=True, capture_output=True, text=True).stdout
    for name in ("ccl_bf16_reduce_host", "ccl_fp16_reduce_host"):
        w = f"{name}(void const*, unsigned long, void*, unsigned long*, ccl::v1::reduction)"
        assert w in out, w


def test_async_empty_reduce_needs_no_device():
    """in_count == 0 completes inside start without touching HIP
    (comp.cpp:132-134); a null request pointer is an error."""
    from oneccl_amd import comp
    buf = (ctypes.c_float * 4)(1, 2, 3, 4)
    req = comp.comp_reduce_start(ctypes.addressof(buf), 0, ctypes.addressof(buf), comp.datatype.float32,
                                 comp.reduction.sum)
    assert req.test()
    req.free()
    assert list(buf) == [1, 2, 3, 4]
    rc = _lib.shim().mi_ccl_comp_reduce_start(None, 1, None, None, 9, 0, _lib.MI_CCL_REDUCTION_FN(), None)
    assert rc == -1 and b"null request" in _lib.shim().mi_ccl_last_error()


def test_reduction_to_str_matches_reference():
    # src/comp/comp.cpp:251-260
    m = _lib.mi()
    assert [m.mi_reduction_to_str(i).decode() for i in range(6)] == ["sum", "prod", "min", "max", "custom",
                                                                      "unknown"]
    s = _lib.shim()
    assert [s.mi_ccl_reduction_to_str(i).decode() for i in range(5)] == ["sum", "prod", "min", "max", "custom"]


def test_dtype_sizes():
    m = _lib.mi()
    assert [m.mi_dtype_size(i) for i in range(12)] == [1, 1, 2, 2, 4, 4, 8, 8, 2, 4, 8, 2]
    assert m.mi_dtype_size(12) == 0


def test_argument_errors_need_no_device():
    m = _lib.mi()
    assert m.mi_reduce(0, 0, 0, 9, 0, 0, None) == 0  # in_count == 0 is success (comp.cpp:132-134)
    assert m.mi_reduce(0, 0, 10, 42, 0, 0, None) == -1
    assert b"datatype" in m.mi_last_error()
    assert m.mi_reduce(0, 0, 10, 9, 4, 0, None) == -1  # custom is host-only
    arr = _lib.void_ptr_array([0] * 17)
    assert m.mi_reduce_multi(arr, 17, 0, 10, 9, 0, 0, None) == -1
    assert m.mi_reduce_batch(None, 0, 9, 0, 0, None) == 0  # empty batch
    assert m.mi_reduce_batch(None, 3, 9, 0, 0, None) == -1
    assert m.mi_reduce_batch(_lib.desc_array([]), -1, 9, 0, 0, None) == -1
    assert m.mi_reduce_batch(_lib.desc_array([(0, 0, 10)]), 1, 42, 0, 0, None) == -1
    assert m.mi_reduce_batch(_lib.desc_array([(0, 0, 0), (0, 0, 0)]), 2, 9, 0, 0, None) == 0  # all empty
    assert m.mi_reduce_batch(_lib.desc_array([(0, 0, 5)]), 1, 9, 0, 0, None) == -1  # null operand


def test_device_entry_points_refuse_pageable_memory():
    """A pageable host pointer handed to an asynchronous device entry point is
    refused before any launch (a kernel touching it would fault the GPU)."""
    m = _lib.mi()
    a = (ctypes.c_float * 64)()
    b = (ctypes.c_float * 64)()
    pa, pb = ctypes.addressof(a), ctypes.addressof(b)
    assert m.mi_reduce(pa, pb, 64, 9, 0, 0, None) == -1
    assert b"pageable" in m.mi_last_error()
    assert m.mi_reduce_out(pa, pb, pb, 64, 9, 0, 0, None) == -1
    assert m.mi_reduce_multi(_lib.void_ptr_array([pa, pb, pa]), 3, pb, 64, 9, 0, 0, None) == -1
    assert m.mi_convert(pa, 9, pb, 11, 64, 0, None) == -1
    assert m.mi_copy(pa, pb, 256, 0, None) == -1
    assert m.mi_reduce_batch(_lib.desc_array([(pa, pb, 64)]), 1, 9, 0, 0, None) == -1


@pytest.mark.parametrize("count", [0, 1, 255, 256, 1000, 1 << 28, (1 << 28) + 3])
@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_shard_range_partitions(count, world):
    m = _lib.mi()
    prev = 0
    for r in range(world):
        b, e = ctypes.c_size_t(), ctypes.c_size_t()
        assert m.mi_shard_range(count, r, world, 256, ctypes.byref(b), ctypes.byref(e)) == 0
        assert b.value == prev and e.value >= b.value
        assert b.value % 256 == 0 or b.value == count
        prev = e.value
    assert prev == count


def test_launch_config():
    m = _lib.mi()
    b, u, mb = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    assert m.mi_get_launch_config(ctypes.byref(b), ctypes.byref(u), ctypes.byref(mb)) == 0
    assert b.value % 64 == 0 and u.value >= 1 and mb.value >= 0
    assert m.mi_set_max_blocks(-1) == -1
    assert m.mi_set_max_blocks(mb.value) == 0


def test_version():
    assert _lib.mi().mi_version() >= 100


def test_residency_plan():
    """The one-wave kernels' resident-wave caps, as the LDS
    granules achieve them: 21 per CU for the 2-input kernel and the
    conversions, 16/11/9/8/5 for a fan-in of <=4/<=6/<=8/<=12/<=16 inputs.
    Without a GPU the LDS size is unknown and no cap is reserved."""
    m = _lib.mi()
    w, lds = ctypes.c_int(), ctypes.c_uint()
    want = {0: 21, 1: 16, 2: 21, 3: 16, 4: 16, 5: 11, 6: 11, 7: 9, 8: 9, 9: 8, 12: 8, 13: 5, 16: 5}
    for k, waves in want.items():
        assert m.mi_get_residency(-1, k, ctypes.byref(w), ctypes.byref(lds)) == 0
        assert w.value == waves, (k, w.value)
        if m.mi_device_count() == 0:
            assert lds.value == 0
    assert m.mi_get_residency(-1, 17, ctypes.byref(w), ctypes.byref(lds)) == -1
    assert m.mi_get_residency(-1, -1, None, None) == -1


def test_residency_override():
    """mi_set_residency (tuning knob): replaces the plan for one k, is
    reported by mi_get_residency, and 0 restores the plan."""
    m = _lib.mi()
    w = ctypes.c_int()
    try:
        assert m.mi_set_residency(2, 18) == 0
        assert m.mi_get_residency(-1, 2, ctypes.byref(w), None) == 0 and w.value == 18
        assert m.mi_get_residency(-1, 8, ctypes.byref(w), None) == 0 and w.value == 9  # other k untouched
        assert m.mi_set_residency(8, 32) == 0
        assert m.mi_get_residency(-1, 8, ctypes.byref(w), None) == 0 and w.value == 32
    finally:
        assert m.mi_set_residency(2, 0) == 0 and m.mi_set_residency(8, 0) == 0
    assert m.mi_get_residency(-1, 2, ctypes.byref(w), None) == 0 and w.value == 21
    assert m.mi_get_residency(-1, 8, ctypes.byref(w), None) == 0 and w.value == 9
    assert m.mi_set_residency(17, 8) == -1 and m.mi_set_residency(-1, 8) == -1
    assert m.mi_set_residency(2, 33) == -1 and m.mi_set_residency(2, -1) == -1


def test_context_stats_need_no_device():
    created, pooled = ctypes.c_size_t(99), ctypes.c_size_t(99)
    assert _lib.mi().mi_context_stats(ctypes.byref(created), ctypes.byref(pooled)) == 0
    assert created.value >= 0 and pooled.value <= created.value
    assert _lib.mi().mi_context_stats(None, None) == 0


def test_host_bucket_device_from_env_and_local_rank(monkeypatch):
    """CCL_COMP_HIP_DEVICE names the host buckets' GPU; without it the local
    rank (MPI_LOCALRANKID / LOCAL_RANK / CCL_LOCAL_RANK, as oneCCL's
    launchers set it) picks one of the visible GPUs, and with at most one
    visible GPU (none here) the calling thread's current device (-1)."""
    from oneccl_amd import comp
    shim = _lib.shim()
    for k in ("CCL_COMP_HIP_DEVICE", "MPI_LOCALRANKID", "LOCAL_RANK", "CCL_LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    try:
        monkeypatch.setenv("CCL_COMP_HIP_DEVICE", "3")
        comp.env_reload()
        assert shim.mi_ccl_comp_device() == 3
        monkeypatch.delenv("CCL_COMP_HIP_DEVICE")
        monkeypatch.setenv("LOCAL_RANK", "5")
        comp.env_reload()
        ndev = _lib.mi().mi_device_count()
        assert shim.mi_ccl_comp_device() == (5 % ndev if ndev > 1 else -1)
    finally:
        monkeypatch.undo()
        comp.env_reload()
