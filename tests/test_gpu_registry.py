"""Declared host ranges on the GPU:
a registration is validated once -- device memory refused, pinned memory kept
pinned so the zero-copy kernel reads it in place -- and every classification
after it, the dispatcher's and the GPU path's (reduce_issue), answers from
the range without HIP's pointer lookup.  Bits against the oracle."""
from __future__ import annotations

import ctypes
import os

import numpy as np
import pytest

import oracle
from oneccl_amd import _lib, comp
from tests.util import BF16, FP32, assert_same, rand_array, wait_os_threads_gone

pytestmark = pytest.mark.gpu

MI_E_INVALID = -1


@pytest.fixture()
def gpu_dispatch():
    """The GPU paths for host buckets of any size (CCL_COMP_HOST_MAX_BYTES=0)."""
    saved = os.environ.get("CCL_COMP_HOST_MAX_BYTES")
    os.environ["CCL_COMP_HOST_MAX_BYTES"] = "0"
    comp.env_reload()
    yield
    if saved is None:
        os.environ.pop("CCL_COMP_HOST_MAX_BYTES", None)
    else:
        os.environ["CCL_COMP_HOST_MAX_BYTES"] = saved
    comp.env_reload()


def _impls():
    b, f = comp.impl_types()
    return int(b), int(f)


def test_device_memory_is_refused():
    import torch
    shim = _lib.shim()
    t = torch.zeros(1 << 16, dtype=torch.float32, device="cuda")
    assert shim.mi_ccl_comp_register_host_buffer(t.data_ptr(), t.numel() * 4) == MI_E_INVALID
    assert b"device" in _lib.mi().mi_last_error()
    assert _lib.mi().mi_host_declared_kind(t.data_ptr(), 64) == -1
    # a host range that runs into device memory is refused too (its last byte)
    assert shim.mi_ccl_comp_register_host_buffer(t.data_ptr() + 4096, 16) == MI_E_INVALID


@pytest.mark.parametrize("dt,n", [(FP32, 4099), (FP32, (40 << 20) // 4 + 33), (BF16, 300001)])
def test_pinned_registration_keeps_zero_copy(gpu_dispatch, dt, n):
    import torch
    shim, m = _lib.shim(), _lib.mi()
    b_impl, f_impl = _impls()
    a = rand_array(dt, n, seed=71, specials=False)
    b = rand_array(dt, n, seed=72, specials=False)
    exp = b.copy()
    oracle.comp_reduce_mt(a, exp, dt, 0, 8, b_impl, f_impl)
    ha = torch.from_numpy(a.view(np.uint8).copy()).pin_memory()
    hb = torch.from_numpy(b.view(np.uint8).copy()).pin_memory()
    pa, pb = ha.data_ptr(), hb.data_ptr()
    assert shim.mi_ccl_comp_register_host_buffer(pa, a.nbytes) == 0
    assert shim.mi_ccl_comp_register_host_buffer(pb, b.nbytes) == 0
    try:
        assert m.mi_host_declared_kind(pa, a.nbytes) == 1 and m.mi_host_declared_kind(pb, b.nbytes) == 1
        dev = ctypes.c_int(-1)
        assert m.mi_pointer_kind_range(pa + 64, 64, ctypes.byref(dev)) == 1
        n0 = shim.mi_ccl_comp_pointer_lookups()
        comp.comp_reduce(pa, n, pb, comp.datatype(dt), comp.reduction.sum)
        assert shim.mi_ccl_comp_pointer_lookups() == n0  # the shim's and the GPU path's classification
    finally:
        assert shim.mi_ccl_comp_unregister_host_buffer(pa) == 0
        assert shim.mi_ccl_comp_unregister_host_buffer(pb) == 0
    got = hb.numpy().view(a.dtype)
    assert_same(got, exp, dt)


@pytest.mark.parametrize("n", [4099, (40 << 20) // 4 + 33])
def test_registered_pageable_gpu_paths_make_no_lookup(gpu_dispatch, n):
    """Pageable operands inside registered buffers: bounce buffers (small),
    the staged pipeline (past one chunk); the lookup count covers
    libmi_reduce's classify() as well as the shim's."""
    shim = _lib.shim()
    b_impl, f_impl = _impls()
    a = rand_array(FP32, n, seed=81, specials=False)
    b = rand_array(FP32, n, seed=82, specials=False)
    exp = b.copy()
    oracle.comp_reduce_mt(a, exp, FP32, 0, 8, b_impl, f_impl)
    assert shim.mi_ccl_comp_register_host_buffer(a.ctypes.data, a.nbytes) == 0
    assert shim.mi_ccl_comp_register_host_buffer(b.ctypes.data, b.nbytes) == 0
    try:
        n0 = shim.mi_ccl_comp_pointer_lookups()
        comp.comp_reduce(a.ctypes.data, n, b.ctypes.data, comp.datatype(FP32), comp.reduction.sum)
        assert shim.mi_ccl_comp_pointer_lookups() == n0
    finally:
        assert shim.mi_ccl_comp_unregister_host_buffer(a.ctypes.data) == 0
        assert shim.mi_ccl_comp_unregister_host_buffer(b.ctypes.data) == 0
    assert_same(b, exp, FP32)


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_host_schedule_large_bucket_bits(mode):
    """Above the dispatcher's threshold a host schedule's bucket is split
    between the calling thread and the GPU as before (its kinds are looked up
    then: pinned vs pageable picks the GPU route); bits are the oracle's in
    every schedule mode."""
    shim = _lib.shim()
    b_impl, f_impl = _impls()
    n = (48 << 20) // 4 + 5
    a = rand_array(FP32, n, seed=90 + mode, specials=False)
    b = rand_array(FP32, n, seed=95 + mode, specials=False)
    exp = b.copy()
    oracle.comp_reduce_mt(a, exp, FP32, 0, 8, b_impl, f_impl)
    prev = shim.mi_ccl_comp_shim_sched(mode)
    try:
        comp.comp_reduce(a.ctypes.data, n, b.ctypes.data, comp.datatype(FP32), comp.reduction.sum)
    finally:
        shim.mi_ccl_comp_shim_sched(prev)
    assert_same(b, exp, FP32)


def test_device_operands_under_a_stream_schedule():
    """A schedule with a stream may hand device memory (the reference's SYCL
    branch, comp.cpp:144-195): the operands are looked up and reduced on the
    GPU in place."""
    import torch
    shim = _lib.shim()
    n = 1 << 20
    a = torch.rand(n, device="cuda")
    b = torch.rand(n, device="cuda")
    exp = (b + a).cpu()
    prev = shim.mi_ccl_comp_shim_sched(2)
    try:
        comp.comp_reduce(a.data_ptr(), n, b.data_ptr(), comp.datatype(FP32), comp.reduction.sum)
    finally:
        shim.mi_ccl_comp_shim_sched(prev)
    torch.cuda.synchronize()
    assert torch.equal(b.cpu().view(torch.int32), exp.view(torch.int32))


def test_host_schedule_concurrent_workers_mixed_sizes():
    """Eight workers under host schedules (as oneCCL's CPU-build entries call)
    reduce host buckets from 4 KiB to 24 MiB at once: the small ones on their
    own CPU with no lookup, the large ones split with the GPU; every result
    is the oracle's."""
    import threading
    b_impl, f_impl = _impls()
    sizes = [1024, 262144, (24 << 20) // 4 + 3]
    errors = []

    def worker(w):
        shim = _lib.shim()
        shim.mi_ccl_comp_shim_sched(1)
        try:
            for rep in range(2):
                for n in sizes:
                    a = rand_array(FP32, n, seed=1000 + 17 * w + n % 97 + rep, specials=False)
                    b = rand_array(FP32, n, seed=2000 + 31 * w + n % 89 + rep, specials=False)
                    exp = b.copy()
                    oracle.comp_reduce(a, exp, FP32, 0, b_impl, f_impl)
                    n0 = shim.mi_ccl_comp_pointer_lookups()
                    rc = shim.mi_ccl_comp_reduce(a.ctypes.data, n, b.ctypes.data, None, FP32, 0)
                    if rc != 0:
                        errors.append((w, n, "rc", shim.mi_ccl_last_error()))
                        continue
                    if n * 4 <= (16 << 20) and shim.mi_ccl_comp_pointer_lookups() != n0:
                        errors.append((w, n, "lookup"))
                    if not np.array_equal(b.view(np.uint32), exp.view(np.uint32)):
                        errors.append((w, n, "bits"))
        finally:
            shim.mi_ccl_comp_shim_sched(0)

    ts = [threading.Thread(target=worker, args=(w,)) for w in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert wait_os_threads_gone([t.native_id for t in ts])
    assert errors == []


PAGE = 4096


def _page_aligned(nbytes):
    raw = np.zeros(nbytes + PAGE, np.uint8)
    off = (-raw.ctypes.data) % PAGE
    return raw, raw[off:off + nbytes]


def test_pinned_ends_with_a_pageable_middle_are_not_zero_copy(gpu_dispatch):
    """a range whose first and last pages are pinned (two
    separate registrations) but whose middle is pageable must not be recorded
    as pinned -- the zero-copy kernel would read unmapped pages.  It is either
    refused (the ends' mappings differ) or recorded pageable and staged; a
    reduce over it then gives the oracle's bits."""
    m = _lib.mi()
    raw, buf = _page_aligned(8 * PAGE)
    p = buf.ctypes.data
    assert m.mi_host_register(p, PAGE) == 0
    assert m.mi_host_register(p + 7 * PAGE, PAGE) == 0
    try:
        rc = m.mi_host_declare(p, 8 * PAGE)
        if rc == 0:
            try:
                assert m.mi_host_declared_kind(p, 8 * PAGE) == 2
                n = 8 * PAGE // 8  # two fp32 operands of 4 pages each, both in the range
                a = buf[:4 * PAGE].view(np.float32)
                b = buf[4 * PAGE:].view(np.float32)
                a[:] = rand_array(FP32, n, seed=5, specials=False)
                b[:] = rand_array(FP32, n, seed=6, specials=False)
                exp = b.copy()
                oracle.comp_reduce(a.copy(), exp, FP32, 0, *_impls())
                comp.comp_reduce(a.ctypes.data, n, b.ctypes.data, comp.datatype(FP32), comp.reduction.sum)
                assert_same(b, exp, FP32)
            finally:
                assert m.mi_host_undeclare(p) == 0
        else:
            assert rc == MI_E_INVALID and b"mappings" in m.mi_last_error()
        # a declaration inside one registration stays pinned (zero-copy)
        assert m.mi_host_declare(p + 7 * PAGE, PAGE) == 0
        assert m.mi_host_declared_kind(p + 7 * PAGE, PAGE) == 1
        assert m.mi_host_undeclare(p + 7 * PAGE) == 0
    finally:
        assert m.mi_host_unregister(p) == 0
        assert m.mi_host_unregister(p + 7 * PAGE) == 0
    del raw


@pytest.mark.parametrize("n", [4099, (40 << 20) // 4 + 33])
def test_unregistering_a_declared_pinned_buffer_demotes_it(gpu_dispatch, n):
    """mi_host_unregister turns the declared ranges over
    the buffer pageable before unpinning it, so a later reduce on the (still
    valid, now pageable) memory is staged instead of read in place."""
    m = _lib.mi()
    raw_a, a8 = _page_aligned(n * 4)
    raw_b, b8 = _page_aligned(n * 4)
    a, b = a8.view(np.float32), b8.view(np.float32)
    a[:] = rand_array(FP32, n, seed=11, specials=False)
    b[:] = rand_array(FP32, n, seed=12, specials=False)
    exp = b.copy()
    oracle.comp_reduce_mt(a.copy(), exp, FP32, 0, 8, *_impls())
    for x in (a, b):
        assert m.mi_host_register(x.ctypes.data, x.nbytes) == 0
        assert m.mi_host_declare(x.ctypes.data, x.nbytes) == 0
        assert m.mi_host_declared_kind(x.ctypes.data, x.nbytes) == 1
    for x in (a, b):
        assert m.mi_host_unregister(x.ctypes.data) == 0
        assert m.mi_host_declared_kind(x.ctypes.data, x.nbytes) == 2
    try:
        comp.comp_reduce(a.ctypes.data, n, b.ctypes.data, comp.datatype(FP32), comp.reduction.sum)
    finally:
        for x in (a, b):
            assert m.mi_host_undeclare(x.ctypes.data) == 0
    assert_same(b, exp, FP32)
    del raw_a, raw_b


def test_operand_running_past_a_pinned_allocation_is_staged():
    """HIP classifies a pointer by its first byte.  An operand that starts in
    a pinned (registered) allocation and runs on into pageable pages must not
    go to the zero-copy kernel, which would read the pageable pages in place
    and fault the GPU: classify() checks the pinned allocation's extent and
    stages such an operand.  The kinds are asserted before any GPU call."""
    m = _lib.mi()
    raw, buf = _page_aligned(8 * PAGE)
    p = buf.ctypes.data
    assert m.mi_host_register(p, 4 * PAGE) == 0
    try:
        dev = ctypes.c_int(-1)
        assert m.mi_pointer_kind_range(p, 4 * PAGE, ctypes.byref(dev)) == 1  # inside the registration
        assert m.mi_pointer_kind_range(p + 64, 4 * PAGE - 64, ctypes.byref(dev)) == 1
        assert m.mi_pointer_kind_range(p, 4 * PAGE + 4, ctypes.byref(dev)) == 2  # one element past it
        assert m.mi_pointer_kind_range(p, 8 * PAGE, ctypes.byref(dev)) == 2
        n = 8 * PAGE // 4
        a = buf.view(np.float32)
        a[:] = rand_array(FP32, n, seed=21, specials=False)
        b = rand_array(FP32, n, seed=22, specials=False)
        exp = b.copy()
        oracle.comp_reduce(a.copy(), exp, FP32, 0, *_impls())
        _lib.check(m.mi_reduce_sync(a.ctypes.data, b.ctypes.data, n, FP32, 0, 0, -1))
        assert_same(b, exp, FP32)
        # and as the accumulator
        c = rand_array(FP32, n, seed=23, specials=False)
        exp2 = a.copy()
        oracle.comp_reduce(c, exp2, FP32, 0, *_impls())
        _lib.check(m.mi_reduce_sync(c.ctypes.data, a.ctypes.data, n, FP32, 0, 0, -1))
        assert_same(a, exp2, FP32)
    finally:
        assert m.mi_host_unregister(p) == 0
    del raw
