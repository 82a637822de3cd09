"""Pageable operands at every 16-byte misalignment through the paths that
hand host memory to the runtime's copies (mi_reduce.hip, h2d_stage /
d2h_pageable): the staged reduce (in place and out of place, 2 and 3
inputs, one chunk and several), the staged conversions and mi_copy_sync in
both directions.  Each operand ends at (or starts at) a PROT_NONE guard
page, so a copy that read or wrote past the operand's pages would fault on
the host; the runtime is given 16-byte-aligned host spans only, which never
leave those pages.  Bits against the oracle / numpy."""
from __future__ import annotations

import ctypes
import mmap

import numpy as np
import pytest

import oracle
from oneccl_amd import _lib, comp
from tests.util import BF16, FP32, assert_same, rand_array

pytestmark = pytest.mark.gpu

PAGE = mmap.PAGESIZE
_libc = ctypes.CDLL(None, use_errno=True)
_libc.mprotect.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]


class Guarded:
    """Anonymous pages with a PROT_NONE page before and after the data."""

    def __init__(self, nbytes):
        self.data_pages = (nbytes + PAGE - 1) // PAGE
        self.m = mmap.mmap(-1, (self.data_pages + 2) * PAGE, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS,
                           prot=mmap.PROT_READ | mmap.PROT_WRITE)
        self.base = ctypes.addressof(ctypes.c_char.from_buffer(self.m))
        for off in (0, (self.data_pages + 1) * PAGE):
            assert _libc.mprotect(self.base + off, PAGE, 0) == 0
        self.lo = self.base + PAGE
        self.hi = self.lo + self.data_pages * PAGE

    def array(self, n, dtype, at_end: bool, mis: int):
        """n elements touching the end guard (or the start guard), shifted by
        `mis` bytes from 16-byte alignment."""
        nbytes = n * np.dtype(dtype).itemsize
        addr = (self.hi - nbytes - mis) if at_end else (self.lo + mis)
        assert self.lo <= addr and addr + nbytes <= self.hi
        buf = (ctypes.c_char * nbytes).from_address(addr)
        return np.frombuffer(buf, dtype=dtype)

    def close(self):
        for off in (0, (self.data_pages + 1) * PAGE):
            _libc.mprotect(self.base + off, PAGE, mmap.PROT_READ | mmap.PROT_WRITE)


@pytest.mark.parametrize("dt", [FP32, BF16, 0])
@pytest.mark.parametrize("mis", [0, 2, 4, 10, 14])
@pytest.mark.parametrize("at_end", [True, False])
def test_staged_reduce_any_misalignment(dt, mis, at_end):
    es = np.dtype(oracle.NP_DTYPE[dt]).itemsize
    if mis % es:
        pytest.skip("operands are aligned to their element size")
    m = _lib.mi()
    flags = comp.reference_flags(comp.datatype(dt))  # the oracle's default impls: avx512bf / avx512f
    n = (3 << 20) // es + 5  # 3 MiB: past the bounce buffers, one staging chunk
    g_in, g_io, g_x = Guarded(n * es + 64), Guarded(n * es + 64), Guarded(n * es + 64)
    try:
        a = g_in.array(n, oracle.NP_DTYPE[dt], at_end, mis)
        b = g_io.array(n, oracle.NP_DTYPE[dt], not at_end, (mis + 6) % 16 // es * es)
        x = g_x.array(n, oracle.NP_DTYPE[dt], at_end, (16 - mis) % 16 // es * es)
        a[:] = rand_array(dt, n, seed=mis + 1, specials=False)
        b[:] = rand_array(dt, n, seed=mis + 2, specials=False)
        x[:] = rand_array(dt, n, seed=mis + 3, specials=False)
        # in place, two inputs
        exp = b.copy()
        oracle.comp_reduce(a.copy(), exp, dt, 3)
        _lib.check(m.mi_reduce_sync(a.ctypes.data, b.ctypes.data, n, dt, 3, flags, -1))
        assert_same(b, exp, dt)
        # three inputs out of place into x
        exp3 = oracle.fanin([b.copy(), a.copy(), b.copy()], dt, 0)
        arr = _lib.void_ptr_array([b.ctypes.data, a.ctypes.data, b.ctypes.data])
        _lib.check(m.mi_reduce_multi_sync(arr, 3, x.ctypes.data, n, dt, 0, flags, -1))
        assert_same(x, exp3, dt)
    finally:
        for g in (g_in, g_io, g_x):
            g.close()


def test_staged_reduce_several_chunks_misaligned():
    """Several 32 MiB chunks (the drain thread's D2H), output 2 bytes off."""
    m = _lib.mi()
    n = (72 << 20) // 2 + 3
    g_in, g_io = Guarded(n * 2 + 64), Guarded(n * 2 + 64)
    try:
        a = g_in.array(n, np.uint16, True, 6)
        b = g_io.array(n, np.uint16, True, 2)
        a[:] = rand_array(BF16, n, seed=5, specials=False)
        b[:] = rand_array(BF16, n, seed=6, specials=False)
        exp = b.copy()
        oracle.comp_reduce(a.copy(), exp, BF16, 0)
        _lib.check(m.mi_reduce_sync(a.ctypes.data, b.ctypes.data, n, BF16, 0, comp.reference_flags(comp.datatype.bfloat16), -1))
        assert_same(b, exp, BF16)
    finally:
        g_in.close()
        g_io.close()


@pytest.mark.parametrize("mis_s,mis_d", [(0, 2), (4, 6), (12, 14), (8, 0)])
def test_staged_convert_misaligned(mis_s, mis_d):
    m = _lib.mi()
    n = (9 << 20) // 4 + 7
    g_s, g_d, g_b = Guarded(n * 4 + 64), Guarded(n * 2 + 64), Guarded(n * 4 + 64)
    try:
        src = g_s.array(n, np.float32, True, mis_s)
        dst = g_d.array(n, np.uint16, True, mis_d)
        back = g_b.array(n, np.float32, False, (mis_s + 4) % 16)
        src[:] = rand_array(FP32, n, seed=9, specials=False)
        _lib.check(m.mi_convert_sync(src.ctypes.data, FP32, dst.ctypes.data, BF16, n, comp.F_BF16_RNE, -1))
        assert np.array_equal(dst, oracle.f32_to_bf16(src, True))
        _lib.check(m.mi_convert_sync(dst.ctypes.data, BF16, back.ctypes.data, FP32, n, 0, -1))
        assert np.array_equal(back.view(np.uint32), oracle.bf16_to_f32(dst).view(np.uint32))
    finally:
        for g in (g_s, g_d, g_b):
            g.close()


@pytest.mark.parametrize("mis", [0, 1, 3, 7, 15])
@pytest.mark.parametrize("nbytes", [5, 4096 + 13, (3 << 20) + 9])
def test_copy_sync_pageable_device_misaligned(mis, nbytes):
    import torch
    m = _lib.mi()
    g_h, g_back = Guarded(nbytes + 64), Guarded(nbytes + 64)
    try:
        h = g_h.array(nbytes, np.uint8, True, mis)
        back = g_back.array(nbytes, np.uint8, False, (mis * 5) % 16)
        h[:] = np.random.default_rng(mis + nbytes).integers(0, 256, nbytes, dtype=np.uint8)
        dev = torch.zeros(nbytes + 32, dtype=torch.uint8, device="cuda")
        dp = dev.data_ptr() + 3  # a device destination off alignment too
        _lib.check(m.mi_copy_sync(h.ctypes.data, dp, nbytes, 0, -1))
        got = dev.cpu().numpy()
        assert np.array_equal(got[3:3 + nbytes], h) and not got[:3].any() and not got[3 + nbytes:].any()
        _lib.check(m.mi_copy_sync(dp, back.ctypes.data, nbytes, 0, -1))
        assert np.array_equal(back, h)
    finally:
        g_h.close()
        g_back.close()
