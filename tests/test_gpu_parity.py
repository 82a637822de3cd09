"""GPU parity: the HIP kernels (through the C ABI, include/mi_reduce.h) against
the CPU oracle (oracle/, a restatement of oneCCL src/comp) on the same seeded
inputs.  Bar: bit-exact for every dtype and op (floating point: NaN payloads
excepted — two NaNs compare equal — because x86 and CDNA produce different
default NaNs; NaN-ness itself must match).
"""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

import oracle
from oneccl_amd import _lib
from oneccl_amd.comp import F_ACC_FP32, F_BF16_RNE, F_BF16_TAIL_TRUNC16, F_MINMAX_INOUT_FIRST, bf16_flags
from tests.util import (ALL_DTYPES, BF16, DT_NAME, FP16, FP32, FP64, INT_DTYPES, OP_NAME, OPS, assert_same,
                        from_dev, rand_array, to_dev)

pytestmark = pytest.mark.gpu

# reference semantics per dtype: (label, kernel flags, oracle bf16 impl, oracle fp16 impl)
VARIANTS = {dt: [("ref", 0, oracle.BF16_AVX512BF, oracle.FP16_AVX512F)] for dt in INT_DTYPES + [FP32, FP64]}
VARIANTS[BF16] = [("scalar", bf16_flags(0), oracle.BF16_SCALAR, 0),
                  ("avx512f", bf16_flags(1), oracle.BF16_AVX512F, 0),
                  ("avx512bf", bf16_flags(2), oracle.BF16_AVX512BF, 0)]
VARIANTS[FP16] = [("avx512f", F_MINMAX_INOUT_FIRST, 0, oracle.FP16_AVX512F)]

CASES = [(dt, op, v) for dt in ALL_DTYPES for op in OPS for v in VARIANTS[dt]]
# element counts of the reference's functional tests (tests/functional/conf.cpp:51-53) + edges
SIZES = [1, 17, 32771, 262144]


def _sync():
    import torch
    torch.cuda.synchronize()


def _stream():
    import torch
    return torch.cuda.current_stream().cuda_stream


def gpu_reduce(a, b, dt, op, flags, off_in=0, off_io=0):
    ta, pa = to_dev(a, offset_elems=off_in)
    tb, pb = to_dev(b, offset_elems=off_io)
    _lib.check(_lib.mi().mi_reduce(pa, pb, a.size, dt, op, flags, _stream()))
    _sync()
    return from_dev(tb, b, off_io)


@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("dt,op,var", CASES, ids=[f"{DT_NAME[d]}-{OP_NAME[o]}-{v[0]}" for d, o, v in CASES])
def test_reduce_inplace_vs_oracle(dt, op, var, n):
    _, flags, bimpl, fimpl = var
    a = rand_array(dt, n, seed=1000 + 17 * dt + op, op=op)
    b = rand_array(dt, n, seed=2000 + 17 * dt + op, op=op)
    exp = b.copy()
    oracle.comp_reduce(a, exp, dt, op, bimpl, fimpl)
    got = gpu_reduce(a, b, dt, op, flags)
    assert_same(got, exp, dt, f"{DT_NAME[dt]} {OP_NAME[op]} n={n}")


@pytest.mark.parametrize("dt", [FP32, BF16, 0, FP64, FP16])
@pytest.mark.parametrize("off_in,off_io", [(1, 1), (3, 3), (1, 0), (0, 2), (5, 7)])
def test_misaligned_pointers(dt, off_in, off_io):
    """Sub-buffer pointers (ring chunks at arbitrary element offsets): common
    misalignment -> scalar head + vector body; different -> element loop."""
    n = 4099
    op = 0
    var = VARIANTS[dt][-1]
    a = rand_array(dt, n, seed=31 + dt)
    b = rand_array(dt, n, seed=37 + dt)
    exp = b.copy()
    oracle.comp_reduce(a, exp, dt, op, var[2], var[3])
    got = gpu_reduce(a, b, dt, op, var[1], off_in, off_io)
    assert_same(got, exp, dt, f"offsets {off_in},{off_io}")


UNALIGNED = [(dt, op) for dt in ALL_DTYPES for op in OPS]


@pytest.fixture
def unaligned_mode():
    """Restore the library's handling of differing misalignments after a test."""
    m = _lib.mi()
    prev = m.mi_set_unaligned_vectors(1)
    yield m
    m.mi_set_unaligned_vectors(prev)


@pytest.mark.parametrize("dt,op", UNALIGNED, ids=[f"{DT_NAME[d]}-{OP_NAME[o]}" for d, o in UNALIGNED])
@pytest.mark.parametrize("vectors", [1, 0], ids=["unaligned-vectors", "element-loop"])
def test_differing_misalignment_2input(dt, op, vectors, unaligned_mode):
    """Ring chunks whose addresses differ mod 16 (element offsets that are not
    multiples of 16 / size): the vector kernels reading unaligned 16-byte
    vectors, and the element loop, both bit-exact to the oracle.  Several
    tiles, partial last tile, scalar head and tail."""
    es = oracle.NP_DTYPE[dt]().itemsize
    n = 3 * 16384 + 16 * 7 + 5
    var = VARIANTS[dt][-1]
    a = rand_array(dt, n, seed=900 + dt + 13 * op, op=op)
    b = rand_array(dt, n, seed=950 + dt + 13 * op, op=op)
    exp = b.copy()
    oracle.comp_reduce(a, exp, dt, op, var[2], var[3])
    unaligned_mode.mi_set_unaligned_vectors(vectors)
    off_in, off_io = (1, 0) if es >= 8 else (16 // es - 1, 1)  # differ mod 16 bytes
    got = gpu_reduce(a, b, dt, op, var[1], off_in, off_io)
    assert_same(got, exp, dt, f"offsets {off_in},{off_io}")


FAN_UNALIGNED = [(FP32, 0, 5), (BF16, 0, 8), (0, 3, 4), (FP16, 2, 3), (FP64, 1, 6), (3, 0, 16), (6, 0, 9)]


@pytest.mark.parametrize("dt,op,k", FAN_UNALIGNED, ids=[f"{DT_NAME[d]}-{OP_NAME[o]}-k{k}" for d, o, k in FAN_UNALIGNED])
@pytest.mark.parametrize("inplace", [False, True], ids=["out", "inplace"])
def test_differing_misalignment_fanin(dt, op, k, inplace, unaligned_mode):
    """K-input fan-in with a different element offset per input (and for the
    output), through the buffer-addressed fan kernel on unaligned bases."""
    n = 2 * 16384 + 16 * 3 + 9
    var = VARIANTS[dt][-1]
    ins = [rand_array(dt, n, seed=1200 + 31 * j + dt, op=op) for j in range(k)]
    exp = oracle.fanin(ins, dt, op, var[2], var[3])
    holders = [to_dev(x, pad_elems=16, offset_elems=(j * 3 + 1) % 7) for j, x in enumerate(ins)]
    if inplace:
        to, po, off_o = holders[0][0], holders[0][1], 1
    else:
        off_o = 2
        to, po = to_dev(np.zeros_like(ins[0]), pad_elems=16, offset_elems=off_o)
    arr = _lib.void_ptr_array([p for _, p in holders])
    _lib.check(_lib.mi().mi_reduce_multi(arr, k, po, n, dt, op, var[1], _stream()))
    _sync()
    assert_same(from_dev(to, ins[0], off_o), exp, dt)


@pytest.mark.parametrize("dt,op", [(FP32, 0), (FP32, 3), (BF16, 0), (4, 1), (FP16, 2)])
def test_reduce_out_of_place(dt, op):
    n = 32771
    var = VARIANTS[dt][-1]
    a = rand_array(dt, n, seed=5, op=op)
    b = rand_array(dt, n, seed=6, op=op)
    exp = b.copy()
    oracle.comp_reduce(a, exp, dt, op, var[2], var[3])
    ta, pa = to_dev(a)
    tb, pb = to_dev(b)
    to, po = to_dev(np.zeros_like(b))
    _lib.check(_lib.mi().mi_reduce_out(pa, pb, po, n, dt, op, var[1], _stream()))
    _sync()
    assert_same(from_dev(to, b), exp, dt)
    assert_same(from_dev(tb, b), b, dt, "in2 must be untouched")


FANIN = [(FP32, 0, 3), (FP32, 0, 8), (FP32, 3, 16), (FP64, 1, 5), (4, 1, 8), (0, 0, 16), (7, 2, 4),
         (BF16, 0, 8), (BF16, 2, 5), (FP16, 0, 8), (FP16, 3, 16)]


@pytest.mark.parametrize("dt,op,k", FANIN, ids=[f"{DT_NAME[d]}-{OP_NAME[o]}-k{k}" for d, o, k in FANIN])
@pytest.mark.parametrize("n", [17, 262144 + 5])
def test_fanin_storage_precision(dt, op, k, n):
    """K-input fan-in == K-1 chained ccl_comp_reduce calls (the ring-chunk
    arrival pattern; ccl_comp_batch_reduce non-keep mode, comp.cpp:236-245)."""
    for var in VARIANTS[dt]:
        ins = [rand_array(dt, n, seed=100 * j + dt, op=op) for j in range(k)]
        exp = oracle.fanin(ins, dt, op, var[2], var[3])
        holders = [to_dev(x) for x in ins]
        to, po = to_dev(np.zeros_like(ins[0]))
        arr = _lib.void_ptr_array([p for _, p in holders])
        _lib.check(_lib.mi().mi_reduce_multi(arr, k, po, n, dt, op, var[1], _stream()))
        _sync()
        assert_same(from_dev(to, ins[0]), exp, dt, f"variant {var[0]}")


@pytest.mark.parametrize("dt", [BF16, FP16])
@pytest.mark.parametrize("op", OPS)
@pytest.mark.parametrize("k", [2, 3, 8, 16])
@pytest.mark.parametrize("rne,inout_first", [(True, False), (False, False), (True, True)])
def test_fanin_fp32_accumulate(dt, op, k, rne, inout_first):
    """bf16/fp16 fan-in with fp32 accumulation and one rounding at the end."""
    if dt == FP16 and not rne:
        pytest.skip("fp16 always rounds RNE")
    n = 20011
    ins = [rand_array(dt, n, seed=7 * j + op, op=op) for j in range(k)]
    exp = oracle.lp_fanin_acc_fp32(ins, dt, op, rne, inout_first)
    holders = [to_dev(x) for x in ins]
    to, po = to_dev(np.zeros_like(ins[0]))
    flags = F_ACC_FP32 | (F_BF16_RNE if rne else 0) | (F_MINMAX_INOUT_FIRST if inout_first else 0)
    arr = _lib.void_ptr_array([p for _, p in holders])
    _lib.check(_lib.mi().mi_reduce_multi(arr, k, po, n, dt, op, flags, _stream()))
    _sync()
    assert_same(from_dev(to, ins[0]), exp, dt)


@pytest.mark.parametrize("bimpl", [oracle.BF16_SCALAR, oracle.BF16_AVX512F, oracle.BF16_AVX512BF])
@pytest.mark.parametrize("k", [1, 2, 4, 9])
@pytest.mark.parametrize("n", [15, 16, 4099])
def test_batch_reduce_keep_precision(bimpl, k, n):
    """ccl_comp_batch_reduce(bf16_keep_precision_mode=1), comp.cpp:214-234,
    including the truncated count%16 tail of the final array conversion."""
    op = 0
    ins = [rand_array(BF16, n, seed=900 + j) for j in range(k)]
    packed = np.concatenate(ins)
    offsets = [j * n for j in range(k)]
    exp = ins[0].copy()
    oracle.batch_reduce(packed, offsets, n, exp, BF16, op, 1, bimpl, 0)
    flags = F_ACC_FP32 | ((F_BF16_RNE | F_BF16_TAIL_TRUNC16) if bimpl == oracle.BF16_AVX512BF else 0)
    holders = [to_dev(x) for x in ins]
    arr = _lib.void_ptr_array([p for _, p in holders])
    _lib.check(_lib.mi().mi_reduce_multi(arr, k, holders[0][1], n, BF16, op, flags, _stream()))
    _sync()
    assert_same(from_dev(holders[0][0], ins[0]), exp, BF16)


def test_pageable_pointer_refused_without_fault():
    """Device entry points refuse pageable host memory instead of launching a
    kernel that would fault; pinned host memory is accepted (zero-copy)."""
    import torch
    m = _lib.mi()
    a = np.ones(4096, np.float32)
    b = np.ones(4096, np.float32)
    assert m.mi_reduce(a.ctypes.data, b.ctypes.data, a.size, FP32, 0, 0, _stream()) == -1
    assert b"pageable" in m.mi_last_error()
    ha = torch.ones(4096, dtype=torch.float32).pin_memory()
    hb = torch.ones(4096, dtype=torch.float32).pin_memory()
    _lib.check(m.mi_reduce(ha.data_ptr(), hb.data_ptr(), 4096, FP32, 0, 0, _stream()))
    _sync()
    assert bool((hb == 2).all())


def test_zero_count_and_errors():
    m = _lib.mi()
    assert m.mi_reduce(0, 0, 0, FP32, 0, 0, _stream()) == 0
    assert m.mi_reduce(0, 0, 10, 99, 0, 0, _stream()) < 0
    assert m.mi_reduce(0, 0, 10, FP32, 4, 0, _stream()) < 0
    assert b"reduction" in m.mi_last_error()


def test_shards_compose():
    """Element-range sharding: reducing each shard separately
    gives the whole-array result bit for bit."""
    n = 1_000_003
    a = rand_array(FP32, n, seed=1)
    b = rand_array(FP32, n, seed=2)
    exp = b.copy()
    oracle.comp_reduce(a, exp, FP32, 0)
    ta, pa = to_dev(a)
    tb, pb = to_dev(b)
    m = _lib.mi()
    for world in (1, 2, 4, 8):
        tb.copy_(to_dev(b)[0])
        for r in range(world):
            lo, hi = ctypes.c_size_t(), ctypes.c_size_t()
            _lib.check(m.mi_shard_range(n, r, world, 256, ctypes.byref(lo), ctypes.byref(hi)))
            _lib.check(m.mi_reduce(pa + 4 * lo.value, pb + 4 * lo.value, hi.value - lo.value, FP32, 0, 0, _stream()))
        _sync()
        assert_same(from_dev(tb, b), exp, FP32, f"world={world}")


# ---- BASELINE.json full-size configurations --------------------------------

def test_full_c2_fp32_sum_1gib():
    """C2: 2-input fp32 sum, 1 GiB device-resident — bit-exact vs the oracle."""
    n = (1 << 30) // 4
    a = rand_array(FP32, n, seed=0xC0FFEE, specials=False)
    b = rand_array(FP32, n, seed=0xBEEF, specials=False)
    exp = b.copy()
    oracle.comp_reduce_mt(a, exp, FP32, 0, 8)
    got = gpu_reduce(a, b, FP32, 0, 0)
    assert_same(got, exp, FP32, "C2")


@pytest.mark.parametrize("dt", [BF16, FP16])
def test_full_c3_lp_sum_256mib(dt):
    """C3: fp16 / bf16 sum with fp32 accumulate, 256 MiB — bit-exact (2-input:
    one rounding of the fp32 sum, as the reference's avx512bf / avx512f)."""
    n = (256 << 20) // 2
    a = rand_array(dt, n, seed=0x1234, specials=False)
    b = rand_array(dt, n, seed=0x4321, specials=False)
    exp = b.copy()
    bimpl, fimpl = (oracle.BF16_AVX512BF, 0) if dt == BF16 else (0, oracle.FP16_AVX512F)
    oracle.comp_reduce_mt(a, exp, dt, 0, 8, bimpl, fimpl)
    flags = bf16_flags(2) if dt == BF16 else F_MINMAX_INOUT_FIRST
    got = gpu_reduce(a, b, dt, 0, flags)
    assert_same(got, exp, dt, "C3")


def test_full_c4_fanin8_fp32_1gib():
    """C4: 8-input fp32 sum fan-in over 1 GiB buffers == 7 chained reduces."""
    n = (1 << 30) // 4
    ins = [rand_array(FP32, n, seed=0xA0 + j, specials=False) for j in range(8)]
    exp = ins[0].copy()
    for x in ins[1:]:
        oracle.comp_reduce_mt(x, exp, FP32, 0, 8)
    holders = [to_dev(x) for x in ins]
    del ins[1:]
    to, po = to_dev(np.zeros(1, np.float32), pad_elems=n - 1)
    arr = _lib.void_ptr_array([p for _, p in holders])
    _lib.check(_lib.mi().mi_reduce_multi(arr, 8, po, n, FP32, 0, 0, _stream()))
    _sync()
    got = to.cpu().numpy().view(np.float32)
    assert_same(got, exp, FP32, "C4")


@pytest.mark.parametrize("dt,n", [(0, (1 << 32) + 4099), (BF16, (1 << 31) + 77)],
                         ids=["int8-2^32+", "bf16-2^31+"])
def test_counts_beyond_32_bit_indices(dt, n):
    """Element counts past 2^31 / 2^32 (288 GB HBM makes them practical).  The
    reference's bf16/fp16 loops index with `int` and break above 2^31
    (bf16_intrisics.hpp:108); the kernels index with 64 bits."""
    import torch
    rng = np.random.default_rng(9)
    st = oracle.NP_DTYPE[dt]
    if dt == BF16:
        a = oracle.f32_to_bf16(rng.standard_normal(n, dtype=np.float32), True)
        b = oracle.f32_to_bf16(rng.standard_normal(n, dtype=np.float32), True)
    else:
        a = rng.integers(-128, 128, n, dtype=st)
        b = rng.integers(-128, 128, n, dtype=st)
    exp = b.copy()
    oracle.comp_reduce_mt(a, exp, dt, 0, 16, oracle.BF16_AVX512BF)
    flags = bf16_flags(2) if dt == BF16 else 0
    ta = torch.from_numpy(a.view(np.int8 if dt == 0 else np.int16)).cuda()
    del a
    tb = torch.from_numpy(b.view(np.int8 if dt == 0 else np.int16)).cuda()
    del b
    _lib.check(_lib.mi().mi_reduce(ta.data_ptr(), tb.data_ptr(), n, dt, 0, flags, _stream()))
    _sync()
    got = tb.cpu().numpy().view(st)
    assert_same(got, exp, dt, f"n={n}")


PACKED = [(dt, op, k) for dt in (0, 1, 2, 3) for op in OPS for k in (3, 8, 16)]


@pytest.mark.parametrize("dt,op,k", PACKED, ids=[f"{DT_NAME[d]}-{OP_NAME[o]}-k{k}" for d, o, k in PACKED])
def test_fanin_packed_small_ints(dt, op, k):
    """8- and 16-bit integer fan-in folds packed on dwords (pk_op4): every
    op, signed and unsigned extremes, wrap-around sum and prod, a partial
    last tile and a scalar tail."""
    n = 3 * 16384 + 16 * 5 + 7
    ins = [rand_array(dt, n, seed=700 + 31 * j + dt, op=op) for j in range(k)]
    exp = oracle.fanin(ins, dt, op)
    holders = [to_dev(x) for x in ins]
    to, po = to_dev(np.zeros_like(ins[0]))
    arr = _lib.void_ptr_array([p for _, p in holders])
    _lib.check(_lib.mi().mi_reduce_multi(arr, k, po, n, dt, op, 0, _stream()))
    _sync()
    assert_same(from_dev(to, ins[0]), exp, dt)


# ---- kernel-form coverage ---------------------------------------------------

FAN_OFFS = [(FP32, 0, 5, 3), (BF16, 0, 5, 1), (0, 0, 7, 9), (FP64, 3, 3, 1), (FP16, 1, 4, 5), (6, 2, 16, 1)]


@pytest.mark.parametrize("dt,op,k,off", FAN_OFFS, ids=[f"{DT_NAME[d]}-{OP_NAME[o]}-k{k}-off{s}"
                                                      for d, o, k, s in FAN_OFFS])
@pytest.mark.parametrize("inplace", [False, True], ids=["out", "inplace"])
def test_fanin_common_misalignment(dt, op, k, off, inplace):
    """Fan-in on sub-buffers that share one misalignment (the fan kernel's
    scalar head + tiled body + partial last tile + scalar tail), written out
    of place or into input 0 as ccl_comp_batch_reduce does (comp.cpp:236-245)."""
    n = 3 * 1024 * (16 // oracle.NP_DTYPE[dt]().itemsize) + 29
    var = VARIANTS[dt][-1]
    ins = [rand_array(dt, n, seed=300 + 11 * j + dt, op=op) for j in range(k)]
    exp = oracle.fanin(ins, dt, op, var[2], var[3])
    holders = [to_dev(x, offset_elems=off) for x in ins]
    if inplace:
        to, po = holders[0]
    else:
        to, po = to_dev(np.zeros_like(ins[0]), offset_elems=off)
    arr = _lib.void_ptr_array([p for _, p in holders])
    _lib.check(_lib.mi().mi_reduce_multi(arr, k, po, n, dt, op, var[1], _stream()))
    _sync()
    assert_same(from_dev(to, ins[0], off), exp, dt)


@pytest.mark.parametrize("dt,op,k", [(FP32, 0, 2), (FP32, 3, 6), (BF16, 0, 2), (BF16, 0, 4), (0, 1, 3),
                                     (FP16, 2, 16), (7, 0, 2)])
def test_grid_stride_general_kernel(dt, op, k):
    """A grid cap (mi_set_max_blocks / MI_REDUCE_MAX_BLOCKS) routes every call
    through the grid-stride general kernel: same results."""
    m = _lib.mi()
    n = 200_003
    var = VARIANTS[dt][-1]
    ins = [rand_array(dt, n, seed=500 + 13 * j + dt, op=op) for j in range(k)]
    exp = oracle.fanin(ins, dt, op, var[2], var[3])
    holders = [to_dev(x) for x in ins]
    to, po = to_dev(np.zeros_like(ins[0]))
    arr = _lib.void_ptr_array([p for _, p in holders])
    _lib.check(m.mi_set_max_blocks(7))
    try:
        _lib.check(m.mi_reduce_multi(arr, k, po, n, dt, op, var[1], _stream()))
        _sync()
    finally:
        _lib.check(m.mi_set_max_blocks(0))
    assert_same(from_dev(to, ins[0]), exp, dt)


def test_fanin_beyond_32_bit_indices():
    """3-input int8 fan-in past 2^32 elements: 64-lane fan tiles of 16-byte
    vectors (1 KiB = 2^10 elements per block, folded packed on dwords), so
    2^22 + 1 blocks."""
    import torch
    n = (1 << 32) + 4099
    rng = np.random.default_rng(11)
    ins = [rng.integers(-128, 128, n, dtype=np.int8) for _ in range(3)]
    exp = ins[0].copy()
    for x in ins[1:]:
        oracle.comp_reduce_mt(x, exp, 0, 0, 16)
    ts = []
    for j in range(3):
        ts.append(torch.from_numpy(ins[j]).cuda())
    del ins
    arr = _lib.void_ptr_array([t.data_ptr() for t in ts])
    _lib.check(_lib.mi().mi_reduce_multi(arr, 3, ts[0].data_ptr(), n, 0, 0, 0, _stream()))
    _sync()
    got = ts[0].cpu().numpy()
    assert_same(got, exp, 0, f"n={n}")


@pytest.mark.gpu
def test_residency_caps_fit_the_device():
    """On the GPU the caps are real: each one-wave workgroup reserves whole
    LDS granules (1/128 of the CU's LDS, 1280 B on MI355X's 160 KiB), so
    exactly `waves` of them fit on a CU by the allocation rule measured with
    tools/residency_probe.hip (floor(128 / granules))."""
    import ctypes
    m = _lib.mi()
    w, lds = ctypes.c_int(), ctypes.c_uint()
    for k in (0, 2, 3, 8, 16):
        assert m.mi_get_residency(0, k, ctypes.byref(w), ctypes.byref(lds)) == 0
        assert lds.value > 0, "the device reported no LDS size: kernels run uncapped"
        per_cu = 160 * 1024
        g = per_cu // 128
        assert lds.value % g == 0, (k, lds.value)
        assert 128 // (lds.value // g) == w.value, (k, w.value, lds.value)
        assert w.value in (21, 16, 11, 9, 8, 5), (k, w.value)


@pytest.mark.gpu
def test_wave_cap_off_same_bits():
    """MI_REDUCE_WAVE_CAP=0 (read once per process, so in a child): no LDS is
    reserved, and the 2-input and fan-in kernels give the same bits."""
    import os
    import subprocess
    import sys
    code = r'''
import ctypes, numpy as np, torch
from oneccl_amd import _lib
import oracle
m = _lib.mi()
w, lds = ctypes.c_int(), ctypes.c_uint()
assert m.mi_get_residency(0, 8, ctypes.byref(w), ctypes.byref(lds)) == 0 and lds.value == 0, lds.value
rng = np.random.default_rng(5)
n = (1 << 22) + 37
xs = [rng.standard_normal(n).astype(np.float32) for _ in range(8)]
exp2 = xs[0].copy(); oracle.comp_reduce_mt(xs[1], exp2, 9, 0, 8)
exp8 = xs[0].copy()
for x in xs[1:]: oracle.comp_reduce_mt(x, exp8, 9, 0, 8)
ts = [torch.from_numpy(x).cuda() for x in xs]
s = torch.cuda.current_stream().cuda_stream
a = ts[0].clone()
_lib.check(m.mi_reduce(ts[1].data_ptr(), a.data_ptr(), n, 9, 0, 0, s))
arr = _lib.void_ptr_array([t.data_ptr() for t in ts])
_lib.check(m.mi_reduce_multi(arr, 8, ts[0].data_ptr(), n, 9, 0, 0, s))
torch.cuda.synchronize()
assert a.cpu().numpy().view(np.uint32).tolist() == exp2.view(np.uint32).tolist()
assert ts[0].cpu().numpy().view(np.uint32).tolist() == exp8.view(np.uint32).tolist()
print("ok")
'''
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MI_REDUCE_WAVE_CAP="0", PYTHONPATH=root)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300, cwd=root)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout + r.stderr


@pytest.mark.parametrize("k,waves", [(2, 16), (2, 32), (2, 1), (8, 8), (8, 32), (0, 25)])
def test_residency_override_same_bits(k, waves):
    """mi_set_residency (tuning knob, tools/residency_ab.py) changes only the
    LDS each one-wave workgroup reserves: the 2-input kernel, the fan-in and
    the conversions give the oracle's bits at other residencies, and 0 puts
    the plan back."""
    m = _lib.mi()
    w, lds = ctypes.c_int(), ctypes.c_uint()
    _lib.check(m.mi_get_residency(0, k, ctypes.byref(w), None))
    plan = w.value
    n = 262144 + 5
    try:
        _lib.check(m.mi_set_residency(k, waves))
        assert m.mi_get_residency(0, k, ctypes.byref(w), ctypes.byref(lds)) == 0 and w.value == waves
        assert lds.value > 0
        if k == 0:  # fp32 -> bf16 (RNE) conversion
            a = rand_array(FP32, n, seed=77)
            exp = oracle.f32_to_bf16(a, rne=True)
            ta, pa = to_dev(a)
            to, po = to_dev(np.zeros(n, dtype=np.uint16))
            _lib.check(m.mi_convert(pa, FP32, po, BF16, n, F_BF16_RNE, _stream()))
            _sync()
            assert np.array_equal(from_dev(to, exp), exp)
        elif k == 2:
            a, b = rand_array(FP32, n, seed=78), rand_array(FP32, n, seed=79)
            exp = b.copy()
            oracle.comp_reduce(a, exp, FP32, 0, oracle.BF16_AVX512BF, oracle.FP16_AVX512F)
            assert_same(gpu_reduce(a, b, FP32, 0, 0), exp, FP32, f"k=2 at {waves} waves")
        else:
            ins = [rand_array(FP32, n, seed=80 + j) for j in range(k)]
            exp = oracle.fanin(ins, FP32, 0, oracle.BF16_AVX512BF, oracle.FP16_AVX512F)
            holders = [to_dev(x) for x in ins]
            to, po = to_dev(np.zeros_like(ins[0]))
            arr = _lib.void_ptr_array([p for _, p in holders])
            _lib.check(m.mi_reduce_multi(arr, k, po, n, FP32, 0, 0, _stream()))
            _sync()
            assert_same(from_dev(to, ins[0]), exp, FP32, f"k={k} at {waves} waves")
    finally:
        _lib.check(m.mi_set_residency(k, 0))
    assert m.mi_get_residency(0, k, ctypes.byref(w), None) == 0 and w.value == plan
