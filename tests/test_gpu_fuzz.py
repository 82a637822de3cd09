"""Seeded random sweep of the whole device surface against the oracle: dtype,
op, semantic variant, input count 1..16, element count (empty, tiny, within
one tile, across tiles), a different element offset per operand (common and
differing misalignments), in place or out of place.  Each case is checked
bit-exactly (bf16/fp16 NaN payloads included) against the oracle's chained
ccl_comp_reduce fold, or its fp32-accumulate fan-in when that variant is set.
The case list is fixed by the seed, so a failure names a reproducible case.
"""
from __future__ import annotations

import os

import numpy as np
import pytest

import oracle
from oneccl_amd import _lib
from oneccl_amd.comp import F_ACC_FP32, F_BF16_RNE, F_MINMAX_INOUT_FIRST, bf16_flags
from tests.util import ALL_DTYPES, BF16, DT_NAME, FP16, OP_NAME, OPS, assert_same, from_dev, rand_array, to_dev

pytestmark = pytest.mark.gpu

N_CASES = int(os.environ.get("MI_FUZZ_CASES", "1000"))  # a longer sweep: MI_FUZZ_CASES=10000


def _cases():
    rng = np.random.default_rng(20261016)
    sizes = [0, 1, 7, 16, 17, 1023, 4096, 16384 + 9, 3 * 16384 + 7, 200_003]
    out = []
    for i in range(N_CASES):
        dt = int(rng.choice(ALL_DTYPES))
        op = int(rng.choice(OPS))
        k = int(rng.integers(1, 17))
        n = int(rng.choice(sizes))
        offs = [int(x) for x in rng.integers(0, 16, size=k + 1)]
        if rng.random() < 0.4:  # common misalignment
            offs = [offs[0]] * (k + 1)
        inplace = bool(rng.random() < 0.5)
        variant = 0
        if dt == BF16:
            variant = int(rng.integers(0, 3))  # bf16 impl: scalar / avx512f / avx512bf
        acc32 = dt in (BF16, FP16) and k >= 2 and rng.random() < 0.3
        out.append((i, dt, op, k, n, offs, inplace, variant, acc32))
    return out


CASES = _cases()


@pytest.mark.parametrize("case", CASES, ids=[f"c{c[0]}-{DT_NAME[c[1]]}-{OP_NAME[c[2]]}-k{c[3]}-n{c[4]}"
                                              for c in CASES])
def test_random_case(case):
    import torch
    i, dt, op, k, n, offs, inplace, variant, acc32 = case
    ins = [rand_array(dt, n, seed=10_000 + 97 * i + j, op=op) for j in range(k)]
    if acc32:
        rne = dt == FP16 or variant == 2
        inout_first = variant != 0 or dt == FP16
        flags = F_ACC_FP32 | (F_BF16_RNE if rne else 0) | (F_MINMAX_INOUT_FIRST if inout_first else 0)
        exp = oracle.lp_fanin_acc_fp32(ins, dt, op, rne, inout_first) if n else ins[0].copy()
    else:
        if dt == BF16:
            flags = bf16_flags(variant)
            bimpl = [oracle.BF16_SCALAR, oracle.BF16_AVX512F, oracle.BF16_AVX512BF][variant]
        else:
            flags = F_MINMAX_INOUT_FIRST if dt == FP16 else 0
            bimpl = oracle.BF16_AVX512BF
        exp = oracle.fanin(ins, dt, op, bimpl, oracle.FP16_AVX512F)
    holders = [to_dev(x, pad_elems=16, offset_elems=offs[j]) for j, x in enumerate(ins)]
    if inplace:
        to, po, off_o = holders[0][0], holders[0][1], offs[0]
    else:
        off_o = offs[k]
        to, po = to_dev(np.zeros_like(ins[0]), pad_elems=16, offset_elems=off_o)
    arr = _lib.void_ptr_array([p for _, p in holders])
    _lib.check(_lib.mi().mi_reduce_multi(arr, k, po, n, dt, op, flags, torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    if n:
        assert_same(from_dev(to, ins[0], off_o), exp, dt, f"case {case}")
    for j, (t, _) in enumerate(holders):  # inputs other than the in-place accumulator are untouched
        if not (inplace and j == 0):
            assert_same(from_dev(t, ins[j], offs[j]), ins[j], dt, f"input {j} modified")


def _sync_cases():
    rng = np.random.default_rng(777)
    sizes = [0, 1, 17, 4096, 100_003, 300_007, 2_000_003, 9_000_001]
    weights = np.array([1, 2, 2, 3, 3, 2, 1, 0.3])
    out = []
    for i in range(N_CASES // 4):
        dt = int(rng.choice(ALL_DTYPES))
        op = int(rng.choice(OPS))
        k = int(rng.integers(1, 17))
        n = int(rng.choice(sizes, p=weights / weights.sum()))
        kinds = [int(x) for x in rng.integers(0, 3, size=k + 1)]  # 0 device, 1 pinned, 2 pageable
        offs = [int(x) for x in rng.integers(0, 16, size=k + 1)]
        inplace = bool(rng.random() < 0.5)
        out.append((i, dt, op, k, n, kinds, offs, inplace))
    return out


SYNC_CASES = _sync_cases()


@pytest.mark.parametrize("case", SYNC_CASES, ids=[f"s{c[0]}-{DT_NAME[c[1]]}-{OP_NAME[c[2]]}-k{c[3]}-n{c[4]}"
                                                   for c in SYNC_CASES])
def test_random_sync_case(case):
    """The synchronous entry with a random pointer kind per operand (device,
    pinned, pageable) at random element offsets: zero-copy, bounce buffers,
    the staged pipeline with its drain thread, and their mixes."""
    import torch
    i, dt, op, k, n, kinds, offs, inplace = case
    ins = [rand_array(dt, n, seed=50_000 + 97 * i + j, op=op) for j in range(k)]
    flags = F_MINMAX_INOUT_FIRST if dt == FP16 else (bf16_flags(2) if dt == BF16 else 0)
    exp = oracle.fanin(ins, dt, op, oracle.BF16_AVX512BF, oracle.FP16_AVX512F)
    es = ins[0].itemsize
    keep = []

    def place(x, kind, off):
        raw = np.zeros(x.size + off + 16, x.dtype)
        raw[off:off + x.size] = x
        if kind == 0:
            t, p = to_dev(x, pad_elems=16, offset_elems=off)
            keep.append(t)
            return p, (lambda: from_dev(t, x, off))
        if kind == 1:
            h = torch.from_numpy(raw.view(np.uint8).copy()).pin_memory()
            keep.append(h)
            return h.data_ptr() + off * es, (lambda: h.numpy().view(x.dtype)[off:off + x.size].copy())
        keep.append(raw)
        return raw.ctypes.data + off * es, (lambda: raw[off:off + x.size].copy())

    placed = [place(x, kinds[j], offs[j]) for j, x in enumerate(ins)]
    if inplace:
        po, read = placed[0]
    else:
        po, read = place(np.zeros_like(ins[0]), kinds[k], offs[k])
    arr = _lib.void_ptr_array([p for p, _ in placed])
    _lib.check(_lib.mi().mi_reduce_multi_sync(arr, k, po, n, dt, op, flags, -1))
    if n:
        assert_same(read(), exp, dt, f"case {case}")
