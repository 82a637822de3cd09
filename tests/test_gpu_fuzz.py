"""Seeded random sweep of the whole device surface against the oracle: dtype,
op, semantic variant, input count 1..16, element count (empty, tiny, within
one tile, across tiles), a different element offset per operand (common and
differing misalignments), in place or out of place.  Each case is checked
bit-exactly (NaN payloads aside) against the oracle's chained
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
