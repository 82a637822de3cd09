"""NaN and Inf bits through every low-precision kernel path, exact.

The kernels fold without NaN fix-ups and refold a row with them only when an
input holds an all-ones exponent, or — for products of three or more inputs —
when the result does (reduce_kernels.hpp fold_vec_x86).  These cases aim at
that screen: NaN payloads of both kinds and signs, infinities, and NaNs that
finite inputs create (a partial product that overflows to Inf, then meets a
zero: x86's default NaN 0xFFC00000 must come out, not the GPU's), placed
sparsely so most rows take the fast path and a few lanes of a wave take the
slow one; sizes cover the scalar head/tail and the vector body; 2 inputs (the
lean kernel), 3, 8 and 16 (the fan-in kernel), and the general kernel via a
launch cap.  Expected bits from the oracle (pinned to the reference's own
code by tests/test_ref_vectors.py); compared with NaN payloads included."""
from __future__ import annotations

import numpy as np
import pytest

import oracle
from oneccl_amd import _lib
from oneccl_amd.comp import F_ACC_FP32, F_BF16_RNE, F_FP16_NATIVE_MINMAX, F_MINMAX_INOUT_FIRST
from tests.util import BF16, FP16, assert_same, from_dev, to_dev

pytestmark = pytest.mark.gpu

BF16_SPECIAL = [0x7FC0, 0xFFC0, 0x7F81, 0xFF81, 0x7FA5, 0x7F80, 0xFF80, 0x0000, 0x8000, 0x7F7F, 0xFF7F]
FP16_SPECIAL = [0x7E00, 0xFE00, 0x7C01, 0xFC01, 0x7D55, 0x7C00, 0xFC00, 0x0000, 0x8000, 0x7BFF, 0xFBFF]

# (name, dtype, flags, oracle fold)
VARIANTS = [
    ("bf16-trunc", BF16, F_MINMAX_INOUT_FIRST,
     lambda ins, op: oracle.fanin(ins, BF16, op, bf16_impl=oracle.BF16_AVX512F)),
    ("bf16-rne", BF16, F_MINMAX_INOUT_FIRST | F_BF16_RNE,
     lambda ins, op: oracle.fanin(ins, BF16, op, bf16_impl=oracle.BF16_AVX512BF)),
    ("fp16", FP16, F_MINMAX_INOUT_FIRST,
     lambda ins, op: oracle.fanin(ins, FP16, op, fp16_impl=oracle.FP16_AVX512F)),
    # CCL_FP16=avx512fp16: VMINPH/VMAXPH keep a NaN accumulator as stored
    ("fp16-native", FP16, F_MINMAX_INOUT_FIRST | F_FP16_NATIVE_MINMAX,
     lambda ins, op: oracle.fanin(ins, FP16, op, fp16_impl=oracle.FP16_AVX512FP16)),
    ("bf16-acc32-rne", BF16, F_ACC_FP32 | F_BF16_RNE | F_MINMAX_INOUT_FIRST,
     lambda ins, op: oracle.lp_fanin_acc_fp32(ins, BF16, op, True, True)),
    ("fp16-acc32", FP16, F_ACC_FP32 | F_MINMAX_INOUT_FIRST,
     lambda ins, op: oracle.lp_fanin_acc_fp32(ins, FP16, op, False, True)),
]


def _inputs(dt, k, n, op, seed):
    rng = np.random.default_rng(seed)
    f = (rng.standard_normal((k, n)) * 4).astype(np.float32)
    ins = [oracle.f32_to_bf16(x, True) if dt == BF16 else oracle.f32_to_fp16(x) for x in f]
    special = np.array(BF16_SPECIAL if dt == BF16 else FP16_SPECIAL, np.uint16)
    for x in ins:  # ~1 % of elements special, so most 8-element rows stay on the fast path
        idx = rng.choice(n, size=max(1, n // 100), replace=False)
        x[idx] = rng.choice(special, size=idx.size)
    if op == 1 and k >= 3 and n >= 64:
        # finite inputs whose partial product overflows, then a zero: NaN from no NaN
        big = 0x7E80 if dt == BF16 else 0x7BFF  # ~8.5e37 / 65504
        rows = rng.choice(n, size=8, replace=False)
        for r in rows:
            for j in range(k - 1):
                ins[j][r] = big
            ins[k - 1][r] = 0
    return ins


@pytest.mark.parametrize("n", [5, 61, 4096 + 13, 300_007])
@pytest.mark.parametrize("k", [2, 3, 8, 16])
@pytest.mark.parametrize("op", [0, 1, 2, 3])
@pytest.mark.parametrize("variant", VARIANTS, ids=[v[0] for v in VARIANTS])
def test_lp_nan_bits_exact(variant, op, k, n):
    import torch
    name, dt, flags, fold = variant
    ins = _inputs(dt, k, n, op, seed=1000 * k + 10 * op + n % 97)
    exp = fold(ins, op)
    holders = [to_dev(x) for x in ins]
    to, po = to_dev(np.zeros(n, np.uint16))
    st = torch.cuda.current_stream().cuda_stream
    _lib.check(_lib.mi().mi_reduce_multi(_lib.void_ptr_array([p for _, p in holders]), k, po, n, dt, op, flags, st))
    torch.cuda.synchronize()
    assert_same(from_dev(to, exp), exp, dt, f"{name} op={op} k={k} n={n}")


@pytest.mark.parametrize("variant", VARIANTS, ids=[v[0] for v in VARIANTS])
@pytest.mark.parametrize("op", [0, 1])
def test_lp_nan_bits_general_kernel(variant, op):
    """The grid-stride general kernel (taken under a launch cap) folds with the
    fix-ups on every row; same bits."""
    import torch
    name, dt, flags, fold = variant
    n, k = 50_003, 5
    ins = _inputs(dt, k, n, op, seed=77 + op)
    exp = fold(ins, op)
    holders = [to_dev(x) for x in ins]
    to, po = to_dev(np.zeros(n, np.uint16))
    m = _lib.mi()
    _lib.check(m.mi_set_max_blocks(64))
    try:
        _lib.check(m.mi_reduce_multi(_lib.void_ptr_array([p for _, p in holders]), k, po, n, dt, op, flags,
                                     torch.cuda.current_stream().cuda_stream))
        torch.cuda.synchronize()
    finally:
        _lib.check(m.mi_set_max_blocks(0))
    assert_same(from_dev(to, exp), exp, dt, f"general {name} op={op}")


@pytest.mark.parametrize("rne", [0, 1])
def test_convert_nan_rows_exact(rne):
    """fp32 -> bf16 / fp16 and fp16 -> fp32 with sparse NaNs and Infs: the
    conversion kernel's screened groups give the reference's NaN bits."""
    import torch
    rng = np.random.default_rng(5 + rne)
    n = 100_003
    u = rng.standard_normal(n).astype(np.float32).view(np.uint32)
    idx = rng.choice(n, size=500, replace=False)
    u[idx] = rng.choice(np.array([0x7FC00000, 0xFFC00000, 0x7F800001, 0xFF812345, 0x7FBFFFFF, 0x7F800000,
                                  0xFF800000], np.uint32), size=idx.size)
    f = u.view(np.float32)
    st = torch.cuda.current_stream().cuda_stream
    m = _lib.mi()
    exp = np.empty(n, np.uint16)
    oracle.lib().orc_convert_fp32_to_bf16_arrays(f.ctypes.data, exp.ctypes.data, n,
                                                 oracle.BF16_AVX512BF if rne else oracle.BF16_AVX512F)
    ts, ps = to_dev(f)
    td, pd = to_dev(np.zeros(n, np.uint16))
    _lib.check(m.mi_convert(ps, 9, pd, BF16, n, (F_BF16_RNE | 0x8) if rne else 0, st))
    torch.cuda.synchronize()
    assert_same(from_dev(td, exp), exp, BF16, "fp32->bf16")
    h = oracle.f32_to_fp16(f)
    _lib.check(m.mi_convert(ps, 9, pd, FP16, n, 0, st))
    torch.cuda.synchronize()
    assert_same(from_dev(td, h), h, FP16, "fp32->fp16")
    h[idx[:100]] = 0x7C01  # signalling fp16 NaNs: VCVTPH2PS quiets them
    th, ph = to_dev(h)
    tf, pf = to_dev(np.zeros(n, np.float32))
    _lib.check(m.mi_convert(ph, FP16, pf, 9, n, 0, st))
    torch.cuda.synchronize()
    ef = oracle.fp16_to_f32(h)
    assert_same(from_dev(tf, ef), ef, 9, "fp16->fp32", nan_payload=True)
