"""BASELINE.json configs[4] (C5): prod/min/max (+sum) on int32 and int64 over
the whole 4 KiB - 1 GiB size sweep (powers of 4), bit-exact against the oracle
(oracle.comp_reduce_mt: CCL_REDUCE, src/comp/comp.cpp:31-58, range-split over
host threads).  The device entry (mi_reduce) covers every size; the drop-in
ccl_comp_reduce on device buffers covers 64 MiB - 1 GiB, the sizes bench.py
times.  Integer results are exact, wrap-around included: every input holds the
type's extremes, and prod inputs mix small factors with extremes so products
wrap."""
from __future__ import annotations

import numpy as np
import pytest

import oracle
from oneccl_amd import _lib, comp
from tests.util import DT_NAME, OP_NAME, assert_same

pytestmark = pytest.mark.gpu

INT32, INT64 = 4, 6
SIZES = [4 << 10, 16 << 10, 64 << 10, 256 << 10, 1 << 20, 4 << 20, 16 << 20, 64 << 20, 256 << 20, 1 << 30]
CASES = [(dt, op) for dt in (INT32, INT64) for op in (0, 1, 2, 3)]


def _label(nbytes):
    return f"{nbytes >> 30}GiB" if nbytes >= 1 << 30 else (f"{nbytes >> 20}MiB" if nbytes >= 1 << 20
                                                           else f"{nbytes >> 10}KiB")


def _inputs(dt, op, n, seed):
    st = oracle.NP_DTYPE[dt]
    info = np.iinfo(st)
    rng = np.random.default_rng(seed)
    if op == 1:
        a = rng.integers(-3, 4, n, dtype=st)
    else:
        a = rng.integers(info.min, info.max, n, dtype=st, endpoint=True)
    # extremes at fixed strides (wrap-around of sum/prod, min/max at the bounds)
    a[::997] = info.min
    a[5::1009] = info.max
    return a


def _dev(a):
    import torch
    return torch.from_numpy(a).cuda()


def _run_case(dt, op, nbytes, via):
    import torch
    es = np.dtype(oracle.NP_DTYPE[dt]).itemsize
    n = nbytes // es
    a = _inputs(dt, op, n, seed=0xC5 + 31 * dt + op)
    b = _inputs(dt, op, n, seed=0x5C + 37 * dt + op)
    ta, tb = _dev(a), _dev(b)
    oracle.comp_reduce_mt(a, b, dt, op, 16)  # b := expected
    del a
    if via == "mi_reduce":
        _lib.check(_lib.mi().mi_reduce(ta.data_ptr(), tb.data_ptr(), n, dt, op, 0,
                                       torch.cuda.current_stream().cuda_stream))
        torch.cuda.synchronize()
    else:
        torch.cuda.synchronize()
        comp.comp_reduce(ta.data_ptr(), n, tb.data_ptr(), comp.datatype(dt), comp.reduction(op))
    del ta
    assert_same(tb.cpu().numpy(), b, dt, f"{DT_NAME[dt]} {OP_NAME[op]} {_label(nbytes)} via {via}")


@pytest.mark.parametrize("nbytes", SIZES, ids=_label)
@pytest.mark.parametrize("dt,op", CASES, ids=[f"{DT_NAME[d]}-{OP_NAME[o]}" for d, o in CASES])
def test_c5_sweep_mi_reduce(dt, op, nbytes):
    _run_case(dt, op, nbytes, "mi_reduce")


@pytest.mark.parametrize("nbytes", SIZES[-3:], ids=_label)
@pytest.mark.parametrize("dt,op", CASES, ids=[f"{DT_NAME[d]}-{OP_NAME[o]}" for d, o in CASES])
def test_c5_sweep_dropin(dt, op, nbytes):
    _run_case(dt, op, nbytes, "ccl_comp_reduce")
