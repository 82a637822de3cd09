"""GPU parity against golden vectors produced by the REFERENCE'S OWN bf16/fp16
reduce code (tests/golden/ref_vectors.npz; producer oracle/ref_harness.cpp over
/root/reference/src/comp/{bf16,fp16}/*_intrisics.*).  The kernels run through
the C ABI with the flags of each impl, and through the drop-in shim with
CCL_BF16 / CCL_FP16 selecting the impl, as oneCCL's env does
(src/common/env/env.cpp:711-720).

Bar: bit-exact, NaN payloads included: the AVX-512 code returns the first NaN
operand quieted and x86's default NaN 0xFFC00000, and the kernels restate
that rule (reduce_kernels.hpp x86_nan_first and the NaN selects of the
narrowing conversions) instead of taking CDNA's ALU NaNs.  The oracle is
pinned to the same vectors in tests/test_ref_vectors.py."""
from __future__ import annotations

import os

import numpy as np
import pytest

from oneccl_amd import _lib, comp
from oneccl_amd.comp import F_BF16_RNE, F_FP16_NATIVE_MINMAX, F_MINMAX_INOUT_FIRST
from tests import refvec
from tests.util import assert_same, from_dev, to_dev

pytestmark = pytest.mark.gpu

# ccl impl type -> kernel flags (oneccl_amd/csrc/comp.cpp bf16_flags / fp16_flags)
BF16_FLAGS = {1: F_MINMAX_INOUT_FIRST, 2: F_MINMAX_INOUT_FIRST | F_BF16_RNE}
FP16_FLAGS = {2: F_MINMAX_INOUT_FIRST, 3: F_MINMAX_INOUT_FIRST, 4: F_MINMAX_INOUT_FIRST | F_FP16_NATIVE_MINMAX}
ENV_NAME = {(refvec.BF16, 1): ("CCL_BF16", "avx512f"), (refvec.BF16, 2): ("CCL_BF16", "avx512bf"),
            (refvec.FP16, 2): ("CCL_FP16", "f16c"), (refvec.FP16, 3): ("CCL_FP16", "avx512f"),
            (refvec.FP16, 4): ("CCL_FP16", "avx512fp16")}


def _cpu_has_avx512fp16():
    try:
        with open("/proc/cpuinfo") as f:
            return "avx512_fp16" in f.read()
    except OSError:
        return False


def _flags(dt, impl):
    return (BF16_FLAGS if dt == refvec.BF16 else FP16_FLAGS)[impl]


def _stream():
    import torch
    return torch.cuda.current_stream().cuda_stream


@pytest.mark.parametrize("c", refvec.reduce_cases(), ids=lambda c: c["key"])
def test_kernel_matches_reference_code(c):
    import torch
    ta, pa = to_dev(c["a"])
    tb, pb = to_dev(c["b"])
    _lib.check(_lib.mi().mi_reduce(pa, pb, c["count"], c["dtype"], c["op"], _flags(c["dtype"], c["impl"]),
                                   _stream()))
    torch.cuda.synchronize()
    assert_same(from_dev(tb, c["b"]), c["expected"], c["dtype"], c["key"])


@pytest.mark.parametrize("c", refvec.fan_cases(), ids=lambda c: c["key"])
def test_fused_fanin_matches_reference_chain(c):
    """The reference folds 8 inputs with 7 chained calls, rounding to storage
    after each; the fused K-input kernel in storage precision gives its bits."""
    import torch
    holders = [to_dev(x) for x in c["inputs"]]
    to, po = to_dev(np.zeros_like(c["inputs"][0]))
    arr = _lib.void_ptr_array([p for _, p in holders])
    _lib.check(_lib.mi().mi_reduce_multi(arr, len(holders), po, c["count"], c["dtype"], c["op"],
                                         _flags(c["dtype"], c["impl"]), _stream()))
    torch.cuda.synchronize()
    assert_same(from_dev(to, c["expected"]), c["expected"], c["dtype"], c["key"])


@pytest.mark.parametrize("impl,f,exp", refvec.conversion_cases(), ids=["avx512f", "avx512bf"])
def test_conversion_matches_reference_stores(impl, f, exp):
    import torch
    tf, pf = to_dev(f)
    tb, pb = to_dev(np.zeros(f.size, np.uint16))
    flags = F_BF16_RNE if impl == 2 else 0
    _lib.check(_lib.mi().mi_convert(pf, 9, pb, 11, f.size, flags, _stream()))
    torch.cuda.synchronize()
    assert_same(from_dev(tb, exp), exp, refvec.BF16, "fp32->bf16")


@pytest.fixture
def impl_env():
    """Set CCL_BF16 / CCL_FP16 for the drop-in, restore afterwards."""
    saved = {k: os.environ.get(k) for k in ("CCL_BF16", "CCL_FP16", "CCL_COMP_HOST_MAX_BYTES")}

    def set_(name, value):
        os.environ[name] = value
        comp.env_reload()

    yield set_
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    comp.env_reload()


@pytest.mark.parametrize("where", ["host", "host_gpu", "device"])
def test_dropin_under_ccl_env_matches_reference_code(where, impl_env):
    """ccl_comp_reduce with the impl chosen by CCL_BF16 / CCL_FP16: every
    2-input case, on host (pageable) buffers — the dispatcher's CPU path, and
    the GPU with that path off — and on device buffers."""
    import torch
    impl_env("CCL_COMP_HOST_MAX_BYTES", "0" if where == "host_gpu" else str(32 << 20))
    for c in refvec.reduce_cases():
        if (c["dtype"], c["impl"]) == (refvec.FP16, 4) and not _cpu_has_avx512fp16():
            continue  # CCL_FP16=avx512fp16 is refused on a CPU without it, as in oneCCL (env.cpp:715-720)
        impl_env(*ENV_NAME[(c["dtype"], c["impl"])])
        if where.startswith("host"):
            a, b = c["a"].copy(), c["b"].copy()
            comp.comp_reduce(a.ctypes.data, c["count"], b.ctypes.data, comp.datatype(c["dtype"]),
                             comp.reduction(c["op"]))
            got = b
        else:
            ta, pa = to_dev(c["a"])
            tb, pb = to_dev(c["b"])
            comp.comp_reduce(pa, c["count"], pb, comp.datatype(c["dtype"]), comp.reduction(c["op"]))
            torch.cuda.synchronize()
            got = from_dev(tb, c["b"])
        assert_same(got, c["expected"], c["dtype"], f"{where} {c['key']}")
