"""GPU parity against golden vectors produced by the REFERENCE'S OWN compiled
src/comp code (tests/golden/ref_comp_vectors.npz; producer
oracle/ref_comp_harness.cpp over /root/reference/src/comp/comp.cpp, bf16.cpp,
... built with the reference's Release flags):

  * CCL_REDUCE (comp.cpp:31-58) for the ten non-LP types x four ops through
    every device kernel family: the lean 2-input kernel (aligned), the
    element loop (operands misaligned differently), the buffer-addressed form
    and the general grid-stride kernel (grid cap), and ccl_comp_reduce of the
    drop-in on device, pinned and pageable buffers;
  * the scalar bf16 impl (bf16.cpp:63-85, flags 0);
  * ccl_comp_batch_reduce's storage-precision chain (comp.cpp:236-245) as one
    fused K-input kernel and through the drop-in.

Bar: identical bits, NaN payloads included.  The reference compiles
`inout op= in` to ADDPS/MULPS with inout as the first source (its NaN wins;
inf - inf gives x86's default NaN 0xFFC00000); CDNA's ALUs choose their own
NaN, so the kernels restate that rule on the rows whose result is NaN
(reduce_kernels.hpp x86_refold)."""
from __future__ import annotations

import numpy as np
import pytest

from oneccl_amd import _lib, comp
from tests import refcomp
from tests.util import assert_same, from_dev, to_dev

pytestmark = pytest.mark.gpu

ALL2 = refcomp.cases("reduce") + refcomp.cases("reduce1") + refcomp.cases("bf16s")


def _stream():
    import torch
    return torch.cuda.current_stream().cuda_stream


def _count(c):
    return c["a"].size


@pytest.mark.parametrize("variant", ["aligned", "misaligned", "gridcap"])
@pytest.mark.parametrize("c", ALL2, ids=lambda c: c["key"])
def test_kernel_matches_reference_code(c, variant):
    import torch
    m = _lib.mi()
    n = _count(c)
    ta, pa = to_dev(c["a"], offset_elems=1 if variant == "misaligned" else 0)
    tb, pb = to_dev(c["b"])
    if variant == "gridcap":
        _lib.check(m.mi_set_max_blocks(2))  # the general grid-stride kernel
    try:
        _lib.check(m.mi_reduce(pa, pb, n, c["dtype"], c["op"], 0, _stream()))
        torch.cuda.synchronize()
    finally:
        if variant == "gridcap":
            _lib.check(m.mi_set_max_blocks(0))
    assert_same(from_dev(tb, c["b"]), c["expected"], c["dtype"], c["key"])


@pytest.mark.parametrize("c", refcomp.cases("batch"), ids=lambda c: c["key"])
def test_fused_batch_matches_reference_batch_reduce(c):
    """ccl_comp_batch_reduce's chain of K-1 storage-precision calls == one
    fused K-input kernel (inout first, then the inputs at their offsets)."""
    import torch
    n = c["count"]
    holders = [to_dev(c["b"])] + [to_dev(c["buf"][o:o + n].copy()) for o in c["offsets"][1:]]
    to, po = to_dev(np.zeros_like(c["b"]))
    arr = _lib.void_ptr_array([p for _, p in holders])
    _lib.check(_lib.mi().mi_reduce_multi(arr, len(holders), po, n, c["dtype"], c["op"], 0, _stream()))
    torch.cuda.synchronize()
    assert_same(from_dev(to, c["b"]), c["expected"], c["dtype"], c["key"])


@pytest.mark.parametrize("c", refcomp.cases("batch"), ids=lambda c: c["key"])
def test_dropin_batch_on_device_matches_reference(c):
    """ccl_comp_batch_reduce of the drop-in on device buffers (one tmp
    buffer holding the inputs at unaligned offsets, as nreduce's)."""
    tbuf, pbuf = to_dev(c["buf"])
    tb, pb = to_dev(c["b"])
    oc = comp.comp_batch_reduce(pbuf, c["offsets"], c["count"], pb, comp.datatype(c["dtype"]),
                                comp.reduction(c["op"]))
    assert oc is None  # the reference leaves out_count alone for non-LP types
    assert_same(from_dev(tb, c["b"]), c["expected"], c["dtype"], c["key"])


@pytest.mark.parametrize("where", ["device", "pinned", "pageable_gpu"])
def test_dropin_reduce_matches_reference(where, monkeypatch):
    """ccl_comp_reduce on device buffers, pinned host buffers (zero-copy
    kernel) and pageable host buffers with the dispatcher's CPU path off
    (staged through the GPU): every CCL_REDUCE case."""
    import torch
    if where == "pageable_gpu":
        monkeypatch.setenv("CCL_COMP_HOST_MAX_BYTES", "0")
    else:
        monkeypatch.setenv("CCL_COMP_HOST_MAX_PINNED_BYTES", "0")
    comp.env_reload()
    try:
        for c in refcomp.cases("reduce"):
            n = _count(c)
            if where == "device":
                ta, pa = to_dev(c["a"])
                tb, pb = to_dev(c["b"])
                comp.comp_reduce(pa, n, pb, comp.datatype(c["dtype"]), comp.reduction(c["op"]))
                got = from_dev(tb, c["b"])
            elif where == "pinned":
                ta = torch.from_numpy(c["a"].view(np.uint8).copy()).pin_memory()
                tb = torch.from_numpy(c["b"].view(np.uint8).copy()).pin_memory()
                comp.comp_reduce(ta.data_ptr(), n, tb.data_ptr(), comp.datatype(c["dtype"]), comp.reduction(c["op"]))
                got = tb.numpy().view(c["b"].dtype).copy()
            else:
                a, b = c["a"].copy(), c["b"].copy()
                comp.comp_reduce(a.ctypes.data, n, b.ctypes.data, comp.datatype(c["dtype"]), comp.reduction(c["op"]))
                got = b
            assert_same(got, c["expected"], c["dtype"], f"{where}:{c['key']}")
    finally:
        monkeypatch.delenv("CCL_COMP_HOST_MAX_BYTES", raising=False)
        monkeypatch.delenv("CCL_COMP_HOST_MAX_PINNED_BYTES", raising=False)
        comp.env_reload()


def test_nan_rule_at_full_bucket_scale():
    """The result screen that sends NaN rows to the fix-ups is per 16-byte
    row: sparse both-NaN / inf-inf pairs across a 64 MiB fp32 and fp64 bucket
    (every kernel block sees some) give the reference's bits, the rest the
    plain sum."""
    import torch
    m = _lib.mi()
    for dt, npdt, u, q, dnan in ((9, np.float32, np.uint32, 0x400000, 0xFFC00000),
                                 (10, np.float64, np.uint64, 0x8000000000000, 0xFFF8000000000000)):
        n = (64 << 20) // np.dtype(npdt).itemsize
        rng = np.random.default_rng(dt)
        a = rng.standard_normal(n).astype(npdt)
        b = rng.standard_normal(n).astype(npdt)
        ia = rng.choice(n, 4096, replace=False)
        a.view(u)[ia] = (rng.integers(1, 1 << 20, ia.size).astype(u) | np.array(0x7F800000 if dt == 9 else
                                                                                 0x7FF0000000000000, u))
        b.view(u)[ia[::2]] = (rng.integers(1, 1 << 20, ia.size // 2 + ia.size % 2).astype(u) |
                              np.array(0xFF800000 if dt == 9 else 0xFFF0000000000000, u))
        ii = rng.choice(n, 1024, replace=False)
        a[ii], b[ii] = np.inf, -np.inf
        with np.errstate(invalid="ignore"):
            exp = a + b
        eb = exp.view(u)
        na, nb = np.isnan(a), np.isnan(b)
        eb[nb] = b.view(u)[nb] | np.array(q, u)          # inout's NaN wins
        eb[na & ~nb] = a.view(u)[na & ~nb] | np.array(q, u)
        eb[np.isnan(exp) & ~na & ~nb] = np.array(dnan, u)
        ta, pa = to_dev(a)
        tb, pb = to_dev(b)
        _lib.check(m.mi_reduce(pa, pb, n, dt, 0, 0, _stream()))
        torch.cuda.synchronize()
        assert_same(from_dev(tb, b), exp, dt, f"dtype {dt} sparse NaN")


def _keep_flags(impl):
    return 0x4 | ((0x2 | 0x8) if impl == 2 else 0)


@pytest.mark.parametrize("c", refcomp.cases("keep"), ids=lambda c: c["key"])
def test_fused_keep_precision_matches_reference_parts(c):
    """ccl_comp_batch_reduce's keep-precision mode (fp32 accumulate, one
    rounding per impl, truncated count % 16 tail under avx512bf) as one fused
    kernel, against the composition of the reference's own compiled parts."""
    import torch
    n = c["count"]
    holders = [to_dev(c["b"])] + [to_dev(c["buf"][o:o + n].copy()) for o in c["offsets"][1:]]
    to, po = to_dev(np.zeros_like(c["b"]))
    arr = _lib.void_ptr_array([p for _, p in holders])
    _lib.check(_lib.mi().mi_reduce_multi(arr, len(holders), po, n, 11, c["op"], _keep_flags(c["impl"]), _stream()))
    torch.cuda.synchronize()
    assert_same(from_dev(to, c["b"]), c["expected"], 11, c["key"])


@pytest.mark.parametrize("c", refcomp.cases("keep"), ids=lambda c: c["key"])
def test_dropin_keep_precision_on_device_matches_reference_parts(c, monkeypatch):
    """The drop-in's ccl_comp_batch_reduce(bf16_keep_precision_mode = 1) on
    device buffers with CCL_BF16 selecting the impl (env.cpp:711-713)."""
    monkeypatch.setenv("CCL_BF16", {1: "avx512f", 2: "avx512bf"}[c["impl"]])
    comp.env_reload()
    try:
        tbuf, pbuf = to_dev(c["buf"])
        tb, pb = to_dev(c["b"])
        comp.comp_batch_reduce(pbuf, c["offsets"], c["count"], pb, comp.datatype.bfloat16, comp.reduction(c["op"]),
                               bf16_keep_precision_mode=1)
        assert_same(from_dev(tb, c["b"]), c["expected"], 11, c["key"])
    finally:
        monkeypatch.delenv("CCL_BF16", raising=False)
        comp.env_reload()


@pytest.mark.parametrize("c", refcomp.cases("bf16s"), ids=lambda c: c["key"])
def test_dropin_scalar_bf16_on_device_matches_reference(c, monkeypatch):
    """ccl_comp_reduce on bf16 device buffers with CCL_BF16=scalar."""
    monkeypatch.setenv("CCL_BF16", "scalar")
    comp.env_reload()
    try:
        ta, pa = to_dev(c["a"])
        tb, pb = to_dev(c["b"])
        oc = comp.comp_reduce(pa, c["a"].size, pb, comp.datatype.bfloat16, comp.reduction(c["op"]))
        assert oc == c["a"].size
        assert_same(from_dev(tb, c["b"]), c["expected"], 11, c["key"])
    finally:
        monkeypatch.delenv("CCL_BF16", raising=False)
        comp.env_reload()
