"""Precision conversions on the GPU (mi_convert / the drop-in's
ccl_convert_* entry points) against the oracle.  The fp32 -> bf16 RNE and
fp32 -> fp16 conversions are checked over ALL 2^32 fp32 bit patterns: the
reduce kernels use the same device functions for every rounding they do, so
this pins their rounding exhaustively, NaN payloads included (the reference's
VCVTNEPS2BF16 / VCVTPS2PH / VCVTPH2PS quiet a NaN and keep its top payload
bits; the kernels restate that rather than take the ALU's NaN)."""
from __future__ import annotations

import numpy as np
import pytest

import oracle
from oneccl_amd import _lib, comp
from tests.util import BF16, FP16, FP32, assert_same, from_dev, to_dev

pytestmark = pytest.mark.gpu

CHUNK = 1 << 27


def _stream():
    import torch
    return torch.cuda.current_stream().cuda_stream


def _gpu_convert(src_np, sdt, ddt, flags, out_dtype, offset_src=0, offset_dst=0):
    import torch
    ts, ps = to_dev(src_np, offset_elems=offset_src)
    out = np.zeros(src_np.size, out_dtype)
    td, pd = to_dev(out, offset_elems=offset_dst)
    _lib.check(_lib.mi().mi_convert(ps, sdt, pd, ddt, src_np.size, flags, _stream()))
    torch.cuda.synchronize()
    return from_dev(td, out, offset_dst)


@pytest.mark.parametrize("ddt,flags", [(BF16, comp.F_BF16_RNE), (FP16, 0), (BF16, 0)],
                         ids=["bf16_rne", "fp16_rne", "bf16_trunc"])
def test_fp32_to_lp_all_bit_patterns(ddt, flags):
    import torch
    L = oracle.lib()
    m = _lib.mi()
    dev_out = torch.empty(CHUNK, dtype=torch.int16, device="cuda")
    exp = np.empty(CHUNK, np.uint16)
    for c in range((1 << 32) // CHUNK):
        host = np.arange(CHUNK, dtype=np.uint32) + np.uint32(c * CHUNK)
        dev_in = torch.arange(c * CHUNK, (c + 1) * CHUNK, dtype=torch.int64, device="cuda").to(torch.int32)
        _lib.check(m.mi_convert(dev_in.data_ptr(), FP32, dev_out.data_ptr(), ddt, CHUNK, flags, _stream()))
        if ddt == BF16:
            L.orc_convert_fp32_to_bf16_arrays(host.ctypes.data, exp.ctypes.data, CHUNK,
                                              oracle.BF16_AVX512BF if flags else oracle.BF16_SCALAR)
        else:
            exp[:] = oracle.f32_to_fp16(host.view(np.float32))
        torch.cuda.synchronize()
        got = dev_out.cpu().numpy().view(np.uint16)
        assert_same(got, exp, ddt, f"chunk {c}")


@pytest.mark.parametrize("sdt", [BF16, FP16])
def test_lp_to_fp32_all_patterns(sdt):
    src = np.arange(65536, dtype=np.uint32).astype(np.uint16)
    got = _gpu_convert(src, sdt, FP32, 0, np.float32)
    L = oracle.lib()
    if sdt == BF16:
        exp = np.empty(65536, np.float32)
        L.orc_convert_bf16_to_fp32_arrays(src.ctypes.data, exp.ctypes.data, 65536)
    else:
        exp = oracle.fp16_to_f32(src)
    assert_same(got, exp, FP32, nan_payload=True)


@pytest.mark.parametrize("n", [1, 15, 16, 17, 4099, 1 << 20])
@pytest.mark.parametrize("impl", [0, 1, 2])
def test_fp32_to_bf16_arrays_tail_semantics(n, impl):
    """ccl_convert_fp32_to_bf16_arrays (bf16.cpp:130-149): avx512bf rounds the
    first (count/16)*16 elements and truncates the tail."""
    rng = np.random.default_rng(n)
    src = (rng.standard_normal(n) * 3).astype(np.float32)
    exp = np.empty(n, np.uint16)
    oracle.lib().orc_convert_fp32_to_bf16_arrays(src.ctypes.data, exp.ctypes.data, n, impl)
    flags = (comp.F_BF16_RNE | comp.F_BF16_TAIL_TRUNC16) if impl == 2 else 0
    got = _gpu_convert(src, FP32, BF16, flags, np.uint16)
    assert_same(got, exp, BF16)
    # the drop-in entry point on host arrays, with the impl forced by CCL_BF16
    import os
    os.environ["CCL_BF16"] = ["scalar", "avx512f", "avx512bf"][impl]
    try:
        comp.env_reload()
        host_out = np.zeros(n, np.uint16)
        _lib.check_shim(_lib.shim().mi_ccl_convert_fp32_to_bf16_arrays(src.ctypes.data, host_out.ctypes.data, n))
        assert_same(host_out, exp, BF16, "drop-in")
        back = np.zeros(n, np.float32)
        _lib.check_shim(_lib.shim().mi_ccl_convert_bf16_to_fp32_arrays(host_out.ctypes.data, back.ctypes.data, n))
        assert_same(back, oracle.bf16_to_f32(host_out), FP32, "drop-in back")
    finally:
        os.environ.pop("CCL_BF16", None)
        comp.env_reload()


@pytest.mark.parametrize("offs", [(1, 0), (0, 1), (3, 5)])
def test_convert_unaligned(offs):
    n = 1001
    src = (np.random.default_rng(2).standard_normal(n) * 100).astype(np.float32)
    got = _gpu_convert(src, FP32, FP16, 0, np.uint16, *offs)
    assert_same(got, oracle.f32_to_fp16(src), FP16)


CONV_PAIRS = [(FP32, BF16, comp.F_BF16_RNE | comp.F_BF16_TAIL_TRUNC16), (FP32, BF16, 0), (FP32, FP16, 0),
              (BF16, FP32, 0), (FP16, FP32, 0)]


@pytest.mark.parametrize("sdt,ddt,flags", CONV_PAIRS, ids=["f32-bf16rne-tail", "f32-bf16trunc", "f32-f16",
                                                           "bf16-f32", "f16-f32"])
@pytest.mark.parametrize("offs", [(0, 0), (1, 0), (0, 1), (3, 5), (2, 7)])
@pytest.mark.parametrize("vectors,cap", [(1, 0), (0, 0), (1, 3), (1, 5)],
                         ids=["unaligned-vectors", "element-loop", "grid-cap-3", "grid-cap-5"])
def test_convert_any_offsets(sdt, ddt, flags, offs, vectors, cap):
    """Conversions between sub-buffers at any element offsets: the vector path
    on dst's 16-byte grid (scalar head, unaligned source vectors, tail) and the
    element loop give the oracle's bits, including the count % 16 truncated
    tail of ccl_convert_fp32_to_bf16_arrays (bf16.cpp:145-148).  A grid cap
    makes every lane stride through many 64-group wave chunks (two runs of 4
    elements per lane) before the partial last chunk."""
    n = 8 * 4099 + 13
    rng = np.random.default_rng(sum(offs) + 10 * sdt + ddt)
    f = (rng.standard_normal(n) * 7).astype(np.float32)
    if sdt == FP32:
        src = f
        exp = np.empty(n, np.uint16)
        if ddt == BF16:
            impl = 2 if flags else 0
            oracle.lib().orc_convert_fp32_to_bf16_arrays(src.ctypes.data, exp.ctypes.data, n, impl)
        else:
            exp = oracle.f32_to_fp16(src)
        out_dtype = np.uint16
    else:
        src = oracle.f32_to_bf16(f, True) if sdt == BF16 else oracle.f32_to_fp16(f)
        exp = oracle.bf16_to_f32(src) if sdt == BF16 else oracle.fp16_to_f32(src)
        out_dtype = np.float32
    m = _lib.mi()
    prev = m.mi_set_unaligned_vectors(vectors)
    _lib.check(m.mi_set_max_blocks(cap))
    try:
        got = _gpu_convert(src, sdt, ddt, flags, out_dtype, *offs)
    finally:
        m.mi_set_unaligned_vectors(prev)
        _lib.check(m.mi_set_max_blocks(0))
    assert_same(got, exp, ddt)


def test_fp16_vector_entry_points():
    src = np.array([1.0, -2.5, 65504.0, 1e-7, 65520.0, -0.0, 3.14159, 1e5], np.float32)
    h = np.zeros(8, np.uint16)
    _lib.check_shim(_lib.shim().mi_ccl_convert_fp32_to_fp16(src.ctypes.data, h.ctypes.data))
    assert_same(h, oracle.f32_to_fp16(src), FP16)
    back = np.zeros(8, np.float32)
    _lib.check_shim(_lib.shim().mi_ccl_convert_fp16_to_fp32(h.ctypes.data, back.ctypes.data))
    assert_same(back, oracle.fp16_to_f32(h), FP32)


def test_unsupported_pair():
    assert _lib.mi().mi_convert(0, 4, 0, 9, 10, 0, None) == -2


@pytest.mark.parametrize("ddt,flags,impl", [(BF16, comp.F_BF16_RNE | comp.F_BF16_TAIL_TRUNC16, 2), (BF16, 0, 0),
                                            (FP16, 0, None)], ids=["bf16rne-tail", "bf16trunc", "fp16"])
@pytest.mark.parametrize("offs", [(0, 0), (1, 0), (0, 3), (5, 2)])
def test_streaming_narrowing_conversions(ddt, flags, impl, offs):
    """Narrowing conversions of 64 MiB of source and more store with sc1 +
    nt through per-wave buffer descriptors (mi_reduce.hip kConvStreamBytes):
    the oracle's bits at shifted offsets, a ragged count % 16 tail and
    nothing written past the destination."""
    import torch
    n = (64 << 20) // 4 + 8 * 37 + 13
    rng = np.random.default_rng(sum(offs) + ddt)
    src = (rng.standard_normal(n) * 9).astype(np.float32)
    if ddt == BF16:
        exp = np.empty(n, np.uint16)
        oracle.lib().orc_convert_fp32_to_bf16_arrays(src.ctypes.data, exp.ctypes.data, n, impl)
    else:
        exp = oracle.f32_to_fp16(src)
    ts, ps = to_dev(src, offset_elems=offs[0])
    td = torch.full((n + offs[1] + 64,), 0x5A5A, dtype=torch.int16, device="cuda")
    pd = td.data_ptr() + 2 * offs[1]
    torch.cuda.synchronize()
    _lib.check(_lib.mi().mi_convert(ps, FP32, pd, ddt, n, flags, _stream()))
    torch.cuda.synchronize()
    got = td.cpu().numpy().view(np.uint16)
    assert_same(got[offs[1]:offs[1] + n], exp, ddt)
    assert (got[:offs[1]] == 0x5A5A).all() and (got[offs[1] + n:] == 0x5A5A).all()
