"""The oracle and the drop-in's CPU path against golden vectors produced by
the REFERENCE'S OWN compiled src/comp code (tests/golden/ref_comp_vectors.npz;
producer: oracle/ref_comp_harness.cpp over /root/reference/src/comp/comp.cpp,
bf16/bf16.cpp, ... with the reference's Release flags):

  * CCL_REDUCE through ccl_comp_reduce_regular (comp.cpp:31-58, 76-121), all
    ten non-LP types x four ops, NaN payloads (both operands NaN included),
    +-0, infinities, denormals, wrapping integers; *out_count left untouched;
  * the scalar bf16 impl (bf16.cpp:63-85);
  * ccl_comp_batch_reduce's storage-precision chain (comp.cpp:236-245).

Bar: identical bits.  Where the reference tree is present the library is
rebuilt and the fixture regenerated and compared with the committed file.
(The GPU kernels are checked against the same fixture in
tests/test_gpu_ref_comp_vectors.py.)"""
from __future__ import annotations

import subprocess
from pathlib import Path

import numpy as np
import pytest

import oracle
from oneccl_amd import _lib
from oneccl_amd.comp import reference_flags
from tests import refcomp

ROOT = Path(__file__).resolve().parent.parent
REF = Path("/root/reference/src/comp")


def _bits(a):
    return a.view({1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[a.itemsize])


def _check(got, exp, key):
    diff = np.flatnonzero(_bits(got) != _bits(exp))
    assert diff.size == 0, f"{key}: {diff.size} differ, first {diff[:5].tolist()}: got " \
                           f"{[hex(x) for x in _bits(got)[diff[:5]]]} reference {[hex(x) for x in _bits(exp)[diff[:5]]]}"


@pytest.mark.parametrize("c", refcomp.cases("reduce"), ids=lambda c: c["key"])
def test_oracle_ccl_reduce_matches_reference_code(c):
    b = c["b"].copy()
    oc = oracle.comp_reduce(c["a"], b, c["dtype"], c["op"])
    _check(b, c["expected"], c["key"])
    assert (oc is not None) == c["out_count_written"]


@pytest.mark.parametrize("c", refcomp.cases("reduce1"), ids=lambda c: c["key"])
def test_oracle_ccl_reduce_scalar_path_matches_reference_code(c):
    b = c["b"].copy()
    for i in range(b.size):
        x = b[i:i + 1].copy()
        oracle.comp_reduce(c["a"][i:i + 1].copy(), x, c["dtype"], c["op"])
        b[i] = x[0]
    _check(b, c["expected"], c["key"])


@pytest.mark.parametrize("c", refcomp.cases("bf16s"), ids=lambda c: c["key"])
def test_oracle_scalar_bf16_matches_reference_code(c):
    b = c["b"].copy()
    oracle.comp_reduce(c["a"], b, 11, c["op"], oracle.BF16_SCALAR)
    _check(b, c["expected"], c["key"])


@pytest.mark.parametrize("c", refcomp.cases("batch"), ids=lambda c: c["key"])
def test_oracle_batch_reduce_matches_reference_code(c):
    b = c["b"].copy()
    oc = oracle.batch_reduce(c["buf"], c["offsets"], c["count"], b, c["dtype"], c["op"], 0)
    _check(b, c["expected"], c["key"])
    assert (oc is not None) == c["out_count_written"]


def keep_flags(impl):
    """The kernel / host-path flags of keep-precision batch reduce per bf16
    impl (comp.cpp batch_reduce_body): fp32 accumulate, and for avx512bf RNE
    with the truncated count % 16 tail."""
    return 0x4 | ((0x2 | 0x8) if impl == 2 else 0)


@pytest.mark.parametrize("c", refcomp.cases("keep"), ids=lambda c: c["key"])
def test_oracle_keep_precision_matches_reference_parts(c):
    b = c["b"].copy()
    oracle.batch_reduce(c["buf"], c["offsets"], c["count"], b, 11, c["op"], 1, c["impl"])
    _check(b, c["expected"], c["key"])


def _host_supported():
    return _lib.shim().mi_host_supported() != 0


def _host_reduce(ins, out, dt, op, flags):
    arr = _lib.void_ptr_array([x.ctypes.data for x in ins])
    rc = _lib.shim().mi_host_reduce(arr, len(ins), out.ctypes.data, out.size, dt, op, flags)
    assert rc == 0, rc


@pytest.mark.parametrize("c", refcomp.cases("reduce") + refcomp.cases("reduce1") + refcomp.cases("bf16s"),
                         ids=lambda c: c["key"])
def test_dropin_host_path_matches_reference_code(c):
    """The dispatcher's CPU side (host_reduce.cpp: buckets <= 16 MiB stay on
    the calling thread) is product code: bit for bit the reference's."""
    if not _host_supported():
        pytest.skip("no AVX2/F16C: the dispatcher sends every bucket to the GPU")
    b = c["b"].copy()
    flags = 0 if c["kind"] == "bf16s" else reference_flags(c["dtype"])
    _host_reduce([b, c["a"]], b, c["dtype"], c["op"], flags)  # acc = inout; acc = op(in, acc)
    _check(b, c["expected"], c["key"])


@pytest.mark.parametrize("c", refcomp.cases("keep"), ids=lambda c: c["key"])
def test_dropin_host_keep_precision_matches_reference_parts(c):
    if not _host_supported():
        pytest.skip("no AVX2/F16C")
    n = c["count"]
    ins = [c["b"].copy()] + [c["buf"][o:o + n].copy() for o in c["offsets"][1:]]
    out = c["b"].copy()
    _host_reduce(ins, out, 11, c["op"], keep_flags(c["impl"]))
    _check(out, c["expected"], c["key"])


@pytest.mark.parametrize("c", refcomp.cases("batch"), ids=lambda c: c["key"])
def test_dropin_host_fanin_matches_reference_batch(c):
    if not _host_supported():
        pytest.skip("no AVX2/F16C")
    n, es = c["count"], c["b"].itemsize
    ins = [c["b"].copy()] + [c["buf"][o:o + n].copy() for o in c["offsets"][1:]]
    out = c["b"].copy()
    _host_reduce(ins, out, c["dtype"], c["op"], 0)
    _check(out, c["expected"], c["key"])
    del es


@pytest.mark.parametrize("dt,flags", [(11, 0x4 | 0x2), (11, 0x4), (8, 0x4)], ids=["bf16-rne", "bf16-trunc", "fp16"])
@pytest.mark.parametrize("k", [2, 3])
@pytest.mark.parametrize("op", [0, 1])
def test_dropin_host_acc32_nan_order(dt, flags, k, op):
    """fp32 accumulation (keep-precision, MI_F_ACC_FP32) takes the
    accumulator's NaN first (CCL_REDUCE(float), pinned by the fixture's float
    cases), also at k = 2, where one step rounds once either way but the NaN
    order differs from a storage-precision step."""
    if not _host_supported():
        pytest.skip("no AVX2/F16C")
    rng = np.random.default_rng(k * 10 + op)
    n = 4099
    nan = (0x7F81, 0xFFC3, 0x7FA5) if dt == 11 else (0x7C01, 0xFE03, 0x7E55)
    ins = []
    for j in range(k):
        x = rng.integers(0, 1 << 16, n, dtype=np.uint32).astype(np.uint16)
        x[j::3] = nan[j % 3]  # overlapping NaN lanes with different payloads
        ins.append(x)
    exp = oracle.lp_fanin_acc_fp32(ins, dt, op, bool(flags & 0x2), False)
    out = np.zeros(n, np.uint16)
    _host_reduce(ins, out, dt, op, flags)
    _check(out, exp, f"dt={dt} k={k} op={op}")


def test_fixture_covers_every_row():
    got = {(c["kind"], c["dtype"], c["op"]) for k in ("reduce", "reduce1", "bf16s", "batch", "keep")
           for c in refcomp.cases(k)}
    want = {("reduce", dt, op) for dt in (0, 1, 2, 3, 4, 5, 6, 7, 9, 10) for op in range(4)}
    want |= {("reduce1", dt, op) for dt in (9, 10) for op in range(4)}
    want |= {("bf16s", 11, op) for op in range(4)}
    want |= {("batch", dt, op) for dt in (4, 6, 9, 10) for op in range(4)}
    want |= {("keep", 11, op) for op in range(4)}
    assert got == want
    # both-NaN pairs are in every floating-point case (the unpinned payload rule of round 2)
    for c in refcomp.cases("reduce"):
        if c["dtype"] in (9, 10):
            both = np.isnan(c["a"]) & np.isnan(c["b"])
            assert both.sum() >= 9


@pytest.mark.skipif(not REF.is_dir(), reason="reference tree absent (GPU box): the committed fixture is used")
def test_fixture_regenerates_from_reference_code():
    r = subprocess.run(["make", "-C", str(ROOT / "oracle"), "refcomp"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    import importlib.util
    spec = importlib.util.spec_from_file_location("mrcv", ROOT / "tests" / "golden" / "make_ref_comp_vectors.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    fresh = m.generate()
    committed, _ = refcomp.load()
    for k, v in fresh.items():
        if k == "meta":
            continue
        assert v.dtype == committed[k].dtype and np.array_equal(v.view(np.uint8), committed[k].view(np.uint8)), k


@pytest.mark.skipif(not REF.is_dir(), reason="reference tree absent")
def test_reference_library_leaves_only_global_state_unbound():
    """The recipe writes no stand-in: the only symbols the reference objects
    need and the library does not define are global_data::get/env (the
    runtime's global state) and datatype_attr::get (the public datatype API),
    all functions, none called on the harness's paths."""
    r = subprocess.run(["make", "-C", str(ROOT / "oracle"), "refcomp"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    so = ROOT / "oracle" / "_ref" / "libref_ccl_comp.so"
    nm = subprocess.run(["nm", "-D", "-u", "-C", str(so)], capture_output=True, text=True, check=True).stdout
    undef = {ln.split(None, 1)[1] for ln in nm.splitlines() if ln.strip().startswith("U ")}
    ours = {u for u in undef if "ccl" in u}
    assert ours == {"ccl::global_data::env()", "ccl::global_data::get()"} | \
        {u for u in ours if u.startswith("ccl::detail::ccl_api_type_attr_traits")}, ours


@pytest.mark.skipif(not oracle.ref_comp_available(), reason="oracle/_ref/libref_ccl_comp.so not built")
@pytest.mark.parametrize("nthreads", [1, 4])
def test_reference_cpu_baseline_call_matches_oracle(nthreads):
    """bench.py's cpu_baseline times the reference's own compiled CCL_REDUCE
    (kind "reference"), range-split over threads: same bits as the oracle."""
    rng = np.random.default_rng(nthreads)
    for dt, op in ((9, 0), (4, 3), (6, 1), (10, 2)):
        if dt in (9, 10):
            a = rng.standard_normal(100_003).astype(oracle.NP_DTYPE[dt])
            b = rng.standard_normal(100_003).astype(oracle.NP_DTYPE[dt])
        else:
            a = rng.integers(-1000, 1000, 100_003).astype(oracle.NP_DTYPE[dt])
            b = rng.integers(-1000, 1000, 100_003).astype(oracle.NP_DTYPE[dt])
        x, y = b.copy(), b.copy()
        oracle.ref_comp_reduce(a, x, dt, op, nthreads)
        oracle.comp_reduce(a, y, dt, op)
        _check(x, y, f"dt={dt} op={op}")


@pytest.mark.skipif(not oracle.ref_comp_available(), reason="oracle/_ref/libref_ccl_comp.so not built")
@pytest.mark.parametrize("nontemporal", [0, 1])
def test_dropin_copy_matches_reference_copy(nontemporal):
    """ccl_comp_copy (comp.cpp:60-74, memcpy / memcpy_nontemporal of
    common/utils/memcpy.cpp): the reference's own compiled copy and the
    drop-in's (host buffers stay on the calling thread's CPU) give the same
    bytes for odd sizes at every source/destination misalignment, and touch
    nothing outside the range."""
    import ctypes
    L = oracle.ref_comp_lib()
    L.ref_ccl_comp_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    L.ref_ccl_comp_copy.restype = ctypes.c_int
    s = _lib.shim()
    rng = np.random.default_rng(nontemporal)
    src = rng.integers(0, 256, 1 << 16, dtype=np.uint8)
    for nbytes in (0, 1, 7, 63, 64, 255, 256, 257, 4099, 40000):
        for so in (0, 1, 13, 64):
            for do in (0, 3, 32):
                a = rng.integers(0, 256, nbytes + 200, dtype=np.uint8)
                b = a.copy()
                assert L.ref_ccl_comp_copy(src.ctypes.data + so, a.ctypes.data + do, nbytes, nontemporal) == 0
                _lib.check_shim(s.mi_ccl_comp_copy(src.ctypes.data + so, b.ctypes.data + do, nbytes, nontemporal),
                                "ccl_comp_copy")
                assert np.array_equal(a, b), (nbytes, so, do)


@pytest.mark.parametrize("c", refcomp.cases("keep"), ids=lambda c: c["key"])
def test_dropin_keep_precision_host_buffers_matches_reference_parts(c, monkeypatch):
    """ccl_comp_batch_reduce(bf16_keep_precision_mode = 1) through the drop-in
    on host buffers (the dispatcher's CPU path), CCL_BF16 selecting the impl."""
    if not _host_supported():
        pytest.skip("no AVX2/F16C")
    from oneccl_amd import comp
    monkeypatch.setenv("CCL_BF16", {1: "avx512f", 2: "avx512bf"}[c["impl"]])
    comp.env_reload()
    try:
        buf, b = c["buf"].copy(), c["b"].copy()
        comp.comp_batch_reduce(buf.ctypes.data, c["offsets"], c["count"], b.ctypes.data, comp.datatype.bfloat16,
                               comp.reduction(c["op"]), bf16_keep_precision_mode=1)
        _check(b, c["expected"], c["key"])
    finally:
        monkeypatch.delenv("CCL_BF16", raising=False)
        comp.env_reload()


@pytest.mark.parametrize("c", refcomp.cases("bf16s"), ids=lambda c: c["key"])
def test_dropin_scalar_bf16_host_buffers_matches_reference(c, monkeypatch):
    """ccl_comp_reduce on bf16 with CCL_BF16=scalar (ccl_bf16_reduce's scalar
    branch, bf16.cpp:98-101) through the drop-in's CPU path."""
    if not _host_supported():
        pytest.skip("no AVX2/F16C")
    from oneccl_amd import comp
    monkeypatch.setenv("CCL_BF16", "scalar")
    comp.env_reload()
    try:
        a, b = c["a"].copy(), c["b"].copy()
        oc = comp.comp_reduce(a.ctypes.data, a.size, b.ctypes.data, comp.datatype.bfloat16, comp.reduction(c["op"]))
        assert oc == a.size  # bf16.cpp:94-96 writes out_count
        _check(b, c["expected"], c["key"])
    finally:
        monkeypatch.delenv("CCL_BF16", raising=False)
        comp.env_reload()
