"""The drop-in's CPU path for small host-resident chunks (oneccl_amd/csrc/
host_reduce.cpp, include/mi_host_reduce.h; SURVEY.md §8f rank 1 dispatcher).

It must give the bits of the reference for every dtype x op x impl variant,
exactly as the GPU kernels do: checked here against the oracle (and against
the golden vectors produced by the reference's own AVX-512 code), directly
and through the shim's entry points on host buffers below the crossover,
where the dispatcher keeps the reduce on the calling thread.  CPU-only: the
host path never touches the GPU.  Bar: bit-exact; NaN payloads included for
the bf16/fp16 paths (the x86 rule is pinned by the reference vectors), for
fp32/fp64 CCL_REDUCE two NaNs compare equal (its payload choice is the
compiler's).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import pytest

import oracle
from oneccl_amd import _lib, comp
from oneccl_amd.comp import F_ACC_FP32, F_BF16_RNE, F_BF16_TAIL_TRUNC16, F_MINMAX_INOUT_FIRST, bf16_flags
from tests import kat, refvec
from tests.util import ALL_DTYPES, BF16, DT_NAME, FP16, FP32, FP64, INT_DTYPES, OP_NAME, OPS, assert_same, rand_array

pytestmark = pytest.mark.skipif(not _lib.shim().mi_host_supported(), reason="CPU lacks AVX2/F16C: no host path")

VARIANTS = {dt: [("ref", 0, oracle.BF16_AVX512BF, oracle.FP16_AVX512F)] for dt in INT_DTYPES + [FP32, FP64]}
VARIANTS[BF16] = [("scalar", bf16_flags(0), oracle.BF16_SCALAR, 0), ("avx512f", bf16_flags(1), oracle.BF16_AVX512F, 0),
                  ("avx512bf", bf16_flags(2), oracle.BF16_AVX512BF, 0)]
VARIANTS[FP16] = [("avx512f", F_MINMAX_INOUT_FIRST, 0, oracle.FP16_AVX512F)]
CASES = [(dt, op, v) for dt in ALL_DTYPES for op in OPS for v in VARIANTS[dt]]
SIZES = [1, 15, 17, 511, 513, 4099, 100_003]


def same(got, exp, dt, what=""):
    if dt in (BF16, FP16) or dt in INT_DTYPES:
        iv = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[got.itemsize]
        d = np.flatnonzero(got.view(iv) != exp.view(iv))
        assert d.size == 0, f"{what}: {d.size} differ, first {d[:5].tolist()}: {got[d[:5]]} vs {exp[d[:5]]}"
    else:
        assert_same(got, exp, dt, what)


def host_fold(ins, dt, op, flags, out=None):
    out = ins[0].copy() if out is None else out
    arr = _lib.void_ptr_array([x.ctypes.data for x in ins])
    rc = _lib.shim().mi_host_reduce(arr, len(ins), out.ctypes.data, out.size, dt, op, flags)
    assert rc == 0, rc
    return out


@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("dt,op,var", CASES, ids=[f"{DT_NAME[d]}-{OP_NAME[o]}-{v[0]}" for d, o, v in CASES])
def test_host_reduce_2input_vs_oracle(dt, op, var, n):
    _, flags, bimpl, fimpl = var
    a = rand_array(dt, n, seed=1000 + 17 * dt + op, op=op)
    b = rand_array(dt, n, seed=2000 + 17 * dt + op, op=op)
    exp = b.copy()
    oracle.comp_reduce(a, exp, dt, op, bimpl, fimpl)
    same(host_fold([b, a], dt, op, flags), exp, dt, f"n={n}")


FAN = [(dt, op, v, k) for dt in (0, 3, 4, 7, FP16, FP32, FP64, BF16) for op in OPS for v in VARIANTS[dt][-1:]
       for k in (1, 3, 16)]


@pytest.mark.parametrize("dt,op,var,k", FAN, ids=[f"{DT_NAME[d]}-{OP_NAME[o]}-{v[0]}-k{k}" for d, o, v, k in FAN])
def test_host_fanin_storage_precision_vs_chained_oracle(dt, op, var, k):
    n = 2 * 512 + 37
    ins = [rand_array(dt, n, seed=300 + 11 * j + dt, op=op) for j in range(k)]
    exp = oracle.fanin(ins, dt, op, var[2], var[3])
    out = np.zeros_like(ins[0])
    same(host_fold(ins, dt, op, var[1], out), exp, dt)


@pytest.mark.parametrize("dt", [BF16, FP16])
@pytest.mark.parametrize("op", OPS)
@pytest.mark.parametrize("rne", [False, True])
@pytest.mark.parametrize("inout_first", [False, True])
def test_host_fanin_fp32_accumulate(dt, op, rne, inout_first):
    if dt == FP16 and not rne:
        pytest.skip("fp16 always rounds RNE")
    n, k = 2011, 5
    ins = [rand_array(dt, n, seed=7 * j + op, op=op) for j in range(k)]
    exp = oracle.lp_fanin_acc_fp32(ins, dt, op, rne, inout_first)
    flags = F_ACC_FP32 | (F_BF16_RNE if rne else 0) | (F_MINMAX_INOUT_FIRST if inout_first else 0)
    same(host_fold(ins, dt, op, flags, np.zeros_like(ins[0])), exp, dt)


@pytest.mark.parametrize("bimpl", [oracle.BF16_SCALAR, oracle.BF16_AVX512F, oracle.BF16_AVX512BF])
@pytest.mark.parametrize("k", [1, 2, 4, 16])
@pytest.mark.parametrize("n", [15, 16, 513, 4099])
def test_host_keep_precision_matches_batch_reduce(bimpl, k, n):
    """ccl_comp_batch_reduce(keep_precision=1) incl. the truncated count%16 tail."""
    ins = [rand_array(BF16, n, seed=900 + j) for j in range(k)]
    exp = ins[0].copy()
    oracle.batch_reduce(np.concatenate(ins), [j * n for j in range(k)], n, exp, BF16, 0, 1, bimpl, 0)
    flags = F_ACC_FP32 | ((F_BF16_RNE | F_BF16_TAIL_TRUNC16) if bimpl == oracle.BF16_AVX512BF else 0)
    out = ins[0].copy()
    assert_same(host_fold(ins, BF16, 0, flags, out), exp, BF16)


@pytest.mark.parametrize("c", refvec.reduce_cases(), ids=lambda c: c["key"])
def test_host_reduce_matches_reference_code(c):
    from oneccl_amd.comp import F_FP16_NATIVE_MINMAX
    flags = ({1: F_MINMAX_INOUT_FIRST, 2: F_MINMAX_INOUT_FIRST | F_BF16_RNE}[c["impl"]] if c["dtype"] == BF16
             else F_MINMAX_INOUT_FIRST | (F_FP16_NATIVE_MINMAX if c["impl"] == 4 else 0))
    b = c["b"].copy()
    arr = _lib.void_ptr_array([b.ctypes.data, c["a"].ctypes.data])
    assert _lib.shim().mi_host_reduce(arr, 2, b.ctypes.data, c["count"], c["dtype"], c["op"], flags) == 0
    same(b, c["expected"], c["dtype"], c["key"])  # payloads included


@pytest.mark.parametrize("rne", [False, True])
@pytest.mark.parametrize("tail", [False, True])
@pytest.mark.parametrize("n", [1, 16, 37, 5000])
def test_host_conversions(rne, tail, n):
    f = rand_array(FP32, n, seed=n)
    got = np.empty(n, np.uint16)
    flags = (F_BF16_RNE if rne else 0) | (F_BF16_TAIL_TRUNC16 if tail else 0)
    assert _lib.shim().mi_host_convert(f.ctypes.data, FP32, got.ctypes.data, BF16, n, flags) == 0
    lim = (n // 16) * 16 if (rne and tail) else (n if rne else 0)
    exp = np.concatenate([oracle.f32_to_bf16(f[:lim], True), oracle.f32_to_bf16(f[lim:], False)])
    same(got, exp, BF16)
    h = np.empty(n, np.uint16)
    assert _lib.shim().mi_host_convert(f.ctypes.data, FP32, h.ctypes.data, FP16, n, 0) == 0
    same(h, oracle.f32_to_fp16(f), FP16)
    back = np.empty(n, np.float32)
    assert _lib.shim().mi_host_convert(h.ctypes.data, FP16, back.ctypes.data, FP32, n, 0) == 0
    assert np.array_equal(back.view(np.uint32), oracle.fp16_to_f32(h).view(np.uint32))


def test_host_reduce_argument_errors():
    s = _lib.shim()
    a = np.zeros(8, np.float32)
    arr = _lib.void_ptr_array([a.ctypes.data, a.ctypes.data])
    assert s.mi_host_reduce(arr, 2, a.ctypes.data, 8, 99, 0, 0) == -1
    assert s.mi_host_reduce(arr, 2, a.ctypes.data, 8, FP32, 4, 0) == -1
    assert s.mi_host_reduce(arr, 17, a.ctypes.data, 8, FP32, 0, 0) == -1
    assert s.mi_host_reduce(arr, 2, a.ctypes.data, 0, FP32, 0, 0) == 0
    assert s.mi_host_convert(a.ctypes.data, FP32, a.ctypes.data, 4, 8, 0) == -2


# ---- through the drop-in: the dispatcher keeps small host buckets here -------

@pytest.fixture
def env():
    saved = {k: os.environ.get(k) for k in ("CCL_BF16", "CCL_FP16", "CCL_COMP_HOST_MAX_BYTES")}

    def set_(**kv):
        for k, v in kv.items():
            os.environ[k] = v
        comp.env_reload()

    yield set_
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    comp.env_reload()


@pytest.mark.parametrize("dt", ALL_DTYPES, ids=[DT_NAME[d] for d in ALL_DTYPES])
def test_dropin_host_buffers_on_cpu(dt, env):
    """ccl_comp_reduce on pageable host buffers under the impl types in force:
    the reference's bits, computed on the calling thread (no GPU here)."""
    env(CCL_COMP_HOST_MAX_BYTES=str(1 << 20))
    b_impl, f_impl = comp.impl_types()
    for op in OPS:
        a = rand_array(dt, 4099, seed=5 + op, op=op)
        b = rand_array(dt, 4099, seed=6 + op, op=op)
        exp = b.copy()
        oc_ref = oracle.comp_reduce(a, exp, dt, op, int(b_impl), int(f_impl))
        oc = comp.comp_reduce(a.ctypes.data, a.size, b.ctypes.data, comp.datatype(dt), comp.reduction(op))
        same(b, exp, dt, OP_NAME[op])
        assert oc == oc_ref


@pytest.mark.parametrize("setting,impl", [("scalar", 0), ("avx512f", 1), ("avx512bf", 2)])
def test_dropin_host_bf16_env(setting, impl, env):
    env(CCL_BF16=setting)
    for op in OPS:
        a = rand_array(BF16, 1000, seed=op)
        b = rand_array(BF16, 1000, seed=op + 10)
        exp = b.copy()
        oracle.comp_reduce(a, exp, BF16, op, impl)
        comp.comp_reduce(a.ctypes.data, a.size, b.ctypes.data, comp.datatype.bfloat16, comp.reduction(op))
        same(b, exp, BF16, f"{setting} {OP_NAME[op]}")


@pytest.mark.parametrize("keep", [0, 1])
@pytest.mark.parametrize("k", [2, 16, 23])
@pytest.mark.parametrize("dt", [BF16, FP32, 4])
def test_dropin_host_batch_reduce(keep, k, dt, env):
    if keep and dt != BF16:
        pytest.skip("keep-precision mode reads bf16")
    b_impl, f_impl = comp.impl_types()
    n = 1043
    ins = [rand_array(dt, n, seed=300 + j) for j in range(k)]
    packed = np.concatenate(ins)
    offsets = [j * n for j in range(k)]
    exp = ins[0].copy()
    oc_ref = oracle.batch_reduce(packed, offsets, n, exp, dt, 0, keep, int(b_impl), int(f_impl))
    got = ins[0].copy()
    oc = comp.comp_batch_reduce(packed.ctypes.data, offsets, n, got.ctypes.data, comp.datatype(dt),
                                comp.reduction.sum, keep)
    assert_same(got, exp, dt)
    assert oc == oc_ref


@pytest.mark.parametrize("nt", [0, 1])
def test_host_copy_offsets_and_sizes(nt):
    """mi_host_copy (host-to-host ccl_comp_copy): with nontemporal, streaming
    stores from the destination's first 64-byte boundary, 128 and 32 bytes per
    step, memcpy head and tail (the reference's memcpy_nontemporal switches at
    256 bytes, src/common/utils/memcpy.cpp:59).  Bytes equal at every offset
    pair and size around those steps; nothing outside the range is written."""
    rng = np.random.default_rng(11)
    src = rng.integers(0, 256, 1 << 16, dtype=np.uint8)
    hc = _lib.shim().mi_host_copy
    for so in (0, 1, 7, 32, 63):
        for do in (0, 1, 31, 32, 60):
            for n in (1, 255, 256, 257, 300, 383, 4096 + 5, 60_000):
                dst = np.zeros(n + 128, np.uint8)
                assert hc(dst.ctypes.data + do, src.ctypes.data + so, n, nt) == 0
                assert np.array_equal(dst[do:do + n], src[so:so + n]), (so, do, n)
                assert not dst[:do].any() and not dst[do + n:].any(), (so, do, n)
    assert hc(0, 0, 0, nt) == 0
    assert hc(0, src.ctypes.data, 5, nt) < 0


def test_dropin_host_conversions_and_copy():
    f = rand_array(FP32, 37, seed=3)
    b_impl, _ = comp.impl_types()
    h = np.empty(37, np.uint16)
    _lib.check_shim(_lib.shim().mi_ccl_convert_fp32_to_bf16_arrays(f.ctypes.data, h.ctypes.data, 37))
    exp = np.empty(37, np.uint16)
    oracle.lib().orc_convert_fp32_to_bf16_arrays(f.ctypes.data, exp.ctypes.data, 37, int(b_impl))
    same(h, exp, BF16)
    src = np.arange(1001, dtype=np.uint8)
    dst = np.zeros_like(src)
    comp.comp_copy(src.ctypes.data, dst.ctypes.data, src.size, True)
    assert np.array_equal(src, dst)


def test_dropin_start_on_small_host_buffers_completes_at_start():
    a = np.ones(4096, np.float32)
    b = np.full(4096, 2.0, np.float32)
    req = comp.comp_reduce_start(a.ctypes.data, a.size, b.ctypes.data, comp.datatype.float32, comp.reduction.sum)
    try:
        assert req.test()
        assert np.all(b == 3.0)
    finally:
        req.free()


def test_reference_functional_kats_through_dropin_on_cpu():
    """oneCCL's tests/functional KATs (SIZE_SMALL/MEDIUM/LARGE) with every
    local reduce done by the drop-in on host buffers: the host path."""
    b_impl, _ = comp.impl_types()
    for case in kat.load():
        if case["suite"] != "tests/functional":
            continue
        dt = case["dtype"]

        def reduce2(a, b):
            comp.comp_reduce(a.ctypes.data, a.size, b.ctypes.data, comp.datatype(dt), comp.reduction(case["op"]))

        for count in case["counts"]:
            err, tol = kat.functional_case(case, count, reduce2, bf16_rne=(b_impl == 2))
            assert err <= tol, (case, count)


def test_threshold_zero_sends_host_buffers_to_the_gpu(env):
    """CCL_COMP_HOST_MAX_BYTES=0: the dispatcher never takes the host path.
    Without a GPU (this container) the call then fails instead of computing;
    on a GPU box the GPU computes it (tests/test_gpu_shim.py)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present: covered by the GPU suite")
    env(CCL_COMP_HOST_MAX_BYTES="0")
    a = np.ones(64, np.float32)
    b = np.ones(64, np.float32)
    rc = _lib.shim().mi_ccl_comp_reduce(a.ctypes.data, 64, b.ctypes.data, None, FP32, 0)
    assert rc == -1 and np.all(b == 1.0)


@pytest.mark.parametrize("isa", ["avx2", "avx512"])
def test_narrower_isa_forms(isa):
    """The bf16/fp16 fold has three forms: 16 AVX-512 lanes with the native
    VCVTNEPS2BF16 (default where the CPU has AVX512_BF16), 16 lanes with the
    integer restatement, 8 AVX2 lanes.  The narrower ones, forced with
    MI_HOST_ISA, give the same bits (reference vectors and fan-in/keep-
    precision cases, in a child process)."""
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-p", "no:cacheprovider", str(Path(__file__)),
                        "-k", "matches_reference_code or fanin or keep_precision"],
                       cwd=str(root), env=dict(os.environ, MI_HOST_ISA=isa), capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert " passed" in r.stdout


def test_dropin_counts_host_bucket_workers(env):
    """The dispatcher counts the threads reducing host buckets (inside a call,
    or returned from one within the last 50 ms): the number of oneCCL workers
    it uses to decide whether a large pageable bucket may still be split with
    the GPU (CCL_COMP_HOST_SPLIT_WORKERS)."""
    import threading
    import time
    env()
    s = _lib.shim()
    time.sleep(0.06)  # earlier tests' callers leave the window
    assert s.mi_ccl_comp_host_workers() == 0
    w = 5
    go = threading.Barrier(w)
    errs = []

    def worker(seed):
        try:
            a = rand_array(FP32, 4096, seed=seed)
            b = rand_array(FP32, 4096, seed=seed + 1)
            exp = b.copy()
            oracle.comp_reduce(a, exp, FP32, 0)
            go.wait()
            comp.comp_reduce(a.ctypes.data, a.size, b.ctypes.data, comp.datatype.float32, comp.reduction.sum)
            assert_same(b, exp, FP32)
        except Exception as e:  # noqa: BLE001 - reported below
            errs.append(e)

    ts = [threading.Thread(target=worker, args=(10 * i,)) for i in range(w)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs
    assert s.mi_ccl_comp_host_workers() == w
    time.sleep(0.06)
    assert s.mi_ccl_comp_host_workers() == 0


@pytest.mark.parametrize("dt", [FP32, 4, 6, FP64], ids=["f32", "i32", "i64", "f64"])
@pytest.mark.parametrize("alias", [None, 0, 2])
def test_host_fanin_out_aliasing(dt, alias):
    """The K-input host fold is a function of the inputs' values before the
    call, wherever `out` points: a distinct buffer, input 0 (in place, the
    batch reduce's accumulator) or a later input (same bits as the GPU fan
    kernel, which loads every input before its store)."""
    k, n = 5, 5000 + 3
    ins = [rand_array(dt, n, seed=60 + j, specials=False) for j in range(k)]
    exp = ins[0].copy()
    for j in range(1, k):
        oracle.comp_reduce(ins[j], exp, dt, 0)
    bufs = [x.copy() for x in ins]
    out = np.zeros_like(ins[0]) if alias is None else bufs[alias]
    arr = (ctypes.c_void_p * k)(*[b.ctypes.data for b in bufs])
    assert _lib.shim().mi_host_reduce(arr, k, out.ctypes.data, n, dt, 0, 0) == 0
    assert_same(out, exp, dt, f"alias={alias}")


@pytest.mark.parametrize("op", [2, 3], ids=["min", "max"])
@pytest.mark.parametrize("k", [2, 3, 8])
def test_host_fp16_native_minmax_keeps_snan_inout(op, k):
    """CCL_FP16=avx512fp16 (MI_F_FP16_NATIVE_MINMAX): VMINPH/VMAXPH return a
    NaN accumulator as stored, a signalling one included; the fp32 route of
    the other impls quiets it.  Against the oracle with each impl."""
    from oneccl_amd.comp import F_FP16_NATIVE_MINMAX
    n = 1031
    rng = np.random.default_rng(5 + op + k)
    ins = [rand_array(FP16, n, seed=700 + j) for j in range(k)]
    snan = rng.choice(n, 64, replace=False)
    ins[0][snan] = (0x7C01 + rng.integers(0, 0x1FF, 64)) | (rng.integers(0, 2, 64) << 15)  # signalling NaNs
    for j in range(1, k):
        ins[j][rng.choice(n, 32, replace=False)] = 0x7E00  # quiet NaNs in the other inputs
    for impl, flags in ((oracle.FP16_AVX512F, F_MINMAX_INOUT_FIRST),
                        (oracle.FP16_AVX512FP16, F_MINMAX_INOUT_FIRST | F_FP16_NATIVE_MINMAX)):
        exp = ins[0].copy()
        for j in range(1, k):
            oracle.comp_reduce(ins[j], exp, FP16, op, oracle.BF16_AVX512BF, impl)
        for inplace in (False, True):
            bufs = [x.copy() for x in ins]
            out = bufs[0] if inplace else np.zeros_like(ins[0])
            arr = (ctypes.c_void_p * k)(*[b.ctypes.data for b in bufs])
            assert _lib.shim().mi_host_reduce(arr, k, out.ctypes.data, n, FP16, op, flags) == 0
            assert_same(out, exp, FP16, f"impl {impl} inplace {inplace}")
        if impl == oracle.FP16_AVX512FP16:
            assert np.array_equal(exp[snan], ins[0][snan])  # signalling, as stored
        else:
            assert np.array_equal(exp[snan], ins[0][snan] | 0x0200)  # quieted
