"""The drop-in src/comp (libccl_comp_hip.so: oneCCL's own ccl_comp_* entry
points over the HIP kernels) driven the way src/sched drives it —
synchronous calls on host staging buffers, device buffers or a mix — checked
against the oracle under the same bf16/fp16 impl types the shim selected
(CPUID + CCL_BF16 / CCL_FP16, src/common/env/env.cpp:711-720)."""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np
import pytest

import oracle
from oneccl_amd import _lib, comp
from tests import kat
from tests.util import ALL_DTYPES, BF16, DT_NAME, FP16, FP32, FP64, OP_NAME, OPS, assert_same, from_dev, rand_array, to_dev, \
    wait_os_threads_gone

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu_dispatch():
    """These tests drive the GPU paths (bounce buffers, staging, zero-copy) on
    host buffers too, so the dispatcher's CPU path for small host buckets is
    off here (CCL_COMP_HOST_MAX_BYTES=0, inherited by child processes);
    tests/test_host_reduce.py and tests/test_gpu_dispatch.py cover it."""
    saved = os.environ.get("CCL_COMP_HOST_MAX_BYTES")
    os.environ["CCL_COMP_HOST_MAX_BYTES"] = "0"
    comp.env_reload()
    yield
    if saved is None:
        os.environ.pop("CCL_COMP_HOST_MAX_BYTES", None)
    else:
        os.environ["CCL_COMP_HOST_MAX_BYTES"] = saved
    comp.env_reload()


@pytest.fixture(autouse=True)
def _reset_env():
    saved = {k: os.environ.get(k) for k in ("CCL_BF16", "CCL_FP16")}
    yield
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    comp.env_reload()


def impls():
    b, f = comp.impl_types()
    return int(b), int(f)


def ptr(a: np.ndarray) -> int:
    return a.ctypes.data


@pytest.mark.parametrize("dt", ALL_DTYPES, ids=[DT_NAME[d] for d in ALL_DTYPES])
@pytest.mark.parametrize("op", OPS, ids=[OP_NAME[o] for o in OPS])
def test_comp_reduce_host_buffers(dt, op):
    """recv_reduce_entry's call: host comm_buf into a host accumulator."""
    n = 32771
    b_impl, f_impl = impls()
    a = rand_array(dt, n, seed=11 + dt, op=op)
    b = rand_array(dt, n, seed=12 + dt, op=op)
    exp = b.copy()
    oc_ref = oracle.comp_reduce(a, exp, dt, op, b_impl, f_impl)
    oc = comp.comp_reduce(ptr(a), n, ptr(b), comp.datatype(dt), comp.reduction(op))
    assert_same(b, exp, dt)
    assert oc == oc_ref  # out_count written only by bf16/fp16 (bf16.cpp:94-96, fp16.cpp:48-50)


@pytest.mark.parametrize("where", ["device", "pinned", "in_host_inout_dev", "in_dev_inout_host"])
@pytest.mark.parametrize("dt", [FP32, BF16, FP16, 6])
def test_comp_reduce_pointer_kinds(where, dt):
    import torch
    n = 100_000
    b_impl, f_impl = impls()
    a = rand_array(dt, n, seed=3)
    b = rand_array(dt, n, seed=4)
    exp = b.copy()
    oracle.comp_reduce(a, exp, dt, 0, b_impl, f_impl)
    if where == "device":
        ta, pa = to_dev(a)
        tb, pb = to_dev(b)
        comp.comp_reduce(pa, n, pb, comp.datatype(dt), comp.reduction.sum)
        got = from_dev(tb, b)
    elif where == "pinned":
        ha = torch.from_numpy(a.view(np.uint8).copy()).pin_memory()
        hb = torch.from_numpy(b.view(np.uint8).copy()).pin_memory()
        comp.comp_reduce(ha.data_ptr(), n, hb.data_ptr(), comp.datatype(dt), comp.reduction.sum)
        got = hb.numpy().view(b.dtype)
    elif where == "in_host_inout_dev":
        tb, pb = to_dev(b)
        comp.comp_reduce(ptr(a), n, pb, comp.datatype(dt), comp.reduction.sum)
        got = from_dev(tb, b)
    else:
        ta, pa = to_dev(a)
        got = b.copy()
        comp.comp_reduce(pa, n, ptr(got), comp.datatype(dt), comp.reduction.sum)
    assert_same(got, exp, dt, where)


@pytest.mark.parametrize("dt,off_in,off_io", [(FP32, 1, 0), (BF16, 3, 6), (0, 5, 2), (FP64, 0, 1), (FP16, 7, 7)])
@pytest.mark.parametrize("mode", [0, 1], ids=["zero_copy", "staged"])
def test_pinned_host_differing_offsets(dt, off_in, off_io, mode):
    """Sub-buffers of pinned staging memory at element offsets whose
    addresses differ mod 16: the zero-copy kernel reads them over PCIe with
    unaligned 16-byte loads; the staged pipeline copies them first."""
    import torch
    n = (3 << 20) + 17
    b_impl, f_impl = impls()
    a = rand_array(dt, n, seed=71, specials=False)
    b = rand_array(dt, n, seed=72, specials=False)
    exp = b.copy()
    oracle.comp_reduce(a, exp, dt, 0, b_impl, f_impl)
    es = a.itemsize
    ha = torch.zeros((n + 16) * es, dtype=torch.uint8).pin_memory()
    hb = torch.zeros((n + 16) * es, dtype=torch.uint8).pin_memory()
    ha.numpy()[off_in * es:(off_in + n) * es] = a.view(np.uint8)
    hb.numpy()[off_io * es:(off_io + n) * es] = b.view(np.uint8)
    m = _lib.mi()
    prev = m.mi_set_host_mode(mode)
    try:
        comp.comp_reduce(ha.data_ptr() + off_in * es, n, hb.data_ptr() + off_io * es, comp.datatype(dt),
                         comp.reduction.sum)
    finally:
        m.mi_set_host_mode(prev)
    got = hb.numpy()[off_io * es:(off_io + n) * es].view(b.dtype)
    assert_same(got, exp, dt)


@pytest.mark.parametrize("mode", [0, 1], ids=["zero_copy", "staged"])
@pytest.mark.parametrize("dt", [FP32, BF16, 4])
def test_pinned_host_modes(mode, dt):
    """Pinned host operands: zero-copy kernel over PCIe (default) or the staged
    H2D / kernel / D2H pipeline — same bits."""
    import torch
    n = (40 << 20) // 4 + 77
    b_impl, f_impl = impls()
    a = rand_array(dt, n, seed=61, specials=False)
    b = rand_array(dt, n, seed=62, specials=False)
    exp = b.copy()
    oracle.comp_reduce_mt(a, exp, dt, 0, 8, b_impl, f_impl)
    ha = torch.from_numpy(a.view(np.uint8).copy()).pin_memory()
    hb = torch.from_numpy(b.view(np.uint8).copy()).pin_memory()
    m = _lib.mi()
    prev = m.mi_set_host_mode(mode)
    try:
        comp.comp_reduce(ha.data_ptr() + 0, n, hb.data_ptr(), comp.datatype(dt), comp.reduction.sum)
    finally:
        m.mi_set_host_mode(prev)
    assert_same(hb.numpy().view(b.dtype), exp, dt)


@pytest.mark.parametrize("dt", [FP32, BF16])
def test_large_host_buffer_pipelined(dt):
    """> 1 staging chunk (32 MiB): the H2D / kernel / D2H pipeline over two
    streams must produce the whole-array result."""
    n = (80 << 20) // 4 + 12345
    b_impl, f_impl = impls()
    a = rand_array(dt, n, seed=21, specials=False)
    b = rand_array(dt, n, seed=22, specials=False)
    exp = b.copy()
    oracle.comp_reduce_mt(a, exp, dt, 0, 8, b_impl, f_impl)
    comp.comp_reduce(ptr(a), n, ptr(b), comp.datatype(dt), comp.reduction.sum)
    assert_same(b, exp, dt)


@pytest.mark.parametrize("setting,impl", [("scalar", 0), ("avx512f", 1), ("avx512bf", 2)])
def test_ccl_bf16_env_selects_semantics(setting, impl):
    """CCL_BF16=<impl> (doc/rst/source/env-variables.rst CCL_BF16) changes the
    bit-level result exactly as it changes the reference's."""
    os.environ["CCL_BF16"] = setting
    comp.env_reload()
    assert impls()[0] == impl
    n = 4099
    for op in OPS:
        a = rand_array(BF16, n, seed=40 + op, op=op)
        b = rand_array(BF16, n, seed=50 + op, op=op)
        exp = b.copy()
        oracle.comp_reduce(a, exp, BF16, op, impl)
        comp.comp_reduce(ptr(a), n, ptr(b), comp.datatype.bfloat16, comp.reduction(op))
        assert_same(b, exp, BF16, f"{setting} {OP_NAME[op]}")


def test_bad_env_value_throws():
    os.environ["CCL_BF16"] = "avx9000"
    with pytest.raises(_lib.MiReduceError):
        comp.env_reload()


def test_bf16_fp16_entry_points():
    """ccl_bf16_reduce / ccl_fp16_reduce: the MPI user-op entries
    (src/atl/mpi/atl_mpi_ctx.cpp:58-124)."""
    s = _lib.shim()
    b_impl, f_impl = impls()
    n = 1000
    for dt, fn in ((BF16, s.mi_ccl_bf16_reduce), (FP16, s.mi_ccl_fp16_reduce)):
        a = rand_array(dt, n, seed=1)
        b = rand_array(dt, n, seed=2)
        exp = b.copy()
        oracle.comp_reduce(a, exp, dt, 3, b_impl, f_impl)
        oc = ctypes.c_size_t(0)
        _lib.check_shim(fn(ptr(a), n, ptr(b), ctypes.byref(oc), 3))
        assert oc.value == n
        assert_same(b, exp, dt)
    # custom / unknown ops abort the process as the reference's CCL_FATAL does: tests/test_fatal.py


@pytest.mark.parametrize("keep", [0, 1])
@pytest.mark.parametrize("k", [1, 2, 5, 16, 23])
@pytest.mark.parametrize("dt", [BF16, FP32, FP16])
def test_comp_batch_reduce(keep, k, dt):
    """Storage-precision folds chain groups of 16; keep-precision past 16
    inputs runs the reference's fp32 scratch chain (comp.cpp:214-234)."""
    if keep and dt != BF16:
        pytest.skip("keep-precision mode reads bf16")
    n = 4099
    b_impl, f_impl = impls()
    ins = [rand_array(dt, n, seed=300 + j) for j in range(k)]
    packed = np.concatenate(ins)
    offsets = [j * n for j in range(k)]
    exp = ins[0].copy()
    oc_ref = oracle.batch_reduce(packed, offsets, n, exp, dt, 0, keep, b_impl, f_impl)
    got = ins[0].copy()
    oc = comp.comp_batch_reduce(ptr(packed), offsets, n, ptr(got), comp.datatype(dt), comp.reduction.sum, keep)
    assert_same(got, exp, dt)
    assert oc == oc_ref


def test_custom_reduction_callback():
    """reduction::custom calls the user's fn on host memory (comp.cpp:84-88);
    device operands are staged through the host (comp.cpp:136-195)."""
    calls = []

    def fn(in_p, count, inout_p, out_count_p, dtype, ctx):
        calls.append((count, dtype))
        src = np.ctypeslib.as_array(ctypes.cast(in_p, ctypes.POINTER(ctypes.c_float)), (count,))
        dst = np.ctypeslib.as_array(ctypes.cast(inout_p, ctypes.POINTER(ctypes.c_float)), (count,))
        dst[:] = dst * 2 + src

    cb = _lib.MI_CCL_REDUCTION_FN(fn)
    n = 1000
    a = np.arange(n, dtype=np.float32)
    b = np.ones(n, np.float32)
    oc = ctypes.c_size_t(0)
    _lib.check_shim(_lib.shim().mi_ccl_comp_reduce_custom(ptr(a), n, ptr(b), ctypes.byref(oc), FP32, cb))
    assert np.array_equal(b, 2 + a)
    ta, pa = to_dev(a)
    tb, pb = to_dev(np.ones(n, np.float32))
    _lib.check_shim(_lib.shim().mi_ccl_comp_reduce_custom(pa, n, pb, ctypes.byref(oc), FP32, cb))
    assert np.array_equal(from_dev(tb, b), 2 + a)
    assert calls == [(n, FP32), (n, FP32)]
    null_fn = ctypes.cast(None, _lib.MI_CCL_REDUCTION_FN)
    assert _lib.shim().mi_ccl_comp_reduce_custom(ptr(a), n, ptr(b), None, FP32, null_fn) == -1
    assert b"callback" in _lib.shim().mi_ccl_last_error()


@pytest.mark.parametrize("cap", [0, 3], ids=["lean", "capped"])
@pytest.mark.parametrize("nt", [0, 1])
def test_comp_copy_any_offsets(nt, cap):
    """ccl_comp_copy between device buffers at every byte offset pair mod 16
    and odd sizes: the copy kernel on the destination's 16-byte grid, as the
    one-tile-per-block kernel (default) and the grid-stride one (a grid cap)."""
    import torch
    m = _lib.mi()
    rng = np.random.default_rng(5)
    src = torch.from_numpy(rng.integers(0, 256, 1 << 20, dtype=np.uint8)).cuda()
    ref = src.cpu().numpy()
    _lib.check(m.mi_set_max_blocks(cap))
    try:
        for so in (0, 1, 3, 4, 8, 15):
            for do in (0, 2, 5, 12):
                for n in (1, 15, 16, 17, 8191, 8193, 4099, (1 << 19) + 3):
                    dst = torch.zeros(n + 64, dtype=torch.uint8, device="cuda")
                    torch.cuda.synchronize()  # the fill runs on torch's stream, the copy on the library's
                    comp.comp_copy(src.data_ptr() + so, dst.data_ptr() + do, n, bool(nt))
                    got = dst.cpu().numpy()
                    assert np.array_equal(got[do:do + n], ref[so:so + n]), (so, do, n)
                    assert not got[:do].any() and not got[do + n:].any(), (so, do, n)
    finally:
        _lib.check(m.mi_set_max_blocks(0))


@pytest.mark.parametrize("nt", [0, 1])
@pytest.mark.parametrize("so,do", [(0, 0), (3, 0), (0, 5), (7, 12), (4, 8)])
def test_comp_copy_streaming_sizes(nt, so, do):
    """Copies of 64 MiB and more store through per-tile buffer descriptors
    with sc1 + nt and no residency cap (mi_reduce.hip kCopyStreamBytes):
    every byte at shifted offsets, nothing written outside the destination,
    at the threshold, one byte under it and past it with a ragged tail."""
    import torch
    base = 64 << 20
    src = torch.randint(0, 256, (base + 4096,), dtype=torch.uint8, device="cuda")
    for n in (base - 1, base, base + 1029):
        dst = torch.zeros(n + 64, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()  # the fills run on torch's stream, the copy on the library's
        comp.comp_copy(src.data_ptr() + so, dst.data_ptr() + do, n, bool(nt))
        assert torch.equal(dst[do:do + n], src[so:so + n]), (so, do, n)
        assert not dst[:do].any() and not dst[do + n:].any(), (so, do, n)
        del dst


@pytest.mark.parametrize("nt", [0, 1])
def test_comp_copy(nt):
    import torch
    n = (5 << 20) + 3
    src = np.random.default_rng(1).integers(0, 255, n, dtype=np.uint8)
    dst = np.zeros_like(src)
    comp.comp_copy(ptr(src), ptr(dst), n, bool(nt))
    assert np.array_equal(src, dst)
    td = torch.zeros(n, dtype=torch.uint8, device="cuda")
    td2 = torch.zeros_like(td)
    torch.cuda.synchronize()  # the fills run on torch's stream, the copies on the library's
    comp.comp_copy(ptr(src), td.data_ptr(), n, bool(nt))
    comp.comp_copy(td.data_ptr(), td2.data_ptr(), n - 16, bool(nt))
    comp.comp_copy(td.data_ptr() + n - 16, td2.data_ptr() + n - 16, 16, bool(nt))
    assert np.array_equal(td2.cpu().numpy(), src)
    comp.comp_copy(0, 0, 0)  # bytes == 0 is success (comp.cpp:61-63)


def test_concurrent_worker_threads():
    """Up to CCL_WORKER_COUNT worker threads call ccl_comp_reduce at once
    (src/exec/thread/worker.cpp:310-379): per-thread streams and scratch."""
    b_impl, f_impl = impls()
    n = 3_000_001
    jobs = []
    for t in range(6):
        dt = [FP32, BF16, 4][t % 3]
        a = rand_array(dt, n, seed=t)
        b = rand_array(dt, n, seed=100 + t)
        exp = b.copy()
        oracle.comp_reduce(a, exp, dt, 0, b_impl, f_impl)
        jobs.append((dt, a, b, exp))
    errs = []

    def work(job):
        dt, a, b, _ = job
        try:
            comp.comp_reduce(ptr(a), n, ptr(b), comp.datatype(dt), comp.reduction.sum)
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=work, args=(j,)) for j in jobs]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs
    for dt, a, b, exp in jobs:
        assert_same(b, exp, dt)


FUNCTIONAL = [c for c in kat.load() if c["suite"] == "tests/functional"]


@pytest.mark.parametrize("case", FUNCTIONAL, ids=[f"dt{c['dtype']}-{OP_NAME[c['op']]}-P{c['P']}-b{c['buf_idx']}"
                                                  for c in FUNCTIONAL])
def test_reference_functional_kats_through_dropin(case):
    """oneCCL's tests/functional allreduce KATs with every local reduce done
    by the drop-in ccl_comp_reduce on the GPU."""
    dt = case["dtype"]
    b_impl, _ = impls()

    def reduce2(a, b):
        comp.comp_reduce(ptr(a), a.size, ptr(b), comp.datatype(dt), comp.reduction(case["op"]))

    for count in case["counts"]:
        err, tol = kat.functional_case(case, count, reduce2, bf16_rne=(b_impl == 2))
        assert err <= tol


def test_reference_example_kats_through_dropin():
    b_impl, _ = impls()
    for c in kat.load():
        if c["suite"] == "examples/cpu/cpu_allreduce_bf16_test":
            assert kat.bf16_example_case(
                c, lambda a, b: comp.comp_reduce(ptr(a), a.size, ptr(b), comp.datatype.bfloat16, comp.reduction.sum),
                b_impl == 2)
        elif c["suite"] == "examples/benchmark":
            assert kat.benchmark_case(
                c, lambda a, b: comp.comp_reduce(ptr(a), a.size, ptr(b), comp.datatype.float32, comp.reduction.sum))


def test_cpp_caller_links_dropin_by_mangled_names():
    """A C++ program written like src/sched's call sites links
    libccl_comp_hip.so and runs host and device reduces through it."""
    import subprocess
    from pathlib import Path
    exe = Path(__file__).resolve().parent / "cpp" / "dropin_caller"
    if not exe.exists():
        from oneccl_amd import build
        build.build_dropin_caller()
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "dropin_caller: ok" in r.stdout


def test_cpp_caller_under_host_asan():
    """Host AddressSanitizer over the product's host code (staging pipeline,
    zero-copy, fan-in chaining, conversions): the drop-in caller linked
    against -Xarch_host -fsanitize=address builds of both libraries.  Device
    code is not instrumented (GPU ASan is not available on this pool)."""
    import os
    import subprocess
    from pathlib import Path
    exe = Path(__file__).resolve().parent / "cpp" / "dropin_caller_asan"
    if not exe.exists():
        # The ASan builds stay out of the GPU push (.gpurunignore); they are
        # built on the box by `tools/gpu_run.sh asan` (python -m
        # oneccl_amd.build --asan) before this test runs there.
        pytest.skip("host-ASan build absent: run `python -m oneccl_amd.build --asan` first")
    # quarantine_size_mb=0: ROCm's ASan runtime tracks pinned host memory
    # (hipHostMalloc) in its device allocator, and a freed pinned chunk still
    # in quarantine when libamdhip64 unloads at exit trips the runtime's own
    # CHECK (sanitizer_allocator_device.h: dev_runtime_unloaded_).  Without a
    # quarantine it is returned at once, while the runtime is alive.
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:halt_on_error=1:quarantine_size_mb=0")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert "dropin_caller: ok" in r.stdout


@pytest.mark.parametrize("dt", [FP32, BF16])
def test_registered_staging_buffer_takes_zero_copy(dt):
    """A pageable staging buffer registered once (what oneCCL's buffer cache
    would do) is classified pinned and reduced in place."""
    import time
    m = _lib.mi()
    n = (64 << 20) // 4 + 3
    b_impl, f_impl = impls()
    a = rand_array(dt, n, seed=81, specials=False)
    b = rand_array(dt, n, seed=82, specials=False)
    exp = b.copy()
    oracle.comp_reduce_mt(a, exp, dt, 0, 8, b_impl, f_impl)
    dev = ctypes.c_int(-1)
    assert m.mi_pointer_kind(ptr(b), ctypes.byref(dev)) == 2  # pageable
    t0 = time.perf_counter()
    _lib.check(m.mi_host_register(ptr(a), a.nbytes))
    _lib.check(m.mi_host_register(ptr(b), b.nbytes))
    t_reg = time.perf_counter() - t0
    try:
        assert m.mi_pointer_kind(ptr(b), ctypes.byref(dev)) == 1  # now pinned
        comp.comp_reduce(ptr(a), n, ptr(b), comp.datatype(dt), comp.reduction.sum)
        assert_same(b, exp, dt)
    finally:
        _lib.check(m.mi_host_unregister(ptr(a)))
        _lib.check(m.mi_host_unregister(ptr(b)))
    assert m.mi_pointer_kind(ptr(b), ctypes.byref(dev)) == 2
    assert t_reg < 30.0


# ---- asynchronous ccl_comp_reduce (include/mi_ccl_comp_async.hpp, §8f rank 4)

def _poll(req, limit_s=60.0):
    """A worker's progress loop: poll update() until the entry completes."""
    import time
    t0 = time.perf_counter()
    while not req.test():
        assert time.perf_counter() - t0 < limit_s, "async reduce did not complete"


@pytest.mark.parametrize("where", ["device", "pinned", "pageable"])
@pytest.mark.parametrize("dt", [FP32, BF16, FP16, 6])
@pytest.mark.parametrize("op", OPS, ids=[OP_NAME[o] for o in OPS])
def test_comp_reduce_start_matches_sync(where, dt, op):
    """start + test polling gives the bits and out_count of ccl_comp_reduce."""
    import torch
    n = 70_001
    b_impl, f_impl = impls()
    a = rand_array(dt, n, seed=31 + op, op=op)
    b = rand_array(dt, n, seed=41 + op, op=op)
    exp = b.copy()
    oc_ref = oracle.comp_reduce(a, exp, dt, op, b_impl, f_impl)
    keep = []
    if where == "device":
        ta, pa = to_dev(a)
        tb, pb = to_dev(b)
        keep += [ta, tb]
    elif where == "pinned":
        ha = torch.from_numpy(a.view(np.uint8).copy()).pin_memory()
        hb = torch.from_numpy(b.view(np.uint8).copy()).pin_memory()
        pa, pb = ha.data_ptr(), hb.data_ptr()
    else:
        hb = b.copy()
        pa, pb = ptr(a), ptr(hb)
    req = comp.comp_reduce_start(pa, n, pb, comp.datatype(dt), comp.reduction(op))
    try:
        _poll(req)
    finally:
        req.free()
    if where == "device":
        got = from_dev(tb, b)
    elif where == "pinned":
        got = hb.numpy().view(b.dtype)
    else:
        got = hb
    assert_same(got, exp, dt, where)
    assert req.out_count == oc_ref


def test_comp_reduce_start_many_in_flight():
    """Eight entries started before any is polled (one worker's queue), each
    on its own device buffers; all complete with the right bits."""
    n = (4 << 20) + 5
    jobs = []
    for e in range(8):
        dt = [FP32, BF16, 4, 6][e % 4]
        a = rand_array(dt, n, seed=200 + e, specials=False)
        b = rand_array(dt, n, seed=300 + e, specials=False)
        exp = b.copy()
        b_impl, f_impl = impls()
        oracle.comp_reduce_mt(a, exp, dt, 0, 8, b_impl, f_impl)
        ta, pa = to_dev(a)
        tb, pb = to_dev(b)
        jobs.append((dt, b, exp, ta, tb, comp.comp_reduce_start(pa, n, pb, comp.datatype(dt), comp.reduction.sum)))
    pending = [j[-1] for j in jobs]
    import time
    t0 = time.perf_counter()
    while pending:
        pending = [r for r in pending if not r.test()]
        assert time.perf_counter() - t0 < 60
    for dt, b, exp, ta, tb, req in jobs:
        req.free()
        assert_same(from_dev(tb, b), exp, dt)


def test_comp_reduce_start_custom_and_empty_complete_at_start():
    """Custom ops run the user callback inside start (host code, comp.cpp:84-88);
    in_count == 0 does nothing (comp.cpp:132-134): both requests are complete
    on return."""
    n = 1000
    a = np.arange(n, dtype=np.float32)
    b = np.ones(n, dtype=np.float32)
    calls = []

    def fn(in_p, count, inout_p, out_count, dtype, ctx):
        calls.append(count)
        src = np.ctypeslib.as_array(ctypes.cast(in_p, ctypes.POINTER(ctypes.c_float)), (count,))
        dst = np.ctypeslib.as_array(ctypes.cast(inout_p, ctypes.POINTER(ctypes.c_float)), (count,))
        dst += 2 * src

    req = comp.comp_reduce_start(ptr(a), n, ptr(b), comp.datatype.float32, comp.reduction.custom, fn=fn)
    assert req.test()
    req.free()
    assert calls == [n] and np.array_equal(b, 1 + 2 * a)
    b2 = np.full(n, 7, np.float32)
    req = comp.comp_reduce_start(ptr(a), 0, ptr(b2), comp.datatype.float32, comp.reduction.sum)
    assert req.test()
    req.wait()
    req.free()
    assert (b2 == 7).all()
    with pytest.raises(_lib.MiReduceError):  # custom without a callback (comp.cpp:85)
        comp.comp_reduce_start(ptr(a), n, ptr(b), comp.datatype.float32, comp.reduction.custom)


def test_comp_request_free_waits_for_pending():
    """Freeing a request still in flight waits for it, so the buffer is never
    written after its owner reclaims it."""
    n = (256 << 20) // 4
    import torch
    x = torch.full((n,), 1.5, device="cuda")
    y = torch.full((n,), 2.0, device="cuda")
    torch.cuda.synchronize()
    req = comp.comp_reduce_start(x.data_ptr(), n, y.data_ptr(), comp.datatype.float32, comp.reduction.sum)
    req.free()
    assert bool((y == 3.5).all())


def test_roctx_range_around_reduce(tmp_path):
    """The ITT event the reference puts around ccl_comp_reduce_regular
    (comp.cpp:90-93) is a roctx range here: `rocprofv3 --marker-trace` records
    comp_reduce_regular and comp_batch_reduce ranges from the drop-in, under
    the reference's own knob (CCL_ITT_LEVEL > 0; off by default, as there)."""
    import os
    import shutil
    import subprocess
    import sys
    from pathlib import Path
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not Path(prof).exists():
        pytest.skip("rocprofv3 not installed")
    root = Path(__file__).resolve().parent.parent
    code = ("import sys; sys.path.insert(0, %r)\n"
            "import numpy as np\n"
            "from oneccl_amd import comp\n"
            "a = np.ones(4096, np.float32); b = np.ones(4096, np.float32)\n"
            "for _ in range(3): comp.comp_reduce(a.ctypes.data, a.size, b.ctypes.data, comp.datatype.float32, "
            "comp.reduction.sum)\n"
            "p = np.ones(3 * 64, np.float32); o = p[:64].copy()\n"
            "comp.comp_batch_reduce(p.ctypes.data, [0, 64, 128], 64, o.ctypes.data, comp.datatype.float32, "
            "comp.reduction.sum)\n"
            "assert (b == 4).all() and (o == 3).all()\n") % str(root)
    env = dict(os.environ, TMPDIR="/tmp", CCL_ITT_LEVEL="1")
    env.pop("MI_ROCTX", None)
    r = subprocess.run([prof, "--marker-trace", "--output-format", "csv", "-d", str(tmp_path), "-o", "trace", "--",
                        sys.executable, "-c", code], cwd="/tmp", env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    text = "".join(p.read_text(errors="replace") for p in tmp_path.rglob("*.csv"))
    assert text.count("comp_reduce_regular") >= 3, (r.stdout + r.stderr)[-2000:]
    assert "comp_batch_reduce" in text


@pytest.mark.parametrize("where", ["device", "pageable"])
@pytest.mark.parametrize("dt,op,k,keep", [(FP32, 0, 5, 0), (FP32, 3, 23, 0), (BF16, 0, 4, 1), (BF16, 2, 9, 0),
                                          (4, 1, 17, 0), (FP16, 0, 3, 0), (BF16, 3, 19, 1)])
def test_comp_batch_reduce_start_matches_sync(where, dt, op, k, keep):
    """ccl_comp_batch_reduce_start (one request; chained launches past 16
    inputs) gives the bits and out_count of the synchronous
    ccl_comp_batch_reduce, which the parity suite pins to the oracle."""
    n = 40_001
    es = oracle.NP_DTYPE[dt]().itemsize
    packed = np.concatenate([rand_array(dt, n, seed=500 + j + 37 * dt, op=op) for j in range(k)])
    offs = [j * n for j in range(k)]
    ref = packed[:n].copy()
    oc_ref = comp.comp_batch_reduce(ptr(packed), offs, n, ptr(ref), comp.datatype(dt), comp.reduction(op), keep)
    if where == "device":
        tp, pp = to_dev(packed)
        to, po = to_dev(packed[:n].copy())
    else:
        host = packed[:n].copy()
        pp, po = ptr(packed), ptr(host)
    req = comp.comp_batch_reduce_start(pp, offs, n, po, comp.datatype(dt), comp.reduction(op), keep)
    try:
        _poll(req)
    finally:
        req.free()
    got = from_dev(to, ref) if where == "device" else host
    assert_same(got, ref, dt)
    assert req.out_count == oc_ref
    assert es == ref.itemsize


def test_concurrent_worker_stress():
    """16 worker threads (CCL_WORKER_COUNT-style), each running 40 reduces that
    mix pointer kinds (device, pinned, pageable), dtypes, ops, synchronous and
    asynchronous entry points and fused fan-ins, concurrently; every result
    checked against the oracle."""
    import threading

    import torch
    b_impl, f_impl = impls()
    errs = []
    tids = []
    n = 33_333

    def worker(t):
        tids.append(threading.get_native_id())
        try:
            rng = np.random.default_rng(t)
            for it in range(40):
                dt = [FP32, BF16, FP16, 4, 6, 0][int(rng.integers(0, 6))]
                op = int(rng.integers(0, 4))
                a = rand_array(dt, n, seed=1000 * t + it, op=op, specials=False)
                b = rand_array(dt, n, seed=1000 * t + it + 500, op=op, specials=False)
                exp = b.copy()
                oracle.comp_reduce(a, exp, dt, op, b_impl, f_impl)
                kind = int(rng.integers(0, 3))
                if kind == 0:
                    ta, pa = to_dev(a)
                    tb, pb = to_dev(b)
                elif kind == 1:
                    ha = torch.from_numpy(a.view(np.uint8).copy()).pin_memory()
                    hb = torch.from_numpy(b.view(np.uint8).copy()).pin_memory()
                    pa, pb = ha.data_ptr(), hb.data_ptr()
                else:
                    hbuf = b.copy()
                    pa, pb = ptr(a), ptr(hbuf)
                if rng.random() < 0.5:
                    comp.comp_reduce(pa, n, pb, comp.datatype(dt), comp.reduction(op))
                else:
                    req = comp.comp_reduce_start(pa, n, pb, comp.datatype(dt), comp.reduction(op))
                    req.wait()
                    req.free()
                got = from_dev(tb, b) if kind == 0 else (hb.numpy().view(b.dtype) if kind == 1 else hbuf)
                assert_same(got, exp, dt, f"thread {t} iter {it} kind {kind}")
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(16)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=240)
    assert not any(x.is_alive() for x in th), "a worker did not finish"
    assert wait_os_threads_gone(tids), "a worker's thread teardown did not finish"
    assert not errs, errs[:3]


@pytest.mark.parametrize("k", [3, 16, 17])
@pytest.mark.parametrize("n", [1000, 70_001, (3 << 20) // 4 + 5])
@pytest.mark.parametrize("dt,op", [(FP32, 0), (BF16, 3), (0, 1)])
def test_batch_reduce_pageable_vs_oracle(k, n, dt, op):
    """ccl_comp_batch_reduce on pageable host memory (oneCCL's tmp buffer
    holding the peers' chunks): small buckets through the pinned bounce
    buffers, larger ones through the staged pipeline; chained past 16 inputs."""
    b_impl, f_impl = impls()
    ins = [rand_array(dt, n, seed=40 + 3 * j + dt, op=op) for j in range(k)]
    exp = oracle.fanin(ins, dt, op, b_impl, f_impl)
    packed = np.concatenate(ins)
    io = ins[0].copy()
    comp.comp_batch_reduce(ptr(packed), [j * n for j in range(k)], n, ptr(io), comp.datatype(dt), comp.reduction(op))
    assert_same(io, exp, dt)


@pytest.mark.parametrize("dt", [FP32, BF16, 4])
def test_shard_devices_env(dt):
    """CCL_COMP_HIP_SHARD_DEVICES splits host-resident reduces over the listed
    GPUs (here the one GPU twice and three times): same bits on pageable,
    pinned and device buffers (device operands never shard), and through the
    fused batch reduce."""
    import os

    import torch
    b_impl, f_impl = impls()
    n = (6 << 20) // 4 + 77
    for devs in ("0,0", "0,0,0"):
        os.environ["CCL_COMP_HIP_SHARD_DEVICES"] = devs
        comp.env_reload()
        try:
            a = rand_array(dt, n, seed=5, specials=False)
            b = rand_array(dt, n, seed=6, specials=False)
            exp = b.copy()
            oracle.comp_reduce(a, exp, dt, 0, b_impl, f_impl)
            got = b.copy()
            comp.comp_reduce(ptr(a), n, ptr(got), comp.datatype(dt), comp.reduction.sum)
            assert_same(got, exp, dt, f"pageable {devs}")
            ha = torch.from_numpy(a.view(np.uint8).copy()).pin_memory()
            hb = torch.from_numpy(b.view(np.uint8).copy()).pin_memory()
            comp.comp_reduce(ha.data_ptr(), n, hb.data_ptr(), comp.datatype(dt), comp.reduction.sum)
            assert_same(hb.numpy().view(b.dtype), exp, dt, f"pinned {devs}")
            ta, pa = to_dev(a)
            tb, pb = to_dev(b)
            comp.comp_reduce(pa, n, pb, comp.datatype(dt), comp.reduction.sum)
            assert_same(from_dev(tb, b), exp, dt, f"device {devs}")
            k = 5
            ins = [rand_array(dt, n, seed=70 + j, specials=False) for j in range(k)]
            fexp = oracle.fanin(ins, dt, 0, b_impl, f_impl)
            packed = np.concatenate(ins)
            io = ins[0].copy()
            comp.comp_batch_reduce(ptr(packed), [j * n for j in range(k)], n, ptr(io), comp.datatype(dt),
                                   comp.reduction.sum)
            assert_same(io, fexp, dt, f"batch {devs}")
        finally:
            os.environ.pop("CCL_COMP_HIP_SHARD_DEVICES", None)
            comp.env_reload()


@pytest.mark.parametrize("where", ["device", "pageable"])
@pytest.mark.parametrize("k,op", [(17, 0), (33, 2), (20, 3)])
def test_keep_precision_past_16_inputs(where, k, op):
    """ccl_comp_batch_reduce(bf16_keep_precision_mode=1) with more inputs than
    one fused pass takes: the fp32 scratch chain of the reference (convert,
    float32 reduce per input, one final rounding) against the oracle's
    restatement of comp.cpp:214-234, under the impl in force, with the
    caller's tmp/acc scratch absent (host scratch is allocated)."""
    b_impl, _ = impls()
    n = 4099  # count % 16 == 3: the truncated tail of the final conversion
    ins = [rand_array(BF16, n, seed=800 + j, op=op) for j in range(k)]
    packed = np.concatenate(ins)
    offsets = [j * n for j in range(k)]
    exp = ins[0].copy()
    oracle.batch_reduce(packed, offsets, n, exp, BF16, op, 1, b_impl, 0)
    if where == "device":
        tp, pp = to_dev(packed)
        to, po = to_dev(ins[0])
    else:
        host = ins[0].copy()
        pp, po = ptr(packed), ptr(host)
    oc = comp.comp_batch_reduce(pp, offsets, n, po, comp.datatype.bfloat16, comp.reduction(op), 1)
    got = from_dev(to, exp) if where == "device" else host
    assert_same(got, exp, BF16, f"k={k}")
    assert oc is None  # float32 CCL_REDUCE steps never write out_count


def test_keep_precision_custom_reduction():
    """keep-precision with reduction::custom: the user's callback runs on the
    fp32 scratch once per input, with datatype float32, and the result is
    rounded to bf16 once at the end (comp.cpp:214-234)."""
    calls = []

    def fn(in_p, count, inout_p, out_count_p, dtype, ctx):
        calls.append(dtype)
        src = np.ctypeslib.as_array(ctypes.cast(in_p, ctypes.POINTER(ctypes.c_float)), (count,))
        dst = np.ctypeslib.as_array(ctypes.cast(inout_p, ctypes.POINTER(ctypes.c_float)), (count,))
        dst[:] = np.maximum(dst, src) + np.float32(0.001)

    cb = _lib.MI_CCL_REDUCTION_FN(fn)
    n, k = 67, 3
    ins = [oracle.f32_to_bf16(np.linspace(j, j + 1, n, dtype=np.float32), True) for j in range(k)]
    packed = np.concatenate(ins)
    offs = (ctypes.c_size_t * k)(*[j * n for j in range(k)])
    b_impl, _ = impls()
    acc = oracle.bf16_to_f32(ins[0]).copy()
    for j in range(1, k):
        acc = np.maximum(acc, oracle.bf16_to_f32(ins[j])) + np.float32(0.001)
    exp = np.empty(n, np.uint16)
    oracle.lib().orc_convert_fp32_to_bf16_arrays(acc.ctypes.data, exp.ctypes.data, n, b_impl)
    for where in ("host", "device"):
        calls.clear()
        if where == "host":
            got = ins[0].copy()
            pp, po = ptr(packed), ptr(got)
        else:
            tp, pp = to_dev(packed)
            to, po = to_dev(ins[0])
        _lib.check_shim(_lib.shim().mi_ccl_comp_batch_reduce_custom(pp, offs, k, n, po, None, BF16, 1, cb))
        if where == "device":
            got = from_dev(to, exp)
        assert calls == [FP32] * (k - 1)
        assert_same(got, exp, BF16, where)
    null_fn = ctypes.cast(None, _lib.MI_CCL_REDUCTION_FN)
    assert _lib.shim().mi_ccl_comp_batch_reduce_custom(ptr(packed), offs, k, n, ptr(ins[0].copy()), None, BF16, 1,
                                                       null_fn) == -1
    assert b"callback" in _lib.shim().mi_ccl_last_error()


_EXIT_RACE = r'''
import sys, threading
import numpy as np
sys.path.insert(0, sys.argv[1])
from oneccl_amd import comp
n = (40 << 20) // 4
def work(i):
    a = np.full(n, 1.0, np.float32)
    b = np.full(n, float(i), np.float32)
    comp.comp_reduce(a.ctypes.data, n, b.ctypes.data, comp.datatype.float32, comp.reduction.sum)
    assert b[0] == i + 1.0 and b[-1] == i + 1.0
ts = [threading.Thread(target=work, args=(i,)) for i in range(12)]
for t in ts: t.start()
for t in ts: t.join()
print("exit-race: ok", flush=True)
'''


def test_process_exit_while_worker_threads_tear_down():
    """Worker threads that staged pageable buckets through the GPU free their
    contexts (hipFree of staging buffers) in thread_local destructors, which
    Python's Thread.join() does not wait for; the process then exits at once.
    Before the library's exit handler this died with SIGSEGV inside
    libamdhip64 (profiles/round2_dispatch/exit_crash_trace.txt)."""
    import subprocess
    import sys
    from pathlib import Path
    root = str(Path(__file__).resolve().parent.parent)
    env = dict(os.environ, CCL_COMP_HOST_MAX_BYTES="0")  # every bucket through the GPU's staging path
    for _ in range(2):
        r = subprocess.run([sys.executable, "-c", _EXIT_RACE, root], capture_output=True, text=True, timeout=120,
                           env=env)
        assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
        assert "exit-race: ok" in r.stdout


# A thread leaves asynchronous pageable requests un-waited and returns; the
# main thread exits at once.  The thread's staging worker finishes the
# requests (HIP calls) from the thread's thread_local destructor while the
# process runs its exit handlers.  The buffers come from libc malloc and are
# never freed, so they outlive Python's own teardown.
_EXIT_ASYNC = r'''
import ctypes, sys, threading
sys.path.insert(0, sys.argv[1])
from oneccl_amd import _lib, comp
libc = ctypes.CDLL(None)
libc.malloc.restype = ctypes.c_void_p
libc.malloc.argtypes = [ctypes.c_size_t]
libc.memset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
n = (48 << 20) // 4
def work():
    for i in range(3):
        a = libc.malloc(n * 4); b = libc.malloc(n * 4)
        libc.memset(a, 0x3F, n * 4); libc.memset(b, 0x3F, n * 4)
        comp.comp_reduce_start(a, n, b, comp.datatype.float32, comp.reduction.sum)  # never waited or freed
t = threading.Thread(target=work)
t.start()
t.join()
print("exit-async: ok", flush=True)
'''


def test_process_exit_with_unwaited_async_requests():
    """process exit while a thread's staging worker still runs
    its un-waited asynchronous requests (profiles/round2_dispatch/
    exit_crash_trace.txt).  The exit handler waits for every job in progress
    (bounded by MI_REDUCE_EXIT_WAIT_S, tests/test_exit_guard.py); jobs not yet
    started are dropped."""
    import subprocess
    import sys
    from pathlib import Path
    root = str(Path(__file__).resolve().parent.parent)
    env = dict(os.environ, CCL_COMP_HOST_MAX_BYTES="0")  # the GPU alone: every request staged on the worker
    r = subprocess.run([sys.executable, "-c", _EXIT_ASYNC, root], capture_output=True, text=True, timeout=120,
                       env=env)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    assert "exit-async: ok" in r.stdout


@pytest.mark.parametrize("n", [4099, (40 << 20) // 4 + 33])
@pytest.mark.parametrize("dt", [FP32, BF16])
def test_registered_pageable_on_gpu_paths(n, dt):
    """Pageable operands inside registered host buffers
    (mi_ccl_comp_register_host_buffer) take the GPU paths — bounce buffers for
    small buckets, the staged pipeline past one chunk — with the oracle's bits
    and without HIP's pointer lookup, in the shim or in libmi_reduce's GPU path
    (one counter, mi_pointer_lookups)."""
    shim = _lib.shim()
    b_impl, f_impl = impls()
    a = rand_array(dt, n, seed=91, specials=False)
    b = rand_array(dt, n, seed=92, specials=False)
    exp = b.copy()
    oracle.comp_reduce_mt(a, exp, dt, 0, 8, b_impl, f_impl)
    assert shim.mi_ccl_comp_register_host_buffer(ptr(a), a.nbytes) == 0
    assert shim.mi_ccl_comp_register_host_buffer(ptr(b), b.nbytes) == 0
    try:
        n0 = shim.mi_ccl_comp_pointer_lookups()
        comp.comp_reduce(ptr(a), n, ptr(b), comp.datatype(dt), comp.reduction.sum)
        assert shim.mi_ccl_comp_pointer_lookups() == n0
    finally:
        assert shim.mi_ccl_comp_unregister_host_buffer(ptr(a)) == 0
        assert shim.mi_ccl_comp_unregister_host_buffer(ptr(b)) == 0
    assert_same(b, exp, dt)


def test_streaming_copy_and_narrowing_on_pinned_host_memory():
    """The streaming copy and narrowing conversion (sc1 + nt buffer stores,
    64 MiB and more) read and write pinned host memory in place as well:
    device -> pinned, pinned -> device, and fp32 device -> bf16 pinned."""
    import torch
    m = _lib.mi()
    n = (64 << 20) + 4099
    src = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
    host = torch.zeros(n, dtype=torch.uint8).pin_memory()
    back = torch.zeros(n, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    _lib.check(m.mi_copy(src.data_ptr(), host.data_ptr(), n, 0, s))
    _lib.check(m.mi_copy(host.data_ptr(), back.data_ptr(), n, 1, s))
    torch.cuda.synchronize()
    assert torch.equal(host.cuda(), src) and torch.equal(back, src)
    count = (64 << 20) // 4 + 21
    f = torch.randn(count, device="cuda") * 5
    out = torch.zeros(count, dtype=torch.int16).pin_memory()
    _lib.check(m.mi_convert(f.data_ptr(), FP32, out.data_ptr(), BF16, count, comp.F_BF16_RNE, s))
    torch.cuda.synchronize()
    exp = oracle.f32_to_bf16(f.cpu().numpy(), True)
    assert_same(out.numpy().view(np.uint16), exp, BF16)
