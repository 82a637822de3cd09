"""The drop-in's dispatcher on a GPU box: host-resident
buckets up to CCL_COMP_HOST_MAX_BYTES run on the calling thread's CPU
(host_reduce.cpp), larger ones and device buffers on the GPU.  Both sides of
the threshold give the reference's bits; a host-path call after an
asynchronous GPU request of the same thread sees that request's result."""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np
import pytest

import oracle
from oneccl_amd import comp
from tests.util import BF16, FP32, assert_same, rand_array, to_dev, from_dev, wait_os_threads_gone

pytestmark = pytest.mark.gpu


KNOBS = ("CCL_COMP_HOST_MAX_BYTES", "CCL_COMP_HOST_MAX_PINNED_BYTES", "CCL_COMP_HOST_SHARE",
         "CCL_COMP_HOST_SHARE_PINNED", "CCL_COMP_HOST_SHARE_ADAPT", "CCL_COMP_HOST_SPLIT_WORKERS",
         "CCL_COMP_HOST_SPLIT_WORKERS_PINNED")


@pytest.fixture
def threshold():
    saved = {k: os.environ.get(k) for k in KNOBS}
    for k in KNOBS:  # every test starts from the defaults
        os.environ.pop(k, None)

    def set_(v, **kv):
        os.environ["CCL_COMP_HOST_MAX_BYTES"] = str(v)
        for k, x in kv.items():
            os.environ[k] = str(x)
        comp.env_reload()

    yield set_
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    comp.env_reload()


@pytest.mark.parametrize("dt", [FP32, BF16, 6])
@pytest.mark.parametrize("kind", ["pageable", "pinned"])
def test_both_sides_of_the_threshold(dt, kind, threshold):
    import torch
    threshold(64 << 10)
    b_impl, f_impl = comp.impl_types()
    es = np.dtype(oracle.NP_DTYPE[dt]).itemsize
    for n in ((64 << 10) // es, (64 << 10) // es + 1, (3 << 20) // es + 7):  # CPU, GPU, GPU
        for op in range(4):
            a = rand_array(dt, n, seed=n + op, op=op)
            b = rand_array(dt, n, seed=n + op + 99, op=op)
            exp = b.copy()
            oracle.comp_reduce(a, exp, dt, op, int(b_impl), int(f_impl))
            if kind == "pinned":
                ta = torch.from_numpy(a.view(np.uint8).copy()).pin_memory()
                tb = torch.from_numpy(b.view(np.uint8).copy()).pin_memory()
                comp.comp_reduce(ta.data_ptr(), n, tb.data_ptr(), comp.datatype(dt), comp.reduction(op))
                got = tb.numpy().view(exp.dtype)
            else:
                comp.comp_reduce(a.ctypes.data, n, b.ctypes.data, comp.datatype(dt), comp.reduction(op))
                got = b
            assert_same(got, exp, dt, f"n={n} op={op}")


def test_host_path_waits_for_earlier_async_request(threshold):
    """A GPU request started asynchronously on a large pageable bucket, then
    a synchronous small reduce (CPU path) that reads part of its output."""
    threshold(1 << 20)
    n = (64 << 20) // 4
    a = rand_array(FP32, n, seed=1, specials=False)
    b = rand_array(FP32, n, seed=2, specials=False)
    c = rand_array(FP32, 4096, seed=3, specials=False)
    exp_b = b.copy()
    oracle.comp_reduce_mt(a, exp_b, FP32, 0, 8)
    exp_c = c.copy()
    oracle.comp_reduce(exp_b[:4096].copy(), exp_c, FP32, 0)
    req = comp.comp_reduce_start(a.ctypes.data, n, b.ctypes.data, comp.datatype.float32, comp.reduction.sum)
    comp.comp_reduce(b.ctypes.data, 4096, c.ctypes.data, comp.datatype.float32, comp.reduction.sum)
    req.wait()
    req.free()
    assert_same(c, exp_c, FP32, "small CPU reduce after the async GPU one")
    assert_same(b, exp_b, FP32, "async GPU reduce")


def test_device_buffers_never_take_the_host_path(threshold):
    threshold(1 << 30)
    import torch
    a = rand_array(FP32, 1000, seed=4)
    b = rand_array(FP32, 1000, seed=5)
    exp = b.copy()
    oracle.comp_reduce(a, exp, FP32, 0)
    ta, pa = to_dev(a)
    tb, pb = to_dev(b)
    comp.comp_reduce(pa, 1000, pb, comp.datatype.float32, comp.reduction.sum)
    torch.cuda.synchronize()
    assert_same(from_dev(tb, b), exp, FP32)


def test_cpp_caller_with_default_dispatch():
    """The C++ drop-in caller (src/sched-style call sites, MPI user ops) with
    the default threshold: small host chunks on the CPU, the rest on the GPU."""
    exe = Path(__file__).resolve().parent / "cpp" / "dropin_caller"
    if not exe.exists():
        from oneccl_amd import build
        build.build_dropin_caller()
    env = {k: v for k, v in os.environ.items() if k != "CCL_COMP_HOST_MAX_BYTES"}
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "dropin_caller: ok" in r.stdout


@pytest.mark.parametrize("kind", ["pageable", "pinned"])
@pytest.mark.parametrize("dt,op", [(FP32, 0), (BF16, 3), (4, 1), (6, 2)])
def test_cooperative_split_same_bits(kind, dt, op, threshold):
    """Above the crossover a host bucket is split: the GPU reduces the tail
    while the calling thread reduces the head.  Same bits as either path."""
    import torch
    threshold(1 << 20, CCL_COMP_HOST_SHARE=0.45, CCL_COMP_HOST_SHARE_PINNED=0.3)
    b_impl, f_impl = comp.impl_types()
    es = np.dtype(oracle.NP_DTYPE[dt]).itemsize
    n = (24 << 20) // es + 13
    a = rand_array(dt, n, seed=71 + op, op=op)
    b = rand_array(dt, n, seed=72 + op, op=op)
    exp = b.copy()
    oracle.comp_reduce_mt(a, exp, dt, op, 8, int(b_impl), int(f_impl))
    if kind == "pinned":
        ta = torch.from_numpy(a.view(np.uint8).copy()).pin_memory()
        tb = torch.from_numpy(b.view(np.uint8).copy()).pin_memory()
        comp.comp_reduce(ta.data_ptr(), n, tb.data_ptr(), comp.datatype(dt), comp.reduction(op))
        got = tb.numpy().view(exp.dtype)
    else:
        comp.comp_reduce(a.ctypes.data, n, b.ctypes.data, comp.datatype(dt), comp.reduction(op))
        got = b
    assert_same(got, exp, dt, f"{kind} split")


@pytest.mark.parametrize("share", ["0.5", "adapt"])
@pytest.mark.parametrize("k", [4, 19])
def test_cooperative_split_keep_precision_tail(k, share, threshold):
    """bf16 keep-precision fan-in across the split: the count % 16 truncated
    tail must land in the GPU's (last) part as in the whole array; with an
    adapting share the head also runs in 8 MiB chunks, none of which may
    truncate."""
    if share == "adapt":
        threshold(1 << 20)
        n = (12 << 20) + 11
    else:
        threshold(1 << 20, CCL_COMP_HOST_SHARE=share)
        n = (3 << 20) + 11
    b_impl, _ = comp.impl_types()
    ins = [rand_array(BF16, n, seed=500 + j, specials=False) for j in range(k)]
    packed = np.concatenate(ins)
    offsets = [j * n for j in range(k)]
    exp = ins[0].copy()
    oracle.batch_reduce(packed, offsets, n, exp, BF16, 0, 1, int(b_impl), 0)
    got = ins[0].copy()
    comp.comp_batch_reduce(packed.ctypes.data, offsets, n, got.ctypes.data, comp.datatype.bfloat16,
                           comp.reduction.sum, 1)
    assert_same(got, exp, BF16)


def _split_share(pinned):
    from oneccl_amd import _lib
    return _lib.shim().mi_ccl_comp_split_share(1 if pinned else 0)


@pytest.mark.parametrize("kind", ["pageable", "pinned"])
@pytest.mark.parametrize("dt", [FP32, BF16])
def test_adaptive_split_keeps_bits_and_bounds_its_share(kind, dt, threshold):
    """With the CPU share left to the dispatcher (no CCL_COMP_HOST_SHARE*),
    each split call times both parts and moves the thread's share toward the
    balance point: every call still gives the oracle's bits, and the share
    stays within [0.1, 0.9]."""
    import time

    import torch
    threshold(1 << 20)
    time.sleep(0.06)  # other tests' worker threads leave the dispatcher's 50 ms window
    b_impl, f_impl = comp.impl_types()
    es = np.dtype(oracle.NP_DTYPE[dt]).itemsize
    n = (48 << 20) // es + 13
    a = rand_array(dt, n, seed=91, specials=False)
    b0 = rand_array(dt, n, seed=92, specials=False)
    exp = b0.copy()
    oracle.comp_reduce_mt(a, exp, dt, 0, 8, int(b_impl), int(f_impl))
    assert _split_share(kind == "pinned") < 0  # env_reload started this thread over
    if kind == "pinned":
        ta = torch.from_numpy(a.view(np.uint8).copy()).pin_memory()
        tb = torch.empty(n * es, dtype=torch.uint8).pin_memory()
        pa, pb = ta.data_ptr(), tb.data_ptr()
        hb = tb.numpy().view(exp.dtype)
    else:
        ta, hb = a, np.empty_like(b0)
        pa, pb = a.ctypes.data, hb.ctypes.data
    shares = []
    for i in range(6):
        hb[:] = b0
        comp.comp_reduce(pa, n, pb, comp.datatype(dt), comp.reduction.sum)
        assert_same(hb, exp, dt, f"{kind} call {i}")
        shares.append(_split_share(kind == "pinned"))
    assert all(0.1 <= s <= 0.9 for s in shares), shares
    assert _split_share(kind != "pinned") < 0  # the other pointer kind's share is its own
    # the 3rd call ran on the GPU alone, timed: whether splitting pays is measured too
    from oneccl_amd import _lib
    left = ctypes.c_uint(0)
    assert _lib.shim().mi_ccl_comp_split_gpu_rate(1 if kind == "pinned" else 0, ctypes.byref(left)) > 0


@pytest.mark.parametrize("env", [{"CCL_COMP_HOST_SHARE": "0.45", "CCL_COMP_HOST_SHARE_PINNED": "0.45"},
                                 {"CCL_COMP_HOST_SHARE_ADAPT": "0"}], ids=["fixed-share", "adapt-off"])
def test_fixed_share_does_not_adapt(env, threshold):
    threshold(1 << 20, **env)
    n = (24 << 20) // 4
    a = rand_array(FP32, n, seed=93, specials=False)
    b = rand_array(FP32, n, seed=94, specials=False)
    exp = b.copy()
    oracle.comp_reduce_mt(a, exp, FP32, 0, 8)
    comp.comp_reduce(a.ctypes.data, n, b.ctypes.data, comp.datatype.float32, comp.reduction.sum)
    assert_same(b, exp, FP32)
    assert _split_share(False) < 0


@pytest.mark.parametrize("limit", ["2", "0"], ids=["limit-2", "no-limit"])
def test_split_yields_to_concurrent_workers(limit, threshold):
    """oneCCL reduces from CCL_WORKER_COUNT threads at once.  Once more than
    CCL_COMP_HOST_SPLIT_WORKERS threads reduce host buckets, a large pageable
    bucket stays on its thread's CPU (the GPU's share of the shared host DRAM
    and PCIe link no longer adds); with the limit off (0) every thread
    splits.  Bits are the oracle's either way."""
    import threading
    import time
    from oneccl_amd import _lib
    threshold(1 << 20, CCL_COMP_HOST_SPLIT_WORKERS=limit)
    time.sleep(0.06)
    w, n = 4, (6 << 20) // 4 + 5
    go = threading.Barrier(w)
    shares, errs = [None] * w, []

    def worker(i):
        try:
            a = rand_array(FP32, n, seed=300 + i, specials=False)
            b0 = rand_array(FP32, n, seed=400 + i, specials=False)
            exp = b0.copy()
            oracle.comp_reduce_mt(a, exp, FP32, 0, 4)
            small = np.ones(1024, np.float32)
            go.wait()
            # every thread is seen as a worker first (a CPU-path reduce)
            comp.comp_reduce(small.ctypes.data, 1024, small.ctypes.data, comp.datatype.float32, comp.reduction.sum)
            go.wait()
            for r in range(3):
                b = b0.copy()
                comp.comp_reduce(a.ctypes.data, n, b.ctypes.data, comp.datatype.float32, comp.reduction.sum)
                assert_same(b, exp, FP32, f"worker {i} round {r}")
            shares[i] = _lib.shim().mi_ccl_comp_split_share(0)
        except Exception as e:  # noqa: BLE001 - reported below
            errs.append(e)
            go.abort()

    ts = [threading.Thread(target=worker, args=(i,)) for i in range(w)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert wait_os_threads_gone([t.native_id for t in ts])
    assert not errs, errs
    if limit == "2":  # 4 workers > 2: nobody split
        assert all(s < 0 for s in shares), shares
    else:
        assert all(0.1 <= s <= 0.9 for s in shares), shares


@pytest.mark.parametrize("kind", ["pageable", "pinned"])
@pytest.mark.parametrize("batch", [False, True], ids=["reduce", "batch-keep-precision"])
def test_async_entry_splits_large_host_buckets(kind, batch, threshold):
    """ccl_comp_reduce_start / ccl_comp_batch_reduce_start on a host bucket
    above the threshold: the head is folded on the thread's staging worker,
    the tail on the GPU (mi_reduce_split_start).  Same bits as the
    synchronous call; the bf16 keep-precision count % 16 tail stays in the
    GPU part."""
    import torch
    threshold(1 << 20)
    b_impl, f_impl = comp.impl_types()
    if batch:
        k, n = 4, (6 << 20) + 11
        ins = [rand_array(BF16, n, seed=700 + j, specials=False) for j in range(k)]
        packed = np.concatenate(ins)
        offsets = [j * n for j in range(k)]
        exp = ins[0].copy()
        oracle.batch_reduce(packed, offsets, n, exp, BF16, 0, 1, int(b_impl), 0)
        got = ins[0].copy()
        if kind == "pinned":
            tp = torch.from_numpy(packed.view(np.uint8).copy()).pin_memory()
            tg = torch.from_numpy(got.view(np.uint8).copy()).pin_memory()
            pp, pg = tp.data_ptr(), tg.data_ptr()
        else:
            pp, pg = packed.ctypes.data, got.ctypes.data
        req = comp.comp_batch_reduce_start(pp, offsets, n, pg, comp.datatype.bfloat16, comp.reduction.sum, 1)
        req.wait()
        req.free()
        res = tg.numpy().view(np.uint16) if kind == "pinned" else got
        assert_same(res, exp, BF16)
        return
    n = (40 << 20) // 4 + 9
    a = rand_array(FP32, n, seed=81, specials=False)
    b = rand_array(FP32, n, seed=82, specials=False)
    exp = b.copy()
    oracle.comp_reduce_mt(a, exp, FP32, 0, 8)
    if kind == "pinned":
        ta = torch.from_numpy(a.view(np.uint8).copy()).pin_memory()
        tb = torch.from_numpy(b.view(np.uint8).copy()).pin_memory()
        pa, pb = ta.data_ptr(), tb.data_ptr()
    else:
        hb = b.copy()
        pa, pb = a.ctypes.data, hb.ctypes.data
    req = comp.comp_reduce_start(pa, n, pb, comp.datatype.float32, comp.reduction.sum)
    req.wait()
    req.free()
    got = tb.numpy().view(np.float32) if kind == "pinned" else hb
    assert_same(got, exp, FP32, kind)


@pytest.mark.parametrize("kind", ["pageable", "pinned"])
def test_async_split_adapts_its_share(kind, threshold):
    """Without CCL_COMP_HOST_SHARE*, each finished asynchronous split moves
    the calling thread's share toward the balance point, from the two parts'
    durations its worker measured (mi_request_split_times): the share leaves
    its 0.45 start and stays within [0.1, 0.9], and every call keeps the
    bits."""
    import time

    import torch
    threshold(1 << 20)
    time.sleep(0.06)
    n = (48 << 20) // 4 + 13
    a = rand_array(FP32, n, seed=95, specials=False)
    b0 = rand_array(FP32, n, seed=96, specials=False)
    exp = b0.copy()
    oracle.comp_reduce_mt(a, exp, FP32, 0, 8)
    if kind == "pinned":
        ta = torch.from_numpy(a.view(np.uint8).copy()).pin_memory()
        tb = torch.empty(n * 4, dtype=torch.uint8).pin_memory()
        pa, pb, hb = ta.data_ptr(), tb.data_ptr(), tb.numpy().view(np.float32)
    else:
        hb = np.empty_like(b0)
        pa, pb = a.ctypes.data, hb.ctypes.data
    shares = []
    for i in range(5):
        hb[:] = b0
        req = comp.comp_reduce_start(pa, n, pb, comp.datatype.float32, comp.reduction.sum)
        while not req.test():
            pass
        req.free()
        assert_same(hb, exp, FP32, f"{kind} call {i}")
        shares.append(_split_share(kind == "pinned"))
    assert all(0.1 <= s <= 0.9 for s in shares), shares
    assert shares[0] == pytest.approx(0.45)  # the first split of a kind only warms up
    assert any(abs(s - 0.45) > 1e-9 for s in shares[1:]), shares
    from oneccl_amd import _lib
    left = ctypes.c_uint(0)
    assert _lib.shim().mi_ccl_comp_split_gpu_rate(1 if kind == "pinned" else 0, ctypes.byref(left)) > 0


def test_pinned_zero_sends_pinned_buckets_to_the_gpu_alone(threshold):
    """CCL_COMP_HOST_MAX_PINNED_BYTES=0: a pinned bucket above
    the pageable threshold is never split with the CPU (the thread's pinned
    share is never started); a pageable one still is."""
    import torch
    threshold(1 << 20, CCL_COMP_HOST_MAX_PINNED_BYTES=0)
    n = (24 << 20) // 4 + 7
    a = rand_array(FP32, n, seed=11, specials=False)
    b = rand_array(FP32, n, seed=12, specials=False)
    exp = b.copy()
    oracle.comp_reduce_mt(a, exp, FP32, 0, 8)
    ta = torch.from_numpy(a.view(np.uint8).copy()).pin_memory()
    tb = torch.from_numpy(b.view(np.uint8).copy()).pin_memory()
    for _ in range(3):
        tb.copy_(torch.from_numpy(b.view(np.uint8)))
        comp.comp_reduce(ta.data_ptr(), n, tb.data_ptr(), comp.datatype.float32, comp.reduction.sum)
        assert_same(tb.numpy().view(np.float32), exp, FP32, "pinned")
    assert _split_share(True) < 0  # no split ever started for pinned buckets
    hb = b.copy()
    comp.comp_reduce(a.ctypes.data, n, hb.ctypes.data, comp.datatype.float32, comp.reduction.sum)
    assert_same(hb, exp, FP32, "pageable")
    assert _split_share(False) >= 0.1  # the pageable bucket was split
