"""Asynchronous requests (mi_reduce_start / mi_test / mi_wait) and the
in-process sharded multi-device call, against the oracle."""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

import oracle
from oneccl_amd import _lib
from tests.util import BF16, FP32, assert_same, from_dev, rand_array, to_dev

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("where", ["device", "pageable", "pinned", "pinned_staged"])
@pytest.mark.parametrize("n", [1000, (70 << 20) // 4 + 5])
def test_start_test_wait(where, n):
    import torch
    m = _lib.mi()
    a = rand_array(FP32, n, seed=1, specials=False)
    b = rand_array(FP32, n, seed=2, specials=False)
    exp = b.copy()
    oracle.comp_reduce_mt(a, exp, FP32, 0, 8)
    keep = []
    if where == "device":
        ta, pa = to_dev(a)
        tb, pb = to_dev(b)
        keep += [ta, tb]
    elif where.startswith("pinned"):
        ha = torch.from_numpy(a.view(np.uint8).copy()).pin_memory()
        hb = torch.from_numpy(b.view(np.uint8).copy()).pin_memory()
        pa, pb = ha.data_ptr(), hb.data_ptr()
    else:
        hb_np = b.copy()
        pa, pb = a.ctypes.data, hb_np.ctypes.data
    prev = m.mi_set_host_mode(1 if where == "pinned_staged" else 0)
    try:
        req = ctypes.c_void_p()
        arr = _lib.void_ptr_array([pb, pa])
        _lib.check(m.mi_reduce_start(arr, 2, pb, n, FP32, 0, 0, -1, ctypes.byref(req)))
        done = ctypes.c_int(0)
        polls = 0
        while True:
            _lib.check(m.mi_test(req, ctypes.byref(done)))
            polls += 1
            if done.value:
                break
            assert polls < 10_000_000
        _lib.check(m.mi_wait(req))
        _lib.check(m.mi_request_free(req))
    finally:
        m.mi_set_host_mode(prev)
    if where == "device":
        got = from_dev(tb, b)
    elif where.startswith("pinned"):
        got = hb.numpy().view(np.float32)
    else:
        got = hb_np
    assert_same(got, exp, FP32, where)


def test_many_outstanding_requests():
    m = _lib.mi()
    n = 1 << 20
    reqs, outs, exps, keep = [], [], [], []
    for j in range(8):
        a = rand_array(BF16, n, seed=10 + j)
        b = rand_array(BF16, n, seed=20 + j)
        exp = b.copy()
        oracle.comp_reduce(a, exp, BF16, 0, oracle.BF16_AVX512BF)
        ta, pa = to_dev(a)
        tb, pb = to_dev(b)
        keep += [ta, tb]
        r = ctypes.c_void_p()
        _lib.check(m.mi_reduce_start(_lib.void_ptr_array([pb, pa]), 2, pb, n, BF16, 0, 0x3, -1, ctypes.byref(r)))
        reqs.append(r)
        outs.append((tb, b))
        exps.append(exp)
    for r in reqs:
        _lib.check(m.mi_wait(r))
        _lib.check(m.mi_request_free(r))
    for (tb, b), exp in zip(outs, exps):
        assert_same(from_dev(tb, b), exp, BF16)


@pytest.mark.parametrize("nshards", [1, 2, 4, 8])
def test_sharded_in_process(nshards):
    """SURVEY §8e inside one process: every shard on its device (here all on
    device 0 — the box has one GPU), launched together, no collective."""
    import torch
    m = _lib.mi()
    n = 3_000_017
    k = 3
    ins = [rand_array(FP32, n, seed=40 + j) for j in range(k)]
    exp = oracle.fanin(ins, FP32, 0)
    dev_ins = [to_dev(x) for x in ins]
    out_t, out_p = to_dev(np.zeros(n, np.float32))
    ndev = torch.cuda.device_count()
    devs, ptrs, outs, counts = [], [], [], []
    for s in range(nshards):
        lo = ctypes.c_size_t()
        hi = ctypes.c_size_t()
        _lib.check(m.mi_shard_range(n, s, nshards, 256, ctypes.byref(lo), ctypes.byref(hi)))
        devs.append(s % ndev if ndev == 1 else 0)
        ptrs += [p + 4 * lo.value for _, p in dev_ins]
        outs.append(out_p + 4 * lo.value)
        counts.append(hi.value - lo.value)
    _lib.check(m.mi_reduce_sharded(nshards, (ctypes.c_int * nshards)(*devs), _lib.void_ptr_array(ptrs), k,
                                   _lib.void_ptr_array(outs), (ctypes.c_size_t * nshards)(*counts), FP32, 0, 0))
    assert_same(from_dev(out_t, ins[0]), exp, FP32)


def test_hipgraph_capture_and_replay():
    """The asynchronous entry points do no allocation or synchronisation while
    launching (cdna_hip_programming.md Guideline 9), so they can be captured
    into a hipGraph and replayed — e.g. a whole bucket schedule as one graph."""
    import torch
    m = _lib.mi()
    n = 1_000_003
    a = rand_array(FP32, n, seed=71, specials=False)
    b = rand_array(FP32, n, seed=72, specials=False)
    c = rand_array(BF16, n, seed=73, specials=False)
    d = rand_array(BF16, n, seed=74, specials=False)
    ta, pa = to_dev(a)
    tb, pb = to_dev(b)
    tc, pc = to_dev(c)
    td, pd = to_dev(d)
    side = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        h = torch.cuda.current_stream().cuda_stream
        _lib.check(m.mi_reduce(pa, pb, n, FP32, 0, 0, h))
        _lib.check(m.mi_reduce(pc, pd, n, BF16, 0, 0x3, h))
    exp_b, exp_d = b.copy(), d.copy()
    replays = 3
    for _ in range(replays):
        oracle.comp_reduce(a, exp_b, FP32, 0)
        oracle.comp_reduce(c, exp_d, BF16, 0, oracle.BF16_AVX512BF)
    tb.copy_(to_dev(b)[0])  # capture does not execute; start from the inputs
    td.copy_(to_dev(d)[0])
    torch.cuda.synchronize()
    for _ in range(replays):
        g.replay()
    torch.cuda.synchronize()
    assert_same(from_dev(tb, b), exp_b, FP32)
    assert_same(from_dev(td, d), exp_d, BF16)


def test_pageable_start_returns_before_the_work_is_done():
    """mi_reduce_start on pageable operands hands the staged pipeline to the
    calling thread's worker and returns at once; requests run in submission
    order, so a request that reads the previous one's output sees it."""
    import time
    m = _lib.mi()
    n = (256 << 20) // 4
    a = rand_array(FP32, n, seed=11, specials=False)
    b = rand_array(FP32, n, seed=12, specials=False)
    c = rand_array(FP32, n, seed=13, specials=False)
    exp_b = b.copy()
    oracle.comp_reduce_mt(a, exp_b, FP32, 0, 8)
    exp_c = c.copy()
    oracle.comp_reduce_mt(exp_b, exp_c, FP32, 0, 8)
    # warm the worker (its streams and staging buffers) with one small request
    w = np.ones(1 << 20, np.float32)
    req = ctypes.c_void_p()
    _lib.check(m.mi_reduce_start(_lib.void_ptr_array([w.ctypes.data, w.ctypes.data]), 2, w.ctypes.data, w.size,
                                 FP32, 0, 0, -1, ctypes.byref(req)))
    _lib.check(m.mi_request_free(req))
    t0 = time.perf_counter()
    r1, r2 = ctypes.c_void_p(), ctypes.c_void_p()
    _lib.check(m.mi_reduce_start(_lib.void_ptr_array([b.ctypes.data, a.ctypes.data]), 2, b.ctypes.data, n, FP32, 0,
                                 0, -1, ctypes.byref(r1)))
    _lib.check(m.mi_reduce_start(_lib.void_ptr_array([c.ctypes.data, b.ctypes.data]), 2, c.ctypes.data, n, FP32, 0,
                                 0, -1, ctypes.byref(r2)))
    t_start = time.perf_counter() - t0
    done = ctypes.c_int(0)
    _lib.check(m.mi_test(r2, ctypes.byref(done)))
    assert done.value == 0  # 2 x 256 MiB staged over PCIe cannot be done yet
    _lib.check(m.mi_wait(r1))
    _lib.check(m.mi_wait(r2))
    t_all = time.perf_counter() - t0
    _lib.check(m.mi_request_free(r1))
    _lib.check(m.mi_request_free(r2))
    assert_same(b, exp_b, FP32, "first request")
    assert_same(c, exp_c, FP32, "second request reads the first one's output")
    assert t_start < 0.25 * t_all, (t_start, t_all)


@pytest.mark.parametrize("where", ["device", "pinned", "pageable", "pageable_small"])
@pytest.mark.parametrize("nshards", [2, 3])
def test_multi_sync_sharded_same_bits(where, nshards):
    """mi_reduce_multi_sync_sharded splits one bucket over several GPUs (here
    the one GPU listed several times, each shard on its own thread, streams
    and staging buffers): same bits as one call, including the bf16
    fp32-accumulate fan-in's count % 16 truncated tail, which must fall in the
    last shard as in the whole array."""
    import torch
    m = _lib.mi()
    n = ((70 << 20) // 2 + 13) if where != "pageable_small" else 100_003
    k = 4
    ins = [rand_array(BF16, n, seed=60 + j, specials=False) for j in range(k)]
    flags = 0x4 | 0x2 | 0x8  # MI_F_ACC_FP32 | MI_F_BF16_RNE | MI_F_BF16_TAIL_TRUNC16
    # ccl_comp_batch_reduce(keep precision) under avx512bf, restated by the oracle
    ref_out = ins[0].copy()
    oracle.batch_reduce(np.concatenate(ins), [j * n for j in range(k)], n, ref_out, BF16, 0, 1,
                        oracle.BF16_AVX512BF, 0)
    if where == "device":
        hs = [to_dev(x) for x in ins]
        ptrs = [p for _, p in hs]
        to, po = to_dev(np.zeros(n, np.uint16))
    elif where == "pinned":
        hs = [torch.from_numpy(x.view(np.uint8).copy()).pin_memory() for x in ins]
        ptrs = [h.data_ptr() for h in hs]
        ho = torch.zeros(n * 2, dtype=torch.uint8).pin_memory()
        po = ho.data_ptr()
    else:
        ptrs = [x.ctypes.data for x in ins]
        out = np.zeros(n, np.uint16)
        po = out.ctypes.data
    devs = (ctypes.c_int * nshards)(*([0] * nshards))
    _lib.check(m.mi_reduce_multi_sync_sharded(_lib.void_ptr_array(ptrs), k, po, n, BF16, 0, flags, nshards, devs))
    if where == "device":
        got = from_dev(to, ref_out)
    elif where == "pinned":
        got = ho.numpy().view(np.uint16)
    else:
        got = out
    assert_same(got, ref_out, BF16, f"{where} x{nshards}")


@pytest.mark.parametrize("first", ["staged", "direct"])
def test_staged_and_direct_requests_keep_submission_order(first):
    """Requests of one thread run in submission order whatever their pointer
    kinds: a staged request (pageable operands, run by the thread's worker)
    and a device-only request (launched on the thread's stream) that reads
    the other's output, in both orders; then a synchronous call that reads
    the last output."""
    import torch
    m = _lib.mi()
    n = (64 << 20) // 4
    a = rand_array(FP32, n, seed=21, specials=False)
    h = rand_array(FP32, n, seed=22, specials=False)  # pageable
    d0 = rand_array(FP32, n, seed=23, specials=False)
    td, pd = to_dev(d0)
    torch.cuda.synchronize()
    reqs = []

    def start(ins, out):
        r = ctypes.c_void_p()
        _lib.check(m.mi_reduce_start(_lib.void_ptr_array(ins), 2, out, n, FP32, 0, 0, -1, ctypes.byref(r)))
        reqs.append(r)

    ta, pa = to_dev(a)
    torch.cuda.synchronize()
    exp_h, exp_d = h.copy(), d0.copy()
    if first == "staged":
        # h += a (staged: pageable h), then d += h (device d reads pageable h: staged)... then d += a on device
        start([h.ctypes.data, pa], h.ctypes.data)
        oracle.comp_reduce(a, exp_h, FP32, 0)
        start([pd, pa], pd)  # device-only: must wait for nothing but keeps order
        oracle.comp_reduce(a, exp_d, FP32, 0)
        start([pd, h.ctypes.data], pd)  # reads the staged request's output
        oracle.comp_reduce(exp_h, exp_d, FP32, 0)
    else:
        start([pd, pa], pd)  # device-only, queued on the thread's stream
        oracle.comp_reduce(a, exp_d, FP32, 0)
        start([h.ctypes.data, pd], h.ctypes.data)  # staged: reads the device request's output
        oracle.comp_reduce(exp_d, exp_h, FP32, 0)
        start([pd, pa], pd)  # device-only again, after a staged one
        oracle.comp_reduce(a, exp_d, FP32, 0)
    # synchronous call on the same thread: runs after every request above
    _lib.check(m.mi_reduce_sync(pd, h.ctypes.data, n, FP32, 0, 0, -1))
    oracle.comp_reduce(exp_d, exp_h, FP32, 0)
    for r in reqs:
        _lib.check(m.mi_wait(r))
        _lib.check(m.mi_request_free(r))
    assert_same(from_dev(td, d0), exp_d, FP32, "device operand")
    assert_same(h, exp_h, FP32, "pageable operand")


def _host_fold_ptr():
    """mi_host_reduce (the shim's CPU fold) as a C function pointer."""
    return ctypes.cast(_lib.shim().mi_host_reduce, ctypes.c_void_p).value


@pytest.mark.parametrize("where", ["pageable", "pinned", "device"])
@pytest.mark.parametrize("dt,op,flags", [(FP32, 0, 0), (BF16, 0, 0x2), (6, 3, 0), (4, 1, 0)],
                         ids=["f32-sum", "bf16-sum-rne", "i64-max", "i32-prod"])
def test_split_start_same_bits(where, dt, op, flags):
    """mi_reduce_split_start: [0, head) folded by the host fold on the
    thread's staging worker while the GPU folds the rest; the same bits as
    the oracle over the whole bucket, for host and device operands."""
    import torch
    m = _lib.mi()
    es = np.dtype(oracle.NP_DTYPE[dt]).itemsize
    n = (40 << 20) // es + 37
    head = (n * 2 // 5) // 256 * 256
    a = rand_array(dt, n, seed=31 + op, op=op)
    b = rand_array(dt, n, seed=32 + op, op=op)
    exp = b.copy()
    oracle.comp_reduce_mt(a, exp, dt, op, 8)  # bf16: the avx512bf impl (RNE) = MI_F_BF16_RNE
    if where == "device":
        ta, pa = to_dev(a)
        tb, pb = to_dev(b)
        torch.cuda.synchronize()
    elif where == "pinned":
        ta = torch.from_numpy(a.view(np.uint8).copy()).pin_memory()
        tb = torch.from_numpy(b.view(np.uint8).copy()).pin_memory()
        pa, pb = ta.data_ptr(), tb.data_ptr()
    else:
        hb = b.copy()
        pa, pb = a.ctypes.data, hb.ctypes.data
    if where == "device":  # the host fold must never see device memory: the GPU takes it whole
        head = 0
    req = ctypes.c_void_p()
    _lib.check(m.mi_reduce_split_start(_lib.void_ptr_array([pb, pa]), 2, pb, n, dt, op, flags, -1, head,
                                       _host_fold_ptr(), ctypes.byref(req)))
    _lib.check(m.mi_wait(req))
    th, tt = ctypes.c_double(), ctypes.c_double()
    rc = m.mi_request_split_times(req, ctypes.byref(th), ctypes.byref(tt))
    if head:
        assert rc == 0 and th.value > 0 and tt.value > 0, (rc, th.value, tt.value)
    else:
        assert rc < 0  # not a split
    _lib.check(m.mi_request_free(req))
    got = from_dev(tb, b) if where == "device" else (tb.numpy().view(exp.dtype) if where == "pinned" else hb)
    assert_same(got, exp, dt, where)


def test_split_start_keeps_submission_order():
    """A split request, then a device-only request that reads its output,
    then a synchronous call on the first one's output: each sees the one
    before, whichever side (host head or GPU tail) wrote the elements."""
    import torch
    m = _lib.mi()
    n = (48 << 20) // 4
    head = (n // 2) // 256 * 256
    a = rand_array(FP32, n, seed=41, specials=False)
    h = rand_array(FP32, n, seed=42, specials=False)
    d0 = rand_array(FP32, n, seed=43, specials=False)
    td, pd = to_dev(d0)
    torch.cuda.synchronize()
    exp_h, exp_d = h.copy(), d0.copy()
    r1, r2 = ctypes.c_void_p(), ctypes.c_void_p()
    _lib.check(m.mi_reduce_split_start(_lib.void_ptr_array([h.ctypes.data, a.ctypes.data]), 2, h.ctypes.data, n,
                                       FP32, 0, 0, -1, head, _host_fold_ptr(), ctypes.byref(r1)))
    oracle.comp_reduce_mt(a, exp_h, FP32, 0, 8)
    _lib.check(m.mi_reduce_start(_lib.void_ptr_array([pd, h.ctypes.data]), 2, pd, n, FP32, 0, 0, -1,
                                 ctypes.byref(r2)))
    oracle.comp_reduce_mt(exp_h, exp_d, FP32, 0, 8)
    _lib.check(m.mi_reduce_sync(pd, h.ctypes.data, n, FP32, 0, 0, -1))
    oracle.comp_reduce_mt(exp_d, exp_h, FP32, 0, 8)
    for r in (r1, r2):
        _lib.check(m.mi_wait(r))
        _lib.check(m.mi_request_free(r))
    assert_same(from_dev(td, d0), exp_d, FP32, "device request after the split")
    assert_same(h, exp_h, FP32, "sync call after both")


def test_split_start_argument_errors():
    m = _lib.mi()
    a = np.ones(4096, np.float32)
    arr = _lib.void_ptr_array([a.ctypes.data, a.ctypes.data])
    req = ctypes.c_void_p()
    assert m.mi_reduce_split_start(arr, 2, a.ctypes.data, a.size, FP32, 0, 0, -1, 256, None, ctypes.byref(req)) < 0
    assert m.mi_reduce_split_start(arr, 2, a.ctypes.data, a.size, FP32, 0, 0, -1, a.size, _host_fold_ptr(),
                                   ctypes.byref(req)) < 0
    assert m.mi_reduce_split_start(arr, 2, a.ctypes.data, a.size, FP32, 4, 0, -1, 256, _host_fold_ptr(),
                                   ctypes.byref(req)) < 0


@pytest.mark.parametrize("where", ["device", "pinned", "pageable"])
def test_timed_request_reports_its_run_time(where):
    """mi_reduce_start_timed: the duration measured where the request ran (a
    HIP event pair around a direct launch, the staging worker's clock for a
    staged one), within the caller's wall time; ADVICE r2 (the dispatcher's
    GPU-alone rate).  An untimed direct request has none."""
    import time

    import torch
    m = _lib.mi()
    n = (32 << 20) // 4
    a = rand_array(FP32, n, seed=5, specials=False)
    b = rand_array(FP32, n, seed=6, specials=False)
    exp = b.copy()
    oracle.comp_reduce_mt(a, exp, FP32, 0, 8)
    if where == "device":
        ta, pa = to_dev(a)
        tb, pb = to_dev(b)
    elif where == "pinned":
        ha = torch.from_numpy(a.view(np.uint8).copy()).pin_memory()
        hb = torch.from_numpy(b.view(np.uint8).copy()).pin_memory()
        pa, pb = ha.data_ptr(), hb.data_ptr()
    else:
        hbn = b.copy()
        pa, pb = a.ctypes.data, hbn.ctypes.data
    ins = _lib.void_ptr_array([pb, pa])
    req = ctypes.c_void_p()
    t0 = time.perf_counter()
    _lib.check(m.mi_reduce_start_timed(ins, 2, pb, n, FP32, 0, 0, -1, ctypes.byref(req)))
    _lib.check(m.mi_wait(req))
    wall = time.perf_counter() - t0
    t = ctypes.c_double(-1)
    _lib.check(m.mi_request_run_time(req, ctypes.byref(t)))
    _lib.check(m.mi_request_free(req))
    assert 0 < t.value <= wall + 1e-3, (t.value, wall)
    got = from_dev(tb, b) if where == "device" else (hb.numpy().view(np.float32) if where == "pinned" else hbn)
    assert_same(got, exp, FP32, where)
    if where == "device":  # untimed direct request: no run time
        req2 = ctypes.c_void_p()
        _lib.check(m.mi_reduce_start(ins, 2, pb, n, FP32, 0, 0, -1, ctypes.byref(req2)))
        _lib.check(m.mi_wait(req2))
        assert m.mi_request_run_time(req2, ctypes.byref(t)) != 0
        _lib.check(m.mi_request_free(req2))
