"""Per-thread device contexts are pooled, not freed, when a thread exits
(mi_reduce.hip, ThreadCtx): a thread's exit makes no HIP call, and the next
thread on the device takes the exited thread's streams and staging buffers.
Short-lived threads one after another then build at most one context, and
each one's staged (pageable) reduce still gives the oracle's bits."""
from __future__ import annotations

import ctypes
import threading

import numpy as np
import pytest

import oracle
from oneccl_amd import _lib
from tests.util import FP32, assert_same, rand_array, wait_os_threads_gone

pytestmark = pytest.mark.gpu


def _stats():
    created, pooled = ctypes.c_size_t(0), ctypes.c_size_t(0)
    _lib.check(_lib.mi().mi_context_stats(ctypes.byref(created), ctypes.byref(pooled)))
    return created.value, pooled.value


def _staged_reduce(seed, n, errs):
    try:
        m = _lib.mi()
        a = rand_array(FP32, n, seed=seed, specials=False)
        b = rand_array(FP32, n, seed=seed + 1, specials=False)
        exp = b.copy()
        oracle.comp_reduce(a, exp, FP32, 0)
        _lib.check(m.mi_reduce_sync(a.ctypes.data, b.ctypes.data, n, FP32, 0, 0, -1))
        assert_same(b, exp, FP32)
    except Exception as e:  # noqa: BLE001
        errs.append(e)


def test_sequential_threads_reuse_one_context():
    n = (3 << 20) // 4 + 7  # 3 MiB per operand: past the bounce buffers, staged
    errs = []
    created0, _ = _stats()
    for t in range(6):
        th = threading.Thread(target=_staged_reduce, args=(100 + 2 * t, n, errs))
        th.start()
        th.join()
        assert wait_os_threads_gone([th.native_id])
    created1, pooled1 = _stats()
    assert not errs, errs[:3]
    assert created1 - created0 <= 1, (created0, created1)
    assert pooled1 >= 1


def test_concurrent_threads_then_reuse():
    n = (3 << 20) // 4 + 7
    errs = []
    ths = [threading.Thread(target=_staged_reduce, args=(300 + 2 * t, n, errs)) for t in range(4)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert wait_os_threads_gone([th.native_id for th in ths])
    created1, pooled1 = _stats()
    assert pooled1 >= 1  # the four threads' contexts (threads that ran apart shared one)
    ths = [threading.Thread(target=_staged_reduce, args=(400 + 2 * t, n, errs)) for t in range(4)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert wait_os_threads_gone([th.native_id for th in ths])
    created2, _ = _stats()
    assert not errs, errs[:3]
    # four threads at once take the pooled contexts first
    assert created2 - created1 <= max(0, 4 - pooled1), (created1, pooled1, created2)


def test_confined_caller_hands_staged_bucket_to_its_worker():
    """A caller pinned to one CPU (as oneCCL pins its workers) has its staged
    pageable buckets run by its staging worker (mi_reduce.hip, sync_entry);
    the bits are the oracle's, in place and through the K-input entry, and
    earlier asynchronous requests of the thread still come first."""
    import os
    n = (5 << 20) // 4 + 3
    errs = []

    def body():
        try:
            cpu = sorted(os.sched_getaffinity(0))[-1]
            os.sched_setaffinity(0, {cpu})
            m = _lib.mi()
            a = rand_array(FP32, n, seed=901, specials=False)
            b = rand_array(FP32, n, seed=902, specials=False)
            c = rand_array(FP32, n, seed=903, specials=False)
            exp = b.copy()
            oracle.comp_reduce(a, exp, FP32, 0)
            # an asynchronous request first (staged: it runs on the worker),
            # then the synchronous one that reads its output
            req = ctypes.c_void_p()
            _lib.check(m.mi_reduce_start(_lib.void_ptr_array([b.ctypes.data, a.ctypes.data]), 2, b.ctypes.data, n,
                                         FP32, 0, 0, -1, ctypes.byref(req)))
            exp_c = c.copy()
            oracle.comp_reduce(exp, exp_c, FP32, 0)
            _lib.check(m.mi_reduce_sync(b.ctypes.data, c.ctypes.data, n, FP32, 0, 0, -1))
            _lib.check(m.mi_wait(req))
            _lib.check(m.mi_request_free(req))
            assert_same(b, exp, FP32)
            assert_same(c, exp_c, FP32)
            out = np.zeros_like(a)
            exp3 = oracle.fanin([a, b, c], FP32, 0)
            _lib.check(m.mi_reduce_multi_sync(_lib.void_ptr_array([a.ctypes.data, b.ctypes.data, c.ctypes.data]),
                                              3, out.ctypes.data, n, FP32, 0, 0, -1))
            assert_same(out, exp3, FP32)
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    th = threading.Thread(target=body)
    th.start()
    th.join()
    assert wait_os_threads_gone([th.native_id])
    assert not errs, errs[:3]


def test_release_pooled_contexts():
    """mi_release_pooled_contexts frees the exited threads' contexts; the
    next thread builds a fresh one and reduces to the same bits."""
    n = (3 << 20) // 4 + 7
    errs = []
    th = threading.Thread(target=_staged_reduce, args=(700, n, errs))
    th.start()
    th.join()
    assert wait_os_threads_gone([th.native_id])
    created0, pooled0 = _stats()
    assert pooled0 >= 1
    freed = _lib.mi().mi_release_pooled_contexts()
    created1, pooled1 = _stats()
    assert freed == pooled0 and pooled1 == 0 and created1 == created0 - freed
    th = threading.Thread(target=_staged_reduce, args=(702, n, errs))
    th.start()
    th.join()
    assert wait_os_threads_gone([th.native_id])
    created2, pooled2 = _stats()
    assert not errs, errs[:3]
    assert created2 == created1 + 1 and pooled2 == 1


def _confined_staged(device, seed, out):
    """A caller confined to one CPU (as oneCCL pins its workers) whose current
    device is `device`: its staged synchronous bucket goes to its staging
    worker (the confined hand-off) with device -1."""
    import os

    import torch
    try:
        os.sched_setaffinity(0, {min(os.sched_getaffinity(0))})
        torch.cuda.set_device(device)
        m = _lib.mi()
        n = (8 << 20) // 4 + 5  # past the bounce size: staged
        a = rand_array(FP32, n, seed=seed, specials=False)
        b = rand_array(FP32, n, seed=seed + 1, specials=False)
        exp = b.copy()
        oracle.comp_reduce(a, exp, FP32, 0)
        _lib.check(m.mi_reduce_sync(a.ctypes.data, b.ctypes.data, n, FP32, 0, 0, -1))
        assert_same(b, exp, FP32)
        out.append(m.mi_test_staged_device())
    except Exception as e:  # noqa: BLE001
        out.append(e)


@pytest.mark.parametrize("device", [0, 1])
def test_confined_handoff_runs_on_the_callers_device(device):
    """device -1 means the calling thread's current
    device, also when a confined caller's bucket runs on its staging worker
    (whose own current device would be HIP's default, 0)."""
    import os

    import torch
    if device >= torch.cuda.device_count():
        pytest.skip(f"needs {device + 1} GPUs")
    if len(os.sched_getaffinity(0)) < 3:
        pytest.skip("the hand-off needs a process CPU set wider than the caller's")
    out = []
    t = threading.Thread(target=_confined_staged, args=(device, 31 + device, out))
    t.start()
    t.join(timeout=120)
    assert not t.is_alive()
    assert len(out) == 1 and not isinstance(out[0], Exception), out
    assert out[0] == device


@pytest.mark.parametrize("confined", [False, True])
def test_sync_bucket_classifies_each_operand_once(confined):
    """a synchronous bucket classifies each operand once,
    also on the confined caller's path (which used to classify them again
    before reduce_issue did).  Pinned, undeclared operands: one HIP lookup
    for the kind and one for the pinned allocation's extent (counted since
    round 6) per operand; in place, `out` is the first input's pointer."""
    import os

    import torch
    if confined and len(os.sched_getaffinity(0)) < 3:
        pytest.skip("the hand-off needs a process CPU set wider than the caller's")
    res = []

    def body():
        try:
            if confined:
                os.sched_setaffinity(0, {min(os.sched_getaffinity(0))})
            m = _lib.mi()
            n = (4 << 20) // 4 + 3
            a = rand_array(FP32, n, seed=41, specials=False)
            b = rand_array(FP32, n, seed=42, specials=False)
            exp = b.copy()
            oracle.comp_reduce(a, exp, FP32, 0)
            ha = torch.from_numpy(a.view(np.uint8).copy()).pin_memory()
            hb = torch.from_numpy(b.view(np.uint8).copy()).pin_memory()
            n0 = m.mi_pointer_lookups()
            _lib.check(m.mi_reduce_sync(ha.data_ptr(), hb.data_ptr(), n, FP32, 0, 0, -1))
            res.append(m.mi_pointer_lookups() - n0)
            assert_same(hb.numpy().view(np.float32), exp, FP32)
        except Exception as e:  # noqa: BLE001
            res.append(e)

    t = threading.Thread(target=body)
    t.start()
    t.join(timeout=120)
    assert not t.is_alive()
    assert res and not isinstance(res[-1], Exception), res
    assert res[0] == 2 * 3, res
