"""The schedule's word on where the operands live (SURVEY.md §8f rank 1,
VERDICT r3 item 1).  The reference's ccl_comp_reduce reads
sched->coll_param.stream (src/comp/comp.cpp:136-142): with no stream the
operands are host memory and it calls the CPU loop without classifying them
(and a CPU build never classifies, :196-198).  The drop-in does the same: a
schedule without a stream routes a small bucket to the calling thread's CPU
with zero HIP pointer lookups, where the lookup of pageable memory is what
serialised concurrent workers.  With a stream, or with no
schedule, the operands are looked up as before.  CPU-only: buckets below the
dispatcher's threshold, bits checked against numpy (IEEE fp32 add)."""
import ctypes
import threading

import numpy as np
import pytest

from oneccl_amd import _lib

FLOAT32, INT32, BF16, SUM, MAX, CUSTOM = 9, 4, 11, 0, 3, 4


@pytest.fixture()
def shim():
    s = _lib.shim()
    prev = s.mi_ccl_comp_shim_sched(0)
    yield s
    s.mi_ccl_comp_shim_sched(prev)


def _pair(n, seed=0, dt=np.float32):
    rng = np.random.default_rng(seed)
    if dt == np.int32:
        return rng.integers(-1000, 1000, n).astype(np.int32), rng.integers(-1000, 1000, n).astype(np.int32)
    return rng.random(n, dtype=np.float32), rng.random(n, dtype=np.float32)


def _lookups_for(shim, mode, fn):
    assert shim.mi_ccl_comp_shim_sched(mode) >= 0
    n0 = shim.mi_ccl_comp_pointer_lookups()
    fn()
    return shim.mi_ccl_comp_pointer_lookups() - n0


@pytest.mark.parametrize("mode,lookups", [(0, 2), (1, 0), (2, 2)])
def test_host_schedule_skips_every_lookup(shim, mode, lookups):
    a, b0 = _pair(1024, mode)
    b = b0.copy()
    got = _lookups_for(shim, mode, lambda: _lib.check_shim(
        shim.mi_ccl_comp_reduce(a.ctypes.data, a.size, b.ctypes.data, None, FLOAT32, SUM), "ccl_comp_reduce"))
    assert got == lookups
    assert np.array_equal(b.view(np.uint32), (b0 + a).view(np.uint32))


def test_host_schedule_every_op_and_dtype_bits(shim):
    """The route changes only who classifies: the bits are the CPU path's."""
    for dt_np, dt, op in ((np.float32, FLOAT32, MAX), (np.int32, INT32, SUM), (np.int32, INT32, MAX)):
        a, b0 = _pair(4099, 7, dt_np)
        b = b0.copy()
        assert _lookups_for(shim, 1, lambda: _lib.check_shim(
            shim.mi_ccl_comp_reduce(a.ctypes.data, a.size, b.ctypes.data, None, dt, op), "reduce")) == 0
        exp = b0 + a if op == SUM else np.maximum(a, b0)
        assert np.array_equal(b, exp)


def test_host_schedule_async_start_skips_lookups(shim):
    a, b0 = _pair(2048, 3)
    b = b0.copy()
    req = ctypes.c_void_p()

    def run():
        _lib.check_shim(shim.mi_ccl_comp_reduce_start(a.ctypes.data, a.size, b.ctypes.data, None, FLOAT32, SUM,
                                                      _lib.MI_CCL_REDUCTION_FN(), ctypes.byref(req)), "start")
        done = ctypes.c_int()
        _lib.check_shim(shim.mi_ccl_comp_request_test(req, ctypes.byref(done)), "test")
        assert done.value == 1  # the CPU path completes inside start
        _lib.check_shim(shim.mi_ccl_comp_request_free(req), "free")

    assert _lookups_for(shim, 1, run) == 0
    assert np.array_equal(b.view(np.uint32), (b0 + a).view(np.uint32))


def test_host_schedule_batch_start_skips_lookups(shim):
    k, n = 4, 512
    rng = np.random.default_rng(5)
    buf = rng.random(k * n, dtype=np.float32)
    acc0 = rng.random(n, dtype=np.float32)
    acc = acc0.copy()
    offs = (ctypes.c_size_t * k)(*[i * n for i in range(k)])
    req = ctypes.c_void_p()

    def run():
        _lib.check_shim(shim.mi_ccl_comp_batch_reduce_start(buf.ctypes.data, offs, k, n, acc.ctypes.data, None,
                                                            FLOAT32, SUM, 0, ctypes.byref(req)), "batch start")
        _lib.check_shim(shim.mi_ccl_comp_request_wait(req), "wait")
        _lib.check_shim(shim.mi_ccl_comp_request_free(req), "free")

    # the batch start reads inout_buf and in_buf + offsets[1..k-1]
    assert _lookups_for(shim, 1, run) == 0
    exp = acc0.copy()
    for i in range(1, k):
        exp = exp + buf[i * n:(i + 1) * n]
    assert np.array_equal(acc.view(np.uint32), exp.view(np.uint32))


def test_host_schedule_custom_reduction_runs_on_the_buffers(shim):
    """A custom op under a host schedule goes straight to the callback on the
    caller's buffers (comp.cpp:139-142 -> :84-88): no lookup, no staging."""
    a, b0 = _pair(64, 11)
    b = b0.copy()
    seen = []

    @_lib.MI_CCL_REDUCTION_FN
    def cb(in_p, n, io_p, out_n, dt, ctx):
        seen.append((in_p, io_p, n))
        x = np.ctypeslib.as_array(ctypes.cast(in_p, ctypes.POINTER(ctypes.c_float)), (n,))
        y = np.ctypeslib.as_array(ctypes.cast(io_p, ctypes.POINTER(ctypes.c_float)), (n,))
        y[:] = x * 2 + y

    assert _lookups_for(shim, 1, lambda: _lib.check_shim(
        shim.mi_ccl_comp_reduce_custom(a.ctypes.data, a.size, b.ctypes.data, None, FLOAT32, cb), "custom")) == 0
    assert seen == [(a.ctypes.data, b.ctypes.data, a.size)]
    assert np.array_equal(b, a * 2 + b0)


def test_shim_sched_mode_is_per_thread_and_checked(shim):
    assert shim.mi_ccl_comp_shim_sched(3) == -1
    assert shim.mi_ccl_comp_shim_sched(-1) == -1
    assert shim.mi_ccl_comp_shim_sched(1) == 0
    other = []
    t = threading.Thread(target=lambda: other.append(shim.mi_ccl_comp_shim_sched(0)))
    t.start()
    t.join()
    assert other == [0]  # a new thread starts with no schedule
    assert shim.mi_ccl_comp_shim_sched(0) == 1


def test_host_schedule_under_concurrent_workers(shim):
    """Eight workers reducing 4 KiB chunks under host schedules make no
    lookup at all and keep exact bits (the regime of VERDICT r3 item 1)."""
    errors = []

    def worker(seed):
        s = _lib.shim()
        s.mi_ccl_comp_shim_sched(1)
        a, b0 = _pair(1024, seed)
        b = b0.copy()
        n0 = s.mi_ccl_comp_pointer_lookups()
        exp = b0.copy()
        for _ in range(300):
            if s.mi_ccl_comp_reduce(a.ctypes.data, a.size, b.ctypes.data, None, FLOAT32, SUM) != 0:
                errors.append("rc")
            exp = exp + a
        if s.mi_ccl_comp_pointer_lookups() != n0:
            errors.append("lookup")
        if not np.array_equal(b.view(np.uint32), exp.view(np.uint32)):
            errors.append("bits")

    ws = [threading.Thread(target=worker, args=(i,)) for i in range(8)]
    for w in ws:
        w.start()
    for w in ws:
        w.join()
    assert errors == []


@pytest.mark.parametrize("nbytes", [1, 255, 4096, 65536 + 7, 1 << 20])
@pytest.mark.parametrize("nt", [0, 1])
def test_copy_entries_host_copy_makes_no_lookup(shim, nbytes, nt):
    """ccl_comp_copy_host (integration/0006): the regular copy of copy_entry
    and recv_copy_entry's copy, host to host by construction
    (copy_entry.cpp:90-97, allreduce.cpp:396-422), copy bytes exactly with no
    pointer lookup; ccl_comp_copy itself still classifies (2 lookups)."""
    rng = np.random.default_rng(nbytes)
    src = rng.integers(0, 256, nbytes + 64, dtype=np.uint8)
    dst = np.zeros(nbytes + 64, np.uint8)
    n0 = shim.mi_ccl_comp_pointer_lookups()
    _lib.check_shim(shim.mi_ccl_comp_copy_host(src.ctypes.data + 3, dst.ctypes.data + 5, nbytes, nt), "copy_host")
    assert shim.mi_ccl_comp_pointer_lookups() == n0
    assert np.array_equal(dst[5:5 + nbytes], src[3:3 + nbytes])
    assert not dst[:5].any() and not dst[5 + nbytes:].any()
    dst[:] = 0
    n0 = shim.mi_ccl_comp_pointer_lookups()
    _lib.check_shim(shim.mi_ccl_comp_copy(src.ctypes.data, dst.ctypes.data, nbytes, nt), "copy")
    assert shim.mi_ccl_comp_pointer_lookups() - n0 == 2
    assert np.array_equal(dst[:nbytes], src[:nbytes])


def test_copy_host_argument_errors(shim):
    a = np.zeros(16, np.uint8)
    assert shim.mi_ccl_comp_copy_host(None, a.ctypes.data, 16, 0) == -1
    assert b"in_buf is null" in shim.mi_ccl_last_error()
    assert shim.mi_ccl_comp_copy_host(a.ctypes.data, None, 16, 0) == -1
    assert shim.mi_ccl_comp_copy_host(None, None, 0, 0) == 0  # empty: nothing checked, as ccl_comp_copy
