"""The drop-in's dispatcher on a GPU box: host-resident
buckets up to CCL_COMP_HOST_MAX_BYTES run on the calling thread's CPU
(host_reduce.cpp), larger ones and device buffers on the GPU.  Both sides of
the threshold give the reference's bits; a host-path call after an
asynchronous GPU request of the same thread sees that request's result."""
from __future__ import annotations

import os
import subprocess
from pathlib import Path

import numpy as np
import pytest

import oracle
from oneccl_amd import comp
from tests.util import BF16, FP32, assert_same, rand_array, to_dev, from_dev

pytestmark = pytest.mark.gpu


@pytest.fixture
def threshold():
    saved = os.environ.get("CCL_COMP_HOST_MAX_BYTES")

    def set_(v):
        os.environ["CCL_COMP_HOST_MAX_BYTES"] = str(v)
        comp.env_reload()

    yield set_
    if saved is None:
        os.environ.pop("CCL_COMP_HOST_MAX_BYTES", None)
    else:
        os.environ["CCL_COMP_HOST_MAX_BYTES"] = saved
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
