"""The MPI user ops' reduce.

With the MPI transport, the default, a build without SYCL selects the
`direct` allreduce at every size (src/coll/selection/selector_allreduce.cpp:
54-57), so bf16/fp16 reductions run inside MPI's user ops on MPI's own host
buffers: bf16_base_op -> ccl_bf16_reduce (src/atl/mpi/atl_mpi_ctx.cpp:87-92)
and fp16_base_op -> the inline ccl_fp16_reduce_impl (:57-63).  integration/
0002 routes both through ccl_{bf16,fp16}_reduce_host
(include/mi_ccl_lp_host.hpp): host memory by the caller's word, so a bucket
up to the dispatcher's threshold is folded on the calling thread's CPU with
no pointer lookup, under any number of concurrent callers.  CPU-only; bits
against the oracle (pinned to the reference's compiled AVX-512 bodies,
tests/test_ref_vectors.py) under every bf16/fp16 impl type."""
import ctypes
import os
import threading

import numpy as np
import pytest

import oracle
from oneccl_amd import _lib, comp
from tests.util import BF16, FP16, OP_NAME, OPS, assert_same, rand_array

BF16_IMPLS = [("scalar", 0), ("avx512f", 1), ("avx512bf", 2)]
FP16_IMPLS = [("f16c", 2), ("avx512f", 3)]


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


def _fold(s, entry, a, b, op, out_count=True):
    oc = ctypes.c_size_t(0)
    rc = getattr(s, entry)(a.ctypes.data, a.size, b.ctypes.data, ctypes.byref(oc) if out_count else None, op)
    _lib.check_shim(rc, entry)
    return oc.value


@pytest.mark.parametrize("setting,impl", BF16_IMPLS)
@pytest.mark.parametrize("n", [1, 15, 4099, 131072])
def test_bf16_user_op_no_lookup_exact_bits(env, setting, impl, n):
    env(CCL_BF16=setting)
    s = _lib.shim()
    for op in OPS:
        a = rand_array(BF16, n, seed=10 + op)
        b0 = rand_array(BF16, n, seed=20 + op)
        exp = b0.copy()
        oracle.comp_reduce(a, exp, BF16, op, impl)
        b = b0.copy()
        n0 = s.mi_ccl_comp_pointer_lookups()
        assert _fold(s, "mi_ccl_bf16_reduce_host", a, b, op) == n  # *out_count, bf16.cpp:94-96
        assert s.mi_ccl_comp_pointer_lookups() == n0, "the MPI user op looked an operand up"
        assert_same(b, exp, BF16, f"bf16 {setting} {OP_NAME[op]}")


@pytest.mark.parametrize("setting,impl", FP16_IMPLS)
@pytest.mark.parametrize("n", [1, 15, 4099, 131072])
def test_fp16_user_op_no_lookup_exact_bits(env, setting, impl, n):
    env(CCL_FP16=setting)
    s = _lib.shim()
    for op in OPS:
        a = rand_array(FP16, n, seed=30 + op)
        b0 = rand_array(FP16, n, seed=40 + op)
        exp = b0.copy()
        oracle.comp_reduce(a, exp, FP16, op, 2, impl)
        b = b0.copy()
        n0 = s.mi_ccl_comp_pointer_lookups()
        _fold(s, "mi_ccl_fp16_reduce_host", a, b, op, out_count=False)  # fp16_base_op passes no out_count
        assert s.mi_ccl_comp_pointer_lookups() == n0, "the MPI user op looked an operand up"
        assert_same(b, exp, FP16, f"fp16 {setting} {OP_NAME[op]}")


def test_plain_entries_still_look_up():
    """Without the caller's word (ccl_bf16_reduce from any other caller) the
    operands are still classified: the host entry is the only change."""
    s = _lib.shim()
    a, b = rand_array(BF16, 1024, 1), rand_array(BF16, 1024, 2)
    n0 = s.mi_ccl_comp_pointer_lookups()
    _fold(s, "mi_ccl_bf16_reduce", a, b, 0)
    assert s.mi_ccl_comp_pointer_lookups() - n0 == 2


def test_host_entry_word_ends_with_the_call():
    """The word holds for one call: a later plain call on the same thread
    classifies again (SchedScope restores the previous word)."""
    s = _lib.shim()
    a, b = rand_array(FP16, 512, 3), rand_array(FP16, 512, 4)
    _fold(s, "mi_ccl_fp16_reduce_host", a, b, 0)
    n0 = s.mi_ccl_comp_pointer_lookups()
    _fold(s, "mi_ccl_fp16_reduce", a, b, 0)
    assert s.mi_ccl_comp_pointer_lookups() - n0 == 2


def test_bad_op_is_fatal_in_a_child():
    """An op outside sum/prod/min/max is CCL_FATAL, as in ccl_bf16_reduce
    (bf16.cpp:73): the process terminates (checked in a child)."""
    import subprocess
    import sys
    code = ("import numpy as np, ctypes\n"
            "from oneccl_amd import _lib\n"
            "a = np.zeros(8, np.uint16); b = np.zeros(8, np.uint16)\n"
            "_lib.shim().mi_ccl_bf16_reduce_host(a.ctypes.data, 8, b.ctypes.data, None, 7)\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode != 0 and "FATAL" in r.stderr, r.stderr[-2000:]


@pytest.mark.parametrize("dt,entry", [(BF16, "mi_ccl_bf16_reduce_host"), (FP16, "mi_ccl_fp16_reduce_host")])
def test_concurrent_user_ops_make_no_lookup(dt, entry):
    """Eight threads folding 4 KiB chunks through the user op at once (MPI
    may call it from several threads): no lookup anywhere, exact bits."""
    errors = []
    b_impl, f_impl = comp.impl_types()

    def worker(seed):
        s = _lib.shim()
        a = rand_array(dt, 2048, seed, specials=False)
        b = rand_array(dt, 2048, seed + 100, specials=False)
        exp = b.copy()
        n0 = s.mi_ccl_comp_pointer_lookups()
        for op in (0, 3, 2, 0):
            for _ in range(50):
                if getattr(s, entry)(a.ctypes.data, a.size, b.ctypes.data, None, op) != 0:
                    errors.append("rc")
                oracle.comp_reduce(a, exp, dt, op, int(b_impl), int(f_impl))
        if s.mi_ccl_comp_pointer_lookups() != n0:
            errors.append("lookup")
        if not np.array_equal(b.view(np.uint16), exp.view(np.uint16)):
            errors.append("bits")

    ws = [threading.Thread(target=worker, args=(i,)) for i in range(8)]
    for w in ws:
        w.start()
    for w in ws:
        w.join()
    assert errors == []


@pytest.mark.gpu
@pytest.mark.parametrize("dt,entry", [(BF16, "mi_ccl_bf16_reduce_host"), (FP16, "mi_ccl_fp16_reduce_host")])
@pytest.mark.parametrize("kind", ["pageable", "pinned"])
def test_large_user_op_bucket_on_the_gpu(dt, entry, kind):
    """Above the dispatcher's threshold (16 MiB) a user op's bucket is split
    between the calling thread and the GPU: its operands are looked up (their
    kinds pick pinned zero-copy or staging), and the bits are the oracle's
    under the impl type in force."""
    import torch
    s = _lib.shim()
    b_impl, f_impl = comp.impl_types()
    n = (40 << 20) // 2 + 77
    a = rand_array(dt, n, seed=61, specials=False)
    b0 = rand_array(dt, n, seed=62, specials=False)
    exp = b0.copy()
    oracle.comp_reduce_mt(a, exp, dt, 0, 8, int(b_impl), int(f_impl))
    if kind == "pinned":
        ha = torch.from_numpy(a.view(np.uint8).copy()).pin_memory()
        hb = torch.from_numpy(b0.view(np.uint8).copy()).pin_memory()
        pa, pb = ha.data_ptr(), hb.data_ptr()
    else:
        b = b0.copy()
        pa, pb = a.ctypes.data, b.ctypes.data
    n0 = s.mi_ccl_comp_pointer_lookups()
    _lib.check_shim(getattr(s, entry)(pa, n, pb, None, 0), entry)
    assert s.mi_ccl_comp_pointer_lookups() - n0 > 0
    got = hb.numpy().view(a.dtype) if kind == "pinned" else b
    assert_same(got, exp, dt, f"{entry} {kind}")
