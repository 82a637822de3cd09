"""Seeded random sweep of the drop-in's dispatcher on host buckets: the CPU
path, the synchronous split and the asynchronous split (head on the worker's
helper thread), through ccl_comp_reduce / ccl_comp_batch_reduce and their
_start forms, against the oracle's restatement of the reference.

Every case draws a dtype, an op, a fan-in K (1 = the 2-input ccl_comp_reduce),
a bucket size around a threshold it also draws (so most cases split and some
stay on the CPU), a pointer kind (pinned / pageable), an element offset, the
entry (synchronous or asynchronous) and, for bf16 fan-ins, keep-precision
mode.  MI_FUZZ_CASES scales it (cases = MI_FUZZ_CASES / 5)."""
from __future__ import annotations

import os

import numpy as np
import pytest

import oracle
from oneccl_amd import comp
from tests.util import ALL_DTYPES, BF16, DT_NAME, OP_NAME, OPS, assert_same, rand_array

pytestmark = pytest.mark.gpu

N_CASES = int(os.environ.get("MI_FUZZ_CASES", "1000")) // 5
KNOBS = ("CCL_COMP_HOST_MAX_BYTES", "CCL_COMP_HOST_MAX_PINNED_BYTES", "CCL_COMP_HOST_SHARE",
         "CCL_COMP_HOST_SHARE_PINNED", "CCL_COMP_HOST_SHARE_ADAPT", "CCL_COMP_HOST_SPLIT_WORKERS",
         "CCL_COMP_HOST_SPLIT_WORKERS_PINNED")


def _cases():
    rng = np.random.default_rng(2026)
    out = []
    for i in range(N_CASES):
        dt = int(rng.choice(ALL_DTYPES))
        op = int(rng.choice(OPS))
        k = int(rng.choice([1, 1, 2, 3, 4, 8, 16, 19]))
        thr_kib = int(rng.choice([16, 64, 256, 1024]))
        es = np.dtype(oracle.NP_DTYPE[dt]).itemsize
        n = max(1, int(thr_kib * 1024 * rng.uniform(0.5, 6.0)) // es + int(rng.integers(0, 300)))
        pinned = bool(rng.random() < 0.4)
        off = int(rng.integers(0, 16))
        asyn = bool(rng.random() < 0.5)
        keep = int(dt == BF16 and k > 1 and rng.random() < 0.5)
        share = str(rng.choice(["adapt", "0.2", "0.45", "0.8"]))
        out.append((i, dt, op, k, n, thr_kib, pinned, off, asyn, keep, share))
    return out


CASES = _cases()


@pytest.fixture
def env():
    saved = {k: os.environ.get(k) for k in KNOBS}
    yield
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    comp.env_reload()


@pytest.mark.parametrize("case", CASES, ids=[f"d{c[0]}-{DT_NAME[c[1]]}-{OP_NAME[c[2]]}-k{c[3]}-n{c[4]}-"
                                             f"{'pin' if c[6] else 'page'}-{'async' if c[8] else 'sync'}"
                                             for c in CASES])
def test_random_dispatch_case(case, env):
    import torch
    i, dt, op, k, n, thr_kib, pinned, off, asyn, keep, share = case
    for kk in KNOBS:
        os.environ.pop(kk, None)
    os.environ["CCL_COMP_HOST_MAX_BYTES"] = str(thr_kib << 10)
    os.environ["CCL_COMP_HOST_MAX_PINNED_BYTES"] = str(thr_kib << 10)
    if share != "adapt":
        os.environ["CCL_COMP_HOST_SHARE"] = share
        os.environ["CCL_COMP_HOST_SHARE_PINNED"] = share
    comp.env_reload()
    b_impl, f_impl = comp.impl_types()
    nin = 2 if k == 1 else k
    ins = [rand_array(dt, n, seed=90_000 + 131 * i + j, op=op, specials=dt not in (BF16,) or not keep)
           for j in range(nin)]
    es = ins[0].itemsize
    if k == 1:  # ccl_comp_reduce: inout = op(in, inout)
        exp = ins[0].copy()
        oracle.comp_reduce(ins[1], exp, dt, op, int(b_impl), int(f_impl))
    else:
        exp = ins[0].copy()
        oracle.batch_reduce(np.concatenate(ins), [j * n for j in range(k)], n, exp, dt, op, keep, int(b_impl),
                            int(f_impl))
    # one host buffer holding every input back to back at an element offset
    packed = np.zeros(off + nin * n + 16, ins[0].dtype)
    for j in range(nin):
        packed[off + j * n:off + (j + 1) * n] = ins[j]
    acc = np.zeros(off + n + 16, ins[0].dtype)
    acc[off:off + n] = ins[0]
    if pinned:
        tp = torch.from_numpy(packed.view(np.uint8).copy()).pin_memory()
        ta = torch.from_numpy(acc.view(np.uint8).copy()).pin_memory()
        p_in, p_acc = tp.data_ptr() + off * es, ta.data_ptr() + off * es

        def read():
            return ta.numpy().view(exp.dtype)[off:off + n].copy()
    else:
        p_in, p_acc = packed.ctypes.data + off * es, acc.ctypes.data + off * es

        def read():
            return acc[off:off + n].copy()
    dtype, red = comp.datatype(dt), comp.reduction(op)
    if k == 1:
        src = p_in + n * es  # input 1
        if asyn:
            req = comp.comp_reduce_start(src, n, p_acc, dtype, red)
            req.wait()
            req.free()
        else:
            comp.comp_reduce(src, n, p_acc, dtype, red)
    else:
        offsets = [j * n for j in range(k)]  # offsets[0] names the accumulator's slot and is not read
        if asyn:
            req = comp.comp_batch_reduce_start(p_in, offsets, n, p_acc, dtype, red, keep)
            req.wait()
            req.free()
        else:
            comp.comp_batch_reduce(p_in, offsets, n, p_acc, dtype, red, keep)
    assert_same(read(), exp, dt, f"case {case}")
