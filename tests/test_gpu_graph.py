"""The asynchronous entry points inside a captured HIP graph.

A oneCCL schedule runs the same chain of entries on the same buffers at
every iteration of a training step: copy the own chunk into the accumulator,
fold each peer's chunk into it, convert the result (the copy_entry /
reduce_local_entry / recv_reduce_entry sequence of the ring algorithms,
src/coll/algorithms/allreduce/allreduce.cpp:333-394, src/sched/entry/).  A
caller can capture that chain once on its stream and replay it as one
submission.  These tests capture mi_copy, mi_reduce, mi_reduce_out,
mi_reduce_multi and mi_convert in a torch CUDA graph (a hipGraph on ROCm),
then replay it on fresh data and check every result against the oracle:
the replay must re-read the buffers, not reuse captured values.
"""
from __future__ import annotations

import numpy as np
import pytest

import oracle
from oneccl_amd import _lib, comp
from tests.util import BF16, FP32, assert_same, rand_array

pytestmark = pytest.mark.gpu

SUM, MAX = 0, 3


def _dev(n, dtype):
    import torch
    return torch.empty(n, dtype=dtype, device="cuda")


@pytest.mark.parametrize("n", [1, 3 * 4096 + 5, 1 << 20])
def test_captured_schedule_replays(n):
    import torch
    m = _lib.mi()
    P = 4
    own = _dev(n, torch.float32)
    peers = [_dev(n, torch.float32) for _ in range(P - 1)]
    acc = _dev(n, torch.float32)
    outp = _dev(n, torch.float32)
    fan = _dev(n, torch.float32)
    bf = _dev(n, torch.int16)

    def fill(seed):
        arrays = [rand_array(FP32, n, seed=seed + j) for j in range(P)]
        for t, a in zip([own] + peers, arrays):
            t.copy_(torch.from_numpy(a))
        for t in (acc, outp, fan):
            t.fill_(-7.0)
        bf.fill_(0)
        return arrays

    fill(1)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    ins = _lib.void_ptr_array([t.data_ptr() for t in [own] + peers])
    with torch.cuda.graph(g):
        s = torch.cuda.current_stream().cuda_stream
        _lib.check(m.mi_copy(own.data_ptr(), acc.data_ptr(), n * 4, 1, s), "mi_copy")
        for p in peers:
            _lib.check(m.mi_reduce(p.data_ptr(), acc.data_ptr(), n, FP32, SUM, 0, s))
        _lib.check(m.mi_reduce_out(own.data_ptr(), peers[0].data_ptr(), outp.data_ptr(), n, FP32, MAX, 0, s))
        _lib.check(m.mi_reduce_multi(ins, P, fan.data_ptr(), n, FP32, SUM, 0, s))
        _lib.check(m.mi_convert(acc.data_ptr(), FP32, bf.data_ptr(), BF16, n, comp.F_BF16_RNE | comp.F_BF16_TAIL_TRUNC16, s),
                   "mi_convert")

    L = oracle.lib()
    for seed in (11, 23, 37):
        arrays = fill(seed)
        g.replay()
        torch.cuda.synchronize()
        exp_acc = arrays[0].copy()
        for a in arrays[1:]:
            oracle.comp_reduce(a, exp_acc, FP32, SUM)
        assert_same(acc.cpu().numpy(), exp_acc, FP32, f"chained reduce, seed {seed}")
        exp_out = arrays[1].copy()
        oracle.comp_reduce(arrays[0], exp_out, FP32, MAX)
        assert_same(outp.cpu().numpy(), exp_out, FP32, f"out-of-place max, seed {seed}")
        assert_same(fan.cpu().numpy(), oracle.fanin(arrays, FP32, SUM), FP32, f"fan-in, seed {seed}")
        exp_bf = np.empty(n, np.uint16)
        L.orc_convert_fp32_to_bf16_arrays(exp_acc.ctypes.data, exp_bf.ctypes.data, n, oracle.BF16_AVX512BF)
        assert_same(bf.cpu().numpy().view(np.uint16), exp_bf, BF16, f"convert, seed {seed}")


def test_capture_refuses_pageable_operand():
    """The pageable-pointer check runs at capture time: the entry returns an
    error and records nothing, so a bad schedule fails when it is built."""
    import torch
    m = _lib.mi()
    host = np.zeros(4096, np.float32)
    dev = _dev(4096, torch.float32)
    dev.zero_()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        s = torch.cuda.current_stream().cuda_stream
        rc = m.mi_reduce(host.ctypes.data, dev.data_ptr(), 4096, FP32, SUM, 0, s)
        dev.fill_(1.0)  # the capture itself stays usable
    assert rc == -1  # MI_E_INVALID
    g.replay()
    torch.cuda.synchronize()
    assert bool((dev == 1.0).all())
