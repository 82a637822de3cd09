"""mi_reduce_batch: many independent in-place reduces in one dispatch, each
checked bit-exactly against the oracle's ccl_comp_reduce on its own
operands (NaN payloads aside).  Descriptor counts cross the 64-per-launch
split.  Counts run from empty to multi-tile, and each operand has its own
element offset: common and differing misalignments, plus a byte-misaligned
fp32 pair that takes the element loop.
"""
from __future__ import annotations

import numpy as np
import pytest

import oracle
from oneccl_amd import _lib
from oneccl_amd.comp import F_MINMAX_INOUT_FIRST, bf16_flags
from tests.util import ALL_DTYPES, BF16, DT_NAME, FP16, FP32, OP_NAME, OPS, assert_same, rand_array

pytestmark = pytest.mark.gpu

SIZES = [0, 1, 7, 17, 255, 4096, 16384 + 9, 100_003]


class Pool:
    """Slots carved from one device allocation, 256 B apart."""

    def __init__(self, nbytes: int):
        import torch
        self.t = torch.zeros(nbytes, dtype=torch.uint8, device="cuda")
        self.base = self.t.data_ptr()
        self.off = 0

    def put(self, a: np.ndarray, byte_off: int) -> int:
        import torch
        o = self.off + byte_off
        raw = a.view(np.uint8)
        self.t[o:o + raw.size].copy_(torch.from_numpy(raw.copy()))
        self.off = (o + raw.size + 256 + 255) // 256 * 256
        return o

    def get(self, o: int, like: np.ndarray) -> np.ndarray:
        return self.t[o:o + like.nbytes].cpu().numpy().view(like.dtype).copy()


def _flags(dt, variant):
    if dt == BF16:
        return bf16_flags(variant), [oracle.BF16_SCALAR, oracle.BF16_AVX512F, oracle.BF16_AVX512BF][variant]
    return (F_MINMAX_INOUT_FIRST if dt == FP16 else 0), oracle.BF16_AVX512BF


def _run_batch(dt, op, variant, n, seed, misalign):
    import torch
    rng = np.random.default_rng(seed)
    flags, bimpl = _flags(dt, variant)
    es = np.dtype(oracle.NP_DTYPE[dt]).itemsize
    cases = []
    total = 0
    for i in range(n):
        cnt = int(rng.choice(SIZES))
        a = rand_array(dt, cnt, seed=seed * 1000 + 2 * i, op=op)
        b = rand_array(dt, cnt, seed=seed * 1000 + 2 * i + 1, op=op)
        if misalign == "common":
            o = int(rng.integers(0, 16 // es)) * es
            offs = (o, o)
        elif misalign == "differing":
            offs = tuple(int(x) * es for x in rng.integers(0, 16 // es, size=2))
        else:
            offs = (0, 0)
        cases.append((a, b, offs))
        total += 2 * (a.nbytes + 2 * 256 + 16)
    pool = Pool(total + 4096)
    placed = []
    for a, b, (oa, ob) in cases:
        pa = pool.put(a, oa)
        pb = pool.put(b, ob)
        placed.append((pa, pb))
    descs = _lib.desc_array([(pool.base + pa, pool.base + pb, a.size) for (a, _, _), (pa, pb) in zip(cases, placed)])
    _lib.check(_lib.mi().mi_reduce_batch(descs, n, dt, op, flags, torch.cuda.current_stream().cuda_stream),
               "mi_reduce_batch")
    torch.cuda.synchronize()
    for i, ((a, b, _), (pa, pb)) in enumerate(zip(cases, placed)):
        exp = b.copy()
        if a.size:
            oracle.comp_reduce(a, exp, dt, op, bimpl, oracle.FP16_AVX512F)
        assert_same(pool.get(pb, b), exp, dt, f"descriptor {i} (count {a.size})")
        assert_same(pool.get(pa, a), a, dt, f"descriptor {i} input modified")


@pytest.mark.parametrize("dt", ALL_DTYPES, ids=[DT_NAME[d] for d in ALL_DTYPES])
@pytest.mark.parametrize("op", OPS, ids=[OP_NAME[o] for o in OPS])
def test_batch_all_dtypes_ops(dt, op):
    _run_batch(dt, op, 2 if dt == BF16 else 0, n=70, seed=dt * 10 + op + 1, misalign="differing")


@pytest.mark.parametrize("variant", [0, 1, 2])
@pytest.mark.parametrize("op", OPS, ids=[OP_NAME[o] for o in OPS])
def test_batch_bf16_variants(variant, op):
    _run_batch(BF16, op, variant, n=20, seed=500 + 10 * variant + op, misalign="common")


@pytest.mark.parametrize("n", [1, 63, 64, 65, 200])
def test_batch_split_across_launches(n):
    _run_batch(FP32, 0, 0, n=n, seed=900 + n, misalign="none")


def test_batch_in_equals_inout_and_byte_misaligned():
    """x = op(x, x) in one descriptor (allowed, as for mi_reduce) next to an
    fp32 pair at odd byte offsets (the element loop, its own launch)."""
    import torch
    pool = Pool(1 << 20)
    x = rand_array(FP32, 5000, seed=1)
    a = rand_array(FP32, 3001, seed=2)
    b = rand_array(FP32, 3001, seed=3)
    px = pool.put(x, 0)
    pa = pool.put(a, 1)
    pb = pool.put(b, 3)
    descs = _lib.desc_array([(pool.base + px, pool.base + px, x.size), (pool.base + pa, pool.base + pb, a.size)])
    _lib.check(_lib.mi().mi_reduce_batch(descs, 2, FP32, 0, 0, torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    ex = x.copy()
    oracle.comp_reduce(x.copy(), ex, FP32, 0)
    eb = b.copy()
    oracle.comp_reduce(a, eb, FP32, 0)
    assert_same(pool.get(px, x), ex, FP32, "in == inout")
    assert_same(pool.get(pb, b), eb, FP32, "byte-misaligned pair")


def test_batch_refuses_overlap():
    import torch
    m = _lib.mi()
    t = torch.zeros(1 << 16, dtype=torch.float32, device="cuda")
    p = t.data_ptr()
    s = torch.cuda.current_stream().cuda_stream
    # two descriptors writing the same range
    assert m.mi_reduce_batch(_lib.desc_array([(p, p + 4096, 100), (p + 8192, p + 4096, 100)]), 2, FP32, 0, 0, s) == -1
    assert b"overlap" in m.mi_last_error()
    # partial overlap of outputs
    assert m.mi_reduce_batch(_lib.desc_array([(p, p + 4096, 100), (p + 8192, p + 4096 + 396, 100)]), 2, FP32, 0, 0,
                             s) == -1
    # one descriptor's input is another's output
    assert m.mi_reduce_batch(_lib.desc_array([(p, p + 4096, 100), (p + 4096 + 200, p + 16384, 100)]), 2, FP32, 0, 0,
                             s) == -1
    # adjacent, touching ranges and a shared input are fine
    assert m.mi_reduce_batch(_lib.desc_array([(p, p + 4096, 100), (p, p + 4096 + 400, 100)]), 2, FP32, 0, 0, s) == 0
    torch.cuda.synchronize()


def test_batch_refuses_wrapping_count():
    """A count whose byte range would wrap past the end of the address space
    is refused (MI_E_INVALID), not launched."""
    import torch
    m = _lib.mi()
    t = torch.zeros(1 << 12, dtype=torch.float32, device="cuda")
    p = t.data_ptr()
    s = torch.cuda.current_stream().cuda_stream
    huge = (1 << 64) // 4 - 1
    assert m.mi_reduce_batch(_lib.desc_array([(p, p + 4096, 16), (p + 8192, p + 12288, huge)]), 2, FP32, 0, 0,
                             s) == -1
    assert b"overflow" in m.mi_last_error()
    torch.cuda.synchronize()
