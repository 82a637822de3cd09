"""Shared helpers for the parity tests: seeded inputs (with the special
values the reference's semantics distinguish, NaNs with payloads of both
signs among them), numpy<->device transfer and the comparison rule
(bit-exact, NaN payloads included for every type: the kernels and the host
path restate x86's NaN rules for the reference's AVX-512 paths and for its
compiled CCL_REDUCE, tests/golden/ref_comp_vectors.npz)."""
from __future__ import annotations

import numpy as np

import oracle

# ccl::datatype ids
INT_DTYPES = [0, 1, 2, 3, 4, 5, 6, 7]
FP16, FP32, FP64, BF16 = 8, 9, 10, 11
ALL_DTYPES = INT_DTYPES + [FP16, FP32, FP64, BF16]
OPS = [0, 1, 2, 3]
DT_NAME = {0: "int8", 1: "uint8", 2: "int16", 3: "uint16", 4: "int32", 5: "uint32", 6: "int64", 7: "uint64",
           8: "float16", 9: "float32", 10: "float64", 11: "bfloat16"}
OP_NAME = {0: "sum", 1: "prod", 2: "min", 3: "max"}

F32_SPECIALS = np.concatenate([
    np.array([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, np.nan, -np.nan, 1e-40, -1e-40, 1e-45,
              3.4e38, -3.4e38, 1.17549435e-38, 65504.0, 6.1e-5, 5.96e-8, 2.0 ** -126], dtype=np.float32),
    # quiet NaNs with payloads of both signs and a signalling NaN
    np.array([0x7FC00123, 0xFFC00456, 0x7F800005], dtype=np.uint32).view(np.float32)])


def rand_array(dtype: int, n: int, seed: int, op: int = 0, specials: bool = True) -> np.ndarray:
    """Seeded input of ccl datatype `dtype` (storage dtype as in oracle.NP_DTYPE)."""
    rng = np.random.default_rng(seed)
    st = oracle.NP_DTYPE[dtype]
    if dtype in INT_DTYPES:
        info = np.iinfo(st)
        if op == 1:  # keep products from being all-zero quickly; wraps still exercised
            a = rng.integers(-3, 4, size=n).astype(np.int64)
            if info.min == 0:
                a = np.abs(a)
            a = a.astype(st)
        else:
            a = rng.integers(info.min, info.max, size=n, endpoint=True, dtype=st)
        if specials and n > 8:
            idx = rng.choice(n, size=min(n, 8), replace=False)
            a[idx[:4]] = info.min
            a[idx[4:]] = info.max
        return a
    if dtype == FP64:
        a = rng.standard_normal(n) * (10.0 ** rng.integers(-3, 4, size=n))
        if specials and n > 40:
            idx = rng.choice(n, size=len(F32_SPECIALS) + 3, replace=False)
            with np.errstate(invalid="ignore"):  # the signalling NaN quiets on widening
                a[idx[:len(F32_SPECIALS)]] = F32_SPECIALS.astype(np.float64)
            a[idx[0]] = 1e-310  # fp64 denormal
            a.view(np.uint64)[idx[len(F32_SPECIALS):]] = np.array(  # fp64 NaN payloads, both signs, signalling
                [0x7FF8000000000123, 0xFFF8000000000456, 0x7FF0000000000007], np.uint64)
        return a
    f = (rng.standard_normal(n) * (2.0 ** rng.integers(-8, 9, size=n))).astype(np.float32)
    if specials and n > 40:
        idx = rng.choice(n, size=len(F32_SPECIALS), replace=False)
        f[idx] = F32_SPECIALS
    if dtype == FP32:
        return f
    if dtype == BF16:
        b = oracle.f32_to_bf16(f, rne=True)
        if specials and n > 40:  # bf16 denormals and tiny values
            idx = rng.choice(n, size=6, replace=False)
            b[idx] = np.array([0x0001, 0x8001, 0x007F, 0x0080, 0x7F7F, 0xFF7F], np.uint16)
        return b
    # fp16
    h = oracle.f32_to_fp16(np.clip(f, -60000, 60000))
    if specials and n > 40:
        idx = rng.choice(n, size=8, replace=False)
        h[idx] = np.array([0x0001, 0x8001, 0x03FF, 0x0400, 0x7BFF, 0xFBFF, 0x7C00, 0x7E00], np.uint16)
    return h


def is_nan_bits(a: np.ndarray, dtype: int) -> np.ndarray:
    if dtype == BF16:
        return ((a & 0x7F80) == 0x7F80) & ((a & 0x007F) != 0)
    if dtype == FP16:
        return ((a & 0x7C00) == 0x7C00) & ((a & 0x03FF) != 0)
    if dtype in (FP32, FP64):
        return np.isnan(a)
    return np.zeros(a.shape, bool)


# NaN payloads count for every type.  Round 2 left the both-NaN choice of
# float/double CCL_REDUCE and of keep-precision's fp32 scratch fold unpinned
# (a compiler-vectorized `inout op= in`); the reference's own compiled
# comp.cpp now pins it (tests/golden/ref_comp_vectors.npz: inout's NaN wins,
# inf - inf gives 0xFFC00000), and the kernels, the host path and the oracle
# restate that rule.  nan_payload=False remains for callers that compare
# against something that does not model payloads (e.g. numpy).


def assert_same(got: np.ndarray, exp: np.ndarray, dtype: int, what: str = "", nan_payload=True) -> None:
    """Bit-exact comparison, NaN payloads included (nan_payload=False: two
    NaNs compare equal)."""
    assert got.shape == exp.shape and got.itemsize == exp.itemsize
    iv = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[got.itemsize]
    cand = np.flatnonzero(got.view(iv) != exp.view(iv))
    if cand.size and not nan_payload:
        both_nan = is_nan_bits(got[cand], dtype) & is_nan_bits(exp[cand], dtype)
        cand = cand[~both_nan]
    if cand.size:
        i = cand
        raise AssertionError(f"{what}: {len(i)} of {got.size} elements differ; first at {i[:5].tolist()}: "
                             f"got {got[i[:5]].tolist()} expected {exp[i[:5]].tolist()}")


# ---- device transfer (torch is plumbing only) ----------------------------
_SIGNED = {1: np.int8, 2: np.int16, 4: np.int32, 8: np.int64}


def to_dev(a: np.ndarray, pad_elems: int = 0, offset_elems: int = 0):
    """Copy to a fresh device buffer; returns (tensor_holder, device_ptr).
    `offset_elems` shifts the data inside the buffer to test misaligned
    pointers."""
    import torch
    es = a.itemsize
    raw = np.zeros(a.size + pad_elems + offset_elems, a.dtype)
    raw[offset_elems:offset_elems + a.size] = a
    t = torch.from_numpy(raw.view(_SIGNED[es])).cuda()
    return t, t.data_ptr() + offset_elems * es


def from_dev(t, like: np.ndarray, offset_elems: int = 0) -> np.ndarray:
    host = t.cpu().numpy().view(like.dtype)
    return host[offset_elems:offset_elems + like.size].copy()


def wait_os_threads_gone(native_ids, timeout=60.0):
    """Wait until the OS threads `native_ids` (threading.get_native_id() of
    each) have exited.  Python's Thread.join() returns when the thread's
    Python function ends, before the OS thread runs its thread_local
    destructors -- for the library, each thread's HIP context teardown
    (streams, staging buffers) -- so a GPU test that starts workers lets
    those teardowns finish here rather than overlap the next test."""
    import os
    import time
    t0 = time.monotonic()
    pending = set(native_ids)
    while pending and time.monotonic() - t0 < timeout:
        pending = {t for t in pending if os.path.exists(f"/proc/self/task/{t}")}
        if pending:
            time.sleep(0.005)
    return not pending
