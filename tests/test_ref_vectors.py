"""The oracle against golden vectors produced by the REFERENCE'S OWN bf16/fp16
reduce code (tests/golden/ref_vectors.npz; producer: oracle/ref_harness.cpp
over /root/reference/src/comp/{bf16,fp16}/*_intrisics.{hpp,cpp}).

Bar: identical bits, NaN payloads included — the oracle restates the x86
NaN propagation the reference's AVX-512 code has (comp_oracle.c
x86_nan_first).  Where the reference tree is present (this container) the
fixture is also regenerated from the reference code and compared with the
committed file, so the fixture cannot drift from what the reference computes.
"""
from __future__ import annotations

import subprocess
import json
from pathlib import Path

import numpy as np
import pytest

import oracle
from tests import refvec

ROOT = Path(__file__).resolve().parent.parent
REF = Path("/root/reference/src/comp")


def _oracle_reduce(c):
    n = c["count"]
    b = c["b"].copy()
    pa, pb = c["a"][:n].copy(), b[:n].copy()
    bimpl = c["impl"] if c["dtype"] == refvec.BF16 else oracle.BF16_AVX512BF
    fimpl = c["impl"] if c["dtype"] == refvec.FP16 else oracle.FP16_AVX512F
    oracle.comp_reduce(pa, pb, c["dtype"], c["op"], bimpl, fimpl)
    b[:n] = pb
    return b


@pytest.mark.parametrize("c", refvec.reduce_cases(), ids=lambda c: c["key"])
def test_oracle_reduce_matches_reference_code(c):
    got = _oracle_reduce(c)
    diff = np.flatnonzero(got != c["expected"])
    assert diff.size == 0, f"{c['key']}: {diff.size} elements differ, first {diff[:5].tolist()}: " \
                           f"oracle {got[diff[:5]].tolist()} reference {c['expected'][diff[:5]].tolist()}"


@pytest.mark.parametrize("c", refvec.fan_cases(), ids=lambda c: c["key"])
def test_oracle_chained_fanin_matches_reference_code(c):
    bimpl = c["impl"] if c["dtype"] == refvec.BF16 else oracle.BF16_AVX512BF
    fimpl = c["impl"] if c["dtype"] == refvec.FP16 else oracle.FP16_AVX512F
    got = oracle.fanin([x.copy() for x in c["inputs"]], c["dtype"], c["op"], bimpl, fimpl)
    assert np.array_equal(got, c["expected"])


@pytest.mark.parametrize("impl,f,exp", refvec.conversion_cases(), ids=["avx512f", "avx512bf"])
def test_oracle_bf16_conversion_matches_reference_code(impl, f, exp):
    got = np.empty(f.size, np.uint16)
    oracle.lib().orc_convert_fp32_to_bf16_arrays(f.ctypes.data, got.ctypes.data, f.size, impl)
    assert np.array_equal(got, exp)


def test_oracle_bf16_load_matches_reference_code():
    src, exp = refvec.load_case()
    got = np.empty(src.size, np.float32)
    oracle.lib().orc_convert_bf16_to_fp32_arrays(src.ctypes.data, got.ctypes.data, src.size)
    assert np.array_equal(got.view(np.uint32), exp.view(np.uint32))


def test_fixture_covers_every_avx512_variant():
    cases = refvec.reduce_cases()
    seen = {(c["dtype"], c["impl"], c["op"]) for c in cases}
    assert seen == {(dt, i, op) for dt, impls in ((refvec.BF16, (1, 2)), (refvec.FP16, (2, 3, 4)))
                    for i in impls for op in range(4)}
    counts = {c["count"] for c in cases if c["impl"] != 4 or c["dtype"] != refvec.FP16}
    assert counts == {2061, 16, 15, 1}  # odd 16- and 8-wide tails, one full vector, a lone element
    native = {c["count"] for c in cases if c["impl"] == 4 and c["dtype"] == refvec.FP16}
    assert native == {2061, 32, 31, 1}  # avx512fp16: 32-wide body, masked tails


@pytest.mark.skipif(not REF.is_dir(), reason="reference tree absent (GPU box): the committed fixture is used")
def test_fixture_regenerates_from_reference_code():
    """Rebuild oracle/_ref from the reference sources and regenerate every
    vector: identical to the committed fixture."""
    r = subprocess.run(["make", "-C", str(ROOT / "oracle"), "ref"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    import importlib.util
    spec = importlib.util.spec_from_file_location("mrv", ROOT / "tests" / "golden" / "make_ref_vectors.py")
    mrv = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mrv)
    fresh = mrv.generate()
    committed, _ = refvec.load()
    for k, v in fresh.items():
        if k == "meta":
            continue
        assert v.dtype == committed[k].dtype and np.array_equal(v.view(np.uint8), committed[k].view(np.uint8)), k


def _has_avx512fp16():
    try:
        return "avx512_fp16" in Path("/proc/cpuinfo").read_text()
    except OSError:
        return False


@pytest.mark.skipif(not REF.is_dir() or not _has_avx512fp16(),
                    reason="needs the reference tree and a CPU with AVX512_FP16 (the committed fixture is used)")
def test_fp16native_fixture_regenerates_from_reference_code():
    """The avx512fp16 vectors: rebuild oracle/_ref/libref_fp16native.so (clang++
    over the reference's fp16_intrisics.cpp) and regenerate; identical."""
    r = subprocess.run(["make", "-C", str(ROOT / "oracle"), "ref"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    import importlib.util
    import sys
    sys.path.insert(0, str(ROOT / "tests" / "golden"))
    spec = importlib.util.spec_from_file_location("mrvn", ROOT / "tests" / "golden" / "make_ref_vectors_fp16native.py")
    mrvn = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mrvn)
    fresh = mrvn.generate()
    z = np.load(refvec.PATH_FP16NATIVE)
    for k, v in fresh.items():
        if k == "meta":
            continue
        assert v.dtype == z[k].dtype and np.array_equal(v.view(np.uint8), z[k].view(np.uint8)), k


def test_fp16native_reference_code_exhaustive_result():
    """oracle/FP16_NATIVE_REF_CHECK.json: the reference's own avx512fp16 code
    against the oracle's model on all 2^32 (in, inout) pairs, every op."""
    d = json.loads((ROOT / "oracle" / "FP16_NATIVE_REF_CHECK.json").read_text())
    assert d["pairs_per_op"] == 1 << 32
    assert all(d["mismatches"][op] == 0 for op in ("sum", "prod", "min", "max"))
