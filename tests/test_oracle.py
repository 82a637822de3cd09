"""Pins the CPU oracle (oracle/comp_oracle.c) before it is trusted as the
checker: against the reference's own known-answer tests, the behaviours the
survey recorded from the compiled reference, and the real x86 instructions
the reference's src/comp calls (exhaustively, see oracle/ISA_CHECK.json)."""
from __future__ import annotations

import json
import subprocess
from pathlib import Path

import numpy as np
import pytest

import oracle
from tests import kat
from tests.util import BF16, FP16, FP32, OP_NAME, rand_array

ROOT = Path(__file__).resolve().parent.parent
IMPLS = {"scalar": oracle.BF16_SCALAR, "avx512f": oracle.BF16_AVX512F, "avx512bf": oracle.BF16_AVX512BF}


def test_isa_check_committed_exhaustive():
    d = json.loads((ROOT / "oracle" / "ISA_CHECK.json").read_text())
    assert d["stride"] == 1 and not d["skipped"]
    assert d["bf16_rne_checked"] == 1 << 32 and d["bf16_rne_bad"] == 0
    assert d["fp16_checked"] == (1 << 32) + 65536 and d["fp16_bad"] == 0
    assert d["minmax_bad"] == 0


def test_isa_check_live_sampled():
    exe = ROOT / "oracle" / "lib" / "isa_check"
    if not exe.exists():
        oracle.build()
    r = subprocess.run([str(exe), "65521"], capture_output=True, text=True)
    if r.returncode == 2:
        pytest.skip("this CPU lacks AVX512_BF16/F16C; the exhaustive run is committed")
    assert r.returncode == 0, r.stdout + r.stderr


def test_vectorised_helpers_match_scalar_oracle():
    L = oracle.lib()
    rng = np.random.default_rng(3)
    bits = np.concatenate([rng.integers(0, 2**32, 20000, dtype=np.uint64).astype(np.uint32),
                           np.array([0, 0x80000000, 0x7F800000, 0xFF800000, 0x7FC00000, 0x7F800001, 0x00000001,
                                     0x807FFFFF, 0x7F7FFFFF, 0x3F808000, 0x3F818000, 0x477FF000, 0x477FEFFF,
                                     0x33000000, 0x33000001, 0x387FFFFF], np.uint32)])
    f = bits.view(np.float32)
    f = np.ascontiguousarray(f[: (f.size // 16) * 16])
    for rne in (False, True):
        vec = oracle.f32_to_bf16(f, rne)
        # array entry point (pointer-based: signalling NaNs reach C unchanged);
        # a multiple of 16 elements so the avx512bf impl rounds all of them
        sc = np.empty(f.size, np.uint16)
        L.orc_convert_fp32_to_bf16_arrays(f.ctypes.data, sc.ctypes.data, f.size,
                                          oracle.BF16_AVX512BF if rne else oracle.BF16_SCALAR)
        assert np.array_equal(vec, sc)
    h = oracle.f32_to_fp16(f)
    sc = np.array([L.orc_fp32_to_fp16_rne(float(x)) for x in f], np.uint16)
    nan = np.isnan(f)
    assert np.array_equal(h[~nan], sc[~nan])
    assert np.all((sc[nan] & 0x7C00) == 0x7C00) and np.all((sc[nan] & 0x3FF) != 0)
    allh = np.arange(65536, dtype=np.uint32).astype(np.uint16)
    w = oracle.fp16_to_f32(allh)
    sc = np.array([L.orc_fp16_to_fp32(int(x)) for x in allh], np.float32)
    ok = np.isnan(w) & np.isnan(sc) | (w.view(np.uint32) == sc.view(np.uint32))
    assert ok.all()


def _roles(res, a, b):
    return ["in" if r == x else ("inout" if r == y else "?") for r, x, y in zip(res, a, b)]


def test_survey_probes():
    d = json.loads((ROOT / "tests" / "golden" / "survey_probes.json").read_text())
    for c in d["cases"]:
        dt = c["dtype"]
        if "expect" in c and dt == 11:
            for name, exp in c["expect"].items():
                a = np.array(c["in"], np.uint16)
                b = np.array(c["inout"], np.uint16)
                oracle.comp_reduce(a, b, dt, c["op"], IMPLS[name])
                assert b.tolist() == exp, (c["what"], name)
        elif "expect" in c:
            a = np.array(c["in"], np.int8)
            b = np.array(c["inout"], np.int8)
            oracle.comp_reduce(a, b, dt, c["op"])
            assert b.tolist() == c["expect"]
        elif dt == 9:
            a = np.array([float(x) for x in c["in_f32"]], np.float32)
            b0 = np.array([float(x) for x in c["inout_f32"]], np.float32)
            for op, name in ((2, "min"), (3, "max")):
                b = b0.copy()
                oracle.comp_reduce(a, b, dt, op)
                assert _roles(b.view(np.uint32), a.view(np.uint32), b0.view(np.uint32)) == c["expect_role"][name]
        else:
            impls = IMPLS if dt == 11 else {"avx512f": oracle.FP16_AVX512F, "f16c": oracle.FP16_F16C}
            for name, roles in c["expect_role"].items():
                for op in (2, 3):
                    a = np.array(c["in"], np.uint16)
                    b0 = np.array(c["inout"], np.uint16)
                    b = b0.copy()
                    if dt == 11:
                        oracle.comp_reduce(a, b, dt, op, impls[name])
                    else:
                        oracle.comp_reduce(a, b, dt, op, oracle.BF16_AVX512BF, impls[name])
                    assert _roles(b, a, b0) == roles, (c["what"], name, op)


FUNCTIONAL = [c for c in kat.load() if c["suite"] == "tests/functional"]


@pytest.mark.parametrize("case", FUNCTIONAL, ids=[f"dt{c['dtype']}-{OP_NAME[c['op']]}-P{c['P']}-b{c['buf_idx']}"
                                                  for c in FUNCTIONAL])
def test_reference_functional_kats(case):
    """oneCCL tests/functional allreduce KATs through the oracle's chained
    2-input reduces, for every bf16/fp16 impl variant."""
    dt = case["dtype"]
    variants = [("avx512bf", oracle.BF16_AVX512BF, True), ("avx512f", oracle.BF16_AVX512F, False),
                ("scalar", oracle.BF16_SCALAR, False)] if dt == BF16 else [("ref", oracle.BF16_AVX512BF, True)]
    for name, bimpl, rne in variants:
        def reduce2(a, b):
            oracle.comp_reduce(a, b, dt, case["op"], bimpl, oracle.FP16_AVX512F)
        for count in case["counts"]:
            err, tol = kat.functional_case(case, count, reduce2, bf16_rne=rne)
            assert err <= tol, f"{name} count={count}: err {err} > tol {tol}"


def test_reference_example_kats():
    for c in kat.load():
        if c["suite"] == "examples/cpu/cpu_allreduce_bf16_test":
            for bimpl, rne in ((oracle.BF16_AVX512BF, True), (oracle.BF16_AVX512F, False)):
                assert kat.bf16_example_case(c, lambda a, b: oracle.comp_reduce(a, b, 11, 0, bimpl), rne)
        elif c["suite"] == "examples/benchmark":
            assert kat.benchmark_case(c, lambda a, b: oracle.comp_reduce(a, b, 9, 0))


@pytest.mark.parametrize("bimpl", [0, 1, 2])
@pytest.mark.parametrize("n", [5, 16, 33, 1000])
def test_batch_keep_precision_matches_numpy_restatement(bimpl, n):
    """comp.cpp:214-234 + bf16.cpp:113-169, restated independently in numpy."""
    k = 4
    ins = [rand_array(BF16, n, seed=50 + j) for j in range(k)]
    packed = np.concatenate(ins)
    out = ins[0].copy()
    oracle.batch_reduce(packed, [j * n for j in range(k)], n, out, BF16, 0, 1, bimpl)
    acc = oracle.bf16_to_f32(ins[0]).copy()
    for x in ins[1:]:
        acc = (acc + oracle.bf16_to_f32(x)).astype(np.float32)
    lim = (n // 16) * 16 if bimpl else 0
    exp = np.concatenate([oracle.f32_to_bf16(acc[:lim], bimpl == 2), oracle.f32_to_bf16(acc[lim:], False)])
    nan = np.isnan(acc)
    assert np.array_equal(out[~nan], exp[~nan])


def test_batch_storage_equals_chain():
    n = 777
    for dt in (FP32, BF16, FP16, 4):
        ins = [rand_array(dt, n, seed=80 + j) for j in range(5)]
        packed = np.concatenate(ins)
        out = ins[0].copy()
        oc = oracle.batch_reduce(packed, [j * n for j in range(5)], n, out, dt, 0, 0)
        exp = oracle.fanin(ins, dt, 0)
        assert out.tobytes() == exp.tobytes()
        assert (oc == n) == (dt in (BF16, FP16))  # out_count written only by bf16/fp16 (bf16.cpp:94-96)


@pytest.mark.parametrize("n", [1 << 20, (70 << 20) // 4 + 5, 64 * 8 + 1, 777])
def test_mt_equals_single_thread(n):
    a = rand_array(FP32, n, seed=1)
    b = rand_array(FP32, n, seed=2)
    e1 = b.copy()
    e2 = b.copy()
    oracle.comp_reduce(a, e1, FP32, 0)
    oracle.comp_reduce_mt(a, e2, FP32, 0, 8)
    assert e1.tobytes() == e2.tobytes()


def test_fp16_no_compiler_impl_is_a_noop():
    """fp16_intrisics.hpp:214-247: an impl type outside f16c/avx512f/avx512fp16
    computes nothing (reproduced, documented trap)."""
    a = rand_array(FP16, 64, seed=1)
    b = rand_array(FP16, 64, seed=2)
    b0 = b.copy()
    oracle.comp_reduce(a, b, FP16, 0, 0, oracle.FP16_NO_COMPILER)
    assert np.array_equal(b, b0)


def test_int_wrap_and_minmax():
    a = np.array([127, -128, 5, -7], np.int8)
    b = np.array([1, -1, -9, 3], np.int8)
    for op, exp in ((0, [-128, 127, -4, -4]), (1, [127, -128, -45, -21]), (2, [1, -128, -9, -7]),
                    (3, [127, -1, 5, 3])):
        x = b.copy()
        oracle.comp_reduce(a, x, 0, op)
        assert x.tolist() == exp, OP_NAME[op]


def test_oracle_is_sanitizer_clean():
    """The restatement under AddressSanitizer + UndefinedBehaviorSanitizer
    (oracle/selftest.c over every entry point, odd sizes, all impls)."""
    r = subprocess.run(["make", "-C", str(ROOT / "oracle"), "asan"], capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip("no sanitizer runtime for this compiler: " + r.stderr[-200:])
    r = subprocess.run([str(ROOT / "oracle" / "lib" / "selftest_asan")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "selftest: ok" in r.stdout


def test_fp16_native_check_committed():
    """oracle/FP16_NATIVE_CHECK.json: on all 2^32 (in, inout) fp16 pairs the
    fp32 route equals IEEE binary16 arithmetic for sum and prod; min/max differ
    exactly on a signalling-NaN inout (65536 x 1022 pairs); the IEEE model
    equals the AVX512_FP16 instructions (VADDPH/VMULPH/VMINPH/VMAXPH, run on
    this container's CPU), and the oracle's avx512fp16 model equals both."""
    d = json.loads((ROOT / "oracle" / "FP16_NATIVE_CHECK.json").read_text())
    assert d["stride"] == 1
    assert d["native_model_vs_avx512fp16_hardware"] is True  # pinned to the instructions themselves
    for op in ("sum", "prod", "min", "max"):
        assert d[f"{op}_checked"] == 1 << 32
        assert d[f"{op}_route_vs_native_unexplained"] == 0
        assert d[f"{op}_oracle_vs_native"] == 0
        assert d[f"{op}_hardware_vs_native"] == 0
    assert d["sum_route_vs_native_snan_inout"] == d["prod_route_vs_native_snan_inout"] == 0
    assert d["min_route_vs_native_snan_inout"] == d["max_route_vs_native_snan_inout"] == 65536 * 1022


def test_fp16_native_check_sample():
    """The same program on a strided sample, rebuilt and run here."""
    import subprocess
    exe = ROOT / "oracle" / "lib" / "fp16_native_check"
    if not exe.exists():
        subprocess.run(["make", "-C", str(ROOT / "oracle"), str(Path("lib") / "fp16_native_check")], check=True)
    r = subprocess.run([str(exe), "65537", "4"], capture_output=True, text=True, timeout=300)
    if r.returncode == 2:
        pytest.skip("CPU lacks F16C")
    assert r.returncode == 0, r.stdout + r.stderr
    d = json.loads(r.stdout)
    assert all(d[f"{op}_oracle_vs_native"] == 0 for op in ("sum", "prod", "min", "max"))
