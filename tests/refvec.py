"""Golden vectors produced by the reference's own bf16/fp16 reduce code
(tests/golden/ref_vectors.npz, made by tests/golden/make_ref_vectors.py through
oracle/_ref/libref_comp.so).  Loaded with numpy's default allow_pickle=False:
the file holds numeric arrays and one JSON string only."""
from __future__ import annotations

import json
from pathlib import Path

import numpy as np

PATH = Path(__file__).resolve().parent / "golden" / "ref_vectors.npz"
# the avx512fp16 impl's vectors (tests/golden/make_ref_vectors_fp16native.py):
# the reference's native half-precision code, run on a CPU with AVX512_FP16
PATH_FP16NATIVE = Path(__file__).resolve().parent / "golden" / "ref_vectors_fp16native.npz"
BF16, FP16 = 11, 8

_cache = None


def load():
    """(arrays, cases): arrays by key, and the case list from the metadata,
    over both fixtures (their shared inputs are the same arrays)."""
    global _cache
    if _cache is None:
        arrs, cases = {}, []
        for path in (PATH, PATH_FP16NATIVE):
            z = np.load(path)
            part = {k: z[k] for k in z.files}
            meta = json.loads(str(part.pop("meta")))
            for k, v in part.items():
                assert k not in arrs or np.array_equal(arrs[k], v), k
                arrs[k] = v
            cases += meta["cases"]
        _cache = (arrs, {"cases": cases})
    return _cache


def reduce_cases():
    """2-input cases: dicts with dtype, impl, op, count, in, inout, expected."""
    arrs, meta = load()
    out = []
    for c in meta["cases"]:
        if c["kind"] not in ("bf16", "fp16"):
            continue
        out.append(dict(c, dtype=BF16 if c["kind"] == "bf16" else FP16, a=arrs[c["kind"] + "_in"],
                        b=arrs[c["kind"] + "_inout"], expected=arrs[c["key"]]))
    return out


def fan_cases():
    """Chained 8-input fan-ins: dicts with dtype, impl, op, inputs (k, n), expected."""
    arrs, meta = load()
    out = []
    for c in meta["cases"]:
        if not c["kind"].startswith("fan_"):
            continue
        out.append(dict(c, dtype=BF16 if "bf16" in c["kind"] else FP16, inputs=arrs[c["kind"]],
                        expected=arrs[c["key"]]))
    return out


def conversion_cases():
    """fp32 -> bf16 16-element stores: (impl, fp32 input, bf16 expected)."""
    arrs, meta = load()
    return [(c["impl"], arrs["cvt_f32"], arrs[c["key"]]) for c in meta["cases"] if c["kind"] == "cvt"]


def load_case():
    arrs, _ = load()
    return arrs["load_bf16"], arrs["load_f32"]
