"""Loader for tests/golden/ref_comp_vectors.npz: vectors produced by the
reference's own compiled src/comp code (CCL_REDUCE for the ten non-LP types,
the scalar bf16 impl, ccl_comp_batch_reduce's storage-precision chain; see
tests/golden/make_ref_comp_vectors.py and oracle/ref_comp_harness.cpp)."""
from __future__ import annotations

import json
from functools import lru_cache
from pathlib import Path

import numpy as np

PATH = Path(__file__).resolve().parent / "golden" / "ref_comp_vectors.npz"


@lru_cache(maxsize=1)
def load():
    z = np.load(PATH)  # allow_pickle=False: arrays and a JSON string only
    arrs = {k: z[k] for k in z.files}
    return arrs, json.loads(str(arrs["meta"]))


def cases(kind: str):
    arrs, meta = load()
    out = []
    for c in meta["cases"]:
        if c["kind"] != kind:
            continue
        d = dict(c)
        d["expected"] = arrs[c["key"]]
        if kind == "reduce":
            d["a"], d["b"] = arrs[f"reduce_{c['dtype']}_in"], arrs[f"reduce_{c['dtype']}_inout"]
        elif kind == "reduce1":
            d["a"], d["b"] = arrs[f"reduce1_{c['dtype']}_in"], arrs[f"reduce1_{c['dtype']}_inout"]
        elif kind == "bf16s":
            d["a"], d["b"] = arrs["bf16s_in"], arrs["bf16s_inout"]
        elif kind == "keep":
            d["buf"], d["b"] = arrs[f"kp_{c['impl']}_buf"], arrs[f"kp_{c['impl']}_inout"]
        else:
            d["buf"], d["b"] = arrs[f"batch_{c['dtype']}_buf"], arrs[f"batch_{c['dtype']}_inout"]
        out.append(d)
    return out
