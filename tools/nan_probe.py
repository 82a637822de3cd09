#!/usr/bin/env python3
"""Which NaN payloads do the GPU kernels produce, against the reference's own
AVX-512 code?  Runs every case of tests/golden/ref_vectors.npz through the C
ABI (2-input mi_reduce and the fused 8-input mi_reduce_multi) and reports, per
case, the elements whose bits differ — the parity tests compare NaNs
payload-agnostic; this counts exact-bit differences and shows the operand
pairs behind them.  One JSON line per case, then a summary line.

  python tools/nan_probe.py
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    import numpy as np
    import torch

    from oneccl_amd import _lib
    from tests import refvec
    from tests.test_gpu_ref_vectors import _flags
    from tests.util import from_dev, to_dev
    m = _lib.mi()
    st = torch.cuda.current_stream().cuda_stream
    total = 0
    for c in refvec.reduce_cases():
        ta, pa = to_dev(c["a"])
        tb, pb = to_dev(c["b"])
        _lib.check(m.mi_reduce(pa, pb, c["count"], c["dtype"], c["op"], _flags(c["dtype"], c["impl"]), st))
        torch.cuda.synchronize()
        got = from_dev(tb, c["b"]).view(np.uint16)
        exp = c["expected"].view(np.uint16)
        d = np.flatnonzero(got != exp)
        total += d.size
        a16, b16 = c["a"].view(np.uint16), c["b"].view(np.uint16)
        print(json.dumps({"key": c["key"], "differ": int(d.size),
                          "samples": [[hex(int(a16[i])), hex(int(b16[i])), hex(int(got[i])), hex(int(exp[i]))]
                                      for i in d[:6]]}), flush=True)
    for c in refvec.fan_cases():
        holders = [to_dev(x) for x in c["inputs"]]
        to, po = to_dev(np.zeros_like(c["inputs"][0]))
        arr = _lib.void_ptr_array([p for _, p in holders])
        _lib.check(m.mi_reduce_multi(arr, len(holders), po, c["count"], c["dtype"], c["op"],
                                     _flags(c["dtype"], c["impl"]), st))
        torch.cuda.synchronize()
        got = from_dev(to, c["expected"]).view(np.uint16)
        exp = c["expected"].view(np.uint16)
        d = np.flatnonzero(got != exp)
        total += d.size
        ins = [x.view(np.uint16) for x in c["inputs"]]
        print(json.dumps({"key": c["key"], "differ": int(d.size),
                          "samples": [[[hex(int(x[i])) for x in ins], hex(int(got[i])), hex(int(exp[i]))]
                                      for i in d[:4]]}), flush=True)
    print(json.dumps({"total_differing_elements": int(total)}), flush=True)


if __name__ == "__main__":
    main()
