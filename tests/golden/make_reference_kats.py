#!/usr/bin/env python3
"""Generate tests/golden/reference_kats.json: the known-answer tests that
oneCCL's own test suites hold for the reduction path, evaluated for a
parameter grid.  No reference code is run or copied: each formula is
restated from the cited file:line, and the fixture records inputs-by-formula,
expected values and tolerances.

Sources (reference snapshot 2024-12-20):
  tests/functional/test_impl.hpp:242-252   int fill:  send[r][b] = r + b (+1 for prod)
  tests/functional/test_impl.hpp:288-299   fp  fill:  c1*r + c2*b (+1 for prod)
  tests/functional/test.hpp:72-86          (c1, c2) = (0.5, 1) bf16, (0.01, 0.01) fp16, (1, 1) otherwise
  tests/functional/test_impl.hpp:268-320   closed-form expected values (computed in T / float)
  tests/functional/test_impl.hpp:160-204   tolerance g = log2(P)*eps / (1 - log2(P)*eps), max_error = g*expected
  tests/functional/lp.hpp:32-35            eps: 2^-10 fp16 (x2), 2^-23 fp32, 2^-52 fp64, 2^-7 bf16 (x2)
  tests/functional/conf.cpp:51-53,59       sizes 17 / 32771 / 262144 (SIZE_SMALL/MEDIUM/LARGE), buffer counts 1 and 4
  examples/cpu/cpu_allreduce_bf16_test.cpp:29-50,80-97   bf16 allreduce of rank+idx, eps 2^-7 (x1)
  examples/benchmark/src/allreduce/cpu_allreduce_coll.hpp:29-57 + include/coll.hpp:152-170  fill = rank,
                                           expected (P-1)*P/2
"""
from __future__ import annotations

import json
import math
from pathlib import Path

import numpy as np

OUT = Path(__file__).resolve().parent / "reference_kats.json"

FP16_PRECISION = 9.77e-4
FP32_PRECISION = 1.19e-7
FP64_PRECISION = 2.22e-16
BF16_PRECISION = 7.81e-3

INT_NP = {0: np.int8, 1: np.uint8, 2: np.int16, 3: np.uint16, 4: np.int32, 5: np.uint32, 6: np.int64,
          7: np.uint64}
COEFF = {11: (0.5, 1.0), 8: (0.01, 0.01)}


def precision(dt):
    return {8: 2 * FP16_PRECISION, 9: FP32_PRECISION, 10: FP64_PRECISION, 11: 2 * BF16_PRECISION}.get(dt, 0.0)


def max_error(dt, P, expected):
    p = precision(dt)
    if not p:
        return 0.0
    if P == 1:
        return p
    lb = math.log(P) / math.log(2)
    g = (lb * p) / (1 - lb * p)
    return g * expected


def int_expected(dt, op, P, b):
    t = INT_NP[dt]
    with np.errstate(over="ignore"):
        if op == 0:
            return t((P * (P - 1)) // 2 + P * b)  # computed in T in the reference
        if op == 1:
            e = t(1)
            for r in range(P):
                e = t(e * t(r + b + 1))
            return e
        if op == 2:
            return t(b)
        return t(P - 1 + b)


def fp_expected(dt, op, P, b):
    c1, c2 = COEFF.get(dt, (1.0, 1.0))
    f = np.float32
    if op == 0:
        return float(f(P) * (f(c1) * f(P - 1) / f(2) + f(c2) * f(b)))
    if op == 1:
        e = f(1)
        for r in range(P):
            e = f(e * (f(c1) * f(r) + f(c2) * f(b) + f(1)))
        return float(e)
    if op == 2:
        return float(f(c2) * f(b))
    return float(f(c1) * f(P - 1) + f(c2) * f(b))


def main():
    cases = []
    for dt in list(range(12)):
        for op in range(4):
            for P in (2, 4, 8):
                for b in (0, 3):
                    if dt in INT_NP:
                        exp = int(int_expected(dt, op, P, b))
                        fill = "r + b + (op == prod)"
                        tol = 0.0
                    else:
                        exp = fp_expected(dt, op, P, b)
                        c1, c2 = COEFF.get(dt, (1.0, 1.0))
                        fill = f"{c1}*r + {c2}*b + (op == prod)"
                        tol = abs(max_error(dt, P, exp))
                    cases.append({"suite": "tests/functional", "dtype": dt, "op": op, "P": P, "buf_idx": b,
                                  "counts": [17, 32771, 262144], "fill": fill, "coeff": list(COEFF.get(dt, (1.0, 1.0))),
                                  "expected": exp, "max_error": tol})
    # examples/cpu/cpu_allreduce_bf16_test.cpp: value rank+idx, bf16 sum, eps 2^-7
    for P in (2, 4, 8):
        idx = np.arange(4096)
        exp = (P * (P - 1) / 2) + idx.astype(np.float32) * P
        lb = math.log(P) / math.log(2)
        g = (lb * BF16_PRECISION) / (1 - lb * BF16_PRECISION)
        cases.append({"suite": "examples/cpu/cpu_allreduce_bf16_test", "dtype": 11, "op": 0, "P": P,
                      "count": 4096, "fill": "rank + idx", "g": g})
    # examples/benchmark allreduce check: fill = rank, expected (P-1)*P/2 (C1 at P=2, 1 MiB fp32)
    for P in (2, 4):
        cases.append({"suite": "examples/benchmark", "dtype": 9, "op": 0, "P": P, "count": 262144,
                      "fill": "rank", "expected": (P - 1) * (P / 2)})
    OUT.write_text(json.dumps({"generator": "tests/golden/make_reference_kats.py", "cases": cases}, indent=0))
    print(f"wrote {len(cases)} cases to {OUT}")


if __name__ == "__main__":
    main()
