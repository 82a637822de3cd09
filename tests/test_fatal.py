"""The reference's error convention at the drop-in boundary: an unknown
datatype or reduction is CCL_FATAL (log + std::terminate,
src/common/log/log.hpp:333-337) — comp.cpp:56,113, bf16.cpp:73,
bf16_intrisics.hpp:131, fp16_intrisics.hpp:222-243 — while a custom reduction
without a callback is CCL_THROW (comp.cpp:85).  The shim reproduces both.

Each fatal case runs in a child process (it must abort); the checks happen
before any GPU work, so they run on CPU."""
from __future__ import annotations

import signal
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent

PRELUDE = f"""
import ctypes, sys
sys.path.insert(0, {str(ROOT)!r})
import numpy as np
from oneccl_amd import _lib
s = _lib.shim()
a = np.zeros(64, np.float32); b = np.zeros(64, np.float32)
pa, pb = a.ctypes.data, b.ctypes.data
"""

FATAL = {
    "unknown dtype": "s.mi_ccl_comp_reduce(pa, 16, pb, None, 99, 0)",
    "unknown op, fp32 (CCL_REDUCE)": "s.mi_ccl_comp_reduce(pa, 16, pb, None, 9, 7)",
    "custom op reaching bf16": "s.mi_ccl_bf16_reduce(pa, 16, pb, None, 4)",
    "unknown op, bf16": "s.mi_ccl_comp_reduce(pa, 16, pb, None, 11, 9)",
    "batch, unknown op": "s.mi_ccl_comp_batch_reduce(pa, (ctypes.c_size_t * 2)(0, 16), 2, 16, pb, None, 9, 5, 0)",
    "async start, unknown dtype": "s.mi_ccl_comp_reduce_start(pa, 16, pb, None, 77, 0, _lib.MI_CCL_REDUCTION_FN(), "
                                  "ctypes.byref(ctypes.c_void_p()))",
}


@pytest.mark.parametrize("what", sorted(FATAL))
def test_unknown_dtype_or_op_is_fatal(what):
    code = PRELUDE + FATAL[what] + "\nprint('returned', flush=True)\n"
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == -signal.SIGABRT, (r.returncode, r.stdout, r.stderr[-2000:])
    assert "FATAL" in r.stderr and "unexpected value" in r.stderr
    assert "returned" not in r.stdout


def test_custom_without_callback_throws_not_fatal():
    """CCL_THROW_IF_NOT(reduction_fn, ...) (comp.cpp:85): an exception the
    caller can catch; the C view reports it as -1 with the message."""
    code = PRELUDE + ("null_fn = ctypes.cast(None, _lib.MI_CCL_REDUCTION_FN)\n"
                      "rc = s.mi_ccl_comp_reduce_custom(pa, 16, pb, None, 9, null_fn)\n"
                      "print(rc, s.mi_ccl_last_error().decode())\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.startswith("-1") and "callback" in r.stdout


def test_batch_with_sizeless_dtype_throws():
    """ccl_comp_batch_reduce strides its inputs by dtype.size(), which
    CCL_THROWs for a non-positive size (datatype.hpp:46-48) before any reduce
    runs: an exception, not CCL_FATAL, in the reference and here."""
    code = PRELUDE + ("rc = s.mi_ccl_comp_batch_reduce(pa, (ctypes.c_size_t * 2)(0, 16), 2, 16, pb, None, 42, 0, 0)\n"
                      "print(rc, s.mi_ccl_last_error().decode())\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.startswith("-1") and "datatype size" in r.stdout
