"""A failing copy injected into the real staged pipeline (mi_test_fail_copy)
surfaces with the operand's geometry in mi_last_error (VERDICT r5 item 2:
a staged-copy fault must be attributable), and the library keeps working
afterwards: the injected failure never reaches the runtime, so no sticky
error is left behind.  The operands are the round-5 faulting case's shape:
bf16 at odd element offsets of pageable buffers, past the bounce size."""
from __future__ import annotations

import numpy as np
import pytest

import oracle
from oneccl_amd import _lib, comp
from tests.test_copy_error_text import expected, parse_geometry
from tests.util import BF16, assert_same, rand_array

pytestmark = pytest.mark.gpu

N = 786437  # elements: 1.5 MiB of bf16, one staging chunk


def _operands(seed):
    raw_a = np.zeros(N + 64, np.uint16)
    raw_b = np.zeros(N + 64, np.uint16)
    a = raw_a[3:3 + N]  # 2-byte aligned: an odd element offset
    b = raw_b[5:5 + N]
    a[:] = rand_array(BF16, N, seed=seed, specials=False)
    b[:] = rand_array(BF16, N, seed=seed + 1, specials=False)
    return raw_a, raw_b, a, b


@pytest.mark.parametrize("nth,what", [(1, "H2D staging copy"), (2, "H2D staging copy"), (3, "D2H result copy")])
def test_injected_copy_failure_is_attributed(nth, what):
    m = _lib.mi()
    flags = comp.reference_flags(comp.datatype.bfloat16)
    _, _, a, b = _operands(11)
    try:
        m.mi_test_fail_copy(nth)
        rc = m.mi_reduce_sync(a.ctypes.data, b.ctypes.data, N, BF16, 0, flags, -1)
    finally:
        m.mi_test_fail_copy(0)
    assert rc != 0
    text = m.mi_last_error().decode()
    assert text.startswith(what), text
    kind, off, nbytes, end, span_off, span, chunk = parse_geometry(text)
    assert kind == "pageable" and chunk == 0 and nbytes == 2 * N
    # copies in order: inout (b, inputs[0]), then in (a); the D2H writes b
    addr = (b if nth != 2 else a).ctypes.data
    assert (off, nbytes, end, span_off, span) == expected(addr, 2 * N, hull=nth != 3)
    m.mi_thread_sync()
    # nothing sticky: the next reduce on the same thread is exact
    _, _, a2, b2 = _operands(21)
    exp = b2.copy()
    oracle.comp_reduce(a2.copy(), exp, BF16, 0)
    _lib.check(m.mi_reduce_sync(a2.ctypes.data, b2.ctypes.data, N, BF16, 0, flags, -1))
    assert_same(b2, exp, BF16)
