"""a failed staged copy names the host operand's geometry.

CPU half (no device needed): mi_test_copy_error formats the text the staged
path's copy sites produce (mi_reduce.hip copy_fail / copy_geometry) and the
fields are checked against the same geometry computed here.  The GPU half
(tests/test_gpu_copy_fault_injection.py) injects a failing copy into the real
staged pipeline with mi_test_fail_copy."""
from __future__ import annotations

import ctypes
import re

import numpy as np
import pytest

from oneccl_amd import _lib

GEOM = re.compile(r"\[(\w+) host operand: addr & 4095 = (\d+), (\d+) bytes, ends at page offset (\d+); "
                  r"runtime span: addr & 4095 = (\d+), (\d+) bytes; chunk (\d+)\]")


def parse_geometry(text):
    m = GEOM.search(text)
    assert m, text
    kind, off, nbytes, end, span_off, span, chunk = m.groups()
    return kind, int(off), int(nbytes), int(end), int(span_off), int(span), int(chunk)


def expected(addr, nbytes, hull):
    if hull:
        lo, hi = addr & ~15, (addr + nbytes + 15) & ~15
    else:
        lo = min((addr + 15) & ~15, addr + nbytes)
        hi = max(lo, (addr + nbytes) & ~15)
    return addr & 4095, nbytes, (addr + nbytes) & 4095, lo & 4095, hi - lo


@pytest.mark.parametrize("mis", [0, 2, 6, 13])
@pytest.mark.parametrize("nbytes", [3, 4096 - 2, (3 << 20) + 10])
@pytest.mark.parametrize("kind,name", [(1, "pinned"), (2, "pageable")])
@pytest.mark.parametrize("hull", [1, 0])
def test_copy_error_names_operand_geometry(mis, nbytes, kind, name, hull):
    m = _lib.mi()
    buf = np.zeros(nbytes + 64, np.uint8)
    addr = buf.ctypes.data + (-buf.ctypes.data) % 16 + mis
    rc = m.mi_test_copy_error(addr, nbytes, 5, kind, hull)
    assert rc != 0
    text = m.mi_last_error().decode()
    assert text.startswith("H2D staging copy (test): ")
    got = parse_geometry(text)
    assert got[0] == name and got[6] == 5
    assert got[1:6] == expected(addr, nbytes, hull)


def test_copy_error_rejects_unknown_kind():
    m = _lib.mi()
    assert m.mi_test_copy_error(ctypes.c_void_p(4096), 16, 0, 7, 1) != 0
    assert "pointer kind" in m.mi_last_error().decode()
