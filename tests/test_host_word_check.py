"""The host word, checked.  Callers that say their operands
are host memory -- a schedule without a stream (comp.cpp:136-142), the MPI
user ops (integration/0002), the copy entries (integration/0006) -- have them
folded or copied on the CPU with no lookup, as the reference does.  Under
CCL_COMP_CHECK_HOST=1 (or CCL_LOG_LEVEL=debug) the drop-in classifies them
anyway and fails loudly on device memory instead of dereferencing it on the
host.  The knob is read once per process, so each case runs in a child."""
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent

HOST_CASE = r"""
import ctypes, numpy as np
from oneccl_amd import _lib
s = _lib.shim()
a = np.ones(1024, np.float32); b = np.ones(1024, np.float32)
s.mi_ccl_comp_shim_sched(1)
n0 = s.mi_ccl_comp_pointer_lookups()
assert s.mi_ccl_comp_reduce(a.ctypes.data, 1024, b.ctypes.data, None, 9, 0) == 0
checked = s.mi_ccl_comp_pointer_lookups() - n0
assert (b == 2).all()
h = np.ones(1024, np.uint16) * 0x3f80
n0 = s.mi_ccl_comp_pointer_lookups()
assert s.mi_ccl_bf16_reduce_host(h.ctypes.data, 512, h[512:].ctypes.data, None, 0) == 0
checked_mpi = s.mi_ccl_comp_pointer_lookups() - n0
n0 = s.mi_ccl_comp_pointer_lookups()
assert s.mi_ccl_comp_copy_host(a.ctypes.data, b.ctypes.data, 4096, 0) == 0
checked_copy = s.mi_ccl_comp_pointer_lookups() - n0
print(checked, checked_mpi, checked_copy)
"""

DEVICE_CASE = r"""
import torch
from oneccl_amd import _lib
s = _lib.shim()
a = torch.ones(1024, device="cuda"); b = torch.ones(1024, device="cuda")
s.mi_ccl_comp_shim_sched(1)
rc = s.mi_ccl_comp_reduce(a.data_ptr(), 1024, b.data_ptr(), None, 9, 0)
print(rc, s.mi_ccl_last_error().decode())
h = torch.zeros(1024, dtype=torch.bfloat16, device="cuda")
rc = s.mi_ccl_bf16_reduce_host(h.data_ptr(), 512, h.data_ptr() + 1024, None, 0)
print(rc, s.mi_ccl_last_error().decode())
rc = s.mi_ccl_comp_copy_host(a.data_ptr(), b.data_ptr(), 4096, 0)
print(rc, s.mi_ccl_last_error().decode())
torch.cuda.synchronize()
"""


def _child(code, **env):
    e = dict(os.environ)
    e.pop("CCL_LOG_LEVEL", None)
    e.pop("CCL_COMP_CHECK_HOST", None)
    e.update(env)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, cwd=ROOT, env=e)
    assert r.returncode == 0, r.stderr[-3000:]
    return r.stdout.strip().splitlines()


def test_unchecked_host_word_makes_no_lookup():
    assert _child(HOST_CASE)[-1] == "0 0 0"


@pytest.mark.parametrize("env", [{"CCL_COMP_CHECK_HOST": "1"}, {"CCL_LOG_LEVEL": "debug"}])
def test_checked_host_word_classifies_and_passes_host_memory(env):
    # reduce: inout counted once (it is both out and the first input) + in;
    # the MPI op the same; the copy both pointers
    assert _child(HOST_CASE, **env)[-1] == "2 2 2"


def test_check_can_be_forced_off_under_debug():
    assert _child(HOST_CASE, CCL_LOG_LEVEL="debug", CCL_COMP_CHECK_HOST="0")[-1] == "0 0 0"


@pytest.mark.gpu
def test_checked_host_word_refuses_device_memory():
    lines = _child(DEVICE_CASE, CCL_COMP_CHECK_HOST="1")
    assert len(lines) >= 3, lines
    for line in lines[-3:]:
        rc, msg = line.split(" ", 1)
        assert rc == "-1" and "device memory passed where the caller says host memory" in msg, line
