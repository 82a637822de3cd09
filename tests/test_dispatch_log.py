"""The dispatcher's decision in oneCCL's log.  The
reference logs its path at debug level (src/comp/bf16/bf16.cpp:92,
fp16/fp16.cpp:46, comp.cpp:149-156, LOG_DEBUG under CCL_LOG_LEVEL).  In-tree
the drop-in uses LOG_DEBUG itself (tests/test_intree_build.py compiles it with
-Werror); standalone it prints the same "|CCL_DEBUG| ..." line to stderr
under CCL_LOG_LEVEL=debug.  Checked in child processes (the environment is
read once), on CPU-path buckets."""
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent

CHILD = r"""
import ctypes, sys, numpy as np
sys.path.insert(0, {root!r})
from oneccl_amd import _lib
s = _lib.shim()
s.mi_ccl_comp_shim_sched({mode})
a = np.ones(1024, np.float32); b = np.ones(1024, np.float32)
_lib.check_shim(s.mi_ccl_comp_reduce(a.ctypes.data, 1024, b.ctypes.data, None, 9, 0), "reduce")
req = ctypes.c_void_p()
_lib.check_shim(s.mi_ccl_comp_reduce_start(a.ctypes.data, 1024, b.ctypes.data, None, 9, 0,
                                           _lib.MI_CCL_REDUCTION_FN(), ctypes.byref(req)), "start")
_lib.check_shim(s.mi_ccl_comp_request_free(req), "free")
assert b[0] == 3.0
print("ok")
"""


def _run(level, mode=0):
    env = dict(os.environ)
    env.pop("CCL_LOG_LEVEL", None)
    if level:
        env["CCL_LOG_LEVEL"] = level
    r = subprocess.run([sys.executable, "-c", CHILD.format(root=str(ROOT), mode=mode)], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip().endswith("ok")
    return [ln for ln in r.stderr.splitlines() if ln.startswith("|CCL_DEBUG|")]


def test_debug_level_logs_each_route():
    lines = _run("debug")
    assert len(lines) == 2, lines
    sync, start = lines
    assert "comp.cpp:" in sync and "reduce: count 1024, dtype 9, bytes 4096, inputs 2" in sync
    assert "operands: host memory, some pageable" in sync and "path: cpu (calling thread)" in sync
    assert "reduce_start: count 1024" in start and "completes in start" in start


def test_host_schedule_is_named_in_the_log():
    lines = _run("trace", mode=1)
    assert len(lines) == 2 and all("host memory by the schedule (no stream; not looked up)" in ln for ln in lines)


def test_quiet_by_default_and_at_info():
    assert _run(None) == []
    assert _run("info") == []
