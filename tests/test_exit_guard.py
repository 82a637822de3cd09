"""Process exit against library sections still running:
the exit handler of libmi_reduce waits for threads inside a guarded section
(a context teardown, a staging worker's job) before HIP's own teardown, but
no longer without limit: past MI_REDUCE_EXIT_WAIT_S it names the section and
ends the process with status 70.  A section that finishes in time is simply
waited for.  Child processes; the hook makes no device call beyond the HIP
runtime's initialisation, so this runs without a GPU."""
import os
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent

CHILD = r"""
import sys, time
sys.path.insert(0, {root!r})
from oneccl_amd import _lib
m = _lib.mi()
assert m.mi_test_hold_exit_guard({hold}) == 0
time.sleep(0.2)
print("exiting", flush=True)
"""


def _run(hold_ms, wait_s):
    env = dict(os.environ, MI_REDUCE_EXIT_WAIT_S=str(wait_s))
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, "-c", CHILD.format(root=str(ROOT), hold=hold_ms)], env=env,
                       capture_output=True, text=True, timeout=120)
    return r, time.monotonic() - t0


def test_blocked_section_ends_the_process_after_the_bound():
    r, dt = _run(-1, 1)
    assert r.returncode == 70, (r.returncode, r.stderr[-1000:])
    assert "exiting" in r.stdout  # stdout flushed before the forced end
    assert "still running after 1 s" in r.stderr and "mi_test_hold_exit_guard" in r.stderr
    assert dt < 60


def test_section_that_finishes_in_time_is_waited_for():
    r, dt = _run(1500, 30)
    assert r.returncode == 0, r.stderr[-1000:]
    assert dt >= 1.3  # the exit waited for the section (started ~0.2 s before exit)
