"""The adaptive dispatcher's bookkeeping, driven with synthetic durations
(CPU; no reduce runs).  These are the functions coop_fold (synchronous) and
settle_split (asynchronous) call after every host bucket above the threshold
(oneccl_amd/csrc/comp.cpp: take_gpu_alone, split_update, split_verdict,
gpu_alone_timed):

* a thread's first split of a kind only warms up; its second schedules one
  GPU-alone bucket (the probe on the 3rd call);
* a split whose whole rate falls below 0.95 of the GPU-alone rate sends the
  next 8 buckets of that kind to the GPU alone;
* every 32nd split re-times the GPU alone;
* the share stays within [0.1, 0.9] whatever the measured rates.

Each case runs in a child process: the state is per thread and the
thresholds are read from the environment at load."""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = str(Path(__file__).resolve().parent.parent)

_PRELUDE = r'''
import ctypes, sys
sys.path.insert(0, sys.argv[1])
from oneccl_amd import _lib
s = _lib.shim()
def state(pk):
    left = ctypes.c_uint(0)
    rate = s.mi_ccl_comp_split_gpu_rate(pk, ctypes.byref(left))
    return s.mi_ccl_comp_split_share(pk), rate, left.value
def feed(pk, count, head, th, tt):
    assert s.mi_ccl_comp_split_feed(pk, count, head, th, tt) == 0, s.mi_ccl_last_error()
N = 1 << 24
'''


def run(body: str, env_extra: dict | None = None) -> str:
    env = dict(os.environ)
    for k in list(env):
        if k.startswith("CCL_COMP_"):
            del env[k]
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, "-c", _PRELUDE + body, ROOT], capture_output=True, text=True, timeout=120,
                       env=env)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    return r.stdout


@pytest.mark.parametrize("pk", [0, 1])
def test_warmup_probe_and_lost_split_stretch(pk):
    out = run(f'''
pk = {pk}
head = int(N * 0.45) // 256 * 256
# call 1: split, warm-up only (share unchanged, nothing scheduled)
assert s.mi_ccl_comp_split_take_gpu_alone(pk) == 0
feed(pk, N, head, 1.0, 1.0)
sh, rate, left = state(pk)
assert abs(sh - 0.45) < 1e-12 and left == 0, (sh, left)
# call 2: split; the share moves halfway to the balance point, and the 3rd call is a GPU-alone probe
assert s.mi_ccl_comp_split_take_gpu_alone(pk) == 0
feed(pk, N, head, 0.010, 0.010)   # CPU part head/0.01, GPU part (N-head)/0.01
sh, rate, left = state(pk)
bal = head / (head + (N - head))
assert abs(sh - (0.5 * 0.45 + 0.5 * bal)) < 1e-9, sh
assert left == 1, left
# call 3: the GPU alone, timed: N elements in 0.02 s
assert s.mi_ccl_comp_split_take_gpu_alone(pk) == 1
feed(pk, N, 0, 0.0, 0.020)
sh, rate, left = state(pk)
assert abs(rate - N / 0.020) < 1e-3 * rate and left == 0, (rate, left)
# a split at 0.96 of the GPU alone keeps splitting
assert s.mi_ccl_comp_split_take_gpu_alone(pk) == 0
feed(pk, N, head, 0.020 / 0.96, 0.020 / 0.96)
assert state(pk)[2] == 0
# a split below 0.95 of the GPU alone: the next 8 buckets go to the GPU alone, the 9th splits again
assert s.mi_ccl_comp_split_take_gpu_alone(pk) == 0
feed(pk, N, head, 0.020 / 0.90, 0.020 / 0.90)
assert state(pk)[2] == 8, state(pk)
for i in range(8):
    assert s.mi_ccl_comp_split_take_gpu_alone(pk) == 1, i
    feed(pk, N, 0, 0.0, 0.020)
assert s.mi_ccl_comp_split_take_gpu_alone(pk) == 0
print("ok")
''')
    assert "ok" in out


def test_every_32nd_split_probes_the_gpu_alone():
    out = run('''
pk = 0
head = int(N * 0.45) // 256 * 256
feed(pk, N, head, 1.0, 1.0)          # warm-up
feed(pk, N, head, 0.01, 0.01)        # 2nd: probe scheduled
assert s.mi_ccl_comp_split_take_gpu_alone(pk) == 1
feed(pk, N, 0, 0.0, 0.02)            # GPU alone: N / 0.02
probes = []
for i in range(1, 100):
    assert s.mi_ccl_comp_split_take_gpu_alone(pk) == 0, i
    feed(pk, N, head, 0.01, 0.01)    # splits at 2x the GPU-alone rate: never judged lost
    if state(pk)[2]:
        probes.append(i)
        assert s.mi_ccl_comp_split_take_gpu_alone(pk) == 1
        feed(pk, N, 0, 0.0, 0.02)
assert probes == [32, 64, 96], probes
print("ok")
''')
    assert "ok" in out


def test_share_stays_within_bounds():
    out = run('''
import random
random.seed(5)
for pk in (0, 1):
    head = int(N * 0.45) // 256 * 256
    feed(pk, N, head, 1.0, 1.0)
    lo = hi = None
    for i in range(400):
        # 20 splits with a CPU 1e6x slower, 20 with it 1e6x faster, then anything between
        if i < 20:
            th, tt = 1e3, 1e-3
        elif i < 40:
            th, tt = 1e-6, 1e0
        else:
            th, tt = 10 ** random.uniform(-6, 6), 10 ** random.uniform(-6, 6)
        sh = state(pk)[0]
        h = max(256, int(N * sh) // 256 * 256)
        if s.mi_ccl_comp_split_take_gpu_alone(pk):
            feed(pk, N, 0, 0.0, tt)
        else:
            feed(pk, N, h, th, tt)
        sh = state(pk)[0]
        assert 0.1 - 1e-12 <= sh <= 0.9 + 1e-12, (i, sh)
        lo = sh if lo is None else min(lo, sh)
        hi = sh if hi is None else max(hi, sh)
    assert lo < 0.12 and hi > 0.88, (lo, hi)   # both bounds were actually reached
print("ok")
''')
    assert "ok" in out


def test_invalid_times_change_nothing():
    out = run('''
head = int(N * 0.45) // 256 * 256
feed(0, N, head, 1.0, 1.0)
before = state(0)
for th, tt in ((0.0, 1.0), (1.0, 0.0), (-1.0, 1.0)):
    feed(0, N, head, th, tt)
feed(0, N, N, 1.0, 1.0)        # head = whole bucket: not a split
assert state(0) == before, (state(0), before)
print("ok")
''')
    assert "ok" in out


def test_pinned_zero_means_gpu_alone_for_pinned_buckets():
    """CCL_COMP_HOST_MAX_PINNED_BYTES=0: pinned buckets are never split with
    the CPU (share 0), pageable ones still are."""
    out = run('''
pg, pn, sh, shp = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_double(), ctypes.c_double()
assert s.mi_ccl_comp_host_max(ctypes.byref(pg), ctypes.byref(pn), ctypes.byref(sh), ctypes.byref(shp)) == 0
print(pg.value, pn.value, sh.value, shp.value)
''', {"CCL_COMP_HOST_MAX_PINNED_BYTES": "0"})
    pg, pn, sh, shp = out.split()
    if int(pg) == 0:
        pytest.skip("host path unsupported on this CPU (no AVX2/F16C)")
    assert int(pn) == 0 and float(shp) == 0.0
    assert int(pg) == 16 << 20 and abs(float(sh) - 0.45) < 1e-12


def test_pageable_zero_means_gpu_alone_everywhere():
    out = run('''
pg, pn, sh, shp = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_double(), ctypes.c_double()
assert s.mi_ccl_comp_host_max(ctypes.byref(pg), ctypes.byref(pn), ctypes.byref(sh), ctypes.byref(shp)) == 0
print(pg.value, pn.value, sh.value, shp.value)
''', {"CCL_COMP_HOST_MAX_BYTES": "0"})
    pg, pn, sh, shp = out.split()
    assert int(pg) == 0 and int(pn) == 0 and float(sh) == 0.0 and float(shp) == 0.0
