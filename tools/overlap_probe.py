#!/usr/bin/env python3
"""Does the reduce's LDS reservation hurt a GEMM running beside it?

The one-wave kernels cap their resident waves per CU by reserving LDS that no
instruction touches.  A GEMM launched on another stream needs
LDS, so while the reduce's blocks sit on a CU the GEMM's cannot.  This probe
times, in one process per mode (the mode is read once per process):
  * a bf16 GEMM alone (torch.matmul -> hipBLASLt), and R in-place 1 GiB fp32
    reduces alone (mi_reduce), each under HIP events on its own stream;
  * both at once on their two streams: the makespan from a common start, and
    each side's own span.
Modes: the default cap, and MI_REDUCE_WAVE_CAP=0 (no reservation).

  python tools/overlap_probe.py            (parent: runs both modes as children)
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def child(mode: str) -> None:
    sys.path.insert(0, str(ROOT))
    import torch

    from oneccl_amd import _lib
    m = _lib.mi()
    n = (1 << 30) // 4
    a = torch.empty(n, device="cuda").uniform_(-1, 1)
    b = torch.empty(n, device="cuda").uniform_(-1, 1)
    x = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    y = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    reps_gemm, reps_red = 6, 8

    def gemm(st):
        with torch.cuda.stream(st):
            for _ in range(reps_gemm):
                torch.matmul(x, y)

    def red(st):
        for _ in range(reps_red):
            _lib.check(m.mi_reduce(b.data_ptr(), a.data_ptr(), n, 9, 0, 0, st.cuda_stream))

    def span(fn, st):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        fn(st)
        e1.record(st)
        return e0, e1

    res = {"mode": mode}
    for _ in range(2):  # warm both
        gemm(s1)
        red(s2)
    torch.cuda.synchronize()
    alone_g, alone_r, both_g, both_r, make = [], [], [], [], []
    for _ in range(5):
        e0, e1 = span(gemm, s1)
        torch.cuda.synchronize()
        alone_g.append(e0.elapsed_time(e1))
        e0, e1 = span(red, s2)
        torch.cuda.synchronize()
        alone_r.append(e0.elapsed_time(e1))
        start = torch.cuda.Event(enable_timing=True)
        start.record(torch.cuda.current_stream())
        s1.wait_event(start)
        s2.wait_event(start)
        g0, g1 = span(gemm, s1)
        r0, r1 = span(red, s2)
        torch.cuda.synchronize()
        both_g.append(g0.elapsed_time(g1))
        both_r.append(r0.elapsed_time(r1))
        make.append(max(start.elapsed_time(g1), start.elapsed_time(r1)))
    med = lambda v: round(sorted(v)[len(v) // 2], 3)  # noqa: E731
    w, lds = __import__("ctypes").c_int(), __import__("ctypes").c_uint()
    m.mi_get_residency(-1, 2, __import__("ctypes").byref(w), __import__("ctypes").byref(lds))
    res.update({"lds_bytes_per_reduce_workgroup": lds.value, "gemm": f"{reps_gemm} x bf16 8192^3 (torch.matmul)",
                "reduce": f"{reps_red} x fp32 sum 1 GiB in place (mi_reduce)",
                "gemm_alone_ms": med(alone_g), "reduce_alone_ms": med(alone_r), "sum_alone_ms":
                round(med(alone_g) + med(alone_r), 3), "gemm_overlapped_ms": med(both_g),
                "reduce_overlapped_ms": med(both_r), "makespan_ms": med(make)})
    print(json.dumps(res), flush=True)


def main() -> None:
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2])
        return
    for mode, env in (("wave cap (default)", {}), ("MI_REDUCE_WAVE_CAP=0", {"MI_REDUCE_WAVE_CAP": "0"})):
        r = subprocess.run([sys.executable, __file__, "--child", mode], env=dict(os.environ, **env),
                           capture_output=True, text=True, timeout=600)
        sys.stdout.write(r.stdout)
        if r.returncode:
            sys.stderr.write(r.stderr)
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
