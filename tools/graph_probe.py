#!/usr/bin/env python3
"""Launch cost of a chain of small reduces: eager calls vs one captured HIP
graph replay vs one mi_reduce_batch dispatch.  A oneCCL ring schedule issues one reduce per chunk per step;
below ~1 MiB each call is bound by dispatch latency, so the
question is what a replayed graph of the same chain costs per reduce.

For each bucket size and chain length L: L in-place fp32 sum reduces
(mi_reduce) on distinct chunk pairs, issued (a) eagerly on one stream, timed
with events around the whole chain, (b) captured once into a torch CUDA graph
and replayed, (c) as one mi_reduce_batch call over the L descriptors.  Prints one JSON line per point.

  python tools/graph_probe.py [--reps 50] > out.jsonl
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from oneccl_amd import _lib  # noqa: E402

FP32, SUM = 9, 0


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    m = _lib.mi()
    for nbytes in (4096, 65536, 1 << 20):
        n = nbytes // 4
        for L in (1, 8, 64):
            acc = [torch.randn(n, device="cuda") for _ in range(L)]
            inp = [torch.randn(n, device="cuda") for _ in range(L)]
            stream = torch.cuda.Stream()

            def chain(s):
                for a, b in zip(acc, inp):
                    _lib.check(m.mi_reduce(b.data_ptr(), a.data_ptr(), n, FP32, SUM, 0, s))

            def timed(fn):
                ts, ws = [], []
                with torch.cuda.stream(stream):
                    for r in range(args.reps + 5):
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        t0 = time.perf_counter()
                        e0.record(stream)
                        fn()
                        e1.record(stream)
                        e1.synchronize()
                        t1 = time.perf_counter()
                        if r >= 5:
                            ts.append(e0.elapsed_time(e1) * 1e3)
                            ws.append((t1 - t0) * 1e6)
                return statistics.median(ts), statistics.median(ws)

            eager, eager_w = timed(lambda: chain(stream.cuda_stream))
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                chain(torch.cuda.current_stream().cuda_stream)
            graph, graph_w = timed(g.replay)
            descs = _lib.desc_array([(b.data_ptr(), a.data_ptr(), n) for a, b in zip(acc, inp)])
            batch, batch_w = timed(lambda: _lib.check(
                m.mi_reduce_batch(descs, L, FP32, SUM, 0, stream.cuda_stream), "mi_reduce_batch"))
            print(json.dumps({"bucket_bytes": nbytes, "chain": L, "eager_us": round(eager, 2),
                              "graph_us": round(graph, 2), "eager_us_per_reduce": round(eager / L, 2),
                              "graph_us_per_reduce": round(graph / L, 2),
                              "eager_wall_us": round(eager_w, 2), "graph_wall_us": round(graph_w, 2),
                              "batch_us": round(batch, 2), "batch_wall_us": round(batch_w, 2),
                              "timing": "torch events on the issuing stream around the chain (gpu) and host clock from "
                                        "first call to completion (wall); median of "
                                        f"{args.reps}"}), flush=True)
            del g


if __name__ == "__main__":
    main()
