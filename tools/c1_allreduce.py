#!/usr/bin/env python3
"""BASELINE.json configs[0] end to end: `examples/benchmark allreduce fp32 sum,
2 ranks loopback, 1 MiB` with the local reduce step done by the drop-in.

Each rank runs oneCCL's nreduce allreduce schedule for P ranks
(src/coll/algorithms/allreduce/allreduce.cpp:292-440): the buffer is split in
P chunks; rank r receives chunk r from every peer into a host staging buffer
(the `comm_buf` of recv_reduce_entry, src/sched/entry/recv_reduce_entry.hpp:66-68)
and folds it with ccl_comp_reduce(in=comm_buf, inout=own chunk); then the
reduced chunks are all-gathered.  Transport: torch.distributed gloo
send/recv on host tensors (the role ATL's MPI/OFI plays).  Fill and check
follow examples/benchmark: send = rank, expected = (P-1)*P/2
(include/coll.hpp:152-170, src/allreduce/cpu_allreduce_coll.hpp:29-57).

  python tools/c1_allreduce.py [--ranks 2] [--count 262144] [--iters 50] [--reduce dropin|oracle]
Rank 0 prints one JSON line with the per-iteration time.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def nreduce_allreduce(buf, rank, world, reduce2, recv_bufs, fused=None):
    """In-place allreduce of a float32 host tensor (nreduce schedule); the
    element count must be a multiple of the rank count.  `fused(recv_all,
    own)`, if given, folds all arrived chunks with one ccl_comp_batch_reduce
    call instead of world-1 chained ccl_comp_reduce calls."""
    import torch
    import torch.distributed as dist
    n = buf.numel()
    assert n % world == 0
    per = n // world
    chunks = [buf[i * per:(i + 1) * per] for i in range(world)]
    own = chunks[rank]
    reqs = []
    for peer in range(world):
        if peer != rank:
            reqs.append(dist.isend(chunks[peer], peer))
            reqs.append(dist.irecv(recv_bufs[peer], peer))
    for r in reqs:
        r.wait()
    t_red = time.perf_counter()
    if fused is not None:
        fused(rank, own)
    else:
        for peer in range(world):  # fold each peer's chunk into the owned chunk
            if peer != rank:
                reduce2(recv_bufs[peer], own)
    t_red = time.perf_counter() - t_red
    gathered = [torch.empty_like(own) for _ in range(world)]
    dist.all_gather(gathered, own)
    for i, g in enumerate(gathered):
        if i != rank:
            chunks[i].copy_(g)
    return t_red


def worker(rank, world, port, count, iters, mode, q, fused_call=False, sched=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if mode == "dropin-gpu":  # the drop-in with its CPU path off: every reduce on the GPU
        os.environ["CCL_COMP_HOST_MAX_BYTES"] = "0"
    import numpy as np
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        if mode in ("dropin", "dropin-gpu"):
            from oneccl_amd import _lib, comp
            if sched:  # the entries' schedule, as a CPU oneCCL build passes it: no stream, host memory
                _lib.shim().mi_ccl_comp_shim_sched(1)

            def reduce2(inp, inout):
                comp.comp_reduce(inp.data_ptr(), inp.numel(), inout.data_ptr(), comp.datatype.float32,
                                 comp.reduction.sum)
        else:
            import oracle

            def reduce2(inp, inout):
                oracle.comp_reduce(inp.numpy(), inout.numpy(), 9, 0)

        per = count // world
        recv_all = torch.empty(world * per, dtype=torch.float32)  # one staging area, chunk p at p*per
        recv = {p: recv_all[p * per:(p + 1) * per] for p in range(world)}
        fused = None
        if fused_call:
            if mode in ("dropin", "dropin-gpu"):
                from oneccl_amd import comp

                def fused(r, own):
                    offs = [0] + [p * per for p in range(world) if p != r]  # offsets[0] unused
                    comp.comp_batch_reduce(recv_all.data_ptr(), offs, per, own.data_ptr(), comp.datatype.float32,
                                           comp.reduction.sum)
            else:
                import oracle

                def fused(r, own):
                    offs = [0] + [p * per for p in range(world) if p != r]
                    oracle.batch_reduce(recv_all.numpy(), offs, per, own.numpy(), 9, 0, 0)
        buf = torch.empty(count, dtype=torch.float32)
        ok = True
        times, red = [], []
        for it in range(iters + 3):
            buf.fill_(float(rank))
            dist.barrier()
            t0 = time.perf_counter()
            tr = nreduce_allreduce(buf, rank, world, reduce2, recv, fused)
            dist.barrier()
            if it >= 3:
                times.append(time.perf_counter() - t0)
                red.append(tr)
            ok = ok and bool(torch.all(buf == (world - 1) * (world / 2)).item())
        t = torch.tensor([min(times), float(np.median(times)), min(red), float(np.median(red))],
                         dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        q.put((rank, ok, t.tolist()))
    finally:
        dist.destroy_process_group()


def run(world=2, count=262144, iters=50, mode="dropin", fused_call=False, sched=False):
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=worker, args=(r, world, port, count, iters, mode, q, fused_call, sched))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=600) for _ in range(world)])
    for p in procs:
        p.join(timeout=60)
    return {"config": "examples/benchmark allreduce fp32 sum, loopback (BASELINE configs[0])", "ranks": world,
            "count": count, "bytes": count * 4, "local_reduce": mode, "fused_batch_reduce": fused_call,
            "host_schedule": sched,
            "iters": iters,
            "correct": all(r[1] for r in res) and all(p.exitcode == 0 for p in procs),
            "best_us": round(res[0][2][0] * 1e6, 1), "median_us": round(res[0][2][1] * 1e6, 1),
            "reduce_best_us": round(res[0][2][2] * 1e6, 1), "reduce_median_us": round(res[0][2][3] * 1e6, 1),
            "reduce_note": "time in the local reduce step (the src/comp calls) per allreduce, max over ranks",
            "reduce_calls_per_rank": 1 if fused_call else world - 1, "reduce_elems_per_call": count // world}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--count", type=int, default=262144)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--reduce", default="dropin", choices=["dropin", "dropin-gpu", "oracle"],
                    help="dropin: the shim with its default dispatch (small host chunks on the CPU); "
                         "dropin-gpu: the shim with every reduce on the GPU; oracle: the CPU restatement")
    ap.add_argument("--fused", action="store_true", help="one ccl_comp_batch_reduce per rank")
    ap.add_argument("--sched", action="store_true",
                    help="pass a schedule without a stream, as the entries of a CPU oneCCL build do (no lookups)")
    a = ap.parse_args()
    print(json.dumps(run(a.ranks, a.count, a.iters, a.reduce, a.fused, a.sched)), flush=True)
