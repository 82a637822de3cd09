"""The N>1 bench path on CPU: world_size-2 gloo process group exercising the
same helpers bench.py uses on the GPU node — element-range planning (no data
exchange between ranks) and the max-over-ranks timing reduction — and that
per-rank shard reduces compose to the whole-bucket result (oracle as the
stand-in compute on CPU; the GPU step itself is covered by tests/test_gpu_*)."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_total, scaling, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    import oracle
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n, first, total = bench.plan(n_total, 4, rank, world, scaling)
        rng = np.random.default_rng(5)
        a = rng.standard_normal(n_total).astype(np.float32)
        b = rng.standard_normal(n_total).astype(np.float32)
        if scaling == "strong":
            part = b[first:first + n].copy()
            oracle.comp_reduce(np.ascontiguousarray(a[first:first + n]), part, 9, 0)
            parts = [None] * world
            dist.all_gather_object(parts, (first, part))
        else:
            parts = None
        mx = bench.max_over_ranks([float(rank + 1), 10.0 - rank], world, "cpu")
        q.put((rank, n, first, total, mx, parts))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("scaling", ["weak", "strong"])
def test_two_rank_gloo_plan_and_timing(scaling):
    world, n_total = 2, 1_000_003
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_total, scaling, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, n, first, total, mx, parts in res:
        assert mx == [2.0, 10.0]  # max over ranks of each value
        if scaling == "weak":
            assert n == n_total and total == n_total * 4 * world
        else:
            assert total == n_total * 4
    if scaling == "strong":
        assert res[0][2] == 0 and res[0][1] + res[1][1] == n_total and res[1][2] == res[0][1]
        import oracle
        rng = np.random.default_rng(5)
        a = rng.standard_normal(n_total).astype(np.float32)
        b = rng.standard_normal(n_total).astype(np.float32)
        oracle.comp_reduce(a, b, 9, 0)
        whole = np.concatenate([p for _, p in sorted(res[0][5], key=lambda x: x[0])])
        assert whole.tobytes() == b.tobytes()


def _c4_worker(rank, world, port, q):
    """BASELINE configs[3] as written: one 8-input fan-in bucket split by
    element range over the ranks (bench.strong_split's plan)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    import oracle
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n_total, k = 300_017, 8
        n, first, total = bench.plan(n_total, 4, rank, world, "strong")
        rng = np.random.default_rng(11)
        ins = [rng.standard_normal(n_total).astype(np.float32) for _ in range(k)]
        shard = oracle.fanin([np.ascontiguousarray(x[first:first + n]) for x in ins], 9, 0)
        parts = [None] * world
        dist.all_gather_object(parts, (first, shard))
        q.put((rank, n, total, parts))
    finally:
        dist.destroy_process_group()


def test_two_rank_c4_strong_split_composes():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_c4_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import oracle
    n_total = 300_017
    assert sum(r[1] for r in res) == n_total and all(r[2] == n_total * 4 for r in res)
    rng = np.random.default_rng(11)
    ins = [rng.standard_normal(n_total).astype(np.float32) for _ in range(8)]
    whole = np.concatenate([p for _, p in sorted(res[0][3], key=lambda x: x[0])])
    assert whole.tobytes() == oracle.fanin(ins, 9, 0).tobytes()


def test_pmc_traffic_scales_to_the_launch():
    """roofline.traffic for a launch of another size (a strong-scaling
    shard) is the measured PMC ratio applied to that launch's bytes."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    full = bench.pmc_traffic("c2", 3 * (1 << 30))
    if full is None:
        pytest.skip("no committed PMC pass")
    half = bench.pmc_traffic("c2", 3 * (1 << 29))
    assert abs(half["bytes_per_launch"] * 2 - full["bytes_per_launch"]) <= 2
    assert half["ratio"] == full["ratio"] and 0.99 < half["ratio"] < 1.01


def test_kernel_identity_is_the_device_code():
    """The PMC pass a bench line cites is matched by the hash of the built
    library's device code (.hip_fatbin), not of source files: a host-only edit
    keeps a pass current, a kernel change makes it stale."""
    import hashlib
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    lib = os.path.join(root, bench.KERNEL_LIB)
    objcopy = "/opt/rocm/lib/llvm/bin/llvm-objcopy"
    if not os.path.exists(lib) or not os.path.exists(objcopy):
        pytest.skip("library or llvm-objcopy absent")
    ident = bench.kernel_identity()
    assert ident and ident.startswith("fatbin:")
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        subprocess.run([objcopy, f"--dump-section=.hip_fatbin={fat}", lib, os.path.join(d, "x.so")], check=True,
                       capture_output=True)
        with open(fat, "rb") as f:
            assert ident == "fatbin:" + hashlib.sha256(f.read()).hexdigest()[:16]
    passes = bench.pmc_passes("c2")
    assert all("hbm_bytes_per_launch" in e for _, e in passes)
