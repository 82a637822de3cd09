#!/usr/bin/env python3
"""Benchmark of the MI355X-native local reduction (oneCCL src/comp hot path).

Headline (BASELINE.json metric): GiB/s of device-resident fp32 sum-reduce of a
1 GiB bucket.  One "step" = one ccl_comp_reduce-equivalent call through the C
ABI (mi_reduce: inout += in over the whole bucket, inputs resident in HBM).

  python bench.py [--gpus N --steps K --warmup W] [--config c2|c3-bf16|c3-fp16|c4|...]
  torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)
With --gpus N > 1 and no launcher (WORLD_SIZE unset), bench.py starts the N
rank processes itself and relays rank 0's line.

Multi-GPU: the element range is sharded — every rank reduces
its own 1 GiB bucket shard with no data-path collective ("scaling": "weak");
torch.distributed is used only for the barrier and the max-over-ranks time.
Rank 0 prints ONE JSON line.  After the timed region every rank re-fills its
bucket, runs one more reduce and compares all of its elements bit for bit with
a torch-computed fold (`parity` in the line; exit 3 on any mismatch).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

GiB = 1 << 30
T0 = time.perf_counter()  # process start (for wall_s_rank0)
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md

# name -> (description, ccl dtype id, element size, op, n_inputs, bucket bytes, flags)
CONFIGS = {
    "c2": ("2-input fp32 sum-reduce, 1 GiB bucket, device-resident (BASELINE configs[1])", 9, 4, 0, 2, GiB, 0),
    "c3-bf16": ("2-input bf16 sum, fp32 math + one RNE rounding, 256 MiB bucket (configs[2])", 11, 2, 0, 2,
                256 << 20, 0x1 | 0x2),
    "c3-fp16": ("2-input fp16 sum, fp32 math + one RNE rounding, 256 MiB bucket (configs[2])", 8, 2, 0, 2,
                256 << 20, 0x1),
    "c4": ("8-input fan-in fp32 sum (ring-chunk arrival pattern), 1 GiB bucket (configs[3])", 9, 4, 0, 8, GiB, 0),
    "c4-bf16acc": ("8-input fan-in bf16 sum, fp32 accumulate, 1 GiB bucket", 11, 2, 0, 8, GiB, 0x4 | 0x2),
    "c4-tmpbuf": ("8-input fan-in fp32 sum, 1 GiB bucket, nreduce layout: the 7 peer chunks in consecutive slots of "
                  "one tmp allocation, folded into the separate reduce_buf in place (allreduce.cpp:333-394)",
                  9, 4, 0, 8, GiB, 0),
    "c5-int32-max": ("2-input int32 max, 1 GiB bucket (configs[4])", 4, 4, 3, 2, GiB, 0),
    "c5-int64-prod": ("2-input int64 prod, 1 GiB bucket (configs[4])", 6, 8, 1, 2, GiB, 0),
}
DTYPE_LABEL = {9: "f32", 11: "bf16 (f32 math)", 8: "f16 (f32 math)", 4: "int32", 6: "int64"}


def mem_mark(tag):
    """MI_BENCH_MEM_TRACE=1: the device bytes torch holds now and its peak so
    far, per phase (checks memory_plan against what the phases allocate)."""
    if os.environ.get("MI_BENCH_MEM_TRACE"):
        import torch
        log(f"mem {tag}: allocated {torch.cuda.memory_allocated() >> 20} MiB, "
            f"peak {torch.cuda.max_memory_allocated() >> 20} MiB")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    p.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                   help="weak: every GPU reduces its own full bucket; strong: one bucket split over the GPUs")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="bound on the CPU baseline's work")
    p.add_argument("--no-host-leg", action="store_true", help="skip the host-resident (PCIe) measurement")
    p.add_argument("--no-config-legs", action="store_true",
                   help="skip the other BASELINE configs' legs (timed launches + full parity) of a c2 run")
    p.add_argument("--layout", default="padded", choices=LAYOUTS,
                   help="padded (default): a config's inputs in one allocation, a 2-input config's second operand "
                        f"{PAIR_OFFSET >> 20} MiB after its first; one: consecutive slices of one allocation; "
                        "separate: one allocation per input (DESIGN.md §6, placement modes)")
    p.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                   help="process group for the barrier / max-over-ranks only (gloo lets several ranks share "
                        "one GPU when rehearsing the N>1 path)")
    p.add_argument("--detail", default=os.environ.get("MI_BENCH_DETAIL", DETAIL_DEFAULT),
                   help="side file for the full result (method notes, probe arrays, per-leg ceilings, the CPU "
                        "sweep); the stdout line names it")
    return p.parse_args()


DETAIL_DEFAULT = "profiles/bench_detail.json"
LINE_LIMIT = 7000  # bytes: under the driver's 8000-character stdout tail, with room to spare


def write_detail(full, path):
    """The full result (everything the stdout line leaves out) as indented
    JSON at `path` (relative to the repo root).  Returns the path the line
    names, or an "unwritten: ..." note: a side file never costs the line."""
    p = Path(path) if Path(path).is_absolute() else ROOT / path
    try:
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_text(json.dumps(full, indent=1) + "\n")
    except OSError as e:
        return f"unwritten: {e}"
    try:
        return str(p.relative_to(ROOT))
    except ValueError:
        return str(p)


def _pick(d, keys):
    return {k: d[k] for k in keys if isinstance(d, dict) and k in d}


def compact_line(full, detail):
    """The ONE stdout line the driver parses, derived from the full result:
    the contract keys, `roofline` and `cpu_baseline` with their numbers, and
    per leg only {GiBps, frac, frac_of_mixed_ceiling, mismatches}.  Prose,
    probe arrays, per-leg ceiling dicts and the CPU sweep stay in the side
    file `detail`.  Kept under LINE_LIMIT bytes (a 21 KB
    line was not parsed); should it still be over, the optional sections
    go, last-listed first, and `trimmed` names them."""
    line = _pick(full, ("metric", "value", "unit", "n_gpus", "ranks", "ranks_per_device", "steps", "warmup",
                        "ms_per_step", "higher_is_better", "scaling", "vs_baseline", "dtype", "data"))
    c = full.get("config", {})
    line["config"] = dict(_pick(c, ("workload", "bucket_bytes_per_gpu", "inputs", "op", "parallelism")),
                          layout=c.get("layout_name", c.get("layout")), entry="mi_reduce")
    r = full.get("roofline", {})
    roof = _pick(r, ("bound", "achieved", "peak", "unit", "frac", "traffic", "traffic_ratio_to_algorithmic",
                     "algorithmic_bytes_per_launch", "avg_kernel_ms", "avg_kernel_ms_max_rank", "kernel_ms_min",
                     "ceiling_TBps", "frac_of_ceiling", "ceiling_mixed_TBps", "frac_of_mixed_ceiling",
                     "frac_by_placement", "traffic_source"))
    if "aggregate" in r:
        roof["aggregate"] = _pick(r["aggregate"], ("achieved", "peak", "frac", "devices"))
    line["roofline"] = roof
    cpu = full.get("cpu_baseline")
    if isinstance(cpu, dict) and "error" not in cpu:
        cb = _pick(cpu, ("value", "unit", "cores", "kind", "sample_short", "cpu_model", "port_1thread",
                         "median"))
        if "sample_short" in cb:
            cb["sample"] = cb.pop("sample_short")
        mt = cpu.get("multi_thread", {})
        cb["multi_thread"] = _pick(mt, ("threads", "value", "median", "spread", "reps", "cgroup_cpu_quota",
                                        "throttled", "throttled_usec", "psi_cpu_some_us"))
        line["cpu_baseline"] = cb
    else:
        line["cpu_baseline"] = cpu
    par = full.get("parity", {})
    line["parity"] = _pick(par, ("elements", "mismatches"))
    if full.get("dropin_sync"):
        d = full["dropin_sync"]
        line["dropin_sync"] = dict(_pick(d, ("value", "best")), mismatches=d.get("parity", {}).get("mismatches"))
    if full.get("strong_split"):
        line["strong_split"] = {k: dict(_pick(v, ("value", "ms_per_step", "avg_kernel_ms_max_rank")),
                                        frac=v.get("aggregate_roofline", {}).get("frac"))
                                for k, v in full["strong_split"].items()}
    if full.get("memory"):
        m = full["memory"]
        line["memory"] = {"planned_peak_bytes_rank0": m.get("planned_peak_bytes_rank0"),
                          "measured_max_rank": m.get("torch_max_allocated_bytes_max_rank")}
    for k in ("rehearsal", "wall_s_rank0"):
        if k in full:
            line[k] = full[k]
    if full.get("host_resident"):
        h = full["host_resident"]
        line["host_resident"] = h if "error" in h else _pick(
            h, ("bucket_bytes", "pinned", "pinned_staged", "pageable", "pageable_registered", "dropin_pinned",
                "dropin_pageable"))
    if full.get("configs"):
        legs = {}
        for name, v in full["configs"].items():
            mism = v.get("parity", {}).get("mismatches")
            if "GiBps" in v:
                legs[name] = dict(_pick(v, ("GiBps", "frac_of_mixed_ceiling")), frac=v.get("roofline_frac"),
                                  mismatches=mism)
            else:  # C1: a host chunk through the drop-in, timed in µs
                legs[name] = dict(_pick(v, ("median_us", "best_us")), mismatches=mism)
        line["configs"] = legs
    line["detail"] = detail
    trimmed = []
    for k in ("host_resident", "strong_split", "memory", "configs"):
        if len(json.dumps(line, separators=(",", ":"))) <= LINE_LIMIT:
            break
        if line.pop(k, None) is not None:
            trimmed.append(k)
    if trimmed:
        line["trimmed"] = trimmed
    return line


def fill(t, seed):
    """Synthetic inputs in [-1, 1) (fp) / small ints, generated on the device."""
    import torch
    g = torch.Generator(device=t.device)
    g.manual_seed(seed)
    if t.dtype.is_floating_point:
        t.uniform_(-1.0, 1.0, generator=g)
    else:
        t.random_(-1000, 1000, generator=g)


LAYOUTS = ("padded", "one", "separate")
PAIR_OFFSET = 1920 << 20  # where a padded layout's second operand starts, from the first
PAIR_GAP = 896 << 20  # past the bucket, for a bucket larger than PAIR_OFFSET


def pair_stride_bytes(nbytes):
    """Offset of a padded layout's second operand from its first."""
    return PAIR_OFFSET if nbytes <= PAIR_OFFSET else nbytes + PAIR_GAP


LAYOUT_NOTE = {
    "padded": f"the inputs in one allocation; a 2-input config's second operand {PAIR_OFFSET >> 20} MiB after the "
              f"first (buckets up to that size; larger: {PAIR_GAP >> 20} MiB past the bucket)",
    "one": "the inputs as consecutive slices of one allocation",
    "separate": "one allocation per input",
}


def alloc_inputs(k, n, tdt, layout, device="cuda"):
    """The k input buffers of n elements.  Where the operands sit relative to
    each other decides the 2-input reduce's rate by up to 7 % (DESIGN.md §6,
    "Where the run-to-run spread comes from"): separate allocations draw a
    placement per run (fast, medium or slow: 0.471-0.511 ms for C2); slices of
    one allocation run at one rate whose level follows their offset (C2: 0.480
    ms at 1 GiB, 0.473-0.475 at 1 GiB + 896 MiB on two boxes,
    profiles/round4_run7/; 256 MiB operands likewise, profiles/round4_run12/).
    "padded" starts a 2-input config's second operand PAIR_OFFSET after its
    first (pair_stride_bytes) and is contiguous for a fan-in (whose rate no gap
    steadied); "one" is contiguous; "separate" is an allocation each."""
    import torch
    if layout == "separate":
        return [torch.empty(n, dtype=tdt, device=device) for _ in range(k)]
    es = torch.empty(0, dtype=tdt).element_size()
    stride = pair_stride_bytes(n * es) // es if layout == "padded" and k == 2 else n
    slab = torch.empty((k - 1) * stride + n, dtype=tdt, device=device)
    return [slab[j * stride:j * stride + n] for j in range(k)]


TMPBUF_NOTE = ("oneCCL's nreduce layout (allreduce.cpp:326-394): reduce_buf is its own allocation, the k - 1 peer "
               "chunks sit in consecutive slots of one tmp allocation")


def alloc_tmpbuf(k, n, tdt, device="cuda"):
    """The nreduce fan-in's operands as oneCCL lays them out: the schedule's
    reduce_buf apart, and the k - 1 peer chunks received into consecutive
    slots of one tmp buffer (src/coll/algorithms/allreduce/allreduce.cpp:
    326-394), folded into reduce_buf in place."""
    import torch
    tmp = torch.empty((k - 1) * n, dtype=tdt, device=device)
    return [torch.empty(n, dtype=tdt, device=device)] + [tmp[j * n:(j + 1) * n] for j in range(k - 1)]


def torch_dtype(dt):
    import torch
    return {9: torch.float32, 11: torch.bfloat16, 8: torch.float16, 4: torch.int32, 6: torch.int64}[dt]


def _cpulist(text):
    """Linux cpulist syntax ("0-3,8,10-11") -> [int]."""
    out = []
    for part in text.strip().split(","):
        if "-" in part:
            a, b = part.split("-")
            out += range(int(a), int(b) + 1)
        elif part:
            out.append(int(part))
    return out


def core_plan():
    """(NUMA node, one CPU per physical core of that node within this
    process's affinity, CPUs in the affinity, cgroup CPU quota or None): the
    node holding most allowed CPUs; of each core's hyperthread siblings the
    first; ordered round robin over the node's L3 domains.  oneCCL pins one worker per core the same way
    (src/exec/thread/worker.cpp:310-379, CCL_WORKER_AFFINITY)."""
    aff = set(os.sched_getaffinity(0))
    nodes = {}
    for d in sorted(Path("/sys/devices/system/node").glob("node[0-9]*")):
        try:
            nodes[int(d.name[4:])] = set(_cpulist((d / "cpulist").read_text()))
        except (OSError, ValueError):
            continue
    if not nodes:
        nodes = {0: set(aff)}
    node = max(nodes, key=lambda x: (len(nodes[x] & aff), -x))
    seen, cores = set(), []
    for c in sorted(nodes[node] & aff):
        try:
            sib = tuple(_cpulist(Path(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list").read_text()))
        except (OSError, ValueError):
            sib = (c,)
        if sib not in seen:
            seen.add(sib)
            cores.append(c)
    # round robin over the L3 domains (a Zen 5 CCD: 8 cores behind one link
    # to the memory side), so T threads draw on min(T, domains) links: the
    # first T cores of one CCD would measure that CCD's link, not the node
    groups = {}
    for c in cores:
        try:
            key = Path(f"/sys/devices/system/cpu/cpu{c}/cache/index3/shared_cpu_list").read_text().strip()
        except OSError:
            key = ""
        groups.setdefault(key, []).append(c)
    lists = list(groups.values())
    cores = [lst[i] for i in range(max(map(len, lists), default=0)) for lst in lists if i < len(lst)]
    quota = None
    try:
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()
        if q != "max":
            quota = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return node, cores, len(aff), quota


class PinnedPool:
    """T threads, thread i pinned to cpus[i] for its whole life; run(job)
    releases all of them on job(i) and returns when every one is done."""

    def __init__(self, cpus):
        import threading
        self.n = len(cpus)
        self.go = threading.Barrier(self.n + 1)
        self.done = threading.Barrier(self.n + 1)
        self.job = None
        self.errors = []
        self.pin_errors = []  # reported, not raised: an unpinned thread still measures

        self.tids = set()

        def body(i, cpu):
            self.tids.add(threading.get_native_id())
            try:
                os.sched_setaffinity(0, {cpu})  # pid 0: the calling thread
            except OSError as e:
                self.pin_errors.append(f"pin cpu {cpu}: {e}")
            while True:
                self.go.wait()
                job = self.job
                if job is None:
                    return
                try:
                    job(i)
                except Exception as e:  # noqa: BLE001
                    self.errors.append(repr(e))
                self.done.wait()

        self.threads = [threading.Thread(target=body, args=(i, c), daemon=True) for i, c in enumerate(cpus)]
        for t in self.threads:
            t.start()

    def run(self, job):
        self.job = job
        self.go.wait()
        self.done.wait()
        if self.errors:
            raise RuntimeError("; ".join(self.errors[:3]))

    def close(self):
        self.job = None
        self.go.wait()
        for t in self.threads:
            t.join()


def cpu_sweep_point(cfg, cpus, seconds, use_ref, pids=None):
    """One thread count of the CPU baseline: len(cpus) threads, each pinned
    to its core, each first-touching its own element range of every buffer
    (so its pages sit on its own NUMA node), then reducing
    that range with the reference's loop: k - 1 chained 2-input calls, as
    CCL_WORKER_COUNT workers would each reduce their chunk.  Whole-bucket
    reps repeated for ~`seconds`; returns (best GiB/s, median GiB/s, reps,
    the threads that could not be pinned)."""
    import ctypes

    import numpy as np
    import oracle
    desc, dt, es, op, k, bucket, flags = cfg
    n = bucket // es
    T = len(cpus)
    per = (n + T - 1) // T
    per += (-per) % 64  # 256-byte aligned ranges: no two threads share a cache line
    parts = [(min(n, i * per), min(n, (i + 1) * per)) for i in range(T)]
    npdt = oracle.NP_DTYPE[dt]
    ins = [np.empty(n, npdt) for _ in range(k - 1)]  # untouched pages until each thread's fill
    acc = np.empty(n, npdt)
    if dt == 11:
        vin, vacc = np.uint16(0x3E80), np.uint16(0x3F80)  # bf16 0.25, 1.0
    elif dt == 8:
        vin, vacc = np.uint16(0x3400), np.uint16(0x3C00)  # fp16 0.25, 1.0
    elif dt in (9, 10):
        vin, vacc = npdt(1.0 if op == 1 else 0.25), npdt(1.0)
    else:
        vin, vacc = npdt(1 if op == 1 else 3), npdt(1)

    def touch(i):
        lo, hi = parts[i]
        for x in ins:
            x[lo:hi] = vin
        acc[lo:hi] = vacc

    if use_ref:
        L = oracle.ref_comp_lib()
        f = L.ref_ccl_comp_reduce_regular
        ptrs = [x.ctypes.data for x in ins]
        pacc = acc.ctypes.data

        def reduce(i):
            lo, hi = parts[i]
            if hi > lo:
                for p in ptrs:
                    f(p + lo * es, hi - lo, pacc + lo * es, None, dt, es, op)
    else:
        def reduce(i):
            lo, hi = parts[i]
            if hi > lo:
                for x in ins:
                    oracle.comp_reduce(x[lo:hi], acc[lo:hi], dt, op)

    pool = PinnedPool(cpus)
    pin_errors = pool.pin_errors
    moved = {}
    try:
        pool.run(touch)
        moved = clear_cores(set(cpus), pool.tids, pids)
        pool.run(reduce)  # warm
        times = []
        st0, ps0 = cgroup_cpu_stat(), psi_totals()
        t_start = time.perf_counter()
        while len(times) < 5 or (time.perf_counter() - t_start < seconds and len(times) < 400):
            t0 = time.perf_counter()
            pool.run(reduce)
            times.append(time.perf_counter() - t0)
        st1, ps1 = cgroup_cpu_stat(), psi_totals()
    finally:
        restore_affinity(moved)
        pool.close()
    del ins, acc
    throttle = {k: st1[k] - st0[k] for k in ("nr_periods", "nr_throttled", "throttled_usec")
                if k in st0 and k in st1}
    # tasks of this machine (or VM) waiting for a CPU / stalled on memory
    # during the timed reps, in microseconds (/proc/pressure, "some")
    throttle.update({f"psi_{k}_some_us": ps1[k] - ps0[k] for k in ps0 if k in ps1})
    return (bucket / GiB / min(times), bucket / GiB / statistics.median(times), len(times), list(pin_errors),
            throttle)


def clear_cores(cores, keep, pids=None):
    """Move every other thread of this process (the main thread, the HIP
    runtime's, the library's helpers) and of `pids` (the other ranks of an
    N-rank run, waiting meanwhile) off `cores` while the timing threads
    (native ids `keep`) run there, so none of them queues behind another
    thread on its core.  Returns {tid: previous affinity} for
    restore_affinity; threads that cannot be moved are left as they are."""
    moved = {}
    tids = []
    for pid in pids or [os.getpid()]:
        try:
            tids += [int(t) for t in os.listdir(f"/proc/{pid}/task")]
        except OSError:
            continue
    for tid in tids:
        if tid in keep:
            continue
        try:
            prev = os.sched_getaffinity(tid)
            rest = prev - cores
            if rest and rest != prev:
                os.sched_setaffinity(tid, rest)
                moved[tid] = prev
        except OSError:
            continue
    return moved


def restore_affinity(moved):
    for tid, prev in moved.items():
        try:
            os.sched_setaffinity(tid, prev)
        except OSError:
            pass  # the thread has exited


def cgroup_cpu_stat(path="/sys/fs/cgroup/cpu.stat"):
    """The cgroup's CPU counters ({nr_periods, nr_throttled, throttled_usec,
    ...}; empty when there is no cgroup v2 cpu controller).  Read around
    each timed sweep point: a point whose threads plus the process's other
    threads exceed the cgroup's quota is throttled, and its spread says
    nothing about the reduce."""
    out = {}
    try:
        for ln in Path(path).read_text().splitlines():
            k, _, v = ln.partition(" ")
            if v.strip().isdigit():
                out[k] = int(v)
    except OSError:
        pass
    return out


def psi_totals(root="/proc/pressure"):
    """Pressure-stall totals ({"cpu": us, "memory": us}, the "some" line;
    empty where the kernel has no PSI)."""
    out = {}
    for k in ("cpu", "memory"):
        try:
            for ln in Path(root, k).read_text().splitlines():
                if ln.startswith("some"):
                    out[k] = int(ln.rsplit("total=", 1)[1])
        except (OSError, ValueError, IndexError):
            pass
    return out


def sweep_counts(n_cores, quota):
    """Thread counts of the CPU sweep: 1, 8, 16, 32, 64 up to the node's
    physical cores; under a cgroup CPU quota Q, capped at Q - 1 (and Q - 1
    itself added), so the timing threads leave the process's main and
    runtime threads one CPU of the quota and are not throttled."""
    limit = n_cores if quota is None else min(n_cores, max(1, int(quota) - 1))
    counts = sorted({t for t in (1, 8, 16, 32, 64) if t <= max(1, limit)} | ({limit} if quota else set()))
    return counts, [t for t in (8, 16, 32, 64) if t not in counts]


def cpu_baseline(cfg, seconds, pids=None):
    """The reference's own CPU reduce (or, for the bf16/fp16 types it cannot
    reach standalone, the oracle's restatement) timed on this host's cores,
    a bounded sample: 1 thread (one ccl_worker, CCL_WORKER_COUNT=1 default)
    and a sweep of 8/16/32/64 pinned threads, each thread first-touching and
    reducing its own range of the same bucket (cpu_sweep_point)."""
    import numpy as np
    import oracle
    desc, dt, es, op, k, bucket, flags = cfg
    # the reference's own compiled CCL_REDUCE (oracle/_ref, its Release flags)
    # when it was built and the type is one it reaches; else the restatement
    use_ref = oracle.ref_comp_available() and dt not in (8, 11)
    node, cores, n_aff, quota = core_plan()
    counts, skipped = sweep_counts(len(cores), quota)
    share = max(seconds / (len(counts) + 1), 1.0)
    res = {}
    for t in counts:
        res[t] = cpu_sweep_point(cfg, cores[:t] if cores else [0], share * (2 if t == 1 else 1), use_ref, pids)
    port_1 = None
    if use_ref:  # the restatement on the same bucket, one thread, for comparison
        port_1 = round(cpu_sweep_point(cfg, cores[:1] if cores else [0], 1.0, False, pids)[0], 3)
    cpu_model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    (b1, m1, r1, _, _) = res[1]
    # sanity probe, independent of the oracle: one core's memcpy bandwidth
    # over the same footprint (numpy's copy is a single-threaded memcpy)
    src = np.ones(bucket // 8, np.float64)
    dst = np.empty_like(src)
    np.copyto(dst, src)
    ct = []
    for _ in range(5):
        t0 = time.perf_counter()
        np.copyto(dst, src)
        ct.append(time.perf_counter() - t0)
    copy_gbps = 2 * src.nbytes / min(ct) / 1e9
    del src, dst
    sweep = [dict({"threads": t, "best": round(b, 3), "median": round(m, 3), "reps": r,
                   "spread": round((b - m) / b, 4), "throttle": th}, **({"pin_errors": pe} if pe else {}))
             for t, (b, m, r, pe, th) in sorted(res.items())]
    # the reported point: the largest count under a quota (quota - 1), else 16
    head = max(res) if quota is not None or 16 not in res else 16
    bn, mn, rn, _, thn = res[head]
    return {
        "value": round(b1, 3), "median": round(m1, 3), "unit": "GiB/s", "cores": 1,
        "kind": "reference" if use_ref else "port",
        "sample_short": ("the reference's own CCL_REDUCE (src/comp/comp.cpp, Release flags, oracle/_ref)" if use_ref
                         else "oracle/comp_oracle.c restatement of CCL_REDUCE") +
                        f", {bucket >> 20} MiB x {k}-input bucket, 1 pinned thread, best of {r1} reps",
        "traffic_GBps_1core": round(b1 * GiB * (k + 1) / 1e9, 1),
        "copy_probe_GBps_1core": round(copy_gbps, 1),
        "traffic_note": f"the 1-core rate moves (k+1) = {k + 1} bucket-sizes of DRAM traffic per reduce; "
                        "copy_probe = 2 x bytes / time of one single-threaded memcpy of the bucket (read + "
                        "write), measured in the same run as an independent ceiling for one core",
        "sample": (("the reference's own ccl_comp_reduce_regular / CCL_REDUCE (src/comp/comp.cpp compiled with its "
                    "Release flags, g++ -O3, oracle/_ref/libref_ccl_comp.so)") if use_ref else
                   "oracle/comp_oracle.c (CPU restatement of src/comp CCL_REDUCE loop, gcc -O3)") +
                  f" on the same {bucket // (1 << 20)} MiB bucket x {k}-input, best of {r1} reps (median {m1:.2f} "
                  f"GiB/s); 1 thread = one ccl_worker (CCL_WORKER_COUNT=1 default), pinned to cpu "
                  f"{cores[0] if cores else 0}, its own first touch",
        "port_1thread": port_1,
        "port_note": "port_1thread = oracle/comp_oracle.c on one thread, the restatement the parity tests use "
                     "(it states the x86 NaN rule explicitly: a checker, not the baseline)"
        if port_1 is not None else None,
        "multi_thread": {"value": round(bn, 3), "median": round(mn, 3), "threads": head, "reps": rn,
                         "spread": round((bn - mn) / bn, 4), "sweep": sweep,
                         "throttled": thn.get("nr_throttled"), "throttled_usec": thn.get("throttled_usec"),
                         "psi_cpu_some_us": thn.get("psi_cpu_some_us"),
                         "numa_node": node, "physical_cores_in_node": len(cores), "cpus_in_affinity": n_aff,
                         "cgroup_cpu_quota": quota, "skipped_thread_counts": skipped,
                         "cpus_used": cores[:max(res)],
                         "note": "range split over threads, emulating CCL_WORKER_COUNT; one thread per physical core "
                                 f"of NUMA node {node} (first hyperthread sibling), taken round robin over the node's L3 "
                                 "domains (CCDs), pinned; each thread first-touches "
                                 "its own range of every buffer, then reduces it; thread counts above the node's "
                                 "physical cores, or above the cgroup's CPU quota - 1, are skipped; throttle = the "
                                 "cgroup's cpu.stat deltas over each point's timed reps; the process's other threads (and the other "
                                 "ranks') are moved off the timing cores while a point runs"},
        "cpu_model": cpu_model, "host_cpus": os.cpu_count(),
    }


def plan(n_total, es, rank, world, scaling):
    """Elements this rank reduces per step, its first element, and the bytes
    all ranks reduce per step.  weak: every rank owns a full bucket (the
    element range of a world x bucket job, sharded); strong: one bucket split
    by element range (mi_shard_range, 256-element aligned)."""
    if scaling == "weak":
        return n_total, rank * n_total, n_total * es * world
    import ctypes

    from oneccl_amd import _lib
    lo, hi = ctypes.c_size_t(), ctypes.c_size_t()
    _lib.check(_lib.mi().mi_shard_range(n_total, rank, world, 256, ctypes.byref(lo), ctypes.byref(hi)))
    return hi.value - lo.value, lo.value, n_total * es


def input_bytes(k, n, es, layout):
    """Device bytes alloc_inputs (or alloc_tmpbuf) takes for k inputs of n."""
    if layout == "padded" and k == 2:
        return pair_stride_bytes(n * es) + n * es
    return k * n * es


PARITY_CHUNK = 1 << 24  # elements per mismatch count (count_mismatches)
# count_nonzero's result and its reduction's scratch beside a chunk's mask:
# six 512-byte blocks of torch's allocator, measured (the N = 2 and N = 8
# rehearsals' peaks, profiles/round5_run10/, profiles/round6_run2/)
PARITY_COUNT_SMALL = 3072


def parity_bytes(n, dt, es, flags=0):
    """Device temporaries of full_parity: the torch fold (expected_result:
    the accumulator, folded in place; for bf16/fp16 an fp32 accumulator and
    one widened input, then the rounding: an int32 shift and the storage copy
    for bf16 truncation, the storage copy otherwise), then the expected result
    beside one chunk's mismatch mask and its int64 count (9 bytes per element
    of a chunk, plus the count's few small blocks).  Measured equal with
    MI_BENCH_MEM_TRACE=1."""
    if dt in (8, 11):
        trunc = dt == 11 and not (flags & 0x2)
        fold = max(8 * n, (4 + 4 + es) * n if trunc else (4 + es) * n)
    else:
        fold = es * n
    return max(fold, es * n + 9 * min(n, PARITY_CHUNK) + PARITY_COUNT_SMALL)


def memory_plan(config, layout, world, rank, scaling="weak"):
    """Device bytes this rank allocates in each phase of `bench.py --gpus
    world`, computed without a GPU (the N = 8 path's
    allocations checked before a node runs it).  Phases: the headline bucket
    (kept through the strong C2 split, which reuses it), its parity check's
    temporaries (the torch fold: the expected result and one step's
    intermediates), at N = 1 for c2 the config legs (each allocated and
    freed in turn while the headline buffers are held), and at N > 1 for c2
    the strong C4 fan-in shard (allocated after the headline bucket is
    freed).  Returns a dict with the peak."""
    desc, dt, es, op, k, bucket, flags = CONFIGS[config]
    n_total = bucket // es
    n, _, _ = plan(n_total, es, rank, world, scaling)
    lay = "tmpbuf" if config == "c4-tmpbuf" else layout
    head = input_bytes(k, n, es, lay)
    parity = parity_bytes(n, dt, es, flags)
    out = {"config": config, "layout": lay, "world": world, "rank": rank, "elements": n,
           "headline_inputs_bytes": head, "parity_temporaries_bytes": parity}
    peak = head + parity
    if world == 1 and config == "c2":
        # the config legs run while the headline buffers are still held
        legs = {}
        for name in ("c3-bf16", "c3-fp16", "c4", "c4-tmpbuf", "c4-bf16acc", "c5-int32-max", "c5-int64-prod",
                     "c2-layout-one", "c2-layout-separate"):
            _, ldt, les, _, lk, lbucket, lflags = CONFIGS["c2" if name.startswith("c2-") else name]
            ln = lbucket // les
            llay = "tmpbuf" if name == "c4-tmpbuf" else name[len("c2-layout-"):] if name.startswith("c2-") else layout
            legs[name] = input_bytes(lk, ln, les, llay) + parity_bytes(ln, ldt, les, lflags)
        legs["f3-copy"] = input_bytes(2, GiB // 4, 4, layout) + 9 * PARITY_CHUNK  # ccl_comp_copy on device
        out["config_legs_bytes"] = legs
        peak = max(peak, head + max(legs.values()))
    if world > 1 and config == "c2":
        n2, _, _ = plan(n_total, es, rank, world, "strong")
        n4, _, _ = plan(GiB // 4, 4, rank, world, "strong")
        out["strong_c2_shard_elements"] = n2  # reuses the headline buffers
        out["strong_c4_inputs_bytes"] = input_bytes(8, n4, 4, layout)
        out["strong_c4_shard_elements"] = n4
        peak = max(peak, out["strong_c4_inputs_bytes"])
    out["peak_bytes"] = peak
    return out


def expected_result(ins, k, dt, op, flags):
    """The whole bucket's expected result, computed on the device by plain
    torch ops, independent of the kernels: the left fold acc = ins[0];
    acc = op(ins[j], acc) of ccl_comp_reduce's CCL_REDUCE loop
    (src/comp/comp.cpp:31-58), chained as the reference chains K-1 calls.
    fp32 add is IEEE RNE on both sides, so the comparison is bit-exact; a
    bf16/fp16 fold computes in fp32 and rounds once (RNE) per step, or once
    at the end under F_ACC_FP32 (ccl_comp_batch_reduce keep-precision,
    comp.cpp:214-234).  Integer prod wraps in two's complement, as in C++."""
    import torch
    lp = dt in (8, 11)
    acc = ins[0].float() if lp else ins[0].clone()
    for j in range(1, k):  # in place: one accumulator, one widened input at a time (parity_bytes)
        x = ins[j].float() if lp else ins[j]
        if op == 0:
            acc.add_(x)
        elif op == 1:
            acc.mul_(x)
        elif op == 2:
            torch.minimum(x, acc, out=acc)
        else:
            torch.maximum(x, acc, out=acc)
        del x
        if lp and not (flags & 0x4):
            acc.copy_(to_storage(acc, dt, flags))  # storage precision after every step
    return to_storage(acc, dt, flags) if lp else acc


def to_storage(acc, dt, flags):
    """fp32 -> bf16/fp16 as the reference rounds: fp16 RNE (cvtps_ph, imm 0);
    bf16 RNE under F_BF16_RNE (avx512bf VCVTNEPS2BF16), otherwise truncation
    to the high 16 bits (scalar and avx512f impls, bf16.cpp:50-61)."""
    import torch
    if dt == 11 and not (flags & 0x2):
        return (acc.view(torch.int32) >> 16).to(torch.int16).view(torch.bfloat16)
    return acc.to(torch.bfloat16 if dt == 11 else torch.float16)


def shim_flags(dt):
    """The semantic flags ccl_comp_reduce applies on this host (CPUID +
    CCL_BF16 / CCL_FP16, comp.cpp's impl selection)."""
    from oneccl_amd import comp
    b, f = comp.impl_types()
    return comp.bf16_flags(b) if dt == 11 else comp.fp16_flags(f) if dt == 8 else 0


def count_mismatches(got, exp):
    """Elements whose bits differ (NaN payloads included)."""
    import torch
    ib = {1: torch.int8, 2: torch.int16, 4: torch.int32, 8: torch.int64}[got.element_size()]
    g, e = got.reshape(-1).view(ib), exp.reshape(-1).view(ib)
    # in chunks: counting a whole bucket's mask makes an int64 copy of it
    # (8 bytes per element, 2 GiB for the headline bucket; measured with
    # MI_BENCH_MEM_TRACE); a chunk bounds the temporaries (PARITY_CHUNK)
    total = 0
    for i in range(0, g.numel(), PARITY_CHUNK):
        total += int(torch.count_nonzero(torch.ne(g[i:i + PARITY_CHUNK], e[i:i + PARITY_CHUNK])).item())
    return total


def full_parity(run_once, ins, k, dt, op, flags, seed0, entry):
    """Outside the timed region: re-fill the bucket, compute the expected
    result on the device with torch, run ONE reduce through `run_once`, and
    compare every element bit for bit.  Returns the JSON `parity` object."""
    import torch
    for j, t in enumerate(ins):
        fill(t, seed0 + j)
    exp = expected_result(ins, k, dt, op, flags)
    torch.cuda.synchronize()
    run_once()
    torch.cuda.synchronize()
    mism = count_mismatches(ins[0], exp)
    del exp
    return {"elements": ins[0].numel(), "mismatches": mism, "entry": entry,
            "checker": "torch on the device (left fold in the reference's order, IEEE RNE; bits compared)"}


def timed_steps(step, steps, warmup, stream, world, probe=10):
    """W untimed steps, then exactly K steps bracketed by a barrier and a
    device synchronize on both sides, issued back to back with one HIP event
    pair around all of them on the launch stream: mean launch time = that
    region / K (the kernels plus their dependent-launch gaps, ~2 us each; no
    per-launch instrumentation inside the timed region).  Afterwards, outside
    it, `probe` launches each between their own event pair give the spread.
    Returns (wall s, mean launch ms, probe launch ms list)."""
    import torch
    import torch.distributed as dist

    from oneccl_amd import _lib
    for _ in range(warmup):
        _lib.check(step(), "mi_reduce")
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(steps):
        rc = step()
        if rc:
            _lib.check(rc, "mi_reduce")
    e1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    avg_ms = e0.elapsed_time(e1) / steps
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(probe)]
    for a, b in ev:
        a.record(stream)
        _lib.check(step(), "mi_reduce")
        b.record(stream)
    torch.cuda.synchronize()
    return elapsed, avg_ms, [a.elapsed_time(b) for a, b in ev]


CEILING_LIB = "oneccl_amd/lib/libmi_ceiling.so"


def measured_ceiling(ins, k, nbytes, stream, launches=10, out=None):
    """The achievable ceiling of a k-input reduce on these buffers, in this
    process: the fastest a memory-only kernel reads the k
    input streams (tools/ceiling_probe.hip mic_read_streams: 16-byte
    non-temporal loads, nothing written) and writes one stream
    (mic_write_stream), each over a few launch shapes, best shape taken.
    Reads and writes share HBM, so the reduce's k reads + 1 write cannot
    beat (k + 1) * nbytes / (t_read + t_write).  Writes over ins[0] (the
    caller refills before its parity check), or over `out` when given (a
    copy: k = 1, out the destination).  None if the probe library is
    missing (it is measurement infrastructure, not product)."""
    import ctypes

    import torch
    path = ROOT / CEILING_LIB
    if not path.exists():
        return None
    L = ctypes.CDLL(str(path))
    L.mic_read_streams.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_size_t, ctypes.c_int,
                                   ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    L.mic_write_stream.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_void_p]
    has_mixed = hasattr(L, "mic_mixed_streams")
    if has_mixed:
        L.mic_mixed_streams.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_void_p,
                                        ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    from oneccl_amd import _lib
    waves = ctypes.c_int(0)
    _lib.check(_lib.mi().mi_get_residency(-1, k, ctypes.byref(waves), None), "mi_get_residency")
    shapes = [(64, waves.value), (64, 0), (256, 0), (1024, 0)]
    arr = _lib.void_ptr_array([t.data_ptr() for t in ins[:k]])
    sink = torch.zeros(1024, dtype=torch.int32, device=ins[0].device)
    sh = stream.cuda_stream
    nb = nbytes - nbytes % 16

    def best(launch, flavors, shapes=shapes):
        res = []
        for fl in flavors:
            for block, w in shapes:
                for _ in range(2):
                    if launch(block, w, fl):
                        break
                else:
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    for _ in range(launches):
                        launch(block, w, fl)
                    e1.record(stream)
                    torch.cuda.synchronize()
                    res.append((e0.elapsed_time(e1) / launches, block, w, fl))
        return min(res) if res else None

    r = best(lambda b, w, fl: L.mic_read_streams(arr, k, nb, b, w, fl, sink.data_ptr(), sh), (0, 1))
    dst = (ins[0] if out is None else out).data_ptr()
    wr = best(lambda b, w, fl: L.mic_write_stream(dst, nb, b, w, fl, sh), (0, 1, 2))
    # the reads and the write in one launch, in place on ins[0] as the reduce
    # runs (stores ins[0]'s own vectors back: no arithmetic)
    # every residency the LDS granules allow for one-wave blocks (the library
    # picks one of them per k), so the ceiling is not the library's own choice
    mixed_shapes = [(64, w) for w in sorted({waves.value, 5, 8, 9, 11, 16, 21, 25})] + shapes[1:]
    mx = best(lambda b, w, fl: L.mic_mixed_streams(arr, k, dst, nb, b, w, fl, sh),
              (0, 1, 2), mixed_shapes) if has_mixed else None
    if not r or not wr:
        return None
    t = (r[0] + wr[0]) / 1e3
    flav = {0: "global nt", 1: "buffer nt", 2: "buffer sc1 nt"}
    mflav = {0: "global nt loads + nt stores", 1: "buffer nt loads + nt stores",
             2: "buffer nt loads + sc1 nt stores"}
    out = {"ceiling_TBps": round((k + 1) * nb / t / 1e12, 3),
           "read_TBps": round(k * nb / (r[0] / 1e3) / 1e12, 3), "read_shape": [r[1], r[2], flav[r[3]]],
           "write_TBps": round(nb / (wr[0] / 1e3) / 1e12, 3), "write_shape": [wr[1], wr[2], flav[wr[3]]],
           "method": f"memory-only probes on this leg's buffers (tools/ceiling_probe.hip): {k} read streams and one "
                     "write stream, each timed alone over block x wave-cap shapes and the load/store flavours the "
                     "kernels use [block, waves/CU (0 = no cap), flavour], best taken; ceiling = (k+1) x bytes / "
                     "(t_read + t_write)"}
    if mx:
        out["mixed_TBps"] = round((k + 1) * nb / (mx[0] / 1e3) / 1e12, 3)
        out["mixed_shape"] = [mx[1], mx[2], mflav[mx[3]]]
        out["mixed_ms"] = round(mx[0], 5)
        out["mixed_method"] = (f"{k} read streams and the write stream in ONE launch (mic_mixed_streams): each lane "
                               f"loads its 16-byte vector of all {k} inputs and stores input 0's back in place, no "
                               "arithmetic; the reduce's own access pattern and K:1 read:write interleave, best over "
                               "one-wave blocks at every residency 5-32 per CU and 256 / 1024-lane blocks, in the "
                               "same flavours")
    return out


def strong_split(m, dt, es, op, k, flags, n_total, rank, world, stream, steps, warmup, coll_dev, ins=None,
                 n_devices=None, layout="padded"):
    """One bucket of n_total elements split by element range over the ranks
    (mi_shard_range, 256-element aligned; BASELINE configs[3] as written):
    this rank reduces its shard of all k inputs.  `ins` (optional) holds
    device buffers at least a shard long to reuse.  value = the whole
    bucket / max-over-ranks wall time."""
    import torch
    n, _, total_bytes = plan(n_total, es, rank, world, "strong")
    tdt = torch_dtype(dt)
    if ins is None:
        ins = alloc_inputs(k, n, tdt, layout)
        for j, t in enumerate(ins):
            fill(t, 0xA0 + j + 7919 * rank)
    from oneccl_amd import _lib
    arr = _lib.void_ptr_array([t.data_ptr() for t in ins[:k]])
    sh = stream.cuda_stream

    def step():
        if k == 2:
            return m.mi_reduce(ins[1].data_ptr(), ins[0].data_ptr(), n, dt, op, flags, sh)
        return m.mi_reduce_multi(arr, k, ins[0].data_ptr(), n, dt, op, flags, sh)

    elapsed, avg_ms, _ = timed_steps(step, steps, warmup, stream, world)
    elapsed, avg_ms_max = max_over_ranks([elapsed, avg_ms], world, coll_dev)
    algo = (k + 1) * n * es
    return {"value": round(total_bytes * steps / elapsed / GiB, 2), "unit": "GiB/s", "inputs": k,
            "bucket_bytes_total": total_bytes, "shard_bytes_per_gpu": n * es,
            "ms_per_step": round(elapsed / steps * 1e3, 4),
            "avg_kernel_ms_max_rank": round(avg_ms_max, 5),
            "aggregate_roofline": {"achieved": round((k + 1) * total_bytes / (avg_ms_max / 1e3) / 1e9, 1),
                                   "peak": HBM_PEAK_GBPS * (n_devices or world),
                                   "frac": round((k + 1) * total_bytes / (avg_ms_max / 1e3) / 1e9 /
                                                 (HBM_PEAK_GBPS * (n_devices or world)), 4)},
            "per_rank_launch_bytes": algo,
            "scaling": "strong", "note": "one bucket split by element range over the ranks, no collective"}


def config_legs(m, stream, layout, launches=10):
    """The other BASELINE.json configs, each at its full size on this GPU, in
    the same run as the headline: mean launch time of `launches` back-to-back
    launches under one event pair, and the whole result checked bit for bit
    (full_parity).  C1 (configs[0]) is the 512 KiB nreduce chunk of a 2-rank
    1 MiB allreduce through ccl_comp_reduce on host buffers: the dispatcher
    keeps it on the calling thread's CPU, as oneCCL runs it."""
    import numpy as np
    import torch

    from oneccl_amd import _lib
    legs = {}
    sh = stream.cuda_stream
    c2_other = {f"c2-layout-{x}": x for x in LAYOUTS if x != layout}  # the headline in the other layouts
    for name in ("c3-bf16", "c3-fp16", "c4", "c4-tmpbuf", "c4-bf16acc", "c5-int32-max", "c5-int64-prod",
                 *c2_other):
        desc, dt, es, op, k, bucket, flags = CONFIGS["c2" if name in c2_other else name]
        n = bucket // es
        if name in c2_other:
            desc = f"the headline (2-input fp32 sum, 1 GiB bucket), layout: {LAYOUT_NOTE[c2_other[name]]}"
        if name == "c4-tmpbuf":
            ins = alloc_tmpbuf(k, n, torch_dtype(dt))
        else:
            ins = alloc_inputs(k, n, torch_dtype(dt), c2_other.get(name, layout))
        for j in range(k):  # (no loop variable left holding a view: `del ins` frees the leg)
            fill(ins[j], 0xC0 + 131 * j)
        arr = _lib.void_ptr_array([t.data_ptr() for t in ins])

        def step():
            if k == 2:
                return m.mi_reduce(ins[1].data_ptr(), ins[0].data_ptr(), n, dt, op, flags, sh)
            return m.mi_reduce_multi(arr, k, ins[0].data_ptr(), n, dt, op, flags, sh)

        for _ in range(2):
            _lib.check(step(), name)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(launches):
            _lib.check(step(), name)
        e1.record(stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / launches
        algo = (k + 1) * n * es
        ceil = measured_ceiling(ins, k, n * es, stream)
        par = full_parity(lambda: _lib.check(step(), name), ins, k, dt, op, flags, 0xE0, "mi_reduce" if k == 2 else
                          "mi_reduce_multi")
        legs[name] = {"workload": desc, "layout": TMPBUF_NOTE if name == "c4-tmpbuf" else
                      LAYOUT_NOTE[c2_other.get(name, layout)],
                      "GiBps": round(bucket / GiB / (ms / 1e3), 2), "avg_launch_ms": round(ms, 5),
                      "roofline_frac": round(algo / (ms / 1e3) / (HBM_PEAK_GBPS * 1e9), 4),
                      "parity": {"elements": par["elements"], "mismatches": par["mismatches"]}}
        if ceil:
            legs[name]["ceiling_TBps"] = ceil["ceiling_TBps"]
            legs[name]["frac_of_ceiling"] = round(algo / (ms / 1e3) / 1e12 / ceil["ceiling_TBps"], 4)
            if "mixed_TBps" in ceil:
                legs[name]["ceiling_mixed_TBps"] = ceil["mixed_TBps"]
                legs[name]["frac_of_mixed_ceiling"] = round(algo / (ms / 1e3) / 1e12 / ceil["mixed_TBps"], 4)
            legs[name]["ceiling"] = ceil
        del ins, arr
        torch.cuda.empty_cache()
    # ccl_comp_copy on device (copy_lean_kernel through
    # mi_copy), 1 GiB from one buffer of the layout to the other
    ins = alloc_inputs(2, GiB // 4, torch.float32, layout)
    dst, src = ins[0], ins[1]
    fill(src, 0xC0C0)
    for _ in range(2):
        _lib.check(m.mi_copy(src.data_ptr(), dst.data_ptr(), GiB, 0, sh), "mi_copy")
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(launches):
        _lib.check(m.mi_copy(src.data_ptr(), dst.data_ptr(), GiB, 0, sh), "mi_copy")
    e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / launches
    ceil = measured_ceiling([src], 1, GiB, stream, out=dst)
    fill(src, 0xC0C1)
    dst.zero_()
    _lib.check(m.mi_copy(src.data_ptr(), dst.data_ptr(), GiB, 0, sh), "mi_copy")
    torch.cuda.synchronize()
    leg = {"workload": "ccl_comp_copy on device (SURVEY §8(f)3): 1 GiB, mi_copy (copy_lean_kernel)",
           "layout": LAYOUT_NOTE[layout], "GiBps": round(1.0 / (ms / 1e3), 2), "avg_launch_ms": round(ms, 5),
           "roofline_frac": round(2 * GiB / (ms / 1e3) / (HBM_PEAK_GBPS * 1e9), 4),
           "parity": {"elements": src.numel(), "mismatches": count_mismatches(dst, src)}}
    if ceil:
        leg["ceiling_TBps"] = ceil["ceiling_TBps"]
        leg["frac_of_ceiling"] = round(2 * GiB / (ms / 1e3) / 1e12 / ceil["ceiling_TBps"], 4)
        if "mixed_TBps" in ceil:
            leg["ceiling_mixed_TBps"] = ceil["mixed_TBps"]
            leg["frac_of_mixed_ceiling"] = round(2 * GiB / (ms / 1e3) / 1e12 / ceil["mixed_TBps"], 4)
        leg["ceiling"] = ceil
    legs["f3-copy"] = leg
    del ins, dst, src
    torch.cuda.empty_cache()
    # C1: host buffers through the drop-in entry point
    n = 131072
    rng = np.random.default_rng(0xC1)
    a = (rng.random(n, dtype=np.float32) * 2 - 1)
    b0 = (rng.random(n, dtype=np.float32) * 2 - 1)
    shim = _lib.shim()
    exp = b0 + a  # IEEE RNE fp32 add, no NaNs in these inputs

    def c1_times(sched_mode):
        # sched_mode 1: a schedule without a stream, as nreduce's reduce
        # entries pass it in a CPU oneCCL build (host memory, no lookup);
        # 0: no schedule (operands looked up)
        prev = shim.mi_ccl_comp_shim_sched(sched_mode)
        try:
            b = b0.copy()
            tt = []
            for _ in range(200):
                t0 = time.perf_counter()
                _lib.check_shim(shim.mi_ccl_comp_reduce(a.ctypes.data, n, b.ctypes.data, None, 9, 0),
                                "ccl_comp_reduce")
                tt.append(time.perf_counter() - t0)
            b = b0.copy()
            _lib.check_shim(shim.mi_ccl_comp_reduce(a.ctypes.data, n, b.ctypes.data, None, 9, 0), "ccl_comp_reduce")
        finally:
            shim.mi_ccl_comp_shim_sched(prev)
        return tt, int(np.count_nonzero(b.view(np.uint32) != exp.view(np.uint32)))

    tt, mism = c1_times(1)
    tt0, mism0 = c1_times(0)
    legs["c1"] = {"workload": "512 KiB fp32 sum chunk (nreduce of a 2-rank 1 MiB allreduce), host buffers through "
                              "ccl_comp_reduce under a schedule without a stream (how a CPU oneCCL build's reduce "
                              "entries call it: the calling thread's CPU, nothing looked up); timed from Python "
                              "(ctypes call included)",
                  "median_us": round(statistics.median(tt) * 1e6, 2), "best_us": round(min(tt) * 1e6, 2),
                  "no_schedule_median_us": round(statistics.median(tt0) * 1e6, 2),
                  "parity": {"elements": 2 * n, "mismatches": mism + mism0}}
    return legs


def max_over_ranks(vals, world, device):
    """Max of each value over all ranks (the driver's contract: the slowest
    rank's time is the job's time)."""
    if world <= 1:
        return list(vals)
    import torch
    import torch.distributed as dist
    t = torch.tensor(vals, dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.tolist()


def sum_over_ranks(vals, world, device):
    """Sum of each value over all ranks (parity counts)."""
    if world <= 1:
        return list(vals)
    import torch
    import torch.distributed as dist
    t = torch.tensor(vals, dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.tolist()


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_plan(n, argv, port, base_env=None):
    """(argv, env) of each of the n rank processes `bench.py --gpus n`
    starts by itself when no launcher set WORLD_SIZE: the same script and
    arguments, one rank per GPU, rendezvous on 127.0.0.1."""
    env0 = dict(os.environ if base_env is None else base_env)
    plans = []
    for r in range(n):
        env = dict(env0, WORLD_SIZE=str(n), RANK=str(r), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        plans.append(([sys.executable, str(Path(__file__).resolve())] + list(argv), env))
    return plans


def launch_ranks(plans, timeout=None):
    """Start every rank as a child process (never exec: the parent has made
    no GPU call and makes none), relay rank 0's JSON line, and return the
    exit code: 0 if every rank exited 0, else the first failing rank's code
    (non-zero).  When one rank fails the others are stopped by PID, so a
    rank left waiting in a barrier cannot hang the job."""
    import subprocess
    procs = []
    for r, (argv, env) in enumerate(plans):
        procs.append(subprocess.Popen(argv, env=env, stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL,
                                      text=True))
    out0 = []

    def pump():
        for line in procs[0].stdout:
            out0.append(line)

    import threading
    th = threading.Thread(target=pump, daemon=True)
    th.start()
    t_end = None if timeout is None else time.monotonic() + timeout
    failed = 0
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad and not failed:
            failed = bad[0]
            for p in procs:
                if p.poll() is None:
                    p.terminate()
        if all(c is not None for c in codes):
            break
        if t_end is not None and time.monotonic() > t_end:
            for p in procs:
                if p.poll() is None:
                    p.kill()
            failed = failed or 124
        time.sleep(0.05)
    th.join(timeout=10)
    for line in out0:
        sys.stdout.write(line)
    sys.stdout.flush()
    if failed:
        log(f"bench: a rank failed (exit {failed}); codes {[p.returncode for p in procs]}")
    return failed if failed >= 0 else 128 - failed  # killed by signal s -> 128 + s


class StdoutToStderr:
    """File descriptor 1 points at stderr inside the block: native libraries
    (gloo prints its rendezvous notes with printf) and stray prints cannot
    put lines before the one JSON line the driver parses, which goes to the
    real stdout through write_line."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)
        return self

    def write_line(self, text):
        sys.stdout.flush()
        data = (text + "\n").encode()
        while data:
            data = data[os.write(self.saved, data):]

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)
        return False


def device_identity(index):
    """A physical device's identity: PCI domain:bus:device and UUID (ranks on
    one GPU share it).  Should the runtime report neither, the identity falls
    back to the visible device index within this node's visible set, so
    ranks on different GPUs never merge into one device."""
    import torch
    p = torch.cuda.get_device_properties(index)
    ids = [getattr(p, a, -1) for a in ("pci_domain_id", "pci_bus_id", "pci_device_id")]
    uuid = str(getattr(p, "uuid", "") or "")
    if all(v in (-1, 0) for v in ids) and uuid.strip("0-") == "":
        return f"visible:{os.environ.get('HIP_VISIBLE_DEVICES', os.environ.get('CUDA_VISIBLE_DEVICES', '*'))}:{index}"
    return ":".join(f"{v:x}" for v in ids) + f"/{uuid}"


def device_plan(idents):
    """From every rank's device identity: (distinct devices, max ranks on one
    device, rehearsal?).  A shared device makes the N-rank line a rehearsal:
    n_gpus counts devices, not ranks, and the aggregate peak is theirs."""
    from collections import Counter
    c = Counter(idents)
    return len(c), max(c.values()), len(c) < len(idents)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `python bench.py --gpus N` with no launcher: become the launcher.
        # torch.cuda.device_count() does not initialise the GPU on this image.
        import torch
        argv = sys.argv[1:]
        ndev = torch.cuda.device_count()
        if args.dist_backend == "nccl" and ndev < args.gpus:
            # RCCL takes one rank per GPU: with fewer GPUs than ranks this can
            # only be a rehearsal of the N-rank path, ranks sharing GPUs over a
            # gloo group; the line says so ("rehearsal": true, n_gpus = the
            # distinct devices, peak = those devices' HBM)
            log(f"note: {args.gpus} ranks but {ndev} visible GPU(s): a REHEARSAL, ranks share GPUs over gloo")
            argv += ["--dist-backend", "gloo"]
        sys.exit(launch_ranks(rank_plan(args.gpus, argv, free_port())))
    # stdout carries the one JSON line and nothing else: whatever the
    # libraries write to file descriptor 1 from here on (gloo's rendezvous
    # notes, runtime messages) goes to stderr, the line to the saved stdout
    line_out = StdoutToStderr().__enter__()
    import torch
    import torch.distributed as dist

    from oneccl_amd import _lib

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    ndev = torch.cuda.device_count()
    torch.cuda.set_device(local_rank % max(ndev, 1))
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group("gloo")
    coll_dev = "cuda" if args.dist_backend == "nccl" else "cpu"
    # a gloo group for the ranks that wait while rank 0 times the host cores:
    # they block in a socket read, where an RCCL barrier's stream wait could
    # poll on the CPUs the baseline is measuring
    idle_pg = dist.new_group(backend="gloo") if world > 1 and args.dist_backend == "nccl" else None
    pg_world = dist.get_world_size() if world > 1 else 1  # the ranks the process group saw
    ident = device_identity(torch.cuda.current_device())
    idents = [ident]
    if world > 1:
        idents = [None] * pg_world
        dist.all_gather_object(idents, ident)
    n_devices, ranks_per_device, rehearsal = device_plan(idents)
    pids = [os.getpid()]  # every rank's process: rank 0 keeps them off its timing cores (cpu_baseline)
    if world > 1:
        pids = [None] * pg_world
        dist.all_gather_object(pids, os.getpid())

    cfg = CONFIGS[args.config]
    desc, dt, es, op, k, bucket, flags = cfg
    n_total = bucket // es
    n, _, total_bytes = plan(n_total, es, rank, world, args.scaling)

    m = _lib.mi()
    tdt = torch_dtype(dt)
    if args.config == "c4-tmpbuf":  # reduce_buf + one tmp buffer holding the k-1 peer chunks
        ins = alloc_tmpbuf(k, n, tdt)
    else:
        ins = alloc_inputs(k, n, tdt, args.layout)
    for j in range(len(ins)):  # (no loop variable left holding a view: `del ins` frees the bucket)
        fill(ins[j], 0xC0FFEE + 7919 * rank + j)
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream
    arr = _lib.void_ptr_array([t.data_ptr() for t in ins])

    def step():
        if k == 2:
            return m.mi_reduce(ins[1].data_ptr(), ins[0].data_ptr(), n, dt, op, flags, sh)  # inout += in
        return m.mi_reduce_multi(arr, k, ins[0].data_ptr(), n, dt, op, flags, sh)

    mem_mark("inputs")
    elapsed, avg_kern_ms, kern_ms = timed_steps(step, args.steps, args.warmup, stream, world)
    elapsed, avg_kern_ms_max = max_over_ranks([elapsed, avg_kern_ms], world, coll_dev)
    mem_mark("timed")
    # the achievable ceiling on these buffers (outside the timed region;
    # overwrites ins[0], which full_parity refills)
    ceil = measured_ceiling(ins, k, n * es, stream)
    mem_mark("ceiling")

    # the whole bucket checked bit for bit, outside the timed region (every
    # rank checks its own; the line reports the sum over ranks)
    seed0 = 0x5EED + 7919 * rank
    parity = full_parity(lambda: _lib.check(step(), "mi_reduce"), ins, k, dt, op, flags, seed0,
                         "mi_reduce" if k == 2 else "mi_reduce_multi")

    units_per_rank = n * es  # bucket bytes this rank reduced per step
    value = total_bytes * args.steps / elapsed / GiB
    traffic_per_launch = (k + 1) * n * es  # read k inputs, write 1 (algorithmic)
    achieved = traffic_per_launch / (avg_kern_ms / 1e3) / 1e9
    # whole job: all ranks' launch bytes over the slowest rank's launch time,
    # against world x one HBM (north star: fraction of aggregate HBM roofline)
    agg_achieved = (k + 1) * total_bytes / (avg_kern_ms_max / 1e3) / 1e9
    agg_peak = HBM_PEAK_GBPS * n_devices  # the distinct devices' HBM, not ranks x one HBM

    # the same bucket through oneCCL's own entry point: ccl_comp_reduce of the
    # drop-in shim (synchronous, as src/sched calls it) — reported beside `value`
    dropin = None
    if k == 2:
        shim = _lib.shim()
        torch.cuda.synchronize()
        tt = []
        for _ in range(max(3, min(10, args.steps))):
            t0 = time.perf_counter()
            rc = shim.mi_ccl_comp_reduce(ins[1].data_ptr(), n, ins[0].data_ptr(), None, dt, op)
            tt.append(time.perf_counter() - t0)
            _lib.check_shim(rc, "ccl_comp_reduce")
        dropin = {"value": round(n * es / GiB / statistics.median(tt), 2), "unit": "GiB/s",
                  "best": round(n * es / GiB / min(tt), 2), "calls": len(tt),
                  "entry": "ccl_comp_reduce (libccl_comp_hip.so, synchronous, oneCCL's C++ signature)"}
        from oneccl_amd import comp as _comp
        if dt == 8 and _comp.impl_types()[1] < 2:  # no fp16 impl: the reference computes nothing
            dropin["parity"] = {"elements": 0, "mismatches": 0, "note": "fp16 impl computes nothing on this host"}
        else:
            dropin["parity"] = full_parity(
                lambda: _lib.check_shim(shim.mi_ccl_comp_reduce(ins[1].data_ptr(), n, ins[0].data_ptr(), None, dt,
                                                                op), "ccl_comp_reduce"),
                ins, k, dt, op, shim_flags(dt), seed0 + 101, "ccl_comp_reduce")
    mem_mark("parity + drop-in")

    # totals over ranks (each rank checked its own bucket shard)
    parity["elements"], parity["mismatches"] = (int(x) for x in sum_over_ranks(
        [parity["elements"], parity["mismatches"]], world, coll_dev))
    if dropin:
        dp = dropin["parity"]
        dp["elements"], dp["mismatches"] = (int(x) for x in sum_over_ranks(
            [dp["elements"], dp["mismatches"]], world, coll_dev))

    host_leg = None
    if rank == 0 and world == 1 and not args.no_host_leg and k == 2:
        host_leg = host_resident_leg(m, dt, es, op, flags, min(n, (256 << 20) // es))

    cpu = None
    if world > 1:
        dist.barrier()  # every rank is past its timed region before rank 0 loads the host cores
    if rank == 0 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(cfg, args.cpu_seconds, pids)
        except Exception as e:  # noqa: BLE001 - a reported baseline never costs the line
            cpu = {"error": f"{type(e).__name__}: {e}"}
            log(f"cpu_baseline failed: {cpu['error']}")
        if world > 1 and "error" not in cpu:
            cpu["note_n_gpus"] = (f"measured on rank 0 after the {world}-rank timed region and a barrier, while the "
                                  "other ranks wait in a gloo barrier; the same bounded sample as at N=1")
    if world > 1:
        dist.barrier(group=idle_pg)  # the other ranks wait here, off the CPUs, until rank 0 is done

    legs = None
    if rank == 0 and world == 1 and args.config == "c2" and not args.no_config_legs:
        legs = config_legs(m, stream, args.layout)

    # BASELINE configs[3] as written at N > 1: one 1 GiB bucket split over the
    # GPUs, beside the weak-scaling `value` (each GPU its own 1 GiB bucket):
    # the 2-input headline bucket and the 8-input fan-in
    strong = None
    if world > 1 and args.config == "c2":
        strong = {"c2": strong_split(m, dt, es, op, k, flags, n_total, rank, world, stream, args.steps,
                                     args.warmup, coll_dev, ins=ins, n_devices=n_devices)}
        mem_mark("strong c2")
        del ins
        torch.cuda.empty_cache()
        mem_mark("headline freed")
        strong["c4_fanin8"] = strong_split(m, 9, 4, 0, 8, 0, GiB // 4, rank, world, stream, args.steps,
                                           args.warmup, coll_dev, n_devices=n_devices, layout=args.layout)
        torch.cuda.empty_cache()
        mem_mark("strong c4")

    traffic = pmc_traffic(args.config, traffic_per_launch)
    mplan = memory_plan(args.config, args.layout, world, rank, args.scaling)
    peak_dev = torch.cuda.max_memory_allocated()
    if world > 1:
        mem_max, = max_over_ranks([peak_dev], world, coll_dev)
        mem_sum, = sum_over_ranks([peak_dev], world, coll_dev)
    else:
        mem_max = mem_sum = peak_dev
    if rank == 0:
        out = {
            "metric": "GiB/s device-resident fp32 sum-reduce of 1 GiB bucket; 1/2/4/8 MI355X"
            if args.config == "c2" else f"GiB/s device-resident {args.config} bucket reduce",
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": n_devices,
            "ranks": pg_world,
            "ranks_per_device": ranks_per_device,
            "devices": sorted(set(idents)),
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": DTYPE_LABEL.get(dt, str(dt)),
            "data": "synthetic (uniform [-1,1) generated on device)",
            "config": {"workload": desc, "bucket_bytes_per_gpu": units_per_rank, "inputs": k,
                       "layout": TMPBUF_NOTE if args.config == "c4-tmpbuf" else LAYOUT_NOTE[args.layout],
                       "layout_name": "tmpbuf" if args.config == "c4-tmpbuf" else args.layout,
                       "op": ["sum", "prod", "min", "max"][op], "dtype_id": dt, "flags": flags,
                       "parallelism": f"element-range shard x{world}, no collective",
                       "entry": "mi_reduce (include/mi_reduce.h) via ctypes, async on the torch stream"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBPS, 4),
                         "traffic": traffic.get("bytes_per_launch") if traffic else None,
                         "traffic_ratio_to_algorithmic": traffic.get("ratio") if traffic else None,
                         "algorithmic_bytes_per_launch": traffic_per_launch,
                         "avg_kernel_ms": round(avg_kern_ms, 5), "avg_kernel_ms_max_rank": round(avg_kern_ms_max, 5),
                         "kernel_ms_min": round(min(kern_ms), 5),
                         "kernel_ms_probe": [round(x, 5) for x in kern_ms],
                         "aggregate": {"achieved": round(agg_achieved, 1), "peak": agg_peak,
                                       "frac": round(agg_achieved / agg_peak, 4), "devices": n_devices,
                                       "note": "all ranks' algorithmic launch bytes / max-over-ranks mean launch "
                                               "time, against the distinct devices' HBM"},
                         "timing": "one hipEvent pair on the launch stream around the K back-to-back timed launches "
                                   "(avg_kernel_ms = that time / K, inter-launch gaps included); kernel_ms_min/_probe: "
                                   "10 launches each between their own event pair, after the timed region",
                         "traffic_source": traffic.get("source") if traffic else None},
            "cpu_baseline": cpu,
            "parity": parity,
        }
        if ceil:
            out["roofline"]["ceiling_TBps"] = ceil["ceiling_TBps"]
            out["roofline"]["frac_of_ceiling"] = round(achieved / 1e3 / ceil["ceiling_TBps"], 4)
            if "mixed_TBps" in ceil:
                out["roofline"]["ceiling_mixed_TBps"] = ceil["mixed_TBps"]
                out["roofline"]["frac_of_mixed_ceiling"] = round(achieved / 1e3 / ceil["mixed_TBps"], 4)
            out["roofline"]["ceiling"] = ceil
        if legs and args.config == "c2":
            # the same kernel and bucket where a caller's operands land: the
            # headline's placement, separate allocations (what recv_reduce_entry
            # hands over: the schedule's comm_buf and the user's buffer) and
            # one allocation's consecutive slices; all in this run
            pl = {args.layout: round(achieved / HBM_PEAK_GBPS, 4)}
            for x in LAYOUTS:
                if f"c2-layout-{x}" in legs:
                    pl[x] = legs[f"c2-layout-{x}"]["roofline_frac"]
            out["roofline"]["frac_by_placement"] = pl
            out["roofline"]["placement_note"] = (
                f"headline: {args.layout}; 'separate' (one allocation per operand) is the placement oneCCL's "
                "recv_reduce_entry produces (comm_buf from the schedule's buffer, inout the user's), DESIGN.md §6")
        out["memory"] = {"planned_peak_bytes_rank0": mplan["peak_bytes"],
                         "torch_max_allocated_bytes_max_rank": int(mem_max),
                         "torch_max_allocated_bytes_sum_ranks": int(mem_sum),
                         "note": "planned = memory_plan() (bench.py, computed without a GPU); measured = "
                                 "torch.cuda.max_memory_allocated() per rank (the config legs' buffers included at "
                                 "N = 1)"}
        out["wall_s_rank0"] = round(time.perf_counter() - T0, 2)
        if rehearsal:
            out["rehearsal"] = True
            out["rehearsal_note"] = (f"{pg_world} ranks on {n_devices} device(s): a rehearsal of the N-rank path, "
                                     "not an N-GPU measurement (ranks share a GPU's HBM)")
        if strong:
            out["strong_split"] = strong
        if dropin:
            out["dropin_sync"] = dropin
        if host_leg:
            out["host_resident"] = host_leg
        if legs:
            out["configs"] = legs
        detail = write_detail(out, args.detail)
        line_out.write_line(json.dumps(compact_line(out, detail), separators=(",", ":")))
    if world > 1:
        dist.destroy_process_group()
    bad = parity["mismatches"] + (dropin["parity"]["mismatches"] if dropin else 0)
    bad += sum(v["parity"]["mismatches"] for v in (legs or {}).values())
    if bad:
        log(f"PARITY FAILURE: {bad} element(s) differ from the expected result")
        sys.exit(3)


def _host_pair(kind, nbytes):
    """Two host buffers of `kind` ("pinned" or pageable), every byte 0x3F:
    0.747 as fp32 (0.746 as bf16), so neither the CPU nor the GPU side meets
    denormals.  (torch.empty's pinned pages held whatever was there before;
    garbage fp32 denormals slowed the CPU head of the split 2.5x in one run.)"""
    import numpy as np
    import torch
    if kind.startswith("pinned"):
        a = torch.full((nbytes,), 0x3F, dtype=torch.uint8).pin_memory()
        b = torch.full((nbytes,), 0x3F, dtype=torch.uint8).pin_memory()
        return a, b, a.data_ptr(), b.data_ptr()
    a = np.full(nbytes, 0x3F, np.uint8)
    b = np.full(nbytes, 0x3F, np.uint8)
    return a, b, a.ctypes.data, b.ctypes.data


def gpu_numa_node(index=None):
    """NUMA node of the GPU's PCI device (sysfs), or None."""
    import torch
    p = torch.cuda.get_device_properties(torch.cuda.current_device() if index is None else index)
    dom, bus, dev = (getattr(p, a, -1) for a in ("pci_domain_id", "pci_bus_id", "pci_device_id"))
    if min(dom, bus, dev) < 0:
        return None
    try:
        node = int(Path(f"/sys/bus/pci/devices/{dom:04x}:{bus:02x}:{dev:02x}.0/numa_node").read_text())
    except (OSError, ValueError):
        return None
    return node if node >= 0 else None


def host_leg_cpu():
    """The core the host leg's calling thread runs on, as oneCCL pins each
    worker to one core (CCL_WORKER_AFFINITY, src/exec/thread/worker.cpp:
    310-379): the first allowed physical core of the GPU's NUMA node (else
    of the node core_plan picks), so the buffers it allocates and first
    touches are local to the GPU's PCIe link; MI_BENCH_HOST_LEG_CPU=c picks
    core c.  Off by default (MI_BENCH_HOST_LEG_PIN=1 turns it on): on two
    boxes pinned and unpinned each won the split once (47 against 37 GiB/s
    and the reverse, profiles/round5_run12/), so the default measures as
    rounds 1-4 did.  None: unpinned."""
    if os.environ.get("MI_BENCH_HOST_LEG_PIN", "0") == "0":
        return None
    aff = set(os.sched_getaffinity(0))
    if os.environ.get("MI_BENCH_HOST_LEG_CPU"):
        c = int(os.environ["MI_BENCH_HOST_LEG_CPU"])
        return c if c in aff else None
    node = gpu_numa_node()
    if node is not None:
        try:
            cpus = sorted(set(_cpulist(Path(f"/sys/devices/system/node/node{node}/cpulist").read_text())) & aff)
        except (OSError, ValueError):
            cpus = []
        if cpus:
            return cpus[0]
    _, cores, _, _ = core_plan()
    return cores[0] if cores else None


def host_resident_leg(m, dt, es, op, flags, n):
    """The path as oneCCL runs it (host staging buffers in, host result out):
    mi_reduce_sync with pinned and with pageable host buffers.  Reported
    beside `value`, never as it (PCIe-inclusive rate).  The
    calling thread is pinned to one core local to the GPU (host_leg_cpu) for
    the leg, as oneCCL's workers are, and allocates its buffers there."""
    cpu = host_leg_cpu()
    prev = os.sched_getaffinity(0)
    if cpu is not None:
        os.sched_setaffinity(0, {cpu})
    try:
        res = _host_resident_leg(m, dt, es, op, flags, n)
    finally:
        os.sched_setaffinity(0, prev)
    if "error" not in res:
        res["calling_thread_cpu"] = cpu
        res["gpu_numa_node"] = gpu_numa_node()
    return res


def _host_resident_leg(m, dt, es, op, flags, n):
    import torch
    res = {}
    nbytes = n * es
    reg_s = None
    for kind in ("pinned", "pinned_staged", "pageable", "pageable_registered"):
        m.mi_set_host_mode(1 if kind == "pinned_staged" else 0)
        a, b, pa, pb = _host_pair(kind, nbytes)
        if kind == "pageable_registered":  # what oneCCL's buffer cache would do once per buffer
            t0 = time.perf_counter()
            m.mi_host_register(pa, nbytes)
            m.mi_host_register(pb, nbytes)
            reg_s = time.perf_counter() - t0
        m.mi_reduce_sync(pa, pb, n, dt, op, flags, -1)  # warm: staging buffers, page faults
        times = []
        for _ in range(5):
            t0 = time.perf_counter()
            rc = m.mi_reduce_sync(pa, pb, n, dt, op, flags, -1)
            times.append(time.perf_counter() - t0)
            if rc:
                return {"error": m.mi_last_error().decode()}
        res[kind] = round(nbytes / GiB / min(times), 3)
        if kind == "pageable_registered":
            m.mi_host_unregister(pa)
            m.mi_host_unregister(pb)
    m.mi_set_host_mode(0)
    res["register_ms_two_buffers"] = round(reg_s * 1e3, 2) if reg_s is not None else None
    # the same bucket through oneCCL's entry point with the dispatcher's
    # defaults: above its threshold the GPU reduces the tail while the
    # calling thread reduces the head
    from oneccl_amd import _lib
    shim = _lib.shim()
    for kind in ("pinned", "pageable"):
        a, b, pa, pb = _host_pair(kind, nbytes)
        shim.mi_ccl_comp_reduce(pa, n, pb, None, dt, op)
        times = []
        for _ in range(5):
            t0 = time.perf_counter()
            rc = shim.mi_ccl_comp_reduce(pa, n, pb, None, dt, op)
            times.append(time.perf_counter() - t0)
            if rc:
                return {"error": shim.mi_ccl_last_error().decode()}
        res[f"dropin_{kind}"] = round(nbytes / GiB / min(times), 3)
    # several GPUs in one node: one pageable bucket split by element range over
    # all of them (mi_reduce_multi_sync_sharded), each shard over its own link.
    # Measured in a child process under a time limit: an extra leg never
    # breaks or stalls the bench line.
    if torch.cuda.device_count() > 1:
        import subprocess
        try:
            r = subprocess.run([sys.executable, str(Path(__file__).resolve()), "--host-shard-probe", str(n), str(dt),
                                str(es), str(op), str(flags)], capture_output=True, text=True, timeout=180)
            res["pageable_all_gpus"] = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else {
                "error": r.stderr[-300:]}
        except Exception as e:  # noqa: BLE001
            res["pageable_all_gpus"] = {"error": str(e)}
    return {"unit": "GiB/s bucket incl. both operands host->GPU and the result GPU->host over PCIe",
            "bucket_bytes": nbytes, **res, "entry": "mi_reduce_sync",
            "modes": "pinned = zero-copy kernel on pinned host memory (default); pinned_staged = chunked "
                     "H2D/kernel/D2H over two streams; pageable = staged; pageable_registered = pageable buffers "
                     "registered once with mi_host_register (cost in register_ms_two_buffers), then zero-copy; "
                     "dropin_* = ccl_comp_reduce with the dispatcher's defaults (GPU tail + calling-thread "
                     "CPU head above 16 MiB)"}


def host_shard_probe(n, dt, es, op, flags):
    """Child-process leg: a pageable bucket of n elements per GPU, split over
    every GPU of the node by mi_reduce_multi_sync_sharded; prints one JSON."""
    import ctypes

    import numpy as np
    import torch

    from oneccl_amd import _lib
    m = _lib.mi()
    ndev = torch.cuda.device_count()
    nn = n * ndev
    a = np.zeros(nn * es, np.uint8)
    b = np.zeros(nn * es, np.uint8)
    arr = _lib.void_ptr_array([b.ctypes.data, a.ctypes.data])
    devs = (ctypes.c_int * ndev)(*range(ndev))
    times = []
    for i in range(4):
        t0 = time.perf_counter()
        _lib.check(m.mi_reduce_multi_sync_sharded(arr, 2, b.ctypes.data, nn, dt, op, flags, ndev, devs))
        if i:
            times.append(time.perf_counter() - t0)
    print(json.dumps({"value": round(nn * es / GiB / min(times), 3), "unit": "GiB/s", "gpus": ndev,
                      "bucket_bytes": nn * es, "entry": "mi_reduce_multi_sync_sharded"}), flush=True)


KERNEL_LIB = "oneccl_amd/lib/libmi_reduce.so"


def kernel_identity():
    """sha256 (16 hex digits) of the device code a PMC pass measured: the
    `.hip_fatbin` section of the built library (the gfx950 code object of
    every kernel, block sizes included as template arguments), so host-side
    edits to mi_reduce.hip leave a pass current and any kernel change does
    not.  tools/pmc_traffic.py stores it with the pass, pmc_traffic() matches
    it.  None when the library is not built."""
    import hashlib
    import struct
    try:
        b = (ROOT / KERNEL_LIB).read_bytes()
    except OSError:
        return None
    shoff, = struct.unpack_from("<Q", b, 0x28)  # ELF64 section header table
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", b, 0x3A)

    def section(i):  # sh_name, sh_offset, sh_size
        name, _, _, _, off, size = struct.unpack_from("<IIQQQQ", b, shoff + i * shentsize)
        return name, off, size
    stroff = section(shstrndx)[1]
    for i in range(shnum):
        name, off, size = section(i)
        if b[stroff + name:b.index(b"\0", stroff + name)] == b".hip_fatbin":
            return "fatbin:" + hashlib.sha256(b[off:off + size]).hexdigest()[:16]
    return None


def pmc_passes(config):
    """Every committed PMC pass for `config` under profiles/ (any depth):
    [(path, entry)] with the entry's recorded identity and time, if any."""
    found = []
    for p in (ROOT / "profiles").rglob("*pmc*.json"):
        try:
            d = json.loads(p.read_text())
        except (OSError, ValueError):
            continue
        e = d.get(config) if isinstance(d, dict) else None
        if isinstance(e, dict) and "hbm_bytes_per_launch" in e and e.get("algorithmic_bytes_per_launch"):
            found.append((p, e))
    return found


def pmc_traffic(config, algo_bytes):
    """HBM bytes per launch from a committed rocprofv3 PMC pass (produced by
    tools/pmc_traffic.py).  The pass chosen is the one recorded against the
    device code of this tree's build (kernel_identity); failing that, the
    most recently recorded one, marked stale.  The pass is a 1-GPU full-bucket
    run; a launch of another size (a strong-scaling shard) gets the measured
    ratio to algorithmic bytes applied to its own algorithmic bytes."""
    passes = pmc_passes(config)
    if not passes:
        return None
    ident = kernel_identity()
    current = [pe for pe in passes if ident and pe[1].get("kernel_code") == ident]
    pool = current or passes
    p, e = max(pool, key=lambda pe: (pe[1].get("recorded_utc", ""), str(pe[0])))
    pmc_algo = e["algorithmic_bytes_per_launch"]
    ratio = e["hbm_bytes_per_launch"] / pmc_algo
    src = str(p.relative_to(ROOT))
    src += " (device code matches this build)" if current else " (STALE: recorded against other device code)"
    if pmc_algo != algo_bytes:
        src += f" (ratio {ratio:.6f} of a {pmc_algo}-B launch, applied to this {algo_bytes}-B launch)"
    return {"bytes_per_launch": int(round(ratio * algo_bytes)), "ratio": round(ratio, 6), "source": src,
            "current": bool(current)}

if __name__ == "__main__":
    if len(sys.argv) == 7 and sys.argv[1] == "--host-shard-probe":
        host_shard_probe(*(int(x) for x in sys.argv[2:]))
    else:
        main()
