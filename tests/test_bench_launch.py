"""bench.py as its own launcher (CPU): `python bench.py --gpus N` with no
WORLD_SIZE starts N rank processes, relays rank 0's JSON line, and exits
non-zero when any rank fails.  Also the full-bucket parity checker's
expected-result fold and the helper-thread CPU set (no GPU needed)."""
from __future__ import annotations

import json
import os
import subprocess
import sys
import textwrap
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402
GIB = 1 << 30


def test_rank_plan_env():
    plans = bench.rank_plan(4, ["--gpus", "4", "--steps", "3"], 29555, base_env={"KEEP": "1"})
    assert len(plans) == 4
    for r, (argv, env) in enumerate(plans):
        assert argv[0] == sys.executable and argv[1].endswith("bench.py")
        assert argv[2:] == ["--gpus", "4", "--steps", "3"]
        assert env["RANK"] == env["LOCAL_RANK"] == str(r)
        assert env["WORLD_SIZE"] == env["LOCAL_WORLD_SIZE"] == "4"
        assert env["MASTER_ADDR"] == "127.0.0.1" and env["MASTER_PORT"] == "29555"
        assert env["KEEP"] == "1"


def _fake(code: str):
    """A fake rank: python -c <code> with the planned env."""
    return [sys.executable, "-c", textwrap.dedent(code)]


def test_launch_relays_rank0_line(capfd):
    code = """
    import json, os
    r = int(os.environ["RANK"])
    if r == 0:
        print(json.dumps({"metric": "m", "n_gpus": int(os.environ["WORLD_SIZE"])}), flush=True)
    """
    plans = [(_fake(code), env) for _, env in bench.rank_plan(3, [], 1, base_env={})]
    rc = bench.launch_ranks(plans, timeout=60)
    out = capfd.readouterr().out.strip().splitlines()
    assert rc == 0
    assert json.loads(out[-1]) == {"metric": "m", "n_gpus": 3}


def test_launch_fails_when_a_rank_fails_and_stops_the_rest(capfd):
    code = """
    import os, sys, time
    r = int(os.environ["RANK"])
    if r == 1:
        sys.exit(7)
    time.sleep(60)          # a rank left waiting (e.g. in a barrier)
    """
    plans = [(_fake(code), env) for _, env in bench.rank_plan(3, [], 1, base_env={})]
    import time
    t0 = time.monotonic()
    rc = bench.launch_ranks(plans, timeout=120)
    assert rc == 7
    assert time.monotonic() - t0 < 30  # the waiting ranks were stopped, not waited for


def test_launch_times_out():
    plans = [(_fake("import time; time.sleep(60)"), env) for _, env in bench.rank_plan(2, [], 1, base_env={})]
    assert bench.launch_ranks(plans, timeout=1) != 0


def test_launch_killed_rank_maps_to_128_plus_signal():
    code = """
    import os, signal
    if os.environ["RANK"] == "1":
        os.kill(os.getpid(), signal.SIGKILL)
    """
    plans = [(_fake(code), env) for _, env in bench.rank_plan(2, [], 1, base_env={})]
    assert bench.launch_ranks(plans, timeout=60) == 128 + 9


def test_bench_gpus2_without_launcher_runs_two_ranks_on_cpu_box():
    """The real script: --gpus 2 with no WORLD_SIZE re-launches itself as two
    ranks.  Without a GPU each rank fails at its first device call, so the
    job must exit non-zero (and not report a 1-rank line)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0",
                        "--no-cpu-baseline", "--no-host-leg"], capture_output=True, text=True, timeout=300, env=env)
    if r.returncode == 0:  # a GPU box: a 2-rank line
        line = json.loads(r.stdout.strip().splitlines()[-1])
        assert line["n_gpus"] == 2
    else:
        assert "metric" not in r.stdout
        assert "ranks share GPUs" in r.stderr or "a rank failed" in r.stderr


def test_expected_result_fold_matches_oracle():
    """The bench's on-device checker (torch ops) folds in the reference's
    order and rounds like it: checked here on CPU tensors against the oracle
    (the restatement of src/comp), for every config the bench runs."""
    import numpy as np
    import torch

    import oracle
    rng = np.random.default_rng(3)
    n = 4099
    for name, (desc, dt, es, op, k, bucket, flags) in bench.CONFIGS.items():
        if dt == 9:
            ins = [rng.standard_normal(n).astype(np.float32) for _ in range(k)]
        elif dt in (4, 6):
            ins = [rng.integers(-1000, 1000, n).astype(oracle.NP_DTYPE[dt]) for _ in range(k)]
        else:
            f = [rng.standard_normal(n).astype(np.float32) for _ in range(k)]
            ins = [oracle.f32_to_bf16(x, True) if dt == 11 else oracle.f32_to_fp16(x) for x in f]
        tdt = bench.torch_dtype(dt)
        view = {2: torch.int16, 4: torch.int32, 8: torch.int64}[es]
        tins = [torch.from_numpy(x.copy()).view(view).view(tdt) if dt in (8, 11) else torch.from_numpy(x.copy())
                for x in ins]
        got = bench.expected_result(tins, k, dt, op, flags)
        if flags & 0x4:  # keep-precision: fp32 accumulate, one rounding (ccl_comp_batch_reduce)
            exp = oracle.lp_fanin_acc_fp32(ins, dt, op, bool(flags & 0x2), bool(flags & 0x1))
        else:
            exp = oracle.fanin(ins, dt, op, oracle.BF16_AVX512BF if flags & 0x2 else oracle.BF16_SCALAR,
                               oracle.FP16_AVX512F)
        gb = got.view(view).numpy()
        assert gb.tobytes() == exp.view(gb.dtype).tobytes(), name


def test_bf16_truncation_in_checker():
    """Without F_BF16_RNE (scalar / avx512f impls) the checker truncates."""
    import torch
    acc = torch.tensor([1.0 + 2 ** -8 + 2 ** -10], dtype=torch.float32)  # RNE rounds up, truncation down
    t = bench.to_storage(acc, 11, 0).view(torch.int16).item() & 0xFFFF
    r = bench.to_storage(acc, 11, 0x2).view(torch.int16).item() & 0xFFFF
    assert t == 0x3F80 and r == 0x3F81


def test_helper_threads_take_the_process_cpu_set():
    """libmi_reduce.so loaded from a thread pinned to one core still gives
    its helper threads the process's CPU set."""
    if len(os.sched_getaffinity(0)) < 2:
        pytest.skip("needs 2+ CPUs")
    code = textwrap.dedent("""
        import os, sys, threading
        sys.path.insert(0, sys.argv[1])
        res = {}
        def loader():
            os.sched_setaffinity(0, {min(os.sched_getaffinity(0))})
            from oneccl_amd import _lib
            res["n"] = _lib.mi().mi_helper_cpu_count()
        t = threading.Thread(target=loader); t.start(); t.join()
        print(res["n"], len(os.sched_getaffinity(0)))
    """)
    r = subprocess.run([sys.executable, "-c", code, str(ROOT)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    n, total = (int(x) for x in r.stdout.split())
    assert n == total > 1


@pytest.mark.parametrize("idents,plan", [
    (["0:3:0/u0"], (1, 1, False)),
    (["0:3:0/u0", "0:3:0/u0"], (1, 2, True)),         # the 2-rank rehearsal on one GPU
    ([f"0:{b:x}:0/u{b}" for b in range(8)], (8, 1, False)),  # one rank per GPU of an 8-GPU node
    (["a", "a", "b", "b"], (2, 2, True)),
])
def test_device_plan_counts_devices_not_ranks(idents, plan):
    """n_gpus = distinct physical devices, ranks_per_device,
    and a shared device marks the line a rehearsal."""
    assert bench.device_plan(idents) == plan


_GLOO_PLAN = """
import os, sys
sys.path.insert(0, sys.argv[1])
import torch.distributed as dist
import bench
dist.init_process_group("gloo")
r, w = dist.get_rank(), dist.get_world_size()
ident = "0:3:0/shared" if r < 2 else f"0:{r:x}:0/own{r}"  # ranks 0 and 1 share a device
idents = [None] * w
dist.all_gather_object(idents, ident)
n, per, reh = bench.device_plan(idents)
peak = bench.HBM_PEAK_GBPS * n
if r == 0:
    print(f"PLAN {n} {per} {reh} {peak}", flush=True)
dist.destroy_process_group()
"""


def test_device_plan_over_a_gloo_group(tmp_path):
    """The plan as bench.py forms it at N > 1: every rank's identity gathered
    over the process group (gloo here; RCCL on the node), the same on every
    rank; 3 ranks on 2 devices -> n_gpus 2, 2 ranks per device, peak 16 TB/s."""
    script = tmp_path / "plan.py"
    script.write_text(_GLOO_PLAN)
    plans = bench.rank_plan(3, [], bench.free_port(), base_env=dict(os.environ))
    procs = [subprocess.Popen([sys.executable, str(script), str(ROOT)], env=env, stdout=subprocess.PIPE, text=True)
             for _, env in plans]
    outs = [p.communicate(timeout=120)[0] for p in procs]
    assert all(p.returncode == 0 for p in procs)
    assert "PLAN 2 2 True 16000.0" in outs[0]


def test_device_identity_uses_pci_and_uuid_and_falls_back(monkeypatch):
    """Distinct GPUs must never merge into one device in the N-rank line: PCI
    ids and UUID when the runtime reports them, else the visible index."""
    import types

    import torch
    props = {0: types.SimpleNamespace(pci_domain_id=0, pci_bus_id=0x11, pci_device_id=0, uuid="abc"),
             1: types.SimpleNamespace(pci_domain_id=0, pci_bus_id=0x2f, pci_device_id=0, uuid="def"),
             2: types.SimpleNamespace(pci_domain_id=0, pci_bus_id=0, pci_device_id=0, uuid=""),
             3: types.SimpleNamespace(pci_domain_id=0, pci_bus_id=0, pci_device_id=0, uuid="")}
    monkeypatch.setattr(torch.cuda, "get_device_properties", lambda i: props[i])
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1,2,3")
    ids = [bench.device_identity(i) for i in range(4)]
    assert ids[0] == "0:11:0/abc" and ids[1] == "0:2f:0/def"
    assert ids[2] != ids[3] and ids[2].startswith("visible:")
    assert bench.device_plan(ids) == (4, 1, False)


@pytest.mark.parametrize("layout,k,dtype", [("padded", 2, "float32"), ("padded", 2, "bfloat16"),
                                            ("padded", 8, "float32"), ("one", 2, "float32"),
                                            ("separate", 2, "float32")])
def test_alloc_inputs_layouts(layout, k, dtype):
    """The bench's input layouts: padded starts a 2-input
    config's second operand PAIR_OFFSET after its first in one allocation and
    is contiguous for a fan-in; one is contiguous; separate is an allocation
    each.  Checked on CPU tensors (the bench allocates on the GPU)."""
    import torch
    tdt = getattr(torch, dtype)
    n = 1024
    ins = bench.alloc_inputs(k, n, tdt, layout, device="cpu")
    es = ins[0].element_size()
    assert len(ins) == k and all(t.numel() == n and t.is_contiguous() for t in ins)
    bases = [t.untyped_storage().data_ptr() for t in ins]
    if layout == "separate":
        assert len(set(bases)) == k
        return
    assert len(set(bases)) == 1  # one allocation
    stride = bench.PAIR_OFFSET if layout == "padded" and k == 2 else n * es
    for j in range(1, k):
        assert ins[j].data_ptr() - ins[j - 1].data_ptr() == stride
    # a bucket larger than the offset: the gap past it
    assert bench.pair_stride_bytes(bench.PAIR_OFFSET + 16) == bench.PAIR_OFFSET + 16 + bench.PAIR_GAP
    assert bench.pair_stride_bytes(1 << 30) == bench.PAIR_OFFSET
    assert layout in bench.LAYOUTS and layout in bench.LAYOUT_NOTE


def test_alloc_tmpbuf_is_oneccl_nreduce_layout():
    """c4-tmpbuf: reduce_buf its own allocation, the k - 1
    peer chunks in consecutive slots of one tmp buffer (allreduce.cpp:326-394)."""
    import torch
    k, n = 8, 1000
    ins = bench.alloc_tmpbuf(k, n, torch.float32, device="cpu")
    assert len(ins) == k and all(t.numel() == n for t in ins)
    tmp_base = ins[1].untyped_storage().data_ptr()
    assert ins[0].untyped_storage().data_ptr() != tmp_base
    for j in range(2, k):
        assert ins[j].untyped_storage().data_ptr() == tmp_base
        assert ins[j].data_ptr() - ins[j - 1].data_ptr() == n * 4


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_memory_plan_n8_without_a_gpu(world):
    """the per-rank allocation plan of `bench.py --gpus N`
    (padded pair, then at N > 1 the strong-split C2 shard reusing it and the
    C4 fan-in shard) is computed on the CPU; the strong shards of all ranks
    tile the bucket, and a rehearsal of 8 ranks on one 288 GB GPU fits."""
    plans = [bench.memory_plan("c2", "padded", world, r) for r in range(world)]
    for p in plans:
        assert p["headline_inputs_bytes"] == bench.PAIR_OFFSET + GIB  # weak: a full 1 GiB bucket per rank
        assert p["peak_bytes"] >= p["headline_inputs_bytes"]
    if world > 1:
        assert sum(p["strong_c2_shard_elements"] for p in plans) == GIB // 4
        assert sum(p["strong_c4_shard_elements"] for p in plans) == GIB // 4
        assert all(p["strong_c4_shard_elements"] % 256 == 0 for p in plans[:-1])
        assert all(p["strong_c4_inputs_bytes"] == 8 * 4 * p["strong_c4_shard_elements"] for p in plans)
    else:
        assert "strong_c4_inputs_bytes" not in plans[0]
    # every rank on one GPU (the rehearsal) stays well inside 288 GB
    assert sum(p["peak_bytes"] for p in plans) < 0.5 * 288e9


def test_memory_plan_layouts_and_tmpbuf():
    assert bench.memory_plan("c2", "separate", 1, 0)["headline_inputs_bytes"] == 2 * GIB
    assert bench.memory_plan("c2", "one", 1, 0)["headline_inputs_bytes"] == 2 * GIB
    p = bench.memory_plan("c4-tmpbuf", "padded", 1, 0)
    assert p["layout"] == "tmpbuf" and p["headline_inputs_bytes"] == 8 * GIB
    p = bench.memory_plan("c3-bf16", "padded", 1, 0)
    # fp32 accumulator + one widened input (the fold is in place; RNE rounding: + the storage copy, less)
    assert p["parity_temporaries_bytes"] == (128 << 20) * (4 + 4)
    assert bench.parity_bytes(128 << 20, 11, 2, 0) == (128 << 20) * (4 + 4 + 2)  # truncation: int32 shift too
    p = bench.memory_plan("c2", "padded", 1, 0)  # the accumulator; then result + one chunk's mask and count
    assert p["parity_temporaries_bytes"] == GIB + 9 * bench.PARITY_CHUNK + bench.PARITY_COUNT_SMALL
    # the rehearsals' measured per-rank peaks (N = 2 and N = 8: head + parity)
    for world in (2, 8):
        assert bench.memory_plan("c2", "padded", world, 0)["peak_bytes"] == 4311747584


@pytest.mark.parametrize("dt,flags", [(9, 0), (4, 0), (6, 0), (11, 0), (11, 0x2), (11, 0x6), (8, 0), (8, 0x4)])
@pytest.mark.parametrize("op", [0, 1, 2, 3])
def test_expected_result_in_place_fold_and_chunked_count(dt, flags, op, monkeypatch):
    """bench.expected_result folds in place; its bits equal the out-of-place
    left fold (CPU tensors), and count_mismatches counts in chunks."""
    import torch
    monkeypatch.setattr(bench, "PARITY_CHUNK", 1000)
    n, k = 4099, 4
    g = torch.Generator().manual_seed(dt * 10 + op)
    tdt = bench.torch_dtype(dt)
    if tdt.is_floating_point:
        ins = [(torch.rand(n, generator=g) * 4 - 2).to(tdt) for _ in range(k)]
    else:
        ins = [torch.randint(-50, 50, (n,), generator=g).to(tdt) for _ in range(k)]
    got = bench.expected_result(ins, k, dt, op, flags)
    lp = dt in (8, 11)
    acc = ins[0].float() if lp else ins[0].clone()
    for j in range(1, k):
        x = ins[j].float() if lp else ins[j]
        acc = [acc + x, acc * x, torch.minimum(x, acc), torch.maximum(x, acc)][op]
        if lp and not (flags & 0x4):
            acc = bench.to_storage(acc, dt, flags).float()
    ref = bench.to_storage(acc, dt, flags) if lp else acc
    assert bench.count_mismatches(got, ref) == 0
    bad = ref.clone()
    bad.view(torch.uint8)[::977] ^= 1
    assert bench.count_mismatches(bad, ref) == len(range(0, bad.numel() * bad.element_size(), 977))


def test_core_plan_one_cpu_per_physical_core():
    import os
    node, cores, n_aff, quota = bench.core_plan()
    assert cores and set(cores) <= set(os.sched_getaffinity(0))
    assert len(cores) == len(set(cores)) and n_aff >= len(cores)
    assert quota is None or quota > 0


def test_cpu_sweep_point_pins_and_reduces():
    """A small sample of the threaded baseline: 2 pinned threads, each first-
    touching and reducing its own range; rates are positive and best >= median."""
    import os
    cfg = ("fp32 sum", 9, 4, 0, 2, 8 << 20, 0)
    cpus = sorted(os.sched_getaffinity(0))[:2]
    b, m, r, pin_errors, throttle = bench.cpu_sweep_point(cfg, cpus, 0.2, False)
    assert pin_errors == []
    assert set(throttle) <= {"nr_periods", "nr_throttled", "throttled_usec", "psi_cpu_some_us",
                             "psi_memory_some_us"}
    assert all(v >= 0 for v in throttle.values())
    assert b >= m > 0 and r >= 5


def test_host_leg_cpu_is_allowed_and_local(monkeypatch):
    """The host leg's calling thread goes to an allowed core of the GPU's
    NUMA node (here node 0, or core_plan's node when the GPU's is unknown)
    under MI_BENCH_HOST_LEG_PIN=1; MI_BENCH_HOST_LEG_PIN=0 (the default)
    leaves it unpinned."""
    import os
    aff = set(os.sched_getaffinity(0))
    monkeypatch.setenv("MI_BENCH_HOST_LEG_PIN", "1")
    monkeypatch.setattr(bench, "gpu_numa_node", lambda index=None: 0)
    c = bench.host_leg_cpu()
    assert c is None or c in aff
    monkeypatch.setattr(bench, "gpu_numa_node", lambda index=None: None)
    c = bench.host_leg_cpu()
    assert c in aff
    monkeypatch.setenv("MI_BENCH_HOST_LEG_PIN", "0")
    assert bench.host_leg_cpu() is None


def _canned_full():
    """A real full result: round 5 run 22's 21 KB line (the one shape the
    driver could not parse), with this round's added fields."""
    full = json.loads((ROOT / "profiles" / "round5_run22" / "bench.json").read_text().strip().splitlines()[-1])
    full["config"]["layout_name"] = "padded"
    full["cpu_baseline"]["sample_short"] = "the reference's own CCL_REDUCE, 1 GiB x 2-input bucket, 1 pinned thread"
    return full


def _strong(v):
    return {"value": v, "unit": "GiB/s", "inputs": 2, "ms_per_step": 1.0, "avg_kernel_ms_max_rank": 0.06,
            "aggregate_roofline": {"achieved": 1.0, "peak": 64000.0, "frac": 0.84}, "note": "x" * 200}


@pytest.mark.parametrize("world", [1, 8])
def test_compact_line_is_small_and_parses(world, tmp_path):
    """the stdout line stays one json.loads-clean line
    under LINE_LIMIT (the driver keeps the last 8000 characters), carries
    roofline and cpu_baseline with their numbers, the per-leg fractions and
    mismatches, and names the side file holding the rest."""
    full = _canned_full()
    if world == 8:
        full.update(n_gpus=1, ranks=8, rehearsal=True, rehearsal_note="y" * 200,
                    strong_split={"c2": _strong(2000.0), "c4_fanin8": _strong(600.0)})
        full.pop("configs")
        full.pop("host_resident")
    path = bench.write_detail(full, str(tmp_path / "detail.json"))
    assert json.loads(Path(path).read_text()) == full
    line = bench.compact_line(full, path)
    text = json.dumps(line, separators=(",", ":"))
    assert "\n" not in text and len(text.encode()) <= bench.LINE_LIMIT < 8000
    back = json.loads(text)
    assert "trimmed" not in back
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "parity", "detail"):
        assert k in back, k
    r = back["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "ceiling_TBps", "ceiling_mixed_TBps"):
        assert r[k] == full["roofline"][k], k
    assert "kernel_ms_probe" not in r and "ceiling" not in r
    cb = back["cpu_baseline"]
    assert cb["value"] == full["cpu_baseline"]["value"] and cb["cores"] == 1 and cb["kind"] == "reference"
    assert cb["sample"] and cb["cpu_model"]
    assert {"threads", "value", "median", "spread"} <= set(cb["multi_thread"])
    assert "sweep" not in cb["multi_thread"]
    if world == 1:
        assert r["frac_by_placement"]["separate"] == full["roofline"]["frac_by_placement"]["separate"]
        legs = back["configs"]
        assert set(legs) == set(full["configs"])
        for name, v in legs.items():
            assert v["mismatches"] == 0
            if name != "c1":
                assert {"GiBps", "frac", "frac_of_mixed_ceiling"} <= set(v)
    else:
        assert back["rehearsal"] is True and back["ranks"] == 8
        assert back["strong_split"]["c4_fanin8"]["frac"] == 0.84


def test_compact_line_trims_when_over_limit(monkeypatch):
    """Should a line still exceed the limit, optional sections go first and
    the line says which; the contract keys always stay."""
    monkeypatch.setattr(bench, "LINE_LIMIT", 2500)
    line = bench.compact_line(_canned_full(), "profiles/bench_detail.json")
    assert "configs" in line["trimmed"] and "roofline" in line and "cpu_baseline" in line
    assert len(json.dumps(line, separators=(",", ":"))) <= 2500 + 80


@pytest.mark.parametrize("n_cores,quota,counts", [(64, 16.0, [1, 8, 15]), (64, None, [1, 8, 16, 32, 64]),
                                                  (12, None, [1, 8]), (64, 8.0, [1, 7]), (4, 2.0, [1])])
def test_sweep_counts_leave_quota_headroom(n_cores, quota, counts):
    """under a cgroup CPU quota Q the timing threads stop
    at Q - 1, so the process's other threads do not push it into throttling."""
    got, skipped = bench.sweep_counts(n_cores, quota)
    assert got == counts
    assert not set(got) & set(skipped)


def test_cgroup_cpu_stat_parses(tmp_path):
    f = tmp_path / "cpu.stat"
    f.write_text("usage_usec 100\nnr_periods 7\nnr_throttled 2\nthrottled_usec 3000\n")
    assert bench.cgroup_cpu_stat(str(f)) == {"usage_usec": 100, "nr_periods": 7, "nr_throttled": 2,
                                               "throttled_usec": 3000}
    assert bench.cgroup_cpu_stat(str(tmp_path / "missing")) == {}


def test_compact_line_of_a_real_8_rank_rehearsal():
    """The full result the 8-rank rehearsal wrote as its side file
    (profiles/round6_run2/) gives back the line it printed."""
    full = json.loads((ROOT / "profiles" / "round6_run2" / "bench_gpus8_detail.json").read_text())
    printed = json.loads((ROOT / "profiles" / "round6_run2" / "bench_gpus8_rehearsal.json").read_text()
                         .strip().splitlines()[-1])
    line = bench.compact_line(full, printed["detail"])
    assert line == printed
    assert len(json.dumps(line, separators=(",", ":"))) <= bench.LINE_LIMIT
    assert line["rehearsal"] is True and line["ranks"] == 8 and line["parity"]["mismatches"] == 0


def test_psi_totals_parse(tmp_path):
    (tmp_path / "cpu").write_text("some avg10=0.45 avg60=0.40 avg300=0.17 total=193073552\n"
                                  "full avg10=0.00 avg60=0.00 avg300=0.00 total=0\n")
    (tmp_path / "memory").write_text("some avg10=0.00 avg60=0.00 avg300=0.00 total=12\n")
    assert bench.psi_totals(str(tmp_path)) == {"cpu": 193073552, "memory": 12}
    assert bench.psi_totals(str(tmp_path / "none")) == {}


def test_stdout_to_stderr_moves_native_writes(capfd):
    """Writes to file descriptor 1 inside the block (as gloo's printf) land
    on stderr; stdout keeps only what is written outside it."""
    print("before", flush=True)
    with bench.StdoutToStderr() as line_out:
        os.write(1, b"native note\n")
        line_out.write_line('{"line": 1}')
    print("after", flush=True)
    out, err = capfd.readouterr()
    assert out == 'before\n{"line": 1}\nafter\n'
    assert "native note" in err


def test_gloo_group_notes_stay_off_stdout():
    """Two gloo ranks created under stdout_to_stderr print nothing on stdout
    but what the script prints (the rank-0 line)."""
    code = textwrap.dedent("""
        import os, sys
        sys.path.insert(0, sys.argv[1])
        import torch.distributed as dist
        import bench
        out = bench.StdoutToStderr().__enter__()
        dist.init_process_group("gloo")
        g = dist.new_group(backend="gloo")
        dist.barrier(group=g)
        print("stray", flush=True)
        if dist.get_rank() == 0:
            out.write_line('{"line": 1}')
        dist.destroy_process_group()
    """)
    plans = bench.rank_plan(2, [], bench.free_port(), base_env=dict(os.environ))
    procs = [subprocess.Popen([sys.executable, "-c", code, str(ROOT)], env=env, stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for _, env in plans]
    outs = [p.communicate(timeout=120) for p in procs]
    assert all(p.returncode == 0 for p in procs), [o[1][-500:] for o in outs]
    assert outs[0][0] == '{"line": 1}\n' and outs[1][0] == ""
    assert "stray" in outs[0][1] and "stray" in outs[1][1]


def test_clear_cores_moves_other_threads_and_restores():
    """During a sweep point every thread of the process but the timing ones
    leaves the timing cores, and gets its affinity back afterwards."""
    import threading
    aff = sorted(os.sched_getaffinity(0))
    if len(aff) < 3:
        pytest.skip("needs 3+ CPUs")
    stop = threading.Event()
    seen = {}

    def idle():
        seen["tid"] = threading.get_native_id()
        stop.wait(30)

    t = threading.Thread(target=idle)
    t.start()
    while "tid" not in seen:
        pass
    try:
        cores = {aff[0]}
        moved = bench.clear_cores(cores, keep=set())
        assert seen["tid"] in moved and threading.get_native_id() in moved
        assert not os.sched_getaffinity(seen["tid"]) & cores
        assert not os.sched_getaffinity(0) & cores
        bench.restore_affinity(moved)
        assert os.sched_getaffinity(seen["tid"]) == set(aff) and os.sched_getaffinity(0) == set(aff)
    finally:
        stop.set()
        t.join()


def test_clear_cores_moves_another_process_threads():
    """An N-rank run's other ranks (their pids) leave the timing cores too."""
    aff = sorted(os.sched_getaffinity(0))
    if len(aff) < 3:
        pytest.skip("needs 3+ CPUs")
    p = subprocess.Popen([sys.executable, "-c", "import time; time.sleep(30)"])
    try:
        cores = {aff[-1]}
        moved = bench.clear_cores(cores, keep=set(), pids=[p.pid])
        assert p.pid in moved and not os.sched_getaffinity(p.pid) & cores
        assert os.getpid() not in moved  # only the pids named
        bench.restore_affinity(moved)
        assert os.sched_getaffinity(p.pid) == set(aff)
    finally:
        p.kill()
        p.wait()


def test_compact_line_keeps_a_failed_cpu_baseline_and_no_legs():
    """A CPU baseline that failed is carried as its error, and a line without
    config legs, host leg or strong split (a --no-config-legs run) stays
    well-formed."""
    full = _canned_full()
    full["cpu_baseline"] = {"error": "OSError: no cores"}
    for k in ("configs", "host_resident", "dropin_sync"):
        full.pop(k)
    line = bench.compact_line(full, "profiles/bench_detail.json")
    assert line["cpu_baseline"] == {"error": "OSError: no cores"}
    assert "configs" not in line and "host_resident" not in line and "trimmed" not in line
    assert json.loads(json.dumps(line)) == line
