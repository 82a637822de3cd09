"""The maintainer's patch set (integration/) against the
reference's own sources.

test_intree_build.py proves the drop-in's translation unit in oneCCL's tree.
This test proves the edits around it: each patch in integration/ applies with
no fuzz to the v2021.14 files it names, the new files of integration/src/ are
laid over the tree, and every touched translation unit compiles with oneCCL's
flags (CMakeLists.txt:172-199, 247: -std=gnu++11 -Wall -Wextra -Werror
-faligned-new ...) against the reference's headers and include/ of this repo.
The symbols the patched objects then need from src/comp are all defined by
the drop-in's in-tree object.  Copies go to a temporary directory; the
reference tree is only read.  Runs where /root/reference exists.

  0001  src/CMakeLists.txt        swap three src/comp sources, link libmi_reduce.so  (§2a)
  0002  atl_mpi_ctx.cpp           MPI bf16/fp16 user ops through the host-word entries (§2b)
  0003  reduce_local_entry, recv_reduce_entry: start the reduce, poll it        (§2d)
  0004  allreduce.cpp nreduce + entry_factory.hpp: one fused fan-in per segment (§2e)
  0005  buffer_cache.cpp: the regular buffer cache declares its host buffers     (§2h)
  0006  copy_entry.cpp, recv_copy_entry.cpp: host copies say so (no lookup)      (§2i)
  0007  global.cpp: finalize frees libmi_reduce's pooled per-thread contexts     (§2j)
"""
from __future__ import annotations

import re
import shutil
import subprocess
from pathlib import Path

import pytest

from tests.test_intree_build import DEFS, REF, ROOT, WARN, _global_defs, _undefs

pytestmark = pytest.mark.skipif(not (REF / "src" / "comp").is_dir(),
                                reason="reference tree absent (GPU box): checked in the build container")

PATCHES = sorted((ROOT / "integration").glob("*.patch"))
NEW_FILES = ROOT / "integration" / "src"
INCS_REF = [f"-I{REF}/include", f"-I{REF}/src", f"-I{REF}/src/atl"] + \
           [f"-I{REF}/deps/{d}/include" for d in ("hwloc", "itt", "ofi", "pmix", "mpi", "level_zero")]
# oneCCL's own gcc flags, -faligned-new included (CMakeLists.txt:244-249)
FLAGS = ["-std=gnu++11", "-O2", "-fPIC", "-faligned-new", "-fvisibility=internal", *WARN, *DEFS]
UNITS = {  # translation units the patches touch (headers through their includers)
    "reduce_local_entry": "src/sched/entry/reduce_local_entry.cpp",
    "allreduce": "src/coll/algorithms/allreduce/allreduce.cpp",  # recv_reduce_entry.hpp, entry_factory.hpp
    "atl_mpi_ctx": "src/atl/mpi/atl_mpi_ctx.cpp",
    "buffer_cache": "src/sched/buffer/buffer_cache.cpp",
    "copy_entry": "src/sched/entry/copy/copy_entry.cpp",
    "recv_copy_entry": "src/sched/entry/recv_copy_entry.cpp",
    "global": "src/common/global/global.cpp",
}


def _patched_files(patch: Path) -> list[str]:
    return [m.group(1) for m in re.finditer(r"^\+\+\+ b/(\S+)", patch.read_text(), re.M)]


@pytest.fixture(scope="module")
def tree(tmp_path_factory):
    """A copy of the files the patches touch, patched, with integration/src laid over it."""
    d = tmp_path_factory.mktemp("patched")
    for p in PATCHES:
        for rel in _patched_files(p):
            dst = d / rel
            if not dst.exists():
                dst.parent.mkdir(parents=True, exist_ok=True)
                shutil.copy2(REF / rel, dst)
    results = {}
    for p in PATCHES:
        results[p.name] = subprocess.run(["patch", "-p1", "-F0", "-N", "-i", str(p)], cwd=d,
                                         capture_output=True, text=True)
    shutil.copytree(NEW_FILES, d / "src", dirs_exist_ok=True)
    return d, results


@pytest.fixture(scope="module")
def objs(tree, tmp_path_factory):
    d, _ = tree
    out = tmp_path_factory.mktemp("patched_objs")
    incs = [f"-I{d / 'src'}", f"-I{ROOT / 'include'}", *INCS_REF]  # patched files shadow the reference's
    res = {}
    for name, rel in UNITS.items():
        o = out / f"{name}.o"
        res[name] = (o, subprocess.run(["g++", *FLAGS, *incs, "-c", str(d / rel), "-o", str(o)],
                                       capture_output=True, text=True))
    o = out / "ours.o"
    res["ours"] = (o, subprocess.run(["g++", *FLAGS, *INCS_REF, "-DMI_ONECCL_TREE", f"-I{ROOT / 'include'}", "-c",
                                      str(ROOT / "oneccl_amd" / "csrc" / "comp.cpp"), "-o", str(o)],
                                     capture_output=True, text=True))
    return res


def test_patch_set_is_complete():
    names = [p.name for p in PATCHES]
    assert names == ["0001-build-swap-src-comp.patch", "0002-atl-mpi-fp16-user-op.patch",
                     "0003-async-host-reduce-entries.patch", "0004-nreduce-fused-fanin.patch",
                     "0005-buffer-cache-declares-host-buffers.patch", "0006-copy-entries-host-copy.patch",
                     "0007-finalize-releases-pooled-contexts.patch"], names
    assert (NEW_FILES / "sched" / "entry" / "batch_reduce_entry.hpp").exists()


def test_every_patch_applies_without_fuzz(tree):
    _, results = tree
    for name, r in results.items():
        assert r.returncode == 0, (name, r.stdout + r.stderr)
        assert "fuzz" not in r.stdout and "offset" not in r.stdout, (name, r.stdout)


def test_build_patch_swaps_three_sources(tree):
    d, _ = tree
    cm = (d / "src" / "CMakeLists.txt").read_text()
    for gone in ("comp/comp.cpp", "comp/bf16/bf16.cpp", "comp/fp16/fp16.cpp"):
        assert f"    {gone}\n" not in cm, gone
    for kept in ("comp/bf16/bf16_intrisics.cpp", "comp/fp16/fp16_intrisics.cpp"):
        assert f"    {kept}\n" in cm, kept
    for src in ("comp.cpp", "host_reduce.cpp", "host_reduce_avx512.cpp"):
        assert f"${{ONECCL_AMD_ROOT}}/oneccl_amd/csrc/{src}" in cm, src
    assert "COMPILE_DEFINITIONS MI_ONECCL_TREE" in cm
    assert "libmi_reduce.so" in cm


def test_patched_units_compile_with_reference_flags(objs):
    for name, (_, r) in objs.items():
        assert r.returncode == 0, (name, r.stderr[-3000:])


def test_patched_units_need_only_what_the_dropin_defines(objs):
    """Every src/comp-side symbol the patched objects use (the asynchronous
    entry points, the fused batch reduce, ccl_fp16_reduce) is defined by the
    drop-in's in-tree object."""
    ours = _global_defs(objs["ours"][0])
    comp_api = re.compile(r"ccl_comp_|ccl_fp16_reduce|ccl_bf16_reduce|ccl_reduction_to_str")
    for name in ("copy_entry", "recv_copy_entry"):  # 0006: the host copy, not the classifying one
        need = _undefs(objs[name][0])
        assert any("ccl_comp_copy_host" in x for x in need), name
        assert not any(re.search(r"ccl_comp_copyPKv", x) for x in need), name
    for name in UNITS:
        need = {s for s in _undefs(objs[name][0]) if comp_api.search(s)}
        missing = sorted(need - ours)
        assert not missing, (name, missing)
    starts = {s for s in _undefs(objs["reduce_local_entry"][0]) if "ccl_comp_reduce_start" in s}
    assert starts, "reduce_local_entry must start the reduce asynchronously"
    assert any("ccl_comp_batch_reduce_start" in s for s in _undefs(objs["allreduce"][0]))
    # the schedule reaches the asynchronous entries (its stream decides
    # whether operands are looked up): ccl_sched* is their first parameter
    assert all("P9ccl_sched" in s for s in starts), starts
    mpi = _undefs(objs["atl_mpi_ctx"][0])
    fp16 = {s for s in mpi if "fp16" in s}
    assert not any("wrap" in s for s in fp16), fp16  # the inline SIMD body is no longer used
    # 0002: both MPI user ops say their operands are host memory
    # (include/mi_ccl_lp_host.hpp), so a small bucket is folded with no lookup
    assert any(s.startswith("_Z20ccl_fp16_reduce_host") for s in mpi), sorted(fp16)
    assert any(s.startswith("_Z20ccl_bf16_reduce_host") for s in mpi), sorted(mpi)
    assert not any(re.match(r"_Z15ccl_(bf16|fp16)_reduce", s) for s in mpi), sorted(mpi)


def test_buffer_cache_declares_exactly_what_it_frees(tree, objs):
    """0005: every buffer the regular cache mallocs is declared, and every
    CCL_FREE of one (clear() and push() without the cache) undeclares it
    first; the declaration symbols it needs are the drop-in's C exports."""
    d, _ = tree
    src = (d / "src" / "sched" / "buffer" / "buffer_cache.cpp").read_text()
    body = src[src.index("void regular_buffer_cache::clear()"):src.index("#ifdef CCL_ENABLE_SYCL\nsycl_buffer_cache")]
    assert body.count("CCL_MALLOC") == 1 and body.count("mi_ccl_comp_register_host_buffer(*pptr, bytes)") == 1
    assert body.count("CCL_FREE") == 2
    for free_at in [m.start() for m in re.finditer(r"CCL_FREE\(", body)]:
        before = body[:free_at].rstrip().splitlines()[-1]
        assert "mi_ccl_comp_unregister_host_buffer" in before, before
    need = _undefs(objs["buffer_cache"][0])
    assert {"mi_ccl_comp_register_host_buffer", "mi_ccl_comp_unregister_host_buffer"} <= need
    assert {"mi_ccl_comp_register_host_buffer", "mi_ccl_comp_unregister_host_buffer"} <= _global_defs(objs["ours"][0])


def test_finalize_releases_pooled_contexts(tree, objs):
    """0007: oneCCL's global reset frees the contexts of the
    exited workers (streams, staging and bounce buffers) once the executor
    has joined them; the call is libmi_reduce's C export."""
    import ctypes
    d, _ = tree
    src = (d / "src" / "common" / "global" / "global.cpp").read_text()
    body = src[src.index("ccl::status global_data::reset()"):]
    assert body.index("executor.reset();") < body.index("mi_release_pooled_contexts();")
    assert "mi_release_pooled_contexts" in _undefs(objs["global"][0])
    lib = ROOT / "oneccl_amd" / "lib" / "libmi_reduce.so"
    if lib.exists():
        assert hasattr(ctypes.CDLL(str(lib)), "mi_release_pooled_contexts")
