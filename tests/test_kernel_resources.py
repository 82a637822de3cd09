"""Register and scratch budget of every kernel in the built library (CPU:
reads the gfx950 code object's metadata, no GPU).  A kernel that spills to
scratch runs an order of magnitude slower and says nothing about it: round 2
found the fp32 8-input fan-in keeping its inputs in scratch (520 B per lane,
33 ms instead of 1.6 ms per GiB) after a refactor that passed every parity
test.  So: no kernel may use scratch or spill, and each fits its launch
bound's VGPR budget.  And no kernel may compute in fp16: the reference
widens to fp32 and rounds with VCVTPS2PH, and LLVM's rewrite of that
sequence into native v_pk_mul_f16 gave different zero signs on gfx950."""
from __future__ import annotations

import re
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
LLVM = Path("/opt/rocm/lib/llvm/bin")
LIBS = [ROOT / "oneccl_amd" / "lib" / "libmi_reduce.so"]


def _code_object(lib: Path, tmp: Path) -> Path:
    fat, co = tmp / "fat.bin", tmp / "co.o"
    subprocess.run([str(LLVM / "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", str(lib), str(tmp / "x.so")],
                   check=True, capture_output=True)
    subprocess.run([str(LLVM / "clang-offload-bundler"), "--unbundle", "--type=o",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fat}", f"--output={co}"],
                   check=True, capture_output=True)
    return co


def _kernels(lib: Path, tmp: Path):
    co = _code_object(lib, tmp)
    notes = subprocess.run([str(LLVM / "llvm-readelf"), "--notes", str(co)], check=True, capture_output=True,
                           text=True).stdout
    out = []
    for block in re.split(r"\n\s+- \.", notes):
        name = re.search(r"\.name:\s+(\S+)", "." + block)
        if not name or "private_segment_fixed_size" not in block:
            continue

        def field(key, default=0):
            m = re.search(rf"\.{key}:\s+(\d+)", block)
            return int(m.group(1)) if m else default
        out.append(dict(name=name.group(1), scratch=field("private_segment_fixed_size"),
                        vgpr=field("vgpr_count"), agpr=field("agpr_count"), vspill=field("vgpr_spill_count"),
                        sspill=field("sgpr_spill_count"), wg=field("max_flat_workgroup_size", 1024)))
    return out


@pytest.mark.parametrize("lib", LIBS, ids=lambda p: p.name)
def test_no_kernel_spills_or_uses_scratch(lib, tmp_path):
    if not lib.exists() or not (LLVM / "clang-offload-bundler").exists():
        pytest.skip("library or ROCm LLVM tools absent")
    if shutil.which("hipcc") is None and not Path("/opt/rocm/bin/hipcc").exists():
        pytest.skip("no ROCm toolchain")
    ks = _kernels(lib, tmp_path)
    assert len(ks) > 100, "code object metadata not found"
    bad = [k for k in ks if k["scratch"] or k["vspill"] or k["sspill"]]
    assert not bad, "kernels using scratch / spilling: " + "; ".join(
        f"{k['name']} scratch={k['scratch']} vspill={k['vspill']} sspill={k['sspill']}" for k in bad[:10])
    for k in ks:
        # 512 VGPRs per SIMD lane; a workgroup of wg lanes puts wg/256 waves on each SIMD
        budget = 512 // max(1, k["wg"] // 256)
        assert k["vgpr"] + k["agpr"] <= budget, k


@pytest.mark.parametrize("lib", LIBS, ids=lambda p: p.name)
def test_no_kernel_computes_in_fp16(lib, tmp_path):
    if not lib.exists() or not (LLVM / "clang-offload-bundler").exists():
        pytest.skip("library or ROCm LLVM tools absent")
    co = _code_object(lib, tmp_path)
    dis = subprocess.run([str(LLVM / "llvm-objdump"), "-d", str(co)], check=True, capture_output=True,
                         text=True).stdout
    fn, hits = None, {}
    for line in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:$", line)
        if m:
            fn = m.group(1)
        elif re.search(r"\bv_(pk_)?(add|sub|mul|fma|mad|min|max)[a-z0-9_]*_f16\b", line):
            hits[fn] = hits.get(fn, 0) + 1
    assert "v_cvt_f32_f16" in dis, "disassembly not as expected"
    assert not hits, f"native fp16 arithmetic in: {sorted(hits)[:8]}"
