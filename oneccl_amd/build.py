"""In-tree build of the native libraries (no JIT cache: the .so files live in
oneccl_amd/lib/ and travel with the repo snapshot to the GPU box).

  libmi_reduce.so     hipcc --offload-arch=gfx950: kernels + C ABI
                      (include/mi_reduce.h)
  libccl_comp_hip.so  g++: the drop-in src/comp shim (oneCCL's C++ entry
                      points, include/mi_ccl_comp.h), linked to libmi_reduce.so
  tools/reduce_sweep  hipcc: launch-geometry / load-policy sweep (bench tool)
  tools/policy_sweep  hipcc: cache-policy / store-form / grid-stride experiment
  tools/fan_sweep     hipcc: fan-in input order experiment
  tools/copy_sweep    hipcc: shapes of the device copy (ccl_comp_copy)
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
LIB = PKG / "lib"
ARCH = os.environ.get("MI_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found: the MI355X build needs ROCm's hipcc")


def _stale(target: Path, deps: list[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def _run(cmd: list[str]) -> None:
    print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


def build_mi_reduce(force: bool = False) -> Path:
    out = LIB / "libmi_reduce.so"
    deps = [CSRC / "mi_reduce.hip", CSRC / "reduce_kernels.hpp", ROOT / "include" / "mi_reduce.h"]
    if force or _stale(out, deps):
        LIB.mkdir(exist_ok=True)
        _run([_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall",
              "-o", str(out), str(CSRC / "mi_reduce.hip")])
    return out


# The host reduce (small host-resident chunks, include/mi_host_reduce.h) is
# compiled for AVX2 + F16C + FMA; comp.cpp calls it only after
# mi_host_supported() has checked the CPU.
HOST_REDUCE_FLAGS = ["-O3", "-mavx2", "-mf16c", "-mfma", "-fPIC", "-Wall", "-Wextra"]
# its 16-lane bf16/fp16 form, called only on CPUs with AVX-512 (+ AVX512_BF16)
HOST_REDUCE_AVX512_FLAGS = HOST_REDUCE_FLAGS + ["-mavx512f", "-mavx512bw", "-mavx512vl", "-mavx512bf16"]


def build_shim(force: bool = False) -> Path:
    out = LIB / "libccl_comp_hip.so"
    deps = [CSRC / "comp.cpp", CSRC / "host_reduce.cpp", CSRC / "host_reduce_avx512.cpp", CSRC / "host_lp.hpp",
            CSRC / "ccl_mirror.hpp", ROOT / "include" / "mi_reduce.h",
            ROOT / "include" / "mi_ccl_comp.h", ROOT / "include" / "mi_ccl_comp_async.hpp",
            ROOT / "include" / "mi_host_reduce.h", LIB / "libmi_reduce.so"]
    if force or _stale(out, deps):
        cxx = os.environ.get("CXX", "g++")
        obj = LIB / "host_reduce.o"
        obj512 = LIB / "host_reduce_avx512.o"
        _run([cxx, *HOST_REDUCE_FLAGS, "-std=c++17", "-c", "-o", str(obj), str(CSRC / "host_reduce.cpp")])
        _run([cxx, *HOST_REDUCE_AVX512_FLAGS, "-std=c++17", "-c", "-o", str(obj512),
              str(CSRC / "host_reduce_avx512.cpp")])
        _run([cxx, "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-Wextra",
              "-o", str(out), str(CSRC / "comp.cpp"), str(obj), str(obj512),
              f"-L{LIB}", "-lmi_reduce", "-ldl", "-Wl,-rpath,$ORIGIN"])
        obj.unlink()
        obj512.unlink()
    return out


def build_sweep(force: bool = False) -> Path:
    out = ROOT / "tools" / "reduce_sweep"
    src = ROOT / "tools" / "reduce_sweep.hip"
    deps = [src, CSRC / "reduce_kernels.hpp"]
    if src.exists() and (force or _stale(out, deps)):
        _run([_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-Wall",
              "-o", str(out), str(src)])
    return out


def build_policy_sweep(force: bool = False) -> Path:
    out = ROOT / "tools" / "policy_sweep"
    src = ROOT / "tools" / "policy_sweep.hip"
    if src.exists() and (force or _stale(out, [src])):
        _run([_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-Wno-unused-result", "-o", str(out), str(src)])
    return out


def build_fan_sweep(force: bool = False) -> Path:
    out = ROOT / "tools" / "fan_sweep"
    src = ROOT / "tools" / "fan_sweep.hip"
    deps = [src, CSRC / "reduce_kernels.hpp"]
    if src.exists() and (force or _stale(out, deps)):
        _run([_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-Wall", "-o", str(out), str(src)])
    return out


def build_burst_sweep(force: bool = False) -> Path:
    out = ROOT / "tools" / "burst_sweep"
    src = ROOT / "tools" / "burst_sweep.hip"
    if src.exists() and (force or _stale(out, [src, CSRC / "reduce_kernels.hpp"])):
        _run([_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-Wall", "-o", str(out), str(src)])
    return out


def build_copy_sweep(force: bool = False) -> Path:
    out = ROOT / "tools" / "copy_sweep"
    src = ROOT / "tools" / "copy_sweep.hip"
    if src.exists() and (force or _stale(out, [src, CSRC / "reduce_kernels.hpp"])):
        _run([_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-Wall", "-o", str(out), str(src)])
    return out


def build_lds_stage_sweep(force: bool = False) -> Path:
    out = ROOT / "tools" / "lds_stage_sweep"
    src = ROOT / "tools" / "lds_stage_sweep.hip"
    if src.exists() and (force or _stale(out, [src, CSRC / "reduce_kernels.hpp"])):
        _run([_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-Wall", "-o", str(out), str(src)])
    return out


def build_occupancy_sweep(force: bool = False) -> Path:
    out = ROOT / "tools" / "occupancy_sweep"
    src = ROOT / "tools" / "occupancy_sweep.hip"
    if src.exists() and (force or _stale(out, [src, CSRC / "reduce_kernels.hpp"])):
        _run([_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-Wall", "-o", str(out), str(src)])
    return out


def build_latency(force: bool = False) -> Path:
    out = ROOT / "tools" / "latency"
    src = ROOT / "tools" / "latency.hip"
    if src.exists() and (force or _stale(out, [src, LIB / "libmi_reduce.so"])):
        _run([_hipcc(), f"--offload-arch={ARCH}", "-O2", "-std=c++17", "-Wno-unused-result", "-o", str(out), str(src),
              f"-L{LIB}", "-lmi_reduce", "-Wl,-rpath,$ORIGIN/../oneccl_amd/lib"])
    return out


def build_pointer_kind_probe(force: bool = False) -> Path:
    """Probe: pointer classification cost against concurrent threads."""
    out = ROOT / "tools" / "pointer_kind_probe"
    src = ROOT / "tools" / "pointer_kind_probe.cpp"
    if src.exists() and (force or _stale(out, [src])):
        _run([_hipcc(), "-O2", "-std=c++17", "-o", str(out), str(src), "-pthread", "-lhsa-runtime64"])
    return out


def build_ceiling(force: bool = False) -> Path:
    """libmi_ceiling.so: the memory-only probes bench.py prices each kernel's
    measured ceiling with (tools/ceiling_probe.hip; not product code)."""
    out = LIB / "libmi_ceiling.so"
    src = ROOT / "tools" / "ceiling_probe.hip"
    if src.exists() and (force or _stale(out, [src])):
        LIB.mkdir(exist_ok=True)
        _run([_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall",
              "-o", str(out), str(src)])
    return out


def build_residency_probe(force: bool = False) -> Path:
    """Probe: resident one-wave workgroups per CU against a dynamic LDS size."""
    out = ROOT / "tools" / "residency_probe"
    src = ROOT / "tools" / "residency_probe.hip"
    if src.exists() and (force or _stale(out, [src])):
        _run([_hipcc(), f"--offload-arch={ARCH}", "-O2", "-std=c++17", "-o", str(out), str(src)])
    return out


def build_small_workers(force: bool = False) -> Path:
    """Probe: small host reduces through the drop-in from T threads at once."""
    out = ROOT / "tools" / "small_workers"
    src = ROOT / "tools" / "small_workers.cpp"
    if src.exists() and (force or _stale(out, [src, LIB / "libccl_comp_hip.so"])):
        _run(["g++", "-O2", "-std=c++17", f"-I{ROOT / 'include'}", "-o", str(out), str(src), f"-L{LIB}",
              "-lccl_comp_hip", "-Wl,-rpath,$ORIGIN/../oneccl_amd/lib", "-pthread", "-ldl"])
    return out


def build_segv_trace(force: bool = False) -> Path:
    """Diagnostic: tools/libsegv_trace.so prints a native backtrace on SIGSEGV."""
    out = ROOT / "tools" / "libsegv_trace.so"
    src = ROOT / "tools" / "segv_trace.c"
    if src.exists() and (force or _stale(out, [src])):
        _run(["gcc", "-O1", "-g", "-fPIC", "-shared", "-Wall", "-o", str(out), str(src)])
    return out


def build_dropin_caller(force: bool = False) -> Path:
    """Test program: a C++ caller linking libccl_comp_hip.so by oneCCL's own
    mangled names (tests/cpp/dropin_caller.cpp)."""
    src = ROOT / "tests" / "cpp" / "dropin_caller.cpp"
    out = ROOT / "tests" / "cpp" / "dropin_caller"
    deps = [src, CSRC / "ccl_mirror.hpp", ROOT / "include" / "mi_ccl_comp_async.hpp", LIB / "libccl_comp_hip.so"]
    if src.exists() and (force or _stale(out, deps)):
        _run([_hipcc(), "-O2", "-std=c++17", "-o", str(out), str(src), f"-L{LIB}", "-lccl_comp_hip",
              "-lmi_reduce", f"-Wl,-rpath,{LIB}", "-Wl,-rpath,$ORIGIN/../../oneccl_amd/lib"])
    return out


def build_asan(force: bool = False) -> Path:
    """Host-AddressSanitizer builds of the product's host code (device code is
    not instrumented: GPU ASan is not available on this pool) plus the C++
    drop-in caller linked against them: lib/asan/*.so, tests/cpp/dropin_caller_asan.
    Run it with ASAN_OPTIONS=detect_leaks=0 (the HIP runtime keeps its allocations)."""
    adir = LIB / "asan"
    adir.mkdir(parents=True, exist_ok=True)
    san = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fno-omit-frame-pointer"]
    mi = adir / "libmi_reduce.so"
    if force or _stale(mi, [CSRC / "mi_reduce.hip", CSRC / "reduce_kernels.hpp"]):
        _run([_hipcc(), f"--offload-arch={ARCH}", "-O1", "-g", "-std=c++17", "-fPIC", "-shared", *san,
              "-o", str(mi), str(CSRC / "mi_reduce.hip")])
    shim = adir / "libccl_comp_hip.so"
    if force or _stale(shim, [CSRC / "comp.cpp", CSRC / "ccl_mirror.hpp", ROOT / "include" / "mi_ccl_comp_async.hpp", mi]):
        # the same compiler (and so the same ASan runtime) as the hipcc-built pieces
        clang = next((c for c in ("/opt/rocm/lib/llvm/bin/clang++", "/opt/rocm/llvm/bin/clang++")
                      if Path(c).exists()), "clang++")
        h512 = adir / "host_reduce_avx512.o"
        _run([clang, "-O1", "-g", "-std=c++17", "-fPIC", "-fsanitize=address", "-fno-omit-frame-pointer",
              *HOST_REDUCE_AVX512_FLAGS[1:], "-c", "-o", str(h512), str(CSRC / "host_reduce_avx512.cpp")])
        _run([clang, "-O1", "-g", "-std=c++17", "-fPIC", "-shared", "-fsanitize=address", "-mavx2", "-mf16c",
              "-mfma", "-fno-omit-frame-pointer", "-o", str(shim), str(CSRC / "comp.cpp"),
              str(CSRC / "host_reduce.cpp"), str(h512), f"-L{adir}", "-lmi_reduce", "-Wl,-rpath,$ORIGIN"])
    src = ROOT / "tests" / "cpp" / "dropin_caller.cpp"
    out = ROOT / "tests" / "cpp" / "dropin_caller_asan"
    if force or _stale(out, [src, shim]):
        _run([_hipcc(), f"--offload-arch={ARCH}", "-O1", "-g", "-std=c++17", *san, "-fsanitize=address", "-o",
              str(out), str(src),
              f"-L{adir}", "-lccl_comp_hip", "-lmi_reduce", f"-Wl,-rpath,{adir}",
              "-Wl,-rpath,$ORIGIN/../../oneccl_amd/lib/asan"])
    return out


def build_oracle(force: bool = False) -> Path:
    """TEST INFRASTRUCTURE: the CPU oracle (oracle/Makefile), and, where the
    reference tree is present (this container, not the GPU box), the harnesses
    over the reference's own compiled code (oracle/_ref, `make -C oracle ref`:
    the AVX-512 bf16/fp16 bodies, the avx512fp16 impl, and src/comp/comp.cpp's
    CCL_REDUCE / scalar bf16 / batch reduce, whose library also serves as
    bench.py's CPU baseline)."""
    odir = ROOT / "oracle"
    if force:
        _run(["make", "-C", str(odir), "clean"])
    _run(["make", "-C", str(odir), "-j4"])
    if Path("/root/reference/src/comp").is_dir():
        _run(["make", "-C", str(odir), "ref"])
    return odir / "lib" / "libcomp_oracle.so"


def build_all(force: bool = False, asan: bool = False) -> None:
    """`force` recompiles the product libraries, the C++ drop-in caller and the
    oracle whatever their timestamps (what __graft_entry__.build() does, so a
    driver-side build never reuses shipped binaries); the research tools are
    rebuilt only when stale.  `asan`: also the host-ASan builds (kept out of
    the GPU push, built on the box by tools/gpu_run.sh asan)."""
    build_mi_reduce(force)
    build_shim(force)
    build_dropin_caller(force)
    build_oracle(force)
    build_ceiling(force)
    build_sweep()
    build_policy_sweep()
    build_fan_sweep()
    build_burst_sweep()
    build_copy_sweep()
    build_lds_stage_sweep()
    build_occupancy_sweep()
    build_latency()
    build_pointer_kind_probe()
    build_small_workers()
    build_residency_probe()
    build_segv_trace()
    if asan:
        build_asan(force)


if __name__ == "__main__":
    if "--asan" in sys.argv:
        build_mi_reduce()
        build_shim()
        build_asan("--force" in sys.argv)
    else:
        build_all(force="--force" in sys.argv)
