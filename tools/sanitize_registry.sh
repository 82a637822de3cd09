#!/usr/bin/env bash
# Host sanitizers over libmi_reduce's declared host ranges (lock-free reads,
# grace-period publication, reader-slot recycling): tests/cpp/registry_stress.cpp
# against TSan and ASan builds of the library's host code (device code is not
# instrumented).  CPU only; ~3 minutes of hipcc.  Output: one line per sanitizer.
#   tools/sanitize_registry.sh [seconds=2] [outdir=/tmp/mi_san]
set -eu
secs=${1:-2}
out=${2:-/tmp/mi_san}
root=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$out"
hipcc=/opt/rocm/bin/hipcc
clang=/opt/rocm/lib/llvm/bin/clang++
for san in thread address; do
    extra=""
    [ $san = address ] && extra="-Xarch_host -fno-omit-frame-pointer"
    $hipcc --offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -shared -Xarch_host -fsanitize=$san $extra \
        -o "$out/libmi_reduce_$san.so" "$root/oneccl_amd/csrc/mi_reduce.hip"
    $clang -O1 -g -std=c++17 -fsanitize=$san -fno-omit-frame-pointer -I"$root/include" \
        -o "$out/registry_stress_$san" "$root/tests/cpp/registry_stress.cpp" \
        -L"$out" -l"mi_reduce_$san" -Wl,-rpath,"$out" -pthread
    echo "== $san"
    ASAN_OPTIONS=detect_leaks=0 TSAN_OPTIONS=halt_on_error=1 "$out/registry_stress_$san" "$secs" 2>&1
done
