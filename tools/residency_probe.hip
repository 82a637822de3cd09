// residency_probe.hip — how many one-wave workgroups a CU actually holds at
// once for a given dynamic LDS reservation (the library sizes its
// reservation as LDS-per-CU / W to cap residency at W waves, but the
// hardware allocates LDS in granules, so the achieved cap may be lower; a
// rocprofv3 kernel trace reports only the kernel's static LDS, 0 here).
//
// Every 64-lane workgroup of the probe reads its CU's identity (HW_REG_HW_ID,
// HW_REG_XCC_ID), raises that CU's counter, records the counter's maximum,
// holds for `hold_us` of wall clock, then lowers the counter.  With the grid
// many times the chip's capacity, each CU's maximum is the residency the
// reservation allows.
//   residency_probe [hold_us=20] [lds_bytes ...]   one JSON line per size
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>

constexpr int kSlots = 2048;  // xcc(3) | se(3) | sh(1) | cu(4)

__global__ void probe(unsigned* cur, unsigned* maxv, unsigned long long hold_ticks) {
    extern __shared__ char lds_cap[];  // never touched
    (void)lds_cap;
    unsigned hwid, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    const unsigned cu = (hwid >> 8) & 0xF, sh = (hwid >> 12) & 1, se = (hwid >> 13) & 7;
    const unsigned idx = ((xcc & 7) << 8) | (se << 5) | (sh << 4) | cu;
    if (threadIdx.x == 0) {
        const unsigned c = atomicAdd(&cur[idx], 1u) + 1u;
        atomicMax(&maxv[idx], c);
    }
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < hold_ticks) __builtin_amdgcn_s_sleep(4);
    if (threadIdx.x == 0) atomicSub(&cur[idx], 1u);
}

int main(int argc, char** argv) {
    const int hold_us = argc > 1 ? atoi(argv[1]) : 20;
    std::vector<unsigned> sizes;
    for (int i = 2; i < argc; i++) sizes.push_back((unsigned)atoi(argv[i]));
    int dev = 0, lds = 0, cus = 0, wall_khz = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, dev);
    if (wall_khz <= 0) wall_khz = 100000;  // s_memrealtime: 100 MHz
    if (sizes.empty())
        for (int w : {0, 6, 8, 10, 12, 16, 24}) sizes.push_back(w ? (unsigned)lds / (unsigned)w : 0u);
    unsigned *cur = nullptr, *maxv = nullptr;
    if (hipMalloc(&cur, kSlots * 4) != hipSuccess || hipMalloc(&maxv, kSlots * 4) != hipSuccess) return 2;
    const unsigned long long ticks = (unsigned long long)hold_us * (unsigned long long)wall_khz / 1000ull;
    const unsigned blocks = (unsigned)std::max(cus, 1) * 64u;  // 64 workgroups per CU: more than any CU holds
    for (unsigned bytes : sizes) {
        (void)hipMemset(cur, 0, kSlots * 4);
        (void)hipMemset(maxv, 0, kSlots * 4);
        hipLaunchKernelGGL(probe, dim3(blocks), dim3(64), bytes, 0, cur, maxv, ticks);
        const hipError_t e = hipDeviceSynchronize();
        if (e != hipSuccess) {
            printf("{\"lds_bytes\": %u, \"error\": \"%s\"}\n", bytes, hipGetErrorString(e));
            return 3;
        }
        std::vector<unsigned> m(kSlots);
        (void)hipMemcpy(m.data(), maxv, kSlots * 4, hipMemcpyDeviceToHost);
        std::map<unsigned, int> hist;
        int seen = 0;
        for (unsigned v : m)
            if (v) {
                hist[v]++;
                seen++;
            }
        printf("{\"lds_bytes\": %u, \"lds_per_cu\": %d, \"planned_waves\": %s%.2f, \"cus_seen\": %d, "
               "\"max_resident_waves_histogram\": {",
               bytes, lds, bytes ? "" : "-", bytes ? (double)lds / bytes : 1.0, seen);
        bool first = true;
        for (auto& kv : hist) {
            printf("%s\"%u\": %d", first ? "" : ", ", kv.first, kv.second);
            first = false;
        }
        printf("}}\n");
        fflush(stdout);
    }
    (void)hipFree(cur);
    (void)hipFree(maxv);
    return 0;
}
