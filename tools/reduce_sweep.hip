// reduce_sweep.hip — launch-geometry / memory-policy sweep of the fp32 sum
// reduce kernel (the same template the library instantiates) on a 1 GiB
// bucket, against two known-good streaming references measured on the same
// device: hipMemcpy D2D and the library's own copy kernel.
//
// Interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24).
// Output: one JSON object per variant on stdout.
//   reduce_sweep [bucket_MiB=1024] [rounds=5] [reps=10]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "../oneccl_amd/csrc/reduce_kernels.hpp"

using namespace mi;

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e = (x);                                                              \
        if (e != hipSuccess) {                                                           \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

// Streaming ceilings on this device: read-only (2 streams, nt loads, one
// float per block written so nothing is dead) and write-only (nt stores).
__global__ __launch_bounds__(kBlock) void read2_kernel(const u32x4* a, const u32x4* b, uint64_t nvec, float* sink) {
    constexpr int U = 4;
    const uint64_t base = (uint64_t)blockIdx.x * kBlock * U + threadIdx.x;
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < U; j++) {
        const uint64_t v = base + (uint64_t)j * kBlock;
        if (v < nvec) {
            u32x4 x = __builtin_nontemporal_load(a + v), y = __builtin_nontemporal_load(b + v);
            acc += __uint_as_float(x[0] ^ y[1]) + __uint_as_float(x[2] ^ y[3]);
        }
    }
    if (acc == 1.2345f) sink[blockIdx.x] = acc;  // practically never taken; keeps the loads live
}

__global__ __launch_bounds__(kBlock) void write_kernel(u32x4* o, uint64_t nvec) {
    constexpr int U = 4;
    const uint64_t base = (uint64_t)blockIdx.x * kBlock * U + threadIdx.x;
#pragma unroll
    for (int j = 0; j < U; j++) {
        const uint64_t v = base + (uint64_t)j * kBlock;
        if (v < nvec) __builtin_nontemporal_store(u32x4{(uint32_t)v, 1u, 2u, 3u}, o + v);
    }
}

// read-only ceiling for K streams at the fan-in's geometry (1024 lanes, one
// 16-B vector per lane per stream)
template <int K>
__global__ __launch_bounds__(1024) void readk_kernel(RKArgs a, float* sink) {
    const uint64_t v = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
    if (v >= a.nvec) return;
    uint32_t acc = 0;
#pragma unroll
    for (int j = 0; j < K; j++) {
        const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a.in[j]) + v);
        acc ^= x[0] ^ x[1] ^ x[2] ^ x[3];
    }
    if (acc == 0x9e3779b9u) sink[blockIdx.x] = 1.f;  // practically never taken; keeps the loads live
}

struct Variant {
    std::string name;
    double traffic;  // bytes per launch
    std::function<void(hipStream_t)> run;
    std::vector<float> ms;
};

template <int U, int MEM, int B = kBlock>
void add_reduce(std::vector<Variant>& vs, KArgs a, int cap, double traffic) {
    const uint64_t tile = (uint64_t)B * U;
    uint64_t blocks = (a.nvec + tile - 1) / tile;
    if (cap > 0) blocks = std::min<uint64_t>(blocks, cap);
    char name[128];
    snprintf(name, sizeof name, "reduce B=%d U=%d mem=%d grid=%s%llu", B, U, MEM, cap ? "cap" : "",
             (unsigned long long)blocks);
    vs.push_back({name, traffic, [a, blocks](hipStream_t s) {
                      hipLaunchKernelGGL((reduce_kernel<float, OP_SUM, 0u, 2, U, MEM, 0, B>), dim3((unsigned)blocks),
                                         dim3(B), 0, s, a);
                  }, {}});
}

template <int U, int B>
void add_reduce2(std::vector<Variant>& vs, KArgs a, double traffic) {
    R2Args r{};
    r.acc = a.in[0];
    r.in = a.in[1];
    r.out = a.out;
    r.nvec = a.nvec;
    r.trunc_from = a.count;
    const uint64_t blocks = (a.nvec + (uint64_t)B * U - 1) / ((uint64_t)B * U);
    char name[128];
    snprintf(name, sizeof name, "reduce2 lean B=%d U=%d grid=%llu", B, U, (unsigned long long)blocks);
    vs.push_back({name, traffic, [r, blocks](hipStream_t s) {
                      hipLaunchKernelGGL((reduce2_kernel<float, OP_SUM, 0u, U, B>), dim3((unsigned)blocks), dim3(B),
                                         0, s, r);
                  }, {}});
}

template <int B>
void add_fan_buf(std::vector<Variant>& vs, KArgs a, double traffic) {
    const uint64_t blocks = (a.nvec + B - 1) / B;
    char name[128];
    snprintf(name, sizeof name, "fan buffer K=%d B=%d grid=%llu%s", a.k, B, (unsigned long long)blocks,
             a.out == a.in[0] ? " inplace" : "");
    vs.push_back({name, traffic, [a, blocks](hipStream_t s) {
                      hipLaunchKernelGGL((fan_kernel<float, OP_SUM, 0u, B>), dim3((unsigned)blocks), dim3(B), 0, s, a);
                  }, {}});
}

template <int B>
void add_reduce2b(std::vector<Variant>& vs, KArgs a, double traffic) {
    R2Args r{};
    r.acc = a.in[0];
    r.in = a.in[1];
    r.out = a.out;
    r.nvec = a.nvec;
    r.trunc_from = a.count;
    const uint64_t blocks = (a.nvec + B - 1) / B;
    char name[128];
    snprintf(name, sizeof name, "reduce2 buffer B=%d grid=%llu", B, (unsigned long long)blocks);
    vs.push_back({name, traffic, [r, blocks](hipStream_t s) {
                      hipLaunchKernelGGL((reduce2b_kernel<float, OP_SUM, 0u, B>), dim3((unsigned)blocks), dim3(B), 0, s, r);
                  }, {}});
}

template <int K, int U, int B>
void add_fanin_lean(std::vector<Variant>& vs, KArgs a, double traffic) {
    RKArgs r{};
    for (int i = 0; i < K; i++) r.in[i] = a.in[i];
    r.out = a.out;
    r.nvec = a.nvec;
    r.trunc_from = a.count;
    const uint64_t blocks = (a.nvec + (uint64_t)B * U - 1) / ((uint64_t)B * U);
    char name[128];
    snprintf(name, sizeof name, "fanin lean K=%d B=%d U=%d grid=%llu", K, B, U, (unsigned long long)blocks);
    vs.push_back({name, traffic, [r, blocks](hipStream_t s) {
                      hipLaunchKernelGGL((reducek_kernel<float, OP_SUM, 0u, K, U, B>), dim3((unsigned)blocks),
                                         dim3(B), 0, s, r);
                  }, {}});
}

template <int KT, int U, int MAP = 0, int B = kBlock>
void add_fanin(std::vector<Variant>& vs, KArgs a, double traffic) {
    const uint64_t tile = (uint64_t)B * U;
    uint64_t blocks = (a.nvec + tile - 1) / tile;
    if (MAP) blocks = (blocks + 7) / 8 * 8;
    char name[128];
    snprintf(name, sizeof name, "fanin B=%d KT=%d U=%d mem=3 map=%d grid=%llu", B, KT, U, MAP,
             (unsigned long long)blocks);
    vs.push_back({name, traffic, [a, blocks](hipStream_t s) {
                      hipLaunchKernelGGL((reduce_kernel<float, OP_SUM, 0u, KT, U, 3, MAP, B>), dim3((unsigned)blocks),
                                         dim3(B), 0, s, a);
                  }, {}});
}

template <int K>
void add_readk(std::vector<Variant>& vs, const std::vector<float*>& fan, uint64_t nvec, float* sink, double bytes) {
    RKArgs r{};
    for (int j = 0; j < K; j++) r.in[j] = fan[j];
    r.nvec = nvec;
    const uint64_t blocks = (nvec + 1023) / 1024;
    vs.push_back({"read-only " + std::to_string(K) + " streams (nt, 1024x1)", K * bytes, [r, blocks, sink](hipStream_t s) {
                      hipLaunchKernelGGL(readk_kernel<K>, dim3((unsigned)blocks), dim3(1024), 0, s, r, sink);
                  }, {}});
}

int main(int argc, char** argv) {
    const size_t mib = argc > 1 ? strtoull(argv[1], nullptr, 10) : 1024;
    const int rounds = argc > 2 ? atoi(argv[2]) : 5;
    const int reps = argc > 3 ? atoi(argv[3]) : 10;
    const size_t bytes = mib << 20;
    const size_t n = bytes / 4;
    float *in, *io, *cp;
    CK(hipMalloc(&in, bytes));
    CK(hipMalloc(&io, bytes));
    CK(hipMalloc(&cp, bytes));
    CK(hipMemset(in, 0x3c, bytes));  // ~0.0115f: finite, non-zero
    CK(hipMemset(io, 0x3c, bytes));
    hipStream_t s;
    CK(hipStreamCreate(&s));

    KArgs a{};
    a.in[0] = io;
    a.in[1] = in;
    a.out = io;
    a.k = 2;
    a.count = n;
    a.nvec = n / 4;
    a.trunc_from = n;
    const double t3 = 3.0 * bytes;

    std::vector<Variant> vs;
    add_reduce<4, 3, 256>(vs, a, 0, t3);  // the general kernel
    add_reduce2<1, 1024>(vs, a, t3);      // the library's 2-input kernel
    add_reduce2<1, 512>(vs, a, t3);
    add_reduce2b<1024>(vs, a, t3);
    add_reduce2b<512>(vs, a, t3);
    add_reduce2b<256>(vs, a, t3);
    // 8-input fan-in (C4): 7 more input buffers, one output
    std::vector<float*> fan(8, nullptr);
    fan[0] = io;
    fan[1] = in;
    for (int j = 2; j < 8; j++) {
        CK(hipMalloc(&fan[j], bytes));
        CK(hipMemset(fan[j], 0x3c, bytes));
    }
    KArgs f8{};
    for (int j = 0; j < 8; j++) f8.in[j] = fan[j];
    f8.out = cp;
    f8.k = 8;
    f8.count = n;
    f8.nvec = n / 4;
    f8.trunc_from = n;
    const double t9 = 9.0 * bytes;
    add_fanin<0, 4>(vs, f8, t9);
    add_fan_buf<1024>(vs, f8, t9);
    add_fan_buf<512>(vs, f8, t9);
    add_fan_buf<256>(vs, f8, t9);
    {
        KArgs ip = f8;  // in place into input 0, as ccl_comp_batch_reduce does
        ip.out = const_cast<void*>(ip.in[0]);
        add_fanin<0, 4>(vs, ip, t9);
        vs.back().name += " inplace";
        add_fan_buf<1024>(vs, ip, t9);
        add_fan_buf<256>(vs, ip, t9);
        KArgs f4 = f8;
        f4.k = 4;
        add_fanin<0, 4>(vs, f4, 5.0 * bytes);
        vs.back().name += " k=4";
        add_fan_buf<1024>(vs, f4, 5.0 * bytes);
        KArgs f3 = f8;
        f3.k = 3;
        add_fanin<0, 4>(vs, f3, 4.0 * bytes);
        vs.back().name += " k=3";
        add_fan_buf<1024>(vs, f3, 4.0 * bytes);
    }
    add_fanin_lean<8, 1, 1024>(vs, f8, t9);
    add_fanin_lean<8, 1, 512>(vs, f8, t9);
    add_fanin_lean<8, 1, 256>(vs, f8, t9);
    add_fanin_lean<8, 2, 256>(vs, f8, t9);
    add_fanin_lean<8, 2, 512>(vs, f8, t9);
    add_fanin_lean<4, 1, 1024>(vs, f8, 5.0 * bytes);
    add_readk<2>(vs, fan, n / 4, cp, (double)bytes);
    add_readk<4>(vs, fan, n / 4, cp, (double)bytes);
    add_readk<8>(vs, fan, n / 4, cp, (double)bytes);
    {
        const uint64_t nvec = bytes / 16;
        const uint64_t blocks = (nvec + kBlock * 4 - 1) / (kBlock * 4);
        float* sink = cp;
        vs.push_back({"read-only 2 streams (nt)", 2.0 * bytes, [=](hipStream_t st) {
                          hipLaunchKernelGGL(read2_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, st,
                                             (const u32x4*)in, (const u32x4*)io, nvec, sink);
                      }, {}});
        vs.push_back({"write-only 1 stream (nt)", 1.0 * bytes, [=](hipStream_t st) {
                          hipLaunchKernelGGL(write_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, st,
                                             (u32x4*)cp, nvec);
                      }, {}});
        vs.push_back({"hipMemsetAsync (write-only)", 1.0 * bytes,
                      [=](hipStream_t st) { (void)hipMemsetAsync(cp, 0, bytes, st); }, {}});
    }
    vs.push_back({"hipMemcpyAsync D2D", 2.0 * bytes,
                  [=](hipStream_t st) { (void)hipMemcpyAsync(cp, in, bytes, hipMemcpyDeviceToDevice, st); }, {}});
    for (int mem : {0, 2}) {
        const uint64_t nvec = bytes / 16;
        const uint64_t blocks = (nvec + kBlock * 4 - 1) / (kBlock * 4);
        vs.push_back({mem ? "copy_kernel nt-store" : "copy_kernel plain", 2.0 * bytes, [=](hipStream_t st) {
                          if (mem)
                              hipLaunchKernelGGL(copy_kernel<2>, dim3((unsigned)blocks), dim3(kBlock), 0, st,
                                                 (const char*)in, (char*)cp, 0u, nvec, 0u);
                          else
                              hipLaunchKernelGGL(copy_kernel<0>, dim3((unsigned)blocks), dim3(kBlock), 0, st,
                                                 (const char*)in, (char*)cp, 0u, nvec, 0u);
                      }, {}});
    }

    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (auto& v : vs) v.run(s);  // warm every variant
    CK(hipStreamSynchronize(s));
    for (int r = 0; r < rounds; r++) {
        for (auto& v : vs) {
            for (int i = 0; i < reps; i++) {
                CK(hipEventRecord(e0, s));
                v.run(s);
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                v.ms.push_back(ms);
            }
        }
        fprintf(stderr, "round %d/%d done\n", r + 1, rounds);
    }
    for (auto& v : vs) {
        std::sort(v.ms.begin(), v.ms.end());
        const float med = v.ms[v.ms.size() / 2], best = v.ms.front();
        printf("{\"variant\": \"%s\", \"bucket_MiB\": %zu, \"median_ms\": %.5f, \"best_ms\": %.5f, "
               "\"median_GBps\": %.1f, \"best_GBps\": %.1f, \"frac_of_8TBps\": %.4f}\n",
               v.name.c_str(), mib, med, best, v.traffic / (med * 1e-3) / 1e9, v.traffic / (best * 1e-3) / 1e9,
               v.traffic / (med * 1e-3) / 8e12);
    }
    return 0;
}
