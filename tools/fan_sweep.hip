// fan_sweep.hip — experiment: does the ORDER in which a block reads the K
// inputs of a fan-in change the HBM rate?
//
// The library's fan_kernel issues one 16-B vector of every input per lane at
// once (input-interleaved: at any moment every block touches all K streams).
// Read-only streams measured 7.0 TB/s for 2 streams but 6.3-6.7 for 4-8
// (profiles/round1_sweep7_fan_buffer.jsonl), so the stream count seen by the
// DRAM looks like the limiter.  Here blocks own U vectors per lane per input
// and walk the inputs G at a time (input-major), double-buffered so 2*G*U
// vectors per lane stay in flight: each block touches at most 2G streams.
//
// Variants, interleaved rounds in one process (cdna_hip_programming.md §5.4):
//   readk      read-only, all K inputs at once (ceiling of the current order)
//   read_im    read-only, input-major G x U
//   fan_im     the fp32 sum fan-in, input-major G x U (+ the nt store)
//   fan_kernel the library's kernel (baseline)
//   fan_kernel over one 8 GiB allocation (inputs contiguous in memory)
//
//   fan_sweep [bucket_MiB=1024] [rounds=5] [reps=8] [layout|pipe|skew]
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

typedef float f32x4 __attribute__((ext_vector_type(4)));

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

// Input-major: block tile = B*U vectors per input (nvec must be a multiple).
// Stage s = inputs [s*G, s*G+G), U vectors each.  Stages 0 and 1 are issued
// up front; stage s+2 is issued right after stage s is consumed, so two
// stages are in flight.  Left alone the compiler hoists every load to the
// top (they are independent), so the address of stage s+2 carries a zero
// laundered through an asm that reads stage s's sum: a real data dependency.
__device__ __forceinline__ uint32_t zero_after(float dep) {
    uint32_t z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z) : "v"(dep));
    return z;
}

template <int K, int G, int U, int B, bool STORE>
__global__ __launch_bounds__(B) void im_kernel(RKArgs a, float* sink) {
    constexpr int S = K / G;
    const uint64_t v0 = (uint64_t)blockIdx.x * (B * U) + threadIdx.x;
    u32x4 buf[S][G][U];  // fully unrolled: only two stages are live at a time
    f32x4 acc[U];
#pragma unroll
    for (int s = 0; s < (S < 2 ? S : 2); s++)
#pragma unroll
        for (int g = 0; g < G; g++)
#pragma unroll
            for (int j = 0; j < U; j++)
                buf[s][g][j] =
                    __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a.in[s * G + g]) + v0 + (uint64_t)j * B);
#pragma unroll
    for (int s = 0; s < S; s++) {
#pragma unroll
        for (int g = 0; g < G; g++)
#pragma unroll
            for (int j = 0; j < U; j++) {
                const f32x4 x = __builtin_bit_cast(f32x4, buf[s][g][j]);
                acc[j] = (s == 0 && g == 0) ? x : acc[j] + x;
            }
        if (s + 2 < S) {
            const uint64_t vz = v0 + zero_after(acc[U - 1][3]);
#pragma unroll
            for (int g = 0; g < G; g++)
#pragma unroll
                for (int j = 0; j < U; j++)
                    buf[s + 2][g][j] = __builtin_nontemporal_load(
                        reinterpret_cast<const u32x4*>(a.in[(s + 2) * G + g]) + vz + (uint64_t)j * B);
        }
    }
    if constexpr (STORE) {
#pragma unroll
        for (int j = 0; j < U; j++)
            __builtin_nontemporal_store(__builtin_bit_cast(u32x4, acc[j]),
                                        reinterpret_cast<u32x4*>(a.out) + v0 + (uint64_t)j * B);
    } else {
        float t = 0.f;
#pragma unroll
        for (int j = 0; j < U; j++) t += acc[j][0] + acc[j][3];
        if (t == 1.2345e-7f) sink[blockIdx.x] = t;
    }
}

// Persistent, software-pipelined fan-in: block b walks tiles b, b+G, ...;
// tile t+G's K loads are issued BEFORE tile t's result is stored, so the
// write of one tile overlaps the reads of the next instead of following
// its own reads.  (pipe mode)
template <int K, int B>
__global__ __launch_bounds__(B) void pipe_kernel(RKArgs a) {
    const uint64_t ntiles = a.nvec / B;
    uint64_t t = blockIdx.x;
    if (t >= ntiles) return;
    u32x4 x[K];
#pragma unroll
    for (int j = 0; j < K; j++)
        x[j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a.in[j]) + t * B + threadIdx.x);
    for (;;) {
        f32x4 acc = __builtin_bit_cast(f32x4, x[0]);
#pragma unroll
        for (int j = 1; j < K; j++) acc = acc + __builtin_bit_cast(f32x4, x[j]);
        const uint64_t tn = t + gridDim.x;
        if (tn < ntiles) {
#pragma unroll
            for (int j = 0; j < K; j++)
                x[j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a.in[j]) + tn * B + threadIdx.x);
        }
        __builtin_nontemporal_store(__builtin_bit_cast(u32x4, acc), reinterpret_cast<u32x4*>(a.out) + t * B + threadIdx.x);
        if (tn >= ntiles) break;
        t = tn;
    }
}

// Skewed read-only K streams (skew mode): block b reads vector v of input j
// at (v + j * skew) mod nvec, so at any moment the K streams are at K
// different offsets instead of one.  Every byte of every input is still read
// exactly once.  Tests whether the multi-stream read penalty (8 streams 6.4-6.8
// TB/s vs 2 streams 7.0) comes from the K streams meeting in the same DRAM
// banks at the same offset.
template <int K>
__global__ __launch_bounds__(1024) void readk_skew_kernel(RKArgs a, uint64_t skew, float* sink) {
    const uint64_t v = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
    if (v >= a.nvec) return;
    uint32_t acc = 0;
#pragma unroll
    for (int j = 0; j < K; j++) {
        uint64_t w = v + (uint64_t)j * skew;
        if (w >= a.nvec) w -= a.nvec;
        const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a.in[j]) + w);
        acc ^= x[0] ^ x[1] ^ x[2] ^ x[3];
    }
    if (acc == 0x9e3779b9u) sink[blockIdx.x] = 1.f;
}

// The fan-in with the same skew: input j's tile t is folded with the other
// inputs' tile t only in the unskewed kernel; here each block folds
// (v + j*skew) of input j into out[v], which is NOT the reduce's result — a
// timing probe of the access pattern with the store included, never a product
// kernel.
template <int K>
__global__ __launch_bounds__(1024) void fan_skew_probe(RKArgs a, uint64_t skew) {
    const uint64_t v = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
    if (v >= a.nvec) return;
    f32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < K; j++) {
        uint64_t w = v + (uint64_t)j * skew;
        if (w >= a.nvec) w -= a.nvec;
        acc = acc + __builtin_bit_cast(f32x4, __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a.in[j]) + w));
    }
    __builtin_nontemporal_store(__builtin_bit_cast(u32x4, acc), reinterpret_cast<u32x4*>(a.out) + v);
}

struct Variant {
    std::string name;
    double traffic;  // bytes per launch
    std::function<void(hipStream_t)> run;
    std::vector<float> ms;
};

template <int K, int G, int U, int B, bool STORE>
void add_im(std::vector<Variant>& vs, const RKArgs& r, float* sink, double bytes) {
    const uint64_t blocks = r.nvec / ((uint64_t)B * U);
    char name[160];
    snprintf(name, sizeof name, "%s input-major K=%d G=%d U=%d B=%d grid=%llu", STORE ? "fan_im" : "read_im", K, G,
             U, B, (unsigned long long)blocks);
    vs.push_back({name, (K + (STORE ? 1 : 0)) * bytes, [r, blocks, sink](hipStream_t s) {
                      hipLaunchKernelGGL((im_kernel<K, G, U, B, STORE>), dim3((unsigned)blocks), dim3(B), 0, s, r,
                                         sink);
                  }, {}});
}

template <int K>
void add_readk(std::vector<Variant>& vs, const RKArgs& r, float* sink, double bytes, const char* tag) {
    const uint64_t blocks = (r.nvec + 1023) / 1024;
    vs.push_back({std::string("readk all-at-once K=") + std::to_string(K) + tag, K * bytes,
                  [r, blocks, sink](hipStream_t s) {
                      hipLaunchKernelGGL(readk_kernel<K>, dim3((unsigned)blocks), dim3(1024), 0, s, r, sink);
                  }, {}});
}

void add_fan(std::vector<Variant>& vs, const RKArgs& r, int k, double bytes, const char* tag) {
    KArgs a{};
    for (int i = 0; i < k; i++) a.in[i] = r.in[i];
    a.out = r.out;
    a.k = k;
    a.nvec = r.nvec;
    a.count = r.nvec * 4;
    a.trunc_from = a.count;
    const uint64_t blocks = (a.nvec + 1023) / 1024;
    vs.push_back({std::string("fan_kernel (library) K=") + std::to_string(k) + tag, (k + 1) * bytes,
                  [a, blocks](hipStream_t s) {
                      hipLaunchKernelGGL((fan_kernel<float, OP_SUM, 0u, 1024>), dim3((unsigned)blocks), dim3(1024), 0,
                                         s, a);
                  }, {}});
}

void add_r2(std::vector<Variant>& vs, const void* acc, const void* in, void* out, uint64_t nvec, double bytes,
            const std::string& tag) {
    R2Args r{};
    r.acc = acc;
    r.in = in;
    r.out = out;
    r.nvec = nvec;
    r.trunc_from = nvec * 4;
    const uint64_t blocks = (nvec + 1023) / 1024;
    vs.push_back({"reduce2_kernel (library) " + tag, 3 * bytes, [r, blocks](hipStream_t s) {
                      hipLaunchKernelGGL((reduce2_kernel<float, OP_SUM, 0u, 1, 1024>), dim3((unsigned)blocks),
                                         dim3(1024), 0, s, r);
                  }, {}});
}

int run(std::vector<Variant>& vs, hipStream_t s, int rounds, int reps, size_t mib) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (auto& v : vs) v.run(s);  // warm every variant
    CK(hipStreamSynchronize(s));
    CK(hipGetLastError());
    for (int rr = 0; rr < rounds; rr++) {
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
        fprintf(stderr, "round %d/%d done\n", rr + 1, rounds);
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

// Layout mode: the same kernels over different placements of the operands
// (separate hipMallocs in different orders, one allocation carved into
// slots, in place vs a separate output).
void layouts(std::vector<Variant>& vs, size_t bytes, float* sink) {
    const uint64_t nvec = bytes / 16;
    const double b = (double)bytes;
    auto alloc = [&](size_t n) {
        char* p;
        CK(hipMalloc(&p, n));
        CK(hipMemset(p, 0x3c, n));
        return p;
    };
    // fan-in K=8
    char* out_first = alloc(bytes);
    std::vector<char*> sep(8);
    for (auto& p : sep) p = alloc(bytes);
    char* out_last = alloc(bytes);
    char* big8 = alloc(8 * bytes);
    char* big9 = alloc(9 * bytes);
    RKArgs r{};
    r.nvec = nvec;
    r.trunc_from = nvec * 4;
    for (int i = 0; i < 8; i++) r.in[i] = sep[i];
    r.out = out_last;
    add_fan(vs, r, 8, b, " separate, out allocated last");
    r.out = out_first;
    add_fan(vs, r, 8, b, " separate, out allocated first");
    r.out = sep[0];
    add_fan(vs, r, 8, b, " separate, in place (out = in0)");
    for (int i = 0; i < 8; i++) r.in[i] = big8 + i * bytes;
    r.out = out_last;
    add_fan(vs, r, 8, b, " one 8x allocation, separate out");
    r.out = big8;
    add_fan(vs, r, 8, b, " one 8x allocation, in place (out = slot 0)");
    for (int i = 0; i < 8; i++) r.in[i] = big9 + i * bytes;
    r.out = big9 + 8 * bytes;
    add_fan(vs, r, 8, b, " one 9x allocation, out = slot 8");
    for (int i = 0; i < 8; i++) r.in[i] = big9 + (i + 1) * bytes;
    r.out = big9;
    add_fan(vs, r, 8, b, " one 9x allocation, out = slot 0");
    for (int i = 0; i < 8; i++) r.in[i] = sep[i];
    add_readk<8>(vs, r, sink, b, " separate");
    for (int i = 0; i < 8; i++) r.in[i] = big8 + i * bytes;
    add_readk<8>(vs, r, sink, b, " one 8x allocation");
    // 2-input (C2): inout += in
    add_r2(vs, sep[0], sep[1], sep[0], nvec, b, "separate allocations");
    add_r2(vs, out_first, out_last, out_first, nvec, b, "separate allocations (far apart)");
    add_r2(vs, big8, big8 + bytes, big8, nvec, b, "one allocation, inout = slot 0, in = slot 1");
    add_r2(vs, big8 + bytes, big8, big8 + bytes, nvec, b, "one allocation, inout = slot 1, in = slot 0");
    add_r2(vs, big9, big9 + 4 * bytes, big9, nvec, b, "one allocation, in 4 slots after inout");
    add_r2(vs, sep[2], sep[3], sep[4], nvec, b, "separate allocations, out of place");
    add_r2(vs, big8, big8 + bytes, big8 + 2 * bytes, nvec, b, "one allocation, out of place slots 0,1 -> 2");
}

template <int K, int B>
void add_pipe(std::vector<Variant>& vs, const RKArgs& r, unsigned grid, double bytes) {
    char name[128];
    snprintf(name, sizeof name, "pipe persistent K=%d B=%d grid=%u", K, B, grid);
    vs.push_back({name, (K + 1) * bytes, [r, grid](hipStream_t s) {
                      hipLaunchKernelGGL((pipe_kernel<K, B>), dim3(grid), dim3(B), 0, s, r);
                  }, {}});
}

template <int K>
void add_skew(std::vector<Variant>& vs, const RKArgs& r, float* sink, double bytes, uint64_t skew, bool store) {
    const uint64_t blocks = (r.nvec + 1023) / 1024;
    char name[160];
    snprintf(name, sizeof name, "%s K=%d skew=%llu vectors (%llu KiB)", store ? "fan_skew_probe" : "readk_skew", K,
             (unsigned long long)skew, (unsigned long long)(skew * 16 / 1024));
    vs.push_back({name, (K + (store ? 1 : 0)) * bytes, [r, blocks, sink, skew, store](hipStream_t s) {
                      if (store)
                          hipLaunchKernelGGL(fan_skew_probe<K>, dim3((unsigned)blocks), dim3(1024), 0, s, r, skew);
                      else
                          hipLaunchKernelGGL(readk_skew_kernel<K>, dim3((unsigned)blocks), dim3(1024), 0, s, r, skew,
                                             sink);
                  }, {}});
}

int main(int argc, char** argv) {
    const size_t mib = argc > 1 ? strtoull(argv[1], nullptr, 10) : 1024;
    const int rounds = argc > 2 ? atoi(argv[2]) : 5;
    const int reps = argc > 3 ? atoi(argv[3]) : 8;
    const bool layout_mode = argc > 4 && std::string(argv[4]) == "layout";
    const bool pipe_mode = argc > 4 && std::string(argv[4]) == "pipe";
    const bool skew_mode = argc > 4 && std::string(argv[4]) == "skew";
    const size_t bytes = mib << 20;
    const uint64_t nvec = bytes / 16;
    std::vector<Variant> vs;
    hipStream_t s;
    CK(hipStreamCreate(&s));
    float* sink;
    CK(hipMalloc(&sink, 1 << 20));
    if (layout_mode) {
        layouts(vs, bytes, sink);
        return run(vs, s, rounds, reps, mib);
    }
    std::vector<float*> sep(8, nullptr);
    for (auto& p : sep) {
        CK(hipMalloc(&p, bytes));
        CK(hipMemset(p, 0x3c, bytes));
    }
    float *out, *big;
    CK(hipMalloc(&out, bytes));
    CK(hipMalloc(&big, 8 * bytes));
    CK(hipMemset(big, 0x3c, 8 * bytes));

    RKArgs r{};
    for (int i = 0; i < 8; i++) r.in[i] = sep[i];
    r.out = out;
    r.nvec = nvec;
    r.trunc_from = nvec * 4;
    RKArgs rc = r;  // contiguous inputs in one allocation
    for (int i = 0; i < 8; i++) rc.in[i] = reinterpret_cast<char*>(big) + i * bytes;
    const double b = (double)bytes;

    if (skew_mode) {  // the multi-stream read penalty vs per-input offsets
        add_readk<8>(vs, r, out, b, "");
        add_readk<2>(vs, r, out, b, "");
        for (uint64_t sk : {1ull, 64ull, 256ull, 1024ull, 1024ull * 7 + 1, 65536ull * 3 + 17})
            add_skew<8>(vs, r, out, b, sk, false);
        add_fan(vs, r, 8, b, "");
        for (uint64_t sk : {0ull, 1024ull, 1024ull * 7 + 1, 65536ull * 3 + 17}) add_skew<8>(vs, r, out, b, sk, true);
        return run(vs, s, rounds, reps, mib);
    }
    if (pipe_mode) {
        add_fan(vs, r, 8, b, "");
        for (unsigned g : {256u, 512u, 1024u, 2048u}) add_pipe<8, 1024>(vs, r, g, b);
        for (unsigned g : {512u, 1024u, 2048u, 4096u}) add_pipe<8, 256>(vs, r, g, b);
        add_readk<8>(vs, r, out, b, "");
        // correctness (all inputs equal bytes -> 8 * x)
        std::vector<float> h(4096), x(4096);
        CK(hipMemcpy(x.data(), sep[0], 4096 * 4, hipMemcpyDeviceToHost));
        hipLaunchKernelGGL((pipe_kernel<8, 1024>), dim3(512), dim3(1024), 0, s, r);
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(h.data(), out, 4096 * 4, hipMemcpyDeviceToHost));
        float e = x[0];
        for (int i = 1; i < 8; i++) e = e + x[0];
        int bad = 0;
        for (int i = 0; i < 4096; i++) bad += (h[i] != e);
        fprintf(stderr, "pipe fan check: %d mismatches\n", bad);
        return run(vs, s, rounds, reps, mib);
    }
    add_readk<8>(vs, r, out, b, "");
    add_readk<2>(vs, r, out, b, "");
    add_readk<8>(vs, rc, out, b, " contiguous-alloc");
    add_im<8, 1, 4, 1024, false>(vs, r, out, b);
    add_im<8, 1, 8, 1024, false>(vs, r, out, b);
    add_im<8, 2, 2, 1024, false>(vs, r, out, b);
    add_im<8, 2, 4, 1024, false>(vs, r, out, b);
    add_im<8, 1, 8, 512, false>(vs, r, out, b);
    add_im<8, 1, 16, 256, false>(vs, r, out, b);
    add_fan(vs, r, 8, b, "");
    add_fan(vs, rc, 8, b, " contiguous-alloc");
    add_im<8, 1, 4, 1024, true>(vs, r, out, b);
    add_im<8, 1, 8, 1024, true>(vs, r, out, b);
    add_im<8, 2, 2, 1024, true>(vs, r, out, b);
    add_im<8, 2, 4, 1024, true>(vs, r, out, b);
    add_im<8, 4, 2, 1024, true>(vs, r, out, b);
    add_im<8, 1, 8, 512, true>(vs, r, out, b);
    add_im<8, 8, 1, 1024, true>(vs, r, out, b);  // == all-at-once through the same code

    // correctness of the input-major fan (all inputs equal -> 8 * x)
    {
        std::vector<float> h(4096), x(4096);
        CK(hipMemcpy(x.data(), sep[0], 4096 * 4, hipMemcpyDeviceToHost));
        hipLaunchKernelGGL((im_kernel<8, 2, 4, 1024, true>), dim3((unsigned)(nvec / 4096)), dim3(1024), 0, s, r, out);
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(h.data(), out, 4096 * 4, hipMemcpyDeviceToHost));
        float e = x[0];
        for (int i = 1; i < 8; i++) e = e + x[0];
        int bad = 0;
        for (int i = 0; i < 4096; i++) bad += (h[i] != e);
        fprintf(stderr, "input-major fan check: %d mismatches\n", bad);
    }
    return run(vs, s, rounds, reps, mib);
}
