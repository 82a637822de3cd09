// burst_sweep.hip — bounded experiment (VERDICT r1 "next" #6): do longer
// read-only phases at the DRAM help the write side of C2 (2-input) and C4
// (8-input fan-in)?
//
// The library's kernels (reduce2_kernel, fan_kernel) are one-shot: every
// block reads its tile and stores it at once, so reads and writes of the
// whole chip interleave at the granularity of one 16 KiB tile.  Here a
// persistent grid of G workgroups walks its contiguous share of the bucket in
// rounds of T tiles: it reads and folds T tiles first, holding each lane's T
// result vectors in registers, then stores the T results back to back (one
// burst of T x 16 KiB per workgroup).  Keeping the results in VGPRs is the
// same burst as staging them through LDS (160 KiB/CU holds ~9 tiles of
// 16 KiB) without the LDS round trip.  With T = 8 and G = 256..2048 the DRAM
// sees read phases of 8 tiles per workgroup between write bursts.
//
// Variants, interleaved rounds in one process; HIP-event time per launch.
//   burst_sweep [bucket_MiB=1024] [rounds=3] [reps=6]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "../oneccl_amd/csrc/reduce_kernels.hpp"

using namespace mi;

#define CK(x)                                                                                \
    do {                                                                                     \
        hipError_t e = (x);                                                                  \
        if (e != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                                         \
        }                                                                                    \
    } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));

// fp32 sum of K inputs, persistent: workgroup w owns tiles [w*per, (w+1)*per)
// of B vectors each and processes them T at a time (reads, then one burst of
// T stores).  nvec must be a multiple of B (1 GiB buckets are).
template <int K, int B, int T>
__global__ __launch_bounds__(B) void burst_kernel(RKArgs a, uint64_t tiles_per_wg) {
    const uint64_t ntiles = a.nvec / B;
    const uint64_t t_begin = (uint64_t)blockIdx.x * tiles_per_wg;
    const uint64_t t_end = t_begin + tiles_per_wg < ntiles ? t_begin + tiles_per_wg : ntiles;
    const u32x4* in[K];
#pragma unroll
    for (int j = 0; j < K; j++) in[j] = reinterpret_cast<const u32x4*>(a.in[j]);
    u32x4* out = reinterpret_cast<u32x4*>(a.out);
    for (uint64_t t0 = t_begin; t0 < t_end; t0 += T) {
        u32x4 res[T];
#pragma unroll
        for (int t = 0; t < T; t++) {
            const uint64_t v = (t0 + t) * B + threadIdx.x;
            if (t0 + t < t_end) {
                f32x4 acc = __builtin_bit_cast(f32x4, __builtin_nontemporal_load(in[0] + v));
#pragma unroll
                for (int j = 1; j < K; j++) acc += __builtin_bit_cast(f32x4, __builtin_nontemporal_load(in[j] + v));
                res[t] = __builtin_bit_cast(u32x4, acc);
            }
        }
#pragma unroll
        for (int t = 0; t < T; t++)
            if (t0 + t < t_end) __builtin_nontemporal_store(res[t], out + (t0 + t) * B + threadIdx.x);
    }
}

struct Variant {
    std::string name;
    double traffic;
    std::function<void(hipStream_t)> run;
    std::vector<float> ms;
};

template <int K, int B, int T>
void add_burst(std::vector<Variant>& vs, const RKArgs& r, unsigned grid, double bucket) {
    const uint64_t ntiles = r.nvec / B;
    const uint64_t per = (ntiles + grid - 1) / grid;
    char name[160];
    snprintf(name, sizeof name, "burst K=%d B=%d T=%d grid=%u", K, B, T, grid);
    vs.push_back({name, (K + 1) * bucket, [r, grid, per](hipStream_t s) {
                      hipLaunchKernelGGL((burst_kernel<K, B, T>), dim3(grid), dim3(B), 0, s, r, per);
                  }, {}});
}

int main(int argc, char** argv) {
    const size_t mib = argc > 1 ? strtoull(argv[1], nullptr, 10) : 1024;
    const int rounds = argc > 2 ? atoi(argv[2]) : 3;
    const int reps = argc > 3 ? atoi(argv[3]) : 6;
    const size_t bytes = mib << 20;
    const uint64_t nvec = bytes / 16;
    const double b = (double)bytes;
    hipStream_t s;
    CK(hipStreamCreate(&s));
    std::vector<float*> in(8, nullptr);
    for (auto& p : in) {
        CK(hipMalloc(&p, bytes));
        CK(hipMemset(p, 0x3c, bytes));
    }
    float *out, *ref;
    CK(hipMalloc(&out, bytes));
    CK(hipMalloc(&ref, bytes));

    std::vector<Variant> vs;
    // the library's kernels, same process (baselines)
    R2Args r2{};
    r2.acc = in[0];
    r2.in = in[1];
    r2.out = out;
    r2.nvec = nvec;
    r2.trunc_from = nvec * 4;
    vs.push_back({"library reduce2_kernel (C2, one-shot)", 3 * b, [r2](hipStream_t st) {
                      hipLaunchKernelGGL((reduce2_kernel<float, OP_SUM, 0u, 1, 1024>), dim3((unsigned)(r2.nvec / 1024)),
                                         dim3(1024), 0, st, r2);
                  }, {}});
    KArgs f{};
    for (int i = 0; i < 8; i++) f.in[i] = in[i];
    f.out = out;
    f.k = 8;
    f.nvec = nvec;
    f.count = nvec * 4;
    f.trunc_from = nvec * 4;
    vs.push_back({"library fan_kernel (C4, one-shot)", 9 * b, [f](hipStream_t st) {
                      hipLaunchKernelGGL((fan_kernel<float, OP_SUM, 0u, 1024, 8>), dim3((unsigned)(f.nvec / 1024)),
                                         dim3(1024), 0, st, f);
                  }, {}});
    RKArgs r{};
    for (int i = 0; i < 8; i++) r.in[i] = in[i];
    r.out = out;
    r.nvec = nvec;
    r.trunc_from = nvec * 4;
    for (unsigned g : {256u, 512u, 1024u, 2048u}) {
        add_burst<2, 1024, 1>(vs, r, g, b);
        add_burst<2, 1024, 4>(vs, r, g, b);
        add_burst<2, 1024, 8>(vs, r, g, b);
        add_burst<8, 1024, 1>(vs, r, g, b);
        add_burst<8, 1024, 4>(vs, r, g, b);
        add_burst<8, 1024, 8>(vs, r, g, b);
    }
    for (unsigned g : {512u, 1024u, 2048u}) {
        add_burst<2, 512, 8>(vs, r, g, b);
        add_burst<8, 512, 8>(vs, r, g, b);
    }

    // correctness: burst results == the library kernels' (fp32 sums of equal inputs)
    for (int K : {2, 8}) {
        if (K == 2)
            hipLaunchKernelGGL((reduce2_kernel<float, OP_SUM, 0u, 1, 1024>), dim3((unsigned)(nvec / 1024)), dim3(1024),
                               0, s, R2Args{in[0], in[1], ref, nvec, 0, 0, nvec * 4});
        else {
            KArgs g = f;
            g.out = ref;
            hipLaunchKernelGGL((fan_kernel<float, OP_SUM, 0u, 1024, 8>), dim3((unsigned)(nvec / 1024)), dim3(1024), 0,
                               s, g);
        }
        CK(hipMemsetAsync(out, 0, bytes, s));
        const uint64_t per = (nvec / 1024 + 511) / 512;
        if (K == 2)
            hipLaunchKernelGGL((burst_kernel<2, 1024, 8>), dim3(512), dim3(1024), 0, s, r, per);
        else
            hipLaunchKernelGGL((burst_kernel<8, 1024, 8>), dim3(512), dim3(1024), 0, s, r, per);
        CK(hipStreamSynchronize(s));
        std::vector<uint32_t> h1(1 << 20), h2(1 << 20);
        size_t bad = 0;
        for (size_t off = 0; off < bytes; off += (size_t)64 << 20) {  // sample 4 MiB every 64 MiB
            CK(hipMemcpy(h1.data(), reinterpret_cast<char*>(out) + off, 4 << 20, hipMemcpyDeviceToHost));
            CK(hipMemcpy(h2.data(), reinterpret_cast<char*>(ref) + off, 4 << 20, hipMemcpyDeviceToHost));
            for (size_t i = 0; i < h1.size(); i++) bad += h1[i] != h2[i];
        }
        fprintf(stderr, "burst K=%d check: %zu mismatching words (sampled)\n", K, bad);
        if (bad) return 3;
    }

    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (auto& v : vs) v.run(s);
    CK(hipStreamSynchronize(s));
    CK(hipGetLastError());
    for (int rr = 0; rr < rounds; rr++) {
        for (auto& v : vs)
            for (int i = 0; i < reps; i++) {
                CK(hipEventRecord(e0, s));
                v.run(s);
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                v.ms.push_back(ms);
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
