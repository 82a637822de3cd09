// lds_stage_sweep.hip — experiment: does staging the inputs through LDS pay
// for the element-wise reduce?
//
// The north star suggests LDS staging for the bf16/fp16 -> fp32 accumulate.
// The library kernels load each lane's 16-byte vectors straight into VGPRs
// (no element ever crosses lanes).  Here the same tiles go
// through LDS by gfx950's LDS-DMA (`global_load_lds_dwordx4`, no VGPR
// destination, cdna_hip_programming.md §5 'Async global->LDS copy'), then
// `ds_read_b128` into the same fold the library runs (fold_row / the fan-in
// fold), then the same non-temporal store.  Each wave reads back only the
// bytes its own DMA wrote, so a `vmcnt(0)` wait is the whole handshake (no
// barrier).  Every variant's output is compared bit for bit with the
// library kernel's on the same inputs before timing.
//
// Variants, interleaved rounds in one process:
//   C3 bf16 sum (avx512bf: RNE)  library reduce2_kernel  vs  LDS-DMA, 1024 / 512 lanes
//   C3 fp16 sum (f16c)           library reduce2_kernel  vs  LDS-DMA, 1024 / 512 lanes
//   C2 fp32 sum                  library reduce2_kernel  vs  LDS-DMA, 1024 / 512 lanes
//   C4 fp32 8-input fan-in       library fan_kernel      vs  LDS-DMA, 512 / 256 / 128 lanes,
//                                and the register path at 256 lanes with and without LDS-capped occupancy
//
//   lds_stage_sweep [C2/C4 bucket_MiB=1024] [rounds=4] [reps=8]   (C3 uses a quarter of the bucket)
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

typedef __attribute__((address_space(1))) void gvoid;
typedef __attribute__((address_space(3))) void lvoid;
constexpr int kDmaAux = 2;  // nt, as the library's loads

__device__ __forceinline__ void dma16(const u32x4* g, u32x4* l) {
    __builtin_amdgcn_global_load_lds((gvoid*)g, (lvoid*)l, 16, 0, kDmaAux);
}

// 2-input reduce, one 16-byte vector per lane per input, staged through LDS.
// Whole tiles only (the host checks nvec % B == 0 and head == tail == 0).
template <typename Tag, int OP, unsigned V, int B>
__global__ __launch_bounds__(B) void reduce2_lds_kernel(R2Args a) {
    using S = typename Tr<Tag>::S;
    constexpr int N = 16 / sizeof(S);
    __shared__ u32x4 lds[2 * B];
    const uint64_t v = (uint64_t)blockIdx.x * B + threadIdx.x;
    const u32x4* p0 = static_cast<const u32x4*>(a.acc) + v;
    const u32x4* p1 = static_cast<const u32x4*>(a.in) + v;
    dma16(p0, &lds[threadIdx.x]);
    dma16(p1, &lds[B + threadIdx.x]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const u32x4 x[2] = {lds[threadIdx.x], lds[B + threadIdx.x]};
    const u32x4 r = fold_row<Tag, OP, V, 2>(x, 2, v * N, a.trunc_from, [&](u32x4 (&y)[2]) {
        y[0] = vload<3>(p0);
        y[1] = vload<3>(p1);
    });
    vstore<3>(static_cast<u32x4*>(a.out) + v, r);
}

// K-input fan-in staged through LDS, the library's fold (fold_row: left fold
// in the reference's order, x86 NaN rule on the rare NaN row).
template <typename Tag, int OP, unsigned V, int K, int B>
__global__ __launch_bounds__(B) void fan_lds_kernel(RKArgs a) {
    using S = typename Tr<Tag>::S;
    constexpr int N = 16 / sizeof(S);
    __shared__ u32x4 lds[K * B];
    const uint64_t v = (uint64_t)blockIdx.x * B + threadIdx.x;
#pragma unroll
    for (int i = 0; i < K; i++) dma16(static_cast<const u32x4*>(a.in[i]) + v, &lds[i * B + threadIdx.x]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    u32x4 x[K];
#pragma unroll
    for (int i = 0; i < K; i++) x[i] = lds[i * B + threadIdx.x];
    vstore<3>(static_cast<u32x4*>(a.out) + v, fold_row<Tag, OP, V, K>(x, K, v * N, a.trunc_from, [&](u32x4 (&y)[K]) {
#pragma unroll
                  for (int i = 0; i < K; i++) y[i] = vload<3>(static_cast<const u32x4*>(a.in[i]) + v);
              }));
}

__global__ void fill_kernel(uint32_t* p, uint64_t nwords, uint32_t seed, uint32_t mask, uint32_t bits) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nwords; i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t h = (uint32_t)i * 0x9E3779B1u ^ seed;
        h ^= h >> 15;
        h *= 0x2C1B3C6Du;
        h ^= h >> 12;
        p[i] = (h & mask) | bits;  // finite normal values of the storage type
    }
}

__global__ void count_diff(const uint32_t* a, const uint32_t* b, uint64_t nwords, unsigned long long* bad) {
    unsigned long long n = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nwords; i += (uint64_t)gridDim.x * blockDim.x)
        n += a[i] != b[i];
    if (n) atomicAdd(bad, n);
}

struct Variant {
    std::string name;
    double traffic;
    std::function<void(hipStream_t)> run;
    void* out;  // checked against ref (nullptr: the reference itself)
    void* ref;
    size_t bytes;
    std::vector<float> ms;
};

template <typename Tag, unsigned V>
void add_pair(std::vector<Variant>& vs, const char* label, void* acc, void* in, void* out_lib, void* out_lds,
              size_t bytes, const uint64_t count) {
    R2Args r{};
    r.acc = acc;
    r.in = in;
    r.nvec = bytes / 16;
    r.trunc_from = count;
    R2Args rl = r;
    rl.out = out_lib;
    const unsigned blocks = (unsigned)(r.nvec / 1024);
    vs.push_back({std::string(label) + " library reduce2_kernel 1024x1", 3.0 * bytes, [rl, blocks](hipStream_t s) {
                      hipLaunchKernelGGL((reduce2_kernel<Tag, OP_SUM, V, 1, 1024>), dim3(blocks), dim3(1024), 0, s, rl);
                  }, nullptr, nullptr, bytes, {}});
    R2Args rd = r;
    rd.out = out_lds;
    vs.push_back({std::string(label) + " LDS-DMA staged 1024x1", 3.0 * bytes, [rd, blocks](hipStream_t s) {
                      hipLaunchKernelGGL((reduce2_lds_kernel<Tag, OP_SUM, V, 1024>), dim3(blocks), dim3(1024), 0, s, rd);
                  }, out_lds, out_lib, bytes, {}});
    vs.push_back({std::string(label) + " LDS-DMA staged 512x1", 3.0 * bytes, [rd, blocks](hipStream_t s) {
                      hipLaunchKernelGGL((reduce2_lds_kernel<Tag, OP_SUM, V, 512>), dim3(blocks * 2), dim3(512), 0, s, rd);
                  }, out_lds, out_lib, bytes, {}});
}

template <int B>
void add_fan_reg(std::vector<Variant>& vs, KArgs k, unsigned blocks, unsigned lds_bytes, size_t bytes, void* out,
                 void* ref) {
    k.out = out;
    char name[160];
    snprintf(name, sizeof name, "C4 fp32 8-input 1 GiB: registers fan_kernel %dx1%s", B,
             lds_bytes ? (", + " + std::to_string(lds_bytes / 1024) + " KiB idle LDS per block").c_str() : "");
    vs.push_back({name, 9.0 * bytes, [k, blocks, lds_bytes](hipStream_t st) {
                      hipLaunchKernelGGL((fan_kernel<float, OP_SUM, 0u, B, 8>), dim3(blocks), dim3(B), lds_bytes, st, k);
                  }, out, ref, bytes, {}});
}

// 2-input: the library kernel holding as much idle LDS as the LDS-DMA kernel
template <typename Tag, unsigned V>
void add_reg_capped(std::vector<Variant>& vs, const char* label, void* acc, void* in, void* out, void* ref,
                    size_t bytes, uint64_t count) {
    R2Args r{};
    r.acc = acc;
    r.in = in;
    r.out = out;
    r.nvec = bytes / 16;
    r.trunc_from = count;
    const unsigned blocks = (unsigned)(r.nvec / 1024);
    vs.push_back({std::string(label) + " library reduce2_kernel 1024x1 + 32 KiB idle LDS", 3.0 * bytes,
                  [r, blocks](hipStream_t s) {
                      hipLaunchKernelGGL((reduce2_kernel<Tag, OP_SUM, V, 1, 1024>), dim3(blocks), dim3(1024), 32768, s, r);
                  }, out, ref, bytes, {}});
}

int main(int argc, char** argv) {
    const size_t mib = argc > 1 ? strtoull(argv[1], nullptr, 10) : 1024;
    const int rounds = argc > 2 ? atoi(argv[2]) : 4;
    const int reps = argc > 3 ? atoi(argv[3]) : 8;
    const size_t bytes = mib << 20, bytes3 = bytes / 4;
    if (bytes3 % (16 * 1024) != 0) {
        fprintf(stderr, "bucket must be a multiple of 64 MiB\n");
        return 2;
    }
    std::vector<void*> buf(11);
    for (auto& p : buf) CK(hipMalloc(&p, bytes));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    // inputs: finite normal values (fp32 [1,2); bf16/fp16 halves in [2^-?, 4))
    for (int i = 0; i < 8; i++)
        hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, s, (uint32_t*)buf[i], bytes / 4, 0xA0u + i,
                           0x007FFFFFu, 0x3F800000u);
    void* lp_a = buf[8];  // bf16/fp16 operands in their own buffers
    void* lp_b = buf[9];
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, s, (uint32_t*)lp_a, bytes3 / 4, 0x1234u, 0x3FFF3FFFu,
                       0x3C003C00u);
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, s, (uint32_t*)lp_b, bytes3 / 4, 0x4321u, 0x3FFF3FFFu,
                       0x3C003C00u);
    void* out_lib = buf[10];
    void* out_lds = static_cast<char*>(buf[9]) + bytes / 2;  // spare halves of the LP buffers
    void* out_lib3 = static_cast<char*>(buf[8]) + bytes / 2;
    CK(hipStreamSynchronize(s));

    std::vector<Variant> vs;
    add_pair<bf16_tag, V_BF16_RNE>(vs, "C3 bf16 sum 256 MiB:", lp_a, lp_b, out_lib3, out_lds, bytes3, bytes3 / 2);
    add_pair<fp16_tag, 0u>(vs, "C3 fp16 sum 256 MiB:", lp_a, lp_b, out_lib3, out_lds, bytes3, bytes3 / 2);
    add_reg_capped<fp16_tag, 0u>(vs, "C3 fp16 sum 256 MiB:", lp_a, lp_b, out_lds, out_lib3, bytes3, bytes3 / 2);
    // C2 in its own output buffers: out-of-place so every rep sees the same inputs
    void* c2_lds = buf[7];  // fan input 7 is refilled after the C2 variants' check (below)
    add_pair<float, 0u>(vs, "C2 fp32 sum 1 GiB:", buf[0], buf[1], out_lib, c2_lds, bytes, bytes / 4);

    std::vector<Variant> fan;
    {
        KArgs k{};
        for (int i = 0; i < 8; i++) k.in[i] = buf[i];
        k.out = out_lib;
        k.k = 8;
        k.count = bytes / 4;
        k.nvec = bytes / 16;
        k.trunc_from = k.count;
        const unsigned blocks = (unsigned)(k.nvec / 1024);
        fan.push_back({"C4 fp32 8-input 1 GiB: library fan_kernel 1024x1", 9.0 * bytes, [k, blocks](hipStream_t st) {
                           hipLaunchKernelGGL((fan_kernel<float, OP_SUM, 0u, 1024, 8>), dim3(blocks), dim3(1024), 0, st,
                                              k);
                       }, nullptr, nullptr, bytes, {}});
        RKArgs r{};
        for (int i = 0; i < 8; i++) r.in[i] = buf[i];
        r.out = buf[8];  // a whole 1 GiB buffer (the LP inputs are done by then)
        r.nvec = k.nvec;
        r.trunc_from = k.count;
        // the library's register kernel at the LDS variants' block sizes, alone
        // and holding as much (unused) LDS as the LDS-DMA kernel of that size
        // (the same blocks per CU), to tell staging from occupancy
        add_fan_reg<128>(fan, k, blocks * 8, 0, bytes, buf[8], out_lib);
        add_fan_reg<128>(fan, k, blocks * 8, 8 * 128 * 16, bytes, buf[8], out_lib);
        add_fan_reg<256>(fan, k, blocks * 4, 8 * 256 * 16, bytes, buf[8], out_lib);
        fan.push_back({"C4 fp32 8-input 1 GiB: LDS-DMA staged 512x1", 9.0 * bytes, [r, blocks](hipStream_t st) {
                           hipLaunchKernelGGL((fan_lds_kernel<float, OP_SUM, 0u, 8, 512>), dim3(blocks * 2), dim3(512), 0,
                                              st, r);
                       }, buf[8], out_lib, bytes, {}});
        fan.push_back({"C4 fp32 8-input 1 GiB: LDS-DMA staged 256x1", 9.0 * bytes, [r, blocks](hipStream_t st) {
                           hipLaunchKernelGGL((fan_lds_kernel<float, OP_SUM, 0u, 8, 256>), dim3(blocks * 4), dim3(256), 0,
                                              st, r);
                       }, buf[8], out_lib, bytes, {}});
        fan.push_back({"C4 fp32 8-input 1 GiB: LDS-DMA staged 128x1", 9.0 * bytes, [r, blocks](hipStream_t st) {
                           hipLaunchKernelGGL((fan_lds_kernel<float, OP_SUM, 0u, 8, 128>), dim3(blocks * 8), dim3(128), 0,
                                              st, r);
                       }, buf[8], out_lib, bytes, {}});
        fan.push_back({"C4 fp32 8-input 1 GiB: LDS-DMA staged 64x1", 9.0 * bytes, [r, blocks](hipStream_t st) {
                           hipLaunchKernelGGL((fan_lds_kernel<float, OP_SUM, 0u, 8, 64>), dim3(blocks * 16), dim3(64), 0,
                                              st, r);
                       }, buf[8], out_lib, bytes, {}});
    }

    unsigned long long* bad;
    CK(hipMalloc(&bad, sizeof(*bad)));
    auto check_group = [&](std::vector<Variant>& g) {
        for (auto& v : g) {
            v.run(s);
            if (v.out) {
                CK(hipMemsetAsync(bad, 0, sizeof(*bad), s));
                hipLaunchKernelGGL(count_diff, dim3(4096), dim3(256), 0, s, (const uint32_t*)v.out,
                                   (const uint32_t*)v.ref, v.bytes / 4, bad);
                unsigned long long h = 0;
                CK(hipMemcpyAsync(&h, bad, sizeof(h), hipMemcpyDeviceToHost, s));
                CK(hipStreamSynchronize(s));
                fprintf(stderr, "check %-60s mismatching words: %llu\n", v.name.c_str(), h);
                if (h) exit(3);
            }
            CK(hipStreamSynchronize(s));
        }
    };
    // the C4 outputs overwrite buf[8] (the LP inputs): check and time the
    // 2-input variants first, then the fan-in group
    check_group(vs);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto time_group = [&](std::vector<Variant>& g) {
        for (int r = 0; r < rounds; r++) {
            for (auto& v : g)
                for (int i = 0; i < reps; i++) {
                    CK(hipEventRecord(e0, s));
                    v.run(s);
                    CK(hipEventRecord(e1, s));
                    CK(hipEventSynchronize(e1));
                    float ms = 0;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    v.ms.push_back(ms);
                }
            fprintf(stderr, "round %d/%d done\n", r + 1, rounds);
        }
    };
    time_group(vs);
    // refill input 7 (C2's LDS output went there) before the fan-in group
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, s, (uint32_t*)buf[7], bytes / 4, 0xA7u, 0x007FFFFFu,
                       0x3F800000u);
    check_group(fan);
    time_group(fan);
    vs.insert(vs.end(), fan.begin(), fan.end());
    for (auto& v : vs) {
        std::sort(v.ms.begin(), v.ms.end());
        const float med = v.ms[v.ms.size() / 2], best = v.ms.front();
        printf("{\"variant\": \"%s\", \"bytes_per_launch\": %.0f, \"median_ms\": %.5f, \"best_ms\": %.5f, "
               "\"median_TBps\": %.3f, \"best_TBps\": %.3f, \"frac_of_8TBps\": %.4f, \"bit_exact_vs_library\": %s}\n",
               v.name.c_str(), v.traffic, med, best, v.traffic / (med * 1e-3) / 1e12, v.traffic / (best * 1e-3) / 1e12,
               v.traffic / (med * 1e-3) / 8e12, v.out ? "true" : "null");
    }
    for (auto& p : buf) CK(hipFree(p));
    return 0;
}
