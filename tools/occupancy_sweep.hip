// occupancy_sweep.hip — experiment: block size and resident waves per CU for
// the library's streaming kernels.
//
// tools/lds_stage_sweep.hip found the 8-input fan-in 2.6 % faster at 128-lane
// blocks than at the library's 1024, and 4.3 % faster again when each block
// also held 16 KiB of idle LDS (10 blocks = 20 waves per CU instead of 32),
// while staging the inputs through LDS itself gained nothing.  Here every
// (kernel, block size, resident-wave cap) is timed in interleaved rounds.
// The cap is set the way a kernel without LDS traffic can set it: dynamic
// LDS that no instruction touches, sized so floor(160 KiB / bytes) blocks fit
// on a CU; hipOccupancyMaxActiveBlocksPerMultiprocessor reports what the
// runtime actually grants.  Outputs are checked bit for bit against the
// library's default launch before timing.
//
//   occupancy_sweep [bucket_MiB=1024] [rounds=6] [reps=8] [c2|c3|c4|all|c4bf|fank|fanu|xcd|r2ab|copyconv|pmcset|r2u|copyu|policy|c5ops|gran]   (all = c2, c3, c4)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <type_traits>
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

constexpr unsigned kLdsPerCU = 160 * 1024;

__global__ void fill_kernel(uint32_t* p, uint64_t nwords, uint32_t seed, uint32_t mask, uint32_t bits) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nwords; i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t h = (uint32_t)i * 0x9E3779B1u ^ seed;
        h ^= h >> 15;
        h *= 0x2C1B3C6Du;
        h ^= h >> 12;
        p[i] = (h & mask) | bits;
    }
}

__global__ void count_diff(const uint32_t* a, const uint32_t* b, uint64_t nwords, unsigned long long* bad) {
    unsigned long long n = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nwords; i += (uint64_t)gridDim.x * blockDim.x)
        n += a[i] != b[i];
    if (n) atomicAdd(bad, n);
}

// copy with U 16-byte vectors per lane (all loads before the first store),
// one tile of B*U vectors per block: the shape question for ccl_comp_copy
template <int B, int U>
__global__ __launch_bounds__(B) void copy_u_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                  uint64_t nvec) {
    const uint64_t v0 = (uint64_t)blockIdx.x * B * U + threadIdx.x;
    u32x4 x[U];
#pragma unroll
    for (int j = 0; j < U; j++)
        if (v0 + (uint64_t)j * B < nvec) x[j] = __builtin_nontemporal_load(src + v0 + (uint64_t)j * B);
#pragma unroll
    for (int j = 0; j < U; j++)
        if (v0 + (uint64_t)j * B < nvec) __builtin_nontemporal_store(x[j], dst + v0 + (uint64_t)j * B);
}

// 2-input fp32 sum through buffer ops with the cache-policy bits as template
// arguments (aux: bit 0 sc0, bit 1 nt, bit 4 sc1), one-wave tiles
template <int LA, int SA>
__global__ __launch_bounds__(64) void r2pol_kernel(const void* in, void* io, uint64_t nvec) {
    const uint64_t t0 = (uint64_t)blockIdx.x * 64;
    if (t0 >= nvec) return;
    const uint32_t bytes = (uint32_t)std::min<uint64_t>(nvec - t0, 64) * 16u;
    const uint32_t off = threadIdx.x * 16u;
    const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(tile_rsrc(io, t0 * 16, bytes), off, 0, LA);
    const u32x4 b = __builtin_amdgcn_raw_buffer_load_b128(tile_rsrc(in, t0 * 16, bytes), off, 0, LA);
    u32x4 r;
#pragma unroll
    for (int e = 0; e < 4; e++) r[e] = __float_as_uint(__uint_as_float(a[e]) + __uint_as_float(b[e]));
    __builtin_amdgcn_raw_buffer_store_b128(r, tile_rsrc(io, t0 * 16, bytes), off, 0, SA);
}

// 8-input fp32 sum fan-in through buffer ops, store policy as a template argument
template <int SA>
__global__ __launch_bounds__(64) void fanpol_kernel(KArgs a) {
    const uint64_t t0 = (uint64_t)blockIdx.x * 64;
    if (t0 >= a.nvec) return;
    const uint32_t bytes = (uint32_t)std::min<uint64_t>(a.nvec - t0, 64) * 16u;
    const uint32_t off = threadIdx.x * 16u;
    u32x4 x[8];
#pragma unroll
    for (int i = 0; i < 8; i++) x[i] = __builtin_amdgcn_raw_buffer_load_b128(tile_rsrc(a.in[i], t0 * 16, bytes), off, 0, 2);
    u32x4 r = x[0];
#pragma unroll
    for (int i = 1; i < 8; i++)
#pragma unroll
        for (int e = 0; e < 4; e++) r[e] = __float_as_uint(__uint_as_float(x[i][e]) + __uint_as_float(r[e]));
    __builtin_amdgcn_raw_buffer_store_b128(r, tile_rsrc(a.out, t0 * 16, bytes), off, 0, SA);
}

// copy through buffer ops, store policy as a template argument, one-wave tiles
template <int SA>
__global__ __launch_bounds__(64) void copypol_kernel(const void* src, void* dst, uint64_t nvec) {
    const uint64_t t0 = (uint64_t)blockIdx.x * 64;
    if (t0 >= nvec) return;
    const uint32_t bytes = (uint32_t)std::min<uint64_t>(nvec - t0, 64) * 16u;
    const uint32_t off = threadIdx.x * 16u;
    const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(tile_rsrc(src, t0 * 16, bytes), off, 0, 2);
    __builtin_amdgcn_raw_buffer_store_b128(x, tile_rsrc(dst, t0 * 16, bytes), off, 0, SA);
}

// the same fan-in with global (flat) loads and stores, guarded per lane
template <int NTST>
__global__ __launch_bounds__(64) void fanglob_kernel(KArgs a) {
    const uint64_t v = (uint64_t)blockIdx.x * 64 + threadIdx.x;
    if (v >= a.nvec) return;
    u32x4 x[8];
#pragma unroll
    for (int i = 0; i < 8; i++) x[i] = __builtin_nontemporal_load(static_cast<const u32x4*>(a.in[i]) + v);
    u32x4 r = x[0];
#pragma unroll
    for (int i = 1; i < 8; i++)
#pragma unroll
        for (int e = 0; e < 4; e++) r[e] = __float_as_uint(__uint_as_float(x[i][e]) + __uint_as_float(r[e]));
    if (NTST)
        __builtin_nontemporal_store(r, static_cast<u32x4*>(a.out) + v);
    else
        static_cast<u32x4*>(a.out)[v] = r;
}

// the 8-input fp32 sum fan-in with U vectors per lane: one wave owns a tile
// of 64*U vectors of every input (U KiB contiguous per stream), the lane's
// j-th vector at tile + j*64 + lane.  IM: loads issued input-major (each
// stream's U requests back to back) instead of vector-major.
template <int U, bool IM>
__global__ __launch_bounds__(64) void fanu_kernel(KArgs a) {
    const uint64_t t0 = (uint64_t)blockIdx.x * 64 * U;
    if (t0 >= a.nvec) return;
    const uint32_t bytes = (uint32_t)std::min<uint64_t>(a.nvec - t0, 64 * U) * 16u;
    const uint32_t off = threadIdx.x * 16u;
    const void* in[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        in[i] = a.in[i];
        asm volatile("" ::"s"(in[i]));
    }
    u32x4 x[8][U];
    if (IM) {
#pragma unroll
        for (int i = 0; i < 8; i++)
#pragma unroll
            for (int j = 0; j < U; j++)
                x[i][j] = __builtin_amdgcn_raw_buffer_load_b128(tile_rsrc(in[i], t0 * 16, bytes), off + j * 1024u, 0, 2);
    } else {
#pragma unroll
        for (int j = 0; j < U; j++)
#pragma unroll
            for (int i = 0; i < 8; i++)
                x[i][j] = __builtin_amdgcn_raw_buffer_load_b128(tile_rsrc(in[i], t0 * 16, bytes), off + j * 1024u, 0, 2);
    }
#pragma unroll
    for (int j = 0; j < U; j++) {
        u32x4 r = x[0][j];
#pragma unroll
        for (int i = 1; i < 8; i++)
#pragma unroll
            for (int e = 0; e < 4; e++) r[e] = __float_as_uint(__uint_as_float(x[i][j][e]) + __uint_as_float(r[e]));
        __builtin_amdgcn_raw_buffer_store_b128(r, tile_rsrc(a.out, t0 * 16, bytes), off + j * 1024u, 0, kAuxNT);
    }
}

// Workgroups are handed to the 8 XCDs round robin (block b -> XCD b % 8).
// remap_tile gives XCD x runs of G consecutive tiles: the j-th block an XCD
// receives takes tile (j / G) * 8G + x * G + j % G (G = 1: the identity).
// nblocks must be a multiple of 8G.
__device__ __forceinline__ uint64_t remap_tile(uint64_t b, uint64_t G) {
    const uint64_t x = b & 7, j = b >> 3;
    return (j / G) * 8 * G + x * G + j % G;
}

// 2-input fp32 sum in place with the library's cache policy (nt loads,
// sc1 + nt stores), tiles remapped per XCD
__global__ __launch_bounds__(64) void r2xcd_kernel(const void* in, void* io, uint64_t nvec, uint64_t G) {
    const uint64_t t0 = remap_tile(blockIdx.x, G) * 64;
    if (t0 >= nvec) return;
    const uint32_t bytes = (uint32_t)std::min<uint64_t>(nvec - t0, 64) * 16u;
    const uint32_t off = threadIdx.x * 16u;
    const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(tile_rsrc(io, t0 * 16, bytes), off, 0, 2);
    const u32x4 b = __builtin_amdgcn_raw_buffer_load_b128(tile_rsrc(in, t0 * 16, bytes), off, 0, 2);
    u32x4 r;
#pragma unroll
    for (int e = 0; e < 4; e++) r[e] = __float_as_uint(__uint_as_float(a[e]) + __uint_as_float(b[e]));
    __builtin_amdgcn_raw_buffer_store_b128(r, tile_rsrc(io, t0 * 16, bytes), off, 0, 18);
}

// 8-input fp32 sum fan-in (nt loads and stores), tiles remapped per XCD
__global__ __launch_bounds__(64) void fanxcd_kernel(KArgs a, uint64_t G) {
    const uint64_t t0 = remap_tile(blockIdx.x, G) * 64;
    if (t0 >= a.nvec) return;
    const uint32_t bytes = (uint32_t)std::min<uint64_t>(a.nvec - t0, 64) * 16u;
    const uint32_t off = threadIdx.x * 16u;
    const void* in[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        in[i] = a.in[i];
        asm volatile("" ::"s"(in[i]));
    }
    u32x4 x[8];
#pragma unroll
    for (int i = 0; i < 8; i++) x[i] = __builtin_amdgcn_raw_buffer_load_b128(tile_rsrc(in[i], t0 * 16, bytes), off, 0, 2);
    u32x4 r = x[0];
#pragma unroll
    for (int i = 1; i < 8; i++)
#pragma unroll
        for (int e = 0; e < 4; e++) r[e] = __float_as_uint(__uint_as_float(x[i][e]) + __uint_as_float(r[e]));
    __builtin_amdgcn_raw_buffer_store_b128(r, tile_rsrc(a.out, t0 * 16, bytes), off, 0, 2);
}

struct Variant {
    std::string name;
    std::string group;
    double traffic;
    std::function<hipError_t(hipStream_t)> run;
    void* out;
    void* ref;  // nullptr: the group's reference launch
    size_t bytes;
    std::vector<float> ms;
};

// dynamic LDS that leaves room for `blocks` blocks per CU (0: none)
unsigned lds_for(int blocks) { return blocks > 0 ? kLdsPerCU / blocks : 0; }

// one variant per (group, kernel, block size, LDS bytes): caps that round to
// the same blocks per CU are timed once
bool seen(const std::string& key) {
    static std::vector<std::string> keys;
    if (std::find(keys.begin(), keys.end(), key) != keys.end()) return true;
    keys.push_back(key);
    return false;
}

template <typename F>
int granted(F kernel, int B, unsigned lds) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, B, lds) != hipSuccess) return -1;
    return nb;
}

template <typename Tag, unsigned V, int B, int U = 1, int OPX = OP_SUM>
void add_r2(std::vector<Variant>& vs, const char* group, R2Args r, size_t bytes, int cap_waves, void* ref) {
    const unsigned blocks = (unsigned)(r.nvec / ((uint64_t)B * U));
    const int waves = B / 64;
    const unsigned lds = cap_waves ? lds_for(cap_waves / waves) : 0;
    if ((cap_waves && cap_waves < waves) || seen(std::string(group) + "r2/" + std::to_string(B) + "x" +
                                                 std::to_string(U) + "/" + std::to_string(lds) + (ref ? "" : "/ref")))
        return;
    auto k = reduce2_kernel<Tag, OPX, V, U, B>;
    const int nb = granted(k, B, lds);
    char name[200];
    snprintf(name, sizeof name, "%s reduce2_kernel<op %d> %dx%d, lds %u B/block -> %d blocks = %d waves per CU", group,
             OPX, B, U, lds, nb, nb * waves);
    vs.push_back({name, group, 3.0 * bytes, [r, blocks, lds](hipStream_t s) {
                      hipLaunchKernelGGL((reduce2_kernel<Tag, OPX, V, U, B>), dim3(blocks), dim3(B), lds, s, r);
                      return hipGetLastError();
                  }, r.out, ref, bytes, {}});
}

template <typename Tag, unsigned V, int B, int KMAX = 8>
void add_fan(std::vector<Variant>& vs, const char* group, KArgs a, size_t bytes, int cap_waves, void* ref) {
    const unsigned blocks = (unsigned)(a.nvec / B);
    const int waves = B / 64;
    const unsigned lds = cap_waves ? lds_for(cap_waves / waves) : 0;
    if ((cap_waves && cap_waves < waves) || seen(std::string(group) + "fan/" + std::to_string(B) + "/" +
                                                 std::to_string(lds) + (ref ? "" : "/ref")))
        return;
    auto k = fan_kernel<Tag, OP_SUM, V, B, KMAX>;
    const int nb = granted(k, B, lds);
    char name[200];
    snprintf(name, sizeof name, "%s fan_kernel %dx1, lds %u B/block -> %d blocks = %d waves per CU", group, B, lds, nb,
             nb * waves);
    vs.push_back({name, group, (a.k + 1.0) * bytes, [a, blocks, lds](hipStream_t s) {
                      hipLaunchKernelGGL((fan_kernel<Tag, OP_SUM, V, B, KMAX>), dim3(blocks), dim3(B), lds, s, a);
                      return hipGetLastError();
                  }, a.out, ref, bytes, {}});
}

// gfx950 allocates LDS in granules of LDS-per-CU / 128 (1280 B of 160 KiB):
// a workgroup reserving `lds` bytes holds ceil(lds / granule) of them, so a
// CU holds 128 / that many one-wave workgroups (tools/residency_probe.hip
// measured it; hipOccupancyMaxActiveBlocksPerMultiprocessor ignores the
// granule).  The one-wave kernels at an exact granule count m: residency
// floor(128 / m), `gran` mode.
constexpr unsigned kGranule = kLdsPerCU / 128;
int resident_of(unsigned lds) { return lds ? (int)std::min(32u, 128u / ((lds + kGranule - 1) / kGranule)) : 32; }

template <typename Tag, unsigned V, int OPX = OP_SUM>
void add_r2_granules(std::vector<Variant>& vs, const char* group, R2Args r, size_t bytes, unsigned m) {
    const unsigned blocks = (unsigned)(r.nvec / 64);
    const unsigned lds = m * kGranule;
    char name[200];
    snprintf(name, sizeof name, "%s reduce2_kernel 64x1, lds %u B = %u granules -> %d waves per CU (measured rule)",
             group, lds, m, resident_of(lds));
    vs.push_back({name, group, 3.0 * bytes, [r, blocks, lds](hipStream_t s) {
                      hipLaunchKernelGGL((reduce2_kernel<Tag, OPX, V, 1, 64>), dim3(blocks), dim3(64), lds, s, r);
                      return hipGetLastError();
                  }, r.out, nullptr, bytes, {}});
}

template <typename Tag, unsigned V>
void add_fan_granules(std::vector<Variant>& vs, const char* group, KArgs a, size_t bytes, unsigned m) {
    const unsigned blocks = (unsigned)(a.nvec / 64);
    const unsigned lds = m * kGranule;
    char name[200];
    snprintf(name, sizeof name, "%s fan_kernel 64x1, lds %u B = %u granules -> %d waves per CU (measured rule)", group,
             lds, m, resident_of(lds));
    vs.push_back({name, group, (a.k + 1.0) * bytes, [a, blocks, lds](hipStream_t s) {
                      hipLaunchKernelGGL((fan_kernel<Tag, OP_SUM, V, 64, 8>), dim3(blocks), dim3(64), lds, s, a);
                      return hipGetLastError();
                  }, a.out, nullptr, bytes, {}});
}

// every block size at every cap (caps a block size cannot meet are skipped)
constexpr int kCaps[] = {0, 24, 20, 16, 12, 8, 6, 4};

template <typename Tag, unsigned V>
void sweep_r2(std::vector<Variant>& vs, const char* group, R2Args r, size_t bytes, void* out_alt) {
    add_r2<Tag, V, 1024>(vs, group, r, bytes, 0, nullptr);  // the library's launch: the reference
    void* ref = r.out;
    r.out = out_alt;
    for (int cap : kCaps) {
        add_r2<Tag, V, 1024>(vs, group, r, bytes, cap, ref);
        add_r2<Tag, V, 512>(vs, group, r, bytes, cap, ref);
        add_r2<Tag, V, 256>(vs, group, r, bytes, cap, ref);
        add_r2<Tag, V, 128>(vs, group, r, bytes, cap, ref);
        add_r2<Tag, V, 64>(vs, group, r, bytes, cap, ref);
    }
}

template <typename Tag, unsigned V>
void sweep_fan(std::vector<Variant>& vs, const char* group, KArgs a, size_t bytes, void* out_alt) {
    add_fan<Tag, V, 1024>(vs, group, a, bytes, 0, nullptr);
    void* ref = a.out;
    a.out = out_alt;
    for (int cap : kCaps) {
        add_fan<Tag, V, 1024>(vs, group, a, bytes, cap, ref);
        add_fan<Tag, V, 128>(vs, group, a, bytes, cap, ref);
        add_fan<Tag, V, 64>(vs, group, a, bytes, cap, ref);
    }
}

int main(int argc, char** argv) {
    const size_t mib = argc > 1 ? strtoull(argv[1], nullptr, 10) : 1024;
    const int rounds = argc > 2 ? atoi(argv[2]) : 6;
    const int reps = argc > 3 ? atoi(argv[3]) : 8;
    const std::string which = argc > 4 ? argv[4] : "all";
    const size_t bytes = mib << 20, bytes3 = bytes / 4;
    if (bytes3 % (64 * 1024) != 0) {
        fprintf(stderr, "bucket must be a multiple of 256 MiB\n");
        return 2;
    }
    std::vector<void*> buf(10);
    for (auto& p : buf) CK(hipMalloc(&p, bytes));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    for (int i = 0; i < 8; i++)
        hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, s, (uint32_t*)buf[i], bytes / 4, 0xA0u + i,
                           0x007FFFFFu, 0x3F800000u);
    CK(hipStreamSynchronize(s));

    std::vector<Variant> vs;
    if (which == "all" || which == "c2") {
        R2Args r{};
        r.acc = buf[0];
        r.in = buf[1];
        r.out = buf[8];
        r.nvec = bytes / 16;
        r.trunc_from = bytes / 4;
        sweep_r2<float, 0u>(vs, "C2 fp32 sum 1 GiB:", r, bytes, buf[9]);
    }
    if (which == "all" || which == "c3") {
        // bf16 operands in buffers of their own
        void *la, *lb;
        CK(hipMalloc(&la, bytes3));
        CK(hipMalloc(&lb, bytes3));
        hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, s, (uint32_t*)la, bytes3 / 4, 0x1234u, 0x3FFF3FFFu,
                           0x3C003C00u);
        hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, s, (uint32_t*)lb, bytes3 / 4, 0x4321u, 0x3FFF3FFFu,
                           0x3C003C00u);
        R2Args r{};
        r.acc = la;
        r.in = lb;
        r.out = static_cast<char*>(buf[8]) + bytes / 2;
        r.nvec = bytes3 / 16;
        r.trunc_from = bytes3 / 2;
        sweep_r2<bf16_tag, V_BF16_RNE>(vs, "C3 bf16 sum 256 MiB:", r, bytes3, static_cast<char*>(buf[9]) + bytes / 2);
    }
    if (which == "all" || which == "c4") {
        KArgs a{};
        for (int i = 0; i < 8; i++) a.in[i] = buf[i];
        a.out = buf[8];
        a.k = 8;
        a.count = bytes / 4;
        a.nvec = bytes / 16;
        a.trunc_from = a.count;
        sweep_fan<float, 0u>(vs, "C4 fp32 8-input 1 GiB:", a, bytes, buf[9]);
        KArgs a4 = a;
        a4.k = 4;
        sweep_fan<float, 0u>(vs, "fan-in fp32 4-input 1 GiB:", a4, bytes, buf[9]);
    }
    if (which == "r2ab") {
        // the 2-input kernel in place (out = the accumulator, as ccl_comp_reduce
        // and the bench run it), a focused set of shapes, per dtype
        void *la, *lb;
        CK(hipMalloc(&la, bytes3));
        CK(hipMalloc(&lb, bytes3));
        hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, s, (uint32_t*)la, bytes3 / 4, 0x1234u, 0x3FFF3FFFu,
                           0x3C003C00u);
        hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, s, (uint32_t*)lb, bytes3 / 4, 0x4321u, 0x3FFF3FFFu,
                           0x3C003C00u);
        auto shapes = [&](auto tag, auto vconst, const char* g, R2Args r, size_t nbytes) {
            using Tag = decltype(tag);
            constexpr unsigned V = decltype(vconst)::value;
            // in place, every variant rewrites the same accumulator: nothing to
            // compare against (the out-of-place modes check the same kernels)
            add_r2<Tag, V, 1024>(vs, g, r, nbytes, 0, nullptr);
            add_r2<Tag, V, 512>(vs, g, r, nbytes, 0, nullptr);
            add_r2<Tag, V, 256>(vs, g, r, nbytes, 0, nullptr);
            add_r2<Tag, V, 128>(vs, g, r, nbytes, 0, nullptr);
            add_r2<Tag, V, 64>(vs, g, r, nbytes, 0, nullptr);
            add_r2<Tag, V, 128>(vs, g, r, nbytes, 24, nullptr);
            add_r2<Tag, V, 64>(vs, g, r, nbytes, 24, nullptr);
            add_r2<Tag, V, 64>(vs, g, r, nbytes, 20, nullptr);
            add_r2<Tag, V, 64>(vs, g, r, nbytes, 16, nullptr);
        };
        R2Args r{};
        r.acc = buf[0];
        r.in = buf[1];
        r.out = buf[0];
        r.nvec = bytes / 16;
        r.trunc_from = bytes / 4;
        shapes(float(), std::integral_constant<unsigned, 0u>(), "C2 fp32 sum 1 GiB in place:", r, bytes);
        R2Args ri = r;
        ri.acc = ri.out = buf[2];
        ri.in = buf[3];
        shapes(int32_t(), std::integral_constant<unsigned, 0u>(), "C5 int32 sum 1 GiB in place:", ri, bytes);
        R2Args rb{};
        rb.acc = rb.out = la;
        rb.in = lb;
        rb.nvec = bytes3 / 16;
        rb.trunc_from = bytes3 / 2;
        shapes(bf16_tag(), std::integral_constant<unsigned, V_BF16_RNE>(), "C3 bf16 sum 256 MiB in place:", rb, bytes3);
        shapes(fp16_tag(), std::integral_constant<unsigned, 0u>(), "C3 fp16 sum 256 MiB in place:", rb, bytes3);
    }
    if (which == "gran") {
        // exact residencies (whole LDS granules): the 2-input kernel in place
        // (fp32, bf16) and the fan-in (8 and 6 inputs), every residency the
        // granules allow from 32 down
        R2Args r{};
        r.acc = r.out = buf[0];
        r.in = buf[1];
        r.nvec = bytes / 16;
        r.trunc_from = bytes / 4;
        for (unsigned m : {0u, 4u, 5u, 6u, 7u, 8u})
            add_r2_granules<float, 0u>(vs, "C2 fp32 sum 1 GiB in place:", r, bytes, m);
        // bf16 operands of their own, every half a finite bf16 (as r2ab fills
        // them): random bits would make NaN/Inf halves common and send rows
        // through the x86 NaN refold
        void *la, *lb;
        CK(hipMalloc(&la, bytes3));
        CK(hipMalloc(&lb, bytes3));
        hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, s, (uint32_t*)la, bytes3 / 4, 0x1234u, 0x3FFF3FFFu,
                           0x3C003C00u);
        hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, s, (uint32_t*)lb, bytes3 / 4, 0x4321u, 0x3FFF3FFFu,
                           0x3C003C00u);
        CK(hipStreamSynchronize(s));
        R2Args rb{};
        rb.acc = rb.out = la;
        rb.in = lb;
        rb.nvec = bytes3 / 16;
        rb.trunc_from = bytes3 / 2;
        for (unsigned m : {0u, 5u, 6u, 7u, 8u})
            add_r2_granules<bf16_tag, V_BF16_RNE>(vs, "C3 bf16 sum 256 MiB in place:", rb, bytes3, m);
        KArgs a{};
        for (int i = 0; i < 8; i++) a.in[i] = buf[i];
        a.out = buf[8];
        a.k = 8;
        a.count = bytes / 4;
        a.nvec = bytes / 16;
        a.trunc_from = a.count;
        for (unsigned m : {8u, 9u, 10u, 11u, 12u, 13u, 15u, 16u, 18u})
            add_fan_granules<float, 0u>(vs, "C4 fp32 8-input 1 GiB:", a, bytes, m);
        KArgs a6 = a;
        a6.k = 6;
        for (unsigned m : {8u, 9u, 10u, 11u, 12u, 13u, 16u})
            add_fan_granules<float, 0u>(vs, "fan-in fp32 6-input 1 GiB:", a6, bytes, m);
    }
    if (which == "c5ops") {
        // the library's 2-input launch over dtypes and ops, same buffers, in place
        auto one = [&](auto tag, auto opc, const char* g, void* acc, void* in, int cap = 24) {
            using Tag = decltype(tag);
            constexpr int OPX = decltype(opc)::value;
            R2Args r{};
            r.acc = r.out = acc;
            r.in = in;
            r.nvec = bytes / 16;
            r.trunc_from = bytes / sizeof(typename Tr<Tag>::S);
            add_r2<Tag, 0u, 64, 1, OPX>(vs, g, r, bytes, cap, nullptr);
        };
        one(float(), std::integral_constant<int, OP_SUM>(), "fp32 sum:", buf[0], buf[1]);
        one(int32_t(), std::integral_constant<int, OP_SUM>(), "int32 sum:", buf[2], buf[3]);
        one(int32_t(), std::integral_constant<int, OP_MAX>(), "int32 max:", buf[4], buf[5]);
        one(int64_t(), std::integral_constant<int, OP_PROD>(), "int64 prod:", buf[6], buf[7]);
        one(int32_t(), std::integral_constant<int, OP_MAX>(), "int32 max (fp32 sum's buffers):", buf[0], buf[1]);
        one(int64_t(), std::integral_constant<int, OP_SUM>(), "int64 sum:", buf[6], buf[7]);
        for (int cap : {28, 32, 0}) one(int64_t(), std::integral_constant<int, OP_PROD>(), "int64 prod:", buf[6], buf[7], cap);
        for (int cap : {28, 32}) one(float(), std::integral_constant<int, OP_PROD>(), "fp32 prod:", buf[0], buf[1], cap);
        one(float(), std::integral_constant<int, OP_PROD>(), "fp32 prod:", buf[0], buf[1], 24);
    }
    if (which == "policy") {
        // cache-policy bits of the one-wave 2-input kernel at 24 waves per CU, in place
        R2Args r{};
        r.acc = r.out = buf[0];
        r.in = buf[1];
        r.nvec = bytes / 16;
        r.trunc_from = bytes / 4;
        add_r2<float, 0u, 64>(vs, "C2 fp32 sum 1 GiB in place:", r, bytes, 24, nullptr);  // the library
        const unsigned lds = lds_for(24);
        const uint64_t nvec = bytes / 16;
        const unsigned blocks = (unsigned)(nvec / 64);
        auto add_pol = [&](auto la, auto sa) {
            constexpr int LA = decltype(la)::value, SA = decltype(sa)::value;
            char name[160];
            snprintf(name, sizeof name, "C2 fp32 sum 1 GiB in place: buffer 64x1 @24, load aux %d, store aux %d", LA, SA);
            const void* in = buf[1];
            void* io = buf[0];
            vs.push_back({name, "pol", 3.0 * bytes, [=](hipStream_t st) {
                              hipLaunchKernelGGL((r2pol_kernel<LA, SA>), dim3(blocks), dim3(64), lds, st, in, io, nvec);
                              return hipGetLastError();
                          }, io, nullptr, bytes, {}});
        };
        using A2 = std::integral_constant<int, 2>;
        using A16 = std::integral_constant<int, 16>;
        using A18 = std::integral_constant<int, 18>;
        using A19 = std::integral_constant<int, 19>;
        add_pol(A2(), A2());
        add_pol(A2(), A16());
        add_pol(A2(), A18());
        add_pol(A2(), A19());
        add_pol(A18(), A18());
        // the 8-input fan-in at the library's cap (10 waves per CU), in place
        KArgs f{};
        for (int i = 0; i < 8; i++) f.in[i] = buf[i + 2];
        f.out = buf[2];
        f.k = 8;
        f.count = bytes / 4;
        f.nvec = nvec;
        f.trunc_from = f.count;
        add_fan<float, 0u, 64>(vs, "C4 fp32 8-input 1 GiB in place:", f, bytes, 10, nullptr);  // the library
        const unsigned flds = lds_for(10);
        auto add_fpol = [&](auto sa) {
            constexpr int SA = decltype(sa)::value;
            char name[160];
            snprintf(name, sizeof name, "C4 fp32 8-input 1 GiB in place: buffer 64x1 @10, store aux %d", SA);
            vs.push_back({name, "fpol", 9.0 * bytes, [=](hipStream_t st) {
                              hipLaunchKernelGGL((fanpol_kernel<SA>), dim3(blocks), dim3(64), flds, st, f);
                              return hipGetLastError();
                          }, f.out, nullptr, bytes, {}});
        };
        add_fpol(A2());
        add_fpol(A16());
        add_fpol(A18());
        vs.push_back({"C4 fp32 8-input 1 GiB in place: global 64x1 @10, nt loads, nt stores", "fglob", 9.0 * bytes,
                      [=](hipStream_t st) {
                          hipLaunchKernelGGL((fanglob_kernel<1>), dim3(blocks), dim3(64), flds, st, f);
                          return hipGetLastError();
                      }, f.out, nullptr, bytes, {}});
        // the copy (1 GiB, buf[1] -> buf[9]), library launch and store policies
        {
            const char* cs = (const char*)buf[1];
            char* cd = (char*)buf[9];
            const unsigned cb = (unsigned)(nvec / kCopyBlock);
            vs.push_back({"copy 1 GiB: library copy_lean_kernel<3>", "cpol", 2.0 * bytes, [=](hipStream_t st) {
                              hipLaunchKernelGGL((copy_lean_kernel<3>), dim3(cb), dim3(kCopyBlock), 0, st, cs, cd, 0u, nvec,
                                                 0u);
                              return hipGetLastError();
                          }, cd, nullptr, bytes, {}});
            auto add_cpol = [&](auto sa) {
                constexpr int SA = decltype(sa)::value;
                char name[120];
                snprintf(name, sizeof name, "copy 1 GiB: buffer 64x1, store aux %d", SA);
                vs.push_back({name, "cpol", 2.0 * bytes, [=](hipStream_t st) {
                                  hipLaunchKernelGGL((copypol_kernel<SA>), dim3(blocks), dim3(64), 0, st, cs, cd, nvec);
                                  return hipGetLastError();
                              }, cd, nullptr, bytes, {}});
            };
            add_cpol(A2());
            add_cpol(A18());
        }
    }
    if (which == "copyu") {
        const uint64_t nvec = bytes / 16;
        auto add_cu = [&](auto bconst, auto uconst, int cap, void* ref) {
            constexpr int B = decltype(bconst)::value;
            constexpr int U = decltype(uconst)::value;
            if (cap && cap < B / 64) return;
            const unsigned lds = cap ? lds_for(cap / (B / 64)) : 0;
            const int nb = granted(copy_u_kernel<B, U>, B, lds);
            char name[200];
            snprintf(name, sizeof name, "copy 1 GiB: copy %dx%d, lds %u B/block -> %d blocks = %d waves per CU", B, U, lds,
                     nb, nb * B / 64);
            const u32x4* src = (const u32x4*)buf[0];
            u32x4* dst = (u32x4*)(ref ? buf[9] : buf[8]);
            const unsigned blocks = (unsigned)(nvec / (B * U));
            vs.push_back({name, "copy", 2.0 * bytes, [=](hipStream_t st) {
                              hipLaunchKernelGGL((copy_u_kernel<B, U>), dim3(blocks), dim3(B), lds, st, src, dst, nvec);
                              return hipGetLastError();
                          }, dst, ref, bytes, {}});
        };
        using I512 = std::integral_constant<int, 512>;
        using I64 = std::integral_constant<int, 64>;
        using U1 = std::integral_constant<int, 1>;
        using U2 = std::integral_constant<int, 2>;
        using U4 = std::integral_constant<int, 4>;
        add_cu(I512(), U1(), 0, nullptr);  // the library's shape
        add_cu(I64(), U1(), 0, buf[8]);
        for (int cap : {0, 24, 16, 12}) add_cu(I64(), U2(), cap, buf[8]);
        for (int cap : {0, 16, 12, 8}) add_cu(I64(), U4(), cap, buf[8]);
    }
    if (which == "r2u") {
        // one-wave tiles of one or two vectors per lane, in place, over the wave cap
        void *la, *lb;
        CK(hipMalloc(&la, bytes3));
        CK(hipMalloc(&lb, bytes3));
        hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, s, (uint32_t*)la, bytes3 / 4, 0x1234u, 0x3FFF3FFFu,
                           0x3C003C00u);
        hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, s, (uint32_t*)lb, bytes3 / 4, 0x4321u, 0x3FFF3FFFu,
                           0x3C003C00u);
        auto shapes = [&](auto tag, auto vconst, const char* g, R2Args r, size_t nbytes) {
            using Tag = decltype(tag);
            constexpr unsigned V = decltype(vconst)::value;
            add_r2<Tag, V, 1024>(vs, g, r, nbytes, 0, nullptr);
            for (int cap : {32, 28, 24, 20}) add_r2<Tag, V, 64>(vs, g, r, nbytes, cap, nullptr);
            for (int cap : {24, 16, 12, 10, 8}) add_r2<Tag, V, 64, 2>(vs, g, r, nbytes, cap, nullptr);
        };
        R2Args r{};
        r.acc = r.out = buf[0];
        r.in = buf[1];
        r.nvec = bytes / 16;
        r.trunc_from = bytes / 4;
        shapes(float(), std::integral_constant<unsigned, 0u>(), "C2 fp32 sum 1 GiB in place:", r, bytes);
        R2Args rb{};
        rb.acc = rb.out = la;
        rb.in = lb;
        rb.nvec = bytes3 / 16;
        rb.trunc_from = bytes3 / 2;
        shapes(bf16_tag(), std::integral_constant<unsigned, V_BF16_RNE>(), "C3 bf16 sum 256 MiB in place:", rb, bytes3);
    }
    if (which == "pmcset") {
        // one variant per kernel template, so rocprofv3's counter rows (which
        // do not show the dynamic LDS) can be told apart: round 2's launch and
        // the library's current one, for C2 in place and the 8-input fan-in
        R2Args r{};
        r.acc = r.out = buf[0];
        r.in = buf[1];
        r.nvec = bytes / 16;
        r.trunc_from = bytes / 4;
        add_r2<float, 0u, 1024>(vs, "C2 fp32 sum 1 GiB in place:", r, bytes, 0, nullptr);
        add_r2<float, 0u, 64>(vs, "C2 fp32 sum 1 GiB in place:", r, bytes, 24, nullptr);
        KArgs a{};
        for (int i = 0; i < 8; i++) a.in[i] = buf[i + 2 < 10 ? i + 2 : 0];
        a.out = buf[2];
        a.k = 8;
        a.count = bytes / 4;
        a.nvec = bytes / 16;
        a.trunc_from = a.count;
        add_fan<float, 0u, 1024>(vs, "C4 fp32 8-input 1 GiB in place:", a, bytes, 0, nullptr);
        add_fan<float, 0u, 64>(vs, "C4 fp32 8-input 1 GiB in place:", a, bytes, 10, nullptr);
    }
    if (which == "copyconv") {
        // ccl_comp_copy's device kernel (1 GiB, nt loads and stores) and the
        // array conversions (2^28 elements): the library's block vs one-wave
        // blocks under wave caps
        const uint64_t nvec = bytes / 16;
        auto add_copy = [&](auto bconst, int cap, void* ref) {
            constexpr int B = decltype(bconst)::value;
            const unsigned lds = cap ? lds_for(cap / (B / 64)) : 0;
            if (cap && cap < B / 64) return;
            const int nb = granted(copy_lean_kernel<3, B>, B, lds);
            char name[200];
            snprintf(name, sizeof name, "copy 1 GiB: copy_lean_kernel %dx1, lds %u B/block -> %d blocks = %d waves per CU",
                     B, lds, nb, nb * B / 64);
            const char* src = (const char*)buf[0];
            char* dst = (char*)(ref ? buf[9] : buf[8]);
            const unsigned blocks = (unsigned)(nvec / B);
            vs.push_back({name, "copy", 2.0 * bytes, [=](hipStream_t st) {
                              hipLaunchKernelGGL((copy_lean_kernel<3, B>), dim3(blocks), dim3(B), lds, st, src, dst, 0u,
                                                 nvec, 0u);
                              return hipGetLastError();
                          }, dst, ref, bytes, {}});
        };
        add_copy(std::integral_constant<int, 512>(), 0, nullptr);
        for (int cap : {0, 24, 16, 12, 8}) add_copy(std::integral_constant<int, 64>(), cap, buf[8]);
        add_copy(std::integral_constant<int, 256>(), 0, buf[8]);
        add_copy(std::integral_constant<int, 128>(), 0, buf[8]);
        // conversions: fp32 -> bf16 (RNE) from buf[1] into buf[2]; bf16 -> fp32 back into buf[3]
        const uint64_t count = bytes / 4;
        auto add_conv = [&](auto st, auto dt, auto vconst, auto bconst, int cap, const char* label, const void* src,
                            void* dst, void* ref, size_t dbytes, auto sc1const) {
            using ST = decltype(st);
            using DT = decltype(dt);
            constexpr unsigned V = decltype(vconst)::value;
            constexpr int B = decltype(bconst)::value;
            constexpr bool SC1 = decltype(sc1const)::value;
            if (cap && cap < B / 64) return;
            const unsigned lds = cap ? lds_for(cap / (B / 64)) : 0;
            CArgs c{};
            c.src = src;
            c.dst = dst;
            c.count = count;
            c.trunc_from = count;
            c.head = 0;
            c.ngroups = count / 8;
            const uint64_t blocks = std::min<uint64_t>((c.ngroups + B - 1) / B, 1u << 20);
            const int nb = granted(convert_kernel<ST, DT, V, B, SC1>, B, lds);
            char name[200];
            snprintf(name, sizeof name, "%s convert_kernel %dx8%s, lds %u B/block -> %d blocks = %d waves per CU", label,
                     B, SC1 ? " sc1-nt stores" : "", lds, nb, nb * B / 64);
            vs.push_back({name, label, 6.0 * count, [=](hipStream_t st) {
                              hipLaunchKernelGGL((convert_kernel<ST, DT, V, B, SC1>), dim3((unsigned)blocks), dim3(B), lds,
                                                 st, c);
                              return hipGetLastError();
                          }, dst, ref, dbytes, {}});
        };
        using I256 = std::integral_constant<int, 256>;
        using I64 = std::integral_constant<int, 64>;
        using V2 = std::integral_constant<unsigned, V_BF16_RNE>;
        using V0 = std::integral_constant<unsigned, 0u>;
        void* nb16 = buf[2];
        void* nb16b = static_cast<char*>(buf[2]) + bytes / 2;
        add_conv(float(), bf16_tag(), V2(), I256(), 0, "fp32->bf16 2^28:", buf[1], nb16, nullptr, bytes / 2, std::false_type());
        for (int cap : {0, 24, 16, 12}) add_conv(float(), bf16_tag(), V2(), I64(), cap, "fp32->bf16 2^28:", buf[1], nb16b, nb16, bytes / 2, std::false_type());
        add_conv(bf16_tag(), float(), V0(), I256(), 0, "bf16->fp32 2^28:", nb16, buf[3], nullptr, bytes, std::false_type());
        for (int cap : {0, 24, 16, 12}) add_conv(bf16_tag(), float(), V0(), I64(), cap, "bf16->fp32 2^28:", nb16, buf[4], buf[3], bytes, std::false_type());
        // round 5: the same with sc1 + nt stores through per-wave buffer descriptors
        for (int cap : {0, 24, 16}) {
            add_conv(float(), bf16_tag(), V2(), I64(), cap, "fp32->bf16 2^28:", buf[1], nb16b, nb16, bytes / 2,
                     std::true_type());
            add_conv(bf16_tag(), float(), V0(), I64(), cap, "bf16->fp32 2^28:", nb16, buf[4], buf[3], bytes,
                     std::true_type());
        }
    }
    if (which == "fank") {
        // the fan-in at 64-lane blocks over the input count and the wave cap
        // (16 inputs: 8 more buffers)
        for (int i = 0; i < 8; i++) {
            void* p;
            CK(hipMalloc(&p, bytes));
            hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, s, (uint32_t*)p, bytes / 4, 0xC0u + i, 0x007FFFFFu,
                               0x3F800000u);
            buf.push_back(p);
        }
        static std::vector<std::string> names;
        for (int k : {3, 4, 6, 8, 12, 16}) {
            KArgs a{};
            for (int i = 0; i < k; i++) a.in[i] = buf[i < 8 ? i : i + 2];  // skip the two output buffers
            a.out = buf[8];
            a.k = k;
            a.count = bytes / 4;
            a.nvec = bytes / 16;
            a.trunc_from = a.count;
            names.push_back("fan-in fp32 " + std::to_string(k) + "-input 1 GiB:");
            const char* g = names.back().c_str();
            if (k <= 8) {
                add_fan<float, 0u, 1024, 8>(vs, g, a, bytes, 0, nullptr);
                KArgs b = a;
                b.out = buf[9];
                for (int cap : {0, 32, 24, 21, 16, 12, 10, 8, 6, 4}) add_fan<float, 0u, 64, 8>(vs, g, b, bytes, cap, a.out);
            } else {
                add_fan<float, 0u, 1024, 16>(vs, g, a, bytes, 0, nullptr);
                KArgs b = a;
                b.out = buf[9];
                for (int cap : {0, 32, 24, 21, 16, 12, 10, 8, 6, 4}) add_fan<float, 0u, 64, 16>(vs, g, b, bytes, cap, a.out);
            }
        }
    }
    if (which == "fanu") {
        // the 8-input fan-in with 1, 2 or 4 vectors per lane, over the wave cap
        KArgs a{};
        for (int i = 0; i < 8; i++) a.in[i] = buf[i];
        a.out = buf[8];
        a.k = 8;
        a.count = bytes / 4;
        a.nvec = bytes / 16;
        a.trunc_from = a.count;
        add_fan<float, 0u, 64>(vs, "C4 fp32 8-input 1 GiB:", a, bytes, 10, nullptr);  // the library's launch
        KArgs b = a;
        b.out = buf[9];
        auto add_u = [&](auto uconst, auto imconst, int cap) {
            constexpr int U = decltype(uconst)::value;
            constexpr bool IM = decltype(imconst)::value;
            const unsigned lds = lds_for(cap);
            const int nb = granted(fanu_kernel<U, IM>, 64, lds);
            char name[200];
            snprintf(name, sizeof name, "C4 fp32 8-input 1 GiB: fanu 64x%d %s, lds %u B/block -> %d waves per CU", U,
                     IM ? "input-major" : "vector-major", lds, nb);
            const unsigned blocks = (unsigned)(b.nvec / (64 * U));
            vs.push_back({name, "fanu", 9.0 * bytes, [=](hipStream_t st) {
                              hipLaunchKernelGGL((fanu_kernel<U, IM>), dim3(blocks), dim3(64), lds, st, b);
                              return hipGetLastError();
                          }, b.out, a.out, bytes, {}});
        };
        using U1 = std::integral_constant<int, 1>;
        using U2 = std::integral_constant<int, 2>;
        using U4 = std::integral_constant<int, 4>;
        using T = std::true_type;
        using F = std::false_type;
        add_u(U1(), F(), 10);
        for (int cap : {12, 10, 8, 6, 5, 4}) {
            add_u(U2(), F(), cap);
            add_u(U2(), T(), cap);
        }
        for (int cap : {8, 6, 5, 4, 3, 2}) {
            add_u(U4(), F(), cap);
            add_u(U4(), T(), cap);
        }
    }
    if (which == "xcd") {
        // one-wave tiles remapped so each XCD takes runs of G consecutive
        // tiles (G = 1 is the hardware's round robin, the library's order)
        const uint64_t nvec = bytes / 16;
        const unsigned blocks = (unsigned)(nvec / 64);
        R2Args r{};
        r.acc = r.out = buf[0];
        r.in = buf[1];
        r.nvec = nvec;
        r.trunc_from = bytes / 4;
        add_r2<float, 0u, 64>(vs, "C2 fp32 sum 1 GiB in place:", r, bytes, 24, nullptr);  // the library
        const unsigned lds24 = lds_for(24), lds10 = lds_for(10);
        const uint64_t gs[] = {1, 2, 4, 16, 64, 1024, blocks / 8};
        for (uint64_t G : gs) {
            char name[160];
            snprintf(name, sizeof name, "C2 fp32 sum 1 GiB in place: xcd runs of %llu tiles, 64x1 @24",
                     (unsigned long long)G);
            const void* in = buf[1];
            void* io = buf[0];
            vs.push_back({name, "r2xcd", 3.0 * bytes, [=](hipStream_t st) {
                              hipLaunchKernelGGL(r2xcd_kernel, dim3(blocks), dim3(64), lds24, st, in, io, nvec, G);
                              return hipGetLastError();
                          }, io, nullptr, bytes, {}});
        }
        KArgs f{};
        for (int i = 0; i < 8; i++) f.in[i] = buf[i + 2];
        f.out = buf[2];
        f.k = 8;
        f.count = bytes / 4;
        f.nvec = nvec;
        f.trunc_from = f.count;
        add_fan<float, 0u, 64>(vs, "C4 fp32 8-input 1 GiB in place:", f, bytes, 10, nullptr);  // the library
        for (uint64_t G : gs) {
            char name[160];
            snprintf(name, sizeof name, "C4 fp32 8-input 1 GiB in place: xcd runs of %llu tiles, 64x1 @10",
                     (unsigned long long)G);
            vs.push_back({name, "fanxcd", 9.0 * bytes, [=](hipStream_t st) {
                              hipLaunchKernelGGL(fanxcd_kernel, dim3(blocks), dim3(64), lds10, st, f, G);
                              return hipGetLastError();
                          }, f.out, nullptr, bytes, {}});
        }
    }
    if (which == "c4bf") {
        // bf16 inputs accumulated in fp32 (the bench's c4-bf16acc leg), in a
        // run of its own: the inputs are refilled as bf16 pairs (fp32 bits
        // read as bf16 would hold NaN patterns)
        for (int i = 0; i < 8; i++)
            hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, s, (uint32_t*)buf[i], bytes / 4, 0xB0u + i,
                               0x3FFF3FFFu, 0x3C003C00u);
        KArgs a{};
        for (int i = 0; i < 8; i++) a.in[i] = buf[i];
        a.out = buf[8];
        a.k = 8;
        a.count = bytes / 2;
        a.nvec = bytes / 16;
        a.trunc_from = a.count;
        sweep_fan<bf16_tag, V_ACC_FP32 | V_BF16_RNE>(vs, "C4 bf16 8-input fp32-acc 1 GiB:", a, bytes, buf[9]);
    }
    CK(hipStreamSynchronize(s));

    // check: each group's reference first (in order), then every variant against it;
    // a variant whose launch fails (a cap the device cannot grant) is dropped
    unsigned long long* bad;
    CK(hipMalloc(&bad, sizeof(*bad)));
    std::vector<Variant> ok;
    for (auto& v : vs) {
        if (v.run(s) != hipSuccess) {
            fprintf(stderr, "skip (launch failed): %s\n", v.name.c_str());
            continue;
        }
        if (v.ref) {
            CK(hipMemsetAsync(bad, 0, sizeof(*bad), s));
            hipLaunchKernelGGL(count_diff, dim3(4096), dim3(256), 0, s, (const uint32_t*)v.out, (const uint32_t*)v.ref,
                               v.bytes / 4, bad);
            unsigned long long h = 0;
            CK(hipMemcpyAsync(&h, bad, sizeof(h), hipMemcpyDeviceToHost, s));
            CK(hipStreamSynchronize(s));
            if (h) {
                fprintf(stderr, "MISMATCH %llu words: %s\n", h, v.name.c_str());
                return 3;
            }
        }
        CK(hipStreamSynchronize(s));
        ok.push_back(v);
    }
    fprintf(stderr, "%zu variants checked bit-exact against the library's launch\n", ok.size());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int r = 0; r < rounds; r++) {
        for (auto& v : ok)
            for (int i = 0; i < reps; i++) {
                CK(hipEventRecord(e0, s));
                CK(v.run(s));
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                v.ms.push_back(ms);
            }
        fprintf(stderr, "round %d/%d done\n", r + 1, rounds);
    }
    for (auto& v : ok) {
        std::sort(v.ms.begin(), v.ms.end());
        const float med = v.ms[v.ms.size() / 2], best = v.ms.front();
        printf("{\"variant\": \"%s\", \"bytes_per_launch\": %.0f, \"median_ms\": %.5f, \"best_ms\": %.5f, "
               "\"median_TBps\": %.3f, \"best_TBps\": %.3f, \"frac_of_8TBps\": %.4f}\n",
               v.name.c_str(), v.traffic, med, best, v.traffic / (med * 1e-3) / 1e12, v.traffic / (best * 1e-3) / 1e12,
               v.traffic / (med * 1e-3) / 8e12);
    }
    for (auto& p : buf) CK(hipFree(p));
    return 0;
}
