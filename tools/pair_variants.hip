// pair_variants.hip — C2's placement mode against the order in which the
// 2-input in-place reduce walks its tiles.
//
// tools/pair_probe.py found that the 1 GiB fp32 reduce runs ~7 % slower for
// some pairs of buffers than for others, that the slow/fast outcome is a
// property of the (acc, in) pair (fresh allocations fall in classes: same
// class fast, different class slow), and that one buffer read or written
// alone is never slower.  The kernel cannot see physical addresses, but it
// decides which tiles are in flight together.  This tool allocates four
// 1 GiB buffers, and for every ordered pair times the library's launch
// (mi_reduce) and the same fold with other tile orders:
//   map 0  tile = block (the library's order, this tool's own kernel)
//   map 1  two halves interleaved: tile = (b % 2) * T/2 + b / 2
//   map 2  8 regions interleaved (one per XCD under round-robin dispatch)
//   map 3  64 regions interleaved
//   map 4  tile = block, `in` loaded before `acc`
//   map 5  walked backwards: tile = T - 1 - block
//   map 6  two windows from both ends: even blocks from the start, odd from the end
// and, in library order, other residencies (the slow mode has fewer reads in
// flight at the L2, placement_pmc/): 16 and 25 resident waves per CU, no cap,
// and two tiles per wave at the library's cap.
// Each variant's output is checked against the library's on the first pair.
// `trials` times the buffers are freed and reallocated behind random pads, so
// that pairs of both placement classes turn up.
//   pair_variants [trials=4] [launches=10]        one JSON line per pair x variant
//   PAIR_RESIDENCY=1 pair_variants ...           the residency variants instead of the orders
//   PAIR_WAVES=12,16,21 pair_variants ...        the library's order at these wave caps
//   PAIR_SPLIT=1 pair_variants ...               acc and in loaded by different waves of a
//                                                tile (through LDS), and read-only probes:
//                                                both buffers per wave, or one per wave
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../include/mi_reduce.h"

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(2);                                                                     \
        }                                                                                \
    } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int MAP>
__global__ __launch_bounds__(64) void fold2(f32x4* acc, const f32x4* in, uint64_t tiles) {
    extern __shared__ char lds_cap[];
    (void)lds_cap;
    const uint64_t b = blockIdx.x;
    uint64_t t;
    if (MAP == 1) t = (b & 1) * (tiles / 2) + (b >> 1);
    else if (MAP == 2) t = (b & 7) * (tiles / 8) + (b >> 3);
    else if (MAP == 3) t = (b & 63) * (tiles / 64) + (b >> 6);
    else if (MAP == 5) t = tiles - 1 - b;
    else if (MAP == 6) t = (b & 1) ? tiles - 1 - (b >> 1) : (b >> 1);
    else t = b;
    const uint64_t v = t * 64 + threadIdx.x;
    f32x4 x, y;
    if (MAP == 4) {
        y = __builtin_nontemporal_load(in + v);
        x = __builtin_nontemporal_load(acc + v);
    } else {
        x = __builtin_nontemporal_load(acc + v);
        y = __builtin_nontemporal_load(in + v);
    }
    const f32x4 r = x + y;
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<char*>(acc + t * 64), (short)0,
                                                                  1024, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, r), rs,
                                           threadIdx.x * 16u, 0, 18 /* sc1 nt, as the library */);
}

// two consecutive tiles per wave: four loads in flight per lane
__global__ __launch_bounds__(64) void fold2x2(f32x4* acc, const f32x4* in, uint64_t tiles) {
    extern __shared__ char lds_cap[];
    (void)lds_cap;
    const uint64_t t = (uint64_t)blockIdx.x * 2;
    const uint64_t v = t * 64 + threadIdx.x;
    const f32x4 x0 = __builtin_nontemporal_load(acc + v), x1 = __builtin_nontemporal_load(acc + v + 64);
    const f32x4 y0 = __builtin_nontemporal_load(in + v), y1 = __builtin_nontemporal_load(in + v + 64);
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<char*>(acc + t * 64), (short)0,
                                                                  2048, 0x00020000);
    typedef __attribute__((ext_vector_type(4))) unsigned u4;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, x0 + y0), rs, threadIdx.x * 16u, 0, 18);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, x1 + y1), rs, 1024u + threadIdx.x * 16u, 0, 18);
}

// two waves per tile: wave 0 brings acc's tile into LDS, wave 1 loads in's
// and folds, so no wave reads both buffers
__global__ __launch_bounds__(128) void fold2_split(f32x4* acc, const f32x4* in, uint64_t tiles) {
    extern __shared__ f32x4 lds_tile[];
    const uint64_t t = blockIdx.x;
    const unsigned w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const uint64_t v = t * 64 + l;
    f32x4 y = {0, 0, 0, 0};
    if (w == 0)
        lds_tile[l] = __builtin_nontemporal_load(acc + v);
    else
        y = __builtin_nontemporal_load(in + v);
    __syncthreads();
    if (w == 1) {
        const f32x4 r = lds_tile[l] + y;
        __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<char*>(acc + t * 64), (short)0,
                                                                      1024, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, r), rs,
                                               l * 16u, 0, 18);
    }
}

// the same with two consecutive tiles per wave (as many loads in flight per
// wave as the library's one-tile wave that loads both buffers)
__global__ __launch_bounds__(128) void fold2_split2(f32x4* acc, const f32x4* in, uint64_t tiles) {
    extern __shared__ f32x4 lds_tile[];
    const uint64_t t = (uint64_t)blockIdx.x * 2;
    const unsigned w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const uint64_t v = t * 64 + l;
    f32x4 y0 = {0, 0, 0, 0}, y1 = {0, 0, 0, 0};
    if (w == 0) {
        lds_tile[l] = __builtin_nontemporal_load(acc + v);
        lds_tile[64 + l] = __builtin_nontemporal_load(acc + v + 64);
    } else {
        y0 = __builtin_nontemporal_load(in + v);
        y1 = __builtin_nontemporal_load(in + v + 64);
    }
    __syncthreads();
    if (w == 1) {
        typedef __attribute__((ext_vector_type(4))) unsigned u4;
        __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<char*>(acc + t * 64), (short)0,
                                                                      2048, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, lds_tile[l] + y0), rs, l * 16u, 0, 18);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, lds_tile[64 + l] + y1), rs, 1024u + l * 16u, 0,
                                               18);
    }
}

// reads only: both buffers per wave (ONE = false) or one buffer per wave,
// alternate blocks taking acc and in (ONE = true)
template <bool ONE>
__global__ __launch_bounds__(64) void read2_probe(const f32x4* acc, const f32x4* in, uint64_t tiles, unsigned* sink) {
    extern __shared__ char lds_cap[];
    (void)lds_cap;
    const uint64_t b = blockIdx.x;
    f32x4 x;
    if (ONE) {  // two consecutive tiles of one buffer: the same loads in flight per wave
        const f32x4* p = ((b & 1) ? in : acc) + (b >> 1) * 128 + threadIdx.x;
        x = __builtin_nontemporal_load(p) + __builtin_nontemporal_load(p + 64);
    } else {
        x = __builtin_nontemporal_load(acc + b * 64 + threadIdx.x) + __builtin_nontemporal_load(in + b * 64 + threadIdx.x);
    }
    if (x.x == 1234.5f && x.y == -1.0f) sink[threadIdx.x] = 1u;
}

__global__ void fill(float* p, uint64_t n, uint32_t seed) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t h = (uint32_t)i * 2654435761u ^ seed;
        h ^= h >> 13;
        h *= 0x5bd1e995u;
        p[i] = (float)(h & 0xFFFF) / 65536.0f - 0.5f;
    }
}

int main(int argc, char** argv) {
    const int trials = argc > 1 ? atoi(argv[1]) : 4;
    const int launches = argc > 2 ? atoi(argv[2]) : 10;
    const uint64_t bytes = 1ull << 30, n = bytes / 4, tiles = bytes / 1024;
    float* buf[4];
    for (auto& p : buf) CK(hipMalloc(&p, bytes));
    std::vector<void*> pads;
    srand(7);
    float *chk_a, *chk_b;
    unsigned* sink = nullptr;
    CK(hipMalloc(&sink, 64 * sizeof(unsigned)));
    CK(hipMalloc(&chk_a, bytes));
    CK(hipMalloc(&chk_b, bytes));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    int dev = 0, ldsb = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&ldsb, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev));
    int waves = 0;
    unsigned lib_lds = 0;
    mi_get_residency(dev, 2, &waves, &lib_lds);
    auto refill = [&](int i) { hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, s, buf[i], n, 0x9E37u + i); };
    for (int i = 0; i < 4; i++) refill(i);
    CK(hipStreamSynchronize(s));

    const unsigned gran = (unsigned)ldsb / 128u;
    auto lds_for = [&](int w) { return (128u / (unsigned)w) * gran; };
    auto run = [&](int v, float* acc, const float* in) -> hipError_t {
        const dim3 g((unsigned)tiles), bl(64);
        switch (v) {
            case 8: hipLaunchKernelGGL(fold2<0>, g, bl, lds_for(16), s, (f32x4*)acc, (const f32x4*)in, tiles); break;
            case 9: hipLaunchKernelGGL(fold2<0>, g, bl, lds_for(25), s, (f32x4*)acc, (const f32x4*)in, tiles); break;
            case 10: hipLaunchKernelGGL(fold2<0>, g, bl, 0, s, (f32x4*)acc, (const f32x4*)in, tiles); break;
            default:
                if (v >= 100) {  // tile = block at a cap of v - 100 waves per CU
                    hipLaunchKernelGGL(fold2<0>, g, bl, lds_for(v - 100), s, (f32x4*)acc, (const f32x4*)in, tiles);
                    break;
                }
                return (hipError_t)mi_reduce(in, acc, n, MI_FLOAT32, MI_OP_SUM, 0, s);
            case 12: {
                const unsigned gran2 = (unsigned)ldsb / 128u;
                hipLaunchKernelGGL(fold2_split, g, dim3(128), std::max(1024u, (128u / 10u) * gran2), s, (f32x4*)acc,
                                   (const f32x4*)in, tiles);
                break;
            }
            case 13: {
                const unsigned gran2 = (unsigned)ldsb / 128u;
                hipLaunchKernelGGL(fold2_split2, dim3((unsigned)(tiles / 2)), dim3(128),
                                   std::max(2048u, (128u / 10u) * gran2), s, (f32x4*)acc, (const f32x4*)in, tiles);
                break;
            }
            case 14:
                hipLaunchKernelGGL(read2_probe<false>, g, bl, lib_lds, s, (const f32x4*)acc, (const f32x4*)in, tiles,
                                   sink);
                break;
            case 15:
                hipLaunchKernelGGL(read2_probe<true>, g, bl, lib_lds, s, (const f32x4*)acc,
                                   (const f32x4*)in, tiles, sink);
                break;
            case 11:
                hipLaunchKernelGGL(fold2x2, dim3((unsigned)(tiles / 2)), bl, lib_lds, s, (f32x4*)acc, (const f32x4*)in,
                                   tiles);
                break;
            case 0: hipLaunchKernelGGL(fold2<0>, g, bl, lib_lds, s, (f32x4*)acc, (const f32x4*)in, tiles); break;
            case 1: hipLaunchKernelGGL(fold2<1>, g, bl, lib_lds, s, (f32x4*)acc, (const f32x4*)in, tiles); break;
            case 2: hipLaunchKernelGGL(fold2<2>, g, bl, lib_lds, s, (f32x4*)acc, (const f32x4*)in, tiles); break;
            case 3: hipLaunchKernelGGL(fold2<3>, g, bl, lib_lds, s, (f32x4*)acc, (const f32x4*)in, tiles); break;
            case 4: hipLaunchKernelGGL(fold2<4>, g, bl, lib_lds, s, (f32x4*)acc, (const f32x4*)in, tiles); break;
            case 6: hipLaunchKernelGGL(fold2<5>, g, bl, lib_lds, s, (f32x4*)acc, (const f32x4*)in, tiles); break;
            case 7: hipLaunchKernelGGL(fold2<6>, g, bl, lib_lds, s, (f32x4*)acc, (const f32x4*)in, tiles); break;
            case 5: return (hipError_t)mi_reduce(in, acc, n, MI_FLOAT32, MI_OP_SUM, 0, s);
        }
        return hipGetLastError();
    };
    const char* names[16] = {"tile = block", "halves interleaved", "8 regions interleaved", "64 regions interleaved",
                             "in loaded first", "library (mi_reduce)", "walked backwards", "two windows from both ends",
                             "16 waves/CU", "25 waves/CU", "no wave cap", "two tiles per wave",
                             "acc and in loaded by different waves (LDS)", "the same, two tiles per wave",
                             "read both per wave (no store)",
                             "read one buffer per wave (no store)"};
    const bool split = getenv("PAIR_SPLIT") != nullptr;  // the split-wave fold and the read-only probes
    const bool resid = getenv("PAIR_RESIDENCY") != nullptr;  // time the residency variants instead of the orders
    std::vector<int> caps;  // PAIR_WAVES=12,16,21: the library's order at these caps instead
    if (const char* w = getenv("PAIR_WAVES"))
        for (const char* q = w; *q;) {
            caps.push_back(100 + atoi(q));
            while (*q && *q != ',') q++;
            if (*q) q++;
        }
    auto name_of = [&](int v) { return v >= 100 ? std::to_string(v - 100) + " waves/CU" : std::string(names[v]); };

    // every variant's bits against the library's on one pair
    for (int v : {0, 1, 2, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13}) {
        CK(hipMemcpyAsync(chk_a, buf[0], bytes, hipMemcpyDeviceToDevice, s));
        CK(hipMemcpyAsync(chk_b, buf[0], bytes, hipMemcpyDeviceToDevice, s));
        CK(run(v, chk_a, buf[1]));
        CK(run(5, chk_b, buf[1]));
        CK(hipStreamSynchronize(s));
        std::vector<uint32_t> ha(1 << 20), hb(1 << 20);
        bool same = true;
        for (uint64_t off = 0; off < n && same; off += (n / 8)) {
            CK(hipMemcpy(ha.data(), chk_a + off, ha.size() * 4, hipMemcpyDeviceToHost));
            CK(hipMemcpy(hb.data(), chk_b + off, hb.size() * 4, hipMemcpyDeviceToHost));
            same = memcmp(ha.data(), hb.data(), ha.size() * 4) == 0;
        }
        printf("{\"check\": \"%s\", \"same_bits_as_library\": %s}\n", names[v], same ? "true" : "false");
        if (!same) return 3;
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int r = 0; r < trials; r++) {
        if (r > 0) {  // new placement: free, pad at random, reallocate, refill
            for (auto& p : buf) CK(hipFree(p));
            for (void* p : pads) CK(hipFree(p));
            pads.clear();
            for (int i = 0; i < 4; i++) {
                void* pad = nullptr;
                CK(hipMalloc(&pad, (size_t)(1 + rand() % 512) << 21));
                pads.push_back(pad);
                CK(hipMalloc(&buf[i], bytes));
                refill(i);
            }
            CK(hipStreamSynchronize(s));
        }
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 4; j++) {
                if (i == j) continue;
                std::vector<int> vs = resid ? std::vector<int>{5, 0, 8, 9, 10, 11} : std::vector<int>{5, 0, 1, 4, 6, 7};
                if (split) vs = {5, 0, 12, 13, 14, 15};
                if (!caps.empty()) {
                    vs = {5};
                    vs.insert(vs.end(), caps.begin(), caps.end());
                }
                for (int v : vs) {
                    for (int w = 0; w < 2; w++) CK(run(v, buf[i], buf[j]));
                    CK(hipEventRecord(e0, s));
                    for (int l = 0; l < launches; l++) CK(run(v, buf[i], buf[j]));
                    CK(hipEventRecord(e1, s));
                    CK(hipEventSynchronize(e1));
                    float ms = 0;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    printf("{\"round\": %d, \"pair\": \"%d%d\", \"variant\": \"%s\", \"ms\": %.5f}\n", r, i, j, name_of(v).c_str(),
                           ms / launches);
                    fflush(stdout);
                }
                refill(i);
            }
    }
    return 0;
}
