// ceiling_probe.hip — libmi_ceiling.so: memory-only probes for the measured
// ceiling bench.py reports beside each kernel's roofline fraction
// (roofline.ceiling_TBps / frac_of_ceiling).
//
// The spec peak (8 TB/s) is not reachable by any access pattern on this
// part; what a K-input reduce can reach is bounded by how fast HBM serves
// its K read streams and its one write stream.  So, on the reduce's own
// buffers and in the same process:
//   mic_read_streams  reads K streams of `bytes` each (16-byte non-temporal
//                     loads, no arithmetic beyond an XOR that keeps the
//                     loads alive; nothing is written unless the XOR hits a
//                     magic value);
//   mic_write_stream  writes one stream of `bytes` (16-byte stores of a
//                     constant);
//   mic_mixed_streams reads the K streams and writes one stream in the same
//                     launch, at the reduce's K:1 ratio, with no arithmetic:
//                     each lane loads its vector of every input, keeps the
//                     loads alive with an empty asm that takes them as
//                     operands, and stores input 0's vector to the output
//                     (the reads and the write interleaved
//                     as the reduce interleaves them, which the separate
//                     probes cannot show).
// Each in the instruction flavours the library's kernels use (`flavor`):
// 0 = global_load/store ... nt; 1 = buffer_load/store ... nt through a
// per-workgroup descriptor; 2 (stores) = buffer_store ... sc1 nt, which the
// 2-input kernel uses (the line leaves L2 as it is written).
// bench.py times each over a few launch shapes and flavours, takes the fastest, and
// prices the reduce's traffic at those rates, reads and writes sharing the
// bus: ceiling = (K + 1) * bytes / (t_read_K + t_write).
// Measurement infrastructure, not product: nothing in libmi_reduce calls it.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

constexpr int kMaxK = 16;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

struct ReadArgs {
    const u32x4* in[kMaxK];
    uint64_t nvec;  // 16-byte vectors per stream
    uint32_t* sink;
};

constexpr int kAuxNT = 2, kAuxSC1NT = 18;  // buffer op aux bits (gfx950), as reduce_kernels.hpp

__device__ __forceinline__ __amdgpu_buffer_rsrc_t block_rsrc(const void* base, uint64_t nvec) {
    const uint64_t v0 = (uint64_t)blockIdx.x * blockDim.x;
    const uint64_t left = nvec - v0;
    const uint32_t bytes = (uint32_t)(left < blockDim.x ? left : blockDim.x) * 16u;
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(static_cast<const char*>(base)) + v0 * 16, (short)0,
                                             (int)bytes, 0x00020000);
}

template <int K>
__global__ void read_streams_buf(ReadArgs a) {
    extern __shared__ char lds_cap[];
    (void)lds_cap;
    if ((uint64_t)blockIdx.x * blockDim.x >= a.nvec) return;
    u32x4 x[K];
#pragma unroll
    for (int j = 0; j < K; j++)
        x[j] = __builtin_amdgcn_raw_buffer_load_b128(block_rsrc(a.in[j], a.nvec), threadIdx.x * 16u, 0, kAuxNT);
    uint32_t acc = 0;
#pragma unroll
    for (int j = 0; j < K; j++) acc ^= x[j].x ^ x[j].y ^ x[j].z ^ x[j].w;
    const uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (acc == 0x9E3779B9u && v < a.nvec) a.sink[v & 1023] = acc;
}

template <int AUX>
__global__ void write_stream_buf(u32x4* out, uint64_t nvec) {
    extern __shared__ char lds_cap[];
    (void)lds_cap;
    if ((uint64_t)blockIdx.x * blockDim.x >= nvec) return;
    const u32x4 one = {0x3F800000u, 0x3F800000u, 0x3F800000u, 0x3F800000u};
    __builtin_amdgcn_raw_buffer_store_b128(one, block_rsrc(out, nvec), threadIdx.x * 16u, 0, AUX);
}

template <int K>
__global__ void read_streams(ReadArgs a) {
    extern __shared__ char lds_cap[];  // never touched: caps resident waves
    (void)lds_cap;
    const uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= a.nvec) return;
    u32x4 x[K];
#pragma unroll
    for (int j = 0; j < K; j++) x[j] = __builtin_nontemporal_load(a.in[j] + v);
    uint32_t acc = 0;
#pragma unroll
    for (int j = 0; j < K; j++) acc ^= x[j].x ^ x[j].y ^ x[j].z ^ x[j].w;
    if (acc == 0x9E3779B9u) a.sink[v & 1023] = acc;
}

__global__ void write_stream(u32x4* out, uint64_t nvec) {
    extern __shared__ char lds_cap[];
    (void)lds_cap;
    const uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= nvec) return;
    const u32x4 one = {0x3F800000u, 0x3F800000u, 0x3F800000u, 0x3F800000u};
    __builtin_nontemporal_store(one, out + v);
}

// The reduce's memory traffic without its arithmetic: K loads, one store
// per lane, a tile of one vector per lane per block (the library's one-wave
// tiles at block 64).  STORE_AUX 0 = global nt store; otherwise buffer_store
// with those aux bits (kAuxNT: the fan-in's nt store, kAuxSC1NT: the 2-input
// kernel's sc1 nt).  Loads: global nt (STORE_AUX 0) or buffer nt, as the
// library's kernels pair them.
struct MixArgs {
    const u32x4* in[kMaxK];
    u32x4* out;
    uint64_t nvec;
};

template <int K, int STORE_AUX>
__global__ void mixed_streams(MixArgs a) {
    extern __shared__ char lds_cap[];
    (void)lds_cap;
    if ((uint64_t)blockIdx.x * blockDim.x >= a.nvec) return;
    u32x4 x[K];
    if constexpr (STORE_AUX == 0) {
        const uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
        if (v >= a.nvec) return;
#pragma unroll
        for (int j = 0; j < K; j++) x[j] = __builtin_nontemporal_load(a.in[j] + v);
#pragma unroll
        for (int j = 1; j < K; j++) asm volatile("" ::"v"(x[j]));
        __builtin_nontemporal_store(x[0], a.out + v);
    } else {
#pragma unroll
        for (int j = 0; j < K; j++)
            x[j] = __builtin_amdgcn_raw_buffer_load_b128(block_rsrc(a.in[j], a.nvec), threadIdx.x * 16u, 0, kAuxNT);
#pragma unroll
        for (int j = 1; j < K; j++) asm volatile("" ::"v"(x[j]));
        __builtin_amdgcn_raw_buffer_store_b128(x[0], block_rsrc(a.out, a.nvec), threadIdx.x * 16u, 0, STORE_AUX);
    }
}

// Other access patterns for the same traffic, no
// arithmetic, as mixed_streams: each workgroup owns a run of T consecutive
// tiles (tile = blockDim vectors).  Read phase: every input's vector of each
// tile, input 0's parked (LDS: in dynamic LDS, T x blockDim x 16 bytes per
// workgroup; else in registers); write phase: the T tiles stored back to
// back, a burst of T x blockDim x 16 bytes per workgroup instead of one
// store per tile between loads.  Each lane stores what it parked itself, so
// no barrier is needed.  Loads buffer nt, stores STORE_AUX (nt / sc1 nt).
template <int K, int T, bool LDS, int STORE_AUX>
__global__ void burst_streams(MixArgs a) {
    extern __shared__ u32x4 stage[];
    const uint64_t B = blockDim.x;
    const uint64_t tile0 = (uint64_t)blockIdx.x * T;
    u32x4 keep[LDS ? 1 : T];
#pragma unroll
    for (int t = 0; t < T; t++) {
        const uint64_t v0 = (tile0 + t) * B;
        if (v0 >= a.nvec) break;
        const uint64_t left = a.nvec - v0;
        const uint32_t bytes = (uint32_t)(left < B ? left : B) * 16u;
        u32x4 x[K];
#pragma unroll
        for (int j = 0; j < K; j++)
            x[j] = __builtin_amdgcn_raw_buffer_load_b128(
                __builtin_amdgcn_make_buffer_rsrc(const_cast<u32x4*>(a.in[j] + v0), (short)0, (int)bytes, 0x00020000),
                threadIdx.x * 16u, 0, kAuxNT);
#pragma unroll
        for (int j = 1; j < K; j++) asm volatile("" ::"v"(x[j]));
        if constexpr (LDS)
            stage[t * B + threadIdx.x] = x[0];
        else
            keep[t] = x[0];
    }
#pragma unroll
    for (int t = 0; t < T; t++) {
        const uint64_t v0 = (tile0 + t) * B;
        if (v0 >= a.nvec) break;
        const uint64_t left = a.nvec - v0;
        const uint32_t bytes = (uint32_t)(left < B ? left : B) * 16u;
        __builtin_amdgcn_raw_buffer_store_b128(LDS ? stage[t * B + threadIdx.x] : keep[LDS ? 0 : t],
                                               __builtin_amdgcn_make_buffer_rsrc(a.out + v0, (short)0, (int)bytes,
                                                                                 0x00020000),
                                               threadIdx.x * 16u, 0, STORE_AUX);
    }
}

// The 2-input fp32 sum in place as the library computes it (an add per
// element, the unordered-compare screen the library's NaN rule runs), but
// with buffer loads (nt) instead of the library's global nt loads, and the
// store flavour STORE_AUX: the load form is the one difference from
// reduce2_kernel<float> (tools/r2_load_ab.py A/Bs the two over placements).
template <int STORE_AUX>
__global__ __launch_bounds__(64) void sum2_buffer(const void* in, void* io, uint64_t nvec, uint32_t* sink) {
    extern __shared__ char lds_cap[];
    (void)lds_cap;
    const uint64_t t0 = (uint64_t)blockIdx.x * 64;
    if (t0 >= nvec) return;
    const uint64_t left = nvec - t0;
    const uint32_t bytes = (uint32_t)(left < 64 ? left : 64) * 16u;
    const uint32_t off = threadIdx.x * 16u;
    const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(static_cast<char*>(io) + t0 * 16, (short)0,
                                                                        (int)bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char*>(static_cast<const char*>(in)) + t0 * 16, (short)0, (int)bytes, 0x00020000);
    const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(ra, off, 0, kAuxNT);
    const u32x4 b = __builtin_amdgcn_raw_buffer_load_b128(rb, off, 0, kAuxNT);
    u32x4 r;
    bool nan = false;
#pragma unroll
    for (int e = 0; e < 4; e++) {
        const float x = __uint_as_float(a[e]), y = __uint_as_float(b[e]);
        const float z = x + y;
        nan = nan || (z != z);
        r[e] = __float_as_uint(z);
    }
    if (nan) sink[threadIdx.x] = 1u;  // the library refolds such a row; the A/B's inputs hold no NaN
    __builtin_amdgcn_raw_buffer_store_b128(r, ra, off, 0, STORE_AUX);
}

typedef hipError_t (*MixFn)(dim3, dim3, unsigned, hipStream_t, const MixArgs&);

template <int K, int T, bool LDS, int AUX>
hipError_t launch_burst(dim3 g, dim3 b, unsigned lds, hipStream_t s, const MixArgs& a) {
    hipLaunchKernelGGL((burst_streams<K, T, LDS, AUX>), g, b, lds, s, a);
    return hipGetLastError();
}

template <int K, bool LDS, int AUX>
MixFn pick_burst_t(int t) {
    switch (t) {
        case 1: return launch_burst<K, 1, LDS, AUX>;
        case 2: return launch_burst<K, 2, LDS, AUX>;
        case 4: return launch_burst<K, 4, LDS, AUX>;
        case 8: return LDS ? launch_burst<K, 8, true, AUX> : nullptr;
        case 16: return LDS ? launch_burst<K, 16, true, AUX> : nullptr;
        case 32: return LDS ? launch_burst<K, 32, true, AUX> : nullptr;
        default: return nullptr;
    }
}

template <int K>
MixFn pick_burst_k(int t, bool lds, int flavor) {
    if (flavor == 1) return lds ? pick_burst_t<K, true, kAuxNT>(t) : pick_burst_t<K, false, kAuxNT>(t);
    if (flavor == 2) return lds ? pick_burst_t<K, true, kAuxSC1NT>(t) : pick_burst_t<K, false, kAuxSC1NT>(t);
    return nullptr;
}

template <int K, int AUX>
hipError_t launch_mix(dim3 g, dim3 b, unsigned lds, hipStream_t s, const MixArgs& a) {
    hipLaunchKernelGGL((mixed_streams<K, AUX>), g, b, lds, s, a);
    return hipGetLastError();
}

template <int AUX>
MixFn pick_mix_k(int k) {
    switch (k) {
        case 1: return launch_mix<1, AUX>;  // a copy (out != ptrs[0]): ccl_comp_copy's traffic
        case 2: return launch_mix<2, AUX>;
        case 3: return launch_mix<3, AUX>;
        case 4: return launch_mix<4, AUX>;
        case 6: return launch_mix<6, AUX>;
        case 8: return launch_mix<8, AUX>;
        case 12: return launch_mix<12, AUX>;
        case 16: return launch_mix<16, AUX>;
        default: return nullptr;
    }
}

MixFn pick_mix(int k, int flavor) {
    return flavor == 0 ? pick_mix_k<0>(k) : flavor == 1 ? pick_mix_k<kAuxNT>(k)
                                                        : flavor == 2 ? pick_mix_k<kAuxSC1NT>(k) : nullptr;
}

template <int K, bool BUF>
hipError_t launch_read(dim3 g, dim3 b, unsigned lds, hipStream_t s, const ReadArgs& a) {
    if (BUF)
        hipLaunchKernelGGL(read_streams_buf<K>, g, b, lds, s, a);
    else
        hipLaunchKernelGGL(read_streams<K>, g, b, lds, s, a);
    return hipGetLastError();
}

typedef hipError_t (*ReadFn)(dim3, dim3, unsigned, hipStream_t, const ReadArgs&);

template <bool BUF>
ReadFn pick_k(int k) {
    switch (k) {
        case 1: return launch_read<1, BUF>;
        case 2: return launch_read<2, BUF>;
        case 3: return launch_read<3, BUF>;
        case 4: return launch_read<4, BUF>;
        case 6: return launch_read<6, BUF>;
        case 8: return launch_read<8, BUF>;
        case 12: return launch_read<12, BUF>;
        case 16: return launch_read<16, BUF>;
        default: return nullptr;
    }
}

ReadFn pick(int k, int flavor) { return flavor == 0 ? pick_k<false>(k) : flavor == 1 ? pick_k<true>(k) : nullptr; }

// dynamic LDS per block so that `waves_per_cu` one-wave blocks fit on a CU
// (0 = no cap), in whole granules of 1/128 of the CU's LDS as the library
// reserves it (mi_reduce.hip wave_cap_bytes); one-wave blocks only
unsigned lds_for(int block, int waves_per_cu) {
    if (waves_per_cu <= 0 || block != 64) return 0;
    int dev = 0, lds = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev) != hipSuccess || lds <= 0)
        return 0;
    const unsigned g = (unsigned)lds / 128u;
    return (128u / (unsigned)waves_per_cu) * g;
}

}  // namespace

extern "C" {

// 0 or the hipError_t; -1 on bad arguments.  `bytes` per stream, a multiple
// of 16; `block` threads per block (64..1024); `waves_per_cu` 0 = uncapped;
// `flavor` as above (reads: 0, 1).
__attribute__((visibility("default"))) int mic_read_streams(const void* const* ptrs, int k, size_t bytes, int block,
                                                            int waves_per_cu, int flavor, void* sink, void* stream) {
    ReadFn fn = pick(k, flavor);
    if (!fn || !ptrs || !sink || bytes % 16 || block < 64 || block > 1024) return -1;
    ReadArgs a{};
    for (int j = 0; j < k; j++) a.in[j] = static_cast<const u32x4*>(ptrs[j]);
    a.nvec = bytes / 16;
    a.sink = static_cast<uint32_t*>(sink);
    const uint64_t blocks = (a.nvec + (uint64_t)block - 1) / (uint64_t)block;
    if (blocks == 0 || blocks > 0x7FFFFFFFull) return -1;
    return (int)fn(dim3((unsigned)blocks), dim3((unsigned)block), lds_for(block, waves_per_cu),
                   static_cast<hipStream_t>(stream), a);
}

__attribute__((visibility("default"))) int mic_write_stream(void* ptr, size_t bytes, int block, int waves_per_cu,
                                                            int flavor, void* stream) {
    if (!ptr || bytes % 16 || block < 64 || block > 1024 || flavor < 0 || flavor > 2) return -1;
    const uint64_t nvec = bytes / 16;
    const uint64_t blocks = (nvec + (uint64_t)block - 1) / (uint64_t)block;
    if (blocks == 0 || blocks > 0x7FFFFFFFull) return -1;
    const dim3 g((unsigned)blocks), b((unsigned)block);
    const unsigned lds = lds_for(block, waves_per_cu);
    hipStream_t s = static_cast<hipStream_t>(stream);
    u32x4* out = static_cast<u32x4*>(ptr);
    if (flavor == 0)
        hipLaunchKernelGGL(write_stream, g, b, lds, s, out, nvec);
    else if (flavor == 1)
        hipLaunchKernelGGL(write_stream_buf<kAuxNT>, g, b, lds, s, out, nvec);
    else
        hipLaunchKernelGGL(write_stream_buf<kAuxSC1NT>, g, b, lds, s, out, nvec);
    return (int)hipGetLastError();
}

// K read streams and one write stream in one launch (see mixed_streams):
// `flavor` 0 = global nt loads + nt stores, 1 = buffer nt loads + nt stores
// (the fan-in's), 2 = buffer nt loads + sc1 nt stores (the 2-input kernel's).
// `out` may be ptrs[0] (in place, as ccl_comp_reduce).  0, the hipError_t,
// or -1 on bad arguments.
__attribute__((visibility("default"))) int mic_mixed_streams(const void* const* ptrs, int k, void* out, size_t bytes,
                                                             int block, int waves_per_cu, int flavor, void* stream) {
    MixFn fn = pick_mix(k, flavor);
    if (!fn || !ptrs || !out || bytes % 16 || block < 64 || block > 1024) return -1;
    MixArgs a{};
    for (int j = 0; j < k; j++) a.in[j] = static_cast<const u32x4*>(ptrs[j]);
    a.out = static_cast<u32x4*>(out);
    a.nvec = bytes / 16;
    const uint64_t blocks = (a.nvec + (uint64_t)block - 1) / (uint64_t)block;
    if (blocks == 0 || blocks > 0x7FFFFFFFull) return -1;
    return (int)fn(dim3((unsigned)blocks), dim3((unsigned)block), lds_for(block, waves_per_cu),
                   static_cast<hipStream_t>(stream), a);
}

// sum2_buffer (see above): io += in over `bytes` of fp32, one-wave
// workgroups capped at `waves_per_cu` (0 = no cap); flavor 1 = nt stores,
// 2 = sc1 nt (the library's).  `sink`: 64 uint32 of device memory.
__attribute__((visibility("default"))) int mic_sum2_buffer(const void* in, void* io, size_t bytes, int waves_per_cu,
                                                           int flavor, void* sink, void* stream) {
    if (!in || !io || !sink || bytes % 16 || (flavor != 1 && flavor != 2)) return -1;
    const uint64_t nvec = bytes / 16;
    const uint64_t blocks = (nvec + 63) / 64;
    if (blocks == 0 || blocks > 0x7FFFFFFFull) return -1;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const unsigned lds = lds_for(64, waves_per_cu);
    if (flavor == 1)
        hipLaunchKernelGGL(sum2_buffer<kAuxNT>, dim3((unsigned)blocks), dim3(64), lds, s, in, io, nvec,
                           static_cast<uint32_t*>(sink));
    else
        hipLaunchKernelGGL(sum2_buffer<kAuxSC1NT>, dim3((unsigned)blocks), dim3(64), lds, s, in, io, nvec,
                           static_cast<uint32_t*>(sink));
    return (int)hipGetLastError();
}

// burst_streams (see above): K reads and one write, each workgroup of
// `block` threads a run of `tiles` tiles; `lds` 1 parks the outputs in LDS
// (tiles x block x 16 bytes per workgroup, at most 160 KiB), 0 in registers
// (tiles <= 4); `waves_per_cu` > 0 adds idle LDS to cap one-wave residency
// (register mode only); flavor 1 = nt stores, 2 = sc1 nt.  K in {2, 8}.
__attribute__((visibility("default"))) int mic_burst_streams(const void* const* ptrs, int k, void* out, size_t bytes,
                                                             int block, int tiles, int lds, int waves_per_cu,
                                                             int flavor, void* stream) {
    MixFn fn = k == 2 ? pick_burst_k<2>(tiles, lds != 0, flavor) : k == 8 ? pick_burst_k<8>(tiles, lds != 0, flavor)
                                                                      : nullptr;
    if (!fn || !ptrs || !out || bytes % 16 || block < 64 || block > 1024 || block % 64) return -1;
    const size_t stage = lds ? (size_t)tiles * (size_t)block * 16u : 0;
    if (stage > 160u * 1024u) return -1;
    MixArgs a{};
    for (int j = 0; j < k; j++) a.in[j] = static_cast<const u32x4*>(ptrs[j]);
    a.out = static_cast<u32x4*>(out);
    a.nvec = bytes / 16;
    const uint64_t per = (uint64_t)block * (uint64_t)tiles;
    const uint64_t blocks = (a.nvec + per - 1) / per;
    if (blocks == 0 || blocks > 0x7FFFFFFFull) return -1;
    const unsigned cap = lds ? 0u : lds_for(block, waves_per_cu);
    return (int)fn(dim3((unsigned)blocks), dim3((unsigned)block), (unsigned)stage > cap ? (unsigned)stage : cap,
                   static_cast<hipStream_t>(stream), a);
}

}  // extern "C"
