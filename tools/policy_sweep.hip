// policy_sweep.hip — experiment: fp32 2-input sum over a 1 GiB bucket with
// one-shot grids, varying block size, vectors per lane, the load/store
// cache-policy bits (buffer ops: aux bit0 = sc0, bit1 = nt, bit4 = sc1) and
// the block -> tile mapping (linear vs XCD-contiguous).  Interleaved rounds,
// one process.  Output: one JSON object per variant.
//   policy_sweep [bucket_MiB=1024] [rounds=5] [reps=10]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e = (x);                                                              \
        if (e != hipSuccess) {                                                           \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// MAP 0: tile = blockIdx.x.  MAP 1: blocks b, b+8, ... (one XCD under the
// observed round-robin dispatch) take a contiguous 1/8 of the tiles.
template <int MAP>
__device__ __forceinline__ uint32_t tile_of(uint32_t b, uint32_t g) {
    if constexpr (MAP == 0) return b;
    const uint32_t per = g / 8;  // host guarantees g % 8 == 0
    return (b % 8) * per + b / 8;
}

template <int B, int U, int LP, int SP, int MAP>
__global__ __launch_bounds__(B) void k_buffer(const float* in, float* io, uint32_t tiles) {
    const uint32_t t = tile_of<MAP>(blockIdx.x, gridDim.x);
    if (t >= tiles) return;
    const size_t tb = (size_t)B * U * 16;
    const char* pin = reinterpret_cast<const char*>(in) + t * tb;
    char* pio = reinterpret_cast<char*>(io) + t * tb;
    __amdgpu_buffer_rsrc_t ri = __builtin_amdgcn_make_buffer_rsrc((void*)pin, (short)0, (int)tb, 0x00020000);
    __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void*)pio, (short)0, (int)tb, 0x00020000);
    u32x4 a[U], b[U];
#pragma unroll
    for (int j = 0; j < U; j++) a[j] = __builtin_amdgcn_raw_buffer_load_b128(ro, (threadIdx.x + j * B) * 16, 0, LP);
#pragma unroll
    for (int j = 0; j < U; j++) b[j] = __builtin_amdgcn_raw_buffer_load_b128(ri, (threadIdx.x + j * B) * 16, 0, LP);
#pragma unroll
    for (int j = 0; j < U; j++) {
        f32x4 x = __builtin_bit_cast(f32x4, a[j]) + __builtin_bit_cast(f32x4, b[j]);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, x), ro, (threadIdx.x + j * B) * 16, 0, SP);
    }
}

template <int B, int U, int NT, int MAP>
__global__ __launch_bounds__(B) void k_global(const u32x4* in, u32x4* io, uint32_t tiles) {
    const uint32_t t = tile_of<MAP>(blockIdx.x, gridDim.x);
    if (t >= tiles) return;
    const size_t base = (size_t)t * B * U + threadIdx.x;
    u32x4 a[U], b[U];
#pragma unroll
    for (int j = 0; j < U; j++) a[j] = NT ? __builtin_nontemporal_load(io + base + j * B) : io[base + j * B];
#pragma unroll
    for (int j = 0; j < U; j++) b[j] = NT ? __builtin_nontemporal_load(in + base + j * B) : in[base + j * B];
#pragma unroll
    for (int j = 0; j < U; j++) {
        f32x4 x = __builtin_bit_cast(f32x4, a[j]) + __builtin_bit_cast(f32x4, b[j]);
        __builtin_nontemporal_store(__builtin_bit_cast(u32x4, x), io + base + j * B);
    }
}

// write-only streams: store form / cache bits / tile size
template <int B, int U, int SP>
__global__ __launch_bounds__(B) void w_buffer(float* o, uint32_t tiles) {
    const uint32_t t = blockIdx.x;
    if (t >= tiles) return;
    const size_t tb = (size_t)B * U * 16;
    char* po = reinterpret_cast<char*>(o) + t * tb;
    __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void*)po, (short)0, (int)tb, 0x00020000);
#pragma unroll
    for (int j = 0; j < U; j++)
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{t, (uint32_t)j, threadIdx.x, 7u}, ro, (threadIdx.x + j * B) * 16, 0, SP);
}

template <int B, int U>
__global__ __launch_bounds__(B) void w_b64(uint64_t* o, uint32_t tiles) {  // 8-byte stores, nt
    const uint32_t t = blockIdx.x;
    if (t >= tiles) return;
    const size_t base = (size_t)t * B * U * 2 + threadIdx.x;
#pragma unroll
    for (int j = 0; j < 2 * U; j++) __builtin_nontemporal_store((uint64_t)(base + j), o + base + (size_t)j * B);
}

// grid-stride streams, the shape of the runtime's fill kernel
// (__amd_rocclr_fillBufferAligned: one 16-B element per lane per iteration,
// pointer advanced by the whole grid)
template <int B, int NT>
__global__ __launch_bounds__(B) void w_stride(u32x4* o, size_t nvec) {
    const size_t step = (size_t)gridDim.x * B;
    for (size_t i = (size_t)blockIdx.x * B + threadIdx.x; i < nvec; i += step) {
        const u32x4 v{(uint32_t)i, 1u, 2u, 3u};
        if (NT) __builtin_nontemporal_store(v, o + i);
        else o[i] = v;
    }
}

template <int B, int NT>
__global__ __launch_bounds__(B) void k_stride(const u32x4* in, u32x4* io, size_t nvec) {
    const size_t step = (size_t)gridDim.x * B;
    for (size_t i = (size_t)blockIdx.x * B + threadIdx.x; i < nvec; i += step) {
        const u32x4 a = __builtin_nontemporal_load(io + i), b = __builtin_nontemporal_load(in + i);
        const u32x4 x = __builtin_bit_cast(u32x4, __builtin_bit_cast(f32x4, a) + __builtin_bit_cast(f32x4, b));
        if (NT) __builtin_nontemporal_store(x, io + i);
        else io[i] = x;
    }
}

// persistent sweep with U vectors per lane per iteration: the grid walks one
// contiguous window of gridDim*B*U vectors at a time (block b owns the b-th
// B*U slice of the window)
template <int B, int U, int NT>
__global__ __launch_bounds__(B) void k_window(const u32x4* in, u32x4* io, size_t nvec) {
    const size_t win = (size_t)gridDim.x * B * U;
    for (size_t w = (size_t)blockIdx.x * B * U + threadIdx.x; w + (U - 1) * B < nvec; w += win) {
        u32x4 a[U], b[U];
#pragma unroll
        for (int j = 0; j < U; j++) a[j] = __builtin_nontemporal_load(io + w + j * B);
#pragma unroll
        for (int j = 0; j < U; j++) b[j] = __builtin_nontemporal_load(in + w + j * B);
#pragma unroll
        for (int j = 0; j < U; j++) {
            const u32x4 x = __builtin_bit_cast(u32x4, __builtin_bit_cast(f32x4, a[j]) + __builtin_bit_cast(f32x4, b[j]));
            if (NT) __builtin_nontemporal_store(x, io + w + j * B);
            else io[w + j * B] = x;
        }
    }
}

// K-input fan-in, in place into input 0 (comp.cpp:217-241 semantics), buffer
// ops with load/store aux bits LP/SP; LAST0 loads input 0 last (closest to
// its store)
template <int K, int B, int LP, int SP, int LAST0>
__global__ __launch_bounds__(B) void k_fan(const float* const* ins, uint32_t tiles) {
    const uint32_t t = blockIdx.x;
    if (t >= tiles) return;
    const int tb = B * 16;
    u32x4 x[K];
#pragma unroll
    for (int jj = 0; jj < K; jj++) {
        const int j = LAST0 ? (jj + 1) % K : jj;
        __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(reinterpret_cast<const char*>(ins[j]) + (size_t)t * tb), (short)0, tb, 0x00020000);
        x[j] = __builtin_amdgcn_raw_buffer_load_b128(r, threadIdx.x * 16, 0, LP);
    }
    f32x4 acc = __builtin_bit_cast(f32x4, x[0]);
#pragma unroll
    for (int j = 1; j < K; j++) acc += __builtin_bit_cast(f32x4, x[j]);
    __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(reinterpret_cast<const char*>(ins[0]) + (size_t)t * tb), (short)0, tb, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc), ro, threadIdx.x * 16, 0, SP);
}

struct Variant {
    std::string name;
    std::function<void(hipStream_t)> run;
    std::vector<float> ms;
};

size_t g_nvec;
const float* g_in;
float* g_io;

template <int B, int U, int NT>
void addwin(std::vector<Variant>& vs, int grid) {
    char name[128];
    snprintf(name, sizeof name, "window B=%d U=%d grid=%d st=%s", B, U, grid, NT ? "nt" : "plain");
    const u32x4* in = (const u32x4*)g_in;
    u32x4* io = (u32x4*)g_io;
    const size_t nv = g_nvec;
    vs.push_back({name, [=](hipStream_t s) { hipLaunchKernelGGL((k_window<B, U, NT>), dim3(grid), dim3(B), 0, s, in, io, nv); }, {}});
}

template <int B, int U, int LP, int SP, int MAP>
void addb(std::vector<Variant>& vs) {
    const uint32_t tiles = (uint32_t)(g_nvec / (B * U));
    uint32_t grid = tiles;
    if (MAP) grid = (tiles + 7) / 8 * 8;
    char name[128];
    snprintf(name, sizeof name, "buffer B=%d U=%d ld=%d st=%d map=%d", B, U, LP, SP, MAP);
    const float* in = g_in;
    float* io = g_io;
    vs.push_back({name, [=](hipStream_t s) {
                      hipLaunchKernelGGL((k_buffer<B, U, LP, SP, MAP>), dim3(grid), dim3(B), 0, s, in, io, tiles);
                  }, {}});
}

template <int B, int U, int NT, int MAP>
void addg(std::vector<Variant>& vs) {
    const uint32_t tiles = (uint32_t)(g_nvec / (B * U));
    uint32_t grid = tiles;
    if (MAP) grid = (tiles + 7) / 8 * 8;
    char name[128];
    snprintf(name, sizeof name, "global B=%d U=%d nt=%d map=%d", B, U, NT, MAP);
    const u32x4* in = (const u32x4*)g_in;
    u32x4* io = (u32x4*)g_io;
    vs.push_back({name, [=](hipStream_t s) {
                      hipLaunchKernelGGL((k_global<B, U, NT, MAP>), dim3(grid), dim3(B), 0, s, in, io, tiles);
                  }, {}});
}

int main(int argc, char** argv) {
    const size_t mib = argc > 1 ? strtoull(argv[1], nullptr, 10) : 1024;
    const int rounds = argc > 2 ? atoi(argv[2]) : 5;
    const int reps = argc > 3 ? atoi(argv[3]) : 10;
    const size_t bytes = mib << 20;
    float *in, *io;
    CK(hipMalloc(&in, bytes));
    CK(hipMalloc(&io, bytes));
    CK(hipMemset(in, 0x3c, bytes));
    CK(hipMemset(io, 0x3c, bytes));
    g_nvec = bytes / 16;
    g_in = in;
    g_io = io;
    hipStream_t s;
    CK(hipStreamCreate(&s));

    std::vector<Variant> vs;
    addg<256, 4, 1, 0>(vs);
    addg<1024, 1, 1, 0>(vs);  // == the library's 2-input configuration
    // fan-in K=8, in place
    std::vector<float*> fan8(8);
    fan8[0] = g_io;
    fan8[1] = const_cast<float*>(g_in);
    for (int j = 2; j < 8; j++) {
        CK(hipMalloc(&fan8[j], bytes));
        CK(hipMemset(fan8[j], 0x3c, bytes));
    }
    float** d_fan8 = nullptr;
    CK(hipMalloc(&d_fan8, 8 * sizeof(float*)));
    CK(hipMemcpy(d_fan8, fan8.data(), 8 * sizeof(float*), hipMemcpyHostToDevice));
    {
        const uint32_t tiles = (uint32_t)(g_nvec / 1024), tiles256 = (uint32_t)(g_nvec / 256);
        const float* const* dp = d_fan8;
#define FAN(B, LP, SP, L0, T)                                                                                     \
    vs.push_back({"FAN8 B=" #B " ld=" #LP " st=" #SP " last0=" #L0, [=](hipStream_t st) {                        \
                      hipLaunchKernelGGL((k_fan<8, B, LP, SP, L0>), dim3(T), dim3(B), 0, st, dp, T);               \
                  }, {}})
        FAN(1024, 2, 2, 0, tiles);
        FAN(1024, 2, 0, 0, tiles);
        FAN(1024, 2, 16, 0, tiles);
        FAN(1024, 2, 18, 0, tiles);
        FAN(1024, 0, 2, 0, tiles);
        FAN(1024, 18, 2, 0, tiles);
        FAN(1024, 2, 2, 1, tiles);
        FAN(256, 2, 2, 0, tiles256);
        FAN(256, 2, 0, 0, tiles256);
        FAN(256, 2, 2, 1, tiles256);
#undef FAN
    }
    for (int g : {256}) {
        addwin<256, 4, 1>(vs, g);
        addwin<256, 8, 1>(vs, g);
    }
    {
        float* wo = io;
        auto addw = [&](const char* name, std::function<void(hipStream_t)> f) {
            vs.push_back({name, f, {}});
            vs.back().name = std::string("WRITE-ONLY ") + name;
        };
        const uint32_t t4 = (uint32_t)(g_nvec / (256 * 4)), t16 = (uint32_t)(g_nvec / (256 * 16));
        addw("buffer B=256 U=4 st=nt", [=](hipStream_t st) { hipLaunchKernelGGL((w_buffer<256, 4, 2>), dim3(t4), dim3(256), 0, st, wo, t4); });
        addw("buffer B=256 U=4 st=plain", [=](hipStream_t st) { hipLaunchKernelGGL((w_buffer<256, 4, 0>), dim3(t4), dim3(256), 0, st, wo, t4); });
        addw("buffer B=256 U=4 st=sc1", [=](hipStream_t st) { hipLaunchKernelGGL((w_buffer<256, 4, 16>), dim3(t4), dim3(256), 0, st, wo, t4); });
        addw("buffer B=256 U=4 st=sc0sc1", [=](hipStream_t st) { hipLaunchKernelGGL((w_buffer<256, 4, 17>), dim3(t4), dim3(256), 0, st, wo, t4); });
        addw("buffer B=256 U=4 st=sc1nt", [=](hipStream_t st) { hipLaunchKernelGGL((w_buffer<256, 4, 18>), dim3(t4), dim3(256), 0, st, wo, t4); });
        addw("buffer B=256 U=16 st=nt", [=](hipStream_t st) { hipLaunchKernelGGL((w_buffer<256, 16, 2>), dim3(t16), dim3(256), 0, st, wo, t16); });
        addw("b64 B=256 U=4 nt", [=](hipStream_t st) { hipLaunchKernelGGL((w_b64<256, 4>), dim3(t4), dim3(256), 0, st, (uint64_t*)wo, t4); });
        for (int wg : {128, 256, 512}) {
            char name[96];
            const size_t nv = g_nvec;
            snprintf(name, sizeof name, "stride B=256 grid=%d st=plain", wg);
            addw(name, [=](hipStream_t st) { hipLaunchKernelGGL((w_stride<256, 0>), dim3(wg), dim3(256), 0, st, (u32x4*)wo, nv); });
            snprintf(name, sizeof name, "stride B=256 grid=%d st=nt", wg);
            addw(name, [=](hipStream_t st) { hipLaunchKernelGGL((w_stride<256, 1>), dim3(wg), dim3(256), 0, st, (u32x4*)wo, nv); });
        }
        addw("hipMemsetAsync", [=](hipStream_t st) { (void)hipMemsetAsync(wo, 0, g_nvec * 16, st); });
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (auto& v : vs) v.run(s);
    CK(hipStreamSynchronize(s));
    CK(hipGetLastError());
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
        fprintf(stderr, "round %d/%d\n", r + 1, rounds);
    }
    for (auto& v : vs) {
        const double traffic = (v.name.rfind("WRITE-ONLY", 0) == 0 ? 1.0 : v.name.rfind("FAN8", 0) == 0 ? 9.0 : 3.0) * bytes;
        std::sort(v.ms.begin(), v.ms.end());
        const float med = v.ms[v.ms.size() / 2], best = v.ms.front();
        printf("{\"variant\": \"%s\", \"median_ms\": %.5f, \"best_ms\": %.5f, \"median_GBps\": %.1f, "
               "\"best_GBps\": %.1f}\n",
               v.name.c_str(), med, best, traffic / (med * 1e-3) / 1e9, traffic / (best * 1e-3) / 1e9);
    }
    return 0;
}
