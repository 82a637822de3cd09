// unaligned_probe.hip — do 16-byte vector loads from element-aligned but not
// 16-byte-aligned addresses return the right bytes on gfx950 (global_load_
// dwordx4 and buffer_load_dwordx4), and at what stream rate?  Decides whether
// operands with different misalignments (oneCCL ring chunks) can take the
// vector kernels instead of the element loop.
//
//   tools/unaligned_probe [MiB]
// One JSON line per (form, byte offset): correct, TB/s of a read+write copy.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define HC(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));      \
            exit(2);                                                                               \
        }                                                                                          \
    } while (0)

// dst[v] = src_bytes[off + 16 v .. +16] (dst aligned), global loads
__global__ __launch_bounds__(1024) void copy_global(const char* __restrict__ src, u32x4* __restrict__ dst,
                                                    uint64_t nvec) {
    const uint64_t v = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
    if (v < nvec) {
        const u32x4* p = reinterpret_cast<const u32x4*>(src + 16 * v);
        __builtin_nontemporal_store(__builtin_nontemporal_load(p), dst + v);
    }
}

// the same with buffer loads (descriptor base = the unaligned address)
__global__ __launch_bounds__(1024) void copy_buffer(const char* __restrict__ src, u32x4* __restrict__ dst,
                                                    uint64_t nvec) {
    const uint64_t t0 = (uint64_t)blockIdx.x * 1024;
    if (t0 >= nvec) return;
    const uint64_t left = nvec - t0;
    const uint32_t bytes = (uint32_t)(left < 1024 ? left : 1024) * 16u;
    __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(src + 16 * t0), (short)0, (int)bytes, 0x00020000);
    const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(r, threadIdx.x * 16u, 0, 2);
    if (t0 + threadIdx.x < nvec) __builtin_nontemporal_store(x, dst + t0 + threadIdx.x);
}

int main(int argc, char** argv) {
    const size_t mib = argc > 1 ? (size_t)atoi(argv[1]) : 256;
    const uint64_t nvec = (mib << 20) / 16;
    const size_t bytes = nvec * 16 + 64;
    char* src;
    u32x4* dst;
    HC(hipMalloc(&src, bytes));
    HC(hipMalloc(&dst, nvec * 16));
    std::vector<unsigned char> h(bytes);
    for (size_t i = 0; i < bytes; i++) h[i] = (unsigned char)(i * 131u + (i >> 8) * 7u + 3u);
    HC(hipMemcpy(src, h.data(), bytes, hipMemcpyHostToDevice));
    std::vector<unsigned char> got(nvec * 16);
    hipEvent_t e0, e1;
    HC(hipEventCreate(&e0));
    HC(hipEventCreate(&e1));
    const int offs[] = {0, 1, 2, 4, 8, 12};
    for (int form = 0; form < 2; form++) {
        for (int off : offs) {
            const dim3 grid((unsigned)((nvec + 1023) / 1024));
            HC(hipMemset(dst, 0, nvec * 16));
            if (form == 0)
                hipLaunchKernelGGL(copy_global, grid, dim3(1024), 0, 0, src + off, dst, nvec);
            else
                hipLaunchKernelGGL(copy_buffer, grid, dim3(1024), 0, 0, src + off, dst, nvec);
            HC(hipGetLastError());
            HC(hipDeviceSynchronize());
            HC(hipMemcpy(got.data(), dst, nvec * 16, hipMemcpyDeviceToHost));
            const bool ok = memcmp(got.data(), h.data() + off, nvec * 16) == 0;
            float best = 1e30f;
            for (int r = 0; r < 10; r++) {
                HC(hipEventRecord(e0, 0));
                if (form == 0)
                    hipLaunchKernelGGL(copy_global, grid, dim3(1024), 0, 0, src + off, dst, nvec);
                else
                    hipLaunchKernelGGL(copy_buffer, grid, dim3(1024), 0, 0, src + off, dst, nvec);
                HC(hipEventRecord(e1, 0));
                HC(hipEventSynchronize(e1));
                float ms = 0;
                HC(hipEventElapsedTime(&ms, e0, e1));
                best = ms < best ? ms : best;
            }
            printf("{\"form\": \"%s\", \"byte_offset\": %d, \"correct\": %s, \"best_ms\": %.4f, \"TB_s\": %.3f}\n",
                   form == 0 ? "global_load_dwordx4" : "buffer_load_dwordx4", off, ok ? "true" : "false", best,
                   2.0 * nvec * 16 / (best * 1e-3) / 1e12);
            fflush(stdout);
        }
    }
    HC(hipFree(src));
    HC(hipFree(dst));
    return 0;
}
