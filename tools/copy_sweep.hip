// copy_sweep.hip — the device copy behind ccl_comp_copy (mi_copy, SURVEY §8
// a13 / (f)3: copy_lean_kernel, and copy_kernel under a grid cap) against
// round 1's copy_kernel<2> default, other shapes of the same 16-byte copy and
// hipMemcpy D2D, interleaved in one process on a 1 GiB buffer.  Also each shape with the
// source 4 bytes off the destination's 16-byte grid (mi_copy's unaligned-source
// case).  Traffic = 2 bytes per byte copied.
// Then the conversion kernel (fp32 <-> bf16 / fp16 arrays, 6 bytes per element)
// at three block sizes, unless the 4th argument is "nocvt".
//   copy_sweep [MiB=1024] [rounds=5] [reps=10] [nocvt]
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

// one 16-byte vector per lane, one tile per block, no loop (reduce2_kernel's shape)
template <int MEM, int B>
__global__ __launch_bounds__(B) void lean_copy(const u32x4* __restrict__ src, u32x4* __restrict__ dst, uint64_t nvec) {
    const uint64_t v = (uint64_t)blockIdx.x * B + threadIdx.x;
    if (v < nvec) vstore<MEM & 2>(dst + v, vload<MEM & 1>(src + v));
}

// U vectors per lane, loads first, one tile per block
template <int MEM, int B, int U>
__global__ __launch_bounds__(B) void lean_copy_u(const u32x4* __restrict__ src, u32x4* __restrict__ dst, uint64_t nvec) {
    const uint64_t base = (uint64_t)blockIdx.x * B * U + threadIdx.x;
    u32x4 r[U];
#pragma unroll
    for (int j = 0; j < U; j++)
        if (base + (uint64_t)j * B < nvec) r[j] = vload<MEM & 1>(src + base + (uint64_t)j * B);
#pragma unroll
    for (int j = 0; j < U; j++)
        if (base + (uint64_t)j * B < nvec) vstore<MEM & 2>(dst + base + (uint64_t)j * B, r[j]);
}

// grid-stride over a fixed grid (the write-only ceiling's best shape: 128-256
// workgroups of 256 lanes, plain stores), U vectors per lane per step
template <int MEM, int U>
__global__ __launch_bounds__(256) void stride_copy(const u32x4* __restrict__ src, u32x4* __restrict__ dst, uint64_t nvec) {
    const uint64_t step = (uint64_t)gridDim.x * 256 * U;
    for (uint64_t base = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; base < nvec; base += step) {
        u32x4 r[U];
#pragma unroll
        for (int j = 0; j < U; j++)
            if (base + (uint64_t)j * 256 < nvec) r[j] = vload<MEM & 1>(src + base + (uint64_t)j * 256);
#pragma unroll
        for (int j = 0; j < U; j++)
            if (base + (uint64_t)j * 256 < nvec) vstore<MEM & 2>(dst + base + (uint64_t)j * 256, r[j]);
    }
}

struct Variant {
    std::string name;
    std::function<void(hipStream_t)> run;
    std::vector<float> ms;
    double traffic = 0;  // bytes per launch; 0 = 2 x the buffer (a copy)
};

// the library's conversion kernel (ccl_convert_*_arrays) at block size B:
// `count` elements, both buffers 16-byte aligned
template <typename ST, typename DT, unsigned V, int B>
void add_convert(std::vector<Variant>& vs, const char* label, const void* src, void* dst, uint64_t count) {
    CArgs a{};
    a.src = src;
    a.dst = dst;
    a.count = count;
    a.head = 0;
    a.ngroups = count / 8;
    a.trunc_from = count;
    a.scalar_only = 0;
    const unsigned blocks = (unsigned)std::min<uint64_t>((a.ngroups + B - 1) / B, 1u << 20);
    const double t = (double)count * (sizeof(typename Tr<ST>::S) + sizeof(typename Tr<DT>::S));
    vs.push_back({std::string("convert ") + label + " B=" + std::to_string(B) + (B == kBlock ? " (round 2's block; the library now launches 64 lanes at 24 waves per CU, tools/occupancy_sweep.hip)" : ""),
                  [a, blocks](hipStream_t st) {
                      hipLaunchKernelGGL((convert_kernel<ST, DT, V, B>), dim3(blocks), dim3(B), 0, st, a);
                  }, {}, t});
}

int main(int argc, char** argv) {
    const size_t mib = argc > 1 ? strtoull(argv[1], nullptr, 10) : 1024;
    const int rounds = argc > 2 ? atoi(argv[2]) : 5;
    const int reps = argc > 3 ? atoi(argv[3]) : 10;
    const size_t bytes = mib << 20;
    char *src, *dst;
    CK(hipMalloc(&src, bytes + 64));
    CK(hipMalloc(&dst, bytes + 64));
    CK(hipMemset(src, 0x3c, bytes + 64));
    CK(hipMemset(dst, 0, bytes + 64));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    const uint64_t nvec = bytes / 16;

    std::vector<Variant> vs;
    for (int off : {0, 4}) {
        const char* sp = src + off;
        const std::string sfx = off ? " src+4" : "";
        const u32x4* s4 = reinterpret_cast<const u32x4*>(sp);
        u32x4* d4 = reinterpret_cast<u32x4*>(dst);
        const uint64_t b_lib = (nvec + kBlock * 4 - 1) / (kBlock * 4);
        const unsigned b_lean = (unsigned)((nvec + kCopyBlock - 1) / kCopyBlock);
        vs.push_back({"library copy_lean_kernel<3> " + std::to_string(kCopyBlock) + "x1 (nt ld, nt st)" + sfx, [=](hipStream_t st) {
                          hipLaunchKernelGGL(copy_lean_kernel<3>, dim3(b_lean), dim3(kCopyBlock), 0, st, sp, dst, 0u,
                                             nvec, 0u);
                      }, {}});
        vs.push_back({"library copy_lean_kernel<1> " + std::to_string(kCopyBlock) + "x1 (nt ld, plain st)" + sfx, [=](hipStream_t st) {
                          hipLaunchKernelGGL(copy_lean_kernel<1>, dim3(b_lean), dim3(kCopyBlock), 0, st, sp, dst, 0u,
                                             nvec, 0u);
                      }, {}});
        vs.push_back({"round-1 copy_kernel<2> 256x4 (plain ld, nt st)" + sfx, [=](hipStream_t st) {
                          hipLaunchKernelGGL(copy_kernel<2>, dim3((unsigned)b_lib), dim3(kBlock), 0, st, sp, dst, 0u,
                                             nvec, 0u);
                      }, {}});
        vs.push_back({"copy_kernel<3> 256x4 (nt ld, nt st)" + sfx, [=](hipStream_t st) {
                          hipLaunchKernelGGL(copy_kernel<3>, dim3((unsigned)b_lib), dim3(kBlock), 0, st, sp, dst, 0u,
                                             nvec, 0u);
                      }, {}});
        vs.push_back({"copy_kernel<1> 256x4 (nt ld, plain st)" + sfx, [=](hipStream_t st) {
                          hipLaunchKernelGGL(copy_kernel<1>, dim3((unsigned)b_lib), dim3(kBlock), 0, st, sp, dst, 0u,
                                             nvec, 0u);
                      }, {}});
        vs.push_back({"lean 1024x1 nt/nt" + sfx, [=](hipStream_t st) {
                          hipLaunchKernelGGL((lean_copy<3, 1024>), dim3((unsigned)((nvec + 1023) / 1024)), dim3(1024), 0,
                                             st, s4, d4, nvec);
                      }, {}});
        vs.push_back({"lean 1024x1 nt ld, plain st" + sfx, [=](hipStream_t st) {
                          hipLaunchKernelGGL((lean_copy<1, 1024>), dim3((unsigned)((nvec + 1023) / 1024)), dim3(1024), 0,
                                             st, s4, d4, nvec);
                      }, {}});
        vs.push_back({"lean 512x1 nt/nt" + sfx, [=](hipStream_t st) {
                          hipLaunchKernelGGL((lean_copy<3, 512>), dim3((unsigned)((nvec + 511) / 512)), dim3(512), 0, st,
                                             s4, d4, nvec);
                      }, {}});
        vs.push_back({"lean 256x1 nt/nt" + sfx, [=](hipStream_t st) {
                          hipLaunchKernelGGL((lean_copy<3, 256>), dim3((unsigned)((nvec + 255) / 256)), dim3(256), 0, st,
                                             s4, d4, nvec);
                      }, {}});
        vs.push_back({"lean 1024x2 nt/nt" + sfx, [=](hipStream_t st) {
                          hipLaunchKernelGGL((lean_copy_u<3, 1024, 2>), dim3((unsigned)((nvec + 2047) / 2048)), dim3(1024),
                                             0, st, s4, d4, nvec);
                      }, {}});
        for (int g : {256, 512, 1024, 2048}) {
            vs.push_back({"stride G=" + std::to_string(g) + " 256x4 nt ld, plain st" + sfx, [=](hipStream_t st) {
                              hipLaunchKernelGGL((stride_copy<1, 4>), dim3(g), dim3(256), 0, st, s4, d4, nvec);
                          }, {}});
            vs.push_back({"stride G=" + std::to_string(g) + " 256x4 nt/nt" + sfx, [=](hipStream_t st) {
                              hipLaunchKernelGGL((stride_copy<3, 4>), dim3(g), dim3(256), 0, st, s4, d4, nvec);
                          }, {}});
        }
        vs.push_back({"hipMemcpyAsync D2D" + sfx,
                      [=](hipStream_t st) { (void)hipMemcpyAsync(dst, sp, bytes, hipMemcpyDeviceToDevice, st); }, {}});
    }

    if (!(argc > 4 && std::string(argv[4]) == "nocvt")) {
        const uint64_t count = bytes / 4;  // fp32 side = the buffer, 16-bit side = half of it
        add_convert<float, bf16_tag, V_BF16_RNE, 256>(vs, "fp32->bf16 RNE", src, dst, count);
        add_convert<float, bf16_tag, V_BF16_RNE, 512>(vs, "fp32->bf16 RNE", src, dst, count);
        add_convert<float, bf16_tag, V_BF16_RNE, 1024>(vs, "fp32->bf16 RNE", src, dst, count);
        add_convert<bf16_tag, float, 0u, 256>(vs, "bf16->fp32", src, dst, count);
        add_convert<bf16_tag, float, 0u, 512>(vs, "bf16->fp32", src, dst, count);
        add_convert<bf16_tag, float, 0u, 1024>(vs, "bf16->fp32", src, dst, count);
        add_convert<float, fp16_tag, 0u, 256>(vs, "fp32->fp16", src, dst, count);
        add_convert<float, fp16_tag, 0u, 1024>(vs, "fp32->fp16", src, dst, count);
        add_convert<fp16_tag, float, 0u, 256>(vs, "fp16->fp32", src, dst, count);
        add_convert<fp16_tag, float, 0u, 1024>(vs, "fp16->fp32", src, dst, count);
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
        const double traffic = v.traffic > 0 ? v.traffic : 2.0 * bytes;
        std::sort(v.ms.begin(), v.ms.end());
        const float med = v.ms[v.ms.size() / 2], best = v.ms.front();
        printf("{\"variant\": \"%s\", \"MiB\": %zu, \"median_ms\": %.5f, \"best_ms\": %.5f, \"median_GBps\": %.1f, "
               "\"best_GBps\": %.1f, \"frac_of_8TBps\": %.4f}\n",
               v.name.c_str(), mib, med, best, traffic / (med * 1e-3) / 1e9, traffic / (best * 1e-3) / 1e9,
               traffic / (med * 1e-3) / 8e12);
    }
    return 0;
}
