// small_sweep.hip — block size of the lean 2-input kernel for small buckets
// (C5's latency end): with 1024-lane tiles a 1 MiB fp32 bucket is 64 blocks,
// a quarter of the CUs.  Times reduce2_kernel<float, sum> at 256/512/1024
// lanes per block for 16 KiB .. 64 MiB buckets, interleaved, hipEvent median
// of `reps` launches back to back on one stream.
//   small_sweep [reps=200]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../oneccl_amd/csrc/reduce_kernels.hpp"

using namespace mi;

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e = (x);                                                                    \
        if (e != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e));   \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

template <int B>
void launch(const R2Args& r, uint64_t nvec, hipStream_t s) {
    const uint64_t blocks = std::max<uint64_t>((nvec + B - 1) / B, 1);
    hipLaunchKernelGGL((reduce2_kernel<float, 0, 0u, 1, B>), dim3((unsigned)blocks), dim3(B), 0, s, r);
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 200;
    const size_t maxb = 64u << 20;
    float *a, *b;
    CK(hipMalloc(&a, maxb));
    CK(hipMalloc(&b, maxb));
    CK(hipMemset(a, 0, maxb));
    CK(hipMemset(b, 0, maxb));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::vector<hipEvent_t> ev(2 * reps);
    for (auto& evt : ev) CK(hipEventCreate(&evt));
    for (size_t bytes = 16u << 10; bytes <= maxb; bytes *= 4) {
        const uint64_t nvec = bytes / 16;
        R2Args r{};
        r.acc = b;
        r.in = a;
        r.out = b;
        r.nvec = nvec;
        r.trunc_from = bytes / 4;
        for (int B : {1024, 512, 256}) {
            auto go = [&] {
                if (B == 1024) launch<1024>(r, nvec, s);
                else if (B == 512) launch<512>(r, nvec, s);
                else launch<256>(r, nvec, s);
            };
            for (int i = 0; i < 20; i++) go();
            for (int i = 0; i < reps; i++) {
                CK(hipEventRecord(ev[2 * i], s));
                go();
                CK(hipEventRecord(ev[2 * i + 1], s));
            }
            CK(hipStreamSynchronize(s));
            std::vector<float> ms(reps);
            for (int i = 0; i < reps; i++) CK(hipEventElapsedTime(&ms[i], ev[2 * i], ev[2 * i + 1]));
            std::sort(ms.begin(), ms.end());
            const double med = ms[reps / 2];
            printf("{\"bucket_KiB\": %zu, \"block\": %d, \"blocks\": %llu, \"median_us\": %.2f, \"min_us\": %.2f, "
                   "\"TB_s\": %.3f}\n",
                   bytes >> 10, B, (unsigned long long)((nvec + B - 1) / B), med * 1e3, ms[0] * 1e3,
                   3.0 * bytes / (med * 1e-3) / 1e12);
            fflush(stdout);
        }
    }
    return 0;
}
