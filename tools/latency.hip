// latency.hip — where the synchronous small-bucket call spends its time.
// Host wall-clock (steady_clock), min and median over many reps, one JSON
// line per item.  Links libmi_reduce.so.
//   latency [reps=2000]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>

#include "../include/mi_reduce.h"
#include "../oneccl_amd/csrc/reduce_kernels.hpp"

__global__ void empty_kernel() {}

static void measure(const char* name, int reps, const std::function<void()>& f) {
    std::vector<double> t(reps);
    for (int i = 0; i < 50; i++) f();
    for (int i = 0; i < reps; i++) {
        auto t0 = std::chrono::steady_clock::now();
        f();
        auto t1 = std::chrono::steady_clock::now();
        t[i] = std::chrono::duration<double, std::micro>(t1 - t0).count();
    }
    std::sort(t.begin(), t.end());
    printf("{\"item\": \"%s\", \"min_us\": %.2f, \"median_us\": %.2f, \"p90_us\": %.2f}\n", name, t[0],
           t[reps / 2], t[reps * 9 / 10]);
    fflush(stdout);
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 2000;
    const size_t n = 1024;  // 4 KiB fp32
    float *a, *b, *ha, *hb;
    (void)hipMalloc(&a, n * 4);
    (void)hipMalloc(&b, n * 4);
    (void)hipMemset(a, 0, n * 4);
    (void)hipMemset(b, 0, n * 4);
    (void)hipHostMalloc(&ha, n * 4, 0);
    (void)hipHostMalloc(&hb, n * 4, 0);
    std::vector<float> pa(n, 1.f), pb(n, 1.f);
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipPointerAttribute_t at;
    int dev = 0;

    measure("empty kernel launch (host side only)", reps, [&] { hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s); });
    (void)hipStreamSynchronize(s);
    measure("empty kernel launch + hipStreamSynchronize", reps, [&] {
        hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
        (void)hipStreamSynchronize(s);
    });
    measure("hipPointerGetAttributes (device ptr)", reps, [&] { (void)hipPointerGetAttributes(&at, a); });
    measure("hipPointerGetAttributes (pageable ptr)", reps, [&] {
        if (hipPointerGetAttributes(&at, pa.data()) != hipSuccess) (void)hipGetLastError();
    });
    measure("hipGetDevice + hipSetDevice", reps, [&] {
        (void)hipGetDevice(&dev);
        (void)hipSetDevice(dev);
    });
    mi::R2Args r{};
    r.acc = b;
    r.in = a;
    r.out = b;
    r.nvec = n / 4;
    r.trunc_from = n;
    measure("reduce2_kernel direct hipLaunchKernelGGL (host side)", reps, [&] {
        hipLaunchKernelGGL((mi::reduce2_kernel<float, 0, 0u, 1, 1024>), dim3(1), dim3(1024), 0, s, r);
    });
    (void)hipStreamSynchronize(s);
    measure("reduce2_kernel direct launch + hipGetLastError", reps, [&] {
        hipLaunchKernelGGL((mi::reduce2_kernel<float, 0, 0u, 1, 1024>), dim3(1), dim3(1024), 0, s, r);
        (void)hipGetLastError();
    });
    (void)hipStreamSynchronize(s);
    measure("hipGetLastError alone", reps, [&] { (void)hipGetLastError(); });
    measure("mi_reduce 4 KiB (async launch, host side)", reps, [&] { mi_reduce(a, b, n, MI_FLOAT32, MI_OP_SUM, 0, s); });
    (void)hipStreamSynchronize(s);
    measure("mi_reduce 4 KiB + hipStreamSynchronize", reps, [&] {
        mi_reduce(a, b, n, MI_FLOAT32, MI_OP_SUM, 0, s);
        (void)hipStreamSynchronize(s);
    });
    measure("mi_reduce_sync 4 KiB device", reps, [&] { mi_reduce_sync(a, b, n, MI_FLOAT32, MI_OP_SUM, 0, -1); });
    measure("mi_reduce_sync 4 KiB pinned host (zero-copy)", reps, [&] { mi_reduce_sync(ha, hb, n, MI_FLOAT32, MI_OP_SUM, 0, -1); });
    {
        const void* ins[2] = {b, a};
        measure("mi_reduce_start + mi_wait + mi_request_free 4 KiB device", reps, [&] {
            mi_request_t r = nullptr;
            mi_reduce_start(ins, 2, b, n, MI_FLOAT32, MI_OP_SUM, 0, -1, &r);
            mi_wait(r);
            mi_request_free(r);
        });
        measure("mi_reduce_start + mi_request_free 4 KiB device (host side; a device request's free does not wait)",
                reps / 4, [&] {
                    mi_request_t r = nullptr;
                    mi_reduce_start(ins, 2, b, n, MI_FLOAT32, MI_OP_SUM, 0, -1, &r);
                    mi_request_free(r);
                });
        (void)hipDeviceSynchronize();
    }
    measure("mi_reduce_sync 4 KiB pageable host (bounce)", reps / 4,
            [&] { mi_reduce_sync(pa.data(), pb.data(), n, MI_FLOAT32, MI_OP_SUM, 0, -1); });
    return 0;
}
