// Pointer classification cost per call against the number of threads calling
// at once: hipPointerGetAttributes vs hsa_amd_pointer_info, on pageable,
// pinned (hipHostMalloc) and device (hipMalloc) memory.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>
#include <algorithm>
#include <functional>
static double run(int T, const std::function<void(int)>& f) {
    const int iters = 100000;
    std::vector<double> us(T);
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++)
        th.emplace_back([&, t] {
            for (int i = 0; i < 2000; i++) f(t);
            auto t0 = std::chrono::steady_clock::now();
            for (int i = 0; i < iters; i++) f(t);
            us[t] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / iters;
        });
    for (auto& x : th) x.join();
    std::sort(us.begin(), us.end());
    return us[T / 2];
}
int main() {
    std::vector<std::vector<float>> pg(16, std::vector<float>(1024));
    void *pin, *dev;
    (void)hipHostMalloc(&pin, 1 << 20, 0);
    (void)hipMalloc(&dev, 1 << 20);
    for (int T : {1, 4, 8, 16}) {
        for (int kind = 0; kind < 3; kind++) {
            auto ptr = [&](int t) -> void* { return kind == 0 ? (void*)pg[t].data() : kind == 1 ? pin : dev; };
            const double a = run(T, [&](int t) {
                hipPointerAttribute_t at;
                if (hipPointerGetAttributes(&at, ptr(t)) != hipSuccess) (void)hipGetLastError();
            });
            const double b = run(T, [&](int t) {
                hsa_amd_pointer_info_t info;
                info.size = sizeof(info);
                (void)hsa_amd_pointer_info(ptr(t), &info, nullptr, nullptr, nullptr);
            });
            int ok_range = 0, ok_attr = 0;
            const double c = run(T, [&](int t) {
                hipDeviceptr_t base;
                size_t size = 0;
                if (hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)ptr(t)) != hipSuccess) (void)hipGetLastError();
            });
            const double d = run(T, [&](int t) {
                unsigned int mt = 0;
                if (hipPointerGetAttribute(&mt, HIP_POINTER_ATTRIBUTE_MEMORY_TYPE, (hipDeviceptr_t)ptr(t)) != hipSuccess)
                    (void)hipGetLastError();
            });
            {
                hipDeviceptr_t base;
                size_t size = 0;
                ok_range = hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)ptr(0)) == hipSuccess;
                (void)hipGetLastError();
                unsigned int mt = 0;
                ok_attr = hipPointerGetAttribute(&mt, HIP_POINTER_ATTRIBUTE_MEMORY_TYPE, (hipDeviceptr_t)ptr(0)) == hipSuccess;
                (void)hipGetLastError();
            }
            printf("{\"threads\": %d, \"memory\": \"%s\", \"hipPointerGetAttributes_us\": %.3f, \"hsa_amd_pointer_info_us\": %.3f, "
                   "\"hipMemGetAddressRange_us\": %.3f, \"hipMemGetAddressRange_ok\": %d, \"hipPointerGetAttribute_memtype_us\": %.3f, "
                   "\"hipPointerGetAttribute_ok\": %d}\n",
                   T, kind == 0 ? "pageable" : kind == 1 ? "pinned" : "device", a, b, c, ok_range, d, ok_attr);
            fflush(stdout);
        }
    }
}
