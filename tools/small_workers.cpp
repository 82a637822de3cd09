// Small host reduces through the drop-in (mi_ccl_comp_reduce, fp32 sum, the
// CPU path) from T threads at once: us per call, median over threads.
//   small_workers T [elements=1024] [reg]   (reg: the buffers are registered as host
//   buffers first, mi_ccl_comp_register_host_buffer, so no HIP pointer lookup runs)
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>
#include <algorithm>
#include <string>
#include "mi_ccl_comp.h"
int main(int argc, char** argv) {
    const int T = atoi(argv[1]);
    const size_t n = argc > 2 ? strtoull(argv[2], 0, 10) : 1024;
    const bool reg = argc > 3 && std::string(argv[3]) == "reg";
    const int iters = 200000;
    std::vector<double> us(T);
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++)
        th.emplace_back([&, t] {
            std::vector<float> a(n, 1.f), b(n, 1.f);
            if (reg) {
                mi_ccl_comp_register_host_buffer(a.data(), n * sizeof(float));
                mi_ccl_comp_register_host_buffer(b.data(), n * sizeof(float));
            }
            for (int i = 0; i < 2000; i++) mi_ccl_comp_reduce(a.data(), n, b.data(), nullptr, 9, 0);
            auto t0 = std::chrono::steady_clock::now();
            for (int i = 0; i < iters; i++) mi_ccl_comp_reduce(a.data(), n, b.data(), nullptr, 9, 0);
            us[t] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / iters;
            if (reg) {
                mi_ccl_comp_unregister_host_buffer(a.data());
                mi_ccl_comp_unregister_host_buffer(b.data());
            }
        });
    for (auto& x : th) x.join();
    std::sort(us.begin(), us.end());
    printf("%sT=%d n=%zu median %.3f us/call max %.3f\n", reg ? "registered: " : "", T, n, us[T / 2], us[T - 1]);
    fflush(stdout);
}
