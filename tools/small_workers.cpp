// Small host reduces (fp32 sum, the CPU path) from T threads at once, each
// on its own buffers: us per call, median and max over the threads.
//   small_workers T [elements=1024] [mode=default]
// modes:
//   default  mi_ccl_comp_reduce with no schedule: every operand looked up
//   reg      the buffers registered first (mi_ccl_comp_register_host_buffer)
//   sched    the call made under a schedule without a stream
//            (mi_ccl_comp_shim_sched(1)): host memory by the schedule's word,
//            nothing looked up -- what reduce_local_entry / recv_reduce_entry
//            pass in a CPU oneCCL build (the reference's comp.cpp:136-142)
//   ref      the reference's own compiled ccl_comp_reduce_regular
//            (oracle/_ref/libref_ccl_comp.so, dlopen'ed lazily): the CPU loop
//            the drop-in must not lose to
//   copy     ccl_comp_copy of the buffer (classifies both pointers)
//   copyhost ccl_comp_copy_host, the copy entries' call after
//            integration/0006 (host to host, nothing looked up)
//   memcpy   plain memcpy: the reference's ccl_comp_copy (comp.cpp:60-74)
// Also prints the HIP pointer lookups the drop-in made per call.
#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "mi_ccl_comp.h"

typedef int (*ref_reduce_t)(const void*, size_t, void*, size_t*, int, size_t, int);

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: small_workers T [elements] [default|reg|sched|ref]\n");
        return 2;
    }
    const int T = atoi(argv[1]);
    const size_t n = argc > 2 ? strtoull(argv[2], 0, 10) : 1024;
    const std::string mode = argc > 3 ? argv[3] : "default";
    ref_reduce_t ref = nullptr;
    if (mode == "ref") {
        const char* path = getenv("REF_COMP_SO") ? getenv("REF_COMP_SO") : "oracle/_ref/libref_ccl_comp.so";
        void* h = dlopen(path, RTLD_LAZY | RTLD_LOCAL);
        if (!h || !(ref = (ref_reduce_t)dlsym(h, "ref_ccl_comp_reduce_regular"))) {
            fprintf(stderr, "cannot load %s: %s\n", path, dlerror());
            return 2;
        }
    }
    // about 0.2 s of work per thread at the size measured alone
    const long iters = std::max<long>(2000, (long)(400000000.0 / (double)(n + 256)));
    std::vector<double> us(T);
    std::vector<double> lookups(T);
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++)
        th.emplace_back([&, t] {
            std::vector<float> a(n, 1.f), b(n, 1.f);
            if (mode == "reg") {
                mi_ccl_comp_register_host_buffer(a.data(), n * sizeof(float));
                mi_ccl_comp_register_host_buffer(b.data(), n * sizeof(float));
            }
            if (mode == "sched") mi_ccl_comp_shim_sched(1);
            const size_t nb = n * sizeof(float);
            auto call = [&] {
                if (ref) ref(a.data(), n, b.data(), nullptr, 9, sizeof(float), 0);
                else if (mode == "copy") mi_ccl_comp_copy(a.data(), b.data(), nb, 0);
                else if (mode == "copyhost") mi_ccl_comp_copy_host(a.data(), b.data(), nb, 0);
                else if (mode == "memcpy") memcpy(b.data(), a.data(), nb);
                else mi_ccl_comp_reduce(a.data(), n, b.data(), nullptr, 9, 0);
            };
            for (long i = 0; i < std::min<long>(2000, iters); i++) call();
            const size_t l0 = mi_ccl_comp_pointer_lookups();
            auto t0 = std::chrono::steady_clock::now();
            for (long i = 0; i < iters; i++) call();
            us[t] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / iters;
            lookups[t] = (double)(mi_ccl_comp_pointer_lookups() - l0) / (double)iters;
            if (mode == "reg") {
                mi_ccl_comp_unregister_host_buffer(a.data());
                mi_ccl_comp_unregister_host_buffer(b.data());
            }
        });
    for (auto& x : th) x.join();
    std::vector<double> s = us;
    std::sort(s.begin(), s.end());
    const double lk = *std::max_element(lookups.begin(), lookups.end());
    // roctx ranges are on only under CCL_ITT_LEVEL > 0 or MI_ROCTX=1 (comp.cpp)
    const char* mi = getenv("MI_ROCTX");
    const char* itt = getenv("CCL_ITT_LEVEL");
    const bool roctx_on = mi ? strcmp(mi, "0") != 0 : (itt && atoi(itt) > 0);
    printf("{\"mode\": \"%s%s\", \"threads\": %d, \"elements\": %zu, \"bytes\": %zu, \"median_us\": %.3f, "
           "\"max_us\": %.3f, \"lookups_per_call\": %.2f, \"iters\": %ld}\n",
           mode.c_str(), roctx_on ? " (roctx on)" : "", T, n, n * sizeof(float), s[T / 2], s[T - 1], lk, iters);
    fflush(stdout);
}
