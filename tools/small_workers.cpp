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
// The MPI user ops (atl_mpi_ctx.cpp:57-63, 87-92; bf16/fp16 sum, elements of
// 2 bytes):
//   mpibf16 / mpifp16  ccl_{bf16,fp16}_reduce_host, integration/0002's call:
//            host memory by the caller's word, nothing looked up
//   bf16 / fp16        ccl_{bf16,fp16}_reduce with no word (every operand
//            looked up): the user ops' call before that patch
//   foldbf16 / foldfp16  mi_host_reduce alone (the drop-in's CPU fold,
//            include/mi_host_reduce.h) with the avx512bf / fp16 flags: the
//            fold without the entry point around it
//   schedbf16 / schedfp16 / schedi16  ccl_comp_reduce of bf16 / fp16 /
//            int16 under a schedule without a stream
//   refbf16 / reffp16  the reference's own AVX-512 body (avx512bf /
//            avx512f impl) from oracle/_ref/libref_comp.so: what the user
//            op runs in the reference (bf16.cpp:98-109, fp16_intrisics.hpp:204)
// Also prints the HIP pointer lookups the drop-in made per call.
// SW_CPUS=c0,c1,...: thread t pins itself to c[t % n] before its buffers are
// allocated (unset: unpinned).
#include <dlfcn.h>
#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "mi_ccl_comp.h"
#include "mi_host_reduce.h"
#include "mi_reduce.h"

typedef int (*ref_reduce_t)(const void*, size_t, void*, size_t*, int, size_t, int);
typedef int (*ref_lp_t)(int, int, const uint16_t*, uint16_t*, size_t);

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: small_workers T [elements] [mode]\n");
        return 2;
    }
    const int T = atoi(argv[1]);
    const size_t n = argc > 2 ? strtoull(argv[2], 0, 10) : 1024;
    const std::string mode = argc > 3 ? argv[3] : "default";
    ref_reduce_t ref = nullptr;
    ref_lp_t ref_lp = nullptr;
    const bool lp = mode.find("bf16") != std::string::npos || mode.find("fp16") != std::string::npos ||
                    mode.find("i16") != std::string::npos;
    const size_t es = lp ? 2 : sizeof(float);
    if (mode == "refbf16" || mode == "reffp16") {
        const char* path = getenv("REF_LP_SO") ? getenv("REF_LP_SO") : "oracle/_ref/libref_comp.so";
        void* h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
        const char* sym = mode == "refbf16" ? "ref_bf16_reduce" : "ref_fp16_reduce";
        if (!h || !(ref_lp = (ref_lp_t)dlsym(h, sym))) {
            fprintf(stderr, "cannot load %s: %s\n", path, dlerror());
            return 2;
        }
    }
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
    enum {
        M_DEFAULT, M_REF, M_REFBF16, M_REFFP16, M_MPIBF16, M_MPIFP16, M_BF16, M_FP16, M_FOLDBF16, M_FOLDFP16,
        M_FOLDI16, M_FOLDF32, M_SCHEDBF16, M_SCHEDFP16, M_SCHEDI16, M_SCHEDI16_FOLDBF16, M_FOLDI16_FOLDBF16,
        M_SCHEDI16X2, M_COPY, M_COPYHOST, M_MEMCPY
    };
    const struct {
        const char* name;
        int id;
    } modes[] = {{"default", M_DEFAULT}, {"reg", M_DEFAULT}, {"sched", M_DEFAULT}, {"ref", M_REF},
                 {"refbf16", M_REFBF16}, {"reffp16", M_REFFP16}, {"mpibf16", M_MPIBF16}, {"mpifp16", M_MPIFP16},
                 {"bf16", M_BF16}, {"fp16", M_FP16}, {"foldbf16", M_FOLDBF16}, {"foldfp16", M_FOLDFP16},
                 {"foldi16", M_FOLDI16}, {"foldf32", M_FOLDF32}, {"schedbf16", M_SCHEDBF16},
                 {"schedfp16", M_SCHEDFP16}, {"schedi16", M_SCHEDI16}, {"schedi16+foldbf16", M_SCHEDI16_FOLDBF16},
                 {"foldi16+foldbf16", M_FOLDI16_FOLDBF16}, {"schedi16x2", M_SCHEDI16X2}, {"copy", M_COPY},
                 {"copyhost", M_COPYHOST}, {"memcpy", M_MEMCPY}};
    int mid = -1;
    for (const auto& m : modes)
        if (mode == m.name) mid = m.id;
    if (mid < 0) {
        fprintf(stderr, "unknown mode %s\n", mode.c_str());
        return 2;
    }
    std::vector<int> pin;
    if (const char* v = getenv("SW_CPUS"))
        for (const char* c = v; *c;) {
            pin.push_back(atoi(c));
            while (*c && *c != ',') c++;
            if (*c == ',') c++;
        }
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++)
        th.emplace_back([&, t] {
            if (!pin.empty()) {
                cpu_set_t cs;
                CPU_ZERO(&cs);
                CPU_SET(pin[t % pin.size()], &cs);
                pthread_setaffinity_np(pthread_self(), sizeof(cs), &cs);
            }
            std::vector<float> a(n, 1.f), b(n, 1.f);
            // 2-byte modes: bf16 1.0 (0x3f80) / fp16 1.0 (0x3c00), n elements
            const uint16_t one = mode.find("bf16") != std::string::npos ? 0x3f80 : 0x3c00;
            std::vector<uint16_t> a2(lp ? n : 0, one), b2(lp ? n : 0, one);
            if (mode == "reg") {
                mi_ccl_comp_register_host_buffer(a.data(), n * sizeof(float));
                mi_ccl_comp_register_host_buffer(b.data(), n * sizeof(float));
            }
            if (mode.compare(0, 5, "sched") == 0) mi_ccl_comp_shim_sched(1);
            const void* fins[2] = {b2.data(), a2.data()};
            const void* f32ins[2] = {b.data(), a.data()};
            const size_t nb = n * sizeof(float);
            // the mode is resolved to an id once: a chain of string compares
            // inside the timed loop cost tens of ns per call (round 5)
            auto call = [&] {
                switch (mid) {
                    case M_REF: ref(a.data(), n, b.data(), nullptr, 9, sizeof(float), 0); break;
                    case M_REFBF16: ref_lp(2, 0, a2.data(), b2.data(), n); break;
                    case M_REFFP16: ref_lp(3, 0, a2.data(), b2.data(), n); break;
                    case M_MPIBF16: mi_ccl_bf16_reduce_host(a2.data(), n, b2.data(), nullptr, 0); break;
                    case M_MPIFP16: mi_ccl_fp16_reduce_host(a2.data(), n, b2.data(), nullptr, 0); break;
                    case M_BF16: mi_ccl_bf16_reduce(a2.data(), n, b2.data(), nullptr, 0); break;
                    case M_FP16: mi_ccl_fp16_reduce(a2.data(), n, b2.data(), nullptr, 0); break;
                    case M_FOLDBF16:
                        mi_host_reduce(fins, 2, b2.data(), n, MI_BFLOAT16, 0, MI_F_MINMAX_INOUT_FIRST | MI_F_BF16_RNE);
                        break;
                    case M_FOLDFP16: mi_host_reduce(fins, 2, b2.data(), n, MI_FLOAT16, 0, MI_F_MINMAX_INOUT_FIRST); break;
                    case M_FOLDI16: mi_host_reduce(fins, 2, b2.data(), n, MI_INT16, 0, 0); break;
                    case M_FOLDF32: mi_host_reduce(f32ins, 2, b.data(), n, MI_FLOAT32, 0, 0); break;
                    case M_SCHEDBF16: mi_ccl_comp_reduce(a2.data(), n, b2.data(), nullptr, 11, 0); break;
                    case M_SCHEDFP16: mi_ccl_comp_reduce(a2.data(), n, b2.data(), nullptr, 8, 0); break;
                    case M_SCHEDI16: mi_ccl_comp_reduce(a2.data(), n, b2.data(), nullptr, 2, 0); break;
                    // diagnostic pairs: does the bf16 fold slow the entry point around it?
                    case M_SCHEDI16_FOLDBF16:
                        mi_ccl_comp_reduce(a2.data(), n, b2.data(), nullptr, 2, 0);
                        mi_host_reduce(fins, 2, b2.data(), n, MI_BFLOAT16, 0, MI_F_MINMAX_INOUT_FIRST | MI_F_BF16_RNE);
                        break;
                    case M_FOLDI16_FOLDBF16:
                        mi_host_reduce(fins, 2, b2.data(), n, MI_INT16, 0, 0);
                        mi_host_reduce(fins, 2, b2.data(), n, MI_BFLOAT16, 0, MI_F_MINMAX_INOUT_FIRST | MI_F_BF16_RNE);
                        break;
                    case M_SCHEDI16X2:
                        mi_ccl_comp_reduce(a2.data(), n, b2.data(), nullptr, 2, 0);
                        mi_ccl_comp_reduce(a2.data(), n, b2.data(), nullptr, 2, 0);
                        break;
                    case M_COPY: mi_ccl_comp_copy(a.data(), b.data(), nb, 0); break;
                    case M_COPYHOST: mi_ccl_comp_copy_host(a.data(), b.data(), nb, 0); break;
                    case M_MEMCPY: memcpy(b.data(), a.data(), nb); break;
                    default: mi_ccl_comp_reduce(a.data(), n, b.data(), nullptr, 9, 0);  // default, reg, sched
                }
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
    printf("{\"mode\": \"%s%s\", \"pinned\": %s, \"threads\": %d, \"elements\": %zu, \"bytes\": %zu, \"median_us\": %.3f, "
           "\"max_us\": %.3f, \"lookups_per_call\": %.2f, \"iters\": %ld}\n",
           mode.c_str(), roctx_on ? " (roctx on)" : "", pin.empty() ? "false" : "true", T, n, n * es, s[T / 2], s[T - 1], lk, iters);
    fflush(stdout);
}
