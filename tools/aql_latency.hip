// aql_latency.hip — feasibility probe: round-trip latency of a synchronous
// small reduce through the HIP runtime vs a raw AQL packet written into our
// own HSA queue (completion signal waited on by spinning).
//
//   tools/aql_latency [iters] [code_object]
// Prints one JSON line per item (min / median / p90 microseconds).
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "../oneccl_amd/csrc/reduce_kernels.hpp"

#define HC(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(2);                                                                   \
        }                                                                              \
    } while (0)
#define SC(x)                                                                          \
    do {                                                                               \
        hsa_status_t s_ = (x);                                                         \
        if (s_ != HSA_STATUS_SUCCESS) {                                                \
            const char* m_ = nullptr;                                                  \
            hsa_status_string(s_, &m_);                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, m_ ? m_ : "?"); \
            exit(3);                                                                   \
        }                                                                              \
    } while (0)

extern "C" __global__ void hip_empty_kernel() {}

using clk = std::chrono::steady_clock;

static void report(const char* item, std::vector<double>& us) {
    std::sort(us.begin(), us.end());
    printf("{\"item\": \"%s\", \"min_us\": %.2f, \"median_us\": %.2f, \"p90_us\": %.2f}\n", item, us[0],
           us[us.size() / 2], us[us.size() * 9 / 10]);
    fflush(stdout);
}

struct Agents {
    hsa_agent_t gpu{0}, cpu{0};
};

static hsa_status_t agent_cb(hsa_agent_t a, void* data) {
    auto* ag = static_cast<Agents*>(data);
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    if (t == HSA_DEVICE_TYPE_GPU && ag->gpu.handle == 0) ag->gpu = a;
    if (t == HSA_DEVICE_TYPE_CPU && ag->cpu.handle == 0) ag->cpu = a;
    return HSA_STATUS_SUCCESS;
}

static hsa_status_t pool_cb(hsa_amd_memory_pool_t p, void* data) {
    hsa_amd_segment_t seg;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
    if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
    uint32_t flags = 0;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
    if (flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT) {
        *static_cast<hsa_amd_memory_pool_t*>(data) = p;
        return HSA_STATUS_INFO_BREAK;
    }
    return HSA_STATUS_SUCCESS;
}

struct Kern {
    uint64_t object = 0;
    uint32_t kernarg = 0, group = 0, priv = 0;
};

static Kern get_kernel(hsa_executable_t exe, hsa_agent_t gpu, const char* name) {
    hsa_executable_symbol_t sym;
    SC(hsa_executable_get_symbol_by_name(exe, name, &gpu, &sym));
    Kern k;
    SC(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &k.object));
    SC(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &k.kernarg));
    SC(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &k.group));
    SC(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &k.priv));
    fprintf(stderr, "kernel %s: kernarg %u group %u private %u\n", name, k.kernarg, k.group, k.priv);
    return k;
}

struct Dispatcher {
    hsa_queue_t* q = nullptr;
    hsa_signal_t sig{0};
    void* kernarg = nullptr;

    // one dispatch, wait for completion; returns false on timeout
    int acq = HSA_FENCE_SCOPE_SYSTEM, rel = HSA_FENCE_SCOPE_SYSTEM;
    bool run(const Kern& k, const void* args, size_t args_bytes, uint32_t grid_blocks, uint32_t block,
             hsa_wait_state_t ws) {
        memset(kernarg, 0, 1024);
        memcpy(kernarg, args, args_bytes);
        hsa_signal_store_relaxed(sig, 1);
        const uint64_t idx = hsa_queue_add_write_index_screlease(q, 1);
        while (idx - hsa_queue_load_read_index_scacquire(q) >= q->size) {
        }
        auto* pkt = static_cast<hsa_kernel_dispatch_packet_t*>(q->base_address) + (idx & (q->size - 1));
        pkt->workgroup_size_x = (uint16_t)block;
        pkt->workgroup_size_y = 1;
        pkt->workgroup_size_z = 1;
        pkt->reserved0 = 0;
        pkt->grid_size_x = grid_blocks * block;
        pkt->grid_size_y = 1;
        pkt->grid_size_z = 1;
        pkt->private_segment_size = k.priv;
        pkt->group_segment_size = k.group;
        pkt->kernel_object = k.object;
        pkt->kernarg_address = kernarg;
        pkt->reserved2 = 0;
        pkt->completion_signal = sig;
        const uint16_t header = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                                (1 << HSA_PACKET_HEADER_BARRIER) |
                                (acq << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                                (rel << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
        const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
        __atomic_store_n(reinterpret_cast<uint32_t*>(pkt), (uint32_t)header | ((uint32_t)setup << 16),
                         __ATOMIC_RELEASE);
        hsa_signal_store_screlease(q->doorbell_signal, (hsa_signal_value_t)idx);
        const hsa_signal_value_t v =
            hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, 2000000000ull, ws);  // ~1 s of ticks
        return v < 1;
    }
};

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 2000;
    std::string co = argc > 2 ? argv[2] : "tools/aql_kernels.hsaco";

    // HIP first: the runtime initialises HSA; ours is a nested hsa_init
    HC(hipSetDevice(0));
    hipStream_t s;
    HC(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const size_t n = 1024;  // 4 KiB fp32
    float *da, *db;
    HC(hipMalloc(&da, n * 4));
    HC(hipMalloc(&db, n * 4));
    std::vector<float> ha(n), hb(n), hr(n);
    for (size_t i = 0; i < n; i++) {
        ha[i] = (float)i * 0.5f;
        hb[i] = 1.0f + (float)i;
    }

    {
        std::vector<double> us;
        for (int i = 0; i < iters + 50; i++) {
            auto t0 = clk::now();
            hipLaunchKernelGGL(hip_empty_kernel, dim3(1), dim3(64), 0, s);
            HC(hipStreamSynchronize(s));
            if (i >= 50) us.push_back(std::chrono::duration<double, std::micro>(clk::now() - t0).count());
        }
        report("hip: empty kernel launch + hipStreamSynchronize", us);
    }
    mi::R2Args ra{};
    ra.acc = db;
    ra.in = da;
    ra.out = db;
    ra.nvec = n / 4;
    {
        std::vector<double> us;
        for (int i = 0; i < iters + 50; i++) {
            auto t0 = clk::now();
            hipLaunchKernelGGL((mi::reduce2_kernel<float, 0, 0u, 1, 1024>), dim3(1), dim3(1024), 0, s, ra);
            HC(hipStreamSynchronize(s));
            if (i >= 50) us.push_back(std::chrono::duration<double, std::micro>(clk::now() - t0).count());
        }
        report("hip: reduce2 4 KiB fp32 launch + hipStreamSynchronize", us);
    }

    SC(hsa_init());
    Agents ag;
    SC(hsa_iterate_agents(agent_cb, &ag));
    if (!ag.gpu.handle || !ag.cpu.handle) {
        fprintf(stderr, "no agents\n");
        return 4;
    }
    char name[64] = {0};
    hsa_agent_get_info(ag.gpu, HSA_AGENT_INFO_NAME, name);
    fprintf(stderr, "gpu agent %s\n", name);

    std::ifstream f(co, std::ios::binary);
    if (!f) {
        fprintf(stderr, "cannot open %s\n", co.c_str());
        return 5;
    }
    std::string blob((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    hsa_code_object_reader_t rd;
    SC(hsa_code_object_reader_create_from_memory(blob.data(), blob.size(), &rd));
    hsa_executable_t exe;
    SC(hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &exe));
    SC(hsa_executable_load_agent_code_object(exe, ag.gpu, rd, nullptr, nullptr));
    SC(hsa_executable_freeze(exe, nullptr));
    Kern ke = get_kernel(exe, ag.gpu, "aql_empty_kernel.kd");
    Kern kr = get_kernel(exe, ag.gpu, "_ZN2mi14reduce2_kernelIfLi0ELj0ELi1ELi1024EEEvNS_6R2ArgsE.kd");
    if (kr.kernarg < sizeof(mi::R2Args) || kr.kernarg > 1024 || kr.group != 0 || kr.priv != 0) {
        fprintf(stderr, "unexpected reduce2 segment sizes\n");
        return 6;
    }

    hsa_amd_memory_pool_t kpool{0};
    hsa_amd_agent_iterate_memory_pools(ag.cpu, pool_cb, &kpool);
    if (!kpool.handle) {
        fprintf(stderr, "no kernarg pool\n");
        return 7;
    }
    Dispatcher d;
    SC(hsa_amd_memory_pool_allocate(kpool, 4096, 0, &d.kernarg));
    SC(hsa_amd_agents_allow_access(1, &ag.gpu, nullptr, d.kernarg));
    SC(hsa_queue_create(ag.gpu, 64, HSA_QUEUE_TYPE_MULTI, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &d.q));
    SC(hsa_signal_create(1, 0, nullptr, &d.sig));

    for (int pass = 0; pass < 2; pass++) {
        const hsa_wait_state_t ws = pass == 0 ? HSA_WAIT_STATE_ACTIVE : HSA_WAIT_STATE_BLOCKED;
        std::vector<double> us;
        for (int i = 0; i < iters + 50; i++) {
            auto t0 = clk::now();
            if (!d.run(ke, nullptr, 0, 1, 64, ws)) {
                fprintf(stderr, "empty dispatch timed out\n");
                return 8;
            }
            if (i >= 50) us.push_back(std::chrono::duration<double, std::micro>(clk::now() - t0).count());
        }
        report(pass == 0 ? "aql: empty kernel, spin wait" : "aql: empty kernel, blocked wait", us);
    }

    {
        const int sc[][2] = {{HSA_FENCE_SCOPE_AGENT, HSA_FENCE_SCOPE_AGENT}, {HSA_FENCE_SCOPE_NONE, HSA_FENCE_SCOPE_AGENT},
                             {HSA_FENCE_SCOPE_AGENT, HSA_FENCE_SCOPE_SYSTEM}, {HSA_FENCE_SCOPE_NONE, HSA_FENCE_SCOPE_NONE}};
        const char* nm[] = {"aql: empty kernel, spin, acquire agent / release agent",
                            "aql: empty kernel, spin, acquire none / release agent",
                            "aql: empty kernel, spin, acquire agent / release system",
                            "aql: empty kernel, spin, acquire none / release none"};
        for (int v = 0; v < 4; v++) {
            d.acq = sc[v][0];
            d.rel = sc[v][1];
            std::vector<double> us;
            for (int i = 0; i < iters + 50; i++) {
                auto t0 = clk::now();
                if (!d.run(ke, nullptr, 0, 1, 64, HSA_WAIT_STATE_ACTIVE)) {
                    fprintf(stderr, "empty dispatch timed out\n");
                    return 8;
                }
                if (i >= 50) us.push_back(std::chrono::duration<double, std::micro>(clk::now() - t0).count());
            }
            report(nm[v], us);
        }
        // a signal with no interrupt: polled only
        hsa_signal_t ps;
        SC(hsa_amd_signal_create(1, 0, nullptr, HSA_AMD_SIGNAL_AMD_GPU_ONLY, &ps));
        (void)ps;
        SC(hsa_signal_destroy(ps));
        d.acq = d.rel = HSA_FENCE_SCOPE_SYSTEM;
    }
    // correctness once, then latency
    HC(hipMemcpy(da, ha.data(), n * 4, hipMemcpyHostToDevice));
    HC(hipMemcpy(db, hb.data(), n * 4, hipMemcpyHostToDevice));
    if (!d.run(kr, &ra, sizeof(ra), 1, 1024, HSA_WAIT_STATE_ACTIVE)) {
        fprintf(stderr, "reduce dispatch timed out\n");
        return 9;
    }
    HC(hipMemcpy(hr.data(), db, n * 4, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < n; i++)
        if (hr[i] != ha[i] + hb[i]) {
            fprintf(stderr, "mismatch at %zu: %f vs %f\n", i, hr[i], ha[i] + hb[i]);
            return 10;
        }
    printf("{\"item\": \"aql reduce2 result check\", \"ok\": true}\n");
    {
        std::vector<double> us;
        for (int i = 0; i < iters + 50; i++) {
            auto t0 = clk::now();
            if (!d.run(kr, &ra, sizeof(ra), 1, 1024, HSA_WAIT_STATE_ACTIVE)) {
                fprintf(stderr, "reduce dispatch timed out\n");
                return 11;
            }
            if (i >= 50) us.push_back(std::chrono::duration<double, std::micro>(clk::now() - t0).count());
        }
        report("aql: reduce2 4 KiB fp32, spin wait", us);
    }
    // the HIP path again after ours, to see that nothing shifted
    {
        std::vector<double> us;
        for (int i = 0; i < iters + 50; i++) {
            auto t0 = clk::now();
            hipLaunchKernelGGL((mi::reduce2_kernel<float, 0, 0u, 1, 1024>), dim3(1), dim3(1024), 0, s, ra);
            HC(hipStreamSynchronize(s));
            if (i >= 50) us.push_back(std::chrono::duration<double, std::micro>(clk::now() - t0).count());
        }
        report("hip: reduce2 4 KiB fp32 launch + hipStreamSynchronize (after)", us);
    }
    SC(hsa_signal_destroy(d.sig));
    SC(hsa_queue_destroy(d.q));
    SC(hsa_amd_memory_pool_free(d.kernarg));
    SC(hsa_executable_destroy(exe));
    SC(hsa_code_object_reader_destroy(rd));
    SC(hsa_shut_down());
    HC(hipFree(da));
    HC(hipFree(db));
    HC(hipStreamDestroy(s));
    return 0;
}
