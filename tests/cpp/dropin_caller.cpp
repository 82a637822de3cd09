// dropin_caller.cpp — a C++ caller of the drop-in src/comp, written the way
// oneCCL's schedule entries call it (src/sched/entry/recv_reduce_entry.hpp:
// 113-132, reduce_local_entry.cpp:98-114): oneCCL types, the C++ entry
// points resolved by their mangled names from libccl_comp_hip.so, buffers
// from a host staging allocation (posix_memalign, like
// sched->alloc_buffer -> src/common/utils/utils.hpp:109-117) and from
// hipMalloc.  Checks results against closed forms.  Exit 0 = all pass.
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../oneccl_amd/csrc/ccl_mirror.hpp"
#include "../../include/mi_ccl_comp_async.hpp"
#include "../../include/mi_ccl_lp_host.hpp"

// reduce_local_entry as INTEGRATION.md §2(d) patches it: start() issues the
// reduce and returns `started`; the worker's progress loop calls update()
// until the entry is complete (src/sched/entry/reduce_local_entry.cpp:116-131,
// src/exec/thread/worker.cpp:310-379).
// The entry's schedule goes along, as the patched entries pass it: a
// collective without a stream works on host memory (nothing is looked up),
// one with a stream may hand device memory (src/comp/comp.cpp:136-142).
enum entry_status { not_started, started, complete };
static ccl_sched g_host_sched;    // coll_param.stream == nullptr
static ccl_sched g_stream_sched;  // coll_param.stream set (never dereferenced)
struct async_reduce_entry {
    ccl_sched* sched;
    const void* in;
    void* inout;
    size_t cnt;
    ccl_datatype dtype;
    ccl::reduction op;
    entry_status status = not_started;
    ccl_comp_request* req = nullptr;
    void start() {
        ccl_comp_reduce_start(sched, in, cnt, inout, nullptr, dtype, op, nullptr, nullptr, &req);
        status = started;
        update();
    }
    void update() {
        if (status == started && ccl_comp_request_test(req)) {
            ccl_comp_request_free(req);
            req = nullptr;
            status = complete;
        }
    }
};

// MPI user ops (MPI_User_function shape) as src/atl/mpi/atl_mpi_ctx.cpp
// registers them, with integration/0002 applied: bf16_base_op (:87-92) and
// fp16_base_op (:57-63) call ccl_{bf16,fp16}_reduce_host, whose operands are
// host memory by the caller's word (include/mi_ccl_lp_host.hpp).  MPI calls
// them from its own progress thread on host buffers.
typedef void (*mpi_user_fn)(void* in, void* inout, int* length, void* datatype);
static void bf16_sum_op(void* in, void* inout, int* length, void*) {
    ccl_bf16_reduce_host(in, *length, inout, nullptr, ccl::reduction::sum);
}
static void fp16_max_op(void* in, void* inout, int* length, void*) {
    size_t len = *length;
    ccl_fp16_reduce_host(in, len, inout, nullptr, ccl::reduction::max);
}

static int failures = 0;
#define EXPECT(cond, ...)                         \
    do {                                          \
        if (!(cond)) {                            \
            fprintf(stderr, "FAIL %s:%d ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);         \
            fprintf(stderr, "\n");                \
            failures++;                           \
        }                                         \
    } while (0)

static void* staging_alloc(size_t bytes) {
    void* p = nullptr;
    if (posix_memalign(&p, 4096, bytes)) return nullptr;
    return p;
}

int main() {
    const size_t n = 131072;  // C1: per-rank nreduce chunk of a 2-rank 1 MiB allreduce
    const ccl_datatype f32(ccl::datatype::float32, sizeof(float));
    const ccl::fn_context ctx = {"match", 0};

    // host staging buffers (recv_reduce_entry's comm_buf and the accumulator)
    float* comm_buf = static_cast<float*>(staging_alloc(n * sizeof(float)));
    float* acc = static_cast<float*>(staging_alloc(n * sizeof(float)));
    for (size_t i = 0; i < n; i++) {
        comm_buf[i] = 1.0f;  // peer rank 1's chunk
        acc[i] = 0.0f;       // own rank 0's chunk
    }
    ccl::status st = ccl_comp_reduce(nullptr, comm_buf, n, acc, nullptr, f32, ccl::reduction::sum, nullptr, &ctx);
    EXPECT(st == ccl::status::success, "status %d", (int)st);
    bool ok = true;
    for (size_t i = 0; i < n; i++) ok = ok && acc[i] == 1.0f;  // (P-1)*P/2 with P = 2
    EXPECT(ok, "host fp32 sum");
    // the same entry under its schedule (no stream: host memory by its word)
    g_stream_sched.coll_param.stream = reinterpret_cast<ccl_stream*>(&g_stream_sched);
    st = ccl_comp_reduce(&g_host_sched, comm_buf, n, acc, nullptr, f32, ccl::reduction::sum, nullptr, &ctx);
    EXPECT(st == ccl::status::success, "status %d", (int)st);
    ok = true;
    for (size_t i = 0; i < n; i++) ok = ok && acc[i] == 2.0f;
    EXPECT(ok, "host fp32 sum under a schedule without a stream");

    // device buffers: reduce_local_entry with device USM (reduce_local_entry.cpp:33-58)
    float *din = nullptr, *dio = nullptr;
    if (hipMalloc(&din, n * sizeof(float)) != hipSuccess || hipMalloc(&dio, n * sizeof(float)) != hipSuccess) {
        fprintf(stderr, "hipMalloc failed\n");
        return 2;
    }
    std::vector<float> h(n);
    for (size_t i = 0; i < n; i++) h[i] = (float)(i % 1000);
    (void)hipMemcpy(din, h.data(), n * sizeof(float), hipMemcpyHostToDevice);
    for (size_t i = 0; i < n; i++) h[i] = (float)(i % 7);
    (void)hipMemcpy(dio, h.data(), n * sizeof(float), hipMemcpyHostToDevice);
    st = ccl_comp_reduce(nullptr, din, n, dio, nullptr, f32, ccl::reduction::max, nullptr, nullptr);
    EXPECT(st == ccl::status::success, "status %d", (int)st);
    (void)hipMemcpy(h.data(), dio, n * sizeof(float), hipMemcpyDeviceToHost);
    ok = true;
    for (size_t i = 0; i < n; i++) ok = ok && h[i] == std::fmax((float)(i % 1000), (float)(i % 7));
    EXPECT(ok, "device fp32 max");

    // bf16 with out_count (bf16.cpp:94-96) and in_count == 0 (comp.cpp:132-134)
    std::vector<uint16_t> a(64, 0x3F80), b(64, 0x4000);  // 1.0 + 2.0
    size_t out_count = 0;
    ccl_comp_reduce(nullptr, a.data(), 64, b.data(), &out_count, ccl_datatype(ccl::datatype::bfloat16, 2),
                    ccl::reduction::sum, nullptr, nullptr);
    EXPECT(out_count == 64, "out_count %zu", out_count);
    EXPECT(b[0] == 0x4040 && b[63] == 0x4040, "bf16 1+2 = %04x", b[0]);
    EXPECT(ccl_comp_reduce(nullptr, a.data(), 0, b.data(), nullptr, f32, ccl::reduction::sum, nullptr, nullptr) ==
               ccl::status::success,
           "zero count");

    // batch reduce: 4 int32 inputs, offsets in elements (comp.cpp:236-245)
    std::vector<int32_t> packed(4 * 100);
    for (int j = 0; j < 4; j++)
        for (int i = 0; i < 100; i++) packed[j * 100 + i] = j + 1;
    std::vector<int32_t> io(packed.begin(), packed.begin() + 100);
    std::vector<size_t> offsets = {0, 100, 200, 300};
    ccl_comp_batch_reduce(packed.data(), offsets, 100, io.data(), nullptr, ccl_datatype(ccl::datatype::int32, 4),
                          ccl::reduction::prod, nullptr, nullptr, 0, nullptr, nullptr);
    EXPECT(io[0] == 24 && io[99] == 24, "batch prod %d", io[0]);

    // copy, to_str, custom op and its error
    std::vector<char> src(1000, 'x'), dst(1000, 0);
    ccl_comp_copy(src.data(), dst.data(), 1000, true);
    EXPECT(memcmp(src.data(), dst.data(), 1000) == 0, "copy");
    EXPECT(strcmp(ccl_reduction_to_str(ccl::reduction::prod), "prod") == 0, "to_str");
    bool threw = false;
    try {
        ccl_comp_reduce(nullptr, a.data(), 64, b.data(), nullptr, f32, ccl::reduction::custom, nullptr, nullptr);
    } catch (const ccl::exception&) {
        threw = true;
    }
    EXPECT(threw, "custom without fn must throw (comp.cpp:85)");

    // large pageable host buffers: more than one 32 MiB staging chunk, odd count
    {
        const size_t m = (80u << 20) / 4 + 5;
        float* x = static_cast<float*>(staging_alloc(m * 4));
        float* y = static_cast<float*>(staging_alloc(m * 4));
        for (size_t i = 0; i < m; i++) {
            x[i] = (float)(i % 97);
            y[i] = 1.0f;
        }
        ccl_comp_reduce(nullptr, x, m, y, nullptr, f32, ccl::reduction::sum, nullptr, nullptr);
        bool okk = true;
        for (size_t i = 0; i < m; i++) okk = okk && y[i] == (float)(i % 97) + 1.0f;
        EXPECT(okk, "pageable multi-chunk");
        // misaligned sub-buffers (ring chunks at odd element offsets)
        ccl_comp_reduce(nullptr, x + 1, m - 3, y + 3, nullptr, f32, ccl::reduction::max, nullptr, nullptr);
        // pinned host buffers: zero-copy kernel path
        float *px = nullptr, *py = nullptr;
        if (hipHostMalloc(&px, m * 4, 0) == hipSuccess && hipHostMalloc(&py, m * 4, 0) == hipSuccess) {
            memcpy(px, x, m * 4);
            for (size_t i = 0; i < m; i++) py[i] = 2.0f;
            ccl_comp_reduce(nullptr, px, m, py, nullptr, f32, ccl::reduction::prod, nullptr, nullptr);
            okk = true;
            for (size_t i = 0; i < m; i++) okk = okk && py[i] == 2.0f * x[i];
            EXPECT(okk, "pinned zero-copy");
            (void)hipHostFree(px);
            (void)hipHostFree(py);
        }
        free(x);
        free(y);
    }

    // batch reduce with more inputs than one fused launch takes (chained groups)
    {
        const size_t k = 23, m = 1001;
        std::vector<float> pk(k * m);
        for (size_t j = 0; j < k; j++)
            for (size_t i = 0; i < m; i++) pk[j * m + i] = 1.0f;
        std::vector<float> out(pk.begin(), pk.begin() + m);
        std::vector<size_t> offs(k);
        for (size_t j = 0; j < k; j++) offs[j] = j * m;
        ccl_comp_batch_reduce(pk.data(), offs, m, out.data(), nullptr, f32, ccl::reduction::sum, nullptr, nullptr, 0,
                              nullptr, nullptr);
        EXPECT(out[0] == 23.0f && out[m - 1] == 23.0f, "batch k=23: %f", out[0]);
        // bf16 keep-precision (fp32 accumulate, one rounding)
        std::vector<uint16_t> bk(4 * 33, 0x3F80);  // 1.0
        std::vector<uint16_t> bo(bk.begin(), bk.begin() + 33);
        std::vector<size_t> o4 = {0, 33, 66, 99};
        ccl_comp_batch_reduce(bk.data(), o4, 33, bo.data(), nullptr, ccl_datatype(ccl::datatype::bfloat16, 2),
                              ccl::reduction::sum, nullptr, nullptr, 1, nullptr, nullptr);
        EXPECT(bo[0] == 0x4080 && bo[32] == 0x4080, "keep precision 4.0 = %04x", bo[0]);
    }

    // conversions with a count%16 tail
    {
        std::vector<float> f(37);
        for (size_t i = 0; i < f.size(); i++) f[i] = 1.0f + (float)i / 3.0f;
        std::vector<uint16_t> h(37);
        ccl_convert_fp32_to_bf16_arrays(f.data(), h.data(), h.size());
        std::vector<float> back(37);
        ccl_convert_bf16_to_fp32_arrays(h.data(), back.data(), back.size());
        bool okk = true;
        for (size_t i = 0; i < f.size(); i++) okk = okk && std::fabs(back[i] - f[i]) <= f[i] / 64;
        EXPECT(okk, "bf16 arrays round trip");
    }

    // asynchronous entries: 4 device + 2 host-staging reduces in flight, one
    // progress loop polling them (bounded: a lost completion fails the test)
    {
        const size_t m = 1u << 20;
        const int nd = 4, nh = 2;
        std::vector<float*> dbufs;
        std::vector<float> hv(m);
        for (int e = 0; e < 2 * nd; e++) {
            float* p = nullptr;
            if (hipMalloc(&p, m * 4) != hipSuccess) {
                fprintf(stderr, "hipMalloc failed\n");
                return 2;
            }
            for (size_t i = 0; i < m; i++) hv[i] = (float)((i + (size_t)e) % 251);
            (void)hipMemcpy(p, hv.data(), m * 4, hipMemcpyHostToDevice);
            dbufs.push_back(p);
        }
        std::vector<float*> hbufs;
        for (int e = 0; e < 2 * nh; e++) {
            float* p = static_cast<float*>(staging_alloc(m * 4));
            for (size_t i = 0; i < m; i++) p[i] = (float)((i + (size_t)e) % 251);
            hbufs.push_back(p);
        }
        std::vector<async_reduce_entry> entries;
        for (int e = 0; e < nd; e++)
            entries.push_back({&g_stream_sched, dbufs[2 * e], dbufs[2 * e + 1], m, f32, ccl::reduction::sum});
        for (int e = 0; e < nh; e++)
            entries.push_back({&g_host_sched, hbufs[2 * e], hbufs[2 * e + 1], m, f32, ccl::reduction::max});
        for (auto& en : entries) en.start();
        size_t spins = 0;
        bool all = false;
        while (!all && spins < 200000000) {
            all = true;
            for (auto& en : entries) {
                en.update();
                all = all && en.status == complete;
            }
            spins++;
        }
        EXPECT(all, "async entries did not complete");
        bool okk = true;
        for (int e = 0; e < nd; e++) {
            (void)hipMemcpy(hv.data(), dbufs[2 * e + 1], m * 4, hipMemcpyDeviceToHost);
            for (size_t i = 0; i < m; i++)
                okk = okk && hv[i] == (float)((i + 2 * e) % 251) + (float)((i + 2 * e + 1) % 251);
        }
        EXPECT(okk, "async device sum");
        okk = true;
        for (int e = 0; e < nh; e++)
            for (size_t i = 0; i < m; i++)
                okk = okk && hbufs[2 * e + 1][i] == std::fmax((float)((i + 2 * e) % 251), (float)((i + 2 * e + 1) % 251));
        EXPECT(okk, "async host max");
        // a host bucket above the dispatcher's threshold (16 MiB): split, the
        // head folded on the worker's helper thread while the GPU takes the tail
        {
            const size_t big = (40u << 20) / 4 + 7;
            float* bx = static_cast<float*>(staging_alloc(big * 4));
            float* by = static_cast<float*>(staging_alloc(big * 4));
            for (size_t i = 0; i < big; i++) {
                bx[i] = (float)(i % 89);
                by[i] = 3.0f;
            }
            async_reduce_entry bigen{&g_host_sched, bx, by, big, f32, ccl::reduction::sum};
            bigen.start();
            size_t sp = 0;
            while (bigen.status != complete && sp++ < 200000000) bigen.update();
            bool okb = bigen.status == complete;
            for (size_t i = 0; i < big && okb; i++) okb = by[i] == (float)(i % 89) + 3.0f;
            EXPECT(okb, "async split of a large host bucket");
            free(bx);
            free(by);
        }
        // empty reduce: complete at start (comp.cpp:132-134)
        async_reduce_entry z{&g_host_sched, hbufs[0], hbufs[1], 0, f32, ccl::reduction::sum};
        z.start();
        EXPECT(z.status == complete, "empty async reduce completes at start");
        for (float* p : dbufs) (void)hipFree(p);
        for (float* p : hbufs) free(p);
    }

    // MPI user ops, called through function pointers as MPI_Reduce_local /
    // the MPI progress engine would (host buffers, odd length)
    {
        const mpi_user_fn ops[2] = {&bf16_sum_op, &fp16_max_op};
        int len = 1001;
        std::vector<uint16_t> in(len, 0x3F80), io(len, 0x4000);  // bf16 1.0 + 2.0
        ops[0](in.data(), io.data(), &len, nullptr);
        EXPECT(io[0] == 0x4040 && io[len - 1] == 0x4040, "MPI bf16 sum op %04x", io[0]);
        std::vector<uint16_t> hin(len, 0x4000), hio(len, 0x3C00);  // fp16 max(2.0, 1.0)
        hin[7] = 0x7E00;  // NaN in `in`: MAXPS(in, inout) returns inout (fp16_intrisics.hpp:72-77)
        ops[1](hin.data(), hio.data(), &len, nullptr);
        EXPECT(hio[0] == 0x4000 && hio[len - 1] == 0x4000 && hio[7] == 0x3C00, "MPI fp16 max op %04x %04x", hio[0],
               hio[7]);
    }

    free(comm_buf);
    free(acc);
    (void)hipFree(din);
    (void)hipFree(dio);
    printf("dropin_caller: %s (%d failures)\n", failures ? "FAIL" : "ok", failures);
    return failures ? 1 : 0;
}
