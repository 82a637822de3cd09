// comp.cpp — drop-in replacement for oneCCL's src/comp/*.cpp, backed by the
// MI355X HIP kernels of libmi_reduce.so (include/mi_reduce.h).
//
// Keeps the reference's signatures and semantics:
//   ccl_comp_copy           src/comp/comp.cpp:60-74
//   ccl_comp_reduce         src/comp/comp.cpp:123-200  (+ _regular :76-121)
//   ccl_comp_batch_reduce   src/comp/comp.cpp:202-249
//   ccl_reduction_to_str    src/comp/comp.cpp:251-260
//   ccl_bf16_reduce         src/comp/bf16/bf16.cpp:87-110
//   ccl_fp16_reduce         src/comp/fp16/fp16.cpp:41-53
//   ccl_{bf16,fp16}_reduce_host  the MPI user ops' call, atl_mpi_ctx.cpp:57-63,87-92
//   bf16_impl_names / fp16_impl_names / fp16_env_impl_names (bf16.cpp:26-30, fp16.cpp:25-39)
// Which bit-level behaviour the reference would show (bf16 truncation vs
// RNE, min/max operand order) is taken from the same place the reference
// takes it: the bf16/fp16 impl type chosen from CPUID and CCL_BF16/CCL_FP16
// (src/common/env/env.cpp:711-720).
//
// Build modes:
//   -DMI_ONECCL_TREE : compiled inside oneCCL's src/ (see INTEGRATION.md),
//                      uses the real headers, ccl::global_data::env() and
//                      CCL_THROW.
//   default          : standalone libccl_comp_hip.so for this repo's tests and
//                      bench (ccl_mirror.hpp; same mangled symbols).
#include <dlfcn.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <memory>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/mi_host_reduce.h"
#include "../../include/mi_reduce.h"

static int mi_local_gpu(int local_idx, int ndev);  // below, after the environment

#ifdef MI_ONECCL_TREE
#include "common/global/global.hpp"
#include "common/log/log.hpp"
#include "comp/bf16/bf16.hpp"
#include "comp/comp.hpp"
#include "comp/fp16/fp16.hpp"
#include "sched/sched.hpp"  // sched->coll_param.stream, as the reference's comp.cpp reads it
#define MI_CCL_THROW(msg) CCL_THROW(msg)
#define MI_CCL_FATAL(msg) CCL_FATAL(msg)
// the dispatcher's decisions go to oneCCL's own log (CCL_LOG_LEVEL=debug),
// as the reference logs its path (bf16.cpp:92, fp16.cpp:46, comp.cpp:149)
#define MI_LOG_DEBUG(...) LOG_DEBUG(__VA_ARGS__)
#include "mi_ccl_comp.h"  // include/ (on the include path)
#include "mi_ccl_comp_async.hpp"
#include "mi_ccl_lp_host.hpp"
static ccl_bf16_impl_type mi_bf16_impl() { return ccl::global_data::env().bf16_impl_type; }
static ccl_fp16_impl_type mi_fp16_impl() { return ccl::global_data::env().fp16_impl_type; }
// CCL_COMP_HIP_DEVICE: the GPU for operands that name none (host buffers).
// Unset: the process's index among the node's processes (global_data, set
// from the launcher at init, global.cpp:96-101,182-220) modulo the GPUs it
// sees (mi_local_gpu).  Read once, like the rest of oneCCL's environment.
static int mi_comp_device() {
    static const int dev = [] {
        if (const char* v = getenv("CCL_COMP_HIP_DEVICE")) return atoi(v);
        return mi_local_gpu(ccl::global_data::get().get_local_proc_idx(), mi_device_count());
    }();
    return dev;
}
struct HostMax;
static HostMax mi_host_max();
#else
#include <sstream>

#include "../../include/mi_ccl_comp.h"
#include "ccl_mirror.hpp"
#define MI_CCL_THROW(msg) throw ccl::exception(msg)
// oneCCL's LOG_DEBUG (src/common/log/log.hpp:302-314) for the standalone
// build: CCL_LOG_LEVEL=debug (or trace) prints the dispatcher's decisions to
// stderr in oneCCL's format; the arguments are only evaluated when it is on.
static bool mi_log_debug_on();
template <typename... A>
static void mi_log_debug(int line, const char* fn, const A&... a) {
    std::ostringstream os;
    os << "|CCL_DEBUG| comp.cpp:" << line << " " << fn << ": ";
    using expand = int[];
    (void)expand{0, ((void)(os << a), 0)...};
    os << "\n";
    fputs(os.str().c_str(), stderr);
}
#define MI_LOG_DEBUG(...)                                                   \
    do {                                                                    \
        if (mi_log_debug_on()) mi_log_debug(__LINE__, __FUNCTION__, __VA_ARGS__); \
    } while (0)
// CCL_FATAL (src/common/log/log.hpp:333-337): log the error, std::terminate().
// The reference uses it for an unknown dtype or reduction (comp.cpp:56,113,
// bf16.cpp:73, bf16_intrisics.hpp:131, fp16_intrisics.hpp:222-243); the
// standalone build does the same, so a caller sees the reference's behaviour.
[[noreturn]] static void mi_ccl_fatal(const std::string& msg) {
    fprintf(stderr, "oneccl_amd: FATAL: %s\n", msg.c_str());
    fflush(stderr);
    std::terminate();
}
#define MI_CCL_FATAL(msg) mi_ccl_fatal(msg)
#include "../../include/mi_ccl_comp_async.hpp"
#include "../../include/mi_ccl_lp_host.hpp"
#endif

// bf16.cpp:26-30, fp16.cpp:25-39 — referenced by env.cpp:711-720, 1101-1102
std::map<ccl_bf16_impl_type, std::string> bf16_impl_names = {
    std::make_pair(ccl_bf16_scalar, "scalar"), std::make_pair(ccl_bf16_avx512f, "avx512f"),
    std::make_pair(ccl_bf16_avx512bf, "avx512bf")};

std::map<ccl_fp16_impl_type, std::string> fp16_impl_names = {
    std::make_pair(ccl_fp16_no_compiler_support, "no_compiler_support"),
    std::make_pair(ccl_fp16_no_hardware_support, "no_hardware_support"),
    std::make_pair(ccl_fp16_f16c, "f16c"), std::make_pair(ccl_fp16_avx512f, "avx512f"),
    std::make_pair(ccl_fp16_avx512fp16, "avx512fp16")};

std::map<ccl_fp16_impl_type, std::string> fp16_env_impl_names = {
    std::make_pair(ccl_fp16_f16c, "f16c"), std::make_pair(ccl_fp16_avx512f, "avx512f"),
    std::make_pair(ccl_fp16_avx512fp16, "avx512fp16")};

// A reduce whose operands are all host memory runs on the calling thread's
// CPU (host_reduce.cpp), as the reference runs every reduce, when its bucket
// is at most
//   CCL_COMP_HOST_MAX_BYTES         bytes, if any operand is pageable memory
//                                   (the GPU would stage it), default 16 MiB;
//   CCL_COMP_HOST_MAX_PINNED_BYTES  bytes, if all are pinned (the GPU reads
//                                   them in place over PCIe), default 16 MiB;
// larger host buckets are split between the GPU and the calling thread (see
// coop_fold), and all device operands run on the GPU.  0 = always the GPU.
// Above the threshold a host bucket is split: the GPU reduces the tail while
// the calling thread reduces a head of this share of the elements
// (CCL_COMP_HOST_SHARE / CCL_COMP_HOST_SHARE_PINNED; 0 = the GPU alone).
// The defaults come from the MI355X sweeps (EPYC 9575F host, DESIGN.md §6,
// profiles/round2_dispatch/): below 16 MiB one core beats a GPU round trip
// (4 KiB: 1.8 vs 16.7 us); from 32 MiB up the split at 0.45 moves 32-46
// GiB/s against 21-23 for one core and 17-25 for the GPU alone.  When the
// share is not set in the environment, each thread adapts it from the
// rates its own split calls measure (coop_fold; CCL_COMP_HOST_SHARE_ADAPT=0
// keeps the default fixed): the best share moved from 0.45 to 0.4 on a box
// whose core read pinned pages at 14 instead of 22 GiB/s.
// Several threads may reduce host buckets at once (oneCCL's CCL_WORKER_COUNT
// workers, worker.cpp:310-379), and they share one PCIe link and the host's
// DRAM.  CCL_COMP_HOST_SPLIT_WORKERS (pageable) / _PINNED caps the number of
// such threads (host_workers) up to which a bucket is still split; beyond it
// every bucket stays on its thread's CPU.  Default 0 = no cap: in paired
// rounds on MI355X boxes the split never lost to all-CPU at 1-16 workers,
// 64 MiB buckets (+10-80 %; profiles/round2_dispatch/workers_paired_*,
// DESIGN.md §6).  The cap is for hosts whose DRAM the staging copies would
// saturate first.
static const size_t kHostMaxPageableDefault = 16ull << 20;
static const size_t kHostMaxPinnedDefault = 16ull << 20;
static const double kHostShareDefault = 0.45;
static const double kHostSharePinnedDefault = 0.45;
static const int kSplitWorkersDefault = 0;
static const int kSplitWorkersPinnedDefault = 0;

struct HostMax {
    size_t pageable = 0, pinned = 0;
    double share = 0, share_pinned = 0;  // cooperative split, see coop_fold
    bool adapt = false, adapt_pinned = false;  // shares not fixed by the environment
    int split_workers = 0, split_workers_pinned = 0;  // 0 = split whatever the number of workers
};

static HostMax parse_host_max() {
    HostMax m;
    if (!mi_host_supported()) return m;  // no AVX2/F16C: the GPU takes everything
    const char* v = getenv("CCL_COMP_HOST_MAX_BYTES");
    const char* p = getenv("CCL_COMP_HOST_MAX_PINNED_BYTES");
    m.pageable = v ? (size_t)strtoull(v, nullptr, 0) : kHostMaxPageableDefault;
    m.pinned = p ? (size_t)strtoull(p, nullptr, 0) : std::min(kHostMaxPinnedDefault, m.pageable);
    const char* sh = getenv("CCL_COMP_HOST_SHARE");
    const char* shp = getenv("CCL_COMP_HOST_SHARE_PINNED");
    m.share = std::min(0.95, std::max(0.0, sh ? atof(sh) : kHostShareDefault));
    m.share_pinned = std::min(0.95, std::max(0.0, shp ? atof(shp) : kHostSharePinnedDefault));
    if (m.pageable == 0) m.share = m.share_pinned = 0;  // "always the GPU"
    if (m.pinned == 0) m.share_pinned = 0;               // pinned buckets: always the GPU, never split
    const char* ad = getenv("CCL_COMP_HOST_SHARE_ADAPT");
    const bool adapt = !(ad && atoi(ad) == 0);
    m.adapt = adapt && !sh && m.share > 0;
    m.adapt_pinned = adapt && !shp && m.share_pinned > 0;
    const char* sw = getenv("CCL_COMP_HOST_SPLIT_WORKERS");
    const char* swp = getenv("CCL_COMP_HOST_SPLIT_WORKERS_PINNED");
    m.split_workers = std::max(0, sw ? atoi(sw) : kSplitWorkersDefault);
    m.split_workers_pinned = std::max(0, swp ? atoi(swp) : kSplitWorkersPinnedDefault);
    return m;
}

#ifdef MI_ONECCL_TREE
static HostMax mi_host_max() {
    // read once, like oneCCL's env; whole cache lines, as MiEnv below
    struct alignas(64) Snap {
        HostMax m;
    };
    static const Snap s{parse_host_max()};
    return s.m;
}
#endif

#ifndef MI_ONECCL_TREE
// ---------------------------------------------------------------------------
// standalone environment: the reference's CPUID detection
// (src/comp/bf16/bf16_utils.hpp:30-68, src/comp/fp16/fp16_utils.hpp:37-88)
// then the CCL_BF16 / CCL_FP16 override (src/common/env/env.cpp:711-720)
// ---------------------------------------------------------------------------
namespace {

// A snapshot owns whole cache lines (alignas, C++17 aligned new): every
// reduce of every worker reads it, and a heap neighbour that some thread
// writes would otherwise make those reads miss across the socket on every
// call (a 4 KiB bf16 MPI user op ran 2.6x slower at 16 threads than at one
// with the snapshot beside a worker's buffer).
struct alignas(64) MiEnv {
    ccl_bf16_impl_type bf16 = ccl_bf16_scalar;
    ccl_fp16_impl_type fp16 = ccl_fp16_no_compiler_support;
    int device = -1;  // CCL_COMP_HIP_DEVICE
    HostMax host_max;  // CCL_COMP_HOST_MAX_BYTES, CCL_COMP_HOST_MAX_PINNED_BYTES
    bool log_debug = false;  // CCL_LOG_LEVEL=debug|trace (env.cpp's log level)
};

// The parsed environment is an immutable snapshot published through an
// atomic pointer: every reduce reads it several times, from up to
// CCL_WORKER_COUNT threads at once, so the read takes no lock.  A reload
// (the standalone test hook mi_ccl_env_reload) publishes a new snapshot and
// keeps the old ones alive, since a reader may still hold a reference.
std::mutex g_env_mu;  // serialises parsing and publishing
std::atomic<const MiEnv*> g_env_cur{nullptr};
std::vector<std::unique_ptr<MiEnv>> g_env_all;  // every snapshot published (under g_env_mu)

void cpuid(uint32_t leaf, uint32_t sub, uint32_t r[4]) {
#if defined(__x86_64__) || defined(__i386__)
    __asm__ __volatile__("cpuid" : "=a"(r[0]), "=b"(r[1]), "=c"(r[2]), "=d"(r[3]) : "a"(leaf), "c"(sub));
#else
    r[0] = r[1] = r[2] = r[3] = 0;
#endif
}

std::set<ccl_bf16_impl_type> bf16_impl_types() {
    std::set<ccl_bf16_impl_type> s{ccl_bf16_scalar};
    uint32_t r[4];
    cpuid(7, 0, r);
    const bool f = ((r[1] >> 16) & 1) && ((r[1] >> 30) & 1) && ((r[1] >> 31) & 1);
    cpuid(7, 1, r);
    const bool bf = (r[0] >> 5) & 1;
    if (f) s.insert(ccl_bf16_avx512f);
    if (bf) s.insert(ccl_bf16_avx512bf);
    return s;
}

std::set<ccl_fp16_impl_type> fp16_impl_types() {
    std::set<ccl_fp16_impl_type> s;
    uint32_t r[4];
    cpuid(1, 0, r);
    const bool f16c = (r[2] >> 29) & 1;
    cpuid(7, 0, r);
    const bool f = ((r[1] >> 16) & 1) && ((r[1] >> 30) & 1) && ((r[1] >> 31) & 1);
    const bool fp16 = ((r[1] >> 30) & 1) && ((r[3] >> 23) & 1);
    if (fp16) s.insert(ccl_fp16_avx512fp16);
    if (f) s.insert(ccl_fp16_avx512f);
    if (f16c) s.insert(ccl_fp16_f16c);
    if (!fp16 && !f && !f16c) s.insert(ccl_fp16_no_hardware_support);
    return s;
}

void parse_env_locked() {
    std::unique_ptr<MiEnv> snap(new MiEnv);
    MiEnv& e = *snap;
    e.bf16 = *bf16_impl_types().rbegin();
    if (const char* v = getenv("CCL_BF16")) {
        bool found = false;
        for (auto& kv : bf16_impl_names)
            if (kv.second == v) {
                e.bf16 = kv.first;
                found = true;
            }
        if (!found) MI_CCL_THROW(std::string("unexpected CCL_BF16 value: ") + v);
    }
    auto fp16_types = fp16_impl_types();
    e.fp16 = *fp16_types.rbegin();
    if (const char* v = getenv("CCL_FP16")) {
        bool found = false;
        for (auto& kv : fp16_env_impl_names)
            if (kv.second == v) {
                e.fp16 = kv.first;
                found = true;
            }
        if (!found) MI_CCL_THROW(std::string("unexpected CCL_FP16 value: ") + v);
    }
    if (fp16_types.find(e.fp16) == fp16_types.end())
        MI_CCL_THROW("unsupported FP16 impl type: " + fp16_impl_names[e.fp16]);
    if (const char* v = getenv("CCL_COMP_HIP_DEVICE")) {
        e.device = atoi(v);
    } else {
        // the launcher's local rank, read as oneCCL's set_local_coord reads
        // it for hydra, torchrun and no launcher (global.cpp:182-220)
        int idx = -1;
        for (const char* name : {"MPI_LOCALRANKID", "LOCAL_RANK", "CCL_LOCAL_RANK"})
            if (const char* v = getenv(name)) {
                idx = atoi(v);
                break;
            }
        // no local rank: no device count either, so a CPU-only first call (a
        // small MPI user-op fold) does not initialise the HIP runtime
        e.device = idx >= 0 ? mi_local_gpu(idx, mi_device_count()) : -1;
    }
    e.host_max = parse_host_max();
    if (const char* v = getenv("CCL_LOG_LEVEL")) e.log_debug = !strcmp(v, "debug") || !strcmp(v, "trace");
    g_env_all.push_back(std::move(snap));
    g_env_cur.store(g_env_all.back().get(), std::memory_order_release);
}

const MiEnv& env() {
    if (const MiEnv* e = g_env_cur.load(std::memory_order_acquire)) return *e;
    std::lock_guard<std::mutex> g(g_env_mu);
    if (!g_env_cur.load(std::memory_order_relaxed)) parse_env_locked();
    return *g_env_cur.load(std::memory_order_relaxed);
}

}  // namespace

static ccl_bf16_impl_type mi_bf16_impl() { return env().bf16; }
static ccl_fp16_impl_type mi_fp16_impl() { return env().fp16; }
static int mi_comp_device() { return env().device; }
static HostMax mi_host_max() { return env().host_max; }
static bool mi_log_debug_on() { return env().log_debug; }
#endif  // !MI_ONECCL_TREE

// The GPU for host buckets when the environment names none: the process's
// local rank modulo the visible GPUs, so the ranks of one node send their
// host buckets over their own GPUs' PCIe links instead of all over GPU 0's;
// -1 (the calling thread's current device) for an unknown rank or one GPU.
static int mi_local_gpu(int local_idx, int ndev) { return local_idx >= 0 && ndev > 1 ? local_idx % ndev : -1; }

// ---------------------------------------------------------------------------
// semantics selection
// ---------------------------------------------------------------------------
namespace {

unsigned bf16_flags(ccl_bf16_impl_type impl) {
    switch (impl) {
        case ccl_bf16_scalar: return 0u;  // std::min/max, truncate (bf16.cpp:63-85)
        case ccl_bf16_avx512f: return MI_F_MINMAX_INOUT_FIRST;  // MINPS order, truncate
        case ccl_bf16_avx512bf: return MI_F_MINMAX_INOUT_FIRST | MI_F_BF16_RNE;
    }
    return 0u;
}

// fp16: f16c / avx512f compute in fp32 with MINPS order and RNE
// (fp16_intrisics.hpp:95-148); avx512fp16 in native fp16 (:150-176), which
// gives the same bits for sum and prod (fp32 has 24 >= 2*11+2 bits) and for
// min/max returns a NaN inout as stored (MI_F_FP16_NATIVE_MINMAX), all proven
// on every operand pair (oracle/FP16_NATIVE_CHECK.json).  Any other impl
// computes nothing (it falls through every branch, :204-248) — reproduced by
// returning false.
bool fp16_flags(ccl_fp16_impl_type impl, unsigned* f) {
    *f = MI_F_MINMAX_INOUT_FIRST | (impl == ccl_fp16_avx512fp16 ? MI_F_FP16_NATIVE_MINMAX : 0u);
    return impl == ccl_fp16_f16c || impl == ccl_fp16_avx512f || impl == ccl_fp16_avx512fp16;
}

// Flags of a 2-input reduce of `dt` under the impl types in force (the
// semantic selection of comp.cpp:96-114 -> bf16.cpp / fp16.cpp).  false: the
// reference computes nothing (fp16 impl outside f16c/avx512f/avx512fp16).
bool reduce_semantics(int dt, unsigned* f) {
    *f = 0u;  // CCL_REDUCE: std::min/std::max operand order
    if (dt == MI_BFLOAT16) {
        *f = bf16_flags(mi_bf16_impl());
        return true;
    }
    if (dt == MI_FLOAT16) return fp16_flags(mi_fp16_impl(), f);
    return true;
}

// sum / prod / min / max: the cases of the reference's op switches; any
// other value (custom included, where it reaches them) is CCL_FATAL there.
bool builtin_op(ccl::reduction op) {
    const int v = static_cast<int>(op);
    return v >= 0 && v <= 3;
}

std::string unexpected(int v) { return "unexpected value " + std::to_string(v); }

void check(int rc, const char* where) {
    if (rc != 0) MI_CCL_THROW(std::string(where) + " failed: " + mi_last_error());
}

// The schedule's word on where the operands live, as the reference takes it
// (src/comp/comp.cpp:136-142): a schedule whose collective has no stream
// (sched->coll_param.stream, src/coll/coll_param.hpp:129) works on host
// memory only -- the reference then calls ccl_comp_reduce_regular on the CPU
// without classifying anything, and a build without SYCL never classifies
// (:196-198).  With a stream, or with no schedule (the MPI user op,
// atl_mpi_ctx.cpp:87-124, and this repo's C view), the operands are looked
// up.  The word holds for the duration of one entry-point call on this
// thread (SchedScope).
thread_local bool t_host_by_sched = false;

bool host_schedule(const ccl_sched* sched) { return sched && !sched->coll_param.stream; }

struct SchedScope {
    const bool prev;
    explicit SchedScope(const ccl_sched* sched) : prev(t_host_by_sched) { t_host_by_sched = host_schedule(sched); }
    // a caller whose operands are host memory by construction (the MPI user
    // ops, include/mi_ccl_lp_host.hpp) gives the same word without a schedule
    explicit SchedScope(bool host) : prev(t_host_by_sched) { t_host_by_sched = host; }
    ~SchedScope() { t_host_by_sched = prev; }
};

bool is_device_ptr(const void* p) {
    int dev = -1;
    return mi_pointer_kind(p, &dev) == 0;
}

// The host word, checked.  A caller that says its operands are host memory
// (a schedule without a stream, the MPI user ops, the copy entries) has them
// dereferenced on the CPU, as the reference does; device memory passed there
// would fault the host instead of being detected.  Under CCL_COMP_CHECK_HOST=1
// (or CCL_LOG_LEVEL=debug|trace) such operands are classified anyway and
// device memory fails loudly (CCL_THROW).  Read once.
bool check_host_word() {
    static const bool on = [] {
        if (const char* v = getenv("CCL_COMP_CHECK_HOST")) return strcmp(v, "0") != 0;
        const char* l = getenv("CCL_LOG_LEVEL");
        return l && (strcmp(l, "debug") == 0 || strcmp(l, "trace") == 0);
    }();
    return on;
}

void verify_host_word(const void* const* ptrs, int n, const char* what) {
    if (!check_host_word()) return;
    for (int i = 0; i < n; i++)
        if (ptrs[i] && is_device_ptr(ptrs[i]))
            MI_CCL_THROW(std::string(what) + ": device memory passed where the caller says host memory "
                         "(a collective without a stream, an MPI user op or a host copy entry)");
}

// reference behaviour for a user callback (comp.cpp:84-88); device operands
// are staged through host memory, as the reference's SYCL branch does
// (comp.cpp:136-195)
void run_custom(const void* in_buf, size_t in_count, void* inout_buf, size_t* out_count,
                const ccl_datatype& dtype, ccl::reduction_fn fn, const ccl::fn_context* context) {
    if (!fn) MI_CCL_THROW("custom reduction requires user callback");
    // host memory by the schedule's word: straight to the callback, as the
    // reference does (comp.cpp:139-142)
    if (t_host_by_sched) {
        const void* ops[2] = {in_buf, inout_buf};
        verify_host_word(ops, 2, "custom reduce");
    }
    const bool din = !t_host_by_sched && is_device_ptr(in_buf), dio = !t_host_by_sched && is_device_ptr(inout_buf);
    if (!din && !dio) {
        fn(in_buf, in_count, inout_buf, out_count, dtype.idx(), context);
        return;
    }
    const size_t bytes = in_count * dtype.size();
    std::vector<char> hin, hio;
    const void* in_h = in_buf;
    void* io_h = inout_buf;
    if (din) {
        hin.resize(bytes);
        check(mi_copy_sync(in_buf, hin.data(), bytes, 0, -1), "mi_copy_sync");
        in_h = hin.data();
    }
    if (dio) {
        hio.resize(bytes);
        check(mi_copy_sync(inout_buf, hio.data(), bytes, 0, -1), "mi_copy_sync");
        io_h = hio.data();
    }
    fn(in_h, in_count, io_h, out_count, dtype.idx(), context);
    if (dio) check(mi_copy_sync(hio.data(), inout_buf, bytes, 0, -1), "mi_copy_sync");
}

int dtype_id(const ccl_datatype& dt) { return static_cast<int>(dt.idx()); }

// ---- tracing ----------------------------------------------------------------
// The reference wraps ccl_comp_reduce_regular in an ITT event of that name
// (comp.cpp:90-93, 116-118), emitted only when CCL_ITT_LEVEL > 0
// (sched_timer.cpp:141-203: event_get/start/end return at once at level 0,
// the default).  The ROCm counterpart is a roctx range, which
// `rocprofv3 --marker-trace` records next to the kernel trace, under the same
// knob (or MI_ROCTX=1; MI_ROCTX=0 forces it off), read once.  The roctx
// library is loaded on first use with dlopen, so the shim has no link-time
// dependency on the profiler SDK; without it ranges are no-ops.  Off, a
// range costs nothing: on, two calls into the SDK (8 ns per 4 KiB reduce on
// MI355X's host, profiles/round4_host/).
struct Roctx {
    int (*push)(const char*) = nullptr;
    int (*pop)() = nullptr;
};

const Roctx& roctx() {
    static const Roctx r = [] {
        Roctx x;
        const char* mi = getenv("MI_ROCTX");
        const char* itt = getenv("CCL_ITT_LEVEL");
        const bool on = mi ? strcmp(mi, "0") != 0 : (itt && atoi(itt) > 0);
        if (!on) return x;
        for (const char* name : {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so",
                                 "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1"}) {
            void* h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
            if (!h) continue;
            x.push = reinterpret_cast<int (*)(const char*)>(dlsym(h, "roctxRangePushA"));
            x.pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
            if (x.push && x.pop) break;
            x = Roctx();
        }
        return x;
    }();
    return r;
}

// CCL_COMP_HIP_SHARD_DEVICES=<d0>,<d1>,...: host-resident reduces are split by
// element range over these GPUs, each shard over its own PCIe link
// (mi_reduce_multi_sync_sharded).  Unset or one device: a single GPU.
// Read on every synchronous reduce: a published snapshot, as env() above.
std::mutex g_shard_mu;
// padded on both sides, so the vector's header shares no cache line with a
// heap neighbour (as MiEnv; padding rather than alignas, since the in-tree
// build is C++11 without aligned new)
struct ShardDevs {
    char pad0[64];
    std::vector<int> v;
    char pad1[64];
};
std::atomic<const std::vector<int>*> g_shard_cur{nullptr};
std::vector<std::unique_ptr<ShardDevs>> g_shard_all;  // under g_shard_mu

const std::vector<int>& shard_devices() {
    if (const std::vector<int>* d = g_shard_cur.load(std::memory_order_acquire)) return *d;
    std::lock_guard<std::mutex> g(g_shard_mu);
    if (const std::vector<int>* d = g_shard_cur.load(std::memory_order_relaxed)) return *d;
    std::unique_ptr<ShardDevs> owner(new ShardDevs);
    std::vector<int>* devs = &owner->v;
    if (const char* v = getenv("CCL_COMP_HIP_SHARD_DEVICES")) {
        std::string cur;
        for (const char* c = v;; c++) {
            if (*c == ',' || *c == 0) {
                if (!cur.empty()) devs->push_back(atoi(cur.c_str()));
                cur.clear();
                if (!*c) break;
            } else {
                cur += *c;
            }
        }
    }
    g_shard_all.push_back(std::move(owner));
    g_shard_cur.store(devs, std::memory_order_release);
    return *devs;
}

#ifndef MI_ONECCL_TREE
void shard_env_reload() {  // standalone only: oneCCL's env is read once, at init
    std::lock_guard<std::mutex> g(g_shard_mu);
    g_shard_cur.store(nullptr, std::memory_order_release);
}
#endif

// Host kind of a set of operands: 0 = some operand is device memory,
// 1 = all pinned host memory, 2 = host memory, some of it pageable,
// 3 = host memory by the schedule's word (kHostBySched, below: not looked up,
// routed as 2).  Each lookup goes to libmi_reduce (mi_pointer_kind_range),
// which answers from the host ranges their owner declared
// (mi_ccl_comp_register_host_buffer -> mi_host_declare) without asking HIP.
constexpr int kHostBySched = 3;

int pointer_kind(const void* p, size_t bytes) {
    int dev = -1;
    return mi_pointer_kind_range(p, bytes, &dev);
}

// Each distinct pointer is classified once: the lookup
// (hipPointerGetAttributes) takes a runtime-wide lock, so with several worker
// threads reducing small host chunks it is the one step that serialises
// them, and the in-place form passes inout both as out and as the first input.
// `bytes` (0 = unknown) is each operand's extent, for the registry.
int host_kind(const void* const* ptrs, int n, const void* out, size_t bytes = 0) {
    if (t_host_by_sched) {
        // host memory by the schedule's word: a bucket that takes the CPU
        // path whatever its pointer kinds needs no lookup at all; above
        // that the kinds still pick pinned zero-copy or staging
        const HostMax m = mi_host_max();
        if (m.pageable > 0 && m.pinned > 0 && bytes <= std::min(m.pageable, m.pinned)) {
            if (check_host_word()) {
                verify_host_word(&out, 1, "reduce");
                for (int i = 0; i < n; i++)
                    if (ptrs[i] != out) verify_host_word(&ptrs[i], 1, "reduce");
            }
            return kHostBySched;
        }
    }
    int kind = pointer_kind(out, bytes);
    if (kind == 0) return 0;
    for (int i = 0; i < n; i++) {
        if (ptrs[i] == out) continue;
        const int k = pointer_kind(ptrs[i], bytes);
        if (k == 0) return 0;
        kind = std::max(kind, k);
    }
    return kind;
}

bool all_host(const void* const* ptrs, int n, const void* out, size_t bytes = 0) {
    return host_kind(ptrs, n, out, bytes) != 0;
}

// ---- the dispatcher's decision, logged ------------------------------------
const char* kind_name(int kind) {
    switch (kind) {
        case 0: return "device memory (or not classified: dispatcher off)";
        case 1: return "pinned host memory";
        case 2: return "host memory, some pageable";
        default: return "host memory by the schedule (no stream; not looked up)";
    }
}

// the GPU's route for operands of this kind (mi_reduce.hip reduce_issue)
const char* gpu_route(int kind) {
    return kind == 0 ? "gpu" : kind == 1 ? "gpu zero-copy (pinned, read in place)" : "gpu staged (pageable)";
}

void log_route(const char* what, size_t count, int dt, int k, int kind, const char* path, double share = -1.0) {
    MI_LOG_DEBUG(what, ": count ", count, ", dtype ", dt, ", bytes ", count * mi_dtype_size(dt), ", inputs ", k,
                 ", operands: ", kind_name(kind), ", path: ", path,
                 share >= 0 ? ", cpu head share " : "", share >= 0 ? std::to_string(share) : std::string());
}

// The dispatcher: host-resident buckets up to the crossover stay on the
// calling thread's CPU: below it a GPU round trip
// costs more than the reduce.
bool host_path(const void* const* ins, int k, const void* out, size_t bytes, int* kind_out = nullptr) {
    const HostMax m = mi_host_max();
    if (bytes > std::max(m.pageable, m.pinned)) return false;  // GPU whatever the kinds: skip classifying
    const int kind = host_kind(ins, k, out, bytes);
    if (kind_out) *kind_out = kind;
    if (kind == 0) return false;
    const size_t lim = kind == 1 ? m.pinned : m.pageable;
    return lim > 0 && bytes <= lim;
}

// the host path runs after this thread's outstanding asynchronous requests,
// which may still be writing these operands
int host_fold(const void* const* ins, int k, void* out, size_t count, int dt, int op, unsigned flags) {
    if (int rc = mi_thread_sync()) return rc;
    return mi_host_reduce(ins, k, out, count, dt, op, flags);
}

// The synchronous fold every entry point ends in: the calling thread's CPU
// for small host-resident buckets, otherwise one GPU, or, for host operands
// under CCL_COMP_HIP_SHARD_DEVICES, several.
// A host bucket above the crossover: the GPU takes the tail [s, count)
// asynchronously (staged on this thread's worker, or the zero-copy kernel on
// pinned memory) while the calling thread reduces the head [0, s) with the
// host path; then it waits for the GPU part.  s is a multiple of 256
// elements, so the bf16 keep-precision count % 16 tail stays in the last
// part exactly as in the whole array.  Element-wise, so the bits are those of
// either path alone.
//
// Adaptive share (`adapt`: not fixed by the environment).  The head runs in
// chunks of ~8 MiB, polling the GPU part between them, so the call knows both
// parts' durations even when the GPU finishes first; the rates give the share
// at which both would have finished together, and the thread's share for
// this pointer kind moves halfway there (kept within [0.1, 0.9]).  A thread's
// first split call of a kind only warms up: it pays for the staging buffers
// and the worker thread, which made it read as a GPU 10x slower than it is
// (profiles/round2_dispatch/adapt_trace.jsonl).  The
// chunks are multiples of 256 elements: each is a whole head region for the
// keep-precision tail rule, as above.
//
// The share only balances the two parts' finishing times; whether splitting
// pays at all is measured too.  Where a core reads the buffers slowly and its
// head slows the GPU's zero-copy reads (hipHostMalloc'd pages on a far NUMA
// node), the split ran up to 25 % below the GPU alone.  So an
// adapting thread times the GPU alone now and then (its 3rd call of a kind,
// then every 32nd split), and when a split's whole rate falls below 0.95 of
// that, the next 8 buckets of that kind go to the GPU alone before a split
// is tried again.
struct SplitShare {
    double share[2] = {-1.0, -1.0};  // [0] some operand pageable, [1] all pinned; < 0: not started
    unsigned calls[2] = {0, 0};
    double gpu_rate[2] = {-1.0, -1.0};  // elements / s of the whole bucket on the GPU alone
    unsigned gpu_left[2] = {0, 0};      // buckets still to run on the GPU alone
    unsigned since_probe[2] = {0, 0};   // split calls since the GPU alone was last timed
};
static thread_local SplitShare t_split;

// After an adaptive split of `count` elements that took `t` seconds in all:
// schedule GPU-alone calls (a probe, or a stretch when the split lost).
static void split_verdict(int pk, size_t count, double t) {
    SplitShare& sp = t_split;
    const unsigned c = sp.calls[pk];
    if (t > 0 && sp.gpu_rate[pk] > 0 && (double)count / t < 0.95 * sp.gpu_rate[pk]) {
        sp.gpu_left[pk] = 8;
        sp.since_probe[pk] = 0;
    } else if (c == 2 || ++sp.since_probe[pk] >= 32) {
        sp.gpu_left[pk] = 1;
        sp.since_probe[pk] = 0;
    }
}

// A bucket the GPU took alone in `t` seconds.
static void gpu_alone_timed(int pk, size_t count, double t) {
    if (t <= 0) return;
    const double r = (double)count / t;
    double& g = t_split.gpu_rate[pk];
    g = g < 0 ? r : 0.5 * g + 0.5 * r;
}

// An adapting thread's next bucket of kind pk: the GPU alone (timed) while
// split_verdict has GPU-alone buckets scheduled; consumes one.
static bool take_gpu_alone(int pk) {
    if (t_split.gpu_left[pk] == 0) return false;
    t_split.gpu_left[pk]--;
    return true;
}

// After a split of `count` elements whose head of `head` took t_cpu seconds
// on the CPU and whose tail took t_gpu on the GPU (both from the split's
// start): move the share halfway toward the balance point, kept within
// [0.1, 0.9], and judge the split against the GPU alone.  A thread's first
// split of a kind only warms up.  Shared by the synchronous (coop_fold) and
// asynchronous (settle_split) paths.
static void split_update(int pk, size_t count, size_t head, double t_cpu, double t_gpu) {
    if (t_cpu <= 0 || t_gpu <= 0 || head == 0 || head >= count) return;
    if (t_split.calls[pk]++ == 0) return;
    const double r_cpu = (double)head / t_cpu, r_gpu = (double)(count - head) / t_gpu;
    double& cur = t_split.share[pk];
    cur = std::min(0.9, std::max(0.1, 0.5 * cur + 0.5 * r_cpu / (r_cpu + r_gpu)));
    split_verdict(pk, count, std::max(t_cpu, t_gpu));
}

static double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int coop_fold(const void* const* ins, int k, void* out, size_t count, int dt, int op, unsigned flags, double share,
              int pinned, bool adapt) {
    const int pk = pinned ? 1 : 0;
    double& cur = t_split.share[pk];
    if (adapt) {
        if (cur < 0) cur = share;
        share = cur;
        if (take_gpu_alone(pk)) {  // the GPU alone, timed
            log_route("reduce", count, dt, k, pinned ? 1 : 2, pinned ? "gpu zero-copy alone (timed against the split)"
                                                                     : "gpu staged alone (timed against the split)");
            const double t0 = now_s();
            const int rc = mi_reduce_multi_sync(ins, k, out, count, dt, op, flags, mi_comp_device());
            if (rc == 0) gpu_alone_timed(pk, count, now_s() - t0);
            return rc;
        }
    }
    const size_t es = mi_dtype_size(dt);
    size_t s = (size_t)((double)count * share);
    s -= s % 256;
    if (s == 0 || s >= count) {
        log_route("reduce", count, dt, k, pinned ? 1 : 2, gpu_route(pinned ? 1 : 2));
        return mi_reduce_multi_sync(ins, k, out, count, dt, op, flags, mi_comp_device());
    }
    log_route("reduce", count, dt, k, pinned ? 1 : 2, "split: calling thread's cpu head + gpu tail", share);
    if (int rc = mi_thread_sync()) return rc;  // earlier requests of this thread first
    const void* gins[MI_MAX_INPUTS];
    for (int i = 0; i < k; i++) gins[i] = static_cast<const char*>(ins[i]) + s * es;
    mi_request_t r = nullptr;
    const double t0 = now_s();
    if (int rc = mi_reduce_start(gins, k, static_cast<char*>(out) + s * es, count - s, dt, op, flags,
                                 mi_comp_device(), &r))
        return rc;
    size_t chunk = adapt ? std::max<size_t>(256, ((size_t)8 << 20) / es) : s;
    chunk -= chunk % 256;
    double t_gpu = -1.0;
    int hrc = 0;
    for (size_t i = 0; i < s && hrc == 0; i += chunk) {
        const void* hins[MI_MAX_INPUTS];
        for (int j = 0; j < k; j++) hins[j] = static_cast<const char*>(ins[j]) + i * es;
        hrc = mi_host_reduce(hins, k, static_cast<char*>(out) + i * es, std::min(chunk, s - i), dt, op, flags);
        int done = 0;
        if (adapt && t_gpu < 0 && mi_test(r, &done) == 0 && done) t_gpu = now_s() - t0;
    }
    const double t_cpu = now_s() - t0;
    const int wrc = mi_wait(r);
    if (t_gpu < 0) t_gpu = now_s() - t0;
    (void)mi_request_free(r);
    if (adapt && hrc == 0 && wrc == 0) split_update(pk, count, s, t_cpu, t_gpu);
    return wrc ? wrc : hrc;
}

// Threads reducing host buckets: each caller of a host-bucket fold owns a
// slot, marked while the call runs and stamped when it returns.  A thread
// counts as a worker while it is inside such a call or returned from one
// within the last kSeenWindowNs, so oneCCL's workers, which reduce chunk
// after chunk, are counted across the gaps between their calls.
constexpr int kSeenSlots = 64;
constexpr int64_t kSeenWindowNs = 50 * 1000 * 1000;
struct alignas(64) SeenSlot {  // one cache line per slot
    std::atomic<int64_t> last_ns;
    std::atomic<int> inside;
};
static SeenSlot g_seen[kSeenSlots];
static std::atomic<unsigned> g_seen_next(0);
static thread_local int t_seen = -1;

// The coarse monotonic clock (a few ms of resolution, against the 50 ms
// window): read on every host-bucket call, where steady_clock's full-
// resolution read cost as much as a quarter of a 4 KiB CPU reduce.
static int64_t now_ns() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC_COARSE, &ts);
    return (int64_t)ts.tv_sec * 1000000000 + ts.tv_nsec;
}

struct HostCall {  // marks the calling thread as reducing a host bucket while `on`
    int slot = -1;
    explicit HostCall(bool on) {
        if (!on) return;
        if (t_seen < 0) t_seen = (int)(g_seen_next.fetch_add(1, std::memory_order_relaxed) % kSeenSlots);
        slot = t_seen;
        g_seen[slot].inside.fetch_add(1, std::memory_order_relaxed);
    }
    ~HostCall() {
        if (slot < 0) return;
        g_seen[slot].last_ns.store(now_ns(), std::memory_order_relaxed);
        g_seen[slot].inside.fetch_sub(1, std::memory_order_relaxed);
    }
};

int host_workers() {
    const int64_t t = now_ns();
    int n = 0;
    for (int i = 0; i < kSeenSlots; i++) {
        const SeenSlot& s = g_seen[i];
        if (s.inside.load(std::memory_order_relaxed) > 0) n++;
        else {
            const int64_t last = s.last_ns.load(std::memory_order_relaxed);
            if (last != 0 && t - last < kSeenWindowNs) n++;
        }
    }
    return n;
}

int fold_sync(const void* const* ins, int k, void* out, size_t count, int dt, int op, unsigned flags) {
    const size_t bytes = count * mi_dtype_size(dt);
    const HostMax m = mi_host_max();
    // 0: some operand is device memory (or the dispatcher is off), 1: all
    // pinned, 2: host memory, some of it pageable
    const int kind = (m.pageable > 0 || m.pinned > 0) ? host_kind(ins, k, out, bytes) : 0;
    const std::vector<int>& devs = shard_devices();
    const HostCall call(kind != 0);  // the thread counts among the host-bucket workers
    if (kind != 0) {
        const size_t lim = kind == 1 ? m.pinned : m.pageable;
        if (lim > 0 && bytes <= lim) {
            log_route("reduce", count, dt, k, kind, "cpu (calling thread)");
            return host_fold(ins, k, out, count, dt, op, flags);
        }
        const double share = kind == 1 ? m.share_pinned : m.share;
        if (devs.size() < 2 && share > 0) {
            const int limit = kind == 1 ? m.split_workers_pinned : m.split_workers;
            if (limit > 0 && host_workers() > limit) {
                log_route("reduce", count, dt, k, kind, "cpu (calling thread; more host workers than the split cap)");
                return host_fold(ins, k, out, count, dt, op, flags);
            }
            return coop_fold(ins, k, out, count, dt, op, flags, share, kind == 1,
                             kind == 1 ? m.adapt_pinned : m.adapt);
        }
    }
    if (devs.size() >= 2) {
        bool host = !is_device_ptr(out);
        for (int i = 0; i < k && host; i++) host = !is_device_ptr(ins[i]);
        if (host) {
            log_route("reduce", count, dt, k, kind == 0 ? 2 : kind, "gpu sharded over CCL_COMP_HIP_SHARD_DEVICES");
            return mi_reduce_multi_sync_sharded(ins, k, out, count, dt, op, flags, (int)devs.size(), devs.data());
        }
    }
    log_route("reduce", count, dt, k, kind, gpu_route(kind));
    return mi_reduce_multi_sync(ins, k, out, count, dt, op, flags, mi_comp_device());
}

// The asynchronous entries' issue.  A host bucket above the threshold is
// split as in the synchronous path (coop_fold), but its head is folded on
// the thread's staging worker (mi_reduce_split_start), not on the calling
// thread the asynchronous form exists to free; the share is the thread's
// adapted one (or the configured one).  Past the worker cap, and for device
// operands, the GPU takes the whole bucket.
struct SplitIssued {      // an adaptive split issued by start_fold, for the share update on completion
    mi_request_t req = nullptr;
    int kind = 0;            // 0: some operand pageable, 1: all pinned
    size_t count = 0, head = 0;  // head 0: a timed GPU-alone bucket
    bool settled = false;    // the share update is done (or not wanted)
};

// On the caller's thread, once its split request is done: the share update
// coop_fold makes, from times measured where the request ran (the staging
// worker's clock, or a HIP event pair around the zero-copy kernel), never
// from when the caller happened to poll it: a oneCCL worker polls between
// other entries, and that delay would read as a slow GPU.
void settle_split(SplitIssued& sp) {
    if (!sp.req || sp.settled) return;
    sp.settled = true;
    if (sp.head == 0) {  // a GPU-alone bucket
        double t = 0;
        if (mi_request_run_time(sp.req, &t) == 0) gpu_alone_timed(sp.kind, sp.count, t);
        return;
    }
    double th = 0, tt = 0;
    if (mi_request_split_times(sp.req, &th, &tt) != 0) return;
    split_update(sp.kind, sp.count, sp.head, th, tt);
}

int start_fold(const void* const* ins, int k, void* out, size_t count, int dt, int op, unsigned flags,
               mi_request_t* r, SplitIssued* sp = nullptr) {
    const HostMax m = mi_host_max();
    const int kind = (m.pageable > 0 || m.pinned > 0) ? host_kind(ins, k, out, count * mi_dtype_size(dt)) : 0;
    if (kind != 0 && shard_devices().size() < 2) {
        const int pk = kind == 1 ? 1 : 0;
        double share = pk ? m.share_pinned : m.share;
        const bool adapt = share > 0 && (pk ? m.adapt_pinned : m.adapt);
        if (adapt) {
            if (t_split.share[pk] < 0) t_split.share[pk] = share;
            share = t_split.share[pk];
        }
        const int limit = pk ? m.split_workers_pinned : m.split_workers;
        if (adapt && sp && !sp->req && take_gpu_alone(pk)) {  // the GPU alone, timed where it runs
            log_route("reduce_start", count, dt, k, kind, pk ? "gpu zero-copy alone (timed against the split)"
                                                             : "gpu staged alone (timed against the split)");
            const int rc = mi_reduce_start_timed(ins, k, out, count, dt, op, flags, mi_comp_device(), r);
            if (rc == 0) {
                sp->req = *r;
                sp->kind = pk;
                sp->count = count;
                sp->head = 0;
            }
            return rc;
        }
        if (share > 0 && !(limit > 0 && host_workers() > limit)) {
            size_t s = (size_t)((double)count * share);
            s -= s % 256;
            if (s > 0 && s < count) {
                log_route("reduce_start", count, dt, k, kind, "split: staging worker's cpu head + gpu tail",
                          (double)s / (double)count);
                const int rc =
                    mi_reduce_split_start(ins, k, out, count, dt, op, flags, mi_comp_device(), s, &mi_host_reduce, r);
                if (rc == 0 && adapt && sp && !sp->req) {
                    sp->req = *r;
                    sp->kind = pk;
                    sp->count = count;
                    sp->head = s;
                }
                return rc;
            }
        }
    }
    log_route("reduce_start", count, dt, k, kind, gpu_route(kind));
    return mi_reduce_start(ins, k, out, count, dt, op, flags, mi_comp_device(), r);
}

// conversions take the same route: the CPU for small host arrays
int convert_sync(const void* src, int sdt, void* dst, int ddt, size_t count, unsigned flags) {
    const void* ins[1] = {src};
    if (host_path(ins, 1, dst, count * std::max(mi_dtype_size(sdt), mi_dtype_size(ddt)))) {
        if (int rc = mi_thread_sync()) return rc;
        return mi_host_convert(src, sdt, dst, ddt, count, flags);
    }
    return mi_convert_sync(src, sdt, dst, ddt, count, flags, mi_comp_device());
}

int reduce2_sync(const void* in, void* inout, size_t count, int dt, int op, unsigned flags) {
    const void* ins[2] = {inout, in};
    return fold_sync(ins, 2, inout, count, dt, op, flags);
}

struct TraceRange {
    const bool on;
    explicit TraceRange(const char* name) : on(roctx().push != nullptr) {
        if (on) roctx().push(name);
    }
    ~TraceRange() {
        if (on) roctx().pop();
    }
};

}  // namespace

// ===========================================================================
// oneCCL entry points
// ===========================================================================

ccl::status ccl_comp_copy(const void* in_buf, void* out_buf, size_t bytes, bool use_nontemporal) {
    if (bytes == 0) return ccl::status::success;
    if (!in_buf) MI_CCL_THROW("in_buf is null");
    if (!out_buf) MI_CCL_THROW("out_buf is null");
    const void* src[1] = {in_buf};
    if (mi_host_max().pageable > 0 && all_host(src, 1, out_buf, bytes)) {  // host to host on the CPU, as the reference
        check(mi_thread_sync(), "mi_thread_sync");
        // (the host path is on only where mi_host_supported(): AVX2 is there)
        check(mi_host_copy(out_buf, in_buf, bytes, use_nontemporal ? 1 : 0), "mi_host_copy");
        return ccl::status::success;
    }
    check(mi_copy_sync(in_buf, out_buf, bytes, use_nontemporal ? 1 : 0, mi_comp_device()), "mi_copy_sync");
    return ccl::status::success;
}

// The copy of a regular (host) copy entry: oneCCL calls ccl_comp_copy only
// there (copy_entry.cpp:201-206, whose copy type is `regular` only without a
// stream or for h2h, and which asserts neither buffer is device USM, :90-97;
// recv_copy_entry.cpp:53 with an h2h attribute, allreduce.cpp:396-422).  So
// the patched entries (integration/0006) say so and no pointer is looked up:
// the reference's memcpy / non-temporal memcpy (comp.cpp:60-74,
// common/utils/memcpy.hpp) on the calling thread, after its own asynchronous
// requests.
ccl::status ccl_comp_copy_host(const void* in_buf, void* out_buf, size_t bytes, bool use_nontemporal) {
    if (bytes == 0) return ccl::status::success;
    if (!in_buf) MI_CCL_THROW("in_buf is null");
    if (!out_buf) MI_CCL_THROW("out_buf is null");
    MI_LOG_DEBUG("copy: bytes ", bytes, ", operands: host memory by the copy entry (not looked up), path: cpu",
                 use_nontemporal ? " (non-temporal)" : "");
    const void* ops[2] = {in_buf, out_buf};
    verify_host_word(ops, 2, "copy");
    check(mi_thread_sync(), "mi_thread_sync");
    check(mi_host_copy(out_buf, in_buf, bytes, use_nontemporal ? 1 : 0), "mi_host_copy");
    return ccl::status::success;
}

void ccl_bf16_reduce(const void* in_buf, size_t in_cnt, void* inout_buf, size_t* out_cnt, ccl::reduction op) {
    if (out_cnt != nullptr) *out_cnt = in_cnt;
    if (!builtin_op(op)) MI_CCL_FATAL(unexpected(static_cast<int>(op)));  // bf16.cpp:73, bf16_intrisics.hpp:131
    check(reduce2_sync(in_buf, inout_buf, in_cnt, MI_BFLOAT16, static_cast<int>(op), bf16_flags(mi_bf16_impl())),
          "mi_reduce_sync(bf16)");
}

// bf16.cpp:63-85: the scalar impl's semantics (std::min/max operand order,
// truncation) whatever impl type is in force; a global symbol of bf16.o.
void ccl_bf16_reduce_scalar_impl(const void* in_buf, void* inout_buf, size_t in_count, ccl::reduction op) {
    if (!builtin_op(op)) MI_CCL_FATAL(unexpected(static_cast<int>(op)));  // bf16.cpp:73
    check(reduce2_sync(in_buf, inout_buf, in_count, MI_BFLOAT16, static_cast<int>(op), bf16_flags(ccl_bf16_scalar)),
          "mi_reduce_sync(bf16 scalar)");
}

void ccl_fp16_reduce(const void* in_buf, size_t in_cnt, void* inout_buf, size_t* out_cnt, ccl::reduction op) {
    if (out_cnt != nullptr) *out_cnt = in_cnt;
    unsigned f = 0;
    if (!fp16_flags(mi_fp16_impl(), &f)) return;  // no impl branch taken: nothing computed, no check
    if (!builtin_op(op)) MI_CCL_FATAL(unexpected(static_cast<int>(op)));  // fp16_intrisics.hpp:222-243
    check(reduce2_sync(in_buf, inout_buf, in_cnt, MI_FLOAT16, static_cast<int>(op), f), "mi_reduce_sync(fp16)");
}

// The MPI user ops' reduce (include/mi_ccl_lp_host.hpp, integration/0002):
// bf16_base_op and fp16_base_op (atl_mpi_ctx.cpp:57-63, 87-92) fold MPI's own
// host buffers, so their word is the one a schedule without a stream gives
// (comp.cpp:136-142): a bucket up to the dispatcher's threshold goes to the
// calling thread's CPU with nothing looked up (host_kind -> kHostBySched);
// a larger one is looked up once to pick the GPU's pinned or staged route.
void ccl_bf16_reduce_host(const void* in_buf, size_t in_cnt, void* inout_buf, size_t* out_cnt, ccl::reduction op) {
    const SchedScope scope(true);
    ccl_bf16_reduce(in_buf, in_cnt, inout_buf, out_cnt, op);
}

void ccl_fp16_reduce_host(const void* in_buf, size_t in_cnt, void* inout_buf, size_t* out_cnt, ccl::reduction op) {
    const SchedScope scope(true);
    ccl_fp16_reduce(in_buf, in_cnt, inout_buf, out_cnt, op);
}

// ---- conversions: bf16.cpp:113-169, fp16.cpp:55-61 ------------------------
// ccl_convert_fp32_to_bf16_arrays: non-scalar impls convert (count/16)*16
// elements with the impl's rounding (avx512bf RNE, avx512f truncate) and
// truncate the tail; the scalar impl truncates all.
static unsigned bf16_conv_flags() {
    return mi_bf16_impl() == ccl_bf16_avx512bf ? (MI_F_BF16_RNE | MI_F_BF16_TAIL_TRUNC16) : 0u;
}

void ccl_convert_fp32_to_bf16_arrays(void* fp32_buf, void* bf16_buf, size_t count) {
    check(convert_sync(fp32_buf, MI_FLOAT32, bf16_buf, MI_BFLOAT16, count, bf16_conv_flags()),
          "mi_convert_sync(fp32->bf16)");
}

void ccl_convert_bf16_to_fp32_arrays(void* bf16_buf, float* fp32_buf, size_t count) {
    check(convert_sync(bf16_buf, MI_BFLOAT16, fp32_buf, MI_FLOAT32, count, 0u), "mi_convert_sync(bf16->fp32)");
}

// 16-element forms (bf16.cpp:113-128): avx512bf -> RNE, otherwise truncate
void ccl_convert_fp32_to_bf16(const void* src, void* dst) {
    const unsigned f = mi_bf16_impl() == ccl_bf16_avx512bf ? MI_F_BF16_RNE : 0u;
    check(convert_sync(src, MI_FLOAT32, dst, MI_BFLOAT16, 16, f), "mi_convert_sync");
}

void ccl_convert_bf16_to_fp32(const void* src, void* dst) {
    check(convert_sync(src, MI_BFLOAT16, dst, MI_FLOAT32, 16, 0u), "mi_convert_sync");
}

// 8-element forms (fp16.cpp:55-61): VCVTPS2PH RNE / VCVTPH2PS
void ccl_convert_fp32_to_fp16(const void* src, void* dst) {
    check(convert_sync(src, MI_FLOAT32, dst, MI_FLOAT16, 8, 0u), "mi_convert_sync");
}

void ccl_convert_fp16_to_fp32(const void* src, void* dst) {
    check(convert_sync(src, MI_FLOAT16, dst, MI_FLOAT32, 8, 0u), "mi_convert_sync");
}

// ccl_comp_reduce_regular, comp.cpp:76-121: a global symbol in the reference too
// (not declared in comp.hpp), kept with its mangled name for the link closure
ccl::status ccl_comp_reduce_regular(const void* in_buf, size_t in_count, void* inout_buf, size_t* out_count,
                                       const ccl_datatype& dtype, ccl::reduction reduction,
                                       ccl::reduction_fn reduction_fn, const ccl::fn_context* context) {
    if (reduction == ccl::reduction::custom) {
        run_custom(in_buf, in_count, inout_buf, out_count, dtype, reduction_fn, context);
        return ccl::status::success;
    }
    const int dt = dtype_id(dtype);
    if (mi_dtype_size(dt) == 0) MI_CCL_FATAL(unexpected(dt));  // comp.cpp:113
    if (!builtin_op(reduction) && dt != MI_BFLOAT16 && dt != MI_FLOAT16)
        MI_CCL_FATAL(unexpected(static_cast<int>(reduction)));  // CCL_REDUCE, comp.cpp:56
    TraceRange range("comp_reduce_regular");
    if (dt == MI_BFLOAT16) {
        ccl_bf16_reduce(in_buf, in_count, inout_buf, out_count, reduction);
    } else if (dt == MI_FLOAT16) {
        ccl_fp16_reduce(in_buf, in_count, inout_buf, out_count, reduction);
    } else {
        // CCL_REDUCE: std::min/std::max operand order, no out_count write
        check(reduce2_sync(in_buf, inout_buf, in_count, dt, static_cast<int>(reduction), 0u), "mi_reduce_sync");
    }
    return ccl::status::success;
}

ccl::status ccl_comp_reduce(ccl_sched* sched, const void* in_buf, size_t in_count, void* inout_buf,
                            size_t* out_count, const ccl_datatype& dtype, ccl::reduction reduction,
                            ccl::reduction_fn reduction_fn, const ccl::fn_context* context) {
    if (!in_count) return ccl::status::success;
    const SchedScope scope(sched);  // comp.cpp:136-142: no stream -> host memory, nothing looked up
    return ccl_comp_reduce_regular(in_buf, in_count, inout_buf, out_count, dtype, reduction, reduction_fn, context);
}

// The reference's keep-precision algorithm as written (comp.cpp:214-234):
// acc = fp32(inout); for every input i >= 1: tmp = fp32(in_i), then
// ccl_comp_reduce_regular(tmp -> acc) on float32 (a user callback for custom);
// finally inout = bf16(acc) with the impl's rounding and truncated count%16
// tail.  Used where the fused kernel does not apply: a custom reduction, or
// more inputs than one fused pass takes (MI_MAX_INPUTS).  `tmp` / `acc` are
// the caller's fp32 scratch of in_count floats (host or device), as in the
// reference's signature; host scratch is allocated when they are absent.
static void keep_precision_chain(const void* in_buf, const std::vector<size_t>& offsets, size_t in_count,
                                 void* inout_buf, size_t* out_count, size_t es, ccl::reduction reduction,
                                 ccl::reduction_fn reduction_fn, const ccl::fn_context* context, float* tmp,
                                 float* acc) {
    std::vector<float> htmp, hacc;
    if (!tmp) {
        htmp.resize(in_count);
        tmp = htmp.data();
    }
    if (!acc) {
        hacc.resize(in_count);
        acc = hacc.data();
    }
    const ccl_datatype f32(ccl::datatype::float32, sizeof(float));
    ccl_convert_bf16_to_fp32_arrays(inout_buf, acc, in_count);
    for (size_t i = 1; i < offsets.size(); i++) {
        ccl_convert_bf16_to_fp32_arrays(const_cast<char*>(static_cast<const char*>(in_buf)) + es * offsets[i], tmp,
                                        in_count);
        ccl_comp_reduce_regular(tmp, in_count, acc, out_count, f32, reduction, reduction_fn, context);
    }
    ccl_convert_fp32_to_bf16_arrays(acc, inout_buf, in_count);
}

// ccl_comp_batch_reduce's body, with the issue of each fused fold (`issue(ins,
// k, out, count, dtype, op, flags)`) left to the caller: synchronous
// (mi_reduce_multi_sync) or asynchronous (mi_reduce_start, one request per
// group of <= 16 inputs; the groups of one call land on the calling thread's
// streams in order, so they chain).
template <typename Issue>
static void batch_reduce_body(const void* in_buf, const std::vector<size_t>& offsets, size_t in_count,
                              void* inout_buf, size_t* out_count, const ccl_datatype& dtype,
                              ccl::reduction reduction, ccl::reduction_fn reduction_fn,
                              const ccl::fn_context* context, int bf16_keep_precision_mode, float* tmp,
                              float* acc, Issue&& issue) {
    // Up to MI_MAX_INPUTS inputs the fp32 scratch `tmp`/`acc` of the
    // reference (comp.cpp:210-234) is not needed: the kernel keeps the fp32
    // accumulator in registers and rounds once.
    const size_t es = dtype.size();
    if (bf16_keep_precision_mode) {
        // keep-precision: buffers read as bf16 whatever dtype says; inputs
        // strided by dtype.size() (comp.cpp:214-234)
        const size_t k = std::max<size_t>(offsets.size(), 1);
        if (in_count == 0) return;
        if (reduction != ccl::reduction::custom && !builtin_op(reduction) && k > 1)
            MI_CCL_FATAL(unexpected(static_cast<int>(reduction)));  // the float32 CCL_REDUCE step, comp.cpp:56
        if (reduction == ccl::reduction::custom || k > MI_MAX_INPUTS) {
            keep_precision_chain(in_buf, offsets, in_count, inout_buf, out_count, es, reduction, reduction_fn,
                                 context, tmp, acc);
            return;
        }
        std::vector<const void*> ins(k);
        ins[0] = inout_buf;
        for (size_t i = 1; i < k; i++) ins[i] = static_cast<const char*>(in_buf) + es * offsets[i];
        // acc uses CCL_REDUCE(float) order (std::min/max); final conversion
        // per impl: avx512bf RNE on (count/16)*16 elements + truncated tail,
        // avx512f / scalar truncate all (bf16.cpp:130-149)
        unsigned f = MI_F_ACC_FP32;
        if (mi_bf16_impl() == ccl_bf16_avx512bf) f |= MI_F_BF16_RNE | MI_F_BF16_TAIL_TRUNC16;
        // one input: only the conversions run (no reduce step checks the op)
        issue(ins.data(), (int)k, inout_buf, in_count, MI_BFLOAT16, k == 1 ? MI_OP_SUM : static_cast<int>(reduction), f);
        return;
    }
    if (offsets.size() <= 1 || in_count == 0) return;
    if (reduction == ccl::reduction::custom) {
        for (size_t i = 1; i < offsets.size(); i++)
            ccl_comp_reduce_regular(static_cast<const char*>(in_buf) + es * offsets[i], in_count, inout_buf,
                                    out_count, dtype, reduction, reduction_fn, context);
        return;
    }
    // storage-precision left fold == the reference's chained reduces, which
    // check dtype and op on every call (ccl_comp_reduce_regular)
    const int dt = dtype_id(dtype);
    if (mi_dtype_size(dt) == 0) MI_CCL_FATAL(unexpected(dt));
    unsigned f = 0;
    if (!reduce_semantics(dt, &f)) return;
    if (!builtin_op(reduction)) MI_CCL_FATAL(unexpected(static_cast<int>(reduction)));
    if ((dt == MI_BFLOAT16 || dt == MI_FLOAT16) && out_count) *out_count = in_count;
    size_t next = 1;
    while (next < offsets.size()) {
        const void* ins[MI_MAX_INPUTS];
        int k = 0;
        ins[k++] = inout_buf;
        while (next < offsets.size() && k < MI_MAX_INPUTS)
            ins[k++] = static_cast<const char*>(in_buf) + es * offsets[next++];
        issue(ins, k, inout_buf, in_count, dt, static_cast<int>(reduction), f);
    }
}

ccl::status ccl_comp_batch_reduce(const void* in_buf, const std::vector<size_t>& offsets, size_t in_count,
                                  void* inout_buf, size_t* out_count, const ccl_datatype& dtype,
                                  ccl::reduction reduction, ccl::reduction_fn reduction_fn,
                                  const ccl::fn_context* context, int bf16_keep_precision_mode, float* tmp,
                                  float* acc) {
    TraceRange range("comp_batch_reduce");
    batch_reduce_body(in_buf, offsets, in_count, inout_buf, out_count, dtype, reduction, reduction_fn, context,
                      bf16_keep_precision_mode, tmp, acc,
                      [](const void* const* ins, int k, void* out, size_t n, int dt, int op, unsigned f) {
                          check(fold_sync(ins, k, out, n, dt, op, f), "mi_reduce_multi_sync");
                      });
    return ccl::status::success;
}

const char* ccl_reduction_to_str(ccl::reduction type) { return mi_reduction_to_str(static_cast<int>(type)); }

// ---- asynchronous ccl_comp_reduce (include/mi_ccl_comp_async.hpp) --------
struct ccl_comp_request {
    std::vector<mi_request_t> r;  // empty: completed inside start (empty, custom, fp16 no-op)
    SplitIssued split;            // the first adaptive split among them, if any
};

ccl::status ccl_comp_reduce_start(ccl_sched* sched, const void* in_buf, size_t in_count, void* inout_buf,
                                  size_t* out_count, const ccl_datatype& dtype, ccl::reduction reduction,
                                  ccl::reduction_fn reduction_fn, const ccl::fn_context* context,
                                  ccl_comp_request** req) {
    if (!req) MI_CCL_THROW("null request pointer");
    *req = nullptr;
    const SchedScope scope(sched);
    std::unique_ptr<ccl_comp_request> q(new ccl_comp_request());
    if (in_count) {  // comp.cpp:132-134
        if (reduction == ccl::reduction::custom) {
            run_custom(in_buf, in_count, inout_buf, out_count, dtype, reduction_fn, context);
        } else {
            const int dt = dtype_id(dtype);
            if (mi_dtype_size(dt) == 0) MI_CCL_FATAL(unexpected(dt));
            if (dt == MI_FLOAT16) {
                unsigned f16 = 0;
                if (fp16_flags(mi_fp16_impl(), &f16) && !builtin_op(reduction))
                    MI_CCL_FATAL(unexpected(static_cast<int>(reduction)));
            } else if (!builtin_op(reduction)) {
                MI_CCL_FATAL(unexpected(static_cast<int>(reduction)));
            }
            if ((dt == MI_BFLOAT16 || dt == MI_FLOAT16) && out_count) *out_count = in_count;
            unsigned f = 0;
            if (reduce_semantics(dt, &f)) {
                const void* ins[2] = {inout_buf, in_buf};
                int kind = 0;
                if (host_path(ins, 2, inout_buf, in_count * mi_dtype_size(dt), &kind)) {  // completes here
                    log_route("reduce_start", in_count, dt, 2, kind, "cpu (calling thread; completes in start)");
                    check(host_fold(ins, 2, inout_buf, in_count, dt, static_cast<int>(reduction), f), "host reduce");
                    *req = q.release();
                    return ccl::status::success;
                }
                mi_request_t r = nullptr;
                check(start_fold(ins, 2, inout_buf, in_count, dt, static_cast<int>(reduction), f, &r, &q->split),
                      "mi_reduce_start");
                q->r.push_back(r);
            }
        }
    }
    *req = q.release();
    return ccl::status::success;
}

ccl::status ccl_comp_batch_reduce_start(ccl_sched* sched, const void* in_buf, const std::vector<size_t>& offsets,
                                        size_t in_count, void* inout_buf, size_t* out_count,
                                        const ccl_datatype& dtype, ccl::reduction reduction,
                                        ccl::reduction_fn reduction_fn, const ccl::fn_context* context,
                                        int bf16_keep_precision_mode, ccl_comp_request** req) {
    if (!req) MI_CCL_THROW("null request pointer");
    *req = nullptr;
    const SchedScope scope(sched);
    std::unique_ptr<ccl_comp_request> q(new ccl_comp_request());
    struct Drop {  // on a throw, wait for and release what was already issued
        ccl_comp_request* q;
        ~Drop() {
            if (!q) return;
            for (mi_request_t r : q->r) {
                (void)mi_wait(r);
                (void)mi_request_free(r);
            }
        }
    } drop{q.get()};
    // (a keep-precision chain — custom op, > MI_MAX_INPUTS inputs — completes
    // inside this call, as a custom reduction does in ccl_comp_reduce_start)
    batch_reduce_body(in_buf, offsets, in_count, inout_buf, out_count, dtype, reduction, reduction_fn, context,
                      bf16_keep_precision_mode, nullptr, nullptr,
                      [&](const void* const* ins, int k, void* out, size_t n, int dt, int op, unsigned f) {
                          int kind = 0;
                          if (host_path(ins, k, out, n * mi_dtype_size(dt), &kind)) {  // small host bucket: done here
                              log_route("batch_reduce_start", n, dt, k, kind,
                                        "cpu (calling thread; completes in start)");
                              check(host_fold(ins, k, out, n, dt, op, f), "host reduce");
                              return;
                          }
                          mi_request_t r = nullptr;
                          check(start_fold(ins, k, out, n, dt, op, f, &r, &q->split), "mi_reduce_start");
                          q->r.push_back(r);
                      });
    drop.q = nullptr;
    *req = q.release();
    return ccl::status::success;
}

bool ccl_comp_request_test(ccl_comp_request* req) {
    if (!req) MI_CCL_THROW("null request");
    for (mi_request_t r : req->r) {  // groups complete in issue order
        int done = 0;
        check(mi_test(r, &done), "mi_test");
        if (!done) return false;
    }
    settle_split(req->split);
    return true;
}

void ccl_comp_request_wait(ccl_comp_request* req) {
    if (!req) MI_CCL_THROW("null request");
    for (mi_request_t r : req->r) check(mi_wait(r), "mi_wait");
    settle_split(req->split);
}

// Waits first if the request is still pending: freeing must never leave a
// kernel writing into a buffer its owner already considers free.
void ccl_comp_request_free(ccl_comp_request* req) {
    if (!req) return;
    int rc = 0;
    for (mi_request_t r : req->r) {
        const int w = mi_wait(r);
        if (w && !rc) rc = w;
        (void)mi_request_free(r);
    }
    delete req;
    check(rc, "mi_wait");
}

// The host buffer registry's entry points (include/mi_ccl_comp.h), in both
// builds: inside oneCCL's tree the regular buffer cache calls them
// (integration/0005).  The ranges live in libmi_reduce (mi_host_declare), so
// every classification -- the dispatcher's here and the GPU path's there --
// answers from them without asking HIP; a range is looked up once, when
// declared: device memory is refused, pinned memory stays pinned.
extern "C" {

int mi_ccl_comp_register_host_buffer(const void* ptr, size_t bytes) { return mi_host_declare(ptr, bytes); }

int mi_ccl_comp_unregister_host_buffer(const void* ptr) { return mi_host_undeclare(ptr); }

size_t mi_ccl_comp_pointer_lookups(void) { return mi_pointer_lookups(); }

}  // extern "C"

#ifndef MI_ONECCL_TREE
// ===========================================================================
// C view of the shim (include/mi_ccl_comp.h) — lets tests and ctypes/FFI
// callers drive exactly the code path src/sched would.
// ===========================================================================
namespace {
thread_local std::string t_shim_err;
ccl_datatype mk_dtype(int dt) { return ccl_datatype(static_cast<ccl::datatype>(dt), mi_dtype_size(dt)); }

// The schedule the C view passes (mi_ccl_comp_shim_sched): none, one whose
// collective has no stream (host memory by the schedule's word), or one with
// a stream (operands looked up).  The stream is never dereferenced.
thread_local int t_shim_sched = 0;
thread_local ccl_sched t_sched_host, t_sched_stream;
ccl_sched* shim_sched() {
    if (t_shim_sched == 1) return &t_sched_host;
    if (t_shim_sched == 2) {
        t_sched_stream.coll_param.stream = reinterpret_cast<ccl_stream*>(&t_sched_stream);
        return &t_sched_stream;
    }
    return nullptr;
}
}  // namespace

#define MI_SHIM_GUARD(body)                 \
    try {                                   \
        body;                               \
    } catch (const std::exception& e) {     \
        t_shim_err = e.what();              \
        return -1;                          \
    }

extern "C" {

int mi_ccl_comp_reduce(const void* in_buf, size_t in_count, void* inout_buf, size_t* out_count, int dtype, int op) {
    MI_SHIM_GUARD(return (int)ccl_comp_reduce(shim_sched(), in_buf, in_count, inout_buf, out_count, mk_dtype(dtype),
                                              static_cast<ccl::reduction>(op), nullptr, nullptr));
}

int mi_ccl_comp_reduce_custom(const void* in_buf, size_t in_count, void* inout_buf, size_t* out_count, int dtype,
                              mi_ccl_reduction_fn fn) {
    MI_SHIM_GUARD(return (int)ccl_comp_reduce(shim_sched(), in_buf, in_count, inout_buf, out_count, mk_dtype(dtype),
                                              ccl::reduction::custom, reinterpret_cast<ccl::reduction_fn>(fn),
                                              nullptr));
}

int mi_ccl_comp_batch_reduce(const void* in_buf, const size_t* offsets, size_t n_offsets, size_t in_count,
                             void* inout_buf, size_t* out_count, int dtype, int op, int bf16_keep_precision_mode) {
    MI_SHIM_GUARD({
        std::vector<size_t> offs(offsets, offsets + n_offsets);
        return (int)ccl_comp_batch_reduce(in_buf, offs, in_count, inout_buf, out_count, mk_dtype(dtype),
                                          static_cast<ccl::reduction>(op), nullptr, nullptr,
                                          bf16_keep_precision_mode, nullptr, nullptr);
    });
}

int mi_ccl_comp_batch_reduce_custom(const void* in_buf, const size_t* offsets, size_t n_offsets, size_t in_count,
                                    void* inout_buf, size_t* out_count, int dtype, int bf16_keep_precision_mode,
                                    mi_ccl_reduction_fn fn) {
    MI_SHIM_GUARD({
        std::vector<size_t> offs(offsets, offsets + n_offsets);
        return (int)ccl_comp_batch_reduce(in_buf, offs, in_count, inout_buf, out_count, mk_dtype(dtype),
                                          ccl::reduction::custom, reinterpret_cast<ccl::reduction_fn>(fn), nullptr,
                                          bf16_keep_precision_mode, nullptr, nullptr);
    });
}

int mi_ccl_comp_copy(const void* in_buf, void* out_buf, size_t bytes, int use_nontemporal) {
    MI_SHIM_GUARD(return (int)ccl_comp_copy(in_buf, out_buf, bytes, use_nontemporal != 0));
}

int mi_ccl_comp_copy_host(const void* in_buf, void* out_buf, size_t bytes, int use_nontemporal) {
    MI_SHIM_GUARD(return (int)ccl_comp_copy_host(in_buf, out_buf, bytes, use_nontemporal != 0));
}

int mi_ccl_bf16_reduce(const void* in_buf, size_t in_cnt, void* inout_buf, size_t* out_cnt, int op) {
    MI_SHIM_GUARD({
        ccl_bf16_reduce(in_buf, in_cnt, inout_buf, out_cnt, static_cast<ccl::reduction>(op));
        return 0;
    });
}

int mi_ccl_fp16_reduce(const void* in_buf, size_t in_cnt, void* inout_buf, size_t* out_cnt, int op) {
    MI_SHIM_GUARD({
        ccl_fp16_reduce(in_buf, in_cnt, inout_buf, out_cnt, static_cast<ccl::reduction>(op));
        return 0;
    });
}

int mi_ccl_bf16_reduce_host(const void* in_buf, size_t in_cnt, void* inout_buf, size_t* out_cnt, int op) {
    MI_SHIM_GUARD({
        ccl_bf16_reduce_host(in_buf, in_cnt, inout_buf, out_cnt, static_cast<ccl::reduction>(op));
        return 0;
    });
}

int mi_ccl_fp16_reduce_host(const void* in_buf, size_t in_cnt, void* inout_buf, size_t* out_cnt, int op) {
    MI_SHIM_GUARD({
        ccl_fp16_reduce_host(in_buf, in_cnt, inout_buf, out_cnt, static_cast<ccl::reduction>(op));
        return 0;
    });
}

int mi_ccl_convert_fp32_to_bf16_arrays(void* fp32_buf, void* bf16_buf, size_t count) {
    MI_SHIM_GUARD({
        ccl_convert_fp32_to_bf16_arrays(fp32_buf, bf16_buf, count);
        return 0;
    });
}

int mi_ccl_convert_bf16_to_fp32_arrays(void* bf16_buf, float* fp32_buf, size_t count) {
    MI_SHIM_GUARD({
        ccl_convert_bf16_to_fp32_arrays(bf16_buf, fp32_buf, count);
        return 0;
    });
}

int mi_ccl_convert_fp32_to_fp16(const void* src, void* dst) {
    MI_SHIM_GUARD({
        ccl_convert_fp32_to_fp16(src, dst);
        return 0;
    });
}

int mi_ccl_convert_fp16_to_fp32(const void* src, void* dst) {
    MI_SHIM_GUARD({
        ccl_convert_fp16_to_fp32(src, dst);
        return 0;
    });
}

int mi_ccl_comp_reduce_start(const void* in_buf, size_t in_count, void* inout_buf, size_t* out_count, int dtype,
                             int op, mi_ccl_reduction_fn fn, struct ccl_comp_request** req) {
    MI_SHIM_GUARD(return (int)ccl_comp_reduce_start(shim_sched(), in_buf, in_count, inout_buf, out_count, mk_dtype(dtype),
                                                    static_cast<ccl::reduction>(op),
                                                    reinterpret_cast<ccl::reduction_fn>(fn), nullptr, req));
}

int mi_ccl_comp_batch_reduce_start(const void* in_buf, const size_t* offsets, size_t n_offsets, size_t in_count,
                                   void* inout_buf, size_t* out_count, int dtype, int op,
                                   int bf16_keep_precision_mode, struct ccl_comp_request** req) {
    MI_SHIM_GUARD({
        std::vector<size_t> offs(offsets, offsets + n_offsets);
        return (int)ccl_comp_batch_reduce_start(shim_sched(), in_buf, offs, in_count, inout_buf, out_count, mk_dtype(dtype),
                                                static_cast<ccl::reduction>(op), nullptr, nullptr,
                                                bf16_keep_precision_mode, req);
    });
}

int mi_ccl_comp_request_test(struct ccl_comp_request* req, int* done) {
    MI_SHIM_GUARD({
        if (!done) throw ccl::exception("null done pointer");
        *done = ccl_comp_request_test(req) ? 1 : 0;
        return 0;
    });
}

int mi_ccl_comp_request_wait(struct ccl_comp_request* req) {
    MI_SHIM_GUARD({
        ccl_comp_request_wait(req);
        return 0;
    });
}

int mi_ccl_comp_request_free(struct ccl_comp_request* req) {
    MI_SHIM_GUARD({
        ccl_comp_request_free(req);
        return 0;
    });
}

const char* mi_ccl_reduction_to_str(int op) { return ccl_reduction_to_str(static_cast<ccl::reduction>(op)); }

int mi_ccl_comp_shim_sched(int mode) {
    if (mode < 0 || mode > 2) return (int)MI_E_INVALID;
    const int prev = t_shim_sched;
    t_shim_sched = mode;
    return prev;
}

int mi_ccl_env_reload(void) {
    MI_SHIM_GUARD({
        std::lock_guard<std::mutex> g(g_env_mu);
        parse_env_locked();
        shard_env_reload();
        t_split = SplitShare();  // the calling thread's adapted shares start over
        return 0;
    });
}

double mi_ccl_comp_split_share(int pinned) { return t_split.share[pinned ? 1 : 0]; }

int mi_ccl_comp_split_take_gpu_alone(int pinned) { return take_gpu_alone(pinned ? 1 : 0) ? 1 : 0; }

int mi_ccl_comp_split_feed(int pinned, size_t count, size_t head, double t_head, double t_tail) {
    MI_SHIM_GUARD({
        const int pk = pinned ? 1 : 0;
        const HostMax m = mi_host_max();
        double& cur = t_split.share[pk];
        if (cur < 0) cur = pk ? m.share_pinned : m.share;  // as coop_fold starts a thread's share
        if (head == 0) gpu_alone_timed(pk, count, t_tail);
        else split_update(pk, count, head, t_head, t_tail);
        return 0;
    });
}

int mi_ccl_comp_host_max(size_t* pageable, size_t* pinned, double* share, double* share_pinned) {
    MI_SHIM_GUARD({
        const HostMax m = mi_host_max();
        if (pageable) *pageable = m.pageable;
        if (pinned) *pinned = m.pinned;
        if (share) *share = m.share;
        if (share_pinned) *share_pinned = m.share_pinned;
        return 0;
    });
}

int mi_ccl_comp_host_workers(void) { return host_workers(); }

double mi_ccl_comp_split_gpu_rate(int pinned, unsigned* gpu_left) {
    if (gpu_left) *gpu_left = t_split.gpu_left[pinned ? 1 : 0];
    return t_split.gpu_rate[pinned ? 1 : 0];
}

int mi_ccl_comp_device(void) { return mi_comp_device(); }

int mi_ccl_impl_types(int* bf16_impl, int* fp16_impl) {
    MI_SHIM_GUARD({
        const MiEnv& e = env();
        if (bf16_impl) *bf16_impl = (int)e.bf16;
        if (fp16_impl) *fp16_impl = (int)e.fp16;
        return 0;
    });
}

const char* mi_ccl_last_error(void) { return t_shim_err.c_str(); }

}  // extern "C"
#endif  // !MI_ONECCL_TREE
