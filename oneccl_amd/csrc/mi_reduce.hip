// mi_reduce.hip — libmi_reduce.so: the C ABI of include/mi_reduce.h.
//
// Host half of the MI355X-native local reduction: variant canonicalisation,
// kernel selection, launch geometry, per-thread streams and the
// host-operand staging pipeline.  Kernels: reduce_kernels.hpp.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <deque>
#include <map>
#include <memory>
#include <thread>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <pthread.h>
#include <sched.h>
#include <stdexcept>
#include <string>
#include <unistd.h>
#include <vector>

#include "../../include/mi_reduce.h"
#include "reduce_kernels.hpp"

using namespace mi;

namespace {

// ---------------------------------------------------------------------------
// errors
// ---------------------------------------------------------------------------
thread_local std::string g_last_error;

int fail(int code, const char* what) {
    g_last_error = what;
    return code;
}
int hip_fail(hipError_t e, const char* what) {
    g_last_error = std::string(what) + ": " + hipGetErrorString(e);
    return (int)e;
}
#define MI_HIP(call)                                   \
    do {                                               \
        hipError_t e_ = (call);                        \
        if (e_ != hipSuccess) return hip_fail(e_, #call); \
    } while (0)

// ---------------------------------------------------------------------------
// launch configuration
// ---------------------------------------------------------------------------
constexpr int kUnroll = 4;  // 16-byte vectors per lane per input per tile
constexpr int kMem = 3;     // non-temporal loads and stores (sweep: profiles/round1_sweep.jsonl)

std::atomic<int> g_max_blocks{-1};  // -1 = not yet read from env; 0 = no cap
std::atomic<int> g_host_mode{-1};   // -1 = not yet read from env

std::atomic<int> g_sync_mode{-1};  // -1 = not yet read from env

int sync_mode() {
    int v = g_sync_mode.load(std::memory_order_relaxed);
    if (v < 0) {
        const char* s = getenv("MI_REDUCE_SYNC");
        v = (s && strcmp(s, "spin") == 0) ? MI_SYNC_SPIN : MI_SYNC_BLOCK;
        g_sync_mode.store(v, std::memory_order_relaxed);
    }
    return v;
}

// Wait for a stream: spin on hipStreamQuery (lowest latency for the
// synchronous src/comp contract) or the runtime's blocking wait.
hipError_t wait_stream(hipStream_t s) {
    if (sync_mode() == MI_SYNC_BLOCK) return hipStreamSynchronize(s);
    for (unsigned spins = 0;; spins++) {
        const hipError_t e = hipStreamQuery(s);
        if (e != hipErrorNotReady) return e;
        if (spins > 4096) sched_yield();
    }
}

int host_mode() {
    int v = g_host_mode.load(std::memory_order_relaxed);
    if (v < 0) {
        const char* s = getenv("MI_REDUCE_HOST_MODE");
        v = (s && strcmp(s, "staged") == 0) ? MI_HOST_STAGED : MI_HOST_AUTO;
        g_host_mode.store(v, std::memory_order_relaxed);
    }
    return v;
}

// Operands whose misalignments differ take the vector kernels (1, default)
// or the element loop (0).  Env MI_REDUCE_UNALIGNED=0 selects the loop.
std::atomic<int> g_unaligned{-1};  // -1 = not yet read from env

int unaligned_vectors() {
    int v = g_unaligned.load(std::memory_order_relaxed);
    if (v < 0) {
        const char* s = getenv("MI_REDUCE_UNALIGNED");
        v = (s && strcmp(s, "0") == 0) ? 0 : 1;
        g_unaligned.store(v, std::memory_order_relaxed);
    }
    return v;
}

int max_blocks() {
    int v = g_max_blocks.load(std::memory_order_relaxed);
    if (v < 0) {
        const char* s = getenv("MI_REDUCE_MAX_BLOCKS");
        v = s ? std::max(0, atoi(s)) : 0;
        g_max_blocks.store(v, std::memory_order_relaxed);
    }
    return v;
}

size_t dtype_size(int dt) {
    switch (dt) {
        case MI_INT8: case MI_UINT8: return 1;
        case MI_INT16: case MI_UINT16: case MI_FLOAT16: case MI_BFLOAT16: return 2;
        case MI_INT32: case MI_UINT32: case MI_FLOAT32: return 4;
        case MI_INT64: case MI_UINT64: case MI_FLOAT64: return 8;
        default: return 0;
    }
}

// Keep only the variant bits that change results for (dtype, op, k).
unsigned canon_flags(int dt, int op, unsigned f, int k) {
    const bool mm = (op == MI_OP_MIN || op == MI_OP_MAX);
    switch (dt) {
        case MI_FLOAT32:
        case MI_FLOAT64: return mm ? (f & V_INOUT_FIRST) : 0u;
        case MI_FLOAT16: {
            unsigned v = (mm ? (f & (V_INOUT_FIRST | V_FP16_NATIVE)) : 0u) | (f & V_ACC_FP32);
            // One step rounds once either way, but a sum/prod step with fp32
            // accumulation takes the accumulator's NaN first (CCL_REDUCE(float)
            // order), a storage-precision step `in`'s: only min/max (and k = 1,
            // no step) may drop the bit.
            if (k <= 1 || (k == 2 && mm)) v &= ~V_ACC_FP32;
            return v;
        }
        case MI_BFLOAT16: {
            unsigned v = (mm ? (f & V_INOUT_FIRST) : 0u) | (f & (V_BF16_RNE | V_ACC_FP32 | V_TAIL_TRUNC));
            if (!((v & V_ACC_FP32) && (v & V_BF16_RNE))) v &= ~V_TAIL_TRUNC;
            if (k == 2 && mm && !(v & V_TAIL_TRUNC)) v &= ~V_ACC_FP32;  // see fp16 above
            return v;
        }
        default: return 0u;  // integers: no variants
    }
}

// ---------------------------------------------------------------------------
// kernel table
// ---------------------------------------------------------------------------
typedef hipError_t (*LaunchFn)(dim3, hipStream_t, const KArgs&);
typedef hipError_t (*LaunchFanFn)(hipStream_t, const KArgs&, unsigned lds);
typedef hipError_t (*Launch2Fn)(dim3, hipStream_t, const R2Args&, unsigned lds);
typedef hipError_t (*LaunchBFn)(dim3, hipStream_t, const BArgs&, unsigned lds);

// Lean 2-input kernel shape: one 16-byte vector per lane, one-wave (64-lane)
// tiles, 21 waves resident per CU (capped by idle LDS, as the fan-in below).
// In place, as ccl_comp_reduce runs it, that took 0.484 ms per GiB of fp32
// against 0.508 for round 2's 1024-lane tiles at 32 waves per CU (-4.8 %;
// int32 -3.5 %, bf16 -4.1 %, fp16 -3.5 %; tools/occupancy_sweep.hip r2ab,
// profiles/round3_occupancy/).  Round 1's sweeps had stopped at 256 lanes.
// (Round 3 sized that reservation for 24 waves; gfx950 allocates LDS in
// granules of 1/128 of the CU's LDS, so it held 21, which is what was
// measured: tools/residency_probe.hip, profiles/round4_host/.  The residencies
// below are the achieved ones, and wave_cap_lds reserves whole granules.)
constexpr int kB2 = 64;
constexpr int kU2 = 1;
constexpr int kLeanWavesPerCU = 21;
// Buffer-addressed fan-in, one tile per block.  One-wave (64-lane) tiles,
// with the waves resident on a CU capped by LDS that no instruction touches
// (a block that reserves 1/W of a CU's LDS leaves room for W of them).  Each
// wave holds K one-KiB loads in flight, and the fan-in streams fastest with
// ~50-100 KiB of loads in flight per CU: at the library's former 1024-lane
// tiles and 32 waves per CU, 8 inputs kept 256 KiB per CU in flight and ran
// 10-11 % slower (tools/occupancy_sweep.hip, profiles/round3_occupancy/:
// 8 inputs 1.65 -> 1.47 ms per GiB, 6 inputs -10.7 %, 4 inputs -4.7 %,
// 16 inputs -7.4 %).  8- and 16-bit integers fold packed on dwords
// (pk_op4), so no type unpacks more than 8 elements per vector.
constexpr int kFanBlock = 64;
// (achieved residencies of round 3's caps 16 / 12 / 10 / 8 / 6, see above)
int fan_waves_per_cu(int k) { return k <= 4 ? 16 : k <= 6 ? 11 : k <= 8 ? 9 : k <= 12 ? 8 : 5; }
constexpr int kConvWavesPerCU = 21;  // the array conversions (achieved residency of round 3's cap of 24)

// mi_set_residency overrides (tuning, per k as mi_get_residency: 0 the
// conversions, 2 the 2-input kernel, 1 and 3..16 the fan-in); 0 = the plan
std::atomic<int> g_residency_override[MI_MAX_INPUTS + 1];

int planned_waves(int k) {
    const int o = g_residency_override[k].load(std::memory_order_relaxed);
    if (o > 0) return o;
    return k == 2 ? kLeanWavesPerCU : k == 0 ? kConvWavesPerCU : fan_waves_per_cu(k);
}

// LDS bytes per CU of each device (read once per device; 0 = unknown: no
// cap).  Lock-free: every launch reads it, from any number of threads.
constexpr int kMaxDevices = 64;
std::atomic<int> g_lds_per_cu[kMaxDevices];  // 0 until read; read value + 1 after

unsigned lds_per_cu(int device) {
    if (device < 0 || device >= kMaxDevices) return 0;
    int v = g_lds_per_cu[device].load(std::memory_order_relaxed);
    if (v == 0) {
        int a = 0;
        if (hipDeviceGetAttribute(&a, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, device) != hipSuccess)
            a = 0;
        v = std::max(a, 0) + 1;
        g_lds_per_cu[device].store(v, std::memory_order_relaxed);
    }
    return (unsigned)(v - 1);
}

// MI_REDUCE_WAVE_CAP=0 launches the one-wave kernels without the LDS
// reservation (every wave slot usable; the reservation also keeps kernels
// that need LDS, on other streams, off the CUs while a reduce runs there).
// Read once.  Uncapped, the 2-input kernel keeps most of its gain (-4.4 %
// against -4.8 %), the fan-in about half (8 inputs -5.5 % against -11 %).
bool wave_cap_enabled() {
    static const bool on = [] {
        const char* e = getenv("MI_REDUCE_WAVE_CAP");
        return !(e && atoi(e) == 0);
    }();
    return on;
}

// LDS is allocated to a workgroup in granules of 1/128 of a CU's LDS
// (gfx950: 1280 B of 160 KiB; 512 B of 64 KiB on gfx942), so a workgroup
// reserving b bytes holds ceil(b / granule) granules and a CU holds
// floor(128 / that) such workgroups.  Measured with tools/residency_probe.hip
// over 11 sizes (profiles/round4_host/residency_probe_run1.jsonl): 6826 B
// (160 KiB / 24) held 21 waves, 16384 B (/ 10) held 9.  The HIP occupancy
// API (hipOccupancyMaxActiveBlocksPerMultiprocessor) ignores the granule.
unsigned lds_granule(unsigned per_cu) { return per_cu / 128; }

// Dynamic LDS (never touched) for a one-wave block so that `waves` of them
// fit on a CU: whole granules, floor(128 / waves) of them.  Exactly `waves`
// fit when waves is one of the residencies granules allow (floor(128 / m):
// 32, 25, 21, 18, 16, 14, 12, 11, 10, 9, 8, ... 5, 4), as every cap here is.
unsigned wave_cap_bytes(unsigned per_cu, int waves) {
    if (per_cu == 0 || waves <= 0) return 0;
    const unsigned g = lds_granule(per_cu);
    if (g == 0) return per_cu / (unsigned)waves;
    return std::max(1u, 128u / (unsigned)waves) * g;
}

unsigned wave_cap_lds(hipStream_t s, int waves) {
    if (!wave_cap_enabled()) return 0;
    int dev = -1;
    if (!s || hipStreamGetDevice(s, &dev) != hipSuccess) (void)hipGetDevice(&dev);
    return wave_cap_bytes(lds_per_cu(dev), waves);
}

template <typename Tag, int OP, unsigned V>
hipError_t launch_general(dim3 grid, hipStream_t s, const KArgs& a) {
    hipLaunchKernelGGL((reduce_kernel<Tag, OP, V, 0, kUnroll, kMem>), grid, dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

template <typename Tag, int OP, unsigned V>
hipError_t launch_lean(dim3 grid, hipStream_t s, const R2Args& a, unsigned lds) {
    hipLaunchKernelGGL((reduce2_kernel<Tag, OP, V, kU2, kB2>), grid, dim3(kB2), lds, s, a);
    return hipGetLastError();
}

template <typename Tag, int OP, unsigned V>
hipError_t launch_batch(dim3 grid, hipStream_t s, const BArgs& a, unsigned lds) {
    hipLaunchKernelGGL((reduce2_batch_kernel<Tag, OP, V, kU2, kB2>), grid, dim3(kB2), lds, s, a);
    return hipGetLastError();
}

template <typename Tag, int OP, unsigned V>
hipError_t launch_fan(hipStream_t s, const KArgs& a, unsigned lds) {
    constexpr int B = kFanBlock;
    const uint64_t blocks = std::max<uint64_t>((a.nvec + B - 1) / B, 1);
    if (blocks > 0x7FFFFFFFull) return hipErrorInvalidConfiguration;
    if (a.k <= 8)
        hipLaunchKernelGGL((fan_kernel<Tag, OP, V, B, 8>), dim3((unsigned)blocks), dim3(B), lds, s, a);
    else
        hipLaunchKernelGGL((fan_kernel<Tag, OP, V, B, kMaxInputs>), dim3((unsigned)blocks), dim3(B), lds, s, a);
    return hipGetLastError();
}

// general: any K (runtime), grid-stride, also the element loop for operands
// with different misalignments; lean: K = 2 with a common alignment; fan:
// any other K with a common alignment
struct Kern {
    LaunchFn general = nullptr;
    Launch2Fn lean = nullptr;
    LaunchFanFn fan = nullptr;
    LaunchBFn batch = nullptr;
};

template <typename Tag, int OP, unsigned V>
constexpr bool valid_v() {
    constexpr bool mm = (OP == OP_MIN || OP == OP_MAX);
    if constexpr (!Tr<Tag>::fp) return V == 0;
    if constexpr (!Tr<Tag>::lp) return V == 0 || (mm && V == V_INOUT_FIRST);
    if ((V & V_INOUT_FIRST) && !mm) return false;
    if ((V & V_FP16_NATIVE) && !(std::is_same<Tag, fp16_tag>::value && mm)) return false;
    if constexpr (std::is_same<Tag, fp16_tag>::value) return (V & (V_BF16_RNE | V_TAIL_TRUNC)) == 0;
    if ((V & V_TAIL_TRUNC) && !((V & V_ACC_FP32) && (V & V_BF16_RNE))) return false;
    return true;
}

template <typename Tag, int OP, unsigned V>
Kern entry() {
    Kern k;
    if constexpr (valid_v<Tag, OP, V>()) {
        k.general = &launch_general<Tag, OP, V>;
        k.lean = &launch_lean<Tag, OP, V>;
        k.fan = &launch_fan<Tag, OP, V>;
        k.batch = &launch_batch<Tag, OP, V>;
    }
    return k;
}

template <typename Tag, int OP>
Kern pick_v(unsigned v) {
    switch (v) {
#define MI_V(n) case n: return entry<Tag, OP, n##u>();
        MI_V(0) MI_V(1) MI_V(2) MI_V(3) MI_V(4) MI_V(5) MI_V(6) MI_V(7)
        MI_V(8) MI_V(9) MI_V(10) MI_V(11) MI_V(12) MI_V(13) MI_V(14) MI_V(15)
        MI_V(16) MI_V(17) MI_V(20) MI_V(21)  // V_FP16_NATIVE: fp16 min/max only (valid_v)
#undef MI_V
        default: return Kern();
    }
}

template <typename Tag>
Kern pick_op(int op, unsigned v) {
    switch (op) {
        case MI_OP_SUM: return pick_v<Tag, OP_SUM>(v);
        case MI_OP_PROD: return pick_v<Tag, OP_PROD>(v);
        case MI_OP_MIN: return pick_v<Tag, OP_MIN>(v);
        case MI_OP_MAX: return pick_v<Tag, OP_MAX>(v);
        default: return Kern();
    }
}

Kern pick(int dt, int op, unsigned v) {
    switch (dt) {
        case MI_INT8: return pick_op<int8_t>(op, v);
        case MI_UINT8: return pick_op<uint8_t>(op, v);
        case MI_INT16: return pick_op<int16_t>(op, v);
        case MI_UINT16: return pick_op<uint16_t>(op, v);
        case MI_INT32: return pick_op<int32_t>(op, v);
        case MI_UINT32: return pick_op<uint32_t>(op, v);
        case MI_INT64: return pick_op<int64_t>(op, v);
        case MI_UINT64: return pick_op<uint64_t>(op, v);
        case MI_FLOAT16: return pick_op<fp16_tag>(op, v);
        case MI_FLOAT32: return pick_op<float>(op, v);
        case MI_FLOAT64: return pick_op<double>(op, v);
        case MI_BFLOAT16: return pick_op<bf16_tag>(op, v);
        default: return Kern();
    }
}

// ---------------------------------------------------------------------------
// pointer classification
// ---------------------------------------------------------------------------
enum PtrKind { PK_DEVICE = 0, PK_PINNED = 1, PK_PAGEABLE = 2 };

// ---- declared host ranges (mi_host_declare) --------------------------------
// HIP's pointer lookup takes a runtime-wide lock, and on pageable memory it
// serialises concurrent callers: 0.07 us alone, 9.5 us per call at 16 threads
// (profiles/round3_host/pointer_kind_probe_run2.jsonl).  A caller that owns
// long-lived host buffers (oneCCL's regular_buffer_cache,
// src/sched/buffer/buffer_cache.cpp:87-123) declares them once; classify()
// answers for an operand lying wholly inside a declared range without asking
// HIP.  Each range is looked up once, when declared, and keeps the kind found
// then (device memory is refused), so a pinned range keeps its zero-copy path.
//
// Readers take no lock.  The ranges are an immutable sorted snapshot behind
// an atomic pointer; a writer publishes a new one and frees the old one after
// a grace period: every reader thread owns a slot whose counter is odd while
// it reads, and the writer waits until each slot it saw odd has moved on.  A
// reader that entered after the publication loads the new snapshot (both
// sides are sequentially consistent), so nothing it can hold is freed.
struct HostRange {
    uintptr_t lo, hi;    // [lo, hi)
    PtrKind kind;        // PK_PINNED or PK_PAGEABLE
    intptr_t dev_delta;  // pinned: device-visible address - host address
};
struct RangeSnap {
    std::vector<HostRange> r;  // sorted by lo, disjoint
};

std::mutex g_rng_mu;  // writers; readers without a slot
std::atomic<const RangeSnap*> g_rng{nullptr};
std::atomic<int> g_rng_n{0};  // ranges declared: 0 lets classify skip all of this

constexpr int kReaderSlots = 256;
struct alignas(64) ReaderSlot {
    std::atomic<uint64_t> seq{0};  // odd: reading a snapshot
    std::atomic<bool> used{false};
};
ReaderSlot g_readers[kReaderSlots];

struct ReaderSlotRef {  // the calling thread's slot, released when it exits
    int idx = -2;       // -2: not taken yet, -1: none free (read under the mutex)
    ~ReaderSlotRef() {
        if (idx >= 0) g_readers[idx].used.store(false, std::memory_order_release);
        // a read later in this thread's exit (another thread_local's
        // destructor) takes the mutex path: the slot may be another thread's now
        idx = -1;
    }
};
thread_local ReaderSlotRef t_reader;
thread_local size_t t_lookups = 0;  // HIP pointer lookups this thread made (mi_pointer_lookups)

ReaderSlot* reader_slot() {
    if (t_reader.idx == -2) {
        t_reader.idx = -1;
        for (int i = 0; i < kReaderSlots; i++) {
            bool f = false;
            // seq_cst, as the writer's load of `used`: a writer that published
            // before this thread's first read either sees the slot taken or
            // is seen by the read (it then loads the new snapshot)
            if (!g_readers[i].used.load(std::memory_order_relaxed) &&
                g_readers[i].used.compare_exchange_strong(f, true, std::memory_order_seq_cst)) {
                t_reader.idx = i;
                break;
            }
        }
    }
    return t_reader.idx >= 0 ? &g_readers[t_reader.idx] : nullptr;
}

bool find_range(const RangeSnap* s, uintptr_t a, size_t bytes, HostRange* out) {
    if (!s) return false;
    auto it = std::upper_bound(s->r.begin(), s->r.end(), a, [](uintptr_t x, const HostRange& r) { return x < r.lo; });
    if (it == s->r.begin()) return false;
    --it;
    if (a < it->lo || a >= it->hi || bytes > it->hi - a) return false;
    *out = *it;
    return true;
}

// [p, p + bytes) wholly inside a declared range: its kind (and, pinned, the
// device-visible address of p)
bool declared(const void* p, size_t bytes, PtrKind* kind, void** devptr) {
    if (g_rng_n.load(std::memory_order_acquire) == 0) return false;
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    HostRange r;
    bool hit;
    if (ReaderSlot* s = reader_slot()) {
        s->seq.fetch_add(1, std::memory_order_seq_cst);  // odd: inside
        hit = find_range(g_rng.load(std::memory_order_seq_cst), a, bytes, &r);
        s->seq.fetch_add(1, std::memory_order_release);
    } else {
        std::lock_guard<std::mutex> lk(g_rng_mu);
        hit = find_range(g_rng.load(std::memory_order_relaxed), a, bytes, &r);
    }
    if (!hit) return false;
    *kind = r.kind;
    if (devptr && r.kind == PK_PINNED) *devptr = reinterpret_cast<void*>(a + r.dev_delta);
    return true;
}

// Writers, under g_rng_mu: publish `next`, wait out the readers that may still
// hold the snapshot it replaces, free that one.
void publish_ranges(RangeSnap* next) {
    const RangeSnap* old = g_rng.exchange(next, std::memory_order_seq_cst);
    for (ReaderSlot& s : g_readers) {
        if (!s.used.load(std::memory_order_seq_cst)) continue;
        const uint64_t v = s.seq.load(std::memory_order_seq_cst);
        if (!(v & 1)) continue;
        while (s.seq.load(std::memory_order_acquire) == v) std::this_thread::yield();
    }
    delete old;
}

// `devptr` (optional): the device-visible address of a pinned host pointer.
// `bytes`: the extent of the operand at p (for the declared ranges).
PtrKind classify_hip(const void* p, int* dev, void** devptr);
bool pinned_extent(uintptr_t a, intptr_t delta, uintptr_t* lo, uintptr_t* hi);

PtrKind classify(const void* p, int* dev, void** devptr = nullptr, size_t bytes = 1) {
    PtrKind dk;
    if (declared(p, bytes ? bytes : 1, &dk, devptr)) return dk;
    void* dv = const_cast<void*>(p);
    const PtrKind k = classify_hip(p, dev, &dv);
    if (k == PK_PINNED && bytes > 1) {
        // HIP answers for the first byte only.  The zero-copy kernel reads the
        // whole operand in place, so a pinned operand must lie inside one
        // pinned allocation (as mi_host_declare requires of a pinned range):
        // one that runs on into pageable memory is staged instead of faulting.
        const uintptr_t a = reinterpret_cast<uintptr_t>(p);
        const intptr_t delta = (intptr_t)(reinterpret_cast<uintptr_t>(dv) - a);
        uintptr_t lo = 0, hi = 0;
        if (!pinned_extent(a, delta, &lo, &hi) || bytes > hi - a) return PK_PAGEABLE;
    }
    if (devptr) *devptr = dv;
    return k;
}

// HIP's answer (one runtime lookup, counted for mi_pointer_lookups)
PtrKind classify_hip(const void* p, int* dev, void** devptr) {
    t_lookups++;
    hipPointerAttribute_t at;
    memset(&at, 0, sizeof(at));
    hipError_t e = hipPointerGetAttributes(&at, p);
    if (e != hipSuccess) {
        (void)hipGetLastError();  // clear the sticky "invalid value" for unregistered memory
        return PK_PAGEABLE;
    }
    if (at.type == hipMemoryTypeDevice || at.type == hipMemoryTypeManaged) {
        *dev = at.device;
        return PK_DEVICE;
    }
    if (at.type == hipMemoryTypeHost) {
        if (devptr) *devptr = at.devicePointer ? at.devicePointer : const_cast<void*>(p);
        return PK_PINNED;
    }
    return PK_PAGEABLE;
}

// A kernel may only touch device memory or pinned host memory: a pageable
// host pointer reaching a device entry point would fault the GPU, so it is
// refused here instead (the *_sync entry points stage pageable memory).
int require_gpu_visible(const void* p, size_t bytes = 1) {
    int dev = -1;
    if (classify(p, &dev, nullptr, bytes) == PK_PAGEABLE)
        return fail(MI_E_INVALID, "pageable host memory passed to a device entry point (use the *_sync form)");
    return 0;
}

// ---------------------------------------------------------------------------
// the asynchronous core: out = fold(inputs[0..k-1]) on device pointers
// ---------------------------------------------------------------------------
// `visible`: the caller already knows every operand is device memory or a
// device-visible pinned address (reduce_issue classified them, or made them:
// staging and bounce buffers), so they are not looked up again.
int launch_reduce(const void* const* inputs, int k, void* out, size_t count, int dt, int op,
                  unsigned flags, hipStream_t stream, bool visible = false) {
    const size_t es = dtype_size(dt);
    if (!es) return fail(MI_E_INVALID, "unknown datatype");
    if (op < MI_OP_SUM || op > MI_OP_MAX) return fail(MI_E_INVALID, "unsupported reduction (device path: sum/prod/min/max)");
    if (k < 1 || k > MI_MAX_INPUTS) return fail(MI_E_INVALID, "input count out of range [1,16]");
    if (count == 0) return 0;
    if (!out) return fail(MI_E_INVALID, "null output");
    for (int i = 0; i < k; i++)
        if (!inputs[i]) return fail(MI_E_INVALID, "null input");

    if (!visible) {
        for (int i = 0; i < k; i++)
            if (int rc = require_gpu_visible(inputs[i], count * es)) return rc;
        if (int rc = require_gpu_visible(out, count * es)) return rc;
    }

    const unsigned v = canon_flags(dt, op, flags, k);
    if (k == 1 && !(v & V_ACC_FP32)) {  // nothing to combine: result is inputs[0]
        if (out != inputs[0]) MI_HIP(hipMemcpyAsync(out, inputs[0], count * es, hipMemcpyDeviceToDevice, stream));
        return 0;
    }
    const Kern kern = pick(dt, op, v);
    if (!kern.general) return fail(MI_E_UNSUPPORTED, "no kernel for this dtype/op/variant");
    // VCVTNEPS2BF16 main part / scalar tail split of ccl_convert_fp32_to_bf16_arrays
    const uint64_t trunc_from = (count / 16) * 16;

    // The vector grid is the output's 16-byte grid: a scalar head up to the
    // first 16-byte boundary of `out`, a vector body, a scalar tail.  Inputs
    // need only be aligned to their element size: gfx950 serves a 16-byte
    // load from any byte address (profiles/round1_unaligned_probe.jsonl: right
    // bytes at every offset; 98-99 % of the aligned stream rate at 4-byte
    // offsets, 89 % at 1- and 2-byte offsets), so ring chunks at arbitrary
    // element offsets still stream as 16-byte vectors.  Operands that are not
    // aligned to their element size take the element loop (general kernel).
    const uintptr_t mis = reinterpret_cast<uintptr_t>(out) & 15u;
    bool elem = (mis % es) == 0;
    bool same = elem;
    for (int i = 0; i < k; i++) {
        const uintptr_t p = reinterpret_cast<uintptr_t>(inputs[i]);
        elem = elem && (p % es) == 0;
        same = same && (p & 15u) == mis;
    }
    const bool vec = same || (elem && unaligned_vectors());
    const size_t n_per_vec = 16 / es;
    const size_t head = vec && mis ? std::min<size_t>((16 - mis) / es, count) : 0;
    const uint64_t nvec = vec ? (count - head) / n_per_vec : 0;
    const size_t tail = vec ? count - head - nvec * n_per_vec : 0;

    // A grid cap (tuning / test knob) routes everything through the
    // grid-stride general kernel; otherwise one tile per block.
    const int cap = max_blocks();
    hipError_t e;
    if (vec && cap == 0 && k == 2) {
        R2Args r;
        r.acc = inputs[0];
        r.in = inputs[1];
        r.out = out;
        r.nvec = nvec;
        r.head = (uint32_t)head;
        r.tail = (uint32_t)tail;
        r.trunc_from = trunc_from;
        const uint64_t tile = (uint64_t)kB2 * kU2;
        uint64_t blocks = std::max<uint64_t>((nvec + tile - 1) / tile, 1);
        if (blocks > 0x7FFFFFFFull) return fail(MI_E_UNSUPPORTED, "bucket too large for one launch");
        e = kern.lean(dim3((unsigned)blocks), stream, r, wave_cap_lds(stream, planned_waves(2)));
    } else {
        KArgs a;
        memset(&a, 0, sizeof(a));
        for (int i = 0; i < k; i++) a.in[i] = inputs[i];
        a.out = out;
        a.k = k;
        a.count = count;
        a.trunc_from = trunc_from;
        if (vec) {
            a.head = head;
            a.nvec = nvec;
            a.tail = tail;
        } else {
            a.scalar_only = 1;
        }
        // fan tiles are 64 vectors: one launch covers 2^37 vectors (2 TiB)
        if (vec && cap == 0 && nvec / kFanBlock < 0x7FFFFFFFull) {
            e = kern.fan(stream, a, wave_cap_lds(stream, planned_waves(k)));
        } else {
            uint64_t blocks;
            if (vec) {
                const uint64_t tile = (uint64_t)kBlock * kUnroll;
                blocks = (a.nvec + tile - 1) / tile;
                if (cap > 0) blocks = std::min<uint64_t>(blocks, (uint64_t)cap);
                if (blocks == 0) blocks = 1;
            } else {
                blocks = std::min<uint64_t>((count + kBlock - 1) / kBlock, 8192);
            }
            if (blocks > 0x7FFFFFFFull) blocks = 0x7FFFFFFFull;  // grid-stride covers the rest
            e = kern.general(dim3((unsigned)blocks), stream, a);
        }
    }
    if (e != hipSuccess) return hip_fail(e, "kernel launch");
    return 0;
}

// ---------------------------------------------------------------------------
// descriptor batch: independent 2-input reduces in one launch
// ---------------------------------------------------------------------------
// Outputs must be pairwise disjoint and disjoint from other descriptors'
// inputs, or the result would depend on which tile ran first.
int check_batch_disjoint(const mi_reduce_desc_t* d, int n, size_t es) {
    struct Rng {
        uintptr_t lo, hi;
        int owner;
    };
    // A range end lo + count * es must not wrap: a corrupt count would
    // otherwise pass the overlap test below with an end below its start.
    for (int i = 0; i < n; i++) {
        if (!d[i].count) continue;
        const uintptr_t lim = UINTPTR_MAX / es;
        const uintptr_t lo_in = reinterpret_cast<uintptr_t>(d[i].in), lo_io = reinterpret_cast<uintptr_t>(d[i].inout);
        if (d[i].count > lim || d[i].count * es > UINTPTR_MAX - lo_in || d[i].count * es > UINTPTR_MAX - lo_io)
            return fail(MI_E_INVALID, "batch descriptor count overflows the address space");
    }
    std::vector<Rng> outs;
    outs.reserve(n);
    for (int i = 0; i < n; i++)
        if (d[i].count) {
            const uintptr_t lo = reinterpret_cast<uintptr_t>(d[i].inout);
            outs.push_back({lo, lo + d[i].count * es, i});
        }
    std::sort(outs.begin(), outs.end(), [](const Rng& x, const Rng& y) { return x.lo < y.lo; });
    for (size_t j = 1; j < outs.size(); j++)
        if (outs[j].lo < outs[j - 1].hi) return fail(MI_E_INVALID, "batch descriptors' outputs overlap");
    // outs are disjoint and sorted, so their ends are sorted too
    for (int i = 0; i < n; i++) {
        if (!d[i].count) continue;
        const uintptr_t lo = reinterpret_cast<uintptr_t>(d[i].in), hi = lo + d[i].count * es;
        auto it = std::upper_bound(outs.begin(), outs.end(), lo,
                                   [](uintptr_t v, const Rng& r) { return v < r.hi; });
        for (; it != outs.end() && it->lo < hi; ++it)
            if (it->owner != i) return fail(MI_E_INVALID, "a batch input overlaps another descriptor's output");
    }
    return 0;
}

int launch_reduce_batch(const mi_reduce_desc_t* d, int n, int dt, int op, unsigned flags,
                        hipStream_t stream) {
    const size_t es = dtype_size(dt);
    if (!es) return fail(MI_E_INVALID, "unknown datatype");
    if (op < MI_OP_SUM || op > MI_OP_MAX) return fail(MI_E_INVALID, "unsupported reduction (device path: sum/prod/min/max)");
    if (n < 0) return fail(MI_E_INVALID, "negative descriptor count");
    if (n == 0) return 0;
    if (!d) return fail(MI_E_INVALID, "null descriptor list");
    for (int i = 0; i < n; i++) {
        if (!d[i].count) continue;
        if (!d[i].in || !d[i].inout) return fail(MI_E_INVALID, "null operand in batch descriptor");
        if (int rc = require_gpu_visible(d[i].in, d[i].count * es)) return rc;
        if (int rc = require_gpu_visible(d[i].inout, d[i].count * es)) return rc;
    }
    if (int rc = check_batch_disjoint(d, n, es)) return rc;
    const unsigned v = canon_flags(dt, op, flags, 2);
    const Kern kern = pick(dt, op, v);
    if (!kern.batch) return fail(MI_E_UNSUPPORTED, "no kernel for this dtype/op/variant");

    const uint64_t tile = (uint64_t)kB2 * kU2;
    const size_t n_per_vec = 16 / es;
    BArgs a;
    memset(&a, 0, sizeof(a));
    uint64_t blocks = 0;
    auto flush = [&]() -> int {
        if (!a.n) return 0;
        a.block0[a.n] = (uint32_t)blocks;
        const hipError_t e = kern.batch(dim3((unsigned)blocks), stream, a, wave_cap_lds(stream, planned_waves(2)));
        if (e != hipSuccess) return hip_fail(e, "kernel launch");
        memset(&a, 0, sizeof(a));
        blocks = 0;
        return 0;
    };
    for (int i = 0; i < n; i++) {
        const size_t count = d[i].count;
        if (!count) continue;
        // the same vector-grid decision as launch_reduce for k = 2
        const uintptr_t mis = reinterpret_cast<uintptr_t>(d[i].inout) & 15u;
        const uintptr_t pin = reinterpret_cast<uintptr_t>(d[i].in);
        const bool elem = (mis % es) == 0 && (pin % es) == 0;
        const bool vec = (elem && (pin & 15u) == mis) || (elem && unaligned_vectors());
        const uint64_t head = vec && mis ? std::min<size_t>((16 - mis) / es, count) : 0;
        const uint64_t nvec = vec ? (count - head) / n_per_vec : 0;
        const uint64_t nb = std::max<uint64_t>((nvec + tile - 1) / tile, 1);
        if (!vec || max_blocks() != 0 || nb > 0x40000000ull) {  // element loop / grid knob / huge: own launch
            const void* ins[2] = {d[i].inout, d[i].in};
            if (int rc = launch_reduce(ins, 2, d[i].inout, count, dt, op, flags, stream)) return rc;
            continue;
        }
        if (a.n == kBatchMax || blocks + nb > 0x7FFFFFFFull)
            if (int rc = flush()) return rc;
        const int j = a.n++;
        a.acc[j] = d[i].inout;
        a.in[j] = d[i].in;
        a.out[j] = d[i].inout;
        a.nvec[j] = nvec;
        a.head[j] = (uint8_t)head;
        a.tail[j] = (uint8_t)(count - head - nvec * n_per_vec);
        a.trunc_from[j] = (count / 16) * 16;
        a.block0[j] = (uint32_t)blocks;
        blocks += nb;
    }
    return flush();
}

// ---------------------------------------------------------------------------
// per-thread device context: stream + scratch for host-operand staging
// ---------------------------------------------------------------------------
constexpr size_t kChunkBytes = 32ull << 20;  // staging chunk per operand

struct DevCtx {
    int device = -1;
    hipStream_t stream[2] = {nullptr, nullptr};
    std::vector<void*> dbuf[2];  // per pipeline slot: one device buffer per host operand
    size_t dbuf_bytes = 0;
    hipStream_t d2h = nullptr;              // the drain thread's stream (created on first use)
    hipEvent_t ready[2] = {nullptr, nullptr};  // per slot: the chunk's result is in dbuf
    std::vector<void*> hbuf;                // pinned bounce buffers for small pageable operands
    size_t hbuf_bytes = 0;
    char* edge = nullptr;                   // pinned scratch for the unaligned ends of D2H copies (Edges)

    ~DevCtx() {
        // Contexts die with their thread; device teardown at process exit may
        // already have happened, so errors here are ignored.
        for (int s = 0; s < 2; s++) {
            for (void* p : dbuf[s]) (void)hipFree(p);
            if (stream[s]) (void)hipStreamDestroy(stream[s]);
            if (ready[s]) (void)hipEventDestroy(ready[s]);
        }
        if (d2h) (void)hipStreamDestroy(d2h);
        for (void* p : hbuf) (void)hipHostFree(p);
        if (edge) (void)hipHostFree(edge);
    }
};

// A copy the synchronous caller makes after the GPU is done (pinned -> `dst`).
struct HostCopy {
    void* dst = nullptr;
    const void* src = nullptr;
    size_t bytes = 0;
};

// ---- the runtime's copies of pageable memory ---------------------------------
// The runtime's copies between pageable host memory and the device get
// 16-byte-aligned host addresses and 16-byte multiples only.  On MI355X /
// ROCm 7.2 an H2D copy from pageable memory whose source was 2-byte aligned
// (a bf16 operand at an odd element offset of a packed buffer: oneCCL's tmp
// buffer of peer chunks) faulted the GPU ("an illegal memory access") in two
// of several full GPU-suite runs, both times at that one case -- the only
// staged copy with such a source -- and never at the 4-byte-aligned fp32 cases
// around it (profiles/round5_host/pytest_gpu_fault_run.txt,
// profiles/round5_run8/).  The staged path's own kernels read only device
// buffers, so the copy itself is the suspect; a fault that depends on where
// the operand lies relative to a page would come and go exactly like this.
// So:
//  * H2D into a staging buffer copies the aligned span around the operand
//    (h2d_stage).  Aligning down the start and up the end by < 16 bytes never
//    leaves the pages the operand touches, so nothing unmapped is read; the
//    kernel reads the operand `shift` bytes into the staging buffer.
//  * D2H into pageable memory copies the aligned interior; the head and tail
//    (< 16 bytes each) go to pinned scratch and are copied to the destination
//    by the CPU after the stream is done (Edges, d2h_pageable).  Nothing
//    outside the destination is written.
constexpr uintptr_t kHostAlign = 16;
constexpr size_t kStageSlack = 2 * kHostAlign;  // a staging buffer holds a chunk and its alignment
inline uintptr_t host_align_dn(uintptr_t a) { return a & ~(kHostAlign - 1); }
inline uintptr_t host_align_up(uintptr_t a) { return (a + kHostAlign - 1) & ~(kHostAlign - 1); }

// Test hook (mi_test_fail_copy): the nth staged host copy from now on fails
// with hipErrorInvalidValue before it reaches the runtime (no sticky state).
std::atomic<long> g_fail_copy_nth{0};
std::atomic<long> g_copy_seq{0};

bool injected_copy_failure() {
    const long n = g_fail_copy_nth.load(std::memory_order_relaxed);
    return n > 0 && g_copy_seq.fetch_add(1, std::memory_order_relaxed) + 1 == n;
}

const char* kind_name(PtrKind k) { return k == PK_DEVICE ? "device" : k == PK_PINNED ? "pinned" : "pageable"; }

// A failed copy between host memory and a staging buffer: the HIP error and
// where the host side lay -- the operand's address within its page and its
// length, the span the runtime was handed (16-byte aligned, h2d_stage /
// d2h_pageable), the chunk and the operand's pointer class -- so that a fault
// surfacing at a copy can be matched to the operand's geometry (VERDICT r5
// item 2).  A sticky error left by an earlier kernel surfaces at the next
// runtime call too: the text names the copy that observed the error, which
// is not necessarily the one that caused it.
// `hull`: the runtime got the operand's aligned hull (h2d_stage), else its
// aligned interior (d2h_pageable, mi_copy_sync's H2D).
std::string copy_geometry(const void* host, size_t bytes, size_t chunk, PtrKind kind, bool hull) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(host);
    const uintptr_t lo = hull ? host_align_dn(a) : std::min(host_align_up(a), a + bytes);
    const uintptr_t hi = hull ? host_align_up(a + bytes) : std::max(lo, host_align_dn(a + bytes));
    char buf[320];
    snprintf(buf, sizeof buf,
             " [%s host operand: addr & 4095 = %zu, %zu bytes, ends at page offset %zu; runtime span: addr & 4095 "
             "= %zu, %zu bytes; chunk %zu]",
             kind_name(kind), (size_t)(a & 4095), bytes, (size_t)((a + bytes) & 4095), (size_t)(lo & 4095),
             (size_t)(hi - lo), chunk);
    return buf;
}

int copy_fail(hipError_t e, const char* what, const void* host, size_t bytes, size_t chunk, PtrKind kind,
              bool hull) {
    g_last_error = std::string(what) + ": " + hipGetErrorString(e) + copy_geometry(host, bytes, chunk, kind, hull);
    return (int)e;
}

hipError_t h2d_stage(void* dst, const void* src, size_t bytes, hipStream_t s, size_t* shift) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(src);
    const uintptr_t lo = host_align_dn(a), hi = host_align_up(a + bytes);
    *shift = a - lo;
    if (injected_copy_failure()) return hipErrorInvalidValue;
    return hipMemcpyAsync(dst, reinterpret_cast<const void*>(lo), hi - lo, hipMemcpyHostToDevice, s);
}

constexpr size_t kEdgeBytes = 8192;            // DevCtx::edge
constexpr size_t kEdgeSlot = 2 * kHostAlign;   // one D2H: head + tail
constexpr size_t kDrainEdge = kEdgeBytes - kEdgeSlot;  // the drain thread's slot (the last one)

struct Edges {
    char* pin = nullptr;  // pinned scratch, kEdgeSlot bytes per D2H
    size_t slots = 0, used = 0;
    std::vector<HostCopy> post;
    bool full() const { return used >= slots; }
    // after the stream(s) carrying the D2H copies are done
    void flush() {
        for (const HostCopy& c : post) memcpy(c.dst, c.src, c.bytes);
        post.clear();
        used = 0;
    }
};

int ensure_edges(DevCtx* d) {
    if (!d->edge) {
        void* p = nullptr;
        MI_HIP(hipHostMalloc(&p, kEdgeBytes, hipHostMallocDefault));
        d->edge = static_cast<char*>(p);
    }
    return 0;
}

// D2H of device [src, src + bytes) into pageable host memory at dst; needs a
// free slot in `e` (the caller flushes a full one first).
hipError_t d2h_pageable(void* dst, const void* src, size_t bytes, hipStream_t s, Edges& e) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(dst);
    const size_t head = std::min(bytes, (size_t)(host_align_up(a) - a));
    const size_t interior = (bytes - head) & ~(size_t)(kHostAlign - 1);
    const size_t tail = bytes - head - interior;
    const char* s8 = static_cast<const char*>(src);
    char* d8 = static_cast<char*>(dst);
    if (injected_copy_failure()) return hipErrorInvalidValue;
    hipError_t r = hipSuccess;
    if (interior) r = hipMemcpyAsync(d8 + head, s8 + head, interior, hipMemcpyDeviceToHost, s);
    if (head || tail) {
        char* slot = e.pin + kEdgeSlot * e.used++;
        if (r == hipSuccess && head) {
            r = hipMemcpyAsync(slot, s8, head, hipMemcpyDeviceToHost, s);
            e.post.push_back(HostCopy{d8, slot, head});
        }
        if (r == hipSuccess && tail) {
            r = hipMemcpyAsync(slot + kHostAlign, s8 + head + interior, tail, hipMemcpyDeviceToHost, s);
            e.post.push_back(HostCopy{d8 + head + interior, slot + kHostAlign, tail});
        }
    }
    return r;
}

// ---------------------------------------------------------------------------
// where helper threads run
// ---------------------------------------------------------------------------
// A new thread inherits its creator's CPU affinity.  oneCCL pins each worker
// thread to one core (CCL_WORKER_AFFINITY), so the staging worker and the
// drain thread a worker creates would share that one core with it, and with
// the cooperative split's CPU head: measured with pinned workers, the GPU
// path then ran at half its rate and the split below one core
// (profiles/round2_dispatch/workers_pinned_inherit.jsonl).  Helpers therefore
// take the process's CPU set: the main thread's allowed list
// (/proc/self/status describes the thread-group leader, which oneCCL does
// not pin), read at library load -- not the loading thread's own mask, which
// is one core when the library is dlopen'ed lazily from a pinned worker.
// MI_REDUCE_HELPER_AFFINITY=inherit keeps the creator's; mi_helper_cpu_count()
// reports the set chosen.
bool parse_cpu_list(const char* s, cpu_set_t* out) {
    CPU_ZERO(out);
    while (*s && *s != '\n') {
        char* end = nullptr;
        const long a = strtol(s, &end, 10);
        if (end == s || a < 0) return false;
        long b = a;
        s = end;
        if (*s == '-') {
            b = strtol(s + 1, &end, 10);
            if (end == s + 1 || b < a) return false;
            s = end;
        }
        for (long c = a; c <= b && c < CPU_SETSIZE; c++) CPU_SET((int)c, out);
        if (*s == ',') s++;
        else if (*s && *s != '\n') return false;
    }
    return CPU_COUNT(out) > 0;
}

struct HelperCpus {
    cpu_set_t mask;
    bool use = false;
    HelperCpus() {
        CPU_ZERO(&mask);
        const char* e = getenv("MI_REDUCE_HELPER_AFFINITY");
        if (e && strcmp(e, "inherit") == 0) return;
        if (FILE* f = fopen("/proc/self/status", "r")) {
            char line[4096];
            while (fgets(line, sizeof line, f))
                if (strncmp(line, "Cpus_allowed_list:", 18) == 0) {
                    const char* p = line + 18;
                    while (*p == ' ' || *p == '\t') p++;
                    use = parse_cpu_list(p, &mask);
                    break;
                }
            fclose(f);
        }
        if (!use) use = sched_getaffinity(0, sizeof(mask), &mask) == 0 && CPU_COUNT(&mask) > 0;
    }
};
const HelperCpus g_helper_cpus;  // at library load

void helper_thread_affinity() {
    if (g_helper_cpus.use) (void)pthread_setaffinity_np(pthread_self(), sizeof(cpu_set_t), &g_helper_cpus.mask);
}

// ---------------------------------------------------------------------------
// drain thread for staged results bound for pageable host memory
// ---------------------------------------------------------------------------
// A D2H copy into pageable memory blocks the thread that issues it until the
// copy is done.  Issued inline, chunk c's D2H therefore sits between chunk
// c's kernel and chunk c+1's H2D, and the staged pipeline uses one PCIe
// direction at a time (17 GiB/s for a 256 MiB bucket).  On a helper thread it
// runs while the calling thread copies the next chunk in, so both directions
// are busy.  Used by the synchronous entry points only; the helper exists for
// the duration of one call.
struct Drain {
    struct Task {
        void* dst;
        const void* src;
        size_t bytes;
        hipEvent_t ready;
        size_t chunk;
    };
    std::mutex mu;
    std::condition_variable cv;
    std::deque<Task> q;
    size_t done = 0;  // tasks finished (or skipped after an error)
    bool stop = false;
    hipError_t err = hipSuccess;
    std::string err_where;  // copy_geometry of the first failed task
    std::thread th;

    // `edge`: pinned scratch for the unaligned ends of its D2H copies (kEdgeSlot bytes)
    void start(int device, hipStream_t s, char* edge) {
        if (th.joinable()) return;
        th = std::thread([this, device, s, edge] { loop(device, s, edge); });
    }
    void loop(int device, hipStream_t s, char* edge) {
        helper_thread_affinity();
        hipError_t e = hipSetDevice(device);
        Edges ed;
        ed.pin = edge;
        ed.slots = 1;
        for (;;) {
            Task t;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return stop || !q.empty(); });
                if (q.empty()) return;
                t = q.front();
                q.pop_front();
            }
            const hipError_t e0 = e;
            if (e == hipSuccess) e = hipEventSynchronize(t.ready);
            if (e == hipSuccess) e = d2h_pageable(t.dst, t.src, t.bytes, s, ed);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            if (e == hipSuccess) ed.flush();
            ed.post.clear();
            ed.used = 0;
            std::lock_guard<std::mutex> lk(mu);
            if (e != hipSuccess && err == hipSuccess) {
                err = e;
                if (e0 == hipSuccess) err_where = copy_geometry(t.dst, t.bytes, t.chunk, PK_PAGEABLE, false);
            }
            done++;
            cv.notify_all();
        }
    }
    void push(const Task& t) {
        std::lock_guard<std::mutex> lk(mu);
        q.push_back(t);
        cv.notify_all();
    }
    // wait until `n` tasks are finished; the first error of the helper, if any
    hipError_t wait_done(size_t n) {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return done >= n; });
        return err;
    }
    hipError_t finish() {
        if (th.joinable()) {
            {
                std::lock_guard<std::mutex> lk(mu);
                stop = true;
            }
            cv.notify_all();
            th.join();
        }
        return err;
    }
    ~Drain() { (void)finish(); }
};

// Process exit against threads that are still exiting or still working.  A
// thread's staging worker (t_stage) finishes the thread's un-waited
// asynchronous requests when the thread exits.  A host program may exit
// while that is still going: Python's Thread.join(), for one, returns before
// the OS thread has run its thread_local destructors.  The HIP runtime's own
// exit-time teardown then pulls the device from under those calls (a SIGSEGV
// inside libamdhip64 from __call_tls_dtors, profiles/round2_dispatch/
// exit_crash_trace.txt).  (A thread's contexts themselves make no HIP call
// when it exits: they go back to a pool, see ThreadCtx.)
//
// So every job a staging worker runs holds an ExitGuard while it makes HIP
// calls.  An exit handler, registered after the runtime's (at the first
// context, when HIP is initialised, so it runs before the runtime's), marks
// the process as exiting and then waits until no guard is held.  A job that
// would start after that mark makes no HIP call: it fails with MI_E_EXITING.  The counter is raised before
// the mark is read (both sequentially consistent), so either the section sees
// the mark or the handler sees the section.
//
// The wait is bounded (MI_REDUCE_EXIT_WAIT_S, default 60 s): a section that
// never ends -- a job blocked on the event of a kernel that hangs, a
// user-supplied head fold that blocks -- would otherwise hold the process at
// exit forever.  Past the bound the handler names the section last entered
// and ends the process with status 70 (EX_SOFTWARE) without the runtime's
// teardown, which would fault under the section still inside HIP.
std::atomic<bool> g_exiting{false};
std::atomic<int> g_active{0};
std::atomic<const char*> g_active_what{nullptr};  // the section most recently entered

double exit_wait_s() {
    const char* e = getenv("MI_REDUCE_EXIT_WAIT_S");
    const double v = e ? atof(e) : 60.0;
    return v > 0 ? v : 60.0;
}

void at_process_exit() {
    g_exiting.store(true);
    const double limit = exit_wait_s();
    const auto t0 = std::chrono::steady_clock::now();
    while (g_active.load() > 0) {
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit) {
            const char* what = g_active_what.load();
            fprintf(stderr,
                    "oneccl_amd: process exit: %d library section(s) still running after %.0f s (last entered: %s); "
                    "ending the process without the HIP runtime's teardown\n",
                    g_active.load(), limit, what ? what : "?");
            fflush(nullptr);
            _exit(70);
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
}

struct ExitGuard {
    bool entered;
    explicit ExitGuard(const char* what) {
        g_active.fetch_add(1);
        entered = !g_exiting.load();
        if (!entered) g_active.fetch_sub(1);
        else g_active_what.store(what);
    }
    ~ExitGuard() {
        if (entered) g_active.fetch_sub(1);
    }
    ExitGuard(const ExitGuard&) = delete;
    ExitGuard& operator=(const ExitGuard&) = delete;
};

// A thread's contexts (streams, staging and bounce buffers) outlive it: when
// the thread exits they go to a process-wide pool, and the next thread that
// needs a context on that device takes one from there.  So a thread exit
// makes no HIP call -- no hipFree / hipHostFree / hipStreamDestroy running
// from __call_tls_dtors while other threads copy and launch (oneCCL's workers
// are long-lived, but a caller that starts short-lived threads, as the test
// suites do, would otherwise free and reallocate gigabytes of staging memory
// per thread) -- and work a thread left queued on its streams stays ordered
// before whatever the next owner queues there.  The pool holds at most as
// many contexts per device as threads ever used one at once; they are freed
// with the process.
// The pool is never destroyed (a thread may exit while the process runs its
// static destructors).
struct CtxPool {
    std::mutex mu;
    std::vector<DevCtx*> free;
};
CtxPool& ctx_pool() {
    static CtxPool* p = new CtxPool();
    return *p;
}
std::atomic<size_t> g_ctx_created{0};

struct ThreadCtx {
    std::vector<DevCtx*> devs;
    ~ThreadCtx() {
        CtxPool& p = ctx_pool();
        std::lock_guard<std::mutex> lk(p.mu);
        for (DevCtx* d : devs)
            if (d) p.free.push_back(d);
        devs.clear();
    }
};
thread_local ThreadCtx t_ctx;

DevCtx* pooled_ctx(int device) {
    CtxPool& p = ctx_pool();
    std::lock_guard<std::mutex> lk(p.mu);
    for (size_t i = p.free.size(); i-- > 0;)
        if (p.free[i]->device == device) {
            DevCtx* d = p.free[i];
            p.free.erase(p.free.begin() + (long)i);
            return d;
        }
    return nullptr;
}
std::once_flag g_exit_hook;

// Register at_process_exit once, after the HIP runtime is initialised (a HIP
// call first), so that it runs before the runtime's own exit teardown.
void ensure_exit_hook() {
    std::call_once(g_exit_hook, [] {
        int dev = 0;
        (void)hipGetDevice(&dev);
        std::atexit(at_process_exit);
    });
}

int get_ctx(int device, DevCtx** out) {
    if (device < 0) MI_HIP(hipGetDevice(&device));
    if ((size_t)device >= t_ctx.devs.size()) t_ctx.devs.resize(device + 1, nullptr);
    if (!t_ctx.devs[device]) t_ctx.devs[device] = pooled_ctx(device);
    if (!t_ctx.devs[device]) {
        // Built in full before it is published: a failure leaves no
        // half-made context (a null stream would be the legacy default
        // stream) cached for the thread, and the caller's device is restored
        // on every path.
        int prev = 0;
        MI_HIP(hipGetDevice(&prev));
        struct Restore {
            int dev;
            ~Restore() { (void)hipSetDevice(dev); }
        } restore{prev};
        MI_HIP(hipSetDevice(device));
        ensure_exit_hook();
        std::unique_ptr<DevCtx> d(new DevCtx());
        d->device = device;
        for (int s = 0; s < 2; s++) MI_HIP(hipStreamCreateWithFlags(&d->stream[s], hipStreamNonBlocking));
        t_ctx.devs[device] = d.release();
        g_ctx_created.fetch_add(1);
    }
    *out = t_ctx.devs[device];
    return 0;
}

// Small pageable operands are copied through pinned bounce buffers by the
// CPU and reduced by the zero-copy kernel: below about 1 MiB the runtime's
// pageable copies cost more than the data (profiles/round1_size_sweep*.jsonl).
constexpr size_t kBounceBytes = 1ull << 20;  // per operand

int ensure_bounce(DevCtx* d, size_t nbuf) {
    if (d->hbuf.size() >= nbuf) return 0;
    while (d->hbuf.size() < nbuf) {
        void* p = nullptr;
        MI_HIP(hipHostMalloc(&p, kBounceBytes, hipHostMallocDefault));
        d->hbuf.push_back(p);
    }
    d->hbuf_bytes = kBounceBytes;
    return 0;
}

int ensure_scratch(DevCtx* d, size_t nbuf, size_t bytes) {
    if (d->dbuf[0].size() >= nbuf && d->dbuf_bytes >= bytes) return 0;
    // grow to the larger of the old and the new shape (a call with fewer but
    // larger operands keeps room for the earlier call's operand count)
    const size_t want = std::max(bytes, d->dbuf_bytes);
    nbuf = std::max(nbuf, d->dbuf[0].size());
    for (int s = 0; s < 2; s++) {
        for (void* p : d->dbuf[s]) MI_HIP(hipFree(p));
        d->dbuf[s].clear();
    }
    d->dbuf_bytes = 0;  // published only once every buffer exists: a failed
                        // hipMalloc leaves no null slot behind for the next call
    for (int s = 0; s < 2; s++) {
        d->dbuf[s].reserve(nbuf);
        while (d->dbuf[s].size() < nbuf) {
            void* p = nullptr;
            MI_HIP(hipMalloc(&p, want));
            d->dbuf[s].push_back(p);
        }
    }
    d->dbuf_bytes = want;
    return 0;
}

// Every operand's kind, device-visible address and device, classified once
// (sync_entry, for a confined caller's hand-off) and handed to reduce_issue,
// which would otherwise classify them again (three
// classifications per bucket for a pinned oneCCL worker, now two).
struct Kinds {
    bool valid = false;
    PtrKind kin[MI_MAX_INPUTS];
    const void* dins[MI_MAX_INPUTS];
    int dev_in[MI_MAX_INPUTS];
    PtrKind kout = PK_PAGEABLE;
    void* dout = nullptr;
    int dev_out = -1;
};

void classify_all(const void* const* inputs, int k, void* out, size_t bytes, Kinds* c) {
    for (int i = 0; i < k; i++) {
        void* dp = const_cast<void*>(inputs[i]);
        c->dev_in[i] = -1;
        c->kin[i] = classify(inputs[i], &c->dev_in[i], &dp, bytes);
        c->dins[i] = dp;
    }
    c->dout = out;
    c->dev_out = -1;
    c->kout = classify(out, &c->dev_out, &c->dout, bytes);
    c->valid = true;
}

// Issue a fold with any pointer kinds on the calling thread's streams of the
// chosen device; *used = the streams that carry work (bit 0: stream[0],
// bit 1: stream[1]).  All-device or zero-copy: one launch on stream[0].
// Otherwise: chunks of kChunkBytes, two pipeline slots on two streams (H2D
// of chunk c+1 overlaps the kernel / D2H of chunk c).
int reduce_issue(const void* const* inputs, int k, void* out, size_t count, int dt, int op,
                 unsigned flags, int device, DevCtx** ctx, int* used, Drain* drain = nullptr,
                 std::vector<HostCopy>* post = nullptr, hipEvent_t* t_start = nullptr,
                 const Kinds* pre = nullptr) {
    *ctx = nullptr;
    *used = 0;
    const size_t es = dtype_size(dt);
    if (!es) return fail(MI_E_INVALID, "unknown datatype");
    if (k < 1 || k > MI_MAX_INPUTS) return fail(MI_E_INVALID, "input count out of range [1,16]");
    if (count == 0) return 0;
    if (!out) return fail(MI_E_INVALID, "null output");
    for (int i = 0; i < k; i++)
        if (!inputs[i]) return fail(MI_E_INVALID, "null input");

    Kinds own;
    if (!pre || !pre->valid) {
        classify_all(inputs, k, out, count * es, &own);
        pre = &own;
    }
    const PtrKind* kin = pre->kin;
    const void* const* dins = pre->dins;
    int pdev = -1;
    bool all_dev = true, mixed_dev = false;
    for (int i = 0; i < k; i++) {
        const int d_i = pre->dev_in[i];
        all_dev = all_dev && kin[i] == PK_DEVICE;
        if (d_i >= 0) {
            mixed_dev = mixed_dev || (pdev >= 0 && d_i != pdev);
            pdev = d_i;
        }
    }
    void* dout = pre->dout;
    const int d_o = pre->dev_out;
    const PtrKind kout = pre->kout;
    all_dev = all_dev && kout == PK_DEVICE;
    if (d_o >= 0) {
        mixed_dev = mixed_dev || (pdev >= 0 && d_o != pdev);
        pdev = d_o;
    }
    // one kernel reads every operand: operands on two GPUs would need peer
    // access the caller never set up — refuse instead of faulting
    if (mixed_dev) return fail(MI_E_UNSUPPORTED, "device operands live on different GPUs");
    if (device < 0 && pdev >= 0) device = pdev;

    DevCtx* d = nullptr;
    int rc = get_ctx(device, &d);
    if (rc) return rc;
    *ctx = d;
    int prev = 0;
    MI_HIP(hipGetDevice(&prev));
    if (prev != d->device) MI_HIP(hipSetDevice(d->device));
    struct Restore {
        int dev, cur;
        ~Restore() {
            if (dev != cur) (void)hipSetDevice(dev);
        }
    } restore{prev, d->device};

    // zero-copy: pinned host operands are read/written by the kernel in place
    // over PCIe (both directions at once); device operands as they are
    bool direct = true;
    for (int i = 0; i < k; i++) direct = direct && (kin[i] == PK_DEVICE || kin[i] == PK_PINNED);
    direct = direct && (kout == PK_DEVICE || kout == PK_PINNED);
    if (!all_dev && direct && host_mode() == MI_HOST_STAGED) direct = false;
    if (all_dev || direct) {
        *used = 1;
        if (t_start) {  // a timed request: an event pair around the one launch
            MI_HIP(hipEventCreateWithFlags(t_start, hipEventDefault));
            MI_HIP(hipEventRecord(*t_start, d->stream[0]));
        }
        return launch_reduce(dins, k, dout, count, dt, op, flags, d->stream[0], true);
    }

    // small pageable operands (synchronous callers only): CPU copy into
    // pinned bounce buffers, zero-copy kernel, CPU copy of the result back
    bool any_pageable = kout == PK_PAGEABLE;
    for (int i = 0; i < k; i++) any_pageable = any_pageable || kin[i] == PK_PAGEABLE;
    if (post && any_pageable && host_mode() == MI_HOST_AUTO && count * es <= kBounceBytes) {
        const void* bins[MI_MAX_INPUTS];
        const void* bsrc[MI_MAX_INPUTS + 1];
        void* bbuf[MI_MAX_INPUTS + 1];
        int nb = 0;
        auto bounce_of = [&](const void* p, bool copy_in) -> void* {
            for (int j = 0; j < nb; j++)
                if (bsrc[j] == p) return bbuf[j];
            bsrc[nb] = p;
            bbuf[nb] = d->hbuf[nb];
            if (copy_in) memcpy(bbuf[nb], p, count * es);
            return bbuf[nb++];
        };
        rc = ensure_bounce(d, (size_t)k + 1);
        if (rc) return rc;
        for (int i = 0; i < k; i++) bins[i] = kin[i] == PK_PAGEABLE ? bounce_of(inputs[i], true) : dins[i];
        void* bout = kout == PK_PAGEABLE ? bounce_of(out, false) : dout;
        *used = 1;
        rc = launch_reduce(bins, k, bout, count, dt, op, flags, d->stream[0], true);
        if (rc) return rc;
        if (kout == PK_PAGEABLE) post->push_back(HostCopy{out, bout, count * es});
        return 0;
    }

    // distinct host operands get a device staging buffer per slot; `out`
    // reuses the buffer of the input it aliases (in-place inout)
    int slot_of[MI_MAX_INPUTS + 1];
    const void* host_ptr[MI_MAX_INPUTS + 1];
    int nhost = 0;
    for (int i = 0; i <= k; i++) {
        const void* p = (i < k) ? inputs[i] : out;
        const PtrKind kk = (i < k) ? kin[i] : kout;
        slot_of[i] = -1;
        if (kk == PK_DEVICE) continue;
        for (int j = 0; j < nhost; j++)
            if (host_ptr[j] == p) slot_of[i] = j;
        if (slot_of[i] < 0) {
            host_ptr[nhost] = p;
            slot_of[i] = nhost++;
        }
    }
    size_t chunk_elems = kChunkBytes / es;
    chunk_elems -= chunk_elems % 16;  // keeps VCVTNEPS2BF16-tail split aligned (see below)
    // each host operand sits at its own 16-byte offset in its staging buffers
    // (h2d_stage); chunk starts are 16-byte multiples apart, so every chunk
    // keeps it
    size_t shift[MI_MAX_INPUTS + 1];
    for (int j = 0; j < nhost; j++) shift[j] = reinterpret_cast<uintptr_t>(host_ptr[j]) & (kHostAlign - 1);
    rc = ensure_scratch(d, (size_t)nhost, chunk_elems * es + kStageSlack);
    if (rc) return rc;

    const size_t nchunks = (count + chunk_elems - 1) / chunk_elems;
    *used = nchunks > 1 ? 3 : 1;
    const bool d2h_pg = kout == PK_PAGEABLE && slot_of[k] >= 0;
    const bool drained = drain && d2h_pg && nchunks > 1;
    Edges edges;  // unaligned ends of the D2H copies this thread issues
    if (d2h_pg) {
        rc = ensure_edges(d);
        if (rc) return rc;
        edges.pin = d->edge;
        edges.slots = kDrainEdge / kEdgeSlot;
    }
    if (drained) {
        if (!d->d2h) MI_HIP(hipStreamCreateWithFlags(&d->d2h, hipStreamNonBlocking));
        for (int s = 0; s < 2; s++)
            if (!d->ready[s]) MI_HIP(hipEventCreateWithFlags(&d->ready[s], hipEventDisableTiming));
        drain->start(d->device, d->d2h, d->edge + kDrainEdge);
    }
    for (size_t c = 0; c < nchunks; c++) {
        const int s = (int)(c & 1);
        hipStream_t st = d->stream[s];
        // slot s holds chunk c-2's result until the helper has copied it out
        if (drained && c >= 2)
            if (hipError_t he = drain->wait_done(c - 1)) {
                hip_fail(he, "staged D2H into pageable memory (drain thread)");
                g_last_error += drain->err_where;
                return (int)he;
            }
        const size_t off = c * chunk_elems;
        const size_t n = std::min(chunk_elems, count - off);
        const size_t bytes = n * es;
        const void* din[MI_MAX_INPUTS];
        std::vector<bool> loaded((size_t)nhost, false);
        for (int i = 0; i < k; i++) {
            if (slot_of[i] < 0) {
                din[i] = static_cast<const char*>(inputs[i]) + off * es;
            } else {
                char* buf = static_cast<char*>(d->dbuf[s][slot_of[i]]);
                if (!loaded[slot_of[i]]) {
                    size_t sh = 0;
                    const void* hsrc = static_cast<const char*>(inputs[i]) + off * es;
                    if (hipError_t he = h2d_stage(buf, hsrc, bytes, st, &sh))
                        return copy_fail(he, "H2D staging copy", hsrc, bytes, c, kin[i], true);
                    loaded[slot_of[i]] = true;
                }
                din[i] = buf + shift[slot_of[i]];
            }
        }
        void* cdst = (slot_of[k] < 0) ? static_cast<char*>(out) + off * es
                                      : static_cast<char*>(d->dbuf[s][slot_of[k]]) + shift[slot_of[k]];
        // The tail-truncation split is defined on the whole array: only the
        // last chunk holds elements >= (count/16)*16, and chunk starts are
        // multiples of 16, so the per-chunk split computed inside
        // launch_reduce is the same split.
        rc = launch_reduce(din, k, cdst, n, dt, op, flags, st, true);
        if (rc) return rc;
        if (slot_of[k] >= 0) {
            void* hdst = static_cast<char*>(out) + off * es;
            if (drained) {
                MI_HIP(hipEventRecord(d->ready[s], st));
                drain->push({hdst, cdst, bytes, d->ready[s], c});
            } else if (d2h_pg) {
                if (edges.full()) {  // every slot holds an end not yet copied out
                    for (int q = 0; q < 2; q++) MI_HIP(wait_stream(d->stream[q]));
                    edges.flush();
                }
                if (hipError_t he = d2h_pageable(hdst, cdst, bytes, st, edges))
                    return copy_fail(he, "D2H result copy", hdst, bytes, c, kout, false);
            } else if (hipError_t he = hipMemcpyAsync(hdst, cdst, bytes, hipMemcpyDeviceToHost, st)) {
                return copy_fail(he, "D2H result copy", hdst, bytes, c, kout, true);
            }
        }
    }
    if (!edges.post.empty()) {
        if (post) {  // copied by the synchronous caller after its wait
            post->insert(post->end(), edges.post.begin(), edges.post.end());
        } else {
            for (int q = 0; q < 2; q++) MI_HIP(wait_stream(d->stream[q]));
            edges.flush();
        }
    }
    return 0;
}

int reduce_sync(const void* const* inputs, int k, void* out, size_t count, int dt, int op,
                unsigned flags, int device, const Kinds* pre = nullptr) {
    DevCtx* d = nullptr;
    int used = 0;
    Drain drain;
    std::vector<HostCopy> post;
    const int rc = reduce_issue(inputs, k, out, count, dt, op, flags, device, &d, &used, &drain, &post, nullptr,
                                pre);
    const hipError_t de = drain.finish();  // every staged result is in `out` after this
    if (rc) return rc;
    if (de != hipSuccess) {
        hip_fail(de, "staged D2H into pageable memory (drain thread)");
        g_last_error += drain.err_where;
        return (int)de;
    }
    for (int s = 0; s < 2; s++)
        if (used & (1 << s)) MI_HIP(wait_stream(d->stream[s]));
    for (const HostCopy& c : post) memcpy(c.dst, c.src, c.bytes);
    return 0;
}

// ---------------------------------------------------------------------------
// asynchronous staging: a worker thread per calling thread
// ---------------------------------------------------------------------------
// The runtime's copies to and from pageable memory are host-synchronous, so an
// mi_reduce_start that staged pageable operands inline would return only when
// the copies were done, and a schedule entry polling it would gain nothing.
// Requests that need staging go instead to a worker thread owned by the
// calling thread. It runs them in submission order through the synchronous
// pipeline (drain thread included), with its own streams and staging buffers
// that persist across requests.
struct AsyncJob {
    // Work the calling thread had already issued on its own streams when the
    // job was submitted: the worker waits for it first, so a staged request
    // never overtakes an earlier direct one (e.g. a device-only reduce that
    // writes an operand this job reads).
    std::vector<hipEvent_t> prior;
    const void* inputs[MI_MAX_INPUTS];
    int k = 0;
    void* out = nullptr;
    size_t count = 0;
    int dt = 0, op = 0;
    unsigned flags = 0;
    int device = -1;
    Kinds kinds;  // the operands as the submitting thread classified them (valid: use them)
    // device < 0 means the submitting thread's current device (mi_reduce.h):
    // that device, read on the submitting thread, made current on the worker
    // before the job runs (the worker's own current device is HIP's default)
    int caller_device = -1;
    // cooperative split (mi_reduce_split_start): [0, head) by head_fold on
    // the worker thread while the GPU folds [head, count)
    size_t head = 0;
    mi_host_fold_t head_fold = nullptr;
    double t_head = -1.0, t_tail = -1.0;  // seconds from the split's start (run_split)
    double t_run = -1.0;                  // seconds the worker spent running it (after `prior`)
    std::mutex mu;
    std::condition_variable cv;
    bool done = false;
    int rc = 0;
    std::string err;

    int wait() {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return done; });
        return rc;
    }
    ~AsyncJob() {
        for (hipEvent_t e : prior) (void)hipEventDestroy(e);  // a job that never ran
    }
};

int run_split(AsyncJob& j);
int split_job(AsyncJob& j) { return run_split(j); }

double mono_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct StageWorker {
    std::thread th;
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::shared_ptr<AsyncJob>> q;
    size_t inflight = 0;  // submitted and not yet finished (guarded by mu)
    bool stop = false;
    std::atomic<int> last_device{-1};  // the worker's current device when its last job ran (diagnostic)

    void submit(const std::shared_ptr<AsyncJob>& j) {
        ensure_exit_hook();  // the job's HIP calls are then covered by the exit handler
        {
            std::lock_guard<std::mutex> lk(mu);
            q.push_back(j);
            inflight++;
        }
        if (!th.joinable()) {
            try {
                th = std::thread([this] { loop(); });
            } catch (...) {
                std::lock_guard<std::mutex> lk(mu);
                q.pop_back();
                inflight--;
                throw;
            }
        }
        cv.notify_all();
    }
    bool busy() {
        std::lock_guard<std::mutex> lk(mu);
        return inflight != 0;
    }
    // Wait until every submitted job has finished (their results are final).
    void wait_idle() {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return inflight == 0; });
    }
    void loop() {
        helper_thread_affinity();
        for (;;) {
            std::shared_ptr<AsyncJob> j;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return stop || !q.empty(); });
                if (q.empty()) return;
                j = q.front();
                q.pop_front();
            }
            int rc = 0;
            {
                ExitGuard g("a staging worker's job");  // the exit handler waits for a job that has started
                if (!g.entered) {
                    rc = fail(MI_E_EXITING, "the process is exiting: asynchronous request not run");
                    j->prior.clear();  // their events go with the process
                } else {
                    for (hipEvent_t e : j->prior) {
                        const hipError_t he = hipEventSynchronize(e);
                        if (he != hipSuccess && !rc)
                            rc = hip_fail(he, "waiting for earlier work of the submitting thread");
                        (void)hipEventDestroy(e);
                    }
                    j->prior.clear();
                    const double t0 = mono_s();
                    if (!rc && j->device < 0 && j->caller_device >= 0) {
                        const hipError_t he = hipSetDevice(j->caller_device);
                        if (he != hipSuccess) rc = hip_fail(he, "hipSetDevice (the submitting thread's device)");
                    }
                    int cur = -1;
                    if (!rc && hipGetDevice(&cur) == hipSuccess) last_device.store(cur, std::memory_order_relaxed);
                    if (!rc)
                        rc = j->head_fold ? split_job(*j)
                                          : reduce_sync(j->inputs, j->k, j->out, j->count, j->dt, j->op, j->flags,
                                                        j->device, &j->kinds);
                    j->t_run = mono_s() - t0;  // published by the done flag below
                }
            }
            {
                std::lock_guard<std::mutex> lk(j->mu);
                j->rc = rc;
                if (rc) j->err = g_last_error;  // the worker's thread-local message
                j->done = true;
                j->cv.notify_all();
            }
            std::lock_guard<std::mutex> lk(mu);
            inflight--;
            cv.notify_all();
        }
    }
    // Thread exit: finish every submitted job (they write the callers'
    // buffers), then stop.  Each job holds an ExitGuard, so a process exit
    // that overlaps this join waits for the job in progress, and the jobs
    // after it fail at once without touching HIP (see at_process_exit).
    ~StageWorker() {
        if (!th.joinable()) return;
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        cv.notify_all();
        th.join();
    }
};
thread_local StageWorker t_stage;
// This thread has started asynchronous requests that mi_thread_sync has not
// yet waited for.
thread_local bool t_async_issued = false;

// A split job, on the staging worker: the GPU part is started from here (a
// pageable one is staged by this thread's own worker, one level down), the
// head is folded on this thread meanwhile, then the GPU part is waited for.
// The head runs in ~8 MiB chunks (multiples of 256 elements, so none holds a
// keep-precision truncated tail), polling the GPU part between them: both
// parts' durations are known even when the GPU finishes first, and the
// caller adapts its share from them (mi_request_split_times).

int run_split(AsyncJob& j) {
    const size_t es = dtype_size(j.dt);
    const void* tail_in[MI_MAX_INPUTS];
    for (int i = 0; i < j.k; i++) tail_in[i] = static_cast<const char*>(j.inputs[i]) + j.head * es;
    mi_request_t r = nullptr;
    const double t0 = mono_s();
    if (int rc = mi_reduce_start(tail_in, j.k, static_cast<char*>(j.out) + j.head * es, j.count - j.head, j.dt, j.op,
                                 j.flags, j.device, &r))
        return rc;
    size_t chunk = std::max<size_t>(256, ((size_t)8 << 20) / es);
    chunk -= chunk % 256;
    int hrc = 0;
    double t_tail = -1.0;
    for (size_t b = 0; b < j.head && hrc == 0; b += chunk) {
        const void* hin[MI_MAX_INPUTS];
        for (int i = 0; i < j.k; i++) hin[i] = static_cast<const char*>(j.inputs[i]) + b * es;
        hrc = j.head_fold(hin, j.k, static_cast<char*>(j.out) + b * es, std::min(chunk, j.head - b), j.dt, j.op,
                          j.flags);
        int done = 0;
        if (t_tail < 0 && mi_test(r, &done) == 0 && done) t_tail = mono_s() - t0;
    }
    const double t_head = mono_s() - t0;
    const int wrc = mi_wait(r);
    if (t_tail < 0) t_tail = mono_s() - t0;
    (void)mi_request_free(r);
    if (wrc) return wrc;
    if (hrc) return fail(hrc, "host fold of the split's head");
    j.t_head = t_head;  // published to the caller by the job's done flag (under its mutex)
    j.t_tail = t_tail;
    return 0;
}

// Events behind the work the calling thread has queued on its own streams
// (every device it used); streams that are already idle need none.
std::vector<hipEvent_t> record_prior() {
    std::vector<hipEvent_t> evs;
    int prev = -1;
    for (DevCtx* d : t_ctx.devs) {
        if (!d) continue;
        for (int s = 0; s < 2; s++) {
            if (!d->stream[s]) continue;
            const hipError_t q = hipStreamQuery(d->stream[s]);
            if (q == hipSuccess) continue;
            (void)hipGetLastError();
            if (prev < 0 && hipGetDevice(&prev) != hipSuccess) prev = -1;
            hipEvent_t e = nullptr;
            if (hipSetDevice(d->device) != hipSuccess ||
                hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
                for (hipEvent_t x : evs) (void)hipEventDestroy(x);
                if (prev >= 0) (void)hipSetDevice(prev);
                throw std::runtime_error("cannot create an ordering event");
            }
            if (hipEventRecord(e, d->stream[s]) != hipSuccess) {
                (void)hipEventDestroy(e);
                (void)hipStreamSynchronize(d->stream[s]);  // order by waiting instead
                continue;
            }
            evs.push_back(e);
        }
    }
    if (prev >= 0) (void)hipSetDevice(prev);
    return evs;
}

// A staged job for the fold out = inputs[0..k-1] (run by a StageWorker);
// `ordered`: it first waits for the work this thread already queued on its
// own streams (record_prior).
std::shared_ptr<AsyncJob> make_job(const void* const* inputs, int k, void* out, size_t count, int dt, int op,
                                   unsigned flags, int device, bool ordered) {
    auto j = std::make_shared<AsyncJob>();
    if (ordered) j->prior = record_prior();
    for (int i = 0; i < k; i++) j->inputs[i] = inputs[i];
    j->k = k;
    j->out = out;
    j->count = count;
    j->dt = dt;
    j->op = op;
    j->flags = flags;
    j->device = device;
    if (device < 0 && hipGetDevice(&j->caller_device) != hipSuccess) {
        (void)hipGetLastError();
        j->caller_device = -1;
    }
    return j;
}

// Does a fold over these operands need host staging (pageable operands, or
// pinned ones under MI_HOST_STAGED)?
bool needs_staging(const void* const* inputs, int k, const void* out, size_t bytes) {
    const bool staged_mode = host_mode() == MI_HOST_STAGED;
    for (int i = 0; i <= k; i++) {
        int dev = -1;
        const PtrKind kind = classify(i < k ? inputs[i] : out, &dev, nullptr, bytes);
        if (kind == PK_PAGEABLE || (kind == PK_PINNED && staged_mode)) return true;
    }
    return false;
}

// ---------------------------------------------------------------------------
// conversions
// ---------------------------------------------------------------------------
typedef hipError_t (*ConvFn)(dim3, hipStream_t, const CArgs&, unsigned lds);

// One-wave blocks, 21 resident per CU (round 3's cap of 24 as allocated), as the 2-input reduce: 2^28 fp32 ->
// bf16 0.253 -> 0.243 ms, bf16 -> fp32 0.262 -> 0.239 ms against round 2's
// 256-lane blocks (tools/occupancy_sweep.hip copyconv, profiles/round3_occupancy/).
constexpr int kConvBlock = 64;

template <typename ST, typename DT, unsigned V, bool SC1 = false>
hipError_t conv_one(dim3 grid, hipStream_t s, const CArgs& a, unsigned lds) {
    hipLaunchKernelGGL((convert_kernel<ST, DT, V, kConvBlock, SC1>), grid, dim3(kConvBlock), lds, s, a);
    return hipGetLastError();
}

// Narrowing conversions of at least kConvStreamBytes of source store with
// sc1 + nt (the line leaves L2 as it is written): 2^28 fp32 -> bf16 0.2430 ->
// 0.2388 ms; widening ones do not (bf16 -> fp32 0.2415 -> 0.2464 ms)
// (tools/occupancy_sweep.hip copyconv, profiles/round5_run20/).
constexpr size_t kConvStreamBytes = 64ull << 20;

template <bool SC1>
ConvFn pick_narrowing(int ddt, unsigned f) {
    if (ddt == MI_BFLOAT16) {
        if (!(f & V_BF16_RNE)) return &conv_one<float, bf16_tag, 0u, SC1>;
        return (f & V_TAIL_TRUNC) ? &conv_one<float, bf16_tag, V_BF16_RNE | V_TAIL_TRUNC, SC1>
                                  : &conv_one<float, bf16_tag, V_BF16_RNE, SC1>;
    }
    return &conv_one<float, fp16_tag, 0u, SC1>;
}

ConvFn pick_conv(int sdt, int ddt, unsigned f, bool streaming = false) {
    if (sdt == MI_FLOAT32 && (ddt == MI_BFLOAT16 || ddt == MI_FLOAT16))
        return streaming ? pick_narrowing<true>(ddt, f) : pick_narrowing<false>(ddt, f);
    if (sdt == MI_BFLOAT16 && ddt == MI_FLOAT32) return &conv_one<bf16_tag, float, 0u>;
    if (sdt == MI_FLOAT16 && ddt == MI_FLOAT32) return &conv_one<fp16_tag, float, 0u>;
    return nullptr;
}

int launch_convert(const void* src, int sdt, void* dst, int ddt, size_t count, unsigned flags, hipStream_t s,
                   uint64_t trunc_from) {
    ConvFn fn = pick_conv(sdt, ddt, flags, count * dtype_size(sdt) >= kConvStreamBytes);
    if (!fn) return fail(MI_E_UNSUPPORTED, "conversion pair not supported (fp32<->bf16, fp32<->fp16)");
    if (count == 0) return 0;
    if (!src || !dst) return fail(MI_E_INVALID, "null pointer");
    if (int rc = require_gpu_visible(src, count * dtype_size(sdt))) return rc;
    if (int rc = require_gpu_visible(dst, count * dtype_size(ddt))) return rc;
    CArgs a;
    memset(&a, 0, sizeof(a));
    a.src = src;
    a.dst = dst;
    a.count = count;
    a.trunc_from = trunc_from;
    // vector path on dst's 16-byte grid (as launch_reduce): both pointers
    // aligned to their element size; the source may sit at any such offset
    const size_t ss = dtype_size(sdt), ds = dtype_size(ddt);
    const uintptr_t sa = reinterpret_cast<uintptr_t>(src), da = reinterpret_cast<uintptr_t>(dst);
    const bool same = (sa & 15u) == 0 && (da & 15u) == 0;
    const bool vec = (sa % ss) == 0 && (da % ds) == 0 && (same || unaligned_vectors());
    a.scalar_only = vec ? 0 : 1;
    a.head = vec ? std::min<uint64_t>(((16 - (da & 15u)) & 15u) / ds, count) : 0;
    a.ngroups = vec ? (count - a.head) / 8 : 0;
    const uint64_t work = a.scalar_only ? count : std::max<uint64_t>(a.ngroups, 1);
    uint64_t blocks = std::min<uint64_t>((work + kConvBlock - 1) / kConvBlock, 1u << 20);
    const int cap = max_blocks();  // a grid cap (mi_set_max_blocks) makes the kernel stride
    if (cap > 0) blocks = std::min<uint64_t>(blocks, (uint64_t)cap);
    blocks = std::max<uint64_t>(blocks, 1);
    hipError_t e = fn(dim3((unsigned)blocks), s, a, wave_cap_lds(s, planned_waves(0)));
    if (e != hipSuccess) return hip_fail(e, "convert kernel launch");
    return 0;
}

}  // namespace

// Host-side failures (a thread, allocation or lock that cannot be had) are
// C++ exceptions; none may cross the C ABI.  They become MI_E_RESOURCE.
template <typename F>
int guarded(F&& f) {
    try {
        return f();
    } catch (const std::exception& e) {
        return fail(MI_E_RESOURCE, e.what());
    } catch (...) {
        return fail(MI_E_RESOURCE, "unexpected host-side exception");
    }
}

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

int mi_reduce(const void* in, void* inout, size_t count, int dtype, int op, unsigned flags,
              void* stream) {
    const void* ins[2] = {inout, in};
    return launch_reduce(ins, 2, inout, count, dtype, op, flags, (hipStream_t)stream);
}

int mi_reduce_out(const void* in1, const void* in2, void* out, size_t count, int dtype, int op,
                  unsigned flags, void* stream) {
    const void* ins[2] = {in2, in1};
    return launch_reduce(ins, 2, out, count, dtype, op, flags, (hipStream_t)stream);
}

int mi_reduce_multi(const void* const* inputs, int k, void* out, size_t count, int dtype, int op,
                    unsigned flags, void* stream) {
    if (!inputs) return fail(MI_E_INVALID, "null input list");
    return launch_reduce(inputs, k, out, count, dtype, op, flags, (hipStream_t)stream);
}

int mi_reduce_batch(const mi_reduce_desc_t* descs, int n, int dtype, int op, unsigned flags,
                    void* stream) {
    return guarded([&]() -> int { return launch_reduce_batch(descs, n, dtype, op, flags, (hipStream_t)stream); });
}

namespace {
// A staged bucket from a caller confined to one or two CPUs -- oneCCL pins
// each worker to one core (CCL_WORKER_AFFINITY, src/exec/thread/worker.cpp:
// 310-379) -- runs on the thread's staging worker, which has the process's
// CPU set, while the caller waits.  The runtime pins pageable pages in place
// on the thread that issues the copy; confined to one core the staged
// pipeline ran at 17-21 GiB/s of bucket against 24 unconfined
// (profiles/round5_run12/host_leg_pin_ab.jsonl).  Below the bounce size the
// CPU copies into pinned buffers on the caller, as before.
// MI_REDUCE_CONFINED_HANDOFF=0 turns it off.
bool handoff_enabled() {
    static const bool on = [] {
        const char* e = getenv("MI_REDUCE_CONFINED_HANDOFF");
        return !(e && strcmp(e, "0") == 0);
    }();
    return on;
}

// some operand is pageable host memory (what the runtime pins in place)
bool any_pageable(const Kinds& c, int k) {
    if (c.kout == PK_PAGEABLE) return true;
    for (int i = 0; i < k; i++)
        if (c.kin[i] == PK_PAGEABLE) return true;
    return false;
}

bool confined_caller() {
    if (!handoff_enabled() || !g_helper_cpus.use) return false;
    cpu_set_t m;
    CPU_ZERO(&m);
    if (sched_getaffinity(0, sizeof(m), &m) != 0) return false;
    const int n = CPU_COUNT(&m);
    return n <= 2 && CPU_COUNT(&g_helper_cpus.mask) > n;
}

int sync_entry(const void* const* inputs, int k, void* out, size_t count, int dtype, int op, unsigned flags,
               int device) {
    t_stage.wait_idle();  // this thread's earlier asynchronous requests come first
    const size_t es = dtype_size(dtype);
    if (es && count * es > kBounceBytes && k >= 1 && k <= MI_MAX_INPUTS && out && confined_caller()) {
        bool nonnull = true;
        for (int i = 0; i < k; i++) nonnull = nonnull && inputs[i];
        if (nonnull) {
            // classified once here; the staging worker (or this thread) reuses it
            Kinds c;
            classify_all(inputs, k, out, count * es, &c);
            if (!any_pageable(c, k)) return reduce_sync(inputs, k, out, count, dtype, op, flags, device, &c);
            auto j = make_job(inputs, k, out, count, dtype, op, flags, device, true);
            j->kinds = c;
            t_stage.submit(j);
            const int rc = j->wait();
            return rc ? fail(rc, j->err.c_str()) : 0;
        }
    }
    return reduce_sync(inputs, k, out, count, dtype, op, flags, device);
}

}  // namespace

int mi_reduce_sync(const void* in, void* inout, size_t count, int dtype, int op, unsigned flags,
                   int device) {
    return guarded([&]() -> int {
        const void* ins[2] = {inout, in};
        return sync_entry(ins, 2, inout, count, dtype, op, flags, device);
    });
}

int mi_reduce_multi_sync(const void* const* inputs, int k, void* out, size_t count, int dtype,
                         int op, unsigned flags, int device) {
    return guarded([&]() -> int {
        if (!inputs) return fail(MI_E_INVALID, "null input list");
        return sync_entry(inputs, k, out, count, dtype, op, flags, device);
    });
}

int mi_convert(const void* src, int src_dtype, void* dst, int dst_dtype, size_t count, unsigned flags,
               void* stream) {
    return launch_convert(src, src_dtype, dst, dst_dtype, count, flags, (hipStream_t)stream, (count / 16) * 16);
}

int mi_convert_sync(const void* src, int src_dtype, void* dst, int dst_dtype, size_t count, unsigned flags,
                    int device) {
    return guarded([&]() -> int {
        t_stage.wait_idle();  // this thread's earlier asynchronous requests come first
        if (!pick_conv(src_dtype, dst_dtype, flags))
            return fail(MI_E_UNSUPPORTED, "conversion pair not supported (fp32<->bf16, fp32<->fp16)");
        if (count == 0) return 0;
        if (!src || !dst) return fail(MI_E_INVALID, "null pointer");
        int pdev = -1;
        const PtrKind ks = classify(src, &pdev, nullptr, count * dtype_size(src_dtype)),
                      kd = classify(dst, &pdev, nullptr, count * dtype_size(dst_dtype));
        if (device < 0 && pdev >= 0) device = pdev;
        DevCtx* d = nullptr;
        int rc = get_ctx(device, &d);
        if (rc) return rc;
        int prev = 0;
        MI_HIP(hipGetDevice(&prev));
        if (prev != d->device) MI_HIP(hipSetDevice(d->device));
        struct Restore {
            int dev, cur;
            ~Restore() {
                if (dev != cur) (void)hipSetDevice(dev);
            }
        } restore{prev, d->device};
        const uint64_t trunc_from = (count / 16) * 16;
        if (ks == PK_DEVICE && kd == PK_DEVICE) {
            rc = launch_convert(src, src_dtype, dst, dst_dtype, count, flags, d->stream[0], trunc_from);
            if (rc) return rc;
            MI_HIP(wait_stream(d->stream[0]));
            return 0;
        }
        const size_t ss = dtype_size(src_dtype), ds = dtype_size(dst_dtype);
        size_t chunk = kChunkBytes / std::max(ss, ds);
        chunk -= chunk % 16;
        rc = ensure_scratch(d, 2, chunk * std::max(ss, ds) + kStageSlack);
        if (rc) return rc;
        Edges edges;  // unaligned ends of D2H copies into pageable memory (d2h_pageable)
        if (kd == PK_PAGEABLE) {
            rc = ensure_edges(d);
            if (rc) return rc;
            edges.pin = d->edge;
            edges.slots = kDrainEdge / kEdgeSlot;
        }
        for (size_t off = 0, c = 0; off < count; off += chunk, c++) {
            const int sl = (int)(c & 1);
            hipStream_t st = d->stream[sl];
            const size_t n = std::min(chunk, count - off);
            const void* sp = static_cast<const char*>(src) + off * ss;
            void* dp = static_cast<char*>(dst) + off * ds;
            const void* dsrc = sp;
            void* ddst = dp;
            if (ks != PK_DEVICE) {
                size_t sh = 0;
                if (hipError_t he = h2d_stage(d->dbuf[sl][0], sp, n * ss, st, &sh))
                    return copy_fail(he, "H2D staging copy (conversion)", sp, n * ss, c, ks, true);
                dsrc = static_cast<const char*>(d->dbuf[sl][0]) + sh;
            }
            if (kd != PK_DEVICE)
                ddst = static_cast<char*>(d->dbuf[sl][1]) + (reinterpret_cast<uintptr_t>(dp) & (kHostAlign - 1));
            // chunk starts are multiples of 16: the tail split is the global one
            rc = launch_convert(dsrc, src_dtype, ddst, dst_dtype, n, flags, st,
                                trunc_from > off ? std::min<uint64_t>(trunc_from - off, n) : 0);
            if (rc) return rc;
            if (kd == PK_PAGEABLE) {
                if (edges.full()) {
                    MI_HIP(wait_stream(d->stream[0]));
                    MI_HIP(wait_stream(d->stream[1]));
                    edges.flush();
                }
                if (hipError_t he = d2h_pageable(dp, ddst, n * ds, st, edges))
                    return copy_fail(he, "D2H result copy (conversion)", dp, n * ds, c, kd, false);
            } else if (kd != PK_DEVICE) {
                if (hipError_t he = hipMemcpyAsync(dp, ddst, n * ds, hipMemcpyDeviceToHost, st))
                    return copy_fail(he, "D2H result copy (conversion)", dp, n * ds, c, kd, true);
            }
        }
        MI_HIP(wait_stream(d->stream[0]));
        MI_HIP(wait_stream(d->stream[1]));
        edges.flush();
        return 0;
    });
}

// ---- asynchronous requests ------------------------------------------------
struct mi_request {
    hipEvent_t ev[2] = {nullptr, nullptr};
    int nev = 0;
    int device = -1;
    hipEvent_t t0 = nullptr;        // timed direct request: recorded before its launch (ev[0] ends it)
    std::shared_ptr<AsyncJob> job;  // staged work running on the calling thread's worker
};

namespace {
int reduce_start(const void* const* inputs, int k, void* out, size_t count, int dtype, int op, unsigned flags,
                 int device, mi_request_t* req, bool timed) {
    return guarded([&]() -> int {
        if (!req) return fail(MI_E_INVALID, "null request pointer");
        *req = nullptr;
        if (!inputs) return fail(MI_E_INVALID, "null input list");
        t_async_issued = true;
        if (!dtype_size(dtype)) return fail(MI_E_INVALID, "unknown datatype");
        if (k < 1 || k > MI_MAX_INPUTS) return fail(MI_E_INVALID, "input count out of range [1,16]");
        if (count > 0) {
            if (!out) return fail(MI_E_INVALID, "null output");
            for (int i = 0; i < k; i++)
                if (!inputs[i]) return fail(MI_E_INVALID, "null input");
            if (op < MI_OP_SUM || op > MI_OP_MAX)
                return fail(MI_E_INVALID, "unsupported reduction (device path: sum/prod/min/max)");
            // Staged work runs on the calling thread's worker.  While that
            // worker still has requests of this thread, later requests go
            // there too, so a thread's requests run in submission order
            // whatever their pointer kinds.
            if (needs_staging(inputs, k, out, count * dtype_size(dtype)) || t_stage.busy()) {
                auto j = make_job(inputs, k, out, count, dtype, op, flags, device, true);
                t_stage.submit(j);
                mi_request* r = new mi_request();
                r->job = j;
                *req = r;
                return 0;
            }
        }
        DevCtx* d = nullptr;
        int used = 0;
        hipEvent_t t0 = nullptr;
        int rc = reduce_issue(inputs, k, out, count, dtype, op, flags, device, &d, &used, nullptr, nullptr,
                              timed ? &t0 : nullptr);
        if (rc) {
            if (t0) (void)hipEventDestroy(t0);
            return rc;
        }
        mi_request* r = new mi_request();
        r->t0 = t0;
        if (d) {
            r->device = d->device;
            int prev = 0;
            MI_HIP(hipGetDevice(&prev));
            if (prev != d->device) MI_HIP(hipSetDevice(d->device));
            for (int s = 0; s < 2 && rc == 0; s++) {
                if (!(used & (1 << s))) continue;
                hipError_t e = hipEventCreateWithFlags(&r->ev[r->nev], t0 ? hipEventDefault : hipEventDisableTiming);
                if (e == hipSuccess) e = hipEventRecord(r->ev[r->nev], d->stream[s]);
                if (e != hipSuccess) rc = hip_fail(e, "hipEventRecord");
                r->nev++;
            }
            if (prev != d->device) (void)hipSetDevice(prev);
        }
        if (rc) {
            mi_request_free(r);
            return rc;
        }
        *req = r;
        return 0;
    });
}
}  // namespace

int mi_reduce_start(const void* const* inputs, int k, void* out, size_t count, int dtype, int op,
                    unsigned flags, int device, mi_request_t* req) {
    return reduce_start(inputs, k, out, count, dtype, op, flags, device, req, false);
}

int mi_reduce_start_timed(const void* const* inputs, int k, void* out, size_t count, int dtype, int op,
                          unsigned flags, int device, mi_request_t* req) {
    return reduce_start(inputs, k, out, count, dtype, op, flags, device, req, true);
}

int mi_request_run_time(mi_request_t req, double* seconds) {
    if (!req || !seconds) return fail(MI_E_INVALID, "null argument");
    if (req->job) {
        std::lock_guard<std::mutex> lk(req->job->mu);
        if (!req->job->done || req->job->rc || req->job->t_run < 0) return fail(MI_E_INVALID, "request not finished");
        *seconds = req->job->t_run;
        return 0;
    }
    if (!req->t0 || req->nev != 1) return fail(MI_E_INVALID, "not a timed request");
    float ms = 0;
    const hipError_t e = hipEventElapsedTime(&ms, req->t0, req->ev[0]);
    if (e == hipErrorNotReady) {
        (void)hipGetLastError();
        return fail(MI_E_INVALID, "request not finished");
    }
    if (e != hipSuccess) return hip_fail(e, "hipEventElapsedTime");
    *seconds = ms * 1e-3;
    return 0;
}

int mi_reduce_split_start(const void* const* inputs, int k, void* out, size_t count, int dtype, int op,
                          unsigned flags, int device, size_t head_count, mi_host_fold_t head_fold,
                          mi_request_t* req) {
    if (head_count == 0 || count == 0) return mi_reduce_start(inputs, k, out, count, dtype, op, flags, device, req);
    return guarded([&]() -> int {
        if (!req) return fail(MI_E_INVALID, "null request pointer");
        *req = nullptr;
        if (!inputs) return fail(MI_E_INVALID, "null input list");
        if (!head_fold) return fail(MI_E_INVALID, "null head fold");
        if (head_count >= count) return fail(MI_E_INVALID, "head_count must leave a GPU part");
        if (!dtype_size(dtype)) return fail(MI_E_INVALID, "unknown datatype");
        if (k < 1 || k > MI_MAX_INPUTS) return fail(MI_E_INVALID, "input count out of range [1,16]");
        if (!out) return fail(MI_E_INVALID, "null output");
        for (int i = 0; i < k; i++)
            if (!inputs[i]) return fail(MI_E_INVALID, "null input");
        if (op < MI_OP_SUM || op > MI_OP_MAX)
            return fail(MI_E_INVALID, "unsupported reduction (device path: sum/prod/min/max)");
        t_async_issued = true;
        auto j = make_job(inputs, k, out, count, dtype, op, flags, device, true);
        j->head = head_count;
        j->head_fold = head_fold;
        t_stage.submit(j);
        mi_request* r = new mi_request();
        r->job = j;
        *req = r;
        return 0;
    });
}

int mi_request_split_times(mi_request_t req, double* head_s, double* tail_s) {
    if (!req || !head_s || !tail_s) return fail(MI_E_INVALID, "null argument");
    if (!req->job || !req->job->head_fold) return fail(MI_E_INVALID, "not a split request");
    std::lock_guard<std::mutex> lk(req->job->mu);
    if (!req->job->done || req->job->rc || req->job->t_head < 0) return fail(MI_E_INVALID, "split not finished");
    *head_s = req->job->t_head;
    *tail_s = req->job->t_tail;
    return 0;
}

int mi_test(mi_request_t req, int* done) {
    if (!req || !done) return fail(MI_E_INVALID, "null request");
    if (req->job) {
        std::lock_guard<std::mutex> lk(req->job->mu);
        *done = req->job->done ? 1 : 0;
        if (req->job->done && req->job->rc) return fail(req->job->rc, req->job->err.c_str());
        return 0;
    }
    *done = 1;
    for (int i = 0; i < req->nev; i++) {
        const hipError_t e = hipEventQuery(req->ev[i]);
        if (e == hipErrorNotReady) {
            (void)hipGetLastError();
            *done = 0;
        } else if (e != hipSuccess) {
            return hip_fail(e, "hipEventQuery");
        }
    }
    return 0;
}

int mi_wait(mi_request_t req) {
    if (!req) return fail(MI_E_INVALID, "null request");
    if (req->job) {
        const int rc = req->job->wait();
        return rc ? fail(rc, req->job->err.c_str()) : 0;
    }
    for (int i = 0; i < req->nev; i++) MI_HIP(hipEventSynchronize(req->ev[i]));
    return 0;
}

int mi_request_free(mi_request_t req) {
    if (!req) return 0;
    if (req->job) (void)req->job->wait();  // the job writes the caller's buffers: never leave it running
    for (int i = 0; i < req->nev; i++)
        if (req->ev[i]) (void)hipEventDestroy(req->ev[i]);
    if (req->t0) (void)hipEventDestroy(req->t0);
    delete req;
    return 0;
}

// ---- one bucket split over several GPUs, any pointer kinds -----------------
int mi_reduce_multi_sync_sharded(const void* const* inputs, int k, void* out, size_t count, int dtype, int op,
                                 unsigned flags, int nshards, const int* devices) {
    return guarded([&]() -> int {
        t_stage.wait_idle();  // this thread's earlier asynchronous requests come first
        if (!inputs || !devices || nshards < 1) return fail(MI_E_INVALID, "bad shard arguments");
        if (k < 1 || k > MI_MAX_INPUTS) return fail(MI_E_INVALID, "input count out of range [1,16]");
        const size_t es = dtype_size(dtype);
        if (!es) return fail(MI_E_INVALID, "unknown datatype");
        if (nshards == 1 || count == 0) return reduce_sync(inputs, k, out, count, dtype, op, flags, devices[0]);
        // Shards start on 256-element boundaries, so the bf16 count % 16 tail
        // (MI_F_BF16_TAIL_TRUNC16) lies in the last shard exactly as in the
        // whole array.  Shard 0 runs on the calling thread, the others on
        // workers owned by it (one per shard slot, persistent streams/staging).
        thread_local std::vector<std::unique_ptr<StageWorker>> t_shard_workers;
        while ((int)t_shard_workers.size() < nshards - 1) t_shard_workers.emplace_back(new StageWorker());
        const size_t per = ((count + (size_t)nshards - 1) / (size_t)nshards + 255) / 256 * 256;
        std::vector<std::shared_ptr<AsyncJob>> jobs;
        // Every shard already submitted finishes before this call returns on
        // any path, a throw included: they write the caller's `out`.
        struct WaitAll {
            std::vector<std::shared_ptr<AsyncJob>>& jobs;
            ~WaitAll() {
                for (auto& j : jobs) (void)j->wait();
            }
        } wait_all{jobs};
        for (int sh = 1; sh < nshards; sh++) {
            const size_t b = std::min(count, per * (size_t)sh), e = std::min(count, b + per);
            if (b >= e) break;
            const void* sins[MI_MAX_INPUTS];
            for (int i = 0; i < k; i++) sins[i] = static_cast<const char*>(inputs[i]) + b * es;
            auto j = make_job(sins, k, static_cast<char*>(out) + b * es, e - b, dtype, op, flags, devices[sh], false);
            jobs.push_back(j);
            try {
                t_shard_workers[sh - 1]->submit(j);
            } catch (...) {
                jobs.pop_back();  // never queued: nothing to wait for
                throw;
            }
        }
        const int rc0 = reduce_sync(inputs, k, out, std::min(count, per), dtype, op, flags, devices[0]);
        std::string err0 = rc0 ? g_last_error : std::string();
        int rc = rc0;
        for (auto& j : jobs) {
            const int r = j->wait();  // every shard finishes before the call returns
            if (r && !rc) {
                rc = r;
                err0 = j->err;
            }
        }
        return rc ? fail(rc, err0.c_str()) : 0;
    });
}

// ---- in-process multi-GPU element-range shards -------------------------------
int mi_reduce_sharded(int nshards, const int* devices, const void* const* inputs, int k, void* const* outs,
                      const size_t* counts, int dtype, int op, unsigned flags) {
    return guarded([&]() -> int {
        if (nshards < 1 || !devices || !inputs || !outs || !counts) return fail(MI_E_INVALID, "bad shard arguments");
        if (k < 1 || k > MI_MAX_INPUTS) return fail(MI_E_INVALID, "input count out of range [1,16]");
        int prev = 0;
        MI_HIP(hipGetDevice(&prev));
        std::vector<DevCtx*> ctx((size_t)nshards, nullptr);
        int rc = 0;
        // launch every shard before waiting for any
        for (int s = 0; s < nshards && rc == 0; s++) {
            rc = get_ctx(devices[s], &ctx[s]);
            if (rc) break;
            hipError_t e = hipSetDevice(devices[s]);
            if (e != hipSuccess) {
                rc = hip_fail(e, "hipSetDevice");
                break;
            }
            rc = launch_reduce(inputs + (size_t)s * k, k, outs[s], counts[s], dtype, op, flags, ctx[s]->stream[0]);
        }
        for (int s = 0; s < nshards; s++) {
            if (!ctx[s]) continue;
            (void)hipSetDevice(devices[s]);
            const hipError_t e = wait_stream(ctx[s]->stream[0]);
            if (e != hipSuccess && rc == 0) rc = hip_fail(e, "hipStreamSynchronize");
        }
        (void)hipSetDevice(prev);
        return rc;
    });
}

// Copies of at least kCopyStreamBytes store with sc1 + nt (each line leaves
// L2 as it is written, as reduce2_kernel's stores), with no residency cap:
// one-wave copies of 1 GiB, uncapped, 0.3204 / 0.3168 ms on two boxes
// against 0.3240 for the library's nt loads + plain stores and 0.3211 with
// nt stores (box 1); a 25-wave cap won on one box (0.3186) and lost on the
// other (0.3205), so none (tools/copy_ab.py, profiles/round5_run17/).  Below
// the threshold the lines a copy writes may be read next from L2 or the
// MALL, so plain stores (or nt, when the caller asks) stay.
constexpr size_t kCopyStreamBytes = 64ull << 20;

int mi_copy(const void* src, void* dst, size_t bytes, int nontemporal, void* stream) {
    if (bytes == 0) return 0;
    if (!src || !dst) return fail(MI_E_INVALID, "null pointer");
    // the whole extent: a pinned operand must lie inside one pinned allocation
    if (int rc = require_gpu_visible(src, bytes)) return rc;
    if (int rc = require_gpu_visible(dst, bytes)) return rc;
    hipStream_t s = (hipStream_t)stream;
    // the destination's 16-byte grid; the source may be at any offset from it
    const uint32_t head = (uint32_t)std::min<size_t>((16 - (reinterpret_cast<uintptr_t>(dst) & 15u)) & 15u, bytes);
    const uint64_t nvec = (bytes - head) / 16;
    const uint32_t tail = (uint32_t)(bytes - head - nvec * 16);
    const char* s8 = static_cast<const char*>(src);
    char* d8 = static_cast<char*>(dst);
    // loads are non-temporal either way (each byte is read once); `nontemporal`
    // picks the stores, as the reference's flag picks its memcpy
    const int cap = max_blocks();
    const uint64_t lean_blocks = (nvec + kCopyBlock - 1) / kCopyBlock;
    if (cap <= 0 && lean_blocks <= 0x7FFFFFFFull) {
        const unsigned blocks = (unsigned)std::max<uint64_t>(lean_blocks, 1);
        if (bytes >= kCopyStreamBytes)  // far past the caches: either flag streams
            hipLaunchKernelGGL(copy_lean_kernel<5>, dim3(blocks), dim3(kCopyBlock), 0, s, s8, d8, head, nvec, tail);
        else if (nontemporal)
            hipLaunchKernelGGL(copy_lean_kernel<3>, dim3(blocks), dim3(kCopyBlock), 0, s, s8, d8, head, nvec, tail);
        else
            hipLaunchKernelGGL(copy_lean_kernel<1>, dim3(blocks), dim3(kCopyBlock), 0, s, s8, d8, head, nvec, tail);
        MI_HIP(hipGetLastError());
        return 0;
    }
    const uint64_t tile = (uint64_t)kBlock * 4;
    uint64_t blocks = (nvec + tile - 1) / tile;
    if (cap > 0) blocks = std::min<uint64_t>(blocks, (uint64_t)cap);
    blocks = std::min<uint64_t>(std::max<uint64_t>(blocks, 1), 0x7FFFFFFFull);
    if (nontemporal)
        hipLaunchKernelGGL(copy_kernel<3>, dim3((unsigned)blocks), dim3(kBlock), 0, s, s8, d8, head, nvec, tail);
    else
        hipLaunchKernelGGL(copy_kernel<1>, dim3((unsigned)blocks), dim3(kBlock), 0, s, s8, d8, head, nvec, tail);
    MI_HIP(hipGetLastError());
    return 0;
}

int mi_copy_sync(const void* src, void* dst, size_t bytes, int nontemporal, int device) {
    return guarded([&]() -> int {
        t_stage.wait_idle();  // this thread's earlier asynchronous requests come first
        if (bytes == 0) return 0;
        if (!src || !dst) return fail(MI_E_INVALID, "null pointer");
        int pdev = -1;
        const PtrKind ks = classify(src, &pdev, nullptr, bytes), kd = classify(dst, &pdev, nullptr, bytes);
        if (device < 0 && pdev >= 0) device = pdev;
        DevCtx* d = nullptr;
        int rc = get_ctx(device, &d);
        if (rc) return rc;
        if (ks == PK_DEVICE && kd == PK_DEVICE) {
            int prev = 0;
            MI_HIP(hipGetDevice(&prev));
            if (prev != d->device) MI_HIP(hipSetDevice(d->device));
            rc = mi_copy(src, dst, bytes, nontemporal, d->stream[0]);
            if (!rc) {
                hipError_t e = wait_stream(d->stream[0]);
                if (e != hipSuccess) rc = hip_fail(e, "hipStreamSynchronize");
            }
            if (prev != d->device) (void)hipSetDevice(prev);
            return rc;
        }
        if (ks != PK_DEVICE && kd != PK_DEVICE) {  // host to host: the CPU's copy
            memcpy(dst, src, bytes);
            return 0;
        }
        int prev = 0;
        MI_HIP(hipGetDevice(&prev));
        if (prev != d->device) MI_HIP(hipSetDevice(d->device));
        struct Restore {
            int dev, cur;
            ~Restore() {
                if (dev != cur) (void)hipSetDevice(dev);
            }
        } restore{prev, d->device};
        hipStream_t st = d->stream[0];
        if (ks == PK_PAGEABLE || kd == PK_PAGEABLE) {  // the runtime gets aligned host spans only (h2d_stage)
            rc = ensure_edges(d);
            if (rc) return rc;
            Edges edges;
            edges.pin = d->edge;
            edges.slots = 1;
            if (kd == PK_PAGEABLE) {
                if (hipError_t he = d2h_pageable(dst, src, bytes, st, edges))
                    return copy_fail(he, "D2H copy (mi_copy_sync)", dst, bytes, 0, kd, false);
                MI_HIP(wait_stream(st));
                edges.flush();
                return 0;
            }
            // pageable -> device: the ends through pinned scratch, the aligned interior direct
            const uintptr_t a = reinterpret_cast<uintptr_t>(src);
            const size_t head = std::min(bytes, (size_t)(host_align_up(a) - a));
            const size_t interior = (bytes - head) & ~(size_t)(kHostAlign - 1);
            const size_t tail = bytes - head - interior;
            const char* s8 = static_cast<const char*>(src);
            char* d8 = static_cast<char*>(dst);
            if (head) {
                memcpy(edges.pin, s8, head);
                MI_HIP(hipMemcpyAsync(d8, edges.pin, head, hipMemcpyHostToDevice, st));
            }
            if (interior)
                if (hipError_t he = hipMemcpyAsync(d8 + head, s8 + head, interior, hipMemcpyHostToDevice, st))
                    return copy_fail(he, "H2D copy (mi_copy_sync)", src, bytes, 0, ks, false);
            if (tail) {
                memcpy(edges.pin + kHostAlign, s8 + head + interior, tail);
                MI_HIP(hipMemcpyAsync(d8 + head + interior, edges.pin + kHostAlign, tail, hipMemcpyHostToDevice, st));
            }
            MI_HIP(wait_stream(st));
            return 0;
        }
        MI_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, st));
        MI_HIP(wait_stream(st));
        return 0;
    });
}

int mi_thread_sync(void) {
    return guarded([&]() -> int {
        if (!t_async_issued) return 0;
        t_stage.wait_idle();
        for (DevCtx* d : t_ctx.devs) {
            if (!d) continue;
            for (int s = 0; s < 2; s++)
                if (d->stream[s]) MI_HIP(hipStreamSynchronize(d->stream[s]));
        }
        t_async_issued = false;
        return 0;
    });
}

int mi_shard_range(size_t count, int rank, int world, size_t align, size_t* begin, size_t* end) {
    if (world < 1 || rank < 0 || rank >= world || !begin || !end) return fail(MI_E_INVALID, "bad shard arguments");
    if (align == 0) align = 256;
    size_t per = (count + (size_t)world - 1) / (size_t)world;
    per = (per + align - 1) / align * align;
    size_t b = std::min(count, per * (size_t)rank);
    size_t e = std::min(count, b + per);
    *begin = b;
    *end = e;
    return 0;
}

const char* mi_reduction_to_str(int op) {
    switch (op) {
        case MI_OP_SUM: return "sum";
        case MI_OP_PROD: return "prod";
        case MI_OP_MIN: return "min";
        case MI_OP_MAX: return "max";
        case MI_OP_CUSTOM: return "custom";
        default: return "unknown";
    }
}

// ---- pinned extents --------------------------------------------------------
// A declared range is recorded as pinned only when it lies inside one pinned
// allocation: its two ends being pinned does not make its middle pinned, and
// a kernel reading pageable pages in place faults the GPU (no XNACK).  The
// allocation is the one mi_host_register pinned, or the one HIP reports for
// the address (hipHostMalloc / a caller's own hipHostRegister).  Anything
// else is recorded as pageable, which is always safe: it is staged.
namespace {
std::mutex g_reg_mu;
std::map<uintptr_t, size_t> g_registered;  // mi_host_register: base -> bytes, under g_reg_mu

bool registered_extent(uintptr_t a, uintptr_t* lo, uintptr_t* hi) {
    std::lock_guard<std::mutex> lk(g_reg_mu);
    auto it = g_registered.upper_bound(a);
    if (it == g_registered.begin()) return false;
    --it;
    if (a - it->first >= it->second) return false;
    *lo = it->first;
    *hi = it->first + it->second;
    return true;
}

// [lo, hi): the pinned allocation holding host address a, whose device-visible
// address is a + delta
bool pinned_extent(uintptr_t a, intptr_t delta, uintptr_t* lo, uintptr_t* hi) {
    if (registered_extent(a, lo, hi)) return true;
    t_lookups++;  // one more HIP query of the pointer (mi_pointer_lookups counts it)
    void* start = nullptr;
    size_t size = 0;
    hipDeviceptr_t q = reinterpret_cast<hipDeviceptr_t>(a + delta);
    if (hipPointerGetAttribute(&start, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, q) != hipSuccess ||
        hipPointerGetAttribute(&size, HIP_POINTER_ATTRIBUTE_RANGE_SIZE, q) != hipSuccess || size == 0) {
        (void)hipGetLastError();
        return false;
    }
    const uintptr_t st = reinterpret_cast<uintptr_t>(start);
    for (const uintptr_t base : {st, st - (uintptr_t)delta})  // host or device-visible answer
        if (base <= a && a - base < size) {
            *lo = base;
            *hi = base + size;
            return true;
        }
    return false;
}

// Declared pinned ranges overlapping [lo, hi) become pageable (staged from
// then on): the memory under them is about to be unpinned.
void demote_declared(uintptr_t lo, uintptr_t hi) {
    std::lock_guard<std::mutex> lk(g_rng_mu);
    const RangeSnap* cur = g_rng.load(std::memory_order_relaxed);
    if (!cur) return;
    bool any = false;
    for (const HostRange& r : cur->r) any |= r.kind == PK_PINNED && r.lo < hi && lo < r.hi;
    if (!any) return;
    std::unique_ptr<RangeSnap> next(new RangeSnap(*cur));
    for (HostRange& r : next->r)
        if (r.kind == PK_PINNED && r.lo < hi && lo < r.hi) {
            r.kind = PK_PAGEABLE;
            r.dev_delta = 0;
        }
    publish_ranges(next.release());
}
}  // namespace

int mi_host_register(void* ptr, size_t bytes) {
    if (!ptr || !bytes) return fail(MI_E_INVALID, "null / empty buffer");
    MI_HIP(hipHostRegister(ptr, bytes, hipHostRegisterMapped | hipHostRegisterPortable));
    try {
        std::lock_guard<std::mutex> lk(g_reg_mu);
        g_registered[reinterpret_cast<uintptr_t>(ptr)] = bytes;
    } catch (const std::exception&) {
        (void)hipHostUnregister(ptr);
        return fail(MI_E_RESOURCE, "out of memory");
    }
    return 0;
}

int mi_host_unregister(void* ptr) {
    if (!ptr) return fail(MI_E_INVALID, "null buffer");
    const uintptr_t a = reinterpret_cast<uintptr_t>(ptr);
    uintptr_t lo = a, hi = a + 1;
    size_t known = 0;
    {
        std::lock_guard<std::mutex> lk(g_reg_mu);
        auto it = g_registered.find(a);
        if (it != g_registered.end()) known = it->second;
    }
    if (known) hi = a + known;
    else if (!pinned_extent(a, 0, &lo, &hi)) hi = a + 1;  // extent unknown: the ranges at ptr
    try {
        demote_declared(lo, hi);  // before the pages are unpinned
    } catch (const std::exception&) {
        return fail(MI_E_RESOURCE, "out of memory");
    }
    MI_HIP(hipHostUnregister(ptr));
    std::lock_guard<std::mutex> lk(g_reg_mu);
    g_registered.erase(a);
    return 0;
}

int mi_pointer_kind(const void* ptr, int* device) {
    int dev = -1;
    const int kind = (int)classify(ptr, &dev);
    if (device) *device = dev;
    return kind;
}

int mi_pointer_kind_range(const void* ptr, size_t bytes, int* device) {
    int dev = -1;
    const int kind = (int)classify(ptr, &dev, nullptr, bytes);
    if (device) *device = dev;
    return kind;
}

int mi_host_declare(const void* ptr, size_t bytes) {
    if (!ptr || bytes == 0) return fail(MI_E_INVALID, "null / empty range");
    const uintptr_t a = reinterpret_cast<uintptr_t>(ptr);
    if (bytes > UINTPTR_MAX - a) return fail(MI_E_INVALID, "range wraps the address space");
    // one lookup of each end, outside the writers' lock: both ends must be
    // host memory of one kind, and a pinned range one mapping
    const uintptr_t last = a + bytes - 1;
    int d0 = -1, d1 = -1;
    void* v0 = const_cast<void*>(ptr);
    void* v1 = reinterpret_cast<void*>(last);
    const PtrKind k0 = classify_hip(ptr, &d0, &v0), k1 = classify_hip(v1, &d1, &v1);
    if (k0 == PK_DEVICE || k1 == PK_DEVICE)
        return fail(MI_E_INVALID, "device or managed memory cannot be declared as host memory");
    if (k0 != k1) return fail(MI_E_INVALID, "the range spans pinned and pageable memory");
    const intptr_t delta = (intptr_t)(reinterpret_cast<uintptr_t>(v0) - a);
    if (k0 == PK_PINNED && (intptr_t)(reinterpret_cast<uintptr_t>(v1) - last) != delta)
        return fail(MI_E_INVALID, "the pinned range spans several mappings");
    PtrKind kind = k0;
    if (kind == PK_PINNED) {  // pinned in place only inside one pinned allocation
        uintptr_t lo = 0, hi = 0;
        if (!pinned_extent(a, delta, &lo, &hi) || bytes > hi - a) kind = PK_PAGEABLE;
    }
    try {
        std::lock_guard<std::mutex> lk(g_rng_mu);
        const RangeSnap* cur = g_rng.load(std::memory_order_relaxed);
        std::unique_ptr<RangeSnap> next(new RangeSnap);
        if (cur) next->r = cur->r;
        auto it = std::upper_bound(next->r.begin(), next->r.end(), a,
                                   [](uintptr_t x, const HostRange& r) { return x < r.lo; });
        if (it != next->r.end() && it->lo < a + bytes) return fail(MI_E_INVALID, "overlaps a declared range");
        if (it != next->r.begin() && std::prev(it)->hi > a) return fail(MI_E_INVALID, "overlaps a declared range");
        next->r.insert(it, HostRange{a, a + bytes, kind, kind == PK_PINNED ? delta : 0});
        publish_ranges(next.release());
        g_rng_n.fetch_add(1, std::memory_order_release);
    } catch (const std::exception&) {
        return fail(MI_E_RESOURCE, "out of memory");
    }
    return 0;
}

int mi_host_undeclare(const void* ptr) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(ptr);
    try {
        std::lock_guard<std::mutex> lk(g_rng_mu);
        const RangeSnap* cur = g_rng.load(std::memory_order_relaxed);
        if (!cur) return fail(MI_E_INVALID, "not a declared range");
        auto it = std::lower_bound(cur->r.begin(), cur->r.end(), a,
                                   [](const HostRange& r, uintptr_t x) { return r.lo < x; });
        if (it == cur->r.end() || it->lo != a) return fail(MI_E_INVALID, "not a declared range");
        std::unique_ptr<RangeSnap> next(new RangeSnap);
        next->r.reserve(cur->r.size() - 1);
        for (const HostRange& r : cur->r)
            if (r.lo != a) next->r.push_back(r);
        g_rng_n.fetch_sub(1, std::memory_order_release);
        publish_ranges(next.release());
    } catch (const std::exception&) {
        return fail(MI_E_RESOURCE, "out of memory");
    }
    return 0;
}

int mi_host_declared_kind(const void* ptr, size_t bytes) {
    PtrKind k;
    return declared(ptr, bytes ? bytes : 1, &k, nullptr) ? (int)k : -1;
}

size_t mi_pointer_lookups(void) { return t_lookups; }

int mi_test_staged_device(void) { return t_stage.last_device.load(std::memory_order_relaxed); }

int mi_test_fail_copy(long nth) {
    g_copy_seq.store(0, std::memory_order_relaxed);
    g_fail_copy_nth.store(nth > 0 ? nth : 0, std::memory_order_relaxed);
    return 0;
}

int mi_test_copy_error(const void* host, size_t bytes, size_t chunk, int kind, int hull) {
    if (kind < PK_DEVICE || kind > PK_PAGEABLE) return fail(MI_E_INVALID, "pointer kind out of range");
    return copy_fail(hipErrorInvalidValue, "H2D staging copy (test)", host, bytes, chunk, (PtrKind)kind, hull != 0);
}

int mi_test_hold_exit_guard(int hold_ms) {
    ensure_exit_hook();
    std::thread([hold_ms] {
        ExitGuard g("mi_test_hold_exit_guard");
        if (hold_ms < 0)
            for (;;) std::this_thread::sleep_for(std::chrono::seconds(1));
        std::this_thread::sleep_for(std::chrono::milliseconds(hold_ms));
    }).detach();
    return 0;
}

size_t mi_dtype_size(int dtype) { return dtype_size(dtype); }

const char* mi_last_error(void) { return g_last_error.c_str(); }

int mi_version(void) { return 100; }  // 0.1.0

int mi_helper_cpu_count(void) { return g_helper_cpus.use ? CPU_COUNT(&g_helper_cpus.mask) : 0; }

int mi_release_pooled_contexts(void) {
    std::vector<DevCtx*> doomed;
    {
        CtxPool& p = ctx_pool();
        std::lock_guard<std::mutex> lk(p.mu);
        doomed.swap(p.free);
    }
    ExitGuard g("releasing pooled contexts");
    if (!g.entered) return 0;  // the process is exiting: its teardown frees them
    for (DevCtx* d : doomed) {
        for (int s = 0; s < 2; s++)
            if (d->stream[s]) (void)hipStreamSynchronize(d->stream[s]);
        if (d->d2h) (void)hipStreamSynchronize(d->d2h);
        delete d;
    }
    g_ctx_created.fetch_sub(doomed.size());
    return (int)doomed.size();
}

int mi_context_stats(size_t* created, size_t* pooled) {
    if (created) *created = g_ctx_created.load();
    if (pooled) {
        CtxPool& p = ctx_pool();
        std::lock_guard<std::mutex> lk(p.mu);
        *pooled = p.free.size();
    }
    return 0;
}

int mi_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return n;
}

int mi_set_host_mode(int mode) {
    if (mode < MI_HOST_AUTO || mode > MI_HOST_ZEROCOPY) return fail(MI_E_INVALID, "bad host mode");
    const int prev = host_mode();
    g_host_mode.store(mode == MI_HOST_ZEROCOPY ? MI_HOST_AUTO : mode, std::memory_order_relaxed);
    return prev;
}

int mi_set_sync_mode(int mode) {
    if (mode != MI_SYNC_SPIN && mode != MI_SYNC_BLOCK) return fail(MI_E_INVALID, "bad sync mode");
    const int prev = sync_mode();
    g_sync_mode.store(mode, std::memory_order_relaxed);
    return prev;
}

int mi_set_unaligned_vectors(int on) {
    const int prev = unaligned_vectors();
    g_unaligned.store(on ? 1 : 0, std::memory_order_relaxed);
    return prev;
}

int mi_get_launch_config(int* block, int* unroll, int* max_blocks_out) {
    if (block) *block = kBlock;
    if (unroll) *unroll = kUnroll;
    if (max_blocks_out) *max_blocks_out = max_blocks();
    return 0;
}

int mi_get_residency(int device, int k, int* waves_per_cu, unsigned* lds_bytes) {
    if (k < 0 || k > MI_MAX_INPUTS) return fail(MI_E_INVALID, "k must be 0..16");
    if (device < 0 && hipGetDevice(&device) != hipSuccess) device = -1;
    const int w = planned_waves(k);
    if (waves_per_cu) *waves_per_cu = w;
    if (lds_bytes) *lds_bytes = wave_cap_enabled() ? wave_cap_bytes(lds_per_cu(device), w) : 0;
    return 0;
}

int mi_set_residency(int k, int waves_per_cu) {
    if (k < 0 || k > MI_MAX_INPUTS) return fail(MI_E_INVALID, "k must be 0..16");
    if (waves_per_cu < 0 || waves_per_cu > 32) return fail(MI_E_INVALID, "waves_per_cu must be 0..32");
    g_residency_override[k].store(waves_per_cu, std::memory_order_relaxed);
    return 0;
}

int mi_set_max_blocks(int mb) {
    if (mb < 0) return fail(MI_E_INVALID, "max_blocks must be >= 0");
    g_max_blocks.store(mb, std::memory_order_relaxed);
    return 0;
}

}  // extern "C"
