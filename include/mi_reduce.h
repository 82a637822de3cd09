/*
 * mi_reduce.h — C ABI of the MI355X-native local element-wise reduction
 * (libmi_reduce.so, built by hipcc for gfx950).
 *
 * This is the drop-in boundary that replaces the *body* of oneCCL's src/comp
 * (reference snapshot 2024-12-20, v2021.14.0).  The C++ shim in
 * oneccl_amd/csrc/comp.cpp keeps oneCCL's own signatures
 * (ccl_comp_reduce / ccl_comp_batch_reduce / ccl_comp_copy /
 * ccl_reduction_to_str / ccl_bf16_reduce / ccl_fp16_reduce) and calls down
 * into the functions below, so src/sched, src/exec, src/coll, src/atl and the
 * ccl:: API are untouched.
 *
 * Plain pointers and sizes only; no torch or HIP C++ types in signatures.
 * `stream` is a hipStream_t passed as void* (NULL = the null stream).
 *
 * Return convention: 0 = success; MI_E_* (< 0) = argument / support errors;
 * > 0 = the hipError_t that failed.  mi_last_error() returns a
 * thread-local human-readable message for the last non-zero return.
 * (The reference returns ccl::status::success always and CCL_FATALs on bad
 * dtype/op, src/comp/comp.cpp:56,113; the C++ shim maps non-zero to
 * CCL_THROW, see oneccl_amd/csrc/comp.cpp.)
 */
#ifndef MI_REDUCE_H
#define MI_REDUCE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- enumerations: numerically identical to the reference's ---------- */

/* ccl::reduction — include/oneapi/ccl/types.hpp:41-47 */
enum mi_op {
    MI_OP_SUM = 0,
    MI_OP_PROD = 1,
    MI_OP_MIN = 2,
    MI_OP_MAX = 3,
    MI_OP_CUSTOM = 4 /* never accepted by the device entry points */
};

/* ccl::datatype — include/oneapi/ccl/types.hpp:52-69 */
enum mi_dtype {
    MI_INT8 = 0,
    MI_UINT8 = 1,
    MI_INT16 = 2,
    MI_UINT16 = 3,
    MI_INT32 = 4,
    MI_UINT32 = 5,
    MI_INT64 = 6,
    MI_UINT64 = 7,
    MI_FLOAT16 = 8,
    MI_FLOAT32 = 9,
    MI_FLOAT64 = 10,
    MI_BFLOAT16 = 11
};

/* ---- semantic variant flags ------------------------------------------- *
 * The reference's CPU reduce has several bit-level behaviours selected by
 * CPUID / CCL_BF16 / CCL_FP16.  The device kernels implement
 * every one of them; the caller picks with these flags.                    */

/* min/max return `inout` when the operands are unordered (NaN) or equal
 * (+0/-0): _mm512_min_ps(in, inout) semantics of the AVX-512 bf16/fp16
 * paths (src/comp/bf16/bf16_intrisics.cpp:28-34,
 * src/comp/fp16/fp16_intrisics.hpp:72-77).  Clear = std::min(in, inout)
 * semantics of CCL_REDUCE and the scalar bf16 path (returns `in`),
 * src/comp/comp.cpp:45-53, src/comp/bf16/bf16.cpp:42-48.                  */
#define MI_F_MINMAX_INOUT_FIRST 0x1u
/* fp32 -> bf16 by round-to-nearest-even with VCVTNEPS2BF16 semantics
 * (denormal fp32 -> signed zero, NaN -> quiet NaN): avx512bf impl,
 * src/comp/bf16/bf16_intrisics.hpp:72-76.  Clear = truncation (scalar and
 * avx512f impls, bf16.cpp:50-54, bf16_intrisics.hpp:67-70).                */
#define MI_F_BF16_RNE 0x2u
/* Low-precision (bf16/fp16) fan-in accumulates in fp32 and rounds once at
 * the end: ccl_comp_batch_reduce(..., bf16_keep_precision_mode=1, ...),
 * src/comp/comp.cpp:214-234.  Clear = round to storage after every
 * pairwise step (chained ccl_comp_reduce, comp.cpp:236-245).               */
#define MI_F_ACC_FP32 0x4u
/* With MI_F_ACC_FP32|MI_F_BF16_RNE: the last (count % 16) elements of the
 * final fp32 -> bf16 conversion are truncated, as the scalar tail loop of
 * ccl_convert_fp32_to_bf16_arrays does (src/comp/bf16/bf16.cpp:145-148).   */
#define MI_F_BF16_TAIL_TRUNC16 0x8u
/* fp16 min/max as VMINPH/VMAXPH (avx512fp16 impl, src/comp/fp16/
 * fp16_intrisics.cpp:30-35): a NaN accumulator (`inout`) is returned as
 * stored, so a signalling NaN stays signalling; clear = the fp32 route of the
 * f16c/avx512f impls, whose VCVTPH2PS quiets it.  The only bits in which the
 * two impls differ (oracle/FP16_NATIVE_CHECK.json).                        */
#define MI_F_FP16_NATIVE_MINMAX 0x10u

/* Error codes (< 0). */
#define MI_E_INVALID (-1)      /* bad dtype / op / k / NULL pointer      */
#define MI_E_UNSUPPORTED (-2)  /* combination not implemented            */
#define MI_E_NO_DEVICE (-3)    /* no HIP device visible                   */
#define MI_E_RESOURCE (-4)     /* host resources (thread, memory) failed  */
#define MI_E_EXITING (-5)      /* process exit began before an asynchronous
                                  request ran; it was not run              */

#define MI_MAX_INPUTS 16 /* the reference's monolithic fan-in covers 16 ranks
                            (src/kernels/kernels.cl:268)                   */

/* ---- device-resident entry points (asynchronous on `stream`) ---------- */

/* inout[i] = op(in[i], inout[i]) for i < count.  Device pointers.
 * Replaces the arithmetic of ccl_comp_reduce_regular, src/comp/comp.cpp:76-121
 * (CCL_REDUCE :31-58; ccl_bf16_reduce bf16/bf16.cpp:87-110; ccl_fp16_reduce
 * fp16/fp16.cpp:41-53) and the device kernel reduce_local_inplace_kernel_*,
 * src/kernels/kernels.cl:236-246.                                           */
int mi_reduce(const void* in, void* inout, size_t count, int dtype, int op,
              unsigned flags, void* stream);

/* out[i] = op(in1[i], in2[i]) with in1 in the `in` role and in2 in the
 * `inout` role.  Replaces reduce_local_outofplace_kernel_*,
 * src/kernels/kernels.cl:219-234.                                           */
int mi_reduce_out(const void* in1, const void* in2, void* out, size_t count,
                  int dtype, int op, unsigned flags, void* stream);

/* K-input fan-in, 2 <= k <= MI_MAX_INPUTS: acc = inputs[0];
 * acc = op(inputs[j], acc) for j = 1..k-1 (left fold, `inputs[j]` in the
 * `in` role); out = acc.  `out` may alias inputs[0].  Replaces
 * ccl_comp_batch_reduce, src/comp/comp.cpp:202-249, and the monolithic
 * fan-in kernels reduce_monolithic_kernel_<N>_*, src/kernels/kernels.cl:269-421. */
int mi_reduce_multi(const void* const* inputs, int k, void* out, size_t count,
                    int dtype, int op, unsigned flags, void* stream);

/* n independent mi_reduce calls in one dispatch: descs[i].inout =
 * op(descs[i].in, descs[i].inout) over descs[i].count elements, all with one
 * dtype / op / flags.  Results are those of the n mi_reduce calls in any
 * order.  So no descriptor's inout may overlap another descriptor's in or
 * inout (MI_E_INVALID); in == inout within one descriptor is allowed, as for
 * mi_reduce.  For schedule phases with many small chunks: a sub-MiB reduce
 * costs one dispatch, and this pays one for up to 64 chunks.
 * No reference counterpart: oneCCL issues one ccl_comp_reduce per entry
 * (reduce_local_entry.cpp:98-114, and one per parallelizer part,
 * parallelizer.cpp:184-320).  An extension for callers that hold several
 * chunks of one phase.                                                      */
typedef struct mi_reduce_desc {
    const void* in;
    void* inout;
    size_t count;
} mi_reduce_desc_t;

int mi_reduce_batch(const mi_reduce_desc_t* descs, int n, int dtype, int op,
                    unsigned flags, void* stream);

/* ---- synchronous, pointer-kind-agnostic entry (what src/comp calls) --- *
 * Same math as mi_reduce, but `in`/`inout` may each be device memory,
 * pinned host memory or pageable host memory; returns only when the result
 * is in `inout` (the entries mark themselves complete right after the call:
 * src/sched/entry/reduce_local_entry.cpp:113, recv_reduce_entry.hpp:133).
 * Host operands are staged through the GPU in pipelined chunks (H2D, kernel,
 * D2H on a per-thread stream).  `device` < 0 = the calling thread's current
 * HIP device.  Thread-safe: each calling thread has its own stream and
 * scratch (threading contract of src/exec/thread/worker.cpp:310-379).  A
 * caller confined to one or two CPUs (a pinned oneCCL worker) has a staged
 * bucket with pageable operands run by its staging worker, whose CPU set is
 * the process's, while it waits (MI_REDUCE_CONFINED_HANDOFF=0: inline).   */
int mi_reduce_sync(const void* in, void* inout, size_t count, int dtype,
                   int op, unsigned flags, int device);

/* Synchronous K-input fan-in with host-or-device operands (staged like
 * mi_reduce_sync).  Used by ccl_comp_batch_reduce.                       */
int mi_reduce_multi_sync(const void* const* inputs, int k, void* out,
                         size_t count, int dtype, int op, unsigned flags,
                         int device);

/* ---- asynchronous form of the pointer-kind-agnostic entry ------------ *
 * Issues the same work as mi_reduce_multi_sync and returns at once with a
 * request; mi_test polls it (done = 1 when inputs may be reused and `out` is
 * final), mi_wait blocks, mi_request_free releases it (after completion).
 * Lets a schedule entry return `started` and poll from update() instead of
 * blocking its worker thread (reduce_local_entry.cpp:
 * 116-135 polls the Level Zero path the same way).  Work that needs host
 * staging (pageable operands) runs on a worker thread owned by the calling
 * thread, in submission order, so mi_reduce_start returns at once for it
 * too.  mi_request_free waits for a request that is still running.       */
typedef struct mi_request* mi_request_t;
int mi_reduce_start(const void* const* inputs, int k, void* out, size_t count,
                    int dtype, int op, unsigned flags, int device,
                    mi_request_t* req);
int mi_test(mi_request_t req, int* done);
/* mi_reduce_start that also times the request where it runs: a staged
 * request on the staging worker's clock (from when it starts, after the
 * thread's earlier work), a direct one by a HIP event pair around its
 * launch.  mi_request_run_time gives that duration in seconds once the
 * request is done (MI_E_INVALID before, or for an untimed direct request).
 * The drop-in's adaptive dispatcher times its GPU-alone buckets with it, so
 * the rate it learns excludes the delay before the caller polls.          */
int mi_reduce_start_timed(const void* const* inputs, int k, void* out, size_t count,
                          int dtype, int op, unsigned flags, int device,
                          mi_request_t* req);
int mi_request_run_time(mi_request_t req, double* seconds);
/* The cooperative split as a request: elements [0, head_count) are folded by
 * `head_fold` (a host reduce with mi_host_reduce's signature and semantics,
 * include/mi_host_reduce.h) on the calling thread's staging worker while the
 * GPU folds [head_count, count) — so neither half waits on the caller's
 * thread.  Ordered with the thread's other requests like a staged one.  The
 * caller keeps head_count a multiple of 256 elements (the bf16 keep-precision
 * count % 16 tail must stay whole in the GPU part); head_count 0 is
 * mi_reduce_start.  Used by ccl_comp_reduce_start / _batch_reduce_start for
 * host buckets above the dispatcher's threshold.                           */
typedef int (*mi_host_fold_t)(const void* const* inputs, int k, void* out, size_t count, int dtype, int op,
                              unsigned flags);
int mi_reduce_split_start(const void* const* inputs, int k, void* out, size_t count, int dtype, int op,
                          unsigned flags, int device, size_t head_count, mi_host_fold_t head_fold,
                          mi_request_t* req);
/* A finished split request's two durations, in seconds from its start: the
 * head (folded in ~8 MiB chunks) and the GPU part (seen done between two
 * chunks, or at the end).  What the caller needs to move its share toward
 * the point where both finish together.  MI_E_INVALID for other requests. */
int mi_request_split_times(mi_request_t req, double* head_s, double* tail_s);
/* Wait until every request this thread has started with mi_reduce_start has
 * finished.  The synchronous entry points do this themselves; a caller about
 * to touch an earlier request's operands on the CPU (the drop-in's host
 * reduce, include/mi_host_reduce.h) calls it first.  Returns at once for a
 * thread that never started a request.                                     */
int mi_thread_sync(void);
int mi_wait(mi_request_t req);
int mi_request_free(mi_request_t req);

/* ---- in-process multi-GPU element-range shards --------- *
 * Shard s folds inputs[s*k .. s*k+k-1] into outs[s] (counts[s] elements) on
 * HIP device devices[s] — all pointers of a shard live on its device.  Every
 * shard is launched before any is waited for; no inter-GPU traffic, no
 * collective.  Synchronous.                                                */
/* One bucket of any pointer kinds split by element range over `nshards`
 * GPUs (devices[s] may repeat), every shard reduced at once: shard 0 on the
 * calling thread, the others on worker threads it owns.  For host-resident
 * buckets each GPU moves its shard over its own PCIe link, so the
 * PCIe-inclusive rate adds up over GPUs.  Synchronous; same bits as
 * mi_reduce_multi_sync (shard boundaries are 256-element aligned).        */
int mi_reduce_multi_sync_sharded(const void* const* inputs, int k, void* out, size_t count,
                                 int dtype, int op, unsigned flags, int nshards,
                                 const int* devices);

int mi_reduce_sharded(int nshards, const int* devices, const void* const* inputs,
                      int k, void* const* outs, const size_t* counts, int dtype,
                      int op, unsigned flags);

/* Byte copy, synchronous, any pointer kinds.  Replaces the body of
 * ccl_comp_copy, src/comp/comp.cpp:60-74 (nontemporal flag honoured on the
 * device path by non-temporal stores).                                     */
int mi_copy_sync(const void* src, void* dst, size_t bytes, int nontemporal,
                 int device);

/* Asynchronous device-to-device copy kernel (non-temporal stores if asked). */
int mi_copy(const void* src, void* dst, size_t bytes, int nontemporal,
            void* stream);

/* ---- precision conversions ------------------------------------------- *
 * fp32 -> bf16 (MI_F_BF16_RNE: VCVTNEPS2BF16 semantics, else truncation;
 * MI_F_BF16_TAIL_TRUNC16: the last count%16 elements truncate), fp32 -> fp16
 * (RNE, VCVTPS2PH imm8=0), bf16 -> fp32 and fp16 -> fp32 (exact).  Replaces
 * ccl_convert_fp32_to_bf16_arrays / ccl_convert_bf16_to_fp32_arrays
 * (src/comp/bf16/bf16.cpp:113-169) and ccl_convert_fp32_to_fp16 /
 * ccl_convert_fp16_to_fp32 (src/comp/fp16/fp16.cpp:55-61).
 * mi_convert: device pointers, asynchronous.  mi_convert_sync: any pointer
 * kinds, returns when dst is written.                                      */
int mi_convert(const void* src, int src_dtype, void* dst, int dst_dtype,
               size_t count, unsigned flags, void* stream);
int mi_convert_sync(const void* src, int src_dtype, void* dst, int dst_dtype,
                    size_t count, unsigned flags, int device);

/* ---- element-range sharding for 1..8 GPUs ------------- *
 * Contiguous [begin,end) of shard `rank` of `world`, boundaries rounded to
 * `align` elements (0 -> 256).  No data moves: each GPU reduces its shard of
 * every input independently; no collective is involved.                  */
int mi_shard_range(size_t count, int rank, int world, size_t align,
                   size_t* begin, size_t* end);

/* ---- pointer classification ------------------------------------------- */
/* 0 = device (or managed) memory of HIP device *device; 1 = pinned host
 * memory; 2 = pageable host memory.  What ccl_comp_reduce's SYCL branch asks
 * sycl::get_pointer_type for (src/comp/comp.cpp:145-147).                 */
int mi_pointer_kind(const void* ptr, int* device);
/* The same for the operand [ptr, ptr + bytes): answered from the declared
 * host ranges below when it lies wholly inside one, else by HIP.          */
int mi_pointer_kind_range(const void* ptr, size_t bytes, int* device);

/* ---- declared host ranges --------------------------------------------- *
 * HIP's pointer lookup serialises concurrent callers on pageable memory
 * (0.07 us alone, 9.5 us per call at 16 threads on MI355X).
 * A caller that owns long-lived host buffers declares them once: every
 * entry point then classifies an operand lying wholly inside a declared
 * range without asking HIP (readers take no lock).  mi_host_declare looks
 * the range up once (both ends): device or managed memory is refused with
 * MI_E_INVALID, as is a range mixing kinds.  A pinned range is recorded as
 * pinned (the zero-copy path) only when it lies inside one pinned
 * allocation (one mi_host_register, or the allocation HIP reports for it);
 * otherwise it is recorded as pageable (staged), since pinned ends do not
 * make the pages between them pinned.  Declare after any mi_host_register of
 * the same buffer; mi_host_unregister turns the declared ranges over the
 * buffer pageable before unpinning it.  Ranges may not overlap.  Undeclare
 * (by the start address) before the memory is freed or unpinned by other
 * means; a range must not be undeclared while a reduce on it is in flight.  oneCCL's
 * regular_buffer_cache declares its buffers (integration/0005, INTEGRATION.md
 * §2f; the place it registers them with Level Zero,
 * src/sched/buffer/buffer_cache.cpp:99-104).                               */
int mi_host_declare(const void* ptr, size_t bytes);
int mi_host_undeclare(const void* ptr);
/* Kind (1 pinned, 2 pageable) of a declared range holding the operand, or
 * -1 when none does.  No HIP call.  Diagnostic.                           */
int mi_host_declared_kind(const void* ptr, size_t bytes);
/* HIP pointer lookups made by the calling thread so far (every entry point's
 * classification, declared ranges excepted).  Diagnostic.                  */
size_t mi_pointer_lookups(void);

/* ---- staging-buffer registration ------------------------------------- *
 * Pin (page-lock and map for every GPU) an existing pageable host buffer, so
 * later mi_*_sync calls on it take the zero-copy path instead of staging.
 * Meant for buffers that live long: oneCCL's regular_buffer_cache reuses its
 * staging buffers and already registers them with Level Zero at this point
 * (src/sched/buffer/buffer_cache.cpp:99-104, import_external_pointer);
 * INTEGRATION.md shows the two-line HIP equivalent.  mi_host_unregister must
 * run before the memory is freed.                                          */
int mi_host_register(void* ptr, size_t bytes);
int mi_host_unregister(void* ptr);

/* ---- host-operand strategy ------------------------------------------- *
 * How mi_*_sync treats host operands.  MI_HOST_AUTO (default): pinned host
 * memory is read and written in place by the kernel over PCIe (zero-copy,
 * full duplex), pageable memory is staged; MI_HOST_STAGED: always stage
 * (chunked H2D -> kernel -> D2H on two streams); MI_HOST_ZEROCOPY: as AUTO.
 * Env: MI_REDUCE_HOST_MODE=auto|staged.  Returns the previous mode.       */
#define MI_HOST_AUTO 0
#define MI_HOST_STAGED 1
#define MI_HOST_ZEROCOPY 2
int mi_set_host_mode(int mode);

/* How the synchronous entry points wait for the GPU: MI_SYNC_BLOCK (default)
 * uses the runtime's stream wait; MI_SYNC_SPIN polls hipStreamQuery (was
 * 1-2 us slower per call on MI355X / ROCm 7.2, profiles/round1_size_sweep2
 * .jsonl).  Env MI_REDUCE_SYNC=spin|block.  Returns the previous mode.     */
#define MI_SYNC_SPIN 0
#define MI_SYNC_BLOCK 1
int mi_set_sync_mode(int mode);

/* Operands whose addresses differ mod 16 bytes (ring chunks at arbitrary
 * element offsets): 1 (default) = the 16-byte vector kernels on the output's
 * 16-byte grid, inputs read by unaligned 16-byte loads; 0 = the element loop.
 * Same bits either way.  Env MI_REDUCE_UNALIGNED=0|1.  Returns the previous
 * setting.                                                                 */
int mi_set_unaligned_vectors(int on);

/* ---- introspection ---------------------------------------------------- */

/* ccl_reduction_to_str, src/comp/comp.cpp:251-260. */
const char* mi_reduction_to_str(int op);
/* Size in bytes of a datatype id (0 if unknown);
 * src/common/datatype/datatype.cpp predefined table.                      */
size_t mi_dtype_size(int dtype);
/* Thread-local message for the last non-zero return on this thread. */
const char* mi_last_error(void);
/* ABI version: major*10000 + minor*100 + patch. */
int mi_version(void);
/* Number of HIP devices (0 when none).  Never initialises a context.      */
int mi_device_count(void);
/* Launch geometry the vector kernels use: threads per block, 16-byte
 * vectors per lane per tile, and the grid cap (0 = one tile per block).   */
int mi_get_launch_config(int* block, int* unroll, int* max_blocks);
/* Residency plan of the one-wave vector kernels on `device` (< 0: the
 * current device) for a k-input launch: k = 2 the 2-input kernel, k = 1 or
 * 3..16 the fan-in, k = 0 the array conversions.  *waves_per_cu = the
 * resident waves per CU the launch is sized for; *lds_bytes = the dynamic
 * LDS (never touched) each one-wave workgroup reserves to cap it there, 0
 * when the device does not report its LDS per CU or MI_REDUCE_WAVE_CAP=0
 * (no cap then).  DESIGN.md §5; tools/occupancy_sweep.hip measured the
 * caps.                                                                    */
int mi_get_residency(int device, int k, int* waves_per_cu, unsigned* lds_bytes);
/* Override that plan for k-input launches (tuning knob, k as above):
 * waves_per_cu 1..32 (the reservation is 128 / waves_per_cu whole LDS
 * granules, so the residency achieved is one of 32, 25, 21, 18, 16, 14, 12,
 * 11, 10, 9, 8, ...), 0 = back to the plan.
 * tools/residency_ab.py A/Bs the plan against other residencies with it.  */
int mi_set_residency(int k, int waves_per_cu);
/* Override the grid cap (tuning knob; env MI_REDUCE_MAX_BLOCKS).  Under a
 * cap the reduce, copy and conversion kernels stride over the buffer.     */
int mi_set_max_blocks(int max_blocks);
/* CPUs the library's helper threads (staging worker, drain thread) run on:
 * the process's allowed set read at load (/proc/self/status), so helpers of
 * a worker oneCCL pinned to one core do not share that core.  0 = helpers
 * inherit their creator's mask (MI_REDUCE_HELPER_AFFINITY=inherit).       */
int mi_helper_cpu_count(void);
/* Per-thread device contexts (two streams, staging and bounce buffers):
 * *created = contexts that exist (built and not released), *pooled = those
 * of exited threads, waiting in the pool for the next thread on their
 * device.  A thread's exit makes no HIP call: its contexts are reused, and
 * freed only by mi_release_pooled_contexts or the process's end.
 * Diagnostic.                                                             */
int mi_context_stats(size_t* created, size_t* pooled);
/* Free the pooled contexts of exited threads (streams, staging and bounce
 * buffers: up to 2 x 32 MiB of device memory per host operand slot each).
 * Work they still hold queued finishes first.  For a point where the
 * process is done reducing for a while (oneCCL's finalize); the next thread
 * that needs a context builds a new one.  Returns the number freed.       */
int mi_release_pooled_contexts(void);
/* Test hook:a library thread holds an exit guard (the section the exit
 * handler waits for) for hold_ms milliseconds, < 0 = forever.  The handler
 * waits at most MI_REDUCE_EXIT_WAIT_S seconds (default 60), then names the
 * section on stderr and ends the process with status 70.                  */
int mi_test_hold_exit_guard(int hold_ms);
/* Test hook: the current device of the calling thread's staging worker when
 * it last ran a job of this thread (-1: none yet).  A job submitted with
 * device < 0 runs on the submitting thread's current device.             */
int mi_test_staged_device(void);
/* Test hook: the nth staged host<->device copy issued from now on (any
 * thread; 1 = the next) fails with hipErrorInvalidValue before it reaches the
 * runtime; 0 turns it off.  The failing call's mi_last_error() then names
 * the copy and the host operand's geometry (page offset, length, the span
 * handed to the runtime, chunk, pointer class).                           */
int mi_test_fail_copy(long nth);
/* Test hook: the error text of a failed copy of [host, host + bytes) in
 * chunk `chunk` of a host operand of pointer kind `kind` (as mi_pointer_kind:
 * 0 device, 1 pinned, 2 pageable), the
 * runtime handed its aligned hull (hull != 0) or interior; sets
 * mi_last_error() and returns hipErrorInvalidValue's code.  No HIP device
 * is needed.                                                              */
int mi_test_copy_error(const void* host, size_t bytes, size_t chunk, int kind, int hull);

#ifdef __cplusplus
}
#endif

#endif /* MI_REDUCE_H */
