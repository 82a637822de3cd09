/*
 * mi_ccl_comp.h — C view of the drop-in src/comp shim (libccl_comp_hip.so,
 * built from oneccl_amd/csrc/comp.cpp in standalone mode).
 *
 * libccl_comp_hip.so exports oneCCL's own C++ entry points with identical
 * mangled names (ccl_comp_reduce(ccl_sched*, ..., ccl::v1::reduction, ...),
 * ccl_comp_batch_reduce, ccl_comp_copy, ccl_reduction_to_str,
 * ccl_bf16_reduce, ccl_fp16_reduce — src/comp/comp.hpp:23-51,
 * src/comp/bf16/bf16.hpp:26-38, src/comp/fp16/fp16.hpp:21-35).  The
 * functions below are thin extern "C" wrappers over exactly those C++
 * functions, so FFI callers (ctypes in this repo's tests, or a cgo/JNI
 * binding) drive the same code path src/sched would.  Each returns the
 * ccl::status value, or -1 if the C++ call threw (message:
 * mi_ccl_last_error()).  dtype / op ids are ccl::datatype / ccl::reduction.
 */
#ifndef MI_CCL_COMP_H
#define MI_CCL_COMP_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ccl::reduction_fn with ccl::datatype passed as int
 * (include/oneapi/ccl/types.hpp:122-124). */
typedef void (*mi_ccl_reduction_fn)(const void* in_buf, size_t in_count, void* inout_buf,
                                    size_t* out_count, int dtype, const void* context);

/* ccl_comp_reduce(sched, ...), src/comp/comp.cpp:123-200; sched = none
 * unless mi_ccl_comp_shim_sched chose one for the calling thread */
int mi_ccl_comp_reduce(const void* in_buf, size_t in_count, void* inout_buf, size_t* out_count,
                       int dtype, int op);
/* ccl_comp_reduce with ccl::reduction::custom and a user callback,
 * src/comp/comp.cpp:84-88 */
int mi_ccl_comp_reduce_custom(const void* in_buf, size_t in_count, void* inout_buf,
                              size_t* out_count, int dtype, mi_ccl_reduction_fn fn);
/* ccl_comp_batch_reduce, src/comp/comp.cpp:202-249 */
int mi_ccl_comp_batch_reduce(const void* in_buf, const size_t* offsets, size_t n_offsets,
                             size_t in_count, void* inout_buf, size_t* out_count, int dtype,
                             int op, int bf16_keep_precision_mode);
/* ccl_comp_batch_reduce with reduction::custom and the user's callback
 * (every input folded by fn, in keep-precision mode on the fp32 scratch). */
int mi_ccl_comp_batch_reduce_custom(const void* in_buf, const size_t* offsets, size_t n_offsets,
                                    size_t in_count, void* inout_buf, size_t* out_count, int dtype,
                                    int bf16_keep_precision_mode, mi_ccl_reduction_fn fn);
/* ccl_comp_copy, src/comp/comp.cpp:60-74 */
int mi_ccl_comp_copy(const void* in_buf, void* out_buf, size_t bytes, int use_nontemporal);
/* ccl_comp_copy_host (mi_ccl_comp_async.hpp): a copy its caller knows to be
 * host to host, with no pointer lookup */
int mi_ccl_comp_copy_host(const void* in_buf, void* out_buf, size_t bytes, int use_nontemporal);
/* ccl_bf16_reduce, src/comp/bf16/bf16.cpp:87-110 (MPI user-op entry,
 * src/atl/mpi/atl_mpi_ctx.cpp:87-92) */
int mi_ccl_bf16_reduce(const void* in_buf, size_t in_cnt, void* inout_buf, size_t* out_cnt, int op);
/* ccl_fp16_reduce, src/comp/fp16/fp16.cpp:41-53 */
int mi_ccl_fp16_reduce(const void* in_buf, size_t in_cnt, void* inout_buf, size_t* out_cnt, int op);
/* ccl_bf16_reduce_host / ccl_fp16_reduce_host (mi_ccl_lp_host.hpp): the MPI
 * user ops' reduce (atl_mpi_ctx.cpp:57-63, 87-92, integration/0002), host
 * memory by construction: no pointer lookup up to the CPU threshold */
int mi_ccl_bf16_reduce_host(const void* in_buf, size_t in_cnt, void* inout_buf, size_t* out_cnt, int op);
int mi_ccl_fp16_reduce_host(const void* in_buf, size_t in_cnt, void* inout_buf, size_t* out_cnt, int op);
/* ccl_convert_fp32_to_bf16_arrays / ccl_convert_bf16_to_fp32_arrays,
 * src/comp/bf16/bf16.cpp:113-169 (rounding per the bf16 impl type) */
int mi_ccl_convert_fp32_to_bf16_arrays(void* fp32_buf, void* bf16_buf, size_t count);
int mi_ccl_convert_bf16_to_fp32_arrays(void* bf16_buf, float* fp32_buf, size_t count);
/* ccl_convert_fp32_to_fp16 / ccl_convert_fp16_to_fp32 (8 elements),
 * src/comp/fp16/fp16.cpp:55-61 */
int mi_ccl_convert_fp32_to_fp16(const void* src, void* dst);
int mi_ccl_convert_fp16_to_fp32(const void* src, void* dst);
/* Asynchronous ccl_comp_reduce (include/mi_ccl_comp_async.hpp, SURVEY.md
 * §8f rank 4): start issues the reduce and returns a request; test sets
 * *done = 1 once inout_buf holds the result; free waits if still pending.
 * `fn` is the user callback for op = custom (run inside start), else NULL. */
struct ccl_comp_request;
int mi_ccl_comp_reduce_start(const void* in_buf, size_t in_count, void* inout_buf,
                             size_t* out_count, int dtype, int op, mi_ccl_reduction_fn fn,
                             struct ccl_comp_request** req);
/* ccl_comp_batch_reduce_start: the fused K-input fold as one request. */
int mi_ccl_comp_batch_reduce_start(const void* in_buf, const size_t* offsets, size_t n_offsets,
                                   size_t in_count, void* inout_buf, size_t* out_count, int dtype,
                                   int op, int bf16_keep_precision_mode,
                                   struct ccl_comp_request** req);
int mi_ccl_comp_request_test(struct ccl_comp_request* req, int* done);
int mi_ccl_comp_request_wait(struct ccl_comp_request* req);
int mi_ccl_comp_request_free(struct ccl_comp_request* req);
/* ccl_reduction_to_str, src/comp/comp.cpp:251-260 */
const char* mi_ccl_reduction_to_str(int op);
/* Re-read CCL_BF16 / CCL_FP16 / CCL_COMP_HIP_DEVICE (env.cpp:711-720). */
int mi_ccl_env_reload(void);
/* The GPU host buckets go to: CCL_COMP_HIP_DEVICE, else the local rank
 * (MPI_LOCALRANKID / LOCAL_RANK / CCL_LOCAL_RANK, as oneCCL's launchers set
 * it) modulo the visible GPUs when more than one is visible, else -1 (the
 * calling thread's current device).  Diagnostic.                          */
int mi_ccl_comp_device(void);
/* The calling thread's CPU share of the cooperative split of host buckets
 * above the dispatcher's threshold (pinned = 1: all operands pinned), as
 * adapted by its own split calls; < 0 before the first one.  Diagnostic. */
double mi_ccl_comp_split_share(int pinned);
/* Threads the dispatcher counts as reducing host buckets now: inside such a
 * call, or returned from one within the last 50 ms.  A host bucket above the
 * threshold is split with the GPU only while this is at most
 * CCL_COMP_HOST_SPLIT_WORKERS (pageable) / _PINNED.  Diagnostic. */
int mi_ccl_comp_host_workers(void);
/* The calling thread's GPU-alone rate for host buckets of that pointer kind
 * (elements/s; < 0 before it was timed) and how many buckets it will still
 * run on the GPU alone (after a split lost to it, or as a probe).  Diagnostic. */
double mi_ccl_comp_split_gpu_rate(int pinned, unsigned* gpu_left);
/* Test hooks for the adaptive split's bookkeeping (no reduce is run):
 * take_gpu_alone = the decision an adapting thread makes before a bucket of
 * that kind (1 = the GPU alone, consuming one scheduled GPU-alone bucket;
 * 0 = split); split_feed = the update after a bucket of `count` elements,
 * a split with a CPU head of `head` elements (t_head, t_tail seconds from
 * its start) or, head = 0, a GPU-alone bucket of t_tail seconds.  The same
 * functions the synchronous and asynchronous paths call.                   */
int mi_ccl_comp_split_take_gpu_alone(int pinned);
int mi_ccl_comp_split_feed(int pinned, size_t count, size_t head, double t_head, double t_tail);
/* The dispatcher's thresholds and default shares in force (after env).     */
int mi_ccl_comp_host_max(size_t* pageable, size_t* pinned, double* share, double* share_pinned);
/* Host buffer registry.  A caller that owns long-lived host memory
 * (oneCCL's regular_buffer_cache, src/sched/buffer/buffer_cache.cpp:87-123;
 * integration/0005) declares [ptr, ptr + bytes) until it unregisters it
 * (by the start address, before freeing).  An operand lying wholly inside a
 * registered buffer is classified without asking HIP, whose lookup of
 * pageable pointers serialises concurrent workers -- by the
 * dispatcher and by libmi_reduce's GPU path alike (mi_host_declare).  The
 * range is looked up once, here: device or managed memory is refused with
 * MI_E_INVALID, pinned memory keeps its zero-copy path.  Buffers may not
 * overlap.  0 or an MI_E_* code.                                           */
int mi_ccl_comp_register_host_buffer(const void* ptr, size_t bytes);
int mi_ccl_comp_unregister_host_buffer(const void* ptr);
/* HIP pointer lookups made by the calling thread so far, in this shim and in
 * libmi_reduce (mi_pointer_lookups).  Diagnostic.                          */
size_t mi_ccl_comp_pointer_lookups(void);
/* Test hook: the schedule this thread's C-view calls pass to
 * ccl_comp_reduce / _start: 0 = none (nullptr, the default), 1 = a schedule
 * whose collective has no stream (operands are host memory by its word and
 * are not looked up, comp.cpp:136-142), 2 = one with a stream (looked up).
 * Returns the previous mode, or MI_E_INVALID.                              */
int mi_ccl_comp_shim_sched(int mode);
/* The impl types in force: ccl_bf16_impl_type / ccl_fp16_impl_type values. */
int mi_ccl_impl_types(int* bf16_impl, int* fp16_impl);
const char* mi_ccl_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
