/*
 * mi_ccl_comp_async.hpp — asynchronous form of oneCCL's ccl_comp_reduce
 * (SURVEY.md §8f rank 4), and the host copy of the copy entries, defined by
 * the drop-in shim oneccl_amd/csrc/comp.cpp for the patched schedule entries.
 *
 * The reference's call is synchronous: reduce_local_entry::start_on_host()
 * (src/sched/entry/reduce_local_entry.cpp:98-114) and
 * recv_reduce_entry::update() (src/sched/entry/recv_reduce_entry.hpp:99-135)
 * call ccl_comp_reduce and mark the entry complete on return.  These four
 * calls split it, so that start() can return with status `started` and
 * update() can poll.  reduce_local_entry::update() already polls the Level
 * Zero device path this way (reduce_local_entry.cpp:123-131).  The patch a
 * maintainer applies is in INTEGRATION.md §2(d).
 *
 * Semantics are those of ccl_comp_reduce (src/comp/comp.cpp:123-200):
 *   - bf16/fp16 write *out_count = in_count (bf16.cpp:94-96, fp16.cpp:48-50),
 *     at start, as the reference writes it before computing;
 *   - rounding and min/max operand order follow the bf16/fp16 impl type
 *     (CPUID + CCL_BF16 / CCL_FP16, env.cpp:711-720);
 *   - ccl::reduction::custom runs the user callback inside start, on host
 *     memory, and returns a request that is already complete;
 *   - in_count == 0 returns a request that is already complete.
 * Until the request tests complete, in_buf and inout_buf stay owned by the
 * library: the caller must not read, write or free them.  Failures throw
 * (CCL_THROW in-tree, ccl::exception standalone), as ccl_comp_reduce does.
 *
 * Include after oneCCL's comp/comp.hpp (in-tree), which declares
 * ccl_datatype, ccl::reduction, ccl::reduction_fn and ccl::fn_context.
 */
#ifndef MI_CCL_COMP_ASYNC_HPP
#define MI_CCL_COMP_ASYNC_HPP

#include <cstddef>
#include <vector>

struct ccl_comp_request;  // opaque; one per started reduce

/* Issue inout_buf = op(in_buf, inout_buf) and return at once; *req receives
 * the request to poll.  Always returns ccl::status::success (errors throw).
 * `sched` is the calling entry's schedule, as for ccl_comp_reduce: when its
 * collective has no stream (sched->coll_param.stream == nullptr) the
 * operands are host memory and are not looked up (the reference's
 * comp.cpp:136-142); nullptr = no schedule, operands looked up.           */
ccl::status ccl_comp_reduce_start(ccl_sched* sched, const void* in_buf, size_t in_count,
                                  void* inout_buf, size_t* out_count, const ccl_datatype& dtype,
                                  ccl::reduction reduction, ccl::reduction_fn reduction_fn,
                                  const ccl::fn_context* context, ccl_comp_request** req);

/* The same for ccl_comp_batch_reduce (src/comp/comp.cpp:202-249): the fused
 * K-input fold of in_buf + offsets[i] * dtype.size() into inout_buf, as one
 * request (several chained launches past 16 inputs).  The fp32 scratch
 * `tmp` / `acc` of the synchronous form is not needed and not taken.     */
ccl::status ccl_comp_batch_reduce_start(ccl_sched* sched, const void* in_buf,
                                        const std::vector<size_t>& offsets,
                                        size_t in_count, void* inout_buf, size_t* out_count,
                                        const ccl_datatype& dtype, ccl::reduction reduction,
                                        ccl::reduction_fn reduction_fn,
                                        const ccl::fn_context* context,
                                        int bf16_keep_precision_mode, ccl_comp_request** req);

/* true once inout_buf holds the result and both buffers may be reused. */
bool ccl_comp_request_test(ccl_comp_request* req);

/* Block until the request is complete. */
void ccl_comp_request_wait(ccl_comp_request* req);

/* Release a request (call after it tested complete, or after wait). */
void ccl_comp_request_free(ccl_comp_request* req);

/* ccl_comp_copy for a copy the caller knows to be host to host: the
 * regular copy of copy_entry (src/sched/entry/copy/copy_entry.cpp:201-206)
 * and recv_copy_entry's (recv_copy_entry.cpp:53), the only callers of
 * ccl_comp_copy in the tree, both on host memory by construction.  The
 * reference's memcpy / non-temporal copy (comp.cpp:60-74) on the calling
 * thread, no pointer classified (integration/0006).  Errors throw.        */
ccl::status ccl_comp_copy_host(const void* in_buf, void* out_buf, size_t bytes, bool use_nontemporal);

#endif
