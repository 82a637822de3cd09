/*
 * mi_ccl_lp_host.hpp — the bf16/fp16 reduce of oneCCL's MPI user ops, for a
 * caller whose operands are host memory by construction.  Defined by the
 * drop-in shim oneccl_amd/csrc/comp.cpp; the patch a maintainer applies is
 * integration/0002.
 *
 * With the MPI transport (the default) a build without SYCL selects the
 * `direct` allreduce for every size (src/coll/selection/selector_allreduce.cpp:
 * 54-57), and MPI then runs the reduction inside its user ops on its own
 * host buffers:
 *   bf16_base_op -> ccl_bf16_reduce(in, *length, inout, nullptr, op)
 *                                      (src/atl/mpi/atl_mpi_ctx.cpp:87-92)
 *   fp16_base_op -> ccl_fp16_reduce_impl(in, inout, len, op)   (:57-63)
 * Those bodies are CPU code: the operands are MPI-owned host memory.  These
 * two entries say so, as a schedule without a stream says so to
 * ccl_comp_reduce (src/comp/comp.cpp:136-142): a bucket at or below the
 * dispatcher's threshold is folded on the calling thread's CPU with no
 * pointer looked up; a larger one looks its operands up once, to choose the
 * GPU's zero-copy (pinned) or staged (pageable) route.
 *
 * Semantics are those of ccl_bf16_reduce (src/comp/bf16/bf16.cpp:87-110) and
 * ccl_fp16_reduce (src/comp/fp16/fp16.cpp:41-53): *out_cnt = in_cnt when
 * out_cnt is not null; rounding and min/max operand order follow the impl
 * type (CPUID + CCL_BF16 / CCL_FP16, src/common/env/env.cpp:711-720); an fp16
 * impl outside {f16c, avx512f, avx512fp16} computes nothing, as
 * fp16_intrisics.hpp:214-247; an op outside sum/prod/min/max is CCL_FATAL.
 * Device pointers must not be passed (they are dereferenced on the host).
 *
 * Include after a header that declares ccl::reduction (oneapi/ccl/types.hpp).
 */
#ifndef MI_CCL_LP_HOST_HPP
#define MI_CCL_LP_HOST_HPP

#include <cstddef>

void ccl_bf16_reduce_host(const void* in_buf, size_t in_cnt, void* inout_buf, size_t* out_cnt,
                          ccl::reduction reduction_op);

void ccl_fp16_reduce_host(const void* in_buf, size_t in_cnt, void* inout_buf, size_t* out_cnt,
                          ccl::reduction reduction_op);

#endif
