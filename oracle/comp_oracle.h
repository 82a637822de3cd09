/*
 * comp_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of oneCCL's local reduction (src/comp, reference snapshot
 * 2024-12-20).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the
 * timed CPU baseline — never as the product path.  The product is the HIP
 * library built from oneccl_amd/csrc (include/mi_reduce.h).
 *
 * Parity pinning: see oracle/README.md (reference KATs from
 * tests/functional + the survey's recorded probes of the compiled reference
 * + exhaustive cross-checks of the conversion/min-max restatements against
 * the x86 instructions the reference calls, run where the CPU has them).
 */
#ifndef COMP_ORACLE_H
#define COMP_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ccl_bf16_impl_type, src/comp/bf16/bf16_utils.hpp:26 */
enum { ORC_BF16_SCALAR = 0, ORC_BF16_AVX512F = 1, ORC_BF16_AVX512BF = 2 };
/* ccl_fp16_impl_type, src/comp/fp16/fp16_utils.hpp:26-32 */
enum {
    ORC_FP16_NO_COMPILER = 0,
    ORC_FP16_NO_HW = 1,
    ORC_FP16_F16C = 2,
    ORC_FP16_AVX512F = 3,
    ORC_FP16_AVX512FP16 = 4
};

/* ccl_comp_reduce_regular, src/comp/comp.cpp:76-121 (custom op excluded).
 * Returns 0, or -1 on an unknown dtype/op (the reference CCL_FATALs). */
int orc_comp_reduce(const void* in_buf, size_t in_count, void* inout_buf,
                    size_t* out_count, int dtype, int op, int bf16_impl,
                    int fp16_impl);

/* Range-split over `nthreads` pthreads — what CCL_WORKER_COUNT=W achieves
 * through the parallelizer (src/parallelizer/parallelizer.cpp:230-244).   */
int orc_comp_reduce_mt(const void* in_buf, size_t in_count, void* inout_buf,
                       int dtype, int op, int bf16_impl, int fp16_impl,
                       int nthreads);

/* ccl_comp_batch_reduce, src/comp/comp.cpp:202-249.  offsets[] are element
 * offsets into in_buf (offsets[0] is unused, as in the reference). */
int orc_comp_batch_reduce(const void* in_buf, const size_t* offsets,
                          size_t n_offsets, size_t in_count, void* inout_buf,
                          size_t* out_count, int dtype, int op,
                          int bf16_keep_precision_mode, float* tmp, float* acc,
                          int bf16_impl, int fp16_impl);

/* ccl_convert_{fp32_to_bf16,bf16_to_fp32}_arrays, src/comp/bf16/bf16.cpp:113-169 */
void orc_convert_fp32_to_bf16_arrays(const float* fp32_buf, uint16_t* bf16_buf,
                                     size_t count, int bf16_impl);
void orc_convert_bf16_to_fp32_arrays(const uint16_t* bf16_buf, float* fp32_buf,
                                     size_t count);
void orc_convert_fp32_to_fp16_arrays(const float* fp32_buf, uint16_t* fp16_buf, size_t count);
void orc_convert_fp16_to_fp32_arrays(const uint16_t* fp16_buf, float* fp32_buf, size_t count);

/* Scalar conversions (exposed for the unit tests). */
float orc_bf16_to_fp32(uint16_t v);
uint16_t orc_fp32_to_bf16_trunc(float f);
uint16_t orc_fp32_to_bf16_rne(float f); /* VCVTNEPS2BF16 semantics */
float orc_fp16_to_fp32(uint16_t h);     /* VCVTPH2PS semantics */
uint16_t orc_fp32_to_fp16_rne(float f); /* VCVTPS2PH imm8=0 semantics */

/* Oracle extension (no reference function): lp fan-in accumulated in fp32
 * for fp16 as well as bf16; single RNE rounding at the end. */
int orc_lp_fanin_acc_fp32(const void* const* inputs, int k, void* out,
                          size_t count, int dtype, int op, int bf16_rne,
                          int minmax_inout_first);

#ifdef __cplusplus
}
#endif
#endif
