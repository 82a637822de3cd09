/*
 * mi_host_reduce.h — the drop-in's CPU reduce for small host-resident chunks
 * (oneccl_amd/csrc/host_reduce.cpp, linked into libccl_comp_hip.so).
 *
 * oneCCL reduces each received chunk on the worker thread that received it,
 * in host staging memory (src/sched/entry/recv_reduce_entry.hpp:99-135).
 * For such a chunk below the crossover of DESIGN.md §6 a GPU round trip costs
 * more than the reduce itself, so the shim (comp.cpp) reduces it here, on the
 * calling thread, and sends larger host chunks and all device buffers to the
 * HIP kernels of mi_reduce.h.  Same semantics, same flags (MI_F_*) as the
 * device entry points: the results are bit-identical to theirs.
 *
 * Host pointers only (pageable or pinned).  Synchronous.  Return codes as in
 * mi_reduce.h (0 ok, MI_E_* < 0).
 */
#ifndef MI_HOST_REDUCE_H
#define MI_HOST_REDUCE_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 1 if this CPU has what the host path is built for (AVX2, F16C, FMA);
 * 0: every reduce goes to the GPU. */
int mi_host_supported(void);

/* out = left fold of inputs[0..k-1] (1 <= k <= MI_MAX_INPUTS): acc =
 * inputs[0]; acc = op(inputs[j], acc); exactly mi_reduce_multi's semantics
 * for (dtype, op, flags).  `out` may alias inputs[0]. */
int mi_host_reduce(const void* const* inputs, int k, void* out, size_t count,
                   int dtype, int op, unsigned flags);

/* Host-to-host copy (ccl_comp_copy, src/comp/comp.cpp:60-74).  nontemporal:
 * streaming stores above 256 bytes, as the reference's memcpy_nontemporal
 * (src/common/utils/memcpy.cpp:49-125); else a memcpy.  No overlap. */
int mi_host_copy(void* dst, const void* src, size_t bytes, int nontemporal);

/* fp32 <-> bf16 / fp16 array conversion, mi_convert's semantics. */
int mi_host_convert(const void* src, int src_dtype, void* dst, int dst_dtype,
                    size_t count, unsigned flags);

#ifdef __cplusplus
}
#endif

#endif /* MI_HOST_REDUCE_H */
