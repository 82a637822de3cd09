// ref_fp16native.cpp — TEST INFRASTRUCTURE ONLY.
//
// The reference's avx512fp16 fp16 reduce (native half-precision math,
// /root/reference/src/comp/fp16/fp16_intrisics.cpp:23-41 and
// fp16_intrisics.hpp:150-176, the 512FP16 instance of
// CCL_FP16_DEFINE_REDUCE_FUNC) behind a C-ABI call, for golden vectors
// (tests/golden/make_ref_vectors.py) on a CPU with AVX512_FP16.  gcc 11 lacks
// the _mm512_*_ph intrinsics (the reference's own cmake switches the impl
// off there, cmake/helpers.cmake:97-102), so `make -C oracle ref` builds this
// one with ROCm's clang++ from the sources where they lie, with
// CCL_FP16_AVX512FP16_COMPILER defined as that cmake check would.  As in
// ref_harness.cpp the env-reading dispatcher (fp16_intrisics.hpp:204-248) is
// bypassed: the per-impl body is called with the op wrap it would pick.
//
// Nothing in the product (oneccl_amd/, include/) links or loads this.
#include "comp/fp16/fp16_intrisics.hpp"

#include <cstddef>

namespace {

ccl_fp16_reduction_func_ptr_512FP16 op_512fp16(int op) {
    switch (op) {
        case 0: return &fp16_sum_wrap_512FP16;
        case 1: return &fp16_prod_wrap_512FP16;
        case 2: return &fp16_min_wrap_512FP16;
        case 3: return &fp16_max_wrap_512FP16;
        default: return nullptr;
    }
}

__attribute__((target("avx512fp16,avx512bw,avx512vl,avx512f"))) void run(const void* in, void* inout, size_t n,
                                                                          ccl_fp16_reduction_func_ptr_512FP16 f) {
    ccl_fp16_reduce_impl_512FP16(in, inout, n, f);
}

}  // namespace

extern "C" {
// 1 when this CPU can run it (AVX512_FP16), else 0
int ref_fp16native_supported(void) { return __builtin_cpu_supports("avx512fp16") ? 1 : 0; }

// inout = op(in, inout) over n fp16 elements by the avx512fp16 impl; 0 ok
int ref_fp16native_reduce(const void* in, void* inout, size_t n, int op) {
    ccl_fp16_reduction_func_ptr_512FP16 f = op_512fp16(op);
    if (!f || !ref_fp16native_supported()) return -1;
    run(in, inout, n, f);
    return 0;
}
}
