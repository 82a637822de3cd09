// ref_harness.cpp — TEST INFRASTRUCTURE ONLY.
//
// A thin C-ABI harness over the reference's OWN bf16/fp16 reduce code, used to
// produce golden vectors (tests/golden/make_ref_vectors.py) and to pin the
// oracle's restatement against the real thing.  Built by `make -C oracle ref`
// from the sources where they lie under /root/reference (nothing is copied):
//
//   /root/reference/src/comp/bf16/bf16_intrisics.hpp  (inline per-impl reduce
//       bodies, :62-114, CCL_BF16_DEFINE_REDUCE_FUNC)
//   /root/reference/src/comp/bf16/bf16_intrisics.cpp  (bf16_{sum,prod,min,max}_wrap, :20-38)
//   /root/reference/src/comp/fp16/fp16_intrisics.hpp  (f16c 256-bit and
//       avx512f 512-bit bodies, :95-148, :179-196)
//   /root/reference/src/comp/fp16/fp16_intrisics.cpp  (fp16_*_wrap_{256,512})
//
// The dispatchers above these bodies (ccl_bf16_reduce_impl / ccl_fp16_reduce_impl,
// bf16_intrisics.hpp:121-147, fp16_intrisics.hpp:204-248) read
// ccl::global_data::env(), whose definition needs the library's global state,
// logger and hwloc/ITT closure — so this harness calls the per-impl bodies
// directly with the impl and op chosen by the caller, exactly as the
// dispatcher would.  The scalar bf16 impl (bf16.cpp:63-85), CCL_REDUCE
// (comp.cpp:31-58) and ccl_comp_batch_reduce (comp.cpp:202-249) live in
// translation units that also need the logger and datatype sources; round 3
// links those from the reference too (oracle/ref_comp_harness.cpp,
// _ref/libref_ccl_comp.so).  AVX512_FP16 native math needs gcc >= 12
// (reference cmake/helpers.cmake:97-102; gcc 11.4 here): ref_fp16native.cpp
// builds it with ROCm's clang++.
//
// Nothing in the product (oneccl_amd/, include/) links or loads this.
#include "comp/bf16/bf16_intrisics.hpp"
#include "comp/fp16/fp16_intrisics.hpp"

#include <cstddef>
#include <cstdint>

#define MI_REF_BF16_TARGET __attribute__((target("avx512bw,avx512vl,avx512f,avx512bf16")))
#define MI_REF_F16C_TARGET __attribute__((target("f16c")))
#define MI_REF_512_TARGET __attribute__((target("avx512f,avx512bw,avx512vl")))

namespace {

// the op switch of ccl_bf16_reduce_impl (bf16_intrisics.hpp:125-132)
ccl_bf16_reduction_func_ptr bf16_op(int op) {
    switch (op) {
        case 0: return &bf16_sum_wrap;
        case 1: return &bf16_prod_wrap;
        case 2: return &bf16_min_wrap;
        case 3: return &bf16_max_wrap;
        default: return nullptr;
    }
}

// the op switches of ccl_fp16_reduce_impl (fp16_intrisics.hpp:217-242)
ccl_fp16_reduction_func_ptr_256 fp16_op_256(int op) {
    switch (op) {
        case 0: return &fp16_sum_wrap_256;
        case 1: return &fp16_prod_wrap_256;
        case 2: return &fp16_min_wrap_256;
        case 3: return &fp16_max_wrap_256;
        default: return nullptr;
    }
}

ccl_fp16_reduction_func_ptr_512 fp16_op_512(int op) {
    switch (op) {
        case 0: return &fp16_sum_wrap_512;
        case 1: return &fp16_prod_wrap_512;
        case 2: return &fp16_min_wrap_512;
        case 3: return &fp16_max_wrap_512;
        default: return nullptr;
    }
}

MI_REF_BF16_TARGET void bf16_avx512f(const void* in, void* inout, size_t n, ccl_bf16_reduction_func_ptr f) {
    ccl_bf16_reduce_impl_avx512f(in, inout, n, f);
}

MI_REF_BF16_TARGET void bf16_avx512bf(const void* in, void* inout, size_t n, ccl_bf16_reduction_func_ptr f) {
    ccl_bf16_reduce_impl_avx512bf(in, inout, n, f);
}

MI_REF_F16C_TARGET void fp16_f16c(const void* in, void* inout, size_t n, ccl_fp16_reduction_func_ptr_256 f) {
    ccl_fp16_reduce_impl_256(in, inout, n, f);
}

MI_REF_512_TARGET void fp16_avx512f(const void* in, void* inout, size_t n, ccl_fp16_reduction_func_ptr_512 f) {
    ccl_fp16_reduce_impl_512(in, inout, n, f);
}

MI_REF_BF16_TARGET void store_bf16_avx512f(const float* src, uint16_t* dst) {
    ccl_fp32_store_as_bf16_avx512f(src, dst);
}

MI_REF_BF16_TARGET void store_bf16_avx512bf(const float* src, uint16_t* dst) {
    ccl_fp32_store_as_bf16_avx512bf(src, dst);
}

MI_REF_BF16_TARGET void load_bf16(const uint16_t* src, float* dst) { ccl_bf16_load_as_fp32(src, dst); }

}  // namespace

extern "C" {

// bf16 reduce through the reference's impl body.  impl: 1 = avx512f
// (truncation), 2 = avx512bf (VCVTNEPS2BF16); ccl_bf16_impl_type values.
// Returns 0, or -1 for an impl/op the reference would reject.
int ref_bf16_reduce(int impl, int op, const uint16_t* in, uint16_t* inout, size_t count) {
    ccl_bf16_reduction_func_ptr f = bf16_op(op);
    if (!f) return -1;
    if (impl == ccl_bf16_avx512f)
        bf16_avx512f(in, inout, count, f);
    else if (impl == ccl_bf16_avx512bf)
        bf16_avx512bf(in, inout, count, f);
    else
        return -1;
    return 0;
}

// fp16 reduce through the reference's impl body.  impl: 2 = f16c (8-wide),
// 3 = avx512f (16-wide); ccl_fp16_impl_type values.
int ref_fp16_reduce(int impl, int op, const uint16_t* in, uint16_t* inout, size_t count) {
    if (impl == ccl_fp16_f16c) {
        ccl_fp16_reduction_func_ptr_256 f = fp16_op_256(op);
        if (!f) return -1;
        fp16_f16c(in, inout, count, f);
        return 0;
    }
    if (impl == ccl_fp16_avx512f) {
        ccl_fp16_reduction_func_ptr_512 f = fp16_op_512(op);
        if (!f) return -1;
        fp16_avx512f(in, inout, count, f);
        return 0;
    }
    return -1;
}

// 16-element fp32 -> bf16 stores of the two AVX-512 impls
// (bf16_intrisics.hpp:67-76); count must be a multiple of 16.
int ref_fp32_to_bf16(int impl, const float* src, uint16_t* dst, size_t count) {
    if (count % 16) return -1;
    for (size_t i = 0; i < count; i += 16) {
        if (impl == ccl_bf16_avx512f)
            store_bf16_avx512f(src + i, dst + i);
        else if (impl == ccl_bf16_avx512bf)
            store_bf16_avx512bf(src + i, dst + i);
        else
            return -1;
    }
    return 0;
}

// 16-element bf16 -> fp32 load (bf16_intrisics.hpp:62-65).
int ref_bf16_to_fp32(const uint16_t* src, float* dst, size_t count) {
    if (count % 16) return -1;
    for (size_t i = 0; i < count; i += 16) load_bf16(src + i, dst + i);
    return 0;
}

}  // extern "C"
