// host_reduce.cpp — the drop-in's CPU reduce for small host-resident chunks
// (include/mi_host_reduce.h).
//
// A oneCCL worker reduces a received chunk that sits in a host staging buffer
// (recv_reduce_entry.hpp:99-135, comm_buf from sched->alloc_buffer).  Below a
// few MiB a GPU round trip (dispatch + completion, plus PCIe for the data)
// costs several times what one core needs for the same chunk,
// so the shim (comp.cpp) keeps such chunks on the calling thread, as the
// reference does, and sends larger ones and every device buffer to the HIP
// kernels.  This file is that CPU path.  It computes exactly what the device
// kernels compute for the same flags (include/mi_reduce.h MI_F_*):
//   * CCL_REDUCE (src/comp/comp.cpp:31-58): wrap-around integer sum/prod,
//     std::min/std::max(in, inout) operand order;
//   * bf16 (bf16.cpp:63-85, bf16_intrisics.hpp:62-114): fp32 math, truncation
//     or VCVTNEPS2BF16 rounding, MINPS/MAXPS(in, inout) order;
//   * fp16 (fp16_intrisics.hpp:95-148): VCVTPH2PS / VCVTPS2PH imm8=0 (F16C),
//     MINPS order;
//   * the K-input left fold, per-step rounding or fp32 accumulation with one
//     final rounding and the truncated count%16 tail of keep-precision mode
//     (comp.cpp:202-249, bf16.cpp:130-149).
// x86 NaN propagation of ADDPS/MULPS(in, inout) is reproduced for bf16/fp16
// (a NaN operand comes back quieted, `in`'s first), so the bits match the
// reference's own AVX-512 code (tests/golden/ref_vectors.npz).
//
// Built with -O3 -mavx2 -mf16c -mfma (oneccl_amd/build.py): every loop below
// is written so that gcc vectorizes it.  mi_host_supported() tells the caller
// whether this CPU can run it; the shim checks it before calling anything
// else here.
#include "../../include/mi_host_reduce.h"

#include <immintrin.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "../../include/mi_reduce.h"
#include "host_lp.hpp"

namespace {

constexpr int kChunk = 512;  // elements per fold block: the accumulator stays in L1
constexpr int kFanChunk = 2048;  // K-input fold of 1-8-byte types: 2-16 KiB of output per block

struct bf16_t {};
struct fp16_t {};

template <typename T>
struct HT {  // storage S, compute C
    using S = T;
    using C = T;
    static constexpr bool lp = false;
};
template <>
struct HT<bf16_t> {
    using S = uint16_t;
    using C = float;
    static constexpr bool lp = true;
};
template <>
struct HT<fp16_t> {
    using S = uint16_t;
    using C = float;
    static constexpr bool lp = true;
};

inline uint32_t f2u(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
}
inline float u2f(uint32_t u) {
    float f;
    memcpy(&f, &u, 4);
    return f;
}

// ---- conversions ----------------------------------------------------------
inline float bf16_widen(uint16_t v) { return u2f((uint32_t)v << 16); }
inline uint16_t bf16_trunc(float f) { return (uint16_t)(f2u(f) >> 16); }
// VCVTNEPS2BF16: zero/denormal -> signed zero, NaN -> quiet NaN (payload's
// high half kept), otherwise round to nearest even.
inline uint16_t bf16_rne(float f) {
    const uint32_t u = f2u(f);
    const uint32_t r = (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
    const uint32_t nan = (u >> 16) | 0x40u;
    const uint32_t zero = (u >> 16) & 0x8000u;
    const uint32_t a = u & 0x7FFFFFFFu;
    return (uint16_t)((u & 0x7F800000u) == 0 ? zero : (a > 0x7F800000u ? nan : r));
}

// fp16 <-> fp32 by the F16C instructions the reference itself uses
// (VCVTPH2PS, VCVTPS2PH imm8 = 0), 8 lanes at a time with a scalar tail.
void fp16_to_f32(const uint16_t* s, float* d, size_t n) {
    size_t i = 0;
    for (; i + 8 <= n; i += 8)
        _mm256_storeu_ps(d + i, _mm256_cvtph_ps(_mm_loadu_si128(reinterpret_cast<const __m128i*>(s + i))));
    for (; i < n; i++) d[i] = _cvtsh_ss(s[i]);
}
void f32_to_fp16(const float* s, uint16_t* d, size_t n) {
    size_t i = 0;
    for (; i + 8 <= n; i += 8)
        _mm_storeu_si128(reinterpret_cast<__m128i*>(d + i), _mm256_cvtps_ph(_mm256_loadu_ps(s + i), 0));
    for (; i < n; i++) d[i] = _cvtss_sh(s[i], 0);
}

// widen storage to compute type / round compute type to storage, per type
// (plain overloads: this file builds with the reference's -std=gnu++11)
template <typename T>
inline void widen(const T* s, T* c, size_t n) {
    for (size_t i = 0; i < n; i++) c[i] = s[i];
}
inline void widen_bf16(const uint16_t* s, float* c, size_t n) {
    for (size_t i = 0; i < n; i++) c[i] = bf16_widen(s[i]);
}

template <typename T>
inline void narrow(const T* c, T* s, size_t n, unsigned, uint64_t, uint64_t) {
    for (size_t i = 0; i < n; i++) s[i] = c[i];
}
// bf16: truncation, or RNE with elements >= trunc_from truncated
// (V_TAIL_TRUNC; the split falls in at most one block)
inline void narrow_bf16(const float* c, uint16_t* s, size_t n, unsigned v, uint64_t idx0, uint64_t trunc_from) {
    if (!(v & MI_F_BF16_RNE)) {
        for (size_t i = 0; i < n; i++) s[i] = bf16_trunc(c[i]);
        return;
    }
    size_t rne_n = n;
    if ((v & MI_F_BF16_TAIL_TRUNC16) && idx0 + n > trunc_from)
        rne_n = idx0 >= trunc_from ? 0 : (size_t)(trunc_from - idx0);
    for (size_t i = 0; i < rne_n; i++) s[i] = bf16_rne(c[i]);
    for (size_t i = rne_n; i < n; i++) s[i] = bf16_trunc(c[i]);
}

template <typename Tag>
struct Conv {  // integers, float, double: storage == compute type
    typedef typename HT<Tag>::S S;
    typedef typename HT<Tag>::C C;
    static void widen_(const S* s, C* c, size_t n) { widen(s, c, n); }
    static void narrow_(const C* c, S* s, size_t n, unsigned v, uint64_t i0, uint64_t tf) {
        narrow(c, s, n, v, i0, tf);
    }
};
template <>
struct Conv<bf16_t> {
    static void widen_(const uint16_t* s, float* c, size_t n) { widen_bf16(s, c, n); }
    static void narrow_(const float* c, uint16_t* s, size_t n, unsigned v, uint64_t i0, uint64_t tf) {
        narrow_bf16(c, s, n, v, i0, tf);
    }
};
template <>
struct Conv<fp16_t> {
    static void widen_(const uint16_t* s, float* c, size_t n) { fp16_to_f32(s, c, n); }
    static void narrow_(const float* c, uint16_t* s, size_t n, unsigned, uint64_t, uint64_t) {
        f32_to_fp16(c, s, n);
    }
};

// ---- the operator: acc' = op(in, acc) -----------------------------------------
// x86 ADDPS/MULPS(first, second) NaN rule: a NaN operand comes back
// quieted, `first`'s when both are; an invalid operation on non-NaN operands
// yields the C result (the default NaN on x86).  The compiler may swap the
// operands of a commutative + or *, so the choice is made explicit:
//   bf16/fp16 steps     first = in   (_mm512_add_ps(in, inout), bf16_intrisics.cpp:20-26)
//   float/double, and   first = acc  (CCL_REDUCE's `inout op= in` as the reference's
//   fp32 accumulation            Release build compiles it: tests/golden/ref_comp_vectors.npz)
template <typename C>
inline C nan_first(C r, C first, C second) {
    // two selects on the bits: the loops stay vectorized (a memcpy-and-branch
    // form of this cost the fp32 fold 4x)
    typedef typename std::conditional<sizeof(C) == 4, uint32_t, uint64_t>::type U;
    const U q = sizeof(C) == 4 ? (U)0x400000u : (U)0x8000000000000ull;
    U o = (second != second) ? (__builtin_bit_cast(U, second) | q) : __builtin_bit_cast(U, r);
    o = (first != first) ? (__builtin_bit_cast(U, first) | q) : o;
    return __builtin_bit_cast(C, o);
}

// integers: CCL_REDUCE's wrap-around sum/prod (computed unsigned) and
// std::min/std::max(in, inout)
template <int OP, bool INOUT_FIRST, bool IN_FIRST, typename C>
inline C op1_impl(C x, C a, std::true_type) {
    typedef typename std::make_unsigned<C>::type U;
    return OP == MI_OP_SUM ? (C)(U)((U)a + (U)x)
         : OP == MI_OP_PROD ? (C)(U)((U)a * (U)x)
         : OP == MI_OP_MIN ? ((a < x) ? a : x)
                           : ((x < a) ? a : x);
}
// floating point: std::min/max(in, inout) or MINPS/MAXPS(in, inout); sum
// and prod with the NaN rule above (IN_FIRST: a bf16/fp16 step in storage
// precision; otherwise the accumulator's NaN wins)
template <int OP, bool INOUT_FIRST, bool IN_FIRST, typename C>
inline C op1_impl(C x, C a, std::false_type) {
    C r;
    if (OP == MI_OP_SUM) r = a + x;
    else if (OP == MI_OP_PROD) r = a * x;
    else if (OP == MI_OP_MIN) r = INOUT_FIRST ? ((x < a) ? x : a) : ((a < x) ? a : x);
    else r = INOUT_FIRST ? ((x > a) ? x : a) : ((x < a) ? a : x);
    if (OP == MI_OP_SUM || OP == MI_OP_PROD) r = IN_FIRST ? nan_first(r, x, a) : nan_first(r, a, x);
    return r;
}
template <int OP, bool INOUT_FIRST, bool IN_FIRST, typename C>
inline C op1(C x, C a) {
    return op1_impl<OP, INOUT_FIRST, IN_FIRST>(x, a, std::is_integral<C>());
}

template <int OP, bool INOUT_FIRST, bool IN_FIRST, typename C>
inline void apply(const C* in, C* acc, size_t n) {
    for (size_t i = 0; i < n; i++) acc[i] = op1<OP, INOUT_FIRST, IN_FIRST>(in[i], acc[i]);
}

// ---- float / double sum and product: ADDPS/MULPS (PD) with the accumulator
// as the first source, as the reference's Release build compiles CCL_REDUCE's
// `inout op= in` (tests/golden/ref_comp_vectors.npz).  The instruction itself
// then gives the reference's NaN bits (first NaN operand quieted, the default
// NaN on an invalid operation); inline asm fixes the operand order, which
// the compiler may otherwise swap for a commutative + or *.
template <int OP>
inline __m256 vop_first(__m256 a, __m256 x) {
    __m256 r;
    if (OP == MI_OP_SUM) asm("vaddps %2, %1, %0" : "=x"(r) : "x"(a), "x"(x));
    else asm("vmulps %2, %1, %0" : "=x"(r) : "x"(a), "x"(x));
    return r;
}
template <int OP>
inline __m256d vop_first(__m256d a, __m256d x) {
    __m256d r;
    if (OP == MI_OP_SUM) asm("vaddpd %2, %1, %0" : "=x"(r) : "x"(a), "x"(x));
    else asm("vmulpd %2, %1, %0" : "=x"(r) : "x"(a), "x"(x));
    return r;
}
inline __m256 vload(const float* p) { return _mm256_loadu_ps(p); }
inline __m256d vload(const double* p) { return _mm256_loadu_pd(p); }
inline void vstore(float* p, __m256 v) { _mm256_storeu_ps(p, v); }
inline void vstore(double* p, __m256d v) { _mm256_storeu_pd(p, v); }

template <typename C, int OP>
inline void fp_group(const C* const* in, int k, size_t i, C* out) {  // W elements at i
    auto acc = vop_first<OP>(vload(in[0] + i), vload(in[1] + i));
    for (int j = 2; j < k; j++) acc = vop_first<OP>(acc, vload(in[j] + i));
    vstore(out + i, acc);
}

template <typename C, int OP>
void fold_fp(const void* const* inputs, int k, void* out, size_t count) {
    constexpr size_t W = 32 / sizeof(C);
    const C* in[MI_MAX_INPUTS];
    for (int j = 0; j < k; j++) in[j] = static_cast<const C*>(inputs[j]);
    C* o = static_cast<C*>(out);
    // Every group reads all its inputs before it stores, so `out` may alias
    // any input (the same elements of a later input are read first).
    size_t i = 0;
    if (k == 2) {  // ccl_comp_reduce: four groups per iteration, loads first
        const C* a = in[0];
        const C* x = in[1];
        for (; i + 4 * W <= count; i += 4 * W) {
            const auto a0 = vload(a + i), a1 = vload(a + i + W), a2 = vload(a + i + 2 * W), a3 = vload(a + i + 3 * W);
            const auto x0 = vload(x + i), x1 = vload(x + i + W), x2 = vload(x + i + 2 * W), x3 = vload(x + i + 3 * W);
            vstore(o + i, vop_first<OP>(a0, x0));
            vstore(o + i + W, vop_first<OP>(a1, x1));
            vstore(o + i + 2 * W, vop_first<OP>(a2, x2));
            vstore(o + i + 3 * W, vop_first<OP>(a3, x3));
        }
    }
    for (; i + W <= count; i += W) fp_group<C, OP>(in, k, i, o);
    if (i < count) {  // zero-padded last group
        const size_t r = count - i;
        alignas(32) C pad[MI_MAX_INPUTS][W] = {};
        const C* p[MI_MAX_INPUTS] = {};
        for (int j = 0; j < k; j++) {
            memcpy(pad[j], in[j] + i, r * sizeof(C));
            p[j] = pad[j];
        }
        alignas(32) C res[W];
        fp_group<C, OP>(p, k, 0, res);
        memcpy(o + i, res, r * sizeof(C));
    }
}

// float / double sum and product take fold_fp (C++11: no if constexpr in
// the in-tree build)
template <typename Tag, int OP,
          bool FP = std::is_floating_point<Tag>::value && (OP == MI_OP_SUM || OP == MI_OP_PROD)>
struct FpFold {
    static bool run(const void* const*, int, void*, size_t) { return false; }
};
template <typename Tag, int OP>
struct FpFold<Tag, OP, true> {
    static bool run(const void* const* inputs, int k, void* out, size_t count) {
        if (k < 2) return false;
        fold_fp<Tag, OP>(inputs, k, out, count);
        return true;
    }
};

// out = fold(inputs[0..k-1]), blockwise
template <typename Tag, int OP, bool INOUT_FIRST>
void fold(const void* const* inputs, int k, void* out, size_t count, unsigned v) {
    if (FpFold<Tag, OP>::run(inputs, k, out, count)) return;
    typedef typename HT<Tag>::S S;
    typedef typename HT<Tag>::C C;
    const bool lp = HT<Tag>::lp;
    const bool acc32 = lp && (v & MI_F_ACC_FP32);
    const uint64_t trunc_from = (count / 16) * 16;
    if (!lp && k == 2) {  // ccl_comp_reduce: one pass, out = op(in, inout)
        const C* a = static_cast<const C*>(inputs[0]);
        const C* x = static_cast<const C*>(inputs[1]);
        C* o = static_cast<C*>(out);
        for (size_t i = 0; i < count; i++) o[i] = op1<OP, INOUT_FIRST, false>(x[i], a[i]);
        return;
    }
    if (!lp) {  // fan-in: every input read once, per L1-sized block of an accumulator
        bool alias = false;  // out is also a later input: fold into a copy, store after every read
        for (int j = 1; j < k; j++) alias = alias || inputs[j] == out;
        alignas(64) C acc[kFanChunk];
        for (size_t b = 0; b < count; b += kFanChunk) {
            const size_t n = std::min<size_t>(kFanChunk, count - b);
            C* o = alias ? acc : static_cast<C*>(out) + b;
            const C* a = static_cast<const C*>(inputs[0]) + b;
            const C* x = static_cast<const C*>(inputs[1]) + b;
            for (size_t i = 0; i < n; i++) o[i] = op1<OP, INOUT_FIRST, false>(x[i], a[i]);
            for (int j = 2; j < k; j++) apply<OP, INOUT_FIRST, false>(static_cast<const C*>(inputs[j]) + b, o, n);
            if (alias) memcpy(static_cast<C*>(out) + b, acc, n * sizeof(C));
        }
        return;
    }
    alignas(64) C acc[kChunk];
    alignas(64) C x[kChunk];
    alignas(64) S tmp[kChunk];
    const unsigned vstep = v & ~MI_F_BF16_TAIL_TRUNC16;
    for (size_t b = 0; b < count; b += kChunk) {
        const size_t n = std::min<size_t>(kChunk, count - b);
        Conv<Tag>::widen_(static_cast<const S*>(inputs[0]) + b, acc, n);
        for (int j = 1; j < k; j++) {
            Conv<Tag>::widen_(static_cast<const S*>(inputs[j]) + b, x, n);
            if (acc32) apply<OP, INOUT_FIRST, false>(x, acc, n);  // fp32 accumulation: CCL_REDUCE(float) order
            else apply<OP, INOUT_FIRST, HT<Tag>::lp>(x, acc, n);
            if (lp && !acc32) {  // round to storage after every step (chained calls)
                Conv<Tag>::narrow_(acc, tmp, n, vstep, b, trunc_from);
                Conv<Tag>::widen_(tmp, acc, n);
            }
        }
        Conv<Tag>::narrow_(acc, static_cast<S*>(out) + b, n, acc32 ? v : vstep, b, trunc_from);
    }
}

// ---- bf16 / fp16: the SIMD fold of host_lp.hpp ----------------------------------
// 8 AVX2 lanes; VCVTNEPS2BF16 (an AVX512_BF16 instruction) restated in the
// integer domain.  CPUs with AVX-512 take the 16-lane form of
// host_reduce_avx512.cpp instead (mi_host_reduce).
struct V8 {
    typedef __m256 F;
    typedef __m128i H;
    static const int W = 8;
    static F widen_bf16(H h) { return _mm256_castsi256_ps(_mm256_slli_epi32(_mm256_cvtepu16_epi32(h), 16)); }
    static F widen_fp16(H h) { return _mm256_cvtph_ps(h); }
    static F load_bf16(const uint16_t* p) { return widen_bf16(_mm_loadu_si128(reinterpret_cast<const __m128i*>(p))); }
    static F load_fp16(const uint16_t* p) { return widen_fp16(_mm_loadu_si128(reinterpret_cast<const __m128i*>(p))); }
    static H pack16(__m256i v) {  // 8 lanes < 2^16 -> 8 x u16, in order
        const __m256i p = _mm256_packus_epi32(v, v);
        return _mm256_castsi256_si128(_mm256_permute4x64_epi64(p, 0x08));
    }
    static H bits_bf16_trunc(F f) { return pack16(_mm256_srli_epi32(_mm256_castps_si256(f), 16)); }
    static H bits_bf16_rne(F f) {  // VCVTNEPS2BF16
        const __m256i u = _mm256_castps_si256(f);
        const __m256i hi = _mm256_srli_epi32(u, 16);
        __m256i r = _mm256_add_epi32(_mm256_add_epi32(u, _mm256_set1_epi32(0x7FFF)),
                                     _mm256_and_si256(hi, _mm256_set1_epi32(1)));
        r = _mm256_srli_epi32(r, 16);
        const __m256i nan = _mm256_or_si256(hi, _mm256_set1_epi32(0x40));
        const __m256i zero = _mm256_and_si256(hi, _mm256_set1_epi32(0x8000));
        const __m256i is_nan =
            _mm256_cmpgt_epi32(_mm256_and_si256(u, _mm256_set1_epi32(0x7FFFFFFF)), _mm256_set1_epi32(0x7F800000));
        const __m256i is_den =
            _mm256_cmpeq_epi32(_mm256_and_si256(u, _mm256_set1_epi32(0x7F800000)), _mm256_setzero_si256());
        r = _mm256_blendv_epi8(r, nan, is_nan);
        return pack16(_mm256_blendv_epi8(r, zero, is_den));
    }
    static H bits_fp16(F f) { return _mm256_cvtps_ph(f, 0); }
    static F keep_hi16(F f) { return _mm256_and_ps(f, _mm256_castsi256_ps(_mm256_set1_epi32((int)0xFFFF0000u))); }
    static F add(F a, F b) { return _mm256_add_ps(a, b); }
    static F mul(F a, F b) { return _mm256_mul_ps(a, b); }
    static F min(F a, F b) { return _mm256_min_ps(a, b); }
    static F max(F a, F b) { return _mm256_max_ps(a, b); }
    // a NaN operand comes back quieted, x (`in`) first
    static F nan_first(F r, F x, F a) {
        const F q = _mm256_castsi256_ps(_mm256_set1_epi32(0x400000));
        r = _mm256_blendv_ps(r, _mm256_or_ps(a, q), _mm256_cmp_ps(a, a, _CMP_UNORD_Q));
        return _mm256_blendv_ps(r, _mm256_or_ps(x, q), _mm256_cmp_ps(x, x, _CMP_UNORD_Q));
    }
    static void store(uint16_t* p, H h) { _mm_storeu_si128(reinterpret_cast<__m128i*>(p), h); }
};

using mi_host::FoldFn;

template <typename Tag, int OP>
struct Pick {
    static FoldFn get(unsigned v) {
        const bool mm = OP == MI_OP_MIN || OP == MI_OP_MAX;
        if (mm && std::is_floating_point<typename HT<Tag>::C>::value && (v & MI_F_MINMAX_INOUT_FIRST))
            return &fold<Tag, OP, true>;
        return &fold<Tag, OP, false>;
    }
};
// bf16 / fp16: 16 AVX-512 lanes where the CPU has them (with the native
// VCVTNEPS2BF16 where it has AVX512_BF16), else 8 AVX2 lanes
struct Isa {
    bool avx512, bf16;
    Isa() {
        __builtin_cpu_init();
        avx512 = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
                 __builtin_cpu_supports("avx512vl");
        bf16 = avx512 && __builtin_cpu_supports("avx512bf16");
        // MI_HOST_ISA=avx2 | avx512 (no AVX512_BF16): narrower forms, for tests
        if (const char* e = getenv("MI_HOST_ISA")) {
            if (strcmp(e, "avx2") == 0) avx512 = bf16 = false;
            if (strcmp(e, "avx512") == 0) bf16 = false;
        }
    }
};
const Isa& isa() {
    static const Isa i;
    return i;
}
FoldFn pick_lp(bool bf, int op, unsigned v) {
    if (isa().avx512) return mi_host::pick_lp_avx512(bf, op, v, isa().bf16);
    return mi_host::pick_lp<V8>(bf, op, v);
}
template <int OP>
struct Pick<bf16_t, OP> {
    static FoldFn get(unsigned v) { return pick_lp(true, OP, v); }
};
template <int OP>
struct Pick<fp16_t, OP> {
    static FoldFn get(unsigned v) { return pick_lp(false, OP, v); }
};

template <typename Tag, int OP>
FoldFn pick_order(unsigned v) {
    return Pick<Tag, OP>::get(v);
}

template <typename Tag>
FoldFn pick_op(int op, unsigned v) {
    switch (op) {
        case MI_OP_SUM: return pick_order<Tag, MI_OP_SUM>(v);
        case MI_OP_PROD: return pick_order<Tag, MI_OP_PROD>(v);
        case MI_OP_MIN: return pick_order<Tag, MI_OP_MIN>(v);
        case MI_OP_MAX: return pick_order<Tag, MI_OP_MAX>(v);
        default: return nullptr;
    }
}

FoldFn pick(int dt, int op, unsigned v) {
    switch (dt) {
        case MI_INT8: return pick_op<int8_t>(op, v);
        case MI_UINT8: return pick_op<uint8_t>(op, v);
        case MI_INT16: return pick_op<int16_t>(op, v);
        case MI_UINT16: return pick_op<uint16_t>(op, v);
        case MI_INT32: return pick_op<int32_t>(op, v);
        case MI_UINT32: return pick_op<uint32_t>(op, v);
        case MI_INT64: return pick_op<int64_t>(op, v);
        case MI_UINT64: return pick_op<uint64_t>(op, v);
        case MI_FLOAT16: return pick_op<fp16_t>(op, v);
        case MI_FLOAT32: return pick_op<float>(op, v);
        case MI_FLOAT64: return pick_op<double>(op, v);
        case MI_BFLOAT16: return pick_op<bf16_t>(op, v);
        default: return nullptr;
    }
}

// Variant bits that change results for (dtype, op, k) — the same
// canonicalisation as the device path (mi_reduce.hip canon_flags).
unsigned canon(int dt, int op, unsigned f, int k) {
    const bool mm = op == MI_OP_MIN || op == MI_OP_MAX;
    switch (dt) {
        case MI_FLOAT32:
        case MI_FLOAT64: return mm ? (f & MI_F_MINMAX_INOUT_FIRST) : 0u;
        case MI_FLOAT16: {
            unsigned v = (mm ? (f & (MI_F_MINMAX_INOUT_FIRST | MI_F_FP16_NATIVE_MINMAX)) : 0u) | (f & MI_F_ACC_FP32);
            if (k <= 1 || (k == 2 && mm)) v &= ~MI_F_ACC_FP32;  // a sum/prod step keeps its NaN order
            return v;
        }
        case MI_BFLOAT16: {
            unsigned v = (mm ? (f & MI_F_MINMAX_INOUT_FIRST) : 0u) |
                         (f & (MI_F_BF16_RNE | MI_F_ACC_FP32 | MI_F_BF16_TAIL_TRUNC16));
            if (!((v & MI_F_ACC_FP32) && (v & MI_F_BF16_RNE))) v &= ~MI_F_BF16_TAIL_TRUNC16;
            if (k == 2 && mm && !(v & MI_F_BF16_TAIL_TRUNC16)) v &= ~MI_F_ACC_FP32;
            return v;
        }
        default: return 0u;
    }
}

size_t dsize(int dt) {
    switch (dt) {
        case MI_INT8: case MI_UINT8: return 1;
        case MI_INT16: case MI_UINT16: case MI_FLOAT16: case MI_BFLOAT16: return 2;
        case MI_INT32: case MI_UINT32: case MI_FLOAT32: return 4;
        case MI_INT64: case MI_UINT64: case MI_FLOAT64: return 8;
        default: return 0;
    }
}

}  // namespace

extern "C" {

int mi_host_supported(void) {
    __builtin_cpu_init();
    return (__builtin_cpu_supports("avx2") && __builtin_cpu_supports("f16c") && __builtin_cpu_supports("fma")) ? 1
                                                                                                              : 0;
}

// VMINPH/VMAXPH return the selected operand as stored, where the fp32 route's
// VCVTPH2PS quiets it; they differ only when the accumulator's start is a
// NaN, which a min/max fold then returns (oracle/fp16_native_check.c).  The
// start is kept per block before the fold, since `out` may be that input.
static int fold_fp16_native(FoldFn fn, const void* const* inputs, int k, void* out, size_t count, unsigned v) {
    uint16_t raw[kChunk];
    for (size_t b = 0; b < count; b += kChunk) {
        const size_t n = std::min<size_t>(kChunk, count - b);
        memcpy(raw, static_cast<const uint16_t*>(inputs[0]) + b, n * 2);
        const void* ins[MI_MAX_INPUTS];
        for (int j = 0; j < k; j++) ins[j] = static_cast<const uint16_t*>(inputs[j]) + b;
        uint16_t* o = static_cast<uint16_t*>(out) + b;
        fn(ins, k, o, n, v);
        for (size_t i = 0; i < n; i++)
            if ((raw[i] & 0x7C00u) == 0x7C00u && (raw[i] & 0x03FFu)) o[i] = raw[i];
    }
    return 0;
}

int mi_host_reduce(const void* const* inputs, int k, void* out, size_t count, int dtype, int op, unsigned flags) {
    if (!dsize(dtype)) return MI_E_INVALID;
    if (op < MI_OP_SUM || op > MI_OP_MAX) return MI_E_INVALID;
    if (k < 1 || k > MI_MAX_INPUTS) return MI_E_INVALID;
    if (count == 0) return 0;
    if (!inputs || !out) return MI_E_INVALID;
    for (int i = 0; i < k; i++)
        if (!inputs[i]) return MI_E_INVALID;
    const unsigned v = canon(dtype, op, flags, k);
    if (k == 1 && !(v & MI_F_ACC_FP32)) {  // nothing to combine
        if (out != inputs[0]) memmove(out, inputs[0], count * dsize(dtype));
        return 0;
    }
    if (v & MI_F_FP16_NATIVE_MINMAX) {  // fp16 min/max as VMINPH/VMAXPH (avx512fp16 impl)
        FoldFn fn = pick(dtype, op, v & ~MI_F_FP16_NATIVE_MINMAX);
        if (!fn) return MI_E_UNSUPPORTED;
        return fold_fp16_native(fn, inputs, k, out, count, v & ~MI_F_FP16_NATIVE_MINMAX);
    }
    FoldFn fn = pick(dtype, op, v);
    if (!fn) return MI_E_UNSUPPORTED;
    fn(inputs, k, out, count, v);
    return 0;
}

// Host-to-host ccl_comp_copy (src/comp/comp.cpp:60-74).  With `nontemporal`
// the destination is written with streaming stores from its first 64-byte
// boundary on (no read-for-ownership of the destination lines, nothing left
// in the caches), as the reference's memcpy_nontemporal does for copies above
// 256 bytes (src/common/utils/memcpy.cpp:49-125); the bytes are the same
// either way.  Unaligned 32-byte loads, 128 bytes per step.
int mi_host_copy(void* dst, const void* src, size_t bytes, int nontemporal) {
    if (bytes == 0) return 0;
    if (!src || !dst) return MI_E_INVALID;
    if (!nontemporal || bytes <= 256) {
        memcpy(dst, src, bytes);
        return 0;
    }
    char* d = static_cast<char*>(dst);
    const char* s = static_cast<const char*>(src);
    const size_t head = (64 - (reinterpret_cast<uintptr_t>(d) & 63)) & 63;
    memcpy(d, s, head);
    size_t i = head;
    for (; i + 128 <= bytes; i += 128) {
        const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i));
        const __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + 32));
        const __m256i c = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + 64));
        const __m256i e = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + 96));
        _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i), a);
        _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i + 32), b);
        _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i + 64), c);
        _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i + 96), e);
    }
    for (; i + 32 <= bytes; i += 32)
        _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i),
                            _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i)));
    memcpy(d + i, s + i, bytes - i);
    _mm_sfence();  // the streaming stores are visible before the caller sends the buffer
    return 0;
}

int mi_host_convert(const void* src, int src_dtype, void* dst, int dst_dtype, size_t count, unsigned flags) {
    if (count == 0) return 0;
    if (!src || !dst) return MI_E_INVALID;
    if (src_dtype == MI_FLOAT32 && dst_dtype == MI_BFLOAT16) {
        const float* s = static_cast<const float*>(src);
        uint16_t* d = static_cast<uint16_t*>(dst);
        const uint64_t trunc_from = (flags & MI_F_BF16_TAIL_TRUNC16) ? (count / 16) * 16 : count;
        for (size_t b = 0; b < count; b += kChunk) {
            const size_t n = std::min<size_t>(kChunk, count - b);
            narrow_bf16(s + b, d + b, n, (flags & MI_F_BF16_RNE) | MI_F_BF16_TAIL_TRUNC16, b, trunc_from);
        }
        return 0;
    }
    if (src_dtype == MI_FLOAT32 && dst_dtype == MI_FLOAT16) {
        f32_to_fp16(static_cast<const float*>(src), static_cast<uint16_t*>(dst), count);
        return 0;
    }
    if (src_dtype == MI_BFLOAT16 && dst_dtype == MI_FLOAT32) {
        widen_bf16(static_cast<const uint16_t*>(src), static_cast<float*>(dst), count);
        return 0;
    }
    if (src_dtype == MI_FLOAT16 && dst_dtype == MI_FLOAT32) {
        fp16_to_f32(static_cast<const uint16_t*>(src), static_cast<float*>(dst), count);
        return 0;
    }
    return MI_E_UNSUPPORTED;
}

}  // extern "C"
