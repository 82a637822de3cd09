// host_reduce_avx512.cpp — the 16-lane (AVX-512) form of the drop-in host
// path's bf16 / fp16 fold (host_lp.hpp).  Built with -mavx512f -mavx512bw
// -mavx512vl -mavx512bf16 (oneccl_amd/build.py); host_reduce.cpp calls into it
// only after checking the CPU (AVX512F/BW/VL; AVX512_BF16 for the native
// VCVTNEPS2BF16 form, the instruction the reference's avx512bf impl uses,
// src/comp/bf16/bf16_intrisics.hpp:72-76).
#include <immintrin.h>

#include <cstdint>

#include "host_lp.hpp"

namespace mi_host {
namespace {

struct V16 {
    typedef __m512 F;
    typedef __m256i H;
    static const int W = 16;
    static F widen_bf16(H h) { return _mm512_castsi512_ps(_mm512_slli_epi32(_mm512_cvtepu16_epi32(h), 16)); }
    static F widen_fp16(H h) { return _mm512_cvtph_ps(h); }
    static F load_bf16(const uint16_t* p) {
        return widen_bf16(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(p)));
    }
    static F load_fp16(const uint16_t* p) {
        return widen_fp16(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(p)));
    }
    static H bits_bf16_trunc(F f) { return _mm512_cvtepi32_epi16(_mm512_srli_epi32(_mm512_castps_si512(f), 16)); }
    static H bits_bf16_rne(F f) {  // VCVTNEPS2BF16 restated (CPUs without AVX512_BF16)
        const __m512i u = _mm512_castps_si512(f);
        const __m512i hi = _mm512_srli_epi32(u, 16);
        __m512i r = _mm512_add_epi32(_mm512_add_epi32(u, _mm512_set1_epi32(0x7FFF)),
                                     _mm512_and_si512(hi, _mm512_set1_epi32(1)));
        r = _mm512_srli_epi32(r, 16);
        const __mmask16 is_nan =
            _mm512_cmpgt_epi32_mask(_mm512_and_si512(u, _mm512_set1_epi32(0x7FFFFFFF)), _mm512_set1_epi32(0x7F800000));
        const __mmask16 is_den = _mm512_testn_epi32_mask(u, _mm512_set1_epi32(0x7F800000));
        r = _mm512_mask_or_epi32(r, is_nan, hi, _mm512_set1_epi32(0x40));
        r = _mm512_mask_and_epi32(r, is_den, hi, _mm512_set1_epi32(0x8000));
        return _mm512_cvtepi32_epi16(r);
    }
    static H bits_fp16(F f) { return _mm512_cvtps_ph(f, 0); }
    static F keep_hi16(F f) { return _mm512_castsi512_ps(_mm512_and_si512(_mm512_castps_si512(f),
                                                                          _mm512_set1_epi32((int)0xFFFF0000u))); }
    static F add(F a, F b) { return _mm512_add_ps(a, b); }
    static F mul(F a, F b) { return _mm512_mul_ps(a, b); }
    static F min(F a, F b) { return _mm512_min_ps(a, b); }
    static F max(F a, F b) { return _mm512_max_ps(a, b); }
    static F nan_first(F r, F x, F a) {  // a NaN operand comes back quieted, x (`in`) first
        const __m512i q = _mm512_set1_epi32(0x400000);
        r = _mm512_mask_mov_ps(r, _mm512_cmp_ps_mask(a, a, _CMP_UNORD_Q),
                               _mm512_castsi512_ps(_mm512_or_si512(_mm512_castps_si512(a), q)));
        return _mm512_mask_mov_ps(r, _mm512_cmp_ps_mask(x, x, _CMP_UNORD_Q),
                                  _mm512_castsi512_ps(_mm512_or_si512(_mm512_castps_si512(x), q)));
    }
    static void store(uint16_t* p, H h) { _mm256_storeu_si256(reinterpret_cast<__m256i*>(p), h); }
};

// ... and with the AVX512_BF16 instruction itself
struct V16B : V16 {
    static H bits_bf16_rne(F f) { return (H)_mm512_cvtneps_pbh(f); }
};

}  // namespace

FoldFn pick_lp_avx512(bool bf, int op, unsigned v, bool native_bf16) {
    return native_bf16 ? pick_lp<V16B>(bf, op, v) : pick_lp<V16>(bf, op, v);
}

}  // namespace mi_host
