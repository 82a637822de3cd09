// host_lp.hpp — the bf16 / fp16 fold of the drop-in's host path, generic
// over the SIMD width (included by host_reduce.cpp with 8 AVX2 lanes and by
// host_reduce_avx512.cpp with 16 AVX-512 lanes).
//
// The reference's own instructions where the ISA has them (VADDPS / VMULPS /
// VMINPS / VMAXPS with `in` as the first source, VCVTPH2PS, VCVTPS2PH imm8 =
// 0, and VCVTNEPS2BF16 on CPUs with AVX512_BF16), so operand order, rounding
// and NaN propagation are those of its AVX-512 bodies
// (src/comp/bf16/bf16_intrisics.hpp:62-114, fp16_intrisics.hpp:95-148).
// Partial groups run on zero-padded copies, as the reference's masked tails
// do.  A traits class V supplies the vectors:
//   F / H       W floats / W u16 storage values
//   load_bf16, load_fp16, widen_bf16, widen_fp16 : storage -> F
//   bits_bf16_trunc, bits_bf16_rne, bits_fp16    : F -> H
//   keep_hi16 (bf16 truncation in place), add, mul, min, max, nan_first, store
#pragma once

#include <cstdint>
#include <cstring>

#include "../../include/mi_reduce.h"

namespace mi_host {

typedef void (*FoldFn)(const void* const*, int, void*, size_t, unsigned);

template <typename V, int OP, bool INOUT_FIRST, bool ACC32>
inline typename V::F vop(typename V::F x, typename V::F a) {  // acc' = op(in = x, acc = a)
    switch (OP) {
        // ADDPS / MULPS(in, acc): the compiler may swap the operands of the
        // commutative intrinsics, so the both-NaN choice is made explicit.
        // The fp32 accumulation of keep-precision is CCL_REDUCE(float)'s
        // `acc += tmp` (comp.cpp:223-229), whose accumulator NaN wins
        // (tests/golden/ref_comp_vectors.npz).
        case MI_OP_SUM: return ACC32 ? V::nan_first(V::add(x, a), a, x) : V::nan_first(V::add(x, a), x, a);
        case MI_OP_PROD: return ACC32 ? V::nan_first(V::mul(x, a), a, x) : V::nan_first(V::mul(x, a), x, a);
        // MINPS(in, inout) | std::min(in, inout) == MINPS(inout, in)
        case MI_OP_MIN: return INOUT_FIRST ? V::min(x, a) : V::min(a, x);
        default: return INOUT_FIRST ? V::max(x, a) : V::max(a, x);
    }
}

template <typename V, bool BF, bool RNE>
struct LpConv {
    typedef typename V::F F;
    typedef typename V::H H;
    static F load(const uint16_t* p) { return BF ? V::load_bf16(p) : V::load_fp16(p); }
    static H store_bits(F v) { return !BF ? V::bits_fp16(v) : (RNE ? V::bits_bf16_rne(v) : V::bits_bf16_trunc(v)); }
    static F round_trip(F v) {  // storage precision between steps
        if (BF && !RNE) return V::keep_hi16(v);
        const H h = store_bits(v);
        return BF ? V::widen_bf16(h) : V::widen_fp16(h);
    }
};

// V::W elements at src[j] + i -> dst + i; OUT_RNE: the final rounding (RNE,
// or truncation for keep-precision's count % 16 tail)
template <typename V, bool BF, int OP, bool INOUT_FIRST, bool ACC32, bool RNE, bool OUT_RNE>
inline void lp_group(const uint16_t* const* src, int k, size_t i, uint16_t* dst) {
    typedef LpConv<V, BF, RNE> C;
    typename V::F acc = C::load(src[0] + i);
    for (int j = 1; j < k; j++) {
        if (!ACC32 && j > 1) acc = C::round_trip(acc);  // the previous step's storage rounding
        acc = vop<V, OP, INOUT_FIRST, ACC32>(C::load(src[j] + i), acc);
    }
    V::store(dst + i, LpConv<V, BF, OUT_RNE>::store_bits(acc));
}

template <typename V, bool BF, int OP, bool INOUT_FIRST, bool ACC32, bool RNE, bool OUT_RNE>
void lp_range(const uint16_t* const* src, int k, uint16_t* dst, size_t begin, size_t end) {
    const size_t W = V::W;
    size_t i = begin;
    for (; i + W <= end; i += W) lp_group<V, BF, OP, INOUT_FIRST, ACC32, RNE, OUT_RNE>(src, k, i, dst);
    if (i < end) {  // zero-padded last group
        const size_t r = end - i;
        uint16_t pad[MI_MAX_INPUTS][V::W] = {};
        const uint16_t* psrc[MI_MAX_INPUTS] = {};
        for (int j = 0; j < k; j++) {
            memcpy(pad[j], src[j] + i, r * 2);
            psrc[j] = pad[j];
        }
        uint16_t res[V::W];
        lp_group<V, BF, OP, INOUT_FIRST, ACC32, RNE, OUT_RNE>(psrc, k, 0, res);
        memcpy(dst + i, res, r * 2);
    }
}

template <typename V, bool BF, int OP, bool INOUT_FIRST, bool ACC32, bool RNE>
void lp_fold(const void* const* inputs, int k, void* out, size_t count, unsigned v) {
    const uint16_t* src[MI_MAX_INPUTS];
    for (int j = 0; j < k; j++) src[j] = static_cast<const uint16_t*>(inputs[j]);
    uint16_t* dst = static_cast<uint16_t*>(out);
    // keep-precision's final conversion truncates the count % 16 tail: a
    // multiple of 16, so whole groups (8 or 16 lanes) fall on either side
    const size_t rne_end = (RNE && ACC32 && (v & MI_F_BF16_TAIL_TRUNC16)) ? (count / 16) * 16 : count;
    lp_range<V, BF, OP, INOUT_FIRST, ACC32, RNE, RNE>(src, k, dst, 0, rne_end);
    if (rne_end < count) lp_range<V, BF, OP, INOUT_FIRST, ACC32, RNE, false>(src, k, dst, rne_end, count);
}

template <typename V, bool BF, int OP, bool IF, bool ACC32>
FoldFn pick_lp_rne(unsigned v) {
    return (BF && (v & MI_F_BF16_RNE)) ? &lp_fold<V, BF, OP, IF, ACC32, true> : &lp_fold<V, BF, OP, IF, ACC32, false>;
}

template <typename V, bool BF, int OP>
FoldFn pick_lp_op(unsigned v) {
    const bool f = (OP == MI_OP_MIN || OP == MI_OP_MAX) && (v & MI_F_MINMAX_INOUT_FIRST);
    if (v & MI_F_ACC_FP32) return f ? pick_lp_rne<V, BF, OP, true, true>(v) : pick_lp_rne<V, BF, OP, false, true>(v);
    return f ? pick_lp_rne<V, BF, OP, true, false>(v) : pick_lp_rne<V, BF, OP, false, false>(v);
}

// the fold for (bf16 or fp16, op, canonical flags)
template <typename V>
FoldFn pick_lp(bool bf, int op, unsigned v) {
    switch (op) {
        case MI_OP_SUM: return bf ? pick_lp_op<V, true, MI_OP_SUM>(v) : pick_lp_op<V, false, MI_OP_SUM>(v);
        case MI_OP_PROD: return bf ? pick_lp_op<V, true, MI_OP_PROD>(v) : pick_lp_op<V, false, MI_OP_PROD>(v);
        case MI_OP_MIN: return bf ? pick_lp_op<V, true, MI_OP_MIN>(v) : pick_lp_op<V, false, MI_OP_MIN>(v);
        case MI_OP_MAX: return bf ? pick_lp_op<V, true, MI_OP_MAX>(v) : pick_lp_op<V, false, MI_OP_MAX>(v);
        default: return nullptr;
    }
}

// host_reduce_avx512.cpp: the 16-lane fold (native VCVTNEPS2BF16 when
// `native_bf16`); call only on CPUs with AVX512F/BW/VL (+AVX512_BF16).
FoldFn pick_lp_avx512(bool bf, int op, unsigned v, bool native_bf16);

}  // namespace mi_host
