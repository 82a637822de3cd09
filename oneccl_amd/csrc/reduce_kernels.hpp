// reduce_kernels.hpp — CDNA4 (gfx950) element-wise reduction kernels.
//
// Device half of the MI355X-native replacement for oneCCL's local reduction:
//   src/comp/comp.cpp:31-58      CCL_REDUCE (int / fp32 / fp64)
//   src/comp/bf16/*              bf16 reduce (scalar / avx512f / avx512bf)
//   src/comp/fp16/*              fp16 reduce (f16c / avx512f / avx512fp16)
//   src/comp/comp.cpp:202-249    ccl_comp_batch_reduce (K-input fan-in,
//                                optional fp32 keep-precision accumulate)
//   src/kernels/kernels.cl:219-421  device in-place / out-of-place / fan-in
//
// Design: the op is a pure HBM stream with zero data reuse,
// so there is no LDS and no MFMA.  Every lane moves 16-byte vectors
// (global_load_dwordx4: one wave-instruction = 1 KiB, fully coalesced into
// 128-byte lines), U independent vectors per input per lane so that
// K*U*16 bytes per lane are in flight before the first use, non-temporal
// stores for the output (written once, never re-read by this op).  bf16 /
// fp16 are widened to fp32 in registers (a shift for bf16, v_cvt for fp16),
// combined, and rounded back once per step (storage-precision chain) or
// once at the end (fp32 accumulate).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace mi {

enum : int { OP_SUM = 0, OP_PROD = 1, OP_MIN = 2, OP_MAX = 3 };

// Semantic variant bits (same values as MI_F_* in include/mi_reduce.h).
enum : unsigned {
    V_INOUT_FIRST = 1u,  // min/max: MINPS/MAXPS(in, inout) order -> inout on NaN/tie
    V_BF16_RNE = 2u,     // bf16 rounding: VCVTNEPS2BF16 (else truncate)
    V_ACC_FP32 = 4u,     // lp fan-in accumulates in fp32, one rounding at the end
    V_TAIL_TRUNC = 8u,   // with ACC|RNE: elements >= trunc_from truncate at the end
    V_FP16_NATIVE = 16u, // fp16 min/max as VMINPH/VMAXPH (avx512fp16): a NaN accumulator as stored
};

constexpr int kMaxInputs = 16;
constexpr int kBlock = 256;  // 4 waves of 64

// storage tags for the two 16-bit float formats
struct bf16_tag {};
struct fp16_tag {};

template <typename Tag>
struct Tr {  // integers, float, double: storage == compute type
    using S = Tag;
    using C = Tag;
    static constexpr bool lp = false;
    static constexpr bool fp = std::is_floating_point<Tag>::value;
};
template <>
struct Tr<bf16_tag> {
    using S = uint16_t;
    using C = float;
    static constexpr bool lp = true;
    static constexpr bool fp = true;
};
template <>
struct Tr<fp16_tag> {
    using S = uint16_t;
    using C = float;
    static constexpr bool lp = true;
    static constexpr bool fp = true;
};

// Kernel arguments (passed by value in the kernarg segment).
struct KArgs {
    const void* in[kMaxInputs];  // in[0] = accumulator start (the `inout` role)
    void* out;
    uint64_t nvec;        // 16-byte vectors in the aligned body
    uint64_t head;        // leading scalar elements (common misalignment)
    uint64_t tail;        // trailing scalar elements
    uint64_t count;       // total elements
    uint64_t trunc_from;  // V_TAIL_TRUNC threshold (element index)
    int k;                // number of inputs (runtime form)
    int scalar_only;      // operands misaligned differently: element loop only
};

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------
// conversions (bit-exact restatements of the x86 instructions the reference
// uses; see oracle/comp_oracle.c and oracle/ISA_CHECK.json)
// ---------------------------------------------------------------------------
__device__ __forceinline__ float bf16_to_f32(uint32_t v) { return __uint_as_float(v << 16); }

__device__ __forceinline__ uint32_t f32_to_bf16_trunc(float f) { return __float_as_uint(f) >> 16; }

// VCVTNEPS2BF16 (Intel SDM convert_fp32_to_bfloat16): zero/denormal ->
// signed zero, NaN -> quiet NaN, otherwise round to nearest even.
// Integer formulation, bit-exact including the NaN payload (~12 VALU ops).
__device__ __forceinline__ uint32_t f32_to_bf16_rne_int(float f) {
    const uint32_t u = __float_as_uint(f);
    uint32_t r = (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
    r = ((u & 0x7FFFFFFFu) > 0x7F800000u) ? ((u >> 16) | 0x40u) : r;
    r = ((u & 0x7F800000u) == 0u) ? ((u >> 16) & 0x8000u) : r;
    return r;
}

__device__ __forceinline__ bool nan_bits(uint32_t u) { return (u & 0x7FFFFFFFu) > 0x7F800000u; }

// Same result via gfx950's v_cvt_pk_bf16_f32 (round to nearest even): flush
// denormals to signed zero first, in the integer domain so the compiler
// cannot fold the flush into the conversion.  Two conversions pack into one
// instruction; ~4 VALU ops per element.  X (exact NaN): a NaN takes
// VCVTNEPS2BF16's quieted upper half explicitly — the hardware's NaN payload
// is its own; the kernels run X only on rows holding an Inf or NaN
// (fold_vec_x86).  Checked against the oracle over all 2^32 fp32 inputs, NaN
// payloads included (tests/test_gpu_convert.py).
template <bool X = true>
__device__ __forceinline__ uint32_t f32_to_bf16_rne(float f) {
    uint32_t u = __float_as_uint(f);
    const uint32_t q = (u >> 16) | 0x40u;
    u = (u & 0x7F800000u) ? u : (u & 0x80000000u);
    const uint32_t r = (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)__uint_as_float(u));
    if constexpr (X) return nan_bits(u) ? q : r;
    return r;
}

// VCVTPH2PS: exact widening (v_cvt_f32_f16; fp16 denormals are on by
// default).  A signalling NaN may stay signalling here; every path that
// stores the value quiets it the way x86 does (x86_nan_first, the narrowing
// below, convert_elem), so stored bits match.
__device__ __forceinline__ float fp16_to_f32(uint32_t h) {
    return (float)__builtin_bit_cast(_Float16, (uint16_t)h);
}
// VCVTPS2PH imm8=0: round to nearest even (v_cvt_f16_f32, default RNE mode);
// X: a NaN keeps its sign and top 10 payload bits, quieted (Intel SDM
// VCVTPS2PH).
template <bool X = true>
__device__ __forceinline__ uint32_t f32_to_fp16_rne(float f) {
    const uint32_t u = __float_as_uint(f);
    const uint32_t q = ((u >> 16) & 0x8000u) | 0x7E00u | ((u >> 13) & 0x3FFu);
    const uint32_t r = (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)f);
    if constexpr (X) return nan_bits(u) ? q : r;
    return r;
}

// x86 NaN propagation of ADDPS/MULPS(first, second) (Intel SDM vol. 1
// §4.8.3.5): a NaN operand comes back quieted, the first source's when both
// are; an invalid operation on numbers (inf - inf, 0 * inf) gives the default
// NaN 0xFFC00000.  CDNA's ALUs choose their own NaN, so the low-precision
// paths — whose reference is explicit AVX-512 code, _mm512_add_ps(in, inout)
// (src/comp/bf16/bf16_intrisics.cpp:20-26, fp16_intrisics.hpp:58-63) — fix the
// result up to those bits (oracle/comp_oracle.c x86_nan_first) on the rows
// that need it (fold_vec_x86).
__device__ __forceinline__ float x86_nan_first(float r, float first, float second) {
    const uint32_t a = __float_as_uint(first), b = __float_as_uint(second);
    uint32_t u = __float_as_uint(r);
    u = nan_bits(u) ? 0xFFC00000u : u;
    u = nan_bits(b) ? (b | 0x400000u) : u;
    u = nan_bits(a) ? (a | 0x400000u) : u;
    return __uint_as_float(u);
}
// The same rule for fp64 (default NaN 0xFFF8000000000000).
__device__ __forceinline__ bool nan_bits64(uint64_t u) { return (u & 0x7FFFFFFFFFFFFFFFull) > 0x7FF0000000000000ull; }
__device__ __forceinline__ double x86_nan_first(double r, double first, double second) {
    const uint64_t a = __double_as_longlong(first), b = __double_as_longlong(second);
    uint64_t u = __double_as_longlong(r);
    u = nan_bits64(u) ? 0xFFF8000000000000ull : u;
    u = nan_bits64(b) ? (b | 0x8000000000000ull) : u;
    u = nan_bits64(a) ? (a | 0x8000000000000ull) : u;
    return __longlong_as_double(u);
}

template <typename Tag>
__device__ __forceinline__ typename Tr<Tag>::C widen(typename Tr<Tag>::S s) {
    if constexpr (std::is_same<Tag, bf16_tag>::value)
        return bf16_to_f32(s);
    else if constexpr (std::is_same<Tag, fp16_tag>::value)
        return fp16_to_f32(s);
    else
        return s;
}

// round a compute value to storage: per-step / final rounding
template <typename Tag, unsigned V, bool X = true>
__device__ __forceinline__ typename Tr<Tag>::S narrow(typename Tr<Tag>::C c) {
    // Keep the fp32 value: left alone, the compiler turns
    // fptrunc(fmul(fpext a, fpext b)) into a native v_pk_mul_f16 (likewise
    // adds), whose zero signs differed from VCVTPS2PH of the fp32 product on
    // the GPU (fp16 prod chains gave +0 for -0; profiles/round2_nan/).  The
    // kernels compute in fp32 and round with the restated conversions only;
    // tests/test_kernel_resources.py checks the built code has no f16 math.
    if constexpr (Tr<Tag>::lp) asm volatile("" : "+v"(c));
    if constexpr (std::is_same<Tag, bf16_tag>::value) {
        if constexpr (V & V_BF16_RNE)
            return (uint16_t)f32_to_bf16_rne<X>(c);
        else
            return (uint16_t)f32_to_bf16_trunc(c);
    } else if constexpr (std::is_same<Tag, fp16_tag>::value) {
        return (uint16_t)f32_to_fp16_rne<X>(c);
    } else {
        return c;
    }
}

// ---------------------------------------------------------------------------
// the reduction operator: acc' = op(in, acc)   (`in` role first, as in
// CCL_REDUCE's std::min(in_buf[i], inout_buf[i]))
// ---------------------------------------------------------------------------
template <int OP, bool INOUT_FIRST, typename C>
__device__ __forceinline__ C apply(C in, C acc) {
    if constexpr (std::is_integral<C>::value) {
        // wrap-around integer arithmetic (defined via unsigned)
        using U = typename std::make_unsigned<C>::type;
        using W = typename std::conditional<(sizeof(C) <= 4), uint32_t, uint64_t>::type;
        if constexpr (OP == OP_SUM) return (C)(U)((W)(U)acc + (W)(U)in);
        if constexpr (OP == OP_PROD) return (C)(U)((W)(U)acc * (W)(U)in);
        if constexpr (OP == OP_MIN) return (acc < in) ? acc : in;
        if constexpr (OP == OP_MAX) return (in < acc) ? acc : in;
    } else {
        if constexpr (OP == OP_SUM) return acc + in;
        if constexpr (OP == OP_PROD) return acc * in;
        if constexpr (OP == OP_MIN) {
            if constexpr (INOUT_FIRST)
                return (in < acc) ? in : acc;  // MINPS(in, inout)
            else
                return (acc < in) ? acc : in;  // std::min(in, inout)
        }
        if constexpr (OP == OP_MAX) {
            if constexpr (INOUT_FIRST)
                return (in > acc) ? in : acc;  // MAXPS(in, inout)
            else
                return (in < acc) ? acc : in;  // std::max(in, inout)
        }
    }
}

// one fold step in the variant's precision (X: x86 NaN bits, see above).
// Which operand is the first source: a bf16/fp16 step in storage precision
// is _mm512_add_ps(in, inout) -> `in`; CCL_REDUCE's `inout op= in` on
// float/double, and the fp32 accumulation of keep-precision (CCL_REDUCE(float),
// comp.cpp:223-229), compile to ADDPS/MULPS with `inout` first -> the
// accumulator (pinned by the reference's compiled comp.cpp,
// tests/golden/ref_comp_vectors.npz).
template <typename Tag, int OP, unsigned V, bool X = true>
__device__ __forceinline__ typename Tr<Tag>::C step(typename Tr<Tag>::C x, typename Tr<Tag>::C acc) {
    auto c = apply<OP, (V & V_INOUT_FIRST) != 0>(x, acc);
    if constexpr (X && Tr<Tag>::fp && (OP == OP_SUM || OP == OP_PROD)) {
        if constexpr (Tr<Tag>::lp && !(V & V_ACC_FP32)) c = x86_nan_first(c, x, acc);
        else c = x86_nan_first(c, acc, x);
    }
    if constexpr (Tr<Tag>::lp && !(V & V_ACC_FP32)) c = widen<Tag>(narrow<Tag, V, X>(c));
    return c;
}

// final rounding of the accumulator for element `idx`
template <typename Tag, unsigned V, bool X = true>
__device__ __forceinline__ typename Tr<Tag>::S finish(typename Tr<Tag>::C acc, uint64_t idx,
                                                      uint64_t trunc_from) {
    if constexpr (std::is_same<Tag, bf16_tag>::value && (V & V_TAIL_TRUNC)) {
        return (idx >= trunc_from) ? (uint16_t)f32_to_bf16_trunc(acc)
                                   : (uint16_t)f32_to_bf16_rne<X>(acc);
    } else {
        return narrow<Tag, V, X>(acc);
    }
}

// final store of a fold's accumulator.  In storage precision (bf16 without
// V_ACC_FP32) every step has already rounded, so the accumulator holds a
// bf16 value exactly and its upper half is the result: no second rounding
// (it cost ~8 VALU ops per element pair on the C3 path).
template <typename Tag, unsigned V, bool X = true>
__device__ __forceinline__ typename Tr<Tag>::S finish_fold(typename Tr<Tag>::C acc, uint64_t idx,
                                                           uint64_t trunc_from) {
    if constexpr (std::is_same<Tag, bf16_tag>::value && !(V & V_ACC_FP32))
        return (uint16_t)f32_to_bf16_trunc(acc);
    else
        return finish<Tag, V, X>(acc, idx, trunc_from);
}


// The avx512fp16 impl's VMINPH/VMAXPH(in, inout) return the selected operand
// as stored; the fp32 route's widening (VCVTPH2PS) has quieted it.  They
// differ only for a signalling NaN, and only the accumulator's start can be
// the NaN a fold returns (a min/max step takes `in` only when in < acc,
// ordered), so the result is that start, as stored, whenever it is a NaN
// (oracle/fp16_native_check.c proves this over all 2^32 operand pairs).
template <typename Tag, int OP, unsigned V>
__device__ __forceinline__ typename Tr<Tag>::S native_minmax(typename Tr<Tag>::S r, typename Tr<Tag>::S acc0) {
    if constexpr (std::is_same<Tag, fp16_tag>::value && (V & V_FP16_NATIVE) && (OP == OP_MIN || OP == OP_MAX)) {
        if (((uint32_t)acc0 & 0x7C00u) == 0x7C00u && ((uint32_t)acc0 & 0x03FFu)) return acc0;
    }
    return r;
}

template <int MEM>
__device__ __forceinline__ u32x4 vload(const u32x4* p) {
    if constexpr (MEM & 1)
        return __builtin_nontemporal_load(p);
    else
        return *p;
}
template <int MEM>
__device__ __forceinline__ void vstore(u32x4* p, u32x4 v) {
    if constexpr (MEM & 2)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}

// Buffer addressing (cdna_hip_programming.md T8/T20): one SGPR descriptor per
// tile, built from kernel arguments and blockIdx only (wave-uniform), whose
// range is the tile's valid bytes, so out-of-range lanes read zeros and their
// stores are dropped.
constexpr int kAuxNT = 2;      // buffer op aux bit 1: non-temporal (gfx950)
constexpr int kAuxSC1NT = 18;  // sc1 + nt: the store drops the line from L2 instead of keeping it

__device__ __forceinline__ __amdgpu_buffer_rsrc_t tile_rsrc(const void* base, uint64_t byte0, uint32_t nbytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(static_cast<const char*>(base) + byte0), (short)0,
                                             (int)nbytes, 0x00020000);
}

template <typename S>
struct alignas(16) Pack {
    S e[16 / sizeof(S)];
};

// ---------------------------------------------------------------------------
// Fold of one 16-byte vector position across inputs x[0..k) (acc = x[0];
// acc = op(x[i], acc); one final rounding) into the output vector.
// fold_vec_x86 runs it without the NaN fix-ups, then screens the inputs for
// an all-ones exponent (Inf or NaN) — 3 integer ops per dword, on the packed
// words — and refolds the row with them only when one is present.  A
// low-precision sum or product is NaN only from a NaN or Inf operand, except
// a product chain whose partial product overflows to Inf and meets a zero
// (K >= 3), which the screen of the result catches.  The fix-ups cost ~10
// VALU ops per element; on every row they made C3 VALU-bound (28 % slower,
// profiles/round2_nan/).
// ---------------------------------------------------------------------------
template <typename Tag>
__device__ __forceinline__ uint32_t inf_nan_word(uint32_t w) {
    // per 16-bit half (bf16, fp16), per word (fp32) or per high word (fp64):
    // exponent field + one ulp of it carries into the top bit exactly when
    // the field is all ones
    if constexpr (std::is_same<Tag, bf16_tag>::value) return (w & 0x7F807F80u) + 0x00800080u;
    else if constexpr (std::is_same<Tag, fp16_tag>::value) return (w & 0x7C007C00u) + 0x04000400u;
    else if constexpr (std::is_same<Tag, double>::value) return (w & 0x7FF00000u) + 0x00100000u;
    else return (w & 0x7F800000u) + 0x00800000u;
}
template <typename Tag>
__device__ __forceinline__ uint32_t inf_nan_bits(u32x4 v) {
    if constexpr (std::is_same<Tag, double>::value) return inf_nan_word<Tag>(v.y) | inf_nan_word<Tag>(v.w);
    return inf_nan_word<Tag>(v.x) | inf_nan_word<Tag>(v.y) | inf_nan_word<Tag>(v.z) | inf_nan_word<Tag>(v.w);
}
template <typename Tag>
__device__ __forceinline__ bool inf_nan_hit(uint32_t bits) {
    return (bits & (sizeof(typename Tr<Tag>::S) == 2 ? 0x80008000u : 0x80000000u)) != 0u;
}

template <typename Tag, int OP, unsigned V, bool X, int KMAX>
__device__ __forceinline__ u32x4 fold_vec(const u32x4 (&x)[KMAX], int k, uint64_t e0, uint64_t trunc_from) {
    using S = typename Tr<Tag>::S;
    using C = typename Tr<Tag>::C;
    constexpr int N = 16 / sizeof(S);
    C acc[N];
    const Pack<S> p0 = __builtin_bit_cast(Pack<S>, x[0]);
#pragma unroll
    for (int e = 0; e < N; e++) acc[e] = widen<Tag>(p0.e[e]);
#pragma unroll
    for (int i = 1; i < KMAX; i++) {
        if (i < k) {
            const Pack<S> pi = __builtin_bit_cast(Pack<S>, x[i]);
#pragma unroll
            for (int e = 0; e < N; e++) acc[e] = step<Tag, OP, V, X>(widen<Tag>(pi.e[e]), acc[e]);
        }
    }
    Pack<S> pr;
#pragma unroll
    for (int e = 0; e < N; e++) {
        pr.e[e] = finish_fold<Tag, V, X>(acc[e], e0 + e, trunc_from);
        if constexpr (X) pr.e[e] = native_minmax<Tag, OP, V>(pr.e[e], p0.e[e]);  // NaN rows take X
    }
    return __builtin_bit_cast(u32x4, pr);
}

// r = the fast fold of x; refold with the fix-ups when the screen hits.
// Low precision: screen the inputs (and a K-input product's result).
// float / double sum and prod: a NaN operand or an invalid operation makes
// the result NaN, and a NaN stays NaN along the fold, so the result's own
// screen finds every row to fix: one unordered compare per element (an
// integer exponent screen cost C2 ~3 %, profiles/round3_run2).  Other types
// and ops: a no-op.
template <typename Tag, int OP, unsigned V, int KMAX>
__device__ __forceinline__ u32x4 x86_refold(u32x4 r, const u32x4 (&x)[KMAX], int k, uint64_t e0,
                                            uint64_t trunc_from) {
    if constexpr (Tr<Tag>::lp) {
        uint32_t bits = inf_nan_bits<Tag>(x[0]);
#pragma unroll
        for (int i = 1; i < KMAX; i++)
            if (i < k) bits |= inf_nan_bits<Tag>(x[i]);
        if constexpr (OP == OP_PROD && KMAX > 2) bits |= inf_nan_bits<Tag>(r);
        if (__builtin_expect(inf_nan_hit<Tag>(bits), 0)) r = fold_vec<Tag, OP, V, true, KMAX>(x, k, e0, trunc_from);
    } else if constexpr (Tr<Tag>::fp && (OP == OP_SUM || OP == OP_PROD)) {
        // unordered self-compares: one v_cmp_u per element pair into a lane mask
        const Pack<Tag> p = __builtin_bit_cast(Pack<Tag>, r);
        bool nan = false;
#pragma unroll
        for (int e = 0; e < 16 / (int)sizeof(Tag); e++) nan |= (p.e[e] != p.e[e]);
        if (__builtin_expect(nan, 0)) r = fold_vec<Tag, OP, V, true, KMAX>(x, k, e0, trunc_from);
    }
    return r;
}

template <typename Tag, int OP, unsigned V, int KMAX>
__device__ __forceinline__ u32x4 fold_vec_x86(const u32x4 (&x)[KMAX], int k, uint64_t e0, uint64_t trunc_from) {
    return x86_refold<Tag, OP, V, KMAX>(fold_vec<Tag, OP, V, false, KMAX>(x, k, e0, trunc_from), x, k, e0,
                                        trunc_from);
}

template <typename Tag>
__device__ __forceinline__ bool row_has_nan(u32x4 r) {
    const Pack<Tag> p = __builtin_bit_cast(Pack<Tag>, r);
    bool nan = false;
#pragma unroll
    for (int e = 0; e < 16 / (int)sizeof(Tag); e++) nan |= (p.e[e] != p.e[e]);
    return nan;
}

// fold_vec_x86 for the lean kernels.  float / double sum and prod: the rare
// NaN row re-reads its inputs (`reload(y)`) instead of keeping x live past the
// fold; kept live, they made the compiler split the guarded load / add / store
// row into three exec-masked blocks and cost the C2 kernel ~3 %
// (profiles/round3_run2).  The compiler barrier stops the re-read from being
// folded into the first read.  Other types: fold_vec_x86.
template <typename Tag, int OP, unsigned V, int KMAX, typename Reload>
__device__ __forceinline__ u32x4 fold_row(const u32x4 (&x)[KMAX], int k, uint64_t e0, uint64_t trunc_from,
                                          Reload&& reload) {
    if constexpr (!Tr<Tag>::lp && Tr<Tag>::fp && (OP == OP_SUM || OP == OP_PROD)) {
        u32x4 r = fold_vec<Tag, OP, V, false, KMAX>(x, k, e0, trunc_from);
        if (__builtin_expect(row_has_nan<Tag>(r), 0)) {
            asm volatile("" ::: "memory");
            u32x4 y[KMAX];
            reload(y);
            r = fold_vec<Tag, OP, V, true, KMAX>(y, k, e0, trunc_from);
        }
        return r;
    } else {
        return fold_vec_x86<Tag, OP, V, KMAX>(x, k, e0, trunc_from);
    }
}

// ---------------------------------------------------------------------------
// Packed 8- and 16-bit integer ops on whole dwords: acc' = op(in, acc) per
// byte / half, with CCL_REDUCE's wrap-around sum and prod.  Unpacking 16 bytes
// of each of up to 16 inputs cost the fan-in 258 VGPRs, one wave per SIMD and
// 1.7 TB/s (profiles/round1_misalign.jsonl).  Packed, the fold stays in the 4
// dwords of the loaded vector.  16-bit lanes map to gfx950's v_pk_*_{i,u}16;
// bytes run as even/odd halves of those, and sum uses the carry-free SWAR add.
// min/max of integers have no tie or NaN cases, so operand order is moot.
// ---------------------------------------------------------------------------
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef short i16x2 __attribute__((ext_vector_type(2)));

template <typename V2>
__device__ __forceinline__ V2 as2(uint32_t x) { return __builtin_bit_cast(V2, x); }
template <typename V2>
__device__ __forceinline__ uint32_t as1(V2 x) { return __builtin_bit_cast(uint32_t, x); }

template <int OP, bool SIGNED>
__device__ __forceinline__ uint32_t pk16_op(uint32_t in, uint32_t acc) {
    if constexpr (OP == OP_SUM) return as1(as2<u16x2>(acc) + as2<u16x2>(in));
    if constexpr (OP == OP_PROD) return as1(as2<u16x2>(acc) * as2<u16x2>(in));
    if constexpr (SIGNED) {
        if constexpr (OP == OP_MIN) return as1(__builtin_elementwise_min(as2<i16x2>(acc), as2<i16x2>(in)));
        if constexpr (OP == OP_MAX) return as1(__builtin_elementwise_max(as2<i16x2>(acc), as2<i16x2>(in)));
    } else {
        if constexpr (OP == OP_MIN) return as1(__builtin_elementwise_min(as2<u16x2>(acc), as2<u16x2>(in)));
        if constexpr (OP == OP_MAX) return as1(__builtin_elementwise_max(as2<u16x2>(acc), as2<u16x2>(in)));
    }
}

template <int OP, bool SIGNED>
__device__ __forceinline__ uint32_t pk8_op(uint32_t in, uint32_t acc) {
    constexpr uint32_t lo7 = 0x7F7F7F7Fu, hi1 = 0x80808080u, evn = 0x00FF00FFu;
    if constexpr (OP == OP_SUM) return ((acc & lo7) + (in & lo7)) ^ ((acc ^ in) & hi1);
    if constexpr (OP == OP_PROD) {  // low byte of each 16-bit product
        const uint32_t pe = as1(as2<u16x2>(acc & evn) * as2<u16x2>(in & evn));
        const uint32_t po = as1(as2<u16x2>((acc >> 8) & evn) * as2<u16x2>((in >> 8) & evn));
        return (pe & evn) | ((po & evn) << 8);
    }
    if constexpr (SIGNED) {  // sign-extend even / odd bytes into 16-bit lanes
        const i16x2 ae = as2<i16x2>(acc << 8) >> 8, ie = as2<i16x2>(in << 8) >> 8;
        const i16x2 ao = as2<i16x2>(acc) >> 8, io = as2<i16x2>(in) >> 8;
        i16x2 re, ro;
        if constexpr (OP == OP_MIN) {
            re = __builtin_elementwise_min(ae, ie);
            ro = __builtin_elementwise_min(ao, io);
        } else {
            re = __builtin_elementwise_max(ae, ie);
            ro = __builtin_elementwise_max(ao, io);
        }
        return (as1(re) & evn) | ((as1(ro) & evn) << 8);
    } else {
        const u16x2 ae = as2<u16x2>(acc & evn), ie = as2<u16x2>(in & evn);
        const u16x2 ao = as2<u16x2>((acc >> 8) & evn), io = as2<u16x2>((in >> 8) & evn);
        u16x2 re, ro;
        if constexpr (OP == OP_MIN) {
            re = __builtin_elementwise_min(ae, ie);
            ro = __builtin_elementwise_min(ao, io);
        } else {
            re = __builtin_elementwise_max(ae, ie);
            ro = __builtin_elementwise_max(ao, io);
        }
        return as1(re) | (as1(ro) << 8);
    }
}

// 8/16-bit integer storage: the fold runs packed on dwords
template <typename Tag>
constexpr bool packed_int() {
    return std::is_integral<Tag>::value && sizeof(Tag) <= 2;
}

template <typename Tag, int OP>
__device__ __forceinline__ u32x4 pk_op4(u32x4 in, u32x4 acc) {
    constexpr bool sg = std::is_signed<Tag>::value;
    u32x4 r;
#pragma unroll
    for (int d = 0; d < 4; d++) {
        if constexpr (sizeof(Tag) == 1)
            r[d] = pk8_op<OP, sg>(in[d], acc[d]);
        else
            r[d] = pk16_op<OP, sg>(in[d], acc[d]);
    }
    return r;
}

// scalar path for one element (head/tail/misaligned)
template <typename Tag, int OP, unsigned V>
__device__ __forceinline__ void reduce_elem(const KArgs& a, int k, uint64_t idx) {
    using S = typename Tr<Tag>::S;
    using C = typename Tr<Tag>::C;
    const S s0 = static_cast<const S*>(a.in[0])[idx];
    C acc = widen<Tag>(s0);
    for (int i = 1; i < k; i++) acc = step<Tag, OP, V>(widen<Tag>(static_cast<const S*>(a.in[i])[idx]), acc);
    static_cast<S*>(a.out)[idx] = native_minmax<Tag, OP, V>(finish_fold<Tag, V>(acc, idx, a.trunc_from), s0);
}

// One tile row: U vectors per lane at v0, v0+B, ...  GUARD = last tile.
template <typename Tag, int OP, unsigned V, int KT, int U, int MEM, bool GUARD, int B>
__device__ __forceinline__ void reduce_tile(const KArgs& a, int k, uint64_t v0) {
    using S = typename Tr<Tag>::S;
    using C = typename Tr<Tag>::C;
    constexpr int N = 16 / sizeof(S);
    const uint64_t hb = a.head * sizeof(S);

    C acc[U][N];
    u32x4 cur[U];
    constexpr bool kNative = std::is_same<Tag, fp16_tag>::value && (V & V_FP16_NATIVE) && (OP == OP_MIN || OP == OP_MAX);
    u32x4 raw0[kNative ? U : 1];  // the accumulator's start as stored (native_minmax)

    const u32x4* p0 = reinterpret_cast<const u32x4*>(static_cast<const char*>(a.in[0]) + hb);
    const u32x4* p1 =
        reinterpret_cast<const u32x4*>(static_cast<const char*>(a.in[(KT == 2 || k >= 2) ? 1 : 0]) + hb);
    // issue input 0 and input 1 loads back to back (2*U*16 B in flight per lane)
#pragma unroll
    for (int j = 0; j < U; j++) {
        const uint64_t v = v0 + (uint64_t)j * B;
        if (!GUARD || v < a.nvec) {
            u32x4 r = vload<MEM>(p0 + v);
            if constexpr (kNative) raw0[j] = r;
            Pack<S> p = __builtin_bit_cast(Pack<S>, r);
#pragma unroll
            for (int e = 0; e < N; e++) acc[j][e] = widen<Tag>(p.e[e]);
        }
    }
    if (KT == 2 || k >= 2) {
#pragma unroll
        for (int j = 0; j < U; j++) {
            const uint64_t v = v0 + (uint64_t)j * B;
            cur[j] = u32x4{0u, 0u, 0u, 0u};
            if (!GUARD || v < a.nvec) cur[j] = vload<MEM>(p1 + v);
        }
    }

    if constexpr (KT == 2) {
#pragma unroll
        for (int j = 0; j < U; j++) {
            Pack<S> p = __builtin_bit_cast(Pack<S>, cur[j]);
#pragma unroll
            for (int e = 0; e < N; e++) acc[j][e] = step<Tag, OP, V>(widen<Tag>(p.e[e]), acc[j][e]);
        }
    } else {
        for (int i = 1; i < k; i++) {
            // prefetch input i+1 while combining input i
            u32x4 nxt[U];
            if (i + 1 < k) {
                const u32x4* pn =
                    reinterpret_cast<const u32x4*>(static_cast<const char*>(a.in[i + 1]) + hb);
#pragma unroll
                for (int j = 0; j < U; j++) {
                    const uint64_t v = v0 + (uint64_t)j * B;
                    nxt[j] = u32x4{0u, 0u, 0u, 0u};
                    if (!GUARD || v < a.nvec) nxt[j] = vload<MEM>(pn + v);
                }
            }
#pragma unroll
            for (int j = 0; j < U; j++) {
                Pack<S> p = __builtin_bit_cast(Pack<S>, cur[j]);
#pragma unroll
                for (int e = 0; e < N; e++) acc[j][e] = step<Tag, OP, V>(widen<Tag>(p.e[e]), acc[j][e]);
            }
            if (i + 1 < k) {
#pragma unroll
                for (int j = 0; j < U; j++) cur[j] = nxt[j];
            }
        }
    }

    u32x4* po = reinterpret_cast<u32x4*>(static_cast<char*>(a.out) + hb);
#pragma unroll
    for (int j = 0; j < U; j++) {
        const uint64_t v = v0 + (uint64_t)j * B;
        if (!GUARD || v < a.nvec) {
            Pack<S> p;
#pragma unroll
            for (int e = 0; e < N; e++)
                p.e[e] = finish_fold<Tag, V>(acc[j][e], a.head + v * N + e, a.trunc_from);
            if constexpr (kNative) {
                const Pack<S> s0 = __builtin_bit_cast(Pack<S>, raw0[j]);
#pragma unroll
                for (int e = 0; e < N; e++) p.e[e] = native_minmax<Tag, OP, V>(p.e[e], s0.e[e]);
            }
            vstore<MEM>(po + v, __builtin_bit_cast(u32x4, p));
        }
    }
}

// Grid-stride over tiles of B*U vectors (B threads per block).  Block 0 also does the
// scalar head/tail (< 16 elements each).  `scalar_only` = operands with
// different misalignments: plain element loop.
// MAP 1: blocks b, b+8, b+16, ... (one XCD under the observed round-robin
// dispatch, MI355X_MICROARCH.md §Workgroup dispatch) take one contiguous
// 1/8 of the tiles (grid must be a multiple of 8; speed only, never
// correctness: every tile is still covered exactly once).
template <typename Tag, int OP, unsigned V, int KT, int U, int MEM, int MAP = 0, int B = kBlock>
__global__ __launch_bounds__(B) void reduce_kernel(KArgs a) {
    const int k = (KT > 0) ? KT : a.k;
    if (a.scalar_only) {
        for (uint64_t i = (uint64_t)blockIdx.x * B + threadIdx.x; i < a.count;
             i += (uint64_t)gridDim.x * B)
            reduce_elem<Tag, OP, V>(a, k, i);
        return;
    }
    using S = typename Tr<Tag>::S;
    constexpr int N = 16 / sizeof(S);
    if (blockIdx.x == 0) {
        if (threadIdx.x < a.head) reduce_elem<Tag, OP, V>(a, k, threadIdx.x);
        if (threadIdx.x < a.tail) reduce_elem<Tag, OP, V>(a, k, a.head + a.nvec * N + threadIdx.x);
    }
    const uint64_t tile = (uint64_t)B * U;
    const uint64_t stride = (uint64_t)gridDim.x * tile;
    uint64_t b = blockIdx.x;
    if constexpr (MAP == 1) b = (uint64_t)(blockIdx.x % 8) * (gridDim.x / 8) + blockIdx.x / 8;
    for (uint64_t base = b * tile; base < a.nvec; base += stride) {
        if (base + tile <= a.nvec)
            reduce_tile<Tag, OP, V, KT, U, MEM, false, B>(a, k, base + threadIdx.x);
        else
            reduce_tile<Tag, OP, V, KT, U, MEM, true, B>(a, k, base + threadIdx.x);
    }
}

// ---------------------------------------------------------------------------
// Lean 2-input kernel (the ccl_comp_reduce case): one tile of B*U vectors per
// block, three pointers, no grid-stride loop.  Per-thread work is a handful
// of address ops around the loads — with 1-vector-per-lane tiles the general
// kernel's argument block and loop structure cost 10-15 % of HBM rate
// (profiles/round1_sweep5_block.jsonl).  Block 0 also does the scalar head
// and tail.  Same element semantics as reduce_kernel (step / finish).
// ---------------------------------------------------------------------------
struct R2Args {
    const void* acc;  // the `inout` role (accumulator start)
    const void* in;   // the `in` role
    void* out;
    uint64_t nvec;        // 16-byte vectors in the aligned body
    uint32_t head, tail;  // scalar elements before / after the body
    uint64_t trunc_from;  // V_TAIL_TRUNC threshold (element index)
};

template <typename Tag, int OP, unsigned V>
__device__ __forceinline__ void reduce2_elem(const R2Args& a, uint64_t idx) {
    using S = typename Tr<Tag>::S;
    using C = typename Tr<Tag>::C;
    const S s0 = static_cast<const S*>(a.acc)[idx];
    C acc = widen<Tag>(s0);
    acc = step<Tag, OP, V>(widen<Tag>(static_cast<const S*>(a.in)[idx]), acc);
    static_cast<S*>(a.out)[idx] = native_minmax<Tag, OP, V>(finish_fold<Tag, V>(acc, idx, a.trunc_from), s0);
}

// One tile (block `blk` of the operand set `a`): the body of reduce2_kernel,
// shared with the descriptor-batched form below.
template <typename Tag, int OP, unsigned V, int U, int B>
__device__ __forceinline__ void reduce2_tile(const R2Args& a, uint32_t blk) {
    using S = typename Tr<Tag>::S;
    constexpr int N = 16 / sizeof(S);
    if (blk == 0) {
        if (threadIdx.x < a.head) reduce2_elem<Tag, OP, V>(a, threadIdx.x);
        if (threadIdx.x < a.tail) reduce2_elem<Tag, OP, V>(a, a.head + a.nvec * N + threadIdx.x);
    }
    const size_t hb = (size_t)a.head * sizeof(S);
    // Every operand through a buffer descriptor per tile (base = the tile's
    // first vector, range = its valid bytes; lanes past the end read zeros
    // and their stores are dropped).  Loads nt: against the global nt loads
    // of rounds 1-5 the same fold ran 0.3-0.5 % faster at the median and in
    // each of 16 fresh placements per layout (tools/r2_load_ab.py), and the
    // library built this way 0.2-0.5 % faster than the round-5 build over 10
    // fresh placements per config, C3 bf16 within noise (tools/ab_c2.py
    // --trials; both in profiles/round6_run6/).  Stores sc1 + nt drop each line from L2 as it
    // is written; nt alone keeps it there, and the 2-input stream then ran
    // 2.3-3.1 % slower (tools/occupancy_sweep.hip policy,
    // profiles/round3_occupancy/).  The fan-in keeps nt (sc1 did not pay there).
    const uint64_t t0 = (uint64_t)blk * (B * U);
    const uint64_t tleft = a.nvec > t0 ? a.nvec - t0 : 0;
    const uint32_t tbytes = (uint32_t)(tleft < (uint64_t)B * U ? tleft : (uint64_t)B * U) * 16u;
    const uint64_t tb = hb + t0 * 16;
    const __amdgpu_buffer_rsrc_t arsrc = tile_rsrc(a.acc, tb, tbytes);
    const __amdgpu_buffer_rsrc_t irsrc = tile_rsrc(a.in, tb, tbytes);
    const __amdgpu_buffer_rsrc_t orsrc = tile_rsrc(a.out, tb, tbytes);
    const uint64_t v0 = t0 + threadIdx.x;
    u32x4 x[U], y[U];
#pragma unroll
    for (int j = 0; j < U; j++)
        x[j] = __builtin_amdgcn_raw_buffer_load_b128(arsrc, (uint32_t)(j * B + threadIdx.x) * 16u, 0, kAuxNT);
#pragma unroll
    for (int j = 0; j < U; j++)
        y[j] = __builtin_amdgcn_raw_buffer_load_b128(irsrc, (uint32_t)(j * B + threadIdx.x) * 16u, 0, kAuxNT);
#pragma unroll
    for (int j = 0; j < U; j++) {
        const uint64_t v = v0 + (uint64_t)j * B;
        if (v < a.nvec) {
            const uint32_t off = (uint32_t)(v - t0) * 16u;
            const u32x4 xs[2] = {x[j], y[j]};
            __builtin_amdgcn_raw_buffer_store_b128(
                fold_row<Tag, OP, V, 2>(xs, 2, a.head + v * N, a.trunc_from, [&](u32x4 (&r)[2]) {
                    r[0] = __builtin_amdgcn_raw_buffer_load_b128(arsrc, off, 0, kAuxNT);
                    r[1] = __builtin_amdgcn_raw_buffer_load_b128(irsrc, off, 0, kAuxNT);
                }),
                orsrc, off, 0, kAuxSC1NT);
        }
    }
}

template <typename Tag, int OP, unsigned V, int U, int B>
__global__ __launch_bounds__(B) void reduce2_kernel(R2Args a) {
    reduce2_tile<Tag, OP, V, U, B>(a, blockIdx.x);
}

// ---------------------------------------------------------------------------
// Descriptor-batched 2-input reduce: up to kBatchMax independent
// (acc, in, out) operand sets in one launch, each cut into reduce2_kernel's
// tiles.  Block b works on descriptor d = the last one with block0[d] <= b
// (a uniform binary search over the kernarg table), tile b - block0[d].  For
// schedules with many small chunks in one phase: one dispatch instead of one
// per chunk (sub-MiB reduces are dispatch-bound).
// ---------------------------------------------------------------------------
constexpr int kBatchMax = 64;

struct BArgs {
    const void* acc[kBatchMax];
    const void* in[kBatchMax];
    void* out[kBatchMax];
    uint64_t nvec[kBatchMax];
    uint64_t trunc_from[kBatchMax];
    uint8_t head[kBatchMax], tail[kBatchMax];  // < 16 elements each
    uint32_t block0[kBatchMax + 1];             // first block of each descriptor; [n] = grid size
    int n;
};

template <typename Tag, int OP, unsigned V, int U, int B>
__global__ __launch_bounds__(B) void reduce2_batch_kernel(BArgs a) {
    const uint32_t b = blockIdx.x;
    int lo = 0, hi = a.n - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (a.block0[mid] <= b) lo = mid;
        else hi = mid - 1;
    }
    R2Args r;
    r.acc = a.acc[lo];
    r.in = a.in[lo];
    r.out = a.out[lo];
    r.nvec = a.nvec[lo];
    r.head = a.head[lo];
    r.tail = a.tail[lo];
    r.trunc_from = a.trunc_from[lo];
    reduce2_tile<Tag, OP, V, U, B>(r, b - a.block0[lo]);
}

// ---------------------------------------------------------------------------
// Lean K-input fan-in (compile-time K): one tile of B*U vectors per block,
// every input's loads issued before the first combine, left fold in the
// reference's order (acc = in[0]; acc = op(in[j], acc)).  Requires a common
// alignment; head/tail by block 0.
// ---------------------------------------------------------------------------
struct RKArgs {
    const void* in[kMaxInputs];
    void* out;
    uint64_t nvec;
    uint32_t head, tail;
    uint64_t trunc_from;
};

template <typename Tag, int OP, unsigned V, int K>
__device__ __forceinline__ void reducek_elem(const RKArgs& a, uint64_t idx) {
    using S = typename Tr<Tag>::S;
    using C = typename Tr<Tag>::C;
    const S s0 = static_cast<const S*>(a.in[0])[idx];
    C acc = widen<Tag>(s0);
#pragma unroll
    for (int i = 1; i < K; i++) acc = step<Tag, OP, V>(widen<Tag>(static_cast<const S*>(a.in[i])[idx]), acc);
    static_cast<S*>(a.out)[idx] = native_minmax<Tag, OP, V>(finish_fold<Tag, V>(acc, idx, a.trunc_from), s0);
}

template <typename Tag, int OP, unsigned V, int K, int U, int B>
__global__ __launch_bounds__(B) void reducek_kernel(RKArgs a) {
    using S = typename Tr<Tag>::S;
    constexpr int N = 16 / sizeof(S);
    if (blockIdx.x == 0) {
        if (threadIdx.x < a.head) reducek_elem<Tag, OP, V, K>(a, threadIdx.x);
        if (threadIdx.x < a.tail) reducek_elem<Tag, OP, V, K>(a, a.head + a.nvec * N + threadIdx.x);
    }
    const size_t hb = (size_t)a.head * sizeof(S);
    const uint64_t v0 = (uint64_t)blockIdx.x * (B * U) + threadIdx.x;
    const bool full = v0 + (uint64_t)(U - 1) * B < a.nvec;
    u32x4 x[K][U];
#pragma unroll
    for (int i = 0; i < K; i++) {
        const u32x4* p = reinterpret_cast<const u32x4*>(static_cast<const char*>(a.in[i]) + hb);
#pragma unroll
        for (int j = 0; j < U; j++)
            if (full || v0 + (uint64_t)j * B < a.nvec) x[i][j] = vload<3>(p + v0 + (uint64_t)j * B);
    }
    u32x4* po = reinterpret_cast<u32x4*>(static_cast<char*>(a.out) + hb);
#pragma unroll
    for (int j = 0; j < U; j++) {
        const uint64_t v = v0 + (uint64_t)j * B;
        if (full || v < a.nvec) {
            u32x4 xs[K];
#pragma unroll
            for (int i = 0; i < K; i++) xs[i] = x[i][j];
            vstore<3>(po + v, fold_row<Tag, OP, V, K>(xs, K, a.head + v * N, a.trunc_from, [&](u32x4 (&r)[K]) {
#pragma unroll
                          for (int i = 0; i < K; i++)
                              r[i] = vload<3>(reinterpret_cast<const u32x4*>(static_cast<const char*>(a.in[i]) + hb) + v);
                      }));
        }
    }
}

// ---------------------------------------------------------------------------
// Buffer-addressed forms (cdna_hip_programming.md T8/T20).  Each block owns one
// tile of B vectors.  Every stream gets one SGPR descriptor per tile, built
// from kernel arguments and blockIdx only (wave-uniform, so no waterfall).
// Its range is the tile's valid bytes, so in the last tile lanes past the end
// read zeros and their stores are dropped by the range check: no guard
// branches.  Lanes carry only a 32-bit byte offset.
// ---------------------------------------------------------------------------

// Fan-in with a runtime K (2..kMaxInputs): all K loads are issued before the
// first combine (uniform branches on k only), then the left fold in the
// reference's order (acc = in[0]; acc = op(in[j], acc)).  Common alignment
// required; head/tail by block 0 through the scalar element path.
template <typename Tag, int OP, unsigned V, int B, int KMAX = kMaxInputs>
__global__ __launch_bounds__(B) void fan_kernel(KArgs a) {
    using S = typename Tr<Tag>::S;
    constexpr int N = 16 / sizeof(S);
    const int k = a.k;
    if (blockIdx.x == 0) {
        if (threadIdx.x < a.head) reduce_elem<Tag, OP, V>(a, k, threadIdx.x);
        if (threadIdx.x < a.tail) reduce_elem<Tag, OP, V>(a, k, a.head + a.nvec * N + threadIdx.x);
    }
    const uint64_t t0 = (uint64_t)blockIdx.x * B;
    if (t0 >= a.nvec) return;
    const uint64_t left = a.nvec - t0;
    const uint32_t bytes = (uint32_t)(left < (uint64_t)B ? left : (uint64_t)B) * 16u;
    const uint64_t byte0 = a.head * sizeof(S) + t0 * 16;
    const uint32_t off = threadIdx.x * 16u;
    // Materialise every input pointer before the first branch: left alone, the
    // compiler sinks each kernarg load into its `i < k` block and every buffer
    // load then waits on its own scalar load.
    const void* in[KMAX];
#pragma unroll
    for (int i = 0; i < KMAX; i++) {
        in[i] = a.in[i];
        asm volatile("" ::"s"(in[i]));
    }
    u32x4 x[KMAX];
#pragma unroll
    for (int i = 0; i < KMAX; i++)
        if (i < k) x[i] = __builtin_amdgcn_raw_buffer_load_b128(tile_rsrc(in[i], byte0, bytes), off, 0, kAuxNT);
    if constexpr (packed_int<Tag>()) {
        u32x4 r = x[0];
#pragma unroll
        for (int i = 1; i < KMAX; i++)
            if (i < k) r = pk_op4<Tag, OP>(x[i], r);
        __builtin_amdgcn_raw_buffer_store_b128(r, tile_rsrc(a.out, byte0, bytes), off, 0, kAuxNT);
        return;
    }
    // The fast fold is written out here rather than through fold_vec: with
    // the runtime-k loop in a callee, the compiler kept the fp32 8-input
    // form's x[] as an aggregate and spilled it to scratch (33 ms instead of
    // 1.6 ms per GiB; tests/test_kernel_resources.py guards every kernel).
    using C = typename Tr<Tag>::C;
    C acc[N];
    const Pack<S> p0 = __builtin_bit_cast(Pack<S>, x[0]);
#pragma unroll
    for (int e = 0; e < N; e++) acc[e] = widen<Tag>(p0.e[e]);
#pragma unroll
    for (int i = 1; i < KMAX; i++) {
        if (i < k) {
            const Pack<S> pi = __builtin_bit_cast(Pack<S>, x[i]);
#pragma unroll
            for (int e = 0; e < N; e++) acc[e] = step<Tag, OP, V, false>(widen<Tag>(pi.e[e]), acc[e]);
        }
    }
    Pack<S> pr;
    const uint64_t e0 = a.head + (t0 + threadIdx.x) * N;
#pragma unroll
    for (int e = 0; e < N; e++) pr.e[e] = finish_fold<Tag, V, false>(acc[e], e0 + e, a.trunc_from);
    __builtin_amdgcn_raw_buffer_store_b128(
        x86_refold<Tag, OP, V, KMAX>(__builtin_bit_cast(u32x4, pr), x, k, e0, a.trunc_from),
        tile_rsrc(a.out, byte0, bytes), off, 0, kAuxNT);
}

// The 2-input form of the same (R2Args: acc, in -> out).
template <typename Tag, int OP, unsigned V, int B>
__global__ __launch_bounds__(B) void reduce2b_kernel(R2Args a) {
    using S = typename Tr<Tag>::S;
    constexpr int N = 16 / sizeof(S);
    if (blockIdx.x == 0) {
        if (threadIdx.x < a.head) reduce2_elem<Tag, OP, V>(a, threadIdx.x);
        if (threadIdx.x < a.tail) reduce2_elem<Tag, OP, V>(a, a.head + a.nvec * N + threadIdx.x);
    }
    const uint64_t t0 = (uint64_t)blockIdx.x * B;
    if (t0 >= a.nvec) return;
    const uint64_t left = a.nvec - t0;
    const uint32_t bytes = (uint32_t)(left < (uint64_t)B ? left : (uint64_t)B) * 16u;
    const uint64_t byte0 = (uint64_t)a.head * sizeof(S) + t0 * 16;
    const uint32_t off = threadIdx.x * 16u;
    const u32x4 xs[2] = {__builtin_amdgcn_raw_buffer_load_b128(tile_rsrc(a.acc, byte0, bytes), off, 0, kAuxNT),
                         __builtin_amdgcn_raw_buffer_load_b128(tile_rsrc(a.in, byte0, bytes), off, 0, kAuxNT)};
    const uint64_t e0 = a.head + (t0 + threadIdx.x) * N;
    __builtin_amdgcn_raw_buffer_store_b128(
        fold_row<Tag, OP, V, 2>(xs, 2, e0, a.trunc_from,
                                [&](u32x4 (&r)[2]) {
                                    r[0] = __builtin_amdgcn_raw_buffer_load_b128(tile_rsrc(a.acc, byte0, bytes), off, 0,
                                                                                 kAuxNT);
                                    r[1] = __builtin_amdgcn_raw_buffer_load_b128(tile_rsrc(a.in, byte0, bytes), off, 0,
                                                                                 kAuxNT);
                                }),
        tile_rsrc(a.out, byte0, bytes), off, 0, kAuxNT);
}

// ---------------------------------------------------------------------------
// element conversions fp32 <-> bf16 / fp16 (ccl_convert_*_arrays,
// src/comp/bf16/bf16.cpp:113-169, src/comp/fp16/fp16.cpp:55-61)
// ---------------------------------------------------------------------------
struct CArgs {
    const void* src;
    void* dst;
    uint64_t count;       // elements
    uint64_t head;        // elements before dst's first 16-byte boundary (vector path)
    uint64_t ngroups;     // groups of 8 elements on the vector path
    uint64_t trunc_from;  // V_TAIL_TRUNC: elements >= trunc_from truncate
    int scalar_only;
};

// X: the reference's NaN bits (the vector body runs X only on groups whose
// source holds an Inf or NaN, as fold_vec_x86 does)
template <typename ST, typename DT, unsigned V, bool X = true>
__device__ __forceinline__ typename Tr<DT>::S convert_elem(typename Tr<ST>::S s, uint64_t idx, uint64_t trunc_from) {
    float f = widen<ST>(s);
    if constexpr (X && std::is_same<ST, fp16_tag>::value)  // VCVTPH2PS quiets a signalling NaN
        f = nan_bits(__float_as_uint(f)) ? __uint_as_float(__float_as_uint(f) | 0x400000u) : f;
    if constexpr (std::is_same<DT, float>::value)
        return f;
    else
        return finish<DT, V, X>(f, idx, trunc_from);
}

template <typename ST, typename DT, unsigned V, bool X, int SV, int DV>
__device__ __forceinline__ void convert_group(const Pack<typename Tr<ST>::S> (&sp)[SV],
                                              Pack<typename Tr<DT>::S> (&dp)[DV], uint64_t e0, uint64_t trunc_from) {
    constexpr int SN = 16 / sizeof(typename Tr<ST>::S), DN = 16 / sizeof(typename Tr<DT>::S);
#pragma unroll
    for (int e = 0; e < 8; e++)
        dp[e / DN].e[e % DN] = convert_elem<ST, DT, V, X>(sp[e / SN].e[e % SN], e0 + e, trunc_from);
}

// The same 8 elements taken as two runs of 4: elements 0-3 have indices
// ea..ea+3, elements 4-7 eb..eb+3.
template <typename ST, typename DT, unsigned V, bool X, int SV, int DV>
__device__ __forceinline__ void convert_runs(const Pack<typename Tr<ST>::S> (&sp)[SV],
                                             Pack<typename Tr<DT>::S> (&dp)[DV], uint64_t ea, uint64_t eb,
                                             uint64_t trunc_from) {
    constexpr int SN = 16 / sizeof(typename Tr<ST>::S), DN = 16 / sizeof(typename Tr<DT>::S);
#pragma unroll
    for (int e = 0; e < 8; e++)
        dp[e / DN].e[e % DN] =
            convert_elem<ST, DT, V, X>(sp[e / SN].e[e % SN], e < 4 ? ea + e : eb + (e - 4), trunc_from);
}

// 8 elements per lane per group: fp32 side 2 x 16 B, 16-bit side 16 B.
// SC1: the vector body's stores go through one buffer descriptor per wave
// chunk with sc1 + nt (the line leaves L2 as it is written, as reduce2_kernel
// stores) instead of global nt stores.
template <typename ST, typename DT, unsigned V, int B = kBlock, bool SC1 = false>
__global__ __launch_bounds__(B) void convert_kernel(CArgs a) {
    using SS = typename Tr<ST>::S;
    using DS = typename Tr<DT>::S;
    const uint64_t stride = (uint64_t)gridDim.x * B;
    uint64_t i = (uint64_t)blockIdx.x * B + threadIdx.x;
    if (a.scalar_only) {
        for (; i < a.count; i += stride)
            static_cast<DS*>(a.dst)[i] = convert_elem<ST, DT, V>(static_cast<const SS*>(a.src)[i], i, a.trunc_from);
        return;
    }
    // vector body on dst's 16-byte grid from element `head` on; the source
    // vectors may be unaligned (element-aligned loads of 16 bytes)
    constexpr int SV = 8 * sizeof(SS) / 16;  // 16-byte source vectors per group
    constexpr int DV = 8 * sizeof(DS) / 16;
    const u32x4* src = reinterpret_cast<const u32x4*>(static_cast<const SS*>(a.src) + a.head);
    u32x4* dst = reinterpret_cast<u32x4*>(static_cast<DS*>(a.dst) + a.head);
    if constexpr (sizeof(SS) != sizeof(DS)) {
        // A lane's 8 elements as two runs of 4, so that every load and store
        // instruction covers one contiguous span across the wave (8 bytes per
        // lane on the 16-bit side, 16 on the fp32 side).  A wave whose 64
        // groups all lie in range (wave-uniform: `stride` and the block size
        // are multiples of 64) takes its 512 elements as the runs [4L, 4L+4)
        // and [256+4L, 256+4L+4) for lane L.  With eight contiguous elements
        // per lane (the loop below) every fp32-side instruction touched every
        // other 16 bytes: widening ran at ~4.1 TB/s, narrowing at ~6.2.
        typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
        for (; (i | 63u) < a.ngroups; i += stride) {
            const uint64_t w = i & ~(uint64_t)63, lane = i & 63u;  // wave chunk: groups [w, w + 64)
            const uint64_t p0 = w * 2 + lane, p1 = p0 + 64;         // the two 4-element runs
            Pack<SS> sp[SV];
            if constexpr (sizeof(SS) < sizeof(DS)) {
                const u32x2* s2 = reinterpret_cast<const u32x2*>(src);
                const u32x2 x0 = __builtin_nontemporal_load(s2 + p0), x1 = __builtin_nontemporal_load(s2 + p1);
                sp[0] = __builtin_bit_cast(Pack<SS>, u32x4{x0.x, x0.y, x1.x, x1.y});
            } else {
                sp[0] = __builtin_bit_cast(Pack<SS>, vload<3>(src + p0));
                sp[1] = __builtin_bit_cast(Pack<SS>, vload<3>(src + p1));
            }
            const uint64_t ea = a.head + 4 * p0, eb = a.head + 4 * p1;  // element indices (V_TAIL_TRUNC)
            Pack<DS> dp[DV];
            convert_runs<ST, DT, V, false>(sp, dp, ea, eb, a.trunc_from);
            if constexpr (!std::is_same<ST, bf16_tag>::value) {  // bf16 -> fp32 is a shift: bits exact as is
                uint32_t bits = 0;
#pragma unroll
                for (int v = 0; v < SV; v++) bits |= inf_nan_bits<ST>(__builtin_bit_cast(u32x4, sp[v]));
                if (__builtin_expect(inf_nan_hit<ST>(bits), 0)) convert_runs<ST, DT, V, true>(sp, dp, ea, eb, a.trunc_from);
            }
            if constexpr (SC1) {
                // the wave chunk's destination: 128 consecutive stores of 16 B
                // (widening) or 8 B (narrowing), the whole chunk in range
                constexpr uint32_t SB = sizeof(SS) < sizeof(DS) ? 16u : 8u;
                const __amdgpu_buffer_rsrc_t o = tile_rsrc(dst, w * 2 * SB, 128u * SB);
                const uint32_t o0 = (uint32_t)lane * SB, o1 = o0 + 64u * SB;
                if constexpr (sizeof(SS) < sizeof(DS)) {
                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, dp[0]), o, o0, 0, kAuxSC1NT);
                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, dp[1]), o, o1, 0, kAuxSC1NT);
                } else {
                    const u32x4 d = __builtin_bit_cast(u32x4, dp[0]);
                    __builtin_amdgcn_raw_buffer_store_b64(u32x2{d.x, d.y}, o, o0, 0, kAuxSC1NT);
                    __builtin_amdgcn_raw_buffer_store_b64(u32x2{d.z, d.w}, o, o1, 0, kAuxSC1NT);
                }
            } else if constexpr (sizeof(SS) < sizeof(DS)) {
                vstore<3>(dst + p0, __builtin_bit_cast(u32x4, dp[0]));
                vstore<3>(dst + p1, __builtin_bit_cast(u32x4, dp[1]));
            } else {
                const u32x4 d = __builtin_bit_cast(u32x4, dp[0]);
                u32x2* d2 = reinterpret_cast<u32x2*>(dst);
                __builtin_nontemporal_store(u32x2{d.x, d.y}, d2 + p0);
                __builtin_nontemporal_store(u32x2{d.z, d.w}, d2 + p1);
            }
        }
    }
    for (; i < a.ngroups; i += stride) {
        Pack<SS> sp[SV];
#pragma unroll
        for (int v = 0; v < SV; v++) sp[v] = __builtin_bit_cast(Pack<SS>, vload<3>(src + i * SV + v));
        Pack<DS> dp[DV];
        convert_group<ST, DT, V, false>(sp, dp, a.head + i * 8, a.trunc_from);
        if constexpr (!std::is_same<ST, bf16_tag>::value) {  // bf16 -> fp32 is a shift: bits exact as is
            uint32_t bits = 0;
#pragma unroll
            for (int v = 0; v < SV; v++) bits |= inf_nan_bits<ST>(__builtin_bit_cast(u32x4, sp[v]));
            if (__builtin_expect(inf_nan_hit<ST>(bits), 0)) convert_group<ST, DT, V, true>(sp, dp, a.head + i * 8, a.trunc_from);
        }
#pragma unroll
        for (int v = 0; v < DV; v++) vstore<3>(dst + i * DV + v, __builtin_bit_cast(u32x4, dp[v]));
    }
    // head (< 16 bytes of dst) and tail (< 8 elements) by the first lanes of block 0
    if (blockIdx.x == 0) {
        if (threadIdx.x < a.head)
            static_cast<DS*>(a.dst)[threadIdx.x] =
                convert_elem<ST, DT, V>(static_cast<const SS*>(a.src)[threadIdx.x], threadIdx.x, a.trunc_from);
        if (threadIdx.x < a.count - a.head - a.ngroups * 8) {
            const uint64_t j = a.head + a.ngroups * 8 + threadIdx.x;
            static_cast<DS*>(a.dst)[j] = convert_elem<ST, DT, V>(static_cast<const SS*>(a.src)[j], j, a.trunc_from);
        }
    }
}

// Byte copy with optional non-temporal stores (ccl_comp_copy), on the
// destination's 16-byte grid: block 0 copies the < 16-byte head and tail byte
// by byte, the body moves 16-byte vectors.  The source may sit at any byte
// offset from that grid (unaligned 16-byte loads, as in the reduce kernels).
template <int MEM>
__global__ __launch_bounds__(kBlock) void copy_kernel(const char* __restrict__ src8, char* __restrict__ dst8,
                                                      uint32_t head, uint64_t nvec, uint32_t tail) {
    if (blockIdx.x == 0) {
        if (threadIdx.x < head) dst8[threadIdx.x] = src8[threadIdx.x];
        if (threadIdx.x < tail) {
            const uint64_t o = head + nvec * 16 + threadIdx.x;
            dst8[o] = src8[o];
        }
    }
    const u32x4* __restrict__ src = reinterpret_cast<const u32x4*>(src8 + head);
    u32x4* __restrict__ dst = reinterpret_cast<u32x4*>(dst8 + head);
    constexpr int U = 4;
    const uint64_t tile = (uint64_t)kBlock * U;
    for (uint64_t base = (uint64_t)blockIdx.x * tile + threadIdx.x; base < nvec;
         base += (uint64_t)gridDim.x * tile) {
        u32x4 r[U];
#pragma unroll
        for (int j = 0; j < U; j++)
            if (base + (uint64_t)j * kBlock < nvec) r[j] = vload<MEM & 1>(src + base + (uint64_t)j * kBlock);
#pragma unroll
        for (int j = 0; j < U; j++)
            if (base + (uint64_t)j * kBlock < nvec) vstore<MEM & 2>(dst + base + (uint64_t)j * kBlock, r[j]);
    }
}

// The same copy as one tile per block, one 16-byte vector per lane, no loop
// (reduce2_kernel's shape); the default grid.  One-wave (64-lane) tiles with
// no residency cap: 1 GiB in 0.320 ms against 0.336 at round 2's 512 lanes
// (-5 %; the 1-read/1-write stream keeps only 1 KiB per wave in flight, so
// unlike the reduce kernels it wants every wave slot; tools/occupancy_sweep.hip
// copyu / copyconv, profiles/round3_occupancy/).  Round 2's sweep
// (tools/copy_sweep.hip) had 512 lanes at 6.44 TB/s against 5.78 for
// copy_kernel<2>, which stays for a capped grid (mi_set_max_blocks).
// MEM bit 0: nt loads; bit 1: nt stores; bit 2: stores through a per-tile
// buffer descriptor with sc1 + nt (each line leaves L2 as it is written, as
// reduce2_kernel stores), for streaming copies far larger than the caches.
constexpr int kCopyBlock = 64;
template <int MEM, int B = kCopyBlock>
__global__ __launch_bounds__(B) void copy_lean_kernel(const char* __restrict__ src8, char* __restrict__ dst8,
                                                      uint32_t head, uint64_t nvec, uint32_t tail) {
    if (blockIdx.x == 0) {
        if (threadIdx.x < head) dst8[threadIdx.x] = src8[threadIdx.x];
        if (threadIdx.x < tail) {
            const uint64_t o = head + nvec * 16 + threadIdx.x;
            dst8[o] = src8[o];
        }
    }
    const uint64_t t0 = (uint64_t)blockIdx.x * B;
    const uint64_t v = t0 + threadIdx.x;
    if (MEM & 4) {
        // global nt loads: buffer loads here ran 0.4-0.7 % slower in every
        // one of 20 fresh placements (tools/ab_c2.py --config copy,
        // profiles/round6_run8/), unlike the 2-input reduce's
        const uint64_t tleft = nvec > t0 ? nvec - t0 : 0;
        const uint32_t tbytes = (uint32_t)(tleft < (uint64_t)B ? tleft : (uint64_t)B) * 16u;
        const __amdgpu_buffer_rsrc_t o = tile_rsrc(dst8 + head, t0 * 16, tbytes);
        if (v < nvec)
            __builtin_amdgcn_raw_buffer_store_b128(vload<MEM & 1>(reinterpret_cast<const u32x4*>(src8 + head) + v), o,
                                                   threadIdx.x * 16u, 0, kAuxSC1NT);
    } else if (v < nvec) {
        vstore<MEM & 2>(reinterpret_cast<u32x4*>(dst8 + head) + v,
                        vload<MEM & 1>(reinterpret_cast<const u32x4*>(src8 + head) + v));
    }
}

}  // namespace mi
