/*
 * comp_oracle.c — TEST INFRASTRUCTURE ONLY (see comp_oracle.h).
 *
 * A plain-C restatement of oneCCL's CPU local reduction, src/comp
 * (reference snapshot 2024-12-20, v2021.14.0).  Every function cites the
 * reference file:line it restates.  The x86 intrinsics the reference calls
 * are restated from their published (Intel SDM) definitions;
 * oracle/isa_check.c cross-checks those restatements against the real
 * instructions on CPUs that have them.
 *
 * Pinned to the reference's own compiled code (oracle/Makefile, target ref):
 *   - oracle/ref_harness.cpp: the AVX-512 bf16 / fp16 bodies
 *     (the _intrisics sources of src/comp/bf16 and src/comp/fp16) -> tests/golden/ref_vectors*.npz;
 *   - oracle/ref_comp_harness.cpp: src/comp/comp.cpp, bf16/bf16.cpp and the
 *     logger/datatype sources they need, built with the reference's Release
 *     flags (ITT off) -> tests/golden/ref_comp_vectors.npz (CCL_REDUCE for the
 *     ten non-LP types, the scalar bf16 impl, the storage-precision batch
 *     reduce).  Only ccl::global_data::get/env stay unresolved (the
 *     runtime's global state), so the LP dispatchers and the keep-precision
 *     batch reduce, which call them, are pinned through their parts.
 *
 * Build: oracle/Makefile -> oracle/lib/libcomp_oracle.so  (gcc -O3, no
 * -ffast-math, no FMA contraction concerns: each element is one op).
 */
#include "comp_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ccl::reduction, include/oneapi/ccl/types.hpp:41-47 */
enum { OP_SUM = 0, OP_PROD = 1, OP_MIN = 2, OP_MAX = 3 };
/* ccl::datatype, include/oneapi/ccl/types.hpp:52-69 */
enum {
    DT_INT8 = 0, DT_UINT8, DT_INT16, DT_UINT16, DT_INT32, DT_UINT32,
    DT_INT64, DT_UINT64, DT_FLOAT16, DT_FLOAT32, DT_FLOAT64, DT_BFLOAT16
};

/* ------------------------------------------------------------------ */
/* conversions                                                         */
/* ------------------------------------------------------------------ */

static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

/* ccl_convert_bf16_to_fp32_scalar, src/comp/bf16/bf16.cpp:56-61 (and the
 * avx512 ccl_bf16_load_as_fp32, bf16_intrisics.hpp:62-65: zero-extend, <<16) */
float orc_bf16_to_fp32(uint16_t v) { return u2f((uint32_t)v << 16); }

/* ccl_convert_fp32_to_bf16_scalar, src/comp/bf16/bf16.cpp:50-54 (high half);
 * ccl_fp32_store_as_bf16_avx512f, bf16_intrisics.hpp:67-70 (bsrli by 2 bytes
 * then cvtepi32_epi16 truncating narrow == the same high half). */
uint16_t orc_fp32_to_bf16_trunc(float f) { return (uint16_t)(f2u(f) >> 16); }

/* ccl_fp32_store_as_bf16_avx512bf, bf16_intrisics.hpp:72-76 ->
 * _mm512_cvtneps_pbh = VCVTNEPS2BF16.  Intel SDM pseudo-code
 * convert_fp32_to_bfloat16(): zero or denormal -> signed zero (the
 * instruction ignores MXCSR and always treats denormals as zero);
 * infinity -> high half; NaN -> high half with bit 6 set (quiet);
 * otherwise round-to-nearest-even by adding 0x7FFF + lsb. */
uint16_t orc_fp32_to_bf16_rne(float f) {
    uint32_t u = f2u(f);
    if ((u & 0x7F800000u) == 0) return (uint16_t)((u >> 16) & 0x8000u);
    if ((u & 0x7FFFFFFFu) > 0x7F800000u) return (uint16_t)((u >> 16) | 0x0040u);
    if ((u & 0x7FFFFFFFu) == 0x7F800000u) return (uint16_t)(u >> 16);
    u += 0x7FFFu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

/* _mm256_cvtph_ps / _mm512_cvtph_ps = VCVTPH2PS (fp16_intrisics.hpp:100,128):
 * exact widening; denormal halves are normalised; a signalling NaN is
 * quietened (payload kept). */
float orc_fp16_to_fp32(uint16_t h) {
    uint32_t sign = ((uint32_t)h & 0x8000u) << 16;
    uint32_t exp = ((uint32_t)h >> 10) & 0x1Fu;
    uint32_t mant = (uint32_t)h & 0x3FFu;
    uint32_t u;
    if (exp == 0) {
        if (mant == 0) {
            u = sign;
        } else {
            int e = 113; /* 127 - 15 + 1 */
            while (!(mant & 0x400u)) { mant <<= 1; e--; }
            mant &= 0x3FFu;
            u = sign | ((uint32_t)e << 23) | (mant << 13);
        }
    } else if (exp == 31) {
        u = sign | 0x7F800000u | (mant << 13);
        if (mant) u |= 0x00400000u;
    } else {
        u = sign | ((exp + 112u) << 23) | (mant << 13);
    }
    return u2f(u);
}

/* _mm256_cvtps_ph(x, 0) / _mm512_cvtps_ph(x, 0) = VCVTPS2PH with imm8 = 0
 * (round to nearest even), fp16_intrisics.hpp:103,131: denormal results are
 * produced (not flushed), overflow -> infinity, NaN -> quiet NaN keeping the
 * top 9 payload bits. */
uint16_t orc_fp32_to_fp16_rne(float f) {
    uint32_t u = f2u(f);
    uint16_t sign = (uint16_t)((u >> 16) & 0x8000u);
    uint32_t a = u & 0x7FFFFFFFu;
    if (a > 0x7F800000u) return (uint16_t)(sign | 0x7E00u | ((a >> 13) & 0x3FFu));
    if (a >= 0x477FF000u) return (uint16_t)(sign | 0x7C00u); /* >= 65520: inf */
    if (a >= 0x38800000u) {                                   /* normal half */
        a += 0xFFFu + ((a >> 13) & 1u);
        return (uint16_t)(sign | ((a - 0x38000000u) >> 13));
    }
    if (a <= 0x33000000u) return sign; /* <= 2^-25 rounds to zero */
    {
        uint32_t e = a >> 23;
        uint32_t m = (a & 0x7FFFFFu) | 0x800000u;
        uint32_t shift = 126u - e; /* units of 2^-24 */
        uint32_t q = m >> shift;
        uint32_t rem = m & ((1u << shift) - 1u);
        uint32_t half = 1u << (shift - 1u);
        if (rem > half || (rem == half && (q & 1u))) q++;
        return (uint16_t)(sign | q);
    }
}

/* ------------------------------------------------------------------ */
/* CCL_REDUCE, src/comp/comp.cpp:31-58                                  */
/* ------------------------------------------------------------------ */
/* sum/prod: inout op= in.  Integer sum/prod wrap (the reference's gcc -O3
 * build wraps; computed here in unsigned arithmetic to stay defined).
 * min: std::min(in, inout) == (inout < in) ? inout : in  (returns `in` on
 * ties and when either operand is NaN); max: std::max(in, inout) ==
 * (in < inout) ? inout : in. */
#define ORC_REDUCE_INT(T, UT, WT)                                                     \
    do {                                                                               \
        const T* a = (const T*)in_buf;                                                 \
        T* b = (T*)inout_buf;                                                          \
        size_t i;                                                                      \
        switch (op) {                                                                  \
            case OP_SUM:                                                               \
                for (i = 0; i < n; i++) b[i] = (T)(UT)((WT)(UT)b[i] + (WT)(UT)a[i]);   \
                break;                                                                 \
            case OP_PROD:                                                              \
                for (i = 0; i < n; i++) b[i] = (T)(UT)((WT)(UT)b[i] * (WT)(UT)a[i]);   \
                break;                                                                 \
            case OP_MIN:                                                               \
                for (i = 0; i < n; i++) b[i] = (b[i] < a[i]) ? b[i] : a[i];            \
                break;                                                                 \
            case OP_MAX:                                                               \
                for (i = 0; i < n; i++) b[i] = (a[i] < b[i]) ? b[i] : a[i];            \
                break;                                                                 \
            default: return -1;                                                        \
        }                                                                              \
    } while (0)

/* Floating point: `inout op= in` as the reference's Release build (g++ -O3)
 * compiles it, SSE ADDPS/MULPS with `inout` as the first source: a NaN operand
 * comes back quieted, inout's when both are; an invalid operation (inf - inf,
 * 0 * inf) gives the x86 default NaN (sign set).  Written out (NAN_IO_F/D)
 * rather than left to this compiler's operand order.  Pinned bit for bit,
 * payloads included, by tests/golden/ref_comp_vectors.npz (the reference's
 * compiled comp.cpp, oracle/ref_comp_harness.cpp). */
/* (written as selects, lowest priority first, so that gcc keeps the loop
 * vectorized) */
static inline float nan_io_f(float r, float io, float in) {
    uint32_t o = (r != r) ? 0xFFC00000u : f2u(r);          /* invalid operation: default NaN */
    o = (in != in) ? (f2u(in) | 0x400000u) : o;             /* else `in`'s NaN, quieted */
    o = (io != io) ? (f2u(io) | 0x400000u) : o;             /* `inout`'s NaN first */
    return u2f(o);
}
static inline uint64_t d2u(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }
static inline double u2d(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }
static inline double nan_io_d(double r, double io, double in) {
    uint64_t o = (r != r) ? 0xFFF8000000000000ull : d2u(r);
    o = (in != in) ? (d2u(in) | 0x8000000000000ull) : o;
    o = (io != io) ? (d2u(io) | 0x8000000000000ull) : o;
    return u2d(o);
}

#define ORC_REDUCE_FP(T, NAN_IO)                                                       \
    do {                                                                               \
        const T* a = (const T*)in_buf;                                                 \
        T* b = (T*)inout_buf;                                                          \
        size_t i;                                                                      \
        switch (op) {                                                                  \
            case OP_SUM: for (i = 0; i < n; i++) b[i] = NAN_IO(b[i] + a[i], b[i], a[i]); break; \
            case OP_PROD: for (i = 0; i < n; i++) b[i] = NAN_IO(b[i] * a[i], b[i], a[i]); break; \
            case OP_MIN:                                                               \
                for (i = 0; i < n; i++) b[i] = (b[i] < a[i]) ? b[i] : a[i];            \
                break;                                                                 \
            case OP_MAX:                                                               \
                for (i = 0; i < n; i++) b[i] = (a[i] < b[i]) ? b[i] : a[i];            \
                break;                                                                 \
            default: return -1;                                                        \
        }                                                                              \
    } while (0)

/* fp32 op on the widened operands.  `simd` selects the _mm512_{min,max}_ps
 * (in, inout) form: MINPS returns the SECOND operand unless first < second
 * (so `inout` on NaN and on +0/-0 ties); MAXPS likewise with >.
 * bf16_intrisics.cpp:28-34, fp16_intrisics.hpp:72-77.  Non-simd = std::
 * forms of bf16.cpp:42-48. */
/* x86 NaN propagation of ADDPS/MULPS (Intel SDM vol. 1 §4.8.3.5, table
 * 4-7): a NaN operand is returned quieted, the FIRST source's when both are
 * NaN; an invalid operation on non-NaN operands (inf - inf, 0 * inf) gives the
 * default NaN, which the C operation below already produces on x86.  The
 * reference computes _mm512_add_ps(in, inout) (bf16_intrisics.cpp:20-26,
 * fp16_intrisics.hpp:58-63), so `in` is the first source.  Pinned bit for bit,
 * payloads included, by tests/golden/ref_vectors.npz (the reference's own
 * code, oracle/ref_harness.cpp).  C's `in + io` alone leaves the both-NaN
 * choice to the compiler's operand order. */
static inline float x86_nan_first(float r, float first, float second) {
    if (first != first) return u2f(f2u(first) | 0x400000u);
    if (second != second) return u2f(f2u(second) | 0x400000u);
    return r;
}

static inline float lp_apply(int op, int simd, float in, float io) {
    switch (op) {
        case OP_SUM: return x86_nan_first(in + io, in, io);
        case OP_PROD: return x86_nan_first(in * io, in, io);
        case OP_MIN: return simd ? ((in < io) ? in : io) : ((io < in) ? io : in);
        default: return simd ? ((in > io) ? in : io) : ((in < io) ? io : in);
    }
}

/* The fp32 accumulation of an fp32-accumulating fan-in: CCL_REDUCE(float)'s
 * step (keep-precision runs ccl_comp_reduce_regular on float32,
 * comp.cpp:223-229), so the accumulator's NaN wins a sum or product. */
static inline float acc32_apply(int op, int simd, float in, float io) {
    switch (op) {
        case OP_SUM: return nan_io_f(io + in, io, in);
        case OP_PROD: return nan_io_f(io * in, io, in);
        case OP_MIN: return simd ? ((in < io) ? in : io) : ((io < in) ? io : in);
        default: return simd ? ((in > io) ? in : io) : ((in < io) ? io : in);
    }
}

/* ccl_bf16_reduce, src/comp/bf16/bf16.cpp:87-110:
 *   scalar   -> ccl_bf16_reduce_scalar_impl (bf16.cpp:63-85): std min/max, truncate
 *   avx512f  -> CCL_BF16_DEFINE_REDUCE_FUNC(avx512f) (bf16_intrisics.hpp:78-114):
 *               MINPS/MAXPS order, truncate
 *   avx512bf -> same with VCVTNEPS2BF16 rounding.
 * The masked tail tile (bf16_intrisics.hpp:96-105) computes the same values
 * on the active lanes.  (The reference's `int i` loop index overflows above
 * 2^31 elements, bf16_intrisics.hpp:108; not reproduced.) */
static int orc_bf16_reduce(const void* in_buf, size_t n, void* inout_buf, int op,
                           int impl) {
    const uint16_t* a = (const uint16_t*)in_buf;
    uint16_t* b = (uint16_t*)inout_buf;
    int simd = (impl != ORC_BF16_SCALAR);
    int rne = (impl == ORC_BF16_AVX512BF);
    if (op < OP_SUM || op > OP_MAX) return -1;
    for (size_t i = 0; i < n; i++) {
        float r = lp_apply(op, simd, orc_bf16_to_fp32(a[i]), orc_bf16_to_fp32(b[i]));
        b[i] = rne ? orc_fp32_to_bf16_rne(r) : orc_fp32_to_bf16_trunc(r);
    }
    return 0;
}

/* ccl_fp16_reduce -> ccl_fp16_reduce_impl, src/comp/fp16/fp16.cpp:41-53,
 * fp16_intrisics.hpp:204-248: f16c (8-wide) and avx512f (16-wide) widen to
 * fp32, apply MINPS/MAXPS-order ops, round RNE.  avx512fp16 does native
 * fp16 arithmetic (fp16_intrisics.cpp:23-41, hpp :150-176): for +,* on fp16
 * operands an fp32 result rounded once to fp16 is the correctly rounded fp16
 * result (fp32 has 24 >= 2*11+2 bits, so no double-rounding error), so sum
 * and prod give the same bits.  VMINPH/VMAXPH select like MINPS/MAXPS but
 * return the selected operand as stored, where the fp32 route's VCVTPH2PS has
 * quieted it: with a NaN `inout` (always the one selected) a signalling NaN
 * stays signalling.  Both proven on all 2^32 operand pairs against IEEE
 * binary16 arithmetic (oracle/fp16_native_check.c, FP16_NATIVE_CHECK.json).
 * Any other impl type falls through and computes nothing (:214-247) —
 * reproduced. */
static int orc_fp16_reduce(const void* in_buf, size_t n, void* inout_buf, int op,
                           int impl) {
    const uint16_t* a = (const uint16_t*)in_buf;
    uint16_t* b = (uint16_t*)inout_buf;
    if (op < OP_SUM || op > OP_MAX) return -1;
    if (impl != ORC_FP16_F16C && impl != ORC_FP16_AVX512F && impl != ORC_FP16_AVX512FP16)
        return 0;
    const int native_mm = impl == ORC_FP16_AVX512FP16 && (op == OP_MIN || op == OP_MAX);
    for (size_t i = 0; i < n; i++) {
        if (native_mm && (b[i] & 0x7C00u) == 0x7C00u && (b[i] & 0x03FFu)) continue; /* NaN inout, as stored */
        float r = lp_apply(op, 1, orc_fp16_to_fp32(a[i]), orc_fp16_to_fp32(b[i]));
        b[i] = orc_fp32_to_fp16_rne(r);
    }
    return 0;
}

/* ccl_comp_reduce_regular, src/comp/comp.cpp:76-121 (dtype switch :96-114).
 * out_count is written only by the bf16/fp16 paths (bf16.cpp:94-96,
 * fp16.cpp:48-50), as in the reference. */
int orc_comp_reduce(const void* in_buf, size_t n, void* inout_buf, size_t* out_count,
                    int dtype, int op, int bf16_impl, int fp16_impl) {
    switch (dtype) {
        case DT_INT8: ORC_REDUCE_INT(int8_t, uint8_t, uint32_t); break;
        case DT_UINT8: ORC_REDUCE_INT(uint8_t, uint8_t, uint32_t); break;
        case DT_INT16: ORC_REDUCE_INT(int16_t, uint16_t, uint32_t); break;
        case DT_UINT16: ORC_REDUCE_INT(uint16_t, uint16_t, uint32_t); break;
        case DT_INT32: ORC_REDUCE_INT(int32_t, uint32_t, uint32_t); break;
        case DT_UINT32: ORC_REDUCE_INT(uint32_t, uint32_t, uint32_t); break;
        case DT_INT64: ORC_REDUCE_INT(int64_t, uint64_t, uint64_t); break;
        case DT_UINT64: ORC_REDUCE_INT(uint64_t, uint64_t, uint64_t); break;
        case DT_FLOAT16:
            if (out_count) *out_count = n;
            return orc_fp16_reduce(in_buf, n, inout_buf, op, fp16_impl);
        case DT_FLOAT32: ORC_REDUCE_FP(float, nan_io_f); break;
        case DT_FLOAT64: ORC_REDUCE_FP(double, nan_io_d); break;
        case DT_BFLOAT16:
            if (out_count) *out_count = n;
            return orc_bf16_reduce(in_buf, n, inout_buf, op, bf16_impl);
        default: return -1;
    }
    return 0;
}

static size_t orc_dtype_size(int dtype) {
    switch (dtype) {
        case DT_INT8: case DT_UINT8: return 1;
        case DT_INT16: case DT_UINT16: case DT_FLOAT16: case DT_BFLOAT16: return 2;
        case DT_INT32: case DT_UINT32: case DT_FLOAT32: return 4;
        case DT_INT64: case DT_UINT64: case DT_FLOAT64: return 8;
        default: return 0;
    }
}

/* ------------------------------------------------------------------ */
/* worker-count emulation                                              */
/* ------------------------------------------------------------------ */
typedef struct {
    const char* in;
    char* inout;
    size_t n;
    int dtype, op, bf16_impl, fp16_impl, rc;
} orc_part_t;

static void* orc_part_run(void* p) {
    orc_part_t* t = (orc_part_t*)p;
    t->rc = orc_comp_reduce(t->in, t->n, t->inout, NULL, t->dtype, t->op, t->bf16_impl,
                            t->fp16_impl);
    return NULL;
}

int orc_comp_reduce_mt(const void* in_buf, size_t n, void* inout_buf, int dtype, int op,
                       int bf16_impl, int fp16_impl, int nthreads) {
    size_t es = orc_dtype_size(dtype);
    if (!es) return -1;
    if (nthreads <= 1 || n < (size_t)nthreads * 64)
        return orc_comp_reduce(in_buf, n, inout_buf, NULL, dtype, op, bf16_impl, fp16_impl);
    orc_part_t* parts = (orc_part_t*)calloc((size_t)nthreads, sizeof(orc_part_t));
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    size_t per = ((n + (size_t)nthreads - 1) / (size_t)nthreads + 63) / 64 * 64;
    int rc = 0;
    for (int t = 0; t < nthreads; t++) {
        size_t b = (size_t)t * per, e = b + per;
        if (b > n) b = n;
        if (e > n) e = n;
        parts[t].in = (const char*)in_buf + b * es;
        parts[t].inout = (char*)inout_buf + b * es;
        parts[t].n = e - b;
        parts[t].dtype = dtype;
        parts[t].op = op;
        parts[t].bf16_impl = bf16_impl;
        parts[t].fp16_impl = fp16_impl;
        pthread_create(&th[t], NULL, orc_part_run, &parts[t]);
    }
    for (int t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        if (parts[t].rc) rc = parts[t].rc;
    }
    free(parts);
    free(th);
    return rc;
}

/* ------------------------------------------------------------------ */
/* array conversions, src/comp/bf16/bf16.cpp:113-169                    */
/* ------------------------------------------------------------------ */
/* Non-scalar impls convert the first (count/16)*16 elements 16 at a time
 * (avx512bf -> RNE, avx512f -> truncate, bf16.cpp:136-143) and the remaining
 * tail with the scalar truncation (:145-148).  Scalar impl: all truncated. */
void orc_convert_fp32_to_bf16_arrays(const float* src, uint16_t* dst, size_t count,
                                     int bf16_impl) {
    size_t limit = 0, i;
    if (bf16_impl != ORC_BF16_SCALAR) {
        limit = (count / 16) * 16;
        for (i = 0; i < limit; i++)
            dst[i] = (bf16_impl == ORC_BF16_AVX512BF) ? orc_fp32_to_bf16_rne(src[i])
                                                      : orc_fp32_to_bf16_trunc(src[i]);
    }
    for (i = limit; i < count; i++) dst[i] = orc_fp32_to_bf16_trunc(src[i]);
}

/* ccl_convert_fp32_to_fp16 (fp16.cpp:55-57) applied over an array: VCVTPS2PH
 * imm8 = 0 on every element. */
void orc_convert_fp32_to_fp16_arrays(const float* src, uint16_t* dst, size_t count) {
    for (size_t i = 0; i < count; i++) dst[i] = orc_fp32_to_fp16_rne(src[i]);
}

/* ccl_convert_fp16_to_fp32 (fp16.cpp:59-61) applied over an array: VCVTPH2PS
 * on every element (a signalling NaN comes back quiet). */
void orc_convert_fp16_to_fp32_arrays(const uint16_t* src, float* dst, size_t count) {
    for (size_t i = 0; i < count; i++) dst[i] = orc_fp16_to_fp32(src[i]);
}

void orc_convert_bf16_to_fp32_arrays(const uint16_t* src, float* dst, size_t count) {
    for (size_t i = 0; i < count; i++) dst[i] = orc_bf16_to_fp32(src[i]);
}

/* ccl_comp_batch_reduce, src/comp/comp.cpp:202-249.
 * keep-precision: acc = fp32(inout); for each input i>=1: tmp = fp32(input);
 * ccl_comp_reduce_regular(tmp, acc, float32) (CCL_REDUCE(float): std::min/
 * max order); inout = bf16(acc) through the array conversion.  The buffers
 * are read as bf16 whatever `dtype` says, as in the reference (it only uses
 * dtype.size() for the input stride, :219-220).
 * Otherwise: chained ccl_comp_reduce_regular in storage precision. */
int orc_comp_batch_reduce(const void* in_buf, const size_t* offsets, size_t n_offsets,
                          size_t in_count, void* inout_buf, size_t* out_count, int dtype,
                          int op, int keep_precision, float* tmp, float* acc,
                          int bf16_impl, int fp16_impl) {
    size_t es = orc_dtype_size(dtype);
    if (!es) return -1;
    if (keep_precision) {
        orc_convert_bf16_to_fp32_arrays((const uint16_t*)inout_buf, acc, in_count);
        for (size_t i = 1; i < n_offsets; i++) {
            orc_convert_bf16_to_fp32_arrays(
                (const uint16_t*)((const char*)in_buf + es * offsets[i]), tmp, in_count);
            if (orc_comp_reduce(tmp, in_count, acc, out_count, DT_FLOAT32, op, bf16_impl,
                                fp16_impl))
                return -1;
        }
        orc_convert_fp32_to_bf16_arrays(acc, (uint16_t*)inout_buf, in_count, bf16_impl);
    } else {
        for (size_t i = 1; i < n_offsets; i++) {
            if (orc_comp_reduce((const char*)in_buf + es * offsets[i], in_count, inout_buf,
                                out_count, dtype, op, bf16_impl, fp16_impl))
                return -1;
        }
    }
    return 0;
}

/* Oracle extension: fp32-accumulating low-precision fan-in (the intent of
 * the keep-precision mode above, also for fp16), single rounding at the end:
 * acc = f32(inputs[0]); acc = op(f32(inputs[j]), acc); out = round(acc). */
int orc_lp_fanin_acc_fp32(const void* const* inputs, int k, void* out, size_t count,
                          int dtype, int op, int bf16_rne, int minmax_inout_first) {
    if (k < 1 || (dtype != DT_BFLOAT16 && dtype != DT_FLOAT16)) return -1;
    if (op < OP_SUM || op > OP_MAX) return -1;
    int bf = (dtype == DT_BFLOAT16);
    for (size_t i = 0; i < count; i++) {
        uint16_t v0 = ((const uint16_t*)inputs[0])[i];
        float acc = bf ? orc_bf16_to_fp32(v0) : orc_fp16_to_fp32(v0);
        for (int j = 1; j < k; j++) {
            uint16_t vj = ((const uint16_t*)inputs[j])[i];
            float x = bf ? orc_bf16_to_fp32(vj) : orc_fp16_to_fp32(vj);
            acc = acc32_apply(op, minmax_inout_first, x, acc);
        }
        ((uint16_t*)out)[i] = bf ? (bf16_rne ? orc_fp32_to_bf16_rne(acc)
                                             : orc_fp32_to_bf16_trunc(acc))
                                 : orc_fp32_to_fp16_rne(acc);
    }
    return 0;
}
