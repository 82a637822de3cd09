/*
 * fp16_native_check.c — TEST INFRASTRUCTURE ONLY.
 *
 * The reference's third fp16 impl, avx512fp16 (src/comp/fp16/fp16_intrisics.cpp:
 * 23-41, fp16_intrisics.hpp:150-176), computes in native half precision:
 * _mm512_add_ph / _mm512_mul_ph / _mm512_min_ph / _mm512_max_ph (in, inout).
 * Its library build needs gcc >= 12 and a CPU with AVX512_FP16, neither of
 * which this image has.  The oracle and the kernels compute that impl by the
 * fp32 route of f16c / avx512f: widen to fp32 (VCVTPH2PS), one fp32 op (x86
 * NaN rules, in as the first source), narrow with VCVTPS2PH imm8=0 (RNE).
 * This program compares the two on every pair of fp16 bit patterns:
 *
 *   fp32 route   the real instructions: F16C conversions, ADDSS / MULSS /
 *                MINSS / MAXSS with `in` as the first source (inline asm, so
 *                the compiler cannot swap the operands);
 *   native model what IEEE 754 binary16 arithmetic gives, which VADDPH /
 *                VMULPH implement: the exact sum or product (exact in double:
 *                at most 50 significant bits) rounded once to fp16, nearest
 *                even, overflow to infinity; NaN operands: the first NaN
 *                source quieted; invalid (inf - inf, 0 * inf): the default NaN
 *                0xFE00; VMINPH / VMAXPH: the second source when either is a
 *                NaN or both are zeros (the MINPS rule).
 *
 * Why sum and prod must agree: fp32 has 24 >= 2*11 + 2 significand bits, so
 * an fp32 add or multiply of two fp16 values rounded to fp16 equals the
 * correctly rounded fp16 operation (no double-rounding error); products are
 * even exact in fp32.  Min and max differ in one case: VMINPH/VMAXPH return
 * the selected operand as stored, while the fp32 route's VCVTPH2PS quiets a
 * signalling NaN, so a signalling-NaN `inout` (the operand selected whenever
 * either is a NaN) comes back quiet from the route and signalling from the
 * native instruction: 65536 x 1022 pairs per op.  The check counts exactly
 * those, and then checks the oracle's avx512fp16 model (orc_comp_reduce with
 * fp16 impl avx512fp16, which keeps a NaN inout as stored) against the
 * native model on every pair: 0 mismatches expected for all four ops.
 *
 * Where the CPU has AVX512_FP16, the native model is itself checked against
 * the instructions (VADDPH / VMULPH / VMINPH / VMAXPH, in first) on every
 * pair, so the reference's avx512fp16 semantics are pinned by the hardware.
 *
 * Usage: fp16_native_check [stride] [threads]  (stride over the 2^32 (in,
 * inout) pairs; 1 = exhaustive).  One JSON line; exit 0 = all equal,
 * 1 = mismatch, 2 = CPU lacks F16C (skipped).
 */
#include <immintrin.h>
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "comp_oracle.h"

static float h2f(uint16_t h) { return _cvtsh_ss(h); }
static uint16_t f2h(float f) { return (uint16_t)_cvtss_sh(f, 0); }

static int is_nan16(uint16_t h) { return (h & 0x7C00) == 0x7C00 && (h & 0x03FF); }

/* the fp32 route, with the instructions the oracle / kernels restate */
static uint16_t route(uint16_t in, uint16_t inout, int op) {
    float r = h2f(in);
    const float b = h2f(inout);
    switch (op) {
        case 0: __asm__("addss %1, %0" : "+x"(r) : "x"(b)); break;  /* r = in + inout, in first */
        case 1: __asm__("mulss %1, %0" : "+x"(r) : "x"(b)); break;
        case 2: __asm__("minss %1, %0" : "+x"(r) : "x"(b)); break;  /* NaN or zeros: inout */
        default: __asm__("maxss %1, %0" : "+x"(r) : "x"(b)); break;
    }
    return f2h(r);
}

/* exact double -> binary16, round to nearest even (x finite) */
static uint16_t d2h_rne(double x) {
    const uint16_t sign = signbit(x) ? 0x8000 : 0;
    const double ax = fabs(x);
    if (ax >= 65520.0) return sign | 0x7C00; /* 65504 + half an ulp ties to 65536: overflow */
    int e;
    (void)frexp(ax, &e);                       /* ax = m * 2^e, m in [0.5, 1) */
    const int q = ax < 0x1p-14 ? -24 : e - 11; /* exponent of the fp16 ulp at ax */
    const double r = nearbyint(ldexp(ax, -q)); /* exact scaling; FE_TONEAREST */
    return sign | (f2h((float)ldexp(r, q)) & 0x7FFF); /* representable: exact conversion */
}

/* IEEE binary16 arithmetic as VADDPH / VMULPH / VMINPH / VMAXPH do it */
static uint16_t native(uint16_t in, uint16_t inout, int op) {
    if (op >= 2) { /* MIN/MAX: the second source on NaN or equal zeros */
        const float a = h2f(in), b = h2f(inout);
        if (is_nan16(in) || is_nan16(inout)) return inout;
        if (op == 2) return a < b ? in : inout;
        return a > b ? in : inout;
    }
    if (is_nan16(in)) return in | 0x0200;
    if (is_nan16(inout)) return inout | 0x0200;
    const double a = h2f(in), b = h2f(inout); /* exact */
    const double r = op == 0 ? a + b : a * b;     /* exact: <= 50 significant bits */
    if (isnan(r)) return 0xFE00;                  /* inf - inf, 0 * inf: the default NaN */
    if (isinf(r)) return (signbit(r) ? 0x8000 : 0) | 0x7C00;
    return d2h_rne(r);
}

static int is_snan16(uint16_t h) { return is_nan16(h) && !(h & 0x0200); }

/* The real instructions, where the CPU has AVX512_FP16 (this build container
 * does; gcc 11 lacks the intrinsics, not the assembler): VADDPH / VMULPH /
 * VMINPH / VMAXPH with `in` as the first source, as _mm512_*_ph(in, inout)
 * issue them, 8 lanes at a time. */
static int has_avx512fp16(void) {
    unsigned a, b, c, d;
    __asm__("cpuid" : "=a"(a), "=b"(b), "=c"(c), "=d"(d) : "a"(7), "c"(0));
    return (b >> 30) & 1 && (d >> 23) & 1; /* AVX512BW (xmm forms need VL: bit 31) and AVX512_FP16 */
}

__attribute__((target("avx512f,avx512vl,avx512bw"))) static void hw8(const uint16_t* in, const uint16_t* inout,
                                                                     uint16_t* out, int op) {
    const __m128i a = _mm_loadu_si128((const __m128i*)in), b = _mm_loadu_si128((const __m128i*)inout);
    __m128i r;
    switch (op) {
        case 0: __asm__("vaddph %2, %1, %0" : "=v"(r) : "v"(a), "v"(b)); break;
        case 1: __asm__("vmulph %2, %1, %0" : "=v"(r) : "v"(a), "v"(b)); break;
        case 2: __asm__("vminph %2, %1, %0" : "=v"(r) : "v"(a), "v"(b)); break;
        default: __asm__("vmaxph %2, %1, %0" : "=v"(r) : "v"(a), "v"(b)); break;
    }
    _mm_storeu_si128((__m128i*)out, r);
}
static int g_hw = 0;

/* the oracle's avx512fp16 model, one pair */
static uint16_t oracle_native(uint16_t in, uint16_t inout, int op) {
    uint16_t io = inout;
    (void)orc_comp_reduce(&in, 1, &io, NULL, 8 /* float16 */, op, 0, ORC_FP16_AVX512FP16);
    return io;
}

struct job {
    uint64_t begin, end, stride, checked, bad, expected_bad, oracle_bad, hw_bad;
    int op;
    uint32_t first_bad;
};

static void* run(void* p) {
    struct job* j = p;
    for (uint64_t v = j->begin; v < j->end; v += j->stride) {
        const uint16_t in = (uint16_t)(v >> 16), inout = (uint16_t)v;
        j->checked++;
        const uint16_t nat = native(in, inout, j->op);
        if (route(in, inout, j->op) != nat) {
            /* the one expected difference: min/max with a signalling-NaN inout */
            if (j->op >= 2 && is_snan16(inout)) j->expected_bad++;
            else {
                if (!j->bad) j->first_bad = (uint32_t)v;
                j->bad++;
            }
        }
        if (oracle_native(in, inout, j->op) != nat) j->oracle_bad++;
        if (g_hw) {  /* the model against the instruction itself */
            uint16_t a8[8] = {in}, b8[8] = {inout}, r8[8];
            hw8(a8, b8, r8, j->op);
            if (r8[0] != nat) j->hw_bad++;
        }
    }
    return NULL;
}

int main(int argc, char** argv) {
    const uint64_t stride = argc > 1 ? strtoull(argv[1], NULL, 10) : 1;
    const int nt = argc > 2 ? atoi(argv[2]) : 8;
    __builtin_cpu_init();
    if (!__builtin_cpu_supports("f16c")) {
        printf("{\"skipped\": true, \"reason\": \"no F16C\"}\n");
        return 2;
    }
    const char* names[4] = {"sum", "prod", "min", "max"};
    uint64_t total_bad = 0;
    g_hw = has_avx512fp16();
    printf("{\"stride\": %llu, \"native_model_vs_avx512fp16_hardware\": %s", (unsigned long long)stride,
           g_hw ? "true" : "false");
    for (int op = 0; op < 4; op++) {
        struct job js[64];
        pthread_t th[64];
        const int n = nt < 1 ? 1 : (nt > 64 ? 64 : nt);
        const uint64_t span = (1ull << 32) / (uint64_t)n;
        for (int t = 0; t < n; t++) {
            uint64_t b = span * (uint64_t)t;
            b += (stride - b % stride) % stride; /* one stride grid across the threads */
            js[t] = (struct job){b, t == n - 1 ? (1ull << 32) : span * (uint64_t)(t + 1), stride, 0, 0, 0, 0, 0, op, 0};
            pthread_create(&th[t], NULL, run, &js[t]);
        }
        uint64_t checked = 0, bad = 0, expected = 0, obad = 0, hbad = 0;
        uint32_t first = 0;
        for (int t = 0; t < n; t++) {
            pthread_join(th[t], NULL);
            checked += js[t].checked;
            if (js[t].bad && !bad) first = js[t].first_bad;
            bad += js[t].bad;
            expected += js[t].expected_bad;
            obad += js[t].oracle_bad;
            hbad += js[t].hw_bad;
        }
        total_bad += bad + obad + hbad;
        printf(", \"%s_checked\": %llu, \"%s_route_vs_native_unexplained\": %llu, "
               "\"%s_route_vs_native_snan_inout\": %llu, \"%s_oracle_vs_native\": %llu",
               names[op], (unsigned long long)checked, names[op], (unsigned long long)bad, names[op],
               (unsigned long long)expected, names[op], (unsigned long long)obad);
        if (g_hw) printf(", \"%s_hardware_vs_native\": %llu", names[op], (unsigned long long)hbad);
        if (bad) printf(", \"%s_first_bad_in_inout\": \"0x%08x\"", names[op], first);
    }
    printf("}\n");
    return total_bad ? 1 : 0;
}
