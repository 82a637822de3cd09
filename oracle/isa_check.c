/*
 * isa_check.c — TEST INFRASTRUCTURE ONLY.
 *
 * Pins the oracle's restated x86 semantics (comp_oracle.c) against the real
 * instructions that oneCCL's src/comp calls, on CPUs that have them:
 *   VCVTNEPS2BF16  (_mm512_cvtneps_pbh,  src/comp/bf16/bf16_intrisics.hpp:72-76)
 *   VCVTPS2PH imm0 (_mm512_cvtps_ph,     src/comp/fp16/fp16_intrisics.hpp:131)
 *   VCVTPH2PS      (_mm512_cvtph_ps,     src/comp/fp16/fp16_intrisics.hpp:128)
 *   VMINPS/VMAXPS  (_mm512_min/max_ps,   src/comp/bf16/bf16_intrisics.cpp:28-34)
 * Usage: isa_check [stride]   (stride over the 2^32 fp32 bit patterns; 1 =
 * exhaustive).  Prints one JSON line; exit 0 = all match, 1 = mismatch,
 * 2 = CPU lacks the instructions (skipped).
 */
#include <immintrin.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "comp_oracle.h"

static int has_avx512bf16(void) {
    return __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
           __builtin_cpu_supports("avx512bf16");
}

__attribute__((target("avx512f,avx512bw,avx512vl,avx512bf16"))) static uint64_t
check_bf16(uint64_t stride, uint64_t* checked) {
    uint64_t bad = 0, n = 0;
    uint32_t buf[16];
    uint16_t out[16];
    for (uint64_t base = 0; base < (1ull << 32); base += 16 * stride) {
        for (int l = 0; l < 16; l++) buf[l] = (uint32_t)(base + (uint64_t)l * stride);
        __m512 v = _mm512_loadu_ps((const float*)buf);
        _mm256_storeu_si256((__m256i*)out, (__m256i)_mm512_cvtneps_pbh(v));
        for (int l = 0; l < 16; l++) {
            float f;
            memcpy(&f, &buf[l], 4);
            if (out[l] != orc_fp32_to_bf16_rne(f)) {
                if (bad < 5)
                    fprintf(stderr, "bf16 rne mismatch %08x: hw %04x oracle %04x\n", buf[l],
                            out[l], orc_fp32_to_bf16_rne(f));
                bad++;
            }
            n++;
        }
    }
    *checked = n;
    return bad;
}

__attribute__((target("avx512f,avx512bw,avx512vl,f16c"))) static uint64_t
check_fp16(uint64_t stride, uint64_t* checked) {
    uint64_t bad = 0, n = 0;
    uint32_t buf[16];
    uint16_t out[16];
    for (uint64_t base = 0; base < (1ull << 32); base += 16 * stride) {
        for (int l = 0; l < 16; l++) buf[l] = (uint32_t)(base + (uint64_t)l * stride);
        __m512 v = _mm512_loadu_ps((const float*)buf);
        _mm256_storeu_si256((__m256i*)out, _mm512_cvtps_ph(v, 0));
        for (int l = 0; l < 16; l++) {
            float f;
            memcpy(&f, &buf[l], 4);
            if (out[l] != orc_fp32_to_fp16_rne(f)) {
                if (bad < 5)
                    fprintf(stderr, "fp16 rne mismatch %08x: hw %04x oracle %04x\n", buf[l],
                            out[l], orc_fp32_to_fp16_rne(f));
                bad++;
            }
            n++;
        }
    }
    /* all 65536 halves widened */
    for (uint32_t h = 0; h < 65536; h += 16) {
        uint16_t hin[16];
        float hw[16];
        for (int l = 0; l < 16; l++) hin[l] = (uint16_t)(h + l);
        _mm512_storeu_ps(hw, _mm512_cvtph_ps(_mm256_loadu_si256((const __m256i*)hin)));
        for (int l = 0; l < 16; l++) {
            float o = orc_fp16_to_fp32(hin[l]);
            if (memcmp(&o, &hw[l], 4) != 0) {
                if (bad < 5) fprintf(stderr, "fp16->fp32 mismatch %04x\n", hin[l]);
                bad++;
            }
            n++;
        }
    }
    *checked = n;
    return bad;
}

/* min/max operand order: the oracle's bf16 avx512 path must equal
 * _mm512_min_ps(in, inout) / _mm512_max_ps(in, inout) bit for bit. */
__attribute__((target("avx512f,avx512bw,avx512vl"))) static uint64_t check_minmax(
    uint64_t* checked) {
    static const uint32_t specials[] = {0x00000000u, 0x80000000u, 0x3F800000u, 0xBF800000u,
                                        0x7F800000u, 0xFF800000u, 0x7FC00000u, 0xFFC00000u,
                                        0x7FA00000u, 0x00010000u, 0x80010000u, 0x40490000u,
                                        0x7F7F0000u, 0xFF7F0000u, 0x3F810000u, 0x00800000u};
    const int ns = (int)(sizeof(specials) / sizeof(specials[0]));
    uint64_t bad = 0, n = 0;
    for (int op = 2; op <= 3; op++) {
        for (int i = 0; i < ns; i++) {
            for (int j = 0; j < ns; j++) {
                /* values are bf16-representable, so the bf16 path's widening is
                 * exact and its truncation is the identity on the selected
                 * operand */
                uint16_t in = (uint16_t)(specials[i] >> 16), io = (uint16_t)(specials[j] >> 16);
                uint16_t got = io;
                orc_comp_reduce(&in, 1, &got, NULL, 11 /*bf16*/, op, ORC_BF16_AVX512F, 0);
                float fin, fio, r[16];
                memcpy(&fin, &specials[i], 4);
                memcpy(&fio, &specials[j], 4);
                __m512 a = _mm512_set1_ps(fin), b = _mm512_set1_ps(fio);
                _mm512_storeu_ps(r, op == 2 ? _mm512_min_ps(a, b) : _mm512_max_ps(a, b));
                uint32_t ru;
                memcpy(&ru, &r[0], 4);
                if ((uint16_t)(ru >> 16) != got) {
                    if (bad < 5)
                        fprintf(stderr, "minmax op%d %08x,%08x: hw %08x oracle %04x\n", op,
                                specials[i], specials[j], ru, got);
                    bad++;
                }
                n++;
            }
        }
    }
    *checked = n;
    return bad;
}

int main(int argc, char** argv) {
    uint64_t stride = (argc > 1) ? strtoull(argv[1], NULL, 10) : 1;
    if (stride == 0) stride = 1;
    if (!has_avx512bf16() || !__builtin_cpu_supports("f16c")) {
        printf("{\"skipped\": true, \"reason\": \"cpu lacks avx512bf16/f16c\"}\n");
        return 2;
    }
    uint64_t n1 = 0, n2 = 0, n3 = 0;
    uint64_t b1 = check_bf16(stride, &n1);
    uint64_t b2 = check_fp16(stride, &n2);
    uint64_t b3 = check_minmax(&n3);
    printf("{\"skipped\": false, \"stride\": %llu, \"bf16_rne_checked\": %llu, "
           "\"bf16_rne_bad\": %llu, \"fp16_checked\": %llu, \"fp16_bad\": %llu, "
           "\"minmax_checked\": %llu, \"minmax_bad\": %llu}\n",
           (unsigned long long)stride, (unsigned long long)n1, (unsigned long long)b1,
           (unsigned long long)n2, (unsigned long long)b2, (unsigned long long)n3,
           (unsigned long long)b3);
    return (b1 || b2 || b3) ? 1 : 0;
}
