/*
 * selftest.c — TEST INFRASTRUCTURE ONLY.  Exercises every oracle entry point
 * on odd sizes and checks internal consistency; built with
 * -fsanitize=address,undefined by `make -C oracle asan` and run by
 * tests/test_oracle.py so the restatement's memory handling and integer
 * arithmetic are sanitizer-clean.  Exit 0 = pass.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "comp_oracle.h"

static unsigned long long rng = 0x9E3779B97F4A7C15ull;
static unsigned long long next(void) {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return rng;
}

static const size_t ES[12] = {1, 1, 2, 2, 4, 4, 8, 8, 2, 4, 8, 2};

int main(void) {
    int fails = 0;
    const size_t sizes[] = {0, 1, 15, 16, 17, 63, 64, 65, 1000, 4099};
    for (size_t si = 0; si < sizeof(sizes) / sizeof(sizes[0]); si++) {
        const size_t n = sizes[si];
        for (int dt = 0; dt < 12; dt++) {
            for (int op = 0; op < 4; op++) {
                for (int impl = 0; impl < 3; impl++) {
                    const size_t bytes = n * ES[dt];
                    unsigned char* a = malloc(bytes + 1);
                    unsigned char* b = malloc(bytes + 1);
                    unsigned char* c = malloc(bytes + 1);
                    for (size_t i = 0; i < bytes; i++) {
                        a[i] = (unsigned char)next();
                        b[i] = (unsigned char)next();
                    }
                    memcpy(c, b, bytes);
                    size_t oc = 0;
                    if (orc_comp_reduce(a, n, b, &oc, dt, op, impl, 3 + (impl % 2))) fails++;
                    /* multi-thread split must equal the single-thread result */
                    if (orc_comp_reduce_mt(a, n, c, dt, op, impl, 3 + (impl % 2), 3)) fails++;
                    if (memcmp(b, c, bytes)) {
                        fprintf(stderr, "mt mismatch dt=%d op=%d n=%zu\n", dt, op, n);
                        fails++;
                    }
                    free(a);
                    free(b);
                    free(c);
                }
            }
        }
        /* batch reduce, both modes, bf16 and fp32 */
        for (int keep = 0; keep < 2; keep++) {
            const size_t k = 5;
            unsigned short* packed = malloc(k * n * 2 + 2);
            unsigned short* io = malloc(n * 2 + 2);
            float* tmp = malloc(n * 4 + 4);
            float* acc = malloc(n * 4 + 4);
            size_t offs[5];
            for (size_t j = 0; j < k; j++) offs[j] = j * n;
            for (size_t i = 0; i < k * n; i++) packed[i] = (unsigned short)next();
            memcpy(io, packed, n * 2);
            if (orc_comp_batch_reduce(packed, offs, k, n, io, NULL, 11, 0, keep, tmp, acc, 2, 3)) fails++;
            free(packed);
            free(io);
            free(tmp);
            free(acc);
        }
        /* conversions round trip: bf16 -> fp32 -> bf16 is the identity except NaN quieting */
        {
            unsigned short* h = malloc(n * 2 + 2);
            unsigned short* h2 = malloc(n * 2 + 2);
            float* f = malloc(n * 4 + 4);
            for (size_t i = 0; i < n; i++) h[i] = (unsigned short)(next() & 0x7F7F);
            orc_convert_bf16_to_fp32_arrays(h, f, n);
            orc_convert_fp32_to_bf16_arrays(f, h2, n, 0);
            if (n && memcmp(h, h2, n * 2)) fails++;
            orc_convert_fp32_to_fp16_arrays(f, h2, n);
            free(h);
            free(h2);
            free(f);
        }
        /* fan-in with fp32 accumulate */
        {
            const void* ins[4];
            unsigned short* bufs[4];
            for (int j = 0; j < 4; j++) {
                bufs[j] = malloc(n * 2 + 2);
                for (size_t i = 0; i < n; i++) bufs[j][i] = (unsigned short)(next() & 0x3FFF);
                ins[j] = bufs[j];
            }
            unsigned short* out = malloc(n * 2 + 2);
            if (orc_lp_fanin_acc_fp32(ins, 4, out, n, 8, 0, 1, 1)) fails++;
            if (orc_lp_fanin_acc_fp32(ins, 4, out, n, 11, 3, 0, 0)) fails++;
            for (int j = 0; j < 4; j++) free(bufs[j]);
            free(out);
        }
    }
    if (orc_comp_reduce(NULL, 0, NULL, NULL, 12, 0, 0, 0) != -1) fails++;  /* unknown dtype */
    printf("selftest: %s (%d failures)\n", fails ? "FAIL" : "ok", fails);
    return fails ? 1 : 0;
}
