/* Offline check behind tf_div_exact3 (tf_internal.h) for the running-average divisors of the
 * TSDF update (w = 1..257) and a few truncation distances mu: q0 = x * RN(1/d),
 * q = fma(-fma(q0, d, -x), RN(1/d), q0) against x / d for every mantissa of the binade [1, 2),
 * both signs.  Scaling x by 2^k scales every step exactly, so one binade covers every binade
 * whose intermediates stay normal (the kernel sends |x| < 2^-100 to the division itself).
 *   gcc -O2 -ffp-contract=off tools/check_div_consts.c -lm && ./a.out [d_lo d_hi]   (0 = exact) */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static long check(float d)
{
    const float r = 1.0f / d;
    long bad = 0;
    for (uint32_t m = 0; m < (1u << 23); ++m) {
        const uint32_t bits = 0x3f800000u | m;
        float x;
        memcpy(&x, &bits, 4);
        for (int s = 0; s < 2; ++s) {
            const float xx = s ? -x : x;
            const float q0 = xx * r;
            const float q = fmaf(-fmaf(q0, d, -xx), r, q0);
            const float ref = xx / d;
            if (memcmp(&q, &ref, 4)) ++bad;
        }
    }
    return bad;
}

int main(int argc, char** argv)
{
    const int lo = argc > 2 ? atoi(argv[1]) : 1, hi = argc > 2 ? atoi(argv[2]) : 257;
    int fail = 0;
    for (int d = lo; d <= hi; ++d) {
        const long b = check((float)d);
        if (b) { printf("w=%d: %ld mismatches\n", d, b); ++fail; }
    }
    const float mus[] = { 0.01f, 0.02f, 0.03f, 0.05f, 0.1f };
    for (int i = 0; i < 5; ++i) {
        const long b = check(mus[i]);
        if (b) { printf("mu=%g: %ld mismatches\n", mus[i], b); ++fail; }
    }
    printf("divisors %d..%d and 5 mu values: %d inexact\n", lo, hi, fail);
    return fail != 0;
}
