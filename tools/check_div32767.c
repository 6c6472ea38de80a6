/* Exhaustive check of the 3-operation division by 32767 used by the raycasting kernels
 * (tf_internal.h: tf_div32767): q0 = x * RN(1/32767), e = fma(q0, 32767, -x),
 * q = fma(-e, RN(1/32767), q0) against the IEEE quotient x / 32767.0f.
 *   gcc -O2 -ffp-contract=off tools/check_div32767.c -lm && ./a.out [lo_bits hi_bits]
 * Default: every float with |x| < 2^21 (bit patterns 0 .. 0x4a000000), both signs -- about two
 * minutes on one core; prints the number of mismatches (0). */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int main(int argc, char** argv)
{
    uint32_t lo = 0, hi = 0x4a000000u;
    if (argc == 3) { lo = (uint32_t)strtoul(argv[1], 0, 0); hi = (uint32_t)strtoul(argv[2], 0, 0); }
    const float r = 1.0f / 32767.0f;
    long bad = 0, tot = 0;
    for (uint32_t bits = lo; bits < hi; ++bits) {
        float x;
        memcpy(&x, &bits, 4);
        for (int sgn = 0; sgn < 2; ++sgn) {
            const float xx = sgn ? -x : x;
            const float q0 = xx * r;
            const float e = fmaf(q0, 32767.0f, -xx);
            const float q = fmaf(-e, r, q0);
            const float ref = xx / 32767.0f;
            if (memcmp(&q, &ref, 4)) {
                if (bad < 5) printf("mismatch x=%a q=%a ref=%a\n", xx, q, ref);
                ++bad;
            }
            ++tot;
        }
    }
    printf("checked %ld values, %ld mismatches\n", tot, bad);
    return bad != 0;
}
