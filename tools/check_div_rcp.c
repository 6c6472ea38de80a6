/* Markstein's correction with a correctly rounded reciprocal, as tf_div_rcp uses it
 * (topfusion_amd/csrc/tf_internal.h): y = RN(1/z), q0 = RN(n*y), q = RN(q0 + RN(n - z*q0)*y)
 * by fma equals RN(n/z) for operands in tf_div_rcp_ok's range.  The device supplies y by a
 * Newton step from v_rcp_f32 and checks that step at tf_create (k_check_rcp); this program checks
 * the quotient step on the host's IEEE arithmetic, which is the same arithmetic (fma, mul):
 *   (1) every mantissa of n in [1, 2) against NZ divisors z spread over the admitted range,
 *   (2) NR random (n, z) pairs over the whole admitted range.
 * gcc -O2 -ffp-contract=off -fopenmp tools/check_div_rcp.c -lm -o /tmp/check_div_rcp */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
static inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float qdiv(float n, float z, float y) { float q0 = n * y; return fmaf(fmaf(-z, q0, n), y, q0); }
static uint64_t mix(uint64_t x) { x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; return x ^ (x >> 33); }
int main(void)
{
    long bad = 0;
    const int NZ = 512;
#pragma omp parallel for reduction(+:bad) schedule(dynamic)
    for (int k = 0; k < NZ; ++k) {
        uint64_t h = mix(0x1234567ull + k);
        uint32_t zb = (uint32_t)(h & 0x7fffffu);
        if (zb == 0x7fffffu) zb = 0;
        int ze = (int)((h >> 23) % 81) - 40;                    /* z in [2^-40, 2^40] */
        float z = ldexpf(u2f(0x3f800000u | zb), ze);
        float y = 1.0f / z;
        for (uint32_t m = 0; m < (1u << 23); ++m) {
            for (int s = 0; s < 2; ++s) {
                float n = u2f((s ? 0xbf800000u : 0x3f800000u) | m);
                if (f2u(qdiv(n, z, y)) != f2u(n / z)) ++bad;
            }
        }
    }
    printf("exhaustive n mantissas x %d divisors: %ld mismatches\n", NZ, bad);
    long bad2 = 0;
    const long NR = 2000000000L;
#pragma omp parallel for reduction(+:bad2)
    for (long i = 0; i < NR; ++i) {
        uint64_t h = mix((uint64_t)i * 0x9e3779b97f4a7c15ull);
        uint32_t zb = (uint32_t)(h & 0x7fffffu), nb = (uint32_t)((h >> 23) & 0x7fffffu);
        if (zb == 0x7fffffu) continue;
        int ze = (int)((h >> 46) % 81) - 40, ne = (int)((h >> 53) % 81) - 40;
        float z = ldexpf(u2f(0x3f800000u | zb), ze);
        float n = ldexpf(u2f(0x3f800000u | nb), ne);
        if (h >> 63) n = -n;
        if (f2u(qdiv(n, z, 1.0f / z)) != f2u(n / z)) ++bad2;
    }
    printf("random pairs: %ld of %ld mismatches\n", bad2, NR);
    return (bad || bad2) ? 1 : 0;
}
