/* svd_lanes_proto.c -- CPU model of the lane-parallel Jacobi SVD solve of tf_icp_tail.h
 * (icp_cv_solve_svd6_lanes): the cyclic sweeps of JacobiSVDImpl_<float> re-ordered by data
 * dependence into levels of up to three disjoint rotations, sweep s+1 started while sweep s
 * finishes, each rotation's (c, s) by the branch-free closed form, and the fast-path of
 * the (c, s) chain with its rounding-margin check (approximate reciprocal square root /
 * reciprocal modelled by a perturbation of up to 2^-APPROX_BITS).  Checked bit for bit against
 * the oracle's serial restatement (oracle/tf_oracle.c, tfo_cv_solve_svd6) on captured ICP
 * systems and on random ones.
 *
 *   gcc -O2 -ffp-contract=off tools/svd_lanes_proto.c -Loracle -loracle -lm -o tools/_build/svd_proto
 *   LD_LIBRARY_PATH=oracle tools/_build/svd_proto tools/_build/svd_systems_C2.f32
 *
 * Test infrastructure (tools/): models the kernel's schedule; the product never runs it. */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

void tfo_cv_solve_svd6(const float A[36], const float b[6], float x[6]);
double tfo_cv_hypot(double x, double y);
void tfo_set_pose_algebra(int mode, int use_libm);

#ifndef APPROX_BITS
#define APPROX_BITS 22
#endif

/* the level table: per level, partner of each row (-1 idle) and whether the pair is sweep s
   (the tail) rather than sweep s + 1 (the head) */
static const int PARTNER[6][6] = {
    { 1, 0, 5, 4, 3, 2 },      /* L0: (0,1)h (2,5)t (3,4)t */
    { 2, -1, 0, 5, -1, 3 },    /* L1: (0,2)h (3,5)t */
    { 3, 2, 1, 0, 5, 4 },      /* L2: (0,3)h (1,2)h (4,5)t */
    { 4, 3, -1, 1, 0, -1 },    /* L3: (0,4)h (1,3)h */
    { 5, 4, 3, 2, 1, 0 },      /* L4: (0,5)h (1,4)h (2,3)h */
    { -1, 5, 4, -1, 2, 1 },    /* L5: (1,5)h (2,4)h */
};
static int is_tail(int L, int i, int j)
{
    if (L == 0) return (i == 2 && j == 5) || (i == 3 && j == 4);
    if (L == 1) return i == 3 && j == 5;
    if (L == 2) return i == 4 && j == 5;
    return 0;
}

static uint64_t g_rng = 0x243F6A8885A308D3ull;
static double approx(double exact)        /* exact * (1 + d), |d| <= 2^-APPROX_BITS */
{
    g_rng = g_rng * 6364136223846793005ull + 1442695040888963407ull;
    const double u = (double)(g_rng >> 11) * (1.0 / 9007199254740992.0) * 2.0 - 1.0;
    return exact * (1.0 + u * ldexp(1.0, -APPROX_BITS));
}
static double rsq_a(double x) { return approx(1.0 / sqrt(x)); }
static double rcp_a(double x) { return approx(1.0 / x); }

/* RN_f(v) equals RN_f(t) for every t within relative E of v?  The 29 bits below a float's
   mantissa must stay clear of the midpoint pattern by more than E's worth of double ulps, and
   the result must be a normal float. */
#define MARGIN_ULPS (1u << 16)             /* relative 2^-37 of a mantissa in [1, 2) */
static int safe_f(double v)
{
    uint64_t b;
    memcpy(&b, &v, 8);
    const unsigned low = (unsigned)b & 0x1fffffffu;
    const unsigned d = low > 0x10000000u ? low - 0x10000000u : 0x10000000u - low;
    const int ex = (int)((b >> 52) & 0x7ff) - 1023;
    return d > MARGIN_ULPS && ex >= -125 && ex <= 126;
}

static uint64_t g_rng_c;
static long long g_fast, g_fallback, g_levels, g_solves;

/* (c, s) of one rotation from p (already doubled), a, b: the serial form (beta < 0 branch and
   all), exactly as the oracle */
static void cs_exact(double p, double a, double b, float* c, float* s)
{
    const double beta = a - b, gamma = tfo_cv_hypot(p, beta);
    if (beta < 0) {
        const double delta = (gamma - beta) * 0.5;
        *s = (float)sqrt(delta / gamma);
        *c = (float)(p / (gamma * *s * 2));
    } else {
        *c = (float)sqrt((gamma + beta) / (gamma * 2));
        *s = (float)(p / (gamma * *c * 2));
    }
}
/* the fast path: approximations with a margin check; falls back to the exact form */
static void cs_fast(double p, double a, double b, float* c, float* s)
{
    const double beta = a - b;
    const double X = fma(p, p, beta * beta);
    const double y = rsq_a(X);
    const double e = fma(-(X * y), y, 1.0);
    const double h = fma(0.25 * y, e, 0.5 * y);
    const double q = fma(fabs(beta), h, 0.5);
    const double y2 = rsq_a(q);
    double U = q * y2;
    const double h2 = 0.5 * y2, r2 = fma(-U, h2, 0.5);
    U = fma(U, r2, U);
    const double z0 = 2.0 * fma(h2, r2, h2);
    const float u = (float)U;
    const double ud = u;
    const double z = fma(fma(-ud, z0, 1.0), z0, z0);
    const double V = (p * h) * z;
    const float v = (float)V;
    if (!(safe_f(U) && safe_f(V))) {
        ++g_fallback;
        cs_exact(p, a, b, c, s);
        return;
    }
    ++g_fast;
    if (beta < 0) { *c = v; *s = u; } else { *c = u; *s = v; }
}

/* the rotation test without its square root (icp_sv_test): p^2 against 2^-44 ab with a 2^-40
   band, the exact test inside it */
static long long g_test_exact;
static int test_fast(double p, double ab)
{
    const double p2 = p * p, t = ab * 5.684341886080802e-14;
    const int skip = p2 <= t * (1.0 - 9.094947017729282e-13);
    const int rot = !skip && p2 >= t * (1.0 + 9.094947017729282e-13);
    if (!skip && !rot) { ++g_test_exact; return !(fabs(p) <= (double)(FLT_EPSILON * 2) * sqrt(ab)); }
    return rot;
}

/* the lane-parallel form's arithmetic (per element exactly the serial operations) */
static void solve_levels(const float A[36], const float bv[6], float x[6], int fast)
{
    float At[6][6], Vt[6][6];
    double W[6];
    for (int i = 0; i < 6; ++i) {
        double sd = 0;
        for (int k = 0; k < 6; ++k) { At[i][k] = A[k * 6 + i]; sd += (double)At[i][k] * At[i][k]; }
        W[i] = sd;
        for (int k = 0; k < 6; ++k) Vt[i][k] = i == k ? 1.f : 0.f;
    }
    const float eps = FLT_EPSILON * 2;
    int changed_tail = 0, changed_head = 0;
    ++g_solves;
    for (int s = -1; s < 30; ++s) {          /* period: tail sweep s, head sweep s + 1 */
        const int head_on = s + 1 < 30;
        for (int L = 0; L < 6; ++L) {
            ++g_levels;
            for (int i = 0; i < 6; ++i) {
                const int j = PARTNER[L][i];
                if (j < i) continue;           /* idle, or the upper row of its pair */
                const int tail = is_tail(L, i, j);
                if (tail ? s < 0 : !head_on) continue;
                double a = W[i], p = 0, b = W[j];
                for (int k = 0; k < 6; k++) p += (double)At[i][k] * At[j][k];
                if (fast ? !test_fast(p, a * b) : fabs(p) <= eps * sqrt(a * b)) continue;
                p *= 2;
                float c, sn;
                if (fast) cs_fast(p, a, b, &c, &sn); else cs_exact(p, a, b, &c, &sn);
                a = b = 0;
                for (int k = 0; k < 6; k++) {
                    const float t0 = c * At[i][k] + sn * At[j][k];
                    const float t1 = -sn * At[i][k] + c * At[j][k];
                    At[i][k] = t0; At[j][k] = t1;
                    a += (double)t0 * t0; b += (double)t1 * t1;
                }
                W[i] = a; W[j] = b;
                for (int k = 0; k < 6; k++) {
                    const float t0 = Vt[i][k] * c + Vt[j][k] * sn;
                    const float t1 = Vt[j][k] * c - Vt[i][k] * sn;
                    Vt[i][k] = t0; Vt[j][k] = t1;
                }
                if (tail) changed_tail = 1; else changed_head = 1;
            }
            if (L == 2 && s >= 0) {            /* sweep s complete */
                if (!changed_tail || s == 29) goto done;
            }
        }
        changed_tail = changed_head;           /* sweep s + 1 becomes the tail */
        changed_head = 0;
    }
done:;
    /* the rest: as the serial form (tfo_cv_jacobi_svd after the sweeps, SVBkSb) */
    for (int i = 0; i < 6; i++) {
        double sd = 0;
        for (int k = 0; k < 6; k++) sd += (double)At[i][k] * At[i][k];
        W[i] = sqrt(sd);
    }
    for (int i = 0; i < 5; i++) {
        int j = i;
        for (int k = i + 1; k < 6; k++) if (W[j] < W[k]) j = k;
        if (i != j) {
            double t = W[i]; W[i] = W[j]; W[j] = t;
            for (int k = 0; k < 6; k++) { float u = At[i][k]; At[i][k] = At[j][k]; At[j][k] = u; }
            for (int k = 0; k < 6; k++) { float u = Vt[i][k]; Vt[i][k] = Vt[j][k]; Vt[j][k] = u; }
        }
    }
    float w[6];
    for (int i = 0; i < 6; i++) w[i] = (float)W[i];
    for (int i = 0; i < 6; i++) {
        double sd = W[i];
        if (i == 0) g_rng_c = 0x12345678;      /* (one generator per solve, as the serial form) */
        for (int ii = 0; ii < 100 && sd <= FLT_MIN; ii++) {   /* a zero singular value: random completion */
            const float val0 = (float)(1. / 6);
            for (int k = 0; k < 6; k++) {
                g_rng_c = (uint64_t)(unsigned)g_rng_c * 4164903690u + (unsigned)(g_rng_c >> 32);
                At[i][k] = ((unsigned)g_rng_c & 256) != 0 ? val0 : -val0;
            }
            for (int it = 0; it < 2; it++)
                for (int j = 0; j < i; j++) {
                    sd = 0;
                    for (int k = 0; k < 6; k++) sd += At[i][k] * At[j][k];
                    float asum = 0;
                    for (int k = 0; k < 6; k++) {
                        const float t = (float)(At[i][k] - sd * At[j][k]);
                        At[i][k] = t;
                        asum += fabsf(t);
                    }
                    asum = asum > eps * 100 ? 1 / asum : 0;
                    for (int k = 0; k < 6; k++) At[i][k] *= asum;
                }
            sd = 0;
            for (int k = 0; k < 6; k++) { const float t = At[i][k]; sd += (double)t * t; }
            sd = sqrt(sd);
        }
        const float sc = (float)(sd > FLT_MIN ? 1 / sd : 0.);
        for (int k = 0; k < 6; k++) At[i][k] *= sc;
    }
    double threshold = 0;
    for (int i = 0; i < 6; i++) threshold += w[i];
    threshold *= (float)(DBL_EPSILON * 2);
    for (int j = 0; j < 6; j++) x[j] = 0;
    for (int i = 0; i < 6; i++) {
        double wi = w[i];
        if ((double)fabs(wi) <= threshold) continue;
        wi = 1 / wi;
        double sacc = 0;
        for (int j = 0; j < 6; j++) sacc += At[i][j] * bv[j];
        sacc *= wi;
        for (int j = 0; j < 6; j++) x[j] = (float)(x[j] + sacc * Vt[i][j]);
    }
}

static void unpack(const float* sm, float A[36], float b[6])
{
    int shift = 0;
    for (int i = 0; i < 6; ++i)
        for (int j = i; j < 7; ++j) {
            const float v = sm[shift++];
            if (j == 6) b[i] = v; else A[j * 6 + i] = A[i * 6 + j] = v;
        }
}

int main(int argc, char** argv)
{
    tfo_set_pose_algebra(4, 0);
    long long n = 0, bad[2] = { 0, 0 };
    float* sys = NULL;
    if (argc > 1) {
        FILE* f = fopen(argv[1], "rb");
        if (!f) { perror(argv[1]); return 2; }
        fseek(f, 0, SEEK_END);
        n = ftell(f) / (27 * 4);
        fseek(f, 0, SEEK_SET);
        sys = malloc(n * 27 * 4);
        if (fread(sys, 4, n * 27, f) != (size_t)(n * 27)) return 2;
        fclose(f);
    }
    const long long nrand = 200000;
    uint64_t st = 12345;
    for (long long q = 0; q < n + nrand; ++q) {
        float sm[27], A[36], b[6], x0[6], x1[6], x2[6];
        if (q < n) memcpy(sm, sys + 27 * q, sizeof(sm));
        else {            /* random ICP-like systems: sums of outer products of 7-vectors */
            memset(sm, 0, sizeof(sm));
            const int rows = 7 + (int)(q % 60);
            for (int r = 0; r < rows; ++r) {
                float v[7];
                for (int k = 0; k < 7; ++k) {
                    st = st * 6364136223846793005ull + 1442695040888963407ull;
                    v[k] = ((float)(st >> 40) / 16777216.0f - 0.5f) * (k < 3 ? 2.f : (k == 6 ? 0.02f : 1.f));
                }
                int s2 = 0;
                for (int a = 0; a < 6; ++a) for (int c = a; c < 7; ++c) sm[s2++] += v[a] * v[c];
            }
        }
        unpack(sm, A, b);
        tfo_cv_solve_svd6(A, b, x0);
        solve_levels(A, b, x1, 0);
        solve_levels(A, b, x2, 1);
        if (memcmp(x0, x1, sizeof(x0))) { if (bad[0]++ < 5) printf("levels/exact differs on system %lld\n", q); }
        if (memcmp(x0, x2, sizeof(x0))) { if (bad[1]++ < 5) printf("levels/fast differs on system %lld\n", q); }
    }
    printf("systems: %lld captured + %lld random; differing: levels-exact %lld, levels-fast %lld\n", n, nrand, bad[0], bad[1]);
    printf("fast-path rotations %lld, fallbacks %lld (%.2e); exact rotation tests %lld; levels per solve %.2f\n", g_fast,
           g_fallback, (double)g_fallback / (double)(g_fast + g_fallback), g_test_exact, (double)g_levels / (double)g_solves);
    return bad[0] || bad[1];
}
