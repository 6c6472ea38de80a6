// tf_icp_tail.h -- the serial tail of an ICP iteration (projective_icp.cpp:197-215): the
// cv::determinant check, the cv::solve replacement and Affine3f(rvec, t)'s Rodrigues, as
// register-resident device functions shared by tf_icp.hip and tools/micro/icp_tail.hip.
#pragma once
#include "tf_internal.h"

// fixed-polynomial sin/cos (replaces std::sin/cos inside cv::Affine3's Rodrigues).  The
// coefficients are compile-time immediates and the Horner loop is fully unrolled: the serial
// ICP tail waits on this chain, and a __constant__ table costs one dependent scalar load per
// term.
__device__ __forceinline__ void icp_sincos(double th, double* s, double* c)
{
    constexpr double inv_sin[14] = { 0.0, 1.0/6.0, 1.0/20.0, 1.0/42.0, 1.0/72.0, 1.0/110.0, 1.0/156.0,
        1.0/210.0, 1.0/272.0, 1.0/342.0, 1.0/420.0, 1.0/506.0, 1.0/600.0, 1.0/702.0 };
    constexpr double inv_cos[14] = { 0.0, 1.0/2.0, 1.0/12.0, 1.0/30.0, 1.0/56.0, 1.0/90.0, 1.0/132.0,
        1.0/182.0, 1.0/240.0, 1.0/306.0, 1.0/380.0, 1.0/462.0, 1.0/552.0, 1.0/650.0 };
    const double PI = 3.14159265358979323846;
    const double TWO_PI = 6.28318530717958647692;
    double r = th;
    if (r > PI || r < -PI) {
        double k = rint(r / TWO_PI);
        r = r - k * TWO_PI;
    }
    double r2 = r * r;
    double ps = 1.0, pc = 1.0;
    if (r2 < 0.015625) {                // |r| < 1/8: 6 terms, first omitted term < 2^-80 relative
#pragma unroll
        for (int n = 6; n >= 1; --n) {
            ps = 1.0 - (r2 * inv_sin[n]) * ps;
            pc = 1.0 - (r2 * inv_cos[n]) * pc;
        }
    } else {
#pragma unroll
        for (int n = 13; n >= 1; --n) {
            ps = 1.0 - (r2 * inv_sin[n]) * ps;
            pc = 1.0 - (r2 * inv_cos[n]) * pc;
        }
    }
    *s = r * ps;
    *c = pc;
}

// Affine3f(rvec, t) rotation (Rodrigues in double).  Sinc form (default): R = cos t I +
// ((1 - cos t) / t^2) r r^T + (sin t / t) [r]x with r = rvec unnormalised and the three even
// functions of t = |rvec| as nested polynomials in t^2 evaluated with fma -- no square root and
// no division on the iteration's serial path, three short independent chains (the sqrt / divide /
// two-chain form it replaces was ~40 dependent f64 operations, 0.9 us of every ICP iteration;
// the CPU restatement computes the same).  t > pi (never for an ICP
// increment) takes that form.  TF_RODRIGUES_SINC=0: the old form throughout (A/B).
#ifndef TF_SOLVE_LDL
#define TF_SOLVE_LDL 0
#endif
#ifndef TF_RODRIGUES_SINC
#define TF_RODRIGUES_SINC 1
#endif
__device__ __forceinline__ void icp_rodrigues_sqrt(const float* rv, float* R);
__device__ __forceinline__ void icp_rodrigues(const float* rv, float* R)
{
#if TF_RODRIGUES_SINC
    constexpr double inv_sin[14] = { 0.0, 1.0/6.0, 1.0/20.0, 1.0/42.0, 1.0/72.0, 1.0/110.0, 1.0/156.0,
        1.0/210.0, 1.0/272.0, 1.0/342.0, 1.0/420.0, 1.0/506.0, 1.0/600.0, 1.0/702.0 };
    constexpr double inv_cos[15] = { 0.0, 1.0/2.0, 1.0/12.0, 1.0/30.0, 1.0/56.0, 1.0/90.0, 1.0/132.0,
        1.0/182.0, 1.0/240.0, 1.0/306.0, 1.0/380.0, 1.0/462.0, 1.0/552.0, 1.0/650.0, 1.0/756.0 };
    const double rx = rv[0], ry = rv[1], rz = rv[2];
    const double t2 = (rx * rx + ry * ry) + rz * rz;
    if (t2 < 4.930380657631324e-32) {             // t < DBL_EPSILON
        for (int k = 0; k < 9; ++k) R[k] = (k % 4 == 0) ? 1.0f : 0.0f;
        return;
    }
    if (t2 > 9.869604401089358) { icp_rodrigues_sqrt(rv, R); return; }   // t > pi
    double pc = 1.0, pa = 1.0, pb = 1.0;          // cos t, sin t / t, 2 (1 - cos t) / t^2
    if (t2 < 0.000244140625) {                    // t < 1/64: 4 terms (first omitted < 2^-60 relative)
#pragma unroll
        for (int n = 4; n >= 1; --n) {
            pc = fma(-(t2 * inv_cos[n]), pc, 1.0);
            pa = fma(-(t2 * inv_sin[n]), pa, 1.0);
            pb = fma(-(t2 * inv_cos[n + 1]), pb, 1.0);
        }
    } else if (t2 < 0.015625) {                   // t < 1/8: 6 terms (first omitted < 2^-80 relative)
#pragma unroll
        for (int n = 6; n >= 1; --n) {
            pc = fma(-(t2 * inv_cos[n]), pc, 1.0);
            pa = fma(-(t2 * inv_sin[n]), pa, 1.0);
            pb = fma(-(t2 * inv_cos[n + 1]), pb, 1.0);
        }
    } else {
#pragma unroll
        for (int n = 13; n >= 1; --n) {
            pc = fma(-(t2 * inv_cos[n]), pc, 1.0);
            pa = fma(-(t2 * inv_sin[n]), pa, 1.0);
            pb = fma(-(t2 * inv_cos[n + 1]), pb, 1.0);
        }
    }
    const double b = 0.5 * pb;
    const double rrt[9] = { rx * rx, rx * ry, rx * rz, rx * ry, ry * ry, ry * rz, rx * rz, ry * rz, rz * rz };
    const double rxm[9] = { 0, -rz, ry, rz, 0, -rx, -ry, rx, 0 };
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        const double I = (k % 4 == 0) ? 1.0 : 0.0;
        R[k] = (float)((pc * I + b * rrt[k]) + pa * rxm[k]);
    }
#else
    icp_rodrigues_sqrt(rv, R);
#endif
}

// the sqrt / sincos / divide form (t > pi, or TF_RODRIGUES_SINC=0)
__device__ __forceinline__ void icp_rodrigues_sqrt(const float* rv, float* R)
{
    double rx = rv[0], ry = rv[1], rz = rv[2];
    double theta = sqrt((rx * rx + ry * ry) + rz * rz);
    if (theta < 2.220446049250313e-16) {
        for (int k = 0; k < 9; ++k) R[k] = (k % 4 == 0) ? 1.0f : 0.0f;
        return;
    }
    double s, c;
    icp_sincos(theta, &s, &c);
    double c1 = 1.0 - c;
    double itheta = 1.0 / theta;
    rx *= itheta; ry *= itheta; rz *= itheta;
    double rrt[9] = { rx * rx, rx * ry, rx * rz, rx * ry, ry * ry, ry * rz, rx * rz, ry * rz, rz * rz };
    double rxm[9] = { 0, -rz, ry, rz, 0, -rx, -ry, rx, 0 };
    for (int k = 0; k < 9; ++k) {
        double I = (k % 4 == 0) ? 1.0 : 0.0;
        R[k] = (float)((c * I + c1 * rrt[k]) + s * rxm[k]);
    }
}

// ---- 6x6 algebra, register resident: every lane runs the same fully unrolled code on
// uniform data (static indices only; pivot rows selected by uniform branches) ------------------
// cv::determinant(Matx66f): LU with partial pivoting in float (eps 10*FLT_EPSILON), pivot
// product in double -- the operations of the serial LU (see oracle/tf_oracle.c:cv_det6)
__device__ __forceinline__ double icp_det6_reg(const float (&A0)[6][6])
{
    float A[6][6];
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = 0; j < 6; ++j) A[i][j] = A0[i][j];
    const float eps = 1.19209290e-07f * 10;
    int p = 1;
#pragma unroll
    for (int i = 0; i < 6; i++) {
        float best = fabsf(A[i][i]);
        int k = i;
#pragma unroll
        for (int j = i + 1; j < 6; j++) { float v = fabsf(A[j][i]); if (v > best) { best = v; k = j; } }
        k = __builtin_amdgcn_readfirstlane(k);          // uniform: swaps become scalar branches
        if (best < eps) return 0.0;
        if (k != i) {
#pragma unroll
            for (int r = i + 1; r < 6; ++r)
                if (r == k) {
#pragma unroll
                    for (int c = i; c < 6; ++c) { float t = A[i][c]; A[i][c] = A[r][c]; A[r][c] = t; }
                }
            p = -p;
        }
        float d = -1 / A[i][i];
#pragma unroll
        for (int j = i + 1; j < 6; j++) {
            float alpha = A[j][i] * d;
#pragma unroll
            for (int c = i + 1; c < 6; c++) A[j][c] += alpha * A[i][c];
        }
    }
    double det = p;
#pragma unroll
    for (int i = 0; i < 6; i++) det *= A[i][i];
    return det;
}

// cv::solve(A, b, DECOMP_SVD) replacement, the canonical form (oracle/tf_oracle.c:solve6, same
// operations in the same order): 2 x 2 block elimination in double with closed-form 3 x 3 inverses,
// A = [P Q; Q^T R], T = Q adj(R) / det R, S = P - T Q^T, x1 = adj(S) (b1 - T b2) / det S,
// x2 = adj(R) (b2 - Q^T x1) / det R.  The serial tail waits on this chain: two 3 x 3 determinants
// and two divisions deep (~35 dependent operations) against ~110 for the column-by-column LDL^T
// below, and x1, which Rodrigues needs, comes before x2.
__device__ __forceinline__ void icp_sym3_adj(const double (&M)[3][3], double (&C)[3][3], double& det)
{
    C[0][0] = M[1][1] * M[2][2] - M[1][2] * M[2][1];
    C[0][1] = M[0][2] * M[2][1] - M[0][1] * M[2][2];
    C[0][2] = M[0][1] * M[1][2] - M[0][2] * M[1][1];
    C[1][0] = M[1][2] * M[2][0] - M[1][0] * M[2][2];
    C[1][1] = M[0][0] * M[2][2] - M[0][2] * M[2][0];
    C[1][2] = M[0][2] * M[1][0] - M[0][0] * M[1][2];
    C[2][0] = M[1][0] * M[2][1] - M[1][1] * M[2][0];
    C[2][1] = M[0][1] * M[2][0] - M[0][0] * M[2][1];
    C[2][2] = M[0][0] * M[1][1] - M[0][1] * M[1][0];
    det = (M[0][0] * C[0][0] + M[0][1] * C[1][0]) + M[0][2] * C[2][0];
}

__device__ __forceinline__ void icp_solve6_schur(const float (&Af)[6][6], const float (&bf)[6], float (&x)[6])
{
    double P[3][3], Q[3][3], R[3][3], b1[3], b2[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            P[i][j] = Af[i][j];
            Q[i][j] = Af[i][3 + j];
            R[i][j] = Af[3 + i][3 + j];
        }
        b1[i] = bf[i];
        b2[i] = bf[3 + i];
    }
    double aR[3][3], dR, aS[3][3], dS, T[3][3], S[3][3], c[3], x1[3], e[3];
    icp_sym3_adj(R, aR, dR);
    const double rR = 1.0 / dR;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
            T[i][j] = ((Q[i][0] * aR[0][j] + Q[i][1] * aR[1][j]) + Q[i][2] * aR[2][j]) * rR;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
#pragma unroll
        for (int j = 0; j < 3; ++j)
            S[i][j] = P[i][j] - ((T[i][0] * Q[j][0] + T[i][1] * Q[j][1]) + T[i][2] * Q[j][2]);
        c[i] = b1[i] - ((T[i][0] * b2[0] + T[i][1] * b2[1]) + T[i][2] * b2[2]);
    }
    icp_sym3_adj(S, aS, dS);
    const double rS = 1.0 / dS;
#pragma unroll
    for (int i = 0; i < 3; ++i) x1[i] = ((aS[i][0] * c[0] + aS[i][1] * c[1]) + aS[i][2] * c[2]) * rS;
#pragma unroll
    for (int i = 0; i < 3; ++i) e[i] = b2[i] - ((Q[0][i] * x1[0] + Q[1][i] * x1[1]) + Q[2][i] * x1[2]);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        x[i] = (float)x1[i];
        x[3 + i] = (float)(((aR[i][0] * e[0] + aR[i][1] * e[1]) + aR[i][2] * e[2]) * rR);
    }
}

// the previous canonical form (rounds 2-4), kept for tools/micro/icp_tail.hip:
// LDL^T of the symmetric normal matrix in double with one reciprocal per pivot, then forward,
// diagonal and backward substitution -- ~270 uniform operations with short dependency chains
// (the pivoting elimination it replaces issued ~2.5x as many, 21 of them full divisions)
__device__ __forceinline__ void icp_solve6_ldl(const float (&Af)[6][6], const float (&bf)[6], float (&x)[6])
{
    double L[6][6], d[6], r[6], y[6], xs[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        double w[6];
#pragma unroll
        for (int k = 0; k < j; ++k) w[k] = L[j][k] * d[k];
        double dj = Af[j][j];
#pragma unroll
        for (int k = 0; k < j; ++k) dj = dj - L[j][k] * w[k];
        d[j] = dj;
        r[j] = 1.0 / dj;
#pragma unroll
        for (int i = j + 1; i < 6; ++i) {
            double sacc = Af[i][j];
#pragma unroll
            for (int k = 0; k < j; ++k) sacc = sacc - L[i][k] * w[k];
            L[i][j] = sacc * r[j];
        }
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        double sacc = bf[i];
#pragma unroll
        for (int k = 0; k < i; ++k) sacc = sacc - L[i][k] * y[k];
        y[i] = sacc;
    }
#pragma unroll
    for (int i = 5; i >= 0; --i) {
        double sacc = y[i] * r[i];
#pragma unroll
        for (int k = i + 1; k < 6; ++k) sacc = sacc - L[k][i] * xs[k];
        xs[i] = sacc;
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) x[i] = (float)xs[i];
}


// =============================================================================================
// The reference's own pose algebra: OpenCV's cv::determinant(Matx66f), cv::solve(A, b, r,
// DECOMP_SVD) and cv::Affine3f(rvec, t) (projective_icp.cpp:197-209; OpenCV >= 2.4.9,
// CMakeLists.txt:18), selected per context (tf_set_pose_algebra / TFUSION_ICP_SOLVE).  The
// operations of the oracle's OpenCV 2.4.9 / 3.x-4.x pose-algebra mode (oracle/tf_oracle.c) with its portable
// transcendental functions (icp_sincos, icp_cv_hypot), in the same order: bit for bit the
// oracle's.  ALG 2: OpenCV 2.4.9 (LU pivot floor FLT_EPSILON, norm(Vec3f) in double); ALG 4:
// OpenCV 3.x / 4.x (10 FLT_EPSILON, norm in float).  One wave evaluates it on uniform data, like
// the LDL^T solve; every register array is indexed statically (rotations are template-unrolled).
// =============================================================================================
constexpr float TF_FLT_EPS = 1.19209290e-07f;
constexpr double TF_FLT_MIN = 1.17549435e-38;

// readlane of a double / float (uniform result)
__device__ __forceinline__ double icp_rl_d(double v, int src)
{
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, src);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), src);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ float icp_rl_f(float v, int src)
{
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), src));
}

// hypot (the oracle's portable hypot): fma-corrected sum of squares
__device__ __forceinline__ double icp_cv_hypot(double x, double y)
{
    x = fabs(x); y = fabs(y);
    if (x < y) { const double t = x; x = y; y = t; }
    if (y == 0.0) return x;
    const double h = sqrt(fma(x, x, y * y));
    const double h_sq = h * h, x_sq = x * x;
    const double e = (fma(-y, y, h_sq - x_sq) + fma(h, h, -h_sq)) - fma(x, x, -x_sq);
    return h - e / (2.0 * h);
}

// cv::determinant(Matx66f) = Matx_DetOp<float, 6>: LU (reciprocal pivots left on the diagonal),
// det = 1 / (p * prod); ALG 0: the canonical form (icp_det6_reg)
template <int ALG>
__device__ __forceinline__ double icp_det6(const float (&A0)[6][6])
{
    if constexpr (ALG == 0) {
        return icp_det6_reg(A0);
    } else {
        float A[6][6];
#pragma unroll
        for (int i = 0; i < 6; ++i)
#pragma unroll
            for (int j = 0; j < 6; ++j) A[i][j] = A0[i][j];
        const float eps = ALG == 2 ? TF_FLT_EPS : TF_FLT_EPS * 10;
        int p = 1;
#pragma unroll
        for (int i = 0; i < 6; i++) {
            float best = fabsf(A[i][i]);
            int k = i;
#pragma unroll
            for (int j = i + 1; j < 6; j++) { float v = fabsf(A[j][i]); if (v > best) { best = v; k = j; } }
            k = __builtin_amdgcn_readfirstlane(k);
            if (best < eps) return 0.0;
            if (k != i) {
#pragma unroll
                for (int r = i + 1; r < 6; ++r)
                    if (r == k) {
#pragma unroll
                        for (int c = i; c < 6; ++c) { float t = A[i][c]; A[i][c] = A[r][c]; A[r][c] = t; }
                    }
                p = -p;
            }
            const float d = -1 / A[i][i];
#pragma unroll
            for (int j = i + 1; j < 6; j++) {
                const float alpha = A[j][i] * d;
#pragma unroll
                for (int c = i + 1; c < 6; c++) A[j][c] += alpha * A[i][c];
            }
            A[i][i] = -d;
        }
        double det = p;
#pragma unroll
        for (int i = 0; i < 6; i++) det *= A[i][i];
        return 1. / det;
    }
}

// one rotation (I, J) of JacobiSVDImpl_<float> (lapack.cpp): true if it rotated
template <int I, int J>
__device__ __forceinline__ bool icp_cv_rot(float (&At)[6][6], float (&Vt)[6][6], double (&W)[6])
{
    constexpr float eps = TF_FLT_EPS * 2;
    double a = W[I], p = 0, b = W[J];
#pragma unroll
    for (int k = 0; k < 6; k++) p += (double)At[I][k] * At[J][k];
    if (fabs(p) <= (double)eps * sqrt(a * b)) return false;
    p *= 2;
    const double beta = a - b, gamma = icp_cv_hypot(p, beta);
    float c, s;
    if (beta < 0) {
        const double delta = (gamma - beta) * 0.5;
        s = (float)sqrt(delta / gamma);
        c = (float)(p / (gamma * s * 2));
    } else {
        c = (float)sqrt((gamma + beta) / (gamma * 2));
        s = (float)(p / (gamma * c * 2));
    }
    a = b = 0;
#pragma unroll
    for (int k = 0; k < 6; k++) {
        const float t0 = c * At[I][k] + s * At[J][k];
        const float t1 = -s * At[I][k] + c * At[J][k];
        At[I][k] = t0; At[J][k] = t1;
        a += (double)t0 * t0; b += (double)t1 * t1;
    }
    W[I] = a; W[J] = b;
#pragma unroll
    for (int k = 0; k < 6; k++) {                 // VBLAS<float>::givens
        const float t0 = Vt[I][k] * c + Vt[J][k] * s;
        const float t1 = Vt[J][k] * c - Vt[I][k] * s;
        Vt[I][k] = t0; Vt[J][k] = t1;
    }
    return true;
}

// cv::RNG::next (multiply-with-carry, CV_RNG_COEFF 4164903690)
__device__ __forceinline__ unsigned icp_cv_rng(unsigned long long& st)
{
    st = (unsigned long long)(unsigned)st * 4164903690ull + (unsigned)(st >> 32);
    return (unsigned)st;
}

// What follows JacobiSVDImpl_<float>'s sweeps: W = |row| sorted descending (rows of At and Vt
// with it), a zero singular value completed at random, the rows of At normalised; then
// SVBkSbImpl_<float>(6, 6, w, u = At (uT), v = Vt (vT), b, nb = 1).  Shared by the serial solve
// below and the lane-parallel one's zero-singular-value path.  The completion is bounded at 100
// draws and a row still zero after them is scaled by 0, as OpenCV 3.x / 4.x write it
// (`ii < 100 && sd <= minval`, `sd > minval ? 1/sd : 0`); 2.4.9 writes an unbounded loop and 1/sd,
// which differ only where 2.4.9 would not terminate.
template <int ALG>
__device__ __forceinline__ void icp_cv_svd_finish(float (&At)[6][6], float (&Vt)[6][6], const float (&bv)[6], float (&x)[6]);

// cv::solve(A, b, x, DECOMP_SVD) for a float 6x6 and one right-hand side (lapack.cpp): the work
// matrix transpose(A), JacobiSVDImpl_<float>(m = n = 6, eps 2 FLT_EPSILON, minval FLT_MIN), then
// SVBkSbImpl_<float> with threshold (sum w) * (float)(2 DBL_EPSILON)
template <int ALG>
__device__ __forceinline__ void icp_cv_solve_svd6(const float (&A)[6][6], const float (&bv)[6], float (&x)[6])
{
    float At[6][6], Vt[6][6];
    double W[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        double sd = 0;
#pragma unroll
        for (int k = 0; k < 6; ++k) { At[i][k] = A[k][i]; sd += (double)At[i][k] * At[i][k]; }
        W[i] = sd;
#pragma unroll
        for (int k = 0; k < 6; ++k) Vt[i][k] = i == k ? 1.f : 0.f;
    }
#pragma unroll 1
    for (int iter = 0; iter < 30; iter++) {        // max_iter = max(m, 30)
        bool ch = false;
        ch |= icp_cv_rot<0, 1>(At, Vt, W); ch |= icp_cv_rot<0, 2>(At, Vt, W); ch |= icp_cv_rot<0, 3>(At, Vt, W);
        ch |= icp_cv_rot<0, 4>(At, Vt, W); ch |= icp_cv_rot<0, 5>(At, Vt, W); ch |= icp_cv_rot<1, 2>(At, Vt, W);
        ch |= icp_cv_rot<1, 3>(At, Vt, W); ch |= icp_cv_rot<1, 4>(At, Vt, W); ch |= icp_cv_rot<1, 5>(At, Vt, W);
        ch |= icp_cv_rot<2, 3>(At, Vt, W); ch |= icp_cv_rot<2, 4>(At, Vt, W); ch |= icp_cv_rot<2, 5>(At, Vt, W);
        ch |= icp_cv_rot<3, 4>(At, Vt, W); ch |= icp_cv_rot<3, 5>(At, Vt, W); ch |= icp_cv_rot<4, 5>(At, Vt, W);
        if (!ch) break;
    }
    icp_cv_svd_finish<ALG>(At, Vt, bv, x);
}

template <int ALG>
__device__ __forceinline__ void icp_cv_svd_finish(float (&At)[6][6], float (&Vt)[6][6], const float (&bv)[6], float (&x)[6])
{
    double W[6];
#pragma unroll
    for (int i = 0; i < 6; i++) {
        double sd = 0;
#pragma unroll
        for (int k = 0; k < 6; k++) sd += (double)At[i][k] * At[i][k];
        W[i] = sqrt(sd);
    }
#pragma unroll
    for (int i = 0; i < 5; i++) {                  // selection sort, descending (strict <: first maximum)
        int j = i;
        double wj = W[i];
#pragma unroll
        for (int k = i + 1; k < 6; k++) if (wj < W[k]) { j = k; wj = W[k]; }
        j = __builtin_amdgcn_readfirstlane(j);
        if (j != i) {
#pragma unroll
            for (int r = i + 1; r < 6; ++r)
                if (r == j) {
                    const double t = W[i]; W[i] = W[r]; W[r] = t;
#pragma unroll
                    for (int k = 0; k < 6; k++) { float u = At[i][k]; At[i][k] = At[r][k]; At[r][k] = u; }
#pragma unroll
                    for (int k = 0; k < 6; k++) { float u = Vt[i][k]; Vt[i][k] = Vt[r][k]; Vt[r][k] = u; }
                }
        }
    }
    float w[6];
#pragma unroll
    for (int i = 0; i < 6; i++) w[i] = (float)W[i];
    unsigned long long rng = 0x12345678ull;
#pragma unroll
    for (int i = 0; i < 6; i++) {
        double sd = W[i];
#pragma unroll 1
        for (int ii = 0; ii < 100 && sd <= TF_FLT_MIN; ii++) {   // a zero singular value: random completion
            const float val0 = (float)(1. / 6);
#pragma unroll
            for (int k = 0; k < 6; k++) At[i][k] = (icp_cv_rng(rng) & 256) != 0 ? val0 : -val0;
#pragma unroll
            for (int it2 = 0; it2 < 2; it2++)
#pragma unroll
                for (int j = 0; j < i; j++) {
                    sd = 0;
#pragma unroll
                    for (int k = 0; k < 6; k++) sd += At[i][k] * At[j][k];
                    float asum = 0;
#pragma unroll
                    for (int k = 0; k < 6; k++) {
                        const float t = (float)(At[i][k] - sd * At[j][k]);
                        At[i][k] = t;
                        asum += fabsf(t);
                    }
                    asum = asum > TF_FLT_EPS * 2 * 100 ? 1 / asum : 0;
#pragma unroll
                    for (int k = 0; k < 6; k++) At[i][k] *= asum;
                }
            sd = 0;
#pragma unroll
            for (int k = 0; k < 6; k++) sd += (double)At[i][k] * At[i][k];
            sd = sqrt(sd);
        }
        const float s = (float)(sd > TF_FLT_MIN ? 1 / sd : 0.);
#pragma unroll
        for (int k = 0; k < 6; k++) At[i][k] *= s;
    }
    // SVBkSbImpl_<float>(6, 6, w, u = At (uT), v = Vt (vT), b, nb = 1)
    double threshold = 0;
#pragma unroll
    for (int i = 0; i < 6; i++) threshold += w[i];
    threshold *= (double)(float)(2.220446049250313e-16 * 2);
#pragma unroll
    for (int j = 0; j < 6; j++) x[j] = 0;
#pragma unroll
    for (int i = 0; i < 6; i++) {
        double wi = w[i];
        if ((double)fabs(wi) <= threshold) continue;
        wi = 1 / wi;
        double s = 0;
#pragma unroll
        for (int j = 0; j < 6; j++) s += At[i][j] * bv[j];         // float product, double sum
        s *= wi;
#pragma unroll
        for (int j = 0; j < 6; j++) x[j] = (float)(x[j] + s * Vt[i][j]);
    }
}

// =============================================================================================
// cv::solve(DECOMP_SVD) lane-parallel (round 6; IP_SVD_LANES).  The serial form above runs each
// sweep's 15 rotations one after another on uniform data.  Here one wave holds the work matrix
// one element per lane -- lane l = 8 r + k holds At[r][k], Vt[r][k] and |row r|^2 (rows 6, 7 and
// columns 6, 7 are padding) -- and:
//  * rotations on disjoint row pairs touch disjoint data, so the sweeps run in dependence order:
//    a period of 6 levels of up to three concurrent rotations per sweep, sweep s + 1 starting
//    while sweep s finishes (SV_PART; every row sees its rotations in the serial order, and a
//    sweep that changed nothing is detected after its last rotation, (4, 5), exactly where the
//    serial loop breaks -- the next sweep's rotations already issued then find the data they
//    would have found and rotate nothing);
//  * a rotation's sums (the dot product, the new |row|^2) keep the serial order: the six exact
//    double products reach the row's lane 0 by DPP row_shl and are added there in order;
//  * (c, s) come from a short sequence (v_rsq_f64 / v_rcp_f64 plus one refinement each,
//    icp_sv_cs) whose double results are accepted only when they lie further from a float
//    rounding boundary than the sequence's error bound -- then their float roundings are the
//    exact sequence's -- and otherwise the exact sequence runs (a wave-uniform branch, about 1 in
//    2000 rotations);
//  * sort, normalisation and back substitution lane-parallel (a zero singular value takes the
//    serial finish on the gathered matrices).
// Every element sees the serial form's operations in the same order: the result is
// icp_cv_solve_svd6's bit for bit (tools/micro/svd_lanes.hip; tools/svd_lanes_proto.c models the
// schedule on the CPU against the oracle).
// =============================================================================================
// partner row of each row r (4-bit fields, 15 = idle) in level L of a period, and the rows whose
// pair belongs to sweep s (the period's tail; the others are sweep s + 1's, its head)
constexpr int SV_P[6][8] = {
    { 1, 0, 5, 4, 3, 2, 15, 15 },        // (0,1)h (2,5)t (3,4)t
    { 2, 15, 0, 5, 15, 3, 15, 15 },      // (0,2)h (3,5)t
    { 3, 2, 1, 0, 5, 4, 15, 15 },        // (0,3)h (1,2)h (4,5)t   -- sweep s complete
    { 4, 3, 15, 1, 0, 15, 15, 15 },      // (0,4)h (1,3)h
    { 5, 4, 3, 2, 1, 0, 15, 15 },        // (0,5)h (1,4)h (2,3)h
    { 15, 5, 4, 15, 2, 1, 15, 15 },      // (1,5)h (2,4)h
};
constexpr unsigned SV_TAIL_ROWS[6] = { 0x3cu, 0x28u, 0x30u, 0u, 0u, 0u };
constexpr unsigned sv_pack(int L)
{
    unsigned v = 0;
    for (int r = 0; r < 8; ++r) v |= (unsigned)SV_P[L][r] << (4 * r);
    return v;
}
constexpr unsigned long long sv_row_lanes(unsigned rows)
{
    unsigned long long m = 0;
    for (int r = 0; r < 8; ++r)
        if ((rows >> r) & 1u) m |= 0xffull << (8 * r);
    return m;
}

// lanes of the rows that are the lower row (I) of their pair in level L; lane 0 of each row whose
// pair is enabled (tail pairs when sweep s exists, head pairs when sweep s + 1 does)
constexpr unsigned long long sv_lower_lanes(int L)
{
    unsigned long long m = 0;
    for (int r = 0; r < 6; ++r)
        if (SV_P[L][r] != 15 && r < SV_P[L][r]) m |= 0xffull << (8 * r);
    return m;
}
constexpr unsigned long long sv_act_base(int L, bool tail_on, bool head_on)
{
    unsigned long long m = 0;
    for (int r = 0; r < 6; ++r) {
        const bool tail = ((SV_TAIL_ROWS[L] >> r) & 1u) != 0;
        if (SV_P[L][r] != 15 && (tail ? tail_on : head_on)) m |= 1ull << (8 * r);
    }
    return m;
}
// per lane: bit `lane` of the wave-uniform mask selects t, else f (one v_cndmask_b32)
__device__ __forceinline__ float icp_lsel(unsigned long long mask, float t, float f)
{
    float r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(f), "v"(t), "s"(mask));
    return r;
}
__device__ __forceinline__ double icp_lsel_d(unsigned long long mask, double t, double f)
{
    const unsigned long long ut = __builtin_bit_cast(unsigned long long, t), uf = __builtin_bit_cast(unsigned long long, f);
    const unsigned lo = __builtin_bit_cast(unsigned, icp_lsel(mask, __builtin_bit_cast(float, (unsigned)ut),
                                                              __builtin_bit_cast(float, (unsigned)uf)));
    const unsigned hi = __builtin_bit_cast(unsigned, icp_lsel(mask, __builtin_bit_cast(float, (unsigned)(ut >> 32)),
                                                              __builtin_bit_cast(float, (unsigned)(uf >> 32))));
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
// each set bit at a row's lane 0 spread over the row's 8 lanes
__device__ __forceinline__ unsigned long long icp_sv_spread(unsigned long long m)
{
    m |= m << 1;
    m |= m << 2;
    return m | (m << 4);
}

template <int CTRL>
__device__ __forceinline__ double icp_dpp_d(double v)
{
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = (unsigned)__builtin_amdgcn_mov_dpp((int)(unsigned)u, CTRL, 0xf, 0xf, false);
    const unsigned hi = (unsigned)__builtin_amdgcn_mov_dpp((int)(unsigned)(u >> 32), CTRL, 0xf, 0xf, false);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ float icp_bperm_f(int src_lane, float v)
{
    return __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(src_lane << 2, __builtin_bit_cast(int, v)));
}
__device__ __forceinline__ double icp_bperm_d(int src_lane, double v)
{
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = (unsigned)__builtin_amdgcn_ds_bpermute(src_lane << 2, (int)(unsigned)u);
    const unsigned hi = (unsigned)__builtin_amdgcn_ds_bpermute(src_lane << 2, (int)(unsigned)(u >> 32));
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
// forward permute: this lane's value lands in lane dst_lane (a permutation of the lanes)
__device__ __forceinline__ float icp_fperm_f(int dst_lane, float v)
{
    return __builtin_bit_cast(float, __builtin_amdgcn_ds_permute(dst_lane << 2, __builtin_bit_cast(int, v)));
}
__device__ __forceinline__ double icp_fperm_d(int dst_lane, double v)
{
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = (unsigned)__builtin_amdgcn_ds_permute(dst_lane << 2, (int)(unsigned)u);
    const unsigned hi = (unsigned)__builtin_amdgcn_ds_permute(dst_lane << 2, (int)(unsigned)(u >> 32));
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
// sum over the row's columns k = 0..5 of q, in order (0 + q0 + q1 + ... + q5, as the serial
// loops add), returned to every lane of the row: q1..q5 reach lane 0 of the 8-lane group by DPP
// row_shl (within a 16-lane DPP row both groups' lanes 0 read in range), the sum is broadcast
// back by row_newbcast:0 / :8
__device__ __forceinline__ double icp_sv_rowsum(double q, int lane)
{
    const double q1 = icp_dpp_d<0x101>(q), q2 = icp_dpp_d<0x102>(q), q3 = icp_dpp_d<0x103>(q);
    const double q4 = icp_dpp_d<0x104>(q), q5 = icp_dpp_d<0x105>(q);
    double s = 0.0 + q;
    s = s + q1;
    s = s + q2;
    s = s + q3;
    s = s + q4;
    s = s + q5;
    const double b0 = icp_dpp_d<0x150>(s), b8 = icp_dpp_d<0x158>(s);
    return (lane & 8) ? b8 : b0;
}

// RN_f(t) == RN_f(v) for every t within the fast sequence's error of v?  The 29 bits a float
// drops from a double's mantissa must stay more than SV_MARGIN double ulps (2^-37 of a mantissa
// in [1, 2), relative) from the midpoint pattern (one add and one unsigned compare), and, where
// the value's range does not already guarantee it (full = true), v must be a normal float.
#define SV_MARGIN (1u << 16)
#ifndef SV_WQ_BPERM
#define SV_WQ_BPERM 0          // 1: |partner row|^2 fetched from the partner's lane 0 (A/B: 0.6% slower)
#endif
template <bool full>
__device__ __forceinline__ bool icp_sv_round_safe(double v)
{
    const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
    const bool clear = (((unsigned)b & 0x1fffffffu) - (0x10000000u - SV_MARGIN)) > 2u * SV_MARGIN;
    if constexpr (!full) return clear;
    const unsigned e = (unsigned)(b >> 52) & 0x7ffu;            // biased exponent (sign dropped)
    return clear & (e - (1023u - 125u) <= 251u);                 // 2^-125 <= |v| < 2^127
}
// (c, s) of a rotation, the serial form's sequence (p already doubled, beta = W[I] - W[J])
__device__ __forceinline__ void icp_sv_cs_exact(double p, double beta, float& c, float& s)
{
    const double gamma = icp_cv_hypot(p, beta);
    if (beta < 0) {
        const double delta = (gamma - beta) * 0.5;
        s = (float)sqrt(delta / gamma);
        c = (float)(p / (gamma * s * 2));
    } else {
        c = (float)sqrt((gamma + beta) / (gamma * 2));
        s = (float)(p / (gamma * c * 2));
    }
}
// The same (c, s) by a short sequence.  Both branches of the serial form compute
// u = RN_f(sqrt((gamma + |beta|) / (2 gamma))) and v = RN_f(p / (gamma u 2)), (c, s) = (u, v) or
// (v, u) by the sign of beta, gamma = hypot(p, beta).  Here h ~ 1 / (2 gamma) from v_rsq_f64 and
// one Newton step, q = 1/2 + |beta| h ~ (gamma + |beta|) / (2 gamma), U ~ sqrt(q) from v_rsq_f64
// and one Goldschmidt step (which also refines 1 / (2 U)), 1 / u from that by one Newton step
// on the rounded u, V = p h / u.  v_rsq_f64 is within 2^-24.2 (relative; all inputs checked,
// profiles/r06/f64_approx.txt), so U and V are within ~2^-47 of the exact sequence's doubles,
// 2^10 below the margin icp_sv_round_safe demands: where both pass it, (c, s)
// are the exact sequence's.  Rotating lanes that fail take icp_sv_cs_exact (uniform branch).
__device__ __forceinline__ void icp_sv_cs(double p, double beta, unsigned long long m, float& c, float& s)
{
    const double X = fma(p, p, beta * beta);
    const double y = __builtin_amdgcn_rsq(X);
    const double e = fma(-(X * y), y, 1.0);
    const double h = fma(0.25 * y, e, 0.5 * y);                 // 1 / (2 gamma)
    const double q = fma(fabs(beta), h, 0.5);
    const double y2 = __builtin_amdgcn_rsq(q);
    double U = q * y2;
    const double h2 = 0.5 * y2, r2 = fma(-U, h2, 0.5);
    U = fma(U, r2, U);
    const double z0 = 2.0 * fma(h2, r2, h2);                   // 1 / U
    const float u = (float)U;
    const double ud = u;
    const double z = fma(fma(-ud, z0, 1.0), z0, z0);           // 1 / u
    const double V = (p * h) * z;
    const float v = (float)V;
    const bool neg = beta < 0;
    c = neg ? v : u;
    s = neg ? u : v;
    const unsigned long long bad =
        m & ~__builtin_amdgcn_ballot_w64((int)icp_sv_round_safe<false>(U) & (int)icp_sv_round_safe<true>(V));
    if (__builtin_expect(bad != 0, 0)) {
#ifdef TF_SV_STATS                                // (tools/micro/svd_lanes.hip: levels that fell back)
        if ((threadIdx.x & 63) == 0) atomicAdd(&g_sv_stats[1], 1ull);
#endif
        float ce, se;
        icp_sv_cs_exact(p, beta, ce, se);
        c = icp_lsel(bad, ce, c);
        s = icp_lsel(bad, se, s);
    }
}

// the serial form's rotation test, !(|p| <= eps sqrt(a b)) with eps = 2 FLT_EPSILON = 2^-22, without
// its square root: p^2 against 2^-44 ab (1 -+ 2^-40), decided there unless p^2 falls between the
// two -- then |p| and 2^-22 RN(sqrt(RN(ab))) are within 2^-41 and the exact test runs (a rare
// wave-uniform branch).  p = 0 or ab = 0 decide as the serial test does (skip, unless p != 0 =
// ab); a NaN fails both comparisons and takes the exact test.  act: the lanes that test; the
// result is the mask of those that rotate.
__device__ __forceinline__ unsigned long long icp_sv_test(unsigned long long act, double p, double ab)
{
    const double p2 = p * p;
    const unsigned long long skip = __builtin_amdgcn_ballot_w64(p2 <= ab * 5.6843418860756883e-14);  // 2^-44 (1 - 2^-40)
    const unsigned long long rot = __builtin_amdgcn_ballot_w64(p2 >= ab * 5.6843418860860254e-14);   // 2^-44 (1 + 2^-40)
    unsigned long long m = act & rot & ~skip;
    const unsigned long long unsure = act & ~rot & ~skip;
    if (__builtin_expect(unsure != 0, 0))
        m |= unsure & __builtin_amdgcn_ballot_w64(!(fabs(p) <= (double)(TF_FLT_EPS * 2) * sqrt(ab)));
    return m;
}

template <int CTRL>
__device__ __forceinline__ float icp_dpp_f(float v)
{
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}
// lane 0 of the lane's 8-lane row group (DPP row_newbcast:0 / :8)
__device__ __forceinline__ float icp_row_bcast(float v, int lane)
{
    const float b0 = icp_dpp_f<0x150>(v), b8 = icp_dpp_f<0x158>(v);
    return (lane & 8) ? b8 : b0;
}

#ifdef TF_SV_TIMING                               // (tools/micro/svd_lanes.hip timing build only)
// a stamp after a value: its phase's cycles since the previous stamp accumulate in registers
// (SvTimes), written to g_sv_t at the end of the solve
struct SvTimes { long long t0, acc[8]; };
#define SV_TPARAM , SvTimes& svt
#define SV_TARG , svt
#define SV_T(k, val_) do { const float d_ = (float)(val_); asm volatile("; sv dep %0" :: "v"(d_)); \
    __builtin_amdgcn_sched_barrier(0); const long long t_ = (long long)__builtin_amdgcn_s_memtime(); \
    __builtin_amdgcn_sched_barrier(0); svt.acc[k] += t_ - svt.t0; svt.t0 = t_; } while (0)
#else
#define SV_TPARAM
#define SV_TARG
#define SV_T(k, val_) do { } while (0)
#endif
// The partner row's element by lane swaps (SV_XOR_PARTNER): in every level each row's partner is
// its index XOR one or two masks, and a row-index XOR of 1 / 2 / 4 is a lane XOR of 8 / 16 / 32 --
// DPP row_ror:8, v_permlane16_swap, v_permlane32_swap (+ one v_cndmask each) -- instead of one
// ds_bpermute round trip.  Rows without a partner (and the padding rows) get some other row's
// element; nothing of theirs is used.  A/B (round 6, tools/micro/svd_lanes.hip, bit-exact): 21 708
// against 20 254 cycles per solve -- the swap chains (up to three deep, each with its select) take
// longer than the one round trip; off.
#ifndef SV_XOR_PARTNER
#define SV_XOR_PARTNER 0
#endif
__device__ __forceinline__ float icp_x8(float x) { return icp_dpp_f<0x128>(x); }
__device__ __forceinline__ float icp_x16(float x)
{
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return icp_lsel(0xffff0000ffff0000ull, __uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float icp_x32(float x)
{
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return icp_lsel(0xffffffff00000000ull, __uint_as_float(r[0]), __uint_as_float(r[1]));
}
template <int L>
__device__ __forceinline__ float icp_sv_partner(float x)
{
    // level L's pairs as row-index XOR masks (SV_P): rows of mask A take a, the rest b
    if constexpr (L == 0) {                 // (0,1) ^1; (2,5) (3,4) ^7
        const float a1 = icp_x8(x), a7 = icp_x32(icp_x16(a1));
        return icp_lsel(sv_row_lanes(0x03u), a1, a7);
    } else if constexpr (L == 1) {          // (0,2) ^2; (3,5) ^6
        const float a2 = icp_x16(x), a6 = icp_x32(a2);
        return icp_lsel(sv_row_lanes(0x05u), a2, a6);
    } else if constexpr (L == 2) {          // (0,3) (1,2) ^3; (4,5) ^1
        const float a1 = icp_x8(x), a3 = icp_x16(a1);
        return icp_lsel(sv_row_lanes(0x0fu), a3, a1);
    } else if constexpr (L == 3) {          // (0,4) ^4; (1,3) ^2
        const float a4 = icp_x32(x), a2 = icp_x16(x);
        return icp_lsel(sv_row_lanes(0x11u), a4, a2);
    } else if constexpr (L == 4) {          // (0,5) (1,4) ^5; (2,3) ^1
        const float a1 = icp_x8(x), a5 = icp_x32(a1);
        return icp_lsel(sv_row_lanes(0x33u), a5, a1);
    } else {                                // (1,5) ^4; (2,4) ^6
        const float a4 = icp_x32(x), a6 = icp_x16(a4);
        return icp_lsel(sv_row_lanes(0x22u), a4, a6);
    }
}
// the partner masks above, checked against SV_P at compile time
constexpr bool sv_xor_ok()
{
    const unsigned A[6] = { 0x03u, 0x05u, 0x0fu, 0x11u, 0x33u, 0x22u };
    const int ma[6] = { 1, 2, 3, 4, 5, 4 }, mb[6] = { 7, 6, 1, 2, 1, 6 };
    for (int L = 0; L < 6; ++L)
        for (int r = 0; r < 6; ++r) {
            if (SV_P[L][r] == 15) continue;
            const int m = ((A[L] >> r) & 1u) ? ma[L] : mb[L];
            if ((r ^ m) != SV_P[L][r]) return false;
        }
    return true;
}
static_assert(sv_xor_ok(), "icp_sv_partner: masks must match SV_P");

// one level of a period: every row with a partner in an enabled sweep rotates with it.  Lane 0
// of each row group gathers its row and the partner row (DPP row_shl) and forms the three sums the
// rotation needs in the serial order -- p = sum_k At[I][k] At[J][k] and both |row|^2, exact double
// products added in order (as fma: the products are exact) -- then the test and (c, s); the row's
// lanes apply (c, s) to their element.  src: the lane holding this lane's element of the partner
// row (own lane when the row is idle); which pairs are enabled is a template argument.
template <int L, bool TAIL_ON, bool HEAD_ON>
__device__ __forceinline__ void icp_sv_level(float& a, float& v, int lane, int src, bool& ch_tail, bool& ch_head SV_TPARAM)
{
    constexpr unsigned long long ACT = sv_act_base(L, TAIL_ON, HEAD_ON);
    constexpr unsigned long long LOW = sv_lower_lanes(L);
    constexpr unsigned long long TL = sv_row_lanes(SV_TAIL_ROWS[L]);
    if constexpr (ACT == 0) return;
    SV_T(0, a);
#if SV_XOR_PARTNER
    const float xa = icp_sv_partner<L>(a), xv = icp_sv_partner<L>(v);
    (void)src;
#else
    const float xa = icp_bperm_f(src, a), xv = icp_bperm_f(src, v);
#endif
    const float a1 = icp_dpp_f<0x101>(a), a2 = icp_dpp_f<0x102>(a), a3 = icp_dpp_f<0x103>(a);
    const float a4 = icp_dpp_f<0x104>(a), a5 = icp_dpp_f<0x105>(a);
    const double d0 = a, d1 = a1, d2 = a2, d3 = a3, d4 = a4, d5 = a5;
    double wo = fma(d0, d0, 0.0);
    wo = fma(d1, d1, wo); wo = fma(d2, d2, wo); wo = fma(d3, d3, wo); wo = fma(d4, d4, wo); wo = fma(d5, d5, wo);
    SV_T(1, xa);
    const float x1 = icp_dpp_f<0x101>(xa), x2 = icp_dpp_f<0x102>(xa), x3 = icp_dpp_f<0x103>(xa);
    const float x4 = icp_dpp_f<0x104>(xa), x5 = icp_dpp_f<0x105>(xa);
    const double e0 = xa, e1 = x1, e2 = x2, e3 = x3, e4 = x4, e5 = x5;
#if SV_WQ_BPERM
    // |partner row|^2: the partner row's lane 0 formed it (its wo), fetched while p is summed
    const double wq = icp_bperm_d(src & ~7, wo);
    double p = fma(d0, e0, 0.0);
    p = fma(d1, e1, p); p = fma(d2, e2, p); p = fma(d3, e3, p); p = fma(d4, e4, p); p = fma(d5, e5, p);
#else
    double wq = fma(e0, e0, 0.0), p = fma(d0, e0, 0.0);
    wq = fma(e1, e1, wq); p = fma(d1, e1, p);
    wq = fma(e2, e2, wq); p = fma(d2, e2, p);
    wq = fma(e3, e3, wq); p = fma(d3, e3, p);
    wq = fma(e4, e4, wq); p = fma(d4, e4, p);
    wq = fma(e5, e5, wq); p = fma(d5, e5, p);
#endif
    SV_T(2, p + wo + wq);
    // beta = W[I] - W[J] on both rows' lanes (RN(y - x) = -RN(x - y)); ab = W[I] W[J]
    const double dw = wo - wq;
    const double beta = icp_lsel_d(LOW, dw, -dw);
    const unsigned long long m = icp_sv_test(ACT, p, wo * wq);      // bits at the rotating rows' lanes 0
    SV_T(3, (float)m);
    if (m != 0) {                                               // (uniform: otherwise nothing changes)
        float c, s;
        icp_sv_cs(p * 2, beta, m, c, s);
        SV_T(4, c + s);
        const float cb = icp_row_bcast(c, lane), sb = icp_row_bcast(s, lane);
        // row I: c Ai + s Aj, Vi c + Vj s;  row J: -s Ai + c Aj, Vj c - Vi s (the same products and
        // one addition each: a + b == b + a and x - y == x + (-y) bit for bit)
        const float sc = icp_lsel(LOW, sb, -sb);
        const float na = cb * a + sc * xa;
        const float nv = v * cb + xv * sc;
        const unsigned long long mr = icp_sv_spread(m);
        a = icp_lsel(mr, na, a);
        v = icp_lsel(mr, nv, v);
        SV_T(5, a + v);
    }
#ifdef TF_SV_STATS                                // (tools/micro/svd_lanes.hip: rotations)
    if (lane == 0) atomicAdd(&g_sv_stats[0], (unsigned long long)__builtin_popcountll(m) / 2);
#endif
    ch_tail = ch_tail || (m & TL) != 0;
    ch_head = ch_head || (m & ~TL) != 0;
}

// tot: lane stride * q holds sum q of the system (StreamHelper layout, projective_icp.cpp:51-61);
// x: the solution, uniform
template <int ALG>
__device__ __forceinline__ void icp_cv_solve_svd6_lanes(float tot, int stride, int lane, float (&x)[6])
{
    const int r = lane >> 3, k = lane & 7;
    const bool valid = r < 6 && k < 6;
    // At = transpose(A) = A (symmetric): element (r, k) is sum idx(min, max), idx(i, j) =
    // i (15 - i) / 2 + j - i; b[k] = sum idx(k, 6)
    const int lo = r < k ? r : k, hi = r < k ? k : r;
    const int ia = valid ? ((lo * (15 - lo)) >> 1) + hi - lo : 0;
    const int kb = k < 6 ? k : 0;
    float a = icp_bperm_f(ia * stride, tot);
    const float bk = icp_bperm_f((((kb * (15 - kb)) >> 1) + 6 - kb) * stride, tot);
    if (!valid) a = 0.f;
    float v = (valid && r == k) ? 1.f : 0.f;
    // partner lane of this lane's element in each level (own lane on an idle row)
    int src[6];
#pragma unroll
    for (int L = 0; L < 6; ++L) {
        const int P = (int)((sv_pack(L) >> (4 * r)) & 15u);
        src[L] = P != 15 ? 8 * P + k : lane;
    }
    bool ch_tail = false, ch_head = false;
#ifdef TF_SV_TIMING
    SvTimes svt = {};
    svt.t0 = (long long)__builtin_amdgcn_s_memtime();
#endif
    // period -1: sweep 0's first levels (no tail)
    icp_sv_level<0, false, true>(a, v, lane, src[0], ch_tail, ch_head SV_TARG);
    icp_sv_level<1, false, true>(a, v, lane, src[1], ch_tail, ch_head SV_TARG);
    icp_sv_level<2, false, true>(a, v, lane, src[2], ch_tail, ch_head SV_TARG);
    icp_sv_level<3, false, true>(a, v, lane, src[3], ch_tail, ch_head SV_TARG);
    icp_sv_level<4, false, true>(a, v, lane, src[4], ch_tail, ch_head SV_TARG);
    icp_sv_level<5, false, true>(a, v, lane, src[5], ch_tail, ch_head SV_TARG);
    ch_tail = ch_head;
    ch_head = false;
    bool done = false;
#pragma unroll 1
    for (int sw = 0; sw < 29; ++sw) {           // period sw: tail sweep sw, head sweep sw + 1
        icp_sv_level<0, true, true>(a, v, lane, src[0], ch_tail, ch_head SV_TARG);
        icp_sv_level<1, true, true>(a, v, lane, src[1], ch_tail, ch_head SV_TARG);
        icp_sv_level<2, true, true>(a, v, lane, src[2], ch_tail, ch_head SV_TARG);
        if (!ch_tail) { done = true; break; }   // sweep sw changed nothing: the serial loop's exit
        icp_sv_level<3, true, true>(a, v, lane, src[3], ch_tail, ch_head SV_TARG);
        icp_sv_level<4, true, true>(a, v, lane, src[4], ch_tail, ch_head SV_TARG);
        icp_sv_level<5, true, true>(a, v, lane, src[5], ch_tail, ch_head SV_TARG);
        ch_tail = ch_head;
        ch_head = false;
    }
    if (!done) {                                // sweep 29, the last (max_iter = 30): its tail only
        icp_sv_level<0, true, false>(a, v, lane, src[0], ch_tail, ch_head SV_TARG);
        icp_sv_level<1, true, false>(a, v, lane, src[1], ch_tail, ch_head SV_TARG);
        icp_sv_level<2, true, false>(a, v, lane, src[2], ch_tail, ch_head SV_TARG);
    }
    // ---- singular values, sorted descending (selection sort, strict <: the first maximum)
    const double Wf = sqrt(icp_sv_rowsum((double)a * (double)a, lane));
    if (__builtin_amdgcn_ballot_w64((r < 6) & (k == 0) & (Wf <= TF_FLT_MIN)) != 0) {
        // a zero singular value: the serial finish (random completion) on the gathered matrices
#ifdef TF_SV_STATS
        if (lane == 0) atomicAdd(&g_sv_stats[2], 1ull);
#endif
        float At[6][6], Vt[6][6], bu[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) {
#pragma unroll
            for (int j = 0; j < 6; ++j) { At[i][j] = icp_rl_f(a, 8 * i + j); Vt[i][j] = icp_rl_f(v, 8 * i + j); }
            bu[i] = icp_rl_f(bk, i);
        }
        icp_cv_svd_finish<ALG>(At, Vt, bu, x);
        return;
    }
    double Wu[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) Wu[i] = icp_rl_d(Wf, 8 * i);
    // Six distinct values: the selection sort's result is the descending order, so row r goes to
    // position #{j : W_j > W_r} -- counted on every lane of the row, moved by one forward permute.
    // Equal values (or a NaN) leave the order to the selection sort's swaps: run it (uniform).
    int rank = 0, eq = 0;
#pragma unroll
    for (int j = 0; j < 6; ++j) { rank += Wu[j] > Wf ? 1 : 0; eq += Wu[j] == Wf ? 1 : 0; }
    float as, vs;
    double sd, Ws[6];
    if (__builtin_expect(__builtin_amdgcn_ballot_w64((r < 6) & (eq != 1)) == 0, 1)) {
        const int dst = r < 6 ? 8 * rank + k : lane;
        as = icp_fperm_f(dst, a);
        vs = icp_fperm_f(dst, v);
        sd = icp_fperm_d(dst, Wf);                // W[r] after the sort
#pragma unroll
        for (int i = 0; i < 6; ++i) Ws[i] = icp_rl_d(sd, 8 * i);
    } else {
        unsigned perm = 0x543210u;                // sorted position i <- row (perm >> 4 i) & 15
#pragma unroll
        for (int i = 0; i < 5; i++) {
            int j = i;
            double wj = Wu[i];
#pragma unroll
            for (int kk = i + 1; kk < 6; kk++) if (wj < Wu[kk]) { j = kk; wj = Wu[kk]; }
            j = __builtin_amdgcn_readfirstlane(j);
            if (j != i) {
#pragma unroll
                for (int rr = i + 1; rr < 6; ++rr)
                    if (rr == j) {
                        const double t = Wu[i]; Wu[i] = Wu[rr]; Wu[rr] = t;
                        const unsigned pi = (perm >> (4 * i)) & 15u, pr = (perm >> (4 * rr)) & 15u;
                        perm = (perm & ~((15u << (4 * i)) | (15u << (4 * rr)))) | (pr << (4 * i)) | (pi << (4 * rr));
                    }
            }
        }
        const int sl = r < 6 ? 8 * (int)((perm >> (4 * r)) & 15u) + k : lane;
        as = icp_bperm_f(sl, a);
        vs = icp_bperm_f(sl, v);
        sd = icp_bperm_d(sl, Wf);
#pragma unroll
        for (int i = 0; i < 6; ++i) Ws[i] = Wu[i];
    }
    SV_T(6, as + vs + sd);
    // the row normalised: RN_f(1 / sd) from v_rcp_f64 and one Newton step (within 2^-48) where that
    // double is clear of a float rounding boundary, else the IEEE division
    {
        const double r0 = __builtin_amdgcn_rcp(sd);
        const double rq = fma(fma(-sd, r0, 1.0), r0, r0);
        float scl = (float)rq;
        const bool exact = icp_sv_round_safe<true>(rq);
        if (__builtin_amdgcn_ballot_w64(!exact) != 0) {
            if (!exact) scl = (float)(1 / sd);
        }
        as *= scl;
    }
    // ---- SVBkSbImpl_<float>: threshold = (sum of the float w[i], in order) * (float)(2 DBL_EPSILON)
    double thr = 0;
#pragma unroll
    for (int i = 0; i < 6; ++i) thr += (float)Ws[i];
    thr *= (double)(float)(2.220446049250313e-16 * 2);
    const float wfl = (float)sd;
    const bool live = !((double)fabs(wfl) <= thr);
    double si = icp_sv_rowsum((double)(as * bk), lane);   // float products, double sum in order
    double wi = wfl;
    wi = 1 / wi;
    si *= wi;
    const double term = si * (double)vs;          // s * Vt[i][j]
    const unsigned long long lm = __builtin_amdgcn_ballot_w64(live && k == 0);
    double ti[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) ti[i] = icp_bperm_d(8 * i + k, term);
    float xj = 0.f;                               // lane (0, j): x[j] over the rows in order
#pragma unroll
    for (int i = 0; i < 6; ++i)
        if ((lm >> (8 * i)) & 1ull) xj = (float)((double)xj + ti[i]);
#pragma unroll
    for (int j = 0; j < 6; ++j) x[j] = icp_rl_f(xj, j);
#ifdef TF_SV_TIMING
    SV_T(7, x[0] + x[5]);
    if (lane == 0)
        for (int q = 0; q < 8; ++q) g_sv_t[q] += svt.acc[q];
#endif
}

// cv::Affine3f(rvec, t)'s rotation: Affine3<float>::rotation(const Vec3f&) (affine.hpp), every
// Matx operation rounded to float
template <int ALG>
__device__ __forceinline__ void icp_cv_rodrigues(const float* rv, float* R)
{
    double theta;
    if constexpr (ALG == 2) {
        double s2 = 0;
#pragma unroll
        for (int i = 0; i < 3; ++i) { const double v = rv[i]; s2 += v * v; }
        theta = sqrt(s2);
    } else {
        float s2 = 0;
#pragma unroll
        for (int i = 0; i < 3; ++i) { const float v = rv[i]; s2 += v * v; }
        theta = sqrtf(s2);
    }
    if (theta < 2.220446049250313e-16) {
#pragma unroll
        for (int k = 0; k < 9; ++k) R[k] = (k % 4 == 0) ? 1.0f : 0.0f;
        return;
    }
    double s, c;
    icp_sincos(theta, &s, &c);
    const double c1 = 1. - c;
    const double itheta = (theta != 0) ? 1. / theta : 0.;
    const float rx = (float)(rv[0] * itheta), ry = (float)(rv[1] * itheta), rz = (float)(rv[2] * itheta);
    const float rrt[9] = { rx * rx, rx * ry, rx * rz, rx * ry, ry * ry, ry * rz, rx * rz, ry * rz, rz * rz };
    const float rxm[9] = { 0, -rz, ry, rz, 0, -rx, -ry, rx, 0 };
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        const float I = (k % 4 == 0) ? 1.0f : 0.0f;
        const float cI = (float)(I * c), crr = (float)(rrt[k] * c1), sx = (float)(rxm[k] * s);
        const float t = cI + crr;
        R[k] = t + sx;
    }
}

// =============================================================================================
// The canonical tail in row layout (round 5).  icp_solve6_schur + icp_rodrigues + tf_rigid_mul on
// one wave issue ~500 instructions, every lane computing every element (the segment is issue-
// bound: ~300 f64 instructions at 4 cycles each).  Here lane i < 3 computes row i of each 3 x 3
// intermediate (T, S, adj S, the rotation) and of the new affine, values every row needs are read
// across with readlane or through LDS, and the uniform parts (adj R, the determinants' sums) run
// once on every lane.  Each element sees exactly the operations, in the same order, of the scalar
// functions above -- the results are theirs bit for bit (tools/micro/icp_tail.hip: 0 of 20 000
// random systems differ; 37 GPU parity tests).  ~280 instructions, and no faster: the tail is a
// dependency chain, not issue-bound (1545 vs 1585 cycles alone; ICP 124.7 -> 128.3 us in the
// kernel, profiles/r05/ab_icp_tail_rows.txt), so it stays an A/B build (IP_TAIL_ROWS=1).
// =============================================================================================
// sums are indexed as StreamHelper lays them out (projective_icp.cpp:51-61): Am[r][c] (r <= c) is
// sum {0, 7, 13, 18, 22, 25}[r] + c - r, bv[r] is Am[r][6]
template <typename T>
__device__ __forceinline__ T icp_sel3(int i, T a, T b, T c) { return i == 0 ? a : (i == 1 ? b : c); }
// sm: the 27 sums (uniform); aff: the current affine (uniform); i: the lane (rows 0-2 used);
// xs: 9 doubles of wave-private LDS.  Out: orow = row i of Tinc * aff, rv = the increment (uniform)
__device__ __forceinline__ void icp_tail_rows(const float (&sm)[27], const float (&aff)[12], int i, double* xs,
                                              float (&orow)[4], float (&rv)[6])
{
    // (indices written out: icp_smi folded by hand, so every sum is a register, never an indexed one)
    double R[3][3], Q[3][3], b2[3];
    R[0][0] = sm[18]; R[0][1] = sm[19]; R[0][2] = sm[20];
    R[1][0] = sm[19]; R[1][1] = sm[22]; R[1][2] = sm[23];
    R[2][0] = sm[20]; R[2][1] = sm[23]; R[2][2] = sm[25];
    Q[0][0] = sm[3]; Q[0][1] = sm[4]; Q[0][2] = sm[5];
    Q[1][0] = sm[9]; Q[1][1] = sm[10]; Q[1][2] = sm[11];
    Q[2][0] = sm[14]; Q[2][1] = sm[15]; Q[2][2] = sm[16];
    b2[0] = sm[21]; b2[1] = sm[24]; b2[2] = sm[26];
    // adj R (uniform): R is symmetric bit for bit, and so is its adjugate (the mirrored formulas
    // are the same products, commuted): six cofactors of icp_sym3_adj, det R as there
    double aR[3][3];
    aR[0][0] = R[1][1] * R[2][2] - R[1][2] * R[2][1];
    aR[0][1] = R[0][2] * R[2][1] - R[0][1] * R[2][2];
    aR[0][2] = R[0][1] * R[1][2] - R[0][2] * R[1][1];
    aR[1][1] = R[0][0] * R[2][2] - R[0][2] * R[2][0];
    aR[1][2] = R[0][2] * R[1][0] - R[0][0] * R[1][2];
    aR[2][2] = R[0][0] * R[1][1] - R[0][1] * R[1][0];
    aR[1][0] = aR[0][1]; aR[2][0] = aR[0][2]; aR[2][1] = aR[1][2];
    const double dR = (R[0][0] * aR[0][0] + R[0][1] * aR[1][0]) + R[0][2] * aR[2][0];
    const double rR = 1.0 / dR;
    // row i's inputs
    double Qi[3], Pi[3], Qc[3], aRi[3];
    Qi[0] = icp_sel3(i, sm[3], sm[9], sm[14]);
    Pi[0] = icp_sel3(i, sm[0], sm[1], sm[2]);
    Qc[0] = icp_sel3(i, sm[3], sm[4], sm[5]);
    aRi[0] = icp_sel3(i, aR[0][0], aR[1][0], aR[2][0]);
    Qi[1] = icp_sel3(i, sm[4], sm[10], sm[15]);
    Pi[1] = icp_sel3(i, sm[1], sm[7], sm[8]);
    Qc[1] = icp_sel3(i, sm[9], sm[10], sm[11]);
    aRi[1] = icp_sel3(i, aR[0][1], aR[1][1], aR[2][1]);
    Qi[2] = icp_sel3(i, sm[5], sm[11], sm[16]);
    Pi[2] = icp_sel3(i, sm[2], sm[8], sm[13]);
    Qc[2] = icp_sel3(i, sm[14], sm[15], sm[16]);
    aRi[2] = icp_sel3(i, aR[0][2], aR[1][2], aR[2][2]);
    const double b1i = icp_sel3(i, sm[6], sm[12], sm[17]);
    const double b2i = icp_sel3(i, sm[21], sm[24], sm[26]);
    // T, S, c: row i
    double Ti[3], Si[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) Ti[j] = ((Qi[0] * aR[0][j] + Qi[1] * aR[1][j]) + Qi[2] * aR[2][j]) * rR;
#pragma unroll
    for (int j = 0; j < 3; ++j) Si[j] = Pi[j] - ((Ti[0] * Q[j][0] + Ti[1] * Q[j][1]) + Ti[2] * Q[j][2]);
    const double ci = b1i - ((Ti[0] * b2[0] + Ti[1] * b2[1]) + Ti[2] * b2[2]);
    // S through LDS: row i of adj S = C[i][j] = S[j+1][i+1] S[j+2][i+2] - S[j+1][i+2] S[j+2][i+1]
    if (i < 3) {
#pragma unroll
        for (int j = 0; j < 3; ++j) xs[3 * i + j] = Si[j];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int i1 = i == 0 ? 1 : (i == 1 ? 2 : 0), i2 = i == 0 ? 2 : (i == 1 ? 0 : 1);
    double SA[3], SB[3];                                    // column i+1, column i+2 of S
#pragma unroll
    for (int r = 0; r < 3; ++r) { SA[r] = xs[3 * r + i1]; SB[r] = xs[3 * r + i2]; }
    const double s0i = xs[i < 3 ? i : 0];                   // S[0][i]
    double aSi[3];
    aSi[0] = SA[1] * SB[2] - SB[1] * SA[2];
    aSi[1] = SA[2] * SB[0] - SB[2] * SA[0];
    aSi[2] = SA[0] * SB[1] - SB[0] * SA[1];
    // det S = (S00 aS00 + S01 aS10) + S02 aS20: term k on lane k
    const double tk = s0i * aSi[0];
    const double dS = (icp_rl_d(tk, 0) + icp_rl_d(tk, 1)) + icp_rl_d(tk, 2);
    const double rS = 1.0 / dS;
    const double c0 = icp_rl_d(ci, 0), c1 = icp_rl_d(ci, 1), c2 = icp_rl_d(ci, 2);
    const double x1i = ((aSi[0] * c0 + aSi[1] * c1) + aSi[2] * c2) * rS;
    const double x10 = icp_rl_d(x1i, 0), x11 = icp_rl_d(x1i, 1), x12 = icp_rl_d(x1i, 2);
    const double ei = b2i - ((Qc[0] * x10 + Qc[1] * x11) + Qc[2] * x12);
    const double e0 = icp_rl_d(ei, 0), e1 = icp_rl_d(ei, 1), e2 = icp_rl_d(ei, 2);
    const float x2f = (float)(((aRi[0] * e0 + aRi[1] * e1) + aRi[2] * e2) * rR);
    rv[0] = (float)x10; rv[1] = (float)x11; rv[2] = (float)x12;
    rv[3] = icp_rl_f(x2f, 0); rv[4] = icp_rl_f(x2f, 1); rv[5] = icp_rl_f(x2f, 2);
    // Rodrigues, row i (icp_rodrigues' operations per element)
    float Ri[3];
    {
        constexpr double inv_sin[14] = { 0.0, 1.0/6.0, 1.0/20.0, 1.0/42.0, 1.0/72.0, 1.0/110.0, 1.0/156.0,
            1.0/210.0, 1.0/272.0, 1.0/342.0, 1.0/420.0, 1.0/506.0, 1.0/600.0, 1.0/702.0 };
        constexpr double inv_cos[15] = { 0.0, 1.0/2.0, 1.0/12.0, 1.0/30.0, 1.0/56.0, 1.0/90.0, 1.0/132.0,
            1.0/182.0, 1.0/240.0, 1.0/306.0, 1.0/380.0, 1.0/462.0, 1.0/552.0, 1.0/650.0, 1.0/756.0 };
        const double rx = rv[0], ry = rv[1], rz = rv[2];
        const double t2 = (rx * rx + ry * ry) + rz * rz;
        if (t2 < 4.930380657631324e-32) {
#pragma unroll
            for (int j = 0; j < 3; ++j) Ri[j] = (i == j) ? 1.0f : 0.0f;
        } else if (t2 > 9.869604401089358) {
            float Rf[9];
            icp_rodrigues_sqrt(rv, Rf);
#pragma unroll
            for (int j = 0; j < 3; ++j) Ri[j] = icp_sel3(i, Rf[j], Rf[3 + j], Rf[6 + j]);
        } else {
            double pc = 1.0, pa = 1.0, pb = 1.0;
            if (t2 < 0.000244140625) {
#pragma unroll
                for (int n = 4; n >= 1; --n) {
                    pc = fma(-(t2 * inv_cos[n]), pc, 1.0);
                    pa = fma(-(t2 * inv_sin[n]), pa, 1.0);
                    pb = fma(-(t2 * inv_cos[n + 1]), pb, 1.0);
                }
            } else if (t2 < 0.015625) {
#pragma unroll
                for (int n = 6; n >= 1; --n) {
                    pc = fma(-(t2 * inv_cos[n]), pc, 1.0);
                    pa = fma(-(t2 * inv_sin[n]), pa, 1.0);
                    pb = fma(-(t2 * inv_cos[n + 1]), pb, 1.0);
                }
            } else {
#pragma unroll
                for (int n = 13; n >= 1; --n) {
                    pc = fma(-(t2 * inv_cos[n]), pc, 1.0);
                    pa = fma(-(t2 * inv_sin[n]), pa, 1.0);
                    pb = fma(-(t2 * inv_cos[n + 1]), pb, 1.0);
                }
            }
            const double b = 0.5 * pb;
            const double ri = icp_sel3(i, rx, ry, rz);
            const double rj[3] = { rx, ry, rz };
            // [r]x row i: (0, -rz, ry), (rz, 0, -rx), (-ry, rx, 0)
            const double m[3] = { icp_sel3(i, 0.0, rz, -ry), icp_sel3(i, -rz, 0.0, rx), icp_sel3(i, ry, -rx, 0.0) };
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const double I = (i == j) ? 1.0 : 0.0;
                Ri[j] = (float)((pc * I + b * (ri * rj[j])) + pa * m[j]);
            }
        }
    }
    // row i of Tinc * aff (tf_rigid_mul)
#pragma unroll
    for (int c = 0; c < 3; ++c) orow[c] = (Ri[0] * aff[0 * 4 + c] + Ri[1] * aff[1 * 4 + c]) + Ri[2] * aff[2 * 4 + c];
    orow[3] = ((Ri[0] * aff[3] + Ri[1] * aff[7]) + Ri[2] * aff[11]) + x2f;
}

// the iteration's solve + Rodrigues under pose algebra ALG
template <int ALG>
__device__ __forceinline__ void icp_solve_rodrigues(const float (&Am)[6][6], const float (&bv)[6], float (&rv)[6], float* R)
{
    if constexpr (ALG == 0) {
#if TF_SOLVE_LDL                                  // A/B only: the rounds 2-4 form (not the oracle's)
        icp_solve6_ldl(Am, bv, rv);
#else
        icp_solve6_schur(Am, bv, rv);
#endif
        icp_rodrigues(rv, R);
    } else {
        icp_cv_solve_svd6<ALG>(Am, bv, rv);
        icp_cv_rodrigues<ALG>(rv, R);
    }
}
