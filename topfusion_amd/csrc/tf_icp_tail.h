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
    if (t2 < 0.015625) {                          // t < 1/8: 6 terms (first omitted < 2^-80 relative)
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

// cv::solve(A, b, DECOMP_SVD) replacement (oracle/tf_oracle.c:solve6, same operation order):
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

