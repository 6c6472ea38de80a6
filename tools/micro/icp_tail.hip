// Latency of the persistent ICP kernel's serial tail on one wave (gfx950): the LDL^T solve,
// Rodrigues and compose of tf_icp.hip, and the f64 primitives they chain, each repeated N times
// with every repetition depending on the last.  hipcc --offload-arch=gfx950 -O3 -ffp-contract=off
//   -fhip-fp32-correctly-rounded-divide-sqrt icp_tail.hip -o icp_tail  (tools/micro/Makefile)
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../topfusion_amd/csrc/tf_icp_tail.h"
#include "../../topfusion_amd/csrc/tf_pose.h"

// one instantiation per variant (its own register allocation: a runtime switch over all of them
// spilled the large ones), one wave
template <int which>
__global__ void __launch_bounds__(64) k_tail(const float* in, float* out, long long* cyc, int n)
{
    float Am[6][6], bv[6], aff[12];
    for (int i = 0; i < 6; ++i) { bv[i] = in[36 + i]; for (int j = 0; j < 6; ++j) Am[i][j] = in[i * 6 + j]; }
    for (int i = 0; i < 12; ++i) aff[i] = (i % 5 == 0) ? 1.f : 0.f;
    double dx = in[0], dacc = 0;
    const long long t0 = clock64();
    for (int it = 0; it < n; ++it) {
        if constexpr (which == 0) {                       // solve + Rodrigues + compose (the tail)
            float rv[6], R[9], tinc[12];
            icp_solve_rodrigues<0>(Am, bv, rv, R);
            for (int j = 0; j < 3; ++j) {
                tinc[j * 4 + 0] = R[j * 3 + 0]; tinc[j * 4 + 1] = R[j * 3 + 1];
                tinc[j * 4 + 2] = R[j * 3 + 2]; tinc[j * 4 + 3] = rv[3 + j];
            }
            tf_rigid_mul(tinc, aff, aff);
            bv[0] += aff[3] * 1e-30f;           // next repetition depends on this one
        } else if constexpr (which == 1) {                // solve only (LDL^T, rounds 2-4)
            float rv[6];
            icp_solve6_ldl(Am, bv, rv);
            bv[0] += rv[0] * 1e-30f;
        } else if constexpr (which == 14) {               // solve only (2 x 2 block Schur, round 5)
            float rv[6];
            icp_solve6_schur(Am, bv, rv);
            bv[0] += rv[0] * 1e-30f;
        } else if constexpr (which == 2) {                // Rodrigues only
            float rv[6] = { bv[0] * 1e-3f, bv[1] * 1e-3f, bv[2] * 1e-3f, 0, 0, 0 }, R[9];
            icp_rodrigues(rv, R);
            bv[0] += R[1] * 1e-30f;
        } else if constexpr (which == 3) {                // 10 dependent f64 divides
            for (int k = 0; k < 10; ++k) dx = 1.0 / (dx + 1.0);
        } else if constexpr (which == 4) {                // 10 dependent f64 sqrt
            for (int k = 0; k < 10; ++k) dx = sqrt(dx + 1.0);
        } else if constexpr (which == 5) {                // 10 dependent f64 fma
            for (int k = 0; k < 10; ++k) dx = fma(dx, 0.999, 1e-3);
        } else if constexpr (which == 6) {                // 10 dependent f32 fma
            float f = (float)dx;
            for (int k = 0; k < 10; ++k) f = fmaf(f, 0.999f, 1e-3f);
            dx = f;
        } else if constexpr (which == 7) {                // 10 dependent f32 IEEE divides
            float f = (float)dx;
            for (int k = 0; k < 10; ++k) f = 1.0f / (f + 1.0f);
            dx = f;
        } else if constexpr (which == 8) {                // the reference's cv::solve(DECOMP_SVD) (ALG 4)
            float rv[6];
            icp_cv_solve_svd6<4>(Am, bv, rv);
            bv[0] += rv[0] * 1e-30f;
        } else if constexpr (which == 9) {                // cv solve + Affine3f rotation + compose
            float rv[6], R[9], tinc[12];
            icp_solve_rodrigues<4>(Am, bv, rv, R);
            for (int j = 0; j < 3; ++j) {
                tinc[j * 4 + 0] = R[j * 3 + 0]; tinc[j * 4 + 1] = R[j * 3 + 1];
                tinc[j * 4 + 2] = R[j * 3 + 2]; tinc[j * 4 + 3] = rv[3 + j];
            }
            tf_rigid_mul(tinc, aff, aff);
            bv[0] += aff[3] * 1e-30f;
        } else if constexpr (which == 10) {               // 10 dependent f64 adds
            for (int k = 0; k < 10; ++k) dx = dx + 1e-3;
        } else if constexpr (which == 11) {               // 10 dependent f64 muls
            for (int k = 0; k < 10; ++k) dx = dx * 0.999;
        } else if constexpr (which == 12) {               // 10 dependent (readlane -> f32 add) round trips
            float f = (float)dx + (float)threadIdx.x;
            for (int k = 0; k < 10; ++k)
                f = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, f), k)) + 1.0f + (float)threadIdx.x;
            dx = f;
        } else if constexpr (which == 13) {               // 10 dependent f32 adds
            float f = (float)dx;
            for (int k = 0; k < 10; ++k) f = f + 1e-3f;
            dx = f;
        }
    }
    const long long t1 = clock64();
    dacc += dx;
    if (threadIdx.x == 0) { cyc[which] = t1 - t0; out[which] = aff[3] + bv[0] + (float)dacc; }
}

// icp_tail_rows (row layout) against the scalar tail on random ICP-like systems: sums of 7-vector
// outer products (the rows), small random increments, a random affine; every output bit compared.
// Also each form's latency with the whole system changing every repetition (nothing hoisted).
__device__ __forceinline__ float rnd(unsigned& st)
{
    st = st * 1664525u + 1013904223u;
    return (float)(st >> 8) * (1.0f / 16777216.0f) - 0.5f;
}
__device__ void make_system(unsigned seed, float (&sm)[27], float (&aff)[12])
{
    unsigned st = seed * 2654435761u + 12345u;
    for (int q = 0; q < 27; ++q) sm[q] = 0.f;
    const int nrow = 8 + (seed % 57);
    for (int n = 0; n < nrow; ++n) {
        float r[7];
        for (int k = 0; k < 6; ++k) r[k] = rnd(st) * (k < 3 ? 2.0f : 1.0f);
        r[6] = rnd(st) * 1e-2f;
        int q = 0;
        for (int a = 0; a < 6; ++a)
            for (int b = a; b < 7; ++b, ++q) sm[q] += r[a] * r[b];
    }
    float rv[3] = { rnd(st) * 0.2f, rnd(st) * 0.2f, rnd(st) * 0.2f }, R[9];
    float rv6[6] = { rv[0], rv[1], rv[2], 0, 0, 0 };
    icp_rodrigues(rv6, R);
    for (int j = 0; j < 3; ++j) {
        for (int c = 0; c < 3; ++c) aff[4 * j + c] = R[3 * j + c];
        aff[4 * j + 3] = rnd(st);
    }
}
__device__ void tail_scalar(const float (&sm)[27], const float (&aff)[12], float (&out)[12], float (&rv)[6])
{
    float Am[6][6], bv[6];
    int shift = 0;
    for (int i = 0; i < 6; ++i)
        for (int j = i; j < 7; ++j) {
            const float v = sm[shift++];
            if (j == 6) bv[i] = v; else { Am[j][i] = v; Am[i][j] = v; }
        }
    float R[9], tinc[12];
    icp_solve6_schur(Am, bv, rv);
    icp_rodrigues(rv, R);
    for (int j = 0; j < 3; ++j) {
        tinc[4 * j + 0] = R[3 * j + 0]; tinc[4 * j + 1] = R[3 * j + 1];
        tinc[4 * j + 2] = R[3 * j + 2]; tinc[4 * j + 3] = rv[3 + j];
    }
    tf_rigid_mul(tinc, aff, out);
}
__global__ void __launch_bounds__(64) k_rows_check(int nsys, int* bad, int* first_bad)
{
    __shared__ double xs[9];
    const int lane = threadIdx.x;
    for (int sys = 0; sys < nsys; ++sys) {
        float sm[27], aff[12], o_s[12], rv_s[6], orow[4], rv_r[6];
        make_system((unsigned)sys, sm, aff);
        tail_scalar(sm, aff, o_s, rv_s);
        icp_tail_rows(sm, aff, lane, xs, orow, rv_r);
        bool ok = true;
        for (int k = 0; k < 6; ++k) ok = ok && __float_as_uint(rv_s[k]) == __float_as_uint(rv_r[k]);
        if (lane < 3)
            for (int c = 0; c < 4; ++c) ok = ok && __float_as_uint(orow[c]) == __float_as_uint(o_s[4 * lane + c]);
        if (__builtin_amdgcn_ballot_w64(!ok && lane < 3) != 0 && lane == 0) {
            if (*bad == 0) *first_bad = sys;
            *bad += 1;
        }
    }
}
template <int ROWS>
__global__ void __launch_bounds__(64) k_rows_time(int n, long long* cyc, float* out)
{
    __shared__ double xs[9];
    const int lane = threadIdx.x;
    float sm[27], aff[12];
    make_system(7u, sm, aff);
    float acc = 0.f;
    const long long t0 = clock64();
    for (int it = 0; it < n; ++it) {
        float rv[6];
        if constexpr (ROWS) {
            float orow[4];
            icp_tail_rows(sm, aff, lane, xs, orow, rv);
            acc = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, orow[3]), 0));
        } else {
            float o[12];
            tail_scalar(sm, aff, o, rv);
            acc = o[3];
        }
        sm[0] += acc * 1e-30f;          // the next repetition's whole system depends on this one
        sm[22] += rv[4] * 1e-30f;
    }
    const long long t1 = clock64();
    if (lane == 0) { cyc[ROWS] = t1 - t0; out[ROWS] = acc; }
}


// candidate: S' = det R * P - Q adj(R) Q^T (one division on the chain; 1/det R off it)
__device__ __forceinline__ void icp_solve6_schur2(const float (&Af)[6][6], const float (&bf)[6], float (&x)[6])
{
    double P[3][3], Q[3][3], R[3][3], b1[3], b2[3];
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) { P[i][j] = Af[i][j]; Q[i][j] = Af[i][3 + j]; R[i][j] = Af[3 + i][3 + j]; }
        b1[i] = bf[i]; b2[i] = bf[3 + i];
    }
    double aR[3][3], dR, aS[3][3], dS, U[3][3], S[3][3], c[3], x1[3], e[3];
    icp_sym3_adj(R, aR, dR);
    const double rR = 1.0 / dR;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) U[i][j] = (Q[i][0] * aR[0][j] + Q[i][1] * aR[1][j]) + Q[i][2] * aR[2][j];
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) S[i][j] = dR * P[i][j] - ((U[i][0] * Q[j][0] + U[i][1] * Q[j][1]) + U[i][2] * Q[j][2]);
        c[i] = dR * b1[i] - ((U[i][0] * b2[0] + U[i][1] * b2[1]) + U[i][2] * b2[2]);
    }
    icp_sym3_adj(S, aS, dS);
    const double rS = 1.0 / dS;
    for (int i = 0; i < 3; ++i) x1[i] = ((aS[i][0] * c[0] + aS[i][1] * c[1]) + aS[i][2] * c[2]) * rS;
    for (int i = 0; i < 3; ++i) e[i] = b2[i] - ((Q[0][i] * x1[0] + Q[1][i] * x1[1]) + Q[2][i] * x1[2]);
    for (int i = 0; i < 3; ++i) {
        x[i] = (float)x1[i];
        x[3 + i] = (float)(((aR[i][0] * e[0] + aR[i][1] * e[1]) + aR[i][2] * e[2]) * rR);
    }
}
__device__ void unpack27(const float (&sm)[27], float (&Am)[6][6], float (&bv)[6])
{
    int shift = 0;
    for (int i = 0; i < 6; ++i)
        for (int j = i; j < 7; ++j) {
            const float v = sm[shift++];
            if (j == 6) bv[i] = v; else { Am[j][i] = v; Am[i][j] = v; }
        }
}
template <int V>
__global__ void __launch_bounds__(64) k_solve_time(int n, long long* cyc, float* out, int* ndiff, float* maxrel)
{
    float sm[27], aff[12];
    make_system(11u, sm, aff);
    float acc = 0.f;
    const long long t0 = clock64();
    for (int it = 0; it < n; ++it) {
        float Am[6][6], bv[6], rv[6];
        unpack27(sm, Am, bv);
        if constexpr (V == 0) icp_solve6_schur(Am, bv, rv); else icp_solve6_schur2(Am, bv, rv);
        acc = rv[0] + rv[4];
        sm[0] += acc * 1e-30f;          // the next repetition's whole system depends on this one
        sm[22] += rv[4] * 1e-30f;
    }
    const long long t1 = clock64();
    if (threadIdx.x == 0) { cyc[V] = t1 - t0; out[V] = acc; }
    if (V == 1 && threadIdx.x == 0) {   // bits: S' against the canonical solve over random systems
        int d = 0; float mr = 0.f;
        for (int sys = 0; sys < 20000; ++sys) {
            float s2[27], a2[12], Am[6][6], bv[6], r0[6], r1[6];
            make_system((unsigned)sys, s2, a2);
            unpack27(s2, Am, bv);
            icp_solve6_schur(Am, bv, r0); icp_solve6_schur2(Am, bv, r1);
            bool same = true;
            for (int k = 0; k < 6; ++k) {
                same = same && __float_as_uint(r0[k]) == __float_as_uint(r1[k]);
                const float rel = fabsf(r0[k] - r1[k]) / fmaxf(fabsf(r0[k]), 1e-30f);
                mr = fmaxf(mr, rel);
            }
            d += !same;
        }
        *ndiff = d; *maxrel = mr;
    }
}

template <int W>
static void launch_t(int w, const float* a, float* o, long long* c, int n)
{
    if (w == W) hipLaunchKernelGGL(k_tail<W>, dim3(1), dim3(64), 0, 0, a, o, c, n);
    if constexpr (W > 0) launch_t<W - 1>(w, a, o, c, n);
}
static void launch(int w, const float* a, float* o, long long* c, int n) { launch_t<14>(w, a, o, c, n); }

int main()
{
    float hA[42];
    // a symmetric positive-definite normal matrix and a right-hand side of ICP's scale
    for (int i = 0; i < 6; ++i) for (int j = 0; j < 6; ++j) hA[i * 6 + j] = (i == j) ? 1000.f + 10 * i : 3.f / (1 + i + j);
    for (int i = 0; i < 6; ++i) hA[36 + i] = 0.01f * (i + 1);
    float *dA, *dO; long long* dC;
    hipMalloc(&dA, sizeof(hA)); hipMalloc(&dO, 64 * 4); hipMalloc(&dC, 16 * sizeof(long long));
    hipMemcpy(dA, hA, sizeof(hA), hipMemcpyHostToDevice);
    const int N = 1000;
    const char* names[] = { "solve+rodrigues+compose (canonical)", "solve (LDL^T, r2-4)", "rodrigues", "10x f64 div", "10x f64 sqrt",
                            "10x f64 fma", "10x f32 fma", "10x f32 div", "cv solve (SVD)", "cv solve+rot+compose",
                            "10x f64 add", "10x f64 mul", "10x readlane+add", "10x f32 add", "solve (block Schur)" };
    {   // the row-layout tail: bit-exact against the scalar one, and each one's latency
        int* dBad; int hb[2] = { 0, -1 };
        hipMalloc(&dBad, 2 * sizeof(int));
        hipMemcpy(dBad, hb, sizeof(hb), hipMemcpyHostToDevice);
        const int nsys = 20000;
        hipLaunchKernelGGL(k_rows_check, dim3(1), dim3(64), 0, 0, nsys, dBad, dBad + 1);
        hipMemcpy(hb, dBad, sizeof(hb), hipMemcpyDeviceToHost);
        printf("row-layout tail vs scalar tail: %d of %d random systems differ in any output bit (first %d)\n", hb[0], nsys, hb[1]);
        long long hc[2];
        for (int w = 0; w < 2; ++w) {
            if (w) { hipLaunchKernelGGL(k_rows_time<1>, dim3(1), dim3(64), 0, 0, 10, dC, dO); hipLaunchKernelGGL(k_rows_time<1>, dim3(1), dim3(64), 0, 0, N, dC, dO); }
            else { hipLaunchKernelGGL(k_rows_time<0>, dim3(1), dim3(64), 0, 0, 10, dC, dO); hipLaunchKernelGGL(k_rows_time<0>, dim3(1), dim3(64), 0, 0, N, dC, dO); }
        }
        hipMemcpy(hc, dC, sizeof(hc), hipMemcpyDeviceToHost);
        printf("%-26s %8.1f cycles per repetition (s_memtime, system changing every repetition)\n", "tail scalar", (double)hc[0] / N);
        printf("%-26s %8.1f cycles per repetition (s_memtime, system changing every repetition)\n", "tail row layout", (double)hc[1] / N);
    }
    {   // the S' solve (one division on the chain) against the canonical Schur solve
        int* dD; float* dM; hipMalloc(&dD, sizeof(int)); hipMalloc(&dM, sizeof(float));
        long long hc[2];
        hipLaunchKernelGGL(k_solve_time<0>, dim3(1), dim3(64), 0, 0, 10, dC, dO, dD, dM);
        hipLaunchKernelGGL(k_solve_time<0>, dim3(1), dim3(64), 0, 0, N, dC, dO, dD, dM);
        hipLaunchKernelGGL(k_solve_time<1>, dim3(1), dim3(64), 0, 0, 10, dC, dO, dD, dM);
        hipLaunchKernelGGL(k_solve_time<1>, dim3(1), dim3(64), 0, 0, N, dC, dO, dD, dM);
        hipMemcpy(hc, dC, sizeof(hc), hipMemcpyDeviceToHost);
        int nd = 0; float mr = 0;
        hipMemcpy(&nd, dD, sizeof(int), hipMemcpyDeviceToHost); hipMemcpy(&mr, dM, sizeof(float), hipMemcpyDeviceToHost);
        printf("%-26s %8.1f cycles per repetition (s_memtime, system changing every repetition)\n", "solve Schur", (double)hc[0] / N);
        printf("%-26s %8.1f cycles per repetition (s_memtime, system changing every repetition)\n", "solve Schur S'", (double)hc[1] / N);
        printf("S' vs Schur: %d of 20000 random systems differ in some output bit, max relative difference %g\n", nd, mr);
    }
    for (int w = 0; w < 15; ++w) {
        launch(w, dA, dO, dC, 10);   // warm
        launch(w, dA, dO, dC, N);
        long long c = 0;
        hipMemcpy(&c, dC + w, sizeof(c), hipMemcpyDeviceToHost);
        printf("%-26s %8.1f cycles per repetition (s_memtime)\n", names[w], (double)c / N);
    }
    return 0;
}
