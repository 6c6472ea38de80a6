// Accuracy of gfx950's f64 approximations (v_rsq_f64, v_rcp_f64) and one Goldschmidt /
// Newton step, plus dependent-chain latencies of the primitives the lane-parallel Jacobi SVD
// chains (tf_icp_tail.h, icp_cv_solve_svd6_lanes).  hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>

__device__ __forceinline__ double rnd01(unsigned long long& s)
{
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    return (double)(s >> 11) * (1.0 / 9007199254740992.0);
}
// max relative errors (as doubles) over many inputs: [0] rsq, [1] rcp, [2] sqrt by one
// Goldschmidt step, [3] 1/(2 sqrt) by the same step, [4] rcp + one Newton step
__global__ void k_acc(int n, double* out)
{
    __shared__ double red[5][256];
    unsigned long long s = 0x9E3779B97F4A7C15ull * (blockIdx.x * 256 + threadIdx.x + 1);
    double m[5] = { 0, 0, 0, 0, 0 };
    for (int i = 0; i < n; ++i) {
        const double e = (rnd01(s) - 0.5) * 400.0;          // exponents 2^-200 .. 2^200
        const double x = exp2(e) * (1.0 + rnd01(s));
        const double t = 1.0 / sqrt(x), tr = 1.0 / x, ts = sqrt(x);
        const double y = __builtin_amdgcn_rsq(x);
        const double r = __builtin_amdgcn_rcp(x);
        double g = x * y, h = 0.5 * y;
        const double rr = fma(-g, h, 0.5);
        g = fma(g, rr, g); h = fma(h, rr, h);
        const double rn = fma(fma(-x, r, 1.0), r, r);
        m[0] = fmax(m[0], fabs(y / t - 1.0));
        m[1] = fmax(m[1], fabs(r / tr - 1.0));
        m[2] = fmax(m[2], fabs(g / ts - 1.0));
        m[3] = fmax(m[3], fabs(2.0 * h * ts - 1.0));
        m[4] = fmax(m[4], fabs(rn / tr - 1.0));
    }
    for (int k = 0; k < 5; ++k) red[k][threadIdx.x] = m[k];
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 0; k < 5; ++k) {
            double mm = 0;
            for (int j = 0; j < 256; ++j) mm = fmax(mm, red[k][j]);
            unsigned long long* o = (unsigned long long*)&out[k];
            atomicMax(o, __double_as_longlong(mm));          // positive doubles order as integers
        }
    }
}

template <int W>
__global__ void __launch_bounds__(64) k_lat(int n, long long* cyc, float* out)
{
    double dx = 1.0 + threadIdx.x * 1e-3;
    float f = 1.0f + threadIdx.x;
    int idx = ((threadIdx.x + 8) & 63) * 4;
    const long long t0 = clock64();
    for (int it = 0; it < n; ++it) {
        if constexpr (W == 0) { for (int k = 0; k < 10; ++k) dx = __builtin_amdgcn_rsq(dx + 1.0); }
        else if constexpr (W == 1) { for (int k = 0; k < 10; ++k) dx = __builtin_amdgcn_rcp(dx + 1.0); }
        else if constexpr (W == 2) {   // ds_bpermute round trips
            for (int k = 0; k < 10; ++k) f = __int_as_float(__builtin_amdgcn_ds_bpermute(idx, __float_as_int(f))) + 1.0f;
        } else if constexpr (W == 3) { // DPP row_shl:1 round trips
            for (int k = 0; k < 10; ++k) f = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(f), 0x101, 0xf, 0xf, false)) + 1.0f;
        } else if constexpr (W == 4) { // f64 -> f32 -> f64 conversions
            for (int k = 0; k < 10; ++k) dx = (double)(float)dx + 1.0;
        } else if constexpr (W == 5) { // v_permlane32_swap round trips
            for (int k = 0; k < 10; ++k) { auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(f), __float_as_uint(f), false, false); f = __uint_as_float(r[0]) + 1.0f; }
        } else if constexpr (W == 6) { // DPP row_share:0 round trips
            for (int k = 0; k < 10; ++k) f = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(f), 0x150, 0xf, 0xf, false)) + 1.0f;
        }
    }
    const long long t1 = clock64();
    if (threadIdx.x == 0) { cyc[W] = t1 - t0; out[W] = (float)dx + f; }
}

int main()
{
    double* dO; long long* dC; float* dF;
    hipMalloc(&dO, 5 * sizeof(double)); hipMalloc(&dC, 16 * sizeof(long long)); hipMalloc(&dF, 64);
    hipMemset(dO, 0, 5 * sizeof(double));
    hipLaunchKernelGGL(k_acc, dim3(1024), dim3(256), 0, 0, 4096, dO);
    double m[5];
    hipMemcpy(m, dO, sizeof(m), hipMemcpyDeviceToHost);
    const char* nm[5] = { "v_rsq_f64", "v_rcp_f64", "sqrt: rsq + 1 Goldschmidt", "1/(2 sqrt): same step", "rcp + 1 Newton" };
    printf("max relative error over %d inputs, exponents 2^-200..2^200\n", 1024 * 256 * 4096);
    for (int k = 0; k < 5; ++k) printf("  %-28s %.3e  (2^%.2f)\n", nm[k], m[k], m[k] > 0 ? log2(m[k]) : -999.0);
    const int N = 1000;
    const char* ln[7] = { "10x v_rsq_f64", "10x v_rcp_f64", "10x ds_bpermute+add", "10x dpp row_shl+add", "10x cvt f64-f32-f64+add",
                          "10x permlane32_swap+add", "10x dpp row_share+add" };
#define LAT(w) hipLaunchKernelGGL(k_lat<w>, dim3(1), dim3(64), 0, 0, 10, dC, dF); hipLaunchKernelGGL(k_lat<w>, dim3(1), dim3(64), 0, 0, N, dC, dF);
    LAT(0) LAT(1) LAT(2) LAT(3) LAT(4) LAT(5) LAT(6)
    long long c[16];
    hipMemcpy(c, dC, sizeof(c), hipMemcpyDeviceToHost);
    for (int w = 0; w < 7; ++w) printf("%-28s %8.1f cycles per repetition (s_memtime)\n", ln[w], (double)c[w] / N);
    return 0;
}
