// The lane-parallel cv::solve(DECOMP_SVD) (tf_icp_tail.h, icp_cv_solve_svd6_lanes) against the
// serial one (icp_cv_solve_svd6) and the oracle (tfo_cv_solve_svd6), bit for bit, on captured ICP
// systems (tools/svd_systems.py), random ICP-like systems and degenerate ones (A = 0, rank
// deficient, huge / tiny scales); then the latency of both forms on one wave, each solve
// depending on the last.
//   make -C tools/micro svd_lanes;  ./tools/micro/svd_lanes tests/golden/icp_systems_C2_opencv4.f32
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#ifdef TF_SV_STATS                               // (the svd_lanes_stats build: counts, not timing)
__device__ unsigned long long g_sv_stats[4];     // rotations, fast-path fallback levels, zero-SV finishes
#endif
#ifdef TF_SV_TIMING                              // (the svd_lanes_timing build: cycles per level phase)
__device__ long long g_sv_t[8];
#endif
#include "../../topfusion_amd/csrc/tf_icp_tail.h"

extern "C" void tfo_cv_solve_svd6(const float A[36], const float b[6], float x[6]);
extern "C" void tfo_set_pose_algebra(int mode, int use_libm);

__device__ __forceinline__ void unpack27(const float (&sm)[27], float (&Am)[6][6], float (&bv)[6])
{
    int shift = 0;
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = i; j < 7; ++j) {
            const float v = sm[shift++];
            if (j == 6) bv[i] = v; else { Am[j][i] = v; Am[i][j] = v; }
        }
}

// one wave per system: x from both forms, a flag when any bit differs
template <int ALG>
__global__ void __launch_bounds__(64) k_check(const float* sys, int n, float* xl, int* bad)
{
    const int lane = threadIdx.x;
    for (int q = blockIdx.x; q < n; q += gridDim.x) {
        float sm[27], Am[6][6], bv[6], x0[6], x1[6];
#pragma unroll
        for (int i = 0; i < 27; ++i) sm[i] = sys[27 * q + i];
        unpack27(sm, Am, bv);
        icp_cv_solve_svd6<ALG>(Am, bv, x0);
        const float tot = lane < 27 ? sys[27 * q + lane] : 0.f;
        icp_cv_solve_svd6_lanes<ALG>(tot, 1, lane, x1);
        bool same = true;
#pragma unroll
        for (int j = 0; j < 6; ++j) same = same && __float_as_uint(x0[j]) == __float_as_uint(x1[j]);
        if (lane < 6) xl[6 * q + lane] = x1[lane];
        if (lane == 0 && !same) atomicAdd(bad, 1);
    }
}

template <int LANES>
__global__ void __launch_bounds__(64) k_time(const float* sys, int nsys, int n, long long* cyc, float* out)
{
    const int lane = threadIdx.x;
    float acc = 0.f;
    const long long t0 = clock64();
    for (int it = 0; it < n; ++it) {
        const int q = it % nsys;
        float x[6];
        if constexpr (LANES) {
            const float tot = lane < 27 ? sys[27 * q + lane] + acc * 1e-30f : 0.f;
            icp_cv_solve_svd6_lanes<4>(tot, 1, lane, x);
        } else {
            float sm[27], Am[6][6], bv[6];
#pragma unroll
            for (int i = 0; i < 27; ++i) sm[i] = sys[27 * q + i] + acc * 1e-30f;
            unpack27(sm, Am, bv);
            icp_cv_solve_svd6<4>(Am, bv, x);
        }
        acc = x[0] + x[5];
    }
    const long long t1 = clock64();
    if (lane == 0) { cyc[LANES] = t1 - t0; out[LANES] = acc; }
}

static unsigned long long g_st = 0x2545F4914F6CDD1Dull;
static float frand() { g_st = g_st * 6364136223846793005ull + 1442695040888963407ull; return (float)(g_st >> 40) / 16777216.0f - 0.5f; }

int main(int argc, char** argv)
{
    std::vector<float> sys;
    int ncap = 0;
    if (argc > 1) {
        FILE* f = fopen(argv[1], "rb");
        if (!f) { perror(argv[1]); return 2; }
        fseek(f, 0, SEEK_END);
        ncap = (int)(ftell(f) / (27 * 4));
        fseek(f, 0, SEEK_SET);
        sys.resize((size_t)ncap * 27);
        if (fread(sys.data(), 4, sys.size(), f) != sys.size()) return 2;
        fclose(f);
    }
    // random ICP-like systems (sums of outer products of 7-vectors, 7..66 rows), at scales 1,
    // 1e-12 and 1e12
    const int nrand = 60000;
    for (int q = 0; q < nrand; ++q) {
        float sm[27] = {};
        const int rows = 7 + q % 60;
        const float scale = q % 3 == 0 ? 1.f : (q % 3 == 1 ? 1e-6f : 1e6f);
        for (int r = 0; r < rows; ++r) {
            float v[7];
            for (int k = 0; k < 7; ++k) v[k] = frand() * scale * (k < 3 ? 2.f : (k == 6 ? 0.02f : 1.f));
            int s2 = 0;
            for (int a = 0; a < 6; ++a) for (int c = a; c < 7; ++c) sm[s2++] += v[a] * v[c];
        }
        sys.insert(sys.end(), sm, sm + 27);
    }
    // degenerate: A = 0; rank 1..5 (fewer rows than unknowns); a zero row/column
    int ndeg = 0;
    for (int rank = 0; rank <= 5; ++rank)
        for (int rep = 0; rep < 40; ++rep) {
            float sm[27] = {};
            for (int r = 0; r < rank; ++r) {
                float v[7];
                for (int k = 0; k < 7; ++k) v[k] = frand();
                int s2 = 0;
                for (int a = 0; a < 6; ++a) for (int c = a; c < 7; ++c) sm[s2++] += v[a] * v[c];
            }
            if (rank == 0) for (int k = 0; k < 27; ++k) sm[k] = (rep == 0) ? 0.f : 0.f;
            sys.insert(sys.end(), sm, sm + 27);
            ++ndeg;
        }
    // equal singular values (the sort's tie path): scaled identities, diagonals with repeated
    // entries, permuted diagonals
    for (int rep = 0; rep < 60; ++rep) {
        float sm[27] = {};
        float d[6];
        for (int i = 0; i < 6; ++i) d[i] = 1.f + (float)((rep + i * (rep % 4)) % 3);
        if (rep % 5 == 0) for (int i = 0; i < 6; ++i) d[i] = 0.5f * (1 + rep);
        int s2 = 0;
        for (int a = 0; a < 6; ++a)
            for (int c = a; c < 7; ++c) sm[s2++] = c == 6 ? frand() : (a == c ? d[a] : 0.f);
        sys.insert(sys.end(), sm, sm + 27);
        ++ndeg;
    }
    const int n = (int)(sys.size() / 27);
    float *dS, *dX, *dO; int* dB; long long* dC;
    hipMalloc(&dS, sys.size() * 4); hipMalloc(&dX, (size_t)n * 6 * 4); hipMalloc(&dB, 4); hipMalloc(&dC, 16 * 8); hipMalloc(&dO, 64);
    hipMemcpy(dS, sys.data(), sys.size() * 4, hipMemcpyHostToDevice);
    unsigned long long z4[4] = {};
    for (int alg = 4; alg >= 2; alg -= 2) {
        hipMemset(dB, 0, 4);
#ifdef TF_SV_STATS
        hipMemcpyToSymbol(HIP_SYMBOL(g_sv_stats), z4, sizeof(z4));
#endif
        (void)z4;
        if (alg == 4) hipLaunchKernelGGL(k_check<4>, dim3(2048), dim3(64), 0, 0, dS, n, dX, dB);
        else hipLaunchKernelGGL(k_check<2>, dim3(2048), dim3(64), 0, 0, dS, n, dX, dB);
        int bad = -1;
        hipMemcpy(&bad, dB, 4, hipMemcpyDeviceToHost);
        unsigned long long st[4] = {};
#ifdef TF_SV_STATS
        hipMemcpyFromSymbol(st, HIP_SYMBOL(g_sv_stats), sizeof(st));
#endif
        printf("ALG %d: lanes vs serial GPU form: %d of %d systems differ (%d captured, %d random, %d degenerate)\n",
               alg, bad, n, ncap, nrand, ndeg);
        printf("  rotations %llu, fast-path fallbacks %llu (%.2e), zero-singular-value finishes %llu\n", st[0], st[1],
               st[0] ? (double)st[1] / (double)st[0] : 0.0, st[2]);
        if (alg == 4) {                      // the oracle (CPU) on every system
            std::vector<float> xl((size_t)n * 6);
            hipMemcpy(xl.data(), dX, xl.size() * 4, hipMemcpyDeviceToHost);
            tfo_set_pose_algebra(4, 0);
            int ob = 0, first = -1;
            for (int q = 0; q < n; ++q) {
                float A[36], b[6], x[6];
                int s2 = 0;
                for (int i = 0; i < 6; ++i)
                    for (int j = i; j < 7; ++j) {
                        const float v = sys[27 * (size_t)q + s2++];
                        if (j == 6) b[i] = v; else A[j * 6 + i] = A[i * 6 + j] = v;
                    }
                tfo_cv_solve_svd6(A, b, x);
                if (memcmp(x, &xl[6 * (size_t)q], 24)) { if (first < 0) first = q; ++ob; }
            }
            printf("  lanes vs oracle (tfo_cv_solve_svd6): %d of %d systems differ (first %d)\n", ob, n, first);
        }
    }
    const int N = 2000, ns = ncap > 0 ? (ncap < 256 ? ncap : 256) : 256;
    hipLaunchKernelGGL(k_time<0>, dim3(1), dim3(64), 0, 0, dS, ns, 20, dC, dO);
    hipLaunchKernelGGL(k_time<0>, dim3(1), dim3(64), 0, 0, dS, ns, N, dC, dO);
#ifdef TF_SV_TIMING
    {
        long long z8[8] = {};
        hipMemcpyToSymbol(HIP_SYMBOL(g_sv_t), z8, sizeof(z8));       // (the check kernels' stamps dropped)
    }
#endif
    hipLaunchKernelGGL(k_time<1>, dim3(1), dim3(64), 0, 0, dS, ns, 20, dC, dO);
    hipLaunchKernelGGL(k_time<1>, dim3(1), dim3(64), 0, 0, dS, ns, N, dC, dO);
    long long c[2];
    hipMemcpy(c, dC, sizeof(c), hipMemcpyDeviceToHost);
#ifdef TF_SV_TIMING
    {
        long long t[8];
        hipMemcpyFromSymbol(t, HIP_SYMBOL(g_sv_t), sizeof(t));
        const char* nm[8] = { "previous level end -> level start", "partner bpermute", "sums (DPP gather + fma)",
                              "test + ballot", "(c, s) chain + checks", "broadcast + update",
                              "after the sweeps: |row|, sort, gather", "normalise + back substitution" };
        printf("per-phase cycles per solve (timing build, stamps included):\n");
        for (int k = 0; k < 8; ++k) printf("  %-36s %9.1f\n", nm[k], (double)t[k] / (N + 20));
    }
#endif
    printf("latency over the first %d systems, one wave, dependent solves (s_memtime cycles per solve):\n", ns);
    printf("  serial  icp_cv_solve_svd6        %9.1f\n", (double)c[0] / N);
    printf("  lanes   icp_cv_solve_svd6_lanes  %9.1f   (%.2fx)\n", (double)c[1] / N, (double)c[0] / (double)c[1]);
    return 0;
}
