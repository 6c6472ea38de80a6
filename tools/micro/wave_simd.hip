// Which SIMD does each wave of a 512-thread workgroup land on (gfx950)?  The persistent ICP
// kernel's grid shape (256 workgroups x 8 waves, 56 KiB dynamic LDS: one workgroup per CU);
// HW_REG_HW_ID's SIMD_ID field per wave, histogrammed over all workgroups.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void __launch_bounds__(512) k_where(unsigned* out)
{
    extern __shared__ float pad[];
    unsigned hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 8 + (threadIdx.x >> 6)] = hw;
    if (threadIdx.x == 1023) pad[0] = 0.f;           // (never: keeps the LDS allocation)
}
int main()
{
    unsigned* d;
    hipMalloc(&d, 256 * 8 * 4);
    unsigned h[256 * 8];
    int hist[8][4] = {};
    int pattern_rr = 0, pattern_packed = 0, other = 0;
    for (int rep = 0; rep < 10; ++rep) {
        hipLaunchKernelGGL(k_where, dim3(256), dim3(512), 56 * 1024, 0, d);
        hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
        for (int b = 0; b < 256; ++b) {
            bool rr = true, pk = true;
            for (int w = 0; w < 8; ++w) {
                const int s = (h[b * 8 + w] >> 4) & 3;
                hist[w][s]++;
                rr = rr && s == (w & 3);
                pk = pk && s == (w >> 1);
            }
            pattern_rr += rr; pattern_packed += pk; other += !rr && !pk;
        }
    }
    for (int w = 0; w < 8; ++w) printf("wave %d: simd0 %5d simd1 %5d simd2 %5d simd3 %5d\n", w, hist[w][0], hist[w][1], hist[w][2], hist[w][3]);
    printf("workgroups: round-robin (w %% 4) %d, packed (w / 2) %d, other %d\n", pattern_rr, pattern_packed, other);
    printf("example hw_id of workgroup 0: ");
    for (int w = 0; w < 8; ++w) printf("%08x ", h[w]);
    printf("\n");
    return 0;
}
