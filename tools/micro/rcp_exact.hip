// Exhaustive check (gfx950): is a short reciprocal sequence -- v_rcp_f32 plus one fma Newton step
// -- equal, bit for bit, to the IEEE-correct 1.0f / z (-fhip-fp32-correctly-rounded-divide-sqrt)
// for every positive float?  If yes for a range, kernels may compute RN(1/z) that way there (the
// canonical value is still RN(1/z); the oracle computes 1.0f / z).
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt
//         -fno-gpu-flush-denormals-to-zero rcp_exact.hip -o rcp_exact   (tools/micro/Makefile)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>

__device__ __forceinline__ float rcp_nr1(float z)
{
    const float r0 = __builtin_amdgcn_rcpf(z);
    const float e = __builtin_fmaf(-z, r0, 1.0f);
    return __builtin_fmaf(e, r0, r0);
}

__device__ __forceinline__ float rcp_nr2(float z)
{
    const float r1 = rcp_nr1(z);
    const float e = __builtin_fmaf(-z, r1, 1.0f);
    return __builtin_fmaf(e, r1, r1);
}

// bins: exponent field of z (0 = subnormal, 1..254 normal); per bin mismatch counts of each form
__global__ void k_check(unsigned long long* mism1, unsigned long long* mism2, unsigned* first1, unsigned base)
{
    const unsigned b = base + blockIdx.x * blockDim.x + threadIdx.x;
    if (b == 0 || b >= 0x7f800000u) return;                 // positive finite, non-zero
    const float z = __uint_as_float(b);
    const float ref = 1.0f / z;
    const unsigned rb = __float_as_uint(ref);
    const unsigned e = b >> 23;
    if (__float_as_uint(rcp_nr1(z)) != rb) {
        atomicAdd(&mism1[e], 1ull);
        atomicMin(&first1[e], b);
    }
    if (__float_as_uint(rcp_nr2(z)) != rb) atomicAdd(&mism2[e], 1ull);
}

int main()
{
    unsigned long long *d1, *d2; unsigned* df;
    hipMalloc(&d1, 256 * 8); hipMalloc(&d2, 256 * 8); hipMalloc(&df, 256 * 4);
    hipMemset(d1, 0, 256 * 8); hipMemset(d2, 0, 256 * 8); hipMemset(df, 0xff, 256 * 4);
    const unsigned chunk = 1u << 28;
    for (unsigned base = 0; base < 0x7f800000u; base += chunk) {
        hipLaunchKernelGGL(k_check, dim3(chunk / 256), dim3(256), 0, 0, d1, d2, df, base);
    }
    hipDeviceSynchronize();
    unsigned long long h1[256], h2[256]; unsigned hf[256];
    hipMemcpy(h1, d1, sizeof(h1), hipMemcpyDeviceToHost);
    hipMemcpy(h2, d2, sizeof(h2), hipMemcpyDeviceToHost);
    hipMemcpy(hf, df, sizeof(hf), hipMemcpyDeviceToHost);
    unsigned long long t1 = 0, t2 = 0, n1 = 0, n2 = 0;
    for (int e = 0; e < 255; ++e) {
        t1 += h1[e]; t2 += h2[e];
        if (e >= 1 && e <= 253) { n1 += h1[e]; n2 += h2[e]; }
        if (h1[e] || h2[e]) {
            float f; unsigned u = hf[e]; std::memcpy(&f, &u, 4);
            printf("exponent field %3d: rcp+1NR mismatches %llu (first z = %a), rcp+2NR mismatches %llu\n", e, h1[e], f, h2[e]);
        }
    }
    printf("all positive finite floats: rcp+1NR %llu mismatches, rcp+2NR %llu; normal z with exponent field 1..253: %llu / %llu\n",
           t1, t2, n1, n2);
    return 0;
}
