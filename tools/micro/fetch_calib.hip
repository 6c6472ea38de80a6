// FETCH_SIZE calibration for the integration pass's depth samples (not part of the product):
// scattered 4-byte gathers over a 640x480 float image from workgroups on every XCD, on one XCD,
// and banded by XCD, against a 16-B-per-lane stream of known size.  Run under
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace -- ./tools/micro/fetch_calib
// and compare each kernel's FETCH_SIZE with the byte counts it prints.
#include <hip/hip_runtime.h>
#include <cstdio>

#define W 640
#define H 480
#define NWG 768

__device__ __forceinline__ unsigned mix(unsigned x)
{
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

// mode 0: every workgroup samples the whole image; 1: workgroup b samples rows of band b % 8
// only (one band per XCD under round-robin dispatch); 2: only workgroups b % 8 == 0 run, whole
// image.  Each thread: 32 samples, 4 consecutive pixels per draw (the integration's x-run).
__global__ void __launch_bounds__(256) k_gather(const float* __restrict__ img, int mode, float* out)
{
    const int b = blockIdx.x;
    if (mode == 2 && (b & 7)) return;
    float acc = 0.f;
    const unsigned seed = (unsigned)(b * 256 + threadIdx.x) * 2654435761u;
#pragma unroll 1
    for (int j = 0; j < 8; ++j) {
        const unsigned r = mix(seed + j);
        int y = (int)(r % H), x = (int)((r >> 12) % (W - 4));
        if (mode == 1) y = (b & 7) * (H / 8) + (int)(r % (H / 8));
#pragma unroll
        for (int k = 0; k < 4; ++k) acc += img[y * W + x + k];
    }
    if (acc == 1234.5f) out[0] = acc;
}

__global__ void __launch_bounds__(256) k_stream(const uint4* __restrict__ p, size_t n, float* out)
{
    unsigned acc = 0;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) acc ^= p[i].x ^ p[i].w;
    if (acc == 0x12345u) out[0] = (float)acc;
}

int main()
{
    float *img, *out;
    uint4* big;
    const size_t nbig = (size_t)64 << 20;                 // 64 MiB streamed (and an L2 flush between runs)
    hipMalloc(&img, W * H * 4); hipMalloc(&out, 64); hipMalloc(&big, nbig);
    hipMemset(img, 0, W * H * 4); hipMemset(big, 1, nbig);
    const char* nm[3] = { "every XCD, whole image", "XCD-banded (1/8 image each)", "one XCD, whole image" };
    for (int m = 0; m < 3; ++m) {
        hipLaunchKernelGGL(k_stream, dim3(2048), dim3(256), 0, 0, big, nbig / 16, out);
        hipLaunchKernelGGL(k_gather, dim3(NWG), dim3(256), 0, 0, img, m, out);
        hipDeviceSynchronize();
        printf("k_gather mode %d (%s): image %d B\n", m, nm[m], W * H * 4);
    }
    printf("k_stream: %zu B per launch (4 launches, 16 B per lane)\n", nbig);
    hipLaunchKernelGGL(k_stream, dim3(2048), dim3(256), 0, 0, big, nbig / 16, out);
    hipDeviceSynchronize();
    return 0;
}
