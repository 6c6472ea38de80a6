// Dependent-launch gaps on one stream by the NEXT kernel's shape (micro-benchmark, not product):
// a writer kernel, then kernels differing in one property each; rocprofv3 --kernel-trace gives
// the end -> start gaps (tools/micro/launch_gap.py).
//   hipcc -O3 --offload-arch=gfx950 tools/micro/launch_gap.hip -o tools/micro/launch_gap
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void __launch_bounds__(256) k_write(float* p, int n)
{
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) p[i] = (float)i;
}
__global__ void __launch_bounds__(256) k_small(float* p) { if (threadIdx.x == 0) p[blockIdx.x] += 1.0f; }
__global__ void __launch_bounds__(256) k_lds32k(float* p)
{
    __shared__ float s[8192];
    s[threadIdx.x * 32] = p[blockIdx.x];
    __syncthreads();
    if (threadIdx.x == 0) p[blockIdx.x] = s[255 * 32] + 1.0f;
}
__global__ void __launch_bounds__(1024) k_wg1024(float* p) { if (threadIdx.x == 0) p[blockIdx.x] += 1.0f; }
struct Big { float v[150]; };
__global__ void __launch_bounds__(256) k_bigarg(float* p, Big b) { if (threadIdx.x == 0) p[blockIdx.x] += b.v[blockIdx.x % 150]; }
__global__ void k_spin(long long cycles)
{   // holds the queue so the host has enqueued everything before the measured kernels run
    const long long t0 = clock64();
    while (clock64() - t0 < cycles) __builtin_amdgcn_s_sleep(100);
}
__global__ void __launch_bounds__(256) k_many(float* p) { if (threadIdx.x == 0) p[blockIdx.x] += 1.0f; }

int main()
{
    float* p;
    hipMalloc(&p, 64 << 20);
    Big b{};
    hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, 0, 200000000LL);
    for (int rep = 0; rep < 200; ++rep) {
        hipLaunchKernelGGL(k_write, dim3(1024), dim3(256), 0, 0, p, 1 << 20);
        hipLaunchKernelGGL(k_small, dim3(288), dim3(256), 0, 0, p);
        hipLaunchKernelGGL(k_small, dim3(288), dim3(256), 0, 0, p);
        hipLaunchKernelGGL(k_lds32k, dim3(288), dim3(256), 0, 0, p);
        hipLaunchKernelGGL(k_small, dim3(288), dim3(256), 0, 0, p);
        hipLaunchKernelGGL(k_wg1024, dim3(68), dim3(1024), 0, 0, p);
        hipLaunchKernelGGL(k_small, dim3(288), dim3(256), 0, 0, p);
        hipLaunchKernelGGL(k_bigarg, dim3(288), dim3(256), 0, 0, p, b);
        hipLaunchKernelGGL(k_small, dim3(288), dim3(256), 0, 0, p);
        hipLaunchKernelGGL(k_many, dim3(2400), dim3(256), 0, 0, p);
        hipLaunchKernelGGL(k_small, dim3(288), dim3(256), 0, 0, p);
    }
    hipDeviceSynchronize();
    printf("done\n");
    return 0;
}
