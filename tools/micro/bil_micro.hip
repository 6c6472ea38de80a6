// Bilateral pass in isolation (gfx950): k_dists_bilateral's tile body, the unrolled interior path
// (FAST) against the loop, 640x480 synthetic depth; per launch time from hipEvents and per
// workgroup duration (s_memrealtime, 100 MHz) to tell the workgroup's own latency from the grid's.
//   make -C tools/micro bil_micro && ./tools/micro/bil_micro
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "../../topfusion_amd/csrc/tf_preproc.h"

template <bool FAST>
__global__ void __launch_bounds__(256) k_bil(BilArgs b, unsigned long long* ts)
{
    __shared__ BilLds L;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    bilateral_block<FAST>(b, blockIdx.x, blockIdx.y, L);
    __syncthreads();
    if (threadIdx.x == 0) {
        const int w = blockIdx.y * gridDim.x + blockIdx.x;
        ts[2 * w] = t0;
        ts[2 * w + 1] = __builtin_amdgcn_s_memrealtime();
    }
}

// variant: 32x8 tiles, one pixel per thread, the 7x7 taps unrolled with dx pairs packed
// (dx = -3..2 in three pairs + dx = 3 alone), for 4x the waves of the pixel-pair layout
struct Lds8 { float f[8 + 2 * HALO][BIL_LD]; };
__global__ void __launch_bounds__(256) k_bil1(BilArgs b, unsigned long long* ts)
{
    __shared__ Lds8 L;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    const int x0 = blockIdx.x * 32, y0 = blockIdx.y * 8;
    for (int i = threadIdx.x; i < 14 * 38; i += 256) {
        const int ly = i / 38, lx = i % 38, gx = x0 + lx - HALO, gy = y0 + ly - HALO;
        const bool in = gx >= 0 && gx < b.W && gy >= 0 && gy < b.H;
        L.f[ly][lx] = in ? (float)b.src[gy * b.W + gx] : 0.f;
    }
    __syncthreads();
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5, x = x0 + tx, y = y0 + ty;
    const float* c0 = &L.f[ty + HALO][tx + HALO];
    const float v = c0[0];
    const tf_f2 vf = { v, v }, sdv = { b.sd, b.sd };
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int dy = -HALO; dy <= HALO; ++dy) {
#pragma unroll
        for (int dx = -HALO; dx <= HALO; dx += 2) {
            const float* q = c0 + dy * BIL_LD + dx;
            const bool two = dx + 1 <= HALO;
            const tf_f2 df = { q[0], two ? q[1] : 0.f };
            const float sp0 = (float)(dx * dx + dy * dy) * b.ss, sp1 = (float)((dx + 1) * (dx + 1) + dy * dy) * b.ss;
            const tf_f2 dd = vf - df;
            const tf_f2 w = bil_weight2((tf_f2){ sp0, sp1 } + dd * dd * sdv);
            const tf_f2 pr = df * w;
            s1 += pr.x; s2 += w.x;
            if (two) { s1 += pr.y; s2 += w.y; }
        }
    }
    if (x < b.W && y < b.H) bil_store(b, x, y, (int)v, s1, s2);
    __syncthreads();
    if (threadIdx.x == 0) {
        const int w = blockIdx.y * gridDim.x + blockIdx.x;
        ts[2 * w] = t0;
        ts[2 * w + 1] = __builtin_amdgcn_s_memrealtime();
    }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main()
{
    const int W = 640, H = 480;
    std::vector<uint16_t> h(W * H);
    unsigned s = 12345;
    for (int i = 0; i < W * H; ++i) { s = s * 1664525u + 1013904223u; h[i] = (uint16_t)(1200 + (i % W) / 2 + (s >> 28)); }
    uint16_t *src, *dst; float* dists; unsigned long long* ts;
    const dim3 grid((W + PRE_TX - 1) / PRE_TX, (H + PRE_TY - 1) / PRE_TY);
    const int nwg = grid.x * grid.y;
    CK(hipMalloc(&src, W * H * 2)); CK(hipMalloc(&dst, W * H * 2)); CK(hipMalloc(&dists, W * H * 4));
    CK(hipMalloc(&ts, 4 * nwg * 16));
    CK(hipMemcpy(src, h.data(), W * H * 2, hipMemcpyHostToDevice));
    BilArgs b;
    b.src = src; b.pitch = W * 2; b.W = W; b.H = H; b.ksz = 7;
    const float sdm = 0.04f * 1000.f;
    b.ss = 0.5f / (4.5f * 4.5f); b.sd = 0.5f / (sdm * sdm);
    b.do_trunc = 0; b.trunc_mm = 0; b.dists = dists; b.dst = dst;
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    std::vector<unsigned long long> t(2 * nwg);
    for (int v = 0; v < 3; ++v) {
        const dim3 g = v == 2 ? dim3((W + 31) / 32, (H + 7) / 8) : grid;
        const int nw = g.x * g.y;
        for (int rep = 0; rep < 3; ++rep) {
            const int N = 50;
            CK(hipEventRecord(e0, 0));
            for (int k = 0; k < N; ++k) {
                if (v == 0) hipLaunchKernelGGL(k_bil<true>, grid, dim3(256), 0, 0, b, ts);
                else if (v == 1) hipLaunchKernelGGL(k_bil<false>, grid, dim3(256), 0, 0, b, ts);
                else hipLaunchKernelGGL(k_bil1, g, dim3(256), 0, 0, b, ts);
            }
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1));
            t.resize(2 * nw);
            CK(hipMemcpy(t.data(), ts, nw * 16, hipMemcpyDeviceToHost));
            unsigned long long lo = ~0ull, hi = 0; double sum = 0, mx = 0;
            for (int w = 0; w < nw; ++w) {
                lo = t[2 * w] < lo ? t[2 * w] : lo; hi = t[2 * w + 1] > hi ? t[2 * w + 1] : hi;
                const double d = (double)(t[2 * w + 1] - t[2 * w]) * 0.01; sum += d; mx = d > mx ? d : mx;
            }
            printf("%s: %.2f us/launch (events, %d back to back); last launch span %.2f us, WG mean %.2f max %.2f us\n",
                   v == 0 ? "FAST" : (v == 1 ? "loop" : "1px "), 1000.f * ms / N, N, (double)(hi - lo) * 0.01, sum / nw, mx);
        }
    }
    return 0;
}
