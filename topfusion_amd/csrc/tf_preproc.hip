// tf_preproc.hip -- depth preprocessing front-end for gfx950.
//
//   k_dists_bilateral : compute_dists_kernel + bilateral_kernel + truncate_depth_kernel
//                       (imgproc.cu:10-89,263-290) fused; 32x8 tiles staged in LDS
//   k_pyr_down        : pyramid_kernel (imgproc.cu:98-140)
//   k_points_normals  : points_normals_kernel (imgproc.cu:214-254), all levels in one launch
//
// All three are HBM/L2-light elementwise-with-halo kernels; the bilateral filter is
// VALU-bound (49 canonical exp per pixel).
#include "tf_internal.h"
#include "tf_pose.h"

#define PRE_TX 32
#define PRE_TY 8
#define HALO 3

// one workgroup = one 32x8 tile; the 7x7 window's source pixels come from an LDS tile
// with a 3-pixel halo (the reference reads them through L1).
__global__ void __launch_bounds__(256)
k_dists_bilateral(const uint16_t* __restrict__ src, size_t pitch, int W, int H, int ksz,
                  float ss, float sd, int do_trunc, unsigned trunc_mm,
                  float* __restrict__ dists, uint16_t* __restrict__ dst)
{
    __shared__ uint16_t tile[PRE_TY + 2 * HALO][PRE_TX + 2 * HALO + 2];
    const int tx = threadIdx.x & (PRE_TX - 1), ty = threadIdx.x / PRE_TX;
    const int x0 = blockIdx.x * PRE_TX, y0 = blockIdx.y * PRE_TY;
    for (int i = threadIdx.x; i < (PRE_TY + 2 * HALO) * (PRE_TX + 2 * HALO); i += 256) {
        int ly = i / (PRE_TX + 2 * HALO), lx = i % (PRE_TX + 2 * HALO);
        int gx = x0 + lx - HALO, gy = y0 + ly - HALO;
        uint16_t v = 0;
        if (gx >= 0 && gx < W && gy >= 0 && gy < H)
            v = *(const uint16_t*)((const char*)src + (size_t)gy * pitch + (size_t)gx * 2);
        tile[ly][lx] = v;
    }
    __syncthreads();
    const int x = x0 + tx, y = y0 + ty;
    if (x >= W || y >= H) return;
    const int value = tile[ty + HALO][tx + HALO];
    // compute_dists_kernel (imgproc.cu:277)
    dists[y * W + x] = (value >= 2047 || value <= 0) ? -1.0f : (float)value * 0.001f;
    // bilateral_kernel (imgproc.cu:25-46): window [max(x-k/2,0), min(x-k/2+k, W-1))
    const int half = ksz / 2;
    int txe = x - half + ksz; if (txe > W - 1) txe = W - 1;
    int tye = y - half + ksz; if (tye > H - 1) tye = H - 1;
    const int cxs = x - half > 0 ? x - half : 0;
    const int cys = y - half > 0 ? y - half : 0;
    float sum1 = 0.f, sum2 = 0.f;
    for (int cy = cys; cy < tye; ++cy)
        for (int cx = cxs; cx < txe; ++cx) {
            int depth = tile[cy - y0 + HALO][cx - x0 + HALO];
            float space2 = (float)((x - cx) * (x - cx) + (y - cy) * (y - cy));
            unsigned dd = (unsigned)(value - depth);
            float color2 = (float)(int)(dd * dd);
            float weight = tf_exp(-(space2 * ss + color2 * sd));
            sum1 += (float)depth * weight;
            sum2 += weight;
        }
    float q = sum1 / sum2;
    int v = (q == q) ? (int)rintf(q) : 0;                 // __float2int_rn
    uint16_t out = (uint16_t)v;
    if (do_trunc && out > trunc_mm) out = 0;              // truncate_depth_kernel (imgproc.cu:76-77)
    dst[y * W + x] = out;
}

// pyramid_kernel (imgproc.cu:98-127)
__global__ void __launch_bounds__(256)
k_pyr_down(const uint16_t* __restrict__ src, int W, int H, uint16_t* __restrict__ dst, int DW, int DH, float sigma3)
{
    const int x = blockIdx.x * 32 + (threadIdx.x & 31), y = blockIdx.y * 8 + (threadIdx.x >> 5);
    if (x >= DW || y >= DH) return;
    const int D = 5;
    int center = src[(2 * y) * W + 2 * x];
    int txe = 2 * x - D / 2 + D; if (txe > W - 1) txe = W - 1;
    int tye = 2 * y - D / 2 + D; if (tye > H - 1) tye = H - 1;
    int sum = 0, count = 0;
    for (int cy = (2 * y - D / 2 > 0 ? 2 * y - D / 2 : 0); cy < tye; ++cy)
        for (int cx = (2 * x - D / 2 > 0 ? 2 * x - D / 2 : 0); cx < txe; ++cx) {
            int val = src[cy * W + cx];
            if ((float)abs(val - center) < sigma3) { sum += val; ++count; }
        }
    dst[y * DW + x] = (uint16_t)((count == 0) ? 0 : sum / count);
}

struct PtsLevels {
    const uint16_t* depth[TF_LEVELS];
    float4* pts[TF_LEVELS];
    float4* nrm[TF_LEVELS];
    int w[TF_LEVELS], h[TF_LEVELS];
    float fx[TF_LEVELS], fy[TF_LEVELS], cx[TF_LEVELS], cy[TF_LEVELS];
};

// points_normals_kernel (imgproc.cu:214-243); blockIdx.z = pyramid level
__global__ void __launch_bounds__(256)
k_points_normals(PtsLevels L)
{
    const int l = blockIdx.z;
    const int W = L.w[l], H = L.h[l];
    const int x = blockIdx.x * 32 + (threadIdx.x & 31), y = blockIdx.y * 8 + (threadIdx.x >> 5);
    if (x >= W || y >= H) return;
    const float qnan = tf_qnan();
    float4 p = make_float4(qnan, qnan, qnan, qnan), n = p;
    if (x < W - 1 && y < H - 1) {
        const uint16_t* d = L.depth[l];
        const float fxi = 1.f / L.fx[l], fyi = 1.f / L.fy[l], cx = L.cx[l], cy = L.cy[l];
        float z00 = (float)d[y * W + x] * 0.001f;
        float z01 = (float)d[y * W + x + 1] * 0.001f;
        float z10 = (float)d[(y + 1) * W + x] * 0.001f;
        if (z00 * z01 * z10 != 0) {
            tf3 v00 = mk3(z00 * ((float)x - cx) * fxi, z00 * ((float)y - cy) * fyi, z00);
            tf3 v01 = mk3(z01 * ((float)(x + 1) - cx) * fxi, z01 * ((float)y - cy) * fyi, z01);
            tf3 v10 = mk3(z10 * ((float)x - cx) * fxi, z10 * ((float)(y + 1) - cy) * fyi, z10);
            tf3 nn = knormalized(kcross(sub3(v01, v00), sub3(v10, v00)));
            n = make_float4(-nn.x, -nn.y, -nn.z, 1.0f);
            p = make_float4(v00.x, v00.y, v00.z, 1.0f);
        }
    }
    L.pts[l][y * W + x] = p;
    L.nrm[l][y * W + x] = n;
}

static inline int div_up(int a, int b) { return (a + b - 1) / b; }

hipError_t tfk_preprocess(tf_ctx* c, const uint16_t* depth, size_t pitch, hipStream_t strm)
{
    const tf_params& p = c->p;
    const int W = c->W, H = c->H;
    float sigma_depth = p.bilateral_sigma_depth * 1000.0f;       // meters -> mm (imgproc.cu:53)
    float ss = 0.5f / (p.bilateral_sigma_spatial * p.bilateral_sigma_spatial);
    float sd = 0.5f / (sigma_depth * sigma_depth);
    int do_trunc = p.icp_truncate_depth_dist > 0;
    unsigned trunc_mm = (unsigned)(uint16_t)(p.icp_truncate_depth_dist * 1000.f);   // imgproc.cu:87
    if (p.bilateral_kernel_size > 2 * HALO + 1) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_dists_bilateral, dim3(div_up(W, PRE_TX), div_up(H, PRE_TY)), dim3(256), 0, strm,
                       depth, pitch, W, H, p.bilateral_kernel_size, ss, sd, do_trunc, trunc_mm, c->dists, c->depth_pyr[0]);
    float sigma3 = sigma_depth * 3.0f;                                               // imgproc.cu:138
    for (int l = 1; l < TF_LEVELS; ++l)
        hipLaunchKernelGGL(k_pyr_down, dim3(div_up(c->lw[l], 32), div_up(c->lh[l], 8)), dim3(256), 0, strm,
                           c->depth_pyr[l - 1], c->lw[l - 1], c->lh[l - 1], c->depth_pyr[l], c->lw[l], c->lh[l], sigma3);
    PtsLevels L;
    for (int l = 0; l < TF_LEVELS; ++l) {
        int div = 1 << l;                                 // Intr::operator()(level), precomp.cpp:10-14
        L.depth[l] = c->depth_pyr[l]; L.pts[l] = c->curr_pts[l]; L.nrm[l] = c->curr_nrm[l];
        L.w[l] = c->lw[l]; L.h[l] = c->lh[l];
        L.fx[l] = p.fx / (float)div; L.fy[l] = p.fy / (float)div; L.cx[l] = p.cx / (float)div; L.cy[l] = p.cy / (float)div;
    }
    hipLaunchKernelGGL(k_points_normals, dim3(div_up(W, 32), div_up(H, 8), TF_LEVELS), dim3(256), 0, strm, L);
    return hipGetLastError();
}
