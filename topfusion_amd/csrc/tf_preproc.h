// tf_preproc.h -- the depth preprocessing front-end's per-workgroup bodies,
// shared by its own kernels (tf_preproc.hip) and by the frame kernels that run later frames'
// preprocessing in their grid's tail when a batch supplies them (k_raycast_pair: the next
// frame's computeDists + pyramids + normals and the bilateral pass of the one after;
// k_alloc_requests: a bilateral pass at the batch start; tf_capi.hip enqueue_frame).
#pragma once
#include "tf_internal.h"
#include "tf_pose.h"

// compute_dists_kernel (imgproc.cu:277)
__device__ __forceinline__ float tf_dist_of(int value)
{
    return (value >= 2047 || value <= 0) ? -1.0f : (float)value * 0.001f;
}

typedef float tf_f2 __attribute__((ext_vector_type(2)));   // packed f32 pair (v_pk_* on gfx950)

#define PRE_TX 32
#define PRE_TY 8
#define HALO 3

// one workgroup = one 32x8 tile; the 7x7 window's source pixels come from an LDS tile
// with a 3-pixel halo (the reference reads them through L1).
struct BilArgs {
    const uint16_t* src; size_t pitch;  // raw depth (pitched)
    int W, H, ksz;
    float ss, sd;
    int do_trunc; unsigned trunc_mm;
    float* dists;                       // computeDists output (nullptr: not written here)
    uint16_t* dst;                      // level-0 depth (bilateral + truncation)
};

// the bilateral pass's LDS (a caller-provided block, so a fused kernel can overlay it with the
// LDS of its other branches)
struct BilLds {
    uint16_t tile[PRE_TY + 2 * HALO][PRE_TX + 2 * HALO + 2];
    float ftile[PRE_TY + 2 * HALO][PRE_TX + 2 * HALO + 2];
    float sptab[2 * HALO + 1][2 * HALO + 2];      // RN(space2 * ss) by (y-cy+3, x-cx+3)
};

// tile (bx, by) of k_dists_bilateral; every thread of the workgroup calls it
__device__ __forceinline__ void bilateral_block(const BilArgs& b, int bx, int by, BilLds& L)
{
    const uint16_t* __restrict__ src = b.src;
    const size_t pitch = b.pitch;
    const int W = b.W, H = b.H, ksz = b.ksz;
    const float ss = b.ss, sd = b.sd;
    float* __restrict__ dists = b.dists;
    uint16_t* __restrict__ dst = b.dst;
    auto& tile = L.tile;
    auto& ftile = L.ftile;
    auto& sptab = L.sptab;
    const int tx = threadIdx.x & (PRE_TX - 1), ty = threadIdx.x / PRE_TX;
    const int x0 = bx * PRE_TX, y0 = by * PRE_TY;
    bool big = false;
    {   // every load of the tile first (clamped to pixel 0 outside the image), then the LDS
        // writes: one memory round trip instead of one per element
        constexpr int NT = (PRE_TY + 2 * HALO) * (PRE_TX + 2 * HALO), PER = (NT + 255) / 256;
        uint16_t vals[PER];
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int i = threadIdx.x + 256 * k;
            const int ly = i / (PRE_TX + 2 * HALO), lx = i % (PRE_TX + 2 * HALO);
            const int gx = x0 + lx - HALO, gy = y0 + ly - HALO;
            const bool in = i < NT && gx >= 0 && gx < W && gy >= 0 && gy < H;
            const uint16_t v = *(const uint16_t*)((const char*)src + (in ? (size_t)gy * pitch + (size_t)gx * 2 : 0));
            vals[k] = in ? v : (uint16_t)0;
        }
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int i = threadIdx.x + 256 * k;
            if (i < NT) {
                const int ly = i / (PRE_TX + 2 * HALO), lx = i % (PRE_TX + 2 * HALO);
                tile[ly][lx] = vals[k];
                ftile[ly][lx] = (float)vals[k];
                big = big || vals[k] >= 46341;
            }
        }
    }
    if (threadIdx.x < (2 * HALO + 1) * (2 * HALO + 1)) {
        const int dy = threadIdx.x / (2 * HALO + 1) - HALO, dx = threadIdx.x % (2 * HALO + 1) - HALO;
        sptab[dy + HALO][dx + HALO] = (float)(dx * dx + dy * dy) * ss;
    }
    // a depth difference of 46341 or more squares past INT_MAX, which the reference's int
    // arithmetic wraps: such tiles take the integer loop
    big = __syncthreads_or(big);
    const int x = x0 + tx, y = y0 + ty;
    if (x >= W || y >= H) return;
    const int value = tile[ty + HALO][tx + HALO];
    // compute_dists_kernel (imgproc.cu:277)
    if (dists) dists[y * W + x] = tf_dist_of(value);
    // bilateral_kernel (imgproc.cu:25-46): window [max(x-k/2,0), min(x-k/2+k, W-1))
    const int half = ksz / 2;
    int txe = x - half + ksz; if (txe > W - 1) txe = W - 1;
    int tye = y - half + ksz; if (tye > H - 1) tye = H - 1;
    const int cxs = x - half > 0 ? x - half : 0;
    const int cys = y - half > 0 ? y - half : 0;
    float sum1 = 0.f, sum2 = 0.f;
    if (!big) {
        // two taps per step in packed f32 (v_pk_*): the same operations per tap as the integer
        // loop below -- space2 * ss from the table, color2 = RN(d * d) == (float)(int)(d * d)
        // for |d| < 46341, tf_exp's own steps (its t >= 128 branch cannot occur: the argument
        // is <= 0) -- and the sums accumulated tap by tap in the reference's order
        const tf_f2 vf = { (float)value, (float)value }, sdv = { sd, sd }, nl2e = { -1.44269504088896341f, -1.44269504088896341f };
        for (int cy = cys; cy < tye; ++cy) {
            const float* frow = &ftile[cy - y0 + HALO][0];
            const float* srow = &sptab[y - cy + HALO][0];
            for (int cx = cxs; cx < txe; cx += 2) {
                const bool two = cx + 1 < txe;
                const tf_f2 df = { frow[cx - x0 + HALO], frow[cx + 1 - x0 + HALO] };
                const tf_f2 spp = { srow[x - cx + HALO], srow[x - cx - 1 + HALO + (two ? 0 : 1)] };
                const tf_f2 dd = vf - df;
                const tf_f2 c2 = dd * dd;
                const tf_f2 arg = spp + c2 * sdv;
                const tf_f2 t = arg * nl2e;                       // == (-arg) * log2(e)
                const float k0 = rintf(t.x), k1 = rintf(t.y);
                const tf_f2 k = { k0, k1 };
                const tf_f2 f = t - k;
                tf_f2 pp = { 1.5403530393381606e-4f, 1.5403530393381606e-4f };
                pp = __builtin_elementwise_fma(pp, f, (tf_f2){ 1.3333558146428443e-3f, 1.3333558146428443e-3f });
                pp = __builtin_elementwise_fma(pp, f, (tf_f2){ 9.6181291076284772e-3f, 9.6181291076284772e-3f });
                pp = __builtin_elementwise_fma(pp, f, (tf_f2){ 5.5504108664821580e-2f, 5.5504108664821580e-2f });
                pp = __builtin_elementwise_fma(pp, f, (tf_f2){ 2.4022650695910071e-1f, 2.4022650695910071e-1f });
                pp = __builtin_elementwise_fma(pp, f, (tf_f2){ 6.9314718055994531e-1f, 6.9314718055994531e-1f });
                pp = __builtin_elementwise_fma(pp, f, (tf_f2){ 1.0f, 1.0f });
                const float w0 = (t.x > -125.0f) ? ldexpf(pp.x, (int)k0) : 0.0f;
                const float w1 = (t.y > -125.0f) ? ldexpf(pp.y, (int)k1) : 0.0f;
                const tf_f2 w = { w0, w1 };
                const tf_f2 prod = df * w;
                sum1 += prod.x; sum2 += w.x;
                if (two) { sum1 += prod.y; sum2 += w.y; }
            }
        }
    } else {
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
    }
    float q = sum1 / sum2;
    int v = (q == q) ? (int)rintf(q) : 0;                 // __float2int_rn
    uint16_t out = (uint16_t)v;
    if (b.do_trunc && out > b.trunc_mm) out = 0;              // truncate_depth_kernel (imgproc.cu:76-77)
    dst[y * W + x] = out;
}

// pyramid_kernel (imgproc.cu:98-127) on a source staged in LDS: destination pixel (x, y) of a
// level whose source is sw x sh; the source sample (gx, gy) lives at lds[(gy - oy) * ld + gx - ox]
template <typename T>
__device__ __forceinline__ int pyr_pixel(const T* lds, int ld, int ox, int oy, int sw, int sh, int x, int y, float sigma3)
{
    const int D = 5;
    const int center = lds[(2 * y - oy) * ld + 2 * x - ox];
    int txe = 2 * x - D / 2 + D; if (txe > sw - 1) txe = sw - 1;
    int tye = 2 * y - D / 2 + D; if (tye > sh - 1) tye = sh - 1;
    int sum = 0, count = 0;
    for (int cy = (2 * y - D / 2 > 0 ? 2 * y - D / 2 : 0); cy < tye; ++cy)
        for (int cx = (2 * x - D / 2 > 0 ? 2 * x - D / 2 : 0); cx < txe; ++cx) {
            const int val = lds[(cy - oy) * ld + cx - ox];
            if ((float)abs(val - center) < sigma3) { sum += val; ++count; }
        }
    return (count == 0) ? 0 : sum / count;
}

struct PyrArgs {
    const uint16_t* raw; size_t raw_pitch;   // raw depth for computeDists (nullptr: not written here)
    float* dists;
    const uint16_t* d0;                 // level-0 depth (bilateral + truncation output)
    uint16_t* d1; uint16_t* d2;         // levels 1, 2
    float4* pts[TF_LEVELS];
    float4* nrm[TF_LEVELS];
    int w[TF_LEVELS], h[TF_LEVELS];
    float fx[TF_LEVELS], fy[TF_LEVELS], cx[TF_LEVELS], cy[TF_LEVELS];
    float sigma3;
};

// points_normals_kernel (imgproc.cu:214-243) for level pixel (x, y), depths from LDS
template <typename T>
__device__ __forceinline__ void pn_pixel(const T* lds, int ld, int ox, int oy, const PyrArgs& a, int l, int x, int y)
{
    const int W = a.w[l], H = a.h[l];
    const float qnan = tf_qnan();
    float4 p = make_float4(qnan, qnan, qnan, qnan), n = p;
    if (x < W - 1 && y < H - 1) {
        const float fxi = 1.f / a.fx[l], fyi = 1.f / a.fy[l], cx = a.cx[l], cy = a.cy[l];
        const int i = (y - oy) * ld + x - ox;
        float z00 = (float)lds[i] * 0.001f;
        float z01 = (float)lds[i + 1] * 0.001f;
        float z10 = (float)lds[i + ld] * 0.001f;
        if (z00 * z01 * z10 != 0) {
            tf3 v00 = mk3(z00 * ((float)x - cx) * fxi, z00 * ((float)y - cy) * fyi, z00);
            tf3 v01 = mk3(z01 * ((float)(x + 1) - cx) * fxi, z01 * ((float)y - cy) * fyi, z01);
            tf3 v10 = mk3(z10 * ((float)x - cx) * fxi, z10 * ((float)(y + 1) - cy) * fyi, z10);
            tf3 nn = knormalized(kcross(sub3(v01, v00), sub3(v10, v00)));
            n = make_float4(-nn.x, -nn.y, -nn.z, 1.0f);
            p = make_float4(v00.x, v00.y, v00.z, 1.0f);
        }
    }
    a.pts[l][y * W + x] = p;
    a.nrm[l][y * W + x] = n;
}

// depthBuildPyramid x2 + computePointNormals x3 (imgproc.cpp:12-41) in one launch.  A workgroup
// owns a 32x32 level-0 tile (16x16 at level 1, 8x8 at level 2) and stages what its outputs
// read: level 0 over the tile +6/+7 pixels (the level-1 windows of the level-2 windows and the
// normals' +1 neighbours), level 1 over its tile -2..+18, level 2 over its tile +1.  The few
// level-1 values next to a tile are computed by both neighbours (identical arithmetic).
#define PN_T0 32
#define PN_R0 45                       // level-0 staging: [X0-6, X0+39)
#define PN_R1 21                       // level-1 staging: [X1-2, X1+19)
#define PN_R2 9                        // level-2 staging: [X2, X2+9)
struct PnLds {
    uint16_t s0[PN_R0 * PN_R0];
    int s1[PN_R1 * PN_R1];
    int s2[PN_R2 * PN_R2];
};
__device__ __forceinline__ void pyr_normals_block(const PyrArgs& a, int bx, int by, PnLds& L)
{
    uint16_t* s0 = L.s0;
    int* s1 = L.s1;
    int* s2 = L.s2;
    const int W0 = a.w[0], H0 = a.h[0], W1 = a.w[1], H1 = a.h[1], W2 = a.w[2], H2 = a.h[2];
    const int X0 = bx * PN_T0, Y0 = by * PN_T0;
    const int X1 = X0 / 2, Y1 = Y0 / 2, X2 = X0 / 4, Y2 = Y0 / 4;
    const int o0x = X0 - 6, o0y = Y0 - 6, o1x = X1 - 2, o1y = Y1 - 2;
    {   // all loads of the staging tile first (clamped), then the LDS writes: one round trip
        constexpr int PER = (PN_R0 * PN_R0 + 255) / 256;
        uint16_t vals[PER];
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int i = threadIdx.x + 256 * k;
            const int gy = o0y + i / PN_R0, gx = o0x + i % PN_R0;
            const bool in = i < PN_R0 * PN_R0 && gx >= 0 && gx < W0 && gy >= 0 && gy < H0;
            const uint16_t v = a.d0[in ? gy * W0 + gx : 0];
            vals[k] = in ? v : (uint16_t)0;
        }
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int i = threadIdx.x + 256 * k;
            if (i < PN_R0 * PN_R0) s0[i] = vals[k];
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < PN_R1 * PN_R1; i += 256) {
        const int y = o1y + i / PN_R1, x = o1x + i % PN_R1;
        int v = 0;
        if (x >= 0 && x < W1 && y >= 0 && y < H1) {
            v = pyr_pixel(s0, PN_R0, o0x, o0y, W0, H0, x, y, a.sigma3);
            if (x >= X1 && x < X1 + 16 && y >= Y1 && y < Y1 + 16) a.d1[y * W1 + x] = (uint16_t)v;
        }
        s1[i] = v;
    }
    __syncthreads();
    if (threadIdx.x < PN_R2 * PN_R2) {
        const int y = Y2 + threadIdx.x / PN_R2, x = X2 + threadIdx.x % PN_R2;
        int v = 0;
        if (x < W2 && y < H2) {
            v = pyr_pixel(s1, PN_R1, o1x, o1y, W1, H1, x, y, a.sigma3);
            if (x < X2 + 8 && y < Y2 + 8) a.d2[y * W2 + x] = (uint16_t)v;
        }
        s2[threadIdx.x] = v;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) {                       // level 0: 32x32, four rows of 8 per thread
        const int t = threadIdx.x + 256 * q;
        const int x = X0 + (t & 31), y = Y0 + (t >> 5);
        if (x < W0 && y < H0) {
            pn_pixel(s0, PN_R0, o0x, o0y, a, 0, x, y);
            if (a.raw) a.dists[y * W0 + x] = tf_dist_of(*(const uint16_t*)((const char*)a.raw + (size_t)y * a.raw_pitch + (size_t)x * 2));
        }
    }
    {
        const int x = X1 + (threadIdx.x & 15), y = Y1 + (threadIdx.x >> 4);
        if (x < W1 && y < H1) pn_pixel(s1, PN_R1, o1x, o1y, a, 1, x, y);
    }
    if (threadIdx.x < 64) {
        const int x = X2 + (threadIdx.x & 7), y = Y2 + (threadIdx.x >> 3);
        if (x < W2 && y < H2) pn_pixel(s2, PN_R2, X2, Y2, a, 2, x, y);
    }
}


static inline int tf_div_up(int a, int b) { return (a + b - 1) / b; }
hipError_t tf_pre_args(tf_ctx* c, const uint16_t* depth, size_t pitch, int lookahead, uint16_t* d0, BilArgs* b, PyrArgs* a);
