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

// one workgroup = one 32x8 tile, one pixel per thread; the 7x7 window's source pixels come from
// an LDS tile with a 3-pixel halo (the reference reads them through L1).
struct BilArgs {
    const uint16_t* src; size_t pitch;  // raw depth (pitched)
    int W, H, ksz;
    float ss, sd;
    int do_trunc; unsigned trunc_mm;
    float* dists;                       // computeDists output (nullptr: not written here)
    uint16_t* dst;                      // level-0 depth (bilateral + truncation)
};

#define BIL_LD (PRE_TX + 2 * HALO + 2)  // LDS row stride (floats / u16)
// the bilateral pass's LDS (a caller-provided block, so a fused kernel can overlay it with the
// LDS of its other branches)
struct BilLds {
    uint16_t tile[PRE_TY + 2 * HALO][BIL_LD];
    float ftile[PRE_TY + 2 * HALO][BIL_LD];
    float sptab[2 * HALO + 1][2 * HALO + 2];      // RN(space2 * ss) by (y-cy+3, x-cx+3)
};

// canonical exp of -arg for two taps (tf_exp's own steps; its t >= 128 branch cannot occur: the
// argument is <= 0)
__device__ __forceinline__ tf_f2 bil_weight2(tf_f2 arg)
{
    const tf_f2 nl2e = { -1.44269504088896341f, -1.44269504088896341f };
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
    return (tf_f2){ w0, w1 };
}

// the pixel's final steps: dists (compute_dists_kernel, imgproc.cu:277), the normalisation and
// __float2int_rn (imgproc.cu:43-45), truncate_depth_kernel (imgproc.cu:76-77)
__device__ __forceinline__ void bil_store(const BilArgs& b, int x, int y, int value, float sum1, float sum2)
{
    if (b.dists) b.dists[y * b.W + x] = tf_dist_of(value);
    const float q = sum1 / sum2;
    const int v = (q == q) ? (int)rintf(q) : 0;
    uint16_t out = (uint16_t)v;
    if (b.do_trunc && out > b.trunc_mm) out = 0;
    b.dst[y * b.W + x] = out;
}

// the unrolled 7x7 window for the thread's pixel (x0 + tx, y0 + ty), taps (dx, dx + 1) as the two
// halves of packed f32 operations (dx = 3 alone); MASK: the window is clamped at the image border
// (taps outside it weigh 0)
template <bool MASK>
__device__ __forceinline__ void bil_taps7(const BilArgs& b, const BilLds& L, int tx, int ty, int x0, int y0)
{
    const int x = x0 + tx, y = y0 + ty;
    const float* c0 = &L.ftile[ty + HALO][tx + HALO];
    const float v = c0[0];
    const tf_f2 vf = { v, v }, sdv = { b.sd, b.sd };
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int dy = -HALO; dy <= HALO; ++dy) {
        const bool rok = !MASK || (y + dy >= 0 && y + dy < b.H - 1);
#pragma unroll
        for (int dx = -HALO; dx <= HALO; dx += 2) {
            const bool two = dx + 1 <= HALO;
            const float* q = c0 + dy * BIL_LD + dx;
            const tf_f2 df = { q[0], two ? q[1] : 0.f };
            const float sp0 = (float)(dx * dx + dy * dy) * b.ss;
            const float sp1 = (float)((dx + 1) * (dx + 1) + dy * dy) * b.ss;
            const tf_f2 dd = vf - df;
            tf_f2 w = bil_weight2((tf_f2){ sp0, sp1 } + dd * dd * sdv);
            if (MASK) {
                const bool c0k = x + dx >= 0 && x + dx < b.W - 1, c1k = x + dx + 1 >= 0 && x + dx + 1 < b.W - 1;
                w = (tf_f2){ (rok && c0k) ? w.x : 0.f, (rok && c1k) ? w.y : 0.f };
            }
            const tf_f2 pr = df * w;
            s1 += pr.x; s2 += w.x;
            if (two) { s1 += pr.y; s2 += w.y; }
        }
    }
    if (x < b.W && y < b.H) bil_store(b, x, y, (int)L.tile[ty + HALO][tx + HALO], s1, s2);
}

// tile (bx, by) of k_dists_bilateral; every thread of the workgroup calls it.  FAST: the unrolled
// interior path (86 VGPRs; the grid tails of the 64-VGPR frame kernels run the loop only)
template <bool FAST>
__device__ __forceinline__ void bilateral_block(const BilArgs& b, int bx, int by, BilLds& L)
{
    const uint16_t* __restrict__ src = b.src;
    const size_t pitch = b.pitch;
    const int W = b.W, H = b.H, ksz = b.ksz;
    const float ss = b.ss, sd = b.sd;
    auto& tile = L.tile;
    auto& ftile = L.ftile;
    auto& sptab = L.sptab;
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
    const int tx = threadIdx.x & (PRE_TX - 1), ty = threadIdx.x / PRE_TX;
    const int x = x0 + tx;
    // bilateral_kernel (imgproc.cu:25-46): window [max(x-k/2,0), min(x-k/2+k, W-1)).  With the
    // default 7-tap window the taps run unrolled, two taps per packed f32 operation: each tap sees
    // exactly the operations of the loop below, in the reference's row-major order, and the
    // spatial term is a compile-time tap constant.  A tile whose every window is the full 7x7
    // (x-3 >= 0 and x+4 <= W-1, the same in y) needs no test; at the image border a tap outside
    // the clamped window gets weight 0, which leaves both sums bit-identical to skipping it (they
    // are +0 or positive, depth * 0 = +0)
    if (FAST && !big && ksz == 7) {
        if (x0 >= HALO && y0 >= HALO && x0 + PRE_TX + HALO <= W - 1 && y0 + PRE_TY + HALO <= H - 1)
            bil_taps7<false>(b, L, tx, ty, x0, y0);
        else
            bil_taps7<true>(b, L, tx, ty, x0, y0);
        return;
    }
    const int half = ksz / 2;
    {
        const int y = y0 + ty;
        if (x >= W || y >= H) return;
        const int value = tile[ty + HALO][tx + HALO];
        int txe = x - half + ksz; if (txe > W - 1) txe = W - 1;
        int tye = y - half + ksz; if (tye > H - 1) tye = H - 1;
        const int cxs = x - half > 0 ? x - half : 0;
        const int cys = y - half > 0 ? y - half : 0;
        float sum1 = 0.f, sum2 = 0.f;
        if (!big) {
            // two taps per step in packed f32 (v_pk_*): the same operations per tap as the integer
            // loop below -- space2 * ss from the table, color2 = RN(d * d) == (float)(int)(d * d)
            // for |d| < 46341 -- and the sums accumulated tap by tap in the reference's order
            const tf_f2 vf = { (float)value, (float)value }, sdv = { sd, sd };
            for (int cy = cys; cy < tye; ++cy) {
                const float* frow = &ftile[cy - y0 + HALO][0];
                const float* srow = &sptab[y - cy + HALO][0];
                for (int cx = cxs; cx < txe; cx += 2) {
                    const bool two = cx + 1 < txe;
                    const tf_f2 df = { frow[cx - x0 + HALO], frow[cx + 1 - x0 + HALO] };
                    const tf_f2 spp = { srow[x - cx + HALO], srow[x - cx - 1 + HALO + (two ? 0 : 1)] };
                    const tf_f2 dd = vf - df;
                    const tf_f2 c2 = dd * dd;
                    const tf_f2 w = bil_weight2(spp + c2 * sdv);
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
        bil_store(b, x, y, value, sum1, sum2);
    }
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
// NT threads per workgroup: 256 in the grid tails of the frame kernels, 1024 in k_pyr_normals
// (the per-call path, where the pass is on the frame's critical path: one level-0 pixel per
// thread, 4x the waves in flight)
template <int NT>
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
        constexpr int PER = (PN_R0 * PN_R0 + NT - 1) / NT;
        uint16_t vals[PER];
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int i = threadIdx.x + NT * k;
            const int gy = o0y + i / PN_R0, gx = o0x + i % PN_R0;
            const bool in = i < PN_R0 * PN_R0 && gx >= 0 && gx < W0 && gy >= 0 && gy < H0;
            const uint16_t v = a.d0[in ? gy * W0 + gx : 0];
            vals[k] = in ? v : (uint16_t)0;
        }
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int i = threadIdx.x + NT * k;
            if (i < PN_R0 * PN_R0) s0[i] = vals[k];
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < PN_R1 * PN_R1; i += NT) {
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
    // the normals: 1024 level-0, 256 level-1 and 64 level-2 pixels, dealt over the threads
    for (int t = threadIdx.x; t < 1024 + 256 + 64; t += NT) {
        if (t < 1024) {
            const int x = X0 + (t & 31), y = Y0 + (t >> 5);
            if (x < W0 && y < H0) {
                pn_pixel(s0, PN_R0, o0x, o0y, a, 0, x, y);
                if (a.raw) a.dists[y * W0 + x] = tf_dist_of(*(const uint16_t*)((const char*)a.raw + (size_t)y * a.raw_pitch + (size_t)x * 2));
            }
        } else if (t < 1024 + 256) {
            const int u = t - 1024;
            const int x = X1 + (u & 15), y = Y1 + (u >> 4);
            if (x < W1 && y < H1) pn_pixel(s1, PN_R1, o1x, o1y, a, 1, x, y);
        } else {
            const int u = t - 1024 - 256;
            const int x = X2 + (u & 7), y = Y2 + (u >> 3);
            if (x < W2 && y < H2) pn_pixel(s2, PN_R2, X2, Y2, a, 2, x, y);
        }
    }
}


static inline int tf_div_up(int a, int b) { return (a + b - 1) / b; }
hipError_t tf_pre_args(tf_ctx* c, const uint16_t* depth, size_t pitch, int lookahead, uint16_t* d0, BilArgs* b, PyrArgs* a);
