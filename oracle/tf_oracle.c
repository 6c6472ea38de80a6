/*
 * tf_oracle.c -- CPU ORACLE (TEST INFRASTRUCTURE ONLY; see tf_oracle.h).
 * Serial restatement of the reference tfusion hot path.  Every function cites the
 * reference file:line it follows (paths relative to the reference root).
 * Build with -ffp-contract=off (oracle/Makefile).
 */
#include "tf_oracle.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>

#define BLK 8           /* SDF_BLOCK_SIZE, VoxelBlockHash.hpp:10 */
#define BLK3 512        /* SDF_BLOCK_SIZE3 */
#define FAR_AWAY 999999.9f   /* VisualisationEngine_Shared.hpp:18 */
#define VERY_CLOSE 0.05f     /* VisualisationEngine_Shared.hpp:22 */
#define SUBSAMPLE 8          /* minmaximg_subsample, VisualisationEngine_Shared.hpp:7 */
#define RB_SIZE 16           /* renderingBlockSizeX/Y, VisualisationEngine_Shared.hpp:25-26 */

static float qnanf_bits(void) { union { uint32_t u; float f; } v; v.u = 0x7fffffffu; return v.f; }

void tfo_default_params(tfo_params* p)
{   /* TopFuParams::default_params, topfu.cpp:12-53 */
    memset(p, 0, sizeof(*p));
    p->cols = 640; p->rows = 480;
    p->fx = 504.261f; p->fy = 503.905f; p->cx = 352.457f; p->cy = 272.202f;
    p->bilateral_sigma_depth = 0.04f;
    p->bilateral_sigma_spatial = 4.5f;
    p->bilateral_kernel_size = 7;
    p->icp_truncate_depth_dist = 2.0f;
    p->icp_dist_thres = 0.1f;
    p->icp_angle_thres = 30.f * 0.017453293f;      /* deg2rad, topfu.cpp:10 */
    p->icp_iter_num[0] = 10; p->icp_iter_num[1] = 5; p->icp_iter_num[2] = 4; p->icp_iter_num[3] = 0;
    p->mu = 0.02f; p->maxW = 100; p->voxelSize = 0.005f;
    p->viewFrustum_min = 0.2f; p->viewFrustum_max = 3.0f;
    p->n_buckets = 0x100000; p->n_excess = 0x20000; p->n_blocks = 0x10000;
    p->vis_capacity = 0x10000 * 4;                  /* SDF_LOCAL_BLOCK_NUM*sizeof(int) elements, RenderState_VH.hpp:42 */
    p->max_render_blocks = 65536 * 4;
    p->use_swapping = 0;                            /* Scene(params, false), topfu.cpp:67 */
    p->swap_transfer_blocks = 0x1000;               /* SDF_TRANSFER_BLOCK_NUM, VoxelBlockHash.hpp:27 */
    p->voxel_rgb = 0;                               /* Voxel_s (Defines.hpp:5) */
    p->depth_to_rgb[0] = p->depth_to_rgb[5] = p->depth_to_rgb[10] = 1.0f;   /* registered RGB-D */
}

/* ------------------------------------------------------------------------- */
/* canonical math                                                            */
/* ------------------------------------------------------------------------- */

/* replacement for CUDA __expf (imgproc.cu:40): 2^(x*log2(e)) */
float tfo_exp(float x)
{
    float t = x * 1.44269504088896341f;
    if (!(t > -125.0f)) return 0.0f;
    if (t >= 128.0f) return INFINITY;
    float k = rintf(t);
    float f = t - k;
    float p = 1.5403530393381606e-4f;
    p = fmaf(p, f, 1.3333558146428443e-3f);
    p = fmaf(p, f, 9.6181291076284772e-3f);
    p = fmaf(p, f, 5.5504108664821580e-2f);
    p = fmaf(p, f, 2.4022650695910071e-1f);
    p = fmaf(p, f, 6.9314718055994531e-1f);
    p = fmaf(p, f, 1.0f);
    return ldexpf(p, (int)k);
}

/* fixed-polynomial double sin/cos (replaces std::sin/cos in cv::Affine3 Rodrigues).  Horner
   over 13 terms; for |r| < 1/8 (every ICP increment in practice) 6 terms, whose first omitted
   term is below 2^-80 relative */
static const double k_inv_sin[14] = { 0.0, 1.0/6.0, 1.0/20.0, 1.0/42.0, 1.0/72.0, 1.0/110.0, 1.0/156.0,
    1.0/210.0, 1.0/272.0, 1.0/342.0, 1.0/420.0, 1.0/506.0, 1.0/600.0, 1.0/702.0 };
static const double k_inv_cos[14] = { 0.0, 1.0/2.0, 1.0/12.0, 1.0/30.0, 1.0/56.0, 1.0/90.0, 1.0/132.0,
    1.0/182.0, 1.0/240.0, 1.0/306.0, 1.0/380.0, 1.0/462.0, 1.0/552.0, 1.0/650.0 };
void tfo_sincos(double th, double* s, double* c)
{
    const double PI = 3.14159265358979323846;
    const double TWO_PI = 6.28318530717958647692;
    double r = th;
    if (r > PI || r < -PI) {
        double k = rint(r / TWO_PI);
        r = r - k * TWO_PI;
    }
    double r2 = r * r;
    double ps = 1.0, pc = 1.0;
    const int nt = r2 < 0.015625 ? 6 : 13;
    for (int n = nt; n >= 1; --n) {
        ps = 1.0 - (r2 * k_inv_sin[n]) * ps;
        pc = 1.0 - (r2 * k_inv_cos[n]) * pc;
    }
    *s = r * ps;
    *c = pc;
}

/* KinFu float3 helpers, src/cuda/device.hpp:26-113 */
typedef struct { float x, y, z; } f3;
typedef struct { float x, y, z, w; } f4;
static inline f3 mk3(float x, float y, float z) { f3 r; r.x = x; r.y = y; r.z = z; return r; }
static inline f3 sub3(f3 a, f3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline f3 add3(f3 a, f3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline f3 mul3s(f3 a, float s) { return mk3(a.x * s, a.y * s, a.z * s); }
/* dot with __fmaf_rn, device.hpp:26-29 */
static inline float kdot(f3 a, f3 b) { return fmaf(a.x, b.x, fmaf(a.y, b.y, a.z * b.z)); }
static inline f3 kcross(f3 a, f3 b) { return mk3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
/* normalized: v * rsqrt(dot(v,v)), device.hpp:100-103 */
static inline f3 knormalized(f3 v) { return mul3s(v, 1.0f / sqrtf(kdot(v, v))); }

void tfo_tsdf_update(int16_t* sdf, uint8_t* w, float eta, float mu, int maxW);
/* InfiniTAM Matrix4f (column-major, m[4c+r]) * Vector4f, Matrix.hpp:126-133 */
static inline void m4v(const float m[16], const float v[4], float r[4])
{
    r[0] = m[0] * v[0] + m[4] * v[1] + m[8] * v[2] + m[12] * v[3];
    r[1] = m[1] * v[0] + m[5] * v[1] + m[9] * v[2] + m[13] * v[3];
    r[2] = m[2] * v[0] + m[6] * v[1] + m[10] * v[2] + m[14] * v[3];
    r[3] = m[3] * v[0] + m[7] * v[1] + m[11] * v[2] + m[15] * v[3];
}

void tfo_m4v(const float m[16], const float v[4], float r[4]) { m4v(m, v, r); }

/* Matrix4f(pose(0,0), pose(1,0), ...): topfu.cpp:246-249, SceneReconstructionEngine_host.cu:94-97 */
static void rt_to_m4(const float rt[12], float m[16])
{
    for (int c = 0; c < 4; ++c) {
        for (int r = 0; r < 3; ++r) m[4 * c + r] = rt[r * 4 + c];
        m[4 * c + 3] = (c == 3) ? 1.0f : 0.0f;
    }
}

/* Matrix4::inv, Matrix.hpp:173-233 (pinned by oracle/ref_pin) */
int tfo_matrix4_inv(const float mm[16], float out[16])
{
    float tmp[12], src[16], det;
    float* dst = out;
    for (int i = 0; i < 4; i++) {
        src[i] = mm[i * 4];
        src[i + 4] = mm[i * 4 + 1];
        src[i + 8] = mm[i * 4 + 2];
        src[i + 12] = mm[i * 4 + 3];
    }
    tmp[0] = src[10] * src[15]; tmp[1] = src[11] * src[14]; tmp[2] = src[9] * src[15];
    tmp[3] = src[11] * src[13]; tmp[4] = src[9] * src[14]; tmp[5] = src[10] * src[13];
    tmp[6] = src[8] * src[15]; tmp[7] = src[11] * src[12]; tmp[8] = src[8] * src[14];
    tmp[9] = src[10] * src[12]; tmp[10] = src[8] * src[13]; tmp[11] = src[9] * src[12];
    dst[0] = (tmp[0] * src[5] + tmp[3] * src[6] + tmp[4] * src[7]) - (tmp[1] * src[5] + tmp[2] * src[6] + tmp[5] * src[7]);
    dst[1] = (tmp[1] * src[4] + tmp[6] * src[6] + tmp[9] * src[7]) - (tmp[0] * src[4] + tmp[7] * src[6] + tmp[8] * src[7]);
    dst[2] = (tmp[2] * src[4] + tmp[7] * src[5] + tmp[10] * src[7]) - (tmp[3] * src[4] + tmp[6] * src[5] + tmp[11] * src[7]);
    dst[3] = (tmp[5] * src[4] + tmp[8] * src[5] + tmp[11] * src[6]) - (tmp[4] * src[4] + tmp[9] * src[5] + tmp[10] * src[6]);
    det = src[0] * dst[0] + src[1] * dst[1] + src[2] * dst[2] + src[3] * dst[3];
    if (det == 0.0f) return 0;
    dst[4] = (tmp[1] * src[1] + tmp[2] * src[2] + tmp[5] * src[3]) - (tmp[0] * src[1] + tmp[3] * src[2] + tmp[4] * src[3]);
    dst[5] = (tmp[0] * src[0] + tmp[7] * src[2] + tmp[8] * src[3]) - (tmp[1] * src[0] + tmp[6] * src[2] + tmp[9] * src[3]);
    dst[6] = (tmp[3] * src[0] + tmp[6] * src[1] + tmp[11] * src[3]) - (tmp[2] * src[0] + tmp[7] * src[1] + tmp[10] * src[3]);
    dst[7] = (tmp[4] * src[0] + tmp[9] * src[1] + tmp[10] * src[2]) - (tmp[5] * src[0] + tmp[8] * src[1] + tmp[11] * src[2]);
    tmp[0] = src[2] * src[7]; tmp[1] = src[3] * src[6]; tmp[2] = src[1] * src[7];
    tmp[3] = src[3] * src[5]; tmp[4] = src[1] * src[6]; tmp[5] = src[2] * src[5];
    tmp[6] = src[0] * src[7]; tmp[7] = src[3] * src[4]; tmp[8] = src[0] * src[6];
    tmp[9] = src[2] * src[4]; tmp[10] = src[0] * src[5]; tmp[11] = src[1] * src[4];
    dst[8] = (tmp[0] * src[13] + tmp[3] * src[14] + tmp[4] * src[15]) - (tmp[1] * src[13] + tmp[2] * src[14] + tmp[5] * src[15]);
    dst[9] = (tmp[1] * src[12] + tmp[6] * src[14] + tmp[9] * src[15]) - (tmp[0] * src[12] + tmp[7] * src[14] + tmp[8] * src[15]);
    dst[10] = (tmp[2] * src[12] + tmp[7] * src[13] + tmp[10] * src[15]) - (tmp[3] * src[12] + tmp[6] * src[13] + tmp[11] * src[15]);
    dst[11] = (tmp[5] * src[12] + tmp[8] * src[13] + tmp[11] * src[14]) - (tmp[4] * src[12] + tmp[9] * src[13] + tmp[10] * src[14]);
    dst[12] = (tmp[2] * src[10] + tmp[5] * src[11] + tmp[1] * src[9]) - (tmp[4] * src[11] + tmp[0] * src[9] + tmp[3] * src[10]);
    dst[13] = (tmp[8] * src[11] + tmp[0] * src[8] + tmp[7] * src[10]) - (tmp[6] * src[10] + tmp[9] * src[11] + tmp[1] * src[8]);
    dst[14] = (tmp[6] * src[9] + tmp[11] * src[11] + tmp[3] * src[8]) - (tmp[10] * src[11] + tmp[2] * src[8] + tmp[7] * src[9]);
    dst[15] = (tmp[10] * src[10] + tmp[4] * src[8] + tmp[9] * src[9]) - (tmp[8] * src[9] + tmp[11] * src[10] + tmp[5] * src[8]);
    float s = 1 / det;
    for (int i = 0; i < 16; ++i) out[i] *= s;
    return 1;
}

/* cv::Affine3f operator*  (canonical float rigid composition, see header) */
void tfo_rigid_mul(const float a[12], const float b[12], float out[12])
{
    float o[12];
    for (int j = 0; j < 3; ++j) {
        for (int i = 0; i < 3; ++i)
            o[j * 4 + i] = (a[j * 4 + 0] * b[0 * 4 + i] + a[j * 4 + 1] * b[1 * 4 + i]) + a[j * 4 + 2] * b[2 * 4 + i];
        o[j * 4 + 3] = ((a[j * 4 + 0] * b[3] + a[j * 4 + 1] * b[7]) + a[j * 4 + 2] * b[11]) + a[j * 4 + 3];
    }
    memcpy(out, o, sizeof(o));
}

/* cv::Affine3f::inv() (canonical rigid inverse) */
void tfo_rigid_inv(const float a[12], float out[12])
{
    float o[12];
    for (int j = 0; j < 3; ++j) {
        for (int i = 0; i < 3; ++i) o[j * 4 + i] = a[i * 4 + j];
        o[j * 4 + 3] = -((a[0 * 4 + j] * a[3] + a[1 * 4 + j] * a[7]) + a[2 * 4 + j] * a[11]);
    }
    memcpy(out, o, sizeof(o));
}

/* cv::Affine3f(rvec, t) rotation part: Rodrigues in double */
/* Affine3f(rvec, t)'s rotation (cv::Affine3::rotation(const Vec3&), OpenCV affine.hpp; OpenCV is
   absent here: parity unpinned).  R = cos t I + ((1 - cos t) / t^2) r r^T + (sin t / t) [r]x with
   r = rvec unnormalised -- the same matrix as cv's c I + (1 - c) u u^T + s [u]x with u = r / t --
   and the three even functions of t as nested polynomials in t^2 with fma (the coefficients of
   tfo_sincos; 2 (1 - cos t) / t^2 = 1 - t^2/12 (1 - t^2/30 (...))).  No square root, no division:
   the GPU's serial ICP tail evaluates exactly this (tf_icp_tail.h icp_rodrigues).  t > pi (never
   for an ICP increment) uses rodrigues_sqrt, the direct form with tfo_sincos' range reduction. */
static void rodrigues_sqrt(const float r[3], float R[9]);
static const double k_inv_cos15 = 1.0 / 756.0;
void tfo_rodrigues(const float r[3], float R[9])
{
    const double rx = r[0], ry = r[1], rz = r[2];
    const double t2 = (rx * rx + ry * ry) + rz * rz;
    if (t2 < DBL_EPSILON * DBL_EPSILON) {
        for (int k = 0; k < 9; ++k) R[k] = (k % 4 == 0) ? 1.0f : 0.0f;
        return;
    }
    if (t2 > 9.869604401089358) { rodrigues_sqrt(r, R); return; }
    double pc = 1.0, pa = 1.0, pb = 1.0;
    /* terms: 4 below t^2 = 2^-12 (an ICP increment past its first iteration; the first omitted term
       is below 2^-60 relative), 6 below 1/64 (below 2^-80), else 13 */
    const int nt = t2 < 0.000244140625 ? 4 : (t2 < 0.015625 ? 6 : 13);
    for (int n = nt; n >= 1; --n) {
        pc = fma(-(t2 * k_inv_cos[n]), pc, 1.0);
        pa = fma(-(t2 * k_inv_sin[n]), pa, 1.0);
        pb = fma(-(t2 * (n + 1 < 14 ? k_inv_cos[n + 1] : k_inv_cos15)), pb, 1.0);
    }
    const double b = 0.5 * pb;
    const double rrt[9] = { rx * rx, rx * ry, rx * rz, rx * ry, ry * ry, ry * rz, rx * rz, ry * rz, rz * rz };
    const double rxm[9] = { 0, -rz, ry, rz, 0, -rx, -ry, rx, 0 };
    for (int k = 0; k < 9; ++k) {
        const double I = (k % 4 == 0) ? 1.0 : 0.0;
        R[k] = (float)((pc * I + b * rrt[k]) + pa * rxm[k]);
    }
}

void tfo_rodrigues_direct(const float r[3], float R[9]) { rodrigues_sqrt(r, R); }

static void rodrigues_sqrt(const float r[3], float R[9])
{
    double rx = r[0], ry = r[1], rz = r[2];
    double theta = sqrt((rx * rx + ry * ry) + rz * rz);
    if (theta < DBL_EPSILON) {
        for (int k = 0; k < 9; ++k) R[k] = (k % 4 == 0) ? 1.0f : 0.0f;
        return;
    }
    double s, c;
    tfo_sincos(theta, &s, &c);
    double c1 = 1.0 - c;
    double itheta = 1.0 / theta;
    rx *= itheta; ry *= itheta; rz *= itheta;
    double rrt[9] = { rx * rx, rx * ry, rx * rz, rx * ry, ry * ry, ry * rz, rx * rz, ry * rz, rz * rz };
    double rxm[9] = { 0, -rz, ry, rz, 0, -rx, -ry, rx, 0 };
    for (int k = 0; k < 9; ++k) {
        double I = (k % 4 == 0) ? 1.0 : 0.0;
        R[k] = (float)((c * I + c1 * rrt[k]) + s * rxm[k]);
    }
}

/* ------------------------------------------------------------------------- */
/* A2-A6: depth preprocessing (src/cuda/imgproc.cu)                          */
/* ------------------------------------------------------------------------- */

/* compute_dists_kernel, imgproc.cu:263-280 */
void tfo_compute_dists(const uint16_t* depth, int W, int H, float* dists)
{
#pragma omp parallel for schedule(static)
    for (int i = 0; i < W * H; ++i) {
        int d = depth[i];
        dists[i] = (d >= 2047 || d <= 0) ? -1.0f : (float)d * 0.001f;
    }
}

/* bilateral_kernel, imgproc.cu:10-47 (+ launch constants :51-59) */
void tfo_bilateral(const uint16_t* src, uint16_t* dst, int W, int H, int ksz, float sigma_spatial, float sigma_depth_m)
{
    float sigma_depth = sigma_depth_m * 1000.0f;
    float ss = 0.5f / (sigma_spatial * sigma_spatial);
    float sd = 0.5f / (sigma_depth * sigma_depth);
#pragma omp parallel for schedule(static)
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            int value = src[y * W + x];
            int tx = x - ksz / 2 + ksz; if (tx > W - 1) tx = W - 1;
            int ty = y - ksz / 2 + ksz; if (ty > H - 1) ty = H - 1;
            float sum1 = 0, sum2 = 0;
            for (int cy = (y - ksz / 2 > 0 ? y - ksz / 2 : 0); cy < ty; ++cy)
                for (int cx = (x - ksz / 2 > 0 ? x - ksz / 2 : 0); cx < tx; ++cx) {
                    int depth = src[cy * W + cx];
                    float space2 = (float)((x - cx) * (x - cx) + (y - cy) * (y - cy));
                    float color2 = (float)((int)((unsigned)(value - depth) * (unsigned)(value - depth)));
                    float weight = tfo_exp(-(space2 * ss + color2 * sd));
                    sum1 += (float)depth * weight;
                    sum2 += weight;
                }
            float q = sum1 / sum2;
            int v = (q == q) ? (int)rintf(q) : 0;  /* __float2int_rn, NaN -> 0 */
            dst[y * W + x] = (uint16_t)v;
        }
}

/* truncate_depth_kernel, imgproc.cu:70-89 */
void tfo_truncate(uint16_t* depth, int W, int H, float max_dist_m)
{
    uint16_t md = (uint16_t)(max_dist_m * 1000.f);
    for (int i = 0; i < W * H; ++i)
        if (depth[i] > md) depth[i] = 0;
}

/* pyramid_kernel, imgproc.cu:98-140 ; dst is (W/2)x(H/2) */
void tfo_pyr_down(const uint16_t* src, int W, int H, uint16_t* dst, float sigma_depth_m)
{
    float sigma3 = sigma_depth_m * 1000.0f * 3.0f;
    int DW = W / 2, DH = H / 2;
    const int D = 5;
#pragma omp parallel for schedule(static)
    for (int y = 0; y < DH; ++y)
        for (int x = 0; x < DW; ++x) {
            int center = src[(2 * y) * W + 2 * x];
            int tx = 2 * x - D / 2 + D; if (tx > W - 1) tx = W - 1;
            int ty = 2 * y - D / 2 + D; if (ty > H - 1) ty = H - 1;
            int sum = 0, count = 0;
            for (int cy = (2 * y - D / 2 > 0 ? 2 * y - D / 2 : 0); cy < ty; ++cy)
                for (int cx = (2 * x - D / 2 > 0 ? 2 * x - D / 2 : 0); cx < tx; ++cx) {
                    int val = src[cy * W + cx];
                    if ((float)abs(val - center) < sigma3) { sum += val; ++count; }
                }
            dst[y * DW + x] = (uint16_t)((count == 0) ? 0 : sum / count);
        }
}

/* points_normals_kernel, imgproc.cu:214-254; Reprojector precomp.cpp:54 / device.hpp:44-48 */
void tfo_points_normals(const uint16_t* depth, int W, int H, float fx, float fy, float cx, float cy,
                        float* points, float* normals)
{
    const float qnan = qnanf_bits();
    float fxi = 1.f / fx, fyi = 1.f / fy;
#pragma omp parallel for schedule(static)
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            float* p = points + 4 * (y * W + x);
            float* n = normals + 4 * (y * W + x);
            p[0] = p[1] = p[2] = p[3] = qnan;
            n[0] = n[1] = n[2] = n[3] = qnan;
            if (x >= W - 1 || y >= H - 1) continue;
            float z00 = (float)depth[y * W + x] * 0.001f;
            float z01 = (float)depth[y * W + x + 1] * 0.001f;
            float z10 = (float)depth[(y + 1) * W + x] * 0.001f;
            if (z00 * z01 * z10 != 0) {
                f3 v00 = mk3(z00 * ((float)x - cx) * fxi, z00 * ((float)y - cy) * fyi, z00);
                f3 v01 = mk3(z01 * ((float)(x + 1) - cx) * fxi, z01 * ((float)y - cy) * fyi, z01);
                f3 v10 = mk3(z10 * ((float)x - cx) * fxi, z10 * ((float)(y + 1) - cy) * fyi, z10);
                f3 nn = knormalized(kcross(sub3(v01, v00), sub3(v10, v00)));
                n[0] = -nn.x; n[1] = -nn.y; n[2] = -nn.z; n[3] = 1.0f;
                p[0] = v00.x; p[1] = v00.y; p[2] = v00.z; p[3] = 1.0f;
            }
        }
}

/* resize_points_normals_kernel, imgproc.cu:355-401 ; src WxH -> dst (W/2)x(H/2) */
void tfo_resize_points_normals(const float* vsrc, const float* nsrc, int W, int H, float* vdst, float* ndst)
{
    const float qnan = qnanf_bits();
    int DW = W / 2, DH = H / 2;
#pragma omp parallel for schedule(static)
    for (int y = 0; y < DH; ++y)
        for (int x = 0; x < DW; ++x) {
            float* vo = vdst + 4 * (y * DW + x);
            float* no = ndst + 4 * (y * DW + x);
            vo[0] = vo[1] = vo[2] = qnan; vo[3] = 0.f;
            no[0] = no[1] = no[2] = qnan; no[3] = 0.f;
            int xs = 2 * x, ys = 2 * y;
            const float* d00 = vsrc + 4 * (ys * W + xs);
            const float* d01 = vsrc + 4 * (ys * W + xs + 1);
            const float* d10 = vsrc + 4 * ((ys + 1) * W + xs);
            const float* d11 = vsrc + 4 * ((ys + 1) * W + xs + 1);
            if (!isnan(d00[0] * d01[0] * d10[0] * d11[0])) {
                for (int k = 0; k < 3; ++k) vo[k] = (((d00[k] + d01[k]) + d10[k]) + d11[k]) * 0.25f;
                vo[3] = 1.0f;
                const float* n00 = nsrc + 4 * (ys * W + xs);
                const float* n01 = nsrc + 4 * (ys * W + xs + 1);
                const float* n10 = nsrc + 4 * ((ys + 1) * W + xs);
                const float* n11 = nsrc + 4 * ((ys + 1) * W + xs + 1);
                for (int k = 0; k < 3; ++k) no[k] = (((n00[k] + n01[k]) + n10[k]) + n11[k]) * 0.25f;
                no[3] = 0.f;
            }
        }
}

/* ------------------------------------------------------------------------- */
/* A7-A9: projective ICP (src/cuda/proj_icp.cu, src/projective_icp.cpp)      */
/* ------------------------------------------------------------------------- */

/* find_coresp (points variant), proj_icp.cu:80-117; row build icp_helper_kernel :359-377 */
static int icp_row(const float* vcurr, const float* ncurr, const float* vprev, const float* nprev,
                   int W, int H, int x, int y, float fx, float fy, float cx, float cy,
                   float min_cosine, float dist2_thres, const float aff[12], float row[7])
{
    const float* sp = vcurr + 4 * (y * W + x);
    f3 s = mk3(sp[0], sp[1], sp[2]);
    if (isnan(s.x)) return 40;
    f3 R0 = mk3(aff[0], aff[1], aff[2]), R1 = mk3(aff[4], aff[5], aff[6]), R2 = mk3(aff[8], aff[9], aff[10]);
    s = mk3(kdot(R0, s) + aff[3], kdot(R1, s) + aff[7], kdot(R2, s) + aff[11]);   /* aff * s, device.hpp:70-72 */
    /* proj, proj_icp.cu:31-37: __fmaf_rn(f, __fdividef(p.x, p.z), c) -- __fdividef is x times an
       approximate reciprocal of y; canonical: x * RN(1 / y), one reciprocal for both coordinates */
    const float rz = 1.0f / s.z;
    float coox = fmaf(fx, s.x * rz, cx);
    float cooy = fmaf(fy, s.y * rz, cy);
    if (s.z <= 0 || coox < 0 || cooy < 0 || coox >= (float)W || cooy >= (float)H) return 80;
    int tx = (int)floorf(coox), ty = (int)floorf(cooy);                         /* point-sampled tex2D */
    const float* dp = vprev + 4 * (ty * W + tx);
    f3 d = mk3(dp[0], dp[1], dp[2]);
    if (isnan(d.x)) return 120;
    f3 sd = sub3(s, d);
    float dist2 = kdot(sd, sd);
    if (dist2 > dist2_thres) return 160;
    const float* ncp = ncurr + 4 * (y * W + x);
    f3 nc = mk3(ncp[0], ncp[1], ncp[2]);
    f3 ns = mk3(kdot(R0, nc), kdot(R1, nc), kdot(R2, nc));
    const float* ndp = nprev + 4 * (ty * W + tx);
    f3 nd = mk3(ndp[0], ndp[1], ndp[2]);
    float cosine = fabsf(kdot(ns, nd));
    if (cosine < min_cosine) return 200;
    f3 cr = kcross(s, nd);
    row[0] = cr.x; row[1] = cr.y; row[2] = cr.z;
    row[3] = nd.x; row[4] = nd.y; row[5] = nd.z;
    row[6] = kdot(nd, sub3(d, s));
    return 0;
}

/* Block::reduce<256> halving tree, src/cuda/temp_utils.hpp:503-523 */
static float tree256(float* v)
{
    for (int s = 128; s >= 1; s >>= 1)
        for (int t = 0; t < s; ++t) v[t] = v[t] + v[t + s];
    return v[0];
}

void tfo_icp_reduce(const float* vcurr, const float* ncurr, const float* vprev, const float* nprev,
                    int W, int H, float fx, float fy, float cx, float cy,
                    float min_cosine, float dist2_thres, const float aff[12], float out27[27])
{
    int gx = (W + 31) / 32, gy = (H + 7) / 8;     /* CTA 32x8, proj_icp.cu:17-19,439-440 */
    int nct = gx * gy;
    float* partial = (float*)malloc(sizeof(float) * 27 * (size_t)nct);
    float v[256];
    /* the CTAs' partial sums are independent (OpenMP build: one CTA per iteration) */
#pragma omp parallel
    {
    float (*rows)[7] = malloc(sizeof(float) * 7 * 256);
    float vt[256];
#pragma omp for schedule(static)
    for (int cta_i = 0; cta_i < nct; ++cta_i) {
        const int by = cta_i / gx, bx = cta_i % gx;
        {
            for (int tid = 0; tid < 256; ++tid) {
                int x = bx * 32 + (tid & 31), y = by * 8 + (tid >> 5);
                int filtered = (x < W && y < H) ? icp_row(vcurr, ncurr, vprev, nprev, W, H, x, y, fx, fy, cx, cy,
                                                          min_cosine, dist2_thres, aff, rows[tid]) : 1;
                if (filtered) for (int k = 0; k < 7; ++k) rows[tid][k] = 0.f;
            }
            int cta = bx + gx * by, k = 0;
            for (int i = 0; i < 6; ++i)
                for (int j = i; j < 7; ++j, ++k) {   /* partial_reduce order, proj_icp.cu:137-356 */
                    for (int tid = 0; tid < 256; ++tid) vt[tid] = rows[tid][i] * rows[tid][j];
                    partial[k * nct + cta] = tree256(vt);
                }
        }
    }
    free(rows);
    }
    for (int k = 0; k < 27; ++k) {              /* icp_final_reduce_kernel, proj_icp.cu:382-403 */
        for (int tid = 0; tid < 256; ++tid) {
            float sum = 0.f;
            for (int j = tid; j < nct; j += 256) sum += partial[k * nct + j];
            v[tid] = sum;
        }
        out27[k] = tree256(v);
    }
    free(partial);
}

/* cv::determinant(Matx66f): LU with partial pivoting in float (eps 10*FLT_EPSILON), pivot product in double */
static double cv_det6(const float Ain[36])
{
    float A[36];
    memcpy(A, Ain, sizeof(A));
    int p = 1;
    const float eps = FLT_EPSILON * 10;
    for (int i = 0; i < 6; i++) {
        int k = i;
        for (int j = i + 1; j < 6; j++)
            if (fabsf(A[j * 6 + i]) > fabsf(A[k * 6 + i])) k = j;
        if (fabsf(A[k * 6 + i]) < eps) return 0.0;
        if (k != i) {
            for (int j = i; j < 6; j++) { float t = A[i * 6 + j]; A[i * 6 + j] = A[k * 6 + j]; A[k * 6 + j] = t; }
            p = -p;
        }
        float d = -1 / A[i * 6 + i];
        for (int j = i + 1; j < 6; j++) {
            float alpha = A[j * 6 + i] * d;
            for (int c = i + 1; c < 6; c++) A[j * 6 + c] += alpha * A[i * 6 + c];
        }
    }
    double det = p;
    for (int i = 0; i < 6; i++) det *= A[i * 6 + i];
    return det;
}

/* cv::solve(A, b, DECOMP_SVD) replacement (the canonical algebra; the reference's own is
   tfo_cv_solve_svd6 below).  A is the symmetric normal matrix J^T J, already past the determinant
   check.  2 x 2 block elimination in double with closed-form 3 x 3 inverses (adjugate / det):
   A = [P Q; Q^T R] (P the rotation block, R the translation block), b = [b1; b2],
     T = Q adj(R) / det(R),  S = P - T Q^T,  c = b1 - T b2,
     x1 = adj(S) c / det(S),  x2 = adj(R) (b2 - Q^T x1) / det(R).
   Its critical path is two 3 x 3 determinants and two divisions deep (~35 dependent operations
   against ~110 for a column-by-column LDL^T), and the rotation part x1 -- what Rodrigues needs --
   comes first.  The GPU's serial ICP tail runs exactly this (tf_icp_tail.h icp_solve6_schur). */
static void sym3_adj(const double M[3][3], double C[3][3], double* det)
{
    C[0][0] = M[1][1] * M[2][2] - M[1][2] * M[2][1];
    C[0][1] = M[0][2] * M[2][1] - M[0][1] * M[2][2];
    C[0][2] = M[0][1] * M[1][2] - M[0][2] * M[1][1];
    C[1][0] = M[1][2] * M[2][0] - M[1][0] * M[2][2];
    C[1][1] = M[0][0] * M[2][2] - M[0][2] * M[2][0];
    C[1][2] = M[0][2] * M[1][0] - M[0][0] * M[1][2];
    C[2][0] = M[1][0] * M[2][1] - M[1][1] * M[2][0];
    C[2][1] = M[0][1] * M[2][0] - M[0][0] * M[2][1];
    C[2][2] = M[0][0] * M[1][1] - M[0][1] * M[1][0];
    *det = (M[0][0] * C[0][0] + M[0][1] * C[1][0]) + M[0][2] * C[2][0];
}

static void solve6(const float Af[36], const float bf[6], float x[6])
{
    double P[3][3], Q[3][3], R[3][3], b1[3], b2[3];
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) {
            P[i][j] = Af[i * 6 + j];
            Q[i][j] = Af[i * 6 + 3 + j];
            R[i][j] = Af[(3 + i) * 6 + 3 + j];
        }
        b1[i] = bf[i];
        b2[i] = bf[3 + i];
    }
    double aR[3][3], dR, aS[3][3], dS, T[3][3], S[3][3], c[3], x1[3], e[3];
    sym3_adj(R, aR, &dR);
    const double rR = 1.0 / dR;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            T[i][j] = ((Q[i][0] * aR[0][j] + Q[i][1] * aR[1][j]) + Q[i][2] * aR[2][j]) * rR;
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j)
            S[i][j] = P[i][j] - ((T[i][0] * Q[j][0] + T[i][1] * Q[j][1]) + T[i][2] * Q[j][2]);
        c[i] = b1[i] - ((T[i][0] * b2[0] + T[i][1] * b2[1]) + T[i][2] * b2[2]);
    }
    sym3_adj(S, aS, &dS);
    const double rS = 1.0 / dS;
    for (int i = 0; i < 3; ++i) x1[i] = ((aS[i][0] * c[0] + aS[i][1] * c[1]) + aS[i][2] * c[2]) * rS;
    for (int i = 0; i < 3; ++i) e[i] = b2[i] - ((Q[0][i] * x1[0] + Q[1][i] * x1[1]) + Q[2][i] * x1[2]);
    for (int i = 0; i < 3; ++i) {
        x[i] = (float)x1[i];
        x[3 + i] = (float)(((aR[i][0] * e[0] + aR[i][1] * e[1]) + aR[i][2] * e[2]) * rR);
    }
}

/* ------------------------------------------------------------------------- */
/* The reference's own pose algebra: OpenCV (>= 2.4.9, CMakeLists.txt:18; not vendored, absent   */
/* here).  TEST-ONLY mode (tfo_set_pose_algebra): estimateTransform's cv::determinant(Matx66f),  */
/* cv::solve(A, b, r, DECOMP_SVD) and cv::Affine3f(rvec, t) (projective_icp.cpp:197-209) as     */
/* OpenCV's published sources define them, so that the canonical algebra above (LDL^T solve,     */
/* sinc Rodrigues: what the GPU runs by default) can be measured against it.                    */
/*   TFO_POSE_OPENCV2 : OpenCV 2.4.9 -- LU pivot floor FLT_EPSILON, norm(Vec3f) in double        */
/*   TFO_POSE_OPENCV4 : OpenCV 3.x / 4.x -- LU floor 10 FLT_EPSILON, norm(Vec3f) in float        */
/* Both: Matx_DetOp (operations.hpp / matx.inl.hpp: LU with the reciprocal pivots left on the    */
/* diagonal, det = 1 / (p * prod)), lapack.cpp's cv::solve DECOMP_SVD path (A transposed into    */
/* the work matrix, JacobiSVDImpl_<float> with eps 2 FLT_EPSILON / minval FLT_MIN, then          */
/* SVBkSbImpl_<float> with threshold eps (float)(2 DBL_EPSILON)), and Affine3::rotation(Vec3)     */
/* (affine.hpp: every Matx operation rounded to float).  The transcendental functions are        */
/* either glibc's (use_libm = 1: what a host build of the reference calls) or portable           */
/* restatements the GPU can run bit for bit (use_libm = 0: tfo_sincos and cv_hypot below).       */
/* ------------------------------------------------------------------------- */
static int g_pose_algebra = TFO_POSE_OPENCV4, g_pose_libm = 0;   /* the reference's own by default */
void tfo_set_pose_algebra(int mode, int use_libm) { g_pose_algebra = mode; g_pose_libm = use_libm; }
int tfo_get_pose_algebra(void) { return g_pose_algebra; }

/* hypot(x, y) for the Jacobi rotation: sqrt(x^2 + y^2) with the rounding error of the sum of
   squares corrected by fma (Borges, "An improved algorithm for hypot(a, b)", 2019, fma variant).
   Inputs here are finite and far from over/underflow (sums of squared float products). */
double tfo_cv_hypot(double x, double y)
{
    if (g_pose_libm) return hypot(x, y);
    x = fabs(x); y = fabs(y);
    if (x < y) { double t = x; x = y; y = t; }
    if (y == 0.0) return x;
    double h = sqrt(fma(x, x, y * y));
    double h_sq = h * h, x_sq = x * x;
    double e = (fma(-y, y, h_sq - x_sq) + fma(h, h, -h_sq)) - fma(x, x, -x_sq);
    return h - e / (2.0 * h);
}

static void pose_sincos(double th, double* s, double* c)
{
    if (g_pose_libm) { *s = sin(th); *c = cos(th); }
    else tfo_sincos(th, s, c);
}

/* cv::LU (lapack.cpp LUImpl, float): partial pivoting; the diagonal keeps the reciprocal pivots */
static int cv_lu_f(float* A, int m, float eps)
{
    int p = 1;
    for (int i = 0; i < m; i++) {
        int k = i;
        for (int j = i + 1; j < m; j++)
            if (fabsf(A[j * m + i]) > fabsf(A[k * m + i])) k = j;
        if (fabsf(A[k * m + i]) < eps) return 0;
        if (k != i) {
            for (int j = i; j < m; j++) { float t = A[i * m + j]; A[i * m + j] = A[k * m + j]; A[k * m + j] = t; }
            p = -p;
        }
        float d = -1 / A[i * m + i];
        for (int j = i + 1; j < m; j++) {
            float alpha = A[j * m + i] * d;
            for (int c = i + 1; c < m; c++) A[j * m + c] += alpha * A[i * m + c];
        }
        A[i * m + i] = -d;
    }
    return p;
}

/* cv::determinant(Matx66f) = Matx_DetOp<float, 6> */
double tfo_cv_det6(const float Ain[36], int mode)
{
    float T[36];
    memcpy(T, Ain, sizeof(T));
    double p = cv_lu_f(T, 6, mode == TFO_POSE_OPENCV2 ? FLT_EPSILON : FLT_EPSILON * 10);
    if (p == 0) return p;
    for (int i = 0; i < 6; i++) p *= T[i * 6 + i];
    return 1. / p;
}

/* cv::RNG::next (core.hpp: multiply-with-carry, CV_RNG_COEFF 4164903690) */
static unsigned cv_rng_next(uint64_t* st)
{
    *st = (uint64_t)(unsigned)*st * 4164903690u + (unsigned)(*st >> 32);
    return (unsigned)*st;
}

/* JacobiSVDImpl_<float>(At, ..., m, n, n1 = n, FLT_MIN, 2 FLT_EPSILON), lapack.cpp: one-sided
   cyclic Jacobi on the rows of At (n rows of m), W in double while iterating, rows sorted by
   singular value, left vectors normalised (random completion of a zero singular value). */
/* statistics of the Jacobi sweeps (test-only diagnostics): calls, sweeps, rotations, max sweeps,
   and a histogram of sweeps per call (index = sweeps, capped at 31) */
static long long g_svd_stats[4 + 32];
void tfo_cv_svd_stats(long long out[36], int reset)
{
    memcpy(out, g_svd_stats, sizeof(g_svd_stats));
    if (reset) memset(g_svd_stats, 0, sizeof(g_svd_stats));
}

void tfo_cv_jacobi_svd(float* At, float* Wout, float* Vt, int m, int n)
{
    const double minval = FLT_MIN;
    const float eps = FLT_EPSILON * 2;
    double W[8], sd;
    int i, j, k, iter, max_iter = m > 30 ? m : 30;
    for (i = 0; i < n; i++) {
        for (k = 0, sd = 0; k < m; k++) { float t = At[i * m + k]; sd += (double)t * t; }
        W[i] = sd;
        for (k = 0; k < n; k++) Vt[i * n + k] = 0;
        Vt[i * n + i] = 1;
    }
    for (iter = 0; iter < max_iter; iter++) {
        int changed = 0;
        for (i = 0; i < n - 1; i++)
            for (j = i + 1; j < n; j++) {
                float *Ai = At + i * m, *Aj = At + j * m;
                double a = W[i], p = 0, b = W[j];
                for (k = 0; k < m; k++) p += (double)Ai[k] * Aj[k];
                if (fabs(p) <= eps * sqrt((double)a * b)) continue;
                p *= 2;
                double beta = a - b, gamma = tfo_cv_hypot(p, beta);
                float c, s;
                if (beta < 0) {
                    double delta = (gamma - beta) * 0.5;
                    s = (float)sqrt(delta / gamma);
                    c = (float)(p / (gamma * s * 2));
                } else {
                    c = (float)sqrt((gamma + beta) / (gamma * 2));
                    s = (float)(p / (gamma * c * 2));
                }
                a = b = 0;
                for (k = 0; k < m; k++) {
                    float t0 = c * Ai[k] + s * Aj[k];
                    float t1 = -s * Ai[k] + c * Aj[k];
                    Ai[k] = t0; Aj[k] = t1;
                    a += (double)t0 * t0; b += (double)t1 * t1;
                }
                W[i] = a; W[j] = b;
                changed = 1;
                g_svd_stats[2]++;
                float *Vi = Vt + i * n, *Vj = Vt + j * n;
                for (k = 0; k < n; k++) {       /* VBLAS<float>::givens: a c + b s, b c - a s */
                    float t0 = Vi[k] * c + Vj[k] * s;
                    float t1 = Vj[k] * c - Vi[k] * s;
                    Vi[k] = t0; Vj[k] = t1;
                }
            }
        if (!changed) break;
    }
    g_svd_stats[0]++;
    g_svd_stats[1] += iter + (iter < max_iter);
    if (iter + 1 > g_svd_stats[3]) g_svd_stats[3] = iter + 1;
    g_svd_stats[4 + (iter < 31 ? iter : 31)]++;
    for (i = 0; i < n; i++) {
        for (k = 0, sd = 0; k < m; k++) { float t = At[i * m + k]; sd += (double)t * t; }
        W[i] = sqrt(sd);
    }
    for (i = 0; i < n - 1; i++) {
        j = i;
        for (k = i + 1; k < n; k++) if (W[j] < W[k]) j = k;
        if (i != j) {
            double t = W[i]; W[i] = W[j]; W[j] = t;
            for (k = 0; k < m; k++) { float u = At[i * m + k]; At[i * m + k] = At[j * m + k]; At[j * m + k] = u; }
            for (k = 0; k < n; k++) { float u = Vt[i * n + k]; Vt[i * n + k] = Vt[j * n + k]; Vt[j * n + k] = u; }
        }
    }
    for (i = 0; i < n; i++) Wout[i] = (float)W[i];
    uint64_t rng = 0x12345678;
    for (i = 0; i < n; i++) {
        sd = W[i];
        /* bounded as OpenCV 3.x / 4.x write it (`ii < 100 && sd <= minval`, then `sd > minval ? 1/sd
           : 0`); 2.4.9's unbounded loop and 1/sd differ only where it would not terminate */
        for (int ii = 0; ii < 100 && sd <= minval; ii++) {
            const float val0 = (float)(1. / m);
            for (k = 0; k < m; k++) At[i * m + k] = (cv_rng_next(&rng) & 256) != 0 ? val0 : -val0;
            for (iter = 0; iter < 2; iter++)
                for (j = 0; j < i; j++) {
                    sd = 0;
                    for (k = 0; k < m; k++) sd += At[i * m + k] * At[j * m + k];
                    float asum = 0;
                    for (k = 0; k < m; k++) {
                        float t = (float)(At[i * m + k] - sd * At[j * m + k]);
                        At[i * m + k] = t;
                        asum += fabsf(t);
                    }
                    asum = asum > eps * 100 ? 1 / asum : 0;
                    for (k = 0; k < m; k++) At[i * m + k] *= asum;
                }
            sd = 0;
            for (k = 0; k < m; k++) { float t = At[i * m + k]; sd += (double)t * t; }
            sd = sqrt(sd);
        }
        float s = (float)(sd > minval ? 1 / sd : 0.);
        for (k = 0; k < m; k++) At[i * m + k] *= s;
    }
}

/* cv::solve(A, b, x, DECOMP_SVD) for a float 6x6 and one right-hand side (lapack.cpp): the work
   matrix is transpose(A); JacobiSVD; SVBkSbImpl_<float>(m, n, w, u = work rows (uT), v = Vt (vT),
   b, nb = 1) with threshold = (sum w) * (float)(2 DBL_EPSILON) */
void tfo_cv_solve_svd6(const float A[36], const float b[6], float x[6])
{
    float At[36], w[6], Vt[36];
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) At[i * 6 + j] = A[j * 6 + i];
    tfo_cv_jacobi_svd(At, w, Vt, 6, 6);
    const float eps = (float)(DBL_EPSILON * 2);
    double threshold = 0;
    for (int i = 0; i < 6; i++) threshold += w[i];
    threshold *= eps;
    for (int j = 0; j < 6; j++) x[j] = 0;
    for (int i = 0; i < 6; i++) {
        double wi = w[i];
        if ((double)fabs(wi) <= threshold) continue;
        wi = 1 / wi;
        double s = 0;
        for (int j = 0; j < 6; j++) s += At[i * 6 + j] * b[j];      /* float product, double sum */
        s *= wi;
        for (int j = 0; j < 6; j++) x[j] = (float)(x[j] + s * Vt[i * 6 + j]);
    }
}

/* cv::Affine3f(rvec, t)'s rotation: Affine3<float>::rotation(const Vec3f&) (affine.hpp) */
void tfo_cv_rodrigues(const float rv[3], float R[9], int mode)
{
    double theta;
    if (mode == TFO_POSE_OPENCV2) {        /* norm(Matx): normL2Sqr<float, double> */
        double s2 = 0;
        for (int i = 0; i < 3; ++i) { double v = rv[i]; s2 += v * v; }
        theta = sqrt(s2);
    } else {                               /* normL2Sqr<float, DataType<float>::work_type = float> */
        float s2 = 0;
        for (int i = 0; i < 3; ++i) { float v = rv[i]; s2 += v * v; }
        theta = sqrtf(s2);
    }
    if (theta < DBL_EPSILON) {
        for (int k = 0; k < 9; ++k) R[k] = (k % 4 == 0) ? 1.0f : 0.0f;
        return;
    }
    double s, c;
    pose_sincos(theta, &s, &c);
    double c1 = 1. - c;
    double itheta = (theta != 0) ? 1. / theta : 0.;
    const float rx = (float)(rv[0] * itheta), ry = (float)(rv[1] * itheta), rz = (float)(rv[2] * itheta);
    const float rrt[9] = { rx * rx, rx * ry, rx * rz, rx * ry, ry * ry, ry * rz, rx * rz, ry * rz, rz * rz };
    const float rxm[9] = { 0, -rz, ry, rz, 0, -rx, -ry, rx, 0 };
    for (int k = 0; k < 9; ++k) {
        const float I = (k % 4 == 0) ? 1.0f : 0.0f;
        const float cI = (float)(I * c), crr = (float)(rrt[k] * c1), sx = (float)(rxm[k] * s);
        const float t = cI + crr;
        R[k] = t + sx;
    }
}

/* one iteration of estimateTransform after the reductions, projective_icp.cpp:187-210
   (StreamHelper::get unpacking :43-62) */
/* the canonical algebra's determinant and solve (the forms tfo_icp_step uses), exported for the
   solve-only parity test (tests/test_gpu_pose_algebra.py) */
void tfo_solve6(const float A[36], const float b[6], float x[6]) { solve6(A, b, x); }
double tfo_det6(const float A[36]) { return cv_det6(A); }

/* test-only capture of every ICP step's 27 sums (tools/svd_systems.py: realistic inputs for the
   Jacobi-SVD micro-benchmarks); off unless a buffer is installed */
static float* g_cap_buf;
static long long g_cap_cap, g_cap_n;
void tfo_capture_sums(float* buf, long long cap) { g_cap_buf = buf; g_cap_cap = cap; g_cap_n = 0; }
long long tfo_captured_sums(void) { return g_cap_n; }

int tfo_icp_step(const float s[27], float affine[12], double* det_out)
{
    if (g_cap_buf && g_cap_n < g_cap_cap) memcpy(g_cap_buf + 27 * g_cap_n++, s, 27 * sizeof(float));
    float A[36], b[6];
    int shift = 0;
    for (int i = 0; i < 6; ++i)
        for (int j = i; j < 7; ++j) {
            float value = s[shift++];
            if (j == 6) b[i] = value;
            else A[j * 6 + i] = A[i * 6 + j] = value;
        }
    const int cv = g_pose_algebra != TFO_POSE_CANONICAL;
    double det = cv ? tfo_cv_det6(A, g_pose_algebra) : cv_det6(A);
    if (det_out) *det_out = det;
    if (fabs(det) < 1e-15 || isnan(det)) return 0;
    float r[6];
    if (cv) tfo_cv_solve_svd6(A, b, r);
    else solve6(A, b, r);
    float tinc[12], R[9];
    if (cv) tfo_cv_rodrigues(r, R, g_pose_algebra);
    else tfo_rodrigues(r, R);
    for (int j = 0; j < 3; ++j) {
        tinc[j * 4 + 0] = R[j * 3 + 0]; tinc[j * 4 + 1] = R[j * 3 + 1]; tinc[j * 4 + 2] = R[j * 3 + 2];
        tinc[j * 4 + 3] = r[3 + j];
    }
    tfo_rigid_mul(tinc, affine, affine);   /* affine = Tinc * affine */
    return 1;
}

/* ------------------------------------------------------------------------- */
/* Scene / pipeline context                                                  */
/* ------------------------------------------------------------------------- */

struct tfo_ctx {
    tfo_params p;
    int n_total;
    tfo_hash_entry* hash;
    int* excessList;
    tfo_voxel* vba;
    int* allocList;
    int lastFreeBlockId, lastFreeExcessListId;
    int alloc_failed[2];      /* the last allocateVoxelBlocksList's failed type-1 / type-2 requests */
    /* SceneReconstructionEngine_CUDA temporaries */
    uint8_t* allocType;
    int16_t* blockCoords;     /* 4 shorts per entry */
    /* RenderState_VH */
    int* visibleIds;
    int noVisibleEntries;
    uint8_t* visType;
    float* range;             /* float2 */
    float* raycast;           /* float4 */
    int noTotalBlocks;
    /* TopFu */
    int frame_counter;
    float pose[12];
    float* dists;
    uint8_t* frame_grey;      /* the image renderImage produced inside the last tracked frame */
    uint16_t* depth_pyr[3];
    float* curr_pts[3]; float* curr_nrm[3];
    float* prev_pts[3]; float* prev_nrm[3];
    int lvl_w[3], lvl_h[3];
    int icp_iterations, icp_ok, n_resets;
    /* swapping: GlobalCache (GlobalCache.hpp:11-134) kept per hash entry */
    uint8_t* swapState;       /* HashSwapState::state */
    uint8_t* hasStored;       /* hasStoredData */
    tfo_voxel* stored;        /* storedVoxelBlocks, 512 voxels per entry */
    int swap_counts[3];       /* last frame: swapped in, swapped out, reallocated */
    long long swap_merged_total;  /* swap-ins that merged stored data (GlobalCache -> VBA), since creation */
    /* colour (voxel_rgb): Voxel_s_rgb's clr + w_color per voxel, r | g << 8 | b << 16 | w << 24,
       beside the Voxel_s plane (VoxelTypes.hpp:39-67); the frame's RGB image while integrating */
    uint32_t* vba_rgb;
    const uint8_t* rgb_in;
    size_t rgb_pitch;
};

static const float k_identity_rt[12] = { 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0 };

/* ResetScene, SceneReconstructionEngine_host.cu:51-73; clear_cache: the TopFu-level resets also
   empty the GlobalCache (see below), the engine's ResetScene (tfo_reset_scene) keeps it */
static void reset_scene_ex(tfo_ctx* c, int clear_cache)
{
    for (size_t i = 0; i < (size_t)c->p.n_blocks * BLK3; ++i) { c->vba[i].sdf = 32767; c->vba[i].w = 0; c->vba[i].pad = 0; }
    for (int i = 0; i < c->p.n_blocks; ++i) c->allocList[i] = i;
    c->lastFreeBlockId = c->p.n_blocks - 1;
    memset(c->hash, 0, sizeof(tfo_hash_entry) * (size_t)c->n_total);
    for (int i = 0; i < c->n_total; ++i) c->hash[i].ptr = -2;
    for (int i = 0; i < c->p.n_excess; ++i) c->excessList[i] = i;
    c->lastFreeExcessListId = c->p.n_excess - 1;
    /* the reference's ResetScene leaves a GlobalCache alone (its swapping is never enabled), and so
       does tfo_reset_scene; the TopFu-level resets (construction, TopFu::reset, the ICP-failure
       reset) also empty it, so no block of the old scene is swapped into the new one */
    if (c->vba_rgb) memset(c->vba_rgb, 0, sizeof(uint32_t) * (size_t)c->p.n_blocks * BLK3);   /* Voxel_s_rgb(): clr 0, w 0 */
    memset(c->swap_counts, 0, sizeof(c->swap_counts));   /* a reset transfers nothing */
    if (c->p.use_swapping && clear_cache) {
        memset(c->swapState, 0, (size_t)c->n_total);
        memset(c->hasStored, 0, (size_t)c->n_total);
    }
}

static void reset_scene(tfo_ctx* c) { reset_scene_ex(c, 1); }

/* SceneReconstructionEngine::ResetScene as an engine call: the GlobalCache stays */
void tfo_reset_scene(tfo_ctx* c) { reset_scene_ex(c, 0); }

long long tfo_swap_merged_total(const tfo_ctx* c) { return c->swap_merged_total; }

tfo_ctx* tfo_create(const tfo_params* p)
{
    tfo_ctx* c = (tfo_ctx*)calloc(1, sizeof(tfo_ctx));
    c->p = *p;
    c->n_total = p->n_buckets + p->n_excess;
    c->hash = (tfo_hash_entry*)malloc(sizeof(tfo_hash_entry) * (size_t)c->n_total);
    c->excessList = (int*)malloc(sizeof(int) * (size_t)p->n_excess);
    c->vba = (tfo_voxel*)malloc(sizeof(tfo_voxel) * (size_t)p->n_blocks * BLK3);
    c->allocList = (int*)malloc(sizeof(int) * (size_t)p->n_blocks);
    c->allocType = (uint8_t*)calloc((size_t)c->n_total, 1);
    c->blockCoords = (int16_t*)calloc((size_t)c->n_total * 4, sizeof(int16_t));
    c->visibleIds = (int*)calloc((size_t)p->vis_capacity, sizeof(int));
    c->visType = (uint8_t*)calloc((size_t)c->n_total, 1);
    size_t npx = (size_t)p->cols * p->rows;
    c->range = (float*)malloc(sizeof(float) * 2 * npx);
    for (size_t i = 0; i < npx; ++i) { c->range[2 * i] = p->viewFrustum_min; c->range[2 * i + 1] = p->viewFrustum_max; } /* RenderState.hpp:56-76 */
    c->raycast = (float*)calloc(4 * npx, sizeof(float));
    c->dists = (float*)calloc(npx, sizeof(float));
    c->frame_grey = (uint8_t*)calloc(npx * 4, 1);
    int w = p->cols, h = p->rows;
    for (int l = 0; l < 3; ++l) {
        c->lvl_w[l] = w; c->lvl_h[l] = h;
        c->depth_pyr[l] = (uint16_t*)calloc((size_t)w * h, sizeof(uint16_t));
        c->curr_pts[l] = (float*)calloc((size_t)w * h * 4, sizeof(float));
        c->curr_nrm[l] = (float*)calloc((size_t)w * h * 4, sizeof(float));
        c->prev_pts[l] = (float*)calloc((size_t)w * h * 4, sizeof(float));
        c->prev_nrm[l] = (float*)calloc((size_t)w * h * 4, sizeof(float));
        w /= 2; h /= 2;
    }
    if (p->use_swapping) {
        c->swapState = (uint8_t*)calloc((size_t)c->n_total, 1);
        c->hasStored = (uint8_t*)calloc((size_t)c->n_total, 1);
        c->stored = (tfo_voxel*)calloc((size_t)c->n_total * BLK3, sizeof(tfo_voxel));
    }
    if (p->voxel_rgb) c->vba_rgb = (uint32_t*)calloc((size_t)p->n_blocks * BLK3, sizeof(uint32_t));
    reset_scene(c);                                   /* topfu.cpp:75 */
    memcpy(c->pose, k_identity_rt, sizeof(c->pose));  /* reset(), topfu.cpp:141-152 */
    c->frame_counter = 0;
    return c;
}

void tfo_destroy(tfo_ctx* c)
{
    if (!c) return;
    free(c->hash); free(c->excessList); free(c->vba); free(c->allocList); free(c->allocType);
    free(c->blockCoords); free(c->visibleIds); free(c->visType); free(c->range); free(c->raycast); free(c->dists); free(c->frame_grey);
    for (int l = 0; l < 3; ++l) {
        free(c->depth_pyr[l]); free(c->curr_pts[l]); free(c->curr_nrm[l]); free(c->prev_pts[l]); free(c->prev_nrm[l]);
    }
    free(c->swapState); free(c->hasStored); free(c->stored); free(c->vba_rgb);
    free(c);
}

/* Deep copy of a context's whole state (scene, render state, pyramids, pose, counters) into
   another created with the same params: a benchmark sample starts at frame k of a stream
   without re-running frames 0..k-1.  Not a reference function.  The serial and OpenMP builds
   compile this same struct, so one build's context may be the source of the other's copy. */
int tfo_copy_state(tfo_ctx* d, const tfo_ctx* s)
{
    if (!d || !s || memcmp(&d->p, &s->p, sizeof(tfo_params)) != 0) return -1;
    const size_t nt = (size_t)s->n_total, nb = (size_t)s->p.n_blocks, npx = (size_t)s->p.cols * s->p.rows;
    memcpy(d->hash, s->hash, sizeof(tfo_hash_entry) * nt);
    memcpy(d->excessList, s->excessList, sizeof(int) * (size_t)s->p.n_excess);
    memcpy(d->vba, s->vba, sizeof(tfo_voxel) * nb * BLK3);
    memcpy(d->allocList, s->allocList, sizeof(int) * nb);
    memcpy(d->allocType, s->allocType, nt);
    memcpy(d->blockCoords, s->blockCoords, sizeof(int16_t) * nt * 4);
    memcpy(d->visibleIds, s->visibleIds, sizeof(int) * (size_t)s->p.vis_capacity);
    memcpy(d->visType, s->visType, nt);
    memcpy(d->range, s->range, sizeof(float) * 2 * npx);
    memcpy(d->raycast, s->raycast, sizeof(float) * 4 * npx);
    memcpy(d->dists, s->dists, sizeof(float) * npx);
    memcpy(d->frame_grey, s->frame_grey, 4 * npx);
    for (int l = 0; l < 3; ++l) {
        const size_t n = (size_t)s->lvl_w[l] * s->lvl_h[l];
        memcpy(d->depth_pyr[l], s->depth_pyr[l], sizeof(uint16_t) * n);
        memcpy(d->curr_pts[l], s->curr_pts[l], sizeof(float) * 4 * n);
        memcpy(d->curr_nrm[l], s->curr_nrm[l], sizeof(float) * 4 * n);
        memcpy(d->prev_pts[l], s->prev_pts[l], sizeof(float) * 4 * n);
        memcpy(d->prev_nrm[l], s->prev_nrm[l], sizeof(float) * 4 * n);
    }
    if (s->p.use_swapping) {
        memcpy(d->swapState, s->swapState, nt);
        memcpy(d->hasStored, s->hasStored, nt);
        memcpy(d->stored, s->stored, sizeof(tfo_voxel) * nt * BLK3);
    }
    if (s->p.voxel_rgb) memcpy(d->vba_rgb, s->vba_rgb, sizeof(uint32_t) * nb * BLK3);
    d->lastFreeBlockId = s->lastFreeBlockId; d->lastFreeExcessListId = s->lastFreeExcessListId;
    d->alloc_failed[0] = s->alloc_failed[0]; d->alloc_failed[1] = s->alloc_failed[1];
    d->noVisibleEntries = s->noVisibleEntries; d->noTotalBlocks = s->noTotalBlocks;
    d->frame_counter = s->frame_counter;
    memcpy(d->pose, s->pose, sizeof(d->pose));
    d->icp_iterations = s->icp_iterations; d->icp_ok = s->icp_ok; d->n_resets = s->n_resets;
    memcpy(d->swap_counts, s->swap_counts, sizeof(d->swap_counts));
    d->swap_merged_total = s->swap_merged_total;
    return 0;
}

void tfo_reset(tfo_ctx* c)
{   /* TopFu::reset, topfu.cpp:141-152 (render state is NOT cleared) */
    if (c->frame_counter) c->n_resets++;
    c->frame_counter = 0;
    memcpy(c->pose, k_identity_rt, sizeof(c->pose));
    reset_scene(c);
}

/* hashIndex, RepresentationAccess.hpp:5-7 */
static inline int hash_index(const tfo_ctx* c, int x, int y, int z)
{
    return (int)((((uint32_t)x * 73856093u) ^ ((uint32_t)y * 19349669u) ^ ((uint32_t)z * 83492791u)) & (uint32_t)(c->p.n_buckets - 1));
}

/* buildHashAllocAndVisibleTypePP, SceneReconstructionEngine.hpp:206-298 */
static void build_hash_alloc_pixel(tfo_ctx* c, int x, int y, const float* depth, const float invM[16],
                                   const float proj[4], float mu, float oneOverVoxelSize)
{
    int W = c->p.cols;
    float depth_measure = depth[x + y * W];
    if (depth_measure <= 0 || (depth_measure - mu) < 0 || (depth_measure - mu) < c->p.viewFrustum_min ||
        (depth_measure + mu) > c->p.viewFrustum_max) return;
    float pc[4];
    pc[2] = depth_measure;
    pc[0] = pc[2] * (((float)x - proj[2]) * proj[0]);
    pc[1] = pc[2] * (((float)y - proj[3]) * proj[1]);
    float norm = sqrtf(pc[0] * pc[0] + pc[1] * pc[1] + pc[2] * pc[2]);
    float buf[4], r[4], point[3], point_e[3], dir[3];
    float s1 = 1.0f - mu / norm;
    buf[0] = pc[0] * s1; buf[1] = pc[1] * s1; buf[2] = pc[2] * s1; buf[3] = 1.0f;
    m4v(invM, buf, r);
    point[0] = r[0] * oneOverVoxelSize; point[1] = r[1] * oneOverVoxelSize; point[2] = r[2] * oneOverVoxelSize;
    float s2 = 1.0f + mu / norm;
    buf[0] = pc[0] * s2; buf[1] = pc[1] * s2; buf[2] = pc[2] * s2; buf[3] = 1.0f;
    m4v(invM, buf, r);
    point_e[0] = r[0] * oneOverVoxelSize; point_e[1] = r[1] * oneOverVoxelSize; point_e[2] = r[2] * oneOverVoxelSize;
    dir[0] = point_e[0] - point[0]; dir[1] = point_e[1] - point[1]; dir[2] = point_e[2] - point[2];
    norm = sqrtf(dir[0] * dir[0] + dir[1] * dir[1] + dir[2] * dir[2]);
    int noSteps = (int)ceilf(2.0f * norm);
    float dv = (float)(noSteps - 1);
    dir[0] /= dv; dir[1] /= dv; dir[2] /= dv;
    for (int i = 0; i < noSteps; i++) {
        int16_t bx = (int16_t)floorf(point[0]), by = (int16_t)floorf(point[1]), bz = (int16_t)floorf(point[2]);
        int hashIdx = hash_index(c, bx, by, bz);
        int isFound = 0;
        tfo_hash_entry e = c->hash[hashIdx];
        if (e.x == bx && e.y == by && e.z == bz && e.ptr >= -1) {
            c->visType[hashIdx] = (e.ptr == -1) ? 2 : 1;
            isFound = 1;
        }
        if (!isFound) {
            int isExcess = 0;
            if (e.ptr >= -1) {
                while (e.offset >= 1) {
                    hashIdx = c->p.n_buckets + e.offset - 1;
                    e = c->hash[hashIdx];
                    if (e.x == bx && e.y == by && e.z == bz && e.ptr >= -1) {
                        c->visType[hashIdx] = (e.ptr == -1) ? 2 : 1;
                        isFound = 1;
                        break;
                    }
                }
                isExcess = 1;
            }
            if (!isFound) {
                c->allocType[hashIdx] = isExcess ? 2 : 1;
                if (!isExcess) c->visType[hashIdx] = 1;
                c->blockCoords[4 * hashIdx + 0] = bx; c->blockCoords[4 * hashIdx + 1] = by;
                c->blockCoords[4 * hashIdx + 2] = bz; c->blockCoords[4 * hashIdx + 3] = 1;
            }
        }
        point[0] += dir[0]; point[1] += dir[1]; point[2] += dir[2];
    }
}

/* checkPointVisibility<false> / checkBlockVisibility<false>, SceneReconstructionEngine.hpp:300-375 */
static inline int check_point_visibility(const float pt[4], const float M[16], const float proj[4], int W, int H)
{
    float b[4];
    m4v(M, pt, b);
    if (b[2] < 1e-10f) return 0;
    b[0] = proj[0] * b[0] / b[2] + proj[2];
    b[1] = proj[1] * b[1] / b[2] + proj[3];
    return (b[0] >= 0 && b[0] < (float)W && b[1] >= 0 && b[1] < (float)H);
}

/* checkPointVisibility<true>'s enlarged frustum (SceneReconstructionEngine.hpp:315-321): the
   image grown by an eighth of its size on every side, integer limits */
static inline int check_point_enlarged(const float pt[4], const float M[16], const float proj[4], int W, int H)
{
    float b[4];
    m4v(M, pt, b);
    if (b[2] < 1e-10f) return 0;
    b[0] = proj[0] * b[0] / b[2] + proj[2];
    b[1] = proj[1] * b[1] / b[2] + proj[3];
    const int lx = -W / 8, ux = W + W / 8, ly = -H / 8, uy = H + H / 8;
    return (b[0] >= (float)lx && b[0] < (float)ux && b[1] >= (float)ly && b[1] < (float)uy);
}

/* checkBlockVisibility<true>'s isVisibleEnlarged: any of the 8 corners in the enlarged frustum
   (a corner inside the image is inside it too, so the early return on isVisible changes nothing) */
static int check_block_enlarged(int16_t px, int16_t py, int16_t pz, const float M[16], const float proj[4],
                                float voxelSize, int W, int H)
{
    float factor = (float)BLK * voxelSize;
    float pt[4];
    pt[0] = (float)px * factor; pt[1] = (float)py * factor; pt[2] = (float)pz * factor; pt[3] = 1.0f;
    if (check_point_enlarged(pt, M, proj, W, H)) return 1;
    pt[2] += factor;
    if (check_point_enlarged(pt, M, proj, W, H)) return 1;
    pt[1] += factor;
    if (check_point_enlarged(pt, M, proj, W, H)) return 1;
    pt[0] += factor;
    if (check_point_enlarged(pt, M, proj, W, H)) return 1;
    pt[2] -= factor;
    if (check_point_enlarged(pt, M, proj, W, H)) return 1;
    pt[1] -= factor;
    if (check_point_enlarged(pt, M, proj, W, H)) return 1;
    pt[0] -= factor; pt[1] += factor;
    if (check_point_enlarged(pt, M, proj, W, H)) return 1;
    pt[0] += factor; pt[1] -= factor; pt[2] += factor;
    if (check_point_enlarged(pt, M, proj, W, H)) return 1;
    return 0;
}

static int check_block_visibility(int16_t px, int16_t py, int16_t pz, const float M[16], const float proj[4],
                                  float voxelSize, int W, int H)
{
    float factor = (float)BLK * voxelSize;
    float pt[4];
    pt[0] = (float)px * factor; pt[1] = (float)py * factor; pt[2] = (float)pz * factor; pt[3] = 1.0f;
    if (check_point_visibility(pt, M, proj, W, H)) return 1;
    pt[2] += factor;                                  /* 0 0 1 */
    if (check_point_visibility(pt, M, proj, W, H)) return 1;
    pt[1] += factor;                                  /* 0 1 1 */
    if (check_point_visibility(pt, M, proj, W, H)) return 1;
    pt[0] += factor;                                  /* 1 1 1 */
    if (check_point_visibility(pt, M, proj, W, H)) return 1;
    pt[2] -= factor;                                  /* 1 1 0 */
    if (check_point_visibility(pt, M, proj, W, H)) return 1;
    pt[1] -= factor;                                  /* 1 0 0 */
    if (check_point_visibility(pt, M, proj, W, H)) return 1;
    pt[0] -= factor; pt[1] += factor;                 /* 0 1 0 */
    if (check_point_visibility(pt, M, proj, W, H)) return 1;
    pt[0] += factor; pt[1] -= factor; pt[2] += factor; /* 1 0 1 */
    if (check_point_visibility(pt, M, proj, W, H)) return 1;
    return 0;
}

/* AllocateSceneFromDepth, SceneReconstructionEngine_host.cu:75-195 (+ kernels :331-479), with the
   onlyUpdateVisibleList (:160-168: no allocation pass) and resetVisibleList (:88) arguments */
void tfo_alloc_ex(tfo_ctx* c, const float pose_rt[12], const float* dists, int only_update_visible, int reset_visible)
{
    int W = c->p.cols, H = c->p.rows;
    float M[16], invM[16];
    rt_to_m4(pose_rt, M);
    tfo_matrix4_inv(M, invM);
    float proj[4] = { c->p.fx, c->p.fy, c->p.cx, c->p.cy };
    float invProj[4] = { 1.0f / proj[0], 1.0f / proj[1], proj[2], proj[3] };
    float mu = c->p.mu;
    float oneOverVoxelSize = 1.0f / (c->p.voxelSize * (float)BLK);
    int noAllocatedVoxelEntries = c->lastFreeBlockId;
    int noAllocatedExcessEntries = c->lastFreeExcessListId;
    int noVisibleEntries = 0;
    if (reset_visible) c->noVisibleEntries = 0;
    memset(c->allocType, 0, (size_t)c->n_total);
    c->alloc_failed[0] = c->alloc_failed[1] = 0;
    /* setToType3, :343-348 */
    for (int i = 0; i < c->noVisibleEntries; ++i) c->visType[c->visibleIds[i]] = 3;
    /* buildHashAllocAndVisibleType_device, :331-341, serial raster order */
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x)
            build_hash_alloc_pixel(c, x, y, dists, invM, invProj, mu, oneOverVoxelSize);
    /* allocateVoxelBlocksList_device, :350-415, serial in index order */
    for (int t = 0; t < c->n_total && !only_update_visible; ++t) {
        int vbaIdx, exlIdx;
        switch (c->allocType[t]) {
        case 1:
            vbaIdx = noAllocatedVoxelEntries--;
            if (vbaIdx >= 0) {
                tfo_hash_entry e;
                e.x = c->blockCoords[4 * t]; e.y = c->blockCoords[4 * t + 1]; e.z = c->blockCoords[4 * t + 2]; e.pad = 0;
                e.ptr = c->allocList[vbaIdx];
                e.offset = 0;
                c->hash[t] = e;
            } else {
                c->visType[t] = 0;
                noAllocatedVoxelEntries++;
                c->alloc_failed[0]++;
            }
            break;
        case 2:
            vbaIdx = noAllocatedVoxelEntries--;
            exlIdx = noAllocatedExcessEntries--;
            if (vbaIdx >= 0 && exlIdx >= 0) {
                tfo_hash_entry e;
                e.x = c->blockCoords[4 * t]; e.y = c->blockCoords[4 * t + 1]; e.z = c->blockCoords[4 * t + 2]; e.pad = 0;
                e.ptr = c->allocList[vbaIdx];
                e.offset = 0;
                int exlOffset = c->excessList[exlIdx];
                c->hash[t].offset = exlOffset + 1;
                c->hash[c->p.n_buckets + exlOffset] = e;
                c->visType[c->p.n_buckets + exlOffset] = 1;
            } else {
                noAllocatedVoxelEntries++;
                noAllocatedExcessEntries++;
                c->alloc_failed[1]++;
            }
            break;
        default: break;
        }
    }
    /* buildVisibleList_device<useSwapping>, :434-479, compaction in index order; swapping
       (:159-160, never with onlyUpdateVisibleList): the enlarged frustum for type-3 entries
       and swap state 1 ("needed") for every listed entry not already in active memory (2) */
    const int swapping = c->p.use_swapping && !only_update_visible;
    for (int t = 0; t < c->n_total; ++t) {
        uint8_t vt = c->visType[t];
        if (vt == 3) {
            const tfo_hash_entry* e = &c->hash[t];
            if (swapping ? !check_block_enlarged(e->x, e->y, e->z, M, proj, c->p.voxelSize, W, H)
                         : !check_block_visibility(e->x, e->y, e->z, M, proj, c->p.voxelSize, W, H)) vt = 0;
            c->visType[t] = vt;
        }
        if (vt > 0) {
            if (swapping && c->swapState[t] != 2) c->swapState[t] = 1;
            if (noVisibleEntries < c->p.vis_capacity) c->visibleIds[noVisibleEntries] = t;
            noVisibleEntries++;
        }
    }
    if (noVisibleEntries > c->p.vis_capacity) noVisibleEntries = c->p.vis_capacity;
    /* reAllocateSwappedOutVoxelBlocks_device (:184-189, 417-432): listed entries whose block
       was swapped out (ptr == -1) get a block again, in ascending index order */
    c->swap_counts[2] = 0;
    if (swapping)
        for (int t = 0; t < c->n_total; ++t) {
            if (c->visType[t] > 0 && c->hash[t].ptr == -1) {
                int vbaIdx = noAllocatedVoxelEntries--;
                if (vbaIdx >= 0) { c->hash[t].ptr = c->allocList[vbaIdx]; c->swap_counts[2]++; }
                else noAllocatedVoxelEntries++;
            }
        }
    c->noVisibleEntries = noVisibleEntries;
    c->lastFreeBlockId = noAllocatedVoxelEntries;
    c->lastFreeExcessListId = noAllocatedExcessEntries;
}

void tfo_alloc(tfo_ctx* c, const float pose_rt[12], const float* dists)
{
    tfo_alloc_ex(c, pose_rt, dists, 0, 0);
}

/* ------------------------------------------------------------------------- */
/* Swapping.  The reference has the GlobalCache (GlobalCache.hpp:11-134: per-entry host
   store, hasStoredData, swap states 0 / 1 / 2, SDF_TRANSFER_BLOCK_NUM blocks per transfer)
   and the swapping branches of AllocateSceneFromDepth (above), but not the engine that moves
   blocks (CUDAInstantiations.cu:8 comments out ITMSwappingEngine_CUDA).  The engine restated
   here is the published algorithm of that lineage (InfiniTAM v3 ITMSwappingEngine_CUDA /
   ITMSwappingEngine_Shared.h, not vendored): after integration,
     IntegrateGlobalIntoLocal: entries in state 1 (ascending index, at most T) take their
       stored block back -- CombineVoxelInformation merges it into the active block by weight
       (skipped where the stored weight is 0) -- and go to state 2;
     SaveToGlobalMemory: entries in state 2 with a block and not visible this frame
       (ascending, at most T) are copied to the store, their block reset to Voxel_s() and
       returned to the free list (cleanMemory: allocList[++lastFreeBlockId] = ptr, ptr = -1),
       state 0.
   Canonical order: ascending hash index where the lineage uses atomics.  One guard: an entry in
   state 1 without a block (its reallocation failed) is not swapped in (the lineage would write
   through ptr = -1). */
/* ------------------------------------------------------------------------- */
/* CombineVoxelInformation (depth part), ITMSwappingEngine_Shared.h: src = stored, dst = active */
static inline void combine_voxel(const tfo_voxel* src, tfo_voxel* dst, int maxW)
{
    int newW = dst->w;
    int oldW = src->w;
    float newF = (float)dst->sdf / 32767.0f;
    float oldF = (float)src->sdf / 32767.0f;
    if (oldW == 0) return;
    newF = (float)oldW * oldF + (float)newW * newF;
    newW = oldW + newW;
    newF /= (float)newW;
    newW = (newW < maxW) ? newW : maxW;
    dst->w = (uint8_t)newW;
    dst->sdf = (int16_t)(newF * 32767.0f);
}

void tfo_swap_in(tfo_ctx* c)                                            /* IntegrateGlobalIntoLocal */
{
    if (!c->p.use_swapping) return;
    const int T = c->p.swap_transfer_blocks;
    int n_in = 0;
    for (int t = 0; t < c->n_total && n_in < T; ++t) {
        if (c->swapState[t] != 1 || c->hash[t].ptr < 0) continue;
        if (c->hasStored[t]) {
            tfo_voxel* dst = c->vba + (size_t)c->hash[t].ptr * BLK3;
            const tfo_voxel* src = c->stored + (size_t)t * BLK3;
            for (int v = 0; v < BLK3; ++v) combine_voxel(&src[v], &dst[v], c->p.maxW);
            c->swap_merged_total++;
        }
        c->swapState[t] = 2;
        n_in++;
    }
    c->swap_counts[0] = n_in;
}

void tfo_swap_out(tfo_ctx* c)                                           /* SaveToGlobalMemory */
{
    if (!c->p.use_swapping) return;
    const int T = c->p.swap_transfer_blocks;
    int n_out = 0;
    for (int t = 0; t < c->n_total && n_out < T; ++t) {
        if (c->swapState[t] != 2 || c->hash[t].ptr < 0 || c->visType[t] != 0) continue;
        tfo_voxel* blk = c->vba + (size_t)c->hash[t].ptr * BLK3;
        memcpy(c->stored + (size_t)t * BLK3, blk, sizeof(tfo_voxel) * BLK3);   /* moveActiveDataToTransferBuffer */
        c->hasStored[t] = 1;
        for (int v = 0; v < BLK3; ++v) { blk[v].sdf = 32767; blk[v].w = 0; blk[v].pad = 0; }
        c->swapState[t] = 0;                                            /* cleanMemory */
        int vbaIdx = c->lastFreeBlockId++;
        if (vbaIdx < c->p.n_blocks - 1) {
            c->allocList[vbaIdx + 1] = c->hash[t].ptr;
            c->hash[t].ptr = -1;
        }
        n_out++;
    }
    c->swap_counts[1] = n_out;
}

void tfo_swap(tfo_ctx* c)
{
    tfo_swap_in(c);
    tfo_swap_out(c);
}

void tfo_swap_counts(const tfo_ctx* c, int out[3]) { memcpy(out, c->swap_counts, sizeof(int) * 3); }
uint8_t* tfo_swap_state(tfo_ctx* c) { return c->swapState; }
uint8_t* tfo_swap_stored_flags(tfo_ctx* c) { return c->hasStored; }
tfo_voxel* tfo_swap_stored(tfo_ctx* c) { return c->stored; }

/* computeUpdatedVoxelDepthInfo, SceneReconstructionEngine.hpp:23-71; returns eta, or -1 where the
   voxel projects behind the camera / outside the image or onto no depth (its return values) */
static inline float update_voxel(tfo_voxel* v, const float pt_model[4], const float M[16], const float proj[4],
                                 float mu, int maxW, const float* depth, int W, int H)
{
    float pc[4];
    m4v(M, pt_model, pc);
    if (pc[2] <= 0) return -1;
    /* fx * x / z under --prec-div=false (CMakeLists.txt:1): canonical (fx x) * RN(1/z) */
    const float rz = 1.0f / pc[2];
    float ix = (proj[0] * pc[0]) * rz + proj[2];
    float iy = (proj[1] * pc[1]) * rz + proj[3];
    if ((ix < 1) || (ix > (float)(W - 2)) || (iy < 1) || (iy > (float)(H - 2))) return -1;
    float depth_measure = depth[(int)(ix + 0.5f) + (int)(iy + 0.5f) * W];
    if (depth_measure <= 0.0f) return -1;
    float eta = depth_measure - pc[2];
    if (eta < -mu) return eta;
    tfo_tsdf_update(&v->sdf, &v->w, eta, mu, maxW);
    return eta;
}

/* Vector3f::toUChar: CLAMP((int)ROUND(v), 0, 255), Vector.hpp:242-244 */
static inline uint32_t u8_round(float v)
{
    int i = (int)((v < 0) ? (v - 0.5f) : (v + 0.5f));
    return (uint32_t)(i < 0 ? 0 : (i > 255 ? 255 : i));
}

/* computeUpdatedVoxelColorInfo, SceneReconstructionEngine.hpp:116-148, with interpolateBilinear
   (PixelUtils.hpp:8-32) of the uchar4 RGB image; called where ComputeUpdatedVoxelInfo<true, ...>
   (:163-176, the lineage's colour path) does: after the depth update, unless
   (eta > mu) || (fabs(eta / mu) > 0.25f).  One guard: a projection with pc.z == 0 (a NaN image
   position, undefined behaviour in the reference) is skipped. */
static inline void update_voxel_colour(uint32_t* clr, const float pt_model[4], const float Mr[16], const float proj[4],
                                       int maxW, const uint8_t* rgb, size_t pitch, int W, int H)
{
    float pc[4];
    m4v(Mr, pt_model, pc);
    const float rz = 1.0f / pc[2];                 /* (as update_voxel) */
    float ix = (proj[0] * pc[0]) * rz + proj[2];
    float iy = (proj[1] * pc[1]) * rz + proj[3];
    if (isnan(ix) || isnan(iy)) return;
    if ((ix < 1) || (ix > (float)(W - 2)) || (iy < 1) || (iy > (float)(H - 2))) return;
    float m4[4];
    tfo_interp_bilinear_u8x4(rgb, pitch, ix, iy, m4);
    *clr = tfo_colour_average(*clr, m4, maxW);
}

/* interpolateBilinear<uchar> (PixelUtils.hpp:8-32) of an RGBA8 image at (ix, iy) */
void tfo_interp_bilinear_u8x4(const uint8_t* rgb, size_t pitch, float ix, float iy, float out[4])
{
    int x0 = (int)floorf(ix), y0 = (int)floorf(iy);
    float dx = ix - (float)x0, dy = iy - (float)y0;
    static const uint8_t zero[4] = { 0, 0, 0, 0 };
    const uint8_t* a = rgb + (size_t)y0 * pitch + 4 * (size_t)x0;
    const uint8_t* b = zero; const uint8_t* cc = zero; const uint8_t* d = zero;
    if (dx != 0) b = a + 4;
    if (dy != 0) cc = a + pitch;
    if (dx != 0 && dy != 0) d = a + pitch + 4;
    for (int k = 0; k < 4; ++k)
        out[k] = ((float)a[k] * (1.0f - dx) * (1.0f - dy) + (float)b[k] * dx * (1.0f - dy) +
                  (float)cc[k] * (1.0f - dx) * dy + (float)d[k] * dx * dy);
}

/* the running colour average of computeUpdatedVoxelColorInfo (SceneReconstructionEngine.hpp:
   124-147) on a colour word r | g << 8 | b << 16 | w_color << 24, given the interpolated sample */
uint32_t tfo_colour_average(uint32_t clr, const float sample[4], int maxW)
{
    float oldW = (float)(clr >> 24);
    float oldC[3], newC[3];
    for (int k = 0; k < 3; ++k) oldC[k] = (float)((clr >> (8 * k)) & 0xffu) / 255.0f;
    float newW = 1;
    for (int k = 0; k < 3; ++k) {
        float m = sample[k] / 255.0f;
        newC[k] = oldC[k] * oldW + m * newW;
    }
    newW = oldW + newW;
    for (int k = 0; k < 3; ++k) newC[k] /= newW;
    float mw = (float)(uint8_t)maxW;
    newW = (newW < mw) ? newW : mw;
    return u8_round(newC[0] * 255.0f) | (u8_round(newC[1] * 255.0f) << 8) | (u8_round(newC[2] * 255.0f) << 16) |
           ((uint32_t)(uint8_t)newW << 24);
}

/* M_rgb = view->calib.trafo_rgb_to_depth.calib_inv * M_d (SceneReconstructionEngine_host.cu:217):
   Matrix4 operator* (Matrix.hpp:113-119), r(x, y) += lhs(k, y) * rhs(x, k) from zero */
static void rgb_matrix(const tfo_ctx* c, const float M[16], float Mr[16])
{
    float D[16];
    rt_to_m4(c->p.depth_to_rgb, D);
    for (int x = 0; x < 4; ++x)
        for (int y = 0; y < 4; ++y) {
            float r = 0.0f;
            for (int k = 0; k < 4; ++k) r += D[4 * k + y] * M[4 * x + k];
            Mr[4 * x + y] = r;
        }
}

static void rgb_proj(const tfo_ctx* c, float proj[4])
{
    const float* q = c->p.rgb_intr;
    if (q[0] == 0 && q[1] == 0 && q[2] == 0 && q[3] == 0) { proj[0] = c->p.fx; proj[1] = c->p.fy; proj[2] = c->p.cx; proj[3] = c->p.cy; }
    else { proj[0] = q[0]; proj[1] = q[1]; proj[2] = q[2]; proj[3] = q[3]; }
}

/* TSDF running average + Voxel_s quantisation, SceneReconstructionEngine.hpp:56-68, VoxelTypes.hpp:71-73 */
void tfo_tsdf_update(int16_t* sdf, uint8_t* w, float eta, float mu, int maxW)
{
    float oldF = (float)*sdf / 32767.0f;
    int oldW = *w;
    float newF = eta / mu;
    newF = (1.0f < newF) ? 1.0f : newF;
    int newW = 1;
    newF = (float)oldW * oldF + (float)newW * newF;
    newW = oldW + newW;
    newF /= (float)newW;
    newW = (newW < maxW) ? newW : maxW;
    *sdf = (int16_t)(newF * 32767.0f);
    *w = (uint8_t)newW;
}

/* IntegrateIntoScene + integrateIntoScene_device<Voxel_s,false>, SceneReconstructionEngine_host.cu:197-251,297-329;
   with voxel_rgb and a frame RGB image (c->rgb_in) the Voxel_s_rgb colour update after each voxel's depth update */
void tfo_integrate(tfo_ctx* c, const float pose_rt[12], const float* dists)
{
    if (c->noVisibleEntries == 0) return;
    float M[16], Mr[16], proj_rgb[4];
    rt_to_m4(pose_rt, M);
    float proj[4] = { c->p.fx, c->p.fy, c->p.cx, c->p.cy };
    float vs = c->p.voxelSize, mu = c->p.mu;
    const int colour = c->vba_rgb && c->rgb_in;
    if (colour) { rgb_matrix(c, M, Mr); rgb_proj(c, proj_rgb); }
#pragma omp parallel for schedule(dynamic, 16)
    for (int i = 0; i < c->noVisibleEntries; ++i) {
        const tfo_hash_entry* e = &c->hash[c->visibleIds[i]];
        if (e->ptr < 0) continue;
        int gx = e->x * BLK, gy = e->y * BLK, gz = e->z * BLK;
        tfo_voxel* blk = c->vba + (size_t)e->ptr * BLK3;
        for (int z = 0; z < BLK; ++z)
            for (int y = 0; y < BLK; ++y)
                for (int x = 0; x < BLK; ++x) {
                    float pm[4];
                    pm[0] = (float)(gx + x) * vs; pm[1] = (float)(gy + y) * vs; pm[2] = (float)(gz + z) * vs; pm[3] = 1.0f;
                    const int lin = x + y * BLK + z * BLK * BLK;
                    float eta = update_voxel(&blk[lin], pm, M, proj, mu, c->p.maxW, dists, c->p.cols, c->p.rows);
                    if (!colour || (eta > mu) || (fabsf(eta / mu) > 0.25f)) continue;
                    update_voxel_colour(&c->vba_rgb[(size_t)e->ptr * BLK3 + lin], pm, Mr, proj_rgb, c->p.maxW, c->rgb_in,
                                        c->rgb_pitch, c->p.cols, c->p.rows);
                }
    }
}

/* the same with the view's RGB image (uchar4 rows of `pitch` bytes, the depth image's size) */
void tfo_integrate_rgb(tfo_ctx* c, const float pose_rt[12], const float* dists, const uint8_t* rgb, size_t pitch)
{
    c->rgb_in = rgb; c->rgb_pitch = pitch ? pitch : (size_t)c->p.cols * 4;
    tfo_integrate(c, pose_rt, dists);
    c->rgb_in = 0;
}

/* ------------------------------------------------------------------------- */
/* voxel access (RepresentationAccess.hpp)                                   */
/* ------------------------------------------------------------------------- */
typedef struct { int bx, by, bz; int blockPtr; } icache;   /* VoxelBlockHash::IndexCache, VoxelBlockHash.hpp:58-62 */

static inline void cache_init(icache* k) { k->bx = k->by = k->bz = 0x7fffffff; k->blockPtr = -1; }

/* pointToVoxelBlockPos, RepresentationAccess.hpp:9-17 */
static inline int point_to_block(int px, int py, int pz, int* bx, int* by, int* bz)
{
    *bx = ((px < 0) ? px - BLK + 1 : px) / BLK;
    *by = ((py < 0) ? py - BLK + 1 : py) / BLK;
    *bz = ((pz < 0) ? pz - BLK + 1 : pz) / BLK;
    return px + (py - *bx) * BLK + (pz - *by) * BLK * BLK - *bz * BLK3;
}

/* readVoxel with cache, RepresentationAccess.hpp:73-104 */
static inline tfo_voxel read_voxel(const tfo_ctx* c, int px, int py, int pz, int* vmIndex, icache* k)
{
    int bx, by, bz;
    int linearIdx = point_to_block(px, py, pz, &bx, &by, &bz);
    if (bx == k->bx && by == k->by && bz == k->bz) {
        *vmIndex = 1;
        return c->vba[k->blockPtr + linearIdx];
    }
    int hashIdx = hash_index(c, bx, by, bz);
    while (1) {
        tfo_hash_entry e = c->hash[hashIdx];
        if (e.x == (int16_t)bx && e.y == (int16_t)by && e.z == (int16_t)bz && e.ptr >= 0) {
            k->bx = bx; k->by = by; k->bz = bz; k->blockPtr = e.ptr * BLK3;
            *vmIndex = hashIdx + 1;
            return c->vba[k->blockPtr + linearIdx];
        }
        if (e.offset < 1) break;
        hashIdx = c->p.n_buckets + e.offset - 1;
    }
    *vmIndex = 0;
    tfo_voxel d; d.sdf = 32767; d.w = 0; d.pad = 0;
    return d;
}

static inline tfo_voxel read_voxel_nc(const tfo_ctx* c, int px, int py, int pz)
{
    icache k; int vm;
    cache_init(&k);
    return read_voxel(c, px, py, pz, &vm, &k);
}

static inline int iround(float x) { return (int)((x < 0) ? (x - 0.5f) : (x + 0.5f)); }   /* ROUND, MathUtils.hpp:20 */

/* a voxel's colour word (readVoxel(...).clr, w_color; Voxel_s_rgb() = 0 where no block) */
static inline uint32_t read_colour(const tfo_ctx* c, int px, int py, int pz)
{
    int bx, by, bz;
    int linearIdx = point_to_block(px, py, pz, &bx, &by, &bz);
    int hashIdx = hash_index(c, bx, by, bz);
    while (1) {
        tfo_hash_entry e = c->hash[hashIdx];
        if (e.x == (int16_t)bx && e.y == (int16_t)by && e.z == (int16_t)bz && e.ptr >= 0)
            return c->vba_rgb[(size_t)e.ptr * BLK3 + linearIdx];
        if (e.offset < 1) return 0;
        hashIdx = c->p.n_buckets + e.offset - 1;
    }
}

/* readFromSDF_color4u_interpolated (RepresentationAccess.hpp:260-294) + drawPixelColour
   (VisualisationEngine_Shared.hpp:312-322): trilinear colour at the raycast point, / 255, then
   (uchar)(v * 255); alpha 255 */
static void colour_at(const tfo_ctx* c, const float pt[3], uint8_t out[4])
{
    int px = (int)floorf(pt[0]), py = (int)floorf(pt[1]), pz = (int)floorf(pt[2]);
    float cx = pt[0] - floorf(pt[0]), cy = pt[1] - floorf(pt[1]), cz = pt[2] - floorf(pt[2]);
    float ret[3] = { 0.0f, 0.0f, 0.0f };
    for (int corner = 0; corner < 8; ++corner) {
        int ux = corner & 1, uy = (corner >> 1) & 1, uz = corner >> 2;
        float w = (ux ? cx : (1.0f - cx)) * (uy ? cy : (1.0f - cy)) * (uz ? cz : (1.0f - cz));
        uint32_t v = read_colour(c, px + ux, py + uy, pz + uz);
        for (int k = 0; k < 3; ++k) ret[k] += w * (float)((v >> (8 * k)) & 0xffu);
    }
    for (int k = 0; k < 3; ++k) out[k] = (uint8_t)((ret[k] / 255.0f) * 255.0f);
    out[3] = 255;
}

/* readFromSDF_float_uninterpolated (cached), RepresentationAccess.hpp:129-135 */
static inline float sdf_uninterp(const tfo_ctx* c, const float pt[3], int* vm, icache* k)
{
    tfo_voxel v = read_voxel(c, iround(pt[0]), iround(pt[1]), iround(pt[2]), vm, k);
    return (float)v.sdf / 32767.0f;
}

/* readFromSDF_float_interpolated, RepresentationAccess.hpp:137-162 */
static inline float sdf_interp(const tfo_ctx* c, const float pt[3], int* vm, icache* k)
{
    float res1, res2, v1, v2;
    int px = (int)floorf(pt[0]), py = (int)floorf(pt[1]), pz = (int)floorf(pt[2]);
    float cx = pt[0] - floorf(pt[0]), cy = pt[1] - floorf(pt[1]), cz = pt[2] - floorf(pt[2]);
    v1 = read_voxel(c, px, py, pz, vm, k).sdf;
    v2 = read_voxel(c, px + 1, py, pz, vm, k).sdf;
    res1 = (1.0f - cx) * v1 + cx * v2;
    v1 = read_voxel(c, px, py + 1, pz, vm, k).sdf;
    v2 = read_voxel(c, px + 1, py + 1, pz, vm, k).sdf;
    res1 = (1.0f - cy) * res1 + cy * ((1.0f - cx) * v1 + cx * v2);
    v1 = read_voxel(c, px, py, pz + 1, vm, k).sdf;
    v2 = read_voxel(c, px + 1, py, pz + 1, vm, k).sdf;
    res2 = (1.0f - cx) * v1 + cx * v2;
    v1 = read_voxel(c, px, py + 1, pz + 1, vm, k).sdf;
    v2 = read_voxel(c, px + 1, py + 1, pz + 1, vm, k).sdf;
    res2 = (1.0f - cy) * res2 + cy * ((1.0f - cx) * v1 + cx * v2);
    *vm = 1;
    return ((1.0f - cz) * res1 + cz * res2) / 32767.0f;
}

/* readWithConfidenceFromSDF_float_interpolated, RepresentationAccess.hpp:164-199 */
static inline float sdf_interp_conf(const tfo_ctx* c, float* confidence, const float pt[3], int* vm, icache* k)
{
    float res1, res2, v1, v2, res1_c, res2_c, v1_c, v2_c;
    tfo_voxel vx;
    int px = (int)floorf(pt[0]), py = (int)floorf(pt[1]), pz = (int)floorf(pt[2]);
    float cx = pt[0] - floorf(pt[0]), cy = pt[1] - floorf(pt[1]), cz = pt[2] - floorf(pt[2]);
    vx = read_voxel(c, px, py, pz, vm, k); v1 = vx.sdf; v1_c = vx.w;
    vx = read_voxel(c, px + 1, py, pz, vm, k); v2 = vx.sdf; v2_c = vx.w;
    res1 = (1.0f - cx) * v1 + cx * v2;
    res1_c = (1.0f - cx) * v1_c + cx * v2_c;
    vx = read_voxel(c, px, py + 1, pz, vm, k); v1 = vx.sdf; v1_c = vx.w;
    vx = read_voxel(c, px + 1, py + 1, pz, vm, k); v2 = vx.sdf; v2_c = vx.w;
    res1 = (1.0f - cy) * res1 + cy * ((1.0f - cx) * v1 + cx * v2);
    res1_c = (1.0f - cy) * res1_c + cy * ((1.0f - cx) * v1_c + cx * v2_c);
    vx = read_voxel(c, px, py, pz + 1, vm, k); v1 = vx.sdf; v1_c = vx.w;
    vx = read_voxel(c, px + 1, py, pz + 1, vm, k); v2 = vx.sdf; v2_c = vx.w;
    res2 = (1.0f - cx) * v1 + cx * v2;
    res2_c = (1.0f - cx) * v1_c + cx * v2_c;
    vx = read_voxel(c, px, py + 1, pz + 1, vm, k); v1 = vx.sdf; v1_c = vx.w;
    vx = read_voxel(c, px + 1, py + 1, pz + 1, vm, k); v2 = vx.sdf; v2_c = vx.w;
    res2 = (1.0f - cy) * res2 + cy * ((1.0f - cx) * v1 + cx * v2);
    res2_c = (1.0f - cy) * res2_c + cy * ((1.0f - cx) * v1_c + cx * v2_c);
    *vm = 1;
    *confidence = (1.0f - cz) * res1_c + cz * res2_c;
    return ((1.0f - cz) * res1 + cz * res2) / 32767.0f;
}

/* debug instrumentation (analysis only; off unless buffers are set): per-pixel ray-march
   sample counts of the last raycast, total and in unallocated blocks */
static int* g_dbg_steps = 0;
static int* g_dbg_empty = 0;
void tfo_debug_ray_buffers(int* steps, int* empty) { g_dbg_steps = steps; g_dbg_empty = empty; }

/* castRay, VisualisationEngine_Shared.hpp:99-172 */
static void cast_ray(tfo_ctx* c, float out[4], int update_visible, int x, int y, const float invM[16],
                     const float invProj[4], float oneOverVoxelSize, float mu, const float* range2)
{
    float pc[4], r[4], ps[3], pe[3], dir[3], pt[3];
    int vmIndex = 0;
    float sdfValue = 1.0f, confidence = 0.0f;
    float totalLength, stepLength, totalLengthMax, stepScale;
    stepScale = mu * oneOverVoxelSize;
    pc[2] = range2[0];
    pc[0] = pc[2] * (((float)x + invProj[2]) * invProj[0]);
    pc[1] = pc[2] * (((float)y + invProj[3]) * invProj[1]);
    pc[3] = 1.0f;
    totalLength = sqrtf(((0.0f + pc[0] * pc[0]) + pc[1] * pc[1]) + pc[2] * pc[2]) * oneOverVoxelSize;
    m4v(invM, pc, r);
    ps[0] = r[0] * oneOverVoxelSize; ps[1] = r[1] * oneOverVoxelSize; ps[2] = r[2] * oneOverVoxelSize;
    pc[2] = range2[1];
    pc[0] = pc[2] * (((float)x + invProj[2]) * invProj[0]);
    pc[1] = pc[2] * (((float)y + invProj[3]) * invProj[1]);
    pc[3] = 1.0f;
    totalLengthMax = sqrtf(((0.0f + pc[0] * pc[0]) + pc[1] * pc[1]) + pc[2] * pc[2]) * oneOverVoxelSize;
    m4v(invM, pc, r);
    pe[0] = r[0] * oneOverVoxelSize; pe[1] = r[1] * oneOverVoxelSize; pe[2] = r[2] * oneOverVoxelSize;
    dir[0] = pe[0] - ps[0]; dir[1] = pe[1] - ps[1]; dir[2] = pe[2] - ps[2];
    float direction_norm = 1.0f / sqrtf(dir[0] * dir[0] + dir[1] * dir[1] + dir[2] * dir[2]);
    dir[0] *= direction_norm; dir[1] *= direction_norm; dir[2] *= direction_norm;
    pt[0] = ps[0]; pt[1] = ps[1]; pt[2] = ps[2];
    icache k; cache_init(&k);
    int n_steps = 0, n_empty = 0;
    while (totalLength < totalLengthMax) {
        sdfValue = sdf_uninterp(c, pt, &vmIndex, &k);
        n_steps++;
        if (!vmIndex) n_empty++;
        if (update_visible) {
            if (vmIndex) c->visType[vmIndex - 1] = 1;
        }
        if (!vmIndex) {
            stepLength = (float)BLK;
        } else {
            if ((sdfValue <= 0.1f) && (sdfValue >= -0.5f)) sdfValue = sdf_interp(c, pt, &vmIndex, &k);
            if (sdfValue <= 0.0f) break;
            float a = sdfValue * stepScale;
            stepLength = (a < 1.0f) ? 1.0f : a;
        }
        pt[0] += stepLength * dir[0]; pt[1] += stepLength * dir[1]; pt[2] += stepLength * dir[2];
        totalLength += stepLength;
    }
    int found;
    if (sdfValue <= 0.0f) {
        stepLength = sdfValue * stepScale;
        pt[0] += stepLength * dir[0]; pt[1] += stepLength * dir[1]; pt[2] += stepLength * dir[2];
        sdfValue = sdf_interp_conf(c, &confidence, pt, &vmIndex, &k);
        stepLength = sdfValue * stepScale;
        pt[0] += stepLength * dir[0]; pt[1] += stepLength * dir[1]; pt[2] += stepLength * dir[2];
        found = 1;
    } else found = 0;
    out[0] = pt[0]; out[1] = pt[1]; out[2] = pt[2];
    out[3] = found ? confidence + 1.0f : 0.0f;
    if (g_dbg_steps) { g_dbg_steps[x + y * c->p.cols] = n_steps; g_dbg_empty[x + y * c->p.cols] = n_empty; }
}

/* GenericRaycast, VisualisationEngine_CUDA.cu:175-218; genericRaycast_device VisualisationHelper.hpp:33-46 */
void tfo_raycast(tfo_ctx* c, const float invM_rt[12], int update_visible)
{
    int W = c->p.cols, H = c->p.rows;
    float invM[16];
    rt_to_m4(invM_rt, invM);
    float oneOverVoxelSize = 1.0f / c->p.voxelSize;
    float invProj[4] = { 1.0f / c->p.fx, 1.0f / c->p.fy, -c->p.cx, -c->p.cy };  /* InvertProjectionParams :28-31 */
    /* rays are independent; castRay<true>'s visibility marks all write the value 1 */
#pragma omp parallel for schedule(dynamic, 4)
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            int locId = x + y * W;
            int locId2 = (int)floorf((float)x / SUBSAMPLE) + (int)floorf((float)y / SUBSAMPLE) * W;
            cast_ray(c, c->raycast + 4 * locId, update_visible, x, y, invM, invProj, oneOverVoxelSize, c->p.mu,
                     c->range + 2 * locId2);
        }
}

/* computeNormalAndAngle<false,false> + processPixelICP, VisualisationEngine_Shared.hpp:205-270,355-397 */
void tfo_render_icp(tfo_ctx* c, const float invM_rt[12], float* points, float* normals)
{
    int W = c->p.cols, H = c->p.rows;
    float vs = c->p.voxelSize;
    float light[3] = { -invM_rt[2], -invM_rt[6], -invM_rt[10] };   /* -Vector3f(invM.getColumn(2)) */
    const float qnan = qnanf_bits();
    const float* ray = c->raycast;
#pragma omp parallel for schedule(static)
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            int locId = x + y * W;
            const float* p = ray + 4 * locId;
            int found = p[3] > 0.0f;
            float n[3] = { 0, 0, 0 }, angle = 0;
            if (found) {
                if (y <= 1 || y >= H - 2 || x <= 1 || x >= W - 2) found = 0;
                else {
                    const float* xp = ray + 4 * ((x + 1) + y * W);
                    const float* yp = ray + 4 * (x + (y + 1) * W);
                    const float* xm = ray + 4 * ((x - 1) + y * W);
                    const float* ym = ray + 4 * (x + (y - 1) * W);
                    if (xp[3] <= 0 || yp[3] <= 0 || xm[3] <= 0 || ym[3] <= 0) found = 0;
                    else {
                        float dx[3] = { xp[0] - xm[0], xp[1] - xm[1], xp[2] - xm[2] };
                        float dy[3] = { yp[0] - ym[0], yp[1] - ym[1], yp[2] - ym[2] };
                        /* length_diff test (:245-248) has no effect when useSmoothing == false */
                        n[0] = -(dx[1] * dy[2] - dx[2] * dy[1]);
                        n[1] = -(dx[2] * dy[0] - dx[0] * dy[2]);
                        n[2] = -(dx[0] * dy[1] - dx[1] * dy[0]);
                        float ns = 1.0f / sqrtf(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
                        n[0] *= ns; n[1] *= ns; n[2] *= ns;
                        angle = n[0] * light[0] + n[1] * light[1] + n[2] * light[2];
                        if (!(angle > 0.0)) found = 0;
                    }
                }
            }
            float* po = points + 4 * locId;
            float* no = normals + 4 * locId;
            if (found) {
                po[0] = p[0] * vs; po[1] = p[1] * vs; po[2] = p[2] * vs; po[3] = 1.0f;
                no[0] = n[0]; no[1] = n[1]; no[2] = n[2]; no[3] = 1.0f;
            } else {
                po[0] = po[1] = po[2] = po[3] = qnan;
                no[0] = no[1] = no[2] = no[3] = qnan;
            }
        }
}

/* computeSingleNormalFromSDF, RepresentationAccess.hpp:340-453 */
static void normal_from_sdf(const tfo_ctx* c, const float pt[3], float ret[3])
{
    int px = (int)floorf(pt[0]), py = (int)floorf(pt[1]), pz = (int)floorf(pt[2]);
    float cx = pt[0] - floorf(pt[0]), cy = pt[1] - floorf(pt[1]), cz = pt[2] - floorf(pt[2]);
    float nx = 1.0f - cx, ny = 1.0f - cy, nz = 1.0f - cz;
#define RV(dx, dy, dz) ((float)read_voxel_nc(c, px + (dx), py + (dy), pz + (dz)).sdf)
    float fx_ = RV(0, 0, 0), fy_ = RV(1, 0, 0), fz_ = RV(0, 1, 0), fw_ = RV(1, 1, 0);
    float bx_ = RV(0, 0, 1), by_ = RV(1, 0, 1), bz_ = RV(0, 1, 1), bw_ = RV(1, 1, 1);
    float tx, ty, tz, tw, p1, p2, v1;
    /* gradient x */
    p1 = fx_ * ny * nz + fz_ * cy * nz + bx_ * ny * cz + bz_ * cy * cz;
    tx = RV(-1, 0, 0); ty = RV(-1, 1, 0); tz = RV(-1, 0, 1); tw = RV(-1, 1, 1);
    p2 = tx * ny * nz + ty * cy * nz + tz * ny * cz + tw * cy * cz;
    v1 = p1 * cx + p2 * nx;
    p1 = fy_ * ny * nz + fw_ * cy * nz + by_ * ny * cz + bw_ * cy * cz;
    tx = RV(2, 0, 0); ty = RV(2, 1, 0); tz = RV(2, 0, 1); tw = RV(2, 1, 1);
    p2 = tx * ny * nz + ty * cy * nz + tz * ny * cz + tw * cy * cz;
    ret[0] = (p1 * nx + p2 * cx - v1) / 32767.0f;
    /* gradient y */
    p1 = fx_ * nx * nz + fy_ * cx * nz + bx_ * nx * cz + by_ * cx * cz;
    tx = RV(0, -1, 0); ty = RV(1, -1, 0); tz = RV(0, -1, 1); tw = RV(1, -1, 1);
    p2 = tx * nx * nz + ty * cx * nz + tz * nx * cz + tw * cx * cz;
    v1 = p1 * cy + p2 * ny;
    p1 = fz_ * nx * nz + fw_ * cx * nz + bz_ * nx * cz + bw_ * cx * cz;
    tx = RV(0, 2, 0); ty = RV(1, 2, 0); tz = RV(0, 2, 1); tw = RV(1, 2, 1);
    p2 = tx * nx * nz + ty * cx * nz + tz * nx * cz + tw * cx * cz;
    ret[1] = (p1 * ny + p2 * cy - v1) / 32767.0f;
    /* gradient z */
    p1 = fx_ * nx * ny + fy_ * cx * ny + fz_ * nx * cy + fw_ * cx * cy;
    tx = RV(0, 0, -1); ty = RV(1, 0, -1); tz = RV(0, 1, -1); tw = RV(1, 1, -1);
    p2 = tx * nx * ny + ty * cx * ny + tz * nx * cy + tw * cx * cy;
    v1 = p1 * cz + p2 * nz;
    p1 = bx_ * nx * ny + by_ * cx * ny + bz_ * nx * cy + bw_ * cx * cy;
    tx = RV(0, 0, 2); ty = RV(1, 0, 2); tz = RV(0, 1, 2); tw = RV(1, 1, 2);
    p2 = tx * nx * ny + ty * cx * ny + tz * nx * cy + tw * cx * cy;
    ret[2] = (p1 * nz + p2 * cz - v1) / 32767.0f;
#undef RV
}

/* baseCol / interpolateCol, VisualisationEngine_Shared.hpp:278-288 */
static float interpolate_col(float val, float y0, float x0, float y1, float x1) { return (val - x0) * (y1 - y0) / (x1 - x0) + y0; }
static float base_col(float val)
{
    if (val <= -0.75f) return 0.0f;
    else if (val <= -0.25f) return interpolate_col(val, 0.0f, -0.75f, 1.0f, -0.25f);
    else if (val <= 0.25f) return 1.0f;
    else if (val <= 0.75f) return interpolate_col(val, 1.0f, 0.25f, 0.0f, 0.75f);
    else return 0.0f;
}

/* Vector4f::toUChar: CLAMP((int)ROUND(v), 0, 255), Vector.hpp:398-404, MathUtils.hpp:16-20 */
static uint8_t round_u8(float v)
{
    int i = (int)((v < 0) ? (v - 0.5f) : (v + 0.5f));
    return (uint8_t)(i < 0 ? 0 : (i > 255 ? 255 : i));
}

/* computeNormalAndAngle<useSmoothing=true, flipNormals=false> on the raycast image,
   VisualisationEngine_Shared.hpp:205-270 */
static int image_normal_angle(const float* ray, int W, int H, int x, int y, float voxelSize, const float light[3], float* angle)
{
    if (y <= 2 || y >= H - 3 || x <= 2 || x >= W - 3) return 0;
    const float *xp = ray + 4 * ((x + 2) + y * W), *yp = ray + 4 * (x + (y + 2) * W);
    const float *xm = ray + 4 * ((x - 2) + y * W), *ym = ray + 4 * (x + (y - 2) * W);
    float dx[3] = { 0, 0, 0 }, dy[3] = { 0, 0, 0 };
    int plus1 = 0;
    if (xp[3] <= 0 || yp[3] <= 0 || xm[3] <= 0 || ym[3] <= 0) plus1 = 1;
    else {
        for (int k = 0; k < 3; ++k) { dx[k] = xp[k] - xm[k]; dy[k] = yp[k] - ym[k]; }
        float lx = dx[0] * dx[0] + dx[1] * dx[1] + dx[2] * dx[2], ly = dy[0] * dy[0] + dy[1] * dy[1] + dy[2] * dy[2];
        float length_diff = (lx < ly) ? ly : lx;                  /* MAX */
        if (length_diff * voxelSize * voxelSize > (0.15f * 0.15f)) plus1 = 1;
    }
    if (plus1) {
        xp = ray + 4 * ((x + 1) + y * W); yp = ray + 4 * (x + (y + 1) * W);
        xm = ray + 4 * ((x - 1) + y * W); ym = ray + 4 * (x + (y - 1) * W);
        for (int k = 0; k < 3; ++k) { dx[k] = xp[k] - xm[k]; dy[k] = yp[k] - ym[k]; }
        if (xp[3] <= 0 || yp[3] <= 0 || xm[3] <= 0 || ym[3] <= 0) return 0;
    }
    float n[3] = { -(dx[1] * dy[2] - dx[2] * dy[1]), -(dx[2] * dy[0] - dx[0] * dy[2]), -(dx[0] * dy[1] - dx[1] * dy[0]) };
    float ns = 1.0f / sqrtf(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
    n[0] *= ns; n[1] *= ns; n[2] *= ns;
    *angle = n[0] * light[0] + n[1] * light[1] + n[2] * light[2];
    return *angle > 0.0f;
}

/* RenderImage_common's pixel stages, VisualisationEngine_CUDA.cu:254-290: renderGrey_device,
   renderGrey_ImageNormals_device<false>, renderColourFromNormal_device,
   renderColourFromConfidence_device (VisualisationHelper.hpp:76-148); processPixel* /
   drawPixel* VisualisationEngine_Shared.hpp:187-310,399-498.  RENDER_COLOUR_FROM_VOLUME falls
   back to greyscale for Voxel_s (:251-252) and reads the colour plane for Voxel_s_rgb.
   drawPixelNormal leaves alpha as it was. */
void tfo_render_type(tfo_ctx* c, const float invM_rt[12], int type, uint8_t* rgba)
{
    int W = c->p.cols, H = c->p.rows;
    float light[3] = { -invM_rt[2], -invM_rt[6], -invM_rt[10] };
#pragma omp parallel for schedule(dynamic, 256)
    for (int i = 0; i < W * H; ++i) {
        const float* p = c->raycast + 4 * i;
        uint8_t* o = rgba + 4 * i;
        int found = p[3] > 0;
        float n[3] = { 0, 0, 0 }, angle = 0;
        if (type == 2 && c->vba_rgb) {          /* renderColour_device / processPixelColour (:464-470) */
            if (found) colour_at(c, p, o);
            else o[0] = o[1] = o[2] = o[3] = 0;
            continue;
        }
        if (type == 1) {
            if (found) found = image_normal_angle(c->raycast, W, H, i % W, i / W, c->p.voxelSize, light, &angle);
            uint8_t v = found ? (uint8_t)((0.8f * angle + 0.2f) * 255.0f) : 0;
            o[0] = o[1] = o[2] = o[3] = v;
            continue;
        }
        if (found) {
            normal_from_sdf(c, p, n);
            float ns = 1.0f / sqrtf(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
            n[0] *= ns; n[1] *= ns; n[2] *= ns;
            angle = n[0] * light[0] + n[1] * light[1] + n[2] * light[2];
            if (!(angle > 0.0)) found = 0;
        }
        if (type == 3) {
            if (found) {
                for (int k = 0; k < 3; ++k) o[k] = (uint8_t)((0.3f + (-n[k] + 1.0f) * 0.35f) * 255.0f);
            } else {
                o[0] = o[1] = o[2] = o[3] = 0;
            }
        } else if (type == 4) {
            if (found) {
                float conf = p[3] - 1.0f;
                float mn = (100.f < conf) ? 100.f : conf;          /* CLAMP(conf, 0, 100.f) */
                float cn = ((0 < mn) ? mn : 0) / 100.0f;
                float col[4] = { (float)(uint8_t)(base_col(cn) * 255.0f), (float)(uint8_t)(base_col(cn - 0.5f) * 255.0f),
                                 (float)(uint8_t)(base_col(cn + 0.5f) * 255.0f), 255.0f };
                float sc = 0.8f * angle + 0.2f;
                for (int k = 0; k < 4; ++k) o[k] = round_u8(sc * col[k]);
            } else {
                o[0] = o[1] = o[2] = o[3] = 0;
            }
        } else {
            uint8_t v = found ? (uint8_t)((0.8f * angle + 0.2f) * 255.0f) : 0;
            o[0] = o[1] = o[2] = o[3] = v;
        }
    }
}

/* renderGrey_device / processPixelGrey / drawPixelGrey,
   VisualisationHelper.hpp:105-118; VisualisationEngine_Shared.hpp:187-203,272-276,450-462 */
void tfo_render_grey(tfo_ctx* c, const float invM_rt[12], uint8_t* rgba)
{
    tfo_render_type(c, invM_rt, 0, rgba);
}

/* VisualisationEngine_CUDA::RenderImage(type, RENDER_FROM_NEW_RAYCAST) from the current pose into
   the context's image (the buffer the frame's renderImage fills) */
void tfo_render_image_type(tfo_ctx* c, int type)
{
    tfo_raycast(c, c->pose, 0);
    tfo_render_type(c, c->pose, type, c->frame_grey);
}

/* TopFu::renderImage -> RenderImage_common(RENDER_SHADED_GREYSCALE), topfu.cpp:332-377,
   VisualisationEngine_CUDA.cu:220-291 */
void tfo_render_image(tfo_ctx* c, uint8_t* rgba)
{
    tfo_raycast(c, c->pose, 0);
    tfo_render_grey(c, c->pose, rgba);
}

/* CreateExpectedDepths, VisualisationEngine_CUDA.cu:119-173; ProjectSingleBlock / CreateRenderingBlocks
   VisualisationEngine_Shared.hpp:33-95; projectAndSplitBlocks_device / fillBlocks_device VisualisationHelper.cu:52-121 */
void tfo_expected_depths(tfo_ctx* c, const float pose_rt[12])
{
    int W = c->p.cols, H = c->p.rows;
    for (int i = 0; i < W * H; ++i) { c->range[2 * i] = FAR_AWAY; c->range[2 * i + 1] = VERY_CLOSE; }
    c->noTotalBlocks = 0;
    if (c->noVisibleEntries == 0) return;
    float M[16];
    rt_to_m4(pose_rt, M);
    float vs = c->p.voxelSize;
    unsigned total = 0;
    for (int i = 0; i < c->noVisibleEntries; ++i) {
        const tfo_hash_entry* e = &c->hash[c->visibleIds[i]];
        if (e->ptr < 0) continue;
        int ulx = W / SUBSAMPLE, uly = H / SUBSAMPLE, lrx = -1, lry = -1;
        float zmin = FAR_AWAY, zmax = VERY_CLOSE;
        for (int corner = 0; corner < 8; ++corner) {
            int16_t tx = (int16_t)(e->x + ((corner & 1) ? 1 : 0));
            int16_t ty = (int16_t)(e->y + ((corner & 2) ? 1 : 0));
            int16_t tz = (int16_t)(e->z + ((corner & 4) ? 1 : 0));
            float p3[4] = { (float)tx * (float)BLK * vs, (float)ty * (float)BLK * vs, (float)tz * (float)BLK * vs, 1.0f }, q[4];
            m4v(M, p3, q);
            if ((double)q[2] < 1e-6) continue;
            float p2x = (c->p.fx * q[0] / q[2] + c->p.cx) / (float)SUBSAMPLE;
            float p2y = (c->p.fy * q[1] / q[2] + c->p.cy) / (float)SUBSAMPLE;
            if ((float)ulx > floorf(p2x)) ulx = (int)floorf(p2x);
            if ((float)lrx < ceilf(p2x)) lrx = (int)ceilf(p2x);
            if ((float)uly > floorf(p2y)) uly = (int)floorf(p2y);
            if ((float)lry < ceilf(p2y)) lry = (int)ceilf(p2y);
            if (zmin > q[2]) zmin = q[2];
            if (zmax < q[2]) zmax = q[2];
        }
        if (ulx < 0) ulx = 0;
        if (uly < 0) uly = 0;
        if (lrx >= W) lrx = W - 1;
        if (lry >= H) lry = H - 1;
        if (ulx > lrx || uly > lry) continue;
        if (zmin < VERY_CLOSE) zmin = VERY_CLOSE;
        if (zmax < VERY_CLOSE) continue;
        int nbx = (int)ceilf((float)(lrx - ulx + 1) / RB_SIZE);
        int nby = (int)ceilf((float)(lry - uly + 1) / RB_SIZE);
        unsigned need = (unsigned)(nbx * nby);
        unsigned off = total;
        total += need;
        if (off + need > (unsigned)c->p.max_render_blocks) continue;   /* projectAndSplitBlocks_device :72 */
        for (int yy = uly; yy <= lry; ++yy)
            for (int xx = ulx; xx <= lrx; ++xx) {
                float* px = c->range + 2 * (xx + yy * W);
                if (zmin < px[0]) px[0] = zmin;           /* atomicMin(fminf), CUDAUtils.hpp:75-84 */
                if (zmax > px[1]) px[1] = zmax;           /* atomicMax(fmaxf), CUDAUtils.hpp:86-95 */
            }
    }
    c->noTotalBlocks = (int)(total > (unsigned)c->p.max_render_blocks ? (unsigned)c->p.max_render_blocks : total);
}

/* CreateICPMaps, VisualisationEngine_CUDA.cu:323-360,473-493 */
static void create_icp_maps(tfo_ctx* c)
{
    tfo_raycast(c, c->pose, 1);
    tfo_render_icp(c, c->pose, c->prev_pts[0], c->prev_nrm[0]);
}

/* ProjectiveICP::estimateTransform(points overload), projective_icp.cpp:169-213 */
static int estimate_transform(tfo_ctx* c, float affine[12])
{
    memcpy(affine, k_identity_rt, sizeof(float) * 12);
    float min_cosine = cosf(c->p.icp_angle_thres);                 /* ComputeIcpHelper ctor, projective_icp.cpp:11-15 */
    float dist2 = c->p.icp_dist_thres * c->p.icp_dist_thres;
    int levels = 4;
    while (levels > 0 && c->p.icp_iter_num[levels - 1] == 0) --levels;   /* getUsedLevelsNum :103-108 */
    if (levels > 3) levels = 3;
    c->icp_iterations = 0;
    for (int l = levels - 1; l >= 0; --l) {
        int div = 1 << l;                                              /* setLevelIntr :17-23 */
        float fx = c->p.fx / (float)div, fy = c->p.fy / (float)div, cx = c->p.cx / (float)div, cy = c->p.cy / (float)div;
        for (int it = 0; it < c->p.icp_iter_num[l]; ++it) {
            float s[27];
            tfo_icp_reduce(c->curr_pts[l], c->curr_nrm[l], c->prev_pts[l], c->prev_nrm[l], c->lvl_w[l], c->lvl_h[l],
                           fx, fy, cx, cy, min_cosine, dist2, affine, s);
            c->icp_iterations++;
            if (!tfo_icp_step(s, affine, NULL)) return 0;
        }
    }
    return 1;
}

/* TopFu::operator()(depth, image) with the image integrated into Voxel_s_rgb voxels (voxel_rgb) */
int tfo_process_frame_rgb(tfo_ctx* c, const uint16_t* depth, const uint8_t* rgb, size_t pitch)
{
    c->rgb_in = rgb; c->rgb_pitch = pitch ? pitch : (size_t)c->p.cols * 4;
    int ok = tfo_process_frame(c, depth);
    c->rgb_in = 0;
    return ok;
}

/* TopFu::operator(), topfu.cpp:161-330 */
int tfo_process_frame(tfo_ctx* c, const uint16_t* depth)
{
    const tfo_params* p = &c->p;
    int W = p->cols, H = p->rows;
    tfo_compute_dists(depth, W, H, c->dists);
    tfo_bilateral(depth, c->depth_pyr[0], W, H, p->bilateral_kernel_size, p->bilateral_sigma_spatial, p->bilateral_sigma_depth);
    if (p->icp_truncate_depth_dist > 0) tfo_truncate(c->depth_pyr[0], W, H, p->icp_truncate_depth_dist);
    for (int l = 1; l < 3; ++l) tfo_pyr_down(c->depth_pyr[l - 1], c->lvl_w[l - 1], c->lvl_h[l - 1], c->depth_pyr[l], p->bilateral_sigma_depth);
    for (int l = 0; l < 3; ++l) {
        int div = 1 << l;                                               /* Intr::operator(), precomp.cpp:10-14 */
        tfo_points_normals(c->depth_pyr[l], c->lvl_w[l], c->lvl_h[l], p->fx / (float)div, p->fy / (float)div,
                           p->cx / (float)div, p->cy / (float)div, c->curr_pts[l], c->curr_nrm[l]);
    }
    c->icp_ok = 1;
    if (c->frame_counter == 0) {
        c->icp_iterations = 0;
        tfo_alloc(c, c->pose, c->dists);                  /* poses_.back() == identity */
        tfo_integrate(c, c->pose, c->dists);
        tfo_swap(c);                                      /* (swapping only) */
        for (int l = 0; l < 3; ++l) {                     /* swap curr <-> prev points/normals */
            float* t = c->curr_pts[l]; c->curr_pts[l] = c->prev_pts[l]; c->prev_pts[l] = t;
            t = c->curr_nrm[l]; c->curr_nrm[l] = c->prev_nrm[l]; c->prev_nrm[l] = t;
        }
        c->frame_counter++;
        return 1;
    }
    float affine[12];
    int ok = estimate_transform(c, affine);
    c->icp_ok = ok;
    tfo_rigid_mul(c->pose, affine, c->pose);              /* poses_.push_back(poses_.back() * affine) */
    if (!ok) { tfo_reset(c); return 0; }
    float pinv[12];
    tfo_rigid_inv(c->pose, pinv);
    tfo_alloc(c, pinv, c->dists);
    tfo_integrate(c, pinv, c->dists);
    tfo_swap(c);                                          /* (swapping only) */
    /* renderImage(image): raycast with the (stale) range image + grey shading (topfu.cpp:284-288) */
    tfo_render_image(c, c->frame_grey);
    tfo_expected_depths(c, pinv);
    create_icp_maps(c);
    for (int l = 1; l < 3; ++l)
        tfo_resize_points_normals(c->prev_pts[l - 1], c->prev_nrm[l - 1], c->lvl_w[l - 1], c->lvl_h[l - 1],
                                  c->prev_pts[l], c->prev_nrm[l]);
    c->frame_counter++;
    return 1;
}

void tfo_get_counters(const tfo_ctx* c, tfo_counters* o)
{
    o->lastFreeBlockId = c->lastFreeBlockId;
    o->lastFreeExcessListId = c->lastFreeExcessListId;
    o->noVisibleEntries = c->noVisibleEntries;
    o->noTotalBlocks = c->noTotalBlocks;
    o->frame_counter = c->frame_counter;
    o->icp_iterations = c->icp_iterations;
    o->icp_ok = c->icp_ok;
    o->n_resets = c->n_resets;
}

void tfo_get_pose(const tfo_ctx* c, float rt[12]) { memcpy(rt, c->pose, sizeof(float) * 12); }

/* the counters of a scene written in place (tfo_hash / tfo_visible_ids), as tf_set_counters */
void tfo_set_counters(tfo_ctx* c, int lastFreeBlockId, int lastFreeExcessListId, int noVisibleEntries)
{
    c->lastFreeBlockId = lastFreeBlockId;
    c->lastFreeExcessListId = lastFreeExcessListId;
    c->noVisibleEntries = noVisibleEntries;
}
tfo_hash_entry* tfo_hash(tfo_ctx* c) { return c->hash; }
int* tfo_alloc_list(tfo_ctx* c) { return c->allocList; }
int* tfo_excess_list(tfo_ctx* c) { return c->excessList; }
void tfo_alloc_failures(const tfo_ctx* c, int out[2]) { out[0] = c->alloc_failed[0]; out[1] = c->alloc_failed[1]; }
tfo_voxel* tfo_vba(tfo_ctx* c) { return c->vba; }
uint32_t* tfo_vba_rgb(tfo_ctx* c) { return c->vba_rgb; }
int* tfo_visible_ids(tfo_ctx* c) { return c->visibleIds; }
uint8_t* tfo_visible_type(tfo_ctx* c) { return c->visType; }
float* tfo_range_image(tfo_ctx* c) { return c->range; }
float* tfo_raycast_result(tfo_ctx* c) { return c->raycast; }
float* tfo_prev_points(tfo_ctx* c, int l) { return c->prev_pts[l]; }
float* tfo_prev_normals(tfo_ctx* c, int l) { return c->prev_nrm[l]; }
float* tfo_curr_points(tfo_ctx* c, int l) { return c->curr_pts[l]; }
float* tfo_curr_normals(tfo_ctx* c, int l) { return c->curr_nrm[l]; }
uint16_t* tfo_curr_depth(tfo_ctx* c, int l) { return c->depth_pyr[l]; }
uint8_t* tfo_frame_grey(tfo_ctx* c) { return c->frame_grey; }
float* tfo_dists(tfo_ctx* c) { return c->dists; }

/* The point conversions used above, exposed for pinning against the reference's own
 * Vector3f::toShortFloor / toIntFloor(residual) / toIntRound and length()
 * (Vector.hpp:210-240, 814-824; golden tests/golden/ref_pin_round.bin).
 * out = {short floor xyz, int floor xyz, residual xyz, round xyz, length}. */
void tfo_point_conv(const float p[3], float out[13])
{
    for (int i = 0; i < 3; ++i) {
        out[i] = (float)(int16_t)floorf(p[i]);
        out[3 + i] = (float)(int)floorf(p[i]);
        out[6 + i] = p[i] - floorf(p[i]);
        out[9 + i] = (float)iround(p[i]);
    }
    out[12] = sqrtf(((0.0f + p[0] * p[0]) + p[1] * p[1]) + p[2] * p[2]);
}

/* hashIndex (RepresentationAccess.hpp:5-7) for a table of n_buckets (power of two) */
int tfo_hash_index(int x, int y, int z, int n_buckets)
{
    return (int)((((uint32_t)x * 73856093u) ^ ((uint32_t)y * 19349669u) ^ ((uint32_t)z * 83492791u)) &
                 (uint32_t)(n_buckets - 1));
}
