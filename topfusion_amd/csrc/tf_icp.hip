// tf_icp.hip -- projective point-to-plane ICP for gfx950.
//
// One iteration = two launches and no host round trip (the reference syncs to the host
// and solves with OpenCV 19 times per frame, projective_icp.cpp:187-210):
//   k_icp_partial : find_coresp + row build (proj_icp.cu:80-117,359-377) and the 27
//                   products reduced per reference CTA.  A wave64 owns one 32x8 reference
//                   CTA (4 pixels per lane: tids l, l+64, l+128, l+192) and reproduces the
//                   reference's 256-wide halving tree (temp_utils.hpp:503-523) with two
//                   in-register adds + a 6-step xor butterfly: no LDS, no barriers.
//   k_icp_solve   : icp_final_reduce_kernel (proj_icp.cu:382-403) in the same order,
//                   then det check (cv::determinant), 6x6 solve, Rodrigues and
//                   affine = Tinc * affine on the device.
// A failed det check sets state->abort; every later ICP / scene kernel of the frame no-ops.
#include "tf_internal.h"

#define ICP_PART_STRIDE 28   // 27 sums padded to 7 float4

struct IcpLevel {
    const float4* vcurr; const float4* ncurr; const float4* vprev; const float4* nprev;
    int W, H, gx, nct;
    float fx, fy, cx, cy;
    float min_cosine, dist2;
};

// find_coresp (points variant) + row (proj_icp.cu:80-117, 365-377)
__device__ __forceinline__ bool icp_row(const IcpLevel& L, const float* aff, int x, int y, float* row)
{
    if (x >= L.W || y >= L.H) return false;
    const int W = L.W;
    float4 sp = L.vcurr[y * W + x];
    tf3 s = mk3(sp.x, sp.y, sp.z);
    if (isnan(s.x)) return false;
    tf3 R0 = mk3(aff[0], aff[1], aff[2]), R1 = mk3(aff[4], aff[5], aff[6]), R2 = mk3(aff[8], aff[9], aff[10]);
    s = mk3(kdot(R0, s) + aff[3], kdot(R1, s) + aff[7], kdot(R2, s) + aff[11]);
    float coox = fmaf(L.fx, s.x / s.z, L.cx);
    float cooy = fmaf(L.fy, s.y / s.z, L.cy);
    if (s.z <= 0 || coox < 0 || cooy < 0 || coox >= (float)L.W || cooy >= (float)L.H) return false;
    int tx = (int)floorf(coox), ty = (int)floorf(cooy);     // point-sampled tex2D
    float4 dp = L.vprev[ty * W + tx];
    tf3 d = mk3(dp.x, dp.y, dp.z);
    if (isnan(d.x)) return false;
    tf3 sd = sub3(s, d);
    if (kdot(sd, sd) > L.dist2) return false;
    float4 ncp = L.ncurr[y * W + x];
    tf3 nc = mk3(ncp.x, ncp.y, ncp.z);
    tf3 ns = mk3(kdot(R0, nc), kdot(R1, nc), kdot(R2, nc));
    float4 ndp = L.nprev[ty * W + tx];
    tf3 nd = mk3(ndp.x, ndp.y, ndp.z);
    if (fabsf(kdot(ns, nd)) < L.min_cosine) return false;
    tf3 cr = kcross(s, nd);
    row[0] = cr.x; row[1] = cr.y; row[2] = cr.z;
    row[3] = nd.x; row[4] = nd.y; row[5] = nd.z;
    row[6] = kdot(nd, sub3(d, s));
    return true;
}

__global__ void __launch_bounds__(256)
k_icp_partial(IcpLevel L, const TfDevState* __restrict__ st, float* __restrict__ partial)
{
    if (st->abort) return;
    const int lane = threadIdx.x & 63;
    const int cta = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (cta >= L.nct) return;                       // whole wave exits together
    float aff[12];
#pragma unroll
    for (int i = 0; i < 12; ++i) aff[i] = st->affine[i];
    const int bx = cta % L.gx, by = cta / L.gx;
    float r[4][7];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        int t = lane + 64 * j;
        int x = bx * 32 + (t & 31), y = by * 8 + (t >> 5);
        if (!icp_row(L, aff, x, y, r[j]))
#pragma unroll
            for (int k = 0; k < 7; ++k) r[j][k] = 0.f;
    }
    float mine = 0.f;
    int k = 0;
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
        for (int b = a; b < 7; ++b, ++k) {
            // step 128: v[t]+v[t+128]; step 64: + (v[t+64]+v[t+192]); then 32..1
            float a0 = r[0][a] * r[0][b] + r[2][a] * r[2][b];
            float a1 = r[1][a] * r[1][b] + r[3][a] * r[3][b];
            float s = tf_wave_tree64(a0 + a1);
            if (lane == k) mine = s;
        }
    if (lane < 27) partial[cta * ICP_PART_STRIDE + lane] = mine;
}

// ---- 6x6 algebra (one thread; double where OpenCV's replacement is double) ----------------
// cv::determinant(Matx66f): LU with partial pivoting in float, eps = 10*FLT_EPSILON
__device__ double icp_det6(const float* Ain)
{
    float A[36];
    for (int i = 0; i < 36; ++i) A[i] = Ain[i];
    int p = 1;
    const float eps = 1.19209290e-07f * 10;
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

// cv::solve(A, b, DECOMP_SVD) replacement: Gaussian elimination, partial pivoting, double
__device__ void icp_solve6(const float* Af, const float* bf, float* x)
{
    double A[36], b[6], xs[6];
    for (int i = 0; i < 36; ++i) A[i] = Af[i];
    for (int i = 0; i < 6; ++i) b[i] = bf[i];
    for (int i = 0; i < 6; ++i) {
        int k = i;
        for (int j = i + 1; j < 6; ++j) if (fabs(A[j * 6 + i]) > fabs(A[k * 6 + i])) k = j;
        if (k != i) {
            for (int j = 0; j < 6; ++j) { double t = A[i * 6 + j]; A[i * 6 + j] = A[k * 6 + j]; A[k * 6 + j] = t; }
            double t = b[i]; b[i] = b[k]; b[k] = t;
        }
        double piv = A[i * 6 + i];
        for (int j = i + 1; j < 6; ++j) {
            double l = A[j * 6 + i] / piv;
            for (int c = i; c < 6; ++c) A[j * 6 + c] = A[j * 6 + c] - l * A[i * 6 + c];
            b[j] = b[j] - l * b[i];
        }
    }
    for (int i = 5; i >= 0; --i) {
        double s = b[i];
        for (int c = i + 1; c < 6; ++c) s = s - A[i * 6 + c] * xs[c];
        xs[i] = s / A[i * 6 + i];
    }
    for (int i = 0; i < 6; ++i) x[i] = (float)xs[i];
}

__constant__ double c_inv_sin[14] = { 0.0, 1.0/6.0, 1.0/20.0, 1.0/42.0, 1.0/72.0, 1.0/110.0, 1.0/156.0,
    1.0/210.0, 1.0/272.0, 1.0/342.0, 1.0/420.0, 1.0/506.0, 1.0/600.0, 1.0/702.0 };
__constant__ double c_inv_cos[14] = { 0.0, 1.0/2.0, 1.0/12.0, 1.0/30.0, 1.0/56.0, 1.0/90.0, 1.0/132.0,
    1.0/182.0, 1.0/240.0, 1.0/306.0, 1.0/380.0, 1.0/462.0, 1.0/552.0, 1.0/650.0 };

// fixed-polynomial sin/cos (replaces std::sin/cos inside cv::Affine3's Rodrigues)
__device__ void icp_sincos(double th, double* s, double* c)
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
    for (int n = 13; n >= 1; --n) {
        ps = 1.0 - (r2 * c_inv_sin[n]) * ps;
        pc = 1.0 - (r2 * c_inv_cos[n]) * pc;
    }
    *s = r * ps;
    *c = pc;
}

// Affine3f(rvec, t) rotation (Rodrigues in double)
__device__ void icp_rodrigues(const float* rv, float* R)
{
    double rx = rv[0], ry = rv[1], rz = rv[2];
    double theta = sqrt((rx * rx + ry * ry) + rz * rz);
    if (theta < 2.220446049250313e-16) {
        for (int k = 0; k < 9; ++k) R[k] = (k % 4 == 0) ? 1.0f : 0.0f;
        return;
    }
    double s, c;
    icp_sincos(theta, &s, &c);
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

// cv::Affine3f operator* (float rigid composition): out = a * b
__device__ void tf_rigid_mul(const float* a, const float* b, float* out)
{
    float o[12];
    for (int j = 0; j < 3; ++j) {
        for (int i = 0; i < 3; ++i)
            o[j * 4 + i] = (a[j * 4 + 0] * b[0 * 4 + i] + a[j * 4 + 1] * b[1 * 4 + i]) + a[j * 4 + 2] * b[2 * 4 + i];
        o[j * 4 + 3] = ((a[j * 4 + 0] * b[3] + a[j * 4 + 1] * b[7]) + a[j * 4 + 2] * b[11]) + a[j * 4 + 3];
    }
    for (int i = 0; i < 12; ++i) out[i] = o[i];
}

// cv::Affine3f::inv() (rigid inverse)
__device__ void tf_rigid_inv(const float* a, float* out)
{
    float o[12];
    for (int j = 0; j < 3; ++j) {
        for (int i = 0; i < 3; ++i) o[j * 4 + i] = a[i * 4 + j];
        o[j * 4 + 3] = -((a[0 * 4 + j] * a[3] + a[1 * 4 + j] * a[7]) + a[2 * 4 + j] * a[11]);
    }
    for (int i = 0; i < 12; ++i) out[i] = o[i];
}

// Matrix4::inv (Matrix.hpp:173-233)
__device__ void tf_matrix4_inv(const float* mm, float* dst)
{
    float tmp[12], src[16], det;
    for (int i = 0; i < 4; i++) {
        src[i] = mm[i * 4]; src[i + 4] = mm[i * 4 + 1]; src[i + 8] = mm[i * 4 + 2]; src[i + 12] = mm[i * 4 + 3];
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
    if (det == 0.0f) return;   // reference leaves dst partially written and returns false
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
    for (int i = 0; i < 16; ++i) dst[i] *= s;
}

// derive the matrices every later stage reads from a camera->world pose
__device__ void tf_set_pose_matrices(TfDevState* st, const float* pose, int alloc_mode)
{
    // alloc_mode 1: world->camera = pose.inv() (topfu.cpp:281-282)
    // alloc_mode 2: pose used as is (frame 0, topfu.cpp:202-203)
    if (alloc_mode) {
        float m[12];
        if (alloc_mode == 1) tf_rigid_inv(pose, m);
        else for (int i = 0; i < 12; ++i) m[i] = pose[i];
        tf_rt_to_m4(m, st->M_alloc);
        tf_matrix4_inv(st->M_alloc, st->invM_alloc);
    }
    tf_rt_to_m4(pose, st->M_ray);
}

__global__ void __launch_bounds__(256)
k_icp_solve(const float* __restrict__ partial, int nct, TfDevState* __restrict__ st, int last_iter)
{
    if (st->abort) return;
    __shared__ float red[27][256];
    __shared__ float sums[27];
    const int t = threadIdx.x;
    // icp_final_reduce_kernel (proj_icp.cu:382-403): per row k, thread t sums t, t+256, ...
    float s[27];
#pragma unroll
    for (int k = 0; k < 27; ++k) s[k] = 0.f;
    for (int j = t; j < nct; j += 256) {
        const float4* p4 = (const float4*)(partial + (size_t)j * ICP_PART_STRIDE);
        float v[28];
#pragma unroll
        for (int q = 0; q < 7; ++q) { float4 f = p4[q]; v[4 * q] = f.x; v[4 * q + 1] = f.y; v[4 * q + 2] = f.z; v[4 * q + 3] = f.w; }
#pragma unroll
        for (int k = 0; k < 27; ++k) s[k] += v[k];
    }
#pragma unroll
    for (int k = 0; k < 27; ++k) red[k][t] = s[k];
    __syncthreads();
    const int wave = t >> 6, lane = t & 63;
    for (int k = wave; k < 27; k += 4) {
        float a0 = red[k][lane] + red[k][lane + 128];
        float a1 = red[k][lane + 64] + red[k][lane + 192];
        float r = tf_wave_tree64(a0 + a1);
        if (lane == 0) sums[k] = r;
    }
    __syncthreads();
    if (t != 0) return;
    // StreamHelper::get unpacking (projective_icp.cpp:51-61)
    float A[36], b[6];
    int shift = 0;
    for (int i = 0; i < 6; ++i)
        for (int j = i; j < 7; ++j) {
            float value = sums[shift++];
            if (j == 6) b[i] = value;
            else A[j * 6 + i] = A[i * 6 + j] = value;
        }
    for (int k = 0; k < 27; ++k) st->sums[k] = sums[k];
    st->icp_iters += 1;
    double det = icp_det6(A);
    if (fabs(det) < 1e-15 || isnan(det)) {          // projective_icp.cpp:197-203
        st->icp_ok = 0;
        st->abort = 1;
        return;
    }
    float r[6], R[9], tinc[12], aff[12];
    icp_solve6(A, b, r);
    icp_rodrigues(r, R);
    for (int j = 0; j < 3; ++j) {
        tinc[j * 4 + 0] = R[j * 3 + 0]; tinc[j * 4 + 1] = R[j * 3 + 1]; tinc[j * 4 + 2] = R[j * 3 + 2];
        tinc[j * 4 + 3] = r[3 + j];
    }
    for (int i = 0; i < 12; ++i) aff[i] = st->affine[i];
    tf_rigid_mul(tinc, aff, aff);
    for (int i = 0; i < 12; ++i) st->affine[i] = aff[i];
    if (last_iter == 1) {
        // poses_.push_back(poses_.back() * affine) (topfu.cpp:243) and the derived matrices
        float pose[12];
        for (int i = 0; i < 12; ++i) pose[i] = st->pose[i];
        tf_rigid_mul(pose, aff, pose);
        for (int i = 0; i < 12; ++i) st->pose[i] = pose[i];
        tf_set_pose_matrices(st, pose, 1);
    }
}

__global__ void k_icp_begin(TfDevState* st)
{
    for (int i = 0; i < 12; ++i) st->affine[i] = (i % 5 == 0) ? 1.0f : 0.0f;   // affine = Identity
    st->icp_ok = 1;
    st->icp_iters = 0;
    st->abort = 0;
}

// explicit pose (stage entry points / frame 0): pose_in -> matrices
__global__ void k_pose_from_input(TfDevState* st, int mode)
{
    float pose[12];
    for (int i = 0; i < 12; ++i) pose[i] = st->pose_in[i];
    int alloc_mode = (mode & TF_POSE_ALLOC) ? 1 : ((mode & TF_POSE_ALLOC_NOINV) ? 2 : 0);
    tf_set_pose_matrices(st, pose, alloc_mode);
}

__global__ void k_frame0_matrices(TfDevState* st)
{
    st->icp_ok = 1;       // frame 0 runs no ICP
    st->icp_iters = 0;
    float pose[12];
    for (int i = 0; i < 12; ++i) pose[i] = st->pose[i];
    tf_set_pose_matrices(st, pose, 2);
}

hipError_t tfk_pose_from_input(tf_ctx* c, int mode)
{
    hipLaunchKernelGGL(k_pose_from_input, dim3(1), dim3(1), 0, c->stream, c->st, mode);
    return hipGetLastError();
}

hipError_t tfk_frame0_matrices(tf_ctx* c)
{
    hipLaunchKernelGGL(k_frame0_matrices, dim3(1), dim3(1), 0, c->stream, c->st);
    return hipGetLastError();
}

// estimateTransform (projective_icp.cpp:169-213): levels coarse -> fine
hipError_t tfk_icp(tf_ctx* c, int pose_update)
{
    const tf_params& p = c->p;
    hipLaunchKernelGGL(k_icp_begin, dim3(1), dim3(1), 0, c->stream, c->st);
    int levels = 4;
    while (levels > 0 && p.icp_iter_num[levels - 1] == 0) --levels;      // getUsedLevelsNum
    if (levels > TF_LEVELS) levels = TF_LEVELS;
    int last_l = -1;
    for (int l = 0; l < levels; ++l) if (p.icp_iter_num[l] > 0) { last_l = l; break; }
    for (int l = levels - 1; l >= 0; --l) {
        IcpLevel L;
        int div = 1 << l;                                                 // setLevelIntr
        L.vcurr = c->curr_pts[l]; L.ncurr = c->curr_nrm[l]; L.vprev = c->prev_pts[l]; L.nprev = c->prev_nrm[l];
        L.W = c->lw[l]; L.H = c->lh[l];
        L.gx = (L.W + 31) / 32;
        L.nct = L.gx * ((L.H + 7) / 8);
        L.fx = p.fx / (float)div; L.fy = p.fy / (float)div; L.cx = p.cx / (float)div; L.cy = p.cy / (float)div;
        L.min_cosine = c->min_cosine; L.dist2 = c->dist2_thres;
        for (int it = 0; it < p.icp_iter_num[l]; ++it) {
            hipLaunchKernelGGL(k_icp_partial, dim3((L.nct + 3) / 4), dim3(256), 0, c->stream, L, c->st, c->icp_partial);
            int last = (pose_update && l == last_l && it == p.icp_iter_num[l] - 1) ? 1 : 0;
            hipLaunchKernelGGL(k_icp_solve, dim3(1), dim3(256), 0, c->stream, c->icp_partial, L.nct, c->st, last);
        }
    }
    return hipGetLastError();
}
