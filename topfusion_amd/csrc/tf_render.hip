// tf_render.hip -- raycasting side of the hot path for gfx950.
//
//   k_raycast     : genericRaycast_device / castRay (VisualisationHelper.hpp:33-46,
//                   VisualisationEngine_Shared.hpp:99-172), incl. the IndexCache behaviour
//                   that decides which entries castRay<true> marks visible
//   k_grey        : renderGrey_device (VisualisationHelper.hpp:105-118)
//   k_icp_maps    : renderICP_device + 2x resizePointsNormals fused: every pyramid level
//                   is recomputed from the raycast result in one launch
//   k_ed_*        : CreateExpectedDepths (VisualisationEngine_CUDA.cu:119-173) as
//                   init+project, (cap check), fill with integer atomics on the positive
//                   float bit patterns (the reference's float CAS loops, CUDAUtils.hpp:75-95)
#include "tf_internal.h"

struct SceneView {
    const TfHashEntry* hash;
    const TfVoxel* vba;
    unsigned mask;
    int n_buckets;
};

struct RCache { int bx, by, bz, blockPtr; };   // VoxelBlockHash::IndexCache (VoxelBlockHash.hpp:58-62)

// readVoxel with cache (RepresentationAccess.hpp:73-104); pointToVoxelBlockPos :9-17
__device__ __forceinline__ TfVoxel rv_read(const SceneView& s, int px, int py, int pz, int* vm, RCache* k)
{
    int bx = ((px < 0) ? px - TF_BLK + 1 : px) / TF_BLK;
    int by = ((py < 0) ? py - TF_BLK + 1 : py) / TF_BLK;
    int bz = ((pz < 0) ? pz - TF_BLK + 1 : pz) / TF_BLK;
    int lin = px + (py - bx) * TF_BLK + (pz - by) * TF_BLK * TF_BLK - bz * TF_BLK3;
    if (bx == k->bx && by == k->by && bz == k->bz) {
        *vm = 1;
        return s.vba[k->blockPtr + lin];
    }
    int hashIdx = tf_hash_index(bx, by, bz, s.mask);
    while (true) {
        TfHashEntry e = s.hash[hashIdx];
        if (e.x == (short)bx && e.y == (short)by && e.z == (short)bz && e.ptr >= 0) {
            k->bx = bx; k->by = by; k->bz = bz; k->blockPtr = e.ptr * TF_BLK3;
            *vm = hashIdx + 1;
            return s.vba[k->blockPtr + lin];
        }
        if (e.offset < 1) break;
        hashIdx = s.n_buckets + e.offset - 1;
    }
    *vm = 0;
    TfVoxel d; d.sdf = 32767; d.w = 0; d.pad = 0;
    return d;
}

__device__ __forceinline__ float rv_sdf_nc(const SceneView& s, int px, int py, int pz)
{
    RCache k; k.bx = k.by = k.bz = 0x7fffffff; k.blockPtr = -1;
    int vm;
    return (float)rv_read(s, px, py, pz, &vm, &k).sdf;
}

__device__ __forceinline__ int tf_round(float x) { return (int)((x < 0) ? (x - 0.5f) : (x + 0.5f)); }

// readFromSDF_float_interpolated (RepresentationAccess.hpp:137-162)
__device__ __forceinline__ float rv_interp(const SceneView& s, const float* pt, int* vm, RCache* k)
{
    float res1, res2, v1, v2;
    float fx = floorf(pt[0]), fy = floorf(pt[1]), fz = floorf(pt[2]);
    int px = (int)fx, py = (int)fy, pz = (int)fz;
    float cx = pt[0] - fx, cy = pt[1] - fy, cz = pt[2] - fz;
    v1 = rv_read(s, px, py, pz, vm, k).sdf;
    v2 = rv_read(s, px + 1, py, pz, vm, k).sdf;
    res1 = (1.0f - cx) * v1 + cx * v2;
    v1 = rv_read(s, px, py + 1, pz, vm, k).sdf;
    v2 = rv_read(s, px + 1, py + 1, pz, vm, k).sdf;
    res1 = (1.0f - cy) * res1 + cy * ((1.0f - cx) * v1 + cx * v2);
    v1 = rv_read(s, px, py, pz + 1, vm, k).sdf;
    v2 = rv_read(s, px + 1, py, pz + 1, vm, k).sdf;
    res2 = (1.0f - cx) * v1 + cx * v2;
    v1 = rv_read(s, px, py + 1, pz + 1, vm, k).sdf;
    v2 = rv_read(s, px + 1, py + 1, pz + 1, vm, k).sdf;
    res2 = (1.0f - cy) * res2 + cy * ((1.0f - cx) * v1 + cx * v2);
    *vm = 1;
    return ((1.0f - cz) * res1 + cz * res2) / 32767.0f;
}

// readWithConfidenceFromSDF_float_interpolated (RepresentationAccess.hpp:164-199)
__device__ __forceinline__ float rv_interp_conf(const SceneView& s, float* conf, const float* pt, int* vm, RCache* k)
{
    float res1, res2, v1, v2, res1_c, res2_c, v1_c, v2_c;
    TfVoxel vx;
    float fx = floorf(pt[0]), fy = floorf(pt[1]), fz = floorf(pt[2]);
    int px = (int)fx, py = (int)fy, pz = (int)fz;
    float cx = pt[0] - fx, cy = pt[1] - fy, cz = pt[2] - fz;
    vx = rv_read(s, px, py, pz, vm, k); v1 = vx.sdf; v1_c = vx.w;
    vx = rv_read(s, px + 1, py, pz, vm, k); v2 = vx.sdf; v2_c = vx.w;
    res1 = (1.0f - cx) * v1 + cx * v2;
    res1_c = (1.0f - cx) * v1_c + cx * v2_c;
    vx = rv_read(s, px, py + 1, pz, vm, k); v1 = vx.sdf; v1_c = vx.w;
    vx = rv_read(s, px + 1, py + 1, pz, vm, k); v2 = vx.sdf; v2_c = vx.w;
    res1 = (1.0f - cy) * res1 + cy * ((1.0f - cx) * v1 + cx * v2);
    res1_c = (1.0f - cy) * res1_c + cy * ((1.0f - cx) * v1_c + cx * v2_c);
    vx = rv_read(s, px, py, pz + 1, vm, k); v1 = vx.sdf; v1_c = vx.w;
    vx = rv_read(s, px + 1, py, pz + 1, vm, k); v2 = vx.sdf; v2_c = vx.w;
    res2 = (1.0f - cx) * v1 + cx * v2;
    res2_c = (1.0f - cx) * v1_c + cx * v2_c;
    vx = rv_read(s, px, py + 1, pz + 1, vm, k); v1 = vx.sdf; v1_c = vx.w;
    vx = rv_read(s, px + 1, py + 1, pz + 1, vm, k); v2 = vx.sdf; v2_c = vx.w;
    res2 = (1.0f - cy) * res2 + cy * ((1.0f - cx) * v1 + cx * v2);
    res2_c = (1.0f - cy) * res2_c + cy * ((1.0f - cx) * v1_c + cx * v2_c);
    *vm = 1;
    *conf = (1.0f - cz) * res1_c + cz * res2_c;
    return ((1.0f - cz) * res1 + cz * res2) / 32767.0f;
}

struct RayArgs {
    SceneView s;
    const float2* range;
    float4* out;
    unsigned char* visType;      // non-null: castRay<true>
    int W, H;
    float invfx, invfy, ncx, ncy; // InvertProjectionParams (VisualisationEngine_Shared.hpp:28-31)
    float oneOverVoxelSize, mu;
};

__global__ void __launch_bounds__(256)
k_raycast(RayArgs a, const TfDevState* __restrict__ st)
{
    if (st->abort) return;
    const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= a.W || y >= a.H) return;
    const float* invM = st->M_ray;
    int locId2 = (int)floorf((float)x / TF_SUBSAMPLE) + (int)floorf((float)y / TF_SUBSAMPLE) * a.W;
    float2 vf = a.range[locId2];
    float r[3], ps[3], pe[3], dir[3], pt[3];
    int vmIndex = 0;
    float sdfValue = 1.0f, confidence = 0.0f, stepLength;
    const float stepScale = a.mu * a.oneOverVoxelSize;
    float pz = vf.x;
    float px = pz * (((float)x + a.ncx) * a.invfx);
    float py = pz * (((float)y + a.ncy) * a.invfy);
    float totalLength = sqrtf(((0.0f + px * px) + py * py) + pz * pz) * a.oneOverVoxelSize;
    tf_m4v3(invM, px, py, pz, 1.0f, r);
    ps[0] = r[0] * a.oneOverVoxelSize; ps[1] = r[1] * a.oneOverVoxelSize; ps[2] = r[2] * a.oneOverVoxelSize;
    pz = vf.y;
    px = pz * (((float)x + a.ncx) * a.invfx);
    py = pz * (((float)y + a.ncy) * a.invfy);
    float totalLengthMax = sqrtf(((0.0f + px * px) + py * py) + pz * pz) * a.oneOverVoxelSize;
    tf_m4v3(invM, px, py, pz, 1.0f, r);
    pe[0] = r[0] * a.oneOverVoxelSize; pe[1] = r[1] * a.oneOverVoxelSize; pe[2] = r[2] * a.oneOverVoxelSize;
    dir[0] = pe[0] - ps[0]; dir[1] = pe[1] - ps[1]; dir[2] = pe[2] - ps[2];
    float dn = 1.0f / sqrtf(dir[0] * dir[0] + dir[1] * dir[1] + dir[2] * dir[2]);
    dir[0] *= dn; dir[1] *= dn; dir[2] *= dn;
    pt[0] = ps[0]; pt[1] = ps[1]; pt[2] = ps[2];
    RCache k; k.bx = k.by = k.bz = 0x7fffffff; k.blockPtr = -1;
    while (totalLength < totalLengthMax) {
        sdfValue = (float)rv_read(a.s, tf_round(pt[0]), tf_round(pt[1]), tf_round(pt[2]), &vmIndex, &k).sdf / 32767.0f;
        if (a.visType && vmIndex) a.visType[vmIndex - 1] = 1;
        if (!vmIndex) {
            stepLength = (float)TF_BLK;
        } else {
            if ((sdfValue <= 0.1f) && (sdfValue >= -0.5f)) sdfValue = rv_interp(a.s, pt, &vmIndex, &k);
            if (sdfValue <= 0.0f) break;
            float q = sdfValue * stepScale;
            stepLength = (q < 1.0f) ? 1.0f : q;
        }
        pt[0] += stepLength * dir[0]; pt[1] += stepLength * dir[1]; pt[2] += stepLength * dir[2];
        totalLength += stepLength;
    }
    float w = 0.0f;
    if (sdfValue <= 0.0f) {
        stepLength = sdfValue * stepScale;
        pt[0] += stepLength * dir[0]; pt[1] += stepLength * dir[1]; pt[2] += stepLength * dir[2];
        sdfValue = rv_interp_conf(a.s, &confidence, pt, &vmIndex, &k);
        stepLength = sdfValue * stepScale;
        pt[0] += stepLength * dir[0]; pt[1] += stepLength * dir[1]; pt[2] += stepLength * dir[2];
        w = confidence + 1.0f;
    }
    a.out[x + y * a.W] = make_float4(pt[0], pt[1], pt[2], w);
}

hipError_t tfk_raycast(tf_ctx* c, int update_visible)
{
    RayArgs a;
    a.s.hash = c->hash; a.s.vba = c->vba; a.s.mask = (unsigned)(c->p.n_buckets - 1); a.s.n_buckets = c->p.n_buckets;
    a.range = (const float2*)c->range; a.out = (float4*)c->raycast;
    a.visType = update_visible ? c->visType : nullptr;
    a.W = c->W; a.H = c->H;
    a.invfx = 1.0f / c->p.fx; a.invfy = 1.0f / c->p.fy; a.ncx = -c->p.cx; a.ncy = -c->p.cy;
    a.oneOverVoxelSize = 1.0f / c->p.voxelSize; a.mu = c->p.mu;
    hipLaunchKernelGGL(k_raycast, dim3((c->W + 15) / 16, (c->H + 15) / 16), dim3(256), 0, c->stream, a, c->st);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// renderGrey_device: computeSingleNormalFromSDF (RepresentationAccess.hpp:340-453),
// computeNormalAndAngle (VisualisationEngine_Shared.hpp:187-203), drawPixelGrey (:272-276)
// ---------------------------------------------------------------------------------------
__device__ void sdf_normal(const SceneView& s, const float* pt, float* ret)
{
    float ffx = floorf(pt[0]), ffy = floorf(pt[1]), ffz = floorf(pt[2]);
    int px = (int)ffx, py = (int)ffy, pz = (int)ffz;
    float cx = pt[0] - ffx, cy = pt[1] - ffy, cz = pt[2] - ffz;
    float nx = 1.0f - cx, ny = 1.0f - cy, nz = 1.0f - cz;
#define RV(dx, dy, dz) rv_sdf_nc(s, px + (dx), py + (dy), pz + (dz))
    float f0 = RV(0, 0, 0), f1 = RV(1, 0, 0), f2 = RV(0, 1, 0), f3 = RV(1, 1, 0);
    float b0 = RV(0, 0, 1), b1 = RV(1, 0, 1), b2 = RV(0, 1, 1), b3 = RV(1, 1, 1);
    float t0, t1, t2, t3, p1, p2, v1;
    p1 = f0 * ny * nz + f2 * cy * nz + b0 * ny * cz + b2 * cy * cz;
    t0 = RV(-1, 0, 0); t1 = RV(-1, 1, 0); t2 = RV(-1, 0, 1); t3 = RV(-1, 1, 1);
    p2 = t0 * ny * nz + t1 * cy * nz + t2 * ny * cz + t3 * cy * cz;
    v1 = p1 * cx + p2 * nx;
    p1 = f1 * ny * nz + f3 * cy * nz + b1 * ny * cz + b3 * cy * cz;
    t0 = RV(2, 0, 0); t1 = RV(2, 1, 0); t2 = RV(2, 0, 1); t3 = RV(2, 1, 1);
    p2 = t0 * ny * nz + t1 * cy * nz + t2 * ny * cz + t3 * cy * cz;
    ret[0] = (p1 * nx + p2 * cx - v1) / 32767.0f;
    p1 = f0 * nx * nz + f1 * cx * nz + b0 * nx * cz + b1 * cx * cz;
    t0 = RV(0, -1, 0); t1 = RV(1, -1, 0); t2 = RV(0, -1, 1); t3 = RV(1, -1, 1);
    p2 = t0 * nx * nz + t1 * cx * nz + t2 * nx * cz + t3 * cx * cz;
    v1 = p1 * cy + p2 * ny;
    p1 = f2 * nx * nz + f3 * cx * nz + b2 * nx * cz + b3 * cx * cz;
    t0 = RV(0, 2, 0); t1 = RV(1, 2, 0); t2 = RV(0, 2, 1); t3 = RV(1, 2, 1);
    p2 = t0 * nx * nz + t1 * cx * nz + t2 * nx * cz + t3 * cx * cz;
    ret[1] = (p1 * ny + p2 * cy - v1) / 32767.0f;
    p1 = f0 * nx * ny + f1 * cx * ny + f2 * nx * cy + f3 * cx * cy;
    t0 = RV(0, 0, -1); t1 = RV(1, 0, -1); t2 = RV(0, 1, -1); t3 = RV(1, 1, -1);
    p2 = t0 * nx * ny + t1 * cx * ny + t2 * nx * cy + t3 * cx * cy;
    v1 = p1 * cz + p2 * nz;
    p1 = b0 * nx * ny + b1 * cx * ny + b2 * nx * cy + b3 * cx * cy;
    t0 = RV(0, 0, 2); t1 = RV(1, 0, 2); t2 = RV(0, 1, 2); t3 = RV(1, 1, 2);
    p2 = t0 * nx * ny + t1 * cx * ny + t2 * nx * cy + t3 * cx * cy;
    ret[2] = (p1 * nz + p2 * cz - v1) / 32767.0f;
#undef RV
}

__global__ void __launch_bounds__(256)
k_grey(SceneView s, const float4* __restrict__ ray, int n, const TfDevState* __restrict__ st, uchar4* __restrict__ out)
{
    if (st->abort) return;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    // lightSource = -Vector3f(pose.getColumn(2)) (VisualisationEngine_CUDA.cu:243)
    const float lx = -st->M_ray[8], ly = -st->M_ray[9], lz = -st->M_ray[10];
    float4 p = ray[i];
    unsigned char v = 0;
    if (p.w > 0) {
        float pt[3] = { p.x, p.y, p.z }, nn[3];
        sdf_normal(s, pt, nn);
        float ns = 1.0f / sqrtf(nn[0] * nn[0] + nn[1] * nn[1] + nn[2] * nn[2]);
        nn[0] *= ns; nn[1] *= ns; nn[2] *= ns;
        float angle = nn[0] * lx + nn[1] * ly + nn[2] * lz;
        if (angle > 0.0f) v = (unsigned char)((0.8f * angle + 0.2f) * 255.0f);
    }
    out[i] = make_uchar4(v, v, v, v);
}

hipError_t tfk_render_grey(tf_ctx* c)
{
    SceneView s; s.hash = c->hash; s.vba = c->vba; s.mask = (unsigned)(c->p.n_buckets - 1); s.n_buckets = c->p.n_buckets;
    int n = c->W * c->H;
    hipLaunchKernelGGL(k_grey, dim3((n + 255) / 256), dim3(256), 0, c->stream, s, (const float4*)c->raycast, n, c->st, c->grey);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// CreateICPMaps: processPixelICP<false,false> (VisualisationEngine_Shared.hpp:355-397 with
// computeNormalAndAngle :205-270) + resizePointsNormals x2 (imgproc.cu:355-388)
// ---------------------------------------------------------------------------------------
struct IcpMapArgs {
    const float4* ray;
    float4* pts[TF_LEVELS];
    float4* nrm[TF_LEVELS];
    int W, H;
    float voxelSize;
};

__device__ __forceinline__ void icp_pixel(const IcpMapArgs& a, float lx, float ly, float lz, int x, int y,
                                          float4* po, float4* no)
{
    const float4* ray = a.ray;
    const int W = a.W, H = a.H;
    float4 p = ray[x + y * W];
    bool found = p.w > 0.0f;
    float n0 = 0, n1 = 0, n2 = 0;
    if (found) {
        if (y <= 1 || y >= H - 2 || x <= 1 || x >= W - 2) found = false;
        else {
            float4 xp = ray[(x + 1) + y * W], yp = ray[x + (y + 1) * W];
            float4 xm = ray[(x - 1) + y * W], ym = ray[x + (y - 1) * W];
            if (xp.w <= 0 || yp.w <= 0 || xm.w <= 0 || ym.w <= 0) found = false;
            else {
                float dx0 = xp.x - xm.x, dx1 = xp.y - xm.y, dx2 = xp.z - xm.z;
                float dy0 = yp.x - ym.x, dy1 = yp.y - ym.y, dy2 = yp.z - ym.z;
                n0 = -(dx1 * dy2 - dx2 * dy1);
                n1 = -(dx2 * dy0 - dx0 * dy2);
                n2 = -(dx0 * dy1 - dx1 * dy0);
                float ns = 1.0f / sqrtf(n0 * n0 + n1 * n1 + n2 * n2);
                n0 *= ns; n1 *= ns; n2 *= ns;
                float angle = n0 * lx + n1 * ly + n2 * lz;
                if (!(angle > 0.0f)) found = false;
            }
        }
    }
    if (found) {
        *po = make_float4(p.x * a.voxelSize, p.y * a.voxelSize, p.z * a.voxelSize, 1.0f);
        *no = make_float4(n0, n1, n2, 1.0f);
    } else {
        float q = tf_qnan();
        *po = make_float4(q, q, q, q);
        *no = *po;
    }
}

// resize_points_normals_kernel body on four source samples
__device__ __forceinline__ void resize4(const float4* v, const float4* n, float4* vo, float4* no)
{
    float q = tf_qnan();
    *vo = make_float4(q, q, q, 0.f);
    *no = make_float4(q, q, q, 0.f);
    if (!isnan(v[0].x * v[1].x * v[2].x * v[3].x)) {
        *vo = make_float4((((v[0].x + v[1].x) + v[2].x) + v[3].x) * 0.25f, (((v[0].y + v[1].y) + v[2].y) + v[3].y) * 0.25f,
                          (((v[0].z + v[1].z) + v[2].z) + v[3].z) * 0.25f, 1.0f);
        *no = make_float4((((n[0].x + n[1].x) + n[2].x) + n[3].x) * 0.25f, (((n[0].y + n[1].y) + n[2].y) + n[3].y) * 0.25f,
                          (((n[0].z + n[1].z) + n[2].z) + n[3].z) * 0.25f, 0.f);
    }
}

__global__ void __launch_bounds__(256)
k_icp_maps(IcpMapArgs a, const TfDevState* __restrict__ st)
{
    if (st->abort) return;
    const int l = blockIdx.z;
    const int lw = a.W >> l, lh = a.H >> l;
    const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= lw || y >= lh) return;
    const float lx = -st->M_ray[8], ly = -st->M_ray[9], lz = -st->M_ray[10];
    float4 po, no;
    if (l == 0) {
        icp_pixel(a, lx, ly, lz, x, y, &po, &no);
    } else if (l == 1) {
        float4 v[4], n[4];
        icp_pixel(a, lx, ly, lz, 2 * x, 2 * y, &v[0], &n[0]);
        icp_pixel(a, lx, ly, lz, 2 * x + 1, 2 * y, &v[1], &n[1]);
        icp_pixel(a, lx, ly, lz, 2 * x, 2 * y + 1, &v[2], &n[2]);
        icp_pixel(a, lx, ly, lz, 2 * x + 1, 2 * y + 1, &v[3], &n[3]);
        resize4(v, n, &po, &no);
    } else {
        float4 v1[4], n1[4];
        for (int q = 0; q < 4; ++q) {
            int x1 = 2 * x + (q & 1), y1 = 2 * y + (q >> 1);
            float4 v[4], n[4];
            icp_pixel(a, lx, ly, lz, 2 * x1, 2 * y1, &v[0], &n[0]);
            icp_pixel(a, lx, ly, lz, 2 * x1 + 1, 2 * y1, &v[1], &n[1]);
            icp_pixel(a, lx, ly, lz, 2 * x1, 2 * y1 + 1, &v[2], &n[2]);
            icp_pixel(a, lx, ly, lz, 2 * x1 + 1, 2 * y1 + 1, &v[3], &n[3]);
            resize4(v, n, &v1[q], &n1[q]);
        }
        resize4(v1, n1, &po, &no);
    }
    a.pts[l][y * lw + x] = po;
    a.nrm[l][y * lw + x] = no;
}

hipError_t tfk_icp_maps(tf_ctx* c)
{
    IcpMapArgs a;
    a.ray = (const float4*)c->raycast;
    for (int l = 0; l < TF_LEVELS; ++l) { a.pts[l] = c->prev_pts[l]; a.nrm[l] = c->prev_nrm[l]; }
    a.W = c->W; a.H = c->H; a.voxelSize = c->p.voxelSize;
    hipLaunchKernelGGL(k_icp_maps, dim3((c->W + 15) / 16, (c->H + 15) / 16, TF_LEVELS), dim3(256), 0, c->stream, a, c->st);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// CreateExpectedDepths
// ---------------------------------------------------------------------------------------
struct EdArgs {
    const TfHashEntry* hash;
    const int* visibleIds;
    float2* range;
    int4* box; float2* z; int* tiles; unsigned char* keep;
    int W, H;
    float fx, fy, cx, cy, voxelSize;
    unsigned cap;
};

// memsetKernel(FAR_AWAY, VERY_CLOSE) + ProjectSingleBlock (VisualisationEngine_Shared.hpp:33-77)
__global__ void __launch_bounds__(256)
k_ed_project(EdArgs a, TfDevState* __restrict__ st)
{
    if (st->abort) return;
    const int tid = blockIdx.x * 256 + threadIdx.x, stride = gridDim.x * 256;
    const int npx = a.W * a.H;
    for (int i = tid; i < npx; i += stride) a.range[i] = make_float2(TF_FAR_AWAY, TF_VERY_CLOSE);
    const int n = st->noVisibleEntries;
    const float* M = st->M_alloc;          // pose.inv() (topfu.cpp:306)
    for (int i = tid; i < n; i += stride) {
        TfHashEntry e = a.hash[a.visibleIds[i]];
        int4 box = make_int4(-1, -1, -1, -1);
        float2 zr = make_float2(0.f, 0.f);
        int ntiles = 0;
        if (e.ptr >= 0) {
            int ulx = a.W / TF_SUBSAMPLE, uly = a.H / TF_SUBSAMPLE, lrx = -1, lry = -1;
            float zmin = TF_FAR_AWAY, zmax = TF_VERY_CLOSE;
            for (int corner = 0; corner < 8; ++corner) {
                short tx = (short)(e.x + ((corner & 1) ? 1 : 0));
                short ty = (short)(e.y + ((corner & 2) ? 1 : 0));
                short tz = (short)(e.z + ((corner & 4) ? 1 : 0));
                float q[3];
                tf_m4v3(M, (float)tx * (float)TF_BLK * a.voxelSize, (float)ty * (float)TF_BLK * a.voxelSize,
                        (float)tz * (float)TF_BLK * a.voxelSize, 1.0f, q);
                if ((double)q[2] < 1e-6) continue;
                float p2x = (a.fx * q[0] / q[2] + a.cx) / (float)TF_SUBSAMPLE;
                float p2y = (a.fy * q[1] / q[2] + a.cy) / (float)TF_SUBSAMPLE;
                if ((float)ulx > floorf(p2x)) ulx = (int)floorf(p2x);
                if ((float)lrx < ceilf(p2x)) lrx = (int)ceilf(p2x);
                if ((float)uly > floorf(p2y)) uly = (int)floorf(p2y);
                if ((float)lry < ceilf(p2y)) lry = (int)ceilf(p2y);
                if (zmin > q[2]) zmin = q[2];
                if (zmax < q[2]) zmax = q[2];
            }
            if (ulx < 0) ulx = 0;
            if (uly < 0) uly = 0;
            if (lrx >= a.W) lrx = a.W - 1;
            if (lry >= a.H) lry = a.H - 1;
            bool valid = !(ulx > lrx || uly > lry);
            if (valid && zmin < TF_VERY_CLOSE) zmin = TF_VERY_CLOSE;
            if (valid && zmax < TF_VERY_CLOSE) valid = false;
            if (valid) {
                int nbx = (int)ceilf((float)(lrx - ulx + 1) / TF_RB_SIZE);
                int nby = (int)ceilf((float)(lry - uly + 1) / TF_RB_SIZE);
                ntiles = nbx * nby;
                box = make_int4(ulx, uly, lrx, lry);
                zr = make_float2(zmin, zmax);
            }
        }
        a.box[i] = box; a.z[i] = zr; a.tiles[i] = ntiles;
        if (ntiles) atomicAdd(&st->tiles_total, (unsigned)ntiles);
    }
}

// MAX_RENDERING_BLOCKS handling (VisualisationHelper.cu:70-74): blocks whose tiles do not fit
// are dropped, in visible-list order.  Only does work when the cap is exceeded.
__global__ void k_ed_cap(EdArgs a, TfDevState* __restrict__ st)
{
    if (st->abort) return;
    unsigned total = st->tiles_total;
    if (threadIdx.x == 0) st->noTotalBlocks = (int)(total > a.cap ? a.cap : total);
    if (total <= a.cap) return;
    if (threadIdx.x != 0) return;
    const int n = st->noVisibleEntries;
    unsigned off = 0;
    for (int i = 0; i < n; ++i) {
        unsigned need = (unsigned)a.tiles[i];
        a.keep[i] = (need && off + need <= a.cap) ? 1 : 0;
        off += need;
    }
}

// fillBlocks_device (VisualisationHelper.cu:105-121): per-pixel min/max of the block z-range
__global__ void __launch_bounds__(256)
k_ed_fill(EdArgs a, const TfDevState* __restrict__ st)
{
    if (st->abort) return;
    const int n = st->noVisibleEntries;
    const bool capped = st->tiles_total > a.cap;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        int4 b = a.box[i];
        if (b.x < 0) continue;
        if (capped && !a.keep[i]) continue;
        float2 zr = a.z[i];
        int zmin = __float_as_int(zr.x), zmax = __float_as_int(zr.y);   // positive floats order as ints
        for (int y = b.y; y <= b.w; ++y)
            for (int x = b.x; x <= b.z; ++x) {
                int* px = (int*)(a.range + x + y * a.W);
                atomicMin(px, zmin);
                atomicMax(px + 1, zmax);
            }
    }
}

hipError_t tfk_expected_depths(tf_ctx* c)
{
    EdArgs a;
    a.hash = c->hash; a.visibleIds = c->visibleIds; a.range = (float2*)c->range;
    a.box = c->blockBox; a.z = c->blockZ; a.tiles = c->blockTiles; a.keep = c->blockKeep;
    a.W = c->W; a.H = c->H;
    a.fx = c->p.fx; a.fy = c->p.fy; a.cx = c->p.cx; a.cy = c->p.cy; a.voxelSize = c->p.voxelSize;
    a.cap = (unsigned)c->p.max_render_blocks;
    hipError_t e = hipMemsetAsync(&c->st->tiles_total, 0, sizeof(unsigned), c->stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_ed_project, dim3(1024), dim3(256), 0, c->stream, a, c->st);
    hipLaunchKernelGGL(k_ed_cap, dim3(1), dim3(64), 0, c->stream, a, c->st);
    hipLaunchKernelGGL(k_ed_fill, dim3(256), dim3(256), 0, c->stream, a, c->st);
    return hipGetLastError();
}
