// tf_render.hip -- raycasting side of the hot path for gfx950.
//
//   k_raycast     : genericRaycast_device / castRay (VisualisationHelper.hpp:33-46,
//                   VisualisationEngine_Shared.hpp:99-172), incl. the IndexCache behaviour
//                   that decides which entries castRay<true> marks visible
//   k_render_type : renderGrey_device and the other RenderImage types (VisualisationHelper.hpp:76-148)
//   k_icp_maps    : renderICP_device + 2x resizePointsNormals fused: every pyramid level
//                   is recomputed from the raycast result in one launch
//   k_ed_*        : CreateExpectedDepths (VisualisationEngine_CUDA.cu:119-173) as
//                   init+project, (cap check), fill with integer atomics on the positive
//                   float bit patterns (the reference's float CAS loops, CUDAUtils.hpp:75-95)
#include "tf_internal.h"
#include "tf_preproc.h"
#include "tf_reset.h"

struct SceneView {
    const TfHashEntry* hash;
    const TfVoxel* vba;      // the guard block before the VBA (tf_ctx::vba_guard): voxel offsets are voff + TF_BLK3 + lin
    const int2* grid;        // block grid (tf_internal.h, TF_GRID_*)
    unsigned mask;
    int n_buckets;
};

// VoxelBlockHash::IndexCache (VoxelBlockHash.hpp:58-62): the cached block position decides castRay's
// visibility marks; the cached pointer is never needed (voxels are read through the grid)
struct RCache { int bx, by, bz; };

// ---------------------------------------------------------------------------------------
// Voxel access through the block grid.  readVoxel (RepresentationAccess.hpp:73-104) walks a
// hash bucket and its excess chain for every block it enters; here a dense grid of
// (hash entry, VBA offset) pairs, kept exact by the allocation kernels (tf_scene.hip), answers
// the same question with one 8-byte load and no chain (blocks outside the grid fall back to
// the hash walk).  Every sample on the raycasting side touches a 2x2x2 (interpolation) or
// 4x4x4 (SDF gradient) voxel neighbourhood, so its <= 2x2x2 blocks are looked up together
// and the voxels then loaded together: two dependent round trips per sample, whatever the
// reference's serial corner order.  Values, the IndexCache state and vmIndex are exactly
// those of the reference's serial reads (RepresentationAccess.hpp:73-199).
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ int vblk(int p) { return p >> 3; }   // floor(p / 8) (:9-17), arithmetic shift
__device__ __forceinline__ int vlin(int x, int y, int z) { return (x & 7) + ((y & 7) << 3) + ((z & 7) << 6); }

// 32-bit byte offset from a uniform (kernel-argument) base: one global_load with an SGPR base
// and a VGPR offset, no 64-bit address arithmetic per lane
template <typename T>
__device__ __forceinline__ T ld_off(const void* base, unsigned byte_off)
{
    return *reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) + byte_off);
}

// the hash walk for a block outside the block grid (rare: the grid spans +-128 blocks)
__device__ __forceinline__ int2 blk_walk(const SceneView& s, int bx, int by, int bz)
{
    int hi = tf_hash_index(bx, by, bz, s.mask);
    while (true) {
        const TfHashEntry e = s.hash[hi];
        if (e.x == (short)bx && e.y == (short)by && e.z == (short)bz && e.ptr >= 0) return make_int2(hi, e.ptr * TF_BLK3);
        if (e.offset < 1) return make_int2(-1, TF_VOFF_NONE);
        hi = s.n_buckets + e.offset - 1;
    }
}

// Cell byte offsets of the 2x2x2 block set {X[i]} x {Y[j]} x {Z[k]} (corner c = i + 2j + 4k;
// X[1] - X[0] etc. are 0 or 1): the base cell's plus the per-axis steps.  False when a block lies
// outside the grid (then the offsets are meaningless and blk_lookup_slow answers).
__device__ __forceinline__ bool blk_offsets8(const int (&X)[2], const int (&Y)[2], const int (&Z)[2], unsigned (&o)[8])
{
    const unsigned x0 = (unsigned)(X[0] + TF_GRID_HALF), y0 = (unsigned)(Y[0] + TF_GRID_HALF), z0 = (unsigned)(Z[0] + TF_GRID_HALF);
    const unsigned x1 = (unsigned)(X[1] + TF_GRID_HALF), y1 = (unsigned)(Y[1] + TF_GRID_HALF), z1 = (unsigned)(Z[1] + TF_GRID_HALF);
    const unsigned base = ((z0 << (2 * TF_GRID_LOG)) | (y0 << TF_GRID_LOG) | x0) * 8u;
    const unsigned dx = (x1 - x0) * 8u, dy = (y1 - y0) << (TF_GRID_LOG + 3), dz = (z1 - z0) << (2 * TF_GRID_LOG + 3);
    o[0] = base; o[1] = base + dx; o[2] = base + dy; o[3] = o[1] + dy;
    o[4] = base + dz; o[5] = o[1] + dz; o[6] = o[2] + dz; o[7] = o[3] + dz;
    return (x0 | x1 | y0 | y1 | z0 | z1) < (unsigned)TF_GRID_DIM;
}
// (hash entry index, VBA voxel offset) per corner, or (-1, TF_VOFF_NONE) when findVoxel fails
__device__ __forceinline__ void blk_load8(const SceneView& s, const unsigned (&o)[8], int2 (&g)[8])
{
#pragma unroll
    for (int c = 0; c < 8; ++c) g[c] = ld_off<int2>(s.grid, o[c]);
}
// the rare case (a block outside the grid, i.e. beyond +-128 blocks): cell or hash walk per corner.
// Callers take it for the whole wave, so the common path's loads stay unbranched and in flight
// together.
// (one rolled loop with a single walk in it: eight inlined walk loops in the ray march's hot
// loop cost it registers and code size for a path the C2 / C3 scenes never take)
__device__ __forceinline__ void blk_lookup_slow(const SceneView& s, const int (&X)[2], const int (&Y)[2], const int (&Z)[2],
                                             int2 (&g)[8])
{
    int x0 = X[0], x1 = X[1], y0 = Y[0], y1 = Y[1], z0 = Z[0], z1 = Z[1];
    // (kept in VGPRs: left alone the optimiser turns the selects below into a private array in scratch)
    asm volatile("" : "+v"(x0), "+v"(x1), "+v"(y0), "+v"(y1), "+v"(z0), "+v"(z1));
#pragma unroll 1
    for (int c = 0; c < 8; ++c) {
        const int bx = (c & 1) ? x1 : x0, by = (c & 2) ? y1 : y0, bz = (c & 4) ? z1 : z0;
        const int2 r = tf_grid_in(bx, by, bz) ? s.grid[tf_grid_cell(bx, by, bz)] : blk_walk(s, bx, by, bz);
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (k == c) g[k] = r;
    }
}
__device__ __forceinline__ bool wave_any(bool p) { return __builtin_amdgcn_ballot_w64(p) != 0; }

__device__ __forceinline__ void blk_find8(const SceneView& s, const int (&X)[2], const int (&Y)[2], const int (&Z)[2],
                                          int (&hidx)[8], int (&voff)[8])
{
    unsigned o[8];
    int2 g[8];
    const bool in = blk_offsets8(X, Y, Z, o);
    if (wave_any(!in)) blk_lookup_slow(s, X, Y, Z, g);
    else blk_load8(s, o, g);
#pragma unroll
    for (int c = 0; c < 8; ++c) { hidx[c] = g[c].x; voff[c] = g[c].y; }
}

// raw Voxel_s word (sdf = low 16 bits, w = bits 16-23) of voxel `lin` of the block at VBA offset
// voff, read relative to the guard block before the VBA (SceneView::vba): a missing block
// (voff = TF_VOFF_NONE) reads the guard's Voxel_s() = (32767, 0).  Byte offsets fit 32 bits:
// the largest is 4 * (ptr*512 + 512 + 511) for ptr = n_blocks - 1, below 2^32 because tf_create
// accepts at most 2^21 - 1 blocks (the guard block is the 2^21-th 2 KiB block of the range).
__device__ __forceinline__ unsigned vox_at(const SceneView& s, int voff, int lin_g)
{
    return ld_off<unsigned>(s.vba, (unsigned)(voff + lin_g) * 4u);
}
// in-block index of voxel coordinate p along one axis, pre-scaled; the guard shift rides on z
__device__ __forceinline__ int lin_x(int x) { return x & 7; }
__device__ __forceinline__ int lin_y(int y) { return (y & 7) << 3; }
__device__ __forceinline__ int lin_zg(int z) { return ((z & 7) << 6) + TF_BLK3; }
__device__ __forceinline__ float raw_sdf(unsigned r) { return (float)(short)(r & 0xffffu); }
__device__ __forceinline__ float raw_w(unsigned r) { return (float)((r >> 16) & 0xffu); }

// v[ux + 2uy + 4uz] for per-axis bits: a 3-level select tree (7 selects on 3 shared conditions)
// (the empty asm keeps the selects as selects: left alone the optimiser rebuilds the tree
// into a dynamically indexed private array in scratch)
template <typename T>
__device__ __forceinline__ T sel_tree(const T (&v)[8], bool ux, bool uy, bool uz)
{
    T w[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) { w[c] = v[c]; asm volatile("" : "+v"(w[c])); }
    const T a0 = ux ? w[1] : w[0], a1 = ux ? w[3] : w[2], a2 = ux ? w[5] : w[4], a3 = ux ? w[7] : w[6];
    const T b0 = uy ? a1 : a0, b1 = uy ? a3 : a2;
    return uz ? b1 : b0;
}

// ROUND (the reference's (int)ROUND(x) for the uninterpolated read)
__device__ __forceinline__ int tf_round(float x) { return (int)((x < 0) ? (x - 0.5f) : (x + 0.5f)); }

// the 8 interpolation corners of pt (floor .. floor+1) in the read order of
// readFromSDF_float_interpolated (RepresentationAccess.hpp:137-162): corner c = (c&1, c>>1&1, c>>2)
struct Corners {
    int fx, fy, fz;          // floor(pt)
    float cx, cy, cz;        // fractions
    int bx, by, bz;          // block of floor(pt)
    int sx, sy, sz;          // 1 when floor+1 is in the next block along that axis
    int cu;                  // ROUND(pt) = corner (cu&1, cu>>1&1, cu>>2) (the uninterpolated read)
    int hU;                  // hash entry of ROUND(pt)'s block (-1: none)
    unsigned valid;          // bit c: corner c's block exists
    int voff[8];             // per corner: VBA offset of its block (TF_VOFF_NONE: none)
    unsigned raw[8];         // per corner: voxel word
};

// A step's corner lookups in phases -- corners_prep (VALU only: floors, blocks, grid offsets),
// the grid loads, corners_vox (block offsets -> the eight voxel loads) -- so that two rays
// interleaved as grid(A) grid(B) vox(A) vox(B) share one round trip per phase.
__device__ __forceinline__ bool corners_prep(const float* pt, Corners& q, unsigned (&o)[8])
{
    const float ffx = floorf(pt[0]), ffy = floorf(pt[1]), ffz = floorf(pt[2]);
    q.fx = (int)ffx; q.fy = (int)ffy; q.fz = (int)ffz;
    q.cx = pt[0] - ffx; q.cy = pt[1] - ffy; q.cz = pt[2] - ffz;
    q.bx = vblk(q.fx); q.by = vblk(q.fy); q.bz = vblk(q.fz);
    q.sx = vblk(q.fx + 1) - q.bx; q.sy = vblk(q.fy + 1) - q.by; q.sz = vblk(q.fz + 1) - q.bz;
    q.cu = (tf_round(pt[0]) - q.fx) + 2 * (tf_round(pt[1]) - q.fy) + 4 * (tf_round(pt[2]) - q.fz);
    const int X[2] = { q.bx, q.bx + q.sx }, Y[2] = { q.by, q.by + q.sy }, Z[2] = { q.bz, q.bz + q.sz };
    return blk_offsets8(X, Y, Z, o);
}
__device__ __forceinline__ void corners_slow(const SceneView& s, const Corners& q, int2 (&g)[8])
{
    const int X[2] = { q.bx, q.bx + q.sx }, Y[2] = { q.by, q.by + q.sy }, Z[2] = { q.bz, q.bz + q.sz };
    blk_lookup_slow(s, X, Y, Z, g);
}
__device__ __forceinline__ void corners_blocks(Corners& q, const int2 (&g)[8])
{
    int hidx[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) { hidx[c] = g[c].x; q.voff[c] = g[c].y; }
    q.valid = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) q.valid |= (q.voff[c] >= 0 ? 1u : 0u) << c;
    q.hU = sel_tree(hidx, (q.cu & 1) != 0, (q.cu & 2) != 0, (q.cu & 4) != 0);
}
__device__ __forceinline__ void corners_vox(const SceneView& s, Corners& q)
{
    const int lx[2] = { lin_x(q.fx), lin_x(q.fx + 1) }, ly[2] = { lin_y(q.fy), lin_y(q.fy + 1) };
    const int lz[2] = { lin_zg(q.fz), lin_zg(q.fz + 1) };
#pragma unroll
    for (int c = 0; c < 8; ++c) q.raw[c] = vox_at(s, q.voff[c], lx[c & 1] + ly[(c >> 1) & 1] + lz[c >> 2]);
}
// the block lookups of pt's corners (one grid round trip; the wave takes the slow path together)
__device__ __forceinline__ void corners_lookup(const SceneView& s, const float* pt, Corners& q)
{
    unsigned o[8];
    int2 g[8];
    const bool in = corners_prep(pt, q, o);
    if (wave_any(!in)) corners_slow(s, q, g);
    else blk_load8(s, o, g);
    corners_blocks(q, g);
}
// the IndexCache after the 8 serial corner reads: the block of the last corner whose block exists
__device__ __forceinline__ void corners_cache(const Corners& q, RCache* k)
{
    if (q.valid) {
        const int last = 31 - __builtin_clz(q.valid);
        k->bx = q.bx + ((last & 1) & q.sx); k->by = q.by + (((last >> 1) & 1) & q.sy); k->bz = q.bz + ((last >> 2) & q.sz);
    }
}

__device__ __forceinline__ float interp_sdf(const Corners& q)
{   // readFromSDF_float_interpolated arithmetic
    const float cx = q.cx, cy = q.cy, cz = q.cz;
    float res1, res2, v1, v2;
    v1 = raw_sdf(q.raw[0]); v2 = raw_sdf(q.raw[1]);
    res1 = (1.0f - cx) * v1 + cx * v2;
    v1 = raw_sdf(q.raw[2]); v2 = raw_sdf(q.raw[3]);
    res1 = (1.0f - cy) * res1 + cy * ((1.0f - cx) * v1 + cx * v2);
    v1 = raw_sdf(q.raw[4]); v2 = raw_sdf(q.raw[5]);
    res2 = (1.0f - cx) * v1 + cx * v2;
    v1 = raw_sdf(q.raw[6]); v2 = raw_sdf(q.raw[7]);
    res2 = (1.0f - cy) * res2 + cy * ((1.0f - cx) * v1 + cx * v2);
    return tf_div32767((1.0f - cz) * res1 + cz * res2);
}

__device__ __forceinline__ float interp_sdf_conf(const Corners& q, float* conf)
{   // readWithConfidenceFromSDF_float_interpolated arithmetic (RepresentationAccess.hpp:164-199)
    const float cx = q.cx, cy = q.cy, cz = q.cz;
    float res1, res2, v1, v2, res1_c, res2_c, v1_c, v2_c;
    v1 = raw_sdf(q.raw[0]); v1_c = raw_w(q.raw[0]); v2 = raw_sdf(q.raw[1]); v2_c = raw_w(q.raw[1]);
    res1 = (1.0f - cx) * v1 + cx * v2;
    res1_c = (1.0f - cx) * v1_c + cx * v2_c;
    v1 = raw_sdf(q.raw[2]); v1_c = raw_w(q.raw[2]); v2 = raw_sdf(q.raw[3]); v2_c = raw_w(q.raw[3]);
    res1 = (1.0f - cy) * res1 + cy * ((1.0f - cx) * v1 + cx * v2);
    res1_c = (1.0f - cy) * res1_c + cy * ((1.0f - cx) * v1_c + cx * v2_c);
    v1 = raw_sdf(q.raw[4]); v1_c = raw_w(q.raw[4]); v2 = raw_sdf(q.raw[5]); v2_c = raw_w(q.raw[5]);
    res2 = (1.0f - cx) * v1 + cx * v2;
    res2_c = (1.0f - cx) * v1_c + cx * v2_c;
    v1 = raw_sdf(q.raw[6]); v1_c = raw_w(q.raw[6]); v2 = raw_sdf(q.raw[7]); v2_c = raw_w(q.raw[7]);
    res2 = (1.0f - cy) * res2 + cy * ((1.0f - cx) * v1 + cx * v2);
    res2_c = (1.0f - cy) * res2_c + cy * ((1.0f - cx) * v1_c + cx * v2_c);
    *conf = (1.0f - cz) * res1_c + cz * res2_c;
    return tf_div32767((1.0f - cz) * res1 + cz * res2);
}


struct RayArgs {
    SceneView s;
    const float2* range;
    float4* out;
    unsigned char* visType;      // non-null: castRay<true>
    uchar4* grey;                // non-null: fused renderGrey (frame path)
    int W, H;
    float invfx, invfy, ncx, ncy; // InvertProjectionParams (VisualisationEngine_Shared.hpp:28-31)
    float oneOverVoxelSize, mu;
};

// castRay's state (VisualisationEngine_Shared.hpp:99-172): ray_init, the march loop
// (ray_march_lite), ray_refine at the surface.
struct Ray {
    float pt[3], dir[3];
    float totalLength, totalLengthMax, sdfValue;
    RCache k;
    bool active;             // inside castRay's while loop
};

// vf: the range image at the ray's /8 pixel (renderingRangeImage[locId2], :104-106)
__device__ __forceinline__ void ray_init(const RayArgs& a, const float* invM, int x, int y, float2 vf, Ray& R)
{
    float r[3], ps[3], pe[3];
    float pz = vf.x;
    float px = pz * (((float)x + a.ncx) * a.invfx);
    float py = pz * (((float)y + a.ncy) * a.invfy);
    R.totalLength = sqrtf(((0.0f + px * px) + py * py) + pz * pz) * a.oneOverVoxelSize;
    tf_m4v3(invM, px, py, pz, 1.0f, r);
    ps[0] = r[0] * a.oneOverVoxelSize; ps[1] = r[1] * a.oneOverVoxelSize; ps[2] = r[2] * a.oneOverVoxelSize;
    pz = vf.y;
    px = pz * (((float)x + a.ncx) * a.invfx);
    py = pz * (((float)y + a.ncy) * a.invfy);
    R.totalLengthMax = sqrtf(((0.0f + px * px) + py * py) + pz * pz) * a.oneOverVoxelSize;
    tf_m4v3(invM, px, py, pz, 1.0f, r);
    pe[0] = r[0] * a.oneOverVoxelSize; pe[1] = r[1] * a.oneOverVoxelSize; pe[2] = r[2] * a.oneOverVoxelSize;
    R.dir[0] = pe[0] - ps[0]; R.dir[1] = pe[1] - ps[1]; R.dir[2] = pe[2] - ps[2];
    float dn = 1.0f / sqrtf(R.dir[0] * R.dir[0] + R.dir[1] * R.dir[1] + R.dir[2] * R.dir[2]);
    R.dir[0] *= dn; R.dir[1] *= dn; R.dir[2] *= dn;
    R.pt[0] = ps[0]; R.pt[1] = ps[1]; R.pt[2] = ps[2];
    R.k.bx = R.k.by = R.k.bz = 0x7fffffff;
    R.sdfValue = 1.0f;
    R.active = R.totalLength < R.totalLengthMax;
}

// castRay's refinement at the surface: the step back onto it; true when there is one (then the
// confidence read at the new pt completes it, ray_march_lite)
__device__ __forceinline__ bool ray_refine(const RayArgs& a, Ray& R)
{
    if (!(R.sdfValue <= 0.0f)) return false;
    const float stepLength = R.sdfValue * (a.mu * a.oneOverVoxelSize);
    R.pt[0] += stepLength * R.dir[0]; R.pt[1] += stepLength * R.dir[1]; R.pt[2] += stepLength * R.dir[2];
    return true;
}
#ifdef TF_RAY_STATS
// diagnostic builds only (tools/ray_stats.py): per ray, steps in unallocated space (bits 0-9),
// steps that read voxels (bits 10-20) and of those the band steps that also read the eight
// interpolation corners (bits 21-31), for the two raycasts of the last pair launch
__device__ unsigned tf_ray_stats_buf[4 * 1280 * 960];   // [2][W*H] counts, then [2][W*H] sdf = 1 voxel steps
extern "C" int tf_debug_ray_stats(void* host, size_t bytes)
{
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(tf_ray_stats_buf), bytes < sizeof(tf_ray_stats_buf) ? bytes : sizeof(tf_ray_stats_buf), 0,
                                    hipMemcpyDeviceToHost);
}
#endif

// (hash entry, VBA offset) of one block: its grid cell, or the hash walk outside the grid (the wave
// takes that branch together; the common path's load stays unbranched)
__device__ __forceinline__ int2 blk_one(const SceneView& s, int bx, int by, int bz)
{
    const bool in = tf_grid_in(bx, by, bz);
    const unsigned off = in ? (unsigned)tf_grid_cell(bx, by, bz) * 8u : 0u;
    int2 g = ld_off<int2>(s.grid, off);
    if (wave_any(!in)) {
        if (!in) g = blk_walk(s, bx, by, bz);
    }
    return g;
}

// readFromSDF_float_interpolated at pt (RepresentationAccess.hpp:137-162) with the IndexCache
// update of its eight serial reads; with conf != nullptr readWithConfidenceFromSDF_float_interpolated
// (:164-199).  One array holds the corners' VBA offsets and then, loaded over them, their voxel
// words: the register footprint of the band steps is what sets the march's occupancy.
__device__ __forceinline__ float interp_at(const SceneView& s, const float* pt, RCache* k, float* conf)
{
    Corners q;
    unsigned o[8];
    const bool in = corners_prep(pt, q, o);
    int v[8];
    if (wave_any(!in)) {
        int2 g[8];
        corners_slow(s, q, g);
#pragma unroll
        for (int c = 0; c < 8; ++c) v[c] = g[c].y;
    } else {
#pragma unroll
        for (int c = 0; c < 8; ++c) v[c] = ld_off<int>(s.grid, o[c] + 4u);
    }
    q.valid = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) q.valid |= (v[c] >= 0 ? 1u : 0u) << c;
    if (k) corners_cache(q, k);
    const int lx[2] = { lin_x(q.fx), lin_x(q.fx + 1) }, ly[2] = { lin_y(q.fy), lin_y(q.fy + 1) };
    const int lz[2] = { lin_zg(q.fz), lin_zg(q.fz + 1) };
#pragma unroll
    for (int c = 0; c < 8; ++c) q.raw[c] = vox_at(s, v[c], lx[c & 1] + ly[(c >> 1) & 1] + lz[c >> 2]);
    return conf ? interp_sdf_conf(q, conf) : interp_sdf(q);
}

// castRay with the uninterpolated read alone on most steps: a step looks up ROUND(pt)'s block
// (one grid load) and reads its one voxel; only a step whose value lies in the band
// [-0.5, 0.1] (where castRay switches to the interpolated read, 1-3 steps a ray) fetches the
// eight interpolation corners.  Against the eight-corner fetch on every step this spends two
// round trips more per band step, and holds far fewer registers across the loop (the ray state
// only): more waves resident to hide the dependent loads.  Values, visibility marks and the
// IndexCache follow castRay's serial reads exactly (VisualisationEngine_Shared.hpp:117-160).
template <bool MARK>
__device__ __forceinline__ float ray_march_lite(const RayArgs& a, const float* invM, int x, int y, float2 vf, float* pt)
{
    Ray R;
    ray_init(a, invM, x, y, vf, R);
    const float stepScale = a.mu * a.oneOverVoxelSize;
#ifdef TF_RAY_STATS
    unsigned n_free = 0, n_found = 0, n_band = 0, n_one = 0;
#endif
    while (R.active) {
        const int rx = tf_round(R.pt[0]), ry = tf_round(R.pt[1]), rz = tf_round(R.pt[2]);
        const int bx = vblk(rx), by = vblk(ry), bz = vblk(rz);
        const int2 g = blk_one(a.s, bx, by, bz);
        const bool found = g.y >= 0;
        int vmIndex = 0;
        if (found) {
            const bool hit = bx == R.k.bx && by == R.k.by && bz == R.k.bz;
            vmIndex = hit ? 1 : g.x + 1;
            R.k.bx = bx; R.k.by = by; R.k.bz = bz;
        }
#ifdef TF_RAY_STATS
        if (found) ++n_found; else ++n_free;
#endif
        unsigned raw = 0;
        if (wave_any(found)) raw = vox_at(a.s, g.y, lin_x(rx) + lin_y(ry) + lin_zg(rz));
        // a missing block reads Voxel_s(): 32767 / 32767 = 1
        float sdfValue = found ? tf_short_to_float((short)(raw & 0xffffu)) : 1.0f;
#ifdef TF_RAY_STATS
        if (found && (raw & 0xffffu) == 0x7fffu) ++n_one;
#endif
        if (MARK && vmIndex) a.visType[vmIndex - 1] = 1;
        float stepLength;
        if (!vmIndex) {
            stepLength = (float)TF_BLK;
        } else {
            if ((sdfValue <= 0.1f) && (sdfValue >= -0.5f)) {
#ifdef TF_RAY_STATS
                ++n_band;
#endif
                sdfValue = interp_at(a.s, R.pt, &R.k, nullptr);
            }
            if (sdfValue <= 0.0f) { R.sdfValue = sdfValue; R.active = false; continue; }   // the loop's break
            const float qq = sdfValue * stepScale;
            stepLength = (qq < 1.0f) ? 1.0f : qq;
        }
        R.sdfValue = sdfValue;
        R.pt[0] += stepLength * R.dir[0]; R.pt[1] += stepLength * R.dir[1]; R.pt[2] += stepLength * R.dir[2];
        R.totalLength += stepLength;
        R.active = R.totalLength < R.totalLengthMax;
    }
#ifdef TF_RAY_STATS
    if (x + y * a.W < 1280 * 960)
    {
        tf_ray_stats_buf[(MARK ? 0 : 1280 * 960) + x + y * a.W] = min(n_free, 1023u) | (min(n_found, 2047u) << 10) | (min(n_band, 2047u) << 21);
        tf_ray_stats_buf[2 * 1280 * 960 + (MARK ? 0 : 1280 * 960) + x + y * a.W] = n_one;
    }
#endif
    float w = 0.0f;
    if (ray_refine(a, R)) {                 // ray_finish on interp_at's confidence read
        float confidence;
        const float sdfValue = interp_at(a.s, R.pt, nullptr, &confidence);
        const float stepLength = sdfValue * (a.mu * a.oneOverVoxelSize);
        R.pt[0] += stepLength * R.dir[0]; R.pt[1] += stepLength * R.dir[1]; R.pt[2] += stepLength * R.dir[2];
        w = confidence + 1.0f;
    }
    pt[0] = R.pt[0]; pt[1] = R.pt[1]; pt[2] = R.pt[2];
    return w;
}

template <bool MARK>
__device__ __forceinline__ float ray_march(const RayArgs& a, const float* invM, int x, int y, float2 vf, float* pt)
{
    return ray_march_lite<MARK>(a, invM, x, y, vf, pt);
}

// ---------------------------------------------------------------------------------------
// renderGrey_device: computeSingleNormalFromSDF (RepresentationAccess.hpp:340-453),
// computeNormalAndAngle (VisualisationEngine_Shared.hpp:187-203), drawPixelGrey (:272-276).
// The 32 uncached reads cover pt's 4x4x4 neighbourhood (floor-1 .. floor+2): <= 2x2x2 blocks.
// ---------------------------------------------------------------------------------------
// vtab: this thread's 8-entry slot in LDS (VTAB_STRIDE ints): the 2x2x2 block offsets, so each
// of the 32 reads finds its block with one LDS load instead of an 8-way select.
#define VTAB_STRIDE 9
#ifndef TF_NORMAL_PHASES
#define TF_NORMAL_PHASES 1
#endif
__device__ void sdf_normal(const SceneView& s, const float* pt, float* ret, int* vtab)
{
    float ffx = floorf(pt[0]), ffy = floorf(pt[1]), ffz = floorf(pt[2]);
    int px = (int)ffx, py = (int)ffy, pz = (int)ffz;
    float cx = pt[0] - ffx, cy = pt[1] - ffy, cz = pt[2] - ffz;
    float nx = 1.0f - cx, ny = 1.0f - cy, nz = 1.0f - cz;
    const int bx = vblk(px - 1), by = vblk(py - 1), bz = vblk(pz - 1);
    const int sx = vblk(px + 2) - bx, sy = vblk(py + 2) - by, sz = vblk(pz + 2) - bz;
    int voff[8], hidx[8];
    const int X[2] = { bx, bx + sx }, Y[2] = { by, by + sy }, Z[2] = { bz, bz + sz };
    blk_find8(s, X, Y, Z, hidx, voff);
#pragma unroll
    for (int c = 0; c < 8; ++c) vtab[c] = voff[c];
    int tx[4], ty[4], tz[4], lx[4], ly[4], lz[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        tx[d] = vblk(px - 1 + d) - bx; ty[d] = 2 * (vblk(py - 1 + d) - by); tz[d] = 4 * (vblk(pz - 1 + d) - bz);
        lx[d] = lin_x(px - 1 + d); ly[d] = lin_y(py - 1 + d); lz[d] = lin_zg(pz - 1 + d);
    }
#define RV(dx, dy, dz) raw_sdf(vox_at(s, vtab[tx[(dx) + 1] + ty[(dy) + 1] + tz[(dz) + 1]], \
                                      lx[(dx) + 1] + ly[(dy) + 1] + lz[(dz) + 1]))
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
    ret[0] = tf_div32767(p1 * nx + p2 * cx - v1);
#if TF_NORMAL_PHASES
    // the y and z reads after the x derivative: 16 + 16 loads in flight instead of 32, so the
    // raycast kernels that end in this gradient keep their register budget (one more round trip
    // per pixel, once, against the march's many)
    __builtin_amdgcn_sched_barrier(0);
#endif
    p1 = f0 * nx * nz + f1 * cx * nz + b0 * nx * cz + b1 * cx * cz;
    t0 = RV(0, -1, 0); t1 = RV(1, -1, 0); t2 = RV(0, -1, 1); t3 = RV(1, -1, 1);
    p2 = t0 * nx * nz + t1 * cx * nz + t2 * nx * cz + t3 * cx * cz;
    v1 = p1 * cy + p2 * ny;
    p1 = f2 * nx * nz + f3 * cx * nz + b2 * nx * cz + b3 * cx * cz;
    t0 = RV(0, 2, 0); t1 = RV(1, 2, 0); t2 = RV(0, 2, 1); t3 = RV(1, 2, 1);
    p2 = t0 * nx * nz + t1 * cx * nz + t2 * nx * cz + t3 * cx * cz;
    ret[1] = tf_div32767(p1 * ny + p2 * cy - v1);
    p1 = f0 * nx * ny + f1 * cx * ny + f2 * nx * cy + f3 * cx * cy;
    t0 = RV(0, 0, -1); t1 = RV(1, 0, -1); t2 = RV(0, 1, -1); t3 = RV(1, 1, -1);
    p2 = t0 * nx * ny + t1 * cx * ny + t2 * nx * cy + t3 * cx * cy;
    v1 = p1 * cz + p2 * nz;
    p1 = b0 * nx * ny + b1 * cx * ny + b2 * nx * cy + b3 * cx * cy;
    t0 = RV(0, 0, 2); t1 = RV(1, 0, 2); t2 = RV(0, 1, 2); t3 = RV(1, 1, 2);
    p2 = t0 * nx * ny + t1 * cx * ny + t2 * nx * cy + t3 * cx * cy;
    ret[2] = tf_div32767(p1 * nz + p2 * cz - v1);
#undef RV
}

// computeNormalAndAngle<TVoxel,TIndex> (VisualisationEngine_Shared.hpp:189-203): the SDF-gradient
// normal at pt, normalised, and its angle to the light; false when the angle is not positive
__device__ __forceinline__ bool sdf_normal_angle(const SceneView& s, const float* pt, float lx, float ly, float lz,
                                                 float* nn, float* angle, int* vtab)
{
    sdf_normal(s, pt, nn, vtab);
    float ns = 1.0f / sqrtf(nn[0] * nn[0] + nn[1] * nn[1] + nn[2] * nn[2]);
    nn[0] *= ns; nn[1] *= ns; nn[2] *= ns;
    *angle = nn[0] * lx + nn[1] * ly + nn[2] * lz;
    return *angle > 0.0f;
}

// drawPixelGrey (VisualisationEngine_Shared.hpp:272-276)
__device__ __forceinline__ unsigned char grey_of(float angle) { return (unsigned char)((0.8f * angle + 0.2f) * 255.0f); }

__device__ __forceinline__ unsigned char grey_pixel(const SceneView& s, const float* pt, float lx, float ly, float lz,
                                                    int* vtab)
{
    float nn[3], angle;
    return sdf_normal_angle(s, pt, lx, ly, lz, nn, &angle, vtab) ? grey_of(angle) : (unsigned char)0;
}

// XCD-aware tile order: consecutive image tiles land on the same XCD (and its L2)
__device__ __forceinline__ int xcd_tile(int bid, int n)
{
    const int per = (n + 7) / 8;
    const int t = (bid % 8) * per + bid / 8;
    return t < n ? t : -1;
}

// MODE 0: castRay<false> -> point image; 1: castRay<true> (visibility marks) -> point image
// (CreateICPMaps); 2: castRay<false> + renderGrey fused (renderImage in the frame path).
// vtab: the caller's LDS for MODE 2's gradient (256 * VTAB_STRIDE ints).  rng (the frame kernel's
// CreateICPMaps rays with CreateExpectedDepths' fill fused in): the tile's four /8 range pixels,
// computed by the caller; else the range image is read.
template <int MODE, bool RNG_LDS = false>
__device__ __forceinline__ void raycast_tile(const RayArgs& a, const TfDevState* __restrict__ st, int tile,
                                             int tiles_x, int* vtab, const float2* rng = nullptr)
{
    const int tx = tile % tiles_x, ty = tile / tiles_x;
    // wave w casts the tile's 8x8 quadrant (w & 1, w >> 1): exactly one /8 pixel of the range
    // image, so the wave's rays start and end on the same range (similar lengths, the wave waits
    // on fewer stragglers), and a load of the wave touches a more compact footprint of voxels
    // (C2: raycast pair 80 -> 73 us against 4x16-pixel waves)
    const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
    const int x = tx * 16 + (wv & 1) * 8 + (ln & 7), y = ty * 16 + (wv >> 1) * 8 + (ln >> 3);
    if (x >= a.W || y >= a.H) return;
    const float2 vf = RNG_LDS ? rng[((y >> 3) - 2 * ty) * 2 + ((x >> 3) - 2 * tx)]
                              : a.range[(int)floorf((float)x / TF_SUBSAMPLE) + (int)floorf((float)y / TF_SUBSAMPLE) * a.W];
    const float* M = MODE == 2 ? st->M_render : st->M_ray;
    float pt[3];
    const float w = ray_march<MODE == 1>(a, M, x, y, vf, pt);
    if (MODE == 2) {
        // renderImage: lightSource = -Vector3f(pose.getColumn(2)) (VisualisationEngine_CUDA.cu:243)
        unsigned char v = 0;
        if (w > 0) v = grey_pixel(a.s, pt, -M[8], -M[9], -M[10], &vtab[threadIdx.x * VTAB_STRIDE]);
        a.grey[x + y * a.W] = make_uchar4(v, v, v, v);
    } else {
        a.out[x + y * a.W] = make_float4(pt[0], pt[1], pt[2], w);
    }
}

// the early exits every raycast workgroup takes first (uniform): the frame's renderImage (MODE 2)
// reads the snapshot render_snapshot took (tf_internal.h); the others run on tracked frames only
template <int MODE>
__device__ __forceinline__ bool raycast_go(const TfDevState* __restrict__ st)
{
    return MODE == 2 ? st->render_go != 0 : !(st->abort || st->mode == 0);
}

// Distinct instantiations also give each use its own kernel name in rocprof.
template <int MODE>
__global__ void __launch_bounds__(256)
k_raycast(RayArgs a, const TfDevState* __restrict__ st, int tiles_x, int n_tiles)
{
    if (!raycast_go<MODE>(st)) return;
    const int tile = xcd_tile(blockIdx.x, n_tiles);            // grid padded to a multiple of 8
    if (tile < 0) return;
    raycast_tile<MODE>(a, st, tile, tiles_x, nullptr);
}

static void ray_args(tf_ctx* c, RayArgs& a)
{
    a.s.hash = c->hash; a.s.vba = c->vba_guard; a.s.grid = c->bgrid; a.s.mask = (unsigned)(c->p.n_buckets - 1); a.s.n_buckets = c->p.n_buckets;
    a.range = (const float2*)c->range; a.out = (float4*)c->raycast;
    a.visType = nullptr;
    a.grey = nullptr;
    a.W = c->W; a.H = c->H;
    a.invfx = 1.0f / c->p.fx; a.invfy = 1.0f / c->p.fy; a.ncx = -c->p.cx; a.ncy = -c->p.cy;
    a.oneOverVoxelSize = 1.0f / c->p.voxelSize; a.mu = c->p.mu;
}

static hipError_t launch_ray(tf_ctx* c, const RayArgs& a, int mode)
{
    const int tx = (c->W + 15) / 16, ty = (c->H + 15) / 16, n = tx * ty;
    const dim3 grid((n + 7) / 8 * 8);
    if (mode == 0) hipLaunchKernelGGL(k_raycast<0>, grid, dim3(256), 0, c->stream, a, c->st, tx, n);
    else hipLaunchKernelGGL(k_raycast<1>, grid, dim3(256), 0, c->stream, a, c->st, tx, n);
    return hipGetLastError();
}

hipError_t tfk_raycast(tf_ctx* c, int update_visible)
{
    RayArgs a;
    ray_args(c, a);
    a.visType = update_visible ? c->visType : nullptr;
    return launch_ray(c, a, update_visible ? 1 : 0);
}

// the renderImage snapshot outside a frame (measurement: tf_time_stage of the raycast pair)
__global__ void k_render_snapshot(TfDevState* st, const float2* range, float2* snap, int W, int H)
{
    render_snapshot(st, range, snap, W, H);
}

hipError_t tfk_render_snapshot(tf_ctx* c)
{
    hipLaunchKernelGGL(k_render_snapshot, dim3(64), dim3(256), 0, c->stream, c->st, (const float2*)c->range,
                       (float2*)c->range_render, c->W, c->H);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// RenderImage_common's pixel stages (VisualisationEngine_CUDA.cu:254-290) on the raycast image:
// the five IVisualisationEngine::RenderImageType values (VisualisationEngine.hpp:15-22).
// ---------------------------------------------------------------------------------------
// baseCol / interpolateCol (VisualisationEngine_Shared.hpp:278-288)
__device__ __forceinline__ float base_col(float val)
{
    if (val <= -0.75f) return 0.0f;
    else if (val <= -0.25f) return (val - -0.75f) * (1.0f - 0.0f) / (-0.25f - -0.75f) + 0.0f;
    else if (val <= 0.25f) return 1.0f;
    else if (val <= 0.75f) return (val - 0.25f) * (0.0f - 1.0f) / (0.75f - 0.25f) + 1.0f;
    else return 0.0f;
}

// Vector4f::toUChar: CLAMP((int)ROUND(v), 0, 255) (Vector.hpp:398-404, MathUtils.hpp:16-20)
__device__ __forceinline__ unsigned char round_u8(float v)
{
    const int i = tf_round(v);
    return (unsigned char)(i < 0 ? 0 : (i > 255 ? 255 : i));
}

// computeNormalAndAngle<useSmoothing = true, flipNormals = false> on the raycast image
// (VisualisationEngine_Shared.hpp:205-270): +-2 neighbours, +-1 where those are missing or
// the difference is longer than 15 cm
__device__ __forceinline__ bool image_normal_angle(const float4* ray, int W, int H, int x, int y, float voxelSize,
                                                   float lx, float ly, float lz, float* angle)
{
    if (y <= 2 || y >= H - 3 || x <= 2 || x >= W - 3) return false;
    float4 xp = ray[(x + 2) + y * W], yp = ray[x + (y + 2) * W];
    float4 xm = ray[(x - 2) + y * W], ym = ray[x + (y - 2) * W];
    float dx0 = 0.f, dx1 = 0.f, dx2 = 0.f, dy0 = 0.f, dy1 = 0.f, dy2 = 0.f;
    bool plus1 = false;
    if (xp.w <= 0 || yp.w <= 0 || xm.w <= 0 || ym.w <= 0) plus1 = true;
    else {
        dx0 = xp.x - xm.x; dx1 = xp.y - xm.y; dx2 = xp.z - xm.z;
        dy0 = yp.x - ym.x; dy1 = yp.y - ym.y; dy2 = yp.z - ym.z;
        const float lx2 = dx0 * dx0 + dx1 * dx1 + dx2 * dx2, ly2 = dy0 * dy0 + dy1 * dy1 + dy2 * dy2;
        const float length_diff = (lx2 < ly2) ? ly2 : lx2;                      // MAX
        if (length_diff * voxelSize * voxelSize > (0.15f * 0.15f)) plus1 = true;
    }
    if (plus1) {
        xp = ray[(x + 1) + y * W]; yp = ray[x + (y + 1) * W];
        xm = ray[(x - 1) + y * W]; ym = ray[x + (y - 1) * W];
        dx0 = xp.x - xm.x; dx1 = xp.y - xm.y; dx2 = xp.z - xm.z;
        dy0 = yp.x - ym.x; dy1 = yp.y - ym.y; dy2 = yp.z - ym.z;
        if (xp.w <= 0 || yp.w <= 0 || xm.w <= 0 || ym.w <= 0) return false;
    }
    float n0 = -(dx1 * dy2 - dx2 * dy1), n1 = -(dx2 * dy0 - dx0 * dy2), n2 = -(dx0 * dy1 - dx1 * dy0);
    const float ns = 1.0f / sqrtf(n0 * n0 + n1 * n1 + n2 * n2);
    n0 *= ns; n1 *= ns; n2 *= ns;
    *angle = n0 * lx + n1 * ly + n2 * lz;
    return *angle > 0.0f;
}

// readFromSDF_color4u_interpolated (RepresentationAccess.hpp:260-294) + drawPixelColour
// (VisualisationEngine_Shared.hpp:312-322): the eight corners' colour words from the colour plane
// (same block offsets as the Voxel_s plane; a missing block reads its zero guard block), weights
// and sums in the reference's order, / 255 then (uchar)(v * 255), alpha 255
__device__ __forceinline__ uchar4 colour_at(const SceneView& s, const unsigned* rgb_guard, const float* pt)
{
    Corners q;
    corners_lookup(s, pt, q);
    const int lx[2] = { lin_x(q.fx), lin_x(q.fx + 1) }, ly[2] = { lin_y(q.fy), lin_y(q.fy + 1) };
    const int lz[2] = { lin_zg(q.fz), lin_zg(q.fz + 1) };
    unsigned cw[8];
#pragma unroll
    for (int c = 0; c < 8; ++c)
        cw[c] = ld_off<unsigned>(rgb_guard, (unsigned)(q.voff[c] + lx[c & 1] + ly[(c >> 1) & 1] + lz[c >> 2]) * 4u);
    float ret[3] = { 0.0f, 0.0f, 0.0f };
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        const float w = ((c & 1) ? q.cx : (1.0f - q.cx)) * ((c & 2) ? q.cy : (1.0f - q.cy)) * ((c & 4) ? q.cz : (1.0f - q.cz));
#pragma unroll
        for (int k = 0; k < 3; ++k) ret[k] += w * (float)((cw[c] >> (8 * k)) & 0xffu);
    }
    return make_uchar4((unsigned char)((ret[0] / 255.0f) * 255.0f), (unsigned char)((ret[1] / 255.0f) * 255.0f),
                       (unsigned char)((ret[2] / 255.0f) * 255.0f), 255);
}

template <int TYPE>
__global__ void __launch_bounds__(256)
k_render_type(SceneView s, const float4* __restrict__ ray, int W, int H, float voxelSize,
              const TfDevState* __restrict__ st, uchar4* __restrict__ out, const unsigned* __restrict__ rgb_guard)
{
    __shared__ int vtab[256 * VTAB_STRIDE];
    if (st->abort || st->mode == 0) return;          // ICP failed, or frame 0 (no rendering)
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= W * H) return;
    const int x = i % W, y = i / W;
    // lightSource = -Vector3f(pose.getColumn(2)) (VisualisationEngine_CUDA.cu:243)
    const float lx = -st->M_ray[8], ly = -st->M_ray[9], lz = -st->M_ray[10];
    const float4 p = ray[i];
    bool found = p.w > 0;
    float nn[3], angle = 0.f;
    if (TYPE == TF_RENDER_COLOUR_FROM_VOLUME) {                      // renderColour_device / processPixelColour
        const float pt[3] = { p.x, p.y, p.z };
        out[i] = found ? colour_at(s, rgb_guard, pt) : make_uchar4(0, 0, 0, 0);
        return;
    }
    if (TYPE == TF_RENDER_SHADED_GREYSCALE_IMAGENORMALS) {           // processPixelGrey_ImageNormals<true,false>
        if (found) found = image_normal_angle(ray, W, H, x, y, voxelSize, lx, ly, lz, &angle);
        const unsigned char v = found ? grey_of(angle) : (unsigned char)0;
        out[i] = make_uchar4(v, v, v, v);
        return;
    }
    if (found) {
        const float pt[3] = { p.x, p.y, p.z };
        found = sdf_normal_angle(s, pt, lx, ly, lz, nn, &angle, &vtab[threadIdx.x * VTAB_STRIDE]);
    }
    if (TYPE == TF_RENDER_COLOUR_FROM_NORMAL) {                      // processPixelNormal / drawPixelNormal
        if (found) {                                                 // r, g, b; alpha is left as it was (:305-310)
            uchar4 o = out[i];
            o.x = (unsigned char)((0.3f + (-nn[0] + 1.0f) * 0.35f) * 255.0f);
            o.y = (unsigned char)((0.3f + (-nn[1] + 1.0f) * 0.35f) * 255.0f);
            o.z = (unsigned char)((0.3f + (-nn[2] + 1.0f) * 0.35f) * 255.0f);
            out[i] = o;
        } else {
            out[i] = make_uchar4(0, 0, 0, 0);
        }
    } else if (TYPE == TF_RENDER_COLOUR_FROM_CONFIDENCE) {           // processPixelConfidence (:290-303)
        if (found) {
            const float conf = p.w - 1.0f;
            const float mn = (100.f < conf) ? 100.f : conf;          // CLAMP(conf, 0, 100.f)
            const float cn = ((0 < mn) ? mn : 0) / 100.0f;
            const float r = (float)(unsigned char)(base_col(cn) * 255.0f);
            const float g = (float)(unsigned char)(base_col(cn - 0.5f) * 255.0f);
            const float b = (float)(unsigned char)(base_col(cn + 0.5f) * 255.0f);
            const float sc = 0.8f * angle + 0.2f;
            out[i] = make_uchar4(round_u8(sc * r), round_u8(sc * g), round_u8(sc * b), round_u8(sc * 255.0f));
        } else {
            out[i] = make_uchar4(0, 0, 0, 0);
        }
    } else {       // RENDER_SHADED_GREYSCALE (RENDER_COLOUR_FROM_VOLUME on Voxel_s is sent here, :251-252)
        const unsigned char v = found ? grey_of(angle) : (unsigned char)0;
        out[i] = make_uchar4(v, v, v, v);
    }
}

hipError_t tfk_render_type(tf_ctx* c, int type)
{
    SceneView s; s.hash = c->hash; s.vba = c->vba_guard; s.grid = c->bgrid; s.mask = (unsigned)(c->p.n_buckets - 1); s.n_buckets = c->p.n_buckets;
    const int n = c->W * c->H;
    const dim3 g((n + 255) / 256), b(256);
    const float4* ray = (const float4*)c->raycast;
    const float vs = c->p.voxelSize;
    const unsigned* cg = c->vba_rgb_guard;
    // RENDER_COLOUR_FROM_VOLUME without colour information: greyscale (VisualisationEngine_CUDA.cu:251-252)
    if (type == TF_RENDER_COLOUR_FROM_VOLUME && !c->p.voxel_rgb) type = TF_RENDER_SHADED_GREYSCALE;
    switch (type) {
    case TF_RENDER_COLOUR_FROM_VOLUME:
        hipLaunchKernelGGL(k_render_type<TF_RENDER_COLOUR_FROM_VOLUME>, g, b, 0, c->stream, s, ray, c->W, c->H, vs, c->st, c->grey, cg); break;
    case TF_RENDER_SHADED_GREYSCALE_IMAGENORMALS:
        hipLaunchKernelGGL(k_render_type<TF_RENDER_SHADED_GREYSCALE_IMAGENORMALS>, g, b, 0, c->stream, s, ray, c->W, c->H, vs, c->st, c->grey, cg); break;
    case TF_RENDER_COLOUR_FROM_NORMAL:
        hipLaunchKernelGGL(k_render_type<TF_RENDER_COLOUR_FROM_NORMAL>, g, b, 0, c->stream, s, ray, c->W, c->H, vs, c->st, c->grey, cg); break;
    case TF_RENDER_COLOUR_FROM_CONFIDENCE:
        hipLaunchKernelGGL(k_render_type<TF_RENDER_COLOUR_FROM_CONFIDENCE>, g, b, 0, c->stream, s, ray, c->W, c->H, vs, c->st, c->grey, cg); break;
    default:
        hipLaunchKernelGGL(k_render_type<TF_RENDER_SHADED_GREYSCALE>, g, b, 0, c->stream, s, ray, c->W, c->H, vs, c->st, c->grey, cg); break;
    }
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

// processPixelICP of pixel (x, y) from it and its four neighbours (already loaded)
__device__ __forceinline__ void icp_pixel(const IcpMapArgs& a, float lx, float ly, float lz, int x, int y,
                                          const float4& p, const float4& xp, const float4& xm, const float4& yp,
                                          const float4& ym, float4* po, float4* no)
{
    const int W = a.W, H = a.H;
    bool found = p.w > 0.0f;
    float n0 = 0, n1 = 0, n2 = 0;
    if (found) {
        if (y <= 1 || y >= H - 2 || x <= 1 || x >= W - 2) found = false;
        else {
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

// One workgroup per 32x32 tile of level 0: thread t owns the 2x2 level-0 quad under level-1
// pixel (t & 15, t >> 4) of the tile's 16x16 level-1 tile, so it computes four processPixelICP
// results and their resizePointsNormals average directly; level 2 (8x8 per tile) is averaged
// from the level-1 values staged in LDS.  Every level-0 pixel is evaluated once (levels 1/2
// are computed from the level-0 results, exactly as the reference's resize of the level-0
// maps).
__device__ __forceinline__ void icp_maps_block(const IcpMapArgs& a, const TfDevState* __restrict__ st, int bx, int by)
{
    if (st->abort || st->mode == 0) return;          // ICP failed, or frame 0 (no rendering)
    __shared__ float4 v1s[16][17], n1s[16][17];
    const int lx1 = threadIdx.x & 15, ly1 = threadIdx.x >> 4;
    const int x1 = bx * 16 + lx1, y1 = by * 16 + ly1;
    const int W = a.W, H = a.H, w1 = W >> 1, h1 = H >> 1, w2 = W >> 2, h2 = H >> 2;
    const float lx = -st->M_ray[8], ly = -st->M_ray[9], lz = -st->M_ray[10];
    float4 v[4], n[4];
    {
        // the 4x4 neighbourhood of the quad minus its corners, twelve loads in flight together
        // (clamped into the image: a clamped sample is only ever needed where processPixelICP's
        // border test has already failed)
        const int xb = 2 * x1, yb = 2 * y1;
        float4 nb[4][4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                if ((j == 0 || j == 3) && (i == 0 || i == 3)) continue;
                const int xx = min(max(xb - 1 + i, 0), W - 1), yy = min(max(yb - 1 + j, 0), H - 1);
                nb[j][i] = a.ray[yy * W + xx];
            }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int qx = q & 1, qy = q >> 1;
            const int x = xb + qx, y = yb + qy;
            if (x < W && y < H) {
                icp_pixel(a, lx, ly, lz, x, y, nb[1 + qy][1 + qx], nb[1 + qy][2 + qx], nb[1 + qy][qx],
                          nb[2 + qy][1 + qx], nb[qy][1 + qx], &v[q], &n[q]);
                a.pts[0][y * W + x] = v[q];
                a.nrm[0][y * W + x] = n[q];
            }
        }
    }
    if (x1 < w1 && y1 < h1) {
        float4 po, no;
        resize4(v, n, &po, &no);
        a.pts[1][y1 * w1 + x1] = po;
        a.nrm[1][y1 * w1 + x1] = no;
        v1s[ly1][lx1] = po;
        n1s[ly1][lx1] = no;
    }
    __syncthreads();
    if (threadIdx.x < 64) {
        const int lx2 = threadIdx.x & 7, ly2 = threadIdx.x >> 3;
        const int x2 = bx * 8 + lx2, y2 = by * 8 + ly2;
        if (x2 < w2 && y2 < h2) {
            float4 vv[4], nn[4], po, no;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                vv[q] = v1s[2 * ly2 + (q >> 1)][2 * lx2 + (q & 1)];
                nn[q] = n1s[2 * ly2 + (q >> 1)][2 * lx2 + (q & 1)];
            }
            resize4(vv, nn, &po, &no);
            a.pts[2][y2 * w2 + x2] = po;
            a.nrm[2][y2 * w2 + x2] = no;
        }
    }
}

__global__ void __launch_bounds__(256)
k_icp_maps(IcpMapArgs a, const TfDevState* __restrict__ st)
{
    icp_maps_block(a, st, blockIdx.x, blockIdx.y);
}

// CreateICPMaps' tiles, then TF_END_BLOCKS workgroups of the frame end (bookkeeping; the
// ResetScene of topfu.cpp:263-264 when ICP failed).  The two share nothing: the maps pass
// reads the raycast and writes the previous-frame maps, and does nothing on a failed frame;
// the frame end writes the pose / counters only, and the scene only on a failed frame.
// n_pyr > 0 (per-call frames, process_frame_early): the next frame's dists / pyramid / normals
// pass in the grid's last workgroups -- it writes only the current maps, the level 1-2 depths and
// dists, which nothing of this frame reads any more, and its level-0 depth came from the
// bilateral pass in this frame's k_raycast_pair.
// Longest-first dispatch order of the next frame's raycast tiles (k_raycast_pair's frame path).
// The pair kernel's run time is its longest workgroups' -- tiles whose rays graze a surface
// inside its truncation band take ~45 us against a median ~20 us -- and a launch holds more
// workgroups than the chip does at once, so a long tile dispatched late ends late
// (tools/pair_timeline.py).  Tile costs are this frame's workgroup times; the camera moves little
// per frame.  Workgroup b of a half runs on XCD b % 8 as its (b / 8)-th tile: each XCD keeps its
// band of consecutive image tiles (xcd_tile: the L2 locality of the voxels its rays read), sorted
// by cost, longest first.  Only the schedule changes: every tile computes the same values.
struct TileSortArgs {
    const unsigned* cost;    // [2][n]
    int* order;              // [2][nb]
    int n, nb;               // tiles, dispatch slots per half (tf_ctx::tile_slots)
    int tx, ty, rows;        // tiles per row / column, tf_ctx::tile_rows
};
// one XCD region of one half: rank sort (each key's rank = the keys above it; keys are distinct,
// the tile index rides in the low bits), a few hundred LDS broadcast reads per thread
__device__ __forceinline__ void tile_sort_block(const TileSortArgs& a, int s, unsigned* keys)
{
    const int h = s >> 3, x = s & 7, per = a.nb >> 3;
    const int cnt = tf_tile_count(x, a.n, a.tx, a.ty, per, a.rows);
    for (int i = threadIdx.x; i < cnt; i += 256)
        keys[i] = (min(a.cost[h * a.n + tf_tile_of(x, i, a.n, a.tx, a.ty, per, a.rows)], 0xfffffu) << 12) | (unsigned)i;
    __syncthreads();
    for (int i = threadIdx.x; i < cnt; i += 256) {
        const unsigned ki = keys[i];
        int rank = 0;
        for (int j = 0; j < cnt; ++j) rank += keys[j] > ki ? 1 : 0;
        a.order[h * a.nb + rank * 8 + x] = tf_tile_of(x, i, a.n, a.tx, a.ty, per, a.rows);   // longest first
    }
    for (int k = cnt + threadIdx.x; k < per; k += 256) a.order[h * a.nb + k * 8 + x] = -1;
}

// the sort's 16 workgroups first (done long before the maps pass), then CreateICPMaps' tiles, the
// frame end and the per-call lookahead
__global__ void __launch_bounds__(256)
k_icp_maps_end(IcpMapArgs a, ResetArgs r, int gx, int nmaps, PyrArgs pyr, int pyr_gx, int n_sort, TileSortArgs ts)
{
    __shared__ union { PnLds pn; unsigned keys[TF_LJF_MAX]; } L;
    const int b = (int)blockIdx.x - n_sort;
    if (b < 0) tile_sort_block(ts, (int)blockIdx.x, L.keys);
    else if (b < nmaps) icp_maps_block(a, r.st, b % gx, b / gx);
    else if (b < nmaps + TF_END_BLOCKS) reset_scene_block(r, b - nmaps, TF_END_BLOCKS);
    else pyr_normals_block<256>(pyr, (b - nmaps - TF_END_BLOCKS) % pyr_gx, (b - nmaps - TF_END_BLOCKS) / pyr_gx, L.pn);
}

__global__ void __launch_bounds__(256) k_tile_sort(TileSortArgs ts)
{
    __shared__ unsigned keys[TF_LJF_MAX];
    tile_sort_block(ts, (int)blockIdx.x, keys);
}

// the XCD-swizzled order (xcd_tile) and zero costs: a new context's first frames
hipError_t tfk_tile_order_init(tf_ctx* c)
{
    const int tx = (c->W + 15) / 16, ty = (c->H + 15) / 16, n = tx * ty, nb = c->tile_slots;
    int* o = (int*)malloc(sizeof(int) * 2 * (size_t)nb);
    if (!o) return hipErrorOutOfMemory;
    const int per = nb / 8;
    for (int b = 0; b < nb; ++b) {
        const int x = b % 8, i = b / 8;
        o[b] = o[nb + b] = i < tf_tile_count(x, n, tx, ty, per, c->tile_rows) ? tf_tile_of(x, i, n, tx, ty, per, c->tile_rows) : -1;
    }
    hipError_t e = hipMemcpy(c->tile_order, o, sizeof(int) * 2 * (size_t)nb, hipMemcpyHostToDevice);
    free(o);
    if (e == hipSuccess) e = hipMemsetAsync(c->tile_cost, 0, sizeof(unsigned) * 2 * (size_t)n, c->stream);
    return e;
}

hipError_t tfk_icp_maps(tf_ctx* c)
{
    IcpMapArgs a;
    a.ray = (const float4*)c->raycast;
    for (int l = 0; l < TF_LEVELS; ++l) { a.pts[l] = c->prev_pts[l]; a.nrm[l] = c->prev_nrm[l]; }
    a.W = c->W; a.H = c->H; a.voxelSize = c->p.voxelSize;
    hipLaunchKernelGGL(k_icp_maps, dim3((c->W + 31) / 32, (c->H + 31) / 32), dim3(256), 0, c->stream, a, c->st);
    return hipGetLastError();
}

hipError_t tfk_icp_maps_end(tf_ctx* c, int slot, TfAhead pyr, size_t pitch)
{
    IcpMapArgs a;
    a.ray = (const float4*)c->raycast;
    for (int l = 0; l < TF_LEVELS; ++l) { a.pts[l] = c->prev_pts[l]; a.nrm[l] = c->prev_nrm[l]; }
    a.W = c->W; a.H = c->H; a.voxelSize = c->p.voxelSize;
    ResetArgs r;
    tf_reset_args(c, &r, 1, slot, 1);
    const int gx = (c->W + 31) / 32, nmaps = gx * ((c->H + 31) / 32);
    PyrArgs pp = PyrArgs{};
    int n_pyr = 0, pyr_gx = 1;
    if (pyr.src) {
        BilArgs bx;
        const hipError_t e = tf_pre_args(c, pyr.src, pitch, 1, pyr.d0, &bx, &pp);
        if (e != hipSuccess) return e;
        pyr_gx = tf_div_up(c->W, PN_T0);
        n_pyr = pyr_gx * tf_div_up(c->H, PN_T0);
    }
    TileSortArgs ts = TileSortArgs{};
    int n_sort = 0;
    if (c->tile_ljf) {                   // 2 halves x 8 XCD regions
        ts.cost = c->tile_cost; ts.order = c->tile_order;
        ts.tx = (c->W + 15) / 16; ts.ty = (c->H + 15) / 16; ts.n = ts.tx * ts.ty;
        ts.nb = c->tile_slots; ts.rows = c->tile_rows;
        n_sort = 16;
    }
    tf_launch(c, k_icp_maps_end, dim3(n_sort + nmaps + TF_END_BLOCKS + n_pyr), dim3(256), 0, a, r, gx, nmaps, pp, pyr_gx,
              n_sort, ts);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// CreateExpectedDepths
// ---------------------------------------------------------------------------------------
#include "tf_ed.h"

__global__ void __launch_bounds__(256)
k_ed_project(EdArgs a, const TfDevState* __restrict__ st)
{
    ed_project_block(a, st, blockIdx.x, gridDim.x);
}

// fillBlocks_device (VisualisationHelper.cu:105-121): per-pixel min/max of the block z-ranges.
// The tile total is the sum of the chunk totals; past MAX_RENDERING_BLOCKS, blocks whose tiles do
// not fit are dropped in visible-list order (the serial semantics of the reference's atomicAdd
// offsets).  Two paths, chosen on the device from the visible count:
//  - n <= a.lds_max_n: workgroup r owns image row r for r < rr + ED_XROWS (the /8 rows, then
//    the first rows below them, where boxes clamped to the full-resolution H-1 spill).  It scans
//    every visible box (one 16-byte record each), reduces its row's pixels in LDS over the full
//    width (min/max as ints: the z values are positive floats) and writes the row with plain
//    stores: the /8 columns always, the columns past them up to the last one a box touched.
//    Rows further down (boxes of blocks close to the camera) take device-scope atomics, spread
//    over the workgroups by entry index; boxes wider than ED_WIDE are queued, one wave each.
//    Each row records the extent it wrote outside the /8 region for the next projection pass.
//  - n > a.lds_max_n: one wave per block, its lanes over the block's pixel box, with
//    device-scope atomics (the projection pass initialised the /8 region).
#ifndef ED_WIDE
#define ED_WIDE 4         // box columns in a row above which a wave fills it (queued)
#endif
#define ED_QUEUE 256      // queued segments per workgroup (beyond: filled by their thread)
#define ED_THREADS 256    // k_ed_fill workgroup
#define ED_INFLIGHT 4     // binned boxes in flight per thread (1024 per workgroup pass)
// a segment: rows y0 .. y1, columns [x0, x1], z range as ints; lds: the workgroup's LDS row,
// else the range image with device-scope atomics
struct EdSeg { int y0, y1, x0, x1, zmin, zmax, lds; };
__device__ __forceinline__ void ed_fill_global(const EdArgs& a, int y0, int y1, int x0, int x1, int zmin, int zmax,
                                               int t, int nt)
{
    const int w = x1 - x0 + 1, nrow = y1 - y0 + 1;
    for (int k = t; k < nrow * w; k += nt) {
        const int r = k / w;
        int* px = (int*)(a.range + (x0 + (k - r * w)) + (y0 + r) * a.W);
        atomicMin(px, zmin);
        atomicMax(px + 1, zmax);
    }
}

// k_ed_fill's workgroup `row` of `nfill` (its own launch, or the leading workgroups of
// k_raycast_pair in the frame path); LW: LDS columns (wider rows take device atomics past them).
// own_zero: the workgroup empties its two bins at the end (else the frame end does, after the
// raycast's ICP tiles have read them too).  With `done` set, the atomic path counts its finished
// workgroups there (release) for the ICP tiles that wait on the range image.
template <int LW>
struct EdLds {
    int lmin[LW], lmax[LW];
    unsigned cpre[ED_LDS_MAX_N / ED_CHUNK];      // tiles of chunks before chunk c (nchunks <= 64)
    EdSeg q[ED_QUEUE];
    int nq, sxy[3];
    unsigned total_s;
    unsigned red[ED_THREADS / 64];
};

template <int LW>
__device__ __forceinline__ void ed_fill_block(const EdArgs& a, TfDevState* __restrict__ st, int row, int nfill,
                                              EdLds<LW>& L, bool own_zero)
{
    // Everything this reads was written by the previous launch, on other XCDs: the state
    // words, the chunk totals and this row's two bin counts are requested together (one round
    // trip); then the binned boxes (the second).
    const int nrow = a.nrows;
    const unsigned cv = threadIdx.x < 64 && (int)threadIdx.x < a.nchunk_max ? (unsigned)a.chunk[threadIdx.x] : 0u;
    const int cnt_row = a.bin_cnt[row], cnt_below = a.bin_cnt[nrow + row];
    if (st->abort || st->mode == 0) return;          // ICP failed, or frame 0 (no rendering)
    const int n = st->noVisibleEntries;
    const int nchunks = (n + ED_CHUNK - 1) / ED_CHUNK;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int rc = a.rc, rr = a.rr;
    if (n > a.lds_max_n) {
        // ---- large lists: one wave per block, its lanes over the block's pixel box, device atomics
        unsigned* red = L.red;
        unsigned part = 0;
        for (int c = threadIdx.x; c < nchunks; c += ED_THREADS) part += (unsigned)a.chunk[c];
        for (int d = 32; d > 0; d >>= 1) part += __shfl_xor(part, d, 64);
        if (lane == 0) red[wv] = part;
        __syncthreads();
        unsigned total = 0;
        for (int w = 0; w < ED_THREADS / 64; ++w) total += red[w];
        const bool capped = total > a.cap;
        if (row == 0 && threadIdx.x == 0) st->noTotalBlocks = (int)(capped ? a.cap : total);
        unsigned cprefix = 0;                    // tiles of chunks [0, cdone)
        int cdone = 0;
        const int nw = nfill * (ED_THREADS / 64);
        for (int i = row * (ED_THREADS / 64) + wv; i < n; i += nw) {
            const uint4 r = a.rec[i];
            if (r.x == 0xffffffffu) continue;
            if (capped) {
                const int ch = i / ED_CHUNK;     // i grows monotonically: extend the chunk prefix
                while (cdone < ch) cprefix += (unsigned)a.chunk[cdone++];
                const unsigned need = (unsigned)a.tiles[i], off = cprefix + (unsigned)a.off[i];
                if (!(need && off + need <= a.cap)) continue;
            }
            ed_fill_global(a, (int)(r.x >> 16), (int)(r.y >> 16), (int)(r.x & 0xffff), (int)(r.y & 0xffff),
                           (int)r.z, (int)r.w, lane, 64);
        }
        // the next projection pass clears the whole buffer (every pixel may have been written)
        if (threadIdx.x == 0) a.spill[row] = row == 0 ? make_int2(a.W, a.H) : make_int2(0, 0);
        if (a.done) {                            // the range image is final once every row has counted
            __syncthreads();
            if (threadIdx.x == 0) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                atomicAdd(a.done, 1u);
            }
        }
        return;
    }
    // ---- one image row per workgroup, reduced in LDS over the full width ----
    const int lw = a.W < LW ? a.W : LW;         // LDS columns
    int* lmin = L.lmin;
    int* lmax = L.lmax;
    unsigned* cpre = L.cpre;
    EdSeg* q = L.q;
    int& nq = L.nq;
    int* sxy = L.sxy;
    unsigned& total_s = L.total_s;
    for (int x = threadIdx.x; x < lw; x += ED_THREADS) { lmin[x] = __float_as_int(TF_FAR_AWAY); lmax[x] = __float_as_int(TF_VERY_CLOSE); }
    if (threadIdx.x < 64) {                      // wave 0: chunk totals -> tile total + chunk prefix
        const unsigned v = (int)threadIdx.x < nchunks ? cv : 0u;
        unsigned incl = v;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const unsigned u = __shfl_up(incl, d, 64);
            if ((int)threadIdx.x >= d) incl += u;
        }
        cpre[threadIdx.x] = incl - v;
        if (threadIdx.x == 63) { total_s = incl; nq = 0; sxy[0] = 0; sxy[1] = 0; sxy[2] = 0; }
    }
    __syncthreads();
    const unsigned total = total_s;
    const bool capped = total > a.cap;
    if (row == 0 && threadIdx.x == 0) st->noTotalBlocks = (int)(capped ? a.cap : total);
    int xt = -1;                                 // last LDS column this thread touched
    int sx = 0, sy = 0;                          // extent of this thread's device-atomic writes
    // this row's boxes (bin row), then its share of the boxes reaching below the LDS rows
    // (bin nrow + row); the projection pass binned them (ed_project_block)
    for (int part = 0; part < 2; ++part) {
        const int m = part ? cnt_below : cnt_row;
        const uint4* bin = a.bins + (size_t)(part ? nrow + row : row) * a.lds_max_n;
        for (int k0 = threadIdx.x; k0 < m; k0 += ED_INFLIGHT * ED_THREADS) {
            uint4 e[ED_INFLIGHT];
#pragma unroll
            for (int k = 0; k < ED_INFLIGHT; ++k) e[k] = bin[k0 + k * ED_THREADS < m ? k0 + k * ED_THREADS : k0];
#pragma unroll
            for (int k = 0; k < ED_INFLIGHT; ++k) {
                if (k0 + k * ED_THREADS >= m) continue;
                const uint4 r = e[k];
                const int bx = (int)(r.x & 0xfffu), by = (int)((r.x >> 12) & 0xfffu);
                const int bz = (int)(r.y & 0xfffu), bw = (int)((r.y >> 12) & 0xfffu);
                const int i = (int)((r.x >> 24) | ((r.y >> 24) << 8));
                if (capped) {
                    const unsigned need = (unsigned)a.tiles[i], off = cpre[i / ED_CHUNK] + (unsigned)a.off[i];
                    if (!(need && off + need <= a.cap)) continue;
                }
                const int zmin = (int)r.z, zmax = (int)r.w;
                if (!part) {                     // by <= row <= bw
                    const int x1 = bz < lw - 1 ? bz : lw - 1;
                    if (x1 >= bx) {
                        xt = max(xt, x1);
                        const int slot = x1 - bx + 1 > ED_WIDE ? atomicAdd(&nq, 1) : ED_QUEUE;
                        if (slot < ED_QUEUE) q[slot] = EdSeg{row, row, bx, x1, zmin, zmax, 1};
                        else for (int x = bx; x <= x1; ++x) { atomicMin(&lmin[x], zmin); atomicMax(&lmax[x], zmax); }
                    }
                    if (bz >= lw) {              // (images wider than ED_MAX_W)
                        sx = max(sx, bz + 1); sy = max(sy, row + 1);
                        ed_fill_global(a, row, row, bx > lw ? bx : lw, bz, zmin, zmax, 0, 1);
                    }
                } else {                         // rows past the LDS rows: device atomics
                    const int y0 = by > nrow ? by : nrow;
                    sx = max(sx, bz + 1); sy = max(sy, bw + 1);
                    const int slot = (bz - bx + 1) * (bw - y0 + 1) > 64 ? atomicAdd(&nq, 1) : ED_QUEUE;
                    if (slot < ED_QUEUE) q[slot] = EdSeg{y0, bw, bx, bz, zmin, zmax, 0};
                    else ed_fill_global(a, y0, bw, bx, bz, zmin, zmax, 0, 1);
                }
            }
        }
    }
    if (xt >= 0) atomicMax(&sxy[2], xt);
    if (sx) atomicMax(&sxy[0], sx);
    if (sy) atomicMax(&sxy[1], sy);
    __syncthreads();
    const int nseg = nq < ED_QUEUE ? nq : ED_QUEUE;
    for (int j = wv; j < nseg; j += ED_THREADS / 64) {   // queued segments: one wave each, lanes over columns
        const EdSeg g = q[j];
        if (g.lds) {
            for (int x = g.x0 + lane; x <= g.x1; x += 64) { atomicMin(&lmin[x], g.zmin); atomicMax(&lmax[x], g.zmax); }
        } else {
            ed_fill_global(a, g.y0, g.y1, g.x0, g.x1, g.zmin, g.zmax, lane, 64);
        }
    }
    __syncthreads();
    // the row: the /8 columns always (rows < rr), and up to the last column a box touched
    const int xlast = sxy[2];
    const int xend = max(row < rr ? rc : 0, xlast + 1);
    float2* out = a.range + (size_t)row * a.W;
    for (int x = threadIdx.x; x < xend; x += ED_THREADS) out[x] = make_float2(__int_as_float(lmin[x]), __int_as_float(lmax[x]));
    if (threadIdx.x == 0) {
        int2 e = make_int2(sxy[0], sxy[1]);      // outside the /8 region: this row past rc, or all of it
        if (xend > (row < rr ? rc : 0)) { e.x = max(e.x, xend); e.y = max(e.y, row + 1); }
        a.spill[row] = e;
        if (own_zero) {                          // the bins are consumed (every thread read the counts)
            a.bin_cnt[row] = 0;
            a.bin_cnt[nrow + row] = 0;
        }
    }
}

__global__ void __launch_bounds__(ED_THREADS)
k_ed_fill(EdArgs a, TfDevState* __restrict__ st)
{
    __shared__ EdLds<ED_MAX_W> L;
    ed_fill_block<ED_MAX_W>(a, st, blockIdx.x, gridDim.x, L, !a.keep_bins);
}

hipError_t ed_spill_all(tf_ctx* c)
{
    hipError_t e = hipMemsetAsync(c->edSpill, 0, sizeof(int2) * ed_nrows(c->H), c->stream);
    const int2 all = make_int2(c->W, c->H);
    if (e == hipSuccess) e = hipMemcpyAsync(c->edSpill, &all, sizeof(int2), hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    return e;
}

void tf_ed_args(tf_ctx* c, EdArgs* out)
{
    EdArgs& a = *out;
    a.hash = c->hash; a.visibleIds = c->visibleIds; a.range = (float2*)c->range;
    a.rec = c->blockRec; a.tiles = c->blockTiles; a.off = c->blockOff; a.chunk = c->edChunk;
    a.spill = c->edSpill;
    a.bins = c->edBins; a.bin_cnt = c->edBinCnt; a.keep_bins = 0; a.done = nullptr; a.fault = 0;
    a.W = c->W; a.H = c->H;
    a.rc = (c->W - 1) / TF_SUBSAMPLE + 1; a.rr = (c->H - 1) / TF_SUBSAMPLE + 1;
    a.nrows = ed_nrows(c->H);
    a.lds_max_n = c->ed_lds_max_n;
    a.vcap = c->p.vis_capacity;
    a.nchunk_max = c->p.vis_capacity / ED_CHUNK + 1;
    a.fx = c->p.fx; a.fy = c->p.fy; a.cx = c->p.cx; a.cy = c->p.cy; a.voxelSize = c->p.voxelSize;
    a.cap = (unsigned)c->p.max_render_blocks;
}

// project_done: k_ed_project's pass already ran in the frame's k_integrate grid (frame path)
hipError_t tfk_expected_depths(tf_ctx* c, int project_done, int keep_bins)
{
    EdArgs a;
    tf_ed_args(c, &a);
    a.keep_bins = keep_bins;
    if (!project_done) hipLaunchKernelGGL(k_ed_project, dim3(TF_ED_BLOCKS), dim3(256), 0, c->stream, a, c->st);
    // one workgroup per LDS row (the atomic path grid-strides the same grid)
    tf_launch(c, k_ed_fill, dim3(a.nrows), dim3(ED_THREADS), 0, a, c->st);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// The frame's raycasts in one launch (k_raycast_pair), with CreateExpectedDepths' fill fused in
// ---------------------------------------------------------------------------------------
#define ED_PAIR_W 1280   // the fused fill's LDS columns: frames up to 1280 wide (wider: k_ed_fill)

// the four /8 range pixels (2tx..2tx+1, 2ty..2ty+1) under a 16x16 ray tile from the projection's
// bins: for each, the min / max over the boxes of its row's bin that cover its column and pass
// the MAX_RENDERING_BLOCKS check -- exactly the value ed_fill_block's LDS row gets (the same
// boxes, min / max commute), so the tile's rays need not wait for the fill
struct IrLds {
    unsigned cpre[ED_LDS_MAX_N / ED_CHUNK];
    unsigned total;
    int mn[4][4], mx[4][4];      // [wave][pixel]
    float2 rng[4];
};
__device__ __forceinline__ void ed_tile_range(const EdArgs& a, int X0, int Y0, int n, IrLds& L)
{
    const int nchunks = (n + ED_CHUNK - 1) / ED_CHUNK;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    // one round trip: the chunk totals and the two bin counts
    const unsigned cv = threadIdx.x < 64 && (int)threadIdx.x < nchunks ? (unsigned)a.chunk[threadIdx.x] : 0u;
    const int c0 = a.bin_cnt[Y0], c1 = a.bin_cnt[Y0 + 1];
    if (threadIdx.x < 64) {                      // chunk totals -> tile total + chunk prefix
        unsigned incl = cv;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const unsigned u = __shfl_up(incl, d, 64);
            if ((int)threadIdx.x >= d) incl += u;
        }
        L.cpre[threadIdx.x] = incl - cv;
        if (threadIdx.x == 63) L.total = incl;
    }
    __syncthreads();
    const bool capped = L.total > a.cap;
    int mn[4], mx[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) { mn[p] = __float_as_int(TF_FAR_AWAY); mx[p] = __float_as_int(TF_VERY_CLOSE); }
#pragma unroll
    for (int part = 0; part < 2; ++part) {
        const int m = part ? c1 : c0;
        const uint4* bin = a.bins + (size_t)(Y0 + part) * a.lds_max_n;
        for (int k0 = threadIdx.x; k0 < m; k0 += 4 * 256) {
            uint4 e[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) e[k] = bin[k0 + k * 256 < m ? k0 + k * 256 : k0];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (k0 + k * 256 >= m) continue;
                const uint4 r = e[k];
                const int bx = (int)(r.x & 0xfffu), bz = (int)(r.y & 0xfffu);
                if (bz < X0 || bx > X0 + 1) continue;
                if (capped) {
                    const int i = (int)((r.x >> 24) | ((r.y >> 24) << 8));
                    const unsigned need = (unsigned)a.tiles[i], off = L.cpre[i / ED_CHUNK] + (unsigned)a.off[i];
                    if (!(need && off + need <= a.cap)) continue;
                }
#pragma unroll
                for (int c = 0; c < 2; ++c)
                    if (bx <= X0 + c && X0 + c <= bz) {
                        mn[2 * part + c] = min(mn[2 * part + c], (int)r.z);
                        mx[2 * part + c] = max(mx[2 * part + c], (int)r.w);
                    }
            }
        }
    }
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            mn[p] = min(mn[p], __shfl_xor(mn[p], o, 64));
            mx[p] = max(mx[p], __shfl_xor(mx[p], o, 64));
        }
    if (lane == 0)
#pragma unroll
        for (int p = 0; p < 4; ++p) { L.mn[wv][p] = mn[p]; L.mx[wv][p] = mx[p]; }
    __syncthreads();
    if (threadIdx.x < 4) {
        const int p = threadIdx.x;
        const int a0 = min(min(L.mn[0][p], L.mn[1][p]), min(L.mn[2][p], L.mn[3][p]));
        const int a1 = max(max(L.mx[0][p], L.mx[1][p]), max(L.mx[2][p], L.mx[3][p]));
        L.rng[p] = make_float2(__int_as_float(a0), __int_as_float(a1));
    }
    __syncthreads();
}

#ifdef TF_PAIR_TIMELINE
// diagnostic builds only (tools/pair_timeline.py): per workgroup of the last k_raycast_pair
// launch, [start, end of wave 0..3, end, kind | xcc << 8 | cu << 16] on the 100 MHz clock
#define PTL_MAX 8192
__device__ unsigned long long tf_pair_tl[PTL_MAX * 7];
extern "C" int tf_debug_pair_timeline(void* host, size_t bytes)
{
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(tf_pair_tl), bytes < sizeof(tf_pair_tl) ? bytes : sizeof(tf_pair_tl), 0,
                                    hipMemcpyDeviceToHost);
}
#endif

// every branch's LDS overlaid: the kernel keeps the raycast's occupancy (8 workgroups per CU)
union PairLds {
    int vtab[256 * VTAB_STRIDE];
    IrLds ir;
    EdLds<ED_PAIR_W> ed;
    PnLds pn;
    BilLds bil;
};

// The frame's two raycasts in one launch: one part of the grid casts CreateICPMaps' rays
// (castRay<true>, new range image), another renderImage's (castRay<false> + grey, range
// snapshot).  Neither writes what the other reads, and a launch's run time is its slowest waves'
// ray length: the halves fill each other's tails instead of each kernel draining alone.
// (Measured: marching both rays of a pixel interleaved in one thread, sharing each step's round
// trips, is slower -- 142 VGPRs halve the resident waves.)
// nfill > 0 (frame path, W <= ED_PAIR_W): the grid starts with CreateExpectedDepths' fill
// (ed_fill_block, one workgroup per LDS row; it writes the range image for the frames after this
// one) and the CreateICPMaps tiles take their four range pixels from the projection's bins
// (ed_tile_range) instead of waiting for it -- one launch and its dependent round trips fewer per
// frame.  Past lds_max_n visible entries the fill takes its atomic path and the tiles wait for
// its rows to count done (the fill workgroups come first in dispatch order, and wait on nothing).
// (8 waves per SIMD: the allocator left alone takes 70 VGPRs over the kernel's branches, each of
// which fits 64 on its own; held to 64 it spills one 8-byte value once per thread)
__device__ __forceinline__ int pair_body(PairLds& L, RayArgs ai, RayArgs ar, TfDevState* __restrict__ st, int tiles_x,
                                         int n_tiles, int nb, PyrArgs pyr, int n_pyr, int pyr_gx, BilArgs bil, int bil_gx,
                                         EdArgs ed, int nfill, int nfill_pad, const int* __restrict__ order,
                                         unsigned* __restrict__ cost);
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8)))
k_raycast_pair(RayArgs ai, RayArgs ar, TfDevState* __restrict__ st, int tiles_x, int n_tiles, int nb,
               PyrArgs pyr, int n_pyr, int pyr_gx, BilArgs bil, int bil_gx, EdArgs ed, int nfill, int nfill_pad,
               const int* __restrict__ order, unsigned* __restrict__ cost)
{
    __shared__ PairLds L;
#ifdef TF_PAIR_TIMELINE
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    const int kind = pair_body(L, ai, ar, st, tiles_x, n_tiles, nb, pyr, n_pyr, pyr_gx, bil, bil_gx, ed, nfill, nfill_pad, order, cost);
    const unsigned long long tw = __builtin_amdgcn_s_memrealtime();
    __syncthreads();
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    // (TFUSION_PTL_LOOKAHEAD builds: only launches that carry later frames' preprocessing)
#ifdef TF_PTL_LOOKAHEAD
    if (n_pyr + (int)gridDim.x - nfill_pad - 2 * nb - n_pyr <= 0) return;
#endif
    if (blockIdx.x < PTL_MAX) {
        unsigned long long* o = &tf_pair_tl[blockIdx.x * 7];
        if ((threadIdx.x & 63) == 0) o[1 + (threadIdx.x >> 6)] = tw;
        if (threadIdx.x == 0) {
            unsigned xcc = 0, hw = 0;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
            o[0] = t0; o[5] = t1;
            o[6] = (unsigned long long)(kind & 0xff) | ((unsigned long long)(xcc & 0xf) << 8) |
                   ((unsigned long long)((hw >> 8) & 0xf) << 16) | ((unsigned long long)((hw >> 13) & 0x7) << 20);
        }
    }
#else
    pair_body(L, ai, ar, st, tiles_x, n_tiles, nb, pyr, n_pyr, pyr_gx, bil, bil_gx, ed, nfill, nfill_pad, order, cost);
#endif
}

// the branch kind (diagnostics): 0 fill, 1 CreateICPMaps tile, 2 renderImage tile, 3 pyramid /
// normals, 4 bilateral, 5 nothing to do
// the ray tiles' workgroup time, for the next frame's longest-first order (tf_ctx::tile_order)
__device__ __forceinline__ void pair_tile_cost(unsigned* cost, int slot, unsigned long long t0)
{
    if (!cost) return;
    __syncthreads();                 // (the workgroup's LDS is held until its last wave anyway)
    if (threadIdx.x == 0) cost[slot] = (unsigned)min(__builtin_amdgcn_s_memrealtime() - t0, 0xffffeull);
}
__device__ __forceinline__ int pair_body(PairLds& L, RayArgs ai, RayArgs ar, TfDevState* __restrict__ st, int tiles_x,
                                         int n_tiles, int nb, PyrArgs pyr, int n_pyr, int pyr_gx, BilArgs bil, int bil_gx,
                                         EdArgs ed, int nfill, int nfill_pad, const int* __restrict__ order,
                                         unsigned* __restrict__ cost)
{
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    int b = (int)blockIdx.x;
    if (b < nfill_pad) {
        if (b < nfill) ed_fill_block<ED_PAIR_W>(ed, st, b, nfill, L.ed, false);
        return b < nfill ? 0 : 5;
    }
    b -= nfill_pad;
    if (b < nb) {
        if (!raycast_go<1>(st)) return 5;
        const int tile = order ? order[b] : xcd_tile(b, n_tiles);
        if (tile < 0) return 5;
        const int tx = tile % tiles_x, ty = tile / tiles_x;
        const int n = st->noVisibleEntries;
        if (nfill > 0 && n <= ed.lds_max_n) {
            ed_tile_range(ed, 2 * tx, 2 * ty, n, L.ir);
        } else {
            if (nfill > 0 && threadIdx.x == 0) {
                // the fill's atomic path writes the range image: wait until every row is done
                unsigned spins = 0;
                while (__hip_atomic_load(ed.done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)nfill) {
                    if (++spins > (1u << 24) || ed.fault) { st->icp_ok = -2; break; }   // the frame end: a sticky HIP error
                    __builtin_amdgcn_s_sleep(2);
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            }
            __syncthreads();
            if (threadIdx.x < 4) {               // the tile's four /8 pixels of the range image
                const int X = 2 * tx + (threadIdx.x & 1), Y = 2 * ty + (threadIdx.x >> 1);
                L.ir.rng[threadIdx.x] = X < ai.W && Y < ai.H ? ai.range[X + Y * ai.W] : make_float2(0.f, 0.f);
            }
            __syncthreads();
        }
        // (one instance of the march for both sources of the range: a second costs registers)
        raycast_tile<1, true>(ai, st, tile, tiles_x, nullptr, L.ir.rng);
        pair_tile_cost(cost, tile, t0);
        return 1;
    }
    b -= nb;
    if (b < nb) {
        if (!raycast_go<2>(st)) return 5;
        const int tile = order ? order[nb + b] : xcd_tile(b, n_tiles);
        if (tile < 0) return 5;
        raycast_tile<2>(ar, st, tile, tiles_x, L.vtab);
        pair_tile_cost(cost, n_tiles + tile, t0);
        return 2;
    }
    b -= nb;
    // Later frames of the batch in this grid's tail, not gated by this frame's abort: the next
    // frame's computeDists + pyramids + normals (this frame's allocation and integration, the
    // last readers of dists and of the current maps, are done; its level-0 depth was filtered
    // a launch or more ago), then the bilateral pass of the frame after it (into the other
    // level-0 buffer: this frame's, whose last reader was its own pyramid pass)
    if (b < n_pyr) { pyr_normals_block<256>(pyr, b % pyr_gx, b / pyr_gx, L.pn); return 3; }
    bilateral_block<false>(bil, (b - n_pyr) % bil_gx, (b - n_pyr) / bil_gx, L.bil);
    return 4;
}

// CreateICPMaps' raycast + the frame's renderImage in one launch (after CreateExpectedDepths'
// projection): the renderImage half reads the range-image snapshot (render_snapshot).
// fuse_ed: CreateExpectedDepths' fill runs in this grid (frame path; W <= ED_PAIR_W)
int tfk_ed_fused(const tf_ctx* c) { return c->W <= ED_PAIR_W; }

hipError_t tfk_raycast_pair_ordered(tf_ctx* c)
{
    hipError_t e = tfk_raycast_pair(c, TfAhead{}, TfAhead{}, 0, 0, 1);
    if (e != hipSuccess || !c->tile_ljf) return e;
    TileSortArgs ts;
    ts.cost = c->tile_cost; ts.order = c->tile_order;
    ts.tx = (c->W + 15) / 16; ts.ty = (c->H + 15) / 16; ts.n = ts.tx * ts.ty;
    ts.nb = c->tile_slots; ts.rows = c->tile_rows;
    hipLaunchKernelGGL(k_tile_sort, dim3(16), dim3(256), 0, c->stream, ts);
    return hipGetLastError();
}

hipError_t tfk_raycast_pair(tf_ctx* c, TfAhead pyr, TfAhead bil, size_t pitch, int fuse_ed, int ljf)
{
    RayArgs ai, ar;
    ray_args(c, ai);
    ai.visType = c->visType;
    ray_args(c, ar);
    ar.range = (const float2*)c->range_render;
    ar.grey = c->grey;
    const int tx = (c->W + 15) / 16, ty = (c->H + 15) / 16, n = tx * ty;
    const int nb = (n + 7) / 8 * 8;
    BilArgs bb = BilArgs{}, bx; PyrArgs pp = PyrArgs{}, px;
    int n_pyr = 0, pyr_gx = 1, n_bil = 0, bil_gx = 1;
    if (pyr.src) {
        const hipError_t e = tf_pre_args(c, pyr.src, pitch, 1, pyr.d0, &bx, &pp);
        if (e != hipSuccess) return e;
        pyr_gx = tf_div_up(c->W, PN_T0);
        n_pyr = pyr_gx * tf_div_up(c->H, PN_T0);
    }
    if (bil.src) {
        const hipError_t e = tf_pre_args(c, bil.src, pitch, 1, bil.d0, &bb, &px);
        if (e != hipSuccess) return e;
        bil_gx = tf_div_up(c->W, PRE_TX);
        n_bil = bil_gx * tf_div_up(c->H, PRE_TY);
    }
    EdArgs ed;
    tf_ed_args(c, &ed);
    int nfill = 0, nfill_pad = 0;
    if (fuse_ed && tfk_ed_fused(c)) {
        nfill = ed.nrows;
        nfill_pad = (nfill + 7) / 8 * 8;        // keeps the tiles' XCD swizzle aligned
        ed.done = c->edDone;
    }
    ed.fault = ++c->pair_launches == c->fill_fault_launch;
    const bool order = ljf && c->tile_ljf;
    const int nbl = order ? c->tile_slots : nb;
    tf_launch(c, k_raycast_pair, dim3(nfill_pad + 2 * nbl + n_pyr + n_bil), dim3(256), 0, ai, ar, c->st, tx, n, nbl,
              pp, n_pyr, pyr_gx, bb, bil_gx, ed, nfill, nfill_pad, order ? (const int*)c->tile_order : nullptr,
              order ? c->tile_cost : nullptr);
    return hipGetLastError();
}
