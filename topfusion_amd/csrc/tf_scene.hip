// tf_scene.hip -- voxel-block hash allocation, visible list and TSDF integration
//  for gfx950.
//
// The reference resolves its data races by "last writer wins" and hands out blocks in
// atomicSub order (SceneReconstructionEngine.hpp:287-292, SceneReconstructionEngine_host.cu:
// 350-479).  Here every decision is deterministic and equal to the serial order:
//   * allocation requests: per-entry atomicMax of key = pixel*64 + step (raster order,
//     last writer wins); the winning block position is recomputed from the key;
//   * block / excess slots: ordered by hash index through a chunked scan whose per-chunk
//     counts the request pass accumulates; capacity exhaustion (the silent failures) is
//     decided per request from the same prefix counts (k_alloc_apply), exactly the serial loop;
//   * visible list: ordered compaction by hash index.
#include "tf_internal.h"
#include "tf_preproc.h"
#include "tf_ed.h"
#include "tf_reset.h"
#include "tf_vis.h"

#ifndef TF_INTEG_STREAM_BLOCKS
#define TF_INTEG_STREAM_BLOCKS 16384   // 32 MiB of voxels
#endif
#ifndef TF_INTEG_NT_STORES
#define TF_INTEG_NT_STORES 0
#endif
#define CHUNK 4096          // hash entries per workgroup in the scan passes (256 thr x 16)

// byte i (0..15) of a 16-byte group held as two 64-bit words (no dynamic register indexing)
__device__ __forceinline__ unsigned byte16(unsigned long long lo, unsigned long long hi, int i)
{
    return (unsigned)(((i < 8) ? (lo >> (8 * i)) : (hi >> (8 * (i - 8)))) & 0xffull);
}
__device__ __forceinline__ void load16(const unsigned char* p, unsigned long long* lo, unsigned long long* hi)
{
    uint4 v = *(const uint4*)p;
    *lo = (unsigned long long)v.x | ((unsigned long long)v.y << 32);
    *hi = (unsigned long long)v.z | ((unsigned long long)v.w << 32);
}

// ---------------------------------------------------------------------------------------
// ResetScene (SceneReconstructionEngine_host.cu:51-73)
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_reset_scene(ResetArgs r)
{
    reset_scene_block(r, blockIdx.x, gridDim.x);
}

void tf_reset_args(tf_ctx* c, ResetArgs* r, int on_failure, int slot, int clear_cache)
{
    r->vba = c->vba; r->n_vox = (size_t)c->p.n_blocks * TF_BLK3;
    r->allocList = c->allocList; r->n_blocks = c->p.n_blocks;
    r->hash = c->hash; r->n_total = c->n_total;
    r->excessList = c->excessList; r->n_excess = c->p.n_excess;
    r->st = c->st; r->grid = c->bgrid;
    r->on_failure = on_failure;
    r->frame_ok = on_failure ? c->frame_ok : nullptr; r->frame_mode = on_failure ? c->frame_mode : nullptr;
    r->slot = on_failure ? slot : 0;
    r->full = on_failure ? 0 : 1;       // (+ st->scene_external, read on the device)
    // swapping: swap-outs push blocks back onto the free list in any order, so its identity (which
    // the clear-what-was-written reset relies on) no longer holds -- every reset is full.  The
    // TopFu-level resets (construction, TopFu::reset, the ICP-failure frame end) also empty the
    // GlobalCache (swap states, stored flags), so no block of the old scene is swapped into the
    // new one; the engine's ResetScene keeps it, as the reference's does (clear_cache = 0)
    r->swapState = c->p.use_swapping && clear_cache ? c->swapState : nullptr;
    r->swapFlags = c->p.use_swapping && clear_cache ? c->swapFlags : nullptr;
    r->vba_rgb = c->p.voxel_rgb ? c->vba_rgb : nullptr;
    r->ed_bin_cnt = on_failure ? c->edBinCnt : nullptr;
    r->ed_nbins = 2 * ed_nrows(c->H);
    r->ed_done = c->edDone;
    if (c->p.use_swapping) r->full = 1;
}

hipError_t tfk_reset_scene(tf_ctx* c, int clear_cache)
{
    ResetArgs r;
    tf_reset_args(c, &r, 0, 0, clear_cache);
    hipLaunchKernelGGL(k_reset_scene, dim3(2048), dim3(256), 0, c->stream, r);
    return hipGetLastError();
}

// the frame's end (every frame; the reset part only when ICP failed): one workgroup per CU, so
// a successful frame pays a small launch; a failed one clears only what the frames wrote (a
// full clear when scene buffers were uploaded since the last full reset)
hipError_t tfk_reset_scene_on_failure(tf_ctx* c, int slot)
{
    ResetArgs r;
    tf_reset_args(c, &r, 1, slot, 1);
    hipLaunchKernelGGL(k_reset_scene, dim3(TF_END_BLOCKS), dim3(256), 0, c->stream, r);
    return hipGetLastError();
}


__global__ void k_grid_build(const TfHashEntry* __restrict__ hash, int n_total, int2* __restrict__ grid)
{
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n_total; i += gridDim.x * blockDim.x)
        grid_set(grid, hash[i], i);
}

__global__ void k_grid_clear(int4* __restrict__ grid2, size_t n2)
{
    const int4 none = make_int4(-1, TF_VOFF_NONE, -1, TF_VOFF_NONE);
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += (size_t)gridDim.x * blockDim.x)
        grid2[i] = none;
}

// every cell "no block" (-1, TF_VOFF_NONE)
hipError_t tfk_grid_clear(tf_ctx* c)
{
    const size_t n2 = (size_t)TF_GRID_DIM * TF_GRID_DIM * TF_GRID_DIM / 2;
    hipLaunchKernelGGL(k_grid_clear, dim3(4096), dim3(256), 0, c->stream, (int4*)c->bgrid, n2);
    return hipGetLastError();
}

// tf_div_exact3 against the division for every mantissa of the binade [1, 2), both signs, on
// the device's own arithmetic (scale invariance extends it to every binade without subnormal
// intermediates)
__global__ void k_check_div3(float d, int* ok)
{
    const unsigned m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= (1u << 23)) return;
    const float rd = 1.0f / d;
    const float x = __uint_as_float(0x3f800000u | m);
    bool good = true;
    for (int s = 0; s < 2; ++s) {
        const float xx = s ? -x : x;
        const float q0 = xx * rd;
        const float q = fmaf(-fmaf(q0, d, -xx), rd, q0);
        good = good && __float_as_uint(q) == __float_as_uint(xx / d);
    }
    if (!good) atomicAnd(ok, 0);
}

hipError_t tfk_check_div3(tf_ctx* c, float d, int* ok)
{
    int* dok = (int*)c->icp_ticket;              // scratch word (the ticket is idle at creation)
    int one = 1;
    hipError_t e = hipMemcpyAsync(dok, &one, sizeof(int), hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_check_div3, dim3((1u << 23) / 256), dim3(256), 0, c->stream, d, dok);
    e = hipMemcpyAsync(ok, dok, sizeof(int), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    int zero = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(dok, &zero, sizeof(int), hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    return e;
}

hipError_t tfk_grid_rebuild(tf_ctx* c)
{
    hipError_t e = tfk_grid_clear(c);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_grid_build, dim3(1024), dim3(256), 0, c->stream, c->hash, c->n_total, c->bgrid);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// buildHashAllocAndVisibleTypePP (SceneReconstructionEngine.hpp:206-298)
// ---------------------------------------------------------------------------------------
struct AllocArgs {
    const float* dists;
    int W, H;
    float invfx, invfy, cx, cy;        // invProjParams_d (SceneReconstructionEngine_host.cu:110-113)
    float mu, oneOverVoxelSize;        // 1/(voxelSize*8)
    float vf_min, vf_max;
    unsigned mask;
    int n_buckets;
    int2* grid;                        // block grid, kept in step with the hash
};

// ray segment [d-mu, d+mu] of pixel (x,y) in block units; false if the pixel is skipped
__device__ __forceinline__ bool alloc_segment(const AllocArgs& a, const float* invM, int x, int y,
                                              float* point, float* dir, int* noSteps)
{
    float depth_measure = a.dists[x + y * a.W];
    if (depth_measure <= 0 || (depth_measure - a.mu) < 0 || (depth_measure - a.mu) < a.vf_min ||
        (depth_measure + a.mu) > a.vf_max) return false;
    float pcz = depth_measure;
    float pcx = pcz * (((float)x - a.cx) * a.invfx);
    float pcy = pcz * (((float)y - a.cy) * a.invfy);
    float norm = sqrtf(pcx * pcx + pcy * pcy + pcz * pcz);
    float r[3], pe[3];
    float s1 = 1.0f - a.mu / norm;
    tf_m4v3(invM, pcx * s1, pcy * s1, pcz * s1, 1.0f, r);
    point[0] = r[0] * a.oneOverVoxelSize; point[1] = r[1] * a.oneOverVoxelSize; point[2] = r[2] * a.oneOverVoxelSize;
    float s2 = 1.0f + a.mu / norm;
    tf_m4v3(invM, pcx * s2, pcy * s2, pcz * s2, 1.0f, r);
    pe[0] = r[0] * a.oneOverVoxelSize; pe[1] = r[1] * a.oneOverVoxelSize; pe[2] = r[2] * a.oneOverVoxelSize;
    dir[0] = pe[0] - point[0]; dir[1] = pe[1] - point[1]; dir[2] = pe[2] - point[2];
    norm = sqrtf(dir[0] * dir[0] + dir[1] * dir[1] + dir[2] * dir[2]);
    int n = (int)ceilf(2.0f * norm);
    float dv = (float)(n - 1);
    dir[0] /= dv; dir[1] /= dv; dir[2] /= dv;
    *noSteps = n;
    return true;
}

// An allocation request of this workgroup's 16x16 pixel tile: requests are aggregated per hash
// entry in LDS (the raster-order maximum key, the request type) and go out as one global
// atomicMax per entry and tile when the tile is done -- every pixel whose segment crosses a new
// block requests it, a few hundred atomics on one word per new block at C2, serialised at the
// memory side.  The maximum and the stores are order-independent: the same winners, types and
// counts.  A full table sends the request straight to memory.
#define AR_SLOTS 256
struct AllocLds {
    int idx[AR_SLOTS];                 // hash entry index, -1 free
    int key[AR_SLOTS];                 // max requesting key
    unsigned char exc[AR_SLOTS];       // request type: excess (chain end) or bucket
    int seen[AR_SLOTS];                // entries found through the block grid (their visType store made)
};

// visType = 1 for an entry the block grid holds: once per entry and tile (a block is found by
// every step of every pixel crossing it; the stores are all the same byte)
__device__ __forceinline__ void alloc_mark_found(AllocLds& t, unsigned char* __restrict__ visType, int hashIdx)
{
    unsigned h = ((unsigned)hashIdx * 2654435761u) >> 24;
    for (int probe = 0; probe < AR_SLOTS; ++probe, h = (h + 1) & (AR_SLOTS - 1)) {
        const int prev = atomicCAS(&t.seen[h], -1, hashIdx);
        if (prev == hashIdx) return;                       // marked by this tile already
        if (prev == -1) break;                             // first in this tile
    }
    visType[hashIdx] = 1;
}

__device__ __forceinline__ void alloc_request_global(int* __restrict__ winnerKey, int* __restrict__ counts, int hashIdx,
                                                     bool isExcess, int key)
{
    // raster-order last writer; the first request of an entry this frame (the key was -1)
    // counts it for its chunk (the hash is read-only here, so an entry's request type is the
    // same for every requester)
    if (atomicMax(&winnerKey[hashIdx], key) < 0) {
        atomicAdd(&counts[2 * (hashIdx / CHUNK)], 1);
        if (isExcess) atomicAdd(&counts[2 * (hashIdx / CHUNK) + 1], 1);
    }
}

__device__ __forceinline__ bool alloc_request_lds(AllocLds& t, int hashIdx, bool isExcess, int key)
{
    unsigned h = ((unsigned)hashIdx * 2654435761u) >> 24;
    for (int probe = 0; probe < AR_SLOTS; ++probe, h = (h + 1) & (AR_SLOTS - 1)) {
        const int prev = atomicCAS(&t.idx[h], -1, hashIdx);
        if (prev == -1 || prev == hashIdx) {
            atomicMax(&t.key[h], key);
            t.exc[h] = isExcess ? 1 : 0;
            return true;
        }
    }
    return false;
}

// the hash probe of one step whose block the grid does not hold: found (outside the grid) ->
// visible type; otherwise an allocation request in the bucket (1) or at the chain end (2)
__device__ __forceinline__ void alloc_probe(const AllocArgs& a, const TfHashEntry* __restrict__ hash,
                                            unsigned char* __restrict__ allocType, unsigned char* __restrict__ visType,
                                            int* __restrict__ winnerKey, int* __restrict__ counts,
                                            int bx, int by, int bz, int key, AllocLds& lt)
{
    {
        int hashIdx = tf_hash_index(bx, by, bz, a.mask);
        TfHashEntry e = hash[hashIdx];
        bool found = false;
        if (e.x == bx && e.y == by && e.z == bz && e.ptr >= -1) {
            visType[hashIdx] = (e.ptr == -1) ? 2 : 1;
            found = true;
        }
        if (!found) {
            bool isExcess = false;
            if (e.ptr >= -1) {
                while (e.offset >= 1) {
                    hashIdx = a.n_buckets + e.offset - 1;
                    e = hash[hashIdx];
                    if (e.x == bx && e.y == by && e.z == bz && e.ptr >= -1) {
                        visType[hashIdx] = (e.ptr == -1) ? 2 : 1;
                        found = true;
                        break;
                    }
                }
                isExcess = true;
            }
            if (!found && !alloc_request_lds(lt, hashIdx, isExcess, key)) {
                allocType[hashIdx] = isExcess ? 2 : 1;
                if (!isExcess) visType[hashIdx] = 1;
                alloc_request_global(winnerKey, counts, hashIdx, isExcess, key);
            }
        }
    }
}

__global__ void __launch_bounds__(256)
k_alloc_requests(AllocArgs a, TfDevState* __restrict__ st, const TfHashEntry* __restrict__ hash,
                 unsigned char* __restrict__ allocType, unsigned char* __restrict__ visType, int* __restrict__ winnerKey,
                 int* __restrict__ counts, int gx, int n_alloc, BilArgs next, int next_gx)
{
    if ((int)blockIdx.x >= n_alloc) {
        // a later frame of the batch: its bilateral pass in this grid's tail (it reads only that
        // frame's raw depth and writes only its level-0 depth buffer; not gated by this
        // frame's abort)
        const int b = (int)blockIdx.x - n_alloc;
        __shared__ BilLds L;
        bilateral_block<false>(next, b % next_gx, b / next_gx, L);
        return;
    }
    if (st->abort) return;
    if (blockIdx.x == 0 && threadIdx.x == 0) { st->alloc_fail[0] = 0; st->alloc_fail[1] = 0; }   // (k_alloc_apply counts)
    __shared__ AllocLds lt;
    lt.idx[threadIdx.x] = -1;
    lt.key[threadIdx.x] = -1;
    lt.seen[threadIdx.x] = -1;
    __syncthreads();
    const int bx = (int)blockIdx.x % gx, by = (int)blockIdx.x / gx;
    const int x = bx * 16 + (threadIdx.x & 15), y = by * 16 + (threadIdx.x >> 4);
    float point[3], dir[3]; int noSteps = 0;
    if (!(x < a.W && y < a.H && alloc_segment(a, st->invM_alloc, x, y, point, dir, &noSteps))) noSteps = 0;
    const int key0 = (y * a.W + x) * 64;
    // Steps in batches of 8: the block grid answers "already allocated" for every step with one
    // batch of independent loads (the grid mirrors the hash exactly, tf_internal.h); only the
    // steps whose block is not in the grid walk the hash (bucket / excess chain) to place their
    // allocation request.  Same outcomes, same raster-order keys as the serial loop.
    for (int i0 = 0; i0 < noSteps; i0 += 8) {
        int sbx[8], sby[8], sbz[8];
        int2 g[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            sbx[j] = (short)floorf(point[0]); sby[j] = (short)floorf(point[1]); sbz[j] = (short)floorf(point[2]);
            const bool in = i0 + j < noSteps && tf_grid_in(sbx[j], sby[j], sbz[j]);
            g[j] = a.grid[in ? tf_grid_cell(sbx[j], sby[j], sbz[j]) : 0];
            if (!in) g[j] = make_int2(-1, -1);
            if (i0 + j < noSteps) { point[0] += dir[0]; point[1] += dir[1]; point[2] += dir[2]; }
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int i = i0 + j;
            if (i >= noSteps) break;
            if (g[j].x >= 0) { alloc_mark_found(lt, visType, g[j].x); continue; }   // found, ptr >= 0 (swapped-out entries have no cell: the probe finds them)
            alloc_probe(a, hash, allocType, visType, winnerKey, counts, sbx[j], sby[j], sbz[j], key0 + i, lt);
        }
    }
    // the tile's requests: one global request per entry
    __syncthreads();
    const int hi = lt.idx[threadIdx.x];
    if (hi >= 0) {
        const bool exc = lt.exc[threadIdx.x] != 0;
        allocType[hi] = exc ? 2 : 1;
        if (!exc) visType[hi] = 1;
        alloc_request_global(winnerKey, counts, hi, exc, lt.key[threadIdx.x]);
    }
}

// recompute the block position written by request `key` (blockCoords in the reference)
__device__ __forceinline__ void alloc_block_from_key(const AllocArgs& a, const float* invM, int key, short* pos)
{
    int pix = key >> 6, step = key & 63;
    int x = pix % a.W, y = pix / a.W;
    float point[3], dir[3]; int noSteps;
    alloc_segment(a, invM, x, y, point, dir, &noSteps);
    for (int i = 0; i < step; ++i) { point[0] += dir[0]; point[1] += dir[1]; point[2] += dir[2]; }
    pos[0] = (short)floorf(point[0]); pos[1] = (short)floorf(point[1]); pos[2] = (short)floorf(point[2]);
}

// setToType3 (SceneReconstructionEngine_host.cu:343-348) over the previous visible list, with
// the checkBlockVisibility<false> test buildVisibleList applies to entries still of type 3
// (:449-476) evaluated here already: it depends only on the entry's block position (which
// the allocation pass does not change for existing entries) and on this frame's pose.  Type 4
// = "type 3, not visible"; the allocation pass overwrites 3/4 exactly as it overwrites 3, and
// k_vis_count turns the 4s that survive into 0.  One entry per thread instead of a dependent
// hash load inside the N_tot scan.
// It also takes the frame's renderImage snapshot (render_snapshot, tf_internal.h) first.
__global__ void __launch_bounds__(256)
k_set_type3(VisArgs v, TfDevState* __restrict__ st, const TfHashEntry* __restrict__ hash,
            const int* __restrict__ visibleIds, unsigned char* __restrict__ visType,
            const float2* __restrict__ range, float2* __restrict__ snap)
{
    if (snap) render_snapshot(st, range, snap, v.W, v.H);
    if (st->abort) return;
    const int n = st->noVisibleEntries;
    const float* M = st->M_alloc;
    set_type3_pass(v, n, M, hash, visibleIds, visType, blockIdx.x * blockDim.x + threadIdx.x, gridDim.x * blockDim.x);
}

// ---------------------------------------------------------------------------------------
// block scan helpers (256 threads)
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ int wave_incl_scan(int v)
{
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int n = __shfl_up(v, o, 64);
        if (lane >= o) v += n;
    }
    return v;
}

// exclusive scan of v over the 256-thread block; *total receives the block sum
__device__ __forceinline__ int block_excl_scan(int v, int* total)
{
    __shared__ int wsum[4];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int inc = wave_incl_scan(v);
    if (lane == 63) wsum[wave] = inc;
    __syncthreads();
    int off = 0, tot = 0;
    for (int w = 0; w < 4; ++w) { int s = wsum[w]; if (w < wave) off += s; tot += s; }
    __syncthreads();
    *total = tot;
    return off + inc - v;
}

__device__ __forceinline__ int block_sum(int v)
{
    int tot;
    block_excl_scan(v, &tot);
    return tot;
}

// four block sums at once (one LDS exchange instead of four)
__device__ __forceinline__ int4 block_sum4(int4 v)
{
    __shared__ int4 wsum4[4];
    const int wave = threadIdx.x >> 6;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        v.x += __shfl_xor(v.x, o, 64); v.y += __shfl_xor(v.y, o, 64);
        v.z += __shfl_xor(v.z, o, 64); v.w += __shfl_xor(v.w, o, 64);
    }
    if ((threadIdx.x & 63) == 0) wsum4[wave] = v;
    __syncthreads();
    int4 t = wsum4[0];
    for (int w = 1; w < 4; ++w) { const int4 u = wsum4[w]; t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w; }
    __syncthreads();
    return t;
}

// ---------------------------------------------------------------------------------------
// allocateVoxelBlocksList_device (SceneReconstructionEngine_host.cu:350-415), ordered
// ---------------------------------------------------------------------------------------
// The serial loop over the requests in index order keeps two counters: v (lastFreeBlockId) and
// e (lastFreeExcessListId).  A type-1 request takes v-- and fails (restoring v, visType = 0)
// when v < 0; a type-2 request takes v-- and e-- and fails (restoring both) when either is < 0
// (:358-413).  Both counters only ever go down, so the outcome of request k is a function of
// prefix counts, with v0 / e0 the counters at the start:
//   q(k)  = type-2 requests before k;   n1(k) = type-1 requests before k
//   S(k)  = n1(k) + min(q(k), e0 + 1)   -- the successes before k while blocks last
//   type 1 succeeds iff S(k) <= v0;  type 2 iff S(k) <= v0 and q(k) <= e0
// (the type-2 successes are the first e0 + 1 type-2 requests until the blocks run out; once
// S(k) > v0 nothing succeeds any more).  A success takes allocList[v0 - S(k)] and, for type 2,
// excessList[e0 - q(k)].  Without exhaustion S(k) is k's rank among all requests.  So every
// request is decided in parallel from the chunk prefix sums, with the serial loop's results.
__global__ void __launch_bounds__(256)
k_alloc_apply(AllocArgs a, TfDevState* __restrict__ st, int n_chunks, const int* __restrict__ counts,
              unsigned char* __restrict__ allocType, int* __restrict__ winnerKey, TfHashEntry* __restrict__ hash,
              unsigned char* __restrict__ visType, const int* __restrict__ allocList,
              const int* __restrict__ excessList, int n_total)
{
    if (st->abort) return;
    // this chunk's request types, loaded before (and in flight with) the counts prefix
    const int base = blockIdx.x * CHUNK + threadIdx.x * 16;
    unsigned long long lo = 0, hi = 0;
    if (base < n_total) load16(allocType + base, &lo, &hi);
    // prefix and totals over the per-chunk counts
    int p12 = 0, p2 = 0, a12 = 0, a2 = 0;
    for (int h = threadIdx.x; h < n_chunks; h += 256) {
        int c12 = counts[2 * h], c2 = counts[2 * h + 1];
        a12 += c12; a2 += c2;
        if (h < (int)blockIdx.x) { p12 += c12; p2 += c2; }
    }
    {
        const int4 t = block_sum4(make_int4(p12, p2, a12, a2));
        p12 = t.x; p2 = t.y; a12 = t.z; a2 = t.w;
    }
    const int v0 = st->lastFreeBlockId, e0 = st->lastFreeExcessListId;
    if (blockIdx.x == 0 && threadIdx.x == 0) { st->pad_[0] = a12; st->pad_[1] = a2; }
    int l12 = 0, l2 = 0;
    if (base < n_total)
        for (int i = 0; i < 16; ++i) { unsigned t = byte16(lo, hi, i); l12 += t != 0; l2 += t == 2; }
    int wg12, tmp;
    const int o12 = block_excl_scan(l12, &wg12);          // this thread's first request in the workgroup
    const int r2_0 = p2 + block_excl_scan(l2, &tmp);
    if (!wg12) return;
    // The workgroup's requests one per thread, in index order: the winner key, the free block and
    // the excess slot are loaded together, then the key's depth sample; a thread holding several
    // requests would chain those round trips.  rq_q: q(k) for a type-2 request, ~q(k) for type 1.
    __shared__ int rq_idx[256], rq_q[256];
    const float* invM = st->invM_alloc;
    for (int k0 = 0; k0 < wg12; k0 += 256) {
        int k = o12, q2 = r2_0;
        for (int i = 0; i < 16 && l12; ++i) {
            const unsigned t = byte16(lo, hi, i);
            if (!t) continue;
            if (k >= k0 && k < k0 + 256) { rq_idx[k - k0] = base + i; rq_q[k - k0] = t == 2 ? q2 : ~q2; }
            ++k;
            if (t == 2) ++q2;
        }
        __syncthreads();
        bool fail1 = false, fail2 = false;
        if (k0 + (int)threadIdx.x < wg12) {
            const int idx = rq_idx[threadIdx.x], qq = rq_q[threadIdx.x];
            const bool is2 = qq >= 0;
            const int q = is2 ? qq : ~qq;
            const int g = p12 + k0 + (int)threadIdx.x;          // rank among all requests
            const int S = (g - q) + (q < e0 + 1 ? q : e0 + 1);    // successes before this request
            const bool ok = S <= v0 && (!is2 || q <= e0);
            if (ok) {
                const int key = winnerKey[idx];
                const int ptr = allocList[v0 - S];
                const int exlOffset = is2 ? excessList[e0 - q] : 0;
                short pos[3];
                alloc_block_from_key(a, invM, key, pos);
                TfHashEntry e; e.x = pos[0]; e.y = pos[1]; e.z = pos[2]; e.pad = 0; e.offset = 0;
                e.ptr = ptr;
                if (!is2) {
                    hash[idx] = e;
                    grid_set(a.grid, e, idx);
                } else {
                    hash[idx].offset = exlOffset + 1;
                    hash[a.n_buckets + exlOffset] = e;
                    grid_set(a.grid, e, a.n_buckets + exlOffset);
                    visType[a.n_buckets + exlOffset] = 1;
                }
            } else if (!is2) {
                visType[idx] = 0;                               // :377
                fail1 = true;
            } else {
                fail2 = true;
            }
            allocType[idx] = 0;
            winnerKey[idx] = -1;
        }
        // failed requests of the frame, one atomic per wave that has any (the counters drop by
        // the successes only: k_vis_count)
        const unsigned long long b1 = __ballot(fail1), b2 = __ballot(fail2);
        if ((threadIdx.x & 63) == 0 && (b1 | b2)) {
            if (b1) atomicAdd(&st->alloc_fail[0], __popcll(b1));
            if (b2) atomicAdd(&st->alloc_fail[1], __popcll(b2));
        }
        __syncthreads();
    }
}


// AllocateSceneFromDepth(..., onlyUpdateVisibleList = true): the requests of this frame are
// dropped unapplied -- request state back to empty, counters unchanged (the reference memsets
// allocType every frame, SceneReconstructionEngine_host.cu:146); the visible types the request
// pass set stay, as in the reference
__global__ void __launch_bounds__(256)
k_alloc_discard(TfDevState* __restrict__ st, const int* __restrict__ counts, unsigned char* __restrict__ allocType,
                int* __restrict__ winnerKey, int n_total)
{
    if (st->abort) return;
    if (blockIdx.x == 0 && threadIdx.x == 0) { st->pad_[0] = 0; st->pad_[1] = 0; }
    if (counts[2 * blockIdx.x] == 0) return;             // no request in this chunk
    for (int i = blockIdx.x * CHUNK + threadIdx.x; i < (int)(blockIdx.x + 1) * CHUNK && i < n_total; i += 256) {
        if (allocType[i]) { allocType[i] = 0; winnerKey[i] = -1; }
    }
}

// ---------------------------------------------------------------------------------------
// buildVisibleList_device<false> (SceneReconstructionEngine_host.cu:434-479) with
// checkBlockVisibility<false> (SceneReconstructionEngine.hpp:300-375), ordered compaction
// ---------------------------------------------------------------------------------------
// one chunk of the count pass: allocation counters reset, type 4 -> 0, swap states marked; the
// thread's 16 types after the clean-up in lo / hi, its count of listed entries returned
__device__ __forceinline__ int vis_count_chunk(const VisArgs& v, TfDevState* __restrict__ st,
                                               unsigned char* __restrict__ visType, int* __restrict__ allocCounts,
                                               unsigned char* __restrict__ swapState, unsigned long long& lo_out,
                                               unsigned long long& hi_out)
{
    if (threadIdx.x == 0) {
        // this frame's allocation is done: its chunk counters go back to zero for the next
        // frame's requests, and (without exhaustion) the free-list counters drop by the totals
        allocCounts[2 * blockIdx.x] = 0;
        allocCounts[2 * blockIdx.x + 1] = 0;
        if (blockIdx.x == 0) {
            // the counters drop by the successful requests (failed ones restored them, :378, :400-401)
            const int f1 = st->alloc_fail[0], f2 = st->alloc_fail[1];
            st->lastFreeBlockId -= st->pad_[0] - f1 - f2;
            st->lastFreeExcessListId -= st->pad_[1] - f2;
            st->tot_alloc_fail1 += f1;
            st->tot_alloc_fail2 += f2;
        }
    }
    const int base = blockIdx.x * CHUNK + threadIdx.x * 16;
    int cnt = 0;
    lo_out = 0; hi_out = 0;
    if (base < v.n_total) {
        unsigned long long lo, hi;
        load16(visType + base, &lo, &hi);
        bool dirty = false;
        for (int i = 0; i < 16; ++i) {
            unsigned t = byte16(lo, hi, i);
            if (t == 4) {              // type 3 that failed checkBlockVisibility (k_set_type3)
                if (i < 8) lo &= ~(0xffull << (8 * i)); else hi &= ~(0xffull << (8 * (i - 8)));
                t = 0;
                dirty = true;
            }
            cnt += t > 0;
        }
        lo_out = lo; hi_out = hi;
        if (dirty) *(uint4*)(visType + base) = make_uint4((unsigned)lo, (unsigned)(lo >> 32), (unsigned)hi, (unsigned)(hi >> 32));
        if (swapState) {
            // buildVisibleList_device<true> (SceneReconstructionEngine_host.cu:466-469): every
            // listed entry not already in active memory (state 2) becomes "needed" (1)
            unsigned long long slo, shi;
            load16(swapState + base, &slo, &shi);
            bool sdirty = false;
            for (int i = 0; i < 16; ++i) {
                if (byte16(lo, hi, i) > 0 && byte16(slo, shi, i) != 2 && byte16(slo, shi, i) != 1) {
                    if (i < 8) slo = (slo & ~(0xffull << (8 * i))) | (1ull << (8 * i));
                    else shi = (shi & ~(0xffull << (8 * (i - 8)))) | (1ull << (8 * (i - 8)));
                    sdirty = true;
                }
            }
            if (sdirty) *(uint4*)(swapState + base) = make_uint4((unsigned)slo, (unsigned)(slo >> 32), (unsigned)shi, (unsigned)(shi >> 32));
        }
    }
    return cnt;
}

__global__ void __launch_bounds__(256)
k_vis_count(VisArgs v, TfDevState* __restrict__ st, const TfHashEntry* __restrict__ hash,
            unsigned char* __restrict__ visType, int* __restrict__ counts, int* __restrict__ allocCounts,
            unsigned char* __restrict__ swapState)
{
    if (st->abort) return;
    unsigned long long lo, hi;
    const int cnt = vis_count_chunk(v, st, visType, allocCounts, swapState, lo, hi);
    int tot = block_sum(cnt);
    if (threadIdx.x == 0) counts[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(256)
k_vis_apply(VisArgs v, TfDevState* __restrict__ st, int n_chunks, const int* __restrict__ counts,
            const unsigned char* __restrict__ visType, int* __restrict__ visibleIds)
{
    if (st->abort) return;
    // this chunk's types, loaded before (and in flight with) the counts prefix
    const int base = blockIdx.x * CHUNK + threadIdx.x * 16;
    unsigned long long lo = 0, hi = 0;
    if (base < v.n_total) load16(visType + base, &lo, &hi);
    int pre = 0, all = 0;
    for (int h = threadIdx.x; h < n_chunks; h += 256) {
        int c = counts[h];
        all += c;
        if (h < (int)blockIdx.x) pre += c;
    }
    pre = block_sum(pre); all = block_sum(all);
    if (blockIdx.x == 0 && threadIdx.x == 0) st->noVisibleEntries = all < v.cap ? all : v.cap;
    int cnt = 0;
    if (base < v.n_total)
        for (int i = 0; i < 16; ++i) cnt += byte16(lo, hi, i) > 0;
    int tmp;
    int r = pre + block_excl_scan(cnt, &tmp);
    if (!cnt) return;
    for (int i = 0; i < 16; ++i) {
        if (byte16(lo, hi, i) > 0) {
            if (r < v.cap) visibleIds[r] = base + i;
            r++;
        }
    }
}

// k_vis_count + k_vis_apply in one launch: each workgroup counts its chunk, publishes the count
// tagged with this launch's generation (agent scope: the readers are on every XCD), waits for
// the counts of every lower chunk and compacts its own entries at their sum -- the same list in
// the same order.  A workgroup waits only on lower-indexed ones, which were dispatched before it,
// so the wait always ends; a bounded spin still turns a lost count into the frame's sticky error.
// The last workgroup, which has waited on all the others, writes noVisibleEntries.
__global__ void __launch_bounds__(256)
k_vis_build(VisArgs v, TfDevState* __restrict__ st, unsigned char* __restrict__ visType,
            int* __restrict__ allocCounts, unsigned char* __restrict__ swapState, unsigned long long* __restrict__ agg,
            unsigned gen, int* __restrict__ visibleIds, int fault)
{
    if (st->abort) return;
    unsigned long long lo, hi;
    const int cnt = vis_count_chunk(v, st, visType, allocCounts, swapState, lo, hi);
    int own;
    int r = block_excl_scan(cnt, &own);
    if (threadIdx.x == 0)
        __hip_atomic_store(&agg[blockIdx.x], ((unsigned long long)gen << 32) | (unsigned)own, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    int pre = 0;
    bool lost = fault && blockIdx.x == gridDim.x - 1;   // TFUSION_VIS_FAULT (tests): the last chunk's wait fails
    for (int h = threadIdx.x; h < (int)blockIdx.x; h += 256) {
        unsigned long long x;
        unsigned spins = 0;
        while (((x = __hip_atomic_load(&agg[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >> 32) != gen) {
            if (++spins > (1u << 22)) { lost = true; break; }
            __builtin_amdgcn_s_sleep(1);
        }
        pre += (int)(unsigned)x;
    }
    pre = block_sum(pre);
    if (__syncthreads_or(lost)) {
        if (threadIdx.x == 0) {
            st->icp_ok = -2;                             // a frame's end turns this into frame_ok -3
            st->sticky_error = 1;                        // engine-level calls have no frame end
        }
        return;
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {
        const int all = pre + own;
        st->noVisibleEntries = all < v.cap ? all : v.cap;
    }
    if (!cnt) return;
    r += pre;
    for (int i = 0; i < 16; ++i) {
        if (byte16(lo, hi, i) > 0) {
            if (r < v.cap) visibleIds[r] = blockIdx.x * CHUNK + threadIdx.x * 16 + i;
            r++;
        }
    }
}

static AllocArgs make_alloc_args(tf_ctx* c)
{
    AllocArgs a;
    a.dists = c->dists; a.W = c->W; a.H = c->H;
    a.invfx = 1.0f / c->p.fx; a.invfy = 1.0f / c->p.fy; a.cx = c->p.cx; a.cy = c->p.cy;
    a.mu = c->p.mu;
    a.oneOverVoxelSize = 1.0f / (c->p.voxelSize * (float)TF_BLK);      // SceneReconstructionEngine_host.cu:138
    a.vf_min = c->p.viewFrustum_min; a.vf_max = c->p.viewFrustum_max;
    a.mask = (unsigned)(c->p.n_buckets - 1);
    a.n_buckets = c->p.n_buckets;
    a.grid = c->bgrid;
    return a;
}

// AllocateSceneFromDepth (SceneReconstructionEngine_host.cu:75-195) with the matrices
// already in st->M_alloc / st->invM_alloc
hipError_t tfk_alloc(tf_ctx* c, int snapshot, TfAhead bil, size_t pitch, int only_update)
{
    AllocArgs a = make_alloc_args(c);
    VisArgs v;
    v.fx = c->p.fx; v.fy = c->p.fy; v.cx = c->p.cx; v.cy = c->p.cy;
    v.factor = (float)TF_BLK * c->p.voxelSize;
    v.W = c->W; v.H = c->H; v.n_total = c->n_total; v.cap = c->p.vis_capacity;
    // swapping (SceneReconstructionEngine_host.cu:159-160, never with onlyUpdateVisibleList):
    // the enlarged frustum for the previous list, swap states marked, swapped-out entries reallocated
    const bool swapping = c->p.use_swapping && !only_update;
    v.enlarged = swapping ? 1 : 0;
    if (snapshot != 2)   // 2: the frame's ICP launch has done it (tfk_icp fold_t3)
        hipLaunchKernelGGL(k_set_type3, dim3(256), dim3(256), 0, c->stream, v, c->st, c->hash, c->visibleIds, c->visType,
                           (const float2*)c->range, snapshot ? (float2*)c->range_render : nullptr);
    const int gx = (c->W + 15) / 16, n_alloc = gx * ((c->H + 15) / 16);
    BilArgs nb; PyrArgs np;
    int n_next = 0, next_gx = 1;
    if (bil.src) {
        const hipError_t e = tf_pre_args(c, bil.src, pitch, 1, bil.d0, &nb, &np);
        if (e != hipSuccess) return e;
        next_gx = tf_div_up(c->W, PRE_TX);
        n_next = next_gx * tf_div_up(c->H, PRE_TY);
    } else nb = BilArgs{};
    hipLaunchKernelGGL(k_alloc_requests, dim3(n_alloc + n_next), dim3(256), 0, c->stream,
                       a, c->st, c->hash, c->allocType, c->visType, c->winnerKey, c->allocCounts, gx, n_alloc, nb, next_gx);
    if (only_update)   // allocateVoxelBlocksList_device is skipped (SceneReconstructionEngine_host.cu:162-168)
        hipLaunchKernelGGL(k_alloc_discard, dim3(c->alloc_chunks), dim3(256), 0, c->stream, c->st, c->allocCounts,
                           c->allocType, c->winnerKey, c->n_total);
    else
        hipLaunchKernelGGL(k_alloc_apply, dim3(c->alloc_chunks), dim3(256), 0, c->stream, a, c->st, c->alloc_chunks,
                           c->allocCounts, c->allocType, c->winnerKey, c->hash, c->visType, c->allocList, c->excessList,
                           c->n_total);
    if (c->vis_fused) {
        hipLaunchKernelGGL(k_vis_build, dim3(c->vis_chunks), dim3(256), 0, c->stream, v, c->st, c->visType,
                           c->allocCounts, swapping ? c->swapState : nullptr, c->visAgg, ++c->vis_gen, c->visibleIds,
                           (int)(++c->vis_launches == c->vis_fault_launch));
    } else {
        hipLaunchKernelGGL(k_vis_count, dim3(c->vis_chunks), dim3(256), 0, c->stream, v, c->st, c->hash, c->visType,
                           c->visCounts, c->allocCounts, swapping ? c->swapState : nullptr);
        hipLaunchKernelGGL(k_vis_apply, dim3(c->vis_chunks), dim3(256), 0, c->stream, v, c->st, c->vis_chunks,
                           c->visCounts, c->visType, c->visibleIds);
    }
    if (swapping) return tfk_swap_realloc(c);      // reAllocateSwappedOutVoxelBlocks (:184-189)
    if (c->p.use_swapping)                         // (an onlyUpdateVisibleList pass reallocates nothing)
        return hipMemsetAsync(&c->st->swap_realloc, 0, sizeof(int), c->stream);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// integrateIntoScene_device<Voxel_s,false> (SceneReconstructionEngine_host.cu:297-329) +
// computeUpdatedVoxelDepthInfo (SceneReconstructionEngine.hpp:23-71).
// 128 lanes per 8^3 block, 4 consecutive voxels (16 B) per lane; blocks grid-strided.
// ---------------------------------------------------------------------------------------
#ifndef TF_INTEG_DIV
#define TF_INTEG_DIV 0
#endif
struct IntegArgs {
    const float* dists;
    int W, H;
    float fx, fy, cx, cy;
    float voxelSize, mu;
    float inv_mu;                       // RN(1/mu) when mu_exact3 (eta / mu in three operations)
    int mu_exact3;
    int maxW;
    // frame 0 of the device-driven frame: prev_ = curr_ (topfu.cpp:205 swaps the pyramids;
    // copying keeps the buffer pointers fixed); levels contiguous, n_maps float4 per map
    const float4* curr_pts; const float4* curr_nrm; float4* prev_pts; float4* prev_nrm;
    int n_maps;
    // colour (voxel_rgb with a frame RGB image): computeUpdatedVoxelColorInfo on the colour plane
    const uchar4* rgb; size_t rgb_pitch;
    unsigned* vba_rgb;
    float rfx, rfy, rcx, rcy;           // projParams_rgb
    float D[16];                        // calib_inv (depth -> rgb) as a column-major Matrix4f
    // engine batches (k_fuse_tail): the frame's world -> camera pose [R|t] as given (so the pass
    // does not read st->M_alloc, which the next frame's begin rewrites in the same grid) and the
    // integration workgroups of the grid
    const float* pose_rt;
    int fuse_nwg;
};

// computeUpdatedVoxelDepthInfo (SceneReconstructionEngine.hpp:23-71) in two halves, so that
// a lane's eight voxels (two blocks) project first, their eight depth loads go out together,
// and the updates follow -- a depth load under the projection's early returns is a branch,
// and eight of them in a row were eight round trips.  integ_project: false when the voxel
// projects behind the camera or outside [1, W-2] x [1, H-2]; else its depth-image index.
__device__ __forceinline__ bool integ_project(float px, float py, float pz, const float* M, const IntegArgs& a,
                                              float* z, int* idx)
{
    float pc[3];
    tf_m4v3(M, px, py, pz, 1.0f, pc);
    *z = pc[2];
    if (pc[2] <= 0) return false;
    // projParams_d.x * pt_camera.x / pt_camera.z (SceneReconstructionEngine.hpp:35-36), built with
    // --prec-div=false (CMakeLists.txt:1): the quotient as a product with the reciprocal -- canonical
    // (fx x) RN(1/z), one reciprocal per voxel for both coordinates (round 5; it was (fx x) / z)
#if TF_INTEG_DIV                                   // A/B only: the IEEE quotients (not the oracle's)
    float ix = a.fx * pc[0] / pc[2] + a.cx;
    float iy = a.fy * pc[1] / pc[2] + a.cy;
#else
    const float rz = tf_rcp_rn(pc[2]);
    float ix = (a.fx * pc[0]) * rz + a.cx;
    float iy = (a.fy * pc[1]) * rz + a.cy;
#endif
    if ((ix < 1) || (ix > (float)(a.W - 2)) || (iy < 1) || (iy > (float)(a.H - 2))) return false;
    *idx = (int)(ix + 0.5f) + (int)(iy + 0.5f) * a.W;
    return true;
}
// *eta_r: computeUpdatedVoxelDepthInfo's return value (eta, or -1 for no depth)
__device__ __forceinline__ unsigned integ_update(unsigned vox, float depth_measure, float z, const IntegArgs& a,
                                                 const float* rw, float* eta_r)
{
    *eta_r = -1.0f;
    if (depth_measure <= 0.0f) return vox;
    float eta = depth_measure - z;
    *eta_r = eta;
    if (eta < -a.mu) return vox;
    short sdf = (short)(vox & 0xffff);
    int oldW = (vox >> 16) & 0xff;
    float oldF = tf_short_to_float(sdf);          // == (float)sdf / 32767.0f, exactly
    float newF = a.mu_exact3 ? tf_div_exact3(eta, a.mu, a.inv_mu) : eta / a.mu;
    newF = (1.0f < newF) ? 1.0f : newF;
    newF = (float)oldW * oldF + 1.0f * newF;
    int newW = oldW + 1;
    newF = tf_div_exact3(newF, (float)newW, rw[newW - 1]);     // newW in 1..256
    newW = (newW < a.maxW) ? newW : a.maxW;
    short nsdf = (short)(newF * 32767.0f);
    return ((unsigned)(unsigned short)nsdf) | ((unsigned)(newW & 0xff) << 16) | (vox & 0xff000000u);
}

// ComputeUpdatedVoxelInfo<true, ...>'s gate (SceneReconstructionEngine.hpp:173): colour only
// unless (eta > mu) || (fabs(eta / mu) > 0.25f).  |eta| > mu fails it whatever the rounding, so
// the division runs only inside the band.
__device__ __forceinline__ bool integ_colour_gate(float eta, const IntegArgs& a)
{
    if (!(fabsf(eta) <= a.mu)) return false;
    const float q = a.mu_exact3 ? tf_div_exact3(eta, a.mu, a.inv_mu) : eta / a.mu;
    return !(fabsf(q) > 0.25f);
}

// Vector3f::toUChar: CLAMP((int)ROUND(v), 0, 255) (Vector.hpp:242-244, MathUtils.hpp:20)
__device__ __forceinline__ unsigned integ_u8(float v)
{
    const int i = (int)((v < 0) ? (v - 0.5f) : (v + 0.5f));
    return (unsigned)(i < 0 ? 0 : (i > 255 ? 255 : i));
}

// computeUpdatedVoxelColorInfo (SceneReconstructionEngine.hpp:116-148) on one colour word
// (r | g << 8 | b << 16 | w << 24) with interpolateBilinear (PixelUtils.hpp:8-32) of the RGB image;
// canonical arithmetic.  A NaN image position (pc.z == 0: undefined in the reference) is skipped.
// its two halves: the image position and the four bilinear samples (issued, not waited for),
// then the running average once they have arrived.  Every sample of an in-image position is in
// bounds (x0 <= W - 2, y0 <= H - 2), so the four loads are unconditional and a zero weight
// selects the reference's zero sample instead.
struct IntegRgbTap {
    uchar4 A, B, C, D;
    float dx, dy;
    bool ok;
};
__device__ __forceinline__ void integ_colour_fetch(float px, float py, float pz, const float* Mr, const IntegArgs& a,
                                                   IntegRgbTap& t)
{
    float pc[3];
    tf_m4v3(Mr, px, py, pz, 1.0f, pc);
    const float rz = tf_rcp_rn(pc[2]);                 // (SceneReconstructionEngine.hpp:132-133, as integ_project)
    const float ix = (a.rfx * pc[0]) * rz + a.rcx;
    const float iy = (a.rfy * pc[1]) * rz + a.rcy;
    t.ok = ix >= 1 && ix <= (float)(a.W - 2) && iy >= 1 && iy <= (float)(a.H - 2);
    const int x0 = t.ok ? (int)floorf(ix) : 1, y0 = t.ok ? (int)floorf(iy) : 1;
    t.dx = ix - (float)x0; t.dy = iy - (float)y0;
    const uchar4* r0 = (const uchar4*)((const char*)a.rgb + (size_t)y0 * a.rgb_pitch);
    const uchar4* r1 = (const uchar4*)((const char*)r0 + a.rgb_pitch);
    t.A = r0[x0]; t.B = r0[x0 + 1]; t.C = r1[x0]; t.D = r1[x0 + 1];
}
__device__ __forceinline__ unsigned integ_colour_apply(unsigned clr, const IntegRgbTap& t, const IntegArgs& a)
{
    if (!t.ok) return clr;
    const float dx = t.dx, dy = t.dy;
    const uchar4 z4 = make_uchar4(0, 0, 0, 0);
    const uchar4 A = t.A;
    const uchar4 B = (dx != 0) ? t.B : z4;
    const uchar4 C = (dy != 0) ? t.C : z4;
    const uchar4 D = (dx != 0 && dy != 0) ? t.D : z4;
    const float oldW = (float)(clr >> 24);
    const float ax = 1.0f - dx, ay = 1.0f - dy;
    const float av[3] = { (float)A.x, (float)A.y, (float)A.z }, bv[3] = { (float)B.x, (float)B.y, (float)B.z };
    const float cv[3] = { (float)C.x, (float)C.y, (float)C.z }, dv[3] = { (float)D.x, (float)D.y, (float)D.z };
    const float newW = oldW + 1.0f;
    float mw = (float)(unsigned char)a.maxW;
    const float wout = (newW < mw) ? newW : mw;
    unsigned out = (unsigned)(unsigned char)wout << 24;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float oldC = (float)((clr >> (8 * k)) & 0xffu) / 255.0f;
        float m = av[k] * ax * ay + bv[k] * dx * ay + cv[k] * ax * dy + dv[k] * dx * dy;
        m = m / 255.0f;
        float nc = oldC * oldW + m * 1.0f;
        nc = nc / newW;
        out |= integ_u8(nc * 255.0f) << (8 * k);
    }
    return out;
}

typedef unsigned int tf_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 nt_load16(const uint4* p)
{
    const tf_u32x4 r = __builtin_nontemporal_load(reinterpret_cast<const tf_u32x4*>(p));
    return make_uint4(r.x, r.y, r.z, r.w);
}
__device__ __forceinline__ void nt_store16(uint4* p, uint4 v)
{
    tf_u32x4 r = { v.x, v.y, v.z, v.w };
    __builtin_nontemporal_store(r, reinterpret_cast<tf_u32x4*>(p));
}

// projection half: the eight voxels' camera z, depth-image index and "projects inside" flag
__device__ __forceinline__ void integ_proj_pair(const TfHashEntry& e, const TfHashEntry& e2, int vx, int vy, int vz,
                                                const float* M, const IntegArgs& a, float (&z)[8], int (&di)[8],
                                                bool (&ok)[8])
{
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        const TfHashEntry& h = b ? e2 : e;
        const int gx = h.x * TF_BLK, gy = h.y * TF_BLK, gz = h.z * TF_BLK;
        const float py = (float)(gy + vy) * a.voxelSize, pz = (float)(gz + vz) * a.voxelSize;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            int idx = 0;
            ok[4 * b + k] = h.ptr >= 0 && integ_project((float)(gx + vx + k) * a.voxelSize, py, pz, M, a, &z[4 * b + k], &idx);
            di[4 * b + k] = ok[4 * b + k] ? idx : 0;
        }
    }
}

// TF_C3X (diagnostic builds only, tools/build_variant.sh; never the product, results wrong):
// bit 0 -- every depth sample reads pixel 0 (no depth-image traffic); bit 1 -- no voxel loads
// (each lane starts from an empty voxel); bits 2 / 3 -- samples rounded down to 16 B / 128 B.  C3I's reads split by source with PMC FETCH_SIZE.
#ifndef TF_C3X
#define TF_C3X 0
#endif
#ifndef TF_INTEG_LANEMAP
#define TF_INTEG_LANEMAP 1
#endif
__device__ __forceinline__ float integ_sample(const float* dists, int di)
{
    if (TF_C3X & 4) di &= ~3;           // (diagnostic: 16-byte aligned: lanes of a segment share an address)
    if (TF_C3X & 8) di &= ~31;          // (diagnostic: 128-byte line starts: the same lines, fewer addresses)
    return dists[(TF_C3X & 1) ? 0 : di];
}
__device__ __forceinline__ void integ_vload(uint4* p, uint4* p2, bool stream, uint4& v, uint4& v2)
{
    if (TF_C3X & 2) { v = make_uint4(0, 0, 0, 0); v2 = v; return; }
    if (stream) { v = nt_load16(p); v2 = nt_load16(p2); }
    else { v = *p; v2 = *p2; }
}

// update half: the eight voxels against their depth samples dm, stores of the changed lanes,
// then (RGB) the colour of the voxels inside the colour gate
template <bool RGB>
__device__ __forceinline__ void integ_apply_pair(uint4 v, uint4 v2, const float (&dm)[8], const float (&z)[8],
                                                 const bool (&ok)[8], const TfHashEntry& e, const TfHashEntry& e2,
                                                 int vx, int vy, int vz, const IntegArgs& a, uint4* p, uint4* p2,
                                                 const float* rw, bool stream, const float* Mr, int lin, int* n_rd,
                                                 int* n_wr)
{
    unsigned w[8] = { v.x, v.y, v.z, v.w, v2.x, v2.y, v2.z, v2.w };
    float eta[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        eta[k] = -1.0f;
        if (ok[k]) w[k] = integ_update(w[k], dm[k], z[k], a, rw, &eta[k]);
    }
    // a lane whose four voxels all kept their value (behind the surface by more than mu, outside
    // the image, no depth) stores nothing: at HBM scale most of a frustum lies behind the surface.
    // (The voxels are still read up front, with the depth samples: skipping the reads of such
    // lanes would put a second dependent round trip on every lane, slower on the C3I scene.)
    const bool ch1 = e.ptr >= 0 && ((w[0] ^ v.x) | (w[1] ^ v.y) | (w[2] ^ v.z) | (w[3] ^ v.w)) != 0;
    const bool ch2 = e2.ptr >= 0 && ((w[4] ^ v2.x) | (w[5] ^ v2.y) | (w[6] ^ v2.z) | (w[7] ^ v2.w)) != 0;
    *n_rd += (int)(e.ptr >= 0) + (int)(e2.ptr >= 0);
    *n_wr += (int)ch1 + (int)ch2;
    if (stream) {
        if (ch1) nt_store16(p, make_uint4(w[0], w[1], w[2], w[3]));
        if (ch2) nt_store16(p2, make_uint4(w[4], w[5], w[6], w[7]));
    } else {
        if (ch1) *p = make_uint4(w[0], w[1], w[2], w[3]);
        if (ch2) *p2 = make_uint4(w[4], w[5], w[6], w[7]);
    }
    if (RGB) {
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            const TfHashEntry& h = b ? e2 : e;
            if (h.ptr < 0) continue;
            unsigned gate = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) gate |= (integ_colour_gate(eta[4 * b + k], a) ? 1u : 0u) << k;
            if (!gate) continue;                   // most lanes: no voxel in the colour band
            uint4* cp = (uint4*)(a.vba_rgb + (size_t)h.ptr * TF_BLK3 + lin);
            const uint4 c4 = *cp;
            const int gx = h.x * TF_BLK, gy = h.y * TF_BLK, gz = h.z * TF_BLK;
            const float py = (float)(gy + vy) * a.voxelSize, pz = (float)(gz + vz) * a.voxelSize;
            // the colour word and every gated voxel's samples in flight together: one round
            // trip per block, not one per voxel
            IntegRgbTap tap[4];
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (gate & (1u << k)) integ_colour_fetch((float)(gx + vx + k) * a.voxelSize, py, pz, Mr, a, tap[k]);
            unsigned cw[4] = { c4.x, c4.y, c4.z, c4.w };
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (gate & (1u << k)) cw[k] = integ_colour_apply(cw[k], tap[k], a);
            *cp = make_uint4(cw[0], cw[1], cw[2], cw[3]);
        }
    }
}

template <bool WITH_ED, bool RGB, bool FUSED = false>
__device__ __forceinline__ void integ_body(IntegArgs a, TfDevState* __restrict__ st, const TfHashEntry* __restrict__ hash,
                                           const int* __restrict__ visibleIds, TfVoxel* __restrict__ vba, EdArgs ed,
                                           long long* __restrict__ cnt);
#ifdef TF_INTEG_TIMELINE
// diagnostic builds only (tools/integ_timeline.py): per workgroup of the last frame-path integrate
// launch, [start, end] on the 100 MHz clock
__device__ unsigned long long tf_integ_tl[4096 * 2];
extern "C" int tf_debug_integ_timeline(void* host, size_t bytes)
{
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(tf_integ_tl), bytes < sizeof(tf_integ_tl) ? bytes : sizeof(tf_integ_tl), 0,
                                    hipMemcpyDeviceToHost);
}
#endif
template <bool WITH_ED, bool RGB>
__global__ void __launch_bounds__(256)
k_integrate(IntegArgs a, TfDevState* __restrict__ st, const TfHashEntry* __restrict__ hash,
            const int* __restrict__ visibleIds, TfVoxel* __restrict__ vba, EdArgs ed, long long* __restrict__ cnt)
{
#ifdef TF_INTEG_TIMELINE
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    integ_body<WITH_ED, RGB>(a, st, hash, visibleIds, vba, ed, cnt);
    __syncthreads();
    if (WITH_ED && threadIdx.x == 0 && blockIdx.x < 4096) {
        tf_integ_tl[2 * blockIdx.x] = t0;
        tf_integ_tl[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
    }
#else
    integ_body<WITH_ED, RGB>(a, st, hash, visibleIds, vba, ed, cnt);
#endif
}
// the frame path with the colour TSDF: its own register budget (TF_INTEG_RGB_WAVES waves per
// SIMD), so that the frame grid's workgroups are resident together
#ifndef TF_INTEG_RGB_WAVES
#define TF_INTEG_RGB_WAVES 3
#endif
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(TF_INTEG_RGB_WAVES)))
k_integrate_rgb(IntegArgs a, TfDevState* __restrict__ st, const TfHashEntry* __restrict__ hash,
                const int* __restrict__ visibleIds, TfVoxel* __restrict__ vba, EdArgs ed, long long* __restrict__ cnt)
{
    integ_body<true, true>(a, st, hash, visibleIds, vba, ed, cnt);
}
// the stand-alone depth-only pass (stage entry points, C3I): its own register budget, so that
// TF_INTEG_PASS_WAVES waves per SIMD are resident on a list of millions of blocks
#ifndef TF_INTEG_PASS_WAVES
#define TF_INTEG_PASS_WAVES 5
#endif
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(TF_INTEG_PASS_WAVES)))
k_integrate_pass(IntegArgs a, TfDevState* __restrict__ st, const TfHashEntry* __restrict__ hash,
                 const int* __restrict__ visibleIds, TfVoxel* __restrict__ vba, EdArgs ed, long long* __restrict__ cnt)
{
    integ_body<false, false>(a, st, hash, visibleIds, vba, ed, cnt);
}
template <bool WITH_ED, bool RGB, bool FUSED>
__device__ __forceinline__ void integ_body(IntegArgs a, TfDevState* __restrict__ st, const TfHashEntry* __restrict__ hash,
                                           const int* __restrict__ visibleIds, TfVoxel* __restrict__ vba, EdArgs ed,
                                           long long* __restrict__ cnt)
{
    // WITH_ED: the first TF_ED_BLOCKS workgroups run CreateExpectedDepths' projection pass (it
    // reads only the visible list and the pose; integration writes only voxels): one launch
    // and its dispatch gap fewer per frame.  The stand-alone instance (stage entry points, C3I)
    // has no such branch: its grid-stride loop is the plain one.
    int bid = blockIdx.x, nblk = FUSED ? a.fuse_nwg : (int)gridDim.x;
    if (WITH_ED) {
        if (bid < TF_ED_BLOCKS) { ed_project_block(ed, st, bid, TF_ED_BLOCKS); return; }
        bid -= TF_ED_BLOCKS; nblk -= TF_ED_BLOCKS;
    }
    __shared__ float rw[256];                    // RN(1/w), w = 1..256: the running average's divisors
    rw[threadIdx.x] = 1.0f / (float)(threadIdx.x + 1);
    __syncthreads();
    if (st->abort) return;
    if (a.n_maps > 0 && st->mode == 0) {
        const int stride = nblk * 256;
        for (int k = bid * 256 + threadIdx.x; k < a.n_maps; k += stride) {
            a.prev_pts[k] = a.curr_pts[k];
            a.prev_nrm[k] = a.curr_nrm[k];
        }
    }
    const int n = st->noVisibleEntries;
    // a pass over more blocks than the L2s hold streams the voxels non-temporally (so they do
    // not evict the depth image every voxel samples); a frame's few hundred blocks stay
    // cached for the raycasts that read them next
    const bool stream = n > TF_INTEG_STREAM_BLOCKS;
    float M[16];
    if (FUSED) {
        tf_rt_to_m4(a.pose_rt, M);               // M_alloc of a given world -> camera pose (alloc_mode 2)
    } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) M[i] = st->M_alloc[i];
    }
    // M_rgb = calib_inv * M_d (SceneReconstructionEngine_host.cu:217), Matrix4 operator*
    // (Matrix.hpp:113-119): r(x, y) += lhs(k, y) * rhs(x, k) from zero
    float Mr[16];
    if (RGB) {
#pragma unroll
        for (int x = 0; x < 4; ++x)
#pragma unroll
            for (int y = 0; y < 4; ++y) {
                float r = 0.0f;
#pragma unroll
                for (int k = 0; k < 4; ++k) r += a.D[4 * k + y] * M[4 * x + k];
                Mr[4 * x + y] = r;
            }
    }
    const int half = threadIdx.x >> 7, t = threadIdx.x & 127;
    // a lane's four voxels: x in {0..3} or {4..7} of one (y, z) row of the block.  Each wave takes
    // four y rows of all eight z layers (TF_INTEG_LANEMAP 1) -- not eight y rows of four layers: a
    // depth-sample instruction then spans half the image rows, and the samples' L1 -> L2 line
    // fetches, not the voxel stream, are what the pass waits on (profiles/r05/c3i_read_attribution.json)
#if TF_INTEG_LANEMAP
    const int vx = (t & 1) * 4, vy = ((t >> 1) & 3) | ((t >> 6) << 2), vz = (t >> 3) & 7;
    const int lin = vx + 8 * vy + 64 * vz;
#else
    const int lin = t * 4;                       // first voxel of this lane: x in {0,4}
    const int vx = lin & 7, vy = (lin >> 3) & 7, vz = lin >> 6;
#endif
    // two blocks per half-workgroup per pass, their id / entry / voxel loads issued before
    // either is computed: twice the bytes in flight per wave (at C3 scale, 2^21 blocks, the
    // pass is a stream over 8.6 GB)
    const int stride = nblk * 2;
    int n_rd = 0, n_wr = 0;
    // Software pipeline over the grid-stride passes, three deep: pass k projects pass k+1's
    // voxels (its entries arrived during pass k-1) and issues their voxel loads and depth
    // samples, issues pass k+2's entry loads and pass k+3's id loads, and only then updates pass
    // k's voxels, whose loads were issued a whole update earlier.  Loads past the list read its
    // last element (valid memory; the results are discarded).
    const int step = 2 * stride;
    int i = bid * 2 + half;
    if (i < n) {
        TfHashEntry e, e2, ne, ne2;
        int nid1, nid2;
        {
            const int id1 = visibleIds[i], id2 = visibleIds[min(i + stride, n - 1)];
            const int n1 = visibleIds[min(i + step, n - 1)], n2 = visibleIds[min(i + step + stride, n - 1)];
            nid1 = visibleIds[min(i + 2 * step, n - 1)]; nid2 = visibleIds[min(i + 2 * step + stride, n - 1)];
            e = hash[id1]; e2 = hash[id2];
            ne = hash[n1]; ne2 = hash[n2];
        }
        if (!(i + stride < n)) e2.ptr = -1;
        float z[8], dm[8];
        bool ok[8];
        uint4 v, v2;
        uint4* p = (uint4*)(vba + (size_t)(e.ptr < 0 ? 0 : e.ptr) * TF_BLK3 + lin);
        uint4* p2 = (uint4*)(vba + (size_t)(e2.ptr < 0 ? 0 : e2.ptr) * TF_BLK3 + lin);
        {
            int di[8];
            integ_vload(p, p2, stream, v, v2);
            integ_proj_pair(e, e2, vx, vy, vz, M, a, z, di, ok);
#pragma unroll
            for (int k = 0; k < 8; ++k) dm[k] = integ_sample(a.dists, di[k]);
        }
        for (; i < n; i += step) {
            // pass k+1: project, issue its voxel loads and depth samples
            const int in = i + step;
            if (!(in + stride < n)) ne2.ptr = -1;
            if (!(in < n)) ne.ptr = -1;
            float zn[8], dmn[8];
            bool okn[8];
            uint4 vn, vn2;
            uint4* pn = (uint4*)(vba + (size_t)(ne.ptr < 0 ? 0 : ne.ptr) * TF_BLK3 + lin);
            uint4* pn2 = (uint4*)(vba + (size_t)(ne2.ptr < 0 ? 0 : ne2.ptr) * TF_BLK3 + lin);
            {
                int di[8];
                integ_vload(pn, pn2, stream, vn, vn2);
                integ_proj_pair(ne, ne2, vx, vy, vz, M, a, zn, di, okn);
#pragma unroll
                for (int k = 0; k < 8; ++k) dmn[k] = integ_sample(a.dists, di[k]);
            }
            // pass k+2's entries, pass k+3's ids
            const TfHashEntry nne = hash[nid1], nne2 = hash[nid2];
            const int nn1 = visibleIds[min(i + 3 * step, n - 1)], nn2 = visibleIds[min(i + 3 * step + stride, n - 1)];
            // pass k: update
            integ_apply_pair<RGB>(v, v2, dm, z, ok, e, e2, vx, vy, vz, a, p, p2, rw, stream || TF_INTEG_NT_STORES, Mr, lin, &n_rd, &n_wr);
            e = ne; e2 = ne2; ne = nne; ne2 = nne2; nid1 = nn1; nid2 = nn2;
            v = vn; v2 = vn2; p = pn; p2 = pn2;
#pragma unroll
            for (int k = 0; k < 8; ++k) { z[k] = zn[k]; dm[k] = dmn[k]; ok[k] = okn[k]; }
        }
    }
    // lanes read / written (profiling / stand-alone passes): the workgroup's running counts in
    // its own slot, plain read-modify-write (launches on one stream; no atomics to contend)
    if (!cnt) return;
    __shared__ int wsum[2][4];
    const int wv = threadIdx.x >> 6;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) { n_rd += __shfl_xor(n_rd, o, 64); n_wr += __shfl_xor(n_wr, o, 64); }
    if ((threadIdx.x & 63) == 0) { wsum[0][wv] = n_rd; wsum[1][wv] = n_wr; }
    __syncthreads();
    if (threadIdx.x == 0) {
        cnt[2 * bid] += (long long)wsum[0][0] + wsum[0][1] + wsum[0][2] + wsum[0][3];
        cnt[2 * bid + 1] += (long long)wsum[1][0] + wsum[1][1] + wsum[1][2] + wsum[1][3];
    }
}

// ---------------------------------------------------------------------------------------
// Engine-level batches (tf_scene_fuse_frames, tf_fuse.hip), four launches per frame.  Frame
// k+1's head -- computeDists of its raw depth into the other dists buffer, its pose matrices, and
// setToType3 over frame k's visible list with frame k+1's visibility test (k_set_type3) --
// shares no data with frame k's IntegrateIntoScene (voxels, read-only list and hash, frame k's
// dists and pose passed as arguments) nor with frame k's record (counters no head writes), so all
// three run in one grid: k_fuse_tail.  The allocation launches then need no head of their own.
// ---------------------------------------------------------------------------------------
struct FuseNext {
    const uint16_t* frame;              // frame k+1's raw depth (nullptr: no next frame)
    size_t pitch;
    float* dists;                       // -> its dists buffer
    const float* pose;                  // its world -> camera pose [R|t]
    int dg_x, n_dists;                  // 16x16 dists tiles
};

// setToType3 with the frame's own visibility test, computeDists, and (workgroup 0) the frame's
// matrices and flags (k_fuse_begin, tf_fuse.hip); b in [0, 256 + n_dists)
__device__ __forceinline__ void fuse_head_part(int b, const FuseNext& f, const VisArgs& v, TfDevState* __restrict__ st,
                                               const TfHashEntry* __restrict__ hash, const int* __restrict__ visibleIds,
                                               unsigned char* __restrict__ visType)
{
    if (b < 256) {
        float pose[12];
#pragma unroll
        for (int i = 0; i < 12; ++i) pose[i] = f.pose[i];
        // (only a frame end writes halt; sticky_error: an engine batch's failed wait, k_vis_build --
        // every later frame of the batch no-ops, and the abort written here equals the one the
        // failing frame's own head wrote unless that frame ran, so the write cannot change what a
        // concurrent reader in this grid sees)
        const int halted = st->halt | st->sticky_error;
        if (b == 0 && threadIdx.x == 0) {
            tf_set_pose_matrices(st, pose, 2);
            st->abort = halted ? 1 : 0;
            st->mode = 1;
        }
        if (halted) return;
        float M[16];
        tf_rt_to_m4(pose, M);
        set_type3_pass(v, st->noVisibleEntries, M, hash, visibleIds, visType, b * 256 + threadIdx.x, 256 * 256);
        return;
    }
    b -= 256;
    const int x = (b % f.dg_x) * 16 + (threadIdx.x & 15), y = (b / f.dg_x) * 16 + (threadIdx.x >> 4);
    if (x >= v.W || y >= v.H) return;
    f.dists[y * v.W + x] = tf_dist_of(*(const uint16_t*)((const char*)f.frame + (size_t)y * f.pitch + (size_t)x * 2));
}

// the batch's first frame: its head alone
__global__ void __launch_bounds__(256)
k_fuse_head(FuseNext f, VisArgs v, TfDevState* __restrict__ st, const TfHashEntry* __restrict__ hash,
            const int* __restrict__ visibleIds, unsigned char* __restrict__ visType)
{
    fuse_head_part((int)blockIdx.x, f, v, st, hash, visibleIds, visType);
}

// frame k: IntegrateIntoScene (workgroups [0, a.fuse_nwg)), its record (tf_fuse_record, the next
// workgroup), then frame k+1's head
__global__ void __launch_bounds__(256)
k_fuse_tail(IntegArgs a, TfDevState* __restrict__ st, const TfHashEntry* __restrict__ hash,
            const int* __restrict__ visibleIds, TfVoxel* __restrict__ vba, long long* __restrict__ cnt,
            int* __restrict__ rec, FuseNext f, VisArgs v, unsigned char* __restrict__ visType)
{
    const int b = (int)blockIdx.x;
    if (b < a.fuse_nwg) {
        // frame k's visible list failed to build (sticky_error, written by its k_vis_build launch,
        // ordered before this one): no integration over it
        if (st->sticky_error) return;
        integ_body<false, false, true>(a, st, hash, visibleIds, vba, EdArgs{}, cnt);
        return;
    }
    if (b == a.fuse_nwg) {
        if (threadIdx.x == 0) {
            rec[0] = st->lastFreeBlockId;
            rec[1] = st->lastFreeExcessListId;
            rec[2] = st->noVisibleEntries;
            rec[3] = st->alloc_fail[0];
            rec[4] = st->alloc_fail[1];
            rec[5] = rec[6] = rec[7] = rec[8] = rec[9] = 0;           // (no swapping on this path)
        }
        return;
    }
    fuse_head_part(b - a.fuse_nwg - 1, f, v, st, hash, visibleIds, visType);
}

static VisArgs make_vis_args(tf_ctx* c)
{
    VisArgs v;
    v.fx = c->p.fx; v.fy = c->p.fy; v.cx = c->p.cx; v.cy = c->p.cy;
    v.factor = (float)TF_BLK * c->p.voxelSize;
    v.W = c->W; v.H = c->H; v.n_total = c->n_total; v.cap = c->p.vis_capacity;
    v.enlarged = 0;
    return v;
}

static FuseNext make_fuse_next(tf_ctx* c, const uint16_t* frame, size_t pitch, float* dists, const float* pose)
{
    FuseNext f;
    f.frame = frame; f.pitch = pitch; f.dists = dists; f.pose = pose;
    f.dg_x = (c->W + 15) / 16;
    f.n_dists = frame ? f.dg_x * ((c->H + 15) / 16) : 0;
    return f;
}

static IntegArgs make_integ_args(tf_ctx* c, int frame_path);

hipError_t tfk_fuse_head(tf_ctx* c, const uint16_t* frame, size_t pitch, float* dists, const float* pose)
{
    const FuseNext f = make_fuse_next(c, frame, pitch, dists, pose);
    hipLaunchKernelGGL(k_fuse_head, dim3(256 + f.n_dists), dim3(256), 0, c->stream, f, make_vis_args(c), c->st, c->hash,
                       c->visibleIds, c->visType);
    return hipGetLastError();
}

// frame k (its dists in c->dists, its pose `pose`, record `rec`) + frame k+1's head (next_frame
// nullptr: none)
hipError_t tfk_fuse_tail(tf_ctx* c, const float* pose, int* rec, const uint16_t* next_frame, size_t pitch,
                         float* next_dists, const float* next_pose)
{
    IntegArgs a = make_integ_args(c, 0);
    a.pose_rt = pose;
    a.fuse_nwg = c->integ_wg_frame;
    const FuseNext f = make_fuse_next(c, next_frame, pitch, next_dists, next_pose);
    const int nwg = a.fuse_nwg + 1 + (next_frame ? 256 + f.n_dists : 0);
    hipLaunchKernelGGL(k_fuse_tail, dim3(nwg), dim3(256), 0, c->stream, a, c->st, c->hash, c->visibleIds, c->vba,
                       c->integ_cnt, rec, f, make_vis_args(c), c->visType);
    return hipGetLastError();
}

static IntegArgs make_integ_args(tf_ctx* c, int frame_path)
{
    IntegArgs a;
    a.curr_pts = c->curr_pts[0]; a.curr_nrm = c->curr_nrm[0]; a.prev_pts = c->prev_pts[0]; a.prev_nrm = c->prev_nrm[0];
    a.n_maps = 0;
    if (frame_path)
        for (int l = 0; l < TF_LEVELS; ++l) a.n_maps += c->lw[l] * c->lh[l];
    a.dists = c->dists; a.W = c->W; a.H = c->H;
    a.fx = c->p.fx; a.fy = c->p.fy; a.cx = c->p.cx; a.cy = c->p.cy;
    a.voxelSize = c->p.voxelSize; a.mu = c->p.mu; a.maxW = c->p.maxW;
    a.inv_mu = 1.0f / c->p.mu; a.mu_exact3 = c->mu_exact3;
    a.rgb = c->rgb_cur; a.rgb_pitch = c->rgb_pitch; a.vba_rgb = c->vba_rgb;
    const float* q = c->p.rgb_intr;
    const bool depth_intr = q[0] == 0 && q[1] == 0 && q[2] == 0 && q[3] == 0;   // rgb_intr all 0
    a.rfx = depth_intr ? c->p.fx : q[0]; a.rfy = depth_intr ? c->p.fy : q[1];
    a.rcx = depth_intr ? c->p.cx : q[2]; a.rcy = depth_intr ? c->p.cy : q[3];
    const float* d = c->p.depth_to_rgb;          // row-major [R|t] -> column-major Matrix4f
    for (int col = 0; col < 4; ++col)
        for (int row = 0; row < 4; ++row)
            a.D[4 * col + row] = row < 3 ? d[4 * row + col] : (col == 3 ? 1.0f : 0.0f);
    a.pose_rt = nullptr;
    a.fuse_nwg = 0;
    return a;
}

hipError_t tfk_integrate(tf_ctx* c, int frame_path, int with_ed)
{
    IntegArgs a = make_integ_args(c, frame_path);
    const bool rgb = c->p.voxel_rgb && c->rgb_cur;
    EdArgs ed = {};
    // stand-alone: 2560 workgroups, two rounds of the 5 per CU that k_integrate_pass's register
    // budget keeps resident (C3I 2.354 -> 2.317 ms against 2048 at 4 per CU; one round of exactly
    // the resident count: 2.43 ms; profiles/r04/ab_integ_pass_waves.txt)
    const int nwg = frame_path ? c->integ_wg_frame : TF_INTEG_WG;
    long long* count = (frame_path ? c->count_lanes : 1) ? c->integ_cnt : nullptr;
    const dim3 b(256);
    if (with_ed) {
        tf_ed_args(c, &ed);
        const dim3 ge(nwg + TF_ED_BLOCKS);
        if (rgb) tf_launch(c, k_integrate_rgb, ge, b, 0, a, c->st, c->hash, c->visibleIds, c->vba, ed, count);
        else tf_launch(c, k_integrate<true, false>, ge, b, 0, a, c->st, c->hash, c->visibleIds, c->vba, ed, count);
    } else {
        const dim3 g(nwg);
        if (rgb) tf_launch(c, k_integrate<false, true>, g, b, 0, a, c->st, c->hash, c->visibleIds, c->vba, ed, count);
        else tf_launch(c, k_integrate_pass, g, b, 0, a, c->st, c->hash, c->visibleIds, c->vba, ed, count);
    }
    return hipGetLastError();
}
