// tf_ed.h -- CreateExpectedDepths' projection pass (VisualisationEngine_CUDA.cu:119-173) as a
// workgroup-level device function, shared by k_ed_project (tf_render.hip) and the leading
// workgroups of k_integrate (tf_scene.hip), which run it beside integration.
#pragma once
#include "tf_internal.h"

struct EdArgs {
    const TfHashEntry* hash;
    const int* visibleIds;
    float2* range;
    uint4* rec;          // per visible entry: ulx | uly << 16, lrx | lry << 16, zmin, zmax bits (x ~0u: none)
    int* tiles; int* off; int* chunk;
    int2* spill;         // per fill row: extent of the pixels the last fill wrote outside the /8 region
    uint4* bins;         // [2 * nrows][lds_max_n] binned boxes (ed_bin_pack): row r's, then row r's
                         // share of the boxes reaching below the LDS rows (entry index % nrows == r)
    int* bin_cnt;        // [2 * nrows] entries in each bin (the fill's workgroup r zeroes its two)
    int keep_bins;       // the fill leaves the counts (tf_time_stage's repeated fills)
    unsigned* done;      // fill fused into k_raycast_pair: its atomic path counts finished rows here
    int W, H;
    int rc, rr;          // the /8 region: (W-1)/8+1 columns, (H-1)/8+1 rows
    int nrows;           // k_ed_fill's LDS rows (ed_nrows: rr + ED_XROWS, at most H)
    int lds_max_n;       // k_ed_fill's LDS-row path up to this many visible entries
    int vcap, nchunk_max;   // box / chunk-total buffer lengths (k_ed_fill's early loads)
    int fault;           // fault injection (tests): the ICP tiles' wait on the fill's atomic path fails
    float fx, fy, cx, cy, voxelSize;
    unsigned cap;
};

#define ED_CHUNK 256     // visible entries per projection chunk (one workgroup pass)
#define ED_MAX_ROWS 520  // k_ed_fill LDS rows for H <= 4096 (ed_nrows); binning needs W, H <= 4096 (tf_create)

// a binned box: its /8 pixel box (12 bits per coordinate), the visible-list index (16 bits, the
// MAX_RENDERING_BLOCKS check) and the z range -- everything the fill reads in one 16-byte load
__device__ __forceinline__ uint4 ed_bin_pack(unsigned ulx, unsigned uly, unsigned lrx, unsigned lry, unsigned i,
                                             unsigned zmin, unsigned zmax)
{
    return make_uint4(ulx | uly << 12 | (i & 0xffu) << 24, lrx | lry << 12 | (i >> 8) << 24, zmin, zmax);
}

// memsetKernel(FAR_AWAY, VERY_CLOSE) + ProjectSingleBlock (VisualisationEngine_Shared.hpp:33-77).
// Visible entries are processed in chunks of 256 (thread t of a chunk pass = entry
// chunk*256 + t).  Each chunk stores its tile total and every entry its exclusive tile offset
// inside the chunk, so the MAX_RENDERING_BLOCKS cap (VisualisationHelper.cu:70-74) is applied
// by k_ed_fill from plain prefix sums: no counter atomics, no last-workgroup ticket, no fence.
// Runs as workgroup `bid` of `nblk`: its own launch (k_ed_project) or the leading workgroups
// of k_integrate's grid (the stages share no data: both only read the visible list).
__device__ __forceinline__ void ed_project_block(const EdArgs& a, const TfDevState* __restrict__ st, int bid, int nblk)
{
    if (st->abort || st->mode == 0) return;          // ICP failed, or frame 0 (no rendering)
    const int tid = bid * 256 + threadIdx.x, stride = nblk * 256;
    // memsetKernel(FAR_AWAY, VERY_CLOSE) over the whole buffer (VisualisationEngine_CUDA.cu:133),
    // restated by what differs from it.  k_ed_fill writes every pixel of the /8 region castRay
    // reads (rc x rr, its LDS rows) with plain stores, so only two parts are written here:
    //  - the pixels the previous fill wrote outside that region (boxes are clamped to the
    //    full-resolution W-1 / H-1, VisualisationEngine_Shared.hpp:67-70): the extents its rows
    //    recorded in a.spill, or the whole buffer after creation / a host upload;
    //  - the /8 region itself when the fill will take its atomic path (n > a.lds_max_n).
    const int n = st->noVisibleEntries;
    {
        __shared__ int sxy[2];
        if (threadIdx.x < 2) sxy[threadIdx.x] = 0;
        __syncthreads();
        int sx = 0, sy = 0;
        for (int r = threadIdx.x; r < a.nrows; r += 256) { const int2 e = a.spill[r]; sx = max(sx, e.x); sy = max(sy, e.y); }
        if (sx) atomicMax(&sxy[0], sx);
        if (sy) atomicMax(&sxy[1], sy);
        __syncthreads();
        const int SX = sxy[0], SY = sxy[1];
        const float2 init = make_float2(TF_FAR_AWAY, TF_VERY_CLOSE);
        if (n > a.lds_max_n)
            for (int i = tid; i < a.rc * a.rr; i += stride) {
                const int y = i / a.rc, x = i - y * a.rc;
                a.range[x + y * a.W] = init;
            }
        if (SX > 0 && SY > 0) {
            if (SX >= a.W && SY >= a.H) {                  // whole buffer, two pixels per 16-byte store
                const int npx = a.W * a.H;
                float4* r4 = (float4*)a.range;
                for (int i = tid; i < (npx >> 1); i += stride) r4[i] = make_float4(init.x, init.y, init.x, init.y);
                if ((npx & 1) && tid == 0) a.range[npx - 1] = init;
            } else {
                for (int i = tid; i < SX * SY; i += stride) {
                    const int y = i / SX, x = i - y * SX;
                    if (x >= a.rc || y >= a.rr) a.range[x + y * a.W] = init;
                }
            }
        }
    }
    __shared__ int wsum[4];
    // binning (n <= lds_max_n): every valid box goes into the bin of each LDS row it covers, and
    // into a "below" bin when it reaches past the LDS rows, so the fill's row workgroup reads its
    // own boxes instead of scanning the whole list.  Counts are aggregated per chunk in LDS (one
    // device atomic per bin and chunk); the order inside a bin is arbitrary -- the fill reduces
    // with min / max only, so its result does not depend on it.
    __shared__ int lcnt[2 * ED_MAX_ROWS], gbase[2 * ED_MAX_ROWS];
    const bool binning = a.lds_max_n > 0 && n <= a.lds_max_n;   // (no bins when lds_max_n is 0)
    const int nb2 = 2 * a.nrows;
    if (binning)
        for (int r = threadIdx.x; r < nb2; r += 256) lcnt[r] = 0;
    const int nchunks = (n + ED_CHUNK - 1) / ED_CHUNK;
    const float* M = st->M_alloc;          // pose.inv() (topfu.cpp:306)
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int ch = bid; ch < nchunks; ch += nblk) {
        const int i = ch * ED_CHUNK + threadIdx.x;
        int ntiles = 0;
        if (i < n) {
            TfHashEntry e = a.hash[a.visibleIds[i]];
            uint4 rec = make_uint4(0xffffffffu, 0xffffffffu, 0u, 0u);
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
                    rec = make_uint4((unsigned)ulx | (unsigned)uly << 16, (unsigned)lrx | (unsigned)lry << 16,
                                     __float_as_uint(zmin), __float_as_uint(zmax));
                }
            }
            a.rec[i] = rec; a.tiles[i] = ntiles;
        }
        if (binning) {
            const uint4 rec = i < n ? a.rec[i] : make_uint4(0xffffffffu, 0u, 0u, 0u);   // (this thread's own store)
            const bool valid = rec.x != 0xffffffffu;
            const int uly = (int)(rec.x >> 16), lry = (int)(rec.y >> 16);
            const int r1 = lry < a.nrows - 1 ? lry : a.nrows - 1;
            const bool below = valid && lry >= a.nrows;
            const int bb = a.nrows + (i % a.nrows);
            if (valid)
                for (int r = uly; r <= r1; ++r) atomicAdd(&lcnt[r], 1);
            if (below) atomicAdd(&lcnt[bb], 1);
            __syncthreads();
            for (int r = threadIdx.x; r < nb2; r += 256) {
                const int c = lcnt[r];
                gbase[r] = c ? atomicAdd(&a.bin_cnt[r], c) : 0;
                lcnt[r] = 0;
            }
            __syncthreads();
            if (valid) {
                const uint4 e = ed_bin_pack(rec.x & 0xffffu, (unsigned)uly, rec.y & 0xffffu, (unsigned)lry, (unsigned)i,
                                            rec.z, rec.w);
                for (int r = uly; r <= r1; ++r) a.bins[(size_t)r * a.lds_max_n + gbase[r] + atomicAdd(&lcnt[r], 1)] = e;
                if (below) a.bins[(size_t)bb * a.lds_max_n + gbase[bb] + atomicAdd(&lcnt[bb], 1)] = e;
            }
            __syncthreads();
            for (int r = threadIdx.x; r < nb2; r += 256) lcnt[r] = 0;
        }
        // exclusive prefix of the tile counts inside the chunk (wave scan + 4 wave totals)
        int incl = ntiles;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            int v = __shfl_up(incl, d, 64);
            if (lane >= d) incl += v;
        }
        if (lane == 63) wsum[wv] = incl;
        __syncthreads();
        int base = 0;
        for (int w = 0; w < wv; ++w) base += wsum[w];
        if (i < n) a.off[i] = base + incl - ntiles;
        if (threadIdx.x == 0) a.chunk[ch] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
        __syncthreads();
    }
}


void tf_ed_args(tf_ctx* c, EdArgs* out);    // tf_render.hip: the context's expected-depth buffers
