// tf_reset.h -- ResetScene (SceneReconstructionEngine_host.cu:51-73) and the device-driven
// frame's end (topfu.cpp:209 / 263-264 / 329) as a workgroup-level device function, shared by
// k_reset_scene (tf_scene.hip) and the fused CreateICPMaps + frame-end launch (tf_render.hip).
#pragma once
#include "tf_internal.h"

struct ResetArgs {
    TfVoxel* vba; size_t n_vox;
    int* allocList; int n_blocks;
    TfHashEntry* hash; int n_total;
    int* excessList; int n_excess;
    TfDevState* st; int2* grid;
    int on_failure;                  // frame end: bookkeeping always, the reset only if ICP failed
    int* frame_ok; int* frame_mode; int slot;
    int full;                        // clear everything (else only what the frames wrote)
    unsigned char* swapState;        // swapping: GlobalCache states / stored flags, cleared with a reset
    unsigned char* swapFlags;
    unsigned* vba_rgb;               // voxel_rgb: the colour plane, cleared with its blocks (Voxel_s_rgb(): 0)
    int* ed_bin_cnt; int ed_nbins;   // frame end: CreateExpectedDepths' bins emptied (the fused fill and the
    unsigned* ed_done;               // ICP tiles that read them are done), its done counter cleared
};

// Runs as workgroup `bid` of `nblk` (256 threads): its own launch (k_reset_scene) or the
// trailing workgroups of the frame's k_icp_maps grid (tf_render.hip, k_icp_maps_end).
__device__ __forceinline__ void reset_scene_block(const ResetArgs& r, int bid, int nblk)
{
    TfVoxel* vba = r.vba; const size_t n_vox = r.n_vox; int* allocList = r.allocList; const int n_blocks = r.n_blocks;
    TfHashEntry* hash = r.hash; const int n_total = r.n_total; int* excessList = r.excessList;
    const int n_excess = r.n_excess; TfDevState* st = r.st; int2* grid = r.grid; const int on_failure = r.on_failure;
    // a full clear when forced (ResetScene entry point) or when the host wrote scene state since
    // the last full reset (tf_upload / tf_set_counters); the last workgroup drops that flag
    const int full = r.full || st->scene_external;
    if (on_failure && bid == 0 && threadIdx.x == 0) {
        // end of the device-driven frame (return values of topfu.cpp:209 / 264 / 329); only
        // frame_counter / n_resets / pose change here, never the mode / icp_ok read below
        const int mode = st->mode, icp_ok = st->icp_ok;
        int ok;
        if (st->halt) ok = -2;                              // skipped: an earlier frame of the batch failed
        else if (mode == 0) { st->frame_counter = 1; ok = 1; }
        else if (icp_ok == -1) {                            // the persistent ICP lost a peer: nothing past the
            ok = -1;                                        // ICP ran, the host re-runs the frame (fallback)
            st->halt = 1;
        } else if (icp_ok < -1) {                           // a later stage's bounded spin timed out: the
            ok = -3;                                        // frame is half done, the context is in error
            st->halt = 1;
            st->sticky_error = 1;
        } else if (icp_ok == 0) {                           // return reset(), false
            st->n_resets++;
            st->frame_counter = 0;
            for (int i = 0; i < 12; ++i) st->pose[i] = (i % 5 == 0) ? 1.0f : 0.0f;
            ok = 0;
        } else { st->frame_counter++; ok = 1; }
        if (ok >= 0) st->tot_frames++;
        if (ok == 0) st->tot_resets++;
        if (ok == 1) st->tot_visible += st->noVisibleEntries;      // the list this frame integrated
        if (ok == 1 && mode == 1) { st->tot_tracked++; st->tot_tiles += st->noTotalBlocks; }
        r.frame_ok[r.slot] = ok;
        r.frame_mode[r.slot] = mode;
    }
    if (on_failure && bid == 0 && r.ed_bin_cnt) {
        for (int k = threadIdx.x; k < r.ed_nbins; k += 256) r.ed_bin_cnt[k] = 0;
        if (threadIdx.x == 0) *r.ed_done = 0u;
    }
    if (on_failure && !(st->mode == 1 && st->icp_ok == 0)) return;   // topfu.cpp:263-264 only
    const size_t tid = (size_t)bid * 256 + threadIdx.x;
    const size_t stride = (size_t)nblk * 256;
    uint4 vfill = make_uint4(32767u, 32767u, 32767u, 32767u);   // Voxel_s(): sdf 32767, w 0
    uint4* v4 = (uint4*)vba;
    uint4* c4 = (uint4*)r.vba_rgb;
    const uint4 cfill = make_uint4(0, 0, 0, 0);
    TfHashEntry e; e.x = e.y = e.z = e.pad = 0; e.offset = 0; e.ptr = -2;
    if (full) {
        for (size_t i = tid; i < n_vox / 4; i += stride) v4[i] = vfill;
        if (c4)
            for (size_t i = tid; i < n_vox / 4; i += stride) c4[i] = cfill;
        for (size_t i = tid; i < (size_t)n_blocks; i += stride) allocList[i] = (int)i;
        for (size_t i = tid; i < (size_t)n_excess; i += stride) excessList[i] = (int)i;
    } else {
        // Same end state from what the frames wrote since the last full reset: allocation only
        // pops the free lists (never writes them) and integration only writes blocks it was
        // handed, so the blocks in use -- allocList[lastFreeBlockId+1 .. n_blocks-1] -- are the
        // only ones not at Voxel_s(), and the free lists are still the identity.
        const int first = st->lastFreeBlockId + 1 < 0 ? 0 : st->lastFreeBlockId + 1;
        const size_t n_used4 = (size_t)(n_blocks - first) * (TF_BLK3 / 4);
        for (size_t i0 = tid; i0 < n_used4; i0 += 8 * stride) {   // 8 list loads in flight per lane
            int blk[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const size_t i = i0 + k * stride;
                blk[k] = allocList[first + (int)((i < n_used4 ? i : i0) / (TF_BLK3 / 4))];
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const size_t i = i0 + k * stride;
                if (i < n_used4) {
                    const size_t o = (size_t)blk[k] * (TF_BLK3 / 4) + i % (TF_BLK3 / 4);
                    v4[o] = vfill;
                    if (c4) c4[o] = cfill;
                }
            }
        }
    }
    if (r.swapState) {                       // the GlobalCache of the old scene goes with it
        for (size_t i = tid; i < (size_t)n_total / 16; i += stride) {
            ((uint4*)r.swapState)[i] = make_uint4(0, 0, 0, 0);
            ((uint4*)r.swapFlags)[i] = make_uint4(0, 0, 0, 0);
        }
    }
    for (size_t i0 = tid; i0 < (size_t)n_total; i0 += 8 * stride) {   // 8 entry loads in flight per lane
        TfHashEntry o[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const size_t i = i0 + k * stride;
            o[k] = hash[i < (size_t)n_total ? i : i0];
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const size_t i = i0 + k * stride;
            // live entries (only they differ from e)
            if (i < (size_t)n_total && (full || o[k].ptr >= 0)) {
                if (o[k].ptr >= 0 && tf_grid_in(o[k].x, o[k].y, o[k].z))   // (swapped-out entries have no cell)
                    grid[tf_grid_cell(o[k].x, o[k].y, o[k].z)] = make_int2(-1, TF_VOFF_NONE);
                hash[i] = e;
            }
        }
    }
    // the counters are reset by the last workgroup to finish (every workgroup has read
    // lastFreeBlockId by then)
    __shared__ int last_s;
    __syncthreads();
    if (threadIdx.x == 0) last_s = atomicAdd(&st->reset_ticket, 1u) == (unsigned)nblk - 1;
    __syncthreads();
    if (last_s && threadIdx.x == 0) {
        st->reset_ticket = 0;
        st->scene_external = 0;
        st->swap_in = 0; st->swap_out = 0; st->swap_realloc = 0;   // a reset frame transfers nothing
        st->lastFreeBlockId = n_blocks - 1;
        st->lastFreeExcessListId = n_excess - 1;
    }
}


// on_failure = 0: ResetScene now (full); 1: the frame end of batch slot `slot`
void tf_reset_args(tf_ctx* c, ResetArgs* r, int on_failure, int slot, int clear_cache);
