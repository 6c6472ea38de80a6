// tf_fuse.hip -- engine-level fusion of a device-resident batch of frames at given poses
// (tf_scene_fuse_frames), for gfx950.
//
// TopFu's call order without the tracker (topfu.cpp:166, 202-203): per frame computeDists on the
// raw depth, AllocateSceneFromDepth and IntegrateIntoScene at the frame's pose, and, in a
// swapping scene, the swapping engine.  These are the launches of the per-call engine entry
// points (tf_scene_alloc / tf_scene_integrate / tf_scene_swap) with the host round trips taken
// out: the frame's dists and pose matrices come from one leading launch that reads the depth
// frame and the pose list on the device, and one trailing one-thread launch writes the frame's
// counters into the batch's record list.  This is the C5 hash-stress driver (capacity
// saturation, silent allocation failure, eviction churn), so the frames carry no ICP and no
// frame-mixing resets.
#include <utility>

#include "tf_internal.h"
#include "tf_preproc.h"

// computeDists (imgproc.cu:263-290) of frame k into the context's dists, and (workgroup 0) the
// frame's pose -> the allocation / integration matrices, as tf_scene_alloc's k_pose_from_input
// with TF_POSE_ALLOC_NOINV (the pose is world -> camera, used as is)
__global__ void __launch_bounds__(256)
k_fuse_begin(const uint16_t* __restrict__ frame, size_t pitch, int W, int H, float* __restrict__ dists,
             const float* __restrict__ pose, TfDevState* __restrict__ st)
{
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
        float p[12];
        for (int i = 0; i < 12; ++i) p[i] = pose[i];
        tf_set_pose_matrices(st, p, 2);
        st->abort = st->halt ? 1 : 0;   // a halted context (an earlier frame failed on the device): the frame no-ops
        st->mode = 1;
    }
    const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= W || y >= H) return;
    dists[y * W + x] = tf_dist_of(*(const uint16_t*)((const char*)frame + (size_t)y * pitch + (size_t)x * 2));
}

// the frame's record (tf_fuse_record, include/tfusion_hip.h)
__global__ void k_fuse_record(const TfDevState* __restrict__ st, int* __restrict__ rec, int swapping)
{
    rec[0] = st->lastFreeBlockId;
    rec[1] = st->lastFreeExcessListId;
    rec[2] = st->noVisibleEntries;
    rec[3] = st->alloc_fail[0];
    rec[4] = st->alloc_fail[1];
    rec[5] = swapping ? st->swap_in : 0;
    rec[6] = swapping ? st->swap_out : 0;
    rec[7] = swapping ? st->swap_realloc : 0;
    rec[8] = swapping ? st->swap_merged : 0;
    rec[9] = 0;
}

hipError_t tfk_fuse_frames(tf_ctx* c, const uint16_t* frames, size_t stride, size_t pitch, int n)
{
    static_assert(sizeof(tf_fuse_record) == 10 * sizeof(int), "tf_fuse_record layout");
    const dim3 dg((c->W + 15) / 16, (c->H + 15) / 16);
    const int swapping = c->p.use_swapping ? 1 : 0;
    if (!swapping && c->fuse_tail && n > 0) {
        // four launches per frame: requests, apply, visible list, then k_fuse_tail -- frame k's
        // integration and record beside frame k+1's head (dists into the other buffer, matrices,
        // setToType3); the batch's first head alone before them.  c->dists alternates between the
        // two buffers and ends on the last frame's.
        if (!c->fuse_dists) {
            const hipError_t e = hipMalloc((void**)&c->fuse_dists, sizeof(float) * (size_t)c->W * c->H);
            if (e != hipSuccess) { c->fuse_dists = nullptr; return e; }
        }
        hipError_t e = tfk_fuse_head(c, frames, pitch, c->dists, c->fuse_pose);
        for (int k = 0; k < n && e == hipSuccess; ++k) {
            e = tfk_alloc(c, 2);                         // (setToType3 ran in the head)
            if (e != hipSuccess) break;
            const bool more = k + 1 < n;
            const uint16_t* nf = more ? (const uint16_t*)((const char*)frames + (size_t)(k + 1) * stride) : nullptr;
            e = tfk_fuse_tail(c, c->fuse_pose + 12 * (size_t)k, c->fuse_rec + 10 * (size_t)k, nf, pitch, c->fuse_dists,
                              more ? c->fuse_pose + 12 * (size_t)(k + 1) : nullptr);
            if (more) std::swap(c->dists, c->fuse_dists);
        }
        return e != hipSuccess ? e : hipGetLastError();
    }
    for (int k = 0; k < n; ++k) {
        const uint16_t* f = (const uint16_t*)((const char*)frames + (size_t)k * stride);
        hipLaunchKernelGGL(k_fuse_begin, dg, dim3(256), 0, c->stream, f, pitch, c->W, c->H, c->dists,
                           c->fuse_pose + 12 * (size_t)k, c->st);
        hipError_t e = tfk_alloc(c);                    // AllocateSceneFromDepth (+ reallocation when swapping)
        if (e == hipSuccess) e = tfk_integrate(c);      // IntegrateIntoScene
        if (e == hipSuccess && swapping) e = tfk_swap(c, 3);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k_fuse_record, dim3(1), dim3(1), 0, c->stream, c->st, c->fuse_rec + 10 * (size_t)k, swapping);
    }
    return hipGetLastError();
}
