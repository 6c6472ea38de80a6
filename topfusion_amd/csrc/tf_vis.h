// tf_vis.h -- checkBlockVisibility<false> and setToType3 over the previous visible list, as
// shared by k_set_type3 (tf_scene.hip) and the tail of the persistent ICP kernel (tf_icp.hip),
// which runs them once the frame's pose is known.
#pragma once
#include "tf_internal.h"

// ---------------------------------------------------------------------------------------
// checkBlockVisibility<false> (SceneReconstructionEngine.hpp:300-375)
// ---------------------------------------------------------------------------------------
struct VisArgs {
    float fx, fy, cx, cy;
    float factor;                 // (float)SDF_BLOCK_SIZE * voxelSize
    int W, H;
    int n_total, cap;
    int enlarged;                 // swapping: checkPointVisibility<true>'s enlarged frustum
};

// isVisible, or with v.enlarged (swapping) isVisibleEnlarged: the image grown by an eighth of its
// size on every side, integer limits (SceneReconstructionEngine.hpp:315-321); a point inside the
// image is inside the enlarged frame too, so "any corner enlarged-visible" is the flag
__device__ __forceinline__ bool vis_point(const float* M, const float* pt, const VisArgs& v)
{
    float b[4];
    tf_m4v(M, pt[0], pt[1], pt[2], pt[3], b);
    if (b[2] < 1e-10f) return false;
    float bx = v.fx * b[0] / b[2] + v.cx;
    float by = v.fy * b[1] / b[2] + v.cy;
    if (v.enlarged) {
        const int lx = -v.W / 8, ux = v.W + v.W / 8, ly = -v.H / 8, uy = v.H + v.H / 8;
        return bx >= (float)lx && bx < (float)ux && by >= (float)ly && by < (float)uy;
    }
    return bx >= 0 && bx < (float)v.W && by >= 0 && by < (float)v.H;
}

__device__ __forceinline__ bool vis_block(const TfHashEntry& e, const float* M, const VisArgs& v)
{
    const float f = v.factor;
    float pt[4] = { (float)e.x * f, (float)e.y * f, (float)e.z * f, 1.0f };
    if (vis_point(M, pt, v)) return true;
    pt[2] += f; if (vis_point(M, pt, v)) return true;                     // 0 0 1
    pt[1] += f; if (vis_point(M, pt, v)) return true;                     // 0 1 1
    pt[0] += f; if (vis_point(M, pt, v)) return true;                     // 1 1 1
    pt[2] -= f; if (vis_point(M, pt, v)) return true;                     // 1 1 0
    pt[1] -= f; if (vis_point(M, pt, v)) return true;                     // 1 0 0
    pt[0] -= f; pt[1] += f; if (vis_point(M, pt, v)) return true;         // 0 1 0
    pt[0] += f; pt[1] -= f; pt[2] += f; if (vis_point(M, pt, v)) return true;  // 1 0 1
    return false;
}

// setToType3 (SceneReconstructionEngine_host.cu:343-348) with the visibility test of the
// entries still of type 3 (:449-476) already applied: 3 = visible, 4 = not (k_set_type3)
__device__ __forceinline__ void set_type3_pass(const VisArgs& v, int n, const float* M, const TfHashEntry* __restrict__ hash,
                                               const int* __restrict__ visibleIds, unsigned char* __restrict__ visType,
                                               int tid, int stride)
{
    for (int i = tid; i < n; i += stride) {
        const int id = visibleIds[i];
        visType[id] = vis_block(hash[id], M, v) ? 3 : 4;
    }
}
