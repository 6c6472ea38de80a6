// tf_pose.h -- device-side pose algebra shared by several kernels (cv::Affine3f *, inv;
// InfiniTAM Matrix4::inv) and the derived per-frame matrices; plus the frame-begin logic of
// the device-driven TopFu::operator() (tf_capi.hip).
#pragma once
#include "tf_internal.h"

// cv::Affine3f operator* (float rigid composition): out = a * b
static __device__ __attribute__((unused)) void tf_rigid_mul(const float* a, const float* b, float* out)
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
static __device__ __attribute__((unused)) void tf_rigid_inv(const float* a, float* out)
{
    float o[12];
    for (int j = 0; j < 3; ++j) {
        for (int i = 0; i < 3; ++i) o[j * 4 + i] = a[i * 4 + j];
        o[j * 4 + 3] = -((a[0 * 4 + j] * a[3] + a[1 * 4 + j] * a[7]) + a[2 * 4 + j] * a[11]);
    }
    for (int i = 0; i < 12; ++i) out[i] = o[i];
}

// Matrix4::inv (Matrix.hpp:173-233)
static __device__ __attribute__((unused)) void tf_matrix4_inv(const float* mm, float* dst)
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
static __device__ __attribute__((unused)) void tf_set_pose_matrices(TfDevState* st, const float* pose, int alloc_mode)
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



// start of a device-driven frame (topfu.cpp:161-209): branch on frame_counter_, reset the
// per-frame flags; frame 0 uses poses_.back() as is for allocation / integration
static __device__ __attribute__((unused)) void tf_frame_begin(TfDevState* st)
{
    st->abort = st->halt ? 1 : 0;       // a halted batch (tf_reset.h): every stage of the frame no-ops
    st->mode = st->frame_counter == 0 ? 0 : 1;
    st->icp_ok = 1;
    st->icp_iters = 0;
    if (st->mode == 0) {
        float pose[12];
        for (int i = 0; i < 12; ++i) pose[i] = st->pose[i];
        tf_set_pose_matrices(st, pose, 2);
    }
}
