/*
 * tfusion_hip.h -- C-ABI of libtfusion_hip.so, the MI355X (gfx950) implementation
 * of the topfusion hot path: depth preprocessing, projective point-to-plane ICP,
 * voxel-block-hash allocation, TSDF integration and raycasting.
 *
 * This is the drop-in boundary.  Plain pointers and sizes only; device pointers
 * are HIP device pointers on the context's device.  Every entry point replaces a
 * reference interface, cited as file:line relative to the 3d-scan/topfusion root.
 * The C++ mirror of the reference API (include/tfusion/topfu.hpp etc.) is a thin layer over
 * these functions; see INTEGRATION.md for the bindings.
 *
 * Error convention: every function returns a tf_status (0 = TF_OK).  The reference
 * prints and exit()s on CUDA errors (tfusion/src/device_memory.cpp:7-11,
 * tfusion/include/tfusion/cuda/CUDADefines.hpp:26-33); here the caller decides.
 * ICP degeneracy is TF_ICP_FAIL and triggers the same reset as the reference
 * (tfusion/src/topfu.cpp:263-264).
 *
 * Device-side failures.  The frame's stages wait on each other inside grids with bounded spins.
 * (1) The persistent ICP launch needs its 256 workgroups resident at once; if another process or
 * kernel holds part of the device, the launch ends with a lost peer.  Nothing past the ICP has
 * run then, and the frame is run again on the per-iteration ICP schedule (tf_totals::icp_fallbacks
 * counts it): the caller sees the frame's normal result.  (2) A bounded spin past the ICP that
 * times out leaves the frame half done: the context is in error from then on -- that frame's
 * call, or the next call that synchronises with the device if the frame's call had already
 * returned (per-call frames return on their ICP verdict), and every later call that
 * synchronises with the device (downloads, uploads, stage / engine / visualisation calls,
 * tf_scene_fuse_frames, stats and pose queries) returns TF_HIP_ERROR until tf_reset.  The same
 * holds for an engine-level call whose visible-list build loses a wait (k_vis_build), which has
 * no frame end to report it.  An engine batch on a context halted by a failed frame no-ops.
 */
#ifndef TFUSION_HIP_H
#define TFUSION_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum tf_status {
    TF_OK = 0,
    TF_ICP_FAIL = 1,        /* estimateTransform returned false; scene was reset */
    TF_INVALID_ARG = 2,
    TF_OOM = 3,
    TF_HIP_ERROR = 4,
    TF_NO_DEVICE = 5
} tf_status;

/* TopFuParams (tfusion/include/tfusion/topfu.hpp:28-60) restricted to the fields the
 * hot path reads, plus SceneParams (tfusion/include/tfusion/SceneParams.hpp:8-66)
 * and the reference's compile-time capacities made run-time. */
typedef struct tf_params {
    int   cols, rows;
    float fx, fy, cx, cy;               /* Intr */
    float bilateral_sigma_depth;        /* m */
    float bilateral_sigma_spatial;      /* px */
    int   bilateral_kernel_size;        /* px (7) */
    float icp_truncate_depth_dist;      /* m; <= 0 disables */
    float icp_dist_thres;               /* m */
    float icp_angle_thres;              /* rad */
    int   icp_iter_num[4];              /* per level 0..3 */
    float mu;                           /* TSDF truncation band (SceneParams::mu) */
    int   maxW;
    float voxelSize;                    /* m */
    float viewFrustum_min, viewFrustum_max;
    int   n_buckets;                    /* SDF_BUCKET_NUM, power of two (VoxelBlockHash.hpp:16) */
    int   n_excess;                     /* SDF_EXCESS_LIST_SIZE (VoxelBlockHash.hpp:18) */
    int   n_blocks;                     /* SDF_LOCAL_BLOCK_NUM (VoxelBlockHash.hpp:14) */
    int   vis_capacity;                 /* visibleEntryIDs capacity (RenderState_VH.hpp:42) */
    int   max_render_blocks;            /* MAX_RENDERING_BLOCKS (VisualisationEngine_Shared.hpp:5) */
    /* swapping: Scene(params, useSwapping) (scene.hpp:29-33) with its GlobalCache
       (GlobalCache.hpp:11-134), kept in HBM; TopFu itself runs without (topfu.cpp:67) */
    int   use_swapping;
    int   swap_transfer_blocks;         /* SDF_TRANSFER_BLOCK_NUM (VoxelBlockHash.hpp:27): blocks per swap */
    /* colour: Voxel_s_rgb voxels (VoxelTypes.hpp:39-67) integrated from the RGB image */
    int   voxel_rgb;                    /* 1: Voxel_s_rgb (colour integrated by the *_rgb entry points) */
    float rgb_intr[4];                  /* projParams_rgb (fx, fy, cx, cy); all 0: the depth intrinsics */
    float depth_to_rgb[12];             /* calib_inv of trafo_rgb_to_depth, row-major [R|t]: M_rgb = it * M_d */
} tf_params;

/* integer counters the reference keeps host-side (LocalVBA.hpp:26, VoxelBlockHash.hpp:69,
 * RenderState_VH.hpp:33, VisualisationEngine_CUDA.cu:160) plus ICP bookkeeping */
typedef struct tf_stats {
    int lastFreeBlockId;
    int lastFreeExcessListId;
    int noVisibleEntries;
    int noTotalBlocks;
    int frame_counter;
    int icp_iterations;                 /* iterations executed by the last estimateTransform */
    int icp_ok;
    int n_resets;
} tf_stats;

typedef struct tf_ctx tf_ctx;

/* buffer ids for tf_download / tf_upload (state inspection for parity tests) */
typedef enum tf_buffer {
    TF_BUF_HASH = 0,          /* HashEntry[n_buckets+n_excess], 16 B each (VoxelBlockHash.hpp:32-44) */
    TF_BUF_VBA = 1,           /* Voxel_s[n_blocks*512], 4 B each (VoxelTypes.hpp:69-92) */
    TF_BUF_VISIBLE_IDS = 2,   /* int[vis_capacity] */
    TF_BUF_VISIBLE_TYPE = 3,  /* uchar[n_buckets+n_excess] */
    TF_BUF_RANGE = 4,         /* float2[rows*cols]  renderingRangeImage */
    TF_BUF_RAYCAST = 5,       /* float4[rows*cols]  raycastResult */
    TF_BUF_DISTS = 6,         /* float[rows*cols] */
    TF_BUF_DEPTH = 7,         /* ushort[level]  filtered depth pyramid */
    TF_BUF_CURR_POINTS = 8,   /* float4[level] */
    TF_BUF_CURR_NORMALS = 9,
    TF_BUF_PREV_POINTS = 10,
    TF_BUF_PREV_NORMALS = 11,
    TF_BUF_GREY = 12,         /* uchar4[rows*cols] last renderImage output */
    TF_BUF_SWAP_STATE = 13,   /* uchar[n_buckets+n_excess] HashSwapState::state (GlobalCache.hpp:11-20) */
    TF_BUF_SWAP_STORED_FLAGS = 14,  /* uchar[n_buckets+n_excess] GlobalCache hasStoredData */
    TF_BUF_SWAP_STORED = 15,  /* Voxel_s[(n_buckets+n_excess)*512] GlobalCache storedVoxelBlocks */
    TF_BUF_VBA_RGB = 16,      /* voxel_rgb: uint32[n_blocks*512] Voxel_s_rgb clr + w_color (VoxelTypes.hpp:39-67),
                                 r | g << 8 | b << 16 | w_color << 24 -- the colour half of each voxel */
    TF_BUF_ALLOC_LIST = 17,   /* int[n_blocks] LocalVBA::allocationList, the free-block stack (LocalVBA.hpp:19, 35) */
    TF_BUF_EXCESS_LIST = 18   /* int[n_excess] VoxelBlockHash::excessAllocationList (VoxelBlockHash.hpp:81, 88) */
} tf_buffer;

/* ---- device ---------------------------------------------------------------- */
/* cuda::getCudaEnabledDeviceCount / setDevice (tfusion/include/tfusion/topfu.hpp:20-21) */
tf_status tf_device_count(int* count);
tf_status tf_set_device(int device);
const char* tf_status_string(tf_status s);

/* ---- context (TopFu) -------------------------------------------------------- */
/* TopFuParams::default_params (tfusion/src/topfu.cpp:12-53) */
tf_status tf_default_params(tf_params* p);
/* TopFu::TopFu (tfusion/src/topfu.cpp:55-84): allocates the scene, render state and
 * ICP buffers on the current device and creates one HIP stream. */
tf_status tf_create(const tf_params* p, tf_ctx** out);
void      tf_destroy(tf_ctx* ctx);
/* TopFu::reset (tfusion/src/topfu.cpp:141-152) */
tf_status tf_reset(tf_ctx* ctx);
/* TopFu::operator()(const cuda::Depth&) (tfusion/src/topfu.cpp:161-330).
 * dev_depth: uint16 millimetres, rows x cols, row pitch in bytes.
 * Returns TF_OK (true) or TF_ICP_FAIL (false, scene reset).  pose_out (optional):
 * getCameraPose() as a row-major 3x4 [R|t].  Returns as soon as the frame's result is known
 * (after its ICP), with its allocation, integration and raycasts still running on the context
 * stream -- the reference likewise returns with its last kernels in flight (topfu.cpp:307-329);
 * every later call that reads the state is ordered after them.  dev_depth has been consumed by
 * then.  stats (optional) waits for the whole frame; so do RGB frames and profiled contexts.
 * Deferred tail: the frame's last two launches (CreateICPMaps' raycast + renderImage, and
 * CreateICPMaps + the frame end) are not enqueued by this call but by the next tf_* call on the
 * context (the next frame's call carries that frame's preprocessing in them).  A caller that
 * synchronises the device or a stream itself must first call tf_get_stream(), which enqueues
 * them; every other entry point does it before its own work. */
tf_status tf_process_frame(tf_ctx* ctx, const uint16_t* dev_depth, size_t pitch_bytes,
                           float pose_out[12], tf_stats* stats);
/* same, host depth (cuda::Depth::upload, device_array.hpp; demo.cpp:100) */
tf_status tf_process_frame_host(tf_ctx* ctx, const uint16_t* host_depth, size_t pitch_bytes,
                                float pose_out[12], tf_stats* stats);
/* Runs n frames (frame i at dev_frames + i*frame_stride_bytes, pitch cols*2) with the
 * exact per-frame semantics of tf_process_frame, but without a host round trip per
 * frame.  ok_out (optional, n ints) receives each frame's bool. */
tf_status tf_process_frames(tf_ctx* ctx, const uint16_t* dev_frames, size_t frame_stride_bytes, int n,
                            int* ok_out);
/* TopFu::operator()(depth, image) (topfu.hpp:80) with the image integrated: with voxel_rgb set,
 * each frame's uchar4 RGB image (rows x cols, pitch bytes; registered to the depth through
 * rgb_intr / depth_to_rgb) updates the Voxel_s_rgb colour of the voxels near the surface
 * (computeUpdatedVoxelColorInfo, SceneReconstructionEngine.hpp:116-148, where the lineage's
 * ComputeUpdatedVoxelInfo<true, ...> calls it, :163-176).  dev_rgb null: as the depth-only call. */
tf_status tf_process_frame_rgb(tf_ctx* ctx, const uint16_t* dev_depth, size_t pitch_bytes, const uint8_t* dev_rgb,
                               size_t rgb_pitch_bytes, float pose_out[12], tf_stats* stats);
/* same, host depth and host RGB (uploaded through the context's staging buffers) */
tf_status tf_process_frame_rgb_host(tf_ctx* ctx, const uint16_t* host_depth, size_t pitch_bytes, const uint8_t* host_rgb,
                                    size_t rgb_pitch_bytes, float pose_out[12], tf_stats* stats);
/* the batch form: frame i's RGB image at dev_rgb_frames + i*rgb_stride_bytes (pitch cols*4) */
tf_status tf_process_frames_rgb(tf_ctx* ctx, const uint16_t* dev_frames, size_t frame_stride_bytes,
                                const uint8_t* dev_rgb_frames, size_t rgb_stride_bytes, int n, int* ok_out);
/* TopFu::renderImage (tfusion/src/topfu.cpp:332-377): raycast + grey shading of the
 * current pose into dev_rgba (uchar4, rows x cols, pitch bytes). */
tf_status tf_render_image(tf_ctx* ctx, uint8_t* dev_rgba, size_t pitch_bytes);
/* IVisualisationEngine::RenderImageType (tfusion/include/tfusion/VisualisationEngine.hpp:15-22) */
typedef enum tf_render_type {
    TF_RENDER_SHADED_GREYSCALE = 0,              /* renderGrey_device (SDF-gradient normals) */
    TF_RENDER_SHADED_GREYSCALE_IMAGENORMALS = 1, /* renderGrey_ImageNormals_device<false> (raycast-image normals) */
    TF_RENDER_COLOUR_FROM_VOLUME = 2,            /* renderColour_device with voxel_rgb; Voxel_s has no colour: greyscale
                                                    (VisualisationEngine_CUDA.cu:251-256) */
    TF_RENDER_COLOUR_FROM_NORMAL = 3,            /* renderColourFromNormal_device (alpha left as it was) */
    TF_RENDER_COLOUR_FROM_CONFIDENCE = 4         /* renderColourFromConfidence_device */
} tf_render_type;
/* VisualisationEngine_CUDA::RenderImage(scene, pose, intr, renderState, image, type,
 * RENDER_FROM_NEW_RAYCAST) (VisualisationEngine_CUDA.cu:220-291, 423-429) from poses_.back():
 * raycast with the current range image, then the type's pixel stage into the context's
 * image buffer (TF_BUF_GREY) and, when dev_rgba is non-null, a copy there. */
tf_status tf_render_image_type(tf_ctx* ctx, int type, uint8_t* dev_rgba, size_t pitch_bytes);
/* TopFu::getCameraPose (tfusion/src/topfu.cpp:154-159), time = -1 only */
tf_status tf_get_pose(tf_ctx* ctx, float rt[12]);
tf_status tf_get_stats(tf_ctx* ctx, tf_stats* stats);
tf_status tf_get_params(tf_ctx* ctx, tf_params* p);
/* HIP stream owned by the context (hipStream_t), for interop */
void*     tf_get_stream(tf_ctx* ctx);
/* execution schedule chosen at tf_create (no reference counterpart): 1 when ICP runs as one
 * persistent launch per frame (k_icp_frame), 0 for one launch per iteration; the environment
 * variable TFUSION_ICP_PERSISTENT=0 forces the latter */
tf_status tf_get_schedule(tf_ctx* ctx, int* icp_persistent);
/* The ICP iterations' pose algebra: estimateTransform's cv::determinant(A), cv::solve(A, b, r,
 * cv::DECOMP_SVD) and Affine3f Tinc(r) (tfusion/src/projective_icp.cpp:197-209).
 *   TF_POSE_ALGEBRA_CANONICAL: the pivoting LU determinant, a 2 x 2 block Schur solve in double
 *     (closed-form 3 x 3 adjugates) and Rodrigues in sinc form -- a short serial tail per iteration;
 *   TF_POSE_ALGEBRA_OPENCV4 / _OPENCV2: OpenCV's published algorithms as the oracle restates them
 *     for OpenCV 3.x-4.x / 2.4.9 (Matx_DetOp's LU, JacobiSVD + SVBkSb in float, Affine3::rotation
 *     with float rounding of every Matx operation; not checked against an OpenCV build, none is
 *     available) -- the reference's algebra (see DESIGN.md §2 for what the two algebras do to a
 *     sequence).
 * Default: TF_POSE_ALGEBRA_OPENCV4 (the reference's algebra; the persistent ICP runs its Jacobi SVD
 * lane-parallel).  The environment variable TFUSION_ICP_SOLVE=opencv4|opencv2|canonical sets it
 * at tf_create.
 * TF_INVALID_ARG if the algebra's persistent ICP kernel would not fit the schedule chosen. */
enum { TF_POSE_ALGEBRA_CANONICAL = 0, TF_POSE_ALGEBRA_OPENCV2 = 2, TF_POSE_ALGEBRA_OPENCV4 = 4 };
tf_status tf_set_pose_algebra(tf_ctx* ctx, int algebra);
tf_status tf_get_pose_algebra(tf_ctx* ctx, int* algebra);
/* One ICP iteration's algebra on caller systems (no context): for each of n systems given as
 * the 27 sums of estimateTransform's reduction (StreamHelper layout, projective_icp.cpp:51-61),
 * det[q] = cv::determinant(A) and x[q] = cv::solve(A, b, DECOMP_SVD) (:197-206) under the
 * algebra TF_POSE_ALGEBRA_* -- the same device code the persistent ICP runs (OpenCV algebras:
 * the lane-parallel Jacobi SVD).  Device buffers: sums 27 n floats, x 6 n floats, det n doubles
 * (may be NULL); asynchronous on `stream` (NULL: the null stream). */
tf_status tf_icp_solve_systems(int algebra, const float* dev_sums, int n, float* dev_x, double* dev_det, void* stream);

/* ---- stage entry points (operate on context state; parity tests) ------------- */
/* computeDists + depthBilateralFilter + depthTruncation + depthBuildPyramid +
 * computePointNormals (topfu.cpp:166-197; imgproc.cpp:3-48) into the curr pyramid */
tf_status tf_stage_preprocess(tf_ctx* ctx, const uint16_t* dev_depth, size_t pitch_bytes);
/* same, host depth */
tf_status tf_stage_preprocess_host(tf_ctx* ctx, const uint16_t* host_depth, size_t pitch_bytes);
/* ProjectiveICP::estimateTransform(points overload) (projective_icp.cpp:169-213) on
 * the context's curr/prev pyramids; affine_rt (out) row-major 3x4. */
tf_status tf_stage_icp(tf_ctx* ctx, float affine_rt[12], int* ok, int* iterations);
/* SceneReconstructionEngine_CUDA::AllocateSceneFromDepth
 * (SceneReconstructionEngine_host.cu:75-195) with the context's dists */
tf_status tf_stage_alloc(tf_ctx* ctx, const float pose_rt[12]);
/* ::IntegrateIntoScene (SceneReconstructionEngine_host.cu:197-251) */
tf_status tf_stage_integrate(tf_ctx* ctx, const float pose_rt[12]);
/* VisualisationEngine_CUDA::CreateExpectedDepths (VisualisationEngine_CUDA.cu:119-173) */
tf_status tf_stage_expected_depths(tf_ctx* ctx, const float pose_rt[12]);
/* GenericRaycast (VisualisationEngine_CUDA.cu:175-218) into raycastResult */
tf_status tf_stage_raycast(tf_ctx* ctx, const float invM_rt[12], int update_visible);
/* renderICP_device + resizePointsNormals (VisualisationEngine_CUDA.cu:323-360,
 * topfu.cpp:308-309): raycastResult -> prev points/normals pyramid */
tf_status tf_stage_icp_maps(tf_ctx* ctx, const float invM_rt[12]);
/* renderGrey_device (VisualisationHelper.hpp:105-118) from raycastResult */
tf_status tf_stage_render_grey(tf_ctx* ctx, const float invM_rt[12]);
/* ResetScene (SceneReconstructionEngine_host.cu:51-73) only */
tf_status tf_stage_reset_scene(tf_ctx* ctx);
/* swap curr <-> prev points/normals pyramids (topfu.cpp:205-207) */
tf_status tf_stage_swap_pyramids(tf_ctx* ctx);

/* ---- engine entry points over caller buffers (the L4 C++ API, include/tfusion/engines.hpp) --
 * Poses are row-major 3x4 [R|t]; intr = {fx, fy, cx, cy} (Intr, types.hpp:20-26) and overrides the
 * context's intrinsics for the call; dists / maps are caller device buffers with a row step in
 * bytes, rows x cols of the context's image size.  All synchronous. */
/* cuda::ProjectiveICP::setDistThreshold / setAngleThreshold / setIterationsNum
 * (projective_icp.cpp:81-101): the tracker parameters the context's frames use from now on */
tf_status tf_icp_set_params(tf_ctx* ctx, float dist_thres, float angle_thres, const int iters[4]);
tf_status tf_icp_get_params(tf_ctx* ctx, float* dist_thres, float* angle_thres, int iters[4]);
/* one level of a point/normal pyramid: float4 maps, row steps in bytes */
typedef struct tf_map_level {
    const void* points; size_t points_step;
    const void* normals; size_t normals_step;
} tf_map_level;
/* cuda::ProjectiveICP::estimateTransform(affine, intr, vcurr, ncurr, vprev, nprev)
 * (projective_icp.cpp:169-213) on caller pyramids (level l is (cols >> l) x (rows >> l)); the
 * maps are copied into the context's current/previous pyramids first.  affine_rt receives the
 * estimate (the last successful composition when *ok == 0, as the reference leaves it). */
tf_status tf_icp_estimate(tf_ctx* ctx, const float intr[4], const tf_map_level* curr, const tf_map_level* prev,
                          int levels, float affine_rt[12], int* ok, int* iterations);
/* SceneReconstructionEngine_CUDA::AllocateSceneFromDepth(scene, intr, pose, dists, renderState,
 * onlyUpdateVisibleList, resetVisibleList) (SceneReconstructionEngine_host.cu:75-195); pose is
 * world -> camera (TopFu passes poses_.back().inv(), topfu.cpp:281) */
tf_status tf_scene_alloc(tf_ctx* ctx, const float intr[4], const float pose_rt[12], const float* dists,
                         size_t dists_step, int only_update_visible_list, int reset_visible_list);
/* ::IntegrateIntoScene(scene, intr, pose, dists, renderState) (SceneReconstructionEngine_host.cu:197-251) */
tf_status tf_scene_integrate(tf_ctx* ctx, const float intr[4], const float pose_rt[12], const float* dists,
                             size_t dists_step);
/* ::IntegrateIntoScene with the view's RGB image (voxel_rgb: the Voxel_s_rgb colour update;
 * SceneReconstructionEngine_host.cu:217 M_rgb = calib_inv * M_d, :245-247 the rgb arguments) */
tf_status tf_scene_integrate_rgb(tf_ctx* ctx, const float intr[4], const float pose_rt[12], const float* dists,
                                 size_t dists_step, const uint8_t* dev_rgb, size_t rgb_step);
/* The swapping engine of the GlobalCache's lineage, run after integration when use_swapping is
 * set (every frame of tf_process_frame(s) does it): IntegrateGlobalIntoLocal + SaveToGlobalMemory
 * (InfiniTAM ITMSwappingEngine_CUDA, whose instantiation the reference comments out,
 * CUDAInstantiations.cu:8); its semantics are written out in DESIGN.md §Swapping. */
tf_status tf_scene_swap(tf_ctx* ctx);
/* the two halves on their own: SwappingEngine::IntegrateGlobalIntoLocal(scene, renderState) and
 * ::SaveToGlobalMemory(scene, renderState); tf_scene_swap == swap_in then swap_out */
tf_status tf_scene_swap_in(tf_ctx* ctx);
tf_status tf_scene_swap_out(tf_ctx* ctx);
/* blocks swapped in / out and reallocated by the last frame (or tf_scene_* call) */
tf_status tf_swap_counts(tf_ctx* ctx, int counts[3]);
/* The state after each frame of tf_scene_fuse_frames (no reference counterpart: the reference keeps
 * these counters host-side, LocalVBA.hpp:26, VoxelBlockHash.hpp:69, RenderState_VH.hpp:33, and its
 * allocation failures are silent, SceneReconstructionEngine_host.cu:374-381, 398-401). */
typedef struct tf_fuse_record {
    int lastFreeBlockId;
    int lastFreeExcessListId;
    int noVisibleEntries;
    int alloc_failed_type1;             /* this frame's requests refused for want of a free block */
    int alloc_failed_type2;             /* ... excess-list requests refused (no block or no excess slot) */
    int swapped_in;                     /* use_swapping: IntegrateGlobalIntoLocal's state 1 -> 2 entries */
    int swapped_out;                    /* SaveToGlobalMemory's blocks moved to the GlobalCache and freed */
    int swap_realloc;                   /* reAllocateSwappedOutVoxelBlocks' blocks */
    int swapped_in_merged;              /* stored blocks merged back into the VBA */
    int pad;
} tf_fuse_record;
/* Engine-level fusion of n device-resident frames at given poses with no host round trip inside,
 * TopFu's call order without the tracker: for frame k, cuda::computeDists(depth_k) (imgproc.cu:
 * 263-290, topfu.cpp:166), SceneReconstructionEngine_CUDA::AllocateSceneFromDepth(scene, intr,
 * poses[k], dists, renderState) and ::IntegrateIntoScene(...) (SceneReconstructionEngine_host.cu:
 * 75-251, topfu.cpp:202-203), then with use_swapping the swapping engine (tf_scene_swap).  The
 * results equal tf_imgproc_compute_dists + tf_scene_alloc + tf_scene_integrate (+ tf_scene_swap)
 * called per frame.  dev_frames: uint16 depth, frame k at dev_frames + k * frame_stride_bytes, rows
 * pitch_bytes apart (0: cols * 2); poses_rt: n world -> camera poses (host, row-major [R|t], as
 * tf_scene_alloc takes them); intr: NULL = the context's; records: NULL or n host records.
 * Returns when the batch is done. */
tf_status tf_scene_fuse_frames(tf_ctx* ctx, const float intr[4], const uint16_t* dev_frames, size_t frame_stride_bytes,
                               size_t pitch_bytes, const float* poses_rt, int n, tf_fuse_record* records);
/* GlobalCache::SaveToFile / ReadFromFile (GlobalCache.hpp:79-110): hasStoredData as one byte per
 * entry, then every entry's 512 voxels (4 B each), n_buckets + n_excess entries */
tf_status tf_swap_save(tf_ctx* ctx, const char* path);
tf_status tf_swap_load(tf_ctx* ctx, const char* path);
/* VisualisationEngine_CUDA::CreateExpectedDepths(scene, pose, intr, renderState)
 * (VisualisationEngine_CUDA.cu:119-173); pose is world -> camera */
tf_status tf_vis_expected_depths(tf_ctx* ctx, const float intr[4], const float pose_rt[12]);
/* ::RenderImage(scene, pose, intr, renderState, image, type, raycastType)
 * (VisualisationEngine_CUDA.cu:220-291, 423-429); pose is camera -> world (Matrix4f(poses_.back()),
 * topfu.cpp:346-352); new_raycast = 1: RENDER_FROM_NEW_RAYCAST, 0: RENDER_FROM_OLD_RAYCAST (the
 * pixel stage on the current raycast result) */
tf_status tf_vis_render_image(tf_ctx* ctx, const float intr[4], const float pose_rt[12], int type, int new_raycast,
                              uint8_t* dev_rgba, size_t step);
/* ::CreateICPMaps(scene, pose, intr, points, normals, renderState) (VisualisationEngine_CUDA.cu:
 * 323-360, 473-493): castRay<true> + renderICP into the caller's level-0 maps; pose is camera -> world */
tf_status tf_vis_icp_maps(tf_ctx* ctx, const float intr[4], const float pose_rt[12], void* points, size_t points_step,
                          void* normals, size_t normals_step);

/* ---- cuda:: image processing over caller buffers (imgproc.hpp:9-31, imgproc.cu) --------
 * Stateless; stream = hipStream_t (NULL: the legacy default stream); all asynchronous on it.
 * Depth is uint16 millimetres, dists float, points / normals float4; steps in bytes. */
/* cuda::computeDists (imgproc.cu:263-290) */
tf_status tf_imgproc_compute_dists(const uint16_t* depth, size_t depth_step, float* dists, size_t dists_step,
                                   int cols, int rows, void* stream);
/* cuda::depthBilateralFilter (imgproc.cu:10-61); sigma_depth in metres as the reference takes it */
tf_status tf_imgproc_bilateral(const uint16_t* in, size_t in_step, uint16_t* out, size_t out_step, int cols, int rows,
                               int ksz, float sigma_spatial, float sigma_depth, void* stream);
/* cuda::depthTruncation (imgproc.cu:70-89), in place; threshold in metres */
tf_status tf_imgproc_truncate(uint16_t* depth, size_t step, int cols, int rows, float threshold, void* stream);
/* cuda::depthBuildPyramid (imgproc.cu:98-140): out is (cols/2) x (rows/2) */
tf_status tf_imgproc_pyr_down(const uint16_t* in, size_t in_step, int cols, int rows, uint16_t* out, size_t out_step,
                              float sigma_depth, void* stream);
/* cuda::computePointNormals (imgproc.cu:214-254) with intr = {fx, fy, cx, cy} of this level */
tf_status tf_imgproc_point_normals(const float intr[4], const uint16_t* depth, size_t depth_step, int cols, int rows,
                                   void* points, size_t points_step, void* normals, size_t normals_step, void* stream);
/* cuda::resizePointsNormals (imgproc.cu:355-401): outputs are (cols/2) x (rows/2) */
tf_status tf_imgproc_resize_points_normals(const void* points, size_t points_step, const void* normals,
                                           size_t normals_step, int cols, int rows, void* points_out,
                                           size_t points_out_step, void* normals_out, size_t normals_out_step,
                                           void* stream);
/* cuda::waitAllDefaultStream (imgproc.cpp:18-19) */
tf_status tf_imgproc_sync(void* stream);

/* ---- state transfer --------------------------------------------------------- */
/* host <-> context buffer copies; level selects the pyramid level for TF_BUF_DEPTH..
 * TF_BUF_PREV_NORMALS.  bytes must equal the buffer size (tf_buffer_bytes). */
tf_status tf_buffer_bytes(tf_ctx* ctx, int which, int level, size_t* bytes);
tf_status tf_download(tf_ctx* ctx, int which, int level, void* host, size_t bytes);
/* bytes [offset, offset + bytes) of a level-0 buffer (one entry of a large table) */
tf_status tf_download_range(tf_ctx* ctx, int which, size_t offset, void* host, size_t bytes);
tf_status tf_upload(tf_ctx* ctx, int which, int level, const void* host, size_t bytes);
tf_status tf_set_pose(tf_ctx* ctx, const float rt[12]);

/* ---- per-stage timing (SampledScopeTime, tfusion/include/tfusion/types.hpp:91-104) --
 * When enabled, every frame records HIP events around each stage on the context stream;
 * durations accumulate until tf_profile_reset.  Stage ids: */
typedef enum tf_stage_id {
    TF_STAGE_PREPROCESS = 0,      /* dists + bilateral + pyramid + vertex/normal maps */
    TF_STAGE_ICP = 1,             /* estimateTransform, all iterations */
    TF_STAGE_ALLOC = 2,           /* AllocateSceneFromDepth */
    TF_STAGE_INTEGRATE = 3,       /* IntegrateIntoScene (k_integrate only) */
    TF_STAGE_RAYCAST_RENDER = 4,  /* renderImage raycast (fused into TF_STAGE_RAYCAST_ICP in the frame) */
    TF_STAGE_GREY = 5,            /* renderGrey (fused likewise) */
    TF_STAGE_EXPECTED_DEPTHS = 6, /* CreateExpectedDepths */
    TF_STAGE_RAYCAST_ICP = 7,     /* CreateICPMaps raycast<true> + renderImage (k_raycast_pair) */
    TF_STAGE_ICP_MAPS = 8         /* renderICP + resizePointsNormals */
} tf_stage_id;
tf_status tf_profile_enable(tf_ctx* ctx, int enable);
/* time only the stages whose bit (1 << tf_stage_id) is set; 0 disables.  Each timed stage
 * adds two event records per frame to the stream, which cost GPU time of their own, so a
 * throughput measurement times only the stage it needs. */
tf_status tf_profile_stages(tf_ctx* ctx, unsigned mask);
/* time only every `period`-th frame enqueued from now on (1 = every frame, the default after
 * tf_profile_enable / tf_profile_stages): a throughput run keeps its stage timing live while
 * all but 1/period of its frames carry no events */
tf_status tf_profile_sample(tf_ctx* ctx, int period);
tf_status tf_profile_reset(tf_ctx* ctx);
/* ms[i] = accumulated milliseconds, counts[i] = frames measured, for i < n (n <= 9) */
tf_status tf_profile_read(tf_ctx* ctx, double* ms, long long* counts, int n);
tf_status tf_set_counters(tf_ctx* ctx, int lastFreeBlockId, int lastFreeExcessListId, int noVisibleEntries);
/* Frame totals accumulated on the device by every frame's end since tf_create or the last
 * tf_reset_totals (measurement; no reference counterpart -- the reference's only metric is the
 * SampledScopeTime average, tfusion/src/core.cpp:202-216). */
typedef struct tf_totals {
    long long frames;               /* TopFu::operator() calls completed */
    long long frames_tracked;       /* tracking path with ICP ok (alloc + integrate + both raycasts) */
    long long resets;               /* ICP failures -> reset (topfu.cpp:263-264) */
    long long visible_sum;          /* noVisibleEntries summed over the frames that integrated */
    long long tiles_sum;            /* noTotalBlocks summed over the tracked frames */
    long long swapped_in;           /* swap-ins (use_swapping): state-1 entries with a block set to state 2,
                                       whether or not the GlobalCache held data for them */
    long long swapped_out;          /* blocks swapped out: each one copied VBA -> GlobalCache and freed */
    long long integrate_lanes_read;     /* 16-B voxel lanes (4 voxels) integration read: those with an update */
    long long integrate_lanes_written;  /* ... and wrote back: those whose value changed */
    long long swapped_in_merged;    /* the swap-ins whose entry held stored data: GlobalCache -> VBA transfers */
    long long alloc_failed_type1;   /* allocation requests that failed silently for want of a free voxel block
                                       (allocateVoxelBlocksList, SceneReconstructionEngine_host.cu:374-381) */
    long long alloc_failed_type2;   /* ... excess-list requests that failed for want of a block or an excess
                                       slot (:386-411) */
    long long icp_fallbacks;        /* frames re-run on the per-iteration ICP schedule because the persistent
                                       launch lost a peer (not all of its workgroups were co-resident) */
} tf_totals;
tf_status tf_get_totals(tf_ctx* ctx, tf_totals* totals);
tf_status tf_reset_totals(tf_ctx* ctx);
/* Measurement: `iters` back-to-back launches of one stage's kernels on the context stream
 * with the pose/matrices of tf_stage_* (stage = TF_STAGE_INTEGRATE: k_integrate;
 * TF_STAGE_EXPECTED_DEPTHS: k_ed_fill over the boxes one projection pass of the current list
 * made first;
 * TF_STAGE_RAYCAST_ICP: castRay<true> into raycastResult; TF_STAGE_RAYCAST_RENDER: the frame's
 * k_raycast_pair -- castRay<true> + renderImage's castRay and grey, over the current range
 * image), timed by HIP events on that stream; *ms_per_iter = elapsed / iters.  The scene is
 * updated by every launch exactly as by tf_stage_integrate / tf_stage_raycast. */
tf_status tf_time_stage(tf_ctx* ctx, int stage, const float pose_rt[12], int iters, float* ms_per_iter);

#ifdef __cplusplus
}
#endif
#endif
