/*
 * tf_oracle.h -- CPU ORACLE for the topfusion hot path (TEST INFRASTRUCTURE ONLY).
 *
 * This is a serial C restatement of the reference algorithm (3d-scan/topfusion,
 * tfusion library) used ONLY as the checker by tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg.  Nothing in the product (topfusion_amd/,
 * include/) includes, links or calls it.
 *
 * Parity status: PARTIALLY PINNED.  The reference has no tests, fixtures or
 * golden vectors, and its CUDA path cannot run here (no nvcc/NVIDIA GPU/OpenCV).
 * The pieces of the reference that compile with plain g++ from their own headers
 * (Matrix.hpp / Vector.hpp / MathUtils.hpp / VoxelTypes.hpp) are built by
 * oracle/ref_pin (outputs in oracle/_ref/) and pin this oracle's matrix inverse,
 * matrix-vector order, floor/round conversions and Voxel_s quantisation
 * (tests/golden/ref_pin_*.bin).  Everything else is "parity unpinned": restated
 * from the cited reference lines under the canonical numerics below.
 *
 * Canonical numerics (the reference's CUDA build uses --ftz --prec-div=false
 * --prec-sqrt=false and fast intrinsics, which are not reproducible off NVIDIA):
 *   - no FMA contraction (-ffp-contract=off); explicit fmaf() exactly where the
 *     reference writes __fmaf_rn (src/cuda/device.hpp:26-29, proj_icp.cu:34-35)
 *   - IEEE-correct f32 division / sqrt; rsqrt(x) -> 1.0f/sqrtf(x);
 *     __fdividef(a,b) -> a/b
 *   - __expf(x) (imgproc.cu:40) -> tfo_exp(): 2^(x*log2e) with an exact range
 *     reduction and a fixed Horner polynomial (results < 2^-125 flushed to 0)
 *   - texture point sampling (proj_icp.cu:102,111) -> floorf() indexing
 *   - races resolved in serial order: allocation requests in raster order
 *     (y, x, step), last writer wins (SceneReconstructionEngine.hpp:287-292);
 *     block / excess allocation and visible-list compaction in ascending hash
 *     index order (SceneReconstructionEngine_host.cu:350-479)
 *   - OpenCV (absent, unpinned): cv::determinant -> LU with partial pivoting in
 *     float (eps 10*FLT_EPSILON) and the pivot product in double;
 *     cv::solve(DECOMP_SVD) -> Gaussian elimination with partial pivoting in
 *     double; Affine3f(rvec,t) -> Rodrigues in double with a fixed-polynomial
 *     sin/cos; Affine3f::operator* and ::inv -> explicit float rigid algebra.
 */
#ifndef TF_ORACLE_H
#define TF_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct tfo_params {
    int cols, rows;                 /* topfu.cpp:19-20 */
    float fx, fy, cx, cy;           /* topfu.cpp:24 */
    float bilateral_sigma_depth;    /* m, topfu.cpp:30 */
    float bilateral_sigma_spatial;  /* px, topfu.cpp:31 */
    int   bilateral_kernel_size;    /* topfu.cpp:32 */
    float icp_truncate_depth_dist;  /* m, topfu.cpp:35 */
    float icp_dist_thres;           /* m, topfu.cpp:36 */
    float icp_angle_thres;          /* rad, topfu.cpp:37 */
    int   icp_iter_num[4];          /* topfu.cpp:14 */
    float mu;                       /* SceneParams, topfu.cpp:50 */
    int   maxW;
    float voxelSize;
    float viewFrustum_min, viewFrustum_max;
    /* capacities (compile-time #defines in the reference, VoxelBlockHash.hpp:10-27,
       RenderState_VH.hpp:41, VisualisationEngine_Shared.hpp:5) */
    int   n_buckets;                /* power of two, SDF_BUCKET_NUM */
    int   n_excess;                 /* SDF_EXCESS_LIST_SIZE */
    int   n_blocks;                 /* SDF_LOCAL_BLOCK_NUM */
    int   vis_capacity;             /* visibleEntryIDs capacity */
    int   max_render_blocks;        /* MAX_RENDERING_BLOCKS */
    /* swapping: Scene(params, useSwapping) (scene.hpp:29-33, GlobalCache.hpp); off in TopFu (topfu.cpp:67) */
    int   use_swapping;
    int   swap_transfer_blocks;     /* SDF_TRANSFER_BLOCK_NUM (VoxelBlockHash.hpp:27) */
    /* colour: Voxel_s_rgb instead of Voxel_s (VoxelTypes.hpp:39-67) and the RGB camera */
    int   voxel_rgb;
    float rgb_intr[4];              /* projParams_rgb (fx, fy, cx, cy); all 0: the depth intrinsics */
    float depth_to_rgb[12];         /* trafo_rgb_to_depth.calib_inv as row-major [R|t] (M_rgb = it * M_d) */
} tfo_params;

typedef struct tfo_hash_entry {     /* VoxelBlockHash.hpp:32-44 (16 B) */
    int16_t x, y, z, pad;
    int32_t offset;
    int32_t ptr;
} tfo_hash_entry;

typedef struct tfo_voxel {          /* VoxelTypes.hpp:69-92 Voxel_s (4 B) */
    int16_t sdf;
    uint8_t w;
    uint8_t pad;
} tfo_voxel;

typedef struct tfo_counters {
    int lastFreeBlockId;            /* LocalVBA.hpp:26 */
    int lastFreeExcessListId;       /* VoxelBlockHash.hpp:69 */
    int noVisibleEntries;           /* RenderState_VH.hpp:33 */
    int noTotalBlocks;              /* rendering tiles, VisualisationEngine_CUDA.cu:160 */
    int frame_counter;
    int icp_iterations;             /* iterations executed in the last estimateTransform */
    int icp_ok;
    int n_resets;
} tfo_counters;

void tfo_default_params(tfo_params* p);

/* ---- stage functions (stateless) ---- */
float tfo_exp(float x);
void tfo_compute_dists(const uint16_t* depth, int W, int H, float* dists);
void tfo_bilateral(const uint16_t* src, uint16_t* dst, int W, int H, int ksz, float sigma_spatial, float sigma_depth_m);
void tfo_truncate(uint16_t* depth, int W, int H, float max_dist_m);
void tfo_pyr_down(const uint16_t* src, int W, int H, uint16_t* dst, float sigma_depth_m);
void tfo_points_normals(const uint16_t* depth, int W, int H, float fx, float fy, float cx, float cy,
                        float* points, float* normals);
void tfo_resize_points_normals(const float* vsrc, const float* nsrc, int W, int H, float* vdst, float* ndst);
/* one ICP iteration: A|b as the 27 reference-ordered sums (proj_icp.cu:120-403) */
void tfo_icp_reduce(const float* vcurr, const float* ncurr, const float* vprev, const float* nprev,
                    int W, int H, float fx, float fy, float cx, float cy,
                    float min_cosine, float dist2_thres, const float aff[12], float out27[27]);
/* det check + solve + Rodrigues + compose (projective_icp.cpp:190-210); returns 1 ok, 0 fail */
int tfo_icp_step(const float sums27[27], float affine_rt[12], double* det_out);
/* test-only: the pose algebra tfo_icp_step uses (canonical = the GPU's default; OpenCV 2.4.9 or
   3.x/4.x as published), with glibc's or the portable transcendental functions */
enum { TFO_POSE_CANONICAL = 0, TFO_POSE_OPENCV2 = 2, TFO_POSE_OPENCV4 = 4 };
void tfo_set_pose_algebra(int mode, int use_libm);
int tfo_get_pose_algebra(void);
double tfo_cv_det6(const float A[36], int mode);
/* the canonical algebra's determinant and solve (test-only exports) */
void tfo_solve6(const float A[36], const float b[6], float x[6]);
double tfo_det6(const float A[36]);
void tfo_cv_jacobi_svd(float* At, float* W, float* Vt, int m, int n);
void tfo_cv_solve_svd6(const float A[36], const float b[6], float x[6]);
void tfo_cv_rodrigues(const float rvec[3], float R[9], int mode);
double tfo_cv_hypot(double x, double y);
/* diagnostics: Jacobi calls, sweeps, rotations, max sweeps, histogram of the converged sweep index */
void tfo_cv_svd_stats(long long out[36], int reset);
/* test-only: record every ICP step's 27 sums into buf (27 floats each, at most cap steps) */
void tfo_capture_sums(float* buf, long long cap);
long long tfo_captured_sums(void);
void tfo_rigid_mul(const float a[12], const float b[12], float out[12]);
void tfo_rigid_inv(const float a[12], float out[12]);
int  tfo_matrix4_inv(const float m[16], float out[16]);
void tfo_sincos(double th, double* s, double* c);
void tfo_m4v(const float m[16], const float v[4], float r[4]);
void tfo_tsdf_update(int16_t* sdf, uint8_t* w, float eta, float mu, int maxW);
void tfo_rodrigues(const float r[3], float R[9]);
/* the direct form (unit axis, sin / cos of the angle, 1 - cos): an independent check of the
   sinc form tfo_rodrigues uses */
void tfo_rodrigues_direct(const float r[3], float R[9]);
void tfo_point_conv(const float p[3], float out[13]);     /* floor/round/length conversions */
void tfo_interp_bilinear_u8x4(const uint8_t* rgb, size_t pitch, float ix, float iy, float out[4]); /* interpolateBilinear<uchar> */
uint32_t tfo_colour_average(uint32_t clr, const float sample[4], int maxW);  /* colour running average */
int  tfo_hash_index(int x, int y, int z, int n_buckets);

/* ---- stateful pipeline (TopFu) ---- */
typedef struct tfo_ctx tfo_ctx;
tfo_ctx* tfo_create(const tfo_params* p);
void tfo_destroy(tfo_ctx* c);
void tfo_reset(tfo_ctx* c);                                   /* TopFu::reset */
int tfo_copy_state(tfo_ctx* dst, const tfo_ctx* src);        /* whole state, same params (bench samples) */
int  tfo_process_frame(tfo_ctx* c, const uint16_t* depth);    /* TopFu::operator() */
/* TopFu::operator()(depth, image): the frame's uchar4 RGB image (pitch bytes per row, 0: cols * 4)
   integrated into the Voxel_s_rgb colour (voxel_rgb) */
int  tfo_process_frame_rgb(tfo_ctx* c, const uint16_t* depth, const uint8_t* rgb, size_t pitch);
void tfo_get_counters(const tfo_ctx* c, tfo_counters* out);
void tfo_set_counters(tfo_ctx* c, int lastFreeBlockId, int lastFreeExcessListId, int noVisibleEntries);
void tfo_get_pose(const tfo_ctx* c, float rt[12]);            /* getCameraPose(): [R|t] row-major */
/* stage-level entry points on the context */
void tfo_reset_scene(tfo_ctx* c);                                             /* ResetScene (keeps the GlobalCache) */
void tfo_alloc(tfo_ctx* c, const float pose_rt[12], const float* dists);      /* AllocateSceneFromDepth */
void tfo_alloc_ex(tfo_ctx* c, const float pose_rt[12], const float* dists, int only_update_visible, int reset_visible);
void tfo_integrate(tfo_ctx* c, const float pose_rt[12], const float* dists);  /* IntegrateIntoScene */
void tfo_integrate_rgb(tfo_ctx* c, const float pose_rt[12], const float* dists, const uint8_t* rgb, size_t pitch);
void tfo_expected_depths(tfo_ctx* c, const float pose_rt[12]);                 /* CreateExpectedDepths */
void tfo_raycast(tfo_ctx* c, const float invM_rt[12], int update_visible);    /* GenericRaycast */
void tfo_render_icp(tfo_ctx* c, const float invM_rt[12], float* points, float* normals); /* renderICP */
void tfo_render_type(tfo_ctx* c, const float invM_rt[12], int type, uint8_t* rgba);
void tfo_render_image_type(tfo_ctx* c, int type);
void tfo_render_grey(tfo_ctx* c, const float invM_rt[12], uint8_t* rgba);     /* renderGrey */
void tfo_render_image(tfo_ctx* c, uint8_t* rgba);                              /* TopFu::renderImage */
/* swapping (GlobalCache + the InfiniTAM-lineage swapping engine, see tf_oracle.c) */
void tfo_swap(tfo_ctx* c);                          /* IntegrateGlobalIntoLocal + SaveToGlobalMemory */
void tfo_swap_in(tfo_ctx* c);                       /* IntegrateGlobalIntoLocal */
void tfo_swap_out(tfo_ctx* c);                      /* SaveToGlobalMemory */
long long tfo_swap_merged_total(const tfo_ctx* c);  /* swap-ins that merged stored data, since creation */
void tfo_swap_counts(const tfo_ctx* c, int out[3]);  /* last frame: swapped in, swapped out, reallocated */
uint8_t* tfo_swap_state(tfo_ctx* c);                /* HashSwapState::state per entry */
uint8_t* tfo_swap_stored_flags(tfo_ctx* c);         /* GlobalCache hasStoredData per entry */
tfo_voxel* tfo_swap_stored(tfo_ctx* c);             /* GlobalCache storedVoxelBlocks, 512 per entry */
/* state access */
tfo_hash_entry* tfo_hash(tfo_ctx* c);
int* tfo_alloc_list(tfo_ctx* c);        /* LocalVBA::allocationList (n_blocks) */
int* tfo_excess_list(tfo_ctx* c);       /* VoxelBlockHash::excessAllocationList (n_excess) */
void tfo_alloc_failures(const tfo_ctx* c, int out[2]);   /* last allocation: failed type-1, type-2 requests */
tfo_voxel* tfo_vba(tfo_ctx* c);
uint32_t* tfo_vba_rgb(tfo_ctx* c);   /* voxel_rgb: per voxel r | g << 8 | b << 16 | w_color << 24 */
int* tfo_visible_ids(tfo_ctx* c);
uint8_t* tfo_visible_type(tfo_ctx* c);
float* tfo_range_image(tfo_ctx* c);     /* W*H float2 */
float* tfo_raycast_result(tfo_ctx* c);  /* W*H float4 */
float* tfo_prev_points(tfo_ctx* c, int level);
float* tfo_prev_normals(tfo_ctx* c, int level);
float* tfo_curr_points(tfo_ctx* c, int level);
float* tfo_curr_normals(tfo_ctx* c, int level);
uint16_t* tfo_curr_depth(tfo_ctx* c, int level);
float* tfo_dists(tfo_ctx* c);
uint8_t* tfo_frame_grey(tfo_ctx* c);    /* W*H rgba: renderImage inside the last tracked frame */

#ifdef __cplusplus
}
#endif
#endif
