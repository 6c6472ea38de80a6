// tf_internal.h -- shared definitions of libtfusion_hip (gfx950).
//
// Numerics are "canonical" (see DESIGN.md §Numerics): every kernel is compiled with
// -ffp-contract=off and IEEE-correct f32 division/sqrt, fmaf() is written exactly where
// the reference writes __fmaf_rn, and the reference's fast intrinsics (__expf, rsqrt,
// __fdividef) are replaced by fixed IEEE sequences, so each stage is bit-reproducible
// against the CPU oracle (oracle/tf_oracle.c, test infrastructure only).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>
#include <stddef.h>
#include "../../include/tfusion_hip.h"

#define TF_BLK 8        // SDF_BLOCK_SIZE (VoxelBlockHash.hpp:10)
#define TF_BLK3 512     // SDF_BLOCK_SIZE3
#define TF_FAR_AWAY 999999.9f   // VisualisationEngine_Shared.hpp:18
#define TF_VERY_CLOSE 0.05f     // VisualisationEngine_Shared.hpp:22
#define TF_SUBSAMPLE 8          // minmaximg_subsample (VisualisationEngine_Shared.hpp:7)
#define TF_RB_SIZE 16           // renderingBlockSizeX/Y (VisualisationEngine_Shared.hpp:25-26)
#define TF_LEVELS 3
#define TF_NUM_STAGES 9     // tf_stage_id in include/tfusion_hip.h
#define TF_PROF_RING 32     // frames enqueued between host syncs (and timing-event ring slots)
#define TF_ST_BYTES (sizeof(TfDevState) + 2 * sizeof(int) * TF_PROF_RING)   // c->st + frame_ok / frame_mode rings
#define TF_ICP_TAG_WORDS (2 * 256 * 28 + 16 + 2 * 8 * 28 + 16 + 8 * 512)   // persistent ICP tagged granules (tf_icp.hip)

// HashEntry, VoxelBlockHash.hpp:32-44 (16 B; one dwordx4 probe)
struct __attribute__((aligned(16))) TfHashEntry {
    short x, y, z, pad;
    int offset;
    int ptr;
};
// Voxel_s, VoxelTypes.hpp:69-92 (4 B)
struct __attribute__((aligned(4))) TfVoxel {
    short sdf;
    unsigned char w;
    unsigned char pad;
};

// Per-context device state: everything the frame's kernels exchange, so that a frame is a
// fixed kernel sequence with no host round trip (graph-capturable).
struct TfDevState {
    float pose[12];          // poses_.back(), camera->world, row-major [R|t]
    float affine[12];        // ICP working transform
    float pose_in[12];       // explicit pose for stage entry points
    float M_alloc[16];       // Matrix4f of the world->camera pose (column-major m[4c+r])
    float invM_alloc[16];    // Matrix4::inv(M_alloc) (SceneReconstructionEngine_host.cu:102-103)
    float M_ray[16];         // Matrix4f(pose) camera->world, raycast invM
    float sums[27];          // last ICP A|b
    int icp_ok;              // estimateTransform result
    int icp_iters;           // iterations executed
    int abort;               // set by ICP failure: remaining kernels of the frame no-op
    int lastFreeBlockId;     // LocalVBA::lastFreeBlockId
    int lastFreeExcessListId;
    int noVisibleEntries;
    int noTotalBlocks;
    int alloc_fail[2];       // this AllocateSceneFromDepth's failed requests: type 1 (no free block), type 2
                             // (no free block or excess slot) -- allocateVoxelBlocksList's silent failures
                             // (SceneReconstructionEngine_host.cu:374-381, 398-401); zeroed by k_alloc_requests
    int pad_[2];             // alloc totals: requests of both types, of type 2 (k_alloc_apply -> k_vis_count)
    unsigned icp_gen;        // last generation tag used by the persistent ICP kernel
    // device-driven frame control (TopFu::operator() branches decided on the device, so a
    // batch of frames is enqueued without host round trips)
    int mode;                // this frame: 0 = frame-0 path (integrate only), 1 = tracking path
    int frame_counter;       // TopFu::frame_counter_
    int n_resets;            // resets taken after ICP failures
    unsigned reset_ticket;   // k_reset_scene: workgroups done (the last one resets the counters)
    int halt;                // set by a frame end whose frame failed on the device (frame_ok < 0): every later
                             // frame of the batch is skipped (frame_ok -2) until the host clears it
    unsigned pad5_;
    int scene_external;      // scene buffers / counters set from the host since the last full reset:
                             // the next reset (in-frame ones too) clears everything, then drops it
    int sticky_error;        // a frame failed past its ICP (a bounded spin in a later stage timed out): the
                             // context reports TF_HIP_ERROR until tf_reset
    // the frame's renderImage runs in k_raycast_pair after CreateExpectedDepths has rewritten the
    // range image; it reads the raycast matrix, go flag and range region snapshotted before
    // (render_snapshot / icp_fold_t3)
    float M_render[16];      // M_ray of the frame being rendered
    int render_go;           // the frame took the tracking path (mode 1, ICP ok)
    int pad3_[3];
    // swapping (tf_swap.hip): the last frame's counts, and the free-list top handed from the
    // swap-in launch to the swap-out launch
    int swap_in, swap_out, swap_realloc, swap_free0;
    int swap_merged;         // the last IntegrateGlobalIntoLocal's merges of stored data (k_swap_count_in zeroes it)
    int pad6_[3];
    // totals since creation / tf_reset_totals, accumulated by the frame end (tf_totals)
    long long tot_frames, tot_tracked, tot_resets, tot_visible, tot_tiles, tot_swap_in, tot_swap_out,
        tot_swap_merged,         // swap-ins whose entry held stored data (a real GlobalCache -> VBA transfer)
        tot_alloc_fail1, tot_alloc_fail2;   // failed allocation requests (alloc_fail), accumulated by k_vis_count
};

// ---------------------------------------------------------------------------------------
// canonical device math
// ---------------------------------------------------------------------------------------
// RN(1 / z), the IEEE-correct reciprocal (= 1.0f / z under -fhip-fp32-correctly-rounded-divide-sqrt),
// in three instructions where that is proven: v_rcp_f32 and one fma Newton step give the correctly
// rounded value for EVERY float z in [2^-126, 2^126) on gfx950 (exhaustive check over all 2^31
// positive floats, tools/micro/rcp_exact.hip, profiles/r05/rcp_exact.txt; mismatches only for
// subnormal z and z >= 2^126).  v_rcp_f32 works on the magnitude and both fma round to nearest,
// so the same holds for z in (-2^126, -2^-126]; NaN gives NaN either way.  The rest (zero,
// subnormal, |z| >= 2^126) takes the IEEE division behind a wave-uniform branch that no wave
// takes on real depth data -- as a select, the division sequence cost ~12 instructions per
// reciprocal on the ICP rows' critical SIMD.
#ifndef TF_RCP_BRANCH
#define TF_RCP_BRANCH 1          // A/B only: 0 = the division computed for every lane and selected
#endif
__device__ __forceinline__ float tf_rcp_fast(float z)
{
    const float r0 = __builtin_amdgcn_rcpf(z);
    const float e = __builtin_fmaf(-z, r0, 1.0f);
    return __builtin_fmaf(e, r0, r0);
}
__device__ __forceinline__ bool tf_rcp_slow(float z)
{
    const float a = __builtin_fabsf(z);
    return a < 0x1p-126f || a >= 0x1p126f;
}
__device__ __forceinline__ float tf_rcp_rn(float z)
{
    float r = tf_rcp_fast(z);
    const bool slow = tf_rcp_slow(z);
#if TF_RCP_BRANCH
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(slow) != 0, 0)) {
        if (slow) r = 1.0f / z;
    }
#else
    if (slow) r = 1.0f / z;
#endif
    return r;
}

// replacement for __expf (imgproc.cu:40): 2^(x log2 e), exact range reduction + Horner
__device__ __forceinline__ float tf_exp(float x)
{
    float t = x * 1.44269504088896341f;
    if (!(t > -125.0f)) return 0.0f;
    if (t >= 128.0f) return __builtin_inff();
    float k = rintf(t);
    float f = t - k;
    float p = 1.5403530393381606e-4f;
    p = fmaf(p, f, 1.3333558146428443e-3f);
    p = fmaf(p, f, 9.6181291076284772e-3f);
    p = fmaf(p, f, 5.5504108664821580e-2f);
    p = fmaf(p, f, 2.4022650695910071e-1f);
    p = fmaf(p, f, 6.9314718055994531e-1f);
    p = fmaf(p, f, 1.0f);
    return ldexpf(p, (int)k);
}

struct tf3 { float x, y, z; };
__device__ __forceinline__ tf3 mk3(float x, float y, float z) { tf3 r; r.x = x; r.y = y; r.z = z; return r; }
__device__ __forceinline__ tf3 sub3(tf3 a, tf3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
// dot with __fmaf_rn (src/cuda/device.hpp:26-29)
__device__ __forceinline__ float kdot(tf3 a, tf3 b) { return fmaf(a.x, b.x, fmaf(a.y, b.y, a.z * b.z)); }
__device__ __forceinline__ tf3 kcross(tf3 a, tf3 b)
{
    return mk3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
// normalized(): v * rsqrt(dot(v,v)) (device.hpp:100-103), rsqrt -> 1/sqrtf
__device__ __forceinline__ tf3 knormalized(tf3 v)
{
    float s = 1.0f / sqrtf(kdot(v, v));
    return mk3(v.x * s, v.y * s, v.z * s);
}

// Matrix4f * Vector4f (Matrix.hpp:126-133), column-major m[4c+r]
__device__ __forceinline__ void tf_m4v(const float* m, float v0, float v1, float v2, float v3, float* r)
{
    r[0] = m[0] * v0 + m[4] * v1 + m[8] * v2 + m[12] * v3;
    r[1] = m[1] * v0 + m[5] * v1 + m[9] * v2 + m[13] * v3;
    r[2] = m[2] * v0 + m[6] * v1 + m[10] * v2 + m[14] * v3;
    r[3] = m[3] * v0 + m[7] * v1 + m[11] * v2 + m[15] * v3;
}
__device__ __forceinline__ void tf_m4v3(const float* m, float v0, float v1, float v2, float v3, float* r)
{
    r[0] = m[0] * v0 + m[4] * v1 + m[8] * v2 + m[12] * v3;
    r[1] = m[1] * v0 + m[5] * v1 + m[9] * v2 + m[13] * v3;
    r[2] = m[2] * v0 + m[6] * v1 + m[10] * v2 + m[14] * v3;
}

// Matrix4f(pose(0,0), pose(1,0), ...) (topfu.cpp:246-249): m[4c+r] = P[r][c]
__device__ __forceinline__ void tf_rt_to_m4(const float* rt, float* m)
{
    for (int c = 0; c < 4; ++c) {
        for (int r = 0; r < 3; ++r) m[4 * c + r] = rt[r * 4 + c];
        m[4 * c + 3] = (c == 3) ? 1.0f : 0.0f;
    }
}

// hashIndex (RepresentationAccess.hpp:5-7)
__device__ __forceinline__ int tf_hash_index(int x, int y, int z, unsigned mask)
{
    return (int)((((unsigned)x * 73856093u) ^ ((unsigned)y * 19349669u) ^ ((unsigned)z * 83492791u)) & mask);
}

__device__ __forceinline__ float tf_qnan() { return __int_as_float(0x7fffffff); }

// (float)s / 32767.0f for a 16-bit integer s (SDF_shortToFloat, VoxelTypes.hpp), IEEE-exact in
// three operations instead of a full division: q0 = s * RN(1/32767), one FMA residual, one FMA
// correction.  Verified equal to the division for all 65536 values of s
// (tests/test_oracle.py::test_short_to_float_division_exact).
__device__ __forceinline__ float tf_short_to_float(int s)
{
    const float x = (float)s;
    const float r = 1.0f / 32767.0f;            // constant-folded RN(1/32767)
    const float q0 = x * r;
    return fmaf(fmaf(-q0, 32767.0f, x), r, q0);
}

// x / 32767.0f for any float |x| < 2^21 (the SDF interpolation and gradient divisions), IEEE-
// exact in three operations: q0 = x * RN(1/32767), e = fma(q0, 32767, -x), q = fma(-e, RN(1/32767),
// q0).  Checked against the division for every float below 2^21 in magnitude, both signs,
// zeros and denormals included (tools/check_div32767.c; tests/test_oracle.py samples it).
__device__ __forceinline__ float tf_div32767(float x)
{
    const float r = 1.0f / 32767.0f;
    const float q0 = x * r;
    return fmaf(-fmaf(q0, 32767.0f, -x), r, q0);
}

// x / d for a divisor d whose three-operation quotient is known exact (rd = RN(1/d)): q0 = x*rd,
// e = fma(q0, d, -x), q = fma(-e, rd, q0) equals the IEEE division for every x of every binade
// where no intermediate is subnormal; that is checked over all mantissas of one binade for
// d = 1..257 (tools/check_div_consts.c) and, at tf_create, for the context's mu.  |x| < 2^-100
// takes the division itself.
__device__ __forceinline__ float tf_div_exact3(float x, float d, float rd)
{
    if (fabsf(x) < 0x1p-100f) return x / d;
    const float q0 = x * rd;
    return fmaf(-fmaf(q0, d, -x), rd, q0);
}

// A missing block's VBA offset in the block grid: the render side reads voxels relative to a
// guard block of Voxel_s() values placed just before the VBA (tf_ctx::vba_guard), so a voxel
// load needs no "is the block there" select -- it lands in the guard and reads (32767, 0).
#define TF_VOFF_NONE (-TF_BLK3)

// Block grid: a dense TF_GRID_DIM^3 array over block coordinates [-HALF, HALF) holding, for
// every block findVoxel would find, (hash entry index, VBA voxel offset = ptr*512), else
// (-1,-1).  It mirrors the hash exactly (written wherever a block is allocated, cleared on
// reset, rebuilt after a hash upload) and replaces the bucket/excess walk on the raycasting
// side by one 8-byte load.  256^3 x 8 B = 128 MiB of HBM.
#define TF_GRID_LOG 8
#define TF_GRID_DIM (1 << TF_GRID_LOG)
#define TF_GRID_HALF (TF_GRID_DIM / 2)
__host__ __device__ __forceinline__ bool tf_grid_in(int bx, int by, int bz)
{
    return ((unsigned)(bx + TF_GRID_HALF) | (unsigned)(by + TF_GRID_HALF) | (unsigned)(bz + TF_GRID_HALF)) <
           (unsigned)TF_GRID_DIM;
}
// (row-major: a layout in 2 x 2 x 4-cell bricks, one 128-byte line each, measured 4 us slower on
// the raycast pair in round 4 -- DESIGN §8)
__host__ __device__ __forceinline__ size_t tf_grid_cell(int bx, int by, int bz)
{
    return ((size_t)(bz + TF_GRID_HALF) << (2 * TF_GRID_LOG)) | ((size_t)(by + TF_GRID_HALF) << TF_GRID_LOG) |
           (size_t)(bx + TF_GRID_HALF);
}

// the cell of a block the hash now holds (allocation, reallocation after a swap-out)
__device__ __forceinline__ void grid_set(int2* grid, const TfHashEntry& e, int idx)
{
    if (e.ptr >= 0 && tf_grid_in(e.x, e.y, e.z)) grid[tf_grid_cell(e.x, e.y, e.z)] = make_int2(idx, e.ptr * TF_BLK3);
}

// wave64 butterfly sum that reproduces the reference's halving tree bit for bit
// (temp_utils.hpp:503-523 for lanes 0..63 after the cross-wave steps)
__device__ __forceinline__ float tf_wave_tree64(float b)
{
    b = b + __shfl_xor(b, 32, 64);
    b = b + __shfl_xor(b, 16, 64);
    b = b + __shfl_xor(b, 8, 64);
    b = b + __shfl_xor(b, 4, 64);
    b = b + __shfl_xor(b, 2, 64);
    b = b + __shfl_xor(b, 1, 64);
    return b;
}

// After this frame's ICP has set the pose (k_set_type3, or the persistent ICP's tail):
// snapshot what the frame's
// renderImage reads and later stages of this frame or the next overwrite -- the raycast
// matrix, the go flag, and the /8 region castRay reads of the range image
// (range[x/8 + (y/8)*W], VisualisationEngine_Shared.hpp:104-106) that CreateExpectedDepths
// rewrites before the render runs.
static __device__ __forceinline__ void render_snapshot(TfDevState* st, const float2* range, float2* snap, int W, int H)
{
    if (blockIdx.x == 0 && threadIdx.x < 16) st->M_render[threadIdx.x] = st->M_ray[threadIdx.x];
    if (blockIdx.x == 0 && threadIdx.x == 0) st->render_go = (st->mode != 0 && !st->abort) ? 1 : 0;
    if (st->mode == 0 || st->abort) return;
    const int rc = (W - 1) / TF_SUBSAMPLE + 1, rr = (H - 1) / TF_SUBSAMPLE + 1;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < rc * rr; i += gridDim.x * blockDim.x) {
        const int y = i / rc, x = i - y * rc;
        snap[x + y * W] = range[x + y * W];
    }
}

// ---------------------------------------------------------------------------------------
// host-side context
// ---------------------------------------------------------------------------------------
struct tf_ctx {
    tf_params p;
    int device;
    hipStream_t stream;
    int n_total;
    int W, H;
    int lw[TF_LEVELS], lh[TF_LEVELS];
    // scene (Scene<Voxel_s,VoxelBlockHash>, scene.hpp:13-44)
    TfHashEntry* hash;
    int* excessList;
    TfVoxel* vba;
    int mu_exact3;          // eta / mu by tf_div_exact3 (checked on the device at tf_create)
    TfVoxel* vba_guard;      // allocation: one guard block of Voxel_s() (TF_VOFF_NONE reads), then vba
    int* allocList;
    int2* bgrid;             // block grid (TF_GRID_*), mirrors the hash
    // swapping (p.use_swapping): the GlobalCache in HBM (GlobalCache.hpp:11-134)
    unsigned char* swapState;    // HashSwapState::state per entry
    unsigned char* swapFlags;    // hasStoredData per entry
    TfVoxel* swapStore;          // storedVoxelBlocks: 512 voxels per entry
    int* swapCounts;             // per 4096-entry chunk: [swap-in candidates, swap-out candidates]
    // colour (p.voxel_rgb): Voxel_s_rgb's clr + w_color as a second plane beside the Voxel_s one
    // (r | g << 8 | b << 16 | w_color << 24 per voxel, same block offsets), so the depth-only
    // passes (raycasts, ICP maps) stream 4 B per voxel, not 8; a guard block of zeros first
    unsigned* vba_rgb_guard;
    unsigned* vba_rgb;
    uchar4* rgb_in;              // staging for host RGB uploads (voxel_rgb)
    const uchar4* rgb_cur;       // the frame's RGB image while it is enqueued (nullptr: none)
    size_t rgb_pitch;            // its row step in bytes
    // SceneReconstructionEngine temporaries
    unsigned char* allocType;
    int* winnerKey;          // per-entry last-writer key (pixel*64+step), replaces blockCoords races
    int* allocCounts;        // per-chunk counts (2 ints per chunk)
    int* visCounts;
    unsigned long long* visAgg;   // [vis_chunks] k_vis_build's tagged chunk counts (generation << 32 | count)
    unsigned vis_gen;        // k_vis_build launches so far (the tag of the next one's counts)
    int vis_fused;           // one k_vis_build launch instead of k_vis_count + k_vis_apply (TFUSION_VIS_FUSED)
    // RenderState_VH
    int* visibleIds;
    unsigned char* visType;
    float* range;            // float2
    float* range_render;     // float2: snapshot of range's ÷8 region for the frame's renderImage
    float* raycast;          // float4
    uchar4* grey;
    // expected-depths scratch
    uint4* blockRec;         // per visible entry: box (4 x u16: ulx, uly, lrx, lry) + z range (invalid: x = ~0u)
    int* blockTiles;
    int* blockOff;           // exclusive tile offset inside the entry's 256-entry chunk
    int* edChunk;            // tile total per chunk
    uint4* edBins;           // k_ed_fill's per-row bins of boxes (tf_ed.h EdArgs::bins)
    int* edBinCnt;
    unsigned* edDone;        // the fused fill's atomic path: rows done (k_raycast_pair)
    // k_raycast_pair's frame path: per CreateICPMaps / renderImage tile the time its workgroup took in
    // the last launch, and the dispatch order that sorts each XCD's tiles longest first (TF_LJF_MAX)
    unsigned* tile_cost;
    int* tile_order;
    int tile_ljf;
    int tile_rows;           // XCD x's tiles: 0 the x-th band of consecutive tiles; 1 the tile rows = x (mod 8)
    int tile_slots;          // dispatch slots per half with the order (8 x the largest XCD share)
    int2* edSpill;           // per k_ed_fill row (ed_nrows): extent [0,x) x [0,y) of the pixels k_ed_fill wrote outside
                             // the /8 region (cleared by the next projection pass)
    int ed_lds_max_n;        // k_ed_fill reduces in LDS per /8 row up to this many visible entries
    int integ_wg_frame;      // integration workgroups in the frame path (<= TF_INTEG_WG)
    // frame buffers
    uint16_t* depth_in;      // staging for host uploads / pitched input
    float* dists;
    uint16_t* depth_pyr[TF_LEVELS];     // [0]: the level-0 buffer of the last frame preprocessed (one of d0_buf)
    uint16_t* d0_buf[2];     // level-0 depth, ping-pong by batch frame parity (two-frame lookahead)
    float4* curr_pts[TF_LEVELS];
    float4* curr_nrm[TF_LEVELS];
    float4* prev_pts[TF_LEVELS];
    float4* prev_nrm[TF_LEVELS];
    // ICP
    float* icp_partial;      // [256][28] column sums
    unsigned* icp_ticket;    // last-workgroup ticket (zero between launches)
    unsigned long long* icp_tagged;   // persistent ICP: [256][28] tagged column sums + [16] broadcast
    int icp_persistent;      // 1: one launch per frame (k_icp_frame), 0: one launch per iteration
    int pose_alg;            // TF_POSE_ALGEBRA_*: the ICP iterations' det / solve / Rodrigues (tf_icp_tail.h)
    int icp_max_cta;
    int count_lanes;         // frame path: count integration's voxel lanes (profiling)
    long long* integ_cnt;    // [TF_INTEG_WG][2] per-workgroup running counts of voxel lanes read / written
    float min_cosine, dist2_thres;
    // device state
    TfDevState* st;
    TfDevState* st_host;     // pinned mirror
    int frame_counter;       // host mirror of st->frame_counter (updated at every sync)
    int n_resets;            // host mirror of st->n_resets
    int* frame_ok;           // per enqueued frame of a batch: 1 ok, 0 ICP failure (reset), -1 error
    int* frame_mode;         // per enqueued frame of a batch: st->mode it ran with
                             // (both rings follow TfDevState in c->st's allocation, TF_ST_BYTES)
    int alloc_chunks;        // N_tot / 4096
    int vis_chunks;
    // per-stage HIP-event timing on the context stream (tf_profile_*)
    int prof_enabled;
    unsigned prof_mask;      // stages timed (bit = tf_stage_id)
    int prof_period;         // time every prof_period-th enqueued frame (1 = every frame)
    long long prof_seq;      // frames enqueued since profiling was configured
    unsigned char prof_slot_on[TF_PROF_RING];   // batch slot carries stage events
    unsigned char prof_slot_pre[TF_PROF_RING];  // batch slot ran its own preprocessing (no lookahead)
    unsigned prof_slot_stages[TF_PROF_RING];    // batch slot: the stages whose events were recorded
    hipEvent_t prof_ev[2 * TF_NUM_STAGES * TF_PROF_RING];
    // a single-kernel stage being timed: its launch (tf_launch) carries these events, which
    // hipExtLaunchKernelGGL ties to the dispatch's own begin / end (what rocprofv3 reports);
    // event records around a launch were measured to include earlier work (ICP: 148 vs 85 us)
    hipEvent_t ev_start, ev_stop;
    // persistent-ICP ordering among the contexts of one device (tf_icp_order_*, tf_capi.hip)
    hipEvent_t icp_ev;
    // engine entry points over caller buffers: orders the context stream after the legacy
    // default stream the caller's producers (cuda:: imgproc, uploads) run on (order_after_caller)
    hipEvent_t caller_ev;
    double prof_ms[TF_NUM_STAGES];
    long long prof_count[TF_NUM_STAGES];
    // per-call frames (tf_process_frame, TopFu::operator()): the persistent ICP launch writes the
    // frame's verdict (return value, pose) into fine-grained host memory and the call returns on
    // it, with the rest of the frame still running on the stream -- as the reference returns with
    // its CreateICPMaps / resize kernels in flight (topfu.cpp:307-329)
    unsigned long long* verdict_host;    // TF_VERDICT_WORDS words (hipHostMallocCoherent)
    unsigned long long* verdict_dev;     // the same memory as the device addresses it
    unsigned verdict_gen;                // generation of the record being armed
    int verdict_arm;                     // the frame being enqueued writes the verdict
    int percall_early;                   // TFUSION_PERCALL_EARLY (default 1)
    // ... and a per-call frame leaves its last two launches (k_raycast_pair, k_icp_maps_end)
    // unenqueued: the next call enqueues them with its own frame's bilateral and pyramid passes in
    // their grid tails (the batch's lookahead), every other entry point first enqueues them as
    // they are (flush_tail, tf_capi.hip)
    int tail_pending;
    int tail_fuse_ed;
    int percall_defer;                   // TFUSION_PERCALL_DEFER (default 1)
    // persistent-ICP fault injection (tests): the icp_fault_launch-th persistent ICP launch of the
    // context reports a lost peer at iteration icp_fault_iter (TFUSION_ICP_FAULT=launch:iteration)
    long long icp_launches;
    long long icp_fault_launch;
    int icp_fault_iter;
    long long icp_fallbacks;             // frames re-run on the per-iteration schedule after a lost peer
    // ... and the fill_fault_launch-th k_raycast_pair launch's range-image wait fails (TFUSION_FILL_FAULT)
    long long pair_launches;
    long long fill_fault_launch;
    // ... and the vis_fault_launch-th k_vis_build launch's wait for the lower chunks fails (TFUSION_VIS_FAULT)
    long long vis_launches;
    long long vis_fault_launch;
    // engine-level batches (tf_scene_fuse_frames, tf_fuse.hip): the batch's poses and per-frame records
    float* fuse_dists;                   // the second dists buffer of a batch (frame k+1's head runs beside frame k)
    int fuse_tail;                       // TFUSION_FUSE_TAIL (default 1): 4 launches per frame (k_fuse_tail)
    float* fuse_pose;                    // [fuse_cap][12] world -> camera, row-major [R|t]
    int* fuse_rec;                       // [fuse_cap] tf_fuse_record
    int fuse_cap;
};
#define TF_VERDICT_WORDS 16

// the launch of a stage's single kernel: timed by the dispatch's own timestamps when the
// stage is being timed (c->ev_start set by STAGE_ON, consumed here), plain otherwise
template <typename... KArgs, typename... Args>
inline void tf_launch(tf_ctx* c, void (*kern)(KArgs...), dim3 grid, dim3 block, unsigned shm, Args... args)
{
    if (c->ev_start) {
        hipExtLaunchKernelGGL(kern, grid, block, shm, c->stream, c->ev_start, c->ev_stop, 0, args...);
        c->ev_start = c->ev_stop = nullptr;
    } else {
        hipLaunchKernelGGL(kern, grid, block, shm, c->stream, args...);
    }
}

// ---------------------------------------------------------------------------------------
// launchers (one per kernel family); all enqueue on ctx->stream
// ---------------------------------------------------------------------------------------
hipError_t tfk_preprocess(tf_ctx* c, const uint16_t* depth, size_t pitch, hipStream_t strm, uint16_t* d0);   // no st access
// fold_t3: k_set_type3's work in the persistent ICP grid's tail (frame path; the caller then
// passes snapshot = 2 to tfk_alloc)
hipError_t tfk_icp(tf_ctx* c, int pose_update, int frame_begin = 0, int fold_t3 = 0);
// Persistent ICP launches of different contexts on one device must not run at the same time:
// each needs all 256 of its workgroups resident at once (one per CU) and spins on the others, so
// two of them dispatched together could each hold part of the chip and wait on each other.  With
// more than one context on a device, every persistent ICP launch waits (on the device) for the
// previous one of another context.  One context per device (the bench, C4) waits on nothing.
hipError_t tf_icp_order_before(tf_ctx* c);
hipError_t tf_icp_order_after(tf_ctx* c);   // frame_begin: frame path (tf_frame_begin)
int tfk_icp_persistent_ok(tf_ctx* c);      // k_icp_frame fits (co-residency, slot count)
hipError_t tfk_pose_from_input(tf_ctx* c, int mode);   // pose_in -> alloc / raycast matrices
// clear_cache: also empty the GlobalCache (TopFu-level resets); 0 = the engine's ResetScene
hipError_t tfk_reset_scene(tf_ctx* c, int clear_cache = 1);
hipError_t tfk_reset_scene_on_failure(tf_ctx* c, int slot);   // frame end + ResetScene if ICP failed
hipError_t tfk_grid_rebuild(tf_ctx* c);   // block grid from the hash (after a hash upload)
hipError_t tfk_grid_clear(tf_ctx* c);     // every cell (-1, TF_VOFF_NONE)
hipError_t tfk_check_div3(tf_ctx* c, float d, int* ok);   // tf_div_exact3(x, d) == x / d over a binade
// a later frame of the batch whose preprocessing (part) runs in a frame kernel's grid tail
struct TfAhead {
    const uint16_t* src;     // raw depth (nullptr: none)
    uint16_t* d0;            // its level-0 depth buffer (d0_buf)
};
hipError_t tfk_alloc(tf_ctx* c, int snapshot = 0,       // snapshot: + the frame's renderImage snapshot
                     TfAhead bil = TfAhead{}, size_t pitch = 0,    // bil: + that frame's bilateral pass
                     int only_update = 0);    // onlyUpdateVisibleList: requests are discarded, not allocated
// frame_path: + frame-0 map copy; with_ed: CreateExpectedDepths' projection pass in the
// grid's first TF_ED_BLOCKS workgroups (then tfk_expected_depths(c, 1) runs only the fill)
hipError_t tfk_integrate(tf_ctx* c, int frame_path = 0, int with_ed = 0);
hipError_t tfk_fuse_head(tf_ctx* c, const uint16_t* frame, size_t pitch, float* dists, const float* pose);
hipError_t tfk_fuse_tail(tf_ctx* c, const float* pose, int* rec, const uint16_t* next_frame, size_t pitch,
                         float* next_dists, const float* next_pose);
hipError_t tfk_raycast(tf_ctx* c, int update_visible);
hipError_t tfk_render_type(tf_ctx* c, int type);   // RenderImage pixel stage (tf_render_type) on raycast
// CreateICPMaps raycast + renderImage, one launch (frame path); next: + that frame's dists/pyramid/normals
// + dists/pyramid/normals of pyr, bilateral of bil; fuse_ed: CreateExpectedDepths' fill in the same
// grid (frame path, when tfk_ed_fused: then no separate tfk_expected_depths launch)
hipError_t tfk_raycast_pair(tf_ctx* c, TfAhead pyr = TfAhead{}, TfAhead bil = TfAhead{}, size_t pitch = 0, int fuse_ed = 0,
                            int ljf = 0);
#define TF_LJF_MAX 1024          // tiles per XCD region the longest-first ordering sorts (one LDS sort)
hipError_t tfk_tile_order_init(tf_ctx* c);   // the XCD-swizzled order, zero costs
// the raycast pair on its own (tf_time_stage, C3R) with the frame path's tile order: the pair
// launch, then the order sort the frame path runs in k_icp_maps_end's grid
hipError_t tfk_raycast_pair_ordered(tf_ctx* c);
// the i-th tile of XCD x's share (-1: none), and the share's size; per = slots / 8
__host__ __device__ __forceinline__ int tf_tile_of(int x, int i, int n, int tx, int ty, int per, int rows)
{
    if (rows) { const int r = x + 8 * (i / tx); return r < ty ? r * tx + i % tx : -1; }
    const int t = x * per + i;
    return (i < per && t < n) ? t : -1;
}
__host__ __device__ __forceinline__ int tf_tile_count(int x, int n, int tx, int ty, int per, int rows)
{
    if (rows) return ty > x ? ((ty - x + 7) / 8) * tx : 0;
    const int c = n - x * per;
    return c < 0 ? 0 : (c < per ? c : per);
}
int tfk_ed_fused(const tf_ctx* c);
hipError_t tfk_icp_maps(tf_ctx* c);
hipError_t tfk_render_snapshot(tf_ctx* c);   // render_snapshot as its own launch
// CreateICPMaps + the frame end (tfk_reset_scene_on_failure) in one grid (the frame path)
// pyr: + that frame's dists / pyramid / normals pass (its level-0 depth already in pyr.d0)
hipError_t tfk_icp_maps_end(tf_ctx* c, int slot, TfAhead pyr = TfAhead{}, size_t pitch = 0);
#define TF_END_BLOCKS 256        // workgroups of the frame-end / in-frame reset pass
// keep_bins: the fill leaves the projection's bins in place (repeated fills of tf_time_stage)
hipError_t tfk_expected_depths(tf_ctx* c, int project_done = 0, int keep_bins = 0);
#define TF_ED_BLOCKS 256         // workgroups of the expected-depth projection pass
#define ED_MAX_W 4096            // k_ed_fill: columns of a row held in LDS (wider images: atomics past it)
#define ED_XROWS 8               // k_ed_fill: LDS rows below the /8 region (where boxes spill)
static inline int ed_nrows(int H) { const int n = (H - 1) / TF_SUBSAMPLE + 1 + ED_XROWS; return n < H ? n : H; }
#define ED_LDS_MAX_N 16384       // k_ed_fill: per-/8-row LDS reduction up to this many visible entries
hipError_t ed_spill_all(tf_ctx* c);   // mark the whole range buffer for clearing by the next projection pass
#define TF_INTEG_WG 2560         // workgroups of the stand-alone integration pass (grid-stride; 2 rounds of 5 per CU)
#define TF_INTEG_WG_FRAME 768    // ... in the frame path (C2-size lists: 3 resident rounds of 256 WGs instead of 2048)
hipError_t tfk_frame0_matrices(tf_ctx* c);
// swapping (tf_swap.hip): reallocation of listed swapped-out entries (after the visible list),
// and IntegrateGlobalIntoLocal + SaveToGlobalMemory (after integration)
hipError_t tfk_swap_realloc(tf_ctx* c);
hipError_t tfk_swap(tf_ctx* c, int which = 3);   // 1 in, 2 out, 3 both

enum { TF_POSE_ALLOC = 1, TF_POSE_RAY = 2, TF_POSE_ALLOC_NOINV = 4 };
