// tf_capi.hip -- context management, frame orchestration and the C-ABI of libtfusion_hip.
//
// TopFu::operator() (tfusion/src/topfu.cpp:161-330) becomes a fixed sequence of kernels on
// the context's stream with ONE host synchronisation at the end of the frame (the
// reference has ~27).  ICP, pose algebra and every counter live on the device
// (TfDevState); the host only reads the frame's bool + counters back.
#include "tf_internal.h"

#include <vector>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <new>

#define TF_CHECK(expr)                                   \
    do {                                                 \
        hipError_t e_ = (expr);                          \
        if (e_ != hipSuccess) return tf_from_hip(e_);    \
    } while (0)

static tf_status tf_from_hip(hipError_t e)
{
    if (e == hipSuccess) return TF_OK;
    if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) return TF_OOM;
    if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return TF_NO_DEVICE;
    return TF_HIP_ERROR;
}

extern "C" const char* tf_status_string(tf_status s)
{
    switch (s) {
    case TF_OK: return "ok";
    case TF_ICP_FAIL: return "icp failed (scene reset)";
    case TF_INVALID_ARG: return "invalid argument";
    case TF_OOM: return "out of device memory";
    case TF_HIP_ERROR: return "HIP error";
    case TF_NO_DEVICE: return "no HIP device";
    }
    return "unknown";
}

extern "C" tf_status tf_device_count(int* count)
{
    if (!count) return TF_INVALID_ARG;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e == hipErrorNoDevice) { *count = 0; return TF_OK; }
    if (e != hipSuccess) { *count = 0; return tf_from_hip(e); }
    *count = n;
    return TF_OK;
}

extern "C" tf_status tf_set_device(int device) { return tf_from_hip(hipSetDevice(device)); }

extern "C" tf_status tf_default_params(tf_params* p)
{   // TopFuParams::default_params (topfu.cpp:12-53) + SceneParams(0.02, 100, 0.005, 0.2, 3.0) (:50)
    if (!p) return TF_INVALID_ARG;
    memset(p, 0, sizeof(*p));
    p->cols = 640; p->rows = 480;
    p->fx = 504.261f; p->fy = 503.905f; p->cx = 352.457f; p->cy = 272.202f;
    p->bilateral_sigma_depth = 0.04f;
    p->bilateral_sigma_spatial = 4.5f;
    p->bilateral_kernel_size = 7;
    p->icp_truncate_depth_dist = 2.0f;
    p->icp_dist_thres = 0.1f;
    p->icp_angle_thres = 30.f * 0.017453293f;
    p->icp_iter_num[0] = 10; p->icp_iter_num[1] = 5; p->icp_iter_num[2] = 4; p->icp_iter_num[3] = 0;
    p->mu = 0.02f; p->maxW = 100; p->voxelSize = 0.005f;
    p->viewFrustum_min = 0.2f; p->viewFrustum_max = 3.0f;
    p->n_buckets = 0x100000; p->n_excess = 0x20000; p->n_blocks = 0x10000;
    p->vis_capacity = 0x40000;
    p->max_render_blocks = 65536 * 4;
    p->use_swapping = 0;                          // Scene(params, false), topfu.cpp:67
    p->swap_transfer_blocks = 0x1000;             // SDF_TRANSFER_BLOCK_NUM, VoxelBlockHash.hpp:27
    p->voxel_rgb = 0;                             // Voxel_s (Defines.hpp:5)
    p->depth_to_rgb[0] = p->depth_to_rgb[5] = p->depth_to_rgb[10] = 1.0f;   // registered RGB-D
    return TF_OK;
}

static bool params_valid(const tf_params* p)
{
    if (p->cols <= 0 || p->rows <= 0 || (p->cols % 4) || (p->rows % 4)) return false;
    if (p->n_buckets <= 0 || (p->n_buckets & (p->n_buckets - 1))) return false;
    if (p->n_excess <= 0 || p->n_blocks <= 0 || p->vis_capacity <= 0 || p->max_render_blocks <= 0) return false;
    // The render side forms 32-bit byte offsets (voff + guard shift + lin) * 4 from the guard
    // block before the VBA (tf_render.hip vox_at): block ptr p reads up to 4 * ((p + 2) * 512 - 1)
    // bytes past the guard, which fits 2^32 only for p <= 2^21 - 2, i.e. n_blocks <= 2^21 - 1.
    if (p->n_blocks > (1 << 21) - 1) return false;
    if ((p->n_buckets + p->n_excess) % 16) return false;
    if (p->bilateral_kernel_size < 1 || p->bilateral_kernel_size > 7) return false;
    if (p->voxelSize <= 0 || p->mu <= 0) return false;
    // steps per pixel ceil(2*|e-s|) with |e-s| ~ 2*mu/(8*voxel) must fit the 6-bit key field
    if (4.0f * p->mu / (8.0f * p->voxelSize) + 2.0f > 60.0f) return false;
    if ((double)p->cols * p->rows * 64.0 > 2147483000.0) return false;
    if (p->cols > 65535 || p->rows > 65535) return false;               // k_ed_fill's 16-bit box records
    if (p->use_swapping && (p->swap_transfer_blocks <= 0 || p->swap_transfer_blocks > p->n_buckets + p->n_excess)) return false;
    // the GlobalCache holds Voxel_s blocks: a swapping colour scene would need the colour half
    // swapped too (CombineVoxelInformation's colour part) -- not built
    if (p->voxel_rgb && p->use_swapping) return false;
    return true;
}

// ---------------------------------------------------------------------------------------
// persistent-ICP ordering among the contexts of one device (see tf_internal.h)
// ---------------------------------------------------------------------------------------
#include <mutex>
#define TF_MAX_DEVICES 64
static std::mutex g_icp_mu;
static int g_icp_ctx_count[TF_MAX_DEVICES];          // live contexts per device
static tf_ctx* g_icp_last[TF_MAX_DEVICES];          // context of the last persistent ICP launch

static void icp_order_register(tf_ctx* c, int add)
{
    if (c->device < 0 || c->device >= TF_MAX_DEVICES) return;
    std::lock_guard<std::mutex> lk(g_icp_mu);
    g_icp_ctx_count[c->device] += add;
    if (add < 0 && g_icp_last[c->device] == c) g_icp_last[c->device] = nullptr;
    // a single context records nothing (an event record per frame costs the device ~4 us): when
    // a second one arrives, the last launcher's stream is marked here, so the newcomer's first
    // ICP waits for everything already enqueued there
    tf_ctx* last = g_icp_last[c->device];
    if (add > 0 && last && last != c) (void)hipEventRecord(last->icp_ev, last->stream);
}

// called with the launch enqueued between before() and after(), from one host thread per context
hipError_t tf_icp_order_before(tf_ctx* c)
{
    if (c->device < 0 || c->device >= TF_MAX_DEVICES || !c->icp_ev) return hipSuccess;
    g_icp_mu.lock();                                  // released by tf_icp_order_after
    tf_ctx* last = g_icp_last[c->device];
    if (g_icp_ctx_count[c->device] > 1 && last && last != c) return hipStreamWaitEvent(c->stream, last->icp_ev, 0);
    return hipSuccess;
}

hipError_t tf_icp_order_after(tf_ctx* c)
{
    if (c->device < 0 || c->device >= TF_MAX_DEVICES || !c->icp_ev) return hipSuccess;
    const hipError_t e = g_icp_ctx_count[c->device] > 1 ? hipEventRecord(c->icp_ev, c->stream) : hipSuccess;
    g_icp_last[c->device] = c;
    g_icp_mu.unlock();
    return e;
}

static void ctx_free(tf_ctx* c)
{
    if (!c) return;
    if (c->icp_ev) {
        icp_order_register(c, -1);
        (void)hipEventDestroy(c->icp_ev);
    }
    if (c->caller_ev) (void)hipEventDestroy(c->caller_ev);
    void* bufs[] = { c->hash, c->excessList, c->vba_guard, c->allocList, c->bgrid, c->allocType, c->winnerKey, c->allocCounts,
                     c->visCounts, c->visAgg, c->visibleIds, c->visType, c->range, c->range_render, c->raycast, c->grey,
                     c->blockRec, c->blockTiles, c->blockOff, c->edChunk, c->edSpill, c->edBins, c->edBinCnt, c->edDone, c->depth_in, c->dists, c->icp_partial, c->icp_ticket, c->icp_tagged, c->st,
                     c->swapState, c->swapFlags, c->swapStore, c->swapCounts,
                     c->vba_rgb_guard, c->rgb_in, c->integ_cnt, c->fuse_pose, c->fuse_rec, c->fuse_dists, c->tile_cost, c->tile_order };
    for (void* b : bufs) if (b) (void)hipFree(b);
    // pyramid maps: one allocation per map (level 0 is the base; swaps keep levels together)
    float4* maps[4] = { c->curr_pts[0], c->curr_nrm[0], c->prev_pts[0], c->prev_nrm[0] };
    for (float4* m : maps) if (m) (void)hipFree(m);
    for (int l = 1; l < TF_LEVELS; ++l) if (c->depth_pyr[l]) (void)hipFree(c->depth_pyr[l]);
    for (int k = 0; k < 2; ++k) if (c->d0_buf[k]) (void)hipFree(c->d0_buf[k]);
    if (c->st_host) (void)hipHostFree(c->st_host);
    if (c->verdict_host) (void)hipHostFree(c->verdict_host);
    for (int i = 0; i < 2 * TF_NUM_STAGES * TF_PROF_RING; ++i) if (c->prof_ev[i]) (void)hipEventDestroy(c->prof_ev[i]);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

template <class T>
static hipError_t dalloc(T** p, size_t bytes)
{
    return hipMalloc((void**)p, bytes < 16 ? 16 : bytes);
}

// A deferred per-call frame's last two launches (TfFramePlan::defer_tail): CreateICPMaps' raycast
// + renderImage (+ CreateExpectedDepths' fill), then CreateICPMaps + the frame end.  nxt: the next
// frame, whose bilateral pass joins the first grid and whose dists / pyramid / normals pass the
// second (the batch's lookahead, enqueue_frame); none when flushed for another entry point.
static tf_status flush_tail(tf_ctx* c, TfAhead nxt = TfAhead{}, size_t pitch = 0)
{
    if (!c->tail_pending) return TF_OK;
    c->tail_pending = 0;
    TF_CHECK(tfk_raycast_pair(c, TfAhead{}, nxt, pitch, c->tail_fuse_ed, 1));
    TF_CHECK(tfk_icp_maps_end(c, 0, nxt, pitch));
    return TF_OK;
}
// every entry point but the per-call frame itself first completes a deferred frame's launches
#define TF_FLUSH(c) do { if (c) { const tf_status fs_ = flush_tail(c); if (fs_ != TF_OK) return fs_; } } while (0)

static tf_status sync_state(tf_ctx* c)
{
    TF_CHECK(hipMemcpyAsync(c->st_host, c->st, sizeof(TfDevState), hipMemcpyDeviceToHost, c->stream));
    TF_CHECK(hipStreamSynchronize(c->stream));
    // a frame that failed past its ICP (tf_reset.h: frame_ok -3) left the context in error until
    // tf_reset -- also when the call that enqueued it had already returned (per-call frames)
    if (c->st_host->sticky_error) return TF_HIP_ERROR;
    return TF_OK;
}

// the end of every synchronous entry point: wait for the stream, then report a context left in
// error by a device-side failure past an ICP (tf_reset.h: frame_ok -3) or by an engine-level
// launch's failed wait (k_vis_build) -- TF_HIP_ERROR from every call until tf_reset
static tf_status sync_checked(tf_ctx* c)
{
    TF_CHECK(hipMemcpyAsync(&c->st_host->sticky_error, &c->st->sticky_error, sizeof(int), hipMemcpyDeviceToHost,
                            c->stream));
    TF_CHECK(hipStreamSynchronize(c->stream));
    return c->st_host->sticky_error ? TF_HIP_ERROR : TF_OK;
}

// TopFu::reset (topfu.cpp:141-152): pose history -> [I], ResetScene.  The render state
// (visible list / types / range image) is deliberately left as is, like the reference.
__global__ void k_host_reset(TfDevState* st)
{
    st->halt = 0;                      // (a device-side failure is cleared by the reset)
    st->sticky_error = 0;
    if (st->frame_counter) st->n_resets++;
    st->frame_counter = 0;
    for (int i = 0; i < 12; ++i) st->pose[i] = (i % 5 == 0) ? 1.0f : 0.0f;
}

static tf_status ctx_reset(tf_ctx* c)
{
    hipLaunchKernelGGL(k_host_reset, dim3(1), dim3(1), 0, c->stream, c->st);
    TF_CHECK(hipGetLastError());
    TF_CHECK(tfk_reset_scene(c));
    const tf_status s = sync_state(c);
    if (s != TF_OK) return s;
    c->frame_counter = c->st_host->frame_counter;
    c->n_resets = c->st_host->n_resets;
    return TF_OK;
}

extern "C" tf_status tf_create(const tf_params* pin, tf_ctx** out)
{
    if (!pin || !out) return TF_INVALID_ARG;
    *out = nullptr;
    if (!params_valid(pin)) return TF_INVALID_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return TF_NO_DEVICE;
    tf_ctx* c = new (std::nothrow) tf_ctx;
    if (!c) return TF_OOM;
    memset((void*)c, 0, sizeof(*c));
    c->p = *pin;
    c->prof_period = 1;
    hipError_t e = hipGetDevice(&c->device);
    if (e != hipSuccess) { ctx_free(c); return tf_from_hip(e); }
    c->W = pin->cols; c->H = pin->rows;
    c->n_total = pin->n_buckets + pin->n_excess;
    for (int l = 0, w = c->W, h = c->H; l < TF_LEVELS; ++l, w /= 2, h /= 2) { c->lw[l] = w; c->lh[l] = h; }
    c->alloc_chunks = (c->n_total + 4095) / 4096;
    c->vis_chunks = c->alloc_chunks;
    const size_t npx = (size_t)c->W * c->H;
    const size_t ntot_pad = (size_t)c->alloc_chunks * 4096;
    c->icp_max_cta = ((c->W + 31) / 32) * ((c->H + 7) / 8);
    // ComputeIcpHelper ctor (projective_icp.cpp:11-15), evaluated on the host like the reference
    c->min_cosine = cosf(pin->icp_angle_thres);
    c->dist2_thres = pin->icp_dist_thres * pin->icp_dist_thres;
#define ALLOC(ptr, bytes) do { e = dalloc(&(ptr), (bytes)); if (e != hipSuccess) { ctx_free(c); return tf_from_hip(e); } } while (0)
    e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->caller_ev, hipEventDisableTiming);
    if (e != hipSuccess) { ctx_free(c); return tf_from_hip(e); }
    ALLOC(c->hash, sizeof(TfHashEntry) * (size_t)c->n_total);
    ALLOC(c->excessList, sizeof(int) * (size_t)pin->n_excess);
    ALLOC(c->vba_guard, sizeof(TfVoxel) * ((size_t)pin->n_blocks + 1) * TF_BLK3);
    c->vba = c->vba_guard + TF_BLK3;
    ALLOC(c->allocList, sizeof(int) * (size_t)pin->n_blocks);
    ALLOC(c->bgrid, sizeof(int2) * (size_t)TF_GRID_DIM * TF_GRID_DIM * TF_GRID_DIM);
    ALLOC(c->allocType, ntot_pad);
    ALLOC(c->winnerKey, sizeof(int) * ntot_pad);
    ALLOC(c->allocCounts, sizeof(int) * 2 * (size_t)c->alloc_chunks);
    ALLOC(c->visCounts, sizeof(int) * (size_t)c->vis_chunks);
    ALLOC(c->visAgg, sizeof(unsigned long long) * (size_t)c->vis_chunks);
    {   // TFUSION_VIS_FUSED=0: the two-launch visible-list build (A/B)
        const char* env = getenv("TFUSION_VIS_FUSED");
        c->vis_fused = !(env && env[0] == '0');
        c->vis_gen = 0;
    }
    ALLOC(c->visibleIds, sizeof(int) * (size_t)pin->vis_capacity);
    ALLOC(c->visType, ntot_pad);
    ALLOC(c->range, sizeof(float) * 2 * npx);
    ALLOC(c->range_render, sizeof(float) * 2 * npx);
    ALLOC(c->raycast, sizeof(float) * 4 * npx);
    ALLOC(c->grey, sizeof(uchar4) * npx);
    ALLOC(c->blockRec, sizeof(uint4) * (size_t)pin->vis_capacity);
    ALLOC(c->blockTiles, sizeof(int) * (size_t)pin->vis_capacity);
    ALLOC(c->blockOff, sizeof(int) * (size_t)pin->vis_capacity);
    ALLOC(c->edChunk, sizeof(int) * ((size_t)pin->vis_capacity / 256 + 1));
    ALLOC(c->edSpill, sizeof(int2) * (size_t)ed_nrows(c->H));
    {   // k_ed_fill: LDS rows up to ED_LDS_MAX_N visible entries, device-scope atomics past that
        // (TFUSION_ED_LDS_MAX_N overrides the threshold; the parity tests run both paths)
        const char* env = getenv("TFUSION_ED_LDS_MAX_N");
        c->ed_lds_max_n = env ? atoi(env) : ED_LDS_MAX_N;
        if (c->ed_lds_max_n > ED_LDS_MAX_N) c->ed_lds_max_n = ED_LDS_MAX_N;
        if (c->ed_lds_max_n > pin->vis_capacity) c->ed_lds_max_n = pin->vis_capacity;   // (a bin holds <= n boxes)
        // the binned boxes hold 12-bit coordinates (tf_ed.h ed_bin_pack), the fill's LDS rows ED_MAX_ROWS
        if (c->W > ED_MAX_W || c->H > ED_MAX_W || c->ed_lds_max_n < 0) c->ed_lds_max_n = 0;
    }
    // the row bins exist only where binning can run: 2 bins per fill row of ed_lds_max_n boxes each
    if (c->ed_lds_max_n > 0) ALLOC(c->edBins, sizeof(uint4) * 2 * (size_t)ed_nrows(c->H) * (size_t)c->ed_lds_max_n);
    ALLOC(c->edBinCnt, sizeof(int) * 2 * (size_t)ed_nrows(c->H));
    ALLOC(c->edDone, 64);
    {   // the raycast tiles' dispatch order, longest first per XCD region (k_raycast_pair, sorted in
        // k_icp_maps_end's grid from the last frame's workgroup times); TFUSION_TILE_ORDER=0: the plain
        // XCD-swizzled order (A/B)
        // TFUSION_TILE_MAP=rows: XCD x takes the tile rows = x (mod 8) instead of the x-th band
        const int tx = (c->W + 15) / 16, ty = (c->H + 15) / 16, nt = tx * ty;
        const char* env = getenv("TFUSION_TILE_ORDER");
        const char* map = getenv("TFUSION_TILE_MAP");
        c->tile_rows = map && strcmp(map, "rows") == 0;
        c->tile_slots = c->tile_rows ? 8 * ((ty + 7) / 8) * tx : (nt + 7) / 8 * 8;
        c->tile_ljf = c->tile_slots / 8 <= TF_LJF_MAX && !(env && env[0] == '0');
        ALLOC(c->tile_cost, sizeof(unsigned) * 2 * (size_t)nt);
        ALLOC(c->tile_order, sizeof(int) * 2 * (size_t)c->tile_slots);
    }
    ALLOC(c->depth_in, sizeof(uint16_t) * npx);
    ALLOC(c->dists, sizeof(float) * npx);
    {   // each map's three pyramid levels are contiguous in one allocation
        size_t ntot = 0;
        for (int l = 0; l < TF_LEVELS; ++l) ntot += (size_t)c->lw[l] * c->lh[l];
        ALLOC(c->curr_pts[0], sizeof(float4) * ntot);
        ALLOC(c->curr_nrm[0], sizeof(float4) * ntot);
        ALLOC(c->prev_pts[0], sizeof(float4) * ntot);
        ALLOC(c->prev_nrm[0], sizeof(float4) * ntot);
        for (int l = 1; l < TF_LEVELS; ++l) {
            const size_t off = (size_t)c->lw[l - 1] * c->lh[l - 1];
            c->curr_pts[l] = c->curr_pts[l - 1] + off; c->curr_nrm[l] = c->curr_nrm[l - 1] + off;
            c->prev_pts[l] = c->prev_pts[l - 1] + off; c->prev_nrm[l] = c->prev_nrm[l - 1] + off;
        }
        for (int l = 1; l < TF_LEVELS; ++l) ALLOC(c->depth_pyr[l], sizeof(uint16_t) * (size_t)c->lw[l] * c->lh[l]);
        for (int k = 0; k < 2; ++k) ALLOC(c->d0_buf[k], sizeof(uint16_t) * (size_t)c->lw[0] * c->lh[0]);
        c->depth_pyr[0] = c->d0_buf[0];
    }
    ALLOC(c->icp_partial, sizeof(float) * 28 * 256);
    ALLOC(c->icp_ticket, 64);
    ALLOC(c->icp_tagged, sizeof(unsigned long long) * TF_ICP_TAG_WORDS);
    // the device state, then the per-slot ok / mode rings: one copy back per host sync
    ALLOC(c->st, TF_ST_BYTES);
    c->frame_ok = (int*)(c->st + 1);
    c->frame_mode = c->frame_ok + TF_PROF_RING;
    ALLOC(c->integ_cnt, sizeof(long long) * 2 * TF_INTEG_WG);
    if (pin->use_swapping) {        // the GlobalCache in HBM: 2 KiB per hash entry + flags
        ALLOC(c->swapState, ntot_pad);
        ALLOC(c->swapFlags, ntot_pad);
        ALLOC(c->swapStore, sizeof(TfVoxel) * (size_t)c->n_total * TF_BLK3);
        ALLOC(c->swapCounts, sizeof(int) * 2 * (size_t)c->alloc_chunks);
        e = hipMemsetAsync(c->swapState, 0, ntot_pad, c->stream);
        if (e == hipSuccess) e = hipMemsetAsync(c->swapFlags, 0, ntot_pad, c->stream);
        if (e != hipSuccess) { ctx_free(c); return tf_from_hip(e); }
    }
    if (pin->voxel_rgb) {           // the Voxel_s_rgb colour plane (guard block + n_blocks blocks of 2 KiB)
        const size_t nb = sizeof(unsigned) * ((size_t)pin->n_blocks + 1) * TF_BLK3;
        ALLOC(c->vba_rgb_guard, nb);
        c->vba_rgb = c->vba_rgb_guard + TF_BLK3;
        ALLOC(c->rgb_in, sizeof(uchar4) * npx);
        e = hipMemsetAsync(c->vba_rgb_guard, 0, nb, c->stream);
        if (e != hipSuccess) { ctx_free(c); return tf_from_hip(e); }
    }
#undef ALLOC
    e = hipHostMalloc((void**)&c->st_host, TF_ST_BYTES, hipHostMallocDefault);
    // per-call frames: the verdict record in fine-grained host memory (written by the ICP launch
    // with system-scope stores)
    if (e == hipSuccess)
        e = hipHostMalloc((void**)&c->verdict_host, sizeof(unsigned long long) * TF_VERDICT_WORDS, hipHostMallocCoherent);
    if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&c->verdict_dev, c->verdict_host, 0);
    if (e != hipSuccess) { ctx_free(c); return tf_from_hip(e); }
    memset(c->verdict_host, 0, sizeof(unsigned long long) * TF_VERDICT_WORDS);
    {   // TFUSION_ICP_FAULT=launch:iteration (tests): that persistent ICP launch of the context reports a
        // lost peer at that iteration, so the run-time fallback to the per-iteration schedule runs
        const char* env = getenv("TFUSION_ICP_FAULT");
        long long fl = 0; int fi = -1;
        if (env && sscanf(env, "%lld:%d", &fl, &fi) == 2 && fl > 0 && fi >= 0) { c->icp_fault_launch = fl; c->icp_fault_iter = fi; }
        else { c->icp_fault_launch = 0; c->icp_fault_iter = -1; }
        // TFUSION_FILL_FAULT=launch: that k_raycast_pair launch's wait for the range image fails
        // (past the ICP: the sticky-error path)
        env = getenv("TFUSION_FILL_FAULT");
        c->fill_fault_launch = env ? atoll(env) : 0;
        // TFUSION_FUSE_TAIL=0: engine batches in the 7-launch form (A/B)
        env = getenv("TFUSION_FUSE_TAIL");
        c->fuse_tail = !(env && env[0] == '0');
        // TFUSION_VIS_FAULT=launch: that k_vis_build launch's wait for the lower chunks' counts fails
        env = getenv("TFUSION_VIS_FAULT");
        c->vis_fault_launch = env ? atoll(env) : 0;
    }
    {   // TFUSION_PERCALL_EARLY=0: per-call frames wait for the whole frame; TFUSION_PERCALL_DEFER=0:
        // they enqueue all their launches (A/B)
        const char* env = getenv("TFUSION_PERCALL_EARLY");
        c->percall_early = !(env && env[0] == '0');
        env = getenv("TFUSION_PERCALL_DEFER");
        c->percall_defer = !(env && env[0] == '0');
    }
    // initial device state
    TfDevState s0;
    memset(&s0, 0, sizeof(s0));
    for (int i = 0; i < 12; ++i) s0.pose[i] = (i % 5 == 0) ? 1.0f : 0.0f;
    s0.icp_ok = 1;
    e = hipMemcpyAsync(c->st, &s0, sizeof(s0), hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipMemsetAsync(c->icp_ticket, 0, 64, c->stream);
    if (e == hipSuccess) e = tfk_grid_clear(c);
    if (e == hipSuccess) e = hipMemsetD32Async((hipDeviceptr_t)c->vba_guard, 0x7fff, TF_BLK3, c->stream);   // Voxel_s()
    if (e == hipSuccess) e = hipMemsetAsync(c->icp_tagged, 0, sizeof(unsigned long long) * TF_ICP_TAG_WORDS, c->stream);
    if (e == hipSuccess) e = hipMemsetAsync(c->integ_cnt, 0, sizeof(long long) * 2 * TF_INTEG_WG, c->stream);
    if (e == hipSuccess) e = hipMemsetAsync(c->visAgg, 0, sizeof(unsigned long long) * (size_t)c->vis_chunks, c->stream);   // no tag yet
    if (e == hipSuccess) e = hipMemsetAsync(c->allocType, 0, ntot_pad, c->stream);
    if (e == hipSuccess) e = hipMemsetAsync(c->winnerKey, 0xff, sizeof(int) * ntot_pad, c->stream);
    // the request pass counts into these; every frame's k_vis_count returns them to zero
    if (e == hipSuccess) e = hipMemsetAsync(c->allocCounts, 0, sizeof(int) * 2 * (size_t)c->alloc_chunks, c->stream);
    if (e == hipSuccess) e = hipMemsetAsync(c->visType, 0, ntot_pad, c->stream);
    if (e == hipSuccess) e = hipMemsetAsync(c->visibleIds, 0, sizeof(int) * (size_t)pin->vis_capacity, c->stream);
    if (e == hipSuccess) e = hipMemsetAsync(c->raycast, 0, sizeof(float) * 4 * npx, c->stream);
    if (e == hipSuccess) e = hipMemsetAsync(c->edBinCnt, 0, sizeof(int) * 2 * (size_t)ed_nrows(c->H), c->stream);
    if (e == hipSuccess) e = hipMemsetAsync(c->edDone, 0, 64, c->stream);
    if (e == hipSuccess) e = tfk_tile_order_init(c);
    if (e == hipSuccess) e = hipMemsetAsync(c->grey, 0, sizeof(uchar4) * npx, c->stream);
    for (int l = 0; l < TF_LEVELS && e == hipSuccess; ++l) {
        size_t n = (size_t)c->lw[l] * c->lh[l];
        e = hipMemsetAsync(c->prev_pts[l], 0, sizeof(float4) * n, c->stream);
        if (e == hipSuccess) e = hipMemsetAsync(c->prev_nrm[l], 0, sizeof(float4) * n, c->stream);
        if (e == hipSuccess) e = hipMemsetAsync(c->curr_pts[l], 0, sizeof(float4) * n, c->stream);
        if (e == hipSuccess) e = hipMemsetAsync(c->curr_nrm[l], 0, sizeof(float4) * n, c->stream);
    }
    if (e != hipSuccess) { ctx_free(c); return tf_from_hip(e); }
    {   // RenderState ctor: renderingRangeImage = (viewFrustum_min, viewFrustum_max) (RenderState.hpp:56-76)
        float2* tmp = (float2*)malloc(sizeof(float2) * npx);
        if (!tmp) { ctx_free(c); return TF_OOM; }
        for (size_t i = 0; i < npx; ++i) tmp[i] = make_float2(pin->viewFrustum_min, pin->viewFrustum_max);
        e = hipMemcpy(c->range, tmp, sizeof(float2) * npx, hipMemcpyHostToDevice);
        free(tmp);
        if (e == hipSuccess) e = ed_spill_all(c);       // the first CreateExpectedDepths clears the whole buffer
        if (e != hipSuccess) { ctx_free(c); return tf_from_hip(e); }
    }
    {   // integration grid of the frame path (TFUSION_INTEG_WG_FRAME overrides; A/B)
        const char* env = getenv("TFUSION_INTEG_WG_FRAME");
        c->integ_wg_frame = env ? atoi(env) : TF_INTEG_WG_FRAME;
        if (c->integ_wg_frame < 64 || c->integ_wg_frame > TF_INTEG_WG) c->integ_wg_frame = TF_INTEG_WG;
    }
    e = tfk_reset_scene(c);                              // topfu.cpp:75
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess) e = tfk_check_div3(c, pin->mu, &c->mu_exact3);   // integrate: eta / mu
    if (e != hipSuccess) { ctx_free(c); return tf_from_hip(e); }
    {   // the ICP iterations' pose algebra (tf_set_pose_algebra): by default the reference's own,
        // cv::determinant / cv::solve(DECOMP_SVD) / Affine3f as OpenCV 3.x-4.x write them;
        // TFUSION_ICP_SOLVE=opencv2 (OpenCV 2.4.9) or canonical (the short block-Schur tail)
        const char* env = getenv("TFUSION_ICP_SOLVE");
        c->pose_alg = !env ? TF_POSE_ALGEBRA_OPENCV4
                    : !strcmp(env, "canonical") ? TF_POSE_ALGEBRA_CANONICAL
                    : !strcmp(env, "opencv2") ? TF_POSE_ALGEBRA_OPENCV2 : TF_POSE_ALGEBRA_OPENCV4;
    }
    {   // ICP: one persistent launch per frame when all its workgroups fit at once; otherwise (or
        // with TFUSION_ICP_PERSISTENT=0) one k_icp_iter launch per iteration
        const char* env = getenv("TFUSION_ICP_PERSISTENT");
        c->icp_persistent = (env && env[0] == '0') ? 0 : tfk_icp_persistent_ok(c);
    }
    if (c->icp_persistent) {
        // ordering only (the contexts share no memory): no system-scope fence at the record --
        // with it, each record wrote back and invalidated the caches, a ~5 us dispatch gap after
        // every persistent ICP launch while two contexts exist (TF_ICP_EV_SYSFENCE=1: the old event)
#ifndef TF_ICP_EV_SYSFENCE
#define TF_ICP_EV_SYSFENCE 0
#endif
        e = hipEventCreateWithFlags(&c->icp_ev, hipEventDisableTiming | (TF_ICP_EV_SYSFENCE ? 0u : hipEventDisableSystemFence));
        if (e != hipSuccess) { c->icp_ev = nullptr; ctx_free(c); return tf_from_hip(e); }
        icp_order_register(c, +1);
    }
    *out = c;
    return TF_OK;
}

extern "C" void tf_destroy(tf_ctx* c)
{
    if (!c) return;
    (void)hipStreamSynchronize(c->stream);
    ctx_free(c);
}

extern "C" tf_status tf_reset(tf_ctx* c)
{
    TF_FLUSH(c);
    if (!c) return TF_INVALID_ARG;
    return ctx_reset(c);
}

// stage entry points run the tracking-path kernels unconditionally
__global__ void k_stage_begin(TfDevState* st)
{
    st->abort = 0;
    st->mode = 1;
}

static hipError_t clear_abort(tf_ctx* c)
{
    hipLaunchKernelGGL(k_stage_begin, dim3(1), dim3(1), 0, c->stream, c->st);
    return hipGetLastError();
}

static void swap_pyramids(tf_ctx* c)
{
    for (int l = 0; l < TF_LEVELS; ++l) {
        float4* t = c->curr_pts[l]; c->curr_pts[l] = c->prev_pts[l]; c->prev_pts[l] = t;
        t = c->curr_nrm[l]; c->curr_nrm[l] = c->prev_nrm[l]; c->prev_nrm[l] = t;
    }
}

// ---- per-stage event timing -----------------------------------------------------------
// Events ring: TF_PROF_RING frames x (start, end) per stage.  Frames are attributed after a
// sync, once their mode / ok flags are known, and only for the stages that did work.
// A single-kernel stage (stage_single) is timed by its dispatch's own timestamps (tf_launch,
// hipExtLaunchKernelGGL); the others by event records around their launches.
#define STAGE_ON(strm, id, expr)                                                              \
    do {                                                                                      \
        const bool timed_ = c->prof_slot_on[slot] && ((c->prof_mask >> (id)) & 1u);          \
        const bool ext_ = timed_ && stage_single(c, id);                                      \
        if (timed_) c->prof_slot_stages[slot] |= 1u << (id);                                  \
        if (ext_) { c->ev_start = prof_event(c, slot, 2 * (id)); c->ev_stop = prof_event(c, slot, 2 * (id) + 1); } \
        else if (timed_) TF_CHECK(hipEventRecord(prof_event(c, slot, 2 * (id)), (strm)));     \
        const hipError_t se_ = (expr);                                                        \
        /* the launcher consumes the events in tf_launch; on every other exit they are dropped */ \
        const bool unused_ = ext_ && c->ev_start;                                             \
        c->ev_start = c->ev_stop = nullptr;                                                   \
        TF_CHECK(se_);                                                                        \
        if (unused_) return TF_HIP_ERROR;                                                     \
        if (timed_ && !ext_) TF_CHECK(hipEventRecord(prof_event(c, slot, 2 * (id) + 1), (strm))); \
    } while (0)
#define STAGE(id, expr) STAGE_ON(c->stream, id, expr)

// stages whose frame-path launcher issues exactly one kernel (through tf_launch)
static bool stage_single(const tf_ctx* c, int id)
{
    return (id == TF_STAGE_ICP && c->icp_persistent) || id == TF_STAGE_INTEGRATE || id == TF_STAGE_EXPECTED_DEPTHS ||
           id == TF_STAGE_RAYCAST_ICP || id == TF_STAGE_ICP_MAPS;
}

static hipEvent_t prof_event(tf_ctx* c, int slot, int k)
{
    return c->prof_ev[(slot % TF_PROF_RING) * 2 * TF_NUM_STAGES + k];
}

static bool stage_ran(int stage, int mode, int ok)
{
    if (stage == TF_STAGE_PREPROCESS) return true;
    // ICP: only frames whose estimateTransform ran all its iterations (a failed det check ends
    // it early, and its launch would understate the per-launch time of the full 19 iterations)
    if (stage == TF_STAGE_ICP) return mode == 1 && ok == 1;
    if (stage == TF_STAGE_ALLOC || stage == TF_STAGE_INTEGRATE) return mode == 0 || ok == 1;
    if (stage == TF_STAGE_GREY) return false;                      // fused into RAYCAST_RENDER
    return mode == 1 && ok == 1;
}

// attribute the timed stages of batch slots [first, first+n) (their events must be complete)
static tf_status prof_collect(tf_ctx* c, int first, int n, const int* ok, const int* mode)
{
    if (!c->prof_enabled) return TF_OK;
    for (int f = 0; f < n; ++f)
        for (int i = 0; i < TF_NUM_STAGES; ++i) {
            if (!c->prof_slot_on[first + f] || !((c->prof_mask >> i) & 1u) || !stage_ran(i, mode[f], ok[f])) continue;
            if (!((c->prof_slot_stages[first + f] >> i) & 1u)) continue;      // not enqueued as its own stage
            if (i == TF_STAGE_PREPROCESS && !c->prof_slot_pre[first + f]) continue;   // done by the previous frame
            if (i == TF_STAGE_RAYCAST_RENDER) continue;                       // fused into RAYCAST_ICP
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, prof_event(c, first + f, 2 * i), prof_event(c, first + f, 2 * i + 1)) == hipSuccess) {
                c->prof_ms[i] += ms;
                c->prof_count[i] += 1;
            }
        }
    return TF_OK;
}

// enqueue one TopFu::operator() frame into batch slot `slot` (no host synchronisation).
// The frame's branches (frame 0 / tracking / ICP failure -> reset, topfu.cpp:161-330) are
// decided on the device: the ICP launch starts the frame (tf_frame_begin sets st->mode), every
// later kernel checks st->mode / st->abort, and the frame end in k_icp_maps_end's tail (frame
// counters, per-slot ok flag, ResetScene on ICP failure) closes it.  A batch is therefore
// enqueued back to back.  Per frame: k_icp_frame (+ setToType3 and the renderImage snapshot in
// its tail) -> k_alloc_requests -> k_alloc_apply -> k_vis_count -> k_vis_apply -> k_integrate
// (+ CreateExpectedDepths' projection) -> k_ed_fill -> k_raycast_pair (CreateICPMaps' castRay
// and renderImage's castRay + grey in one grid) -> k_icp_maps_end.
//
// Lookahead (batches): later frames' preprocessing runs in this frame's grid tails and their
// enqueues skip it.  k_raycast_pair of frame j runs frame j+1's computeDists + pyramids +
// normals and frame j+2's bilateral pass, whose level-0 depth goes to the buffer of j's parity
// (d0_buf, ping-pong); the batch's first frame also runs frame 1's bilateral pass in
// k_alloc_requests.  Preprocessing is a pure function of the raw frame; what it writes is past
// its last reader of this frame by then (level-0 depth: this frame's pyramid pass; dists and
// the current maps: this frame's allocation, integration and ICP).
struct TfFramePlan {
    int pre_done;            // this frame's preprocessing ran in earlier launches
    uint16_t* d0;            // this frame's level-0 depth buffer
    TfAhead alloc_bil, pair_pyr, pair_bil;
    int defer_tail;          // leave k_raycast_pair + k_icp_maps_end to the next call (flush_tail)
};

// the view's RGB image for the integrations enqueued while in scope (voxel_rgb)
struct RgbScope {
    tf_ctx* c;
    RgbScope(tf_ctx* ctx, const uint8_t* rgb, size_t pitch) : c(ctx)
    {
        c->rgb_cur = (const uchar4*)rgb;
        c->rgb_pitch = pitch ? pitch : (size_t)c->W * 4;
    }
    ~RgbScope() { c->rgb_cur = nullptr; }
};

#ifdef TF_DIAG_NOP_AFTER_ICP
__global__ void k_diag_nop() {}
#endif

static tf_status enqueue_frame(tf_ctx* c, const uint16_t* depth, size_t pitch, int slot,
                               const TfFramePlan* plan = nullptr)
{
    static const TfFramePlan none = { 0, nullptr, {}, {}, {}, 0 };
    if (!plan) plan = &none;
    uint16_t* d0 = plan->d0 ? plan->d0 : c->d0_buf[0];
    c->prof_slot_on[slot] = c->prof_enabled && (c->prof_seq++ % c->prof_period) == 0;
    c->prof_slot_pre[slot] = !plan->pre_done;
    c->prof_slot_stages[slot] = 0;
    // preprocessing (topfu.cpp:166-197)
    if (!plan->pre_done) STAGE(TF_STAGE_PREPROCESS, tfk_preprocess(c, depth, pitch, c->stream, d0));
    c->depth_pyr[0] = d0;
    // frame begin + estimateTransform + poses_.push_back (topfu.cpp:200, 242-243); with the
    // persistent ICP, setToType3 / the renderImage snapshot run in its tail
    const bool t3_fold = c->icp_persistent != 0;
    STAGE(TF_STAGE_ICP, tfk_icp(c, 1, 1, t3_fold));
#ifdef TF_DIAG_NOP_AFTER_ICP
    // diagnostic builds only: an empty launch between the ICP and the allocation, to tell in a
    // kernel trace which side of that boundary its dispatch gap belongs to
    hipLaunchKernelGGL(k_diag_nop, dim3(1), dim3(64), 0, c->stream);
#endif
    STAGE(TF_STAGE_ALLOC, tfk_alloc(c, t3_fold ? 2 : 1, plan->alloc_bil, pitch));   // topfu.cpp:202 / 281
    // (+ CreateExpectedDepths' projection pass in the same grid)
    STAGE(TF_STAGE_INTEGRATE, tfk_integrate(c, 1, 1));              // topfu.cpp:203 / 282 (+ frame-0 prev_ = curr_)
    if (c->p.use_swapping) TF_CHECK(tfk_swap(c));                   // swap in / out after integration
    // CreateExpectedDepths (topfu.cpp:306): its projection ran in k_integrate's grid; its fill runs
    // in k_raycast_pair's grid when the frame is narrow enough (tfk_ed_fused), else on its own
    const int fuse_ed = tfk_ed_fused(c);
    if (!fuse_ed) STAGE(TF_STAGE_EXPECTED_DEPTHS, tfk_expected_depths(c, 1));
    if (plan->defer_tail) {                   // per-call frame: the last two launches wait for the next call
        c->tail_pending = 1;
        c->tail_fuse_ed = fuse_ed;
        return TF_OK;
    }
    // CreateICPMaps' raycast + renderImage (topfu.cpp:284-285 + 307) in one launch (snapshot range)
    STAGE(TF_STAGE_RAYCAST_ICP, tfk_raycast_pair(c, plan->pair_pyr, plan->pair_bil, pitch, fuse_ed, 1));
    // renderICP + resizePointsNormals (topfu.cpp:308-309) + the frame end (topfu.cpp:263-264)
    STAGE(TF_STAGE_ICP_MAPS, tfk_icp_maps_end(c, slot));
    return TF_OK;
}


// sync, read back slots [first, first+n) and the state; ok_out gets 1/0 per frame.  *lost: the
// slot whose persistent ICP lost a peer (frame_ok -1: nothing of it ran past the ICP, and the
// later slots were skipped, -2), for the caller to re-run from there; -1 if none.  A frame that
// failed past its ICP (-3) is TF_HIP_ERROR.
static tf_status finish_frames(tf_ctx* c, int first, int n, int* ok_out, int* lost = nullptr)
{
    if (lost) *lost = -1;
    // one device-to-host copy into the pinned mirror: the state and the slots' ok / mode
    TF_CHECK(hipMemcpyAsync(c->st_host, c->st, TF_ST_BYTES, hipMemcpyDeviceToHost, c->stream));
    TF_CHECK(hipStreamSynchronize(c->stream));
    const int* okb = (const int*)(c->st_host + 1) + first;
    const int* modeb = (const int*)(c->st_host + 1) + TF_PROF_RING + first;
    c->frame_counter = c->st_host->frame_counter;
    c->n_resets = c->st_host->n_resets;
    prof_collect(c, first, n, okb, modeb);
    if (c->st_host->sticky_error) return TF_HIP_ERROR;
    tf_status r = TF_OK;
    for (int i = 0; i < n; ++i) {
        if (okb[i] == -1 && lost) { *lost = i; break; }
        if (okb[i] < 0) return TF_HIP_ERROR;
        if (ok_out) ok_out[i] = okb[i];
        if (okb[i] == 0) r = TF_ICP_FAIL;
    }
    return r;
}

// Run-time fallback of the persistent ICP: a frame whose persistent launch lost a peer (some of
// its 256 workgroups could not be co-resident -- another process or kernel on the device; the
// bounded spins ended it: frame_ok -1, the frame end halted the batch) is enqueued again, whole,
// on the per-iteration schedule (k_icp_iter: one launch per iteration, no co-residency needed).
// Nothing of the failed attempt changed the scene (every stage after the ICP no-oped on abort),
// so the re-run is the frame as it would have run.  Synchronous; *ok = its frame_ok.
static tf_status rerun_frame_fallback(tf_ctx* c, const uint16_t* depth, size_t pitch, int* ok)
{
    TF_CHECK(hipMemsetAsync((char*)c->st + offsetof(TfDevState, halt), 0, sizeof(int), c->stream));
    const int saved = c->icp_persistent;
    c->icp_persistent = 0;
    c->icp_fallbacks++;
    tf_status s = enqueue_frame(c, depth, pitch, 0);
    c->icp_persistent = saved;
    if (s != TF_OK) return s;
    int okv = 0;
    s = finish_frames(c, 0, 1, &okv);
    if (s != TF_OK && s != TF_ICP_FAIL) return s;
    if (ok) *ok = okv;
    return s;
}

extern "C" tf_status tf_profile_enable(tf_ctx* c, int enable)
{
    if (!c) return TF_INVALID_ARG;
    if (enable && !c->prof_ev[0]) {
        // timing only (read after the stream is synchronised): no system-scope fence at the record,
        // whose cache writeback and invalidate were a dispatch gap after every timed stage
        for (int i = 0; i < 2 * TF_NUM_STAGES * TF_PROF_RING; ++i)
            TF_CHECK(hipEventCreateWithFlags(&c->prof_ev[i], hipEventDisableSystemFence));
    }
    c->prof_enabled = enable ? 1 : 0;
    c->count_lanes = enable ? 1 : 0;
    c->prof_mask = (1u << TF_NUM_STAGES) - 1;
    c->prof_period = 1;
    c->prof_seq = 0;
    return TF_OK;
}

extern "C" tf_status tf_profile_stages(tf_ctx* c, unsigned mask)
{
    if (!c) return TF_INVALID_ARG;
    tf_status s = tf_profile_enable(c, mask != 0);
    if (s != TF_OK) return s;
    c->prof_mask = mask;
    c->count_lanes = 0;          // (selected stages: a timed run, no counting atomics in it)
    return TF_OK;
}

extern "C" tf_status tf_profile_sample(tf_ctx* c, int period)
{
    if (!c || period < 1) return TF_INVALID_ARG;
    c->prof_period = period;
    c->prof_seq = 0;
    return TF_OK;
}

extern "C" tf_status tf_profile_reset(tf_ctx* c)
{
    if (!c) return TF_INVALID_ARG;
    for (int i = 0; i < TF_NUM_STAGES; ++i) { c->prof_ms[i] = 0; c->prof_count[i] = 0; }
    return TF_OK;
}

extern "C" tf_status tf_profile_read(tf_ctx* c, double* ms, long long* counts, int n)
{
    if (!c || n < 0 || n > TF_NUM_STAGES) return TF_INVALID_ARG;
    for (int i = 0; i < n; ++i) {
        if (ms) ms[i] = c->prof_ms[i];
        if (counts) counts[i] = c->prof_count[i];
    }
    return TF_OK;
}

static void fill_stats(tf_ctx* c, tf_stats* st)
{
    if (!st) return;
    const TfDevState* d = c->st_host;
    st->lastFreeBlockId = d->lastFreeBlockId;
    st->lastFreeExcessListId = d->lastFreeExcessListId;
    st->noVisibleEntries = d->noVisibleEntries;
    st->noTotalBlocks = d->noTotalBlocks;
    st->frame_counter = c->frame_counter;   // mirrors of the device counters (last sync)
    st->icp_iterations = d->icp_iters;
    st->icp_ok = d->icp_ok;
    st->n_resets = c->n_resets;
}

// A per-call frame returns on its verdict (early) when nothing the caller asked for needs the
// whole frame: no stats, no stage timing, no RGB image (k_integrate reads the caller's image
// directly, so the call must not return before the integration has run), and the persistent
// ICP (the per-iteration fallback writes no verdict).
static bool percall_early(const tf_ctx* c, const tf_stats* stats)
{
    return c->percall_early && c->icp_persistent && !c->prof_enabled && !stats && !c->rgb_cur;
}

// TopFu::operator() returning on its verdict.  Enqueues the whole frame, then waits only until
// the persistent ICP launch has written the frame's verdict (topfu.cpp:209 / 263-264 / 329:
// frame-0 path, reset + false, true; and poses_.back()) into host memory.  The allocation,
// integration, raycasts and frame end are still running on the context stream when it returns;
// everything that reads their results later (tf_download, tf_render_image, tf_get_*) is ordered
// after them on that stream, and the next frame's launches queue behind them, so the device does
// not wait for the host between frames.  The frame's preprocessing has read the depth by then.
// host_depth: the tf_process_frame_host form.
static tf_status process_frame_early(tf_ctx* c, const uint16_t* depth, size_t pitch, const uint16_t* host_depth,
                                     float pose_out[12])
{
    if (host_depth) {
        TF_CHECK(hipMemcpy2DAsync(c->depth_in, (size_t)c->W * 2, host_depth, pitch, (size_t)c->W * 2, c->H,
                                  hipMemcpyHostToDevice, c->stream));
        depth = c->depth_in;
        pitch = (size_t)c->W * 2;
    }
    // the previous frame's deferred launches carry this frame's preprocessing in their grid tails
    TfFramePlan plan = { 0, nullptr, {}, {}, {}, c->percall_defer };
    if (c->tail_pending) {
        const TfAhead nxt = { depth, c->d0_buf[0] };
        tf_status fs = flush_tail(c, nxt, pitch);
        if (fs != TF_OK) return fs;
        plan.pre_done = 1;
        plan.d0 = c->d0_buf[0];
    }
    if (++c->verdict_gen == 0) c->verdict_gen = 1;
    const unsigned gen = c->verdict_gen;
    c->verdict_arm = 1;
    tf_status s = enqueue_frame(c, depth, pitch, 0, &plan);
    c->verdict_arm = 0;
    if (s != TF_OK) return s;
    // wait for the verdict: every word tagged with this generation
    volatile unsigned long long* v = c->verdict_host;
    unsigned long long w[13];
    bool drained = false;
    for (unsigned spins = 0;; ++spins) {
        int k = 0;
        for (; k < 13; ++k) {
            w[k] = v[k];
            if ((unsigned)(w[k] >> 32) != gen) break;
        }
        if (k == 13) break;
        if (drained) return TF_HIP_ERROR;        // the stream finished without writing it
        if ((spins & 1023u) == 1023u) {
            const hipError_t q = hipStreamQuery(c->stream);
            if (q == hipSuccess) drained = true;   // read the record once more, then give up
            else if (q != hipErrorNotReady) return tf_from_hip(q);
        }
        __builtin_ia32_pause();
    }
    const int mode = (int)(w[0] & 15u), ok = (int)((w[0] >> 4) & 15u) - 1;
    if (ok < 0) {
        // the frame's launches end on the device (the halted / failed frame no-ops); its deferred
        // tail holds the frame end, enqueued now without a lookahead
        const tf_status fs = flush_tail(c);
        if (fs != TF_OK) return fs;
        TF_CHECK(hipStreamSynchronize(c->stream));
        if ((w[0] >> 16) & 1u) return TF_HIP_ERROR;           // halted: an earlier frame failed past its ICP
        // a lost peer in the persistent ICP: the frame again, on the per-iteration schedule
        int okv = 0;
        const tf_status s2 = rerun_frame_fallback(c, depth, pitch, &okv);
        if (s2 != TF_OK && s2 != TF_ICP_FAIL) return s2;
        if (pose_out) memcpy(pose_out, c->st_host->pose, sizeof(float) * 12);
        return s2;
    }
    // host mirrors of the counters the frame end writes (tf_reset.h)
    if (mode == 0) c->frame_counter = 1;
    else if (ok) c->frame_counter++;
    else { c->frame_counter = 0; c->n_resets++; }
    if (pose_out)
        for (int i = 0; i < 12; ++i) {
            const unsigned bits = (unsigned)w[1 + i];
            memcpy(&pose_out[i], &bits, sizeof(float));
        }
    return ok ? TF_OK : TF_ICP_FAIL;
}

extern "C" tf_status tf_process_frame(tf_ctx* c, const uint16_t* dev_depth, size_t pitch, float pose_out[12],
                                      tf_stats* stats)
{
    if (!c || !dev_depth) return TF_INVALID_ARG;
    if (pitch == 0) pitch = (size_t)c->W * 2;
    if (percall_early(c, stats)) return process_frame_early(c, dev_depth, pitch, nullptr, pose_out);
    TF_FLUSH(c);
    tf_status s = enqueue_frame(c, dev_depth, pitch, 0);
    if (s != TF_OK) return s;
    int lost = -1;
    s = finish_frames(c, 0, 1, nullptr, &lost);
    if (lost == 0) s = rerun_frame_fallback(c, dev_depth, pitch, nullptr);   // the persistent ICP lost a peer
    if (s != TF_OK && s != TF_ICP_FAIL) return s;
    if (pose_out) memcpy(pose_out, c->st_host->pose, sizeof(float) * 12);
    fill_stats(c, stats);
    return s;
}

extern "C" tf_status tf_process_frame_rgb(tf_ctx* c, const uint16_t* dev_depth, size_t pitch, const uint8_t* dev_rgb,
                                          size_t rgb_pitch, float pose_out[12], tf_stats* stats)
{
    TF_FLUSH(c);
    if (!c) return TF_INVALID_ARG;
    if (dev_rgb && !c->p.voxel_rgb) return TF_INVALID_ARG;
    RgbScope rs(c, dev_rgb, rgb_pitch);
    return tf_process_frame(c, dev_depth, pitch, pose_out, stats);
}

extern "C" tf_status tf_process_frame_rgb_host(tf_ctx* c, const uint16_t* host_depth, size_t pitch, const uint8_t* host_rgb,
                                               size_t rgb_pitch, float pose_out[12], tf_stats* stats)
{
    TF_FLUSH(c);
    if (!c || !host_depth) return TF_INVALID_ARG;
    if (host_rgb && !c->p.voxel_rgb) return TF_INVALID_ARG;
    if (!host_rgb) return tf_process_frame_host(c, host_depth, pitch, pose_out, stats);
    if (rgb_pitch == 0) rgb_pitch = (size_t)c->W * 4;
    TF_CHECK(hipMemcpy2DAsync(c->rgb_in, (size_t)c->W * 4, host_rgb, rgb_pitch, (size_t)c->W * 4, c->H,
                              hipMemcpyHostToDevice, c->stream));
    if (pitch == 0) pitch = (size_t)c->W * 2;
    TF_CHECK(hipMemcpy2DAsync(c->depth_in, (size_t)c->W * 2, host_depth, pitch, (size_t)c->W * 2, c->H,
                              hipMemcpyHostToDevice, c->stream));
    return tf_process_frame_rgb(c, c->depth_in, (size_t)c->W * 2, (const uint8_t*)c->rgb_in, (size_t)c->W * 4, pose_out,
                                stats);
}

extern "C" tf_status tf_process_frame_host(tf_ctx* c, const uint16_t* host_depth, size_t pitch, float pose_out[12],
                                           tf_stats* stats)
{
    if (!c || !host_depth) return TF_INVALID_ARG;
    if (pitch == 0) pitch = (size_t)c->W * 2;
    if (percall_early(c, stats)) return process_frame_early(c, nullptr, pitch, host_depth, pose_out);
    TF_FLUSH(c);
    TF_CHECK(hipMemcpy2DAsync(c->depth_in, (size_t)c->W * 2, host_depth, pitch, (size_t)c->W * 2, c->H,
                              hipMemcpyHostToDevice, c->stream));
    return tf_process_frame(c, c->depth_in, (size_t)c->W * 2, pose_out, stats);
}

// a batch of device-resident frames: enqueued TF_PROF_RING at a time with no host round trip
// inside a group (the frame's branches are decided on the device)
static tf_status process_frames(tf_ctx* c, const uint16_t* dev_frames, size_t stride, const uint8_t* rgb_frames,
                                size_t rgb_stride, int n, int* ok_out);

extern "C" tf_status tf_process_frames(tf_ctx* c, const uint16_t* dev_frames, size_t stride, int n, int* ok_out)
{
    TF_FLUSH(c);
    return process_frames(c, dev_frames, stride, nullptr, 0, n, ok_out);
}

extern "C" tf_status tf_process_frames_rgb(tf_ctx* c, const uint16_t* dev_frames, size_t stride, const uint8_t* rgb_frames,
                                          size_t rgb_stride, int n, int* ok_out)
{
    TF_FLUSH(c);
    if (c && rgb_frames && !c->p.voxel_rgb) return TF_INVALID_ARG;
    return process_frames(c, dev_frames, stride, rgb_frames, rgb_stride, n, ok_out);
}

static tf_status process_frames(tf_ctx* c, const uint16_t* dev_frames, size_t stride, const uint8_t* rgb_frames,
                                size_t rgb_stride, int n, int* ok_out)
{
    if (!c || !dev_frames || n < 0) return TF_INVALID_ARG;
    if (rgb_frames && rgb_stride == 0) rgb_stride = (size_t)c->W * c->H * 4;
    auto frame = [&](int j) { return (const uint16_t*)((const char*)dev_frames + (size_t)j * stride); };
    int s0 = 0;                 // the frame the lookahead chain starts at (0, or after a fallback re-run)
    for (int first = 0; first < n;) {
        const int m = n - first < TF_PROF_RING ? n - first : TF_PROF_RING;
        for (int i = 0; i < m; ++i) {
            const int j = first + i;
            // two-frame lookahead (enqueue_frame): frame j+1's pyramid pass and frame j+2's
            // bilateral pass run in frame j's grid tails
            TfFramePlan p = { j > s0, c->d0_buf[j & 1], {}, {}, {}, 0 };
            if (j + 1 < n) {
                TfAhead next = { frame(j + 1), c->d0_buf[(j + 1) & 1] };
                p.pair_pyr = next;
                if (j == s0) p.alloc_bil = next;
                if (j + 2 < n) p.pair_bil = TfAhead{ frame(j + 2), c->d0_buf[j & 1] };
            }
            RgbScope rs(c, rgb_frames ? rgb_frames + (size_t)j * rgb_stride : nullptr, (size_t)c->W * 4);
            tf_status s = enqueue_frame(c, frame(j), (size_t)c->W * 2, i, &p);
            if (s != TF_OK) return s;
        }
        int lost = -1;
        tf_status s = finish_frames(c, 0, m, ok_out ? ok_out + first : nullptr, &lost);
        if (s != TF_OK && s != TF_ICP_FAIL) return s;
        if (lost < 0) { first += m; continue; }
        // frame first+lost lost an ICP peer, the rest of the group was skipped: re-run it on the
        // per-iteration schedule (its own preprocessing: its maps were overwritten by the lookahead
        // of the skipped frames), then continue the batch after it with a fresh lookahead chain
        const int j = first + lost;
        RgbScope rs(c, rgb_frames ? rgb_frames + (size_t)j * rgb_stride : nullptr, (size_t)c->W * 4);
        int okv = 0;
        s = rerun_frame_fallback(c, frame(j), (size_t)c->W * 2, &okv);
        if (s != TF_OK && s != TF_ICP_FAIL) return s;
        if (ok_out) ok_out[j] = okv;
        first = s0 = j + 1;
    }
    return TF_OK;
}

extern "C" tf_status tf_render_image(tf_ctx* c, uint8_t* dev_rgba, size_t pitch)
{   // TopFu::renderImage: raycast from poses_.back() with the current range image + grey
    TF_FLUSH(c);
    return tf_render_image_type(c, TF_RENDER_SHADED_GREYSCALE, dev_rgba, pitch);
}

extern "C" tf_status tf_render_image_type(tf_ctx* c, int type, uint8_t* dev_rgba, size_t pitch)
{   // VisualisationEngine_CUDA::RenderImage(..., type, RENDER_FROM_NEW_RAYCAST) from poses_.back()
    TF_FLUSH(c);
    if (!c || type < TF_RENDER_SHADED_GREYSCALE || type > TF_RENDER_COLOUR_FROM_CONFIDENCE) return TF_INVALID_ARG;
    TF_CHECK(clear_abort(c));
    TF_CHECK(hipMemcpyAsync(c->st->pose_in, c->st->pose, sizeof(float) * 12, hipMemcpyDeviceToDevice, c->stream));
    TF_CHECK(tfk_pose_from_input(c, 0));
    TF_CHECK(tfk_raycast(c, 0));
    TF_CHECK(tfk_render_type(c, type));
    if (dev_rgba) {
        if (pitch == 0) pitch = (size_t)c->W * 4;
        TF_CHECK(hipMemcpy2DAsync(dev_rgba, pitch, c->grey, (size_t)c->W * 4, (size_t)c->W * 4, c->H,
                                  hipMemcpyDeviceToDevice, c->stream));
    }
    return sync_checked(c);
}

extern "C" tf_status tf_get_pose(tf_ctx* c, float rt[12])
{
    TF_FLUSH(c);
    if (!c || !rt) return TF_INVALID_ARG;
    tf_status s = sync_state(c);
    if (s != TF_OK) return s;
    memcpy(rt, c->st_host->pose, sizeof(float) * 12);
    return TF_OK;
}

extern "C" tf_status tf_get_stats(tf_ctx* c, tf_stats* stats)
{
    TF_FLUSH(c);
    if (!c || !stats) return TF_INVALID_ARG;
    tf_status s = sync_state(c);
    if (s != TF_OK) return s;
    fill_stats(c, stats);
    return TF_OK;
}

extern "C" tf_status tf_get_params(tf_ctx* c, tf_params* p)
{
    if (!c || !p) return TF_INVALID_ARG;
    *p = c->p;
    return TF_OK;
}

extern "C" void* tf_get_stream(tf_ctx* c)
{   // (a caller that synchronises the stream itself sees every frame complete)
    if (c) (void)flush_tail(c);
    return c ? (void*)c->stream : nullptr;
}

extern "C" tf_status tf_get_schedule(tf_ctx* c, int* icp_persistent)
{
    if (!c) return TF_INVALID_ARG;
    if (icp_persistent) *icp_persistent = c->icp_persistent;
    return TF_OK;
}

extern "C" tf_status tf_set_pose_algebra(tf_ctx* c, int algebra)
{
    if (!c) return TF_INVALID_ARG;
    if (algebra != TF_POSE_ALGEBRA_CANONICAL && algebra != TF_POSE_ALGEBRA_OPENCV2 && algebra != TF_POSE_ALGEBRA_OPENCV4)
        return TF_INVALID_ARG;
    TF_FLUSH(c);
    const int old = c->pose_alg;
    c->pose_alg = algebra;
    if (c->icp_persistent && !tfk_icp_persistent_ok(c)) {     // the schedule stays what tf_create chose
        c->pose_alg = old;
        return TF_INVALID_ARG;
    }
    return TF_OK;
}

extern "C" tf_status tf_get_pose_algebra(tf_ctx* c, int* algebra)
{
    if (!c || !algebra) return TF_INVALID_ARG;
    *algebra = c->pose_alg;
    return TF_OK;
}

// ---- stage entry points ---------------------------------------------------------------
static tf_status set_pose_in(tf_ctx* c, const float* rt, int mode)
{
    TF_CHECK(clear_abort(c));
    TF_CHECK(hipMemcpyAsync(c->st->pose_in, rt, sizeof(float) * 12, hipMemcpyHostToDevice, c->stream));
    TF_CHECK(tfk_pose_from_input(c, mode));
    return TF_OK;
}

extern "C" tf_status tf_stage_preprocess(tf_ctx* c, const uint16_t* dev_depth, size_t pitch)
{
    TF_FLUSH(c);
    if (!c || !dev_depth) return TF_INVALID_ARG;
    if (pitch == 0) pitch = (size_t)c->W * 2;
    TF_CHECK(clear_abort(c));
    TF_CHECK(tfk_preprocess(c, dev_depth, pitch, c->stream, c->d0_buf[0]));
    c->depth_pyr[0] = c->d0_buf[0];
    return sync_checked(c);
}

extern "C" tf_status tf_stage_preprocess_host(tf_ctx* c, const uint16_t* host_depth, size_t pitch)
{
    TF_FLUSH(c);
    if (!c || !host_depth) return TF_INVALID_ARG;
    if (pitch == 0) pitch = (size_t)c->W * 2;
    TF_CHECK(hipMemcpy2DAsync(c->depth_in, (size_t)c->W * 2, host_depth, pitch, (size_t)c->W * 2, c->H,
                              hipMemcpyHostToDevice, c->stream));
    return tf_stage_preprocess(c, c->depth_in, (size_t)c->W * 2);
}

extern "C" tf_status tf_stage_icp(tf_ctx* c, float affine_rt[12], int* ok, int* iterations)
{
    TF_FLUSH(c);
    if (!c) return TF_INVALID_ARG;
    TF_CHECK(clear_abort(c));                      // tracking-path kernels run (st->mode = 1)
    TF_CHECK(tfk_icp(c, 0));
    tf_status s = sync_state(c);
    if (s != TF_OK) return s;
    if (c->st_host->icp_ok < 0) return TF_HIP_ERROR;
    if (affine_rt) memcpy(affine_rt, c->st_host->affine, sizeof(float) * 12);
    if (ok) *ok = c->st_host->icp_ok;
    if (iterations) *iterations = c->st_host->icp_iters;
    TF_CHECK(clear_abort(c));
    return TF_OK;
}

extern "C" tf_status tf_stage_alloc(tf_ctx* c, const float pose_rt[12])
{
    TF_FLUSH(c);
    if (!c || !pose_rt) return TF_INVALID_ARG;
    TF_CHECK(clear_abort(c));                      // tracking-path kernels run (st->mode = 1)
    tf_status s = set_pose_in(c, pose_rt, TF_POSE_ALLOC_NOINV);
    if (s != TF_OK) return s;
    TF_CHECK(tfk_alloc(c));
    return sync_checked(c);
}

extern "C" tf_status tf_stage_integrate(tf_ctx* c, const float pose_rt[12])
{
    TF_FLUSH(c);
    if (!c || !pose_rt) return TF_INVALID_ARG;
    TF_CHECK(clear_abort(c));                      // tracking-path kernels run (st->mode = 1)
    tf_status s = set_pose_in(c, pose_rt, TF_POSE_ALLOC_NOINV);
    if (s != TF_OK) return s;
    TF_CHECK(tfk_integrate(c));
    return sync_checked(c);
}

extern "C" tf_status tf_stage_expected_depths(tf_ctx* c, const float pose_rt[12])
{
    TF_FLUSH(c);
    if (!c || !pose_rt) return TF_INVALID_ARG;
    TF_CHECK(clear_abort(c));                      // tracking-path kernels run (st->mode = 1)
    tf_status s = set_pose_in(c, pose_rt, TF_POSE_ALLOC_NOINV);
    if (s != TF_OK) return s;
    TF_CHECK(tfk_expected_depths(c));
    return sync_checked(c);
}

extern "C" tf_status tf_stage_raycast(tf_ctx* c, const float invM_rt[12], int update_visible)
{
    TF_FLUSH(c);
    if (!c || !invM_rt) return TF_INVALID_ARG;
    TF_CHECK(clear_abort(c));                      // tracking-path kernels run (st->mode = 1)
    tf_status s = set_pose_in(c, invM_rt, 0);
    if (s != TF_OK) return s;
    TF_CHECK(tfk_raycast(c, update_visible));
    return sync_checked(c);
}

extern "C" tf_status tf_stage_icp_maps(tf_ctx* c, const float invM_rt[12])
{
    TF_FLUSH(c);
    if (!c || !invM_rt) return TF_INVALID_ARG;
    TF_CHECK(clear_abort(c));                      // tracking-path kernels run (st->mode = 1)
    tf_status s = set_pose_in(c, invM_rt, 0);
    if (s != TF_OK) return s;
    TF_CHECK(tfk_icp_maps(c));
    return sync_checked(c);
}

extern "C" tf_status tf_stage_render_grey(tf_ctx* c, const float invM_rt[12])
{
    TF_FLUSH(c);
    if (!c || !invM_rt) return TF_INVALID_ARG;
    TF_CHECK(clear_abort(c));                      // tracking-path kernels run (st->mode = 1)
    tf_status s = set_pose_in(c, invM_rt, 0);
    if (s != TF_OK) return s;
    TF_CHECK(tfk_render_type(c, TF_RENDER_SHADED_GREYSCALE));
    return sync_checked(c);
}

extern "C" tf_status tf_time_stage(tf_ctx* c, int stage, const float pose_rt[12], int iters, float* ms_per_iter)
{
    TF_FLUSH(c);
    if (!c || !pose_rt || iters <= 0 || !ms_per_iter) return TF_INVALID_ARG;
    if (stage != TF_STAGE_INTEGRATE && stage != TF_STAGE_RAYCAST_ICP && stage != TF_STAGE_RAYCAST_RENDER &&
        stage != TF_STAGE_EXPECTED_DEPTHS)
        return TF_INVALID_ARG;
    TF_CHECK(clear_abort(c));                      // tracking-path kernels run (st->mode = 1)
    tf_status s = set_pose_in(c, pose_rt, stage == TF_STAGE_INTEGRATE || stage == TF_STAGE_EXPECTED_DEPTHS ? TF_POSE_ALLOC_NOINV : 0);
    if (s != TF_OK) return s;
    if (stage == TF_STAGE_EXPECTED_DEPTHS) TF_CHECK(tfk_expected_depths(c, 0, 1));    // boxes of the current list
    // the pair's renderImage half reads the snapshot of the raycast matrix / range region
    if (stage == TF_STAGE_RAYCAST_RENDER) TF_CHECK(tfk_render_snapshot(c));
    hipEvent_t e0, e1;
    TF_CHECK(hipEventCreate(&e0));
    TF_CHECK(hipEventCreate(&e1));
    hipError_t e = hipEventRecord(e0, c->stream);
    for (int i = 0; i < iters && e == hipSuccess; ++i)
        e = stage == TF_STAGE_INTEGRATE ? tfk_integrate(c)
          : stage == TF_STAGE_EXPECTED_DEPTHS ? tfk_expected_depths(c, 1, 1)
          : stage == TF_STAGE_RAYCAST_ICP ? tfk_raycast(c, 1) : tfk_raycast_pair_ordered(c);
    if (e == hipSuccess) e = hipEventRecord(e1, c->stream);
    if (e == hipSuccess) e = hipEventSynchronize(e1);
    float ms = 0.f;
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
    // the repeated fills kept the bins: empty them for the next projection pass
    if (e == hipSuccess && stage == TF_STAGE_EXPECTED_DEPTHS)
        e = hipMemsetAsync(c->edBinCnt, 0, sizeof(int) * 2 * (size_t)ed_nrows(c->H), c->stream);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (e != hipSuccess) return tf_from_hip(e);
    *ms_per_iter = ms / (float)iters;
    return TF_OK;
}

extern "C" tf_status tf_stage_reset_scene(tf_ctx* c)
{   // SceneReconstructionEngine::ResetScene: the GlobalCache stays (SceneReconstructionEngine_host.cu:51-73)
    TF_FLUSH(c);
    if (!c) return TF_INVALID_ARG;
    TF_CHECK(tfk_reset_scene(c, 0));
    return sync_checked(c);
}

extern "C" tf_status tf_stage_swap_pyramids(tf_ctx* c)
{
    TF_FLUSH(c);
    if (!c) return TF_INVALID_ARG;
    swap_pyramids(c);
    return TF_OK;
}

// ---- engine entry points over caller buffers (include/tfusion/engines.hpp) -------------
// the call's intrinsics (the reference engines take Intr per call) in place of the context's
// for as long as the scope lives; every launcher reads c->p when it builds its arguments
struct IntrScope {
    tf_ctx* c;
    float saved[4];
    IntrScope(tf_ctx* ctx, const float* intr) : c(ctx)
    {
        saved[0] = c->p.fx; saved[1] = c->p.fy; saved[2] = c->p.cx; saved[3] = c->p.cy;
        if (intr) { c->p.fx = intr[0]; c->p.fy = intr[1]; c->p.cx = intr[2]; c->p.cy = intr[3]; }
    }
    ~IntrScope() { c->p.fx = saved[0]; c->p.fy = saved[1]; c->p.cx = saved[2]; c->p.cy = saved[3]; }
};

extern "C" tf_status tf_icp_set_params(tf_ctx* c, float dist_thres, float angle_thres, const int iters[4])
{
    TF_FLUSH(c);
    if (!c || !iters || !(dist_thres >= 0) || !(angle_thres >= 0)) return TF_INVALID_ARG;
    if (iters[3] != 0) return TF_INVALID_ARG;            // three pyramid levels (TF_LEVELS)
    for (int l = 0; l < 4; ++l) if (iters[l] < 0) return TF_INVALID_ARG;
    c->p.icp_dist_thres = dist_thres;
    c->p.icp_angle_thres = angle_thres;
    for (int l = 0; l < 4; ++l) c->p.icp_iter_num[l] = iters[l];
    // ComputeIcpHelper ctor (projective_icp.cpp:11-15)
    c->min_cosine = cosf(angle_thres);
    c->dist2_thres = dist_thres * dist_thres;
    return TF_OK;
}

extern "C" tf_status tf_icp_get_params(tf_ctx* c, float* dist_thres, float* angle_thres, int iters[4])
{
    TF_FLUSH(c);
    if (!c) return TF_INVALID_ARG;
    if (dist_thres) *dist_thres = c->p.icp_dist_thres;
    if (angle_thres) *angle_thres = c->p.icp_angle_thres;
    if (iters) for (int l = 0; l < 4; ++l) iters[l] = c->p.icp_iter_num[l];
    return TF_OK;
}

// The context stream is non-blocking, so it does not wait for the legacy default stream on
// which the reference-shaped callers produce their inputs (cuda:: imgproc wrappers with
// stream 0, asynchronous uploads): in the reference everything runs on the default stream and
// that order is implicit.  Entry points that read caller device buffers therefore make the
// context stream wait for all work already enqueued on stream 0 before their first read.
static hipError_t order_after_caller(tf_ctx* c)
{
    hipError_t e = hipEventRecord(c->caller_ev, nullptr);
    return e == hipSuccess ? hipStreamWaitEvent(c->stream, c->caller_ev, 0) : e;
}

// caller pitched float4 map -> the context's packed level buffer
static hipError_t copy_map_in(tf_ctx* c, float4* dst, int l, const void* src, size_t step)
{
    const size_t row = sizeof(float4) * (size_t)c->lw[l];
    return hipMemcpy2DAsync(dst, row, src, step ? step : row, row, c->lh[l], hipMemcpyDeviceToDevice, c->stream);
}

extern "C" tf_status tf_icp_estimate(tf_ctx* c, const float intr[4], const tf_map_level* curr, const tf_map_level* prev,
                                     int levels, float affine_rt[12], int* ok, int* iterations)
{
    TF_FLUSH(c);
    if (!c || !curr || !prev || levels < 1 || levels > TF_LEVELS) return TF_INVALID_ARG;
    int used = 4;                                         // getUsedLevelsNum (projective_icp.cpp:103-108)
    while (used > 0 && c->p.icp_iter_num[used - 1] == 0) --used;
    if (used > levels) return TF_INVALID_ARG;
    for (int l = 0; l < levels; ++l)
        if (!curr[l].points || !curr[l].normals || !prev[l].points || !prev[l].normals) return TF_INVALID_ARG;
    TF_CHECK(order_after_caller(c));
    for (int l = 0; l < levels; ++l) {
        TF_CHECK(copy_map_in(c, c->curr_pts[l], l, curr[l].points, curr[l].points_step));
        TF_CHECK(copy_map_in(c, c->curr_nrm[l], l, curr[l].normals, curr[l].normals_step));
        TF_CHECK(copy_map_in(c, c->prev_pts[l], l, prev[l].points, prev[l].points_step));
        TF_CHECK(copy_map_in(c, c->prev_nrm[l], l, prev[l].normals, prev[l].normals_step));
    }
    IntrScope is(c, intr);
    return tf_stage_icp(c, affine_rt, ok, iterations);
}

// caller dists (pitched) -> the context's dists buffer
static hipError_t copy_dists_in(tf_ctx* c, const float* dists, size_t step)
{
    const size_t row = sizeof(float) * (size_t)c->W;
    return hipMemcpy2DAsync(c->dists, row, dists, step ? step : row, row, c->H, hipMemcpyDeviceToDevice, c->stream);
}

extern "C" tf_status tf_scene_alloc(tf_ctx* c, const float intr[4], const float pose_rt[12], const float* dists,
                                   size_t dists_step, int only_update_visible_list, int reset_visible_list)
{
    TF_FLUSH(c);
    if (!c || !pose_rt || !dists) return TF_INVALID_ARG;
    TF_CHECK(order_after_caller(c));
    TF_CHECK(copy_dists_in(c, dists, dists_step));
    IntrScope is(c, intr);
    tf_status s = set_pose_in(c, pose_rt, TF_POSE_ALLOC_NOINV);
    if (s != TF_OK) return s;
    if (reset_visible_list) {          // renderState_vh->noVisibleEntries = 0 (SceneReconstructionEngine_host.cu:88)
        static const int zero = 0;
        TF_CHECK(hipMemcpyAsync((char*)c->st + offsetof(TfDevState, noVisibleEntries), &zero, sizeof(int),
                                hipMemcpyHostToDevice, c->stream));
    }
    TF_CHECK(tfk_alloc(c, 0, TfAhead{}, 0, only_update_visible_list ? 1 : 0));
    return sync_checked(c);
}

extern "C" tf_status tf_scene_integrate(tf_ctx* c, const float intr[4], const float pose_rt[12], const float* dists,
                                       size_t dists_step)
{
    TF_FLUSH(c);
    if (!c || !pose_rt || !dists) return TF_INVALID_ARG;
    TF_CHECK(order_after_caller(c));
    TF_CHECK(copy_dists_in(c, dists, dists_step));
    IntrScope is(c, intr);
    tf_status s = set_pose_in(c, pose_rt, TF_POSE_ALLOC_NOINV);
    if (s != TF_OK) return s;
    TF_CHECK(tfk_integrate(c));
    return sync_checked(c);
}

extern "C" tf_status tf_scene_integrate_rgb(tf_ctx* c, const float intr[4], const float pose_rt[12], const float* dists,
                                           size_t dists_step, const uint8_t* dev_rgb, size_t rgb_step)
{
    TF_FLUSH(c);
    if (!c || !pose_rt || !dists) return TF_INVALID_ARG;
    if (dev_rgb && !c->p.voxel_rgb) return TF_INVALID_ARG;
    RgbScope rs(c, dev_rgb, rgb_step);
    return tf_scene_integrate(c, intr, pose_rt, dists, dists_step);
}

static tf_status scene_swap(tf_ctx* c, int which)
{
    if (!c) return TF_INVALID_ARG;
    if (!c->p.use_swapping) return TF_INVALID_ARG;
    TF_CHECK(clear_abort(c));
    TF_CHECK(tfk_swap(c, which));
    return sync_checked(c);
}

extern "C" tf_status tf_scene_swap(tf_ctx* c) { TF_FLUSH(c); return scene_swap(c, 3); }
extern "C" tf_status tf_scene_swap_in(tf_ctx* c) { TF_FLUSH(c); return scene_swap(c, 1); }
extern "C" tf_status tf_scene_swap_out(tf_ctx* c) { TF_FLUSH(c); return scene_swap(c, 2); }

hipError_t tfk_fuse_frames(tf_ctx* c, const uint16_t* frames, size_t stride, size_t pitch, int n);   // tf_fuse.hip

extern "C" tf_status tf_scene_fuse_frames(tf_ctx* c, const float intr[4], const uint16_t* dev_frames, size_t stride,
                                         size_t pitch, const float* poses_rt, int n, tf_fuse_record* records)
{
    TF_FLUSH(c);
    if (!c || !dev_frames || !poses_rt || n < 0) return TF_INVALID_ARG;
    if (pitch == 0) pitch = (size_t)c->W * 2;
    if (pitch < (size_t)c->W * 2 || (n > 1 && stride < pitch * (size_t)c->H)) return TF_INVALID_ARG;
    if (c->st_host->sticky_error) return TF_HIP_ERROR;     // (in error since an earlier call: nothing runs)
    if (n == 0) return TF_OK;
    if (n > c->fuse_cap) {              // the pose / record lists grow to the largest batch seen
        TF_CHECK(hipStreamSynchronize(c->stream));
        if (c->fuse_pose) TF_CHECK(hipFree(c->fuse_pose));
        if (c->fuse_rec) TF_CHECK(hipFree(c->fuse_rec));
        c->fuse_pose = nullptr; c->fuse_rec = nullptr; c->fuse_cap = 0;
        TF_CHECK(dalloc(&c->fuse_pose, sizeof(float) * 12 * (size_t)n));
        TF_CHECK(dalloc(&c->fuse_rec, sizeof(tf_fuse_record) * (size_t)n));
        c->fuse_cap = n;
    }
    TF_CHECK(order_after_caller(c));
    TF_CHECK(hipMemcpyAsync(c->fuse_pose, poses_rt, sizeof(float) * 12 * (size_t)n, hipMemcpyHostToDevice, c->stream));
    IntrScope is(c, intr);
    TF_CHECK(tfk_fuse_frames(c, dev_frames, stride, pitch, n));
    if (records)
        TF_CHECK(hipMemcpyAsync(records, c->fuse_rec, sizeof(tf_fuse_record) * (size_t)n, hipMemcpyDeviceToHost, c->stream));
    return sync_checked(c);
}

extern "C" tf_status tf_swap_counts(tf_ctx* c, int counts[3])
{
    TF_FLUSH(c);
    if (!c || !counts) return TF_INVALID_ARG;
    tf_status s = sync_state(c);
    if (s != TF_OK) return s;
    counts[0] = c->st_host->swap_in; counts[1] = c->st_host->swap_out; counts[2] = c->st_host->swap_realloc;
    return TF_OK;
}

// GlobalCache::SaveToFile / ReadFromFile (GlobalCache.hpp:79-110): hasStoredData (1 byte per
// entry), then 512 voxels of 4 bytes per entry
extern "C" tf_status tf_swap_save(tf_ctx* c, const char* path)
{
    TF_FLUSH(c);
    if (!c || !path || !c->p.use_swapping) return TF_INVALID_ARG;
    const size_t nf = (size_t)c->n_total, nv = sizeof(TfVoxel) * (size_t)c->n_total * TF_BLK3;
    void* host = malloc(nf + nv);
    if (!host) return TF_OOM;
    hipError_t e = hipMemcpyAsync(host, c->swapFlags, nf, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync((char*)host + nf, c->swapStore, nv, hipMemcpyDeviceToHost, c->stream);
    tf_status s = tf_from_hip(e);
    if (s == TF_OK) s = sync_checked(c);
    if (s == TF_OK) {
        FILE* f = fopen(path, "wb");
        if (!f || fwrite(host, 1, nf + nv, f) != nf + nv) s = TF_INVALID_ARG;
        if (f) fclose(f);
    }
    free(host);
    return s;
}

extern "C" tf_status tf_swap_load(tf_ctx* c, const char* path)
{
    TF_FLUSH(c);
    if (!c || !path || !c->p.use_swapping) return TF_INVALID_ARG;
    const size_t nf = (size_t)c->n_total, nv = sizeof(TfVoxel) * (size_t)c->n_total * TF_BLK3;
    FILE* f = fopen(path, "rb");
    if (!f) return TF_INVALID_ARG;
    void* host = malloc(nf + nv);
    if (!host) { fclose(f); return TF_OOM; }
    const size_t got = fread(host, 1, nf + nv, f);
    fclose(f);
    tf_status s = TF_OK;
    if (got == nf + nv) {       // the reference reads the blocks only when the flags are complete
        hipError_t e = hipMemcpyAsync(c->swapFlags, host, nf, hipMemcpyHostToDevice, c->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(c->swapStore, (char*)host + nf, nv, hipMemcpyHostToDevice, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        s = tf_from_hip(e);
    } else s = TF_INVALID_ARG;
    free(host);
    return s;
}

extern "C" tf_status tf_vis_expected_depths(tf_ctx* c, const float intr[4], const float pose_rt[12])
{
    TF_FLUSH(c);
    if (!c || !pose_rt) return TF_INVALID_ARG;
    IntrScope is(c, intr);
    return tf_stage_expected_depths(c, pose_rt);
}

extern "C" tf_status tf_vis_render_image(tf_ctx* c, const float intr[4], const float pose_rt[12], int type, int new_raycast,
                                        uint8_t* dev_rgba, size_t step)
{
    TF_FLUSH(c);
    if (!c || !pose_rt || type < TF_RENDER_SHADED_GREYSCALE || type > TF_RENDER_COLOUR_FROM_CONFIDENCE) return TF_INVALID_ARG;
    IntrScope is(c, intr);
    tf_status s = set_pose_in(c, pose_rt, 0);
    if (s != TF_OK) return s;
    if (new_raycast) TF_CHECK(tfk_raycast(c, 0));        // RENDER_FROM_NEW_RAYCAST (VisualisationEngine_CUDA.cu:227-240)
    TF_CHECK(tfk_render_type(c, type));
    if (dev_rgba) {
        TF_CHECK(order_after_caller(c));                  // the caller may still read the image on stream 0
        const size_t row = (size_t)c->W * 4;
        TF_CHECK(hipMemcpy2DAsync(dev_rgba, step ? step : row, c->grey, row, row, c->H, hipMemcpyDeviceToDevice, c->stream));
    }
    return sync_checked(c);
}

extern "C" tf_status tf_vis_icp_maps(tf_ctx* c, const float intr[4], const float pose_rt[12], void* points,
                                    size_t points_step, void* normals, size_t normals_step)
{
    TF_FLUSH(c);
    if (!c || !pose_rt) return TF_INVALID_ARG;
    IntrScope is(c, intr);
    tf_status s = set_pose_in(c, pose_rt, 0);
    if (s != TF_OK) return s;
    TF_CHECK(tfk_raycast(c, 1));                          // castRay<true> (VisualisationEngine_CUDA.cu:340-345)
    TF_CHECK(tfk_icp_maps(c));                            // renderICP (:347-359) + the context's resized levels
    const size_t row = sizeof(float4) * (size_t)c->W;
    if (points || normals) TF_CHECK(order_after_caller(c));
    if (points)
        TF_CHECK(hipMemcpy2DAsync(points, points_step ? points_step : row, c->prev_pts[0], row, row, c->H,
                                  hipMemcpyDeviceToDevice, c->stream));
    if (normals)
        TF_CHECK(hipMemcpy2DAsync(normals, normals_step ? normals_step : row, c->prev_nrm[0], row, row, c->H,
                                  hipMemcpyDeviceToDevice, c->stream));
    return sync_checked(c);
}

// ---- state transfer -------------------------------------------------------------------
static void* buffer_ptr(tf_ctx* c, int which, int level, size_t* bytes)
{
    const size_t npx = (size_t)c->W * c->H;
    if (level < 0 || level >= TF_LEVELS) level = 0;
    const size_t nl = (size_t)c->lw[level] * c->lh[level];
    switch (which) {
    case TF_BUF_HASH: *bytes = sizeof(TfHashEntry) * (size_t)c->n_total; return c->hash;
    case TF_BUF_VBA: *bytes = sizeof(TfVoxel) * (size_t)c->p.n_blocks * TF_BLK3; return c->vba;
    case TF_BUF_VISIBLE_IDS: *bytes = sizeof(int) * (size_t)c->p.vis_capacity; return c->visibleIds;
    case TF_BUF_VISIBLE_TYPE: *bytes = (size_t)c->n_total; return c->visType;
    case TF_BUF_RANGE: *bytes = sizeof(float) * 2 * npx; return c->range;
    case TF_BUF_RAYCAST: *bytes = sizeof(float) * 4 * npx; return c->raycast;
    case TF_BUF_DISTS: *bytes = sizeof(float) * npx; return c->dists;
    case TF_BUF_DEPTH: *bytes = sizeof(uint16_t) * nl; return c->depth_pyr[level];
    case TF_BUF_CURR_POINTS: *bytes = sizeof(float4) * nl; return c->curr_pts[level];
    case TF_BUF_CURR_NORMALS: *bytes = sizeof(float4) * nl; return c->curr_nrm[level];
    case TF_BUF_PREV_POINTS: *bytes = sizeof(float4) * nl; return c->prev_pts[level];
    case TF_BUF_PREV_NORMALS: *bytes = sizeof(float4) * nl; return c->prev_nrm[level];
    case TF_BUF_GREY: *bytes = sizeof(uchar4) * npx; return c->grey;
    case TF_BUF_SWAP_STATE: *bytes = c->swapState ? (size_t)c->n_total : 0; return c->swapState;
    case TF_BUF_SWAP_STORED_FLAGS: *bytes = c->swapFlags ? (size_t)c->n_total : 0; return c->swapFlags;
    case TF_BUF_SWAP_STORED: *bytes = c->swapStore ? sizeof(TfVoxel) * (size_t)c->n_total * TF_BLK3 : 0; return c->swapStore;
    case TF_BUF_VBA_RGB: *bytes = c->vba_rgb ? sizeof(unsigned) * (size_t)c->p.n_blocks * TF_BLK3 : 0; return c->vba_rgb;
    case TF_BUF_ALLOC_LIST: *bytes = sizeof(int) * (size_t)c->p.n_blocks; return c->allocList;
    case TF_BUF_EXCESS_LIST: *bytes = sizeof(int) * (size_t)c->p.n_excess; return c->excessList;
    }
    *bytes = 0;
    return nullptr;
}

extern "C" tf_status tf_buffer_bytes(tf_ctx* c, int which, int level, size_t* bytes)
{
    TF_FLUSH(c);
    if (!c || !bytes) return TF_INVALID_ARG;
    return buffer_ptr(c, which, level, bytes) ? TF_OK : TF_INVALID_ARG;
}

extern "C" tf_status tf_download(tf_ctx* c, int which, int level, void* host, size_t bytes)
{
    TF_FLUSH(c);
    if (!c || !host) return TF_INVALID_ARG;
    size_t n;
    void* p = buffer_ptr(c, which, level, &n);
    if (!p || n != bytes) return TF_INVALID_ARG;
    TF_CHECK(hipMemcpyAsync(host, p, n, hipMemcpyDeviceToHost, c->stream));
    return sync_checked(c);
}

extern "C" tf_status tf_download_range(tf_ctx* c, int which, size_t offset, void* host, size_t bytes)
{
    TF_FLUSH(c);
    if (!c || !host) return TF_INVALID_ARG;
    size_t n;
    void* p = buffer_ptr(c, which, 0, &n);
    if (!p || offset > n || bytes > n - offset) return TF_INVALID_ARG;
    TF_CHECK(hipMemcpyAsync(host, (const char*)p + offset, bytes, hipMemcpyDeviceToHost, c->stream));
    return sync_checked(c);
}

extern "C" tf_status tf_upload(tf_ctx* c, int which, int level, const void* host, size_t bytes)
{
    TF_FLUSH(c);
    if (!c || !host) return TF_INVALID_ARG;
    size_t n;
    void* p = buffer_ptr(c, which, level, &n);
    if (!p || n != bytes) return TF_INVALID_ARG;
    TF_CHECK(hipMemcpyAsync(p, host, n, hipMemcpyHostToDevice, c->stream));
    if (which == TF_BUF_HASH) TF_CHECK(tfk_grid_rebuild(c));       // keep the block grid exact
    if (which == TF_BUF_RANGE) TF_CHECK(ed_spill_all(c));          // next CreateExpectedDepths: whole buffer
    static const int one = 1;
    if (which == TF_BUF_HASH || which == TF_BUF_VBA || which == TF_BUF_VBA_RGB || which == TF_BUF_ALLOC_LIST ||
        which == TF_BUF_EXCESS_LIST)                               // next reset (in-frame ones too): full clear
        TF_CHECK(hipMemcpyAsync((char*)c->st + offsetof(TfDevState, scene_external), &one, sizeof(int), hipMemcpyHostToDevice, c->stream));
    return sync_checked(c);
}

extern "C" tf_status tf_set_pose(tf_ctx* c, const float rt[12])
{
    TF_FLUSH(c);
    if (!c || !rt) return TF_INVALID_ARG;
    TF_CHECK(hipMemcpyAsync(c->st->pose, rt, sizeof(float) * 12, hipMemcpyHostToDevice, c->stream));
    return sync_checked(c);
}

extern "C" tf_status tf_set_counters(tf_ctx* c, int lastFreeBlockId, int lastFreeExcessListId, int noVisibleEntries)
{
    TF_FLUSH(c);
    if (!c) return TF_INVALID_ARG;
    tf_status s = sync_state(c);
    if (s != TF_OK) return s;
    c->st_host->lastFreeBlockId = lastFreeBlockId;
    c->st_host->lastFreeExcessListId = lastFreeExcessListId;
    c->st_host->noVisibleEntries = noVisibleEntries;
    c->st_host->scene_external = 1;                                 // next reset: full clear
    TF_CHECK(hipMemcpyAsync(c->st, c->st_host, sizeof(TfDevState), hipMemcpyHostToDevice, c->stream));
    return sync_checked(c);
}

extern "C" tf_status tf_get_totals(tf_ctx* c, tf_totals* t)
{
    TF_FLUSH(c);
    if (!c || !t) return TF_INVALID_ARG;
    tf_status s = sync_state(c);
    if (s != TF_OK) return s;
    const TfDevState* d = c->st_host;
    t->frames = d->tot_frames; t->frames_tracked = d->tot_tracked; t->resets = d->tot_resets;
    t->visible_sum = d->tot_visible; t->tiles_sum = d->tot_tiles;
    t->swapped_in = d->tot_swap_in; t->swapped_out = d->tot_swap_out;
    t->swapped_in_merged = d->tot_swap_merged;
    t->alloc_failed_type1 = d->tot_alloc_fail1; t->alloc_failed_type2 = d->tot_alloc_fail2;
    t->icp_fallbacks = c->icp_fallbacks;
    t->integrate_lanes_read = t->integrate_lanes_written = 0;
    std::vector<long long> h(2 * TF_INTEG_WG);
    TF_CHECK(hipMemcpyAsync(h.data(), c->integ_cnt, sizeof(long long) * h.size(), hipMemcpyDeviceToHost, c->stream));
    TF_CHECK(hipStreamSynchronize(c->stream));
    for (int i = 0; i < TF_INTEG_WG; ++i) { t->integrate_lanes_read += h[2 * i]; t->integrate_lanes_written += h[2 * i + 1]; }
    return TF_OK;
}

extern "C" tf_status tf_reset_totals(tf_ctx* c)
{
    TF_FLUSH(c);
    if (!c) return TF_INVALID_ARG;
    const size_t b = offsetof(TfDevState, tot_frames), e = offsetof(TfDevState, tot_alloc_fail2) + sizeof(long long);
    TF_CHECK(hipMemsetAsync((char*)c->st + b, 0, e - b, c->stream));
    TF_CHECK(hipMemsetAsync(c->integ_cnt, 0, sizeof(long long) * 2 * TF_INTEG_WG, c->stream));
    TF_CHECK(hipStreamSynchronize(c->stream));
    c->icp_fallbacks = 0;
    return TF_OK;
}
