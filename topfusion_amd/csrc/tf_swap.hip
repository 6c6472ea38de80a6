// tf_swap.hip -- voxel-block swapping between the active VBA and the GlobalCache, for gfx950
// (SURVEY §8f-2).  Enabled per context (tf_params::use_swapping, Scene(params, useSwapping),
// scene.hpp:29-33); TopFu itself runs without it (topfu.cpp:67).
//
// The reference holds the GlobalCache (GlobalCache.hpp:11-134: per-entry store, hasStoredData,
// HashSwapState 0 / 1 / 2, SDF_TRANSFER_BLOCK_NUM blocks per transfer) and the swapping
// branches of AllocateSceneFromDepth (enlarged-frustum visibility, swap-state marking,
// reAllocateSwappedOutVoxelBlocks; SceneReconstructionEngine_host.cu:159-189, 417-479), but
// not the engine that moves blocks (CUDAInstantiations.cu:8 comments ITMSwappingEngine_CUDA
// out).  The engine here is the published algorithm of that lineage, restated in
// the CPU oracle (test infrastructure) with serial ascending-index order where the lineage uses
// atomics:
//   IntegrateGlobalIntoLocal: entries in state 1 with a block, first T in index order: the
//     stored block is merged into the active one (CombineVoxelInformation) if there is one;
//     state 2.
//   SaveToGlobalMemory: entries in state 2 with a block and not visible this frame, first T:
//     block -> store, block reset to Voxel_s(), block returned to the free list
//     (allocList[lastFreeBlockId + 1 + rank] = ptr, ptr = -1, its grid cell cleared), state 0.
//
// MI355X design: the GlobalCache lives in HBM (2 KiB per hash entry: 2.4 GB at the reference's
// 1.18 M entries -- the "host" of the lineage is a second tier in the 288 GB of the same
// device), so a transfer is a device-side copy inside the frame's launches, with no host round
// trip and no staging buffer; hipMemcpy moves it to / from a file (tf_swap_save / _load).
// Three launches per frame after integration, over 4096-entry chunks like the allocation scans:
// count swap-in candidates; swap in (ordered by a chunk prefix) + count swap-out candidates;
// swap out.  The reallocation of listed swapped-out entries is the same count + prefix pattern
// over the visible list (ascending, so its serial free-list order is a prefix sum).
#include "tf_internal.h"

#define SW_CHUNK 4096          // entries per workgroup (256 threads x 16)

// byte i (0..15) of 16 bytes held as two 64-bit words
__device__ __forceinline__ unsigned sw_byte(unsigned long long lo, unsigned long long hi, int i)
{
    return (unsigned)(((i < 8) ? (lo >> (8 * i)) : (hi >> (8 * (i - 8)))) & 0xffull);
}
__device__ __forceinline__ void sw_load16(const unsigned char* p, unsigned long long* lo, unsigned long long* hi)
{
    uint4 v = *(const uint4*)p;
    *lo = (unsigned long long)v.x | ((unsigned long long)v.y << 32);
    *hi = (unsigned long long)v.z | ((unsigned long long)v.w << 32);
}

// exclusive scan over the 256-thread workgroup; *total receives the sum
__device__ __forceinline__ int sw_excl_scan(int v, int* total)
{
    __shared__ int wsum[4];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int n = __shfl_up(inc, o, 64);
        if (lane >= o) inc += n;
    }
    if (lane == 63) wsum[wave] = inc;
    __syncthreads();
    int off = 0, tot = 0;
    for (int w = 0; w < 4; ++w) { const int s = wsum[w]; if (w < wave) off += s; tot += s; }
    __syncthreads();
    *total = tot;
    return off + inc - v;
}

// ---------------------------------------------------------------------------------------
// reAllocateSwappedOutVoxelBlocks_device (SceneReconstructionEngine_host.cu:417-432): entries of
// visible type > 0 whose block was swapped out (ptr == -1) take blocks from the free list in
// ascending index order; once it is empty the rest keep ptr -1.  The candidates are the visible
// list's entries (ascending, so the serial free-list order is a prefix sum over the list); when
// the list is full (noVisibleEntries == cap: entries past the capacity may be of type > 0
// without being listed, and the reference's pass covers every entry) every hash entry with
// visType > 0.  Two launches over 4096-candidate chunks, as the swap-in / swap-out passes:
// count per chunk, then each chunk assigns allocList[v - prefix - rank].
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ int sw_realloc_flags(const TfDevState* st, const TfHashEntry* __restrict__ hash,
                                                const int* __restrict__ visibleIds, const unsigned char* __restrict__ visType,
                                                int cap, int n_total, int* ids)
{
    const int nv = st->noVisibleEntries;
    const bool full = nv >= cap;
    const int n = full ? n_total : nv;
    const int base = blockIdx.x * SW_CHUNK + threadIdx.x * 16;
    int flags = 0;
    if (base >= n) return 0;
    if (full) {
        if (base + 16 <= n_total) {
            unsigned long long vlo, vhi;
            sw_load16(visType + base, &vlo, &vhi);
#pragma unroll
            for (int i = 0; i < 16; ++i) ids[i] = sw_byte(vlo, vhi, i) > 0 ? base + i : -1;
        } else {
            for (int i = 0; i < 16; ++i) ids[i] = base + i < n_total && visType[base + i] > 0 ? base + i : -1;
        }
    } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) ids[i] = base + i < n ? visibleIds[base + i] : -1;
    }
    int ptr[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) ptr[i] = ids[i] >= 0 ? hash[ids[i]].ptr : 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) if (ptr[i] == -1) flags |= 1 << i;
    return flags;
}

__global__ void __launch_bounds__(256)
k_swap_realloc_count(TfDevState* __restrict__ st, const TfHashEntry* __restrict__ hash, const int* __restrict__ visibleIds,
                     const unsigned char* __restrict__ visType, int* __restrict__ counts, int cap, int n_total)
{
    if (st->abort) return;
    int ids[16];
    const int flags = sw_realloc_flags(st, hash, visibleIds, visType, cap, n_total, ids);
    int tot;
    sw_excl_scan(__popc(flags), &tot);
    if (threadIdx.x == 0) counts[2 * blockIdx.x] = tot;
    if (blockIdx.x == 0 && threadIdx.x == 0) counts[1] = st->lastFreeBlockId;   // the free-list top both passes use
}

__global__ void __launch_bounds__(256)
k_swap_realloc(TfDevState* __restrict__ st, TfHashEntry* __restrict__ hash, const int* __restrict__ visibleIds,
               const unsigned char* __restrict__ visType, const int* __restrict__ allocList, int2* __restrict__ grid,
               const int* __restrict__ counts, int n_chunks, int cap, int n_total)
{
    if (st->abort) return;
    int pre = 0, all = 0;
    for (int h = threadIdx.x; h < n_chunks; h += 256) {
        const int c = counts[2 * h];
        all += c;
        if (h < (int)blockIdx.x) pre += c;
    }
    sw_excl_scan(pre, &pre);
    sw_excl_scan(all, &all);
    const int v = counts[1];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const int got = all < v + 1 ? all : (v + 1 > 0 ? v + 1 : 0);
        st->lastFreeBlockId = v - got;
        st->swap_realloc = got;
    }
    int ids[16];
    const int flags = sw_realloc_flags(st, hash, visibleIds, visType, cap, n_total, ids);
    int nchunk;
    int r = pre + sw_excl_scan(__popc(flags), &nchunk);
    if (!flags) return;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        if (!(flags & (1 << i))) continue;
        if (v - r >= 0) {
            TfHashEntry e = hash[ids[i]];
            e.ptr = allocList[v - r];
            hash[ids[i]].ptr = e.ptr;
            grid_set(grid, e, ids[i]);
        }
        ++r;
    }
}

// swap-in candidates of a chunk: state 1 with a block
__global__ void __launch_bounds__(256)
k_swap_count_in(TfDevState* __restrict__ st, const unsigned char* __restrict__ swapState,
                const TfHashEntry* __restrict__ hash, int* __restrict__ counts, int n_total)
{
    if (st->abort) return;
    const int base = blockIdx.x * SW_CHUNK + threadIdx.x * 16;
    int c = 0;
    if (base < n_total) {
        unsigned long long lo, hi;
        sw_load16(swapState + base, &lo, &hi);
        for (int i = 0; i < 16; ++i)
            if (sw_byte(lo, hi, i) == 1 && hash[base + i].ptr >= 0) ++c;
    }
    int tot;
    sw_excl_scan(c, &tot);
    if (threadIdx.x == 0) counts[2 * blockIdx.x] = tot;
    if (blockIdx.x == 0 && threadIdx.x == 0) st->swap_merged = 0;   // (k_swap_in counts this pass's merges)
}

// CombineVoxelInformation (depth part): src = stored, dst = active; canonical arithmetic
__device__ __forceinline__ unsigned sw_combine(unsigned src, unsigned dst, int maxW)
{
    const int oldW = (src >> 16) & 0xff, newW0 = (dst >> 16) & 0xff;
    if (oldW == 0) return dst;
    const float oldF = tf_short_to_float((short)(src & 0xffff)), newF0 = tf_short_to_float((short)(dst & 0xffff));
    float newF = (float)oldW * oldF + (float)newW0 * newF0;
    int newW = oldW + newW0;
    newF = newF / (float)newW;
    newW = newW < maxW ? newW : maxW;
    const short sdf = (short)(newF * 32767.0f);
    return (unsigned)(unsigned short)sdf | ((unsigned)(newW & 0xff) << 16) | (dst & 0xff000000u);
}

// IntegrateGlobalIntoLocal for this chunk's candidates of rank < T, then the chunk's swap-out
// candidates (its states are final once its own swap-ins are done: no other workgroup touches
// this chunk's entries)
__global__ void __launch_bounds__(256)
k_swap_in(TfDevState* __restrict__ st, unsigned char* __restrict__ swapState, const unsigned char* __restrict__ swapFlags,
          const TfVoxel* __restrict__ store, const TfHashEntry* __restrict__ hash, TfVoxel* __restrict__ vba,
          const unsigned char* __restrict__ visType, int* __restrict__ counts, int n_chunks, int n_total, int T, int maxW)
{
    if (st->abort) return;
    __shared__ int list[SW_CHUNK];
    int pre = 0, all = 0;
    for (int h = threadIdx.x; h < n_chunks; h += 256) {
        const int c = counts[2 * h];
        all += c;
        if (h < (int)blockIdx.x) pre += c;
    }
    int tmp;
    sw_excl_scan(pre, &pre);
    sw_excl_scan(all, &all);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        st->swap_in = all < T ? all : T;
        st->tot_swap_in += all < T ? all : T;
        st->swap_free0 = st->lastFreeBlockId;            // for k_swap_out (nobody writes it in between)
    }
    const int base = blockIdx.x * SW_CHUNK + threadIdx.x * 16;
    unsigned long long lo = 0, hi = 0;
    if (base < n_total) sw_load16(swapState + base, &lo, &hi);
    int flags = 0, nmine = 0;
    if (base < n_total)
        for (int i = 0; i < 16; ++i)
            if (sw_byte(lo, hi, i) == 1 && hash[base + i].ptr >= 0) { flags |= 1 << i; ++nmine; }
    int nchunk;
    const int r0 = sw_excl_scan(nmine, &nchunk);
    // the chunk's candidates in index order, those of global rank < T
    int take = T - pre;                                  // how many of this chunk's candidates go in
    take = take < 0 ? 0 : (take > nchunk ? nchunk : take);
    {
        int r = r0;
        for (int i = 0; i < 16; ++i)
            if (flags & (1 << i)) { if (r < take) list[r] = base + i; ++r; }
    }
    __syncthreads();
    int merged = 0;
    for (int k = 0; k < take; ++k) {
        const int id = list[k];
        if (swapFlags[id]) {
            const uint2* src = (const uint2*)(store + (size_t)id * TF_BLK3);
            uint2* dst = (uint2*)(vba + (size_t)hash[id].ptr * TF_BLK3);
            const uint2 s2 = src[threadIdx.x], d2 = dst[threadIdx.x];
            dst[threadIdx.x] = make_uint2(sw_combine(s2.x, d2.x, maxW), sw_combine(s2.y, d2.y, maxW));
            ++merged;
        }
        if (threadIdx.x == 0) swapState[id] = 2;
    }
    if (threadIdx.x == 0 && merged) {
        atomicAdd((unsigned long long*)&st->tot_swap_merged, (unsigned long long)merged);
        atomicAdd(&st->swap_merged, merged);
    }
    __syncthreads();
    // swap-out candidates of the chunk: state 2 (after the swap-ins above), a block, not visible
    int c = 0;
    if (base < n_total) {
        sw_load16(swapState + base, &lo, &hi);
        unsigned long long vlo, vhi;
        sw_load16(visType + base, &vlo, &vhi);
        for (int i = 0; i < 16; ++i)
            if (sw_byte(lo, hi, i) == 2 && sw_byte(vlo, vhi, i) == 0 && hash[base + i].ptr >= 0) ++c;
    }
    int tot;
    sw_excl_scan(c, &tot);
    if (threadIdx.x == 0) counts[2 * blockIdx.x + 1] = tot;
    (void)tmp;
}

// swap-out candidates of a chunk, for a SaveToGlobalMemory on its own (k_swap_in counts them
// when the two run together); also records the free-list top k_swap_out starts from
__global__ void __launch_bounds__(256)
k_swap_count_out(TfDevState* __restrict__ st, const unsigned char* __restrict__ swapState,
                 const unsigned char* __restrict__ visType, const TfHashEntry* __restrict__ hash,
                 int* __restrict__ counts, int n_total)
{
    if (st->abort) return;
    const int base = blockIdx.x * SW_CHUNK + threadIdx.x * 16;
    int c = 0;
    if (base < n_total) {
        unsigned long long lo, hi, vlo, vhi;
        sw_load16(swapState + base, &lo, &hi);
        sw_load16(visType + base, &vlo, &vhi);
        for (int i = 0; i < 16; ++i)
            if (sw_byte(lo, hi, i) == 2 && sw_byte(vlo, vhi, i) == 0 && hash[base + i].ptr >= 0) ++c;
    }
    int tot;
    sw_excl_scan(c, &tot);
    if (threadIdx.x == 0) counts[2 * blockIdx.x + 1] = tot;
    if (blockIdx.x == 0 && threadIdx.x == 0) st->swap_free0 = st->lastFreeBlockId;
}

// SaveToGlobalMemory for the chunk's candidates of rank < T
__global__ void __launch_bounds__(256)
k_swap_out(TfDevState* __restrict__ st, unsigned char* __restrict__ swapState, unsigned char* __restrict__ swapFlags,
           TfVoxel* __restrict__ store, TfHashEntry* __restrict__ hash, TfVoxel* __restrict__ vba,
           const unsigned char* __restrict__ visType, int* __restrict__ allocList, int2* __restrict__ grid,
           const int* __restrict__ counts, int n_chunks, int n_total, int T, int n_blocks)
{
    if (st->abort) return;
    __shared__ int list[SW_CHUNK];
    int pre = 0, all = 0;
    for (int h = threadIdx.x; h < n_chunks; h += 256) {
        const int c = counts[2 * h + 1];
        all += c;
        if (h < (int)blockIdx.x) pre += c;
    }
    sw_excl_scan(pre, &pre);
    sw_excl_scan(all, &all);
    const int free0 = st->swap_free0;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const int n_out = all < T ? all : T;
        st->swap_out = n_out;
        st->lastFreeBlockId = free0 + n_out;             // cleanMemory's increments, taken or not
        st->tot_swap_out += n_out;
    }
    const int base = blockIdx.x * SW_CHUNK + threadIdx.x * 16;
    int flags = 0, nmine = 0;
    if (base < n_total) {
        unsigned long long lo, hi, vlo, vhi;
        sw_load16(swapState + base, &lo, &hi);
        sw_load16(visType + base, &vlo, &vhi);
        for (int i = 0; i < 16; ++i)
            if (sw_byte(lo, hi, i) == 2 && sw_byte(vlo, vhi, i) == 0 && hash[base + i].ptr >= 0) { flags |= 1 << i; ++nmine; }
    }
    int nchunk;
    const int r0 = sw_excl_scan(nmine, &nchunk);
    int take = T - pre;
    take = take < 0 ? 0 : (take > nchunk ? nchunk : take);
    {
        int r = r0;
        for (int i = 0; i < 16; ++i)
            if (flags & (1 << i)) { if (r < take) list[r] = base + i; ++r; }
    }
    __syncthreads();
    const uint2 fill = make_uint2(32767u, 32767u);      // Voxel_s(): sdf 32767, w 0
    for (int k = 0; k < take; ++k) {
        const int id = list[k];
        const TfHashEntry e = hash[id];
        uint2* blk = (uint2*)(vba + (size_t)e.ptr * TF_BLK3);
        ((uint2*)(store + (size_t)id * TF_BLK3))[threadIdx.x] = blk[threadIdx.x];   // moveActiveDataToTransferBuffer
        blk[threadIdx.x] = fill;
        __syncthreads();                                // every lane has read the entry before it changes
        if (threadIdx.x == 0) {
            swapFlags[id] = 1;
            swapState[id] = 0;                          // cleanMemory
            const int vbaIdx = free0 + pre + k;
            if (vbaIdx < n_blocks - 1) {
                allocList[vbaIdx + 1] = e.ptr;
                hash[id].ptr = -1;
                if (tf_grid_in(e.x, e.y, e.z)) grid[tf_grid_cell(e.x, e.y, e.z)] = make_int2(-1, TF_VOFF_NONE);
            }
        }
    }
}

hipError_t tfk_swap_realloc(tf_ctx* c)
{
    // chunks over the table: the visible list never holds more than n_total entries
    const int nch = (c->n_total + SW_CHUNK - 1) / SW_CHUNK;
    hipLaunchKernelGGL(k_swap_realloc_count, dim3(nch), dim3(256), 0, c->stream, c->st, c->hash, c->visibleIds, c->visType,
                       c->swapCounts, c->p.vis_capacity, c->n_total);
    hipLaunchKernelGGL(k_swap_realloc, dim3(nch), dim3(256), 0, c->stream, c->st, c->hash, c->visibleIds, c->visType,
                       c->allocList, c->bgrid, c->swapCounts, nch, c->p.vis_capacity, c->n_total);
    return hipGetLastError();
}

// which: 1 = IntegrateGlobalIntoLocal, 2 = SaveToGlobalMemory, 3 = both (the frame's order)
hipError_t tfk_swap(tf_ctx* c, int which)
{
    const int nch = (c->n_total + SW_CHUNK - 1) / SW_CHUNK, T = c->p.swap_transfer_blocks;
    if (which & 1) {
        hipLaunchKernelGGL(k_swap_count_in, dim3(nch), dim3(256), 0, c->stream, c->st, c->swapState, c->hash, c->swapCounts,
                           c->n_total);
        hipLaunchKernelGGL(k_swap_in, dim3(nch), dim3(256), 0, c->stream, c->st, c->swapState, c->swapFlags, c->swapStore,
                           c->hash, c->vba, c->visType, c->swapCounts, nch, c->n_total, T, c->p.maxW);
    }
    if (which & 2) {
        if (!(which & 1))
            hipLaunchKernelGGL(k_swap_count_out, dim3(nch), dim3(256), 0, c->stream, c->st, c->swapState, c->visType, c->hash,
                               c->swapCounts, c->n_total);
        hipLaunchKernelGGL(k_swap_out, dim3(nch), dim3(256), 0, c->stream, c->st, c->swapState, c->swapFlags, c->swapStore,
                           c->hash, c->vba, c->visType, c->allocList, c->bgrid, c->swapCounts, nch, c->n_total, T,
                           c->p.n_blocks);
    }
    return hipGetLastError();
}
