// tf_icp.hip -- projective point-to-plane ICP for gfx950.
//
// ONE launch per ICP iteration and no host round trip (the reference syncs to the host and
// solves with OpenCV 19 times per frame, projective_icp.cpp:187-210).  k_icp_iter:
//   * find_coresp + row build (proj_icp.cu:80-117,359-377).  A wave64 owns one 32x8
//     reference CTA, 4 pixels per lane (reference tids l, l+64, l+128, l+192), and reproduces
//     the reference's 256-wide halving tree (temp_utils.hpp:503-523) bit for bit: two adds
//     in registers, then a *transposed* xor butterfly that halves the live sums at every
//     step (32 lane exchanges for all 27 sums instead of 27 x 6).
//   * workgroup w owns reference CTAs w, w+256, w+512, ... so it produces exactly the
//     column sum that thread w of icp_final_reduce_kernel computes (proj_icp.cu:389-391),
//     in the same order; no [27 x #CTA] partial buffer.
//   * the last workgroup to finish (agent-scope ticket, write-through sc1 stores/loads,
//     MI355X_MICROARCH.md "Valid forms" row 1) runs the final 256-wide tree, the det check
//     (cv::determinant), the 6x6 solve, Rodrigues and affine = Tinc * affine with one wave
//     holding the 6x7 system one element per lane.
// A failed det check sets state->abort; every later ICP / scene kernel of the frame no-ops.
#include "tf_internal.h"
#include <string.h>

#define ICP_T_STRIDE 28        // 27 column sums per workgroup, padded
#define ICP_NWG 256            // = FINAL_REDUCE_CTA_SIZE (proj_icp.cu:25-26)
#define ICP_WAVES 5
#define ICP_MAX_SLOTS 40       // reference CTAs per workgroup (40*256 CTAs = 2560x1024 pixels)

#ifdef TF_ICP_TIMING
// debug build only: per-phase wall clock of the last workgroup (s_memrealtime, 100 MHz)
__device__ unsigned long long g_icp_ts[16];
#define ICP_TS0() const unsigned long long ts0_ = __builtin_amdgcn_s_memrealtime()
#define ICP_TS(k) do { if (threadIdx.x == 0) g_icp_ts[k] += __builtin_amdgcn_s_memrealtime() - ts0_; } while (0)
extern "C" int tf_debug_icp_ts(unsigned long long* out)
{
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_icp_ts), sizeof(g_icp_ts), 0, hipMemcpyDeviceToHost);
}
#define IPT_NOW() __builtin_amdgcn_s_memrealtime()
#define IPT_ADD(k, v) do { } while (0)
// timeline of the last persistent launch: per iteration [256 starts][256 publishes][8 WG0 events]
#define IPT_STRIDE (2 * ICP_NWG + 10)
__device__ unsigned long long g_icp_tl[64 * IPT_STRIDE];
#define IPT_REC(it, slot) IPT_REC_T(it, slot, 0)
// a stamp after a value: the value is an operand of a volatile asm placed before the stamp, so
// the compiler cannot sink the work it depends on past the stamp (VALU issue is in order; what is
// left in flight is a pipeline depth); workgroup 0 alone records (the slots are shared)
#define IPT_REC_DEP(it, slot, val_) do { \
    const float d_ = (float)(val_); \
    asm volatile("; ipt dependency %0" :: "v"(d_)); \
    __builtin_amdgcn_sched_barrier(0); \
    if (blockIdx.x == 0 && threadIdx.x == 0 && (it) < 64) g_icp_tl[(it) * IPT_STRIDE + (slot)] = IPT_NOW(); \
    __builtin_amdgcn_sched_barrier(0); } while (0)
// the stamp is fenced against the scheduler (no instruction moves across it) and issued after the
// VALU work before it has been issued; the data it measures lives in registers, so the segment
// between two stamps is that segment's issue time
#define IPT_REC_T(it, slot, t) do { __builtin_amdgcn_sched_barrier(0); \
    if (threadIdx.x == (t) && (it) < 64) g_icp_tl[(it) * IPT_STRIDE + (slot)] = IPT_NOW(); \
    __builtin_amdgcn_sched_barrier(0); } while (0)
extern "C" int tf_debug_icp_timeline(unsigned long long* out)
{
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_icp_tl), sizeof(g_icp_tl), 0, hipMemcpyDeviceToHost);
}
// workgroup 0's shader clock (s_memtime) beside the 100 MHz clock at each iteration start: the
// shader clock the kernel ran at
__device__ unsigned long long g_icp_clk[64 * 2];
#define IPT_CLK(it) do { if (blockIdx.x == 0 && threadIdx.x == 0 && (it) < 64) { \
    g_icp_clk[2 * (it)] = __builtin_amdgcn_s_memtime(); g_icp_clk[2 * (it) + 1] = __builtin_amdgcn_s_memrealtime(); } } while (0)
// the tail's halves on the shader clock, each run twice in a row (solve, solve again, Rodrigues,
// Rodrigues again) per iteration of workgroup 0
__device__ long long g_icp_tail_cyc[64 * 4];
#define IPT_CYC(val_) ({ const float d_ = (float)(val_); asm volatile("; ipt dependency %0" :: "v"(d_)); \
    __builtin_amdgcn_sched_barrier(0); const long long t_ = (long long)__builtin_amdgcn_s_memtime(); \
    __builtin_amdgcn_sched_barrier(0); t_; })
extern "C" int tf_debug_icp_tail_cycles(long long* out)
{
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_icp_tail_cyc), sizeof(g_icp_tail_cyc), 0, hipMemcpyDeviceToHost);
}
extern "C" int tf_debug_icp_clock(unsigned long long* out)
{
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_icp_clk), sizeof(g_icp_clk), 0, hipMemcpyDeviceToHost);
}
#else
#define ICP_TS0()
#define ICP_TS(k)
#define IPT_NOW() 0ull
#define IPT_ADD(k, v) do { } while (0)
#define IPT_REC(it, slot) do { } while (0)
#define IPT_REC_T(it, slot, t) do { } while (0)
#define IPT_REC_DEP(it, slot, val_) do { } while (0)
#define IPT_CLK(it) do { } while (0)
#endif

struct IcpLevel {
    const float4* vcurr; const float4* ncurr; const float4* vprev; const float4* nprev;
    int W, H, gx, nct;
    float fx, fy, cx, cy;
    float min_cosine, dist2;
};

// One exchange step of the transposed butterfly: lanes with (lane & OFF) keep the upper half
// of the N live sums, the others the lower half; each kept sum is completed with the
// partner lane's copy, so every sum sees the same pairings as a full xor butterfly.  The
// exchanges are cross-lane register moves, no LDS: v_permlane32_swap / v_permlane16_swap for
// the 32- and 16-lane steps (one instruction swaps the halves of two sums), DPP for the rest
// (xor 8 = row_ror:8, xor 4 = row_half_mirror then quad_perm xor 3, xor 2/1 = quad_perm).
// a + b == b + a bit for bit, so which operand is the kept one does not matter.
template <int CTRL>
__device__ __forceinline__ float dppf(float v)
{
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float xor1(float v) { return dppf<0xB1>(v); }                  // quad_perm [1,0,3,2]
__device__ __forceinline__ float xor2(float v) { return dppf<0x4E>(v); }                  // quad_perm [2,3,0,1]
__device__ __forceinline__ float xor4(float v) { return dppf<0x1B>(dppf<0x141>(v)); }     // half_mirror, [3,2,1,0]
__device__ __forceinline__ float xor8(float v) { return dppf<0x128>(v); }                 // row_ror:8

template <int N, int OFF>
__device__ __forceinline__ void tstep(float* v, int lane)
{
#pragma unroll
    for (int j = 0; j < N / 2; ++j) {
        if constexpr (OFF == 32 || OFF == 16) {
            auto r = OFF == 32 ? __builtin_amdgcn_permlane32_swap(__float_as_uint(v[j]), __float_as_uint(v[j + N / 2]), false, false)
                               : __builtin_amdgcn_permlane16_swap(__float_as_uint(v[j]), __float_as_uint(v[j + N / 2]), false, false);
            v[j] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
        } else {
            const bool hi = (lane & OFF) != 0;
            const float send = hi ? v[j] : v[j + N / 2];
            const float keep = hi ? v[j + N / 2] : v[j];
            const float recv = OFF == 8 ? xor8(send) : (OFF == 4 ? xor4(send) : xor2(send));
            v[j] = keep + recv;
        }
    }
}

#ifndef IP_SVD_LANES
#define IP_SVD_LANES 1         // the OpenCV algebra's cv::solve(DECOMP_SVD): 1 = lane-parallel, 0 = serial (A/B)
#endif
#include "tf_icp_tail.h"
#include "tf_pose.h"
#include "tf_vis.h"

// rows of 4 pixels per lane with the current-frame point/normal already in registers and both
// previous-map gathers issued before the dependent tests (defined with the persistent kernel)
typedef float ip_f2 __attribute__((ext_vector_type(2)));   // two pixels' values: v_pk_* arithmetic
// the current-frame point / normal of a lane's pixel pair (2h, 2h + 1), one packed pair per component
struct IpPix { ip_f2 vx, vy, vz, nx, ny, nz; };
// pixel j of the lane: (map index valid, point, normal) -> pair j / 2, element j % 2
__device__ __forceinline__ void ip_set(IpPix (&px)[2], int j, float4 v, float4 n)
{
    IpPix& p = px[j >> 1];
    if (j & 1) { p.vx.y = v.x; p.vy.y = v.y; p.vz.y = v.z; p.nx.y = n.x; p.ny.y = n.y; p.nz.y = n.z; }
    else { p.vx.x = v.x; p.vy.x = v.y; p.vz.x = v.z; p.nx.x = n.x; p.ny.x = n.y; p.nz.x = n.z; }
}
__device__ __forceinline__ void ip_rows4(const IcpLevel& L, const float* aff, const IpPix (&px)[2],
                                         const int (&xy)[4], ip_f2 (&r01)[7], ip_f2 (&r23)[7]);
__device__ __forceinline__ float ip_cta_reduce(const ip_f2 (&r01)[7], const ip_f2 (&r23)[7], int lane);

template <int ALG>
__global__ void __launch_bounds__(64 * ICP_WAVES)
k_icp_iter(IcpLevel L, TfDevState* __restrict__ st, float* __restrict__ T, unsigned* __restrict__ ticket,
           int nwg, int slots, int last_iter)
{
    __shared__ float red[ICP_MAX_SLOTS][ICP_T_STRIDE];
    __shared__ float tv[27][ICP_NWG + 1];   // +1: the gather's (col, q) stores hit distinct banks
    __shared__ int is_last;
    if (st->abort || st->mode == 0) return;
    ICP_TS0();
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    float aff[12];
#pragma unroll
    for (int i = 0; i < 12; ++i) aff[i] = st->affine[i];
    for (int s = wave; s < slots; s += ICP_WAVES) {
        const int cta = blockIdx.x + ICP_NWG * s;
        if (cta >= L.nct) break;
        const int bx = cta % L.gx, by = cta / L.gx;
        // the CTA's current maps with unconditional loads, then ip_rows4 (the per-pixel
        // per-pixel early returns make every load a branch: ~10 round trips per CTA)
        IpPix q[2];
        int qxy[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int t = lane + 64 * j;
            const int x = bx * 32 + (t & 31), y = by * 8 + (t >> 5);
            const bool in = x < L.W && y < L.H;
            qxy[j] = in ? 1 : -1;
            const int pi = in ? y * L.W + x : 0;
            float4 v = L.vcurr[pi], n = L.ncurr[pi];
            if (!in) { v = make_float4(0.f, 0.f, 0.f, 0.f); n = v; }
            ip_set(q, j, v, n);
        }
        ip_f2 r01[7], r23[7];
        ip_rows4(L, aff, q, qxy, r01, r23);
        const float tot = ip_cta_reduce(r01, r23, lane);    // lane l ends with sum (l >> 1)
        const int sidx = lane >> 1;
        if (!(lane & 1) && sidx < 27) red[s][sidx] = tot;
    }
    __syncthreads();
    // column sum of icp_final_reduce_kernel thread blockIdx.x: 0 + P[w] + P[w+256] + ...
    if (tid < 27) {
        float sum = 0.f;
        for (int s = 0; s < slots; ++s) {
            if (blockIdx.x + ICP_NWG * s >= L.nct) break;
            sum += red[s][tid];
        }
        __hip_atomic_store(&T[blockIdx.x * ICP_T_STRIDE + tid], sum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        unsigned old = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        is_last = (old == (unsigned)nwg - 1);
    }
    __syncthreads();
    if (!is_last) return;
    ICP_TS(1);
    // ---- last workgroup: final 256-wide tree over the column sums --------------------------
    // (write-through sc1 loads: 7 x 16 B per column, aux 16 = sc1)
    if (tid < ICP_NWG) {
        float4 q4[7];
        if (tid < nwg) {
            __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(T, 0, ICP_NWG * ICP_T_STRIDE * 4, 0x00020000);
#pragma unroll
            for (int q = 0; q < 7; ++q) {
                q4[q] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                    rs, (tid * ICP_T_STRIDE + 4 * q) * 4, 0, 16));
            }
        } else {
#pragma unroll
            for (int q = 0; q < 7; ++q) q4[q] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int q = 0; q < 7; ++q) {
            tv[4 * q + 0][tid] = q4[q].x;
            if (4 * q + 1 < 27) tv[4 * q + 1][tid] = q4[q].y;
            if (4 * q + 2 < 27) tv[4 * q + 2][tid] = q4[q].z;
            if (4 * q + 3 < 27) tv[4 * q + 3][tid] = q4[q].w;
        }
    }
    __syncthreads();
    ICP_TS(2);
    if (wave != 0) return;
    if (lane == 0) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // halving tree over the 256 columns: steps 128 and 64 from LDS, then the transposed butterfly
    float v[32];
#pragma unroll
    for (int q = 0; q < 27; ++q) {
        float a0 = tv[q][lane] + tv[q][lane + 128];
        float a1 = tv[q][lane + 64] + tv[q][lane + 192];
        v[q] = a0 + a1;
    }
#pragma unroll
    for (int q = 27; q < 32; ++q) v[q] = 0.f;
    tstep<32, 32>(v, lane);
    tstep<16, 16>(v, lane);
    tstep<8, 8>(v, lane);
    tstep<4, 4>(v, lane);
    tstep<2, 2>(v, lane);
    const float tot = v[0] + xor1(v[0]);     // lane l holds sum (l >> 1)
    float sm[27];
#pragma unroll
    for (int q = 0; q < 27; ++q) sm[q] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, tot), 2 * q));
    if (lane < 27) st->sums[lane] = __shfl(tot, 2 * lane, 64);
    if (lane == 0) st->icp_iters += 1;
    // StreamHelper::get unpacking (projective_icp.cpp:51-61)
    float Am[6][6], bv[6];
    {
        int shift = 0;
#pragma unroll
        for (int i = 0; i < 6; ++i)
#pragma unroll
            for (int j = i; j < 7; ++j) {
                float value = sm[shift++];
                if (j == 6) bv[i] = value;
                else { Am[j][i] = value; Am[i][j] = value; }
            }
    }
    ICP_TS(3);
    double det = icp_det6<ALG>(Am);
    ICP_TS(4);
    if (fabs(det) < 1e-15 || isnan(det)) {                     // projective_icp.cpp:197-203
        if (lane == 0) { st->icp_ok = 0; st->abort = 1; }
        return;
    }
    float rv[6];
    float R[9], tinc[12], A[12];
    if constexpr (ALG != 0 && IP_SVD_LANES) {                  // (tot: lane 2q holds sum q)
        icp_cv_solve_svd6_lanes<ALG>(tot, 2, lane, rv);
        icp_cv_rodrigues<ALG>(rv, R);
    } else {
        icp_solve_rodrigues<ALG>(Am, bv, rv, R);
    }
    ICP_TS(5);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        tinc[j * 4 + 0] = R[j * 3 + 0]; tinc[j * 4 + 1] = R[j * 3 + 1]; tinc[j * 4 + 2] = R[j * 3 + 2];
        tinc[j * 4 + 3] = rv[3 + j];
    }
#pragma unroll
    for (int i = 0; i < 12; ++i) A[i] = aff[i];
    tf_rigid_mul(tinc, A, A);
    if (lane < 12) st->affine[lane] = A[lane];
    ICP_TS(6);
#ifdef TF_ICP_TIMING
    if (threadIdx.x == 0) g_icp_ts[0] += 1;
#endif
    if (last_iter == 1 && lane == 0) {
        // poses_.push_back(poses_.back() * affine) (topfu.cpp:243) and the derived matrices
        float pose[12];
        for (int i = 0; i < 12; ++i) pose[i] = st->pose[i];
        tf_rigid_mul(pose, A, pose);
        for (int i = 0; i < 12; ++i) st->pose[i] = pose[i];
        tf_set_pose_matrices(st, pose, 1);
    }
}

// =========================================================================================
// Persistent ICP: ONE launch per frame for all levels and iterations.
//
// 256 workgroups x 8 waves stay resident.  Workgroup w owns reference CTAs w, w+256, ... of
// every level (the column of icp_final_reduce_kernel it reproduces); its current-frame maps
// stay in registers for the whole level, so an iteration costs one dependent gather (previous
// maps) instead of a launch plus four dependent loads.  Cross-workgroup exchange uses 64-bit
// TAGGED slots: each value is stored as (generation << 32 | float bits) with one agent-scope
// (sc1) 8-byte atomic store, so a reader that sees the current generation also sees the data
// -- no ticket counter, no fence.  The exchange of an iteration is the hierarchical gather
// described above k_icp_frame.  Every spin is bounded (status 2 -> the host reports a HIP
// error) so no wave can outlive a missing peer.
// =========================================================================================
#define IP_WAVES 8
#ifndef TF_PROJ_DIV
#define TF_PROJ_DIV 0
#endif
#define IP_SREG 1                       // CTA slots kept in registers per wave (8 per WG; larger images use k_icp_iter)
#define IP_SPIN_LIMIT (1u << 21)
#ifndef IP_SLEEP
#define IP_SLEEP 0                      // s_sleep between hand-off polls (x 64 cycles); round 6 A/B under the
                                        // OpenCV 4 algebra: 0 vs 1 = 2829 / 2825 vs 2816 / 2819 frames/s, ICP
                                        // 0.304 vs 0.306 ms (profiles/r06/ab_icp_poll_sleep.txt); 2 = as 1
#endif
#define IP_PART (2 * ICP_NWG * ICP_T_STRIDE + 16)   // column slots (double-buffered by generation parity), then
                                                 // the 8 residue-class partials, double-buffered
#define IP_NPART 8                               // residue classes of the final tree's first five steps
#define IP_LDS_PAD (56 * 1024)
#define IP_DETW (IP_WAVES - 1)                   // the wave that runs the det check off the critical path
// Column sums go to the residue-class leader (workgroup wg % 8).  Each leader publishes its XCD
// (HW_REG_XCC_ID) at launch; a workgroup that finds its leader on its own XCD publishes its
// columns with plain stores (kept in the shared L2), any other with write-through sc1 stores.
// Placement is checked, never assumed: an unknown or different XCD takes the sc1 path.
#ifndef IP_XCD_STORE
#define IP_XCD_STORE 1
#endif
#define IP_XCC_AT (IP_PART + 2 * IP_NPART * ICP_T_STRIDE)   // the leaders' XCD ids (TF_ICP_TAG_WORDS)
// Hop 2's readers are all 256 workgroups, polling 8 x 27 granules.  Each leader publishes its
// partials IP_PCOPY = 8 times, 4 KiB apart, and the workgroups of residue class x (one XCD
// under round-robin dispatch) poll copy x: 32 pollers per line instead of 256 (ICP -1.5 us per
// launch, A/B profiles/r05/ab_icp_hop2_copies.txt).
#ifndef IP_TAIL_ROWS
#define IP_TAIL_ROWS 0                           // A/B: 1 = the row-layout tail (bit-exact, slower: DESIGN 8)
#endif
#ifndef IP_OK_BITWISE
#define IP_OK_BITWISE 1                          // A/B: 0 = short-circuit correspondence flags
#endif
#ifndef IP_PCOPY
#define IP_PCOPY 8                               // A/B: 1 = one copy polled by every workgroup
#endif
#define IP_PCOPY_AT (IP_XCC_AT + 16)
#define IP_PCOPY_STRIDE 512
static_assert(IP_PCOPY_AT + 8 * IP_PCOPY_STRIDE <= TF_ICP_TAG_WORDS, "TF_ICP_TAG_WORDS");
__device__ __forceinline__ int ip_part_at(int copy)
{
    return IP_PCOPY == 1 ? IP_PART : IP_PCOPY_AT + copy * IP_PCOPY_STRIDE;
}

struct IcpFrameArgs {
    IcpLevel lv[TF_LEVELS];             // in processing order (coarse -> fine)
    int iters[TF_LEVELS];
    int slots[TF_LEVELS];
    int nlev;
    int total_iters;
    int pose_update;
    int frame_begin;                    // frame path: the launch starts the frame (tf_frame_begin)
    TfDevState* st;
    unsigned long long* tag;            // [256][28] column sums, then [16] broadcast
    // fold_t3: the frame's setToType3 + visibility test and renderImage snapshot (k_set_type3)
    // run in this grid's tail, once the pose is known (frame path)
    int fold_t3;
    VisArgs vis;
    const TfHashEntry* hash;
    const int* visibleIds;
    unsigned char* visType;
    const float2* range;
    float2* snap;
    // per-call frames (tf_process_frame): the frame's verdict -- TopFu::operator()'s return value
    // and poses_.back() -- written to host memory as soon as it is known, so the host returns
    // while the rest of the frame runs (tf_verdict_*, tf_capi.hip); nullptr: not requested
    unsigned long long* verdict;
    unsigned verdict_gen;
    int fault_iter;                     // >= 0: report a lost peer at this iteration (fault injection, tests)
};

// the verdict record: TF_VERDICT_WORDS 64-bit words, each (generation << 32 | payload), written
// with system-scope stores into fine-grained host memory; the host accepts the record once every
// word carries the generation it armed.  Word 0: mode | (ok + 1) << 4 | iterations << 8;
// words 1..12: the pose's float bits.  Bit 16 of word 0: the context is halted by an earlier
// frame (tf_reset.h) -- this frame did not run.
static __device__ void icp_verdict(const IcpFrameArgs& a, int mode, int ok, int iters, const float* pose, int halted = 0)
{
    const unsigned long long g = (unsigned long long)a.verdict_gen << 32;
    for (int i = 0; i < 12; ++i)
        __hip_atomic_store(&a.verdict[1 + i], g | __float_as_uint(pose[i]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&a.verdict[0], g | (unsigned)(mode | (ok + 1) << 4 | iters << 8 | (halted ? 1u << 16 : 0u)),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// k_set_type3's work (render_snapshot + set_type3_pass) in every workgroup of the persistent
// ICP grid after its last iteration: pose0 = poses_.back() read at launch (only workgroup 0
// writes st->pose, after every hand-off); mode 0 = frame-0 path (pose as is), else status 1 =
// ICP succeeded (pose0 * affine).  The matrices are those tf_set_pose_matrices derives,
// computed by the same operations.
__device__ void icp_fold_t3(const IcpFrameArgs& a, const float* pose0, const float* aff, int mode, int status)
{
    __shared__ float M_s[16], Mr_s[16];
    TfDevState* st = a.st;
    const bool go = mode == 0 || status == 1;              // !abort
    const int tid = blockIdx.x * blockDim.x + threadIdx.x, stride = gridDim.x * blockDim.x;
    // the thread's first previous-list entry, loaded while thread 0 derives the matrices
    const int n = go ? st->noVisibleEntries : 0;
    int id0 = -1;
    TfHashEntry e0 = {};
    if (tid < n) { id0 = a.visibleIds[tid]; e0 = a.hash[id0]; }
    if (threadIdx.x == 0) {
        float pose[12], m[12];
        for (int i = 0; i < 12; ++i) pose[i] = pose0[i];
        if (mode != 0 && status == 1) tf_rigid_mul(pose, aff, pose);
        if (mode != 0) tf_rigid_inv(pose, m);
        else for (int i = 0; i < 12; ++i) m[i] = pose[i];
        tf_rt_to_m4(m, M_s);
        tf_rt_to_m4(pose, Mr_s);
    }
    __syncthreads();
    // render_snapshot (tf_internal.h): M_render = M_ray (unchanged by a failed ICP), render_go
    if (blockIdx.x == 0 && threadIdx.x < 16) st->M_render[threadIdx.x] = go ? Mr_s[threadIdx.x] : st->M_ray[threadIdx.x];
    if (blockIdx.x == 0 && threadIdx.x == 0) st->render_go = (mode != 0 && go) ? 1 : 0;
    if (!go) return;
    if (mode != 0) {
        const int W = a.vis.W, rc = (W - 1) / TF_SUBSAMPLE + 1, rr = (a.vis.H - 1) / TF_SUBSAMPLE + 1;
        for (int i = tid; i < rc * rr; i += stride) {
            const int y = i / rc, x = i - y * rc;
            a.snap[x + y * W] = a.range[x + y * W];
        }
    }
    if (id0 >= 0) a.visType[id0] = vis_block(e0, M_s, a.vis) ? 3 : 4;
    set_type3_pass(a.vis, n, M_s, a.hash, a.visibleIds, a.visType, tid + stride, stride);
}

__device__ __forceinline__ unsigned long long ip_pack(unsigned gen, float v)
{
    return ((unsigned long long)gen << 32) | (unsigned long long)__float_as_uint(v);
}
__device__ __forceinline__ void ip_store(unsigned long long* p, unsigned long long v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ip_load(const unsigned long long* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// a granule for a reader on this workgroup's own XCD: a plain 8-byte store stays in the XCD's
// L2, where the reader's agent-scope (L1-bypassing) loads find it; an sc1 store would drop the
// line and send the reader to memory
__device__ __forceinline__ void ip_store_xcd(unsigned long long* p, unsigned long long v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ unsigned ip_xcc_id()
{
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
    return x;
}

// find_coresp (points variant) + row (proj_icp.cu:80-117, 365-377) for 4 pixels per lane, with
// the current-frame point/normal in registers and both previous-map loads issued before any of
// the dependent tests (IpPix is declared above k_icp_iter)

// kdot / kcross (tf_internal.h) on two pixels at once: the same operations per element, as
// v_pk_mul / v_pk_fma / v_pk_add (the rows are VALU-bound: two reference CTAs share a SIMD at
// level 0, one CTA's rows are ~700 instructions)
__device__ __forceinline__ ip_f2 ip_bc(float v) { return ip_f2{ v, v }; }
__device__ __forceinline__ ip_f2 kdot2(ip_f2 ax, ip_f2 ay, ip_f2 az, ip_f2 bx, ip_f2 by, ip_f2 bz)
{
    return __builtin_elementwise_fma(ax, bx, __builtin_elementwise_fma(ay, by, az * bz));
}

// a pixel pair: projection into the previous frame (find_coresp's first half)
__device__ __forceinline__ void ip_project2(const IcpLevel& L, const float* aff, ip_f2 vx, ip_f2 vy, ip_f2 vz,
                                           int xy0, int xy1, ip_f2& sx, ip_f2& sy, ip_f2& sz, bool& ok0, bool& ok1,
                                           int& idx0, int& idx1)
{
    sx = kdot2(ip_bc(aff[0]), ip_bc(aff[1]), ip_bc(aff[2]), vx, vy, vz) + ip_bc(aff[3]);
    sy = kdot2(ip_bc(aff[4]), ip_bc(aff[5]), ip_bc(aff[6]), vx, vy, vz) + ip_bc(aff[7]);
    sz = kdot2(ip_bc(aff[8]), ip_bc(aff[9]), ip_bc(aff[10]), vx, vy, vz) + ip_bc(aff[11]);
    // __fdividef(p.x, p.z) = p.x times an approximate reciprocal (proj_icp.cu:34-35): canonical
    // p.x * RN(1 / p.z), one reciprocal per pixel for both coordinates, the products packed
#if TF_PROJ_DIV                                   // A/B only: the IEEE division sequence for RN(1 / z)
    const ip_f2 rz = { 1.0f / sz.x, 1.0f / sz.y };
#else
    // (one wave-uniform branch for the pair's rare IEEE fallback, tf_internal.h)
    ip_f2 rz = { tf_rcp_fast(sz.x), tf_rcp_fast(sz.y) };
    const bool slow0 = tf_rcp_slow(sz.x), slow1 = tf_rcp_slow(sz.y);
#if TF_RCP_BRANCH
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(slow0 | slow1) != 0, 0)) {
        if (slow0) rz.x = 1.0f / sz.x;
        if (slow1) rz.y = 1.0f / sz.y;
    }
#else
    if (slow0) rz.x = 1.0f / sz.x;
    if (slow1) rz.y = 1.0f / sz.y;
#endif
#endif
    const ip_f2 qx = sx * rz, qy = sy * rz;
    const ip_f2 coox = __builtin_elementwise_fma(ip_bc(L.fx), qx, ip_bc(L.cx));
    const ip_f2 cooy = __builtin_elementwise_fma(ip_bc(L.fy), qy, ip_bc(L.cy));
#if IP_OK_BITWISE            // (bitwise, not short-circuit: no exec-mask branches)
    ok0 = (xy0 >= 0) & !isnan(vx.x) &
          !((sz.x <= 0) | (coox.x < 0) | (cooy.x < 0) | (coox.x >= (float)L.W) | (cooy.x >= (float)L.H));
    ok1 = (xy1 >= 0) & !isnan(vx.y) &
          !((sz.y <= 0) | (coox.y < 0) | (cooy.y < 0) | (coox.y >= (float)L.W) | (cooy.y >= (float)L.H));
#else
    ok0 = xy0 >= 0 && !isnan(vx.x) &&
          !(sz.x <= 0 || coox.x < 0 || cooy.x < 0 || coox.x >= (float)L.W || cooy.x >= (float)L.H);
    ok1 = xy1 >= 0 && !isnan(vx.y) &&
          !(sz.y <= 0 || coox.y < 0 || cooy.y < 0 || coox.y >= (float)L.W || cooy.y >= (float)L.H);
#endif
    idx0 = ok0 ? (int)floorf(cooy.x) * L.W + (int)floorf(coox.x) : 0;
    idx1 = ok1 ? (int)floorf(cooy.y) * L.W + (int)floorf(coox.y) : 0;
}

// a pixel pair: the correspondence tests and the row (find_coresp's second half, the
// row of proj_icp.cu:365-377), zero where a test fails
__device__ __forceinline__ void ip_row2(const IcpLevel& L, const float* aff, ip_f2 ncx, ip_f2 ncy, ip_f2 ncz,
                                       ip_f2 sx, ip_f2 sy, ip_f2 sz, bool ok0, bool ok1, float4 dp0, float4 dp1,
                                       float4 ndp0, float4 ndp1, ip_f2 (&r)[7])
{
    const ip_f2 dx = { dp0.x, dp1.x }, dy = { dp0.y, dp1.y }, dz = { dp0.z, dp1.z };
    const ip_f2 ex = sx - dx, ey = sy - dy, ez = sz - dz;              // sd = s - d
    const ip_f2 dd = kdot2(ex, ey, ez, ex, ey, ez);
    const ip_f2 nsx = kdot2(ip_bc(aff[0]), ip_bc(aff[1]), ip_bc(aff[2]), ncx, ncy, ncz);
    const ip_f2 nsy = kdot2(ip_bc(aff[4]), ip_bc(aff[5]), ip_bc(aff[6]), ncx, ncy, ncz);
    const ip_f2 nsz = kdot2(ip_bc(aff[8]), ip_bc(aff[9]), ip_bc(aff[10]), ncx, ncy, ncz);
    const ip_f2 ndx = { ndp0.x, ndp1.x }, ndy = { ndp0.y, ndp1.y }, ndz = { ndp0.z, ndp1.z };
    const ip_f2 cs = kdot2(nsx, nsy, nsz, ndx, ndy, ndz);
    // kcross(s, nd), kdot(nd, d - s)
    const ip_f2 crx = sy * ndz - sz * ndy, cry = sz * ndx - sx * ndz, crz = sx * ndy - sy * ndx;
    const ip_f2 b = kdot2(ndx, ndy, ndz, dx - sx, dy - sy, dz - sz);
    const bool g0 = ok0 && !isnan(dx.x) && !(dd.x > L.dist2) && !(fabsf(cs.x) < L.min_cosine);
    const bool g1 = ok1 && !isnan(dx.y) && !(dd.y > L.dist2) && !(fabsf(cs.y) < L.min_cosine);
    auto sel = [g0, g1](ip_f2 v) { return ip_f2{ g0 ? v.x : 0.f, g1 ? v.y : 0.f }; };
    r[0] = sel(crx); r[1] = sel(cry); r[2] = sel(crz);
    r[3] = sel(ndx); r[4] = sel(ndy); r[5] = sel(ndz); r[6] = sel(b);
}

__device__ __forceinline__ void ip_rows4(const IcpLevel& L, const float* aff, const IpPix (&px)[2],
                                         const int (&xy)[4], ip_f2 (&r01)[7], ip_f2 (&r23)[7])
{
    ip_f2 sx0, sy0, sz0, sx1, sy1, sz1;
    bool ok0, ok1, ok2, ok3;
    int i0, i1, i2, i3;
    ip_project2(L, aff, px[0].vx, px[0].vy, px[0].vz, xy[0], xy[1], sx0, sy0, sz0, ok0, ok1, i0, i1);
    ip_project2(L, aff, px[1].vx, px[1].vy, px[1].vz, xy[2], xy[3], sx1, sy1, sz1, ok2, ok3, i2, i3);
    // both previous-map gathers of all four pixels issued before any dependent test
    const float4 d0 = L.vprev[i0], d1 = L.vprev[i1], d2 = L.vprev[i2], d3 = L.vprev[i3];
    const float4 n0 = L.nprev[i0], n1 = L.nprev[i1], n2 = L.nprev[i2], n3 = L.nprev[i3];
    ip_row2(L, aff, px[0].nx, px[0].ny, px[0].nz, sx0, sy0, sz0, ok0, ok1, d0, d1, n0, n1, r01);
    ip_row2(L, aff, px[1].nx, px[1].ny, px[1].nz, sx1, sy1, sz1, ok2, ok3, d2, d3, n2, n3, r23);
}

// 256-pixel CTA reduction (partial_reduce order): lane l ends holding sum (l >> 1).  Steps 128
// and 64 in registers: (r0a r0b + r2a r2b) + (r1a r1b + r3a r3b), the first two pairs as one
// v_pk_mul each over the pixel pairs and one v_pk_add.
__device__ __forceinline__ float ip_cta_reduce(const ip_f2 (&r01)[7], const ip_f2 (&r23)[7], int lane)
{
    float v[32];
    int k = 0;
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
        for (int b = a; b < 7; ++b, ++k) {
            const ip_f2 s = r01[a] * r01[b] + r23[a] * r23[b];      // (a0, a1)
            v[k] = s.x + s.y;
        }
#pragma unroll
    for (int j = 27; j < 32; ++j) v[j] = 0.f;
    tstep<32, 32>(v, lane);
    tstep<16, 16>(v, lane);
    tstep<8, 8>(v, lane);
    tstep<4, 4>(v, lane);
    tstep<2, 2>(v, lane);
    return v[0] + xor1(v[0]);
}

__device__ __forceinline__ void ip_unpack(const float (&sm)[27], float (&Am)[6][6], float (&bv)[6])
{   // StreamHelper::get (projective_icp.cpp:51-61)
    int shift = 0;
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = i; j < 7; ++j) {
            float value = sm[shift++];
            if (j == 6) bv[i] = value;
            else { Am[j][i] = value; Am[i][j] = value; }
        }
}

// Partial tree of one residue class.  icp_final_reduce_kernel's 256-wide halving tree
// (temp_utils.hpp:503-523) pairs column t with t+128, t+64, t+32, t+16, t+8 in its first five
// steps, so after them slot x < 8 holds a sum over the 32 columns x + 8k only, in a fixed
// pairing: c[k] + c[k+16], then +8, +4, +2, +1 (k = 0..31).  Bit-identical to the full tree.
__device__ __forceinline__ float ip_residue_tree(const float* c)
{
    float b[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) b[k] = c[k] + c[k + 16];
#pragma unroll
    for (int k = 0; k < 8; ++k) b[k] = b[k] + b[k + 8];
#pragma unroll
    for (int k = 0; k < 4; ++k) b[k] = b[k] + b[k + 4];
    b[0] = b[0] + b[2];
    b[1] = b[1] + b[3];
    return b[0] + b[1];
}

// Per iteration (hierarchical gather, no broadcast): every workgroup publishes its 27 column
// sums; workgroup x < 8 gathers the 32 columns of residue class x (the workgroups dispatched
// round-robin onto its own XCD), runs the first five steps of the final tree on them
// (ip_residue_tree) and publishes 27 partials; every workgroup then gathers the 8 x 27
// partials, runs the last three tree steps and the solve / Rodrigues / compose itself,
// redundantly and bit-identically -- two small hops per iteration, no broadcast.  The det check
// of iteration k (cv::determinant, projective_icp.cpp:197-203) runs on wave IP_DETW while
// iteration k+1 computes its rows and is settled before anything of k+1 is published: on
// failure the affine of k-1 is restored and the loop ends exactly where the serial order ends
// it.  The solve (wave 0) is the only serial work between two iterations.
template <int ALG>
__global__ void __launch_bounds__(64 * IP_WAVES)
k_icp_frame(IcpFrameArgs a)
{
    __shared__ float red[ICP_MAX_SLOTS][ICP_T_STRIDE];
    __shared__ float tl[27][33];                // a residue class's 32 columns (+1 pad)
    __shared__ float tv[27][IP_NPART + 1];      // the 8 residue-class partials per sum
    __shared__ float aff_s[12];
    __shared__ int det_ok_s;
    // the det check's sums and the affine it may restore live in LDS, not in registers across the
    // iteration: the serial tail runs in the registers they would hold
    __shared__ float det_sm_s[27], aff_prev_s[12];
#if IP_TAIL_ROWS
    __shared__ double xs_s[9];                  // icp_tail_rows' exchange of S (wave 0)
#endif
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, wg = blockIdx.x;
    TfDevState* st = a.st;
    unsigned long long* tag = a.tag;
    __shared__ float pose0_s[12];
    if (a.fold_t3 && tid < 12) pose0_s[tid] = st->pose[tid];
    if (a.frame_begin) {
        // the device-driven frame starts here (TopFu::operator(), topfu.cpp:200): frame 0 of a
        // run (frame_counter == 0) takes the integrate-only path.  Workgroup 0 records the
        // frame's mode; every workgroup derives it from frame_counter, which only the previous
        // frame's end wrote (so the preprocessing stream never touches the state)
        const bool frame0 = st->frame_counter == 0;
        const bool halted = st->halt != 0;              // (only a frame end writes it: uniform)
        if (wg == 0 && tid == 0) tf_frame_begin(st);
        if (halted) {                                   // an earlier frame failed: this one is skipped
            if (a.verdict && wg == 0 && tid == 0) {
                float pose[12];
                for (int i = 0; i < 12; ++i) pose[i] = st->pose[i];
                icp_verdict(a, frame0 ? 0 : 1, -1, 0, pose, 1);
            }
            if (a.fold_t3) {                            // (the renderImage snapshot's go flag: off)
                __syncthreads();
                icp_fold_t3(a, pose0_s, nullptr, 1, 2);
            }
            return;
        }
        if (frame0) {
            if (a.verdict && wg == 0 && tid == 0) {             // return ++frame_counter_, true (topfu.cpp:209)
                float pose[12];
                for (int i = 0; i < 12; ++i) pose[i] = st->pose[i];
                icp_verdict(a, 0, 1, 0, pose);
            }
            if (a.fold_t3) {
                __syncthreads();
                icp_fold_t3(a, pose0_s, nullptr, 0, 1);
            }
            return;
        }
    } else if (st->mode == 0) {
        return;                                // frame 0 runs no ICP (uniform over the grid)
    }
    const unsigned base = st->icp_gen;
    unsigned gen = base;
#if IP_XCD_STORE
    const unsigned my_xcc = ip_xcc_id();
    if (wg < IP_NPART && tid == 0) ip_store(&tag[IP_XCC_AT + wg], ip_pack(base, __uint_as_float(my_xcc)));
    int leader_same = wg < IP_NPART ? 1 : -1;          // -1: the leader's XCD not yet known
#endif
    float aff[12];
#pragma unroll
    for (int i = 0; i < 12; ++i) aff[i] = (i % 5 == 0) ? 1.0f : 0.0f;     // affine = Identity
    int status = 1, done = 0;
    float last_sums = 0.f;

    bool det_pending = false;

#pragma unroll 1
    for (int li = 0; li < a.nlev && status == 1; ++li) {
        // uniform selects instead of a dynamic index into the kernel arguments (no scratch copy)
        const IcpLevel L = li == 0 ? a.lv[0] : (li == 1 ? a.lv[1] : a.lv[2]);
        const int slots = li == 0 ? a.slots[0] : (li == 1 ? a.slots[1] : a.slots[2]);
        IPT_REC(done, 2 * ICP_NWG + 8);                 // (timing build: the level's set-up begins)
        // current-frame maps of my CTA slots -> registers (constant over the level)
        IpPix px[IP_SREG][2];
        int xy[IP_SREG][4];
#pragma unroll
        for (int rr = 0; rr < IP_SREG; ++rr) {
            const int sl = wave + IP_WAVES * rr;
            const int cta = wg + ICP_NWG * sl;
            const bool live = sl < slots && cta < L.nct;
            const int bx = live ? cta % L.gx : 0, by = live ? cta / L.gx : 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int t = lane + 64 * j;
                const int x = bx * 32 + (t & 31), y = by * 8 + (t >> 5);
                const bool in = live && x < L.W && y < L.H;
                xy[rr][j] = in ? 1 : -1;
                // unconditional loads (pixel 0 when outside): a load under a per-lane condition
                // is a branch, and the eight of a level start would be eight round trips
                const int pi = in ? y * L.W + x : 0;
                float4 v = L.vcurr[pi], n = L.ncurr[pi];
                if (!in) { v = make_float4(0.f, 0.f, 0.f, 0.f); n = v; }
                ip_set(px[rr], j, v, n);
            }
        }
        IPT_REC_DEP(done, 2 * ICP_NWG + 9, px[0][0].vx.x + px[0][1].nz.y);   // (its maps arrived)
        const int iters = li == 0 ? a.iters[0] : (li == 1 ? a.iters[1] : a.iters[2]);
#pragma unroll 1
        for (int it = 0; it < iters; ++it) {
            ++gen;
            IPT_REC(done, wg);
            IPT_CLK(done);
            if (det_pending && wave == IP_DETW) {
                float Am[6][6], bv[6], det_sm[27];
#pragma unroll
                for (int q = 0; q < 27; ++q) det_sm[q] = det_sm_s[q];
                ip_unpack(det_sm, Am, bv);
                const double det = icp_det6<ALG>(Am);
                if (lane == 0) det_ok_s = !(fabs(det) < 1e-15 || isnan(det));
                IPT_REC_T(done - 1, 2 * ICP_NWG + 5, 64 * IP_DETW);
            }
            // ---- per-CTA reductions -> column sum of this workgroup -> tagged slot
#pragma unroll
            for (int rr = 0; rr < IP_SREG; ++rr) {
                const int sl = wave + IP_WAVES * rr;
                if (sl < slots && wg + ICP_NWG * sl < L.nct) {
                    ip_f2 r01[7], r23[7];
                    ip_rows4(L, aff, px[rr], xy[rr], r01, r23);
                    const float tot = ip_cta_reduce(r01, r23, lane);
                    if (!(lane & 1) && (lane >> 1) < 27) red[sl][lane >> 1] = tot;
                }
            }
            // slots beyond the register-resident ones (large images): current maps re-read
#pragma unroll 1
            for (int sl = wave + IP_WAVES * IP_SREG; sl < slots; sl += IP_WAVES) {
                const int cta = wg + ICP_NWG * sl;
                if (cta >= L.nct) break;
                IpPix q[2];
                int qxy[4];
                const int bx = cta % L.gx, by = cta / L.gx;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int t = lane + 64 * j;
                    const int x = bx * 32 + (t & 31), y = by * 8 + (t >> 5);
                    const bool in = x < L.W && y < L.H;
                    qxy[j] = in ? 1 : -1;
                    const int pi = in ? y * L.W + x : 0;                 // unconditional loads
                    float4 v = L.vcurr[pi], n = L.ncurr[pi];
                    if (!in) { v = make_float4(0.f, 0.f, 0.f, 0.f); n = v; }
                    ip_set(q, j, v, n);
                }
                ip_f2 r01[7], r23[7];
                ip_rows4(L, aff, q, qxy, r01, r23);
                const float tot = ip_cta_reduce(r01, r23, lane);
                if (!(lane & 1) && (lane >> 1) < 27) red[sl][lane >> 1] = tot;
            }
            __syncthreads();
            if (det_pending) {                                    // settle iteration k's det check
                det_pending = false;
                if (!det_ok_s) {
                    status = 0;
#pragma unroll
                    for (int i = 0; i < 12; ++i) aff[i] = aff_prev_s[i];
                    break;
                }
            }
            if (tid < 27) {
                float sum = 0.f;                                   // 0 + P[w] + P[w+256] + ...
                for (int sl = 0; sl < slots; ++sl) {
                    if (wg + ICP_NWG * sl >= L.nct) break;
                    sum += red[sl][tid];
                }
#if IP_XCD_STORE
                if (leader_same < 0) {
                    const unsigned long long x = ip_load(&tag[IP_XCC_AT + (wg & (IP_NPART - 1))]);
                    if ((unsigned)(x >> 32) == base) leader_same = __float_as_uint(__uint_as_float((unsigned)x)) == my_xcc ? 1 : 0;
                }
                if (leader_same > 0)
                    ip_store_xcd(&tag[(gen & 1) * ICP_NWG * ICP_T_STRIDE + wg * ICP_T_STRIDE + tid], ip_pack(gen, sum));
                else
#endif
                ip_store(&tag[(gen & 1) * ICP_NWG * ICP_T_STRIDE + wg * ICP_T_STRIDE + tid], ip_pack(gen, sum));
            }
            IPT_REC(done, ICP_NWG + wg);
            if (wg < IP_NPART) {
                // ---- residue-class leader: gather columns wg + 8k, partial tree, publish
                constexpr int PER = (32 * 27 + 64 * IP_WAVES - 1) / (64 * IP_WAVES);
                const unsigned long long* cols = &tag[(gen & 1) * ICP_NWG * ICP_T_STRIDE];
                unsigned long long v[PER];
#pragma unroll
                for (int k = 0; k < PER; ++k) {
                    const int e = tid + 64 * IP_WAVES * k;
                    const int kk = e / 27, q = e - kk * 27;
                    v[k] = e < 32 * 27 ? ip_load(&cols[(wg + IP_NPART * kk) * ICP_T_STRIDE + q]) : ((unsigned long long)gen << 32);
                }
                bool timeout = false;
                for (unsigned spins = 0;; ++spins) {
                    bool ready = true;
#pragma unroll
                    for (int k = 0; k < PER; ++k) {
                        if ((unsigned)(v[k] >> 32) != gen) {
                            ready = false;
                            const int e = tid + 64 * IP_WAVES * k;
                            const int kk = e / 27, q = e - kk * 27;
                            v[k] = ip_load(&cols[(wg + IP_NPART * kk) * ICP_T_STRIDE + q]);
                        }
                    }
                    if (ready) break;
                    if (spins > IP_SPIN_LIMIT) { timeout = true; break; }
                    __builtin_amdgcn_s_sleep(IP_SLEEP);
                }
#pragma unroll
                for (int k = 0; k < PER; ++k) {
                    const int e = tid + 64 * IP_WAVES * k;
                    const int kk = e / 27, q = e - kk * 27;
                    if (e < 32 * 27) tl[q][kk] = __uint_as_float((unsigned)v[k]);
                }
                const int lead_timeout = __syncthreads_or(timeout);
                if (!lead_timeout && tid < 27) {        // a missing column: publish nothing, WG0 times out
                    const unsigned long long pv = ip_pack(gen, ip_residue_tree(tl[tid]));
#pragma unroll
                    for (int c = 0; c < IP_PCOPY; ++c)
                        ip_store(&tag[ip_part_at(c) + (gen & 1) * IP_NPART * ICP_T_STRIDE + wg * ICP_T_STRIDE + tid], pv);
                }
            }
            {
                // ---- gather the 8 x 27 partials, last three tree steps, det / solve / compose
                // (every workgroup, redundantly and bit-identically -- no broadcast hop)
                const unsigned long long* parts = &tag[ip_part_at(wg & (IP_PCOPY - 1)) + (gen & 1) * IP_NPART * ICP_T_STRIDE];
                bool timeout = false;
                if (tid < IP_NPART * 27) {
                    const int x = tid / 27, q = tid - x * 27;
                    const unsigned long long* pp = &parts[x * ICP_T_STRIDE + q];
                    unsigned long long v = ip_load(pp);
                    for (unsigned spins = 0; (unsigned)(v >> 32) != gen; ++spins) {
                        if (spins > IP_SPIN_LIMIT) { timeout = true; break; }
                        __builtin_amdgcn_s_sleep(IP_SLEEP);
                        v = ip_load(pp);
                    }
                    tv[q][x] = __uint_as_float((unsigned)v);
                }
                const int any_timeout = __syncthreads_or(timeout || done == a.fault_iter);
                IPT_REC(done, 2 * ICP_NWG + 0);
                if (!any_timeout && (wave == 0 || wave == IP_DETW)) {
                    // steps 4, 2, 1: ((P0+P4) + (P2+P6)) + ((P1+P5) + (P3+P7)); lane q holds sum q
                    float tot = 0.f;
                    if (lane < 27) {
                        const float* P = tv[lane];
                        tot = ((P[0] + P[4]) + (P[2] + P[6])) + ((P[1] + P[5]) + (P[3] + P[7]));
                    }
                    float sm[27], Am[6][6], bv[6];
#pragma unroll
                    for (int q = 0; q < 27; ++q)
                        sm[q] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, tot), q));
                    IPT_REC_DEP(done, 2 * ICP_NWG + 6, sm[26] + sm[0]);
                    ip_unpack(sm, Am, bv);
                    IPT_REC(done, 2 * ICP_NWG + 2);
                    if (wave == IP_DETW) {                             // det after the barrier
                        if (lane < 27) det_sm_s[lane] = tot;
                    } else {                                           // solve -> Rodrigues -> compose
#if IP_TAIL_ROWS
                      if constexpr (ALG == 0) {                          // row layout (tf_icp_tail.h)
                        float orow[4], rvr[6];
                        icp_tail_rows(sm, aff, lane, xs_s, orow, rvr);
                        IPT_REC_DEP(done, 2 * ICP_NWG + 7, orow[0] + orow[3]);
                        if (lane < 3) {
#pragma unroll
                            for (int c = 0; c < 4; ++c) aff_s[4 * lane + c] = orow[c];
                        }
                        IPT_REC_DEP(done, 2 * ICP_NWG + 4, orow[1]);
                        last_sums = tot;
                      } else
#endif
                      {
                        float rv[6], R[9], tinc[12];
#ifdef TF_ICP_TIMING
                        if constexpr (ALG == 0) {                       // the two halves stamped apart
                            // each half run twice back to back on the shader clock: the second
                            // run finds its code in the instruction cache (g_icp_tail_cyc)
                            const long long c0 = IPT_CYC(0.f);
                            icp_solve6_schur(Am, bv, rv);
                            const long long c1 = IPT_CYC(rv[0] + rv[5]);
                            float bv2[6], rv2[6], R2[9];
#pragma unroll
                            for (int i = 0; i < 6; ++i) bv2[i] = bv[i] + rv[i] * 0.0f;
                            icp_solve6_schur(Am, bv2, rv2);
                            const long long c2 = IPT_CYC(rv2[0] + rv2[5]);
                            IPT_REC_DEP(done, 2 * ICP_NWG + 3, rv[0] + rv[5] + rv2[1] * 0.0f);
                            const long long c3 = IPT_CYC(0.f);
                            icp_rodrigues(rv, R);
                            const long long c4 = IPT_CYC(R[0] + R[8]);
                            float rvb[6];
#pragma unroll
                            for (int i = 0; i < 6; ++i) rvb[i] = rv[i] + R[i] * 0.0f;
                            icp_rodrigues(rvb, R2);
                            const long long c5 = IPT_CYC(R2[0] + R2[8]);
                            if (blockIdx.x == 0 && lane == 0 && done < 64) {
                                g_icp_tail_cyc[4 * done + 0] = c1 - c0; g_icp_tail_cyc[4 * done + 1] = c2 - c1;
                                g_icp_tail_cyc[4 * done + 2] = c4 - c3; g_icp_tail_cyc[4 * done + 3] = c5 - c4;
                            }
                            R[0] = R[0] + R2[0] * 0.0f;
                        } else
#endif
                        if constexpr (ALG != 0 && IP_SVD_LANES) {       // projective_icp.cpp:206-209
                            icp_cv_solve_svd6_lanes<ALG>(tot, 1, lane, rv);
                            icp_cv_rodrigues<ALG>(rv, R);
                        } else {
                            icp_solve_rodrigues<ALG>(Am, bv, rv, R);
                        }
                        IPT_REC_DEP(done, 2 * ICP_NWG + 7, R[0] + R[8]);
#pragma unroll
                        for (int j = 0; j < 3; ++j) {
                            tinc[j * 4 + 0] = R[j * 3 + 0]; tinc[j * 4 + 1] = R[j * 3 + 1];
                            tinc[j * 4 + 2] = R[j * 3 + 2]; tinc[j * 4 + 3] = rv[3 + j];
                        }
                        float A[12];
#pragma unroll
                        for (int i = 0; i < 12; ++i) A[i] = aff[i];
                        tf_rigid_mul(tinc, A, A);
                        if (lane < 12) aff_s[lane] = A[lane];
                        IPT_REC_DEP(done, 2 * ICP_NWG + 4, A[0] + A[11]);
                        last_sums = tot;
                      }
                    }
                }
                __syncthreads();
                IPT_REC(done, 2 * ICP_NWG + 1);
                status = any_timeout ? 2 : 1;
                det_pending = !any_timeout;
                if (wave == 0 && lane == 0) {
#pragma unroll
                    for (int i = 0; i < 12; ++i) aff_prev_s[i] = aff[i];
                }
                if (status == 1) {
#pragma unroll
                    for (int i = 0; i < 12; ++i) aff[i] = aff_s[i];
                }
            }
            ++done;
            if (status != 1) break;
            __syncthreads();                       // red[] / aff_s reuse in the next iteration
        }
    }
    if (det_pending) {                                            // the last iteration's det check
        if (wave == IP_DETW) {
            float Am[6][6], bv[6], det_sm[27];
#pragma unroll
            for (int q = 0; q < 27; ++q) det_sm[q] = det_sm_s[q];
            ip_unpack(det_sm, Am, bv);
            const double det = icp_det6<ALG>(Am);
            if (lane == 0) det_ok_s = !(fabs(det) < 1e-15 || isnan(det));
        }
        __syncthreads();
        if (!det_ok_s) {
            status = 0;
#pragma unroll
            for (int i = 0; i < 12; ++i) aff[i] = aff_prev_s[i];
        }
    }
    // ---- workgroup 0 records the frame's ICP result
    if (wg == 0 && wave == 0) {
        if (lane < 27 && done > 0 && status != 2) st->sums[lane] = last_sums;
        if (lane == 0) {
            st->icp_gen = base + (unsigned)a.total_iters;   // every generation this launch could use
            st->icp_iters = done;
            st->icp_ok = status == 1 ? 1 : (status == 0 ? 0 : -1);
            st->abort = status == 1 ? 0 : 1;
            for (int i = 0; i < 12; ++i) st->affine[i] = aff[i];
            if (status == 1 && a.pose_update) {
                // poses_.push_back(poses_.back() * affine) (topfu.cpp:243) and the derived matrices
                float pose[12];
                for (int i = 0; i < 12; ++i) pose[i] = st->pose[i];
                tf_rigid_mul(pose, aff, pose);
                for (int i = 0; i < 12; ++i) st->pose[i] = pose[i];
                tf_set_pose_matrices(st, pose, 1);
                if (a.verdict) icp_verdict(a, 1, 1, done, pose);
            } else if (a.verdict) {
                // failure: the frame end resets the pose history to [I] (topfu.cpp:263-264, reset())
                float pose[12];
                for (int i = 0; i < 12; ++i) pose[i] = (i % 5 == 0) ? 1.0f : 0.0f;
                icp_verdict(a, 1, status == 1 ? 1 : (status == 0 ? 0 : -1), done, pose);
            }
        }
    }
    if (a.fold_t3) {
        __syncthreads();
        icp_fold_t3(a, pose0_s, aff, 1, status);
    }
}

__global__ void k_icp_begin(TfDevState* st, int frame_begin)
{
    if (frame_begin) tf_frame_begin(st);       // frame path: the frame starts here
    if (st->mode == 0) return;                 // frame 0 runs no ICP
    for (int i = 0; i < 12; ++i) st->affine[i] = (i % 5 == 0) ? 1.0f : 0.0f;   // affine = Identity
    st->icp_ok = 1;
    st->icp_iters = 0;
    st->abort = st->halt ? 1 : 0;              // a halted batch: the iterations no-op
}

// explicit pose (stage entry points / frame 0): pose_in -> matrices
__global__ void k_pose_from_input(TfDevState* st, int mode)
{
    float pose[12];
    for (int i = 0; i < 12; ++i) pose[i] = st->pose_in[i];
    int alloc_mode = (mode & TF_POSE_ALLOC) ? 1 : ((mode & TF_POSE_ALLOC_NOINV) ? 2 : 0);
    tf_set_pose_matrices(st, pose, alloc_mode);
}

__global__ void k_frame0_matrices(TfDevState* st)
{
    if (st->mode != 0) return;
    st->icp_ok = 1;       // frame 0 runs no ICP
    st->icp_iters = 0;
    float pose[12];
    for (int i = 0; i < 12; ++i) pose[i] = st->pose[i];
    tf_set_pose_matrices(st, pose, 2);
}

hipError_t tfk_pose_from_input(tf_ctx* c, int mode)
{
    hipLaunchKernelGGL(k_pose_from_input, dim3(1), dim3(1), 0, c->stream, c->st, mode);
    return hipGetLastError();
}

hipError_t tfk_frame0_matrices(tf_ctx* c)
{
    hipLaunchKernelGGL(k_frame0_matrices, dim3(1), dim3(1), 0, c->stream, c->st);
    return hipGetLastError();
}

// estimateTransform (projective_icp.cpp:169-213): levels coarse -> fine.
// Persistent path: one k_icp_frame launch; fallback: one k_icp_iter launch per iteration.
static void icp_level(tf_ctx* c, int l, IcpLevel& L)
{
    const tf_params& p = c->p;
    const int div = 1 << l;                                               // setLevelIntr
    L.vcurr = c->curr_pts[l]; L.ncurr = c->curr_nrm[l]; L.vprev = c->prev_pts[l]; L.nprev = c->prev_nrm[l];
    L.W = c->lw[l]; L.H = c->lh[l];
    L.gx = (L.W + 31) / 32;
    L.nct = L.gx * ((L.H + 7) / 8);
    L.fx = p.fx / (float)div; L.fy = p.fy / (float)div; L.cx = p.cx / (float)div; L.cy = p.cy / (float)div;
    L.min_cosine = c->min_cosine; L.dist2 = c->dist2_thres;
}

static int icp_used_levels(const tf_params& p)
{
    int levels = 4;
    while (levels > 0 && p.icp_iter_num[levels - 1] == 0) --levels;      // getUsedLevelsNum
    return levels > TF_LEVELS ? TF_LEVELS : levels;
}

// can every workgroup of k_icp_frame be resident at once, and do the levels fit its slots?
int tfk_icp_persistent_ok(tf_ctx* c)
{
    int per_cu = 0, cus = 0;
    const hipError_t oe = c->pose_alg == 0
        ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_icp_frame<0>, 64 * IP_WAVES, IP_LDS_PAD)
        : c->pose_alg == 2 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_icp_frame<2>, 64 * IP_WAVES, IP_LDS_PAD)
                           : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_icp_frame<4>, 64 * IP_WAVES, IP_LDS_PAD);
    if (oe != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess) return 0;
    if (per_cu * cus < ICP_NWG) return 0;
    for (int l = 0; l < TF_LEVELS; ++l) {
        IcpLevel L;
        icp_level(c, l, L);
        if ((L.nct + ICP_NWG - 1) / ICP_NWG > ICP_MAX_SLOTS) return 0;
    }
    return 1;
}

hipError_t tfk_icp(tf_ctx* c, int pose_update, int frame_begin, int fold_t3)
{
    const tf_params& p = c->p;
    const int levels = icp_used_levels(p);
    if (c->icp_persistent) {
        IcpFrameArgs a;
        memset(&a, 0, sizeof(a));
        for (int l = levels - 1; l >= 0; --l) {
            if (p.icp_iter_num[l] <= 0) continue;
            IcpLevel& L = a.lv[a.nlev];
            icp_level(c, l, L);
            a.iters[a.nlev] = p.icp_iter_num[l];
            a.slots[a.nlev] = (L.nct + ICP_NWG - 1) / ICP_NWG;
            a.total_iters += p.icp_iter_num[l];
            a.nlev++;
        }
        a.pose_update = pose_update;
        a.frame_begin = frame_begin;
        a.st = c->st;
        a.tag = c->icp_tagged;
        if (fold_t3 && pose_update && frame_begin) {
            a.fold_t3 = 1;
            a.vis.fx = c->p.fx; a.vis.fy = c->p.fy; a.vis.cx = c->p.cx; a.vis.cy = c->p.cy;
            a.vis.factor = (float)TF_BLK * c->p.voxelSize;
            a.vis.W = c->W; a.vis.H = c->H; a.vis.n_total = c->n_total; a.vis.cap = c->p.vis_capacity;
            a.vis.enlarged = c->p.use_swapping ? 1 : 0;
            a.hash = c->hash; a.visibleIds = c->visibleIds; a.visType = c->visType;
            a.range = (const float2*)c->range; a.snap = (float2*)c->range_render;
        }
        if (c->verdict_arm && pose_update && frame_begin) {     // tf_process_frame's early return
            a.verdict = c->verdict_dev;
            a.verdict_gen = c->verdict_gen;
        }
        a.fault_iter = ++c->icp_launches == c->icp_fault_launch ? c->icp_fault_iter : -1;
        // IP_LDS_PAD bytes of dynamic LDS (unused) take the workgroup above 80 KiB: at most one
        // workgroup per CU, so the 256 workgroups spread over all CUs instead of doubling up
        hipError_t e = tf_icp_order_before(c);
        if (e == hipSuccess) {
            if (c->pose_alg == 0) tf_launch(c, k_icp_frame<0>, dim3(ICP_NWG), dim3(64 * IP_WAVES), IP_LDS_PAD, a);
            else if (c->pose_alg == 2) tf_launch(c, k_icp_frame<2>, dim3(ICP_NWG), dim3(64 * IP_WAVES), IP_LDS_PAD, a);
            else tf_launch(c, k_icp_frame<4>, dim3(ICP_NWG), dim3(64 * IP_WAVES), IP_LDS_PAD, a);
            e = hipGetLastError();
        }
        const hipError_t e2 = tf_icp_order_after(c);     // (always: releases the ordering lock)
        return e != hipSuccess ? e : e2;
    }
    hipLaunchKernelGGL(k_icp_begin, dim3(1), dim3(1), 0, c->stream, c->st, frame_begin);
    int last_l = -1;
    for (int l = 0; l < levels; ++l) if (p.icp_iter_num[l] > 0) { last_l = l; break; }
    for (int l = levels - 1; l >= 0; --l) {
        IcpLevel L;
        icp_level(c, l, L);
        const int nwg = L.nct < ICP_NWG ? L.nct : ICP_NWG;
        const int slots = (L.nct + ICP_NWG - 1) / ICP_NWG;
        if (slots > ICP_MAX_SLOTS) return hipErrorInvalidValue;
        for (int it = 0; it < p.icp_iter_num[l]; ++it) {
            int last = (pose_update && l == last_l && it == p.icp_iter_num[l] - 1) ? 1 : 0;
            auto kern = c->pose_alg == 0 ? k_icp_iter<0> : (c->pose_alg == 2 ? k_icp_iter<2> : k_icp_iter<4>);
            hipLaunchKernelGGL(kern, dim3(nwg), dim3(64 * ICP_WAVES), 0, c->stream, L, c->st, c->icp_partial,
                               c->icp_ticket, nwg, slots, last);
        }
    }
    return hipGetLastError();
}

// ---- the iteration's algebra on caller systems (tf_icp_solve_systems): one wave per system,
// the forms k_icp_frame runs (canonical: LU determinant + block Schur solve; OpenCV: Matx_DetOp +
// the lane-parallel cv::solve(DECOMP_SVD))
template <int ALG>
__global__ void __launch_bounds__(64) k_solve_systems(const float* __restrict__ sums, int n, float* __restrict__ x,
                                                      double* __restrict__ det)
{
    const int lane = threadIdx.x;
    for (int q = blockIdx.x; q < n; q += gridDim.x) {
        float sm[27], Am[6][6], bv[6], xs[6];
#pragma unroll
        for (int i = 0; i < 27; ++i) sm[i] = sums[27 * (size_t)q + i];
        ip_unpack(sm, Am, bv);
        const double d = icp_det6<ALG>(Am);
        if constexpr (ALG != 0 && IP_SVD_LANES) {
            const float tot = lane < 27 ? sums[27 * (size_t)q + lane] : 0.f;
            icp_cv_solve_svd6_lanes<ALG>(tot, 1, lane, xs);
        } else if constexpr (ALG != 0) {
            icp_cv_solve_svd6<ALG>(Am, bv, xs);
        } else {
            icp_solve6_schur(Am, bv, xs);
        }
        if (lane < 6) x[6 * (size_t)q + lane] = xs[lane];
        if (lane == 0 && det) det[q] = d;
    }
}

extern "C" tf_status tf_icp_solve_systems(int algebra, const float* dev_sums, int n, float* dev_x, double* dev_det,
                                          void* stream)
{
    if (n < 0 || (n > 0 && (!dev_sums || !dev_x))) return TF_INVALID_ARG;
    if (algebra != TF_POSE_ALGEBRA_CANONICAL && algebra != TF_POSE_ALGEBRA_OPENCV2 && algebra != TF_POSE_ALGEBRA_OPENCV4)
        return TF_INVALID_ARG;
    if (n == 0) return TF_OK;
    const hipStream_t s = (hipStream_t)stream;
    const dim3 grid(n < 4096 ? n : 4096);
    if (algebra == 0) hipLaunchKernelGGL(k_solve_systems<0>, grid, dim3(64), 0, s, dev_sums, n, dev_x, dev_det);
    else if (algebra == 2) hipLaunchKernelGGL(k_solve_systems<2>, grid, dim3(64), 0, s, dev_sums, n, dev_x, dev_det);
    else hipLaunchKernelGGL(k_solve_systems<4>, grid, dim3(64), 0, s, dev_sums, n, dev_x, dev_det);
    return hipGetLastError() == hipSuccess ? TF_OK : TF_HIP_ERROR;
}
