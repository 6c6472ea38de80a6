// Stress test of the persistent ICP's same-XCD hand-off (micro-benchmark, not product).
//
// k_icp_frame (topfusion_amd/csrc/tf_icp.hip) publishes a workgroup's 27 column sums to its
// residue-class leader (workgroup wg % 8) as tagged 8-byte granules (generation << 32 | float
// bits).  When the leader's HW_REG_XCC_ID equals the producer's, the producer uses a plain
// (workgroup-scope) store, which stays in the XCD's shared L2; the leader polls with agent-scope
// (sc1, L1-bypassing) loads.  That is not one of MI355X_MICROARCH.md's validated forms, so this
// kernel runs the same pattern -- same grid (256 workgroups x 512 threads, one per CU), same
// granules, same placement check, same polling -- for many rounds under UNEVEN load (every
// workgroup sleeps a pseudo-random 0-4 us before publishing), with the leaders' lines kept
// L1/L2-warm by the previous rounds, and checks EVERY granule the leaders accept:
//   * payload: a granule carrying the round's tag must carry that round's value (a torn or stale
//     granule would show here);
//   * liveness and latency: each producer also publishes its publish time; the leader takes the
//     time from that to its first sight of the granule, for the producers that published after it
//     began polling (a plain store that never reached the shared L2 would run into the spin limit);
//   * placement: how many producer publishes took the plain-store path.
// Then the leaders publish the round's end with sc1 stores and every workgroup waits for all
// eight (the ICP's second hop), so rounds never overlap.  A second mode (argv[1] == "sc1") uses sc1
// stores for every publish: the validated form, for the latency comparison.
//   hipcc -O3 --offload-arch=gfx950 tools/micro/xcd_handoff.hip -o tools/micro/xcd_handoff
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>
#include <algorithm>

#define NWG 256
#define NPART 8
#define STRIDE 28
#define SPIN_LIMIT (1u << 22)
#define TAGS (2 * NWG * STRIDE + 2 * NPART * STRIDE + 16)
#define XCC_AT (2 * NWG * STRIDE + 2 * NPART * STRIDE)

__device__ __forceinline__ unsigned long long pack(unsigned g, float v)
{
    return ((unsigned long long)g << 32) | __float_as_uint(v);
}
__device__ __forceinline__ void st_agent(unsigned long long* p, unsigned long long v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_xcd(unsigned long long* p, unsigned long long v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ unsigned long long ld_agent(const unsigned long long* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned xcc_id()
{
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
    return x;
}
// the value producer `wg` publishes for sum q in round r (exact in float)
__device__ __forceinline__ float val(int wg, unsigned r, int q) { return (float)((wg * 131 + q * 7 + (int)(r & 0xfff)) & 0xffff); }

struct Stats {
    unsigned long long checked, bad, timeouts, plain_pub, sc1_pub;
    unsigned long long poll_cycles_sum, poll_cycles_max;   // per leader and round: the slowest producer's hand-off
                                                           // (publish -> first sight by the leader), 100 MHz ticks
    unsigned hist[64];                                     // ... in 0.1 us bins (last bin: >= 6.3 us)
};

__global__ void __launch_bounds__(512) k_handoff(unsigned long long* tag, Stats* st, unsigned base, int rounds, int mode_sc1)
{
    const int tid = threadIdx.x, wg = blockIdx.x;
    __shared__ int leader_same_s, bad_s, tmo_s;
    const unsigned my_xcc = xcc_id();
    if (wg < NPART && tid == 0) st_agent(&tag[XCC_AT + wg], pack(base, __uint_as_float(my_xcc)));
    if (tid == 0) { leader_same_s = -1; bad_s = 0; tmo_s = 0; }
    __syncthreads();
    unsigned long long plain = 0, sc1 = 0, checked = 0, psum = 0, pmax = 0;
    for (int r = 0; r < rounds; ++r) {
        const unsigned gen = base + 1 + (unsigned)r;
        // uneven load: 0..4 us of sleep, pseudo-random per workgroup and round
        unsigned h = (unsigned)wg * 2654435761u ^ (gen * 40503u);
        h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
        const unsigned long long t_sleep = __builtin_amdgcn_s_memrealtime() + (h % 400);
        while (__builtin_amdgcn_s_memrealtime() < t_sleep) __builtin_amdgcn_s_sleep(2);
        if (tid < 28) {
            if (leader_same_s < 0 && !mode_sc1) {
                const unsigned long long x = ld_agent(&tag[XCC_AT + (wg & (NPART - 1))]);
                if ((unsigned)(x >> 32) == base) leader_same_s = (unsigned)x == my_xcc ? 1 : 0;
            }
            // granules 0..26: the sums; granule 27: the publish time (100 MHz clock, low 32 bits)
            const float f = tid < 27 ? val(wg, gen, tid) : __uint_as_float((unsigned)__builtin_amdgcn_s_memrealtime());
            unsigned long long* p = &tag[(gen & 1) * NWG * STRIDE + wg * STRIDE + tid];
            if (leader_same_s > 0) { st_xcd(p, pack(gen, f)); if (tid == 0) ++plain; }
            else { st_agent(p, pack(gen, f)); if (tid == 0) ++sc1; }
        }
        if (wg < NPART) {
            // leader: gather the 32 producers' 28 granules (2 per thread), check every sum, and
            // time each producer's hand-off (first sight of its time granule - its publish time)
            const unsigned long long* cols = &tag[(gen & 1) * NWG * STRIDE];
            __shared__ unsigned lat_max_s;
            if (tid == 0) lat_max_s = 0;
            unsigned long long v[2];
            bool ok[2];
            for (int k = 0; k < 2; ++k) {
                const int e = tid + 512 * k;
                const int kk = e / STRIDE, q = e - kk * STRIDE;
                ok[k] = e >= 32 * STRIDE;
                v[k] = ok[k] ? 0 : ld_agent(&cols[(wg + NPART * kk) * STRIDE + q]);
            }
            __syncthreads();
            const unsigned t0 = (unsigned)__builtin_amdgcn_s_memrealtime();   // poll start
            bool tmo = false;
            unsigned lat = 0;
            for (unsigned spins = 0;; ++spins) {
                bool ready = true;
                for (int k = 0; k < 2; ++k) {
                    const int e = tid + 512 * k;
                    if (e >= 32 * STRIDE) continue;
                    const int kk = e / STRIDE, q = e - kk * STRIDE;
                    if ((unsigned)(v[k] >> 32) == gen) {
                        if (!ok[k]) {
                            ok[k] = true;
                            if (q < 27) {
                                ++checked;
                                if (__uint_as_float((unsigned)v[k]) != val(wg + NPART * kk, gen, q)) atomicAdd(&bad_s, 1);
                            } else {
                                // observable only when the producer published after the poll began
                                const unsigned pub = (unsigned)v[k];
                                const unsigned d = (unsigned)__builtin_amdgcn_s_memrealtime() - pub;
                                if ((int)(pub - t0) >= 0) lat = d > lat ? d : lat;
                            }
                        }
                    } else {
                        ready = false;
                        v[k] = ld_agent(&cols[(wg + NPART * kk) * STRIDE + q]);
                    }
                }
                if (ready) break;
                if (spins > SPIN_LIMIT) { tmo = true; break; }
                __builtin_amdgcn_s_sleep(1);
            }
            if (tmo) atomicAdd(&tmo_s, 1);
            if (lat) atomicMax(&lat_max_s, lat);
            __syncthreads();
            const unsigned long long dt = lat_max_s;     // the round's slowest hand-off to this leader
            if (tid == 0) {
                psum += dt; pmax = dt > pmax ? dt : pmax;
                atomicAdd(&st->hist[dt / 10 >= 63 ? 63 : dt / 10], 1u);
            }
            if (tid == 0) st_agent(&tag[2 * NWG * STRIDE + (gen & 1) * NPART * STRIDE + wg], pack(gen, 1.0f));
        }
        // the second hop: every workgroup waits for the eight leaders' end of round
        if (tid < NPART) {
            const unsigned long long* p = &tag[2 * NWG * STRIDE + (gen & 1) * NPART * STRIDE + tid];
            unsigned long long x = ld_agent(p);
            for (unsigned spins = 0; (unsigned)(x >> 32) != gen; ++spins) {
                if (spins > SPIN_LIMIT) { atomicAdd(&tmo_s, 1); break; }
                __builtin_amdgcn_s_sleep(1);
                x = ld_agent(p);
            }
        }
        __syncthreads();
    }
    if (tid == 0) {
        atomicAdd(&st->plain_pub, plain); atomicAdd(&st->sc1_pub, sc1);
        atomicAdd(&st->bad, (unsigned long long)bad_s); atomicAdd(&st->timeouts, (unsigned long long)tmo_s);
        atomicAdd(&st->poll_cycles_sum, psum);
        atomicMax(&st->poll_cycles_max, pmax);
    }
    if (wg < NPART) {
        __shared__ unsigned long long cs;
        if (tid == 0) cs = 0;
        __syncthreads();
        atomicAdd(&cs, checked);
        __syncthreads();
        if (tid == 0) atomicAdd(&st->checked, cs);
    }
}

int main(int argc, char** argv)
{
    const int sc1 = argc > 1 && !strcmp(argv[1], "sc1");
    const int launches = argc > 2 ? atoi(argv[2]) : 20, rounds = 2000;
    unsigned long long* tag;
    Stats* st;
    if (hipMalloc(&tag, sizeof(unsigned long long) * TAGS) != hipSuccess) return 1;
    if (hipMalloc(&st, sizeof(Stats)) != hipSuccess) return 1;
    hipMemset(tag, 0, sizeof(unsigned long long) * TAGS);
    hipMemset(st, 0, sizeof(Stats));
    unsigned base = 1000;
    for (int l = 0; l < launches; ++l) {
        hipLaunchKernelGGL(k_handoff, dim3(NWG), dim3(512), 56 * 1024, 0, tag, st, base, rounds, sc1);
        if (hipDeviceSynchronize() != hipSuccess) { printf("{\"error\": \"launch %d failed\"}\n", l); return 1; }
        base += rounds + 8;
    }
    Stats h;
    hipMemcpy(&h, st, sizeof(Stats), hipMemcpyDeviceToHost);
    const unsigned long long nleader = (unsigned long long)launches * rounds * NPART;
    // percentiles of the per-round slowest hand-off (0.1 us bins)
    std::vector<unsigned> hist(h.hist, h.hist + 64);
    auto pct = [&](double f) {
        unsigned long long acc = 0, tot = 0;
        for (unsigned x : hist) tot += x;
        for (int i = 0; i < 64; ++i) { acc += hist[i]; if (acc >= f * tot) return (i + 1) * 0.1; }
        return 6.4;
    };
    printf("{\"mode\": \"%s\", \"launches\": %d, \"rounds_per_launch\": %d, \"granules_checked\": %llu, "
           "\"payload_mismatches\": %llu, \"timeouts\": %llu, \"publishes_plain\": %llu, \"publishes_sc1\": %llu, "
           "\"handoff_us_mean\": %.3f, \"handoff_us_max\": %.3f, \"handoff_us_p50\": %.2f, "
           "\"handoff_us_p99\": %.2f, \"handoff_is\": \"per leader and round, the slowest of its 32 producers: publish "
           "-> first sight of the granule by the leader's polling sc1 loads (p50 / p99: upper edge of a 0.1 us bin)\"}\n",
           sc1 ? "sc1 stores (validated form)" : "plain store when the leader shares the XCD (ICP default)", launches, rounds,
           h.checked, h.bad, h.timeouts, h.plain_pub, h.sc1_pub,
           nleader ? h.poll_cycles_sum / (double)nleader * 0.01 : 0.0, h.poll_cycles_max * 0.01, pct(0.5), pct(0.99));
    return h.bad || h.timeouts ? 2 : 0;
}
