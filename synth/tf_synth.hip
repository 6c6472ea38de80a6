// tf_synth.hip -- synthetic depth streams rendered on the GPU (bench / test input, not the
// product): the C2 / C5 room (render_room) and the C5E hall (render_hall) of
// topfusion_amd/synth.py, bit for bit.
//
// The numpy renderer is the definition; this is the same float64 arithmetic in the same order
// (compiled with -ffp-contract=off: no contraction, IEEE-correct division), so a frame rendered
// here equals synth.render_hall's.  It links the HIP runtime of /opt/rocm, the one
// libtfusion_hip.so uses, so frames and fusion share one runtime and one device context.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#define HALL_FLOOR 0.55
#define HALL_CEIL (-0.75)
#define HALL_PERIOD 0.8
#define HALL_REACH 3
#define HALL_CELLS ((2 * HALL_REACH + 1) * (2 * HALL_REACH + 1))

__host__ __device__ static inline uint32_t mix32(uint32_t h)
{
    h ^= h >> 16; h *= 0x7FEB352Du; h ^= h >> 15; h *= 0x846CA68Bu; h ^= h >> 16;
    return h;
}
__host__ __device__ static inline double unit32(uint32_t h) { return (double)h * (1.0 / 4294967296.0); }

struct HallBox { double lo[3], hi[3]; int kind; };

// synth.hall_cell
__device__ static void hall_cell(long long i, long long j, HallBox* b)
{
    uint32_t h = mix32((uint32_t)i * 0x9E3779B1u ^ mix32((uint32_t)j + 0x632BE5ABu));
    double u[6];
    u[0] = unit32(h);
    for (int k = 1; k < 6; ++k) { h = mix32(h + 0x9E3779B9u); u[k] = unit32(h); }
    const int kind = u[0] < 0.45 ? 1 : (u[0] < 0.8 ? 2 : 0);
    const double cx = ((double)i + 0.5) * HALL_PERIOD + (u[1] - 0.5) * 0.2;
    const double cz = ((double)j + 0.5) * HALL_PERIOD + (u[2] - 0.5) * 0.2;
    const double hx = 0.08 + 0.14 * u[3];
    const double hz = 0.08 + 0.14 * u[4];
    const double ylo = kind == 1 ? 0.2 + 0.2 * u[5] : HALL_CEIL;
    const double yhi = kind == 1 ? HALL_FLOOR : -0.35 - 0.2 * u[5];
    b->lo[0] = cx - hx; b->lo[1] = ylo; b->lo[2] = cz - hz;
    b->hi[0] = cx + hx; b->hi[1] = yhi; b->hi[2] = cz + hz;
    b->kind = kind;
}

// synth._slab
__device__ static inline double slab(const double* o, const double* d, const HallBox& b)
{
    double tn = -INFINITY, tf = INFINITY;
    for (int a = 0; a < 3; ++a) {
        double t1, t2;
        if (d[a] == 0.0) {
            const bool inside = o[a] >= b.lo[a] && o[a] <= b.hi[a];
            t1 = inside ? -INFINITY : INFINITY;
            t2 = inside ? INFINITY : -INFINITY;
        } else {
            t1 = (b.lo[a] - o[a]) / d[a];
            t2 = (b.hi[a] - o[a]) / d[a];
        }
        tn = fmax(tn, fmin(t1, t2));
        tf = fmin(tf, fmax(t1, t2));
    }
    return (tn <= tf && tn > 1e-6) ? tn : INFINITY;
}

struct HallArgs {
    uint16_t* out; size_t stride;      // frame f at out + f * stride bytes
    const double* poses;               // [n][12]: R row-major, then t (camera -> world)
    int first, W, H;
    double fx, fy, cx, cy, noise_mm;
    uint32_t seed;
};

__global__ void __launch_bounds__(256) k_render_hall(HallArgs a)
{
    __shared__ HallBox box[HALL_CELLS];
    __shared__ double P[12];
    const int f = blockIdx.z;
    if (threadIdx.x < 12) P[threadIdx.x] = a.poses[12 * (size_t)f + threadIdx.x];
    __syncthreads();
    const double o[3] = { P[9], P[10], P[11] };
    if (threadIdx.x < HALL_CELLS) {
        const long long ci = (long long)floor(o[0] / HALL_PERIOD), cj = (long long)floor(o[2] / HALL_PERIOD);
        const int di = (int)threadIdx.x / (2 * HALL_REACH + 1) - HALL_REACH, dj = (int)threadIdx.x % (2 * HALL_REACH + 1) - HALL_REACH;
        hall_cell(ci + di, cj + dj, &box[threadIdx.x]);
    }
    __syncthreads();
    const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= a.W || y >= a.H) return;
    const double xc = ((double)x - a.cx) / a.fx, yc = ((double)y - a.cy) / a.fy;
    const double d[3] = { (P[0] * xc + P[1] * yc) + P[2], (P[3] * xc + P[4] * yc) + P[5], (P[6] * xc + P[7] * yc) + P[8] };
    double best = INFINITY;
    {
        const double y0s[2] = { HALL_FLOOR, HALL_CEIL };
        for (int k = 0; k < 2; ++k) {
            const double tt = (y0s[k] - o[1]) / d[1];      // d[1] == 0: +-inf or nan, never > 1e-6 unless +inf
            const double v = (tt > 1e-6) ? tt : INFINITY;
            best = fmin(best, v);
        }
    }
    for (int c = 0; c < HALL_CELLS; ++c) {
        if (box[c].kind == 0) continue;
        best = fmin(best, slab(o, d, box[c]));
    }
    double mm = best * 1000.0;
    if (a.noise_mm > 0) {
        const uint32_t frame = (uint32_t)(a.first + f);
        const uint32_t base = mix32(mix32(a.seed + 0x2545F491u) ^ frame);
        const uint32_t pix = (uint32_t)(y * a.W + x);
        double s = 0.0;
        for (int k = 0; k < 4; ++k) s = s + unit32(mix32(base ^ mix32(pix * 4u + (uint32_t)k + 0x68E31DA4u)));
        mm = mm + a.noise_mm * ((s - 2.0) * 1.7320508075688772);
    }
    double r = isfinite(mm) ? rint(mm) : 0.0;
    r = r < 0.0 ? 0.0 : (r > 65535.0 ? 65535.0 : r);
    *(uint16_t*)((char*)a.out + (size_t)f * a.stride + ((size_t)y * a.W + x) * 2) = (uint16_t)r;
}

struct RoomArgs {
    uint16_t* out; size_t stride;
    const double* poses;
    int first, W, H, sphere;
    double fx, fy, cx, cy, noise_mm;
    uint32_t seed;
};

__device__ static inline double hashed_noise(uint32_t seed, uint32_t frame, uint32_t pix)
{
    const uint32_t base = mix32(mix32(seed + 0x2545F491u) ^ frame);
    double s = 0.0;
    for (int k = 0; k < 4; ++k) s = s + unit32(mix32(base ^ mix32(pix * 4u + (uint32_t)k + 0x68E31DA4u)));
    return (s - 2.0) * 1.7320508075688772;
}

// synth.render_room: the room of render_depth (six walls + the sphere) with the hashed noise
__global__ void __launch_bounds__(256) k_render_room(RoomArgs a)
{
    __shared__ double P[12];
    const int f = blockIdx.z;
    if (threadIdx.x < 12) P[threadIdx.x] = a.poses[12 * (size_t)f + threadIdx.x];
    __syncthreads();
    const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= a.W || y >= a.H) return;
    const double o[3] = { P[9], P[10], P[11] };
    const double xc = ((double)x - a.cx) / a.fx, yc = ((double)y - a.cy) / a.fy;
    const double d[3] = { (P[0] * xc + P[1] * yc) + P[2], (P[3] * xc + P[4] * yc) + P[5], (P[6] * xc + P[7] * yc) + P[8] };
    const int ax[6] = { 2, 1, 0, 0, 1, 2 };
    const double off[6] = { 1.8, 0.6, -0.8, 1.1, -0.9, -0.6 };
    double best = INFINITY;
    for (int k = 0; k < 6; ++k) {
        const double tt = (off[k] - o[ax[k]]) / d[ax[k]];
        best = fmin(best, (tt > 1e-6) ? tt : INFINITY);
    }
    if (a.sphere) {
        const double oc[3] = { o[0] - 0.15, o[1] - 0.25, o[2] - 1.3 };
        const double b = (d[0] * oc[0] + d[1] * oc[1]) + d[2] * oc[2];
        const double aa = (d[0] * d[0] + d[1] * d[1]) + d[2] * d[2];
        const double cc = ((oc[0] * oc[0] + oc[1] * oc[1]) + oc[2] * oc[2]) - 0.09;
        const double disc = b * b - aa * cc;
        const double t0 = (-b - sqrt(fmax(disc, 0.0))) / aa;
        best = fmin(best, (disc >= 0 && t0 > 1e-6) ? t0 : INFINITY);
    }
    double mm = best * 1000.0;
    if (a.noise_mm > 0) mm = mm + a.noise_mm * hashed_noise(a.seed, (uint32_t)(a.first + f), (uint32_t)(y * a.W + x));
    double r = isfinite(mm) ? rint(mm) : 0.0;
    r = r < 0.0 ? 0.0 : (r > 65535.0 ? 65535.0 : r);
    *(uint16_t*)((char*)a.out + (size_t)f * a.stride + ((size_t)y * a.W + x) * 2) = (uint16_t)r;
}

// synth.render_colour: the colour camera's view of the room (uchar4, alpha 255, black where no
// surface is hit) -- the RGB stream of the colour TSDF lines.  Not bit-identical with numpy (sin /
// cos of the device's libm): only the GPU renders it, and the parity tests feed both sides the
// same downloaded images.
__global__ void __launch_bounds__(256) k_render_room_rgb(RoomArgs a, uchar4* out)
{
    __shared__ double P[12];
    const int f = blockIdx.z;
    if (threadIdx.x < 12) P[threadIdx.x] = a.poses[12 * (size_t)f + threadIdx.x];
    __syncthreads();
    const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= a.W || y >= a.H) return;
    const double o[3] = { P[9], P[10], P[11] };
    const double xc = ((double)x - a.cx) / a.fx, yc = ((double)y - a.cy) / a.fy;
    const double d[3] = { (P[0] * xc + P[1] * yc) + P[2], (P[3] * xc + P[4] * yc) + P[5], (P[6] * xc + P[7] * yc) + P[8] };
    const int ax[6] = { 2, 1, 0, 0, 1, 2 };
    const double off[6] = { 1.8, 0.6, -0.8, 1.1, -0.9, -0.6 };
    double best = INFINITY;
    for (int k = 0; k < 6; ++k) {
        const double tt = (off[k] - o[ax[k]]) / d[ax[k]];
        best = fmin(best, (tt > 1e-6) ? tt : INFINITY);
    }
    if (a.sphere) {
        const double oc[3] = { o[0] - 0.15, o[1] - 0.25, o[2] - 1.3 };
        const double b = (d[0] * oc[0] + d[1] * oc[1]) + d[2] * oc[2];
        const double aa = (d[0] * d[0] + d[1] * d[1]) + d[2] * d[2];
        const double cc = ((oc[0] * oc[0] + oc[1] * oc[1]) + oc[2] * oc[2]) - 0.09;
        const double disc = b * b - aa * cc;
        const double t0 = (-b - sqrt(fmax(disc, 0.0))) / aa;
        best = fmin(best, (disc >= 0 && t0 > 1e-6) ? t0 : INFINITY);
    }
    uchar4 c = make_uchar4(0, 0, 0, 0);
    if (isfinite(best)) {
        const double p[3] = { o[0] + d[0] * best, o[1] + d[1] * best, o[2] + d[2] * best };
        const double tp = 6.283185307179586;
        c.x = (unsigned char)rint(127.5 + 120.0 * sin(tp * p[0] / 0.13));
        c.y = (unsigned char)rint(127.5 + 120.0 * sin(tp * (p[1] + p[2]) / 0.17));
        c.z = (unsigned char)rint(127.5 + 120.0 * cos(tp * (p[2] - p[0]) / 0.23));
        c.w = 255;
    }
    *(uchar4*)((char*)out + (size_t)f * a.stride + ((size_t)y * a.W + x) * 4) = c;
}

extern "C" {

// frames first..first+n-1 of the colour camera's view of the room (uchar4), the RGB stream of the
// colour TSDF lines; stride in bytes (>= W * H * 4).  Synchronous.  0 = ok.
int tfs_render_room_rgb(uchar4* dev_out, size_t stride, const double* poses, int n, int W, int H,
                        double fx, double fy, double cx, double cy, int sphere)
{
    if (!dev_out || !poses || n < 0 || W <= 0 || H <= 0 || stride < (size_t)W * H * 4) return 1;
    const int B = 256;
    double* dp = nullptr;
    if (hipMalloc((void**)&dp, sizeof(double) * 12 * (size_t)(n < B ? n : B) + 16) != hipSuccess) return 2;
    int rc = 0;
    for (int f0 = 0; f0 < n && !rc; f0 += B) {
        const int nb = n - f0 < B ? n - f0 : B;
        if (hipMemcpy(dp, poses + 12 * (size_t)f0, sizeof(double) * 12 * nb, hipMemcpyHostToDevice) != hipSuccess) { rc = 3; break; }
        RoomArgs a;
        a.out = nullptr; a.stride = stride; a.poses = dp; a.first = f0; a.W = W; a.H = H; a.sphere = sphere;
        a.fx = fx; a.fy = fy; a.cx = cx; a.cy = cy; a.noise_mm = 0; a.seed = 0;
        hipLaunchKernelGGL(k_render_room_rgb, dim3((W + 15) / 16, (H + 15) / 16, nb), dim3(256), 0, 0, a,
                           (uchar4*)((char*)dev_out + (size_t)f0 * stride));
        if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) rc = 4;
    }
    (void)hipFree(dp);
    return rc;
}

// frames first..first+n-1 of the room at the host poses [n][12] (camera -> world), as
// tfs_render_hall; sphere: render_depth's sphere in the room.  Synchronous.  0 = ok.
int tfs_render_room(uint16_t* dev_out, size_t stride, const double* poses, int n, int first, int W, int H,
                    double fx, double fy, double cx, double cy, unsigned seed, double noise_mm, int sphere)
{
    if (!dev_out || !poses || n < 0 || W <= 0 || H <= 0 || stride < (size_t)W * H * 2) return 1;
    const int B = 256;
    double* dp = nullptr;
    if (hipMalloc((void**)&dp, sizeof(double) * 12 * (size_t)(n < B ? n : B) + 16) != hipSuccess) return 2;
    int rc = 0;
    for (int f0 = 0; f0 < n && !rc; f0 += B) {
        const int nb = n - f0 < B ? n - f0 : B;
        if (hipMemcpy(dp, poses + 12 * (size_t)f0, sizeof(double) * 12 * nb, hipMemcpyHostToDevice) != hipSuccess) { rc = 3; break; }
        RoomArgs a;
        a.out = (uint16_t*)((char*)dev_out + (size_t)f0 * stride); a.stride = stride;
        a.poses = dp; a.first = first + f0; a.W = W; a.H = H; a.sphere = sphere;
        a.fx = fx; a.fy = fy; a.cx = cx; a.cy = cy; a.noise_mm = noise_mm; a.seed = seed;
        hipLaunchKernelGGL(k_render_room, dim3((W + 15) / 16, (H + 15) / 16, nb), dim3(256), 0, 0, a);
        if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) rc = 4;
    }
    (void)hipFree(dp);
    return rc;
}

// device-to-device copy bandwidth (read + write bytes / s) over `bytes`, HIP events, reps copies
double tfs_copy_gbs(size_t bytes, int reps)
{
    void *a = nullptr, *b = nullptr;
    double gbs = -1.0;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (hipMalloc(&a, bytes) == hipSuccess && hipMalloc(&b, bytes) == hipSuccess &&
        hipEventCreate(&e0) == hipSuccess && hipEventCreate(&e1) == hipSuccess &&
        hipMemcpy(b, a, bytes, hipMemcpyDeviceToDevice) == hipSuccess) {
        (void)hipEventRecord(e0, 0);
        for (int i = 0; i < reps; ++i) (void)hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, 0);
        (void)hipEventRecord(e1, 0);
        float ms = 0.f;
        if (hipEventSynchronize(e1) == hipSuccess && hipEventElapsedTime(&ms, e0, e1) == hipSuccess && ms > 0)
            gbs = 2.0 * (double)bytes * reps / (ms * 1e-3) / 1e9;
    }
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (a) (void)hipFree(a);
    if (b) (void)hipFree(b);
    return gbs;
}

// frames first..first+n-1 of the hall walk into dev_out (frame k - first at k * stride bytes);
// poses: host float64 [n][12] camera -> world (R row-major, t).  Synchronous.  0 = ok.
int tfs_render_hall(uint16_t* dev_out, size_t stride, const double* poses, int n, int first, int W, int H,
                    double fx, double fy, double cx, double cy, unsigned seed, double noise_mm)
{
    if (!dev_out || !poses || n < 0 || W <= 0 || H <= 0 || stride < (size_t)W * H * 2) return 1;
    const int B = 256;                  // frames per launch
    double* dp = nullptr;
    if (hipMalloc((void**)&dp, sizeof(double) * 12 * (size_t)(n < B ? n : B) + 16) != hipSuccess) return 2;
    int rc = 0;
    for (int f0 = 0; f0 < n && !rc; f0 += B) {
        const int nb = n - f0 < B ? n - f0 : B;
        if (hipMemcpy(dp, poses + 12 * (size_t)f0, sizeof(double) * 12 * nb, hipMemcpyHostToDevice) != hipSuccess) { rc = 3; break; }
        HallArgs a;
        a.out = (uint16_t*)((char*)dev_out + (size_t)f0 * stride); a.stride = stride;
        a.poses = dp; a.first = first + f0; a.W = W; a.H = H;
        a.fx = fx; a.fy = fy; a.cx = cx; a.cy = cy; a.noise_mm = noise_mm; a.seed = seed;
        hipLaunchKernelGGL(k_render_hall, dim3((W + 15) / 16, (H + 15) / 16, nb), dim3(256), 0, 0, a);
        if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) rc = 4;
    }
    (void)hipFree(dp);
    return rc;
}

// device memory for the frames (the same runtime as libtfusion_hip.so)
int tfs_malloc(void** p, size_t bytes) { return hipMalloc(p, bytes) == hipSuccess ? 0 : 1; }
int tfs_free(void* p) { return hipFree(p) == hipSuccess ? 0 : 1; }
int tfs_download(void* host, const void* dev, size_t bytes)
{
    return hipMemcpy(host, dev, bytes, hipMemcpyDeviceToHost) == hipSuccess ? 0 : 1;
}
int tfs_upload(void* dev, const void* host, size_t bytes)
{
    return hipMemcpy(dev, host, bytes, hipMemcpyHostToDevice) == hipSuccess ? 0 : 1;
}
int tfs_sync(void) { return hipDeviceSynchronize() == hipSuccess ? 0 : 1; }

}
