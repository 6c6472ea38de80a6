// tf_imgproc.hip -- the cuda:: image-processing functions of the reference API
// (tfusion/include/tfusion/cuda/imgproc.hpp:9-31, tfusion/src/cuda/imgproc.cu) as stateless
// kernels over caller-owned pitched device buffers, for users of the L4 API outside TopFu.
//
// TopFu's own frames never run these: its preprocessing is the fused two-launch front-end of
// tf_preproc.hip (LDS-staged tiles, lookahead in later launches' tails).  These are the same
// per-pixel arithmetic -- the device functions of tf_preproc.h / tf_internal.h -- one thread per
// output pixel reading its window straight from global memory (L1/L2 serve the reuse), so the
// results are bit-identical to the fused path and to the oracle.
#include "tf_internal.h"
#include "tf_preproc.h"

template <typename T>
__device__ __forceinline__ const T* row_of(const void* base, size_t step, int y)
{
    return reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) + (size_t)y * step);
}
template <typename T>
__device__ __forceinline__ T* row_of(void* base, size_t step, int y)
{
    return reinterpret_cast<T*>(reinterpret_cast<char*>(base) + (size_t)y * step);
}

// compute_dists_kernel (imgproc.cu:263-280)
__global__ void __launch_bounds__(256) k_ip_dists(const uint16_t* d, size_t ds, float* o, size_t os, int W, int H)
{
    const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= W || y >= H) return;
    row_of<float>(o, os, y)[x] = tf_dist_of(row_of<uint16_t>(d, ds, y)[x]);
}

// bilateral_kernel (imgproc.cu:10-47): window [max(x-k/2,0), min(x-k/2+k, W-1)), the reference's
// integer colour difference (wrapping past 46340 like its int arithmetic), canonical exp
__global__ void __launch_bounds__(256) k_ip_bilateral(const uint16_t* in, size_t is, uint16_t* out, size_t os, int W,
                                                      int H, int ksz, float ss, float sd)
{
    const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= W || y >= H) return;
    const int value = row_of<uint16_t>(in, is, y)[x];
    const int half = ksz / 2;
    int txe = x - half + ksz; if (txe > W - 1) txe = W - 1;
    int tye = y - half + ksz; if (tye > H - 1) tye = H - 1;
    float sum1 = 0.f, sum2 = 0.f;
    for (int cy = (y - half > 0 ? y - half : 0); cy < tye; ++cy) {
        const uint16_t* r = row_of<uint16_t>(in, is, cy);
        for (int cx = (x - half > 0 ? x - half : 0); cx < txe; ++cx) {
            const int depth = r[cx];
            const float space2 = (float)((x - cx) * (x - cx) + (y - cy) * (y - cy));
            const unsigned dd = (unsigned)(value - depth);
            const float color2 = (float)(int)(dd * dd);
            const float weight = tf_exp(-(space2 * ss + color2 * sd));
            sum1 += (float)depth * weight;
            sum2 += weight;
        }
    }
    const float q = sum1 / sum2;
    row_of<uint16_t>(out, os, y)[x] = (uint16_t)((q == q) ? (int)rintf(q) : 0);   // __float2int_rn
}

// truncate_depth_kernel (imgproc.cu:70-78)
__global__ void __launch_bounds__(256) k_ip_truncate(uint16_t* d, size_t ds, int W, int H, unsigned max_mm)
{
    const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= W || y >= H) return;
    uint16_t* r = row_of<uint16_t>(d, ds, y);
    if (r[x] > max_mm) r[x] = 0;
}

// pyramid_kernel (imgproc.cu:98-127) on a pitched source
__global__ void __launch_bounds__(256) k_ip_pyr(const uint16_t* in, size_t is, int W, int H, uint16_t* out, size_t os,
                                                float sigma3)
{
    const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= W / 2 || y >= H / 2) return;
    const int D = 5;
    const int center = row_of<uint16_t>(in, is, 2 * y)[2 * x];
    int txe = 2 * x - D / 2 + D; if (txe > W - 1) txe = W - 1;
    int tye = 2 * y - D / 2 + D; if (tye > H - 1) tye = H - 1;
    int sum = 0, count = 0;
    for (int cy = (2 * y - D / 2 > 0 ? 2 * y - D / 2 : 0); cy < tye; ++cy) {
        const uint16_t* r = row_of<uint16_t>(in, is, cy);
        for (int cx = (2 * x - D / 2 > 0 ? 2 * x - D / 2 : 0); cx < txe; ++cx) {
            const int val = r[cx];
            if ((float)abs(val - center) < sigma3) { sum += val; ++count; }
        }
    }
    row_of<uint16_t>(out, os, y)[x] = (uint16_t)((count == 0) ? 0 : sum / count);
}

// points_normals_kernel (imgproc.cu:214-243)
__global__ void __launch_bounds__(256) k_ip_point_normals(const uint16_t* d, size_t ds, int W, int H, float fx, float fy,
                                                          float cx, float cy, float4* p, size_t ps, float4* n, size_t ns)
{
    const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= W || y >= H) return;
    const float qnan = tf_qnan();
    float4 po = make_float4(qnan, qnan, qnan, qnan), no = po;
    if (x < W - 1 && y < H - 1) {
        const float fxi = 1.f / fx, fyi = 1.f / fy;
        const uint16_t* r0 = row_of<uint16_t>(d, ds, y);
        const uint16_t* r1 = row_of<uint16_t>(d, ds, y + 1);
        const float z00 = (float)r0[x] * 0.001f, z01 = (float)r0[x + 1] * 0.001f, z10 = (float)r1[x] * 0.001f;
        if (z00 * z01 * z10 != 0) {
            tf3 v00 = mk3(z00 * ((float)x - cx) * fxi, z00 * ((float)y - cy) * fyi, z00);
            tf3 v01 = mk3(z01 * ((float)(x + 1) - cx) * fxi, z01 * ((float)y - cy) * fyi, z01);
            tf3 v10 = mk3(z10 * ((float)x - cx) * fxi, z10 * ((float)(y + 1) - cy) * fyi, z10);
            tf3 nn = knormalized(kcross(sub3(v01, v00), sub3(v10, v00)));
            no = make_float4(-nn.x, -nn.y, -nn.z, 1.0f);
            po = make_float4(v00.x, v00.y, v00.z, 1.0f);
        }
    }
    row_of<float4>(p, ps, y)[x] = po;
    row_of<float4>(n, ns, y)[x] = no;
}

// resize_points_normals_kernel (imgproc.cu:355-388): 2x2 mean, NaN if any point is NaN; the
// normals are not renormalised, w_p = 1, w_n = 0
__global__ void __launch_bounds__(256) k_ip_resize(const float4* p, size_t ps, const float4* n, size_t ns, int W, int H,
                                                   float4* po, size_t pos, float4* no, size_t nos)
{
    const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= W / 2 || y >= H / 2) return;
    const float q = tf_qnan();
    const float4* p0 = row_of<float4>(p, ps, 2 * y);
    const float4* p1 = row_of<float4>(p, ps, 2 * y + 1);
    const float4 d00 = p0[2 * x], d01 = p0[2 * x + 1], d10 = p1[2 * x], d11 = p1[2 * x + 1];
    float4 vo = make_float4(q, q, q, 0.f), nout = make_float4(q, q, q, 0.f);
    if (!isnan(d00.x * d01.x * d10.x * d11.x)) {
        vo = make_float4((((d00.x + d01.x) + d10.x) + d11.x) * 0.25f, (((d00.y + d01.y) + d10.y) + d11.y) * 0.25f,
                         (((d00.z + d01.z) + d10.z) + d11.z) * 0.25f, 1.0f);
        const float4* n0 = row_of<float4>(n, ns, 2 * y);
        const float4* n1 = row_of<float4>(n, ns, 2 * y + 1);
        const float4 m00 = n0[2 * x], m01 = n0[2 * x + 1], m10 = n1[2 * x], m11 = n1[2 * x + 1];
        nout = make_float4((((m00.x + m01.x) + m10.x) + m11.x) * 0.25f, (((m00.y + m01.y) + m10.y) + m11.y) * 0.25f,
                           (((m00.z + m01.z) + m10.z) + m11.z) * 0.25f, 0.f);
    }
    row_of<float4>(po, pos, y)[x] = vo;
    row_of<float4>(no, nos, y)[x] = nout;
}

static tf_status ip_status(hipError_t e)
{
    if (e == hipSuccess) return TF_OK;
    if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) return TF_OOM;
    if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return TF_NO_DEVICE;
    return TF_HIP_ERROR;
}

static dim3 ip_grid(int w, int h) { return dim3((unsigned)((w + 15) / 16), (unsigned)((h + 15) / 16)); }
#define IP_ARGS_OK(cols, rows) ((cols) > 0 && (rows) > 0)

extern "C" tf_status tf_imgproc_compute_dists(const uint16_t* depth, size_t ds, float* dists, size_t os, int cols,
                                              int rows, void* stream)
{
    if (!depth || !dists || !IP_ARGS_OK(cols, rows)) return TF_INVALID_ARG;
    hipLaunchKernelGGL(k_ip_dists, ip_grid(cols, rows), dim3(256), 0, (hipStream_t)stream, depth, ds, dists, os, cols, rows);
    return ip_status(hipGetLastError());
}

extern "C" tf_status tf_imgproc_bilateral(const uint16_t* in, size_t is, uint16_t* out, size_t os, int cols, int rows,
                                          int ksz, float sigma_spatial, float sigma_depth, void* stream)
{
    if (!in || !out || in == out || !IP_ARGS_OK(cols, rows) || ksz < 1) return TF_INVALID_ARG;
    const float sd_mm = sigma_depth * 1000.0f;                       // meters -> mm (imgproc.cu:53)
    const float ss = 0.5f / (sigma_spatial * sigma_spatial), sd = 0.5f / (sd_mm * sd_mm);
    hipLaunchKernelGGL(k_ip_bilateral, ip_grid(cols, rows), dim3(256), 0, (hipStream_t)stream, in, is, out, os, cols, rows,
                       ksz, ss, sd);
    return ip_status(hipGetLastError());
}

extern "C" tf_status tf_imgproc_truncate(uint16_t* depth, size_t ds, int cols, int rows, float threshold, void* stream)
{
    if (!depth || !IP_ARGS_OK(cols, rows)) return TF_INVALID_ARG;
    const unsigned max_mm = (unsigned)(uint16_t)(threshold * 1000.f);   // imgproc.cu:87
    hipLaunchKernelGGL(k_ip_truncate, ip_grid(cols, rows), dim3(256), 0, (hipStream_t)stream, depth, ds, cols, rows, max_mm);
    return ip_status(hipGetLastError());
}

extern "C" tf_status tf_imgproc_pyr_down(const uint16_t* in, size_t is, int cols, int rows, uint16_t* out, size_t os,
                                         float sigma_depth, void* stream)
{
    if (!in || !out || !IP_ARGS_OK(cols / 2, rows / 2)) return TF_INVALID_ARG;
    const float sigma3 = sigma_depth * 1000.0f * 3.0f;                 // imgproc.cu:133-138
    hipLaunchKernelGGL(k_ip_pyr, ip_grid(cols / 2, rows / 2), dim3(256), 0, (hipStream_t)stream, in, is, cols, rows, out, os,
                       sigma3);
    return ip_status(hipGetLastError());
}

extern "C" tf_status tf_imgproc_point_normals(const float intr[4], const uint16_t* depth, size_t ds, int cols, int rows,
                                              void* points, size_t ps, void* normals, size_t ns, void* stream)
{
    if (!intr || !depth || !points || !normals || !IP_ARGS_OK(cols, rows)) return TF_INVALID_ARG;
    hipLaunchKernelGGL(k_ip_point_normals, ip_grid(cols, rows), dim3(256), 0, (hipStream_t)stream, depth, ds, cols, rows,
                       intr[0], intr[1], intr[2], intr[3], (float4*)points, ps, (float4*)normals, ns);
    return ip_status(hipGetLastError());
}

extern "C" tf_status tf_imgproc_resize_points_normals(const void* points, size_t ps, const void* normals, size_t ns,
                                                      int cols, int rows, void* points_out, size_t pos,
                                                      void* normals_out, size_t nos, void* stream)
{
    if (!points || !normals || !points_out || !normals_out || !IP_ARGS_OK(cols / 2, rows / 2)) return TF_INVALID_ARG;
    hipLaunchKernelGGL(k_ip_resize, ip_grid(cols / 2, rows / 2), dim3(256), 0, (hipStream_t)stream, (const float4*)points, ps,
                       (const float4*)normals, ns, cols, rows, (float4*)points_out, pos, (float4*)normals_out, nos);
    return ip_status(hipGetLastError());
}

extern "C" tf_status tf_imgproc_sync(void* stream)
{
    return ip_status(stream ? hipStreamSynchronize((hipStream_t)stream) : hipDeviceSynchronize());
}
