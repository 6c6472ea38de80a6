// tf_preproc.hip -- depth preprocessing front-end for gfx950.
//
//   k_dists_bilateral : compute_dists_kernel + bilateral_kernel + truncate_depth_kernel
//                       (imgproc.cu:10-89,263-290) fused; 32x8 tiles staged in LDS
//   k_pyr_normals     : pyramid_kernel x2 (imgproc.cu:98-140) + points_normals_kernel x3
//                       (imgproc.cu:214-254), all levels in one launch from LDS-staged tiles
//
// All three are HBM/L2-light elementwise-with-halo kernels; the bilateral filter is
// VALU-bound (49 canonical exp per pixel).
#include "tf_preproc.h"

__global__ void __launch_bounds__(256) k_dists_bilateral(BilArgs b)
{
    __shared__ BilLds L;
    bilateral_block<true>(b, blockIdx.x, blockIdx.y, L);
}
__global__ void __launch_bounds__(1024) k_pyr_normals(PyrArgs a)
{
    __shared__ PnLds L;
    pyr_normals_block<1024>(a, blockIdx.x, blockIdx.y, L);
}

// the preprocessing arguments of raw frame `depth`; lookahead: the frame-path split in which
// the bilateral pass leaves dists alone (the current frame's allocation / integration still
// read them) and the pyramid pass writes them
hipError_t tf_pre_args(tf_ctx* c, const uint16_t* depth, size_t pitch, int lookahead, uint16_t* d0, BilArgs* b, PyrArgs* a)
{
    const tf_params& p = c->p;
    float sigma_depth = p.bilateral_sigma_depth * 1000.0f;       // meters -> mm (imgproc.cu:53)
    if (p.bilateral_kernel_size > 2 * HALO + 1) return hipErrorInvalidValue;
    b->src = depth; b->pitch = pitch; b->W = c->W; b->H = c->H; b->ksz = p.bilateral_kernel_size;
    b->ss = 0.5f / (p.bilateral_sigma_spatial * p.bilateral_sigma_spatial);
    b->sd = 0.5f / (sigma_depth * sigma_depth);
    b->do_trunc = p.icp_truncate_depth_dist > 0;
    b->trunc_mm = (unsigned)(uint16_t)(p.icp_truncate_depth_dist * 1000.f);   // imgproc.cu:87
    b->dists = lookahead ? nullptr : c->dists;
    b->dst = d0;
    a->raw = lookahead ? depth : nullptr; a->raw_pitch = pitch;
    a->dists = c->dists;
    a->sigma3 = sigma_depth * 3.0f;                                                    // imgproc.cu:138
    a->d0 = d0; a->d1 = c->depth_pyr[1]; a->d2 = c->depth_pyr[2];
    for (int l = 0; l < TF_LEVELS; ++l) {
        int div = 1 << l;                                 // Intr::operator()(level), precomp.cpp:10-14
        a->pts[l] = c->curr_pts[l]; a->nrm[l] = c->curr_nrm[l];
        a->w[l] = c->lw[l]; a->h[l] = c->lh[l];
        a->fx[l] = p.fx / (float)div; a->fy[l] = p.fy / (float)div; a->cx[l] = p.cx / (float)div; a->cy[l] = p.cy / (float)div;
    }
    return hipSuccess;
}

hipError_t tfk_preprocess(tf_ctx* c, const uint16_t* depth, size_t pitch, hipStream_t strm, uint16_t* d0)
{
    BilArgs b; PyrArgs a;
    hipError_t e = tf_pre_args(c, depth, pitch, 0, d0, &b, &a);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_dists_bilateral, dim3(tf_div_up(c->W, PRE_TX), tf_div_up(c->H, PRE_TY)), dim3(256), 0, strm, b);
    hipLaunchKernelGGL(k_pyr_normals, dim3(tf_div_up(c->W, PN_T0), tf_div_up(c->H, PN_T0)), dim3(1024), 0, strm, a);
    return hipGetLastError();
}
