// tfusion/topfu.hpp -- the tfusion pipeline API (TopFuParams, TopFu) for MI355X, header-only
// over the C-ABI of libtfusion_hip.so (include/tfusion_hip.h).
//
// Drop-in for tfusion/include/tfusion/topfu.hpp:17-110 as used by apps/demo.cpp:27-38,100-115,
// 141-168: TopFuParams::default_params, TopFu(params), operator()(Depth), renderImage(image4u&),
// getCameraPose(time), reset(), params(), icp(); cuda::{setDevice, getCudaEnabledDeviceCount,
// getDeviceName, checkIfPreFermiGPU, printShortCudaDeviceInfo, printCudaDeviceInfo}.
// Behaviour mirrored from topfu.cpp: frame 0 integrates only; later frames track and return
// false after an ICP failure, which resets the pipeline (poses_ back to {Identity},
// topfu.cpp:141-152, 263-264); getCameraPose(time) indexes the pose history (:154-159).
// Errors: a HIP failure throws std::runtime_error (the reference exits, device_memory.cpp:7-11).
#pragma once
#include "../tfusion_hip.h"
#include "types.hpp"
#include "cuda/projective_icp.hpp"

#include <memory>

namespace tfusion
{
    namespace cuda
    {
        inline int getCudaEnabledDeviceCount()
        {
            int n = 0;
            return tf_device_count(&n) == TF_OK ? n : 0;
        }
        inline void setDevice(int device)
        {
            if (tf_set_device(device) != TF_OK) throw std::runtime_error("tfusion::cuda::setDevice failed");
        }
        inline std::string getDeviceName(int device)
        {
            hipDeviceProp_t p;
            hip_check(hipGetDeviceProperties(&p, device), "hipGetDeviceProperties");
            return p.name;
        }
        inline bool checkIfPreFermiGPU(int) { return false; }   // no such GPUs on this path
        inline void printShortCudaDeviceInfo(int device)
        {
            hipDeviceProp_t p;
            hip_check(hipGetDeviceProperties(&p, device), "hipGetDeviceProperties");
            std::printf("Device %d: \"%s\" %s, %d CUs, %.0f GB\n", device, p.name, p.gcnArchName, p.multiProcessorCount,
                        p.totalGlobalMem / 1e9);
        }
        inline void printCudaDeviceInfo(int device) { printShortCudaDeviceInfo(device); }
    }

    // SceneParams (SceneParams.hpp:9-63)
    struct SceneParams {
        float voxelSize, viewFrustum_min, viewFrustum_max, mu;
        int maxW;
        bool stopIntegratingAtMaxW;
        SceneParams() : voxelSize(0.005f), viewFrustum_min(0.2f), viewFrustum_max(3.0f), mu(0.02f), maxW(100),
                        stopIntegratingAtMaxW(false) {}
        SceneParams(float mu_, int maxW_, float voxelSize_, float vmin, float vmax, bool stop)
            : voxelSize(voxelSize_), viewFrustum_min(vmin), viewFrustum_max(vmax), mu(mu_), maxW(maxW_),
              stopIntegratingAtMaxW(stop) {}
    };

    // TopFuParams (topfu.hpp:28-60).  Fields the hot path does not read (volume_*, tsdf_*,
    // raycast_step_factor, gradient_delta_factor, light_pose) are kept for source compatibility.
    // The capacities (hash buckets / excess / blocks / visible list / render blocks) are MI355X
    // additions with the reference's values as defaults (VoxelBlockHash.hpp:10-27).
    struct TopFuParams {
        static TopFuParams default_params()   // topfu.cpp:12-53
        {
            TopFuParams p;
            p.cols = 640; p.rows = 480;
            p.intr = Intr(504.261f, 503.905f, 352.457f, 272.202f);
            p.volume_dims = Vec3i::all(512);
            p.volume_size = Vec3f::all(3.f);
            p.volume_pose = Affine3f().translate(Vec3f(-1.5f, -1.5f, 0.5f));
            p.bilateral_sigma_depth = 0.04f;
            p.bilateral_sigma_spatial = 4.5f;
            p.bilateral_kernel_size = 7;
            p.icp_truncate_depth_dist = 2.0f;
            p.icp_dist_thres = 0.1f;
            p.icp_angle_thres = deg2rad(30.f);
            p.icp_iter_num = { 10, 5, 4, 0 };
            p.tsdf_min_camera_movement = 0.f;
            p.tsdf_trunc_dist = 0.04f;
            p.tsdf_max_weight = 64;
            p.raycast_step_factor = 0.75f;
            p.gradient_delta_factor = 0.5f;
            p.light_pose = Vec3f::all(0.f);
            p.sceneParams = std::make_shared<SceneParams>(0.02f, 100, 0.005f, 0.2f, 3.0f, false);
            tf_params d;
            tf_default_params(&d);
            p.n_buckets = d.n_buckets; p.n_excess = d.n_excess; p.n_blocks = d.n_blocks;
            p.vis_capacity = d.vis_capacity; p.max_render_blocks = d.max_render_blocks;
            p.integrate_colour = false;
            p.rgb_intr = Intr(0.f, 0.f, 0.f, 0.f);
            p.depth_to_rgb = Affine3f::Identity();
            return p;
        }

        int cols, rows;
        Intr intr;
        Vec3i volume_dims;
        Vec3f volume_size;
        Affine3f volume_pose;
        float bilateral_sigma_depth, bilateral_sigma_spatial;
        int bilateral_kernel_size;
        float icp_truncate_depth_dist, icp_dist_thres, icp_angle_thres;
        std::vector<int> icp_iter_num;
        float tsdf_min_camera_movement, tsdf_trunc_dist;
        int tsdf_max_weight;
        float raycast_step_factor, gradient_delta_factor;
        Vec3f light_pose;
        std::shared_ptr<SceneParams> sceneParams;   // the reference leaks a raw pointer (topfu.cpp:50)
        int n_buckets, n_excess, n_blocks, vis_capacity, max_render_blocks;
        // colour (an addition): Voxel_s_rgb voxels, the RGB image of operator()(depth, rgba)
        // integrated (VoxelTypes.hpp:39-67, SceneReconstructionEngine.hpp:116-148); rgb_intr all 0
        // = the depth intrinsics; depth_to_rgb = trafo_rgb_to_depth.calib_inv (identity: registered)
        bool integrate_colour;
        Intr rgb_intr;
        Affine3f depth_to_rgb;

        tf_params to_c() const
        {
            tf_params c;
            tf_default_params(&c);
            c.cols = cols; c.rows = rows;
            c.fx = intr.fx; c.fy = intr.fy; c.cx = intr.cx; c.cy = intr.cy;
            c.bilateral_sigma_depth = bilateral_sigma_depth;
            c.bilateral_sigma_spatial = bilateral_sigma_spatial;
            c.bilateral_kernel_size = bilateral_kernel_size;
            c.icp_truncate_depth_dist = icp_truncate_depth_dist;
            c.icp_dist_thres = icp_dist_thres;
            c.icp_angle_thres = icp_angle_thres;
            for (int i = 0; i < 4; ++i) c.icp_iter_num[i] = i < (int)icp_iter_num.size() ? icp_iter_num[i] : 0;
            if (sceneParams) {
                c.mu = sceneParams->mu; c.maxW = sceneParams->maxW; c.voxelSize = sceneParams->voxelSize;
                c.viewFrustum_min = sceneParams->viewFrustum_min; c.viewFrustum_max = sceneParams->viewFrustum_max;
            }
            c.n_buckets = n_buckets; c.n_excess = n_excess; c.n_blocks = n_blocks;
            c.vis_capacity = vis_capacity; c.max_render_blocks = max_render_blocks;
            c.voxel_rgb = integrate_colour ? 1 : 0;
            c.rgb_intr[0] = rgb_intr.fx; c.rgb_intr[1] = rgb_intr.fy; c.rgb_intr[2] = rgb_intr.cx; c.rgb_intr[3] = rgb_intr.cy;
            affine_to_rt(depth_to_rgb, c.depth_to_rgb);
            return c;
        }
    };

    class TopFu
    {
    public:
        typedef SharedPtr<TopFu> Ptr;   // cv::Ptr<TopFu> (topfu.hpp:65); std::shared_ptr without OpenCV

        explicit TopFu(const TopFuParams& params) : params_(params)
        {
            const tf_params c = params_.to_c();
            check(tf_create(&c, &ctx_), "tf_create");
            // topfu.cpp:77-80: the tracker takes the TopFu's thresholds and iterations
            icp_.bind(ctx_);
            icp_.setDistThreshold(params_.icp_dist_thres);
            icp_.setAngleThreshold(params_.icp_angle_thres);
            icp_.setIterationsNum(params_.icp_iter_num);
            poses_.reserve(30000);
            poses_.push_back(Affine3f::Identity());
        }
        ~TopFu() { tf_destroy(ctx_); }
        TopFu(const TopFu&) = delete;
        TopFu& operator=(const TopFu&) = delete;

        const TopFuParams& params() const { return params_; }
        TopFuParams& params() { return params_; }

        // topfu.hpp:75-76: the frame tracker; its setters change the parameters the following
        // frames use, and estimateTransform runs it on caller pyramids (through this context,
        // whose current / previous maps it overwrites)
        const cuda::ProjectiveICP& icp() const { return icp_; }
        cuda::ProjectiveICP& icp() { return icp_; }

        void reset()                                  // topfu.cpp:141-152
        {
            check(tf_reset(ctx_), "tf_reset");
            frame_counter_ = 0;
            poses_.clear();
            poses_.push_back(Affine3f::Identity());
        }

        // TopFu::operator() (topfu.cpp:161-330); the colour image is unused by the reference too
        bool operator()(const cuda::Depth& depth, const cuda::Image& = cuda::Image())
        {
            return frame(depth, nullptr);
        }
        // with params().integrate_colour: the frame's RGBA image (Vector4u, the engine's view->rgb)
        // integrated into the Voxel_s_rgb colour (an addition)
        bool operator()(const cuda::Depth& depth, const cuda::image4u& rgba)
        {
            return frame(depth, &rgba);
        }

    private:
        bool frame(const cuda::Depth& depth, const cuda::image4u* rgba)
        {
            float rt[12];
            // no tf_stats: the call returns once the frame's result is known (stats() waits for the rest)
            const tf_status s = rgba && !rgba->empty()
                ? tf_process_frame_rgb(ctx_, depth.ptr(), depth.step(), reinterpret_cast<const uint8_t*>(rgba->ptr()),
                                       rgba->step(), rt, nullptr)
                : tf_process_frame(ctx_, depth.ptr(), depth.step(), rt, nullptr);
            if (s == TF_ICP_FAIL) {                   // reset(), return false (topfu.cpp:263-264)
                frame_counter_ = 0;
                poses_.clear();
                poses_.push_back(Affine3f::Identity());
                return false;
            }
            check(s, "tf_process_frame");
            if (frame_counter_ > 0) poses_.push_back(affine_from_rt(rt));   // poses_.back() * affine
            ++frame_counter_;
            return true;
        }

    public:

        // TopFu::renderImage (topfu.cpp:332-377): grey shading of the current pose.  The type
        // argument (default: the reference's RENDER_SHADED_GREYSCALE) selects one of the engine's
        // RenderImageType modes (VisualisationEngine.hpp:15-22) -- an addition, source compatible.
        enum RenderImageType {
            RENDER_SHADED_GREYSCALE = TF_RENDER_SHADED_GREYSCALE,
            RENDER_SHADED_GREYSCALE_IMAGENORMALS = TF_RENDER_SHADED_GREYSCALE_IMAGENORMALS,
            RENDER_COLOUR_FROM_VOLUME = TF_RENDER_COLOUR_FROM_VOLUME,
            RENDER_COLOUR_FROM_NORMAL = TF_RENDER_COLOUR_FROM_NORMAL,
            RENDER_COLOUR_FROM_CONFIDENCE = TF_RENDER_COLOUR_FROM_CONFIDENCE
        };
        void renderImage(cuda::image4u& image, RenderImageType type = RENDER_SHADED_GREYSCALE)
        {
            image.create(params_.rows, params_.cols);
            check(tf_render_image_type(ctx_, (int)type, reinterpret_cast<uint8_t*>(image.ptr()), image.step()),
                  "tf_render_image_type");
        }

        Affine3f getCameraPose(int time = -1) const   // topfu.cpp:154-159
        {
            if (time > (int)poses_.size() || time < 0) time = (int)poses_.size() - 1;
            return poses_[time];
        }

        tf_stats stats() const
        {
            tf_stats s;
            check(tf_get_stats(ctx_, &s), "tf_get_stats");
            return s;
        }
        tf_ctx* handle() { return ctx_; }
        hipStream_t stream() const { return (hipStream_t)tf_get_stream(ctx_); }

    private:
        static void check(tf_status s, const char* what)
        {
            if (s != TF_OK) throw std::runtime_error(std::string(what) + ": " + tf_status_string(s));
        }
        TopFuParams params_;
        tf_ctx* ctx_ = nullptr;
        cuda::ProjectiveICP icp_;
        int frame_counter_ = 0;
        std::vector<Affine3f> poses_;
    };
}
