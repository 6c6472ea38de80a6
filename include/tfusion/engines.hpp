// tfusion/engines.hpp -- the L4 engine API of the reference (scene, render state, reconstruction
// and visualisation engines, cuda:: image processing) for MI355X, header-only over the C-ABI of
// libtfusion_hip.so.  Mirrors:
//   Scene<TVoxel, TIndex>                   tfusion/include/tfusion/scene.hpp:13-44
//   RenderState / RenderState_VH            tfusion/include/tfusion/RenderState.hpp:12-88, RenderState_VH.hpp:15-61
//   SceneReconstructionEngine_CUDA          tfusion/include/tfusion/cuda/SceneReconstructionEngine_host.hpp:42-74
//   VisualisationEngine_CUDA                tfusion/include/tfusion/cuda/VisualisationEngine_CUDA.hpp:12-47
//   IVisualisationEngine enums              tfusion/include/tfusion/VisualisationEngine.hpp:12-40
//   cuda::{computeDists, depthBilateralFilter, depthTruncation, depthBuildPyramid,
//          computePointNormals, resizePointsNormals, waitAllDefaultStream}
//                                           tfusion/include/tfusion/cuda/imgproc.hpp:9-31
//
// One difference of structure: a Scene owns one libtfusion_hip context, which holds the scene
// (hash, voxel blocks, block grid) AND the render state it is rendered with (visible list and
// types, range image, raycast result).  A RenderState object is therefore a handle that the
// engines accept for source compatibility; everything goes to the scene's context, so a scene
// has exactly one render state.  The context is sized at construction: the image size and the
// capacities come from the TopFuParams the Scene is given (defaults: the reference's
// default_params, VoxelBlockHash.hpp:10-27).
#pragma once
#include "../tfusion_hip.h"
#include "topfu.hpp"
#include "types.hpp"

#include <stdexcept>
#include <string>

namespace tfusion
{
    inline void tf_engine_check(tf_status s, const char* what)
    {
        if (s != TF_OK) throw std::runtime_error(std::string(what) + ": " + tf_status_string(s));
    }

    // voxel / index type tags (VoxelTypes.hpp:69-92, VoxelBlockHash.hpp:53-122)
    struct Voxel_s {
        short sdf;
        unsigned char w_depth;
        unsigned char pad;
        static short SDF_initialValue() { return 32767; }
        static float valueToFloat(float x) { return x / 32767.0f; }
        static short floatToValue(float x) { return (short)(x * 32767.0f); }
        static const bool hasColorInformation = false;
    };
    // Voxel_s_rgb (VoxelTypes.hpp:39-67): the context keeps its colour half (clr, w_color) as a
    // second plane (TF_BUF_VBA_RGB); this struct is the combined view a caller assembles
    struct Voxel_s_rgb {
        short sdf;
        unsigned char w_depth;
        Vector3u clr;
        unsigned char w_color;
        static short SDF_initialValue() { return 32767; }
        static float valueToFloat(float x) { return x / 32767.0f; }
        static short floatToValue(float x) { return (short)(x * 32767.0f); }
        static const bool hasColorInformation = true;
    };
    struct VoxelBlockHash {
        enum { noTotalEntries = 0x100000 + 0x20000 };   // SDF_BUCKET_NUM + SDF_EXCESS_LIST_SIZE (defaults)
    };

    // IVisualisationEngine::RenderImageType / RenderRaycastSelection (VisualisationEngine.hpp:15-27)
    struct IVisualisationEngine {
        enum RenderImageType {
            RENDER_SHADED_GREYSCALE = TF_RENDER_SHADED_GREYSCALE,
            RENDER_SHADED_GREYSCALE_IMAGENORMALS = TF_RENDER_SHADED_GREYSCALE_IMAGENORMALS,
            RENDER_COLOUR_FROM_VOLUME = TF_RENDER_COLOUR_FROM_VOLUME,
            RENDER_COLOUR_FROM_NORMAL = TF_RENDER_COLOUR_FROM_NORMAL,
            RENDER_COLOUR_FROM_CONFIDENCE = TF_RENDER_COLOUR_FROM_CONFIDENCE
        };
        enum RenderRaycastSelection { RENDER_FROM_NEW_RAYCAST, RENDER_FROM_OLD_RAYCAST, RENDER_FROM_OLD_FORWARDPROJ };
    };

    // HashSwapState (GlobalCache.hpp:11-20): 0 data on the host side only, 1 in both (not yet
    // combined), 2 most recent in active memory
    struct HashSwapState { unsigned char state; };

    // GlobalCache<TVoxel> (GlobalCache.hpp:22-134): a view of the scene context's cache, which
    // lives in HBM next to the active voxel blocks, not in host memory;
    // the accessors copy out.  The transfer buffers of the reference (synced blocks, needed ids)
    // have no counterpart: a transfer is a device-side copy.
    template <class TVoxel>
    class GlobalCache
    {
    public:
        int noTotalEntries;

        explicit GlobalCache(tf_ctx* ctx) : noTotalEntries(0), ctx_(ctx)
        {
            tf_params p;
            tf_engine_check(tf_get_params(ctx, &p), "GlobalCache: tf_get_params");
            noTotalEntries = p.n_buckets + p.n_excess;
        }
        bool HasStoredData(int address) const { return byte_at(TF_BUF_SWAP_STORED_FLAGS, address) != 0; }
        // the stored block of an entry (SDF_BLOCK_SIZE3 voxels) copied into `out`
        void GetStoredVoxelBlock(int address, TVoxel* out) const
        {
            size_t n = 0;
            tf_engine_check(tf_buffer_bytes(ctx_, TF_BUF_SWAP_STORED, 0, &n), "tf_buffer_bytes");
            const size_t blk = sizeof(TVoxel) * 512;
            if (address < 0 || address >= noTotalEntries) throw std::out_of_range("GetStoredVoxelBlock");
            tf_engine_check(tf_download_range(ctx_, TF_BUF_SWAP_STORED, (size_t)address * blk, out, blk),
                            "GetStoredVoxelBlock");
        }
        HashSwapState GetSwapState(int address) const { return HashSwapState{ byte_at(TF_BUF_SWAP_STATE, address) }; }
        void SaveToFile(const char* fileName) const { tf_engine_check(tf_swap_save(ctx_, fileName), "SaveToFile"); }
        void ReadFromFile(const char* fileName) { tf_engine_check(tf_swap_load(ctx_, fileName), "ReadFromFile"); }

    private:
        unsigned char byte_at(int which, int address) const
        {
            if (address < 0 || address >= noTotalEntries) throw std::out_of_range("GlobalCache entry");
            unsigned char b = 0;
            tf_engine_check(tf_download_range(ctx_, which, (size_t)address, &b, 1), "GlobalCache");
            return b;
        }
        tf_ctx* ctx_;
    };

    // Scene<TVoxel, TIndex> (scene.hpp:13-44): owns the context
    template <class TVoxel, class TIndex>
    class Scene
    {
    public:
        const SceneParams* sceneParams;
        GlobalCache<TVoxel>* globalCache = nullptr;     // scene.hpp:27, set when useSwapping

        // scene.hpp:29-34; `frame` (an addition, defaulted) gives the image size, intrinsics and
        // capacities the context is created with; useSwapping sets tf_params::use_swapping
        Scene(const SceneParams* params, bool useSwapping, const TopFuParams& frame = TopFuParams::default_params())
            : sceneParams(params)
        {
            TopFuParams tp = frame;
            tf_params c = tp.to_c();
            if (params) {
                c.mu = params->mu; c.maxW = params->maxW; c.voxelSize = params->voxelSize;
                c.viewFrustum_min = params->viewFrustum_min; c.viewFrustum_max = params->viewFrustum_max;
            }
            c.use_swapping = useSwapping ? 1 : 0;
            c.voxel_rgb = TVoxel::hasColorInformation ? 1 : 0;    // Scene<Voxel_s_rgb, ...>
            tf_engine_check(tf_create(&c, &ctx_), "Scene: tf_create");
            intr_ = tp.intr;
            if (useSwapping) globalCache = new GlobalCache<TVoxel>(ctx_);
        }
        ~Scene()
        {
            delete globalCache;
            tf_destroy(ctx_);
        }
        Scene(const Scene&) = delete;
        Scene& operator=(const Scene&) = delete;

        tf_ctx* context() const { return ctx_; }
        const Intr& intr() const { return intr_; }
        // LocalVBA::lastFreeBlockId, VoxelBlockHash::lastFreeExcessListId, RenderState_VH::noVisibleEntries
        tf_stats counters() const
        {
            tf_stats s;
            tf_engine_check(tf_get_stats(ctx_, &s), "tf_get_stats");
            return s;
        }

    private:
        tf_ctx* ctx_ = nullptr;
        Intr intr_;
    };

    // RenderState (RenderState.hpp:12-88) / RenderState_VH (RenderState_VH.hpp:15-61): handles
    // (the state itself lives in the scene's context, see the header comment)
    class RenderState
    {
    public:
        RenderState(const Vector2i& imgSize, float vf_min, float vf_max) : imgSize_(imgSize), vf_min_(vf_min), vf_max_(vf_max) {}
        virtual ~RenderState() {}
        const Vector2i& imgSize() const { return imgSize_; }
    private:
        Vector2i imgSize_;
        float vf_min_, vf_max_;
    };
    class RenderState_VH : public RenderState
    {
    public:
        RenderState_VH(int noTotalEntries, const Vector2i& imgSize, float vf_min, float vf_max)
            : RenderState(imgSize, vf_min, vf_max), noTotalEntries_(noTotalEntries) {}
    private:
        int noTotalEntries_;
    };

    namespace detail
    {
        inline void intr4(const Intr& i, float out[4]) { out[0] = i.fx; out[1] = i.fy; out[2] = i.cx; out[3] = i.cy; }
        inline void rt_of(const Affine3f& a, float rt[12]) { affine_to_rt(a, rt); }
        inline void rt_of(const Matrix4f& m, float rt[12]) { m.toRt(rt); }
    }

    // SceneReconstructionEngine_CUDA<TVoxel, TIndex> (SceneReconstructionEngine_host.hpp:42-74)
    template <class TVoxel, class TIndex>
    class SceneReconstructionEngine_CUDA
    {
    public:
        // ResetScene (SceneReconstructionEngine_host.cu:51-73)
        void ResetScene(Scene<TVoxel, TIndex>* scene)
        {
            tf_engine_check(tf_stage_reset_scene(scene->context()), "ResetScene");
        }
        // AllocateSceneFromDepth (:75-195); pose is world -> camera, as TopFu passes it
        void AllocateSceneFromDepth(Scene<TVoxel, TIndex>* scene, const Intr intr, const Affine3f pose, cuda::Dists& dist,
                                    const RenderState* = nullptr, bool onlyUpdateVisibleList = false,
                                    bool resetVisibleList = false)
        {
            float in[4], rt[12];
            detail::intr4(intr, in);
            detail::rt_of(pose, rt);
            tf_engine_check(tf_scene_alloc(scene->context(), in, rt, dist.ptr(), dist.step(), onlyUpdateVisibleList ? 1 : 0,
                                           resetVisibleList ? 1 : 0), "AllocateSceneFromDepth");
        }
        // IntegrateIntoScene (:197-251)
        void IntegrateIntoScene(Scene<TVoxel, TIndex>* scene, const Intr intr, const Affine3f pose, cuda::Dists& dist,
                                const RenderState* = nullptr)
        {
            float in[4], rt[12];
            detail::intr4(intr, in);
            detail::rt_of(pose, rt);
            tf_engine_check(tf_scene_integrate(scene->context(), in, rt, dist.ptr(), dist.step()), "IntegrateIntoScene");
        }
        // with the view's RGBA image (view->rgb, :225): the colour update of a Voxel_s_rgb scene
        void IntegrateIntoScene(Scene<TVoxel, TIndex>* scene, const Intr intr, const Affine3f pose, cuda::Dists& dist,
                                const cuda::image4u& rgb, const RenderState* = nullptr)
        {
            float in[4], rt[12];
            detail::intr4(intr, in);
            detail::rt_of(pose, rt);
            tf_engine_check(tf_scene_integrate_rgb(scene->context(), in, rt, dist.ptr(), dist.step(),
                                                   reinterpret_cast<const uint8_t*>(rgb.ptr()), rgb.step()),
                            "IntegrateIntoScene(rgb)");
        }
    };

    // SwappingEngine_CUDA<TVoxel, TIndex>: the engine of the GlobalCache's lineage (InfiniTAM
    // ITMSwappingEngine_CUDA; its instantiation is commented out in the reference,
    // CUDAInstantiations.cu:8), called after IntegrateIntoScene on a swapping scene
    template <class TVoxel, class TIndex>
    class SwappingEngine_CUDA
    {
    public:
        // stored blocks of the entries marked "needed" (state 1) merged into their active blocks
        void IntegrateGlobalIntoLocal(Scene<TVoxel, TIndex>* scene, RenderState* = nullptr)
        {
            tf_engine_check(tf_scene_swap_in(scene->context()), "IntegrateGlobalIntoLocal");
        }
        // active blocks not visible this frame moved to the cache, their VBA blocks freed
        void SaveToGlobalMemory(Scene<TVoxel, TIndex>* scene, RenderState* = nullptr)
        {
            tf_engine_check(tf_scene_swap_out(scene->context()), "SaveToGlobalMemory");
        }
    };

    // VisualisationEngine_CUDA<TVoxel, TIndex> (VisualisationEngine_CUDA.hpp:12-47)
    template <class TVoxel, class TIndex>
    class VisualisationEngine_CUDA
    {
    public:
        // CreateExpectedDepths (VisualisationEngine_CUDA.cu:119-173); pose is world -> camera
        void CreateExpectedDepths(const Scene<TVoxel, TIndex>* scene, const Affine3f pose, const Intr intrinsics,
                                  RenderState* = nullptr) const
        {
            float in[4], rt[12];
            detail::intr4(intrinsics, in);
            detail::rt_of(pose, rt);
            tf_engine_check(tf_vis_expected_depths(scene->context(), in, rt), "CreateExpectedDepths");
        }
        // RenderImage (:220-291, 423-429); pose is camera -> world (TopFu's Matrix4f(poses_.back()))
        void RenderImage(const Scene<TVoxel, TIndex>* scene, Matrix4f pose, const Vector4f intrinsics, RenderState* renderState,
                         cuda::image4u& outputImage,
                         IVisualisationEngine::RenderImageType type = IVisualisationEngine::RENDER_SHADED_GREYSCALE,
                         IVisualisationEngine::RenderRaycastSelection raycastType =
                             IVisualisationEngine::RENDER_FROM_NEW_RAYCAST) const
        {
            if (raycastType == IVisualisationEngine::RENDER_FROM_OLD_FORWARDPROJ)
                throw std::invalid_argument("RenderImage: RENDER_FROM_OLD_FORWARDPROJ is not on this path");
            (void)renderState;
            float in[4] = { intrinsics.x, intrinsics.y, intrinsics.z, intrinsics.w }, rt[12];
            detail::rt_of(pose, rt);
            tf_params p;
            tf_engine_check(tf_get_params(scene->context(), &p), "tf_get_params");
            outputImage.create(p.rows, p.cols);
            tf_engine_check(tf_vis_render_image(scene->context(), in, rt, (int)type,
                                                raycastType == IVisualisationEngine::RENDER_FROM_NEW_RAYCAST ? 1 : 0,
                                                reinterpret_cast<uint8_t*>(outputImage.ptr()), outputImage.step()),
                            "RenderImage");
        }
        // CreateICPMaps (:473-493 -> 323-360); pose is camera -> world
        void CreateICPMaps(const Scene<TVoxel, TIndex>* scene, const Matrix4f pose, const Intr intr, cuda::Cloud& points,
                           cuda::Normals& normals, RenderState* = nullptr) const
        {
            float in[4], rt[12];
            detail::intr4(intr, in);
            detail::rt_of(pose, rt);
            tf_params p;
            tf_engine_check(tf_get_params(scene->context(), &p), "tf_get_params");
            points.create(p.rows, p.cols);
            normals.create(p.rows, p.cols);
            tf_engine_check(tf_vis_icp_maps(scene->context(), in, rt, points.ptr(), points.step(), normals.ptr(),
                                            normals.step()), "CreateICPMaps");
        }
    };

    // cuda:: image processing (imgproc.hpp:9-31) on the legacy default stream
    namespace cuda
    {
        // computeDists (imgproc.cpp:44-48): mm -> m, >= 2047 mm or 0 -> -1
        inline void computeDists(const Depth& depth, Dists& dists, const Intr&)
        {
            dists.create(depth.rows(), depth.cols());
            tf_engine_check(tf_imgproc_compute_dists(depth.ptr(), depth.step(), dists.ptr(), dists.step(), depth.cols(),
                                                     depth.rows(), nullptr), "computeDists");
        }
        // depthBilateralFilter (imgproc.cpp:3-7); sigma_depth in metres
        inline void depthBilateralFilter(const Depth& in, Depth& out, int ksz, float sigma_spatial, float sigma_depth)
        {
            out.create(in.rows(), in.cols());
            tf_engine_check(tf_imgproc_bilateral(in.ptr(), in.step(), out.ptr(), out.step(), in.cols(), in.rows(), ksz,
                                                 sigma_spatial, sigma_depth, nullptr), "depthBilateralFilter");
        }
        // depthTruncation (imgproc.cpp:9-10); threshold in metres
        inline void depthTruncation(Depth& depth, float threshold)
        {
            tf_engine_check(tf_imgproc_truncate(depth.ptr(), depth.step(), depth.cols(), depth.rows(), threshold, nullptr),
                            "depthTruncation");
        }
        // depthBuildPyramid (imgproc.cpp:12-16)
        inline void depthBuildPyramid(const Depth& depth, Depth& pyramid, float sigma_depth)
        {
            pyramid.create(depth.rows() / 2, depth.cols() / 2);
            tf_engine_check(tf_imgproc_pyr_down(depth.ptr(), depth.step(), depth.cols(), depth.rows(), pyramid.ptr(),
                                                pyramid.step(), sigma_depth, nullptr), "depthBuildPyramid");
        }
        // computePointNormals (imgproc.cpp:31-41)
        inline void computePointNormals(const Intr& intr, const Depth& depth, Cloud& points, Normals& normals)
        {
            points.create(depth.rows(), depth.cols());
            normals.create(depth.rows(), depth.cols());
            const float in[4] = { intr.fx, intr.fy, intr.cx, intr.cy };
            tf_engine_check(tf_imgproc_point_normals(in, depth.ptr(), depth.step(), depth.cols(), depth.rows(), points.ptr(),
                                                     points.step(), normals.ptr(), normals.step(), nullptr),
                            "computePointNormals");
        }
        // resizePointsNormals (imgproc.cpp:64-73)
        inline void resizePointsNormals(const Cloud& points, const Normals& normals, Cloud& points_out, Normals& normals_out)
        {
            points_out.create(points.rows() / 2, points.cols() / 2);
            normals_out.create(normals.rows() / 2, normals.cols() / 2);
            tf_engine_check(tf_imgproc_resize_points_normals(points.ptr(), points.step(), normals.ptr(), normals.step(),
                                                             points.cols(), points.rows(), points_out.ptr(),
                                                             points_out.step(), normals_out.ptr(), normals_out.step(),
                                                             nullptr), "resizePointsNormals");
        }
        // waitAllDefaultStream (imgproc.cpp:18-19)
        inline void waitAllDefaultStream() { tf_engine_check(tf_imgproc_sync(nullptr), "waitAllDefaultStream"); }
    }
}
