// engine_check.cpp -- the L4 engine API against the pipeline API.  Every frame of a synthetic
// orbit goes through
//   A: tfusion::TopFu::operator() (include/tfusion/topfu.hpp), and
//   B: TopFu::operator()'s body spelled out over the engine API (include/tfusion/engines.hpp):
//      cuda::computeDists / depthBilateralFilter / depthTruncation / depthBuildPyramid /
//      computePointNormals, cuda::ProjectiveICP::estimateTransform (a stand-alone tracker with
//      TopFu's parameters), SceneReconstructionEngine_CUDA::{ResetScene,
//      AllocateSceneFromDepth, IntegrateIntoScene}, VisualisationEngine_CUDA::{RenderImage,
//      CreateExpectedDepths, CreateICPMaps}, cuda::resizePointsNormals -- in the order of
//      tfusion/src/topfu.cpp:161-330 (reset(): :141-152),
// and the two must agree bit for bit after every frame: the frame's bool, the pose, the
// allocation / visibility counters, the in-frame renderImage grey image, and at the end the
// previous-frame ICP maps.  Also checks TopFu::icp()'s parameters and the SampledScopeTime
// static counter (prints once at the 34th scope).
//
//   ./engine_check [frames=40] [cols=320] [rows=240]
#include <tfusion/engines.hpp>

#include "synth_depth.hpp"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

using namespace tfusion;

static int fails = 0;
#define EXPECT(cond, ...)                                     \
    do {                                                      \
        if (!(cond)) {                                        \
            ++fails;                                          \
            std::printf("MISMATCH: " __VA_ARGS__);            \
            std::printf("\n");                                \
        }                                                     \
    } while (0)

template <typename T>
static std::vector<T> download(const cuda::DeviceArray2D<T>& a)
{
    std::vector<T> h((size_t)a.rows() * a.cols());
    a.download(h.data(), sizeof(T) * (size_t)a.cols());
    return h;
}

static std::vector<unsigned char> download_ctx(tf_ctx* c, int which, int level = 0)
{
    size_t n = 0;
    tf_buffer_bytes(c, which, level, &n);
    std::vector<unsigned char> h(n);
    if (tf_download(c, which, level, h.data(), n) != TF_OK) std::printf("tf_download failed\n");
    return h;
}

int main(int argc, char** argv)
{
    const int frames = argc > 1 ? std::atoi(argv[1]) : 40;
    const int cols = argc > 2 ? std::atoi(argv[2]) : 320;
    const int rows = argc > 3 ? std::atoi(argv[3]) : 240;
    // "nowait": no cuda::waitAllDefaultStream() between the imgproc calls (legacy default
    // stream) and the engines (the context's own stream): the entry points must order
    // themselves after the caller's stream-0 work
    const bool wait_default = !(argc > 4 && std::strcmp(argv[4], "nowait") == 0);
    cuda::setDevice(0);

    TopFuParams p = TopFuParams::default_params();
    p.cols = cols;
    p.rows = rows;
    const double s = cols / 640.0;
    p.intr = Intr(504.261f * s, 503.905f * s, 352.457f * s, 272.202f * s);

    // A: the pipeline
    TopFu topfu(p);
    EXPECT(topfu.icp().getDistThreshold() == p.icp_dist_thres, "icp().getDistThreshold");
    EXPECT(topfu.icp().getAngleThreshold() == p.icp_angle_thres, "icp().getAngleThreshold");
    EXPECT(topfu.icp().getUsedLevelsNum() == 3, "icp().getUsedLevelsNum");

    // B: TopFu's members and constructor (topfu.cpp:55-84, 104-139)
    Scene<Voxel_s, VoxelBlockHash> scene(p.sceneParams.get(), false, p);
    SceneReconstructionEngine_CUDA<Voxel_s, VoxelBlockHash> sceneEngine;
    VisualisationEngine_CUDA<Voxel_s, VoxelBlockHash> visEngine;
    RenderState_VH renderState(VoxelBlockHash::noTotalEntries, Vector2i(cols, rows), p.sceneParams->viewFrustum_min,
                               p.sceneParams->viewFrustum_max);
    cuda::ProjectiveICP icp;
    icp.setDistThreshold(p.icp_dist_thres);
    icp.setAngleThreshold(p.icp_angle_thres);
    icp.setIterationsNum(p.icp_iter_num);
    const int LEVELS = icp.getUsedLevelsNum();
    cuda::Dists dists;
    cuda::Frame curr, prev;
    curr.depth_pyr.resize(LEVELS); curr.points_pyr.resize(LEVELS); curr.normals_pyr.resize(LEVELS);
    prev.depth_pyr.resize(LEVELS); prev.points_pyr.resize(LEVELS); prev.normals_pyr.resize(LEVELS);
    std::vector<Affine3f> poses{ Affine3f::Identity() };
    int frame_counter = 0;
    sceneEngine.ResetScene(&scene);

    cuda::Depth depth_device;
    cuda::image4u image;
    std::vector<unsigned short> depth;
    double time_ms = 0;
    int n_ok = 0, n_reset = 0;
    for (int i = 0; i < frames; ++i) {
        double R[9], t[3];
        tfusion_apps::orbit_pose(i, R, t);
        tfusion_apps::render_depth(R, t, cols, rows, p.intr, depth);
        depth_device.upload(depth.data(), (size_t)cols * 2, rows, cols);

        bool okA;
        {
            SampledScopeTime fps(time_ms);
            okA = topfu(depth_device);
        }

        // ---- B: topfu.cpp:161-330
        bool okB = true, tracked = false;
        cuda::computeDists(depth_device, dists, p.intr);
        cuda::depthBilateralFilter(depth_device, curr.depth_pyr[0], p.bilateral_kernel_size, p.bilateral_sigma_spatial,
                                   p.bilateral_sigma_depth);
        if (p.icp_truncate_depth_dist > 0) cuda::depthTruncation(curr.depth_pyr[0], p.icp_truncate_depth_dist);
        for (int l = 1; l < LEVELS; ++l) cuda::depthBuildPyramid(curr.depth_pyr[l - 1], curr.depth_pyr[l], p.bilateral_sigma_depth);
        for (int l = 0; l < LEVELS; ++l) cuda::computePointNormals(p.intr(l), curr.depth_pyr[l], curr.points_pyr[l], curr.normals_pyr[l]);
        if (wait_default) cuda::waitAllDefaultStream();
        if (frame_counter == 0) {
            sceneEngine.AllocateSceneFromDepth(&scene, p.intr, poses.back(), dists, &renderState);
            sceneEngine.IntegrateIntoScene(&scene, p.intr, poses.back(), dists, &renderState);
            curr.points_pyr.swap(prev.points_pyr);
            curr.normals_pyr.swap(prev.normals_pyr);
            ++frame_counter;
        } else {
            Affine3f affine;
            const bool ok = icp.estimateTransform(affine, p.intr, curr.points_pyr, curr.normals_pyr, prev.points_pyr,
                                                  prev.normals_pyr);
            poses.push_back(poses.back() * affine);
            const Affine3f pose = poses.back();
            if (!ok) {                                         // reset(), false (topfu.cpp:141-152, 263-264)
                frame_counter = 0;
                poses.clear();
                poses.push_back(Affine3f::Identity());
                sceneEngine.ResetScene(&scene);
                okB = false;
            } else {
                sceneEngine.AllocateSceneFromDepth(&scene, p.intr, pose.inv(), dists, &renderState);
                sceneEngine.IntegrateIntoScene(&scene, p.intr, pose.inv(), dists, &renderState);
                // renderImage (topfu.cpp:284-285, 332-377): the previous frame's range image
                const Matrix4f M_d = Matrix4f::fromAffine(pose);
                visEngine.RenderImage(&scene, M_d, Vector4f(p.intr.fx, p.intr.fy, p.intr.cx, p.intr.cy), &renderState,
                                      image, IVisualisationEngine::RENDER_SHADED_GREYSCALE,
                                      IVisualisationEngine::RENDER_FROM_NEW_RAYCAST);
                visEngine.CreateExpectedDepths(&scene, pose.inv(), p.intr, &renderState);
                visEngine.CreateICPMaps(&scene, M_d, p.intr, prev.points_pyr[0], prev.normals_pyr[0], &renderState);
                for (int l = 1; l < LEVELS; ++l)
                    cuda::resizePointsNormals(prev.points_pyr[l - 1], prev.normals_pyr[l - 1], prev.points_pyr[l],
                                              prev.normals_pyr[l]);
                ++frame_counter;
                tracked = true;
            }
        }

        // ---- compare
        EXPECT(okA == okB, "frame %d ok: TopFu %d engines %d", i, (int)okA, (int)okB);
        n_ok += okA;
        n_reset += !okA;
        const Affine3f pa = topfu.getCameraPose(), pb = poses.back();
        EXPECT(std::memcmp(pa.matrix.val, pb.matrix.val, sizeof(float) * 12) == 0, "frame %d pose", i);
        const tf_stats sa = topfu.stats(), sb = scene.counters();
        EXPECT(sa.lastFreeBlockId == sb.lastFreeBlockId && sa.lastFreeExcessListId == sb.lastFreeExcessListId &&
                   sa.noVisibleEntries == sb.noVisibleEntries,
               "frame %d counters: TopFu (%d %d %d) engines (%d %d %d)", i, sa.lastFreeBlockId, sa.lastFreeExcessListId,
               sa.noVisibleEntries, sb.lastFreeBlockId, sb.lastFreeExcessListId, sb.noVisibleEntries);
        if (tracked) {
            const std::vector<unsigned char> ga = download_ctx(topfu.handle(), TF_BUF_GREY);
            const std::vector<Vector4u> gb = download(image);
            EXPECT(ga.size() == gb.size() * 4 && std::memcmp(ga.data(), gb.data(), ga.size()) == 0,
                   "frame %d renderImage grey", i);
        }
    }
    for (int l = 0; l < LEVELS; ++l) {
        const std::vector<unsigned char> pa = download_ctx(topfu.handle(), TF_BUF_PREV_POINTS, l);
        const std::vector<unsigned char> na = download_ctx(topfu.handle(), TF_BUF_PREV_NORMALS, l);
        const std::vector<Point> pb = download(prev.points_pyr[l]);
        const std::vector<Normal> nb = download(prev.normals_pyr[l]);
        EXPECT(pa.size() == pb.size() * 16 && std::memcmp(pa.data(), pb.data(), pa.size()) == 0, "final prev points L%d", l);
        EXPECT(na.size() == nb.size() * 16 && std::memcmp(na.data(), nb.data(), na.size()) == 0, "final prev normals L%d", l);
    }
    std::printf("engine_check frames %d ok %d resets %d: %s\n", frames, n_ok, n_reset, fails ? "MISMATCH" : "MATCH");
    return fails ? 1 : 0;
}
