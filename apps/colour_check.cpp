// colour_check.cpp -- the colour TSDF through both C++ APIs.  Every frame of a synthetic orbit
// (depth + the colour camera's RGBA view) goes through
//   A: tfusion::TopFu with params.integrate_colour, operator()(depth, rgba), and
//   B: the same frame over the engine API: a Scene<Voxel_s_rgb, VoxelBlockHash> with
//      SceneReconstructionEngine_CUDA::IntegrateIntoScene(..., rgb) (the view's colour) and the
//      rest of TopFu::operator()'s body as in engine_check.cpp,
// and after the run the two scenes must agree bit for bit -- hash, Voxel_s plane, colour plane --
// as must RenderImage(RENDER_COLOUR_FROM_VOLUME) from the last pose.  The colour camera sits
// 2.5 cm beside the depth camera with its own intrinsics (rgb_intr / depth_to_rgb).
//
//   ./colour_check [frames=24] [cols=320] [rows=240]
#include <tfusion/engines.hpp>

#include "synth_depth.hpp"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

using namespace tfusion;

static std::vector<unsigned char> download_ctx(tf_ctx* c, int which)
{
    size_t n = 0;
    tf_buffer_bytes(c, which, 0, &n);
    std::vector<unsigned char> h(n);
    if (tf_download(c, which, 0, h.data(), n) != TF_OK) std::printf("tf_download failed\n");
    return h;
}

int main(int argc, char** argv)
{
    const int frames = argc > 1 ? std::atoi(argv[1]) : 24;
    const int cols = argc > 2 ? std::atoi(argv[2]) : 320;
    const int rows = argc > 3 ? std::atoi(argv[3]) : 240;
    cuda::setDevice(0);

    TopFuParams p = TopFuParams::default_params();
    p.cols = cols;
    p.rows = rows;
    const double s = cols / 640.0;
    p.intr = Intr(504.261f * s, 503.905f * s, 352.457f * s, 272.202f * s);
    p.integrate_colour = true;
    p.rgb_intr = Intr(p.intr.fx * 1.03f, p.intr.fy * 1.03f, p.intr.cx - 3.5f, p.intr.cy + 2.25f);
    const double a = 1.0 * M_PI / 180.0;        // depth -> rgb: 1 deg about y, 2.5 cm along x
    const double DR[9] = { std::cos(a), 0, std::sin(a), 0, 1, 0, -std::sin(a), 0, std::cos(a) }, Dt[3] = { 0.025, 0.0, 0.004 };
    {
        float rt[12];
        for (int r = 0; r < 3; ++r) {
            for (int c = 0; c < 3; ++c) rt[4 * r + c] = (float)DR[3 * r + c];
            rt[4 * r + 3] = (float)Dt[r];
        }
        p.depth_to_rgb = affine_from_rt(rt);
    }

    TopFu topfu(p);                                                  // A
    Scene<Voxel_s_rgb, VoxelBlockHash> scene(p.sceneParams.get(), false, p);   // B
    SceneReconstructionEngine_CUDA<Voxel_s_rgb, VoxelBlockHash> sceneEngine;
    VisualisationEngine_CUDA<Voxel_s_rgb, VoxelBlockHash> visEngine;
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
    int frame_counter = 0, fails = 0, n_ok = 0;
    sceneEngine.ResetScene(&scene);

    cuda::Depth depth_device;
    cuda::image4u rgb_device, image;
    std::vector<unsigned short> depth;
    std::vector<unsigned char> rgb;
    for (int i = 0; i < frames; ++i) {
        double R[9], t[3];
        tfusion_apps::orbit_pose(i, R, t);
        tfusion_apps::render_depth(R, t, cols, rows, p.intr, depth);
        // the colour camera: c2w_d * D^-1
        double Rc[9], tc[3];
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) {
                Rc[3 * r + c] = 0;
                for (int k = 0; k < 3; ++k) Rc[3 * r + c] += R[3 * r + k] * DR[3 * c + k];
            }
        for (int r = 0; r < 3; ++r) tc[r] = t[r] - (Rc[3 * r] * Dt[0] + Rc[3 * r + 1] * Dt[1] + Rc[3 * r + 2] * Dt[2]);
        tfusion_apps::render_colour(Rc, tc, cols, rows, p.rgb_intr, rgb);
        depth_device.upload(depth.data(), (size_t)cols * 2, rows, cols);
        rgb_device.upload(rgb.data(), (size_t)cols * 4, rows, cols);

        const bool okA = topfu(depth_device, rgb_device);

        // B: topfu.cpp:161-330 with the colour view
        bool okB = true;
        cuda::computeDists(depth_device, dists, p.intr);
        cuda::depthBilateralFilter(depth_device, curr.depth_pyr[0], p.bilateral_kernel_size, p.bilateral_sigma_spatial,
                                   p.bilateral_sigma_depth);
        if (p.icp_truncate_depth_dist > 0) cuda::depthTruncation(curr.depth_pyr[0], p.icp_truncate_depth_dist);
        for (int l = 1; l < LEVELS; ++l) cuda::depthBuildPyramid(curr.depth_pyr[l - 1], curr.depth_pyr[l], p.bilateral_sigma_depth);
        for (int l = 0; l < LEVELS; ++l) cuda::computePointNormals(p.intr(l), curr.depth_pyr[l], curr.points_pyr[l], curr.normals_pyr[l]);
        cuda::waitAllDefaultStream();
        if (frame_counter == 0) {
            sceneEngine.AllocateSceneFromDepth(&scene, p.intr, poses.back(), dists, &renderState);
            sceneEngine.IntegrateIntoScene(&scene, p.intr, poses.back(), dists, rgb_device, &renderState);
            curr.points_pyr.swap(prev.points_pyr);
            curr.normals_pyr.swap(prev.normals_pyr);
            ++frame_counter;
        } else {
            Affine3f affine;
            const bool ok = icp.estimateTransform(affine, p.intr, curr.points_pyr, curr.normals_pyr, prev.points_pyr,
                                                  prev.normals_pyr);
            poses.push_back(poses.back() * affine);
            const Affine3f pose = poses.back();
            if (!ok) {
                frame_counter = 0;
                poses.clear();
                poses.push_back(Affine3f::Identity());
                sceneEngine.ResetScene(&scene);
                okB = false;
            } else {
                sceneEngine.AllocateSceneFromDepth(&scene, p.intr, pose.inv(), dists, &renderState);
                sceneEngine.IntegrateIntoScene(&scene, p.intr, pose.inv(), dists, rgb_device, &renderState);
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
            }
        }
        if (okA != okB) { ++fails; std::printf("MISMATCH frame %d ok: TopFu %d engines %d\n", i, (int)okA, (int)okB); }
        n_ok += okA;
    }
    // the scenes: hash, Voxel_s plane, colour plane
    const int bufs[3] = { TF_BUF_HASH, TF_BUF_VBA, TF_BUF_VBA_RGB };
    const char* names[3] = { "hash", "voxel plane", "colour plane" };
    long coloured = 0;
    for (int b = 0; b < 3; ++b) {
        const std::vector<unsigned char> ha = download_ctx(topfu.handle(), bufs[b]);
        const std::vector<unsigned char> hb = download_ctx(scene.context(), bufs[b]);
        if (ha.size() != hb.size() || std::memcmp(ha.data(), hb.data(), ha.size())) { ++fails; std::printf("MISMATCH %s\n", names[b]); }
        if (bufs[b] == TF_BUF_VBA_RGB)
            for (size_t k = 3; k < ha.size(); k += 4) coloured += ha[k] > 0;
    }
    // RenderImage(RENDER_COLOUR_FROM_VOLUME) from the last pose through both APIs
    cuda::image4u ia, ib;
    topfu.renderImage(ia, TopFu::RENDER_COLOUR_FROM_VOLUME);
    visEngine.RenderImage(&scene, Matrix4f::fromAffine(poses.back()), Vector4f(p.intr.fx, p.intr.fy, p.intr.cx, p.intr.cy),
                          &renderState, ib, IVisualisationEngine::RENDER_COLOUR_FROM_VOLUME,
                          IVisualisationEngine::RENDER_FROM_NEW_RAYCAST);
    std::vector<Vector4u> va((size_t)rows * cols), vb((size_t)rows * cols);
    ia.download(va.data(), sizeof(Vector4u) * cols);
    ib.download(vb.data(), sizeof(Vector4u) * cols);
    long lit = 0;
    for (const Vector4u& v : va) lit += v.w == 255;
    if (std::memcmp(va.data(), vb.data(), va.size() * sizeof(Vector4u))) { ++fails; std::printf("MISMATCH colour render\n"); }
    std::printf("colour_check frames %d ok %d coloured voxels %ld lit pixels %ld: %s\n", frames, n_ok, coloured, lit,
                fails ? "MISMATCH" : "MATCH");
    return fails ? 1 : 0;
}
