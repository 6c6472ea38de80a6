// demo_headless.cpp -- apps/demo.cpp's loop (tfusion/apps/demo.cpp:27-168) without OpenCV /
// OpenNI: depth frames are uploaded with cuda::Depth::upload, fused by TopFu::operator(), and
// the grey rendering is fetched with renderImage + download, exactly as the reference demo
// does.  Frames are either synthetic (the C2 orbit of SURVEY.md §8d, rendered analytically on
// the host) or read from a numbered 16-bit PGM sequence like the reference demo's
// "%04d.pgm" / "%04d.ppm" pairs (demo.cpp:91-97) through tfusion::io::FrameSequenceSource.
//
//   ./demo_headless [frames=100] [cols=640] [rows=480]
//   ./demo_headless --pgm 'dir/%04d.pgm' [--ppm 'dir/%04d.ppm'] [max_frames]
#include <tfusion/io.hpp>
#include <tfusion/topfu.hpp>

#include "synth_depth.hpp"

#include <cstring>
#include <string>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <limits>
#include <vector>

using namespace tfusion;

int main(int argc, char** argv)
{
    std::string pgm, ppm;
    std::vector<const char*> pos;
    for (int i = 1; i < argc; ++i) {
        if (!std::strcmp(argv[i], "--pgm") && i + 1 < argc) pgm = argv[++i];
        else if (!std::strcmp(argv[i], "--ppm") && i + 1 < argc) ppm = argv[++i];
        else pos.push_back(argv[i]);
    }
    int frames = pos.size() > 0 ? std::atoi(pos[0]) : (pgm.empty() ? 100 : 1 << 30);
    int cols = pos.size() > 1 ? std::atoi(pos[1]) : 640;
    int rows = pos.size() > 2 ? std::atoi(pos[2]) : 480;
    io::FrameSequenceSource source(pgm, ppm);
    std::vector<unsigned short> depth;
    std::vector<unsigned char> image;
    bool have_first = false;
    if (!pgm.empty()) {                        // frame size from the first file
        if (!source.grab(depth, image)) { std::fprintf(stderr, "no frame %s\n", pgm.c_str()); return 1; }
        cols = source.cols(); rows = source.rows();
        have_first = true;
    }

    int device = 0;
    cuda::setDevice(device);
    cuda::printShortCudaDeviceInfo(device);
    if (cuda::checkIfPreFermiGPU(device)) return 1;

    TopFuParams params = TopFuParams::default_params();
    params.cols = cols;
    params.rows = rows;
    const double s = cols / 640.0;
    params.intr = Intr(504.261f * s, 503.905f * s, 352.457f * s, 272.202f * s);
    TopFu::Ptr topfu(new TopFu(params));

    cuda::Depth depth_device;
    cuda::image4u view_device;
    std::vector<unsigned char> view_host((size_t)cols * rows * 4);
    double time_ms = 0;
    int n_ok = 0, n = 0;
    for (int i = 0; i < frames; ++i) {
        if (!pgm.empty()) {
            if (!have_first && !source.grab(depth, image)) break;         // end of the sequence
            have_first = false;
            if (source.cols() != cols || source.rows() != rows) { std::fprintf(stderr, "frame size changed\n"); return 1; }
        } else {
            double R[9], t[3];
            tfusion_apps::orbit_pose(i, R, t);
            tfusion_apps::render_depth(R, t, cols, rows, params.intr, depth);
        }
        ++n;
        depth_device.upload(depth.data(), (size_t)cols * 2, rows, cols);
        bool has_image;
        {
            SampledScopeTime fps(time_ms); (void)fps;
            has_image = (*topfu)(depth_device);
        }
        if (has_image) {
            ++n_ok;
            topfu->renderImage(view_device);
            view_device.download(view_host.data(), (size_t)cols * 4);
        }
    }
    const Affine3f pose = topfu->getCameraPose();
    const tf_stats st = topfu->stats();
    std::printf("frames %d ok %d resets %d visible %d  pose t = (%.4f %.4f %.4f)\n", n, n_ok, st.n_resets,
                st.noVisibleEntries, pose.translation()[0], pose.translation()[1], pose.translation()[2]);
    long lit = 0;
    for (size_t k = 0; k < view_host.size(); k += 4) lit += view_host[k] > 0;
    std::printf("rendered pixels lit: %ld of %d\n", lit, cols * rows);
    return n_ok > 0 && lit > 0 ? 0 : 2;
}
