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

#include <cstring>
#include <string>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <limits>
#include <vector>

using namespace tfusion;

// analytic room (+ sphere) seen from camera->world pose (R, t); uint16 millimetres
static void render_depth(const double R[9], const double t[3], int cols, int rows, const Intr& in,
                         std::vector<unsigned short>& out)
{
    out.assign((size_t)cols * rows, 0);
    const int axes[6] = { 2, 1, 0, 0, 1, 2 };
    const double offs[6] = { 1.8, 0.6, -0.8, 1.1, -0.9, -0.6 };
    const double c[3] = { 0.15, 0.25, 1.3 }, r = 0.3;
    for (int v = 0; v < rows; ++v)
        for (int u = 0; u < cols; ++u) {
            const double dc[3] = { (u - in.cx) / in.fx, (v - in.cy) / in.fy, 1.0 };
            double dw[3];
            for (int i = 0; i < 3; ++i) dw[i] = R[i * 3 + 0] * dc[0] + R[i * 3 + 1] * dc[1] + R[i * 3 + 2] * dc[2];
            double best = std::numeric_limits<double>::infinity();
            for (int p = 0; p < 6; ++p) {
                const double tt = (offs[p] - t[axes[p]]) / dw[axes[p]];
                if (tt > 1e-6 && tt < best) best = tt;
            }
            double oc[3] = { t[0] - c[0], t[1] - c[1], t[2] - c[2] };
            const double b = dw[0] * oc[0] + dw[1] * oc[1] + dw[2] * oc[2];
            const double a = dw[0] * dw[0] + dw[1] * dw[1] + dw[2] * dw[2];
            const double cc = oc[0] * oc[0] + oc[1] * oc[1] + oc[2] * oc[2] - r * r;
            const double disc = b * b - a * cc;
            if (disc >= 0) {
                const double t0 = (-b - std::sqrt(disc)) / a;
                if (t0 > 1e-6 && t0 < best) best = t0;
            }
            if (std::isfinite(best)) {
                const double mm = std::nearbyint(best * 1000.0);
                out[(size_t)v * cols + u] = (unsigned short)(mm > 65535 ? 65535 : mm);
            }
        }
}

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
            const double ang = 0.25 * i * M_PI / 180.0, ca = std::cos(ang), sa = std::sin(ang);
            const double R[9] = { ca, 0, sa, 0, 1, 0, -sa, 0, ca };
            const double t[3] = { -sa * 1.2, 0.0, 1.2 - ca * 1.2 };     // orbit about a pivot 1.2 m ahead
            render_depth(R, t, cols, rows, params.intr, depth);
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
