// synth_depth.hpp -- the synthetic C2 scene of SURVEY.md §8d for the C++ apps: an analytic room
// (+ sphere) rendered from a camera pose, and the orbit the bench / tests use (0.25 deg per
// frame about a pivot 1.2 m ahead, swinging +-25 deg).  Same geometry as topfusion_amd/synth.py (no noise).
#pragma once
#include <tfusion/types.hpp>

#include <cmath>
#include <limits>
#include <vector>

namespace tfusion_apps
{
using tfusion::Intr;

// analytic room (+ sphere) seen from camera->world pose (R, t); uint16 millimetres
inline void render_depth(const double R[9], const double t[3], int cols, int rows, const Intr& in,
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

// the colour camera's view of the same room (pose R, t camera -> world): the texture of
// topfusion_amd/synth.py render_colour, RGBA, black where nothing is hit
inline void render_colour(const double R[9], const double t[3], int cols, int rows, const Intr& in,
                          std::vector<unsigned char>& out)
{
    out.assign((size_t)cols * rows * 4, 0);
    const int axes[6] = { 2, 1, 0, 0, 1, 2 };
    const double offs[6] = { 1.8, 0.6, -0.8, 1.1, -0.9, -0.6 };
    const double c[3] = { 0.15, 0.25, 1.3 }, r = 0.3, two_pi = 2.0 * M_PI;
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
            const double disc = b * b - a * (oc[0] * oc[0] + oc[1] * oc[1] + oc[2] * oc[2] - r * r);
            if (disc >= 0) {
                const double t0 = (-b - std::sqrt(disc)) / a;
                if (t0 > 1e-6 && t0 < best) best = t0;
            }
            if (!std::isfinite(best)) continue;
            const double p[3] = { t[0] + dw[0] * best, t[1] + dw[1] * best, t[2] + dw[2] * best };
            unsigned char* o = &out[4 * ((size_t)v * cols + u)];
            o[0] = (unsigned char)std::nearbyint(127.5 + 120 * std::sin(two_pi * p[0] / 0.13));
            o[1] = (unsigned char)std::nearbyint(127.5 + 120 * std::sin(two_pi * (p[1] + p[2]) / 0.17));
            o[2] = (unsigned char)std::nearbyint(127.5 + 120 * std::cos(two_pi * (p[2] - p[0]) / 0.23));
            o[3] = 255;
        }
}

// orbit angle of frame i in degrees: a ping-pong between -25 and +25 deg at 0.25 deg per frame
// (synth.orbit_angle_deg), so the camera stays inside the room however long the stream is
inline double orbit_angle_deg(int i)
{
    const double A = 25.0, a = 0.25 * i, ph = std::fmod(a, 4.0 * A);
    if (ph <= A) return ph;
    if (ph <= 3.0 * A) return 2.0 * A - ph;
    return ph - 4.0 * A;
}

// frame i of the orbit: camera -> world rotation about y and translation
inline void orbit_pose(int i, double R[9], double t[3])
{
    const double ang = orbit_angle_deg(i) * M_PI / 180.0, ca = std::cos(ang), sa = std::sin(ang);
    const double Rr[9] = { ca, 0, sa, 0, 1, 0, -sa, 0, ca };
    for (int k = 0; k < 9; ++k) R[k] = Rr[k];
    t[0] = -sa * 1.2; t[1] = 0.0; t[2] = 1.2 - ca * 1.2;      // orbit about a pivot 1.2 m ahead
}
}
