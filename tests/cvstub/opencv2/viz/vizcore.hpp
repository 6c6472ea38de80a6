// TEST-ONLY stand-in for the cv::viz declarations apps/demo.cpp uses (OpenCV viz/types.hpp,
// widgets.hpp, viz3d.hpp: KeyboardEvent, Color, WCube, WCoordinateSystem, Viz3d), for the
// compile-only test tests/test_cpp_api.py::test_reference_demo_compiles.  Never used by the product.
#pragma once
#include "../core/core.hpp"
#include "../core/affine.hpp"

namespace cv
{
namespace viz
{
    struct Color {
        double v[3] = { 0, 0, 0 };
        static Color apricot() { Color c; c.v[0] = 177; c.v[1] = 206; c.v[2] = 251; return c; }
        static Color white() { Color c; c.v[0] = c.v[1] = c.v[2] = 255; return c; }
    };
    struct KeyboardEvent {
        enum { NONE = 0, ALT = 1, CTRL = 2, SHIFT = 4 };
        enum Action { KEY_UP = 0, KEY_DOWN = 1 };
        Action action;
        String symbol;
        unsigned char code;
        int modifiers;
    };
    struct Widget {};
    struct Widget3D : Widget {};
    struct WCube : Widget3D {
        WCube(const Vec3d& min_point = Vec3d::all(-0.5), const Vec3d& max_point = Vec3d::all(0.5),
              bool wire_frame = true, const Color& color = Color::white())
        { (void)min_point; (void)max_point; (void)wire_frame; (void)color; }
    };
    struct WCoordinateSystem : Widget3D {
        explicit WCoordinateSystem(double scale = 1.0) { (void)scale; }
    };
    class Viz3d {
    public:
        typedef void (*KeyboardCallback)(const KeyboardEvent&, void*);
        Viz3d() {}
        void showWidget(const String& id, const Widget& widget, const Affine3d& pose = Affine3d::Identity())
        { (void)id; (void)widget; (void)pose; }
        void registerKeyboardCallback(KeyboardCallback callback, void* cookie = 0) { (void)callback; (void)cookie; }
        bool wasStopped() const { return true; }
        void setViewerPose(const Affine3d& pose) { (void)pose; }
        void spinOnce(int time = 1, bool force_redraw = false) { (void)time; (void)force_redraw; }
    };
}
}
