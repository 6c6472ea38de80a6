// TEST-ONLY compile check (tests/test_cpp_api.py::test_cv_types_alias_compiles): with
// TFUSION_OPENCV_TYPES on, the tfusion headers' value types ARE OpenCV's, and every use
// apps/demo.cpp makes of the API (demo.cpp:27-38, 100-115, 141-168) compiles -- written out here
// against the stand-in cv headers of this directory (OpenCV is absent from this image).
#include <type_traits>

#include <io/capture.hpp>
#include <tfusion/topfu.hpp>

using namespace tfusion;

static_assert(std::is_same<Affine3f, cv::Affine3f>::value, "Affine3f is cv::Affine3f");
static_assert(std::is_same<Vec3f, cv::Vec3f>::value, "Vec3f is cv::Vec3f");
static_assert(std::is_same<Vec3i, cv::Vec3i>::value, "Vec3i is cv::Vec3i");
static_assert(std::is_same<Mat3f, cv::Matx33f>::value, "Mat3f is cv::Matx33f");
static_assert(std::is_same<TopFu::Ptr, cv::Ptr<TopFu>>::value, "TopFu::Ptr is cv::Ptr<TopFu>");

static void viz_pose(const cv::Affine3d&) {}         // cv::viz::Viz3d::setViewerPose / showWidget's pose
static void viz_size(const cv::Vec3d&) {}            // cv::viz::WCube's corner

int main(int argc, char**)
{
    if (argc > 100) {                                 // compile-only: nothing runs
        int device = 0;
        cuda::setDevice(device);                      // demo.cpp:151-155
        cuda::printShortCudaDeviceInfo(device);
        if (cuda::checkIfPreFermiGPU(device)) return 1;
        OpenNISource capture;                         // demo.cpp:157-158
        capture.open(0);
        capture.setRegistration(true);                // demo.cpp:32
        TopFuParams params = TopFuParams::default_params();       // demo.cpp:29-30
        TopFu::Ptr topfu_ = TopFu::Ptr(new TopFu(params));
        viz_size(cv::Vec3d(params.volume_size));      // demo.cpp:34-35
        viz_pose(params.volume_pose);
        TopFu& topfu = *topfu_;
        cuda::Depth depth_device_;
        cuda::image4u view_device_;
        cuda::DeviceArray<Point> cloud_buffer;        // demo.cpp:146
        unsigned short host[16] = {};
        depth_device_.upload(host, 8, 2, 4);          // demo.cpp:100
        double time_ms = 0;
        bool has_image;
        {
            SampledScopeTime fps(time_ms); (void)fps;  // demo.cpp:102-105
            has_image = topfu(depth_device_);
        }
        if (has_image) {
            topfu.renderImage(view_device_);          // demo.cpp:51
            unsigned char view[64];
            view_device_.download(view, 16);
        }
        viz_pose(topfu.getCameraPose());              // demo.cpp:115
    }
    return 0;
}
