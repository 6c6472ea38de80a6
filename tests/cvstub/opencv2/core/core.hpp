// TEST-ONLY stand-in for the few OpenCV core declarations include/tfusion/types.hpp names when
// TFUSION_OPENCV_TYPES is on (OpenCV is absent from this image).  Signatures follow OpenCV's
// public headers (core/matx.hpp, core/cvstd.hpp); no behaviour beyond what the compile-only test
// tests/test_cpp_api.py::test_cv_types_alias_compiles instantiates.  Never used by the product.
#pragma once
#include <memory>
#include <string>

namespace cv
{
    template <typename T> struct Ptr : std::shared_ptr<T> {        // cvstd.hpp (OpenCV >= 3: a shared_ptr)
        Ptr() = default;
        explicit Ptr(T* p) : std::shared_ptr<T>(p) {}
    };

    template <typename T, int m, int n> struct Matx {
        T val[m * n];
        Matx() { for (int i = 0; i < m * n; ++i) val[i] = T(0); }
        T operator()(int r, int c) const { return val[r * n + c]; }
        T& operator()(int r, int c) { return val[r * n + c]; }
    };
    typedef Matx<float, 3, 3> Matx33f;
    typedef Matx<float, 4, 4> Matx44f;
    typedef Matx<double, 4, 4> Matx44d;

    template <typename T, int cn> struct Vec : Matx<T, cn, 1> {
        Vec() {}
        Vec(T a, T b, T c) { this->val[0] = a; this->val[1] = b; this->val[2] = c; }
        template <typename T2> explicit Vec(const Vec<T2, cn>& o) { for (int i = 0; i < cn; ++i) this->val[i] = T(o.val[i]); }
        static Vec all(T v) { Vec r; for (int i = 0; i < cn; ++i) r.val[i] = v; return r; }
        T operator[](int i) const { return this->val[i]; }
        T& operator[](int i) { return this->val[i]; }
    };
    typedef Vec<float, 3> Vec3f;
    typedef Vec<double, 3> Vec3d;
    typedef Vec<int, 3> Vec3i;

    typedef std::string String;
    enum { CV_8U = 0, CV_16U = 2 };                                    // core/hal/interface.h depths
    struct Mat {                                                       // core/mat.hpp: what demo.cpp uses
        int rows = 0, cols = 0;
        unsigned char* data = nullptr;
        size_t step = 0;
        void create(int r, int c, int type) { rows = r; cols = c; (void)type; }
        template <typename T> T* ptr(int y = 0) { return reinterpret_cast<T*>(data + step * (size_t)y); }
        void convertTo(Mat& m, int rtype, double alpha = 1, double beta = 0) const { (void)m; (void)rtype; (void)alpha; (void)beta; }
    };
}
#define CV_8U 0
#define CV_16U 2
#define CV_8UC4 24
