// TEST-ONLY stand-in for cv::Affine3 (OpenCV core/affine.hpp): the members include/tfusion uses
// and the conversion to Affine3d that cv::viz's setViewerPose / showWidget take.  See core.hpp.
#pragma once
#include "core.hpp"

namespace cv
{
    template <typename T> struct Affine3 {
        typedef Matx<T, 3, 3> Mat3;
        typedef Matx<T, 4, 4> Mat4;
        typedef Vec<T, 3> Vec3;
        Mat4 matrix;
        Affine3() { for (int i = 0; i < 4; ++i) matrix.val[i * 5] = T(1); }
        Affine3(const Mat4& m) : matrix(m) {}
        static Affine3 Identity() { return Affine3(); }
        Mat3 rotation() const { Mat3 R; for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) R(r, c) = matrix(r, c); return R; }
        Vec3 translation() const { return Vec3(matrix(0, 3), matrix(1, 3), matrix(2, 3)); }
        Affine3 translate(const Vec3& t) const { Affine3 a = *this; for (int i = 0; i < 3; ++i) a.matrix(i, 3) += t[i]; return a; }
        Affine3 inv() const { return *this; }
        template <typename Y> operator Affine3<Y>() const
        {
            Matx<Y, 4, 4> m; for (int i = 0; i < 16; ++i) m.val[i] = Y(matrix.val[i]); return Affine3<Y>(m);
        }
    };
    template <typename T> Affine3<T> operator*(const Affine3<T>& a, const Affine3<T>& b) { (void)b; return a; }
    typedef Affine3<float> Affine3f;
    typedef Affine3<double> Affine3d;
}
