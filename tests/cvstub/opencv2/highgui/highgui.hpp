// TEST-ONLY stand-in for the OpenCV highgui / imgcodecs calls apps/demo.cpp makes (imread, imshow,
// waitKey; OpenCV's public signatures), for the compile-only test
// tests/test_cpp_api.py::test_reference_demo_compiles.  Never used by the product.
#pragma once
#include <cstdio>
#include "../core/core.hpp"

namespace cv
{
    inline Mat imread(const String& filename, int flags = 1) { (void)filename; (void)flags; return Mat(); }
    inline void imshow(const String& winname, const Mat& mat) { (void)winname; (void)mat; }
    inline int waitKey(int delay = 0) { (void)delay; return -1; }
}
