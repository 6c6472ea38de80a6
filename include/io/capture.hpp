// io/capture.hpp -- the capture interface apps/demo.cpp includes (tfusion/include/io/capture.hpp,
// OpenNISource, :8-41).  OpenNI capture is out of scope for this build: the class
// keeps the reference's interface so demo.cpp compiles unchanged, and reports that no OpenNI
// device or .oni file can be opened.  Frames come from PGM / PPM files instead (demo.cpp's own
// loop reads them with cv::imread; tfusion/io.hpp reads them without OpenCV).
#pragma once
#include <cstdio>
#include <string>

#include <tfusion/types.hpp>

namespace tfusion
{
    struct PixelRGB { unsigned char r, g, b; };    // types.hpp:50-53

    class OpenNISource
    {
    public:
        typedef tfusion::PixelRGB RGB24;
        enum { PROP_OPENNI_REGISTRATION_ON = 104 };

        OpenNISource() {}
        explicit OpenNISource(int device) { open(device); }
        explicit OpenNISource(const std::string& oni_filename, bool repeat = false) { open(oni_filename, repeat); }
        ~OpenNISource() { release(); }

        void open(int device)
        {
            std::fprintf(stderr, "OpenNISource: device %d: this build has no OpenNI capture (frames: PGM/PPM files)\n", device);
        }
        void open(const std::string& oni_filename, bool /*repeat*/ = false)
        {
            std::fprintf(stderr, "OpenNISource: %s: this build has no OpenNI capture (frames: PGM/PPM files)\n",
                         oni_filename.c_str());
        }
        void release() {}
#if TFUSION_OPENCV_TYPES
        bool grab(cv::Mat& /*depth*/, cv::Mat& /*image*/) { return false; }
#endif
        bool setRegistration(bool /*value*/ = false) { return false; }

        // parameters taken from camera / oni (capture.hpp:27-32): none without a device
        int shadow_value = 0, no_sample_value = 0;
        float depth_focal_length_VGA = 0.f;
        float baseline = 0.f;
        double pixelSize = 0.0;
        unsigned short max_depth = 0;
    };
}
