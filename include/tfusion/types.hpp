// tfusion/types.hpp -- host-side value types and device containers of the tfusion API,
// re-declared for the MI355X build (header-only, over include/tfusion_hip.h + HIP runtime).
//
// Mirrors tfusion/include/tfusion/types.hpp (Intr :19-26, Point/Normal :30-40, cuda typedefs
// :56-82, ScopeTime/SampledScopeTime :86-108) and tfusion/include/tfusion/cuda/device_array.hpp
// (DeviceArray2D create/upload/download/ptr/step/rows/cols/release, :19-222).
//
// The value types.  The reference typedefs them to OpenCV's (types.hpp:15-18: Mat3f = cv::Matx33f,
// Vec3f / Vec3i = cv::Vec3f / cv::Vec3i, Affine3f = cv::Affine3f; TopFu::Ptr = cv::Ptr<TopFu>,
// topfu.hpp:65), and apps/demo.cpp hands them to cv::viz (demo.cpp:35 volume_pose / volume_size,
// :115 getCameraPose()).  Where OpenCV's headers exist (TFUSION_OPENCV_TYPES, detected with
// __has_include(<opencv2/core/affine.hpp>); -DTFUSION_OPENCV_TYPES=0/1 overrides) they are the same
// cv:: types, so demo.cpp compiles unchanged.  Without OpenCV they are small own types with the
// cv:: member names the callers use (matrix, rotation(), translation(), inv(), operator*,
// Identity(), translate(), all()).  Code here touches them only through that common subset and
// the free functions affine_from_rt / affine_to_rt.
#pragma once
#include <hip/hip_runtime_api.h>

#include <chrono>
#include <cmath>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#ifndef TFUSION_OPENCV_TYPES
#  if defined(__has_include)
#    if __has_include(<opencv2/core/affine.hpp>)
#      define TFUSION_OPENCV_TYPES 1
#    endif
#  endif
#endif
#ifndef TFUSION_OPENCV_TYPES
#  define TFUSION_OPENCV_TYPES 0
#endif

#if TFUSION_OPENCV_TYPES
#include <opencv2/core/core.hpp>
#include <opencv2/core/affine.hpp>

namespace tfusion
{
    typedef cv::Matx33f Mat3f;                 // types.hpp:15-18
    typedef cv::Vec3f Vec3f;
    typedef cv::Vec3i Vec3i;
    typedef cv::Affine3f Affine3f;
    typedef cv::Matx44f Matx44f;
    template <class T> using SharedPtr = cv::Ptr<T>;     // TopFu::Ptr (topfu.hpp:65)
}
#else
namespace tfusion
{
    template <class T> using SharedPtr = std::shared_ptr<T>;

    struct Vec3f {
        float val[3];
        Vec3f() : val{ 0.f, 0.f, 0.f } {}
        Vec3f(float x, float y, float z) : val{ x, y, z } {}
        static Vec3f all(float v) { return Vec3f(v, v, v); }
        float& operator[](int i) { return val[i]; }
        float operator[](int i) const { return val[i]; }
    };
    struct Vec3i {
        int val[3];
        Vec3i() : val{ 0, 0, 0 } {}
        Vec3i(int x, int y, int z) : val{ x, y, z } {}
        static Vec3i all(int v) { return Vec3i(v, v, v); }
        int& operator[](int i) { return val[i]; }
        int operator[](int i) const { return val[i]; }
    };
    struct Mat3f {
        float val[9];   // row-major
        float operator()(int r, int c) const { return val[r * 3 + c]; }
        float& operator()(int r, int c) { return val[r * 3 + c]; }
    };

    // cv::Matx44f subset: row-major 4x4, element (r, c) = val[4r + c], zero-initialised like cv::Matx
    struct Matx44f {
        float val[16];
        Matx44f() : val{} {}
        float operator()(int r, int c) const { return val[r * 4 + c]; }
        float& operator()(int r, int c) { return val[r * 4 + c]; }
    };

    // cv::Affine3f subset: the 4x4 matrix of a rigid transform (camera -> world for poses), with
    // the member names the reference's callers use: matrix(r, c) (topfu.cpp:246-249),
    // rotation(), translation(), inv(), operator*, Identity(), translate()
    struct Affine3f {
        Matx44f matrix;
        Affine3f() { *this = Identity(); }
        explicit Affine3f(const Matx44f& m) : matrix(m) {}
        static Affine3f Identity()
        {
            Affine3f a(0);
            for (int i = 0; i < 4; ++i) a.matrix.val[i * 5] = 1.f;
            return a;
        }
        Mat3f rotation() const
        {
            Mat3f R;
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 3; ++c) R(r, c) = matrix(r, c);
            return R;
        }
        Vec3f translation() const { return Vec3f(matrix(0, 3), matrix(1, 3), matrix(2, 3)); }
        Affine3f translate(const Vec3f& t) const
        {
            Affine3f a = *this;
            a.matrix(0, 3) += t[0]; a.matrix(1, 3) += t[1]; a.matrix(2, 3) += t[2];
            return a;
        }
        Affine3f operator*(const Affine3f& b) const   // rigid composition in float
        {
            Affine3f o(0);
            for (int r = 0; r < 3; ++r) {
                for (int c = 0; c < 3; ++c)
                    o.matrix(r, c) = matrix(r, 0) * b.matrix(0, c) + matrix(r, 1) * b.matrix(1, c) + matrix(r, 2) * b.matrix(2, c);
                o.matrix(r, 3) = matrix(r, 0) * b.matrix(0, 3) + matrix(r, 1) * b.matrix(1, 3) + matrix(r, 2) * b.matrix(2, 3) +
                                 matrix(r, 3);
            }
            o.matrix(3, 3) = 1.f;
            return o;
        }
        Affine3f inv() const                            // rigid inverse [R^T | -R^T t]
        {
            Affine3f o(0);
            for (int r = 0; r < 3; ++r) {
                for (int c = 0; c < 3; ++c) o.matrix(r, c) = matrix(c, r);
                o.matrix(r, 3) = -(matrix(0, r) * matrix(0, 3) + matrix(1, r) * matrix(1, 3) + matrix(2, r) * matrix(2, 3));
            }
            o.matrix(3, 3) = 1.f;
            return o;
        }
    private:
        explicit Affine3f(int) : matrix() {}
    };
}
#endif

namespace tfusion
{
    // the C-ABI's row-major 3x4 [R|t] <-> Affine3f (own or cv::)
    inline Affine3f affine_from_rt(const float rt[12])
    {
        Matx44f m;
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 4; ++c) m(r, c) = rt[r * 4 + c];
        m(3, 3) = 1.f;
        return Affine3f(m);
    }
    inline void affine_to_rt(const Affine3f& a, float rt[12])
    {
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 4; ++c) rt[r * 4 + c] = a.matrix(r, c);
    }

    // Matrix4f (tfusion/include/Matrix.hpp:22-66, 126-133): column-major, m[4c + r]; the 16-value
    // constructor fills m in argument order, so Matrix4f(P(0,0), P(1,0), P(2,0), P(3,0), P(0,1), ...)
    // holds P (the reference's conversion, topfu.cpp:246-249); operator()(x, y) is column x, row y
    struct Matrix4f {
        float m[16];
        Matrix4f() : m{} { for (int i = 0; i < 4; ++i) m[i * 5] = 1.f; }
        Matrix4f(float a00, float a01, float a02, float a03, float a10, float a11, float a12, float a13,
                 float a20, float a21, float a22, float a23, float a30, float a31, float a32, float a33)
            : m{ a00, a01, a02, a03, a10, a11, a12, a13, a20, a21, a22, a23, a30, a31, a32, a33 } {}
        float& operator()(int x, int y) { return m[y | (x << 2)]; }
        float operator()(int x, int y) const { return m[y | (x << 2)]; }
        // the rigid transform it holds as a row-major 3x4 [R|t] (the C-ABI's pose layout)
        void toRt(float rt[12]) const
        {
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 4; ++c) rt[r * 4 + c] = m[4 * c + r];
        }
        static Matrix4f fromAffine(const Affine3f& a)
        {
            const Matx44f& P = a.matrix;
            return Matrix4f(P(0, 0), P(1, 0), P(2, 0), P(3, 0), P(0, 1), P(1, 1), P(2, 1), P(3, 1),
                            P(0, 2), P(1, 2), P(2, 2), P(3, 2), P(0, 3), P(1, 3), P(2, 3), P(3, 3));
        }
    };

    struct Intr {
        float fx, fy, cx, cy;
        Intr() : fx(0), fy(0), cx(0), cy(0) {}
        Intr(float fx_, float fy_, float cx_, float cy_) : fx(fx_), fy(fy_), cx(cx_), cy(cy_) {}
        Intr operator()(int level_index) const   // precomp.cpp:10-14
        {
            const int div = 1 << level_index;
            return Intr(fx / div, fy / div, cx / div, cy / div);
        }
    };

    struct Point { union { float data[4]; struct { float x, y, z; }; }; };
    typedef Point Normal;
    struct Vector3u { unsigned char x, y, z; };
    struct Vector4u { unsigned char x, y, z, w; };
    struct Vector4f {
        float x, y, z, w;
        Vector4f() : x(0), y(0), z(0), w(0) {}
        Vector4f(float x_, float y_, float z_, float w_) : x(x_), y(y_), z(z_), w(w_) {}
    };
    struct Vector2i {
        int x, y;
        Vector2i() : x(0), y(0) {}
        Vector2i(int x_, int y_) : x(x_), y(y_) {}
    };

    inline float deg2rad(float alpha) { return alpha * 0.017453293f; }

    namespace cuda
    {
        inline void hip_check(hipError_t e, const char* what)
        {   // the reference prints and exits (device_memory.cpp:7-11); the build throws
            if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
        }

        // DeviceArray2D<T>: pitched device image, reference-counted like the reference's
        // DeviceMemory2D (shallow copies share the allocation, freed with the last owner)
        template <typename T>
        class DeviceArray2D
        {
        public:
            DeviceArray2D() = default;
            DeviceArray2D(int rows, int cols) { create(rows, cols); }
            DeviceArray2D(const DeviceArray2D& o) : data_(o.data_), step_(o.step_), rows_(o.rows_), cols_(o.cols_), ref_(o.ref_)
            {
                if (ref_) ++*ref_;
            }
            DeviceArray2D& operator=(const DeviceArray2D& o)
            {
                if (this != &o) { release(); data_ = o.data_; step_ = o.step_; rows_ = o.rows_; cols_ = o.cols_; ref_ = o.ref_; if (ref_) ++*ref_; }
                return *this;
            }
            ~DeviceArray2D() { release(); }

            void create(int rows, int cols)
            {
                if (data_ && rows == rows_ && cols == cols_) return;
                release();
                size_t pitch = 0;
                hip_check(hipMallocPitch(&data_, &pitch, sizeof(T) * (size_t)cols, (size_t)rows), "DeviceArray2D::create");
                step_ = pitch; rows_ = rows; cols_ = cols;
                ref_ = new int(1);
            }
            void release()
            {
                if (ref_ && --*ref_ == 0) { (void)hipFree(data_); delete ref_; }
                data_ = nullptr; ref_ = nullptr; step_ = 0; rows_ = cols_ = 0;
            }
            void upload(const void* host, size_t host_step, int rows, int cols)
            {
                create(rows, cols);
                hip_check(hipMemcpy2D(data_, step_, host, host_step, sizeof(T) * (size_t)cols, (size_t)rows, hipMemcpyHostToDevice),
                          "DeviceArray2D::upload");
            }
            void download(void* host, size_t host_step) const
            {
                hip_check(hipMemcpy2D(host, host_step, data_, step_, sizeof(T) * (size_t)cols_, (size_t)rows_, hipMemcpyDeviceToHost),
                          "DeviceArray2D::download");
            }
            void swap(DeviceArray2D& o)
            {
                std::swap(data_, o.data_); std::swap(step_, o.step_); std::swap(rows_, o.rows_);
                std::swap(cols_, o.cols_); std::swap(ref_, o.ref_);
            }
            bool empty() const { return data_ == nullptr; }
            T* ptr(int y = 0) { return reinterpret_cast<T*>(reinterpret_cast<char*>(data_) + (size_t)y * step_); }
            const T* ptr(int y = 0) const { return reinterpret_cast<const T*>(reinterpret_cast<const char*>(data_) + (size_t)y * step_); }
            size_t step() const { return step_; }
            int rows() const { return rows_; }
            int cols() const { return cols_; }
            size_t elem_step() const { return step_ / sizeof(T); }

        private:
            void* data_ = nullptr;
            size_t step_ = 0;
            int rows_ = 0, cols_ = 0;
            int* ref_ = nullptr;
        };

        // DeviceArray<T> (device_array.hpp:19-96): a linear device buffer, reference-counted like
        // DeviceArray2D (apps/demo.cpp:146 declares a DeviceArray<Point> cloud buffer)
        template <typename T>
        class DeviceArray
        {
        public:
            typedef T type;
            enum { elem_size = sizeof(T) };
            DeviceArray() = default;
            explicit DeviceArray(size_t size) { create(size); }
            DeviceArray(const DeviceArray& o) : data_(o.data_), size_(o.size_), ref_(o.ref_) { if (ref_) ++*ref_; }
            DeviceArray& operator=(const DeviceArray& o)
            {
                if (this != &o) { release(); data_ = o.data_; size_ = o.size_; ref_ = o.ref_; if (ref_) ++*ref_; }
                return *this;
            }
            ~DeviceArray() { release(); }
            void create(size_t size)
            {
                if (data_ && size == size_) return;
                release();
                if (size == 0) return;
                hip_check(hipMalloc(&data_, sizeof(T) * size), "DeviceArray::create");
                size_ = size;
                ref_ = new int(1);
            }
            void release()
            {
                if (ref_ && --*ref_ == 0) { (void)hipFree(data_); delete ref_; }
                data_ = nullptr; ref_ = nullptr; size_ = 0;
            }
            void upload(const T* host, size_t size)
            {
                create(size);
                hip_check(hipMemcpy(data_, host, sizeof(T) * size, hipMemcpyHostToDevice), "DeviceArray::upload");
            }
            void download(T* host) const
            {
                hip_check(hipMemcpy(host, data_, sizeof(T) * size_, hipMemcpyDeviceToHost), "DeviceArray::download");
            }
            void upload(const std::vector<T>& v) { upload(v.data(), v.size()); }
            void download(std::vector<T>& v) const { v.resize(size_); if (size_) download(v.data()); }
            void swap(DeviceArray& o) { std::swap(data_, o.data_); std::swap(size_, o.size_); std::swap(ref_, o.ref_); }
            bool empty() const { return data_ == nullptr; }
            size_t size() const { return size_; }
            size_t sizeBytes() const { return size_ * sizeof(T); }
            T* ptr() { return static_cast<T*>(data_); }
            const T* ptr() const { return static_cast<const T*>(data_); }

        private:
            void* data_ = nullptr;
            size_t size_ = 0;
            int* ref_ = nullptr;
        };

        typedef DeviceArray2D<unsigned short> Depth;
        typedef DeviceArray2D<float> Dists;
        typedef DeviceArray2D<Vector4u> image4u;
        typedef DeviceArray2D<Vector4f> image4f;
        typedef DeviceArray2D<Point> Cloud;
        typedef DeviceArray2D<Normal> Normals;
        struct RGB { union { struct { unsigned char b, g, r; }; int bgra; }; };
        typedef DeviceArray2D<RGB> Image;
        typedef DeviceArray2D<int> imageInt;

        // cuda::Frame (types.hpp:73-79): one frame's pyramids
        struct Frame {
            bool use_points = true;
            std::vector<Depth> depth_pyr;
            std::vector<Cloud> points_pyr;
            std::vector<Normals> normals_pyr;
        };
    }

    // ScopeTime / SampledScopeTime (types.hpp:83-104; core.cpp:202-231): wall-clock timers with the
    // reference's output.  SampledScopeTime keeps the reference's function-static call counter
    // (core.cpp:208): one counter for the whole program, so a loop that constructs one per frame
    // (demo.cpp:102-105) prints the average after 33 more frames each time, starting at the 34th.
    struct ScopeTime {
        const char* name;
        std::chrono::steady_clock::time_point start;
        explicit ScopeTime(const char* n) : name(n), start(std::chrono::steady_clock::now()) {}
        ~ScopeTime()
        {
            double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - start).count();
            std::printf("Time(%s) = %gms\n", name, ms);
        }
    };

    struct SampledScopeTime {
        enum { EACH = 33 };
        explicit SampledScopeTime(double& time_ms) : time_ms_(time_ms), start_(std::chrono::steady_clock::now()) {}
        ~SampledScopeTime()
        {
            static int i_ = 0;                  // function-static, as core.cpp:208 (inline: one per program)
            time_ms_ += getTime();
            if (i_ % EACH == 0 && i_) {
                std::printf("Average frame time = %gms ( %gfps )\n", time_ms_ / EACH, 1000.f * EACH / time_ms_);
                std::fflush(stdout);
                time_ms_ = 0.0;
            }
            ++i_;
        }
    private:
        double getTime() const
        {
            return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - start_).count();
        }
        SampledScopeTime(const SampledScopeTime&) = delete;
        SampledScopeTime& operator=(const SampledScopeTime&) = delete;
        double& time_ms_;
        std::chrono::steady_clock::time_point start_;
    };
}
