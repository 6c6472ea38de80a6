// tfusion/types.hpp -- host-side value types and device containers of the tfusion API,
// re-declared for the MI355X build (header-only, over include/tfusion_hip.h + HIP runtime).
//
// Mirrors tfusion/include/tfusion/types.hpp (Intr :19-26, Point/Normal :30-40, cuda typedefs
// :56-82, ScopeTime/SampledScopeTime :86-108) and tfusion/include/tfusion/cuda/device_array.hpp
// (DeviceArray2D create/upload/download/ptr/step/rows/cols/release, :19-222).  OpenCV is not
// required: Affine3f / Vec3f / Matx33f are small own types with the cv:: member names the
// reference's callers use (matrix, rotation(), translation(), inv(), operator*, Identity()).
#pragma once
#include <hip/hip_runtime_api.h>

#include <chrono>
#include <cmath>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace tfusion
{
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

    // cv::Affine3f subset: 4x4 row-major matrix of a rigid transform (camera -> world for poses)
    struct Affine3f {
        float matrix[16];
        Affine3f() { *this = Identity(); }
        static Affine3f Identity()
        {
            Affine3f a(0);
            for (int i = 0; i < 4; ++i) a.matrix[i * 5] = 1.f;
            return a;
        }
        // from the C-ABI's row-major 3x4 [R|t]
        static Affine3f fromRt(const float rt[12])
        {
            Affine3f a(0);
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 4; ++c) a.matrix[r * 4 + c] = rt[r * 4 + c];
            a.matrix[15] = 1.f;
            return a;
        }
        void toRt(float rt[12]) const
        {
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 4; ++c) rt[r * 4 + c] = matrix[r * 4 + c];
        }
        Mat3f rotation() const
        {
            Mat3f R;
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 3; ++c) R(r, c) = matrix[r * 4 + c];
            return R;
        }
        Vec3f translation() const { return Vec3f(matrix[3], matrix[7], matrix[11]); }
        Affine3f translate(const Vec3f& t) const
        {
            Affine3f a = *this;
            a.matrix[3] += t[0]; a.matrix[7] += t[1]; a.matrix[11] += t[2];
            return a;
        }
        Affine3f operator*(const Affine3f& b) const   // rigid composition in float
        {
            Affine3f o(0);
            for (int r = 0; r < 3; ++r) {
                for (int c = 0; c < 3; ++c)
                    o.matrix[r * 4 + c] = matrix[r * 4 + 0] * b.matrix[0 * 4 + c] + matrix[r * 4 + 1] * b.matrix[1 * 4 + c] +
                                          matrix[r * 4 + 2] * b.matrix[2 * 4 + c];
                o.matrix[r * 4 + 3] = matrix[r * 4 + 0] * b.matrix[3] + matrix[r * 4 + 1] * b.matrix[7] +
                                      matrix[r * 4 + 2] * b.matrix[11] + matrix[r * 4 + 3];
            }
            o.matrix[15] = 1.f;
            return o;
        }
        Affine3f inv() const                            // rigid inverse [R^T | -R^T t]
        {
            Affine3f o(0);
            for (int r = 0; r < 3; ++r) {
                for (int c = 0; c < 3; ++c) o.matrix[r * 4 + c] = matrix[c * 4 + r];
                o.matrix[r * 4 + 3] = -(matrix[0 * 4 + r] * matrix[3] + matrix[1 * 4 + r] * matrix[7] +
                                        matrix[2 * 4 + r] * matrix[11]);
            }
            o.matrix[15] = 1.f;
            return o;
        }
    private:
        explicit Affine3f(int) : matrix{} {}
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
    struct Vector4u { unsigned char x, y, z, w; };
    struct Vector4f { float x, y, z, w; };

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

        typedef DeviceArray2D<unsigned short> Depth;
        typedef DeviceArray2D<float> Dists;
        typedef DeviceArray2D<Vector4u> image4u;
        typedef DeviceArray2D<Vector4f> image4f;
        typedef DeviceArray2D<Point> Cloud;
        typedef DeviceArray2D<Normal> Normals;
        struct RGB { union { struct { unsigned char b, g, r; }; int bgra; }; };
        typedef DeviceArray2D<RGB> Image;
    }

    // ScopeTime / SampledScopeTime (types.hpp:86-108; core.cpp:180-216): wall-clock timers.
    // SampledScopeTime averages over EACH = 33 scopes per instance (the reference keeps the
    // counter in a function static; here it lives in the object so several streams can time).
    struct ScopeTime {
        const char* name;
        std::chrono::steady_clock::time_point start;
        explicit ScopeTime(const char* n) : name(n), start(std::chrono::steady_clock::now()) {}
        ~ScopeTime()
        {
            double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - start).count();
            std::printf("Time(%s) = %.3f ms\n", name, ms);
        }
    };

    struct SampledScopeTime {
        enum { EACH = 33 };
        explicit SampledScopeTime(double& time_ms, int* counter = nullptr)
            : time_ms_(time_ms), counter_(counter), start_(std::chrono::steady_clock::now()) {}
        ~SampledScopeTime()
        {
            time_ms_ += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - start_).count();
            int& c = counter_ ? *counter_ : local_;
            if (++c == EACH) {
                std::printf("Average frame time = %.3f ms ( %.1f fps )\n", time_ms_ / EACH, 1000.0 * EACH / time_ms_);
                time_ms_ = 0; c = 0;
            }
        }
    private:
        SampledScopeTime(const SampledScopeTime&) = delete;
        SampledScopeTime& operator=(const SampledScopeTime&) = delete;
        double& time_ms_;
        int* counter_;
        int local_ = 0;
        std::chrono::steady_clock::time_point start_;
    };
}
