// tfusion/io.hpp -- frame input for the tfusion API without OpenCV / OpenNI.
//
// The reference demo reads its frames as 16-bit PGM depth + 8-bit PPM colour pairs
// (apps/demo.cpp:91-97: cv::imread("...\\%04d.pgm", CV_16U) and cv::imread("...\\%04d.ppm")).
// These readers return the same pixels OpenCV's imread gives for those files:
//   * P5 (PGM) with maxval > 255: big-endian 16-bit samples -> uint16 in host order
//     (imread's IMREAD_ANYDEPTH = CV_16U = 2 keeps the 16 bits); maxval <= 255: 8-bit samples
//     widened to uint16;
//   * P6 (PPM), maxval <= 255: RGB triplets -> B, G, R order (imread's 3-channel BGR Mat).
// Header comments (#...) and any whitespace between header fields are accepted, as netpbm
// allows.  Header-only, no dependencies beyond the C++ standard library.
#pragma once

#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <vector>

namespace tfusion {
namespace io {

namespace detail {
inline int next_field(std::FILE* f)
{   // netpbm header integer: skip whitespace and '#' comments
    int c = std::fgetc(f);
    while (c != EOF) {
        if (c == '#') { while (c != EOF && c != '\n') c = std::fgetc(f); }
        else if (c == ' ' || c == '\t' || c == '\r' || c == '\n') c = std::fgetc(f);
        else break;
    }
    if (c == EOF || c < '0' || c > '9') throw std::runtime_error("netpbm: bad header");
    long v = 0;
    while (c >= '0' && c <= '9') {
        v = v * 10 + (c - '0');
        if (v > 1 << 30) throw std::runtime_error("netpbm: header value too large");
        c = std::fgetc(f);
    }
    // exactly one whitespace character separates the last header field from the raster
    return (int)v;
}

struct File {
    std::FILE* f;
    explicit File(const std::string& path) : f(std::fopen(path.c_str(), "rb"))
    {
        if (!f) throw std::runtime_error("cannot open " + path);
    }
    ~File() { if (f) std::fclose(f); }
};

inline void magic(std::FILE* f, char want, const std::string& path)
{
    char m[2];
    if (std::fread(m, 1, 2, f) != 2 || m[0] != 'P' || m[1] != want)
        throw std::runtime_error(path + ": not a binary P" + std::string(1, want) + " file");
}
}  // namespace detail

// 16-bit depth (millimetres) of a P5 PGM, row-major cols x rows
inline void readPGM16(const std::string& path, std::vector<uint16_t>& px, int& cols, int& rows)
{
    detail::File file(path);
    detail::magic(file.f, '5', path);
    cols = detail::next_field(file.f);
    rows = detail::next_field(file.f);
    const int maxval = detail::next_field(file.f);
    if (cols <= 0 || rows <= 0 || maxval <= 0 || maxval > 65535) throw std::runtime_error(path + ": bad PGM header");
    const size_t n = (size_t)cols * rows;
    px.resize(n);
    if (maxval > 255) {
        std::vector<unsigned char> raw(2 * n);
        if (std::fread(raw.data(), 1, raw.size(), file.f) != raw.size()) throw std::runtime_error(path + ": short PGM");
        for (size_t i = 0; i < n; ++i) px[i] = (uint16_t)((raw[2 * i] << 8) | raw[2 * i + 1]);   // big-endian
    } else {
        std::vector<unsigned char> raw(n);
        if (std::fread(raw.data(), 1, raw.size(), file.f) != raw.size()) throw std::runtime_error(path + ": short PGM");
        for (size_t i = 0; i < n; ++i) px[i] = raw[i];
    }
}

// 8-bit colour of a P6 PPM as B, G, R triplets, row-major cols x rows
inline void readPPM(const std::string& path, std::vector<uint8_t>& bgr, int& cols, int& rows)
{
    detail::File file(path);
    detail::magic(file.f, '6', path);
    cols = detail::next_field(file.f);
    rows = detail::next_field(file.f);
    const int maxval = detail::next_field(file.f);
    if (cols <= 0 || rows <= 0 || maxval <= 0 || maxval > 255) throw std::runtime_error(path + ": bad PPM header");
    const size_t n = (size_t)cols * rows * 3;
    bgr.resize(n);
    if (std::fread(bgr.data(), 1, n, file.f) != n) throw std::runtime_error(path + ": short PPM");
    for (size_t i = 0; i < n; i += 3) std::swap(bgr[i], bgr[i + 2]);      // RGB -> BGR
}

inline void writePGM16(const std::string& path, const uint16_t* px, int cols, int rows)
{
    std::FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) throw std::runtime_error("cannot write " + path);
    std::fprintf(f, "P5\n%d %d\n65535\n", cols, rows);
    std::vector<unsigned char> raw((size_t)cols * rows * 2);
    for (size_t i = 0; i < (size_t)cols * rows; ++i) { raw[2 * i] = (unsigned char)(px[i] >> 8); raw[2 * i + 1] = (unsigned char)px[i]; }
    const bool ok = std::fwrite(raw.data(), 1, raw.size(), f) == raw.size();
    std::fclose(f);
    if (!ok) throw std::runtime_error("short write " + path);
}

// A numbered frame sequence in place of the reference's capture source (OpenNISource::grab,
// io/capture.hpp): depth from printf(depth_pattern, i) (e.g. "frames/%04d.pgm"), colour from
// printf(image_pattern, i) when a pattern is given.  grab() returns false at the first
// missing depth file.
class FrameSequenceSource {
public:
    FrameSequenceSource(std::string depth_pattern, std::string image_pattern = std::string(), int first = 0)
        : depth_pattern_(std::move(depth_pattern)), image_pattern_(std::move(image_pattern)), next_(first) {}

    bool grab(std::vector<uint16_t>& depth, std::vector<uint8_t>& image)
    {
        const std::string dp = format(depth_pattern_, next_);
        if (std::FILE* f = std::fopen(dp.c_str(), "rb")) std::fclose(f);
        else return false;
        readPGM16(dp, depth, cols_, rows_);
        if (!image_pattern_.empty()) {
            int c = 0, r = 0;
            readPPM(format(image_pattern_, next_), image, c, r);
            if (c != cols_ || r != rows_) throw std::runtime_error("colour / depth frame size mismatch");
        } else {
            image.clear();
        }
        ++next_;
        return true;
    }
    int cols() const { return cols_; }
    int rows() const { return rows_; }
    int index() const { return next_; }

private:
    static std::string format(const std::string& pattern, int i)
    {
        std::vector<char> buf(pattern.size() + 32);
        std::snprintf(buf.data(), buf.size(), pattern.c_str(), i);
        return std::string(buf.data());
    }
    std::string depth_pattern_, image_pattern_;
    int next_ = 0, cols_ = 0, rows_ = 0;
};

}  // namespace io
}  // namespace tfusion
