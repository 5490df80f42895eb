// Minimal cv::Mat stand-in for compiling stereomatch_amd/shim/stereo3dmst_shim.cpp in the test suite
// (the image has no OpenCV).  Test infrastructure: only the members the shim uses, plus a padded-row
// constructor (an ROI-like non-continuous image) for the shim's stride handling.
#pragma once
#include <cstddef>
#include <cstring>
#include <vector>
#define CV_8UC3 16
#define CV_32F 5
namespace cv {
struct Size {
    int width = 0, height = 0;
    bool operator!=(const Size& o) const { return width != o.width || height != o.height; }
};
struct Mat {
    int rows = 0, cols = 0, t = 0;
    size_t step = 0;
    unsigned char* data = nullptr;
    std::vector<unsigned char> buf;
    Mat() = default;
    Mat(const Mat& o) { *this = o; }
    Mat& operator=(const Mat& o) {
        rows = o.rows, cols = o.cols, t = o.t, step = o.step;
        buf = o.buf;
        data = buf.empty() ? nullptr : buf.data();
        return *this;
    }
    static size_t elem(int type) { return type == CV_32F ? 4 : 3; }
    void create(int r, int c, int type) { create_padded(r, c, type, 0); }
    // rows of cols * elem bytes, each followed by pad bytes
    void create_padded(int r, int c, int type, size_t pad) {
        rows = r, cols = c, t = type;
        step = (size_t)c * elem(type) + pad;
        buf.assign(step * r, 0);
        data = buf.data();
    }
    int type() const { return t; }
    Size size() const { return Size{cols, rows}; }
    bool isContinuous() const { return step == (size_t)cols * elem(t); }
    Mat clone() const {  // continuous copy
        Mat m;
        m.create(rows, cols, t);
        for (int y = 0; y < rows; ++y) std::memcpy(m.data + m.step * y, data + step * y, (size_t)cols * elem(t));
        return m;
    }
    template <typename T>
    T* ptr(int row) { return reinterpret_cast<T*>(data + step * row); }
};
}  // namespace cv
