// Minimal cv::Mat stand-in for compiling stereomatch_amd/shim/stereo3dmst_shim.cpp in the CPU test
// suite (the image has no OpenCV).  Test infrastructure: only the members the shim uses.
#pragma once
#include <cstddef>
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
    void create(int r, int c, int type) {
        rows = r, cols = c, t = type;
        step = (size_t)c * (type == CV_32F ? 4 : 3);
        buf.assign(step * r, 0);
        data = buf.data();
    }
    int type() const { return t; }
    Size size() const { return Size{cols, rows}; }
    bool isContinuous() const { return true; }
    Mat clone() const { return *this; }
    template <typename T>
    T* ptr(int row) { return reinterpret_cast<T*>(data + step * row); }
};
}  // namespace cv
