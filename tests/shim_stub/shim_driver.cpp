// Test driver of the drop-in shim (stereomatch_amd/shim/stereo3dmst_shim.cpp): what src/stereo_Yin.cpp
// does around the call (:205-210) -- startTimer(); stereo3dmst(names, L, R, dL, dR, data_cost, Dmax);
// getTimer() -- with the images in (stub) cv::Mat objects.  Built as a shared library (tests load it
// with ctypes and call shim_run in-process).  Test infrastructure.
#include <cstring>

#include "../../include/Stereo3DMST.h"

// pad > 0: the input images get padded rows (non-continuous, like an ROI), so the shim's clone path runs.
// Returns 0 and fills outl / outr (H*W floats) and *ms; 1: the output maps have the wrong geometry.
extern "C" int shim_run(const unsigned char* l, const unsigned char* r, int W, int H, int pad, const char* data_cost,
                        int Dmax, float* outl, float* outr, double* ms) {
    cv::Mat L, R, dL, dR;
    L.create_padded(H, W, CV_8UC3, (size_t)pad);
    R.create_padded(H, W, CV_8UC3, (size_t)pad);
    for (int y = 0; y < H; ++y) {
        std::memcpy(L.data + L.step * y, l + (size_t)3 * W * y, (size_t)3 * W);
        std::memcpy(R.data + R.step * y, r + (size_t)3 * W * y, (size_t)3 * W);
    }
    startTimer();
    stereo3dmst("img1r.png", "img2r.png", L, R, dL, dR, data_cost, Dmax);
    *ms = getTimer();
    if (dL.rows != H || dL.cols != W || dL.type() != CV_32F || dR.rows != H || dR.cols != W || dR.type() != CV_32F)
        return 1;
    for (int y = 0; y < H; ++y) {
        std::memcpy(outl + (size_t)W * y, dL.ptr<float>(y), (size_t)4 * W);
        std::memcpy(outr + (size_t)W * y, dR.ptr<float>(y), (size_t)4 * W);
    }
    return 0;
}
