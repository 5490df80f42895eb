/* Stereo3DMST.h -- drop-in replacement for the reference's public header
 * (lr-xiang/StereoMatch include/Stereo3DMST.h:1-13), same declarations so src/stereo_Yin.cpp
 * (:7, :205-209) compiles and links unchanged against libstereo3dmst_shim.so.
 *
 *   stereo3dmst : unmangled (extern "C") like the reference's exported symbol; C++ types in the
 *                 signature exactly as the reference (std::string by value, cv::Mat&).
 *   startTimer / getTimer : C++ linkage (_Z10startTimerv / _Z8getTimerv), milliseconds.
 *
 * Implemented in stereomatch_amd/shim/stereo3dmst_shim.cpp over the C-ABI of stereomst.h;
 * built only where OpenCV headers exist. */
#ifndef STEREOMATCH_AMD_STEREO3DMST_H
#define STEREOMATCH_AMD_STEREO3DMST_H

#include <string>

#include <opencv2/highgui/highgui.hpp>
#include <opencv2/imgproc/imgproc.hpp>

extern "C" void stereo3dmst(std::string left_name, std::string right_name, cv::Mat& leftImg, cv::Mat& rightImg,
                            cv::Mat& leftDisp, cv::Mat& rightDisp, std::string data_cost, int Dmax);

void startTimer();

double getTimer();

#endif
