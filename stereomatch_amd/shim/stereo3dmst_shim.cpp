// stereo3dmst_shim.cpp -- the reference's entry points (include/Stereo3DMST.h) over the C-ABI.
//
// stereo3dmst (src/Stereo3DMST.cpp:714-912 contract):
//   * creates leftDisp / rightDisp as CV_32F rows x cols (:722-723);
//   * data_cost "MCCNN_fst" without an mc-cnn-master folder prints "no mc-cnn-master folder" and
//     returns (:727-731); "MCCNN_acrt" without it returns silently (:744-745); an unknown string
//     prints "wrong data cost" (:756-759) -- maps are left allocated but unset, as the reference;
//   * "AGD" runs this framework's GPU path: AGD cost volume, MST tree filter per disparity slice,
//     strict-< WTA, then the reference's output step: left map left-right checked without fill
//     (:900-904); both maps in [0, Dmax-1].  MC-CNN volume ingest is not implemented yet
//     (SURVEY.md 8f rank 2): with an mc-cnn-master folder present the MCCNN_* kinds print a
//     notice and return.
// One process-global context behind a mutex (the reference is not reentrant either: :15, :727).
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <iostream>
#include <mutex>

#include "../../include/Stereo3DMST.h"
#include "../../include/stereomst.h"

namespace {
std::mutex g_mu;
sm_ctx* g_ctx = nullptr;
double g_timer = 0.0;

bool has_mccnn_dir() {
    struct stat st;
    return stat("mc-cnn-master", &st) == 0 && S_ISDIR(st.st_mode);
}
}  // namespace

extern "C" void stereo3dmst(std::string left_name, std::string right_name, cv::Mat& leftImg, cv::Mat& rightImg,
                            cv::Mat& leftDisp, cv::Mat& rightDisp, std::string data_cost, int Dmax) {
    (void)left_name;
    (void)right_name;
    const int cols = leftImg.cols, rows = leftImg.rows;
    leftDisp.create(rows, cols, CV_32F);
    rightDisp.create(rows, cols, CV_32F);
    if (data_cost == "MCCNN_fst" || data_cost == "MCCNN_acrt") {
        if (!has_mccnn_dir()) {
            if (data_cost == "MCCNN_fst") std::cout << "no mc-cnn-master folder\n";
            return;
        }
        std::cout << "stereo3dmst: MC-CNN volume ingest is not implemented in this build; use data_cost=\"AGD\"\n";
        return;
    }
    if (data_cost != "AGD") {
        std::cout << "wrong data cost\n";
        return;
    }
    if (leftImg.type() != CV_8UC3 || rightImg.type() != CV_8UC3 || rightImg.size() != leftImg.size()) {
        std::cout << "stereo3dmst: expected two same-sized CV_8UC3 BGR images\n";
        return;
    }
    std::lock_guard<std::mutex> lock(g_mu);
    if (!g_ctx) {
        sm_config cfg{0, cols, rows, Dmax};
        if (sm_create(&g_ctx, &cfg) != SM_OK) {
            std::cout << "stereo3dmst: no HIP device\n";
            g_ctx = nullptr;
            return;
        }
    }
    sm_params p;
    sm_default_params(&p);
    p.disp_total = Dmax;
    p.post = SM_POST_LR_CHECK;
    const cv::Mat l = leftImg.isContinuous() ? leftImg : leftImg.clone();
    const cv::Mat r = rightImg.isContinuous() ? rightImg : rightImg.clone();
    const sm_status st = sm_match(g_ctx, l.data, r.data, cols, rows, (int)l.step, Dmax, &p, leftDisp.ptr<float>(0),
                                  rightDisp.ptr<float>(0), nullptr, nullptr, nullptr, nullptr);
    if (st != SM_OK) std::cout << "stereo3dmst: " << sm_last_error(g_ctx) << "\n";
}

void startTimer() { sm_start_timer(&g_timer); }

double getTimer() { return sm_get_timer_ms(&g_timer); }
