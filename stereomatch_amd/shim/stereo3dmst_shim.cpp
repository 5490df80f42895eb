// stereo3dmst_shim.cpp -- the reference's entry points (include/Stereo3DMST.h) over the C-ABI.
//
// stereo3dmst (src/Stereo3DMST.cpp:714-912 contract):
//   * creates leftDisp / rightDisp as CV_32F rows x cols (:722-723);
//   * data_cost "MCCNN_fst" without an mc-cnn-master folder prints "no mc-cnn-master folder" and
//     returns (:727-731); "MCCNN_acrt" without it returns silently (:744-745); an unknown string
//     prints "wrong data cost" (:756-759) -- maps are left allocated but unset, as the reference;
//   * "AGD" runs this framework's GPU path on the AGD cost volume.  The algorithm is the reference's
//     own (env SM_STEREO3DMST_ALGO unset or "pms"): the segment forest with c = 5000, min_size = 200,
//     random plane labels and 100 MST_PMS calls per view (:830-832, :546-629, :851-889; env
//     SM_PMS_ITERS overrides the count), or with SM_STEREO3DMST_ALGO=slices the per-slice
//     restatement (MST tree filter per disparity slice, strict-< WTA); then the reference's output
//     step: LabelToDisp + scaling, left map left-right checked without fill (:900-904), both maps in
//     [0, Dmax-1];
//   * "MCCNN_fst" / "MCCNN_acrt" with an mc-cnn-master folder: like the reference, run the network
//     there (system(), :733-750; its exit status is ignored unless system() itself fails) and
//     read mc-cnn-master/{left,right}.bin, [Dmax][rows][cols] float (:764-775); the clamp
//     (:785-803), tree filter and WTA run on the GPU (SM_COST_VOLUME), then the same output step.
// One process-global context behind a mutex (the reference is not reentrant either: :15, :727).
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <mutex>
#include <vector>

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

// the reference's MC-CNN step (Stereo3DMST.cpp:725-775): the network in mc-cnn-master, then the
// two raw volumes; false (message printed) when a volume is missing or short
bool mccnn_volumes(const std::string& left_name, const std::string& right_name, const std::string& data_cost, int rows,
                   int cols, int Dmax, std::vector<float>& lv, std::vector<float>& rv) {
    const bool fast = data_cost == "MCCNN_fst";
    const std::string net = fast ? "fast" : "slow";
    const std::string cmd = "cd mc-cnn-master && ./main.lua mb " + net + " -a predict -net_fname net/net_mb_" + net +
                            "_-a_train_all.t7 -left ../" + left_name + " -right ../" + right_name + " -disp_max " +
                            std::to_string(Dmax) + " -sm_terminate cnn";
    if (system(cmd.c_str()) < 0) return false;  // the reference returns only when system() fails
    const size_t n = (size_t)Dmax * rows * cols;
    const char* names[2] = {"mc-cnn-master/left.bin", "mc-cnn-master/right.bin"};
    std::vector<float>* outs[2] = {&lv, &rv};
    for (int v = 0; v < 2; ++v) {
        std::ifstream f(names[v], std::ios::binary);
        outs[v]->resize(n);
        if (!f.read(reinterpret_cast<char*>(outs[v]->data()), (std::streamsize)(n * sizeof(float)))) {
            std::cout << "stereo3dmst: " << names[v] << " missing or shorter than Dmax*rows*cols floats\n";
            return false;
        }
    }
    return true;
}
}  // namespace

extern "C" void stereo3dmst(std::string left_name, std::string right_name, cv::Mat& leftImg, cv::Mat& rightImg,
                            cv::Mat& leftDisp, cv::Mat& rightDisp, std::string data_cost, int Dmax) {
    const int cols = leftImg.cols, rows = leftImg.rows;
    leftDisp.create(rows, cols, CV_32F);
    rightDisp.create(rows, cols, CV_32F);
    const bool mccnn = data_cost == "MCCNN_fst" || data_cost == "MCCNN_acrt";
    std::vector<float> lv, rv;
    if (mccnn) {
        if (!has_mccnn_dir()) {
            if (data_cost == "MCCNN_fst") std::cout << "no mc-cnn-master folder\n";
            return;
        }
        if (!mccnn_volumes(left_name, right_name, data_cost, rows, cols, Dmax, lv, rv)) return;
    } else if (data_cost != "AGD") {
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
    p.post = SM_POST_LABEL_TO_DISP | SM_POST_LR_CHECK;  // LabelToDisp + scaling, then the L-R check (:900-904)
    const char* algo = getenv("SM_STEREO3DMST_ALGO");
    if (!algo || std::string(algo) == "pms") {  // the reference's own label search (:830-832, :854)
        p.aggregator = SM_AGG_PMS;
        p.c = 5000.0f;
        p.min_size = 200;
        const char* it = getenv("SM_PMS_ITERS");
        p.pms_iters = it ? atoi(it) : 100;
    }
    if (mccnn) {
        if (sm_upload_cost_volumes(g_ctx, lv.data(), rv.data(), cols, rows, Dmax) != SM_OK) {
            std::cout << "stereo3dmst: " << sm_last_error(g_ctx) << "\n";
            return;
        }
        p.cost_kind = SM_COST_VOLUME;
    }
    const cv::Mat l = leftImg.isContinuous() ? leftImg : leftImg.clone();
    const cv::Mat r = rightImg.isContinuous() ? rightImg : rightImg.clone();
    const sm_status st = sm_match(g_ctx, l.data, r.data, cols, rows, (int)l.step, Dmax, &p, leftDisp.ptr<float>(0),
                                  rightDisp.ptr<float>(0), nullptr, nullptr, nullptr, nullptr);
    if (st != SM_OK) std::cout << "stereo3dmst: " << sm_last_error(g_ctx) << "\n";
}

void startTimer() { sm_start_timer(&g_timer); }

double getTimer() { return sm_get_timer_ms(&g_timer); }
