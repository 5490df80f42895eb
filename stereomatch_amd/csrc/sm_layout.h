// sm_layout.h -- tree layout consumed by the walker kernels (see sm_layout.cpp).
#pragma once
#include <stdint.h>

#include <vector>

#include "sm_common.h"

struct SmLayout {
    std::vector<SmMeta> meta;               // [slot]
    std::vector<SmPath> paths;              // all rounds, round r = [round_path_begin[r], round_path_begin[r+1])
    std::vector<uint32_t> round_path_begin; // nrounds+1
    std::vector<uint32_t> round_slot_begin; // nrounds+1 (slots of light depth r)
    std::vector<uint32_t> max_path_len;     // per round
    std::vector<uint32_t> parent_pix;       // [pix] (SM_NONE for roots)
    std::vector<uint32_t> subtree_size;     // [pix]
    std::vector<uint32_t> slot_of_pix;      // [pix]
    uint32_t nrounds = 0, nroots = 0, n_light = 0;
};

void sm_build_layout(int W, int H, const uint8_t* mR, const uint8_t* mD, const uint16_t* wR, const uint16_t* wD,
                     SmLayout& L);
