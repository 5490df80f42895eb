// sm_knob.cpp -- the knob table behind sm_set_knob (include/stereomst.h) and sm_knob (sm_knob.h).
#include "sm_knob.h"

#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <string>

#include "../../include/stereomst.h"

namespace {

// Every knob a product build reads.  Schedule knobs never change a result (the engines are exact
// under any schedule); diagnostics print to stderr or count; SM_TEST_PMS_CYCLE is the
// forest test's fault injection.
const char* const kKnobs[] = {
    // segment forest launch schedules (sm_api.cpp, sm_seg_gpu.hip)
    "SM_SEG_HOST", "SM_SEG_FLATTEN", "SM_SEG_NOSPLIT", "SM_SEG_NORUN", "SM_SEG_GLOBAL_ROUNDS", "SM_SEG_SMALL",
    "SM_SEG_TAIL_GLOBAL", "SM_SEG_TAIL_MIN", "SM_SEG_ACT_MAX",
    // MST engine schedules (sm_kernels.hip)
    "SM_MST_PIXEL_ROUNDS", "SM_MST_LOCAL_ITERS",
    // tree filter: pieces, repairs, bounded waits, heavy-leaf f32 rows (sm_chain.hip, sm_walk.hip)
    "SM_PIECE_LEN", "SM_REPAIR_MAX", "SM_WAIT_ITERS", "SM_NO_LEAF_COST",
    // MST_PMS schedules (sm_pms.hip, sm_pms_forest.hip)
    "SM_PMS_SERIAL", "SM_PMS_MAX_ROUNDS", "SM_PMS_PIECE", "SM_PMS_BIG", "SM_PMS_CHAIN_MIN", "SM_PMS_CHAIN_NSU",
    "SM_PMS_CHAIN_NSD", "SM_PMS_HOST_FOREST", "SM_PMS_FOREST_CHECK", "SM_PREP_THREADS",
    // guided-filter kernel variants (sm_guided.hip)
    "SM_GF_UNFUSED", "SM_GF_DIRECT_X",
    // diagnostics (stderr, counters)
    "SM_LAYOUT_DEBUG", "SM_LAYOUT_CHECK", "SM_MST_DEBUG", "SM_SEG_DEBUG", "SM_SEG_PROF", "SM_PIECE_DEBUG", "SM_PMS_PROF",
    "SM_PMS_TREE_TIMES", "SM_PMS_COUNT_RUN", "SM_PREP_DEBUG",
    // fault injection of test_pms_forest_cycle_is_an_error
    "SM_TEST_PMS_CYCLE",
};

std::mutex g_mu;
std::map<std::string, const char*> g_set;  // name -> value (interned, never freed)
std::deque<std::string> g_pool;            // the interned values: a reader's pointer stays valid

bool known(const char* name) {
    for (const char* k : kKnobs)
        if (strcmp(k, name) == 0) return true;
    return false;
}

}  // namespace

const char* sm_knob(const char* name) {
    {
        std::lock_guard<std::mutex> lk(g_mu);
        auto it = g_set.find(name);
        if (it != g_set.end()) return it->second;
    }
#ifdef SM_DEV
    return getenv(name);
#else
    return nullptr;
#endif
}

int sm_knob_int(const char* name, int dflt) {
    const char* v = sm_knob(name);
    return v ? atoi(v) : dflt;
}

extern "C" sm_status sm_set_knob(const char* name, const char* value) {
    if (!name || !known(name)) return SM_ERR_ARG;
    std::lock_guard<std::mutex> lk(g_mu);
    if (!value) {
        g_set.erase(name);
    } else {
        g_pool.emplace_back(value);
        g_set[name] = g_pool.back().c_str();
    }
    return SM_OK;
}

extern "C" int sm_knob_names(const char** out, int cap) {
    const int n = (int)(sizeof(kKnobs) / sizeof(kKnobs[0]));
    for (int i = 0; i < n && out && i < cap; ++i) out[i] = kKnobs[i];
    return n;
}
