// sm_api.cpp -- C-ABI (include/stereomst.h): context, orchestration of the HIP stages,
// RCCL min+argmin reduce for disparity sharding, timers.
//
// Pipeline of one frame (both views in every launch, blockIdx selects the view):
//   prep -> median -> weights -> Boruvka MST -> tree layout -> up rounds -> down rounds (+WTA)
//   [-> RCCL allreduce(min f64) + allreduce(min i32 candidate index) when sharded over ranks]
// There is no CPU fallback: without a HIP device every entry returns SM_ERR_NODEVICE.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <sys/time.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/stereomst.h"
#include "sm_common.h"
#include "sm_launch.h"
#include "sm_layout_gpu.h"
#include "sm_pms.h"
#include "sm_pms_forest.h"
#include "sm_reduce_rule.h"
#include "sm_seg_gpu.h"
#include "sm_segment.h"
#include "sm_tables.inc"
#include "sm_knob.h"

hipError_t launch_cand(hipStream_t st, const double* minc, const double* gmin, const int32_t* idx, int32_t* cand, size_t N);
hipError_t launch_finalize(hipStream_t st, const double* gmin, const int32_t* gidx, double* minc, int32_t* idx, float* disp,
                           size_t N);
hipError_t launch_cand64(hipStream_t st, const double* minc, const double* gmin, const int32_t* idx, const float* disp,
                         unsigned long long* cand, size_t N);
hipError_t launch_finalize64(hipStream_t st, const double* gmin, const unsigned long long* gkey, double* minc, int32_t* idx,
                             float* disp, size_t N);

namespace {

constexpr size_t RREC_FWD = (SM_NBUCKETS + 1) + SM_NBUCKETS + SM_NBUCKETS + 2 + SM_NBUCKETS + (SM_NBUCKETS + 1) + SM_NBUCKETS +
                            (SM_NBUCKETS + 1);

struct DevBuf {
    void* p = nullptr;
    size_t n = 0;
};

// pinned host array (segment mode's weight / mask copies: the copies run asynchronously to the host
// thread and read or fill the memory when the stream reaches them)
template <class T>
struct PinnedVec {
    T* p = nullptr;
    size_t n = 0;
    PinnedVec() = default;
    PinnedVec(const PinnedVec&) = delete;
    PinnedVec& operator=(const PinnedVec&) = delete;
    ~PinnedVec() {
        if (p) (void)hipHostFree(p);
    }
    bool resize(size_t m) {  // capacity; contents undefined
        if (p && m <= n) return true;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
        if (hipHostMalloc((void**)&p, (m ? m : 1) * sizeof(T)) != hipSuccess) return false;
        n = m;
        return true;
    }
    T* data() { return p; }
    const T* data() const { return p; }
    T& operator[](size_t i) { return p[i]; }
    const T& operator[](size_t i) const { return p[i]; }
};

// MST_PMS state of one view (SM_AGG_PMS, sm_pms.hip): the host forest and schedule, their device
// copies, labels, aggregation rows, cost rows and the speculation scratch
// buffers of the GPU forest build (sm_pms_forest.hip), kept between calls
struct PfBufs {
    DevBuf par, flag, tree_of, nbr, nbw, root_pix, tsize, gpix, gpar, gtree, gw, gfc, gnc, gsize, ghk, iota, rot, pdir, psize,
        bpos, a_dist, a_cid, nchains, c_last, c_len, cnw, tval, tval_s, tkey0, tkey1, tpix0, tpix1,
        bglob, gtree_s, g2b, bpar, bch0, J0, J1, D0, D1, plen, ld, rowof, rowstart, hflag, hidx, hkey0, hkey1, cutof,
        hcnt[4], hoff[4], rtc[4], rt[4], pairs0, pairs1, npairs, uflag, uidx, nbcnt, cut_round, tree_cut, tot, temp;
};

struct PmsState {
    PmsForest f;
    PfBufs pf;
    DevBuf rows, rtree, paths, items, rt_path, rt_item, tree_rounds, tree_start, bfs_pix, nb_start, nb, tree_pt, tree_abase,
        tree_lab, nref, lab, labq, abc, minc, abc_bak, minc_bak, A, vrows, off, oguess, cnt, flag, result, prof, cuts, reps,
        cut_bak, Abak, labu, nprop, rep_flag, pt_ph, ab_ph, plan_cnt, plan_path, plan_item, plan_base, plan_ibase;
    std::vector<int32_t> h_rtree, h_pt, h_lab;
    std::vector<long long> h_abase;
    long long dice_need = 0;
    PmsDev dev{};
};

// segment mode's GPU segmentation of one view (sm_seg_gpu.hip): union-find state, bucketed edges,
// candidate / rejected / hooked lists, counters; pinned copies of the bucket starts, the counters and
// the min-size candidates, and the host merge's hooks
struct SegGpu {
    DevBuf par, sz, wl, best, first, ebuf, bcnt, list0, list1, rej, hooked, cnt, mlist, hooks, mkey, mval, msorted, stemp;
    DevBuf keep, kpos, lmark, lid, dense, lsize, lroot;  // the pair dedupe (seg_launch_dedupe)
    size_t stemp_bytes = 0;
    uint32_t gen = 0;  // next Boruvka generation (keys of older ones lose every atomicMin)
    PinnedVec<uint32_t> h_b, h_cnt, h_hooks, h_lsize, h_lroot;
    PinnedVec<SegEdge> h_dense;
    std::vector<SegEdge> h_dsort;  // seg_sort_dense's scratch
    std::vector<uint32_t> mpar, msize;  // the merge's union-find over local ids
};

struct MstPending {
    bool active = false;
    int nviews = 0, r = 0;  // contracted rounds enqueued
    MstArgs a{};
    MstCompact c{};
};

}  // namespace

struct sm_ctx {
    int device = 0;
    hipStream_t st = nullptr;
    // Stream of the long-path chain engine.  Measured (round 1): running it on a second stream
    // concurrently with the short-path walkers loses -- every round boundary then costs a
    // ~30 us cross-stream join and the throughput-bound k_up_pre only competes with the walkers --
    // so it aliases st; the round code keeps the two-stream structure (join() is then a no-op).
    hipStream_t st2 = nullptr;
    // Everything of a call runs on st.  A tree stream of its own (prep / MST / layout, the filter
    // waiting by event) was measured slower at either priority: the tree at the lowest priority, C2
    // 4.82 -> 5.43-5.50 ms/frame (round 2); at the highest, 4.80-4.82 -> 5.12-5.16 (round 5).
    std::string err;
    int W = 0, H = 0, stride = 0;
    DevBuf img[2], bgrx[2], gray[2], med[2], wR[2], wD[2], comp[2], best[2], root[2], mR[2], mD[2];
    DevBuf changed, mst_ok, atab, slut, s2lut, meta[2], paths[2], U[2], Cst[2], idx[2], minc[2], disp[2];
    DevBuf cand[2], gmin[2], gidx[2], vol[2], rec[2], rec4[2];
    DevBuf post_mask, post_scratch;  // output step (sm_post.hip): marks, scan positions
    // guided-filter aggregator (sm_guided.hip): guide planes / means, per-view statistics, batch
    // planes, box scratch, WTA state
    DevBuf gf_planes, gf_means, gf_stats[2], gf_pl, gf_tmp, gf_state[2];
    // segment mode (finite c, sm_segment.cpp): layout weights with the virtual edges, and host copies
    DevBuf fwR[2], fwD[2];
    bool seg = false;  // the current tree is a segment forest (layout reads fwR / fwD)
    bool want_size = false;  // the layout writes subtree sizes (sm_build_tree reports them)
    bool sub = false;  // the current call's WTA carries subpixel disparities (SM_POST_SUBPIXEL)
    int seg_trees[2] = {0, 0};
    PinnedVec<uint16_t> h_w[2][2], h_fw[2][2];
    PinnedVec<uint8_t> h_m[2][2];
    SegGpu sg[2];  // GPU segmentation (default; SM_SEG_HOST=1: the host sweep of sm_segment.cpp)
    // asynchronous segment mode (sm_match_begin): the host segmentation runs on a worker thread that
    // waits for the weights' copy (ev_segw), uploads the forest and enqueues the layout; sm_match_finish
    // joins it
    std::thread seg_worker;
    sm_status seg_status = SM_OK;
    hipEvent_t ev_segw = nullptr;
    size_t rec_pad_n[2] = {0, 0};  // pixel count the record pads were zeroed for
    size_t rec_pad_z[2] = {0, 0};  // pad length (records) they were zeroed with
    // records of padding on each side of the image records: the walkers read the matched image
    // at pix +- (disp_begin + Dpad) (sm_walk_util.h load_recs), so the pad follows the call's range
    size_t rec_pad = SM_REC_PAD;
    DevBuf vin[2];               // MC-CNN ingest: caller volumes [vin_D][H][W] f32 per view
    int vin_W = 0, vin_H = 0, vin_D = 0;
    bool use_vol = false;        // the current call takes its costs from vin (SM_COST_VOLUME)
    int views = 3;               // views of the last call (sm_params.views; bit 0 left, bit 1 right)
    DevBuf cedge[2], clab[2], chook[2], ccnt[2];  // contracted Boruvka (component graph)
    uint32_t epoch = 0;      // bumped per filter call; status words are zeroed only on (re)allocation
    // GPU layout buffers (sm_layout_gpu.hip)
    DevBuf adj[2], pdir[2], heavy[2], size[2], arcpix[2], hk[2], pixpre[2];
    DevBuf a_dist[2], a_cid[2], ccount[2], c_last[2], c_len[2];
    DevBuf segtab[2], pathpos[2], plen[2], slotpix[2], lrank[2], wrow[2];
    DevBuf pieces[2], pieces_tmp[2], agg[2], pstat[2], fix[2], pdbg;  // long-path pieces: table, segment aggregates, status words
    // the down pass's A rows of light children's parents (compact: n_has_light rows, SmMeta::cslot[3]), and
    // every node's A row by slot for the debug calls only (round 6: A was one dense row per slot)
    DevBuf acmp[2], adbg[2];
    DevBuf cnw[2], tour[2], spart[2], rounds[2];
    int* h_changed = nullptr;
    uint32_t* h_err = nullptr;  // pinned, device-visible error word of the chain engine's waits
    uint32_t* d_err = nullptr;  // its device address
    int mst_rounds = 12;  // contracted Boruvka rounds the previous frame needed
    MstPending mst_pend;  // rounds enqueued without a host check (stage_mst -> mst_finish)
    uint32_t* h_rounds = nullptr;  // pinned: per view [SM_MAX_ROUNDS+1 begin | nrounds | n_has_light]
    struct HostRounds {
        uint32_t nrounds = 0, npaths = 0, n_has_light = 0;
        std::vector<uint32_t> begin, maxlen, seg_begin, nodes, piece_begin;  // per bucket
    } layout[2];
    hipEvent_t ev[8] = {};
    hipEvent_t ev_layout = nullptr;  // after the layout's round-count copy (stage_layout_finish waits)
    // sm_match_begin -> sm_match_finish: the call in between (0: none, 1: tree enqueued, 2: guided,
    // fully enqueued by begin)
    int pending = 0;
    int pend_D = 0;
    bool exp_layout_ok = false;  // SM_EXP_FILTER_ONLY (timing experiment): a layout of these images exists
    sm_params pend_p{};
    // tree-filter launch timing: timed launch k runs between events fev[fam_ev[k]] on its stream
    std::vector<hipEvent_t> fev;
    std::vector<int> fam;
    std::vector<double> fam_vox;  // voxels of launch k
    std::vector<std::pair<int, int>> fam_ev;  // its start / end event
    int nfev = 0;
    bool ev_open = false;  // the last op on ev_stream was a timed launch's end event
    hipStream_t ev_stream = nullptr;
    std::vector<hipEvent_t> sev;  // stream-ordering events of the filter rounds
    int nsev = 0;
    sm_filter_stats stats{};
    sm_kernel_stat kstats[8]{};  // >= KF_N
    unsigned ktiming = ~0u;      // families timed with events (sm_set_kernel_timing)
    float stage_ms[7] = {0};
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;
    bool reduced = false;
    // MST_PMS (SM_AGG_PMS)
    PmsState pms[2];
    DevBuf pms_dice, pms_rnd, pms_evals;
    hipStream_t st_pms = nullptr;  // view 1's MST_PMS calls (view 0's run on st), created on first use
    hipEvent_t ev_pms = nullptr;
    long long pms_dice_n = 0;  // dice values on the device (the stream prefix every call replays)
    std::vector<float> pms_init;   // random plane labels of (W, H, Dmax) (both views start from them)
    int pms_init_key[3] = {0, 0, 0};
    std::vector<double> pms_dblmax;
    std::vector<int32_t> pms_hrnd;
    int32_t* h_pms_res = nullptr;  // pinned: the validation result
    bool pms_last = false;         // the last call was SM_AGG_PMS (labels available)
    int pms_W = 0, pms_H = 0;      // its image size (the labels' extent)
    sm_pms_stats pms_stats{};
};

namespace {

// (the two view threads of an MST_PMS call may fail at once: the message is written under a lock)
std::mutex g_err_mu;
sm_status fail(sm_ctx* c, sm_status s, const std::string& msg) {
    if (c) {
        std::lock_guard<std::mutex> lk(g_err_mu);
        c->err = msg;
    }
    return s;
}

#define HIPC(call)                                                                                    \
    do {                                                                                              \
        hipError_t e_ = (call);                                                                       \
        if (e_ != hipSuccess)                                                                         \
            return fail(ctx, e_ == hipErrorOutOfMemory ? SM_ERR_OOM : SM_ERR_HIP,                     \
                        std::string(#call) + ": " + hipGetErrorString(e_));                         \
    } while (0)

#define RCCLC(call)                                                                                   \
    do {                                                                                              \
        ncclResult_t r_ = (call);                                                                     \
        if (r_ != ncclSuccess) return fail(ctx, SM_ERR_RCCL, std::string(#call) + ": " + ncclGetErrorString(r_)); \
    } while (0)

#define CHECK(expr)                  \
    do {                             \
        sm_status s_ = (expr);       \
        if (s_ != SM_OK) return s_;  \
    } while (0)

sm_status ensure(sm_ctx* ctx, DevBuf& b, size_t bytes) {
    if (b.n >= bytes && b.p) return SM_OK;
    if (b.p) HIPC(hipFree(b.p));
    b.p = nullptr;
    b.n = 0;
    HIPC(hipMalloc(&b.p, bytes ? bytes : 16));
    b.n = bytes;
    return SM_OK;
}

template <class T>
T* P(DevBuf& b) {
    return reinterpret_cast<T*>(b.p);
}

int spl_for(int D) { return D <= 64 ? 1 : D <= 128 ? 2 : 4; }
// row length of a call of D slices: 64 * SPL, or 32 for D <= 32 (a 32-slice shard moves 32-slice
// rows; SM_NO_DPAD32=1 restores 64 for A/B)
int dpad_for(int D) {
    static const bool off = sm_dev_knob("SM_NO_DPAD32") != nullptr;
    return (D <= 32 && !off) ? 32 : 64 * spl_for(D);
}

float agd_color_term(int l1) {
    // 0.11f*fminf(color_l1*0.33333333333, 7.0f) (PatchMatchStereoGPU.cu:1539)
    const float scaled = (float)((double)(float)l1 * 0.33333333333);
    return 0.11f * fminf(scaled, 7.0f);
}

sm_status check_params(sm_ctx* ctx, const sm_params* p, int D) {
    if (!p) return fail(ctx, SM_ERR_ARG, "null params");
    if (std::isnan(p->c) || p->c < 0) return fail(ctx, SM_ERR_ARG, "c must be >= 0 (finite: segment mode) or +INFINITY (MST mode)");
    if (p->median_ksize != 3) return fail(ctx, SM_ERR_ARG, "only median_ksize=3 is supported");
    if (p->cost_kind != SM_COST_AGD && p->cost_kind != SM_COST_VOLUME) return fail(ctx, SM_ERR_ARG, "unknown cost_kind");
    if (p->gamma != 1.0f / 12.f)
        return fail(ctx, SM_ERR_ARG, "only gamma=1/12 (embedded correctly-rounded tables) is supported");
    if (D < 1 || D > 256) return fail(ctx, SM_ERR_ARG, "D must be in [1, 256] per call (shard larger ranges)");
    if (p->disp_begin < 0) return fail(ctx, SM_ERR_ARG, "disp_begin < 0");
    if (p->disp_begin > (1 << 20)) return fail(ctx, SM_ERR_ARG, "disp_begin > 2^20");
    if (p->disp_total != 0 && p->disp_total < p->disp_begin + D)
        return fail(ctx, SM_ERR_ARG, "disp_total < disp_begin + D (shard beyond the total range)");
    const int known = SM_POST_LR_CHECK | SM_POST_LABEL_TO_DISP | SM_POST_LR_FILL | SM_POST_OCCLUSION | SM_POST_OCCLUSION_ZERO |
                      SM_POST_SUBPIXEL;
    if (p->post & ~known) return fail(ctx, SM_ERR_ARG, "unknown post-processing bits");
    if ((p->post & SM_POST_LR_FILL) && !(p->post & SM_POST_LR_CHECK))
        return fail(ctx, SM_ERR_ARG, "SM_POST_LR_FILL needs SM_POST_LR_CHECK");
    if ((p->post & SM_POST_OCCLUSION) && (p->post & SM_POST_OCCLUSION_ZERO))
        return fail(ctx, SM_ERR_ARG, "SM_POST_OCCLUSION and SM_POST_OCCLUSION_ZERO are exclusive");
    if (p->aggregator != SM_AGG_TREE && p->aggregator != SM_AGG_GUIDED && p->aggregator != SM_AGG_PMS)
        return fail(ctx, SM_ERR_ARG, "unknown aggregator");
    if (p->aggregator == SM_AGG_PMS) {
        if (p->disp_begin != 0 || (p->disp_total != 0 && p->disp_total != D))
            return fail(ctx, SM_ERR_ARG, "SM_AGG_PMS: unsharded only (disp_begin 0, D = Dmax)");
        if (p->views != 0 && p->views != 3) return fail(ctx, SM_ERR_ARG, "SM_AGG_PMS computes both views");
        if (D < 2) return fail(ctx, SM_ERR_ARG, "SM_AGG_PMS needs Dmax >= 2");
        if (p->pms_iters < 0 || p->pms_iters > 100000) return fail(ctx, SM_ERR_ARG, "SM_AGG_PMS: pms_iters out of range");
        if (p->post & SM_POST_SUBPIXEL) return fail(ctx, SM_ERR_ARG, "SM_AGG_PMS: no subpixel step (labels are planes)");
        return SM_OK;
    }
    if (p->views < 0 || p->views > 3) return fail(ctx, SM_ERR_ARG, "views must be 1 (left), 2 (right) or 3 / 0 (both)");
    if (p->views == 1 || p->views == 2) {
        if (p->aggregator != SM_AGG_TREE) return fail(ctx, SM_ERR_ARG, "a one-view call needs SM_AGG_TREE");
        if (p->post & ~SM_POST_SUBPIXEL)
            return fail(ctx, SM_ERR_ARG, "a one-view call takes no post-processing that needs both maps (only SM_POST_SUBPIXEL)");
    }
    if (p->aggregator == SM_AGG_GUIDED) {
        if (p->cost_kind != SM_COST_AGD) return fail(ctx, SM_ERR_ARG, "SM_AGG_GUIDED filters the AGD cost only");
        if (p->gf_radius < 1 || p->gf_radius > 64 || !(p->gf_eps > 0)) return fail(ctx, SM_ERR_ARG, "bad guided-filter radius / eps");
        if ((p->post & SM_POST_SUBPIXEL) && (p->disp_begin > 0 || (p->disp_total > 0 && p->disp_total != D)))
            return fail(ctx, SM_ERR_ARG, "SM_AGG_GUIDED: subpixel on a shard is not supported");
        return SM_OK;
    }
    if (p->post & SM_POST_SUBPIXEL) {
        const int dtot = p->disp_total > 0 ? p->disp_total : p->disp_begin + D;
        const int halo = (p->disp_begin > 0) + (p->disp_begin + D < dtot);
        if (D + halo > 256)
            return fail(ctx, SM_ERR_ARG, "SM_POST_SUBPIXEL on a shard needs D + its 1-slice halos <= 256");
    }
    return SM_OK;
}

// the slices a call computes: [disp_begin, disp_begin + D), plus for SM_POST_SUBPIXEL on a shard a
// one-slice halo on each inner side, so the parabola of the shard's winner has both neighbours
// locally; the WTA itself covers the shard only
struct CallRange {
    int d0, D;  // computed slices (global first, count)
    WtaCfg w;
};
CallRange call_range(const sm_params* p, int D) {
    const int dtot = p->disp_total > 0 ? p->disp_total : p->disp_begin + D;
    const int sub = (p->post & SM_POST_SUBPIXEL) ? 1 : 0;
    const int h0 = sub && p->disp_begin > 0 ? 1 : 0, h1 = sub && p->disp_begin + D < dtot ? 1 : 0;
    CallRange r;
    r.d0 = p->disp_begin - h0;
    r.D = D + h0 + h1;
    r.w = WtaCfg{h0, h0 + D, r.d0, dtot, sub};
    return r;
}

// image-record pad for a call over slices [disp_begin, disp_begin + Dpad): load_recs reads records
// pix - disp_begin - Dpad .. pix + disp_begin + Dpad + 1 (sm_walk_util.h)
size_t rec_pad_for(int disp_begin, int D) {
    const size_t need = (size_t)disp_begin + 64 * (size_t)spl_for(D) + 64;
    return need <= SM_REC_PAD ? SM_REC_PAD : (need + 1023) / 1024 * 1024;
}

// views of a call: bit 0 = left, bit 1 = right (sm_params.views); stages that run view-agnostic
// kernels (MST, layout) pack the active views into the kernels' view slots 0 .. n-1
struct ViewSet {
    int n = 0;
    int v[2] = {0, 1};
    explicit ViewSet(int mask) {
        for (int q = 0; q < 2; ++q)
            if ((mask >> q) & 1) v[n++] = q;
        if (n == 1) v[1] = v[0];  // an unused kernel slot aliases the active view: never an unallocated buffer
    }
};
inline bool view_on(int mask, int v) { return ((mask >> v) & 1) != 0; }

// ----------------------------------------------------------------------------- stages
sm_status stage_prep(sm_ctx* ctx) {
    const int W = ctx->W, H = ctx->H;
    const size_t N = (size_t)W * H;
    for (int v = 0; v < 2; ++v) {
        CHECK(ensure(ctx, ctx->bgrx[v], N * 4));
        CHECK(ensure(ctx, ctx->gray[v], N * 4));
        CHECK(ensure(ctx, ctx->med[v], N * 4));
        CHECK(ensure(ctx, ctx->wR[v], N * 2));
        CHECK(ensure(ctx, ctx->wD[v], N * 2));
        const void* old = ctx->rec[v].p;
        const void* old4 = ctx->rec4[v].p;
        const size_t pad = ctx->rec_pad;
        CHECK(ensure(ctx, ctx->rec[v], (N + 2 * pad) * 8));
        CHECK(ensure(ctx, ctx->rec4[v], (N + 2 * pad) * 4));
        if (ctx->rec[v].p != old || ctx->rec4[v].p != old4 || ctx->rec_pad_n[v] != N || ctx->rec_pad_z[v] != pad) {
            // zero pads around the records: once per allocation, size and pad
            ctx->rec_pad_n[v] = N;
            ctx->rec_pad_z[v] = pad;
            HIPC(hipMemsetAsync(ctx->rec[v].p, 0, pad * 8, ctx->st));
            HIPC(hipMemsetAsync(P<uint2>(ctx->rec[v]) + pad + N, 0, pad * 8, ctx->st));
            HIPC(hipMemsetAsync(ctx->rec4[v].p, 0, pad * 4, ctx->st));
            HIPC(hipMemsetAsync(P<uint32_t>(ctx->rec4[v]) + pad + N, 0, pad * 4, ctx->st));
        }
    }
    HIPC(launch_prep(ctx->st, P<uint8_t>(ctx->img[0]), P<uint8_t>(ctx->img[1]), W, H, ctx->stride, P<uint32_t>(ctx->bgrx[0]),
                     P<float>(ctx->gray[0]), P<uint32_t>(ctx->bgrx[1]), P<float>(ctx->gray[1]),
                     P<uint2>(ctx->rec[0]) + ctx->rec_pad, P<uint2>(ctx->rec[1]) + ctx->rec_pad,
                     P<uint32_t>(ctx->rec4[0]) + ctx->rec_pad, P<uint32_t>(ctx->rec4[1]) + ctx->rec_pad));
    HIPC(launch_median_weights(ctx->st, P<uint32_t>(ctx->bgrx[0]), P<uint32_t>(ctx->bgrx[1]), P<uint32_t>(ctx->med[0]),
                               P<uint32_t>(ctx->med[1]), P<uint16_t>(ctx->wR[0]), P<uint16_t>(ctx->wD[0]),
                               P<uint16_t>(ctx->wR[1]), P<uint16_t>(ctx->wD[1]), W, H));
    return SM_OK;
}

static bool hooked_any(const int* hf, int nviews, int q) {
    return hf[q] != 0 || (nviews > 1 && hf[SM_MST_MAX_ROUNDS + q] != 0);
}

sm_status stage_mst(sm_ctx* ctx, int views);

// Segment mode: the reference's order-dependent Felzenszwalb segmentation + min-size merge on the host
// (sm_segment.cpp), from the GPU's edge weights; the forest, linked into one tree by S = 0 virtual
// edges, goes back as the MST masks and the layout's weights.  Replaces stage_mst.  Three parts:
// the weights' copy to pinned host memory (recorded by ev_segw), the host segmentation of the views
// (one thread each), the forest's copy back.
sm_status segment_download(sm_ctx* ctx, int views) {
    const size_t N = (size_t)ctx->W * ctx->H;
    const ViewSet vs(views);
    for (int i = 0; i < vs.n; ++i) {
        const int v = vs.v[i];
        CHECK(ensure(ctx, ctx->mR[v], N));
        CHECK(ensure(ctx, ctx->mD[v], N));
        CHECK(ensure(ctx, ctx->fwR[v], N * 2));
        CHECK(ensure(ctx, ctx->fwD[v], N * 2));
        for (int k = 0; k < 2; ++k)
            if (!ctx->h_w[v][k].resize(N) || !ctx->h_fw[v][k].resize(N) || !ctx->h_m[v][k].resize(N))
                return fail(ctx, SM_ERR_OOM, "segment mode: pinned host buffers");
        HIPC(hipMemcpyAsync(ctx->h_w[v][0].data(), ctx->wR[v].p, N * 2, hipMemcpyDeviceToHost, ctx->st));
        HIPC(hipMemcpyAsync(ctx->h_w[v][1].data(), ctx->wD[v].p, N * 2, hipMemcpyDeviceToHost, ctx->st));
    }
    CHECK(ensure(ctx, ctx->mst_ok, sizeof(int)));
    HIPC(hipEventRecord(ctx->ev_segw, ctx->st));
    return SM_OK;
}

sm_status segment_host(sm_ctx* ctx, int views, float c, int min_size) {
    const int W = ctx->W, H = ctx->H;
    const ViewSet vs(views);
    HIPC(hipEventSynchronize(ctx->ev_segw));
    std::thread other;
    auto run = [ctx, W, H, c, min_size](int v) {
        ctx->seg_trees[v] = sm_segment_forest(ctx->h_w[v][0].data(), ctx->h_w[v][1].data(), W, H, c, min_size,
                                              ctx->h_m[v][0].data(), ctx->h_m[v][1].data(), ctx->h_fw[v][0].data(),
                                              ctx->h_fw[v][1].data());
    };
    if (vs.n > 1) other = std::thread(run, vs.v[1]);
    run(vs.v[0]);
    if (other.joinable()) other.join();
    return SM_OK;
}

sm_status segment_upload(sm_ctx* ctx, int views) {
    const size_t N = (size_t)ctx->W * ctx->H;
    const ViewSet vs(views);
    for (int i = 0; i < vs.n; ++i) {
        const int v = vs.v[i];
        HIPC(hipMemcpyAsync(ctx->mR[v].p, ctx->h_m[v][0].data(), N, hipMemcpyHostToDevice, ctx->st));
        HIPC(hipMemcpyAsync(ctx->mD[v].p, ctx->h_m[v][1].data(), N, hipMemcpyHostToDevice, ctx->st));
        HIPC(hipMemcpyAsync(ctx->fwR[v].p, ctx->h_fw[v][0].data(), N * 2, hipMemcpyHostToDevice, ctx->st));
        HIPC(hipMemcpyAsync(ctx->fwD[v].p, ctx->h_fw[v][1].data(), N * 2, hipMemcpyHostToDevice, ctx->st));
    }
    HIPC(hipMemsetAsync(ctx->mst_ok.p, 1, sizeof(int), ctx->st));
    return SM_OK;
}

// SM_SEG_HOST=1: segment mode's segmentation by the host sweep (sm_segment.cpp) instead of the GPU
bool seg_host() { return sm_knob("SM_SEG_HOST") != nullptr; }

// SM_SEG_FLATTEN: bit 0: point every pixel at its root before each run of one-workgroup buckets (default),
// bit 1: before each whole-GPU bucket as well; 0: never
int seg_flatten() { return sm_knob("SM_SEG_FLATTEN") ? atoi(sm_knob("SM_SEG_FLATTEN")) : 1; }

// a small-bucket run starts with k_seg_split (SM_SEG_NOSPLIT=1: every edge of the run through k_seg_small)
bool seg_split() { return sm_knob("SM_SEG_NOSPLIT") == nullptr; }

// Boruvka rounds launched over the whole GPU before a bucket's single-workgroup tail, for buckets of
// more than SM_SEG_SMALL edges (env SM_SEG_GLOBAL_ROUNDS, default 3: the LDS tail then gets the ~2.7k
// still-crossing candidates at most; latency 9.96 -> 9.7 ms, profiles/r04/seg/r04ao/)
int seg_global_rounds() { return sm_knob("SM_SEG_GLOBAL_ROUNDS") ? atoi(sm_knob("SM_SEG_GLOBAL_ROUNDS")) : 3; }

// buckets of at most this many edges run in one workgroup, consecutive ones in one launch (k_seg_small;
// env SM_SEG_SMALL, default 16384)
uint32_t seg_small() { return sm_knob("SM_SEG_SMALL") ? (uint32_t)atoi(sm_knob("SM_SEG_SMALL")) : 16384u; }

// the hashed pair dedupe's kept candidates (unordered) into the merge's (w, id) order: LSD radix sort of the
// key (w << 32) | id in four 11-bit digits (w < 2^10, id < 2^23 for images below 4.19 M pixels; the full
// 42 bits otherwise) -- ~23k edges per C2 view, well under 0.1 ms
void seg_sort_dense(SegEdge* e, uint32_t n, std::vector<SegEdge>& tmp) {
    if (n < 2) return;
    uint32_t idmax = 0;
    for (uint32_t i = 0; i < n; ++i) idmax = std::max(idmax, e[i].id);
    int idbits = 1;
    while (idbits < 32 && (1ull << idbits) <= idmax) ++idbits;
    const int bits = idbits + 10;  // w < 1024
    tmp.resize(n);
    SegEdge* src = e;
    SegEdge* dst = tmp.data();
    auto key = [idbits](const SegEdge& x) { return ((unsigned long long)x.w << idbits) | x.id; };
    std::vector<uint32_t> cnt(2048);
    for (int sh = 0; sh < bits; sh += 11) {
        std::fill(cnt.begin(), cnt.end(), 0u);
        for (uint32_t i = 0; i < n; ++i) ++cnt[(key(src[i]) >> sh) & 2047u];
        uint32_t run = 0;
        for (uint32_t& c : cnt) {
            const uint32_t t = c;
            c = run;
            run += t;
        }
        for (uint32_t i = 0; i < n; ++i) dst[cnt[(key(src[i]) >> sh) & 2047u]++] = src[i];
        std::swap(src, dst);
    }
    if (src != e) std::copy(src, src + n, e);
}

// The reference's min-size merge (Stereo3DMST.cpp:293-307) over the deduplicated candidates (the first
// candidate of each pair of sweep roots, in (w, id) order, with the roots as dense local ids; lsize /
// lroot: their sizes and pixels): the serial rule on a union-find.  Emits the hooks (child root, parent
// root) and the joined edge ids for k_seg_apply.
int seg_minsize_dense(const SegEdge* e, uint32_t n, uint32_t nl, const uint32_t* lsize, const uint32_t* lroot, uint32_t ms,
                      uint32_t* out, std::vector<uint32_t>& par, std::vector<uint32_t>& size) {
    par.resize(nl);
    size.assign(lsize, lsize + nl);
    for (uint32_t i = 0; i < nl; ++i) par[i] = i;
    uint32_t* P = par.data();
    uint32_t* S = size.data();
    auto find = [P](uint32_t x) {
        while (P[x] != x) x = P[x] = P[P[x]];
        return x;
    };
    uint32_t* ids = out + 2 * (size_t)n;  // scratch: the marked ids, moved behind the k pairs at the end
    int k = 0;
    for (uint32_t j = 0; j < n; ++j) {
        if (j + 16 < n) {
            __builtin_prefetch(&P[e[j + 16].la]);
            __builtin_prefetch(&P[e[j + 16].lb]);
        }
        uint32_t a = find(e[j].la), b = find(e[j].lb);
        if (a == b) continue;
        uint32_t sa = S[a], sb = S[b];
        if (sa >= ms && sb >= ms) continue;
        if (sa < sb) {
            std::swap(a, b);
            std::swap(sa, sb);
        }
        P[b] = a;
        S[a] = sa + sb;
        out[2 * k] = lroot[b];
        out[2 * k + 1] = lroot[a];
        ids[k] = e[j].id;
        ++k;
    }
    memmove(out + 2 * (size_t)k, ids, (size_t)k * 4);
    return k;
}

double now_ms();

// Segment mode's segmentation on the GPU (sm_seg_gpu.h): the masks and layout weights of the forest
// land in mR / mD / fwR / fwD as segment_upload leaves them.  Both views go through every launch, on
// the context's stream, bucket by bucket in lockstep.  Host synchronisations: the bucket sizes (once),
// the min-size candidates (twice).  With host_copy the weights, masks and layout weights are copied to
// the h_w / h_m / h_fw host arrays as well (MST_PMS, sm_build_tree_p).
sm_status segment_gpu(sm_ctx* ctx, int views, float c, int min_size, bool host_copy) {
    const bool dbg = sm_knob("SM_SEG_DEBUG") != nullptr;
    const int flatten = seg_flatten();
    const double t0 = dbg ? now_ms() : 0.0;
    double t1 = 0, t2 = 0, t3 = 0, t4 = 0;
    const int W = ctx->W, H = ctx->H;
    const size_t N = (size_t)W * H, E = 2 * N;
    const ViewSet vs(views);
    hipStream_t st = ctx->st;
    SegPair sp{};
    sp.nv = vs.n;
    bool reset = false;
    uint32_t gen = 1;
    for (int i = 0; i < vs.n; ++i) {
        const SegGpu& g = ctx->sg[vs.v[i]];
        reset |= g.best.n < N * 8 || g.gen > 0xF0000000u;
        gen = std::max(gen, g.gen);
    }
    if (reset) gen = 1;  // keys of generation >= 1 beat the initial all-ones
    for (int i = 0; i < vs.n; ++i) {
        const int v = vs.v[i];
        SegGpu& g = ctx->sg[v];
        CHECK(ensure(ctx, ctx->mR[v], N));
        CHECK(ensure(ctx, ctx->mD[v], N));
        CHECK(ensure(ctx, ctx->fwR[v], N * 2));
        CHECK(ensure(ctx, ctx->fwD[v], N * 2));
        CHECK(ensure(ctx, g.par, N * 4));
        CHECK(ensure(ctx, g.sz, N * 4));
        CHECK(ensure(ctx, g.wl, N * 2));
        CHECK(ensure(ctx, g.best, N * 8));
        CHECK(ensure(ctx, g.first, N * 4));
        CHECK(ensure(ctx, g.ebuf, E * 4));
        CHECK(ensure(ctx, g.bcnt, (3 * SM_SEG_NB + 1) * 4));
        CHECK(ensure(ctx, g.list0, E * 16));
        CHECK(ensure(ctx, g.list1, E * 16));
        CHECK(ensure(ctx, g.rej, E * 4));
        CHECK(ensure(ctx, g.hooked, N * 4));
        CHECK(ensure(ctx, g.cnt, SM_SEG_NCOUNT * 4));
        CHECK(ensure(ctx, g.mlist, E * sizeof(SegMin)));
        CHECK(ensure(ctx, g.msorted, E * sizeof(SegMin)));
        CHECK(ensure(ctx, g.mkey, E * 16));
        CHECK(ensure(ctx, g.mval, E * 8));
        CHECK(ensure(ctx, g.keep, (E + 1) * 4));
        CHECK(ensure(ctx, g.kpos, (E + 1) * 4));
        CHECK(ensure(ctx, g.lmark, (N + 1) * 4));
        CHECK(ensure(ctx, g.lid, (N + 1) * 4));
        CHECK(ensure(ctx, g.dense, E * sizeof(SegEdge)));
        CHECK(ensure(ctx, g.lsize, N * 4));
        CHECK(ensure(ctx, g.lroot, N * 4));
        g.stemp_bytes = seg_sort_temp_bytes((uint32_t)E);  // enough for any candidate count (<= E)
        CHECK(ensure(ctx, g.stemp, g.stemp_bytes));
        if (!g.h_b.resize(SM_SEG_NB + 1) || !g.h_cnt.resize(8)) return fail(ctx, SM_ERR_OOM, "segment mode: pinned host buffers");
        if (reset) HIPC(hipMemsetAsync(g.best.p, 0xFF, N * 8, st));
        HIPC(hipMemsetAsync(g.bcnt.p, 0, (3 * SM_SEG_NB + 1) * 4, st));
        HIPC(hipMemsetAsync(g.cnt.p, 0, SM_SEG_NCOUNT * 4, st));
        SegView& s = sp.v[i];
        s.W = W;
        s.H = H;
        s.wR = P<uint16_t>(ctx->wR[v]);
        s.wD = P<uint16_t>(ctx->wD[v]);
        s.par = P<uint32_t>(g.par);
        s.sz = P<uint32_t>(g.sz);
        s.wl = P<uint16_t>(g.wl);
        s.best = P<unsigned long long>(g.best);
        s.first = P<uint32_t>(g.first);
        s.ebuf = P<uint32_t>(g.ebuf);
        s.bcnt = P<uint32_t>(g.bcnt);
        s.list[0] = P<uint4>(g.list0);
        s.list[1] = P<uint4>(g.list1);
        s.rej = P<uint32_t>(g.rej);
        s.hooked = P<uint32_t>(g.hooked);
        s.cnt = P<uint32_t>(g.cnt);
        s.mlist = P<SegMin>(g.mlist);
        s.msorted = P<SegMin>(g.msorted);
        s.mkey[0] = P<unsigned long long>(g.mkey);
        s.mkey[1] = P<unsigned long long>(g.mkey) + E;
        s.mval[0] = P<uint32_t>(g.mval);
        s.mval[1] = P<uint32_t>(g.mval) + E;
        s.mR = P<uint8_t>(ctx->mR[v]);
        s.mD = P<uint8_t>(ctx->mD[v]);
        s.fwR = P<uint16_t>(ctx->fwR[v]);
        s.fwD = P<uint16_t>(ctx->fwD[v]);
        s.keep = P<uint32_t>(g.keep);
        s.act = P<uint32_t>(g.keep);  // the sweep's small-run active lists; the pair dedupe reuses it afterwards
        s.kpos = P<uint32_t>(g.kpos);
        s.lmark = P<uint32_t>(g.lmark);
        s.lid = P<uint32_t>(g.lid);
        s.dense = P<SegEdge>(g.dense);
        s.lsize = P<uint32_t>(g.lsize);
        s.lroot = P<uint32_t>(g.lroot);
    }
    HIPC(seg_launch_init(st, sp));
    for (int i = 0; i < vs.n; ++i) {
        SegGpu& g = ctx->sg[vs.v[i]];
        HIPC(hipMemcpyAsync(g.h_b.data(), P<uint32_t>(g.bcnt) + SM_SEG_NB, (SM_SEG_NB + 1) * 4, hipMemcpyDeviceToHost, st));
    }
    HIPC(seg_launch_scatter(st, sp));
    HIPC(hipStreamSynchronize(st));
    if (dbg) t1 = now_ms();
    // buckets in lockstep: a bucket is small if it is small in every view of the call
    auto bsize = [&](int w) {
        uint32_t m = 0;
        for (int i = 0; i < vs.n; ++i) {
            const SegGpu& g = ctx->sg[vs.v[i]];
            m = std::max(m, g.h_b[w + 1] - g.h_b[w]);
        }
        return m;
    };
    const int R = seg_global_rounds();
    const uint32_t small = seg_small();
    int L = 0;
    uint32_t rej_max = 0;
    for (int i = 0; i < vs.n; ++i) rej_max = std::max(rej_max, ctx->sg[vs.v[i]].h_b[SM_SEG_NB]);
    for (int w = 0; w < SM_SEG_NB; ++w) {
        const uint32_t m = bsize(w);
        if (!m) continue;
        if (m <= small) {  // a run of small buckets in one workgroup per view: classify, rounds, sizes
            int w1 = w + 1, nb = 1;
            for (uint32_t m1; w1 < SM_SEG_NB && (m1 = bsize(w1)) <= small; ++w1) nb += m1 > 0;
            if (flatten & 1) HIPC(seg_launch_flatten(st, sp));
            const bool split = seg_split();
            if (split) {
                uint32_t ne = 0;
                for (int i = 0; i < vs.n; ++i) {
                    const SegGpu& g = ctx->sg[vs.v[i]];
                    ne = std::max(ne, g.h_b[w1] - g.h_b[w]);
                }
                HIPC(seg_launch_split(st, sp, w, w1, c, ne));
            }
            HIPC(seg_launch_small(st, sp, w, w1, c, gen, split));
            gen += SM_SEG_TAIL_GENS * (uint32_t)nb;
            w = w1 - 1;
            continue;
        }
        if (L + R + 2 >= SM_SEG_MAXL) return fail(ctx, SM_ERR_STATE, "segment mode: list counters exhausted");
        int lin = L++;
        if (flatten & 2) HIPC(seg_launch_flatten(st, sp));
        HIPC(seg_launch_classify(st, sp, w, m, c, lin, gen++));  // + the first round's hooks
        for (int r = 1; r < R; ++r) {
            HIPC(seg_launch_round(st, sp, m, lin, lin + 1, gen++));
            lin = L++;
        }
        HIPC(seg_launch_tail(st, sp, lin, gen));
        gen += SM_SEG_TAIL_GENS;
        HIPC(seg_launch_sizes(st, sp, w, m));
    }
    for (int i = 0; i < vs.n; ++i) ctx->sg[vs.v[i]].gen = gen;
    HIPC(seg_launch_minsize(st, sp, min_size, rej_max));
    for (int i = 0; i < vs.n; ++i) {
        SegGpu& g = ctx->sg[vs.v[i]];
        HIPC(hipMemcpyAsync(g.h_cnt.data(), P<uint32_t>(g.cnt), 8 * 4, hipMemcpyDeviceToHost, st));
    }
    if (dbg) t2 = now_ms();
    HIPC(hipStreamSynchronize(st));
    if (dbg) t3 = now_ms();
    if (sm_knob("SM_SEG_PROF")) {  // k_seg_small's timings (sm_seg_gpu.hip SEG_PROF_SLOT): prologue, then per bucket
        for (int i = 0; i < vs.n; ++i) {
            std::vector<uint32_t> pr(2 + SM_SEG_NB);
            HIPC(hipMemcpy(pr.data(), P<uint32_t>(ctx->sg[vs.v[i]].cnt) + SM_SEG_C_LIST + 60000, pr.size() * 4,
                           hipMemcpyDeviceToHost));
            fprintf(stderr, "seg prof view %d: small-run prologue %.1f us, active %u; buckets (us):", i, pr[0] * 0.01, pr[1]);
            double tot = 0;
            for (int w = 0; w < SM_SEG_NB; ++w)
                if (pr[2 + w]) {
                    fprintf(stderr, " %d:%.1f%s", w, (pr[2 + w] & 0x7FFFFFFFu) * 0.01, (pr[2 + w] >> 31) ? "B" : "");
                    tot += (pr[2 + w] & 0x7FFFFFFFu) * 0.01;
                }
            fprintf(stderr, " | total %.1f us\n", tot);
        }
    }
    void* temp[2] = {nullptr, nullptr};
    size_t tbytes[2] = {0, 0};
    for (int i = 0; i < vs.n; ++i) {
        SegGpu& g = ctx->sg[vs.v[i]];
        if (g.h_cnt[SM_SEG_C_ERR]) return fail(ctx, SM_ERR_STATE, "segment mode: a Boruvka tail did not converge");
        const uint32_t nm = g.h_cnt[SM_SEG_C_MIN];
        if (!g.h_hooks.resize(3 * (size_t)nm + 1))
            return fail(ctx, SM_ERR_OOM, "segment mode: pinned host buffers");
        sp.v[i].nmin = nm;
        temp[i] = g.stemp.p;
        tbytes[i] = g.stemp_bytes;
    }
    // the pair dedupe by hashing: no sort of the ~260k candidates (round 4: the sorts cost 0.55 ms of
    // kernels plus their gaps); a table that would not fit the key buffers sorts them instead
    uint32_t hcap = 0;
    {
        uint32_t nmax = 0;
        for (int i = 0; i < vs.n; ++i) nmax = std::max(nmax, sp.v[i].nmin);
        hcap = 1024;
        while (hcap < 2 * nmax) hcap <<= 1;
        if ((size_t)hcap > E) hcap = 0;  // (the table lives in the E-entry key buffers)
    }
    if (!hcap) HIPC(seg_launch_sort(st, sp, temp, tbytes));
    {  // the first candidate of each root pair, dense root ids: their counts, then the lists
        if (hcap)
            HIPC(seg_launch_dedupe_hash(st, sp, temp, tbytes, hcap));
        else
            HIPC(seg_launch_dedupe(st, sp, temp, tbytes));
        for (int i = 0; i < vs.n; ++i)
            HIPC(hipMemcpyAsync(ctx->sg[vs.v[i]].h_cnt.data() + SM_SEG_C_UNIQ, P<uint32_t>(ctx->sg[vs.v[i]].cnt) + SM_SEG_C_UNIQ,
                                8, hipMemcpyDeviceToHost, st));
        HIPC(hipStreamSynchronize(st));
        for (int i = 0; i < vs.n; ++i) {
            SegGpu& g = ctx->sg[vs.v[i]];
            const uint32_t nu = g.h_cnt[SM_SEG_C_UNIQ], nl = g.h_cnt[SM_SEG_C_LOCAL];
            if (nu > sp.v[i].nmin || nl > 2 * nu) return fail(ctx, SM_ERR_STATE, "segment mode: bad min-size dedupe counts");
            if (!g.h_dense.resize(nu) || !g.h_lsize.resize(nl) || !g.h_lroot.resize(nl))
                return fail(ctx, SM_ERR_OOM, "segment mode: pinned host buffers");
            if (nu) HIPC(hipMemcpyAsync(g.h_dense.data(), g.dense.p, nu * sizeof(SegEdge), hipMemcpyDeviceToHost, st));
            if (nl) {
                HIPC(hipMemcpyAsync(g.h_lsize.data(), g.lsize.p, nl * 4, hipMemcpyDeviceToHost, st));
                HIPC(hipMemcpyAsync(g.h_lroot.data(), g.lroot.p, nl * 4, hipMemcpyDeviceToHost, st));
            }
        }
    }
    HIPC(hipStreamSynchronize(st));
    if (dbg) t4 = now_ms();
    const uint32_t ms = (uint32_t)(min_size < 2 ? 2 : min_size);
    int nk[2] = {0, 0};
    {  // the views' merges in parallel
        auto merge = [ctx, ms, hcap](int v) {
            SegGpu& g = ctx->sg[v];
            if (hcap) seg_sort_dense(g.h_dense.data(), g.h_cnt[SM_SEG_C_UNIQ], g.h_dsort);  // hashed: unordered
            return seg_minsize_dense(g.h_dense.data(), g.h_cnt[SM_SEG_C_UNIQ], g.h_cnt[SM_SEG_C_LOCAL], g.h_lsize.data(),
                                     g.h_lroot.data(), ms, g.h_hooks.data(), g.mpar, g.msize);
        };
        std::thread other;
        if (vs.n > 1) other = std::thread([&] { nk[1] = merge(vs.v[1]); });
        nk[0] = merge(vs.v[0]);
        if (other.joinable()) other.join();
    }
    for (int i = 0; i < vs.n; ++i) {
        SegGpu& g = ctx->sg[vs.v[i]];
        const int k = nk[i];
        CHECK(ensure(ctx, g.hooks, (3 * (size_t)k + 1) * 4));
        if (k) HIPC(hipMemcpyAsync(g.hooks.p, g.h_hooks.data(), 3 * (size_t)k * 4, hipMemcpyHostToDevice, st));
        sp.v[i].hooks = P<uint32_t>(g.hooks);
        sp.v[i].nhooks = k;
    }
    HIPC(seg_launch_apply(st, sp));
    HIPC(seg_launch_trees(st, sp));
    for (int i = 0; i < vs.n; ++i) {
        const int v = vs.v[i];
        SegGpu& g = ctx->sg[v];
        HIPC(hipMemcpyAsync(g.h_cnt.data() + 4, P<uint32_t>(g.cnt) + SM_SEG_C_TREES, 4, hipMemcpyDeviceToHost, st));
        if (host_copy) {
            for (int q = 0; q < 2; ++q)
                if (!ctx->h_w[v][q].resize(N) || !ctx->h_fw[v][q].resize(N) || !ctx->h_m[v][q].resize(N))
                    return fail(ctx, SM_ERR_OOM, "segment mode: pinned host buffers");
            HIPC(hipMemcpyAsync(ctx->h_w[v][0].data(), ctx->wR[v].p, N * 2, hipMemcpyDeviceToHost, st));
            HIPC(hipMemcpyAsync(ctx->h_w[v][1].data(), ctx->wD[v].p, N * 2, hipMemcpyDeviceToHost, st));
            HIPC(hipMemcpyAsync(ctx->h_m[v][0].data(), ctx->mR[v].p, N, hipMemcpyDeviceToHost, st));
            HIPC(hipMemcpyAsync(ctx->h_m[v][1].data(), ctx->mD[v].p, N, hipMemcpyDeviceToHost, st));
            HIPC(hipMemcpyAsync(ctx->h_fw[v][0].data(), ctx->fwR[v].p, N * 2, hipMemcpyDeviceToHost, st));
            HIPC(hipMemcpyAsync(ctx->h_fw[v][1].data(), ctx->fwD[v].p, N * 2, hipMemcpyDeviceToHost, st));
        }
    }
    if (host_copy) {
        HIPC(hipStreamSynchronize(st));
        for (int i = 0; i < vs.n; ++i) ctx->seg_trees[vs.v[i]] = (int)ctx->sg[vs.v[i]].h_cnt[4];
    }
    CHECK(ensure(ctx, ctx->mst_ok, sizeof(int)));
    HIPC(hipMemsetAsync(ctx->mst_ok.p, 1, sizeof(int), st));
    if (dbg) {
        const double t5 = now_ms();
        fprintf(stderr, "segment_gpu: init+buckets %.2f ms, enqueue %.2f, sweep wait %.2f, min-size copy %.2f, host merge + rest %.2f;",
                t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4);
        for (int i = 0; i < vs.n; ++i)
            fprintf(stderr, " view %d: rejected %u, small %u, first of their pair %u, roots %u, hooks %u", vs.v[i],
                    ctx->sg[vs.v[i]].h_cnt[SM_SEG_C_REJ], ctx->sg[vs.v[i]].h_cnt[SM_SEG_C_MIN], ctx->sg[vs.v[i]].h_cnt[SM_SEG_C_UNIQ],
                    ctx->sg[vs.v[i]].h_cnt[SM_SEG_C_LOCAL], ctx->sg[vs.v[i]].h_cnt[SM_SEG_C_HOOK]);
        fprintf(stderr, "\n");
    }
    return SM_OK;
}

sm_status stage_segment(sm_ctx* ctx, int views, float c, int min_size, bool host_copy = true) {
    if (!seg_host()) {
        CHECK(segment_gpu(ctx, views, c, min_size, host_copy));
        ctx->mst_pend.active = false;
        ctx->seg = true;
        return SM_OK;
    }
    CHECK(segment_download(ctx, views));
    CHECK(segment_host(ctx, views, c, min_size));
    CHECK(segment_upload(ctx, views));
    HIPC(hipStreamSynchronize(ctx->st));  // the host buffers are reused by the next call
    ctx->mst_pend.active = false;
    ctx->seg = true;
    return SM_OK;
}

// SM_SEG_SYNC=1: segment mode's host segmentation inside sm_match_begin (A/B of the worker thread)
bool seg_sync() {
    static const bool s = sm_dev_knob("SM_SEG_SYNC") != nullptr;
    return s;
}

// tree of the call: the MST (Boruvka) or, for finite c, the segment forest
sm_status stage_tree(sm_ctx* ctx, int views, const sm_params* p, bool host_copy) {
    if (p && !std::isinf(p->c)) return stage_segment(ctx, views, p->c, p->min_size, host_copy);
    ctx->seg = false;
    return stage_mst(ctx, views);
}

sm_status stage_mst(sm_ctx* ctx, int views) {
    const int W = ctx->W, H = ctx->H;
    const size_t N = (size_t)W * H;
    const ViewSet vs(views);
    const int nviews = vs.n;
    MstArgs a{};
    a.nviews = nviews;
    for (int i = 0; i < 2; ++i) {  // kernel view slot i = view vs.v[i] (slot 1 unused for one view)
        const int v = vs.v[i];
        CHECK(ensure(ctx, ctx->comp[v], N * 4));
        CHECK(ensure(ctx, ctx->best[v], 2 * N * 8));
        CHECK(ensure(ctx, ctx->root[v], N * 4));
        CHECK(ensure(ctx, ctx->mR[v], N));
        CHECK(ensure(ctx, ctx->mD[v], N));
        a.wR[i] = P<uint16_t>(ctx->wR[v]);
        a.wD[i] = P<uint16_t>(ctx->wD[v]);
        a.comp[i] = P<uint32_t>(ctx->comp[v]);
        a.best[i] = P<unsigned long long>(ctx->best[v]);
        a.root[i] = P<uint32_t>(ctx->root[v]);
        a.mR[i] = P<uint8_t>(ctx->mR[v]);
        a.mD[i] = P<uint8_t>(ctx->mD[v]);
    }
    CHECK(ensure(ctx, ctx->changed, 2 * SM_MST_MAX_ROUNDS * sizeof(int)));
    CHECK(ensure(ctx, ctx->mst_ok, sizeof(int)));
    ZeroList z{};
    for (int i = 0; i < nviews; ++i) {  // the active views only: an inactive view's buffers may not exist
        const int v = vs.v[i];
        CHECK(ensure(ctx, ctx->ccnt[v], 16));
        z.add(ctx->ccnt[v].p, 16);  // (the masks are zeroed by k_bor_local, tile by tile)
    }
    z.add(ctx->changed.p, 2 * SM_MST_MAX_ROUNDS * sizeof(int));
    HIPC(launch_zero(ctx->st, z));
    a.flags[0] = P<int>(ctx->changed);
    a.flags[1] = P<int>(ctx->changed) + SM_MST_MAX_ROUNDS;
    const bool pixel_rounds = sm_knob("SM_MST_PIXEL_ROUNDS") != nullptr;  // A/B path (tests, tools)
    {
        uint32_t* cc[2] = {nullptr, nullptr};
        uint32_t* cl[2] = {nullptr, nullptr};
        if (!pixel_rounds)
            for (int i = 0; i < nviews; ++i) {
                const int v = vs.v[i];
                CHECK(ensure(ctx, ctx->clab[v], N * 4));
                cc[i] = P<uint32_t>(ctx->ccnt[v]);
                cl[i] = P<uint32_t>(ctx->clab[v]);
            }
        HIPC(launch_bor_local(ctx->st, a, W, H, cc, cl, N));
    }
    if (pixel_rounds) {
        for (int i = 0; i < nviews; ++i) HIPC(hipMemsetAsync(ctx->best[vs.v[i]].p, 0xFF, N * 8, ctx->st));
        // global rounds: every kernel of round r exits at once if round r-1 hooked nothing, so the
        // host only synchronises every 4 rounds to decide whether to enqueue more
        for (int r = 0; r < SM_MST_MAX_ROUNDS; ++r) {
            HIPC(launch_bor_round(ctx->st, a, W, H, r));
            if ((r & 3) == 3) {
                HIPC(hipMemcpyAsync(ctx->h_changed, P<int>(ctx->changed) + r, sizeof(int), hipMemcpyDeviceToHost, ctx->st));
                HIPC(hipMemcpyAsync(ctx->h_changed + 1, P<int>(ctx->changed) + SM_MST_MAX_ROUNDS + r, sizeof(int),
                                    hipMemcpyDeviceToHost, ctx->st));
                HIPC(hipStreamSynchronize(ctx->st));
                if (ctx->h_changed[0] == 0 && (nviews < 2 || ctx->h_changed[1] == 0)) break;
            }
        }
        HIPC(hipMemsetAsync(ctx->mst_ok.p, 1, sizeof(int), ctx->st));  // checked on the host above
        ctx->mst_pend.active = false;
        return SM_OK;
    }
    // contracted rounds on the component graph left by the tile phase
    MstCompact c{};
    c.emax = 2 * N;
    c.bstride = N;
    for (int i = 0; i < 2; ++i) {
        const int v = vs.v[i];
        CHECK(ensure(ctx, ctx->cedge[v], 2 * (2 * N) * 16));
        CHECK(ensure(ctx, ctx->clab[v], N * 4));
        CHECK(ensure(ctx, ctx->chook[v], N * 4));
        c.cid[i] = P<uint32_t>(ctx->root[v]);
        c.counts[i] = P<uint32_t>(ctx->ccnt[v]);
        c.edges[i] = ctx->cedge[v].p;
        c.lab[i] = P<uint32_t>(ctx->clab[v]);
        c.hook[i] = P<uint32_t>(ctx->chook[v]);
    }
    HIPC(launch_bor_compact(ctx->st, a, c, W, H));
    // Enqueue the rounds the previous frame needed (the last of them hooked nothing) and the copy
    // of the hook flags, without waiting: the layout is enqueued behind them and the flags are
    // checked after the layout's own synchronisation (mst_finish).  Every kernel of round r exits
    // at once when round r-1 hooked nothing.
    const int first = std::min(std::max(ctx->mst_rounds, 2), SM_MST_MAX_ROUNDS);
    const bool dbg = sm_knob("SM_MST_DEBUG") != nullptr;
    int r = 0;
    for (; r < first; ++r) {
        HIPC(launch_bor_cround(ctx->st, a, c, W, r));
        if (dbg) {
            uint32_t h[4];
            HIPC(hipMemcpyAsync(h, c.counts[0], 16, hipMemcpyDeviceToHost, ctx->st));
            HIPC(hipStreamSynchronize(ctx->st));
            fprintf(stderr, "mst round %d: K %u live edges %u / %u\n", r, h[0], h[1], h[2]);
        }
    }
    HIPC(launch_mst_done(ctx->st, a, r - 1, P<int>(ctx->mst_ok)));
    HIPC(hipMemcpyAsync(ctx->h_changed, ctx->changed.p, 2 * SM_MST_MAX_ROUNDS * sizeof(int), hipMemcpyDeviceToHost, ctx->st));
    ctx->mst_pend = MstPending{true, nviews, r, a, c};
    return SM_OK;
}

// After a synchronisation that covers stage_mst's flag copy: if the last enqueued round still
// hooked an edge, run more rounds (synchronously) and report that the MST grew (the layout built
// on the incomplete forest must then be redone).  Records the rounds needed for the next frame.
sm_status mst_finish(sm_ctx* ctx, bool* grew) {
    *grew = false;
    MstPending& m = ctx->mst_pend;
    if (!m.active) return SM_OK;
    m.active = false;
    int r = m.r;
    while (hooked_any(ctx->h_changed, m.nviews, r - 1) && r < SM_MST_MAX_ROUNDS) {
        *grew = true;
        const int end = std::min(r + 4, SM_MST_MAX_ROUNDS);
        for (; r < end; ++r) HIPC(launch_bor_cround(ctx->st, m.a, m.c, ctx->W, r));
        HIPC(hipMemcpyAsync(ctx->h_changed, ctx->changed.p, 2 * SM_MST_MAX_ROUNDS * sizeof(int), hipMemcpyDeviceToHost,
                            ctx->st));
        HIPC(hipStreamSynchronize(ctx->st));
    }
    if (*grew) HIPC(launch_mst_done(ctx->st, m.a, r - 1, P<int>(ctx->mst_ok)));
    // rounds needed: through the first one that hooked nothing in any view
    int need = 1;
    while (need < r && hooked_any(ctx->h_changed, m.nviews, need - 1)) ++need;
    ctx->mst_rounds = need;
    return SM_OK;
}

// nodes per piece: SM_PIECE, or env SM_PIECE_LEN (multiple of SM_PRE_SEG, >= 64)
int piece_len() {  // read per call: tests switch it between matches
    const char* e = sm_knob("SM_PIECE_LEN");
    const int v = e ? atoi(e) : SM_PIECE;
    return (v >= 64 && v % SM_PRE_SEG == 0) ? v : SM_PIECE;
}

// device-side rounds record: [0, SM_NBUCKETS] bucket begin, then count, cursor, nrounds, n_has_light
constexpr size_t RREC = RREC_FWD;

// The layout in two halves: stage_layout_enqueue launches it and the copy of the per-round
// counts; stage_layout_finish waits for that copy (the host sizes the walker grids from it) and
// reads it.  sm_match_begin / sm_match_finish put the host wait between them, so a caller can
// enqueue the next frame's tree before it waits for this frame's layout.
sm_status stage_layout_enqueue(sm_ctx* ctx, int views);
sm_status stage_layout_finish(sm_ctx* ctx, int views);
sm_status stage_layout(sm_ctx* ctx, int views) {
    CHECK(stage_layout_enqueue(ctx, views));
    return stage_layout_finish(ctx, views);
}

sm_status stage_layout_enqueue(sm_ctx* ctx, int views) {
    const ViewSet vs(views);
    const int nviews = vs.n;
    const int W = ctx->W, H = ctx->H;
    const size_t N = (size_t)W * H;
    const uint32_t ntiles = (uint32_t)(((W + 31) / 32) * ((H + 31) / 32));
    const uint32_t max_chains = ntiles * 129u + 1u;
    const size_t nscan = scan_tiles(N);
    if (N >= ((size_t)1 << 27))  // 32-bit tour values and path records hold the preorder in 27 bits (sm_layout_gpu.hip)
        return fail(ctx, SM_ERR_ARG, "tree layout: images of 2^27 pixels or more are not supported");
    LayoutPair LP{};
    ZeroList z{};
    for (int i = 0; i < nviews; ++i) {
        const int v = vs.v[i];
        CHECK(ensure(ctx, ctx->adj[v], N));
        CHECK(ensure(ctx, ctx->pdir[v], N));
        CHECK(ensure(ctx, ctx->heavy[v], N));
        CHECK(ensure(ctx, ctx->size[v], N * 4));
        CHECK(ensure(ctx, ctx->arcpix[v], 2 * N * 4));
        CHECK(ensure(ctx, ctx->hk[v], N * 4));
        CHECK(ensure(ctx, ctx->pixpre[v], N * 4));
        CHECK(ensure(ctx, ctx->a_dist[v], 4 * N * 2));
        CHECK(ensure(ctx, ctx->a_cid[v], 4 * N * 4));
        CHECK(ensure(ctx, ctx->ccount[v], 16));
        CHECK(ensure(ctx, ctx->c_last[v], max_chains * 4));
        CHECK(ensure(ctx, ctx->c_len[v], max_chains * 4));
        CHECK(ensure(ctx, ctx->cnw[v], max_chains * 8));
        CHECK(ensure(ctx, ctx->tour[v], 2 * N * 4 + 16));
        CHECK(ensure(ctx, ctx->spart[v], nscan * 8));
        CHECK(ensure(ctx, ctx->meta[v], N * sizeof(SmMeta)));
        CHECK(ensure(ctx, ctx->paths[v], N * sizeof(SmPath)));
        CHECK(ensure(ctx, ctx->rounds[v], RREC * 4));
        CHECK(ensure(ctx, ctx->segtab[v], (N / 16 + 64) * sizeof(uint2)));  // <= N/32 segments + N/32 long paths
        CHECK(ensure(ctx, ctx->pieces[v], (N / 16 + 64) * sizeof(uint4)));  // <= N/32 long paths + N/SM_PIECE
        CHECK(ensure(ctx, ctx->pieces_tmp[v], (N / 16 + 64) * sizeof(uint4)));
        CHECK(ensure(ctx, ctx->pathpos[v], N * 4));
        CHECK(ensure(ctx, ctx->plen[v], N * 4));
        CHECK(ensure(ctx, ctx->slotpix[v], N * 4));
        CHECK(ensure(ctx, ctx->lrank[v], N));
        CHECK(ensure(ctx, ctx->wrow[v], 4 * (size_t)ntiles * 4));
        z.add(ctx->ccount[v].p, 16);
        z.add(ctx->rounds[v].p, RREC * 4);
        LayoutView& L = LP.v[i];
        L.mR = P<uint8_t>(ctx->mR[v]);
        L.mD = P<uint8_t>(ctx->mD[v]);
        L.wR = P<uint16_t>(ctx->seg ? ctx->fwR[v] : ctx->wR[v]);
        L.wD = P<uint16_t>(ctx->seg ? ctx->fwD[v] : ctx->wD[v]);
        L.adj = P<uint8_t>(ctx->adj[v]);
        L.pdir = P<int8_t>(ctx->pdir[v]);
        L.heavy = P<int8_t>(ctx->heavy[v]);
        L.size = P<uint32_t>(ctx->size[v]);
        L.arcpix = P<uint32_t>(ctx->arcpix[v]);
        L.hk = P<uint32_t>(ctx->hk[v]);
        L.pixpre = P<uint32_t>(ctx->pixpre[v]);
        L.a_dist = P<uint16_t>(ctx->a_dist[v]);
        L.a_cid = P<uint32_t>(ctx->a_cid[v]);
        L.nchains = P<uint32_t>(ctx->ccount[v]);
        L.c_last = P<uint32_t>(ctx->c_last[v]);
        L.c_len = P<uint32_t>(ctx->c_len[v]);
        L.cnw = P<uint64_t>(ctx->cnw[v]);
        L.tour = P<uint32_t>(ctx->tour[v]);
        LP.scan.part[i] = P<uint64_t>(ctx->spart[v]);
        L.meta = P<SmMeta>(ctx->meta[v]);
        L.paths = P<SmPath>(ctx->paths[v]);
        L.pathpos = P<uint32_t>(ctx->pathpos[v]);
        L.plen = P<uint32_t>(ctx->plen[v]);
        L.slotpix = P<uint32_t>(ctx->slotpix[v]);
        L.lrank = P<uint8_t>(ctx->lrank[v]);
        L.wrow = P<uint32_t>(ctx->wrow[v]);
        uint32_t* R = P<uint32_t>(ctx->rounds[v]);
        L.round_begin = R;
        L.round_count = R + SM_NBUCKETS + 1;
        L.round_cursor = R + 2 * SM_NBUCKETS + 1;
        L.nrounds = R + 3 * SM_NBUCKETS + 1;
        L.n_has_light = R + 3 * SM_NBUCKETS + 2;
        L.round_maxlen = R + 3 * SM_NBUCKETS + 3;
        L.seg_begin = R + 4 * SM_NBUCKETS + 3;
        L.round_nodes = R + 5 * SM_NBUCKETS + 4;
        L.segtab = P<uint2>(ctx->segtab[v]);
        L.piece_begin = R + 6 * SM_NBUCKETS + 4;
        L.pieces = P<uint4>(ctx->pieces[v]);
        L.pieces_tmp = P<uint4>(ctx->pieces_tmp[v]);
    }
    if (nviews == 1) LP.v[1] = LP.v[0];
    LP.mst_ok = P<int>(ctx->mst_ok);
    if (nviews == 1) LP.scan.part[1] = LP.scan.part[0];
    LP.scan.err = ctx->d_err;
    LP.want_size = ctx->want_size ? 1 : 0;
    HIPC(launch_zero(ctx->st, z));
    HIPC(launch_layout(ctx->st, LP, nviews, W, H, max_chains, (uint32_t)piece_len()));
    // the host needs the per-round path counts to size the walker grids
    for (int i = 0; i < nviews; ++i)
        HIPC(hipMemcpyAsync(ctx->h_rounds + vs.v[i] * RREC, ctx->rounds[vs.v[i]].p, RREC * 4, hipMemcpyDeviceToHost, ctx->st));
    HIPC(hipEventRecord(ctx->ev_layout, ctx->st));
    return SM_OK;
}

sm_status stage_layout_finish(sm_ctx* ctx, int views) {
    HIPC(hipEventSynchronize(ctx->ev_layout));
    // a layout index out of range (bit 1, the layout kernels' guards): the metadata is not a tree
    // layout, so no filter may run over it (its indices would be wild).  Only bit 1 is the layout's: the
    // other bits belong to the filter of a frame still in flight.
    if (__atomic_fetch_and(ctx->h_err, ~2u, __ATOMIC_ACQ_REL) & 2u)
        return fail(ctx, SM_ERR_STATE, "tree layout: an index out of range (the MST tour is not a spanning tree's)");
    bool grew = false;
    CHECK(mst_finish(ctx, &grew));
    if (grew) return stage_layout(ctx, views);  // the forest was incomplete: lay out the final MST
    for (int v = 0; v < 2; ++v) {
        auto& L = ctx->layout[v];
        if (!view_on(views, v)) { L.nrounds = 0; L.npaths = 0; L.begin.assign(1, 0); L.maxlen.assign(SM_NBUCKETS, 0); L.seg_begin.assign(SM_NBUCKETS + 1, 0); L.nodes.assign(SM_NBUCKETS, 0); L.piece_begin.assign(SM_NBUCKETS + 1, 0); continue; }
        const uint32_t* R = ctx->h_rounds + v * RREC;
        L.nrounds = R[3 * SM_NBUCKETS + 1];
        L.n_has_light = R[3 * SM_NBUCKETS + 2];
        L.begin.assign(R, R + SM_NBUCKETS + 1);
        L.maxlen.assign(R + 3 * SM_NBUCKETS + 3, R + 4 * SM_NBUCKETS + 3);
        L.seg_begin.assign(R + 4 * SM_NBUCKETS + 3, R + 5 * SM_NBUCKETS + 4);
        L.nodes.assign(R + 5 * SM_NBUCKETS + 4, R + 6 * SM_NBUCKETS + 4);
        L.piece_begin.assign(R + 6 * SM_NBUCKETS + 4, R + 7 * SM_NBUCKETS + 5);
        L.npaths = R[SM_NBUCKETS];
        if (L.nrounds == 0 || L.npaths == 0) return fail(ctx, SM_ERR_STATE, "layout produced no paths");
        if (sm_knob("SM_LAYOUT_DEBUG"))  // per-round path statistics (tools/gpu_layout_dbg.sh)
            for (uint32_t r = 0; r < L.nrounds; ++r)
                fprintf(stderr, "view %d round %u: long %u paths %u nodes maxlen %u | short %u paths %u nodes maxlen %u\n", v, r,
                        L.begin[2 * r + 1] - L.begin[2 * r], L.nodes[2 * r], L.maxlen[2 * r], L.begin[2 * r + 2] - L.begin[2 * r + 1],
                        L.nodes[2 * r + 1], L.maxlen[2 * r + 1]);
    }
    return SM_OK;
}

WalkArgs walk_args(sm_ctx* ctx, int Dpad, int D, int dglob0) {
    WalkArgs a{};
    for (int v = 0; v < 2; ++v) {
        a.meta[v] = P<SmMeta>(ctx->meta[v]);
        a.U[v] = P<double>(ctx->U[v]);
        a.A[v] = nullptr;  // set by setup_sync (compact rows)
        a.Adbg[v] = nullptr;  // debug calls only (stage_filter)
        a.Cst[v] = P<float>(ctx->Cst[v]);
        a.idx[v] = P<int32_t>(ctx->idx[v]);
        a.minc[v] = P<double>(ctx->minc[v]);
        a.disp[v] = P<float>(ctx->disp[v]);
    }
    a.Lrec = P<uint2>(ctx->rec[0]) + ctx->rec_pad;
    a.Rrec = P<uint2>(ctx->rec[1]) + ctx->rec_pad;
    a.Lrec4 = P<uint32_t>(ctx->rec4[0]) + ctx->rec_pad;
    a.Rrec4 = P<uint32_t>(ctx->rec4[1]) + ctx->rec_pad;
    a.atab = P<float>(ctx->atab);
    a.slut = P<double>(ctx->slut);
    a.s2lut = P<double>(ctx->s2lut);
    a.W = ctx->W;
    a.Dpad = Dpad;
    a.dcall = D;
    a.dglob0 = dglob0;
    a.wta = WtaCfg{0, D, dglob0, dglob0 + D, 0};  // stage_filter sets the call's own
    return a;
}

bool no_pieces() { return sm_dev_knob("SM_NO_PIECES") != nullptr; }

// capacity of the per-view piece arrays (<= N/32 long paths + N/SM_PIECE pieces)
size_t piece_cap(size_t N) { return N / 16 + 64; }

void set_bucket(sm_ctx* ctx, WalkArgs& a, uint32_t r, bool long_paths, int views) {
    a.maxlen = 0;
    for (int v = 0; v < 2; ++v) {
        const auto& L = ctx->layout[v];
        if (!view_on(views, v) || r >= L.nrounds) {
            a.paths[v] = P<SmPath>(ctx->paths[v]);
            a.npaths[v] = 0;
            a.segtab[v] = P<uint2>(ctx->segtab[v]);
            a.nseg[v] = 0;
            a.pieces[v] = nullptr;
            a.npieces[v] = 0;
            a.bucket_plen[v] = a.piece_len;
        } else {
            const uint32_t b = 2 * r + (long_paths ? 0 : 1);
            a.paths[v] = P<SmPath>(ctx->paths[v]) + L.begin[b];
            a.npaths[v] = (int)(L.begin[b + 1] - L.begin[b]);
            a.maxlen = std::max(a.maxlen, (int)L.maxlen[b]);
            a.segtab[v] = P<uint2>(ctx->segtab[v]) + L.seg_begin[b];
            a.nseg[v] = (int)(L.seg_begin[b + 1] - L.seg_begin[b]);
            // long buckets: pieces (sm_chain.hip "Pieces"), unless SM_NO_PIECES (A/B)
            const bool pieces = long_paths && ctx->agg[v].p && !no_pieces();
            a.pieces[v] = pieces ? P<uint4>(ctx->pieces[v]) + L.piece_begin[b] : nullptr;
            a.bucket_plen[v] = (int)sm_bucket_piece_len(L.nodes[b], (uint32_t)a.piece_len);
            a.npieces[v] = pieces ? (int)(L.piece_begin[b + 1] - L.piece_begin[b]) : 0;
            a.agg[v] = pieces ? P<double>(ctx->agg[v]) + (size_t)L.seg_begin[b] * 2 * a.Dpad : nullptr;
            // the bucket's cut paths' rows (sm_chain.hip FixRows): 32 per segment
            a.fix[v] = P<double>(ctx->fix[v]) + (size_t)L.seg_begin[b] * SM_PRE_SEG * a.Dpad;
            a.pstat[v] = pieces ? P<uint32_t>(ctx->pstat[v]) + L.piece_begin[b] : nullptr;
        }
    }
}

// Timing-only events skip the system-scope fence on record (hipEventDisableSystemFence): the
// default record writes back and invalidates the caches, which put ~5.7 us of idle GPU between
// the bracketed launches and left the next kernel with cold caches.  Elapsed times are read after
// a stream synchronisation, so nothing needs the fence.  SM_EVENT_FENCE=1: default events (A/B).
static unsigned timing_event_flags() {
    static const bool fence = sm_dev_knob("SM_EVENT_FENCE") != nullptr;
    return fence ? hipEventDefault : hipEventDisableSystemFence;
}

sm_status ensure_events(sm_ctx* ctx, std::vector<hipEvent_t>& evs, size_t n, unsigned flags = hipEventDefault) {
    while (evs.size() < n) {
        hipEvent_t e;
        HIPC(hipEventCreateWithFlags(&e, flags));
        evs.push_back(e);
    }
    return SM_OK;
}

// kernel families of the tree filter and their algorithmic bytes per voxel (SURVEY.md 8(d):
// K1 cost write 4 B, K2 up 8 B, K3 down 8 B, K4 WTA 4 B; DESIGN.md "Roofline accounting").
// Both up families compute the cost on the fly (K1 + K2); k_up_pre only folds the cut paths'
// segment aggregates and accounts no bytes.
enum { KF_UP_WALK, KF_UP_PRE, KF_UP_CHAIN, KF_DOWN_CHAIN, KF_DOWN_WALK, KF_N };
const char* const kf_name[KF_N] = {"k_up_walk", "k_up_pre", "k_up_chain", "k_down_chain", "k_down_walk"};
const double kf_bytes[KF_N] = {12.0, 0.0, 12.0, 12.0, 12.0};
static bool kf_up(int f) { return f <= KF_UP_CHAIN; }

// A timed launch of family f on stream s.  HIP events bracket the launch, but consecutive timed
// launches on the filter stream share the event between them (the end of one is the start of
// the next, so a launch's time includes the dispatch gap before it); empty buckets launch
// nothing and record nothing.  Each event record costs the host ~3 us and the deep rounds are
// host-bound: two events per launch added ~0.45 ms per C2 frame, one adds ~0.15 ms.  Launches
// below SM_TIMED_MIN_VOX voxels may be left untimed (and out of the per-family stats); 0 keeps
// every launch timed so rocprof's per-kernel averages compare launch for launch.
#ifndef SM_TIMED_MIN_VOX
#define SM_TIMED_MIN_VOX 0.0
#endif
template <class F>
sm_status timed(sm_ctx* ctx, hipStream_t s, int f, double vox, F&& launch, double acct = -1.0) {
    // vox: voxels of the launch (0: nothing to launch); acct: voxels its algorithmic bytes count
    // (default vox)
    static const bool off = sm_dev_knob("SM_NO_KTIMING") != nullptr;  // A/B: no events at all
    if (vox <= 0) return SM_OK;                                   // empty bucket: nothing to launch
    if (off || vox < SM_TIMED_MIN_VOX || !((ctx->ktiming >> f) & 1u)) {
        HIPC(launch());
        ctx->ev_open = false;
        return SM_OK;
    }
    CHECK(ensure_events(ctx, ctx->fev, (size_t)ctx->nfev + 2, timing_event_flags()));
    int start;
    if (ctx->ev_open && s == ctx->ev_stream) {
        start = ctx->nfev - 1;  // the previous timed launch's end event
    } else {
        start = ctx->nfev;
        HIPC(hipEventRecord(ctx->fev[ctx->nfev++], s));
    }
    HIPC(launch());
    HIPC(hipEventRecord(ctx->fev[ctx->nfev], s));
    ctx->fam.push_back(f);
    ctx->fam_vox.push_back(acct < 0 ? vox : acct);
    ctx->fam_ev.push_back(std::make_pair(start, ctx->nfev));
    ctx->nfev += 1;
    ctx->ev_open = true;
    ctx->ev_stream = s;
    return SM_OK;
}

// make stream `waiter` wait for everything enqueued so far on stream `src`
sm_status join(sm_ctx* ctx, hipStream_t waiter, hipStream_t src) {
    if (waiter == src) return SM_OK;
    CHECK(ensure_events(ctx, ctx->sev, (size_t)ctx->nsev + 1));
    hipEvent_t e = ctx->sev[ctx->nsev++];
    HIPC(hipEventRecord(e, src));
    HIPC(hipStreamWaitEvent(waiter, e, 0));
    return SM_OK;
}

double bucket_voxels(sm_ctx* ctx, uint32_t r, bool long_paths, int views, int D) {
    double n = 0;
    for (int v = 0; v < 2; ++v) {
        const auto& L = ctx->layout[v];
        if (view_on(views, v) && r < L.nrounds) n += L.nodes[2 * r + (long_paths ? 0 : 1)];
    }
    return n * D;
}

// One light-depth round of a pass: short paths by the chunked walkers on st, long paths by the
// chain engine on st2, concurrently (they touch disjoint rows; both only read rows finished in
// earlier rounds).  Rounds are ordered by joining the two streams at every round boundary.
sm_status up_round(sm_ctx* ctx, WalkArgs& a, uint32_t r, int spl, int views) {
    CHECK(join(ctx, ctx->st, ctx->st2));
    CHECK(join(ctx, ctx->st2, ctx->st));
    set_bucket(ctx, a, r, true, views);
    const WalkArgs al = a;
    const double vl = bucket_voxels(ctx, r, true, views, a.dcall);
    // segment aggregates (the pieces' guesses): only buckets with a path cut into pieces need them
    bool cut = false;
    for (int v = 0; v < 2; ++v)
        cut = cut || (al.pieces[v] && sm_piece_cut((uint32_t)al.maxlen, (uint32_t)al.bucket_plen[v]));
    set_bucket(ctx, a, r, false, views);
    const WalkArgs as = a;
    double vs = bucket_voxels(ctx, r, false, views, a.dcall);
#ifdef SM_DEV  // timing experiment only (wrong results): no walker launch for buckets below this many nodes
    if (const char* e = sm_dev_knob("SM_EXP_SKIP_SMALL_WALK"))
        if (vs < atof(e) * a.dcall) vs = 0.0;
#endif
#ifndef SM_PRE_FUSED  // the aggregates in a launch of their own, before the chains
    if (cut) CHECK(timed(ctx, ctx->st2, KF_UP_PRE, vl, [&] { return launch_up_pre(ctx->st2, al, spl); }, 0.0));
    CHECK(timed(ctx, ctx->st2, KF_UP_CHAIN, vl, [&] { return launch_up_chain(ctx->st2, al, spl); }));
    CHECK(timed(ctx, ctx->st, KF_UP_WALK, vs, [&] { return launch_up(ctx->st, as, spl, false); }));
#else  // A/B: the aggregates run as extra blocks of the walker launch; the chains read them, so
    // they follow it.  Filter wall clock -0.02 ms at C2, but +0.03..0.08 ms per frame with frames in
    // flight (the separate launch's idle GPU is filled by the other frames)
    CHECK(timed(ctx, ctx->st, KF_UP_WALK, (vs > 0 || cut) ? std::max(vs, 1.0) : 0.0,
                [&] { return launch_up(ctx->st, as, spl, false, cut ? &al : nullptr); }, vs));
    CHECK(join(ctx, ctx->st2, ctx->st));
    CHECK(timed(ctx, ctx->st2, KF_UP_CHAIN, vl, [&] { return launch_up_chain(ctx->st2, al, spl); }));
#endif
    return SM_OK;
}

sm_status down_round(sm_ctx* ctx, WalkArgs& a, uint32_t r, int spl, int views, bool store_all) {
    CHECK(join(ctx, ctx->st, ctx->st2));
    CHECK(join(ctx, ctx->st2, ctx->st));
    set_bucket(ctx, a, r, true, views);
    const WalkArgs al = a;
    CHECK(timed(ctx, ctx->st2, KF_DOWN_CHAIN, bucket_voxels(ctx, r, true, views, a.dcall),
                [&] { return launch_down_long(ctx->st2, al, spl, store_all ? 1 : 0); }));
    set_bucket(ctx, a, r, false, views);
    const WalkArgs as = a;
    double vs = bucket_voxels(ctx, r, false, views, a.dcall);
#ifdef SM_DEV  // timing experiment only (wrong results), as up_round
    if (const char* e = sm_dev_knob("SM_EXP_SKIP_SMALL_WALK"))
        if (vs < atof(e) * a.dcall) vs = 0.0;
#endif
    CHECK(timed(ctx, ctx->st, KF_DOWN_WALK, vs, [&] {
        return store_all ? launch_down_debug(ctx->st, as, spl, false) : launch_down(ctx->st, as, spl, false);
    }));
    return SM_OK;
}

sm_status ensure_filter_bufs(sm_ctx* ctx, int Dpad) {
    const size_t N = (size_t)ctx->W * ctx->H;
    for (int v = 0; v < 2; ++v) {
        if (!view_on(ctx->views, v)) continue;  // a one-view call: the kernels never touch the other view's rows
        CHECK(ensure(ctx, ctx->U[v], N * (size_t)Dpad * 8));
        if (ctx->use_vol) CHECK(ensure(ctx, ctx->Cst[v], N * (size_t)Dpad * 4));  // ingested cost rows only
        CHECK(ensure(ctx, ctx->idx[v], N * 4));
        CHECK(ensure(ctx, ctx->minc[v], N * 8));
        CHECK(ensure(ctx, ctx->disp[v], N * 4));
    }
    return SM_OK;
}

// cross-workgroup synchronisation state of one filter call: piece aggregates and status words, and
// the call's epoch (no per-call reset of any word)
sm_status setup_sync(sm_ctx* ctx, WalkArgs& a, size_t N, int Dpad) {
    // piece buffers: segment aggregates and 8 status-word arrays (up: done/merged/final, down: same
    // + aggregate published)
    const size_t pcap = piece_cap(N);
    a.pstride = (int)pcap;
    a.piece_len = piece_len();
    {
        const char* e = sm_knob("SM_REPAIR_MAX");
        a.repair_max = e ? std::max(1, atoi(e)) : 1 << 30;
    }
    a.err = ctx->d_err;
    {
        const char* e = sm_knob("SM_WAIT_ITERS");  // read per call: the forced-timeout test lowers it
        a.wait_iters = e ? std::max(0, atoi(e)) : 1 << 24;
    }
    a.piece_dbg = nullptr;
    if (sm_knob("SM_PIECE_DEBUG")) {  // per-call repair statistics on stderr (tools)
        CHECK(ensure(ctx, ctx->pdbg, 128));
        HIPC(hipMemsetAsync(ctx->pdbg.p, 0, 128, ctx->st));
        if (atoi(sm_knob("SM_PIECE_DEBUG")) == 2) {
            const unsigned long long one = 1;
            HIPC(hipMemcpyAsync(P<unsigned long long>(ctx->pdbg) + 15, &one, 8, hipMemcpyHostToDevice, ctx->st));
            HIPC(hipStreamSynchronize(ctx->st));
        }
        a.piece_dbg = P<unsigned long long>(ctx->pdbg);
    }
    for (int v = 0; v < 2; ++v) {
        if (view_on(ctx->views, v)) {
            // the segment aggregates of the cut paths (2 rows per 32-node segment; a bucket's down pieces,
            // listed first among its items, write theirs at the piece index, below the bucket's segment
            // count since a piece spans >= 16 segments), the rows of the cut paths' nodes (32 per segment:
            // the up repair's corrections, the down pieces' last rows) and the compact A rows of light
            // children's parents, all sized by this layout's counts with 1/16 of headroom, so frames whose
            // counts vary a little do not reallocate (hipFree synchronises the device).  Round 6: the
            // aggregates were sized by the piece capacity (N/16 segments: 4.2 GB of a C3 context, against
            // ~0.5 GB used); a C3 context is now below 50 GB
            const auto& L = ctx->layout[v];
            const size_t nseg = (size_t)L.seg_begin[SM_NBUCKETS];
            if (ctx->agg[v].n < nseg * 2 * Dpad * 8 || !ctx->agg[v].p)
                CHECK(ensure(ctx, ctx->agg[v], (nseg + nseg / 16 + 64) * 2 * (size_t)Dpad * 8));
            const size_t nfix = nseg * SM_PRE_SEG, nacmp = L.n_has_light;
            if (ctx->fix[v].n < nfix * Dpad * 8) CHECK(ensure(ctx, ctx->fix[v], (nfix + nfix / 16 + 64) * Dpad * 8));
            if (ctx->acmp[v].n < nacmp * Dpad * 8) CHECK(ensure(ctx, ctx->acmp[v], (nacmp + nacmp / 16 + 64) * Dpad * 8));
        }
        a.fix[v] = P<double>(ctx->fix[v]);   // (set per bucket by set_bucket)
        a.A[v] = P<double>(ctx->acmp[v]);
        const bool fresh = ctx->pstat[v].n < pcap * 8 * 4;
        CHECK(ensure(ctx, ctx->pstat[v], pcap * 8 * 4));
        if (fresh) HIPC(hipMemsetAsync(ctx->pstat[v].p, 0, pcap * 8 * 4, ctx->st));
    }
    a.epoch = ++ctx->epoch;
    if (a.epoch == 0 || a.epoch >= 0x7FFFFFFFu) {  // wrapped (merged words hold 2*epoch+1): clear every word
        for (int v = 0; v < 2; ++v) HIPC(hipMemsetAsync(ctx->pstat[v].p, 0, pcap * 8 * 4, ctx->st));
        a.epoch = ctx->epoch = 1;
    }
    return SM_OK;
}

// up + down passes over all rounds for nviews views; debug_store_all stores every A row
sm_status stage_filter(sm_ctx* ctx, int D, int dglob0, int views, bool debug_store_all, const WtaCfg* wta = nullptr) {
    const size_t N = (size_t)ctx->W * ctx->H;
    const int spl = spl_for(D);
    const int Dpad = dpad_for(D);
    CHECK(ensure_filter_bufs(ctx, Dpad));
    uint32_t nr = 0;
    for (int v = 0; v < 2; ++v)
        if (view_on(views, v)) nr = std::max(nr, ctx->layout[v].nrounds);
    WalkArgs a = walk_args(ctx, Dpad, D, dglob0);
    if (wta) a.wta = *wta;
    CHECK(setup_sync(ctx, a, N, Dpad));
    if (debug_store_all)  // every node's A row by slot (sm_aggregate_debug)
        for (int v = 0; v < 2; ++v)
            if (view_on(views, v)) {
                CHECK(ensure(ctx, ctx->adbg[v], N * (size_t)Dpad * 8));
                a.Adbg[v] = P<double>(ctx->adbg[v]);
            }
    a.vol = ctx->use_vol ? 1 : 0;
    a.leaf_cost = (!a.vol && !debug_store_all && !sm_knob("SM_NO_LEAF_COST")) ? 1 : 0;  // SM_NO_LEAF_COST: A/B
    if (a.vol)  // cost rows of every slot from the caller's volumes (slots come from the layout)
        for (int v = 0; v < 2; ++v)
            if (view_on(views, v))
                HIPC(launch_vol_rows(ctx->st, P<float>(ctx->vin[v]), N, dglob0, D, Dpad, P<uint32_t>(ctx->slotpix[v]),
                                 P<float>(ctx->Cst[v])));
    ctx->nfev = ctx->nsev = 0;
    ctx->fam.clear();
    ctx->fam_vox.clear();
    ctx->fam_ev.clear();
    ctx->ev_open = false;
    for (uint32_t i = 0; i < nr; ++i) CHECK(up_round(ctx, a, nr - 1 - i, spl, views));  // deepest first
    CHECK(join(ctx, ctx->st, ctx->st2));
    HIPC(hipEventRecord(ctx->ev[6], ctx->st));  // up | down boundary (stage times)
    ctx->ev_open = false;
    for (uint32_t r = 0; r < nr; ++r) CHECK(down_round(ctx, a, r, spl, views, debug_store_all));
    CHECK(join(ctx, ctx->st, ctx->st2));  // everything after the filter runs on st
    if (a.piece_dbg) {
        unsigned long long h[16];
        HIPC(hipMemcpyAsync(h, a.piece_dbg, 128, hipMemcpyDeviceToHost, ctx->st));
        HIPC(hipStreamSynchronize(ctx->st));
        fprintf(stderr, "pieces: fast %llu slow %llu repair nodes sum %llu max %llu | merge <8 %llu <16 %llu <32 %llu <64 %llu <128 %llu >=128 %llu never %llu\n",
                h[0], h[1], h[2], h[3], h[8], h[9], h[10], h[11], h[12], h[13], h[14]);
        fprintf(stderr, "down pieces: fast %llu slow %llu repair nodes sum %llu max %llu\n", h[4], h[5], h[6], h[7]);
    }
    (void)N;
    return SM_OK;
}

// per-family totals of the last filter call (after the stream has been synchronised)
sm_status collect_filter_stats(sm_ctx* ctx) {
    sm_kernel_stat ks[KF_N]{};
    for (int f = 0; f < KF_N; ++f) {
        snprintf(ks[f].name, sizeof(ks[f].name), "%s", kf_name[f]);
        ks[f].bytes_per_voxel = kf_bytes[f];
    }
    for (size_t k = 0; k < ctx->fam.size(); ++k) {
        float ms;
        HIPC(hipEventElapsedTime(&ms, ctx->fev[ctx->fam_ev[k].first], ctx->fev[ctx->fam_ev[k].second]));
        const int f = ctx->fam[k];
        ks[f].launches += 1;  // only launches are recorded (a bucket without paths launches nothing)
        ks[f].ms += ms;
        ks[f].voxels += ctx->fam_vox[k];
    }
    static_assert(sizeof(ctx->kstats) >= sizeof(ks), "kstats holds every family");
    memcpy(ctx->kstats, ks, sizeof(ks));
    sm_filter_stats fs{};
    for (int f = 0; f < KF_N; ++f) {
        const bool up = kf_up(f);
        (up ? fs.up_ms : fs.down_ms) += ks[f].ms;
        (up ? fs.up_bytes : fs.down_bytes) += ks[f].voxels * ks[f].bytes_per_voxel;
        (up ? fs.up_launches : fs.down_launches) += ks[f].launches;
    }
    ctx->stats = fs;
    return SM_OK;
}

// Runs whenever the context has a communicator, a one-rank one included (the exchange then reduces
// over that rank alone: tests drive k_cand / k_finalize and the RCCL calls on one GPU).
sm_status stage_reduce(sm_ctx* ctx) {
    if (!ctx->comm) return SM_OK;
    const size_t N = (size_t)ctx->W * ctx->H;
    for (int v = 0; v < 2; ++v)
        if (view_on(ctx->views, v)) {
        CHECK(ensure(ctx, ctx->gmin[v], N * 8));
        CHECK(ensure(ctx, ctx->cand[v], N * 4));
        CHECK(ensure(ctx, ctx->gidx[v], N * 4));
    }
    // lexicographic (cost, global d) minimum: the reference's strict-< first-minimum rule
    // (Stereo3DMST.cpp:177, PatchMatchStereoGPU.cu:1712) over contiguous ascending shards.
    RCCLC(ncclGroupStart());
    for (int v = 0; v < 2; ++v)
        if (view_on(ctx->views, v))
        RCCLC(ncclAllReduce(ctx->minc[v].p, ctx->gmin[v].p, N, ncclFloat64, ncclMin, ctx->comm, ctx->st));
    RCCLC(ncclGroupEnd());
    if (!ctx->sub)
        for (int v = 0; v < 2; ++v)
        if (view_on(ctx->views, v))
            HIPC(launch_cand(ctx->st, P<double>(ctx->minc[v]), P<double>(ctx->gmin[v]), P<int32_t>(ctx->idx[v]),
                             P<int32_t>(ctx->cand[v]), N));
    if (ctx->sub) {
        // subpixel: the candidate is (global index << 32 | float bits of the rank's subpixel disparity),
        // so the MIN over ranks carries the winning rank's disparity with the lowest index
        for (int v = 0; v < 2; ++v)
        if (view_on(ctx->views, v)) {
            CHECK(ensure(ctx, ctx->cand[v], N * 8));
            CHECK(ensure(ctx, ctx->gidx[v], N * 8));
            HIPC(launch_cand64(ctx->st, P<double>(ctx->minc[v]), P<double>(ctx->gmin[v]), P<int32_t>(ctx->idx[v]),
                               P<float>(ctx->disp[v]), P<unsigned long long>(ctx->cand[v]), N));
        }
        RCCLC(ncclGroupStart());
        for (int v = 0; v < 2; ++v)
        if (view_on(ctx->views, v))
            RCCLC(ncclAllReduce(ctx->cand[v].p, ctx->gidx[v].p, N, ncclUint64, ncclMin, ctx->comm, ctx->st));
        RCCLC(ncclGroupEnd());
        for (int v = 0; v < 2; ++v)
        if (view_on(ctx->views, v))
            HIPC(launch_finalize64(ctx->st, P<double>(ctx->gmin[v]), P<unsigned long long>(ctx->gidx[v]), P<double>(ctx->minc[v]),
                                   P<int32_t>(ctx->idx[v]), P<float>(ctx->disp[v]), N));
        return SM_OK;
    }
    RCCLC(ncclGroupStart());
    for (int v = 0; v < 2; ++v)
        if (view_on(ctx->views, v))
        RCCLC(ncclAllReduce(ctx->cand[v].p, ctx->gidx[v].p, N, ncclInt32, ncclMin, ctx->comm, ctx->st));
    RCCLC(ncclGroupEnd());
    for (int v = 0; v < 2; ++v)
        if (view_on(ctx->views, v))
        HIPC(launch_finalize(ctx->st, P<double>(ctx->gmin[v]), P<int32_t>(ctx->gidx[v]), P<double>(ctx->minc[v]),
                             P<int32_t>(ctx->idx[v]), P<float>(ctx->disp[v]), N));
    return SM_OK;
}

// Guided-filter aggregator (sm_guided.hip): guide statistics per view, then batches of up to 32
// slices of AGD cost (k_cost_volume), each through the colour guided filter and the running WTA.
sm_status stage_guided(sm_ctx* ctx, int D, int d0, int dtot, int sub, int rad, float eps) {
    const int W = ctx->W, H = ctx->H;
    const size_t N = (size_t)W * H;
    const int S = std::min(D, 32);
    const size_t NS = std::max(N, gf_band_plane(W, H));  // planes of the row band layout (fused path)
    CHECK(ensure(ctx, ctx->gf_planes, 9 * N * 4));
    CHECK(ensure(ctx, ctx->gf_means, 9 * N * 4));
    CHECK(ensure(ctx, ctx->gf_pl, 4 * (size_t)S * NS * 4));
    CHECK(ensure(ctx, ctx->gf_tmp, std::max<size_t>(9, 4 * (size_t)S) * N * 4));
    for (int v = 0; v < 2; ++v) {
        CHECK(ensure(ctx, ctx->gf_stats[v], 9 * NS * 4));
        CHECK(ensure(ctx, ctx->gf_state[v], 5 * N * 4));
        CHECK(ensure(ctx, ctx->vol[v], (size_t)S * N * 4));
        CHECK(ensure(ctx, ctx->idx[v], N * 4));
        CHECK(ensure(ctx, ctx->minc[v], N * 8));
        CHECK(ensure(ctx, ctx->disp[v], N * 4));
    }
    GfStateArgs sa[2];
    for (int v = 0; v < 2; ++v) {
        float* b = P<float>(ctx->gf_state[v]);
        sa[v] = GfStateArgs{b, reinterpret_cast<int32_t*>(b + N), b + 2 * N, b + 3 * N, b + 4 * N};
        HIPC(launch_gf_guide(ctx->st, P<uint32_t>(ctx->bgrx[v]), W, H, rad, eps, P<float>(ctx->gf_planes), P<float>(ctx->gf_tmp),
                             P<float>(ctx->gf_means), P<float>(ctx->gf_stats[v])));
        HIPC(launch_gf_init(ctx->st, sa[v], N));
    }
    for (int b = 0; b < D; b += S) {
        const int s = std::min(S, D - b);
        HIPC(launch_cost_volume(ctx->st, P<uint32_t>(ctx->bgrx[0]), P<float>(ctx->gray[0]), P<uint32_t>(ctx->bgrx[1]),
                                P<float>(ctx->gray[1]), P<float>(ctx->atab), W, H, d0 + b, s, P<float>(ctx->vol[0]),
                                P<float>(ctx->vol[1])));
        for (int v = 0; v < 2; ++v)
            HIPC(launch_gf_batch(ctx->st, P<float>(ctx->vol[v]), P<uint32_t>(ctx->bgrx[v]), P<float>(ctx->gf_stats[v]), W, H,
                                 rad, s, b, P<float>(ctx->gf_pl), P<float>(ctx->gf_tmp), sa[v]));
    }
    for (int v = 0; v < 2; ++v)
        HIPC(launch_gf_out(ctx->st, sa[v], N, d0, dtot, sub, P<int32_t>(ctx->idx[v]), P<double>(ctx->minc[v]),
                           P<float>(ctx->disp[v])));
    return SM_OK;
}

// output step on the final (reduced) float maps, in the reference's order: LabelToDisp + scaling
// (Stereo3DMST.cpp:189-201, 900-902), L-R check (+ fill) (:632-709, 904), then the GPU PatchMatch's
// occlusion handling (PatchMatchStereoGPU.cu:1128-1288).  dmax = the total disparity range.
sm_status stage_post(sm_ctx* ctx, int post, int dmax) {
    if (!post) return SM_OK;
    const int W = ctx->W, H = ctx->H;
    const size_t N = (size_t)W * H;
    float* L = P<float>(ctx->disp[0]);
    float* R = P<float>(ctx->disp[1]);
    if (post & (SM_POST_LR_FILL | SM_POST_OCCLUSION | SM_POST_OCCLUSION_ZERO)) {
        CHECK(ensure(ctx, ctx->post_mask, 2 * N));
        CHECK(ensure(ctx, ctx->post_scratch, 2 * N * 4));
    }
    if (post & SM_POST_LABEL_TO_DISP) HIPC(launch_label_to_disp(ctx->st, L, R, N, dmax));
    if (post & SM_POST_LR_CHECK) {
        const bool fill = (post & SM_POST_LR_FILL) != 0;
        HIPC(launch_lr_check(ctx->st, L, R, W, H, dmax, fill ? P<uint8_t>(ctx->post_mask) : nullptr));
        if (fill) HIPC(launch_lr_fill(ctx->st, L, P<uint8_t>(ctx->post_mask), W, H, P<int>(ctx->post_scratch)));
    }
    if (post & (SM_POST_OCCLUSION | SM_POST_OCCLUSION_ZERO))
        HIPC(launch_occlusion(ctx->st, L, R, W, H, 1.0f, (post & SM_POST_OCCLUSION_ZERO) ? 1 : 0, 0.0f,
                              P<uint8_t>(ctx->post_mask), P<int>(ctx->post_scratch)));
    return SM_OK;
}

// ----------------------------------------------------------------------------- MST_PMS (SM_AGG_PMS)
double now_ms();

template <class T>
sm_status upload_vec(sm_ctx* ctx, DevBuf& b, const std::vector<T>& v) {
    CHECK(ensure(ctx, b, std::max<size_t>(v.size(), 1) * sizeof(T)));
    if (!v.empty()) HIPC(hipMemcpyAsync(b.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, ctx->st));
    return SM_OK;
}

// SM_PMS_SERIAL=1: every MST_PMS call in serial mode (tests compare the two modes); SM_PMS_MAX_ROUNDS:
// speculative passes per call before the rest of the call runs serially
bool pms_serial_only() {
    const char* e = sm_knob("SM_PMS_SERIAL");
    return e && atoi(e) == 1;
}
int pms_max_rounds() {
    const char* e = sm_knob("SM_PMS_MAX_ROUNDS");
    return e ? std::max(1, atoi(e)) : 8;
}

// The forest, schedule and per-tree tables of view v on the device (host forest built already).
sm_status pms_upload_view(sm_ctx* ctx, int v, int L) {
    PmsState& S = ctx->pms[v];
    const PmsForest& f = S.f;
    const int K = f.K;
    const size_t N = (size_t)f.W * f.H;
    S.h_rtree.resize(N);
    S.h_pt.resize(K);
    S.h_lab.resize(K + 1);
    S.h_abase.resize(K + 1);
    long long abase = 0, deg_sum = 0;
    int lab = 0;
    for (int t = 0; t < K; ++t) {
        const int deg = f.nb_start[t + 1] - f.nb_start[t];
        const int pt = (std::max(deg, L) + 1) & ~1;  // proposals per A row (16-byte rows)
        S.h_pt[t] = pt;
        S.h_abase[t] = abase;
        S.h_lab[t] = lab;
        abase += (long long)(f.tree_start[t + 1] - f.tree_start[t]) * pt;
        lab += deg + L;
        deg_sum += deg;
        if (!f.on_device)
            for (int r = f.tree_start[t]; r < f.tree_start[t + 1]; ++r) S.h_rtree[r] = t;
    }
    S.h_abase[K] = abase;
    S.h_lab[K] = lab;
    S.dice_need = deg_sum + 4ll * L * K + 8;
    // pieces: backup offsets of the cut paths' non-head rows (A_up, saved before the down pass)
    std::vector<long long> cut_bak(std::max<size_t>(f.cuts.size(), 1), 0);
    long long bak = 0;
    for (size_t c = 0; c < f.cuts.size(); ++c) {
        cut_bak[c] = bak;
        bak += (long long)(f.cuts[c].len - f.piece) * S.h_pt[f.cuts[c].tree];
    }
    if (!f.on_device) {
        CHECK(upload_vec(ctx, S.cuts, f.cuts));
        CHECK(upload_vec(ctx, S.reps, f.reps));
    }
    CHECK(ensure(ctx, S.rep_flag, std::max<size_t>(f.reps.size(), 1) * 4));
    CHECK(ensure(ctx, S.pt_ph, (size_t)std::max(K, 1) * 4));
    CHECK(ensure(ctx, S.ab_ph, (size_t)std::max(K, 1) * 8));
    HIPC(hipMemsetAsync(S.rep_flag.p, 0, std::max<size_t>(f.reps.size(), 1) * 4, ctx->st));
    CHECK(upload_vec(ctx, S.cut_bak, cut_bak));
    CHECK(ensure(ctx, S.Abak, (size_t)std::max(bak, 1ll) * 8));
    if (!f.on_device) {  // the GPU build leaves these in place
        CHECK(upload_vec(ctx, S.rows, f.rows));
        CHECK(upload_vec(ctx, S.rtree, S.h_rtree));
        CHECK(upload_vec(ctx, S.paths, f.paths));
        CHECK(upload_vec(ctx, S.items, f.items));
        CHECK(upload_vec(ctx, S.rt_path, f.rt_path));
        CHECK(upload_vec(ctx, S.rt_item, f.rt_item));
        CHECK(upload_vec(ctx, S.tree_rounds, f.tree_rounds));
        CHECK(upload_vec(ctx, S.tree_start, f.tree_start));
        CHECK(upload_vec(ctx, S.bfs_pix, f.bfs_pix));
        CHECK(upload_vec(ctx, S.nb_start, f.nb_start));
        CHECK(upload_vec(ctx, S.nb, f.nb));
    }
    CHECK(upload_vec(ctx, S.tree_pt, S.h_pt));
    CHECK(upload_vec(ctx, S.tree_abase, S.h_abase));
    CHECK(upload_vec(ctx, S.tree_lab, S.h_lab));
    CHECK(ensure(ctx, S.nref, (size_t)std::max(K, 1) * 4));
    CHECK(ensure(ctx, S.lab, (size_t)std::max(lab, 1) * 16));
    CHECK(ensure(ctx, S.labu, (size_t)std::max(lab, 1) * 16));
    CHECK(ensure(ctx, S.labq, (size_t)std::max(lab, 1) * 4));
    CHECK(ensure(ctx, S.nprop, (size_t)(f.K + 1) * 4));
    CHECK(ensure(ctx, S.abc, N * 12));
    CHECK(ensure(ctx, S.minc, N * 8));
    CHECK(ensure(ctx, S.abc_bak, N * 12));
    CHECK(ensure(ctx, S.minc_bak, N * 8));
    CHECK(ensure(ctx, S.A, (size_t)std::max(abase, 1ll) * 8));
    CHECK(ensure(ctx, S.off, 16));
    CHECK(ensure(ctx, S.oguess, (size_t)std::max(K, 1) * 8));
    CHECK(ensure(ctx, S.cnt, (size_t)std::max(K, 1) * 4));
    CHECK(ensure(ctx, S.flag, (size_t)std::max(K, 1) * 4));
    CHECK(ensure(ctx, S.result, 16));
    // the planned walks' lists (k_pms_plan): per round, two lane-group classes of paths, and (path, chunk)
    // items of any phase (at most the round's prop items + one per path)
    {
        const int R = f.nrounds;
        std::vector<int32_t> pb(std::max(R, 1), 0), ib(std::max(R, 1), 0);
        for (int r = 0; r < R; ++r) {
            pb[r] = f.rt_path[(size_t)r * (K + 1)];
            ib[r] = f.rt_item[(size_t)r * (K + 1)] + f.rt_path[(size_t)r * (K + 1)];
        }
        CHECK(upload_vec(ctx, S.plan_base, pb));
        CHECK(upload_vec(ctx, S.plan_ibase, ib));
        CHECK(ensure(ctx, S.plan_cnt, (size_t)std::max(R, 1) * PMS_NCNT * 4));
        CHECK(ensure(ctx, S.plan_path, (size_t)std::max(f.npaths, 1) * (PMS_NCLS - 1) * 4));
        // wave items at [0, cap), chain items at [cap, 2 cap)
        CHECK(ensure(ctx, S.plan_item, 2 * (size_t)std::max(f.nitems + f.npaths, 1) * sizeof(PmsItem)));
    }
    return SM_OK;
}

PmsDev pms_dev(sm_ctx* ctx, int v, int D) {
    PmsState& S = ctx->pms[v];
    PmsDev d{};
    d.rows = P<PmsRow>(S.rows);
    d.rtree = P<int32_t>(S.rtree);
    d.paths = P<PmsPath>(S.paths);
    d.items = P<PmsItem>(S.items);
    d.rt_path = P<int32_t>(S.rt_path);
    d.rt_item = P<int32_t>(S.rt_item);
    d.tree_rounds = P<int32_t>(S.tree_rounds);
    d.tree_start = P<int32_t>(S.tree_start);
    d.bfs_pix = P<int32_t>(S.bfs_pix);
    d.nb_start = P<int32_t>(S.nb_start);
    d.nb = P<int32_t>(S.nb);
    d.tree_pt = P<int32_t>(S.tree_pt);
    d.tree_abase = P<long long>(S.tree_abase);
    d.tree_lab = P<int32_t>(S.tree_lab);
    d.nref = P<int32_t>(S.nref);
    d.lab = P<float4>(S.lab);
    d.labu = P<float4>(S.labu);
    d.nprop = nullptr;  // set for the speculative passes' propagation phase only (pms_speculative_call)
    d.labq = P<int32_t>(S.labq);
    d.abc = P<float>(S.abc);
    d.minc = P<double>(S.minc);
    d.abc_bak = P<float>(S.abc_bak);
    d.minc_bak = P<double>(S.minc_bak);
    d.A = P<double>(S.A);
    d.vol = P<float>(S.vrows);
    d.dice = P<float>(ctx->pms_dice);
    d.dice_n = ctx->pms_dice_n;
    d.rnd = nullptr;
    d.off = P<long long>(S.off);
    d.oguess = P<long long>(S.oguess);
    d.cnt = P<int32_t>(S.cnt);
    d.flag = P<int32_t>(S.flag);
    d.result = P<int32_t>(S.result);
    d.err = ctx->d_err + 1 + v;  // a word per view: the views' calls run concurrently (h_err[1 + v])
    d.prof = nullptr;
    d.evals = nullptr;
    if (sm_knob("SM_PMS_PROF")) {  // diagnostics: serial-kernel segment times, printed per call
        if (ensure(ctx, S.prof, 16 * 8) == SM_OK) d.prof = P<long long>(S.prof);
    }
    d.slut = P<double>(ctx->slut);
    d.s2lut = P<double>(ctx->s2lut);
    d.cuts = P<PmsCut>(S.cuts);
    d.reps = P<PmsRep>(S.reps);
    d.cut_bak = P<long long>(S.cut_bak);
    d.plan_cnt = P<int32_t>(S.plan_cnt);
    d.plan_path = P<int32_t>(S.plan_path);
    d.plan_item = P<PmsItem>(S.plan_item);
    d.plan_base = P<int32_t>(S.plan_base);
    d.plan_ibase = P<int32_t>(S.plan_ibase);
    d.npaths_total = S.f.npaths;
    d.item_cap = std::max(S.f.nitems + S.f.npaths, 1);
    d.Abak = P<double>(S.Abak);
    d.rep_flag = P<uint32_t>(S.rep_flag);
    d.piece = S.f.piece;
    d.hi_bak = 0;
    d.W = ctx->W;
    d.Dv = D;
    d.Dmax = D;
    d.K = S.f.K;
    d.nrounds = S.f.nrounds;
    return d;
}

// MST_PMS pieces: heavy paths of at least 2 x this many rows are cut (SM_PMS_PIECE; 0: none).  512
// balances a piece's walk against the repairs of the pieces above it (~30-60 rows each at C2).
int pms_piece() {
    const char* e = sm_knob("SM_PMS_PIECE");
    return e ? std::max(0, atoi(e)) : 512;
}

// trees whose work (nodes x 64-proposal chunks) is at least this run over the whole GPU in serial mode
// (their rounds as launches); smaller ones go to the one-workgroup k_pms_serial in runs.  C2 first
// call per view (tools/pms_bench.py): 32768 -> 376 ms, 8192 -> 278, 2048 -> 229, 1024 -> 223, 512 ->
// 221, 128 -> 226 ms.
long long pms_big_tree() {
    const char* e = sm_knob("SM_PMS_BIG");
    return e ? std::max(1ll, atoll(e)) : 1024;
}

// One phase (0: propagation, 1: refinement) of trees [t_lo, t_hi) over the whole GPU: the data terms
// into the A rows, the up rounds deepest first, the cut paths' pieces repaired after each round, the cut paths' A_up rows saved, the
// down rounds root first (repaired likewise), then the per-pixel update.
sm_status pms_phase(sm_ctx* ctx, hipStream_t st, int v, const PmsDev& d0, int phase, int t_lo, int t_hi) {
    const PmsForest& f = ctx->pms[v].f;
    // the phase's A rows packed by its proposal counts (k_pms_layout; round 4: 1.2 GB of static max-degree
    // rows per phase at C2 before)
    PmsDev d = d0;
    const size_t K1 = (size_t)f.K + 1;
    int R = 0;
    for (int t = t_lo; t < t_hi; ++t) R = std::max(R, f.tree_rounds[t]);
    // (the layout launch also zeroes the plan's counters)
    HIPC(launch_pms_layout(st, d0, phase, t_lo, t_hi, P<int32_t>(ctx->pms[v].pt_ph), P<long long>(ctx->pms[v].ab_ph),
                           d0.plan_cnt, PMS_NCNT * R));
    d.tree_pt = P<int32_t>(ctx->pms[v].pt_ph);
    d.tree_abase = P<long long>(ctx->pms[v].ab_ph);
    const std::vector<int32_t>& rt = phase == 0 ? f.rt_item : f.rt_path;
    HIPC(launch_pms_cost(st, d, phase, f.tree_start[t_lo], f.tree_start[t_hi]));
    // planned walks (k_pms_plan / k_pms_walk_plan): the round's paths in lane-group classes by their
    // tree's proposal count, over a persistent grid of at most PMS_WALK_WAVES waves (round 4; one wave per
    // (path, 64-proposal chunk) item before)
    constexpr int PMS_WALK_WAVES = 16384;
    std::vector<int> bound(std::max(R, 1), 0);
    {
        int maxp = 0;
        for (int r = 0; r < R; ++r) {
            const int np = f.rt_path[r * K1 + t_hi] - f.rt_path[r * K1 + t_lo];
            maxp = std::max(maxp, np);
            // virtual tasks: at most one per path of the classes, plus the chunks of the rest
            bound[r] = std::min(PMS_WALK_WAVES, np + (phase == 0 ? rt[r * K1 + t_hi] - rt[r * K1 + t_lo] : 0));
        }
        // SM_PMS_CHAIN_MIN: the chain threshold (at least SM_PMS_CHAIN_LEN, whose counts bound the grid;
        // tests lower it to put more chain items on small images)
        const char* cm = sm_knob("SM_PMS_CHAIN_MIN");
        HIPC(launch_pms_plan(st, d, phase, t_lo, t_hi, R, maxp, cm ? atoi(cm) : SM_PMS_CHAIN_DEFAULT, true));
    }
    // pieces: every guessed piece repairs at once, then a gated sequential pass; maxp[r] = the most pieces
    // of a cut repaired in round r
    std::vector<int> maxp(std::max(R, 1), 0);
    for (int r = 0; r < R; ++r)
        for (int k = f.rt_rep[r * K1 + t_lo]; k < f.rt_rep[r * K1 + t_hi]; ++k)
            maxp[r] = std::max(maxp[r], f.cuts[f.reps[k].cut].npieces);
    // chain items (paths / pieces of >= SM_PMS_CHAIN_LEN rows, k_pms_chain): the host's bound per round
    std::vector<int> nlong(std::max(R, 1), 0);
    for (int r = 0; r < R; ++r) nlong[r] = f.rt_long[r * K1 + t_hi] - f.rt_long[r * K1 + t_lo];
    // a round's chain items and walker tasks are disjoint paths whose inputs are final; one after the
    // other on the view's stream (a chain stream beside the walkers cost more in event fork / join than
    // the overlap won: 960 against 670 ms per 100-call frame, round 4)
    auto round = [&](int r, bool up) -> sm_status {
        HIPC(launch_pms_chain(st, d, phase, up, r, nlong[r]));
        HIPC(launch_pms_walk_plan(st, d, phase, up, r, bound[r]));
        HIPC(launch_pms_repair(st, d, phase, up, f.rt_rep[r * K1 + t_lo], f.rt_rep[r * K1 + t_hi], maxp[r]));
        return SM_OK;
    };
    for (int r = R - 1; r >= 0; --r) CHECK(round(r, true));
    HIPC(launch_pms_cut_backup(st, d, f.tree_cut[t_lo], f.tree_cut[t_hi]));
    for (int r = 0; r < R; ++r) CHECK(round(r, false));
    HIPC(launch_pms_update(st, d, phase, f.tree_start[t_lo], f.tree_start[t_hi]));
    return SM_OK;
}


// Trees [t0, t1) in the reference's order from the dice offset *off.  Runs of small trees go to one
// workgroup (k_pms_serial); a large tree's phases are launched over the whole GPU, round by round.
sm_status pms_serial_range(sm_ctx* ctx, hipStream_t st, int v, const PmsDev& d, int t0, int t1) {
    const PmsForest& f = ctx->pms[v].f;
    const long long big = pms_big_tree();
    int run = t0;
    for (int t = t0; t <= t1; ++t) {
        bool is_big = false;
        if (t < t1) {
            const long long n = f.tree_start[t + 1] - f.tree_start[t];
            const int deg = f.nb_start[t + 1] - f.nb_start[t];
            // a tree with cut paths needs the repair launches: never in the one-workgroup kernel
            is_big = n * ((std::max(deg, 1) + 63) / 64) >= big || f.tree_cut[t + 1] > f.tree_cut[t];
        }
        if (t < t1 && !is_big) continue;
        HIPC(launch_pms_serial(st, d, run, t));
        if (t > run) {  // the run's distinct propagation counts (nprop: k_pms_count's input)
            PmsDev dd = d;
            dd.labu = P<float4>(ctx->pms[v].labu);
            dd.nprop = P<int32_t>(ctx->pms[v].nprop);
            HIPC(launch_pms_prop_dedupe(st, dd, run, t));
        }
        run = t + 1;
        if (t == t1) break;
        const int deg = f.nb_start[t + 1] - f.nb_start[t];
        if (deg > 0) {  // its labels, then over its distinct propagation labels (one launch: k_pms_prop_tree)
            PmsDev dd = d;
            dd.labu = P<float4>(ctx->pms[v].labu);
            dd.nprop = P<int32_t>(ctx->pms[v].nprop);
            HIPC(launch_pms_prop_tree(st, dd, t));
            dd.lab = dd.labu;
            CHECK(pms_phase(ctx, st, v, dd, 0, t, t + 1));
        }
        HIPC(launch_pms_ref_one(st, d, t));
        // a refinement that drew no in-range level (nref == 0, most of a first call's trees) has nothing to
        // walk: its ~20 launches would all be empty, so read the count back (the view's pinned result slot)
        // and skip the phase
        int32_t* h_nref = ctx->h_pms_res + 4 * v + 3;
        HIPC(hipMemcpyAsync(h_nref, P<int32_t>(ctx->pms[v].nref) + t, 4, hipMemcpyDeviceToHost, st));
        HIPC(hipStreamSynchronize(st));
        if (*h_nref == 0) continue;
        CHECK(pms_phase(ctx, st, v, d, 1, t, t + 1));
    }
    return SM_OK;
}

// One speculative MST_PMS call of one view (iteration > 0).  A pass over the trees [t_lo, K): guessed
// offsets, every tree's propagation and refinement, validation.  Every tree before the first invalid
// one (t*) is exact.  t* goes back to the call's starting state and runs serially (its inputs are exact
// now).  If t* failed on its offset, every later tree drew from the wrong place: they are restored as
// well and the next pass speculates from t* + 1.  If only its sampled inputs were stale, the later
// trees keep their results and are validated again against t*'s exact labels and offset (a tree whose
// count changed shows up as the next offset failure), so a stale input costs one serial tree instead
// of a pass.
// Per view counters of the concurrent view threads (summed into sm_pms_stats after the calls)
struct PmsRun {
    hipStream_t st = nullptr;
    int32_t* h_res = nullptr;  // pinned: the validation result
    int spec_rounds = 0, serial_trees = 0;
    double first_ms = 0.0, later_ms = 0.0;
};

sm_status pms_speculative_call(sm_ctx* ctx, PmsRun& run, int v, PmsDev& d) {
    const hipStream_t st = run.st;
    PmsState& S = ctx->pms[v];
    const PmsForest& f = S.f;
    const int K = f.K;
    const size_t N = (size_t)f.W * f.H;
    const int max_rounds = pms_max_rounds();
    HIPC(launch_pms_backup(st, d, N));
    HIPC(hipMemsetAsync(S.off.p, 0, 16, st));
    int t_lo = 0, rounds = 0;
    bool pass = true;
    while (t_lo < K) {
        if (pass) {
            if (rounds >= max_rounds) {  // pathological: finish the call in order
                CHECK(pms_serial_range(ctx, st, v, d, t_lo, K));
                run.serial_trees += K - t_lo;
                break;
            }
            ++rounds;
            ++run.spec_rounds;
            // the draws trees [t_lo, K) can consume: their propagation draws + 4 per refinement level
            const long long wn =
                (long long)(f.nb_start[K] - f.nb_start[t_lo]) + 4ll * sm_pms_levels(d.Dmax) * (K - t_lo) + 8;
            HIPC(launch_pms_guess(st, d, t_lo, wn));
            HIPC(launch_pms_prop_setup(st, d, t_lo, f.nb_start[K] - f.nb_start[t_lo]));
            {  // propagation over each tree's distinct labels (k_pms_prop_dedupe)
                PmsDev dd = d;
                dd.nprop = P<int32_t>(S.nprop);
                HIPC(launch_pms_prop_dedupe(st, dd, t_lo, K));  // lab -> labu
                dd.lab = P<float4>(S.labu);                        // the phase reads the distinct labels
                CHECK(pms_phase(ctx, st, v, dd, 0, t_lo, K));
            }
            HIPC(launch_pms_ref_setup(st, d, t_lo));
            CHECK(pms_phase(ctx, st, v, d, 1, t_lo, K));
        }
        HIPC(launch_pms_validate(st, d, t_lo));
        HIPC(hipMemcpyAsync(run.h_res, S.result.p, 16, hipMemcpyDeviceToHost, st));
        HIPC(hipStreamSynchronize(st));
        const int ts = run.h_res[0], why = run.h_res[1];
        if (ts < t_lo || ts > K || (ts < K && why != 1 && why != 2))
            return fail(ctx, SM_ERR_STATE, "MST_PMS validation returned a bad tree index");
        if (ts == K) break;
        pass = why == 1;
        HIPC(launch_pms_restore(st, d, f.tree_start[ts], pass ? (int)N : f.tree_start[ts + 1]));
        HIPC(hipMemcpyAsync(S.off.p, P<int32_t>(S.result) + 2, 8, hipMemcpyDeviceToDevice, st));
        PmsDev dk = d;
        dk.hi_bak = pass ? 0 : 1;  // later trees keep their (modified) labels: sample the starting ones
        CHECK(pms_serial_range(ctx, st, v, dk, ts, ts + 1));
        run.serial_trees += 1;
        t_lo = ts + 1;
    }
    return SM_OK;
}

// The schedule forest of view v on the GPU (sm_pms_forest.hip), from the segmentation's device masks, on
// stream st: the outputs go straight into the PmsState buffers the kernels read; the host keeps the
// per-tree and per-round tables (K, tree_start, nb_start, rounds, cuts, repair items, round lists).
sm_status pms_forest_gpu(sm_ctx* ctx, int v, hipStream_t st, int piece) {
    PmsState& S = ctx->pms[v];
    PfBufs& B = S.pf;
    PmsForest& f = S.f;
    const int W = ctx->W, H = ctx->H, N = W * H;
    const size_t n1 = (size_t)N + 1;
    PfView pv{};
    pv.W = W;
    pv.H = H;
    pv.N = N;
    pv.mR = P<uint8_t>(ctx->mR[v]);
    pv.mD = P<uint8_t>(ctx->mD[v]);
    pv.fwR = P<uint16_t>(ctx->fwR[v]);
    pv.fwD = P<uint16_t>(ctx->fwD[v]);
    pv.wR = P<uint16_t>(ctx->wR[v]);
    pv.wD = P<uint16_t>(ctx->wD[v]);
    pv.piece = piece;
    struct A {
        DevBuf* b;
        size_t bytes;
        void** out;
    };
    const A bufs[] = {
        {&B.par, n1 * 4, (void**)&pv.par}, {&B.flag, n1 * 4, (void**)&pv.flag}, {&B.tree_of, n1 * 4, (void**)&pv.tree_of},
        {&B.nbr, n1 * 16, (void**)&pv.nbr}, {&B.nbw, n1 * 8, (void**)&pv.nbw}, {&B.root_pix, n1 * 4, (void**)&pv.root_pix},
        {&B.tsize, n1 * 4, (void**)&pv.tsize}, {&B.gpix, n1 * 4, (void**)&pv.gpix}, {&B.gpar, n1 * 4, (void**)&pv.gpar},
        {&B.gtree, n1 * 4, (void**)&pv.gtree}, {&B.gw, n1 * 2, (void**)&pv.gw}, {&B.gfc, n1 * 4, (void**)&pv.gfc},
        {&B.gnc, n1, (void**)&pv.gnc}, {&B.gsize, n1 * 4, (void**)&pv.gsize}, {&B.ghk, n1, (void**)&pv.ghk},
        {&B.iota, n1 * 4, (void**)&pv.iota}, {&B.rot, n1 * 4, (void**)&pv.rot}, {&B.pdir, n1, (void**)&pv.pdir},
        {&B.psize, n1 * 4, (void**)&pv.psize}, {&B.bpos, n1 * 4, (void**)&pv.bpos}, {&B.a_dist, 4 * n1 * 2, (void**)&pv.a_dist},
        {&B.a_cid, 4 * n1 * 4, (void**)&pv.a_cid},
        {&B.nchains, 16, (void**)&pv.nchains}, {&B.tval, 2 * n1 * 8, (void**)&pv.tval}, {&B.tval_s, 2 * n1 * 8, (void**)&pv.tval_s},
        {&B.tkey0, n1 * 8, (void**)&pv.tkey[0]}, {&B.tkey1, n1 * 8, (void**)&pv.tkey[1]}, {&B.tpix0, n1 * 4, (void**)&pv.tpix[0]},
        {&B.tpix1, n1 * 4, (void**)&pv.tpix[1]},
        {&B.bglob, n1 * 4, (void**)&pv.bglob}, {&B.gtree_s, n1 * 4, (void**)&pv.gtree_s}, {&B.g2b, n1 * 4, (void**)&pv.g2b},
        {&B.bpar, n1 * 4, (void**)&pv.bpar}, {&B.bch0, n1 * 4, (void**)&pv.bch0}, {&B.J0, n1 * 4, (void**)&pv.J[0]},
        {&B.J1, n1 * 4, (void**)&pv.J[1]}, {&B.D0, n1 * 4, (void**)&pv.Dj[0]}, {&B.D1, n1 * 4, (void**)&pv.Dj[1]},
        {&B.plen, n1 * 4, (void**)&pv.plen}, {&B.ld, n1 * 4, (void**)&pv.ld}, {&B.rowof, n1 * 4, (void**)&pv.rowof},
        {&B.rowstart, n1 * 4, (void**)&pv.rowstart}, {&B.hflag, n1 * 4, (void**)&pv.hflag}, {&B.hidx, n1 * 4, (void**)&pv.hidx},
        {&B.hkey0, n1 * 8, (void**)&pv.hkey[0]}, {&B.hkey1, n1 * 8, (void**)&pv.hkey[1]}, {&B.cutof, n1 * 4, (void**)&pv.cutof},
        {&B.hcnt[0], n1 * 4, (void**)&pv.hcnt[0]}, {&B.hcnt[1], n1 * 4, (void**)&pv.hcnt[1]},
        {&B.hcnt[2], n1 * 4, (void**)&pv.hcnt[2]}, {&B.hcnt[3], n1 * 4, (void**)&pv.hcnt[3]},
        {&B.hoff[0], n1 * 4, (void**)&pv.hoff[0]}, {&B.hoff[1], n1 * 4, (void**)&pv.hoff[1]},
        {&B.hoff[2], n1 * 4, (void**)&pv.hoff[2]}, {&B.hoff[3], n1 * 4, (void**)&pv.hoff[3]},
        {&B.pairs0, 4 * n1 * 8, (void**)&pv.pairs[0]}, {&B.pairs1, 4 * n1 * 8, (void**)&pv.pairs[1]},
        {&B.npairs, 16, (void**)&pv.npairs}, {&B.uflag, 4 * n1 * 4, (void**)&pv.uflag}, {&B.uidx, 4 * n1 * 4, (void**)&pv.uidx},
        {&B.nbcnt, n1 * 4, (void**)&pv.nbcnt}, {&B.cut_round, n1 * 4, (void**)&pv.cut_round},
        {&B.tree_cut, n1 * 4, (void**)&pv.tree_cut}, {&B.tot, 64, (void**)&pv.tot},
        // outputs the PMS kernels read (K <= N, rows = N)
        {&S.rows, (size_t)N * sizeof(PmsRow), (void**)&pv.rows}, {&S.rtree, (size_t)N * 4, (void**)&pv.rtree},
        {&S.bfs_pix, (size_t)N * 4, (void**)&pv.bfs_pix}, {&S.nb_start, n1 * 4, (void**)&pv.nb_start},
        {&S.nb, 4 * n1 * 4, (void**)&pv.nb}, {&S.tree_start, n1 * 4, (void**)&pv.tree_start},
        {&S.tree_rounds, n1 * 4, (void**)&pv.tree_rounds}, {&S.cuts, n1 * sizeof(PmsCut), (void**)&pv.cuts},
    };
    for (const A& a : bufs) {
        CHECK(ensure(ctx, *a.b, a.bytes));
        *a.out = a.b->p;
    }
    pv.temp_bytes = pf_temp_bytes(N);
    CHECK(ensure(ctx, B.temp, pv.temp_bytes));
    pv.temp = B.temp.p;
    int K = 0;
    HIPC(pf_trees(st, pv, &K));
    // the BFS tours' chains (sm_tour.h): their count depends on K
    const size_t mch = pf_max_chains(W, H, K);
    CHECK(ensure(ctx, B.c_last, mch * 4));
    CHECK(ensure(ctx, B.c_len, mch * 4));
    CHECK(ensure(ctx, B.cnw, mch * 8));
    pv.c_last = P<uint32_t>(B.c_last);
    pv.c_len = P<uint32_t>(B.c_len);
    pv.cnw = P<uint64_t>(B.cnw);
    pv.max_chains = (uint32_t)mch;
    int rb[3];
    HIPC(pf_bfs(st, pv, K, rb));
    if (rb[2]) return fail(ctx, SM_ERR_STATE, rb[2] == 1   ? "MST_PMS: the segment forest's masks contain a cycle"
                                              : rb[2] == 4 ? "MST_PMS GPU forest: inconsistent tree tour"
                                                           : "MST_PMS GPU forest: unresolved light depths");
    const int R = rb[0], nh = rb[1];
    const size_t T = (size_t)R * (K + 1) + 1;
    // round tables: rt_path and rt_item are kernel inputs (PmsDev), built in place; rt_rep and rt_long are
    // read on the host only
    DevBuf* rtb[4] = {&S.rt_path, &S.rt_item, &B.rt[2], &B.rt[3]};
    for (int q = 0; q < 4; ++q) {
        CHECK(ensure(ctx, B.rtc[q], T * 4));
        CHECK(ensure(ctx, *rtb[q], T * 4));
        pv.rtc[q] = P<int32_t>(B.rtc[q]);
        pv.rt[q] = P<int32_t>(*rtb[q]);
    }
    int cnt[7];
    HIPC(pf_lists(st, pv, K, R, nh, cnt));
    if (cnt[6]) return fail(ctx, SM_ERR_STATE, "MST_PMS GPU forest: rows out of range");
    CHECK(ensure(ctx, S.paths, (size_t)std::max(cnt[0], 1) * sizeof(PmsPath)));
    CHECK(ensure(ctx, S.items, (size_t)std::max(cnt[1], 1) * sizeof(PmsItem)));
    CHECK(ensure(ctx, S.reps, (size_t)std::max(cnt[2], 1) * sizeof(PmsRep)));
    pv.paths = P<PmsPath>(S.paths);
    pv.items = P<PmsItem>(S.items);
    pv.reps = P<PmsRep>(S.reps);
    HIPC(pf_fill(st, pv, nh));
    // the host's tables
    f.W = W;
    f.H = H;
    f.K = K;
    f.nrounds = R;
    f.piece = piece > 0 ? piece : 0;
    f.npaths = cnt[0];
    f.nitems = cnt[1];
    f.on_device = true;
    f.tree_start.resize(K + 1);
    f.nb_start.resize(K + 1);
    f.tree_rounds.resize(K);
    f.tree_cut.resize(K + 1);
    f.cuts.resize(cnt[4]);
    f.cut_round.resize(cnt[4]);
    f.reps.resize(cnt[2]);
    std::vector<int32_t>* rts[4] = {&f.rt_path, &f.rt_item, &f.rt_rep, &f.rt_long};
    for (int q = 0; q < 4; ++q) {
        rts[q]->resize((size_t)R * (K + 1));
        HIPC(hipMemcpyAsync(rts[q]->data(), rtb[q]->p, (size_t)R * (K + 1) * 4, hipMemcpyDeviceToHost, st));
    }
    HIPC(hipMemcpyAsync(f.tree_start.data(), S.tree_start.p, (K + 1) * 4, hipMemcpyDeviceToHost, st));
    HIPC(hipMemcpyAsync(f.nb_start.data(), S.nb_start.p, (K + 1) * 4, hipMemcpyDeviceToHost, st));
    HIPC(hipMemcpyAsync(f.tree_rounds.data(), S.tree_rounds.p, K * 4, hipMemcpyDeviceToHost, st));
    HIPC(hipMemcpyAsync(f.tree_cut.data(), B.tree_cut.p, (K + 1) * 4, hipMemcpyDeviceToHost, st));
    if (cnt[4]) {
        HIPC(hipMemcpyAsync(f.cuts.data(), S.cuts.p, cnt[4] * sizeof(PmsCut), hipMemcpyDeviceToHost, st));
        HIPC(hipMemcpyAsync(f.cut_round.data(), B.cut_round.p, cnt[4] * 4, hipMemcpyDeviceToHost, st));
    }
    if (cnt[2]) HIPC(hipMemcpyAsync(f.reps.data(), S.reps.p, cnt[2] * sizeof(PmsRep), hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    f.rows.clear();
    f.paths.clear();
    f.items.clear();
    f.bfs_pix.clear();
    f.nb.clear();
    return SM_OK;
}

// SM_PMS_FOREST_CHECK=1 (tests): the GPU forest of view v against the host construction, array by array
sm_status pms_forest_check(sm_ctx* ctx, int v, hipStream_t st, const PmsForest& h) {
    const PmsState& S = ctx->pms[v];
    const PmsForest& g = S.f;
    auto bad = [&](const char* what) { return fail(ctx, SM_ERR_STATE, std::string("MST_PMS GPU forest differs from the host build: ") + what); };
    if (g.K != h.K || g.nrounds != h.nrounds || g.npaths != h.npaths || g.nitems != h.nitems) return bad("sizes");
    if (g.tree_start != h.tree_start) return bad("tree_start");
    if (g.nb_start != h.nb_start) return bad("nb_start");
    if (g.tree_rounds != h.tree_rounds) return bad("tree_rounds");
    if (g.tree_cut != h.tree_cut || g.cut_round != h.cut_round) return bad("tree_cut / cut_round");
    if (g.rt_path != h.rt_path || g.rt_item != h.rt_item || g.rt_rep != h.rt_rep || g.rt_long != h.rt_long) return bad("round lists");
    if (g.cuts.size() != h.cuts.size() || (g.cuts.size() && memcmp(g.cuts.data(), h.cuts.data(), g.cuts.size() * sizeof(PmsCut))))
        return bad("cuts");
    if (g.reps.size() != h.reps.size() || (g.reps.size() && memcmp(g.reps.data(), h.reps.data(), g.reps.size() * sizeof(PmsRep))))
        return bad("reps");
    const size_t N = (size_t)g.W * g.H;
    std::vector<PmsRow> rows(N);
    std::vector<PmsPath> paths(g.npaths);
    std::vector<PmsItem> items(g.nitems);
    std::vector<int32_t> pix(N), nb(h.nb.size()), rtree(N);
    HIPC(hipMemcpyAsync(rows.data(), S.rows.p, N * sizeof(PmsRow), hipMemcpyDeviceToHost, st));
    if (g.npaths) HIPC(hipMemcpyAsync(paths.data(), S.paths.p, paths.size() * sizeof(PmsPath), hipMemcpyDeviceToHost, st));
    if (g.nitems) HIPC(hipMemcpyAsync(items.data(), S.items.p, items.size() * sizeof(PmsItem), hipMemcpyDeviceToHost, st));
    HIPC(hipMemcpyAsync(pix.data(), S.bfs_pix.p, N * 4, hipMemcpyDeviceToHost, st));
    if (!nb.empty()) HIPC(hipMemcpyAsync(nb.data(), S.nb.p, nb.size() * 4, hipMemcpyDeviceToHost, st));
    HIPC(hipMemcpyAsync(rtree.data(), S.rtree.p, N * 4, hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    if (pix != h.bfs_pix) return bad("bfs_pix");
    if (nb != h.nb) return bad("nb");
    if (memcmp(rows.data(), h.rows.data(), N * sizeof(PmsRow))) return bad("rows");
    if (paths.size() != h.paths.size() || (paths.size() && memcmp(paths.data(), h.paths.data(), paths.size() * sizeof(PmsPath))))
        return bad("paths");
    if (items.size() != h.items.size() || (items.size() && memcmp(items.data(), h.items.data(), items.size() * sizeof(PmsItem))))
        return bad("items");
    for (int t = 0; t < h.K; ++t)
        for (int r = h.tree_start[t]; r < h.tree_start[t + 1]; ++r)
            if (rtree[r] != t) return bad("rtree");
    return SM_OK;
}

// SM_AGG_PMS: Stereo3DMST's stereo3dmst() after its cost volume (Stereo3DMST.cpp:805-904) -- segment
// forests, random plane labels, pms_iters MST_PMS calls on the left view, then on the right, plane
// disparities.  Runs to completion (host synchronisations between speculative passes).
// Joins a thread on every way out of a scope: destroying a joinable std::thread calls std::terminate,
// so an early return (HIPC, CHECK) or an exception between its start and its join would kill the host
// process instead of returning an error.
struct Joiner {
    std::thread& t;
    ~Joiner() {
        if (t.joinable()) t.join();
    }
};

sm_status stage_pms(sm_ctx* ctx, int D, const sm_params* p) {
    const int W = ctx->W, H = ctx->H;
    const size_t N = (size_t)W * H;
    const int iters = p->pms_iters;
    const int L = sm_pms_levels(D);
    sm_pms_stats& st = ctx->pms_stats;
    st = sm_pms_stats{};
    st.iters = iters;
    const double t0 = now_ms();
    // the rand() stream's skip over random_rgb's 3 draws per pixel of both views does not depend on the
    // forests: it runs on a thread of its own from the start (the calls' values are drawn after step 2)
    GlibcRandom grnd;
    std::thread skip([&grnd, N] { grnd.seed_skip(1u, (long)(6 * N)); });
    Joiner jskip{skip};  // joined on every way out (early returns, exceptions)
    // 1. the forests: the reference's order-dependent segmentation (c = +inf: the MST)
    // the schedule forests are built on the GPU (sm_pms_forest.hip) from the device masks;
    // SM_PMS_HOST_FOREST=1: on host threads (pms_build_forest, A/B); SM_PMS_FOREST_CHECK=1 (tests): both,
    // compared array by array
    const bool host_forest = sm_knob("SM_PMS_HOST_FOREST") && atoi(sm_knob("SM_PMS_HOST_FOREST")) == 1;
    const bool forest_check = sm_knob("SM_PMS_FOREST_CHECK") && atoi(sm_knob("SM_PMS_FOREST_CHECK")) == 1;
    const sm_status seg_st = stage_segment(ctx, 3, p->c, p->min_size, host_forest || forest_check);
    if (seg_st != SM_OK) {
        skip.join();
        return seg_st;
    }
    st.prep_seg_ms = now_ms() - t0;
    // 2. reference-numbered forests and walk schedules, both views in parallel (view 1 on st_pms)
    if (!ctx->st_pms) {
        if (hipStreamCreateWithFlags(&ctx->st_pms, hipStreamNonBlocking) != hipSuccess) {
            skip.join();
            return fail(ctx, SM_ERR_HIP, "hipStreamCreateWithFlags (MST_PMS view stream)");
        }
    }
    {
        auto host_build = [ctx, W, H, N](int v, PmsForest& f) {
            std::vector<uint8_t> mR(N), mD(N);
            for (size_t i = 0; i < N; ++i) {
                mR[i] = ctx->h_m[v][0][i] && ctx->h_fw[v][0][i] != SM_VIRTUAL_W;
                mD[i] = ctx->h_m[v][1][i] && ctx->h_fw[v][1][i] != SM_VIRTUAL_W;
            }
            pms_build_forest(W, H, ctx->h_w[v][0].data(), ctx->h_w[v][1].data(), mR.data(), mD.data(), f, pms_piece());
        };
        sm_status fs[2] = {SM_OK, SM_OK};
        auto build = [&](int v) {
            const hipStream_t sv = v == 0 ? ctx->st : ctx->st_pms;
            if (host_forest) {
                host_build(v, ctx->pms[v].f);
                return;
            }
            if (hipSetDevice(ctx->device) != hipSuccess) {
                fs[v] = SM_ERR_HIP;
                return;
            }
            fs[v] = pms_forest_gpu(ctx, v, sv, pms_piece());
            if (fs[v] == SM_OK && forest_check) {
                PmsForest h;
                host_build(v, h);
                fs[v] = pms_forest_check(ctx, v, sv, h);
            }
        };
        const double tf = now_ms();
        HIPC(hipEventRecord(ctx->ev_pms, ctx->st));
        HIPC(hipStreamWaitEvent(ctx->st_pms, ctx->ev_pms, 0));  // the segmentation's masks
        auto guarded = [&](int v) {
            try {
                build(v);
            } catch (const std::bad_alloc&) {
                fs[v] = SM_ERR_OOM;
            } catch (...) {
                fs[v] = SM_ERR_STATE;
            }
        };
        std::thread other([&] { guarded(1); });
        Joiner jother{other};
        guarded(0);
        other.join();
        st.prep_forest_ms = now_ms() - tf;
        if (fs[0] != SM_OK || fs[1] != SM_OK) {
            skip.join();
            return fs[0] != SM_OK ? fs[0] : fs[1];
        }
    }
    // 3. random streams: the replayed dice prefix, the rand() values of every call (after random_rgb's
    // 3 draws per pixel of both views), the initial labels (one stream, so both views start equal)
    const int K0 = ctx->pms[0].f.K, K1 = ctx->pms[1].f.K;
    ctx->pms_hrnd.resize((size_t)iters * (K0 + K1) + 1);
    skip.join();
    std::thread rng([ctx, iters, K0, K1, &grnd] { grnd.draw((long)iters * (K0 + K1), ctx->pms_hrnd.data()); });
    Joiner jrng{rng};
    if (ctx->pms_init_key[0] != W || ctx->pms_init_key[1] != H || ctx->pms_init_key[2] != D) {
        ctx->pms_init.resize(3 * N);
        sm_pms_init_labels(W, H, D, ctx->pms_init.data());
        ctx->pms_init_key[0] = W;
        ctx->pms_init_key[1] = H;
        ctx->pms_init_key[2] = D;
    }
    if (ctx->pms_dblmax.size() != N) ctx->pms_dblmax.assign(N, DBL_MAX);
    rng.join();
    const double t1 = now_ms();
    st.prep_ms = t1 - t0;
    st.ntrees[0] = K0;
    st.ntrees[1] = K1;
    for (int v = 0; v < 2; ++v) CHECK(pms_upload_view(ctx, v, L));
    const long long need = std::max(ctx->pms[0].dice_need, ctx->pms[1].dice_need);
    if (need > ctx->pms_dice_n) {
        std::vector<float> dice((size_t)need);
        sm_pms_dice((long)need, dice.data());
        CHECK(ensure(ctx, ctx->pms_dice, (size_t)need * 4));
        HIPC(hipMemcpy(ctx->pms_dice.p, dice.data(), (size_t)need * 4, hipMemcpyHostToDevice));
        ctx->pms_dice_n = need;
    }
    CHECK(upload_vec(ctx, ctx->pms_rnd, ctx->pms_hrnd));
    // 4. cost rows [N][D]: the AGD volume, or the uploaded MC-CNN volumes with the reference's clamp
    for (int v = 0; v < 2; ++v) CHECK(ensure(ctx, ctx->pms[v].vrows, N * (size_t)D * 4));
    if (ctx->use_vol) {
        for (int v = 0; v < 2; ++v)
            HIPC(launch_pms_vol_rows(ctx->st, P<float>(ctx->vin[v]), N, D, D, 1, P<float>(ctx->pms[v].vrows)));
    } else {
        for (int v = 0; v < 2; ++v) CHECK(ensure(ctx, ctx->vol[v], N * (size_t)D * 4));
        HIPC(launch_cost_volume(ctx->st, P<uint32_t>(ctx->bgrx[0]), P<float>(ctx->gray[0]), P<uint32_t>(ctx->bgrx[1]),
                                P<float>(ctx->gray[1]), P<float>(ctx->atab), W, H, 0, D, P<float>(ctx->vol[0]),
                                P<float>(ctx->vol[1])));
        for (int v = 0; v < 2; ++v)
            HIPC(launch_pms_vol_rows(ctx->st, P<float>(ctx->vol[v]), N, D, D, 0, P<float>(ctx->pms[v].vrows)));
    }
    for (int v = 0; v < 2; ++v) {
        HIPC(hipMemcpyAsync(ctx->pms[v].abc.p, ctx->pms_init.data(), N * 12, hipMemcpyHostToDevice, ctx->st));
        HIPC(hipMemcpyAsync(ctx->pms[v].minc.p, ctx->pms_dblmax.data(), N * 8, hipMemcpyHostToDevice, ctx->st));
    }
    HIPC(hipStreamSynchronize(ctx->st));
    const double t2 = now_ms();
    st.setup_ms = t2 - t1;
    // 5. the MST_PMS calls: left view, then right (:858-889).  The two views share nothing but read-only
    // tables (each view's rand() values sit at fixed offsets of the precomputed stream, the dice prefix is
    // replayed), so each view's calls run on a host thread and stream of their own, concurrently (round
    // 4: one after the other took 0.81 -> 0.67 s per 100-call frame).  Every call is timed; the node-label
    // evaluations each call needed are counted on the device (k_pms_count).
    const bool serial_only = pms_serial_only();
    CHECK(ensure(ctx, ctx->pms_evals, 16 * 8));
    HIPC(hipMemsetAsync(ctx->pms_evals.p, 0, 16 * 8, ctx->st));
    HIPC(hipEventRecord(ctx->ev_pms, ctx->st));
    HIPC(hipStreamWaitEvent(ctx->st_pms, ctx->ev_pms, 0));  // view 1's stream after the set-up above
    PmsRun run[2];
    run[0].st = ctx->st;
    run[1].st = ctx->st_pms;
    run[0].h_res = ctx->h_pms_res;
    run[1].h_res = ctx->h_pms_res + 4;
    const size_t roff0[2] = {0, (size_t)iters * K0};
    // evaluations the device ran (speculation and repeats included): a diagnostic, SM_PMS_COUNT_RUN=1
    const bool count_run = sm_knob("SM_PMS_COUNT_RUN") && atoi(sm_knob("SM_PMS_COUNT_RUN")) == 1;
    auto calls = [ctx, D, iters, serial_only, count_run, &roff0](PmsRun& r, int v) -> sm_status {
        HIPC(hipSetDevice(ctx->device));
        const hipStream_t st = r.st;
        PmsDev d = pms_dev(ctx, v, D);
        // per view: [needed, reference's count] of the first call, of the later calls; evaluations run
        // (speculation and repeats included) of the first call, of the later calls
        unsigned long long* acc = P<unsigned long long>(ctx->pms_evals) + 8 * v;
        const int K = d.K;
        size_t roff = roff0[v];
        for (int i = 0; i < iters; ++i) {
            const double a = now_ms();
            d.rnd = P<int32_t>(ctx->pms_rnd) + roff;
            d.evals = count_run ? acc + (i == 0 ? 4 : 5) : nullptr;
            roff += (size_t)K;
            if (d.prof) HIPC(hipMemsetAsync(d.prof, 0, 16 * 8, st));
            if (i == 0 || serial_only) {
                HIPC(hipMemsetAsync(ctx->pms[v].off.p, 0, 16, st));
                const bool tree_times = sm_knob("SM_PMS_TREE_TIMES") != nullptr;  // diagnostics (tools)
                if (tree_times && i == 0) {
                    std::vector<hipEvent_t> ev(K + 1);
                    for (auto& e : ev) HIPC(hipEventCreate(&e));
                    HIPC(hipEventRecord(ev[0], st));
                    for (int t = 0; t < K; ++t) {
                        CHECK(pms_serial_range(ctx, st, v, d, t, t + 1));
                        HIPC(hipEventRecord(ev[t + 1], st));
                    }
                    HIPC(hipStreamSynchronize(st));
                    const PmsForest& f = ctx->pms[v].f;
                    for (int t = 0; t < K; ++t) {
                        float ms = 0;
                        HIPC(hipEventElapsedTime(&ms, ev[t], ev[t + 1]));
                        fprintf(stderr, "pms tree v%d t%d n %d deg %d rounds %d ms %.3f\n", v, t,
                                f.tree_start[t + 1] - f.tree_start[t], f.nb_start[t + 1] - f.nb_start[t], f.tree_rounds[t], ms);
                    }
                    for (auto& e : ev) HIPC(hipEventDestroy(e));
                } else {
                    CHECK(pms_serial_range(ctx, st, v, d, 0, K));
                }
                r.serial_trees += K;
            } else {
                CHECK(pms_speculative_call(ctx, r, v, d));
            }
            {  // the call's node-label evaluations (a speculative call with the dedupe: nprop holds the counts)
                PmsDev dc = d;
                dc.nprop = (i > 0 && !serial_only) ? P<int32_t>(ctx->pms[v].nprop) : nullptr;
                HIPC(launch_pms_count(st, dc, acc + (i == 0 ? 0 : 2)));
            }
            HIPC(hipStreamSynchronize(st));
            const uint32_t e = __atomic_load_n(ctx->h_err + 1 + v, __ATOMIC_ACQUIRE);  // this view's word
            if (e) {
                __atomic_store_n(ctx->h_err + 1 + v, 0u, __ATOMIC_RELEASE);
                return fail(ctx, SM_ERR_STATE, (e & 4u) ? "MST_PMS: dice stream exhausted (internal sizing error)"
                                                        : "MST_PMS: a propagation index fell outside its tree (the "
                                                          "reference would read outside mst_vertices_vec)");
            }
            (i == 0 ? r.first_ms : r.later_ms) += now_ms() - a;
            if (d.prof) {
                long long h[16];
                HIPC(hipMemcpy(h, d.prof, 16 * 8, hipMemcpyDeviceToHost));
                fprintf(stderr, "pms prof v%d call %d (ms): prop setup %.2f up %.2f down %.2f update %.2f | ref setup %.2f up %.2f "
                        "down %.2f update %.2f | rounds %lld | guess staging %.3f chain %.3f | up chain items %lld: longest %.1f us "
                        "(%lld rows), mean %.1f us, mean %.0f rows\n", v, i, h[0] * 1e-5, h[1] * 1e-5,
                        h[2] * 1e-5, h[3] * 1e-5, h[4] * 1e-5, h[5] * 1e-5, h[6] * 1e-5, h[7] * 1e-5, h[8], h[9] * 1e-5, h[10] * 1e-5,
                        h[14], (double)(h[11] >> 24) * 1e-2, h[11] & 0xFFFFFF, h[14] ? h[12] * 1e-2 / h[14] : 0.0,
                        h[14] ? (double)h[13] / h[14] : 0.0);
            }
        }
        return SM_OK;
    };
    const double tc0 = now_ms();
    sm_status rs[2] = {SM_OK, SM_OK};
    {
        auto guarded = [&](int v) {
            try {
                rs[v] = calls(run[v], v);
            } catch (const std::bad_alloc&) {
                rs[v] = SM_ERR_OOM;
            } catch (...) {
                rs[v] = SM_ERR_STATE;
            }
        };
        std::thread other([&] { guarded(1); });
        Joiner jother{other};
        guarded(0);
        other.join();
    }
    const double tc1 = now_ms();
    CHECK(rs[0]);
    CHECK(rs[1]);
    // outputs: the plane disparity, the per-pixel aggregated minimum, idx = -1
    for (int v = 0; v < 2; ++v) {
        CHECK(ensure(ctx, ctx->disp[v], N * 4));
        CHECK(ensure(ctx, ctx->minc[v], N * 8));
        CHECK(ensure(ctx, ctx->idx[v], N * 4));
        HIPC(launch_pms_disp(ctx->st, P<float>(ctx->pms[v].abc), W, N, P<float>(ctx->disp[v])));
        HIPC(hipMemcpyAsync(ctx->minc[v].p, ctx->pms[v].minc.p, N * 8, hipMemcpyDeviceToDevice, ctx->st));
        HIPC(hipMemsetAsync(ctx->idx[v].p, 0xFF, N * 4, ctx->st));
    }
    unsigned long long ev[16];
    HIPC(hipMemcpyAsync(ev, ctx->pms_evals.p, sizeof(ev), hipMemcpyDeviceToHost, ctx->st));
    HIPC(hipStreamSynchronize(ctx->st));
    // wall clock of the calls: the first calls of the views (the longer one), then the rest
    const double iter0 = std::max(run[0].first_ms, run[1].first_ms);
    const double rest = (tc1 - tc0) - iter0;
    st.spec_rounds = run[0].spec_rounds + run[1].spec_rounds;
    st.serial_trees = run[0].serial_trees + run[1].serial_trees;
    st.calls_ms = tc1 - tc0;
    st.concurrent_views = 1;
    for (int v = 0; v < 2; ++v) {
        st.first_ms_view[v] = run[v].first_ms;
        st.later_ms_view[v] = run[v].later_ms;
    }
    st.evals_first = (double)(ev[0] + ev[8]);
    st.evals_first_ref = (double)(ev[1] + ev[9]);
    st.evals_later = (double)(ev[2] + ev[10]);
    st.evals_later_ref = (double)(ev[3] + ev[11]);
    st.evals_first_run = (double)(ev[4] + ev[12]);
    st.evals_later_run = (double)(ev[5] + ev[13]);
    st.iter0_ms = iter0;
    st.iters_ms = rest;
    st.total_ms = now_ms() - t0;
    ctx->pms_last = true;
    ctx->pms_W = W;
    ctx->pms_H = H;
    return SM_OK;
}

// the tree layout packs preorder positions in 27 bits (sm_layout_gpu.hip): every tree-based call
// (MST, segment forest, MST_PMS) refuses images of 2^27 pixels or more with its other argument checks,
// before anything is uploaded or allocated (stage_layout_enqueue keeps its own check as a backstop)
sm_status check_tree_size(sm_ctx* ctx, long long W, long long H, const sm_params* p) {
    if (p && p->aggregator == SM_AGG_GUIDED) return SM_OK;
    if (W > 0 && H > 0 && W * H >= (1ll << 27))
        return fail(ctx, SM_ERR_ARG, "images of 2^27 pixels or more are not supported by the tree layout");
    return SM_OK;
}

sm_status upload(sm_ctx* ctx, const uint8_t* l, const uint8_t* r, int W, int H, int stride) {
    if (!l || !r) return fail(ctx, SM_ERR_ARG, "null image");
    if (W < 1 || H < 1 || stride < 3 * W) return fail(ctx, SM_ERR_ARG, "bad image geometry");
    if ((long long)W * H > (1ll << 30)) return fail(ctx, SM_ERR_ARG, "image too large");
    ctx->W = W;
    ctx->H = H;
    ctx->stride = stride;
    const size_t bytes = (size_t)H * stride;
    for (int v = 0; v < 2; ++v) CHECK(ensure(ctx, ctx->img[v], bytes));
    HIPC(hipMemcpyAsync(ctx->img[0].p, l, bytes, hipMemcpyHostToDevice, ctx->st));
    HIPC(hipMemcpyAsync(ctx->img[1].p, r, bytes, hipMemcpyHostToDevice, ctx->st));
    return SM_OK;
}

// Host check of one view's tree metadata (knob SM_LAYOUT_CHECK, tests): every light children's parent
// holds a distinct compact A row below n_has_light in cslot[3], every path head's parent word is
// SM_HEAD | its parent's row, every other node's the previous slot (or SM_NONE at the root)
sm_status layout_check(sm_ctx* ctx, int v, size_t N) {
    std::vector<SmMeta> m(N);
    HIPC(hipMemcpy(m.data(), ctx->meta[v].p, N * sizeof(SmMeta), hipMemcpyDeviceToHost));
    const uint32_t nl = ctx->layout[v].n_has_light;
    std::vector<uint8_t> seen(nl + 1, 0);
    size_t nlight = 0, nroot = 0;
    char msg[160];
    for (size_t s = 0; s < N; ++s) {
        const SmMeta& x = m[s];
        if (sm_meta_has_light(x)) {
            ++nlight;
            const uint32_t r = x.cslot[3];
            if (r >= nl || seen[r]) {
                snprintf(msg, sizeof msg, "layout check: slot %zu compact row %u (n_has_light %u)%s", s, r, nl, r < nl ? " twice" : "");
                return fail(ctx, SM_ERR_STATE, msg);
            }
            seen[r] = 1;
            if (sm_meta_nch(x) > 3) return fail(ctx, SM_ERR_STATE, "layout check: a light children's parent with 4 children");
        }
        const uint32_t w = x.parent;
        if (w == SM_NONE) {
            ++nroot;
        } else if (w != (uint32_t)s - 1u) {
            if (!(w & SM_HEAD) || sm_arow(w) >= nl) {
                snprintf(msg, sizeof msg, "layout check: slot %zu parent word %08x (n_has_light %u)", s, w, nl);
                return fail(ctx, SM_ERR_STATE, msg);
            }
        }
    }
    if (nlight != nl || nroot != 1) {
        snprintf(msg, sizeof msg, "layout check: %zu light parents against n_has_light %u, %zu roots", nlight, nl, nroot);
        return fail(ctx, SM_ERR_STATE, msg);
    }
    return SM_OK;
}

// the chain engine's error word (written by the device through the host mapping): reported once,
// then cleared so the context stays usable
sm_status check_device_error(sm_ctx* ctx) {
    // (bit 1 is the tree layout's, checked by stage_layout_finish: a later frame's may be in flight)
    const uint32_t e = __atomic_fetch_and(ctx->h_err, 2u, __ATOMIC_ACQ_REL) & ~2u;
    if (!e) return SM_OK;
    return fail(ctx, SM_ERR_STATE,
                "long-path chain engine: a cross-workgroup wait timed out (piece status word never published); "
                "the results of this call are invalid");
}

double now_ms() {
    struct timeval t;
    gettimeofday(&t, nullptr);
    return t.tv_sec * 1000.0 + t.tv_usec / 1000.0;
}

}  // namespace

// ============================================================================ C-ABI
extern "C" {

const char* sm_version(void) { return "stereomst-mi355x 0.1 (gfx950)"; }

void sm_default_params(sm_params* p) {
    if (!p) return;
    p->gamma = 1.0f / 12.f;        // Stereo3DMST.cpp:830
    p->c = INFINITY;               // MST mode (north star); reference segment mode uses 5000 (:831)
    p->min_size = 200;             // :832
    p->median_ksize = 3;           // :214
    p->cost_kind = SM_COST_AGD;
    p->disp_begin = 0;
    p->disp_total = 0;
    p->post = 0;
    p->aggregator = SM_AGG_TREE;
    p->gf_radius = 9;                                  // PatchMatchStereoGPU.cu:9001
    p->gf_eps = (float)(std::pow(0.01, 2.0) * 255 * 255);  // :9000
    p->views = 3;                                      // both views
    p->pms_iters = 100;                                // Stereo3DMST.cpp:854
}

sm_status sm_device_count(int* count) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    if (count) *count = n;
    return n > 0 ? SM_OK : SM_ERR_NODEVICE;
}

sm_status sm_create(sm_ctx** out, const sm_config* cfg) {
    if (!out) return SM_ERR_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return SM_ERR_NODEVICE;
    sm_ctx* ctx = new sm_ctx();
    ctx->device = cfg ? cfg->device : 0;
    if (ctx->device < 0 || ctx->device >= n) { delete ctx; return SM_ERR_ARG; }
    if (hipSetDevice(ctx->device) != hipSuccess || hipStreamCreateWithFlags(&ctx->st, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return SM_ERR_HIP;
    }
    ctx->st2 = ctx->st;  // (the chain engine's stream: an alias, see sm_ctx::st2)
    if (hipHostMalloc((void**)&ctx->h_err, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer((void**)&ctx->d_err, ctx->h_err, 0) != hipSuccess) {
        delete ctx;
        return SM_ERR_HIP;
    }
    ctx->h_err[0] = 0;
    if (hipHostMalloc((void**)&ctx->h_pms_res, 32) != hipSuccess ||
        hipEventCreateWithFlags(&ctx->ev_pms, hipEventDisableTiming) != hipSuccess ||
        hipHostMalloc((void**)&ctx->h_changed, (2 * SM_MST_MAX_ROUNDS + 8) * sizeof(int)) != hipSuccess ||
        hipHostMalloc((void**)&ctx->h_rounds, 2 * RREC_FWD * sizeof(uint32_t)) != hipSuccess) {
        delete ctx;
        return SM_ERR_HIP;
    }
    for (auto& e : ctx->ev)  // stage-boundary timing events
        if (hipEventCreateWithFlags(&e, timing_event_flags()) != hipSuccess) { delete ctx; return SM_ERR_HIP; }
    if (hipEventCreateWithFlags(&ctx->ev_layout, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&ctx->ev_segw, hipEventDisableTiming) != hipSuccess) {
        delete ctx;
        return SM_ERR_HIP;
    }
    // tables: S/S2 (correctly rounded, tools/gen_tables.py) and the AGD colour term
    std::vector<float> atab(SM_MAX_W + 1);
    for (int i = 0; i <= SM_MAX_W; ++i) atab[i] = agd_color_term(i);
    if (ensure(ctx, ctx->atab, atab.size() * 4) != SM_OK || ensure(ctx, ctx->slut, 766 * 8) != SM_OK ||
        ensure(ctx, ctx->s2lut, 766 * 8) != SM_OK ||
        hipMemcpy(ctx->atab.p, atab.data(), atab.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(ctx->slut.p, SM_S_LUT, 766 * 8, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(ctx->s2lut.p, SM_S2_LUT, 766 * 8, hipMemcpyHostToDevice) != hipSuccess) {
        sm_destroy(ctx);
        return SM_ERR_HIP;
    }
    *out = ctx;
    return SM_OK;
}

void sm_destroy(sm_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->seg_worker.joinable()) ctx->seg_worker.join();  // a begun segment-mode call's host worker
    if (ctx->st) (void)hipStreamSynchronize(ctx->st);
    if (ctx->st2 && ctx->st2 != ctx->st) (void)hipStreamSynchronize(ctx->st2);
    if (ctx->comm) ncclCommDestroy(ctx->comm);
    DevBuf* all[] = {&ctx->changed, &ctx->mst_ok, &ctx->atab, &ctx->slut, &ctx->s2lut, &ctx->post_mask, &ctx->post_scratch,
                     &ctx->gf_planes, &ctx->gf_means, &ctx->gf_pl, &ctx->gf_tmp, &ctx->gf_stats[0], &ctx->gf_stats[1],
                     &ctx->gf_state[0], &ctx->gf_state[1]};
    for (DevBuf* b : all) if (b->p) (void)hipFree(b->p);
    for (int v = 0; v < 2; ++v) {
        DevBuf* per[] = {&ctx->img[v], &ctx->bgrx[v], &ctx->gray[v], &ctx->med[v], &ctx->wR[v], &ctx->wD[v], &ctx->comp[v],
                         &ctx->best[v], &ctx->root[v], &ctx->mR[v], &ctx->mD[v], &ctx->meta[v], &ctx->paths[v], &ctx->U[v], &ctx->Cst[v],
                         &ctx->idx[v], &ctx->minc[v], &ctx->disp[v], &ctx->cand[v], &ctx->gmin[v], &ctx->gidx[v], &ctx->vol[v], &ctx->rec[v], &ctx->rec4[v], &ctx->vin[v],
                         &ctx->cedge[v], &ctx->clab[v], &ctx->chook[v], &ctx->ccnt[v], &ctx->fwR[v], &ctx->fwD[v]};
        for (DevBuf* b : per) if (b->p) (void)hipFree(b->p);
        SegGpu& g = ctx->sg[v];
        DevBuf* sg[] = {&g.par, &g.sz, &g.wl, &g.best, &g.first, &g.ebuf, &g.bcnt, &g.list0, &g.list1, &g.rej, &g.hooked,
                        &g.cnt, &g.mlist, &g.hooks, &g.mkey, &g.mval, &g.msorted, &g.stemp};
        for (DevBuf* b : sg) if (b->p) (void)hipFree(b->p);
    }
    for (auto e : ctx->ev) if (e) (void)hipEventDestroy(e);
    if (ctx->ev_layout) (void)hipEventDestroy(ctx->ev_layout);
    if (ctx->ev_segw) (void)hipEventDestroy(ctx->ev_segw);
    for (auto e : ctx->fev) (void)hipEventDestroy(e);
    for (auto e : ctx->sev) (void)hipEventDestroy(e);
    for (int v = 0; v < 2; ++v) {
        PmsState& S = ctx->pms[v];
        DevBuf* pb[] = {&S.rows, &S.rtree, &S.paths, &S.items, &S.rt_path, &S.rt_item, &S.tree_rounds, &S.tree_start,
                        &S.bfs_pix, &S.nb_start, &S.nb, &S.tree_pt, &S.tree_abase, &S.tree_lab, &S.nref, &S.lab, &S.labq,
                        &S.abc, &S.minc, &S.abc_bak, &S.minc_bak, &S.A, &S.vrows, &S.off, &S.oguess, &S.cnt, &S.flag,
                        &S.result, &S.prof, &S.labu, &S.nprop, &S.vrows, &S.cuts, &S.reps, &S.cut_bak, &S.Abak,
                        &S.plan_cnt, &S.plan_path, &S.plan_item, &S.plan_base, &S.plan_ibase, &S.rep_flag, &S.pt_ph,
                        &S.ab_ph};
        for (DevBuf* b : pb) if (b->p) (void)hipFree(b->p);
    }
    if (ctx->pms_dice.p) (void)hipFree(ctx->pms_dice.p);
    if (ctx->pms_evals.p) (void)hipFree(ctx->pms_evals.p);
    if (ctx->st_pms) {
        (void)hipStreamSynchronize(ctx->st_pms);
        (void)hipStreamDestroy(ctx->st_pms);
    }
    if (ctx->ev_pms) (void)hipEventDestroy(ctx->ev_pms);
    for (int v = 0; v < 2; ++v) {
    }
    if (ctx->pms_rnd.p) (void)hipFree(ctx->pms_rnd.p);
    if (ctx->h_pms_res) (void)hipHostFree(ctx->h_pms_res);
    if (ctx->h_changed) (void)hipHostFree(ctx->h_changed);
    if (ctx->h_err) (void)hipHostFree(ctx->h_err);
    if (ctx->h_rounds) (void)hipHostFree(ctx->h_rounds);
    for (int v = 0; v < 2; ++v) {
        DevBuf* lay[] = {&ctx->adj[v], &ctx->pdir[v], &ctx->heavy[v], &ctx->size[v], &ctx->arcpix[v],
                         &ctx->hk[v], &ctx->pixpre[v], &ctx->a_dist[v], &ctx->a_cid[v],
                         &ctx->ccount[v], &ctx->c_last[v], &ctx->c_len[v], &ctx->cnw[v],
                         &ctx->tour[v], &ctx->spart[v],
                         &ctx->rounds[v], &ctx->segtab[v], &ctx->pathpos[v], &ctx->plen[v],
                         &ctx->slotpix[v], &ctx->pieces[v], &ctx->pieces_tmp[v], &ctx->agg[v], &ctx->pstat[v], &ctx->fix[v],
                         &ctx->acmp[v], &ctx->adbg[v], &ctx->lrank[v], &ctx->wrow[v]};
        if (v == 0 && ctx->pdbg.p) (void)hipFree(ctx->pdbg.p);
        for (DevBuf* b : lay) if (b->p) (void)hipFree(b->p);
    }
    if (ctx->st2 && ctx->st2 != ctx->st) (void)hipStreamDestroy(ctx->st2);
    if (ctx->st) (void)hipStreamDestroy(ctx->st);
    delete ctx;
}

const char* sm_last_error(const sm_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

sm_status sm_upload_images(sm_ctx* ctx, const uint8_t* l, const uint8_t* r, int W, int H, int stride) {
    if (!ctx) return SM_ERR_ARG;
    if (ctx->pending) return fail(ctx, SM_ERR_STATE, "sm_upload_images: a call begun with sm_match_begin is not finished (sm_match_finish)");
    HIPC(hipSetDevice(ctx->device));
    return upload(ctx, l, r, W, H, stride);
}

sm_status sm_upload_cost_volumes(sm_ctx* ctx, const float* left_vol, const float* right_vol, int W, int H, int D) {
    if (!ctx) return SM_ERR_ARG;
    if (ctx->pending) return fail(ctx, SM_ERR_STATE, "sm_upload_cost_volumes: a call begun with sm_match_begin is not finished (sm_match_finish)");
    if (!left_vol || !right_vol) return fail(ctx, SM_ERR_ARG, "null volume");
    if (W < 1 || H < 1 || D < 1 || (long long)W * H > (1ll << 30)) return fail(ctx, SM_ERR_ARG, "bad volume geometry");
    HIPC(hipSetDevice(ctx->device));
    const size_t bytes = (size_t)W * H * D * sizeof(float);
    for (int v = 0; v < 2; ++v) CHECK(ensure(ctx, ctx->vin[v], bytes));
    HIPC(hipMemcpyAsync(ctx->vin[0].p, left_vol, bytes, hipMemcpyHostToDevice, ctx->st));
    HIPC(hipMemcpyAsync(ctx->vin[1].p, right_vol, bytes, hipMemcpyHostToDevice, ctx->st));
    HIPC(hipStreamSynchronize(ctx->st));  // the caller may free or reuse its buffers on return
    ctx->vin_W = W;
    ctx->vin_H = H;
    ctx->vin_D = D;
    return SM_OK;
}

static sm_status match_begin_impl(sm_ctx* ctx, int D, const sm_params* p);
static sm_status match_finish_impl(sm_ctx* ctx);

// No C++ exception crosses the C-ABI: host allocations (std::vector, std::thread) that throw in a
// stage become SM_ERR_OOM / SM_ERR_STATE.
sm_status sm_match_begin(sm_ctx* ctx, int D, const sm_params* p) {
    try {
        return match_begin_impl(ctx, D, p);
    } catch (const std::bad_alloc&) {
        return ctx ? fail(ctx, SM_ERR_OOM, "sm_match_begin: host allocation failed") : SM_ERR_OOM;
    } catch (...) {
        return ctx ? fail(ctx, SM_ERR_STATE, "sm_match_begin: host exception") : SM_ERR_STATE;
    }
}

sm_status sm_match_finish(sm_ctx* ctx) {
    try {
        return match_finish_impl(ctx);
    } catch (const std::bad_alloc&) {
        return ctx ? fail(ctx, SM_ERR_OOM, "sm_match_finish: host allocation failed") : SM_ERR_OOM;
    } catch (...) {
        return ctx ? fail(ctx, SM_ERR_STATE, "sm_match_finish: host exception") : SM_ERR_STATE;
    }
}

static sm_status match_begin_impl(sm_ctx* ctx, int D, const sm_params* p) {
    if (!ctx) return SM_ERR_ARG;
    if (ctx->pending) return fail(ctx, SM_ERR_STATE, "sm_match_begin: the previous call was not finished (sm_match_finish)");
    if (ctx->seg_worker.joinable()) ctx->seg_worker.join();  // a worker left by a failed finish
    if (ctx->W == 0) return fail(ctx, SM_ERR_STATE, "no images uploaded");
    CHECK(check_params(ctx, p, D));
    CHECK(check_tree_size(ctx, ctx->W, ctx->H, p));
    const CallRange cr = call_range(p, D);
    ctx->use_vol = p->cost_kind == SM_COST_VOLUME;
    ctx->views = p->views == 0 ? 3 : p->views;
    if (ctx->use_vol) {
        if (ctx->vin_D == 0) return fail(ctx, SM_ERR_STATE, "SM_COST_VOLUME: no volumes uploaded (sm_upload_cost_volumes)");
        if (ctx->vin_W != ctx->W || ctx->vin_H != ctx->H) return fail(ctx, SM_ERR_ARG, "cost volumes and images differ in size");
        if (cr.d0 + cr.D > ctx->vin_D) return fail(ctx, SM_ERR_ARG, "slices beyond the uploaded cost volumes");
    }
    HIPC(hipSetDevice(ctx->device));
    ctx->rec_pad = rec_pad_for(cr.d0, cr.D);
    ctx->sub = cr.w.sub != 0;
#ifdef SM_DEV  // (compiled out of product builds: these skip work)
    // timing experiments only (tools): with a layout of these images from an earlier frame,
    // SM_EXP_FILTER_ONLY=1 re-filters it without re-running prep / MST / layout (the filter's streaming
    // cost alone); SM_EXP_SKIP=mst keeps the previous MST (prep + layout + filter), SM_EXP_SKIP=layout
    // keeps the previous layout (prep + MST + filter): the tree stages' streaming cost, stage by stage
    static const bool exp_filter_only = sm_dev_knob("SM_EXP_FILTER_ONLY") != nullptr;
    static const int exp_skip = sm_dev_knob("SM_EXP_SKIP") ? (strcmp(sm_dev_knob("SM_EXP_SKIP"), "mst") == 0 ? 1 : 2) : 0;
    const bool exp_on = ctx->exp_layout_ok && p->aggregator == SM_AGG_TREE && std::isinf(p->c);
    if (exp_on && exp_skip) {
        HIPC(hipEventRecord(ctx->ev[0], ctx->st));
        CHECK(stage_prep(ctx));
        HIPC(hipEventRecord(ctx->ev[1], ctx->st));
        if (exp_skip == 2) CHECK(stage_tree(ctx, ctx->views, p, false));
        HIPC(hipEventRecord(ctx->ev[2], ctx->st));
        if (exp_skip == 1) {
            ctx->mst_pend.active = false;
            CHECK(stage_layout_enqueue(ctx, ctx->views));
        } else {
            HIPC(hipEventRecord(ctx->ev_layout, ctx->st));  // (finish waits for the MST's rounds record)
        }
        ctx->pending = 1;
        ctx->pend_D = D;
        ctx->pend_p = *p;
        return SM_OK;
    }
    if (exp_filter_only && exp_on) {
        for (int i = 0; i < 3; ++i) HIPC(hipEventRecord(ctx->ev[i], ctx->st));
        ctx->pending = 3;
        ctx->pend_D = D;
        ctx->pend_p = *p;
        return SM_OK;
    }
#endif
    HIPC(hipEventRecord(ctx->ev[0], ctx->st));
    CHECK(stage_prep(ctx));
    HIPC(hipEventRecord(ctx->ev[1], ctx->st));
    ctx->pms_last = false;
    if (p->aggregator == SM_AGG_PMS) {  // runs to completion here (host waits between its passes)
        ctx->sub = false;
        ctx->nfev = ctx->nsev = 0;
        ctx->fam.clear();
        ctx->fam_vox.clear();
        ctx->fam_ev.clear();
        HIPC(hipEventRecord(ctx->ev[2], ctx->st));
        HIPC(hipEventRecord(ctx->ev[3], ctx->st));
        CHECK(stage_pms(ctx, D, p));
        HIPC(hipEventRecord(ctx->ev[6], ctx->st));
        HIPC(hipEventRecord(ctx->ev[4], ctx->st));
        CHECK(stage_post(ctx, p->post, D));
        HIPC(hipEventRecord(ctx->ev[5], ctx->st));
        ctx->pending = 2;
        return SM_OK;
    }
    if (p->aggregator == SM_AGG_GUIDED) {  // no tree: stage times MST / layout / down read 0
        // with a communicator the exchange must carry the guided WTA's subpixel disparities (the 64-bit
        // candidate path); the int32 path would overwrite them with the index
        ctx->sub = (p->post & SM_POST_SUBPIXEL) != 0;
        ctx->nfev = ctx->nsev = 0;
        ctx->fam.clear();
        ctx->fam_vox.clear();
        ctx->fam_ev.clear();
        HIPC(hipEventRecord(ctx->ev[2], ctx->st));
        HIPC(hipEventRecord(ctx->ev[3], ctx->st));
        CHECK(stage_guided(ctx, D, p->disp_begin, p->disp_total > 0 ? p->disp_total : p->disp_begin + D,
                           (p->post & SM_POST_SUBPIXEL) ? 1 : 0, p->gf_radius, p->gf_eps));
        HIPC(hipEventRecord(ctx->ev[6], ctx->st));
        HIPC(hipEventRecord(ctx->ev[4], ctx->st));
        CHECK(stage_reduce(ctx));
        CHECK(stage_post(ctx, p->post, p->disp_total > 0 ? p->disp_total : p->disp_begin + D));
        HIPC(hipEventRecord(ctx->ev[5], ctx->st));
        ctx->pending = 2;
        return SM_OK;
    }
    if (!std::isinf(p->c) && !seg_sync()) {
        // segment mode: the host segmentation on a worker thread, so begin returns at once and the
        // caller's other contexts keep the GPU busy; the worker uploads the forest and enqueues the
        // layout on this context's stream, and sm_match_finish joins it before using the layout
        const bool gpu = !seg_host();
        if (!gpu) CHECK(segment_download(ctx, ctx->views));
        ctx->mst_pend.active = false;
        ctx->seg = true;
        const int views = ctx->views;
        const float c = p->c;
        const int min_size = p->min_size;
        ctx->seg_status = SM_OK;
        ctx->seg_worker = std::thread([ctx, views, c, min_size, gpu] {
            auto work = [&]() -> sm_status {
                HIPC(hipSetDevice(ctx->device));
                if (gpu) {
                    CHECK(segment_gpu(ctx, views, c, min_size, false));
                } else {
                    CHECK(segment_host(ctx, views, c, min_size));
                    CHECK(segment_upload(ctx, views));
                }
                HIPC(hipEventRecord(ctx->ev[2], ctx->st));
                return stage_layout_enqueue(ctx, views);
            };
            try {
                ctx->seg_status = work();
            } catch (const std::bad_alloc&) {
                ctx->seg_status = SM_ERR_OOM;
            } catch (...) {
                ctx->seg_status = SM_ERR_STATE;
            }
        });
        ctx->pending = 1;
        ctx->pend_D = D;
        ctx->pend_p = *p;
        return SM_OK;
    }
    CHECK(stage_tree(ctx, ctx->views, p, false));
    HIPC(hipEventRecord(ctx->ev[2], ctx->st));
    CHECK(stage_layout_enqueue(ctx, ctx->views));
    ctx->pending = 1;
    ctx->pend_D = D;
    ctx->pend_p = *p;
    return SM_OK;
}

static sm_status match_finish_impl(sm_ctx* ctx) {
    if (!ctx) return SM_ERR_ARG;
    if (!ctx->pending) return fail(ctx, SM_ERR_STATE, "sm_match_finish without sm_match_begin");
    const int kind = ctx->pending;
    ctx->pending = 0;
    if (kind == 2) return SM_OK;  // guided / MST_PMS: enqueued in full by sm_match_begin
    // the asynchronous segment-mode tree (sm_match_begin): joined before anything can return early
    const bool had_worker = ctx->seg_worker.joinable();
    if (had_worker) ctx->seg_worker.join();
    HIPC(hipSetDevice(ctx->device));
    const sm_params* p = &ctx->pend_p;
    const int D = ctx->pend_D;
    const CallRange cr = call_range(p, D);
    if (had_worker) CHECK(ctx->seg_status);
    if (kind != 3) CHECK(stage_layout_finish(ctx, ctx->views));
    ctx->exp_layout_ok = kind == 3 || (!ctx->seg && ctx->views == 3);
    HIPC(hipEventRecord(ctx->ev[3], ctx->st));
    CHECK(stage_filter(ctx, cr.D, cr.d0, ctx->views, false, &cr.w));
    HIPC(hipEventRecord(ctx->ev[4], ctx->st));
    CHECK(stage_reduce(ctx));
    CHECK(stage_post(ctx, p->post, p->disp_total > 0 ? p->disp_total : p->disp_begin + D));
    HIPC(hipEventRecord(ctx->ev[5], ctx->st));
    return SM_OK;
}

sm_status sm_match_async(sm_ctx* ctx, int D, const sm_params* p) {
    CHECK(sm_match_begin(ctx, D, p));
    return sm_match_finish(ctx);
}

sm_status sm_synchronize(sm_ctx* ctx) {
    if (!ctx) return SM_ERR_ARG;
    if (ctx->pending) return fail(ctx, SM_ERR_STATE, "sm_synchronize: a call begun with sm_match_begin is not finished (sm_match_finish)");
    HIPC(hipSetDevice(ctx->device));
    HIPC(hipStreamSynchronize(ctx->st));
    CHECK(check_device_error(ctx));
    float t[5];
    for (int i = 0; i < 5; ++i) HIPC(hipEventElapsedTime(&t[i], ctx->ev[i], ctx->ev[i + 1]));
    ctx->stage_ms[0] = t[0];
    ctx->stage_ms[1] = t[1];
    ctx->stage_ms[2] = t[2];
    CHECK(collect_filter_stats(ctx));
    // up / down pass wall time (events at the filter's start, the pass boundary and its end)
    HIPC(hipEventElapsedTime(&ctx->stage_ms[3], ctx->ev[3], ctx->ev[6]));
    HIPC(hipEventElapsedTime(&ctx->stage_ms[4], ctx->ev[6], ctx->ev[4]));
    ctx->stage_ms[5] = t[4];
    float tot;
    HIPC(hipEventElapsedTime(&tot, ctx->ev[0], ctx->ev[5]));
    ctx->stage_ms[6] = tot;
    return SM_OK;
}

sm_status sm_download_results(sm_ctx* ctx, float* ld, float* rd, int32_t* li, int32_t* ri, double* lm, double* rm) {
    if (!ctx) return SM_ERR_ARG;
    if (ctx->pending) return fail(ctx, SM_ERR_STATE, "sm_download_results: a call begun with sm_match_begin is not finished (sm_match_finish)");
    HIPC(hipSetDevice(ctx->device));
    const size_t N = (size_t)ctx->W * ctx->H;
    void* outs[2][3] = {{ld, li, lm}, {rd, ri, rm}};
    for (int v = 0; v < 2; ++v) {
        if (!view_on(ctx->views, v)) continue;  // a one-view call: the other view's buffers are untouched
        if (outs[v][0]) HIPC(hipMemcpyAsync(outs[v][0], ctx->disp[v].p, N * 4, hipMemcpyDeviceToHost, ctx->st));
        if (outs[v][1]) HIPC(hipMemcpyAsync(outs[v][1], ctx->idx[v].p, N * 4, hipMemcpyDeviceToHost, ctx->st));
        if (outs[v][2]) HIPC(hipMemcpyAsync(outs[v][2], ctx->minc[v].p, N * 8, hipMemcpyDeviceToHost, ctx->st));
    }
    HIPC(hipStreamSynchronize(ctx->st));
    return SM_OK;
}

sm_status sm_match(sm_ctx* ctx, const uint8_t* l, const uint8_t* r, int W, int H, int stride, int D, const sm_params* p,
                   float* ld, float* rd, int32_t* li, int32_t* ri, double* lm, double* rm) {
    if (!ctx) return SM_ERR_ARG;
    if (!p) return fail(ctx, SM_ERR_ARG, "null params");
    CHECK(check_tree_size(ctx, W, H, p));
    CHECK(sm_upload_images(ctx, l, r, W, H, stride));
    CHECK(sm_match_async(ctx, D, p));
    CHECK(sm_synchronize(ctx));
    return sm_download_results(ctx, ld, rd, li, ri, lm, rm);
}

sm_status sm_cost_volume(sm_ctx* ctx, const uint8_t* l, const uint8_t* r, int W, int H, int stride, int d0, int D,
                         float* lvol, float* rvol) {
    if (!ctx) return SM_ERR_ARG;
    if (ctx->pending) return fail(ctx, SM_ERR_STATE, "sm_cost_volume: a call begun with sm_match_begin is not finished (sm_match_finish)");
    if (D < 1 || d0 < 0) return fail(ctx, SM_ERR_ARG, "bad disparity range");
    HIPC(hipSetDevice(ctx->device));
    CHECK(upload(ctx, l, r, W, H, stride));
    CHECK(stage_prep(ctx));
    const size_t bytes = (size_t)W * H * D * 4;
    for (int v = 0; v < 2; ++v) CHECK(ensure(ctx, ctx->vol[v], bytes));
    HIPC(launch_cost_volume(ctx->st, P<uint32_t>(ctx->bgrx[0]), P<float>(ctx->gray[0]), P<uint32_t>(ctx->bgrx[1]),
                            P<float>(ctx->gray[1]), P<float>(ctx->atab), W, H, d0, D, P<float>(ctx->vol[0]),
                            P<float>(ctx->vol[1])));
    if (lvol) HIPC(hipMemcpyAsync(lvol, ctx->vol[0].p, bytes, hipMemcpyDeviceToHost, ctx->st));
    if (rvol) HIPC(hipMemcpyAsync(rvol, ctx->vol[1].p, bytes, hipMemcpyDeviceToHost, ctx->st));
    HIPC(hipStreamSynchronize(ctx->st));
    return SM_OK;
}

sm_status sm_build_tree_p(sm_ctx* ctx, const uint8_t* bgr, int W, int H, int stride, const sm_params* p, uint8_t* mask,
                          int32_t* parent_pix, int32_t* subtree_size, int32_t* slot_of_pix, int32_t* ntrees) {
    if (!ctx) return SM_ERR_ARG;
    if (ctx->pending) return fail(ctx, SM_ERR_STATE, "sm_build_tree_p: a call begun with sm_match_begin is not finished (sm_match_finish)");
    if (p && (std::isnan(p->c) || p->c < 0)) return fail(ctx, SM_ERR_ARG, "c must be >= 0 or +INFINITY");
    CHECK(check_tree_size(ctx, W, H, nullptr));
    HIPC(hipSetDevice(ctx->device));
    CHECK(upload(ctx, bgr, bgr, W, H, stride));
    CHECK(stage_prep(ctx));
    CHECK(stage_tree(ctx, 1, p, true));  // the image is uploaded as both views: view 0 only
    ctx->want_size = true;
    const sm_status ls = stage_layout(ctx, 1);
    ctx->want_size = false;
    CHECK(ls);
    const size_t N = (size_t)W * H;
    if (sm_knob("SM_LAYOUT_CHECK")) CHECK(layout_check(ctx, 0, N));  // diagnostics: the metadata's invariants
    // segment mode: the virtual edges that link the trees are not part of the reported forest
    const bool seg = ctx->seg;
    auto virt = [&](size_t i, int k) { return seg && ctx->h_fw[0][k][i] == SM_VIRTUAL_W; };
    if (mask) {
        std::vector<uint8_t> mR(N), mD(N);
        HIPC(hipMemcpy(mR.data(), ctx->mR[0].p, N, hipMemcpyDeviceToHost));
        HIPC(hipMemcpy(mD.data(), ctx->mD[0].p, N, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < N; ++i)
            mask[i] = (uint8_t)((mR[i] && !virt(i, 0) ? 1 : 0) | (mD[i] && !virt(i, 1) ? 2 : 0));
    }
    std::vector<int8_t> pdir(N);
    std::vector<uint32_t> size(N), pre(N);
    HIPC(hipMemcpy(pdir.data(), ctx->pdir[0].p, N, hipMemcpyDeviceToHost));
    HIPC(hipMemcpy(size.data(), ctx->size[0].p, N * 4, hipMemcpyDeviceToHost));
    HIPC(hipMemcpy(pre.data(), ctx->slotpix[0].p, N * 4, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < N; ++i) {
        if (parent_pix) {
            const int k = pdir[i];
            const size_t q = k == 0 ? i + 1 : k == 1 ? i + W : k == 2 ? i - 1 : i - W;
            // the edge to the parent is stored at its left / upper pixel
            const bool v = k >= 0 && (k == 0 ? virt(i, 0) : k == 1 ? virt(i, 1) : k == 2 ? virt(q, 0) : virt(q, 1));
            parent_pix[i] = (k < 0 || v) ? -1 : (int32_t)q;
        }
        if (subtree_size) subtree_size[i] = (int32_t)size[i];
        if (slot_of_pix) slot_of_pix[i] = (int32_t)pre[i];
    }
    if (ntrees) *ntrees = seg ? ctx->seg_trees[0] : 1;
    return SM_OK;
}

sm_status sm_build_tree(sm_ctx* ctx, const uint8_t* bgr, int W, int H, int stride, uint8_t* mask, int32_t* parent_pix,
                        int32_t* subtree_size, int32_t* slot_of_pix) {
    return sm_build_tree_p(ctx, bgr, W, H, stride, nullptr, mask, parent_pix, subtree_size, slot_of_pix, nullptr);
}

sm_status sm_aggregate_debug(sm_ctx* ctx, const uint8_t* l, const uint8_t* r, int W, int H, int stride, int view, int d0,
                             int D, double* A_up, double* A) {
    return sm_aggregate_debug_p(ctx, l, r, W, H, stride, nullptr, view, d0, D, A_up, A);
}

sm_status sm_aggregate_debug_p(sm_ctx* ctx, const uint8_t* l, const uint8_t* r, int W, int H, int stride, const sm_params* p,
                               int view, int d0, int D, double* A_up, double* A) {
    if (!ctx) return SM_ERR_ARG;
    if (ctx->pending) return fail(ctx, SM_ERR_STATE, "sm_aggregate_debug_p: a call begun with sm_match_begin is not finished (sm_match_finish)");
    if (p && (std::isnan(p->c) || p->c < 0)) return fail(ctx, SM_ERR_ARG, "c must be >= 0 or +INFINITY");
    if (view != 0 && view != 1) return fail(ctx, SM_ERR_ARG, "view must be 0 or 1");
    ctx->use_vol = false;  // AGD costs
    if (D < 1 || D > 256 || d0 < 0 || d0 > (1 << 20)) return fail(ctx, SM_ERR_ARG, "bad disparity range");
    CHECK(check_tree_size(ctx, W, H, nullptr));
    HIPC(hipSetDevice(ctx->device));
    ctx->rec_pad = rec_pad_for(d0, D);
    CHECK(upload(ctx, l, r, W, H, stride));
    CHECK(stage_prep(ctx));
    ctx->views = 3;
    CHECK(stage_tree(ctx, 3, p, false));
    CHECK(stage_layout(ctx, 3));
    const size_t N = (size_t)W * H;
    const int Dpad = dpad_for(D);
    CHECK(ensure(ctx, ctx->vol[0], N * (size_t)D * 8));
    // up pass only, snapshot A_up
    {
        CHECK(ensure_filter_bufs(ctx, Dpad));
        WalkArgs a = walk_args(ctx, Dpad, D, d0);
        CHECK(setup_sync(ctx, a, N, Dpad));
        const uint32_t nr = std::max(ctx->layout[0].nrounds, ctx->layout[1].nrounds);
        ctx->nfev = ctx->nsev = 0;
        ctx->fam.clear();
        ctx->fam_vox.clear();
        ctx->fam_ev.clear();
        ctx->ev_open = false;
        for (uint32_t i = 0; i < nr; ++i) CHECK(up_round(ctx, a, nr - 1 - i, spl_for(D), 3));
        CHECK(join(ctx, ctx->st, ctx->st2));
        HIPC(launch_rows_to_volume(ctx->st, P<SmMeta>(ctx->meta[view]), P<double>(ctx->U[view]), (int)N, Dpad, D, N,
                                   P<double>(ctx->vol[0])));
        if (A_up) HIPC(hipMemcpyAsync(A_up, ctx->vol[0].p, N * D * 8, hipMemcpyDeviceToHost, ctx->st));
        HIPC(hipStreamSynchronize(ctx->st));
        CHECK(check_device_error(ctx));
    }
    CHECK(stage_filter(ctx, D, d0, 3, true));
    HIPC(launch_rows_to_volume(ctx->st, P<SmMeta>(ctx->meta[view]), P<double>(ctx->adbg[view]), (int)N, Dpad, D, N,
                               P<double>(ctx->vol[0])));
    if (A) HIPC(hipMemcpyAsync(A, ctx->vol[0].p, N * D * 8, hipMemcpyDeviceToHost, ctx->st));
    HIPC(hipStreamSynchronize(ctx->st));
    return check_device_error(ctx);
}

int sm_stage_times(sm_ctx* ctx, float* out, int n) {
    if (!ctx || !out) return 0;
    int k = n < 7 ? n : 7;
    for (int i = 0; i < k; ++i) out[i] = ctx->stage_ms[i];
    return k;
}

sm_status sm_set_kernel_timing(sm_ctx* ctx, unsigned family_mask) {
    if (!ctx) return SM_ERR_ARG;
    ctx->ktiming = family_mask;
    return SM_OK;
}

int sm_get_kernel_stats(sm_ctx* ctx, sm_kernel_stat* out, int n) {
    if (!ctx || !out) return 0;
    const int k = n < KF_N ? n : KF_N;
    for (int i = 0; i < k; ++i) {
        out[i] = ctx->kstats[i];
        snprintf(out[i].name, sizeof(out[i].name), "%s", kf_name[i]);  // also before the first call
        out[i].bytes_per_voxel = kf_bytes[i];
    }
    return k;
}

sm_status sm_get_filter_stats(sm_ctx* ctx, sm_filter_stats* out) {
    if (!ctx || !out) return SM_ERR_ARG;
    *out = ctx->stats;
    return SM_OK;
}

// Host form of the exchange rule (sm_reduce_rule.h), library-internal: the CPU tests run the gloo
// exchange through these, the GPU path through k_cand / k_finalize.  disp may be NULL when !sub.
void sm_reduce_candidates(const double* minc, const double* gmin, const int32_t* idx, const float* disp, int sub, void* cand,
                          size_t N) {
    for (size_t i = 0; i < N; ++i) {
        if (sub) {
            uint32_t bits;
            memcpy(&bits, disp + i, 4);
            static_cast<unsigned long long*>(cand)[i] = sm_rule_cand64(minc[i], gmin[i], idx[i], bits);
        } else {
            static_cast<int32_t*>(cand)[i] = sm_rule_cand32(minc[i], gmin[i], idx[i]);
        }
    }
}

void sm_reduce_finalize(const double* gmin, const void* gcand, int sub, double* minc, int32_t* idx, float* disp, size_t N) {
    for (size_t i = 0; i < N; ++i) {
        if (sub) {
            uint32_t bits;
            sm_rule_finalize64(gmin[i], static_cast<const unsigned long long*>(gcand)[i], minc[i], idx[i], bits);
            memcpy(disp + i, &bits, 4);
        } else {
            sm_rule_finalize32(gmin[i], static_cast<const int32_t*>(gcand)[i], minc[i], idx[i], disp[i]);
        }
    }
}

sm_status sm_download_labels(sm_ctx* ctx, float* left_abc, float* right_abc) {
    if (!ctx) return SM_ERR_ARG;
    if (!ctx->pms_last) return fail(ctx, SM_ERR_STATE, "sm_download_labels: the last call was not SM_AGG_PMS");
    if (ctx->pending) return fail(ctx, SM_ERR_STATE, "sm_download_labels: a begun call is not finished");
    HIPC(hipSetDevice(ctx->device));
    // the labels' size is the PMS call's (a later upload may have changed W / H)
    const size_t N = (size_t)ctx->pms_W * ctx->pms_H;
    float* out[2] = {left_abc, right_abc};
    for (int v = 0; v < 2; ++v)
        if (out[v]) HIPC(hipMemcpyAsync(out[v], ctx->pms[v].abc.p, N * 12, hipMemcpyDeviceToHost, ctx->st));
    HIPC(hipStreamSynchronize(ctx->st));
    return SM_OK;
}

sm_status sm_get_pms_stats(sm_ctx* ctx, sm_pms_stats* out) {
    return sm_get_pms_stats_n(ctx, out, sizeof(sm_pms_stats));
}

sm_status sm_get_pms_stats_n(sm_ctx* ctx, sm_pms_stats* out, size_t out_bytes) {
    if (!ctx || !out) return SM_ERR_ARG;
    memcpy(out, &ctx->pms_stats, std::min(out_bytes, sizeof(sm_pms_stats)));
    return SM_OK;
}

sm_status sm_labels_extent(sm_ctx* ctx, int* W, int* H) {
    if (!ctx || !W || !H) return SM_ERR_ARG;
    if (!ctx->pms_last) return fail(ctx, SM_ERR_STATE, "sm_labels_extent: the last call was not SM_AGG_PMS");
    *W = ctx->pms_W;
    *H = ctx->pms_H;
    return SM_OK;
}

sm_status sm_comm_unique_id(uint8_t out[SM_UNIQUE_ID_BYTES]) {
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return SM_ERR_RCCL;
    static_assert(sizeof(id) <= SM_UNIQUE_ID_BYTES, "unique id size");
    memcpy(out, &id, sizeof(id));
    return SM_OK;
}

sm_status sm_comm_init(sm_ctx* ctx, int nranks, int rank, const uint8_t id[SM_UNIQUE_ID_BYTES]) {
    if (!ctx || nranks < 1 || rank < 0 || rank >= nranks) return SM_ERR_ARG;
    HIPC(hipSetDevice(ctx->device));
    if (ctx->comm) RCCLC(ncclCommDestroy(ctx->comm));
    ctx->comm = nullptr;
    ncclUniqueId uid;
    memcpy(&uid, id, sizeof(uid));
    RCCLC(ncclCommInitRank(&ctx->comm, nranks, uid, rank));
    ctx->nranks = nranks;
    ctx->rank = rank;
    return SM_OK;
}

sm_status sm_comm_destroy(sm_ctx* ctx) {
    if (!ctx) return SM_ERR_ARG;
    if (ctx->comm) RCCLC(ncclCommDestroy(ctx->comm));
    ctx->comm = nullptr;
    ctx->nranks = 1;
    ctx->rank = 0;
    return SM_OK;
}

void sm_start_timer(double* t0) {
    if (t0) *t0 = now_ms();
}

double sm_get_timer_ms(const double* t0) { return t0 ? now_ms() - *t0 : 0.0; }

}  // extern "C"
