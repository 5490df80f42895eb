// sm_launch.h -- host-side launchers of the kernels in sm_kernels.hip (library-internal).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "sm_common.h"

// WTA configuration of the down pass (sm_walk_util.h wta_nodes): the call computes local slices
// [0, dcall) = global [dglob0, dglob0 + dcall); the WTA takes local [lo, hi); dtot = the total range
#ifndef SM_WTACFG_DEFINED
#define SM_WTACFG_DEFINED
struct WtaCfg {
    int lo, hi, dglob0, dtot, sub;
};
#endif

// byte ranges zeroed by one launch (each base 16-byte aligned: hipMalloc'd buffers)
#define SM_ZERO_MAX 12
struct ZeroList {
    void* p[SM_ZERO_MAX];
    size_t n[SM_ZERO_MAX];
    int count;
    void add(void* ptr, size_t bytes) { p[count] = ptr; n[count] = bytes; ++count; }
};

struct MstArgs {
    int nviews;
    const uint16_t* wR[2];
    const uint16_t* wD[2];
    uint32_t* comp[2];
    unsigned long long* best[2];
    uint32_t* root[2];
    uint8_t* mR[2];
    uint8_t* mD[2];
    int* flags[2];   // per view: flags[r] for r < SM_MST_MAX_ROUNDS
};

// contracted Boruvka (after the tile phase): component graph buffers per view
struct MstCompact {
    uint32_t* cid[2];     // [pixel] compact id of a tile-phase representative
    uint32_t* counts[2];  // [0] K, [1] E' of edge list 0, [2] of list 1
    void* edges[2];       // two CEdge lists of emax (16 B each)
    size_t emax;
    size_t bstride;  // second best[] array at best + bstride (best holds 2 * bstride keys)
    uint32_t* lab[2];     // [K]
    uint32_t* hook[2];    // [K]
};

#define SM_MST_MAX_ROUNDS 64
#define SM_REC_PAD 1024  // records of padding before/after each image (walker loads stay in bounds)

struct WalkArgs {
    const SmMeta* meta[2];
    const SmPath* paths[2];
    int npaths[2];
    double* U[2];
    double* A[2];        // down-pass A rows of light children's parents (compact: SmMeta::cslot[3])
    double* Adbg[2];     // every node's A row by slot (debug calls, store_all), else nullptr
    int32_t* idx[2];
    double* minc[2];
    float* disp[2];
    const uint2* Lrec;   // {bgrx, gray} records, padded by SM_REC_PAD records on both sides
    const uint2* Rrec;
    const uint32_t* Lrec4;  // bgrx alone, same padding: the up walker recomputes the gray
    const uint32_t* Rrec4;
    const float* atab;
    const double* slut;
    const double* s2lut;
    float* Cst[2];       // cost rows [slot][Dpad]: long-path AGD staging, or every slot's volume row
    int vol;             // costs from Cst rows (MC-CNN ingest, k_vol_rows) instead of the AGD cost
    // 1: the short-path walkers treat leaves specially.  A leaf's A_up is its cost ((double)C, no
    // children), so the up walker does not store the rows of heavy leaves (read by nobody: their
    // parent takes the value from registers, light children are path heads) and the down walker
    // recomputes every leaf's A_up from the image records instead of reading U.  0: AGD costs
    // unavailable (vol) or a debug call that reads every U row.
    int leaf_cost;
    int maxlen;          // longest path of the current bucket (both views)
    const uint2* segtab[2];  // long buckets: {path, segment} per SM_PRE_SEG-node segment
    int nseg[2];
    int W, Dpad, dcall, dglob0;
    WtaCfg wta;          // down pass: the WTA's slice range, output offset, subpixel (sm_walk_util.h)
    uint32_t epoch;       // filter call counter (status words hold it)
    // long-path pieces of the current long bucket (sm_chain.hip "Pieces"); pieces[v] == nullptr:
    // one workgroup per path, no pieces
    const uint4* pieces[2];
    int npieces[2];
    // rows of cut paths' nodes, 32 per segment (row = 32 * segment of the path + node offset in the
    // path; per bucket from its first segment): the up repair's buffered corrections, the down
    // pieces' published last rows
    double* fix[2];
    double* agg[2];       // per bucket segment: [P row | B row] (2 * Dpad doubles), affine aggregates
    uint32_t* pstat[2];   // status words of the bucket's first piece: done / merged / final at
    int pstride;          // offsets 0, pstride, 2 * pstride
    int piece_len;        // P (SM_PIECE or env SM_PIECE_LEN)
    int bucket_plen[2];   // the current long bucket's piece length per view (sm_bucket_piece_len)
    int repair_max;       // fast-repair node cap (env SM_REPAIR_MAX; tests force the slow path)
    unsigned long long* piece_dbg;  // SM_PIECE_DEBUG counters (nullptr otherwise)
    uint32_t* err;        // device error word of the call (host-mapped; sm_synchronize checks it)
    int wait_iters;       // polls before a cross-workgroup wait gives up (env SM_WAIT_ITERS, tests)
};

hipError_t launch_prep(hipStream_t st, const uint8_t* l, const uint8_t* r, int W, int H, int stride, uint32_t* lb,
                       float* lg, uint32_t* rb, float* rg, uint2* lrec, uint2* rrec, uint32_t* lrec4, uint32_t* rrec4);
hipError_t launch_median_weights(hipStream_t st, const uint32_t* lb, const uint32_t* rb, uint32_t* lmed, uint32_t* rmed,
                                 uint16_t* lwR, uint16_t* lwD, uint16_t* rwR, uint16_t* rwD, int W, int H);
hipError_t launch_cost_volume(hipStream_t st, const uint32_t* lb, const float* lg, const uint32_t* rb, const float* rg,
                              const float* atab, int W, int H, int d0, int D, float* lvol, float* rvol);
// ccount / clab: null for the pixel rounds; otherwise the contracted rounds' K counter and label array,
// whose initial state k_bor_local writes with the compact ids (minima: best, best + bstride)
hipError_t launch_bor_local(hipStream_t st, const MstArgs& a, int W, int H, uint32_t* const ccount[2],
                            uint32_t* const clab[2], size_t bstride);
hipError_t launch_bor_round(hipStream_t st, const MstArgs& a, int W, int H, int r);
hipError_t launch_bor_compact(hipStream_t st, const MstArgs& a, const MstCompact& c, int W, int H);
hipError_t launch_bor_cround(hipStream_t st, const MstArgs& a, const MstCompact& c, int W, int r);
hipError_t launch_zero(hipStream_t st, const ZeroList& z);
hipError_t launch_mst_done(hipStream_t st, const MstArgs& a, int r, int* ok);
hipError_t launch_vol_rows(hipStream_t st, const float* vin, size_t N, int d0, int D, int Dpad, const uint32_t* slotpix,
                           float* Cst);
// guided-filter aggregator (sm_guided.hip): per-pixel WTA state of one view
struct GfStateArgs {
    float* mn;
    int32_t* best;
    float* pre;
    float* nxt;
    float* prevq;
};
hipError_t launch_gf_guide(hipStream_t st, const uint32_t* bgrx, int W, int H, int r, float eps, float* planes, float* tmp,
                           float* means, float* stats);
hipError_t launch_gf_batch(hipStream_t st, const float* cost, const uint32_t* bgrx, const float* stats, int W, int H, int r,
                           int S, int dloc0, float* pl, float* tmp, GfStateArgs sa);
hipError_t launch_gf_init(hipStream_t st, GfStateArgs sa, size_t N);
// the fused tile path (radius 9) keeps its statistics and (b, a) planes in the row band layout:
// planes of gf_band_plane(W, H) elements
bool gf_fused(int r);
size_t gf_band_plane(int W, int H);
hipError_t launch_gf_out(hipStream_t st, GfStateArgs sa, size_t N, int dglob0, int dtot, int sub, int32_t* idx, double* minc,
                         float* disp);

// output step (sm_post.hip)
hipError_t launch_label_to_disp(hipStream_t st, float* d0, float* d1, size_t N, int dmax);
hipError_t launch_lr_check(hipStream_t st, float* left, const float* right, int W, int H, int max_disp, uint8_t* mask);
hipError_t launch_lr_fill(hipStream_t st, float* left, const uint8_t* mask, int W, int H, int* scratch);
hipError_t launch_occlusion(hipStream_t st, float* left, float* right, int W, int H, float thresh, int remove, float min_disp,
                            uint8_t* occ, int* scratch);
// The segment aggregates of a round's cut long paths (sm_walk_util.h up_pre_segment).
struct UpPreArgs {
    const SmPath* paths[2];  // the round's long bucket
    const uint2* seg[2];     // its segment table (cut paths only)
    int nseg[2];
    double* agg[2];          // segment aggregates (nullptr: no pieces in that view)
    int plen[2];             // the bucket's piece length
    int walk_blocks;         // fused walker launch: blocks [0, walk_blocks) walk, the rest are segments
};
UpPreArgs up_pre_args(const WalkArgs& long_bucket);
// pre: the round's long bucket when its segment aggregates run as extra blocks of this launch
hipError_t launch_up(hipStream_t st, const WalkArgs& a, int spl, bool long_paths, const WalkArgs* pre = nullptr);
hipError_t launch_down(hipStream_t st, const WalkArgs& a, int spl, bool long_paths);
// long-path engine (sm_chain.hip): buckets of paths with >= SM_LONG_PATH nodes; k_up_pre only
// computes the segment aggregates of paths cut into pieces
hipError_t launch_up_pre(hipStream_t st, const WalkArgs& a, int spl);
hipError_t launch_up_chain(hipStream_t st, const WalkArgs& a, int spl);
hipError_t launch_down_long(hipStream_t st, const WalkArgs& a, int spl, int store_all);
hipError_t launch_down_debug(hipStream_t st, const WalkArgs& a, int spl, bool long_paths);
hipError_t launch_rows_to_volume(hipStream_t st, const SmMeta* meta, const double* U, int nslots, int Dpad, int D,
                                 size_t N, double* out);
