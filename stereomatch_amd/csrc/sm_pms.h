// sm_pms.h -- launchers of the MST_PMS kernels (sm_pms.hip), library-internal.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sm_pms_host.h"

// Device view of one view's MST_PMS state (kernel argument).  Rows of tree t are [tree_start[t],
// tree_start[t+1]) in the schedule order of PmsForest; A rows of tree t start at tree_abase[t] with
// tree_pt[t] doubles per row.  The label table of tree t (tree_lab[t]) holds deg(t) propagation
// labels, then the refinement labels of the current iteration (compacted: nref[t] of them).
struct PmsDev {
    const PmsRow* rows;
    const int32_t* rtree;        // row -> tree
    const PmsPath* paths;
    const PmsItem* items;
    const int32_t* rt_path;      // nrounds x (K+1)
    const int32_t* rt_item;
    const int32_t* tree_rounds;
    const int32_t* tree_start;
    const int32_t* bfs_pix;
    const int32_t* nb_start;
    const int32_t* nb;
    const int32_t* tree_pt;
    const long long* tree_abase;
    const int32_t* tree_lab;
    int32_t* nref;
    float4* lab;                 // (a, b, c, 0)
    // speculative passes: each tree's propagation labels without repeats (first occurrences, in order)
    // and their count; nprop == nullptr: every tree's phase 0 has deg(t) proposals in lab
    float4* labu;
    int32_t* nprop;
    int32_t* labq;               // pixel each propagation label was sampled at
    float* abc;                  // [N][3] current labels
    double* minc;                // [N] current minimum aggregated costs
    float* abc_bak;              // [N][3] labels at the start of the iteration (speculation)
    double* minc_bak;
    double* A;                   // aggregation rows
    const float* vol;            // cost rows [N][Dv]
    const float* dice;           // the replayed (-1, 1) dice stream
    long long dice_n;
    const int32_t* rnd;          // this iteration's rand() values, one per tree
    long long* off;              // the dice offset of the next tree (serial mode); [1]: scratch
    long long* oguess;           // per tree: its speculated dice offset
    int32_t* cnt;                // per tree: dice values it consumed (given oguess)
    int32_t* flag;               // per tree: its propagation inputs were stale (speculation)
    int32_t* result;             // [0] first invalid tree (K: none), [1..2] its exact offset (int64)
    uint32_t* err;               // bit 1: a sampled index fell outside its tree; bit 2: dice stream exhausted
    long long* prof;             // SM_PMS_PROF: k_pms_serial segment totals (nullptr: off)
    unsigned long long* evals;   // node-label evaluations the per-pixel updates ran (nullptr: not counted)
    // walk plan of one phase (k_pms_plan): per round r, the paths of trees with few proposals in lists of
    // lane-group classes (PMS_NCLS - 1 of them: P <= 2, P <= 8) and (path, chunk) items of the others;
    // plan_cnt[r * PMS_NCLS + c] entries at plan_path + plan_base[r] (classes) / plan_item + plan_ibase[r]
    int32_t* plan_cnt;
    int32_t* plan_path;          // class c of round r at plan_path + c * npaths_total + plan_base[r]
    PmsItem* plan_item;
    const int32_t* plan_base;    // nrounds: first path of round r (rt_path[r][0])
    const int32_t* plan_ibase;   // nrounds: rt_item[r][0] + rt_path[r][0] (big items: chunks of any phase)
    int npaths_total;
    int item_cap;                // plan_item: wave items at [0, item_cap), chain items at [item_cap, 2 item_cap)
    const double* slut;
    const double* s2lut;
    // pieces (sm_pms_host.h PmsCut): cut paths, repair items, per-cut backup offsets into Abak (the
    // A_up rows of a cut path's non-head pieces, saved before the down pass overwrites them)
    const PmsCut* cuts;
    const PmsRep* reps;
    const long long* cut_bak;
    double* Abak;
    uint32_t* rep_flag;          // per repair item: pieces whose parallel repair rewrote a boundary row (bit i)
    int W, Dv, Dmax, K, nrounds, piece;
    int hi_bak;  // 1: propagation samples higher neighbours (u > t) from abc_bak, the call's starting labels
                 // (a serial re-run in the middle of a speculative call, whose later trees keep results)
};

// serial: trees [t0, t1) one after the other in one workgroup (the reference's order), starting at the
// dice offset *off and leaving the next one there
hipError_t launch_pms_serial(hipStream_t st, const PmsDev& d, int t0, int t1);
// the propagation labels of trees [t_lo, t_hi) without repeats -> labu / nprop (k_pms_prop_dedupe)
hipError_t launch_pms_prop_dedupe(hipStream_t st, const PmsDev& d, int t_lo, int t_hi);
// serial mode, one large tree over the whole GPU: propagation labels from *off, and the refinement
// labels (after the propagation update), which advance *off
hipError_t launch_pms_prop_tree(hipStream_t st, const PmsDev& d, int t);  // d: labu / nprop set (labels + dedupe)
hipError_t launch_pms_ref_one(hipStream_t st, const PmsDev& d, int t);
// speculative iteration over trees [t_lo, K): every tree at once from the guessed offsets and the
// labels at the start of the iteration, then validation (sm_pms.hip "Speculation")
// wn: stream floats from off[0] a pass can consume (staged in LDS when the window fits)
hipError_t launch_pms_guess(hipStream_t st, const PmsDev& d, int t_lo, long long wn);
hipError_t launch_pms_prop_setup(hipStream_t st, const PmsDev& d, int t_lo, int total_deg);
// lane-group classes of the planned walks: paths of trees with P <= 2 / P <= 8 proposals share a wave
// (32 / 8 paths per wave), the rest are (path, 64-proposal chunk) items of one wave each
#define PMS_NCLS 3
// plan counters per round: the PMS_NCLS walk classes, then the chain items (paths of >= PMS_CHAIN_LEN rows)
#define PMS_NCNT 4
// one round's chain items (k_pms_chain): `items` workgroups (the host's bound on the round's long items)
hipError_t launch_pms_chain(hipStream_t st, const PmsDev& d, int phase, bool up, int r, int items);
// the phase's A-row layout of trees [t_lo, t_hi): stride P rounded up to even, packed (k_pms_layout)
// (and zeroes zero[0, nzero): the phase's plan counters, so launch_pms_plan needs no memset)
hipError_t launch_pms_layout(hipStream_t st, const PmsDev& d, int phase, int t_lo, int t_hi, int32_t* pt_out,
                             long long* ab_out, int32_t* zero = nullptr, int nzero = 0);
// the walk plan of trees [t_lo, t_hi) for a phase (plan_cnt zeroed here unless `zeroed`); r_lo..r_hi: rounds to plan
// chain_len > 0: paths of >= max(chain_len, SM_PMS_CHAIN_LEN) rows become chain items (k_pms_chain);
// 0: none (wave items)
hipError_t launch_pms_plan(hipStream_t st, const PmsDev& d, int phase, int t_lo, int t_hi, int nrounds, int max_paths,
                           int chain_len, bool zeroed = false);
// one round's planned walk, a persistent grid of `waves` waves (the host's bound on the work)
hipError_t launch_pms_walk_plan(hipStream_t st, const PmsDev& d, int phase, bool up, int r, int waves);
hipError_t launch_pms_cost(hipStream_t st, const PmsDev& d, int phase, int row_lo, int row_hi);
hipError_t launch_pms_update(hipStream_t st, const PmsDev& d, int phase, int row_lo, int row_hi);
hipError_t launch_pms_ref_setup(hipStream_t st, const PmsDev& d, int t_lo);
// pieces: re-walk the cut paths' guessed pieces from their exact neighbours (repair items [lo, hi)),
// and save the A_up rows of cuts [c_lo, c_hi) before the down pass
// maxp > 0: first every guessed piece at once (k_pms_repair_par, maxp = the most pieces of a cut in the
// range), then the sequential pass only for the items it flagged; maxp = 0: the sequential pass alone
hipError_t launch_pms_repair(hipStream_t st, const PmsDev& d, int phase, bool up, int lo, int hi, int maxp);
hipError_t launch_pms_cut_backup(hipStream_t st, const PmsDev& d, int c_lo, int c_hi);
hipError_t launch_pms_validate(hipStream_t st, const PmsDev& d, int t_lo);
hipError_t launch_pms_restore(hipStream_t st, const PmsDev& d, int row_lo, int row_hi);
hipError_t launch_pms_backup(hipStream_t st, const PmsDev& d, size_t N);
// after a call: the node-label evaluations it needed, acc[0] += sum_t size(t) * (distinct propagation labels
// + refinement labels), and the reference's count, acc[1] += sum_t size(t) * (deg(t) + refinement labels)
hipError_t launch_pms_count(hipStream_t st, const PmsDev& d, unsigned long long* acc);
// [D][N] volume slices (MC-CNN layout; clamp: NaN -> 0.5, min(0.5, x), Stereo3DMST.cpp:785-803) ->
// [N][Dv] cost rows
hipError_t launch_pms_vol_rows(hipStream_t st, const float* in, size_t N, int D, int Dv, int clamp, float* out);
// plane disparity of every pixel's label, fma(x, a, y*b) + c (LabelToDisp before its clamp, :197)
hipError_t launch_pms_disp(hipStream_t st, const float* abc, int W, size_t N, float* disp);
