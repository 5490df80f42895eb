// sm_pms_forest.h -- the MST_PMS schedule forest built on the GPU (sm_pms_forest.hip): the same
// arrays as the host construction pms_build_forest (sm_pms_host.cpp), bit for bit.  Library-internal.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sm_pms_host.h"

// Device buffers of one view's GPU forest build.  Capacities are set by the caller (pms_forest_gpu
// in sm_api.cpp allocates them); the outputs (rows ... rt_long) are the PmsDev inputs.
struct PfView {
    int W, H, N;
    // inputs: forest masks with the segment forest's virtual links (weight code SM_VIRTUAL_W), weights
    const uint8_t* mR;
    const uint8_t* mD;
    const uint16_t* fwR;
    const uint16_t* fwD;
    const uint16_t* wR;
    const uint16_t* wD;
    // pixels (N)
    int32_t* par;       // union-find parents (root: the tree's first pixel)
    int32_t* flag;      // N + 1: root flags -> (scan) tree id of a root pixel, [N] = K
    int32_t* tree_of;
    int4* nbr;          // real tree neighbours in (w, a, b) key order, -1: none
    uint2* nbw;         // their weight codes, 4 x u16
    // trees (K)
    int32_t* root_pix;
    int32_t* tsize;     // K + 1 -> (scan) tree_start
    int32_t* tree_start;
    int32_t* tree_rounds;
    // the BFS by Euler tours (sm_tour.h): per pixel
    uint32_t* rot;      // rotation word: real edges by direction, the tour's next direction per arrival
    int8_t* pdir;       // direction to the parent (-1: a root)
    int32_t* psize;     // subtree size
    int32_t* bpos;      // BFS position
    // per arc (4N) and per chain (max_chains) of the list ranking
    uint16_t* a_dist;
    uint32_t* a_cid;
    uint32_t* nchains;
    uint32_t* c_last;
    uint32_t* c_len;
    uint64_t* cnw;
    uint32_t max_chains;
    long long* tval;    // 2(N - K): the tours' values, concatenated by tree, and their inclusive scan
    long long* tval_s;
    unsigned long long* tkey[2];  // (tree, depth) at the global preorder position, sorted
    int32_t* tpix[2];
    // BFS order (N) of every tree at once (tree-major: the level-order arrays of the round-4 build)
    int32_t* gpix;
    int32_t* gpar;      // parent's index (-1: a root)
    int32_t* gtree;
    uint16_t* gw;       // weight code of the edge to the parent
    int32_t* gfc;       // first child's index
    uint8_t* gnc;       // children
    int32_t* gsize;     // subtree size
    int8_t* ghk;        // heavy child (index among the children, -1: a leaf)
    // BFS numbering (N): the stable sort of the level order by tree
    int32_t* iota;
    int32_t* bglob;     // BFS node -> level-order index
    int32_t* gtree_s;   // sorted keys (scratch)
    int32_t* g2b;       // level-order index -> BFS node
    int32_t* bpar;
    int32_t* bch0;      // first child (BFS), -1: a leaf
    int32_t* J[2];      // pointer jumping: path head
    int32_t* Dj[2];     //                  offset on the path
    int32_t* plen;      // [head] path length
    int32_t* ld;        // [node] light depth (heads first, then every node)
    int32_t* rowof;
    int32_t* rowstart;  // [head]
    // heads (<= N)
    int32_t* hflag;     // N + 1: head flags
    int32_t* hidx;      // N + 1: their scan (a head's index; [N] = heads)
    unsigned long long* hkey[2];
    int32_t* cutof;     // [head node] -> cut index (-1: not cut)
    int32_t* hcnt[4];   // per sorted head (n + 1 each): scan inputs -- A order: path length, cut flag;
    int32_t* hoff[4];   //   B order: pieces, prop items, repair items, chain items -- and their scans
    int32_t* rtc[4];    // nrounds x (K + 1) + 1: per (round, tree) counts of the four lists
    // tree graph
    unsigned long long* pairs[2];  // <= 4N
    int32_t* npairs;    // [0]: pairs
    int32_t* uflag;     // 4N + 1: first of its run in the sorted pairs
    int32_t* uidx;      // 4N + 1: their scan
    int32_t* nbcnt;     // K + 1: per tree count (cuts, then neighbours) -> (scan) tree_cut / nb_start
    // outputs
    PmsRow* rows;
    int32_t* rtree;
    int32_t* bfs_pix;
    int32_t* nb_start;
    int32_t* nb;
    PmsPath* paths;
    PmsItem* items;
    PmsCut* cuts;
    int32_t* cut_round;
    PmsRep* reps;
    int32_t* tree_cut;  // K + 1
    int32_t* rt[4];     // nrounds x (K + 1): rt_path, rt_item, rt_rep, rt_long
    int32_t* tot;       // [0..3] paths, items, reps, long; [4] cuts; [5] nrounds; [6] heads; [7] inconsistent; [8] edges
    void* temp;         // hipcub scratch
    size_t temp_bytes;
    int piece;
};

// hipcub scratch bytes for N pixels (the largest sort / scan / select of the build)
size_t pf_temp_bytes(int N);
// steps of the build; each ends with a host sync for the sizes the next one allocates by
hipError_t pf_trees(hipStream_t st, PfView& v, int* K_out);   // union-find, tree ids, sizes
size_t pf_max_chains(int W, int H, int K);                      // chain capacity of the BFS's tours
// BFS, sizes, heavy paths, light depths; out[0] = rounds, out[1] = heads, out[2] != 0: the masks had a cycle (1),
// a light depth stayed unresolved (2) or a tour was inconsistent (4)
hipError_t pf_bfs(hipStream_t st, PfView& v, int K, int* out);
// rows, cuts, tree graph, round-major counts and tables; counts: paths, items, reps, chain items, cuts, pairs,
// error flag
hipError_t pf_lists(hipStream_t st, PfView& v, int K, int nrounds, int nheads, int* counts);
hipError_t pf_fill(hipStream_t st, PfView& v, int nheads);  // paths, items, repair items
