// sm_seg_gpu.h -- segment mode's Felzenszwalb segmentation on the GPU (sm_seg_gpu.hip), driven per
// view by segment_gpu() in sm_api.cpp.  Library-internal.
//
// Reference: segment_graph (include/segment-graph.h:54-89) over the (w, a, b)-sorted grid edges of
// Stereo3DMST.cpp:242-282, then the min-size merge of :293-307.  Bit-exact restatement of the serial
// sweep, bucket by bucket:
//   * within one weight bucket w, a component is OPEN if w <= wl + c/size at the bucket's start (the
//     reference's threshold).  A closed component rejects every edge of the bucket (its threshold only
//     changes when it joins, and joining needs its acceptance), and a component that joined in the
//     bucket has threshold w + c/size >= w, so it accepts every later edge of the bucket.  So the
//     bucket joins exactly the open components that its open-open edges connect, whatever the order,
//     and the edges the serial sweep marks are the first (by edge id = the reference's (a, b) order)
//     edge to connect two groups: the minimum spanning forest of the bucket's open-open edges keyed by
//     id, which Boruvka finds in parallel;
//   * the sweep rejects exactly the edges whose two components differ and one of them is closed; a
//     closed component never joins again in the sweep, so such an edge still joins two different
//     components afterwards.  The min-size merge only joins an edge with a component smaller than
//     min_size, and sizes only grow, so it only needs the rejected edges with a small end: those go
//     to the host (few), which runs the merge's serial rule over them in (w, id) order.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define SM_SEG_NB 766        // weight buckets: |dR| + |dG| + |dB| in [0, 765]
#define SM_SEG_TILE 4096     // pixels per block of the bucketing kernels
#define SM_SEG_MAXL 65536    // list counters per view and frame
#define SM_SEG_TAIL_GENS 64  // Boruvka rounds reserved for one tail launch

// counters (uint32) of one view: [0] rejected, [1] hooked roots, [2] trees, [3] min-size candidates,
// [4] error flags, [8 + L] the length of candidate list L, [8 + SM_SEG_MAXL + b] bucket b's first
// hooked-root index
#define SM_SEG_C_REJ 0
#define SM_SEG_C_HOOK 1
#define SM_SEG_C_TREES 2
#define SM_SEG_C_MIN 3
#define SM_SEG_C_ERR 4
#define SM_SEG_C_UNIQ 5   // candidates that are the first of their root pair (k_seg_dense)
#define SM_SEG_C_LOCAL 6  // distinct roots of those (dense local ids)
#define SM_SEG_C_ACT 7    // edges of a small-bucket run with both ends open at its start (k_seg_split)
#define SM_SEG_C_LIST 8
#define SM_SEG_C_BUCKET (8 + SM_SEG_MAXL)
#define SM_SEG_NCOUNT (8 + SM_SEG_MAXL + SM_SEG_NB)

// a rejected edge with a component smaller than min_size at the end of the sweep
struct SegMin {
    uint32_t id, w, ra, rb, sa, sb;
};

// a min-size candidate that is the first (in (w, id) order) of its pair of sweep roots, with the roots
// as dense local ids (lsize / lroot give their sizes and pixels)
struct SegEdge {
    uint32_t la, lb, id, w;
};

struct SegView {
    int W, H;
    const uint16_t* wR;
    const uint16_t* wD;
    uint32_t* par;              // [N] union-find parent (roots: par == self)
    uint32_t* sz;               // [N] component size (roots)
    uint16_t* wl;               // [N] weight of the root's last join (threshold wl + c/size)
    unsigned long long* best;   // [N] Boruvka keys ((~gen) << 32 | edge id), never reset
    uint32_t* first;            // [N] a tree's first pixel in raster order
    uint32_t* ebuf;             // [E] edge ids grouped by weight
    uint32_t* bcnt;             // [NB] counts, [NB + 1] starts (at bcnt + NB), [NB] cursors (at bcnt + 2 NB + 1)
    uint4* list[2];             // candidate lists {id, ra, rb, 0}
    uint32_t* rej;              // rejected edge ids
    uint32_t* hooked;           // roots hooked by the sweep, bucket after bucket
    uint32_t* cnt;              // SM_SEG_NCOUNT counters
    SegMin* mlist;              // min-size candidates
    unsigned long long* mkey[2];  // their (w, id) keys, unsorted / sorted
    uint32_t* mval[2];            // their indices, unsorted / sorted
    SegMin* msorted;              // min-size candidates in (w, id) order
    uint32_t nmin;                // their count (host-set before the sort)
    // pair dedupe (seg_launch_dedupe): only the first candidate of each root pair can join
    uint32_t* keep;               // [E + 1] first of its pair, by position -> (scan) kpos
    uint32_t* act;                // [E] a small-bucket run's active edges (k_seg_split; the keep buffer, free then)
    uint32_t* kpos;               // [E + 1]
    uint32_t* lmark;              // [N + 1] roots of the kept candidates -> (scan) lid
    uint32_t* lid;                // [N + 1]
    SegEdge* dense;               // [E] the kept candidates in (w, id) order
    uint32_t* lsize;              // [N] per local id: the root's size at the end of the sweep
    uint32_t* lroot;              // [N] per local id: the root pixel
    const uint32_t* hooks;        // the host merge's hooks and marked edges (k_seg_apply)
    int nhooks;
    uint8_t* mR;
    uint8_t* mD;
    uint16_t* fwR;
    uint16_t* fwD;
};

// both views of a call in every launch (blockIdx.y, or blockIdx.x for the one-workgroup kernels)
struct SegPair {
    SegView v[2];
    int nv;
};

hipError_t seg_launch_init(hipStream_t st, const SegPair& p);
hipError_t seg_launch_scatter(hipStream_t st, const SegPair& p);
hipError_t seg_launch_classify(hipStream_t st, const SegPair& p, int w, uint32_t m, float c, int lout, uint32_t gen);
hipError_t seg_launch_round(hipStream_t st, const SegPair& p, uint32_t m, int lin, int lout, uint32_t gen);
hipError_t seg_launch_tail(hipStream_t st, const SegPair& p, int lin, uint32_t gen0);
// split = the run's edges were classified by seg_launch_split first (the run then only walks its active edges)
hipError_t seg_launch_small(hipStream_t st, const SegPair& p, int w0, int w1, float c, uint32_t gen0, bool split);
// a small-bucket run's edges at its start: internal ones dropped, those with a closed end rejected at once,
// the rest listed (SM_SEG_C_ACT); nedges = the run's largest edge count over the views
hipError_t seg_launch_split(hipStream_t st, const SegPair& p, int w0, int w1, float c, uint32_t nedges);
// every pixel's parent := its root
hipError_t seg_launch_flatten(hipStream_t st, const SegPair& p);
hipError_t seg_launch_sizes(hipStream_t st, const SegPair& p, int w, uint32_t m);
hipError_t seg_launch_minsize(hipStream_t st, const SegPair& p, int min_size, uint32_t nrej_max);
size_t seg_sort_temp_bytes(uint32_t n);
hipError_t seg_launch_sort(hipStream_t st, const SegPair& p, void* const* temp, const size_t* temp_bytes);
// after seg_launch_sort: the first candidate of each root pair, dense root ids; counts at SM_SEG_C_UNIQ / _LOCAL
hipError_t seg_launch_dedupe(hipStream_t st, const SegPair& p, void* const* temp, const size_t* temp_bytes);
// the same without sorting (SM_SEG_SORTDEDUP=1 keeps the sorts): each root pair's minimum (w, id) key by
// atomicMin in a hash table over the pair keys (cap slots, a power of two >= 2 nmin, in mkey[0] / mkey[1]);
// dense is then unordered (the host sorts its kept candidates); needs 2 nmin <= cap <= E
hipError_t seg_launch_dedupe_hash(hipStream_t st, const SegPair& p, void* const* temp, const size_t* temp_bytes,
                                  uint32_t cap);
hipError_t seg_launch_apply(hipStream_t st, const SegPair& p);
hipError_t seg_launch_trees(hipStream_t st, const SegPair& p);
