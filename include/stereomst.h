/*
 * stereomst.h -- C-ABI of the MI355X-native Stereo3DMST cost-aggregation path.
 *
 * One entry point per reference operation on the hot path; plain pointers and sizes,
 * integer status codes, no C++/torch/OpenCV types.  The reference-compatible C++
 * surface (stereo3dmst / startTimer / getTimer, include/Stereo3DMST.h) is a thin shim
 * over these calls (stereomatch_amd/csrc/shim/stereo3dmst_cv.cpp, built iff OpenCV
 * is found); ctypes bindings live in stereomatch_amd/_lib.py.
 *
 * Reference interfaces replaced (file:line under /root/reference):
 *   sm_match            <- stereo3dmst()                         src/Stereo3DMST.cpp:714-912
 *                           (include/Stereo3DMST.h:7), per-slice restatement of the
 *                           MST_PMS label search
 *   sm_cost_volume      <- buildCostVolumeSharedMemoryBGR         src/PatchMatchStereoGPU.cu:1482-1550
 *   sm_upload_cost_volumes <- MC-CNN volume mmap + clamp          src/Stereo3DMST.cpp:764-803
 *   sm_build_tree[_p]   <- segment_image_other_init (MST / segment mode) src/Stereo3DMST.cpp:213-543
 *                           + segment_graph/universe              include/segment-graph.h:54-89
 *   sm_aggregate_debug  <- aggregateCostFromChildren/Parent       src/Stereo3DMST.cpp:120-158
 *   WTA inside sm_match <- MSTCostAggregationAndLabelUpdate :160-186 / selectDisparity
 *                                                                 src/PatchMatchStereoGPU.cu:1688-1737
 *   sm_start_timer/sm_get_timer_ms <- startTimer/getTimer         src/Stereo3DMST.cpp:15-26
 *   SM_AGG_PMS, sm_download_labels <- MST_PMS label search + abc_map  src/Stereo3DMST.cpp:546-629, 851-889
 *
 * Threading: one sm_ctx per host thread; the only global mutable state is the knob table
 * (sm_set_knob), which tests set between calls.
 * All calls are synchronous w.r.t. the host unless named *_async.
 */
#ifndef STEREOMST_H
#define STEREOMST_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    SM_OK = 0,
    SM_ERR_ARG = 1,      /* bad argument (sizes, null pointers, unsupported mode)      */
    SM_ERR_HIP = 2,      /* a HIP runtime call failed (message in sm_last_error)       */
    SM_ERR_OOM = 3,      /* device allocation failed                                  */
    SM_ERR_RCCL = 4,     /* an RCCL call failed                                       */
    SM_ERR_STATE = 5,    /* call order violated (e.g. comm not initialised)           */
    SM_ERR_NODEVICE = 6  /* no HIP device: the library never falls back to the CPU    */
} sm_status;

typedef enum { SM_VIEW_LEFT = 0, SM_VIEW_RIGHT = 1 } sm_view;

typedef enum {
    SM_COST_AGD = 0,     /* truncated colour-AD + gradient cost built on the GPU (.cu:1482) */
    SM_COST_VOLUME = 1   /* caller-supplied [D][H][W] float volumes (MC-CNN .bin ingest)    */
} sm_cost_kind;

/* Cost aggregator of a call (sm_params.aggregator). */
typedef enum {
    SM_AGG_TREE = 0,   /* the MST / segment-forest tree filter (Stereo3DMST.cpp:120-186)          */
    SM_AGG_GUIDED = 1, /* the colour guided filter of the cost volume, each view guided by its own
                          image, then selectDisparity (PatchMatchStereoGPU.cu:8251-8470, 1688-1737);
                          float arithmetic; radius gf_radius, eps gf_eps (the reference: 9 and
                          0.01^2*255^2, :9000-9001); AGD cost only */
    SM_AGG_PMS = 2     /* Stereo3DMST's own label search: the segment forest (c, min_size; c = +INFINITY
                          gives the MST), random slanted-plane labels (Stereo3DMST.cpp:390-430), then
                          pms_iters MST_PMS calls per view (:546-629, :851-889) -- neighbour-tree
                          propagation and random refinement, each label aggregated over its tree with
                          the lerp data term (:103-118) and taken per pixel with strict <.  The float
                          disparity is the plane's, fma(x, a, y*b) + c (LabelToDisp before its clamp,
                          :197; SM_POST_LABEL_TO_DISP applies the clamp and scaling); min = each pixel's
                          aggregated cost; idx = -1.  Both views, unsharded (disp_begin 0), D = Dmax */
} sm_aggregator;

typedef struct {
    int device;        /* HIP device ordinal                                        */
    int max_width;     /* workspace capacity                                        */
    int max_height;
    int max_disp;      /* max slices per call on this device (after sharding)       */
} sm_config;

typedef struct {
    float gamma;       /* S = exp(-w*gamma); reference 1/12 (Stereo3DMST.cpp:830)    */
    float c;           /* segment threshold: +INFINITY = MST mode (one tree); finite c >= 0 = segment
                          mode, the forest of segment_graph(c) + the min-size merge, filtered per tree
                          (segment-graph.h:54-89, Stereo3DMST.cpp:242-384; the reference uses 5000, :831) */
    int min_size;      /* min component size of the merge (Stereo3DMST.cpp:293-307, 832); segment mode */
    int median_ksize;  /* 3 (Stereo3DMST.cpp:214); only 3 is supported             */
    int cost_kind;     /* sm_cost_kind                                              */
    int disp_begin;    /* first global disparity of this call (D sharding)          */
    int disp_total;    /* total disparities across all shards (== D unsharded)      */
    int post;          /* sm_post bits applied to the final maps (default 0)         */
    int aggregator;    /* sm_aggregator (default SM_AGG_TREE)                        */
    int gf_radius;     /* SM_AGG_GUIDED: box radius (default 9)                      */
    float gf_eps;      /* SM_AGG_GUIDED: regularisation (default 6.5025 = 0.01^2*255^2) */
    int views;         /* views this call computes: 1 = left, 2 = right, 3 = both (default; 0 = both).
                          A one-view call builds that view's tree only, filters it and (with a
                          communicator) reduces it across the ranks of its group; the other view's
                          outputs are left untouched.  Multi-GPU partitioning: see DESIGN.md 7 */
    int pms_iters;     /* SM_AGG_PMS: MST_PMS calls per view (default 100, Stereo3DMST.cpp:854)    */
} sm_params;

/* Post-processing of the final (cross-rank reduced) float disparity maps (idx / min untouched),
 * applied in this order.  Dmax below = p->disp_total (or disp_begin + D when 0).  stereo3dmst's
 * own output step is SM_POST_LABEL_TO_DISP | SM_POST_LR_CHECK (Stereo3DMST.cpp:900-904). */
typedef enum {
    SM_POST_LR_CHECK = 1,       /* left-right check: a left pixel whose disparity d (rounded) has x-d
                                   outside the image, d outside [0, Dmax), or |d - right(x-d)| > 1 is
                                   set to 0 in left_disp (Stereo3DMST.cpp:632-662, at :904) */
    SM_POST_LABEL_TO_DISP = 2,  /* LabelToDisp + scaling, both maps: disp = clamp(d / (Dmax-1.f), 0, 1)
                                   * (Dmax-1.f) in float (:189-201, :900-902); applied before the check */
    SM_POST_LR_FILL = 4,        /* with SM_POST_LR_CHECK: the check's fill step, fill=true (:664-709) */
    SM_POST_OCCLUSION = 8,      /* handleOcclusionSharedMemory (PatchMatchStereoGPU.cu:1128-1288),
                                   both maps: occluded pixels take the min of the nearest valid
                                   neighbours in the row (255 if none) */
    SM_POST_OCCLUSION_ZERO = 16, /* the same check with remove_occlusion=true: occluded pixels = 0 */
    SM_POST_SUBPIXEL = 32       /* the float disparity of the WTA gets selectDisparity's parabola through
                                   the neighbouring slices' aggregated costs (as float), d - s when
                                   |s| < 1 (PatchMatchStereoGPU.cu:1726-1736); a shard computes a
                                   1-slice halo on each inner side and the cross-rank exchange carries
                                   the winner's disparity (idx / min unchanged).  Applied in the WTA,
                                   i.e. before the steps above */
} sm_post;

typedef struct sm_ctx sm_ctx;

/* Library / context --------------------------------------------------------- */
const char* sm_version(void);
void sm_default_params(sm_params* p);
sm_status sm_create(sm_ctx** out, const sm_config* cfg);
void sm_destroy(sm_ctx* ctx);
const char* sm_last_error(const sm_ctx* ctx);
sm_status sm_device_count(int* count);

/* Whole path, host buffers (the stereo3dmst() boundary) ----------------------
 * left_bgr/right_bgr: H rows of W packed BGR u8 pixels, row_stride bytes apart.
 * Computes slices [p->disp_begin, p->disp_begin + D) for both views and returns,
 * per view, the strict-< argmin slice (global index), its aggregated cost (fp64) and the
 * disparity as float.  Any output pointer may be NULL.  When the context has an RCCL
 * communicator (sm_comm_init) the per-rank results are reduced (min+argmin) across ranks
 * and every rank receives the global answer.  W * H must be below 2^27 pixels (the tree layout
 * packs preorder positions in 27 bits): larger images return SM_ERR_ARG. */
sm_status sm_match(sm_ctx* ctx, const uint8_t* left_bgr, const uint8_t* right_bgr, int W, int H,
                   int row_stride, int D, const sm_params* p,
                   float* left_disp, float* right_disp, int32_t* left_idx, int32_t* right_idx,
                   double* left_min, double* right_min);

/* Device-resident variant for throughput runs: images already in device memory (uploaded
 * with sm_upload_images); outputs stay on the device until sm_download_results.
 * Enqueued on the context stream; returns without synchronising. */
sm_status sm_upload_images(sm_ctx* ctx, const uint8_t* left_bgr, const uint8_t* right_bgr, int W, int H,
                           int row_stride);
sm_status sm_match_async(sm_ctx* ctx, int D, const sm_params* p);
/* sm_match_async in two halves.  sm_match_begin enqueues prep, MST and tree layout and returns
 * without waiting; sm_match_finish waits for the layout's per-round counts (the host sizes the
 * filter launches from them) and enqueues the filter, the cross-rank reduce and the output step.
 * A caller streaming frames over several contexts begins frame i+1 before it finishes frame i,
 * so the GPU has the next frame's tree queued while the host waits.  One begin per finish, per
 * context (SM_ERR_STATE otherwise); sm_match_async == begin + finish. */
sm_status sm_match_begin(sm_ctx* ctx, int D, const sm_params* p);
sm_status sm_match_finish(sm_ctx* ctx);
sm_status sm_synchronize(sm_ctx* ctx);
sm_status sm_download_results(sm_ctx* ctx, float* left_disp, float* right_disp, int32_t* left_idx,
                              int32_t* right_idx, double* left_min, double* right_min);

/* MC-CNN ingest (SM_COST_VOLUME): the raw matching-cost volumes stereo3dmst mmaps from
 * mc-cnn-master/{left,right}.bin (src/Stereo3DMST.cpp:764-775), [D][H][W] float per view, host
 * buffers.  Copied to the device (synchronously: the caller may free them on return); every
 * following sm_match / sm_match_async with p->cost_kind == SM_COST_VOLUME on images of the same
 * W x H filters slices [p->disp_begin, p->disp_begin + D) of them after the reference's clamp,
 * NaN -> 0.5 else min(0.5, x) (:785-803), instead of the AGD cost.  The tree still comes from
 * the images. */
sm_status sm_upload_cost_volumes(sm_ctx* ctx, const float* left_vol, const float* right_vol, int W, int H, int D);

/* Stage entry points (parity tests, MC-CNN ingest) --------------------------- */
/* AGD cost volumes [D][H][W] float for slices [d0, d0+D); host output buffers. */
sm_status sm_cost_volume(sm_ctx* ctx, const uint8_t* left_bgr, const uint8_t* right_bgr, int W, int H,
                         int row_stride, int d0, int D, float* left_vol, float* right_vol);

/* MST of one view's image (MST mode), rooted at pixel 0.  Outputs (host, W*H each, any may
 * be NULL): mask bit0 = edge (p,p+1) in MST, bit1 = edge (p,p+W); parent pixel (root: -1);
 * subtree size; heavy-first preorder slot. */
sm_status sm_build_tree(sm_ctx* ctx, const uint8_t* bgr, int W, int H, int row_stride, uint8_t* mst_mask,
                        int32_t* parent_pix, int32_t* subtree_size, int32_t* slot_of_pix);

/* The same with the tree of params p (NULL: MST mode): for finite p->c the segment forest of
 * segment_graph(c) + the min-size merge (segment-graph.h:54-89, Stereo3DMST.cpp:242-307), each tree
 * rooted at its first pixel (:342-384).  mask / parent_pix report the forest (roots: -1); subtree
 * size and slot refer to the schedule tree the GPU builds (the forest linked at its roots);
 * ntrees (may be NULL) gets the number of trees. */
sm_status sm_build_tree_p(sm_ctx* ctx, const uint8_t* bgr, int W, int H, int row_stride, const sm_params* p,
                          uint8_t* mst_mask, int32_t* parent_pix, int32_t* subtree_size, int32_t* slot_of_pix,
                          int32_t* ntrees);

/* Debug/parity: aggregated volumes of one view in [D][H][W] fp64 (A_up after the leaf->root
 * pass, A after root->leaf), slices [d0, d0+D).  Memory-hungry: for small images. */
sm_status sm_aggregate_debug(sm_ctx* ctx, const uint8_t* left_bgr, const uint8_t* right_bgr, int W, int H,
                             int row_stride, int view, int d0, int D, double* A_up, double* A);
/* ... over the tree of params p (NULL: MST mode; finite c: the segment forest, filtered per tree). */
sm_status sm_aggregate_debug_p(sm_ctx* ctx, const uint8_t* left_bgr, const uint8_t* right_bgr, int W, int H,
                               int row_stride, const sm_params* p, int view, int d0, int D, double* A_up, double* A);

/* Per-stage timings of the last sm_match/sm_match_async (ms, from HIP events on the ctx
 * stream): [0] prep+median+weights, [1] MST, [2] tree layout, [3] up pass, [4] down pass+WTA,
 * [5] cross-rank reduce, [6] total.  n = capacity of out. Returns entries written. */
int sm_stage_times(sm_ctx* ctx, float* out, int n);

/* Tree-filter pass totals of the last call: summed HIP-event durations of the leaf->root
 * and root->leaf passes, and their algorithmic HBM bytes at SURVEY.md 8(d)'s per-voxel
 * figures (leaf->root = K1 cost 4 B + K2 up 8 B; root->leaf = K3 down 8 B + K4 WTA 4 B). */
typedef struct {
    double up_ms, down_ms;
    double up_bytes, down_bytes;
    int up_launches, down_launches;
} sm_filter_stats;
sm_status sm_get_filter_stats(sm_ctx* ctx, sm_filter_stats* out);

/* Per kernel family of the tree filter (k_up_walk, k_up_pre, k_up_chain, k_down_chain,
 * k_down_walk, k_long_costs -- the long paths' AGD cost rows, computed up front): launches,
 * summed HIP-event duration (ms) over the last call, voxels processed (path nodes x
 * disparities, both views) and algorithmic bytes per voxel (DESIGN.md "Roofline accounting").
 * Only timed families report (see sm_set_kernel_timing).  Returns the number of entries
 * written (<= n). */
typedef struct {
    char name[32];
    int launches;
    double ms;
    double voxels;
    double bytes_per_voxel;
} sm_kernel_stat;
int sm_get_kernel_stats(sm_ctx* ctx, sm_kernel_stat* out, int n);

/* Which kernel families the following calls time with HIP events: bit i = entry i of
 * sm_get_kernel_stats (default: all).  Each timed launch costs one event record (~2 us of
 * GPU time per launch at C2); untimed families launch back to back.  No reference
 * counterpart: measurement plumbing of this library. */
sm_status sm_set_kernel_timing(sm_ctx* ctx, unsigned family_mask);

/* MST_PMS (SM_AGG_PMS) ----------------------------------------------------------
 * The plane labels (a, b, c) of every pixel after the last SM_AGG_PMS call, [H*W][3] float per view
 * (abc_map, Stereo3DMST.cpp:814-815); either pointer may be NULL. */
sm_status sm_download_labels(sm_ctx* ctx, float* left_abc, float* right_abc);
/* The extent (W, H) of the labels sm_download_labels copies: the last SM_AGG_PMS call's image size,
 * which a later upload does not change.  Size the label buffers from this (W*H*3 floats each). */
sm_status sm_labels_extent(sm_ctx* ctx, int* W, int* H);
/* Timings and counters of the last SM_AGG_PMS call.  The first MST_PMS call of a view runs its trees
 * one after the other (serial); later calls run every tree at once from guessed dice offsets and the
 * labels at the start of the call, validate, and redo from the first tree whose inputs differed
 * (spec_rounds counts those passes; serial_trees the trees run one by one). */
typedef struct {
    int iters;              /* MST_PMS calls per view */
    int ntrees[2];          /* trees per view */
    int spec_rounds;        /* speculative passes, both views */
    int serial_trees;       /* trees run in serial mode, both views */
    double prep_ms;         /* host: segmentation, forests, schedules, tables (wall) */
    double setup_ms;        /* device: uploads, cost rows, labels (wall) */
    double iter0_ms;        /* the first call of both views (wall) */
    double iters_ms;        /* the remaining calls of both views (wall) */
    double total_ms;        /* the whole SM_AGG_PMS call (wall) */
    /* appended (round 4) */
    double calls_ms;        /* all MST_PMS calls of both views (wall) */
    int concurrent_views;   /* 1: the two views' calls ran concurrently (own host thread + stream each) */
    double first_ms_view[2];  /* per view: its first call (wall, its own thread) */
    double later_ms_view[2];  /* per view: its later calls (wall, its own thread) */
    /* node-label evaluations (one label's data term + up + down + update at one tree node), both views:
     * needed = distinct propagation labels + refinement labels per tree, times its size; _ref = the
     * reference's count (every sampled propagation label); _run = what the device ran, speculation and
     * serial re-runs included (counted only under env SM_PMS_COUNT_RUN=1, else 0) */
    double evals_first, evals_first_ref, evals_first_run;
    double evals_later, evals_later_ref, evals_later_run;
    double prep_seg_ms;     /* host wall of prep_ms: the segmentation (GPU) and its host copies */
    double prep_forest_ms;  /* the reference-numbered forests and walk schedules, both views */
} sm_pms_stats;
sm_status sm_get_pms_stats(sm_ctx* ctx, sm_pms_stats* out);
/* The same, writing at most out_bytes bytes (pass sizeof(sm_pms_stats) of the header the caller was
 * compiled against): a caller built against an older, shorter struct gets its prefix only.  Fields
 * are only ever appended. */
sm_status sm_get_pms_stats_n(sm_ctx* ctx, sm_pms_stats* out, size_t out_bytes);

/* Multi-GPU (one process per GPU, RCCL over xGMI) ----------------------------- */
#define SM_UNIQUE_ID_BYTES 128
sm_status sm_comm_unique_id(uint8_t out[SM_UNIQUE_ID_BYTES]);
sm_status sm_comm_init(sm_ctx* ctx, int nranks, int rank, const uint8_t id[SM_UNIQUE_ID_BYTES]);
sm_status sm_comm_destroy(sm_ctx* ctx);

/* Timers (reference startTimer/getTimer semantics, but per call site, no global). */
void sm_start_timer(double* t0);
double sm_get_timer_ms(const double* t0);

/* Tuning / diagnostic knobs (test and tool hook; no reference counterpart).  Schedule knobs never
 * change a result (every engine is exact under any schedule: piece lengths, repair caps, launch
 * schedules of the segmentation and MST); diagnostic knobs print or count; SM_TEST_PMS_CYCLE is
 * the MST_PMS forest test's fault injection.  The library reads knobs only from this process-wide
 * table, never from the environment (builds with -DSM_DEV excepted).  value: decimal string, or
 * NULL to restore the default.  Set knobs between calls, not while one is running.  Returns
 * SM_ERR_ARG for a name that is not a knob; sm_knob_names lists them (returns the count, writes
 * at most cap names). */
sm_status sm_set_knob(const char* name, const char* value);
int sm_knob_names(const char** out, int cap);

#ifdef __cplusplus
}
#endif
#endif
