// sm_pms_host.h -- host side of the MST_PMS slanted-plane label search (sm_pms_host.cpp): the
// reference-ordered forest (BFS numbering, tree graph), the heavy-path schedule of every tree, and
// the random streams.  Library-internal; the C-linkage functions at the bottom are exported so the
// CPU tests can compare them with the oracle.
#pragma once
#include <stdint.h>

#ifdef __cplusplus
#include <vector>

// One tree node in schedule ("row") order: per tree, its heavy paths by (light depth, head BFS id),
// each path a contiguous row range from its head down to its bottom.  40 bytes.
struct PmsRow {
    int32_t pix;        // pixel y*W + x
    int32_t parent;     // parent row, -1 at a tree root
    int32_t child[4];   // child rows in DESCENDING BFS id order (the up pass's fold order), -1 unused
    uint16_t w;         // weight code of the edge to the parent (S = exp(-w/12))
    uint8_t nch;        // children
    uint8_t hk;         // index in child[] of the heavy child (0xFF: a leaf); the heavy child is row + 1
    uint16_t wch[4];    // weight codes of the child edges (order of child[])
    uint16_t x, y;      // pixel coordinates
};

// Paths (and pieces) of at least SM_PMS_CHAIN_DEFAULT rows are walked by the chain kernel (sm_pms.hip
// k_pms_chain; env SM_PMS_CHAIN_MIN moves the threshold, down to SM_PMS_CHAIN_LEN, the floor the schedule's
// chain-item counts rt_long are kept for)
#define SM_PMS_CHAIN_LEN 48
#define SM_PMS_CHAIN_DEFAULT 64  // (96 before the chain loaders lost their scratch memory: 100-call frame 470 -> 465 ms)

// A heavy path: rows [row, row + len), head first.
struct PmsPath {
    int32_t tree, row, len, pad;
};

// One work item of a walk: a path and the 64-proposal chunk it covers.
struct PmsItem {
    int32_t path, chunk;
};

// A heavy path cut into pieces (len >= 2 * piece): pieces i < npieces - 1 are rows
// [row + i*piece, row + (i+1)*piece), the last one takes the rest.  Each piece is its own PmsPath in
// f.paths, run from a guessed input (up: its bottom node's heavy child x = 0; down: its head's parent
// row as found); k_pms_repair then re-walks each piece from its neighbour's exact boundary row until
// the recomputed rows agree bitwise with the stored ones.
struct PmsCut {
    int32_t tree, row, len, npieces;
};

// One repair item: a cut path and the 64-proposal chunk
struct PmsRep {
    int32_t cut, chunk;
};

// The forest of one view, in the reference's numbering (Stereo3DMST.cpp:342-384, 434-522) and in the
// walkers' schedule order.
struct PmsForest {
    int W = 0, H = 0, K = 0;
    std::vector<int32_t> tree_start;  // K+1: tree t has BFS nodes (and rows) [tree_start[t], tree_start[t+1])
    std::vector<int32_t> bfs_pix;     // N: BFS node -> pixel (mst_vertices_vec[t][i])
    std::vector<int32_t> nb_start, nb;  // tree_g (:377-384) as CSR, ascending neighbour ids (boost setS)
    std::vector<PmsRow> rows;         // N rows
    std::vector<PmsPath> paths;       // round-major: sorted by (light depth, tree, head BFS id)
    std::vector<PmsItem> items;       // the prop phase's work items (paths x 64-proposal chunks), round-major
    int nrounds = 0;                  // 1 + max light depth
    std::vector<int32_t> rt_path;     // nrounds x (K+1): paths of tree t in round r
    std::vector<int32_t> rt_item;     // nrounds x (K+1): prop items of tree t in round r
    std::vector<int32_t> tree_rounds; // K
    // pieces (piece > 0): cut paths in tree order, their repair items round-major
    int piece = 0;                    // rows per piece, 0: no cuts
    std::vector<PmsCut> cuts;
    std::vector<int32_t> tree_cut;    // K+1: cuts of tree t are [tree_cut[t], tree_cut[t+1])
    std::vector<int32_t> cut_round;   // per cut: its round (light depth)
    std::vector<PmsRep> reps;         // round-major
    std::vector<int32_t> rt_rep;      // nrounds x (K+1)
    std::vector<int32_t> rt_long;     // nrounds x (K+1): paths / pieces of >= SM_PMS_CHAIN_LEN rows x max(1, chunks)
    int npaths = 0, nitems = 0;       // list sizes (the host build: paths.size(), items.size())
    bool on_device = false;           // built on the GPU (sm_pms_forest.hip): rows, paths, items, bfs_pix, nb
                                      // and the row -> tree map live in device buffers only
};

// glibc's random() after srandom(seed) (TYPE_3, the generator sm_pms_glibc_random restates), as a state:
// seed_skip discards the first `skip` outputs, draw continues the stream
struct GlibcRandom {
    int32_t st[31];
    int f = 3, r = 0;
    void seed_skip(unsigned seed, long skip);
    void draw(long n, int32_t* out);
};

// Build the forest from the forest masks (real edges only: mR[p] = edge (p, p+1), mD[p] = (p, p+W)) and
// the edge weights.  Returns the number of trees.
// piece > 0 cuts every heavy path of at least 2 * piece rows into pieces.
// nthreads host threads (0: SM_PREP_THREADS, or min(8, cores / 2)); the result does not depend on it.
int pms_build_forest(int W, int H, const uint16_t* wR, const uint16_t* wD, const uint8_t* mR, const uint8_t* mD,
                     PmsForest& f, int piece = 0, int nthreads = 0);
#endif

#ifdef __cplusplus
extern "C" {
#endif
// The reference's BFS numbering of a forest given as a per-pixel mask (bit 0: edge (p, p+1), bit 1:
// (p, p+W)): the layout of orc_bfs (oracle/sm_oracle.h).  Returns the number of trees.
int sm_pms_forest_bfs(int W, int H, const uint16_t* wR, const uint16_t* wD, const uint8_t* mask, int32_t* tree_start,
                      int32_t* node_pix, int32_t* node_parent, uint16_t* node_w, uint8_t* node_nch, int32_t* node_child);
// tree_g of that forest as CSR (nb capacity nb_cap); returns the entries or -1.
int sm_pms_tree_graph(int W, int H, const uint8_t* mask, const uint16_t* wR, const uint16_t* wD, int32_t* nb_start,
                      int32_t* nb, int nb_cap);
// pms_build_forest over a mask forest: digests of its arrays (rows, paths, items, round lists, cuts, tree
// graph) into out[6], its tree_start (K+1) and bfs_pix (N); returns K
int sm_pms_forest_digest(int W, int H, const uint16_t* wR, const uint16_t* wD, const uint8_t* mask, int piece, int nthreads,
                         uint64_t* out, int32_t* tree_start, int32_t* bfs_pix);
// dice values 0..n-1 of uniform_real_distribution<float>(-1, 1) over a default-seeded minstd_rand0
void sm_pms_dice(long n, float* out);
// glibc random() after srandom(seed): outputs skip .. skip+n-1
void sm_pms_glibc_random(unsigned seed, long skip, long n, int32_t* out);
// segment_image_other_init's random plane labels (Stereo3DMST.cpp:390-430), abc[3N]
void sm_pms_init_labels(int W, int H, int max_disp, float* abc);
// refinement levels per tree (:597-600)
int sm_pms_levels(int max_disp);
#ifdef __cplusplus
}
#endif
