/*
 * sm_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the lr-xiang/StereoMatch Stereo3DMST cost-aggregation path,
 * used as the parity checker for the HIP product (stereomatch_amd/) and as the
 * cpu_baseline leg of bench.py.  Nothing in the product links, loads or calls
 * this library: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline.
 *
 * Parity status (details in DESIGN.md "Oracle"):
 *  - MST (orc_segment) is pinned against the reference's own include/segment-graph.h
 *    + include/disjoint-set.h, compiled here into oracle/_ref (tests/golden fixtures).
 *  - Tree filter arithmetic is pinned by static disassembly of the shipped
 *    build/StereoYin (vfmadd/vfnmadd pattern), not by executed reference outputs.
 *  - AGD cost volume restates src/PatchMatchStereoGPU.cu:1482-1550; the reference
 *    ships no fixtures for it (parity unpinned for that row).
 *
 * Layouts: images are packed BGR uint8 rows (OpenCV CV_8UC3) with a row stride in
 * bytes; pixel index p = y*W + x; volumes are [d][y][x] (Stereo3DMST.cpp:117).
 */
#ifndef SM_ORACLE_H
#define SM_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* mst/segment mask bits per pixel */
#define ORC_EDGE_RIGHT 1u /* edge (p, p+1) */
#define ORC_EDGE_DOWN 2u  /* edge (p, p+W) */

/* cv::medianBlur(ksize=3) per channel, BORDER_REPLICATE (Stereo3DMST.cpp:226-228). out: packed W*3. */
void orc_median3(const uint8_t* img, int W, int H, int stride, uint8_t* out);

/* 4-connected edge weights, L1 RGB (Stereo3DMST.cpp:83-94, 242-262). wR[p] for x<W-1, wD[p] for y<H-1,
 * 0xFFFF where the edge does not exist. */
void orc_edge_weights(const uint8_t* med, int W, int H, uint16_t* wR, uint16_t* wD);

/* segment_graph (include/segment-graph.h:54-89) + min-size merge (Stereo3DMST.cpp:293-307).
 * c = +INFINITY is MST mode; min_size < 0 skips the merge (oracle-only).  Returns the number of components; mask gets ORC_EDGE_* bits. */
int orc_segment(int W, int H, const uint16_t* wR, const uint16_t* wD, float c, int min_size, uint8_t* mask);

/* Component enumeration + BFS rooting/renumbering (Stereo3DMST.cpp:342-369, 434-522).
 * Trees in order of their first raster pixel; root = first pixel; children in ascending
 * (w,a,b) edge order (Boost vecS insertion order).  Node arrays are indexed by global BFS
 * node id (tree_start[t] + bfs id).  node_parent[root] = root; node_w[root] = 0.
 * node_child[4*n+i] for i < node_nch[n], ascending BFS id.  Returns number of trees. */
int orc_bfs(int W, int H, const uint16_t* wR, const uint16_t* wD, const uint8_t* mask,
            int32_t* tree_start, int32_t* node_pix, int32_t* node_parent, uint16_t* node_w,
            uint8_t* node_nch, int32_t* node_child);

/* buildCostVolumeSharedMemoryBGR (PatchMatchStereoGPU.cu:1482-1550), slices d0..d1-1:
 * right[d][y][x] (right reference) and left[d][y][x+d]; invalid = 3.0f; the left column
 * the reference never writes (x = W-1, x >= d) is defined as 3.0f. Volumes [(d1-d0)][H][W]. */
void orc_set_gf_contract(int mode);  /* 1: the guided filter helpers as nvcc --fmad=true would contract them */
void orc_set_agd_contract(int mode); /* 0: shipped (uncontracted) AGD; 1: nvcc --fmad=true contraction */
void orc_cost_agd(const uint8_t* left, const uint8_t* right, int W, int H, int stride, int d0, int d1,
                  float* left_vol, float* right_vol, int nthreads);

/* Per-slice tree filter in the shipped order (Stereo3DMST.cpp:120-186):
 *   up   (descending BFS id): A[p] = A[p] + C ; A[parent] = fma(S, A[p], A[parent])
 *   down (ascending BFS id) : A[c] = fma(S_c, A[p], S2_c * A[c])
 * then strict-< argmin over slices (first minimum wins, init DBL_MAX); idx is absolute (d0+..).  vol: [nd][H][W]
 * slices d0..d0+nd-1.  idx/minc: W*H (may be NULL); Aup/A: [nd][H][W] (may be NULL).
 * OpenMP over slices with nthreads threads (<=0: default). */
void orc_tree_filter(int W, int H, int nd, int d0, int ntrees, const int32_t* tree_start,
                     const int32_t* node_pix, const int32_t* node_parent, const uint16_t* node_w,
                     const uint8_t* node_nch, const int32_t* node_child, const float* vol,
                     int32_t* idx, double* minc, double* Aup, double* A, int nthreads);

/* The S / S2 tables the oracle uses (for tests). */
const double* orc_s_lut(void);
const double* orc_s2_lut(void);

/* AGD color term table a(l1) = 0.11f*fminf((float)(l1*0.33333333333), 7.0f), l1 in [0,765]. */
float orc_agd_color_term(int l1);

/* Stereo3DMST.cpp:632-662 (fill=false, as called at :904): in place on left. */
void orc_lr_check(float* left, const float* right, int W, int H, int max_disp);
/* leftRightConsistencyCheck with the fill step (Stereo3DMST.cpp:632-709), fill = 0 / 1. */
void orc_lr_check_fill(float* left, const float* right, int W, int H, int max_disp, int fill);
/* LabelToDisp of the per-slice label (0, 0, d) and the *= (Dmax-1) scaling (:189-201, 900-902). */
void orc_label_to_disp(float* disp, long n, int dmax);
/* handleOcclusionSharedMemory (PatchMatchStereoGPU.cu:1128-1288), marks computed before the search. */
/* Colour guided filter of a cost volume [nd][H][W] with the view's own BGR image as guide, radius
 * rad, eps (costVolumeColorGuidedFilterCUDA2Streams, PatchMatchStereoGPU.cu:8251-8470; box means of
 * :495-580); OpenMP over slices. */
void orc_guided_filter(const uint8_t* img, int W, int H, int stride, const float* vol, int nd, int rad, float eps,
                       float* out, int nthreads);
/* the reference's box mean of one plane: 32-block sliding sums, x pass then y pass (.cu:495-580) */
void orc_box_mean(const float* in, float* out, int W, int H, int r);
/* selectDisparity (PatchMatchStereoGPU.cu:1688-1737), with the subpixel parabola when sub. */
void orc_select_disparity(const float* vol, int nd, int d0, int dtot, size_t N, int sub, int32_t* idx, float* mn,
                          float* disp);
void orc_occlusion(float* left, float* right, int W, int H, int min_disp, float thresh, int remove);

/* ---- MST_PMS, the slanted-plane label search (Stereo3DMST.cpp:546-629; sm_oracle_pms.c) ---- */
uint32_t orc_minstd0_next(uint32_t s);        /* minstd_rand0 step */
float orc_canon_f(uint32_t u);                /* generate_canonical<float,24> of the shipped libstdc++ */
void orc_pms_dice(long n, float* out);        /* the (-1,1) dice stream every MST_PMS call replays */
void orc_glibc_random(unsigned seed, long skip, long n, int32_t* out); /* glibc random()/rand() */
void orc_pms_init_labels(int W, int H, int max_disp, float* abc);     /* :390-430, abc[3N] */
float orc_label_cost(const float* vol, float a, float b, float c, int pix, int max_disp, int W, size_t N); /* :103-118 */
void orc_pms_label_to_disp(const float* abc, int W, int H, int max_disp, float* disp); /* :189-201 + :900-902 */
void orc_pms_plane_disp(const float* abc, int W, int H, float* disp); /* fma(x, a, y*b) + c, unclamped */
int orc_tree_graph(int W, int H, int ntrees, const int32_t* tree_start, const int32_t* node_pix, int32_t* nb_start,
                   int32_t* nb, int nb_cap);  /* tree_g (:377-384) as CSR, ascending */
long orc_mst_pms(int W, int H, int max_disp, int ntrees, const int32_t* tree_start, const int32_t* node_pix,
                 const int32_t* node_parent, const uint16_t* node_w, const uint8_t* node_nch, const int32_t* node_child,
                 const int32_t* nb_start, const int32_t* nb, const float* vol, float* abc, double* min_cost,
                 const float* dice, long dice_n, const int32_t* rnd, int32_t* stats);

#ifdef __cplusplus
}
#endif
#endif
