/*
 * sm_oracle.c -- TEST INFRASTRUCTURE ONLY (see sm_oracle.h).
 *
 * Plain-C restatement of the reference path, kept deliberately literal:
 * array-of-pixels accumulation exactly as Stereo3DMST.cpp does it, sequential
 * per slice.  Compiled with -ffp-contract=off; every fused multiply-add the
 * shipped binary performs is an explicit fma() here (DESIGN.md "Shipped arithmetic").
 */
#include "sm_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "orc_tables.inc"

const double* orc_s_lut(void) { return SM_S_LUT; }
const double* orc_s2_lut(void) { return SM_S2_LUT; }

/* ------------------------------------------------------------------ median */
#define ORC_CS(a, b) do { const int lo_ = a < b ? a : b, hi_ = a < b ? b : a; a = lo_; b = hi_; } while (0)

static inline int median9(int p0, int p1, int p2, int p3, int p4, int p5, int p6, int p7, int p8) {
    /* exact median of 9 (exchange network; any exact median gives the same value) */
    ORC_CS(p1, p2); ORC_CS(p4, p5); ORC_CS(p7, p8); ORC_CS(p0, p1);
    ORC_CS(p3, p4); ORC_CS(p6, p7); ORC_CS(p1, p2); ORC_CS(p4, p5);
    ORC_CS(p7, p8); ORC_CS(p0, p3); ORC_CS(p5, p8); ORC_CS(p4, p7);
    ORC_CS(p3, p6); ORC_CS(p1, p4); ORC_CS(p2, p5); ORC_CS(p4, p7);
    ORC_CS(p4, p2); ORC_CS(p6, p4); ORC_CS(p4, p2);
    return p4;
}

void orc_median3(const uint8_t* img, int W, int H, int stride, uint8_t* out) {
    /* OpenCV medianBlur ksize 3: replicate border in x and y, exact median of 9. */
    for (int y = 0; y < H; ++y) {
        const uint8_t* r0 = img + (size_t)(y > 0 ? y - 1 : 0) * stride;
        const uint8_t* r1 = img + (size_t)y * stride;
        const uint8_t* r2 = img + (size_t)(y < H - 1 ? y + 1 : H - 1) * stride;
        for (int x = 0; x < W; ++x) {
            const int j0 = 3 * (x > 0 ? x - 1 : 0), j1 = 3 * x, j2 = 3 * (x < W - 1 ? x + 1 : W - 1);
            for (int c = 0; c < 3; ++c)
                out[((size_t)y * W + x) * 3 + c] = (uint8_t)median9(r0[j0 + c], r0[j1 + c], r0[j2 + c], r1[j0 + c],
                                                                    r1[j1 + c], r1[j2 + c], r2[j0 + c], r2[j1 + c],
                                                                    r2[j2 + c]);
        }
    }
}

/* ------------------------------------------------------------------ edges */
void orc_edge_weights(const uint8_t* med, int W, int H, uint16_t* wR, uint16_t* wD) {
    /* diff(): double differences of integer-valued planes, abs, summed r+g+b -> integer. */
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const size_t p = (size_t)y * W + x;
            const uint8_t* a = med + 3 * p;
            if (x < W - 1) {
                const uint8_t* b = a + 3;
                wR[p] = (uint16_t)(abs(a[2] - b[2]) + abs(a[1] - b[1]) + abs(a[0] - b[0]));
            } else {
                wR[p] = 0xFFFF;
            }
            if (y < H - 1) {
                const uint8_t* b = a + 3 * (size_t)W;
                wD[p] = (uint16_t)(abs(a[2] - b[2]) + abs(a[1] - b[1]) + abs(a[0] - b[0]));
            } else {
                wD[p] = 0xFFFF;
            }
        }
}

/* ------------------------------------------------------------------ union-find */
typedef struct { int rank, p, size; } uelt;

static int uf_find(uelt* e, int x) {
    int y = x;
    while (y != e[y].p) y = e[y].p;
    e[x].p = y;
    return y;
}

static void uf_join(uelt* e, int x, int y) {
    if (e[x].rank > e[y].rank) {
        e[y].p = x;
        e[x].size += e[y].size;
    } else {
        e[x].p = y;
        e[y].size += e[x].size;
        if (e[x].rank == e[y].rank) e[y].rank++;
    }
}

/* Edge emission order of Stereo3DMST.cpp:244-262 is ascending (a, b): for each pixel the
 * right edge (b=a+1) then the down edge (b=a+W).  A stable counting sort by w therefore
 * yields exactly std::sort's (w, a, b) order (include/segment-graph.h:34-42, 57). */
typedef struct { int a, b; uint16_t w; uint8_t dir; } orc_edge;

static orc_edge* sorted_edges(int W, int H, const uint16_t* wR, const uint16_t* wD, int* num_out) {
    const int N = W * H;
    int num = 0;
    int* count = (int*)calloc(SM_NUM_WEIGHTS + 1, sizeof(int));
    for (int p = 0; p < N; ++p) {
        const int x = p % W, y = p / W;
        if (x < W - 1) { count[wR[p] + 1]++; num++; }
        if (y < H - 1) { count[wD[p] + 1]++; num++; }
    }
    for (int i = 0; i < SM_NUM_WEIGHTS; ++i) count[i + 1] += count[i];
    orc_edge* e = (orc_edge*)malloc(sizeof(orc_edge) * (size_t)(num > 0 ? num : 1));
    for (int p = 0; p < N; ++p) {
        const int x = p % W, y = p / W;
        if (x < W - 1) { orc_edge t = {p, p + 1, wR[p], 0}; e[count[wR[p]]++] = t; }
        if (y < H - 1) { orc_edge t = {p, p + W, wD[p], 1}; e[count[wD[p]]++] = t; }
    }
    free(count);
    *num_out = num;
    return e;
}

int orc_segment(int W, int H, const uint16_t* wR, const uint16_t* wD, float c, int min_size, uint8_t* mask) {
    const int N = W * H;
    int num;
    orc_edge* e = sorted_edges(W, H, wR, wD, &num);
    uelt* u = (uelt*)malloc(sizeof(uelt) * (size_t)N);
    double* thr = (double*)malloc(sizeof(double) * (size_t)N);
    for (int i = 0; i < N; ++i) { u[i].rank = 0; u[i].size = 1; u[i].p = i; thr[i] = (double)(c / 1.0f); }
    memset(mask, 0, (size_t)N);
    int nsets = N;
    /* segment_graph: THRESHOLD(size,c) = c/size evaluated in float, added to a double w. */
    for (int i = 0; i < num; ++i) {
        int a = uf_find(u, e[i].a), b = uf_find(u, e[i].b);
        if (a != b) {
            const double w = (double)e[i].w;
            if (w <= thr[a] && w <= thr[b]) {
                uf_join(u, a, b);
                nsets--;
                a = uf_find(u, a);
                thr[a] = w + (double)(c / (float)u[a].size);
                mask[e[i].a] |= e[i].dir ? ORC_EDGE_DOWN : ORC_EDGE_RIGHT;
            }
        }
    }
    /* min-size merge, Stereo3DMST.cpp:293-307 (a no-op in MST mode: one component).
     * min_size < 0 skips it (oracle-only switch, to compare bare segment_graph output). */
    const int do_merge = min_size >= 0;
    if (min_size < 2) min_size = 2;
    for (int i = 0; do_merge && i < num; ++i) {
        int a = uf_find(u, e[i].a), b = uf_find(u, e[i].b);
        if (a != b && (u[a].size < min_size || u[b].size < min_size)) {
            uf_join(u, a, b);
            nsets--;
            mask[e[i].a] |= e[i].dir ? ORC_EDGE_DOWN : ORC_EDGE_RIGHT;
        }
    }
    free(thr);
    free(u);
    free(e);
    return nsets;
}

/* ------------------------------------------------------------------ BFS rooting */
static inline uint64_t edge_key(int W, int p, int k, const uint16_t* wR, const uint16_t* wD) {
    /* (w, a, b) order as a 64-bit key: b is a+1 (right) or a+W (down), so (w, a, dir). */
    int a, vert;
    uint16_t w;
    switch (k) {
        case 0: a = p; vert = 0; w = wR[p]; break;          /* right */
        case 1: a = p; vert = 1; w = wD[p]; break;          /* down  */
        case 2: a = p - 1; vert = 0; w = wR[p - 1]; break;  /* left  */
        default: a = p - W; vert = 1; w = wD[p - W]; break; /* up    */
    }
    return ((uint64_t)w << 33) | ((uint64_t)a << 1) | (uint64_t)vert;
}

static int mst_neighbors(int W, int p, const uint8_t* mask, int* nb, int* dir) {
    int n = 0;
    if (mask[p] & ORC_EDGE_RIGHT) { nb[n] = p + 1; dir[n++] = 0; }
    if (mask[p] & ORC_EDGE_DOWN) { nb[n] = p + W; dir[n++] = 1; }
    if ((p % W) > 0 && (mask[p - 1] & ORC_EDGE_RIGHT)) { nb[n] = p - 1; dir[n++] = 2; }
    if (p >= W && (mask[p - W] & ORC_EDGE_DOWN)) { nb[n] = p - W; dir[n++] = 3; }
    return n;
}

int orc_bfs(int W, int H, const uint16_t* wR, const uint16_t* wD, const uint8_t* mask,
            int32_t* tree_start, int32_t* node_pix, int32_t* node_parent, uint16_t* node_w,
            uint8_t* node_nch, int32_t* node_child) {
    const int N = W * H;
    /* components of the mask forest, numbered by first raster appearance (:352-369) */
    uelt* u = (uelt*)malloc(sizeof(uelt) * (size_t)N);
    for (int i = 0; i < N; ++i) { u[i].rank = 0; u[i].size = 1; u[i].p = i; }
    for (int p = 0; p < N; ++p) {
        if (mask[p] & ORC_EDGE_RIGHT) { int a = uf_find(u, p), b = uf_find(u, p + 1); if (a != b) uf_join(u, a, b); }
        if (mask[p] & ORC_EDGE_DOWN) { int a = uf_find(u, p), b = uf_find(u, p + W); if (a != b) uf_join(u, a, b); }
    }
    int* cc_of_rep = (int*)malloc(sizeof(int) * (size_t)N);
    for (int i = 0; i < N; ++i) cc_of_rep[i] = -1;
    int* cc = (int*)malloc(sizeof(int) * (size_t)N);
    int* tsize = (int*)calloc((size_t)N + 1, sizeof(int));
    int ntrees = 0;
    int* root_pix = (int*)malloc(sizeof(int) * (size_t)N);
    for (int p = 0; p < N; ++p) {
        const int r = uf_find(u, p);
        if (cc_of_rep[r] < 0) { cc_of_rep[r] = ntrees; root_pix[ntrees] = p; ntrees++; }
        cc[p] = cc_of_rep[r];
        tsize[cc[p]]++;
    }
    tree_start[0] = 0;
    for (int t = 0; t < ntrees; ++t) tree_start[t + 1] = tree_start[t] + tsize[t];
    /* BFS per tree (:450-522): queue order = new ids; children in ascending edge key */
    int* node_of_pix = (int*)malloc(sizeof(int) * (size_t)N);
    for (int i = 0; i < N; ++i) node_of_pix[i] = -1;
    for (int t = 0; t < ntrees; ++t) {
        int head = tree_start[t], tail = tree_start[t];
        const int root = root_pix[t];
        node_pix[tail] = root;
        node_parent[tail] = tail;
        node_w[tail] = 0;
        node_of_pix[root] = tail;
        tail++;
        while (head < tail) {
            const int n = head++;
            const int p = node_pix[n];
            int nb[4], dr[4];
            const int k = mst_neighbors(W, p, mask, nb, dr);
            uint64_t key[4];
            int ord[4];
            for (int i = 0; i < k; ++i) { key[i] = edge_key(W, p, dr[i], wR, wD); ord[i] = i; }
            for (int i = 1; i < k; ++i) /* insertion sort, ascending key */
                for (int j = i; j > 0 && key[ord[j]] < key[ord[j - 1]]; --j) { int s = ord[j]; ord[j] = ord[j - 1]; ord[j - 1] = s; }
            int nch = 0;
            for (int i = 0; i < k; ++i) {
                const int q = nb[ord[i]];
                if (node_of_pix[q] >= 0) continue; /* the parent (already coloured) */
                node_pix[tail] = q;
                node_parent[tail] = n;
                node_w[tail] = (uint16_t)(key[ord[i]] >> 33);
                node_of_pix[q] = tail;
                node_child[4 * n + nch++] = tail;
                tail++;
            }
            node_nch[n] = (uint8_t)nch;
            for (int i = nch; i < 4; ++i) node_child[4 * n + i] = -1;
        }
    }
    free(node_of_pix);
    free(root_pix);
    free(tsize);
    free(cc);
    free(cc_of_rep);
    free(u);
    return ntrees;
}

/* ------------------------------------------------------------------ AGD cost */
float orc_agd_color_term(int l1) {
    /* 0.11f*fminf(color_l1*0.33333333333, 7.0f): the product is double (double literal),
     * fminf converts it to float (PatchMatchStereoGPU.cu:1539). */
    const float scaled = (float)((double)(float)l1 * 0.33333333333);
    return 0.11f * fminf(scaled, 7.0f);
}

/* Contraction variant (oracle-only switch, DESIGN.md "AGD contraction"): 0 = the shipped restatement,
 * no contraction; 1 = what an LLVM-based CUDA compiler with --fmad=true (nvcc's default; the
 * reference's CMakeLists.txt:19-20 sets no --fmad) forms from the same expressions:
 * a*b + c*d -> fma(a, b, c*d) and (..) + e*f -> fma(e, f, ..). */
static int g_agd_contract = 0;
void orc_set_agd_contract(int mode) { g_agd_contract = mode; }

static inline float gray_of(const uint8_t* bgr) {
    /* 0.114f*B + 0.587f*G + 0.299f*R, left-to-right, no contraction (:1529-1530) */
    const float b = (float)bgr[0], g = (float)bgr[1], r = (float)bgr[2];
    if (g_agd_contract) return fmaf(0.299f, r, fmaf(0.114f, b, 0.587f * g));
    float t = 0.114f * b;
    t = t + 0.587f * g;
    t = t + 0.299f * r;
    return t;
}

static inline float agd_cost(const uint8_t* r0, const uint8_t* l0) {
    /* r0 = right(x), r0+3 = right(x+1); l0 = left(x+d), l0+3 = left(x+d+1) (:1518-1540) */
    float color_l1 = 0.0f;
    for (int i = 0; i < 3; ++i) color_l1 += fabsf((float)r0[i] - (float)l0[i]);
    float ref_gray = gray_of(r0), match_gray = gray_of(l0);
    float g = match_gray - ref_gray;
    ref_gray = gray_of(r0 + 3);
    match_gray = gray_of(l0 + 3);
    g += ref_gray - match_gray;
    const float x = fminf((float)((double)color_l1 * 0.33333333333), 7.0f);
    const float y = fminf(fabsf(g), 2.0f);
    if (g_agd_contract) return 0.f + fmaf(0.11f, x, 0.89f * y);
    const float a = 0.11f * x;
    const float b = 0.89f * y;
    float cost = 0.f;
    cost += a + b;
    return cost;
}

void orc_cost_agd(const uint8_t* left, const uint8_t* right, int W, int H, int stride, int d0, int d1,
                  float* left_vol, float* right_vol, int nthreads) {
    /* slices are independent: OpenMP over d (nthreads <= 0: the OpenMP default) */
    const size_t N = (size_t)W * H;
#ifdef _OPENMP
    const int nt = nthreads > 0 ? nthreads : omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(nt)
#else
    (void)nthreads;
#endif
    for (int d = d0; d < d1; ++d) {
        float* rv = right_vol ? right_vol + (size_t)(d - d0) * N : NULL;
        float* lv = left_vol ? left_vol + (size_t)(d - d0) * N : NULL;
        for (int y = 0; y < H; ++y) {
            const uint8_t* rrow = right + (size_t)y * stride;
            const uint8_t* lrow = left + (size_t)y * stride;
            if (lv) for (int x = 0; x < W; ++x) lv[(size_t)y * W + x] = 3.0f; /* x<d and column W-1 */
            for (int x = 0; x < W; ++x) {
                const size_t p = (size_t)y * W + x;
                if (d + x + 1 < W) {
                    const float c = agd_cost(rrow + 3 * x, lrow + 3 * (x + d));
                    if (rv) rv[p] = c;
                    if (lv) lv[p + d] = c;
                } else if (rv) {
                    rv[p] = 3.0f;
                }
            }
        }
    }
}

/* ------------------------------------------------------------------ tree filter */
void orc_tree_filter(int W, int H, int nd, int d0, int ntrees, const int32_t* tree_start,
                     const int32_t* node_pix, const int32_t* node_parent, const uint16_t* node_w,
                     const uint8_t* node_nch, const int32_t* node_child, const float* vol,
                     int32_t* idx, double* minc, double* Aup, double* A, int nthreads) {
    const size_t N = (size_t)W * H;
    int nt = 1;
#ifdef _OPENMP
    nt = nthreads > 0 ? nthreads : omp_get_max_threads();
    if (nt > nd) nt = nd;
    if (nt < 1) nt = 1;
#else
    (void)nthreads;
#endif
    /* per-thread partial argmin over a contiguous block of slices; merged in block order,
     * which preserves the strict-< / first-minimum rule of Stereo3DMST.cpp:177. */
    double* pmin = NULL;
    int32_t* pidx = NULL;
    if (idx || minc) {
        pmin = (double*)malloc(sizeof(double) * N * (size_t)nt);
        pidx = (int32_t*)malloc(sizeof(int32_t) * N * (size_t)nt);
    }
#pragma omp parallel num_threads(nt)
    {
        int tid = 0;
#ifdef _OPENMP
        tid = omp_get_thread_num();
#endif
        const int dbeg = (int)((long)nd * tid / nt), dend = (int)((long)nd * (tid + 1) / nt);
        double* agg = (double*)malloc(sizeof(double) * N);
        double* my_min = pmin ? pmin + N * (size_t)tid : NULL;
        int32_t* my_idx = pidx ? pidx + N * (size_t)tid : NULL;
        if (my_min) for (size_t p = 0; p < N; ++p) { my_min[p] = DBL_MAX; my_idx[p] = 0; }
        for (int dl = dbeg; dl < dend; ++dl) {
            const float* C = vol + (size_t)dl * N;
            for (int t = 0; t < ntrees; ++t) {
                const int ts = tree_start[t], te = tree_start[t + 1];
                for (int n = ts; n < te; ++n) agg[node_pix[n]] = 0.0;                 /* :165 */
                for (int n = te - 1; n > ts; --n) {                                    /* :125-135 */
                    const int pix = node_pix[n], ppix = node_pix[node_parent[n]];
                    agg[pix] = agg[pix] + (double)C[pix];
                    agg[ppix] = fma(SM_S_LUT[node_w[n]], agg[pix], agg[ppix]);
                }
                agg[node_pix[ts]] = agg[node_pix[ts]] + (double)C[node_pix[ts]];    /* :137 */
                if (Aup) for (int n = ts; n < te; ++n) Aup[(size_t)dl * N + node_pix[n]] = agg[node_pix[n]];
                for (int n = ts; n < te; ++n) {                                        /* :145-157 */
                    const int p = node_pix[n];
                    for (int i = 0; i < node_nch[n]; ++i) {
                        const int c = node_child[4 * n + i];
                        const int cp = node_pix[c];
                        agg[cp] = fma(SM_S_LUT[node_w[c]], agg[p], SM_S2_LUT[node_w[c]] * agg[cp]);
                    }
                }
            }
            if (A) memcpy(A + (size_t)dl * N, agg, sizeof(double) * N);
            if (my_min)
                for (size_t p = 0; p < N; ++p)
                    if (agg[p] < my_min[p]) { my_min[p] = agg[p]; my_idx[p] = d0 + dl; } /* :177 strict < */
        }
        free(agg);
    }
    if (pmin) {
        for (size_t p = 0; p < N; ++p) {
            double best = DBL_MAX;
            int32_t bi = 0;
            for (int t = 0; t < nt; ++t)
                if (pmin[N * (size_t)t + p] < best) { best = pmin[N * (size_t)t + p]; bi = pidx[N * (size_t)t + p]; }
            if (idx) idx[p] = bi;
            if (minc) minc[p] = best;
        }
        free(pmin);
        free(pidx);
    }
}

/* LabelToDisp (Stereo3DMST.cpp:189-201) of the per-slice label a = b = 0, c = d:
 * MAX(0.0f, min(1.0f, (x*a + y*b + c)/(max_disp-1.0f))), x*0 + y*0 + d == d exactly; then
 * leftDisp *= (Dmax-1.f) (:900-902), OpenCV convertTo with scale: one float multiply. */
void orc_label_to_disp(float* disp, long n, int dmax) {
    const float dm1 = (float)dmax - 1.0f;
    for (long i = 0; i < n; ++i) {
        float v = disp[i] / dm1;
        v = (v < 1.0f) ? v : 1.0f;  /* std::min(1.0f, v) */
        v = (0.0f < v) ? v : 0.0f;  /* MAX(0.0f, v) (OpenCV: a < b ? b : a) */
        disp[i] = v * dm1;
    }
}

/* Left-right consistency check (Stereo3DMST.cpp:632-709), literal: d = round(left); a pixel with
 * x-d < 0, d < 0, d >= max_disp or |left - right(x-d)| > 1 becomes 0 and is masked (:642-662);
 * with fill, each row is walked left to right: a masked pixel copies the nearest pixel to its left
 * whose mask is 0 and clears its mask, then takes the nearest mask-0 pixel to its right if that is
 * smaller or if its own mask is still 1 (:664-709).  Rows are independent (the OpenMP loop is over
 * y), so the serial loop equals the reference. */
void orc_lr_check_fill(float* left, const float* right, int W, int H, int max_disp, int fill) {
    unsigned char* mask = (unsigned char*)calloc((size_t)W * H, 1);
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const long idx = (long)y * W + x;
            const float df = left[idx];
            const int d = (int)roundf(df);
            if (x - d >= 0 && d >= 0 && d < max_disp) {
                if (fabsf(df - right[idx - d]) > 1.0f) { mask[idx] = 1; left[idx] = 0.0f; }
            } else {
                mask[idx] = 1;
                left[idx] = 0.0f;
            }
        }
    if (fill) {
        for (int y = 0; y < H; ++y)
            for (int x = 0; x < W; ++x) {
                const long idx = (long)y * W + x;
                if (mask[idx] == 0) continue;
                for (int i = 1; x - i >= 0; ++i)
                    if (mask[idx - i] == 0) { left[idx] = left[idx - i]; mask[idx] = 0; break; }
                for (int i = 1; x + i < W; ++i)
                    if (mask[idx + i] == 0) {
                        if (left[idx + i] < left[idx] || mask[idx] == 1) left[idx] = left[idx + i];
                        break;
                    }
            }
    }
    free(mask);
}

void orc_lr_check(float* left, const float* right, int W, int H, int max_disp) {
    orc_lr_check_fill(left, right, W, H, max_disp, 0); /* as called at :904 */
}

/* handleOcclusionSharedMemory (PatchMatchStereoGPU.cu:1128-1288), literal per row with the copy
 * tile: marks (1e18f) are written into the copies for both maps first (the race-free reading of
 * the kernel, which has no barrier between marking and searching), then every marked pixel is
 * set to min_disp (remove) or to fminf of the nearest unmarked ORIGINAL values to its left and
 * right (1e18f when absent; 255 when both are absent). */
void orc_occlusion(float* left, float* right, int W, int H, int min_disp, float thresh, int remove) {
    const float inv = 1e18f;
    float* t = (float*)malloc(sizeof(float) * 4 * (size_t)W);
    for (int y = 0; y < H; ++y) {
        float* L = left + (size_t)y * W;
        float* R = right + (size_t)y * W;
        for (int x = 0; x < W; ++x) { t[x] = L[x]; t[x + W] = R[x]; t[x + 2 * W] = L[x]; t[x + 3 * W] = R[x]; }
        for (int x = 0; x < W; ++x) {
            int right_x = (int)((float)x - t[x]);
            int left_x = x;
            if ((right_x >= 0 && fabsf(t[right_x + W] - t[left_x]) > thresh) || right_x < 0) t[left_x + 2 * W] = inv;
            left_x = (int)((float)x + t[x + W]);
            right_x = x;
            if ((left_x < W && fabsf(t[right_x + W] - t[left_x]) > thresh) || left_x >= W) t[right_x + 3 * W] = inv;
        }
        for (int x = 0; x < W; ++x) {
            if (remove) {
                if (t[x + 2 * W] == inv) L[x] = (float)min_disp;
                if (t[x + 3 * W] == inv) R[x] = (float)min_disp;
                continue;
            }
            for (int v = 0; v < 2; ++v) {
                const float* orig = t + v * W;
                const float* marks = t + (2 + v) * W;
                float* out = v ? R : L;
                if (marks[x] != inv) continue;
                float ls = inv, rs = inv;
                for (int q = x - 1; q >= 0; --q) if (marks[q] != inv) { ls = orig[q]; break; }
                for (int q = x + 1; q < W; ++q) if (marks[q] != inv) { rs = orig[q]; break; }
                out[x] = (ls == inv && rs == inv) ? 255.f : fminf(ls, rs);
            }
        }
    }
    free(t);
}

/* ------------------------------------------------------------------ guided-filter aggregation */
/* Sliding box mean of radius r (boxFilter_x_global_shared / boxFilter_y_global,
 * PatchMatchStereoGPU.cu:495-580): the running sum restarts at every 32-pixel block (the kernels'
 * block width), starts as sum_{i=x0-r}^{x0+r} in ascending i (0 outside the image), then slides
 * t += in[x+r]; t -= in[x-r-1] (0 outside); out = t * (1.0f/(2r+1)). */
#define ORC_GF_BLOCK 32
static void orc_box_x(const float* in, float* out, int W, int H, int r) {
    const float scale = 1.0f / (float)((r << 1) + 1);
    for (int y = 0; y < H; ++y) {
        const float* row = in + (size_t)y * W;
        float* o = out + (size_t)y * W;
        for (int x0 = 0; x0 < W; x0 += ORC_GF_BLOCK) {
            float t = 0.0f;
            for (int i = x0 - r; i <= x0 + r; ++i) t += (i < 0 || i >= W) ? 0.0f : row[i];
            o[x0] = t * scale;
            const int end = W - x0 < ORC_GF_BLOCK ? W : x0 + ORC_GF_BLOCK;
            for (int x = x0 + 1; x < end; ++x) {
                t += (x + r >= W) ? 0.0f : row[x + r];
                t -= (x - r - 1 < 0) ? 0.0f : row[x - r - 1];
                o[x] = t * scale;
            }
        }
    }
}

static void orc_box_y(const float* in, float* out, int W, int H, int r) {
    const float scale = 1.0f / (float)((r << 1) + 1);
    for (int x = 0; x < W; ++x)
        for (int y0 = 0; y0 < H; y0 += ORC_GF_BLOCK) {
            float t = 0.0f;
            for (int i = y0 - r; i <= y0 + r; ++i) t += (i < 0 || i >= H) ? 0.0f : in[(size_t)i * W + x];
            out[(size_t)y0 * W + x] = t * scale;
            const int end = H - y0 < ORC_GF_BLOCK ? H : y0 + ORC_GF_BLOCK;
            for (int y = y0 + 1; y < end; ++y) {
                t += (y + r >= H) ? 0.0f : in[(size_t)(y + r) * W + x];
                t -= (y - r - 1 < 0) ? 0.0f : in[(size_t)(y - r - 1) * W + x];
                out[(size_t)y * W + x] = t * scale;
            }
        }
}

static void orc_box(const float* in, float* out, float* tmp, int W, int H, int r) {
    orc_box_x(in, tmp, W, H, r);
    orc_box_y(tmp, out, W, H, r);
}

/* Colour guided filter of one cost slice p with guide planes (r, g, b) -- the per-pixel steps of
 * costVolumeColorGuidedFilterCUDA2Streams (PatchMatchStereoGPU.cu:8251-8470) in source order,
 * no contraction: the guide statistics st[] (mean_r, mean_g, mean_b, inv_rr, inv_rg, inv_rb,
 * inv_gg, inv_gb, inv_bb; see orc_gf_guide) are precomputed. */
/* g_gf_contract = 1: the helper kernels' a*b +/- c*d chains as nvcc's default --fmad=true would
 * contract them (the first product of a sum fused, each later product fused into the running sum;
 * the convention of orc_set_agd_contract) -- a what-if for tools/gf_contraction.py, never the
 * shipped arithmetic */
static int g_gf_contract = 0;
void orc_set_gf_contract(int mode) { g_gf_contract = mode; }

static void orc_gf_slice(const float* p, const float* gr, const float* gg, const float* gb, const float* const* st,
                         int W, int H, int rad, float* q, float* w /* 12 planes of N */) {
    const size_t N = (size_t)W * H;
    float *mp = w, *mr = w + N, *mg = w + 2 * N, *mb = w + 3 * N, *t = w + 4 * N, *ar = w + 5 * N, *ag = w + 6 * N,
          *ab = w + 7 * N, *bb = w + 8 * N, *x = w + 9 * N;
    orc_box(p, mp, t, W, H, rad);                               /* mean_p */
    for (size_t i = 0; i < N; ++i) x[i] = gr[i] * p[i];
    orc_box(x, mr, t, W, H, rad);                               /* mean_I_r = box(r .* p) */
    for (size_t i = 0; i < N; ++i) x[i] = gg[i] * p[i];
    orc_box(x, mg, t, W, H, rad);
    for (size_t i = 0; i < N; ++i) x[i] = gb[i] * p[i];
    orc_box(x, mb, t, W, H, rad);
    const float *m_r = st[0], *m_g = st[1], *m_b = st[2];
    const float *irr = st[3], *irg = st[4], *irb = st[5], *igg = st[6], *igb = st[7], *ibb = st[8];
    for (size_t i = 0; i < N; ++i) {
        if (g_gf_contract) {
            const float cr = fmaf(-m_r[i], mp[i], mr[i]), cg = fmaf(-m_g[i], mp[i], mg[i]), cb = fmaf(-m_b[i], mp[i], mb[i]);
            ar[i] = fmaf(irb[i], cb, fmaf(irr[i], cr, irg[i] * cg));
            ag[i] = fmaf(igb[i], cb, fmaf(irg[i], cr, igg[i] * cg));
            ab[i] = fmaf(ibb[i], cb, fmaf(irb[i], cr, igb[i] * cg));
            bb[i] = fmaf(-ab[i], m_b[i], fmaf(-ag[i], m_g[i], fmaf(-ar[i], m_r[i], mp[i])));
            continue;
        }
        const float cr = mr[i] - m_r[i] * mp[i];                /* Helper3: s1 - s2*s3 */
        const float cg = mg[i] - m_g[i] * mp[i];
        const float cb = mb[i] - m_b[i] * mp[i];
        ar[i] = irr[i] * cr + irg[i] * cg + irb[i] * cb;        /* Helper2 */
        ag[i] = irg[i] * cr + igg[i] * cg + igb[i] * cb;
        ab[i] = irb[i] * cr + igb[i] * cg + ibb[i] * cb;
        bb[i] = mp[i] - ar[i] * m_r[i] - ag[i] * m_g[i] - ab[i] * m_b[i];  /* Helper4 */
    }
    orc_box(ar, mr, t, W, H, rad);
    orc_box(ag, mg, t, W, H, rad);
    orc_box(ab, mb, t, W, H, rad);
    orc_box(bb, x, t, W, H, rad);
    for (size_t i = 0; i < N; ++i)                                   /* Helper5 */
        q[i] = g_gf_contract ? fmaf(mb[i], gb[i], fmaf(mg[i], gg[i], fmaf(mr[i], gr[i], x[i])))
                             : x[i] + mr[i] * gr[i] + mg[i] * gg[i] + mb[i] * gb[i];
}

/* guide statistics of one view (PatchMatchStereoGPU.cu:8261-8420), eps added to the diagonal */
static void orc_gf_guide(const float* gr, const float* gg, const float* gb, int W, int H, int rad, float eps, float** st,
                         float* w /* 4 planes */) {
    const size_t N = (size_t)W * H;
    float *t = w, *x = w + N, *m = w + 2 * N;
    float *vrr = malloc(sizeof(float) * N), *vgg = malloc(sizeof(float) * N), *vbb = malloc(sizeof(float) * N);
    float *vrg = malloc(sizeof(float) * N), *vrb = malloc(sizeof(float) * N), *vgb = malloc(sizeof(float) * N);
    orc_box(gr, st[0], t, W, H, rad);
    orc_box(gg, st[1], t, W, H, rad);
    orc_box(gb, st[2], t, W, H, rad);
    const float* pl[3] = {gr, gg, gb};
    float* var[6] = {vrr, vgg, vbb, vrg, vrb, vgb};
    const int pa[6] = {0, 1, 2, 0, 0, 1}, pb[6] = {0, 1, 2, 1, 2, 2};
    for (int k = 0; k < 6; ++k) {
        for (size_t i = 0; i < N; ++i) x[i] = pl[pa[k]][i] * pl[pb[k]][i];
        orc_box(x, m, t, W, H, rad);
        for (size_t i = 0; i < N; ++i) {
            const float mm = st[pa[k]][i] * st[pb[k]][i];
            var[k][i] = k < 3 ? m[i] - mm + eps : m[i] - mm;      /* Helper0 */
        }
    }
    for (size_t i = 0; i < N; ++i) {                              /* Helper1 ... */
        if (g_gf_contract) {
            const float irr = fmaf(vgg[i], vbb[i], -(vgb[i] * vgb[i])), igg = fmaf(vrr[i], vbb[i], -(vrb[i] * vrb[i]));
            const float ibb = fmaf(vrr[i], vgg[i], -(vrg[i] * vrg[i])), irg = fmaf(vgb[i], vrb[i], -(vrg[i] * vbb[i]));
            const float irb = fmaf(vrg[i], vgb[i], -(vgg[i] * vrb[i])), igb = fmaf(vrb[i], vrg[i], -(vrr[i] * vgb[i]));
            const float det = fmaf(irb, vrb[i], fmaf(irr, vrr[i], irg * vrg[i]));
            st[3][i] = irr / det;
            st[4][i] = irg / det;
            st[5][i] = irb / det;
            st[6][i] = igg / det;
            st[7][i] = igb / det;
            st[8][i] = ibb / det;
            continue;
        }
        float irr = vgg[i] * vbb[i] - vgb[i] * vgb[i];
        float igg = vrr[i] * vbb[i] - vrb[i] * vrb[i];
        float ibb = vrr[i] * vgg[i] - vrg[i] * vrg[i];
        float irg = vgb[i] * vrb[i] - vrg[i] * vbb[i];
        float irb = vrg[i] * vgb[i] - vgg[i] * vrb[i];
        float igb = vrb[i] * vrg[i] - vrr[i] * vgb[i];
        const float det = irr * vrr[i] + irg * vrg[i] + irb * vrb[i];  /* Helper2 */
        st[3][i] = irr / det;
        st[4][i] = irg / det;
        st[5][i] = irb / det;
        st[6][i] = igg / det;
        st[7][i] = igb / det;
        st[8][i] = ibb / det;
    }
    free(vrr); free(vgg); free(vbb); free(vrg); free(vrb); free(vgb);
}

void orc_guided_filter(const uint8_t* img, int W, int H, int stride, const float* vol, int nd, int rad, float eps,
                       float* out, int nthreads) {
    const size_t N = (size_t)W * H;
    float* g3 = malloc(sizeof(float) * 3 * N);
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const uint8_t* px = img + (size_t)y * stride + 3 * x;
            g3[(size_t)y * W + x] = (float)px[2];          /* r */
            g3[N + (size_t)y * W + x] = (float)px[1];      /* g */
            g3[2 * N + (size_t)y * W + x] = (float)px[0];  /* b */
        }
    float* stb = malloc(sizeof(float) * 9 * N);
    float* st[9];
    for (int k = 0; k < 9; ++k) st[k] = stb + k * N;
    float* w0 = malloc(sizeof(float) * 3 * N);
    orc_gf_guide(g3, g3 + N, g3 + 2 * N, W, H, rad, eps, st, w0);
    free(w0);
    int nt = 1;
#ifdef _OPENMP
    nt = nthreads > 0 ? nthreads : omp_get_max_threads();
#else
    (void)nthreads;
#endif
#pragma omp parallel num_threads(nt)
    {
        float* w = malloc(sizeof(float) * 10 * N);
#pragma omp for schedule(dynamic, 1)
        for (int d = 0; d < nd; ++d)
            orc_gf_slice(vol + (size_t)d * N, g3, g3 + N, g3 + 2 * N, (const float* const*)st, W, H, rad, out + (size_t)d * N, w);
        free(w);
    }
    free(stb);
    free(g3);
}

/* selectDisparity (PatchMatchStereoGPU.cu:1688-1737) on a float volume of slices d0..: strict <
 * from 1e10f over ascending d; no minimum -> disp 0 (idx 0); with sub the parabola through the
 * neighbouring slices (0 at the ends of [0, dtot)). */
void orc_select_disparity(const float* vol, int nd, int d0, int dtot, size_t N, int sub, int32_t* idx, float* mn,
                          float* disp) {
    for (size_t p = 0; p < N; ++p) {
        float m = 1e10f;
        int best = -1;
        for (int d = 0; d < nd; ++d) {
            const float c = vol[(size_t)d * N + p];
            if (c < m) { m = c; best = d; }
        }
        if (best < 0) {
            idx[p] = 0;
            mn[p] = m;
            disp[p] = 0.0f;
            continue;
        }
        const int g = d0 + best;
        idx[p] = g;
        mn[p] = m;
        float dd = (float)g;
        if (sub) {
            const float pre = g == 0 ? 0.0f : vol[(size_t)(best - 1) * N + p];
            const float cur = vol[(size_t)best * N + p];
            const float nxt = g == dtot - 1 ? 0.0f : vol[(size_t)(best + 1) * N + p];
            const float s = (nxt - pre) * 0.5f / (nxt - 2.0f * cur + pre);
            if (fabsf(s) < 1.0f) dd = (float)g - s;
        }
        disp[p] = dd;
    }
}

/* box mean of one plane (x pass, then y pass): test access to orc_box */
void orc_box_mean(const float* in, float* out, int W, int H, int r) {
    float* t = malloc(sizeof(float) * (size_t)W * H);
    orc_box(in, out, t, W, H, r);
    free(t);
}
