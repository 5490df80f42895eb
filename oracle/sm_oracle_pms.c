/*
 * sm_oracle_pms.c -- TEST INFRASTRUCTURE ONLY (see sm_oracle.h).
 *
 * Restatement of Stereo3DMST's slanted-plane label search, MST_PMS (src/Stereo3DMST.cpp:546-629),
 * with its random plane init (:388-430), its lerp data term (compute3DLabelCost, :103-118), the
 * per-label tree aggregation + strict-< update (MSTCostAggregationAndLabelUpdate, :160-186) and
 * LabelToDisp (:189-201).  Serial, in the reference's tree order: the shipped StereoYin was linked
 * without OpenMP, so this is the order it ran in.
 *
 * Float arithmetic follows the shipped binary (build/StereoYin, GCC 5.4 -O3 -march=native, read
 * with objdump only; DESIGN.md "MST_PMS arithmetic"): every vfmadd it performs is an explicit fmaf /
 * fma here, everything else is compiled with -ffp-contract=off.
 *
 * Random streams (third-party published algorithms, pinned against this container's libc/libstdc++
 * by tests/golden/make_rng_golden.py):
 *  - std::default_random_engine = minstd_rand0 (x <- 16807 x mod 2^31-1, seed 1; the mangled
 *    MST_PMS signature names linear_congruential_engine<unsigned long,16807,0,2147483647>);
 *  - std::uniform_real_distribution<float>(a, b) over it, GCC 5.4's generate_canonical<float,24>:
 *    one engine call, (float)(u - 1) * 2^-31 (no clamp below 1 in the shipped code), then
 *    fma(r, b - a, a);
 *  - glibc random()/rand() (TYPE_3 additive feedback, seed 1): random_rgb draws 3 per pixel per
 *    view (:72-80, :316) before any MST_PMS call, then rand() once per tree (:584).
 */
#include "sm_oracle.h"

#include <float.h>
#include <limits.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "orc_tables.inc"

/* ------------------------------------------------------------------ random streams */
uint32_t orc_minstd0_next(uint32_t s) { return (uint32_t)(((uint64_t)s * 16807u) % 2147483647u); }

/* generate_canonical<float, 24>(minstd_rand0) of the shipped libstdc++: k = 1 engine call,
 * sum = (float)(u - min), tmp = (float)(max - min + 1) = 2^31; the division is a multiply by 2^-31
 * in the binary (exact), and there is no `ret >= 1` clamp (build/StereoYin 0x40ff38-0x40ff63). */
float orc_canon_f(uint32_t u) { return (float)(int32_t)(u - 1u) * 0x1p-31f; }

/* dice() of uniform_real_distribution<float>(-1, 1) bound to a copy of a default-seeded
 * minstd_rand0 (:554, :851-852): value k (k >= 0) of the stream every MST_PMS call replays. */
void orc_pms_dice(long n, float* out) {
    uint32_t s = 1u;
    for (long k = 0; k < n; ++k) {
        s = orc_minstd0_next(s);
        out[k] = fmaf(orc_canon_f(s), 2.0f, -1.0f); /* fma(r, b - a, a) (0x40ff6b) */
    }
}

/* glibc random_r, TYPE_3 (degree 31, separation 3), srandom(seed): outputs skip..skip+n-1. */
void orc_glibc_random(unsigned seed, long skip, long n, int32_t* out) {
    int32_t st[31];
    if (seed == 0) seed = 1;
    st[0] = (int32_t)seed;
    long word = (long)seed;
    for (int i = 1; i < 31; ++i) {
        const long hi = word / 127773, lo = word % 127773;
        word = 16807 * lo - 2836 * hi;
        if (word < 0) word += 2147483647;
        st[i] = (int32_t)word;
    }
    int f = 3, b = 0; /* fptr = &state[3], rptr = &state[0] */
    const long total = 310 + skip + n;
    for (long k = 0; k < total; ++k) {
        const uint32_t val = (uint32_t)st[f] + (uint32_t)st[b];
        st[f] = (int32_t)val;
        if (k >= 310 + skip) out[k - 310 - skip] = (int32_t)(val >> 1);
        if (++f >= 31) { f = 0; ++b; }
        else if (++b >= 31) b = 0;
    }
}

/* ------------------------------------------------------------------ labels */
/* x86 cvttss2si: truncation; NaN and out-of-range values give INT_MIN. */
static inline int cvtt(float f) {
    if (!(f >= -2147483648.0f && f < 2147483648.0f)) return INT_MIN;
    return (int)f;
}

/* random abc init of segment_image_other_init (:390-430): a fresh default-seeded minstd_rand0 per
 * call with uniform_real_distribution<float>(0, 1); pixels in raster order.  Arithmetic as in
 * build/StereoYin 0x4125ea-0x4127f7: the loop squares are reused (no fma), nz^2 = fnma chains. */
void orc_pms_init_labels(int W, int H, int max_disp, float* abc) {
    uint32_t s = 1u;
    const float fmax = (float)max_disp;
#define ORC_DICE01() (s = orc_minstd0_next(s), orc_canon_f(s))
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const size_t idx = (size_t)y * W + x;
            const float d = ORC_DICE01() * fmax;
            float x1, x2, s1, s2;
            for (;;) {
                x1 = ORC_DICE01();
                x2 = ORC_DICE01();
                s1 = x1 * x1;
                s2 = x2 * x2;
                if (s1 + s2 < 1.0f) break;
            }
            const float root = sqrtf((1.0f - s1) - s2);
            const float nx = (x1 + x1) * root;
            const float ny = (x2 + x2) * root;
            const float nz = sqrtf(fmaf(-ny, ny, fmaf(-nx, nx, 1.0f)));
            abc[3 * idx + 0] = -nx / nz;
            abc[3 * idx + 1] = -ny / nz;
            abc[3 * idx + 2] = fmaf(nz, d, fmaf((float)x, nx, ny * (float)y)) / nz;
        }
#undef ORC_DICE01
}

/* compute3DLabelCost (:103-118), build/StereoYin 0x40f930: disp = fma(x, a, y*b) + c; out of
 * [0, max_disp) -> 0.5; else fma(ceil - disp, C[floor], (disp - floor) * C[ceil]). */
float orc_label_cost(const float* vol, float a, float b, float c, int pix, int max_disp, int W, size_t N) {
    const float xf = (float)(pix % W), yf = (float)(pix / W);
    const float disp = fmaf(xf, a, yf * b) + c;
    const float dc = ceilf(disp), dfl = floorf(disp);
    const int ic = cvtt(dc);
    if (ic >= max_disp) return 0.5f;
    const int ifl = cvtt(dfl);
    if (ifl < 0) return 0.5f;
    return fmaf(dc - disp, vol[(size_t)ifl * N + pix], (disp - dfl) * vol[(size_t)ic * N + pix]);
}

/* LabelToDisp (:189-201) then *= (Dmax - 1.f) (:900-902): v = (fma(x, a, y*b) + c) / (Dmax - 1);
 * v >= 1 or NaN -> 1, v <= 0 -> 0 (0x40fd60) */
void orc_pms_label_to_disp(const float* abc, int W, int H, int max_disp, float* disp) {
    const float dm1 = (float)max_disp - 1.0f;
    for (long i = 0; i < (long)W * H; ++i) {
        const float xf = (float)(i % W), yf = (float)(i / W);
        float v = (fmaf(xf, abc[3 * i], yf * abc[3 * i + 1]) + abc[3 * i + 2]) / dm1;
        v = (v < 1.0f) ? v : 1.0f;
        v = (0.0f < v) ? v : 0.0f;
        disp[i] = v * dm1;
    }
}

/* the plane disparity of every pixel's label, fma(x, a, y*b) + c (LabelToDisp before its clamp) */
void orc_pms_plane_disp(const float* abc, int W, int H, float* disp) {
    for (long i = 0; i < (long)W * H; ++i)
        disp[i] = fmaf((float)(i % W), abc[3 * i], (float)(i / W) * abc[3 * i + 1]) + abc[3 * i + 2];
}

/* ------------------------------------------------------------------ tree graph */
static int cmp64(const void* a, const void* b) {
    const int64_t x = *(const int64_t*)a, y = *(const int64_t*)b;
    return x < y ? -1 : x > y;
}

/* tree_g (:377-384): trees adjacent through any 4-connected grid edge, boost setS (no duplicates,
 * ascending target id).  Trees are the orc_bfs trees (numbered by first raster pixel).  CSR:
 * nb[nb_start[t] .. nb_start[t+1]).  nb_cap: capacity of nb; returns the number of entries (or -1
 * if nb_cap is too small). */
int orc_tree_graph(int W, int H, int ntrees, const int32_t* tree_start, const int32_t* node_pix, int32_t* nb_start,
                   int32_t* nb, int nb_cap) {
    const int N = W * H;
    int32_t* cc = (int32_t*)malloc(sizeof(int32_t) * (size_t)N);
    for (int t = 0; t < ntrees; ++t)
        for (int n = tree_start[t]; n < tree_start[t + 1]; ++n) cc[node_pix[n]] = t;
    /* pairs (t, u) for every crossing edge, both directions, then sort + unique per tree */
    long np = 0;
    for (int p = 0; p < N; ++p) {
        const int x = p % W, y = p / W;
        if (x < W - 1 && cc[p] != cc[p + 1]) np += 2;
        if (y < H - 1 && cc[p] != cc[p + W]) np += 2;
    }
    int64_t* pr = (int64_t*)malloc(sizeof(int64_t) * (size_t)(np > 0 ? np : 1));
    long k = 0;
    for (int p = 0; p < N; ++p) {
        const int x = p % W, y = p / W;
        const int q[2] = {x < W - 1 ? p + 1 : -1, y < H - 1 ? p + W : -1};
        for (int j = 0; j < 2; ++j) {
            if (q[j] < 0 || cc[p] == cc[q[j]]) continue;
            pr[k++] = ((int64_t)cc[p] << 32) | (uint32_t)cc[q[j]];
            pr[k++] = ((int64_t)cc[q[j]] << 32) | (uint32_t)cc[p];
        }
    }
    qsort(pr, (size_t)np, sizeof(int64_t), cmp64);
    int cnt = 0, t = 0;
    nb_start[0] = 0;
    for (long i = 0; i < np; ++i) {
        if (i > 0 && pr[i] == pr[i - 1]) continue;
        const int a = (int)(pr[i] >> 32), b = (int)(pr[i] & 0xffffffff);
        while (t < a) nb_start[++t] = cnt;
        if (cnt >= nb_cap) { cnt = -1; break; }
        nb[cnt++] = b;
    }
    if (cnt >= 0) while (t < ntrees) nb_start[++t] = cnt;
    free(pr);
    free(cc);
    return cnt;
}

/* ------------------------------------------------------------------ MST_PMS */
typedef struct {
    int W, max_disp;
    size_t N;
    const int32_t *tree_start, *node_pix, *node_parent, *node_child;
    const uint16_t* node_w;
    const float* vol;
    float* abc;
    double *min_cost, *agg;
} pms_view;

/* MSTCostAggregationAndLabelUpdate (:160-186) for tree t and label (a, b, c); returns the number
 * of pixels whose label changed. */
static int pms_update(const pms_view* v, int t, float a, float b, float c, const uint8_t* nch) {
    const int ts = v->tree_start[t], te = v->tree_start[t + 1];
    double* agg = v->agg;
    for (int n = ts; n < te; ++n) agg[v->node_pix[n]] = 0.0; /* :165 */
    for (int n = te - 1; n > ts; --n) {                     /* :125-135 */
        const int pix = v->node_pix[n], ppix = v->node_pix[v->node_parent[n]];
        agg[pix] = (double)orc_label_cost(v->vol, a, b, c, pix, v->max_disp, v->W, v->N) + agg[pix];
        agg[ppix] = fma(agg[pix], SM_S_LUT[v->node_w[n]], agg[ppix]);
    }
    {
        const int rp = v->node_pix[ts];
        agg[rp] = (double)orc_label_cost(v->vol, a, b, c, rp, v->max_disp, v->W, v->N) + agg[rp]; /* :137 */
    }
    for (int n = ts; n < te; ++n) { /* :145-157 */
        const int p = v->node_pix[n];
        for (int i = 0; i < nch[n]; ++i) {
            const int ch = v->node_child[4 * n + i];
            const int cp = v->node_pix[ch];
            agg[cp] = fma(SM_S_LUT[v->node_w[ch]], agg[p], SM_S2_LUT[v->node_w[ch]] * agg[cp]);
        }
    }
    int changed = 0;
    for (int n = ts; n < te; ++n) { /* :173-185 strict < */
        const int p = v->node_pix[n];
        if (agg[p] < v->min_cost[p]) {
            v->min_cost[p] = agg[p];
            v->abc[3 * (size_t)p] = a;
            v->abc[3 * (size_t)p + 1] = b;
            v->abc[3 * (size_t)p + 2] = c;
            changed++;
        }
    }
    return changed;
}

/* One MST_PMS call (:546-629) over one view's forest.  dice: the replayed (-1, 1) stream (orc_pms_dice,
 * at least dice_n values); rnd: the ntrees rand() values this call draws (:584), in tree order.
 * abc [3N] and min_cost [N] are updated in place (min_cost starts at DBL_MAX, :820-821).
 * stats (may be NULL): per tree {dice values consumed, pixels changed in propagation, pixels changed
 * in refinement, test pixel}.  Returns the dice values consumed, or -1 when dice_n is exceeded or a
 * propagation index falls outside its tree (the reference would read past the vector). */
long orc_mst_pms(int W, int H, int max_disp, int ntrees, const int32_t* tree_start, const int32_t* node_pix,
                 const int32_t* node_parent, const uint16_t* node_w, const uint8_t* node_nch, const int32_t* node_child,
                 const int32_t* nb_start, const int32_t* nb, const float* vol, float* abc, double* min_cost,
                 const float* dice, long dice_n, const int32_t* rnd, int32_t* stats) {
    pms_view v;
    v.W = W;
    v.max_disp = max_disp;
    v.N = (size_t)W * H;
    v.tree_start = tree_start;
    v.node_pix = node_pix;
    v.node_parent = node_parent;
    v.node_child = node_child;
    v.node_w = node_w;
    v.vol = vol;
    v.abc = abc;
    v.min_cost = min_cost;
    v.agg = (double*)malloc(sizeof(double) * v.N);
    long k = 0;
    long ret = 0;
    const float fmax = (float)max_disp;
    for (int t = 0; t < ntrees && ret >= 0; ++t) {
        const long k0 = k;
        int chp = 0, chr = 0;
        /* spatial propagation (:562-580): one label per neighbour tree, ascending tree id */
        for (int j = nb_start[t]; j < nb_start[t + 1]; ++j) {
            const int u = nb[j];
            if (k >= dice_n) { ret = -1; break; }
            const int sz = tree_start[u + 1] - tree_start[u];
            const int i = cvtt(((dice[k++] + 1.0f) * 0.5f) * (float)sz);
            if (i < 0 || i >= sz) { ret = -1; break; }
            const size_t q = (size_t)node_pix[tree_start[u] + i];
            chp += pms_update(&v, t, abc[3 * q], abc[3 * q + 1], abc[3 * q + 2], node_nch);
        }
        if (ret < 0) break;
        /* random refinement (:582-625) around the test pixel's current label */
        const int sz = tree_start[t + 1] - tree_start[t];
        const int tp = node_pix[tree_start[t] + (int)((unsigned long)(long)rnd[t] % (unsigned long)sz)];
        const float px = (float)(tp % W), py = (float)(tp / W);
        const float la = abc[3 * (size_t)tp], lb = abc[3 * (size_t)tp + 1], lc = abc[3 * (size_t)tp + 2];
        const float nz = 1.0f / sqrtf(fmaf(la, la, lb * lb) + 1.0f);
        const float nx = -la * nz, ny = -lb * nz;
        const float d = fmaf(la, px, lb * py) + lc;
        float max_n = 1.0f, max_d = 0.5f * fmax;
        for (; max_d > 0.1f; max_d *= 0.5f, max_n *= 0.5f) {
            if (k + 4 > dice_n) { ret = -1; break; }
            const float rand_d = fmaf(dice[k++], max_d, d);
            if (rand_d < 0.0f || rand_d > fmax) continue;
            float rnx = fmaf(max_n, dice[k++], nx);
            float rny = fmaf(max_n, dice[k++], ny);
            float rnz = fmaf(max_n, dice[k++], nz);
            const float ni = 1.0f / sqrtf(fmaf(rnz, rnz, fmaf(rnx, rnx, rny * rny)));
            rnx *= ni;
            rny *= ni;
            rnz = fabsf(rnz * ni);
            const float a = -rnx / rnz, b = -rny / rnz;
            const float c = fmaf(rand_d, rnz, fmaf(rnx, px, rny * py)) / rnz;
            chr += pms_update(&v, t, a, b, c, node_nch);
        }
        if (stats) {
            stats[4 * t + 0] = (int32_t)(k - k0);
            stats[4 * t + 1] = chp;
            stats[4 * t + 2] = chr;
            stats[4 * t + 3] = tp;
        }
    }
    free(v.agg);
    return ret < 0 ? -1 : k;
}
