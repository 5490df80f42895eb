// sm_pms.hip -- MST_PMS, Stereo3DMST's slanted-plane label search (src/Stereo3DMST.cpp:546-629), on the GPU.
//
// One MST_PMS call visits the trees of a view in order.  Tree t evaluates deg(t) propagation labels
// (one from each neighbour tree, at a pixel the dice pick, :562-580), then up to L refinement labels
// around the label of a random pixel of its own (:582-625).  Each label is a full aggregation over the
// tree (MSTCostAggregationAndLabelUpdate, :160-186): the lerp data term (:103-118) of every node, the
// leaf->root and root->leaf passes, and a strict-< update of every pixel's (min_cost, label).
//
// Parallel form.  The labels of one phase (propagation or refinement) of one tree are independent of
// each other: they are "slices".  Lane j of a wave walks proposal j along a heavy path of the tree, and
// the per-pixel update then scans the proposals in order with strict <, which is the reference's
// sequential rule.  Trees are scheduled as heavy paths by light depth (sm_pms_host.cpp): the up pass
// runs depths deepest first, the down pass root first; the A rows are updated in place (A_up, then A),
// as the reference does in agg_cost.
//
// Serial dependencies between trees: (1) the dice offset -- tree t's draws start where tree t-1's
// ended, and a refinement level whose disparity falls outside [0, Dmax] consumes 1 draw instead of 4
// (:604); (2) propagation reads a lower neighbour's label after that tree ran (Gauss-Seidel).  Two
// modes keep these exact:
//   * serial (k_pms_serial): one workgroup walks the trees in order;
//   * speculative: every tree at once from guessed offsets and the labels at the start of the
//     iteration; a validation scan finds the first tree whose offset or sampled labels differ from
//     what the serial order gives, everything before it is exact, and the host redoes the rest.
//
// Arithmetic follows the shipped binary (build/StereoYin, read with objdump; DESIGN.md "MST_PMS"):
// the data term fma(x, a, y*b) + c and fma(ceil - d, C[floor], (d - floor) * C[ceil]); the up pass
// fma(A_child, S, acc) over children in descending BFS id then (double)C + acc; the down pass
// fma(S, A_parent, S2 * A_up).  Compiled with -ffp-contract=off; divisions and square roots are
// correctly rounded (sqrt_rn / div_rn), as x86's sqrtss / divss are.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdlib>

#include "sm_pms.h"
#include "sm_knob.h"

namespace {

constexpr int PMS_CH = 8;  // nodes whose loads a walker issues together

// x86 cvttss2si: NaN and out-of-range values give INT_MIN (the GPU's v_cvt_i32_f32 saturates)
__device__ __forceinline__ int cvtt(float f) {
    return (f >= -2147483648.0f && f < 2147483648.0f) ? (int)f : INT_MIN;
}

// compute3DLabelCost (:103-118), build/StereoYin 0x40f930
__device__ __forceinline__ float label_cost(const float* __restrict__ vol, int Dv, int Dmax, float a, float b, float c,
                                            int pix, float xf, float yf) {
    const float disp = fmaf(xf, a, yf * b) + c;
    const float dc = ceilf(disp), dfl = floorf(disp);
    const int ic = cvtt(dc), ifl = cvtt(dfl);
    const bool out = ic >= Dmax || ifl < 0;  // 0.5 (:108-111)
    // branch-free: both words are loaded from clamped indices and the result selected, so a walker's
    // loads stay straight-line code (a load under a branch makes the wait counters fall back to a full
    // drain before the next node's loads)
    const float* r = vol + (size_t)pix * Dv;
    const float vf = r[out ? 0 : ifl], vc = r[out || ic < 0 ? 0 : ic];
    return out ? 0.5f : fmaf(dc - disp, vf, (disp - dfl) * vc);
}

// Correctly rounded float sqrt and division, as x86's sqrtss / divss.  HIP's __fsqrt_rn is the native
// (1-ulp) sqrt unless OCML_BASIC_ROUNDED_OPERATIONS is defined, so the hardware result is fixed up here
// and does not depend on compiler defaults: a candidate within an ulp is moved to the float whose
// rounding interval holds the exact value, decided by exact double products (the midpoint of two
// adjacent floats has <= 26 significant bits; its square or its product with a float is exact in
// double).  Neither an exact square root nor an exact quotient can fall on a midpoint.
// neighbours of a positive finite float
__device__ __forceinline__ float next_up(float f) { return __uint_as_float(__float_as_uint(f) + 1u); }
__device__ __forceinline__ float next_dn(float f) { return __uint_as_float(__float_as_uint(f) - 1u); }

__device__ float sqrt_rn(float x) {
    float s = __builtin_sqrtf(x);
    if (!(x > 0.0f) || !(x < INFINITY)) return s;  // 0, negatives, NaN, inf: the hardware is exact
    const double xd = (double)x;
    for (int i = 0; i < 2; ++i) {
        const float up = next_up(s), dn = next_dn(s);
        const double mu = ((double)s + (double)up) * 0.5, md = ((double)s + (double)dn) * 0.5;
        if (xd > mu * mu) s = up;
        else if (xd < md * md) s = dn;
        else break;
    }
    return s;
}

__device__ float div_rn(float a, float b) {
    const float q = a / b;
    if (!(fabsf(q) < INFINITY) || q == 0.0f || !(fabsf(a) < INFINITY) || !(fabsf(b) < INFINITY)) return q;
    const double A = fabs((double)a), B = fabs((double)b);
    float m = fabsf(q);
    for (int i = 0; i < 2; ++i) {
        const float up = next_up(m), dn = next_dn(m);
        const double mu = ((double)m + (double)up) * 0.5, md = ((double)m + (double)dn) * 0.5;
        if (A > mu * B) m = up;
        else if (A < md * B) m = dn;
        else break;
    }
    return q < 0.0f ? -m : m;
}

__device__ __forceinline__ int tree_deg(const PmsDev& d, int t) { return d.nb_start[t + 1] - d.nb_start[t]; }

// proposals of a phase: count and label-table base
__device__ __forceinline__ void phase_labels(const PmsDev& d, int phase, int t, int& P, int& base) {
    const int deg = tree_deg(d, t);
    if (phase == 0) {
        P = d.nprop ? d.nprop[t] : deg;
        base = d.tree_lab[t];
    } else {
        P = d.nref[t];
        base = d.tree_lab[t] + deg;
    }
}

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

// Chunk metadata staged across the wave: the PmsRow words of rows [first, first + n) (10 dwords
// each, n <= PMS_CH), word j of the block in lane j (m0) or lane j - 64 (m1).  One coalesced load per
// lane instead of a chain of per-field loads; the walkers read fields with v_readlane (uniform index).
struct ChunkMeta {
    uint32_t m0, m1;
};
static_assert(sizeof(PmsRow) == 40, "PmsRow is 10 dwords");
static_assert(PMS_CH * 10 <= 128, "a chunk's metadata fits two words per lane");

__device__ __forceinline__ ChunkMeta meta_load(const PmsRow* rows, int first, int n) {
    const uint32_t* b = reinterpret_cast<const uint32_t*>(rows + first);
    const int lane = (int)(threadIdx.x & 63), nd = n * 10;
    ChunkMeta m;
    m.m0 = b[lane < nd ? lane : 0];  // unconditional (clamped) loads
    m.m1 = b[lane + 64 < nd ? lane + 64 : 0];
    return m;
}

__device__ __forceinline__ uint32_t meta_dw(const ChunkMeta& m, int j) {  // j wave-uniform
    const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)m.m0, j & 63);
    const uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)m.m1, j & 63);
    return j < 64 ? a : b;
}

// Leaf->root walk of rows [top, bot] of tree t (a heavy path or a piece of one) for proposals
// [64*chunk, 64*chunk+64), bottom to head, from x0 = the value of the bottom row's heavy child (a
// path's bottom is a leaf; a cut piece's bottom takes the guess 0, or in a repair the exact row of
// the piece below).  A node's value folds its children in descending BFS id, the heavy child (the row
// below, walked just before) from a register, the light ones from their rows (finished in a deeper
// round).  Software-pipelined in chunks of PMS_CH nodes: a chunk's light-child rows and cost-row
// words are issued from metadata staged during the previous chunk, then the next chunk's metadata,
// so each chunk pays one memory latency; the serial part reads only registers and the LDS weight
// tables sS / sS2.  REPAIR: the stored rows are loaded with the chunk, and the walk stops at the
// first node where every lane's recomputed value equals the stored one bitwise (two trajectories of
// the recurrence that agree at a node agree from there on); until then it overwrites.  PRE: the data
// term of every row was written into its A row beforehand (k_pms_cost / cost_rows), so a chunk loads
// tree-contiguous A rows instead of gathering from the cost volume (a dependent load per node, and
// a TLB miss at most of them: the volume is ~1 GB).
template <bool REPAIR, bool PRE>
__device__ bool up_walk(const PmsDev& d, const double* __restrict__ sS, int phase, int t, int top, int bot, int chunk,
                        double x0) {
    int P, base;
    phase_labels(d, phase, t, P, base);
    const int j = chunk * 64 + (int)(threadIdx.x & 63);
    if (chunk * 64 >= P) return true;
    const bool act = j < P;
    float4 L = make_float4(0.f, 0.f, 0.f, 0.f);
    if (!PRE && act) L = d.lab[base + j];
    const int ts = d.tree_start[t], pt = d.tree_pt[t];
    double* __restrict__ A = d.A + d.tree_abase[t] + j;
    const double* __restrict__ Al = d.A + d.tree_abase[t] + (act ? j : 0);  // loads: every lane in bounds
    const int row0 = top, len = bot - top + 1;
    int i0 = len - 1;                                       // top (last walked) index of this chunk
    int lo = i0 - PMS_CH + 1 > 0 ? i0 - PMS_CH + 1 : 0;     // its first index
    ChunkMeta mc = meta_load(d.rows, row0 + lo, i0 - lo + 1);
    double x = x0;
    while (i0 >= 0) {
        const int n = i0 - lo + 1;
        double cv[PMS_CH][4];
        double cost[PMS_CH];
        double old[PMS_CH];
        int nch[PMS_CH], hk[PMS_CH], wc[PMS_CH][4];
        // straight-line issue: every load unconditional from a valid address (nodes past the chunk's end
        // re-read its first node; lanes past P read column 0), and no select on a loaded value -- a
        // select would make the compiler wait for the load where it is issued.  Lanes past P compute
        // garbage and never store.
#pragma unroll
        for (int k = 0; k < PMS_CH; ++k) {
            const int kk = k < n ? k : 0;
            const int row = row0 + i0 - kk;
            const int w0 = (i0 - kk - lo) * 10;  // node row0 + i0 - kk
            const uint32_t w6 = meta_dw(mc, w0 + 6), w7 = meta_dw(mc, w0 + 7), w8 = meta_dw(mc, w0 + 8);
            nch[k] = k < n ? (int)((w6 >> 16) & 255u) : 0;
            hk[k] = (int)(w6 >> 24);
            wc[k][0] = (int)(w7 & 0xFFFFu);
            wc[k][1] = (int)(w7 >> 16);
            wc[k][2] = (int)(w8 & 0xFFFFu);
            wc[k][3] = (int)(w8 >> 16);
#pragma unroll
            for (int q = 0; q < 4; ++q) {  // only the light children's rows (wave-uniform tests, no dummy loads)
                cv[k][q] = 0.0;
                if (q < nch[k] && q != hk[k]) cv[k][q] = Al[(size_t)((int)meta_dw(mc, w0 + 2 + q) - ts) * pt];
            }
            if (PRE) {
                cost[k] = Al[(size_t)(row - ts) * pt];
            } else {
                const uint32_t w9 = meta_dw(mc, w0 + 9);
                const float c = label_cost(d.vol, d.Dv, d.Dmax, L.x, L.y, L.z, (int)meta_dw(mc, w0), (float)(w9 & 0xFFFFu),
                                           (float)(w9 >> 16));
                cost[k] = (double)c;
            }
            if (REPAIR) old[k] = Al[(size_t)(row - ts) * pt];
        }
        const int i0n = lo - 1;
        const int lon = i0n - PMS_CH + 1 > 0 ? i0n - PMS_CH + 1 : 0;
        // unconditional (past the head: a dummy reload of row0), so no branch precedes the serial part
        const ChunkMeta mn = meta_load(d.rows, row0 + lon, i0n >= 0 ? i0n - lon + 1 : 1);
#pragma unroll
        for (int k = 0; k < PMS_CH; ++k) {
            if (k >= n) break;
            double sv[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) sv[q] = sS[wc[k][q]];
            double acc = 0.0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (q >= nch[k]) break;
                const double v = q == hk[k] ? x : cv[k][q];
                acc = fma(v, sv[q], acc);  // A[parent] = fma(A[v], S, A[parent]) (0x40fad5)
            }
            x = cost[k] + acc;  // A[v] = C + A[v] (0x40fac5); cost[k] is a float widened exactly
            if (REPAIR) {
                const bool same = !act || __double_as_longlong(x) == __double_as_longlong(old[k]);
                if (__all(same)) return true;
                if (!same) A[(size_t)(row0 + i0 - k - ts) * pt] = x;
            } else if (act) {
                A[(size_t)(row0 + i0 - k - ts) * pt] = x;
            }
        }
        mc = mn;
        i0 = i0n;
        lo = lon;
    }
    return !REPAIR;  // a repair that never agreed rewrote the head row
}

__device__ void up_item(const PmsDev& d, const double* __restrict__ sS, int phase, int path, int chunk) {
    const PmsPath pa = d.paths[path];
    up_walk<false, true>(d, sS, phase, uni(pa.tree), uni(pa.row), uni(pa.row) + uni(pa.len) - 1, chunk, 0.0);
}

// the data term C (:103-118) of proposals [j0, P) step js of row `row` of tree t into its A row: the
// up walk's starting values (PRE)
__device__ __forceinline__ void cost_row(const PmsDev& d, int row, int t, int P, int base, int j0, int js) {
    const PmsRow& rw = d.rows[row];
    const int pix = rw.pix;
    const float xf = (float)rw.x, yf = (float)rw.y;
    double* a = d.A + d.tree_abase[t] + (size_t)(row - d.tree_start[t]) * d.tree_pt[t];
    for (int j = j0; j < P; j += js) {
        const float4 L = d.lab[base + j];
        a[j] = (double)label_cost(d.vol, d.Dv, d.Dmax, L.x, L.y, L.z, pix, xf, yf);
    }
}

// Root->leaf walk of rows [top, bot] of tree t, head to bottom: A(c) = fma(S_c, A(p), S2_c * A_up(c))
// in place (0x40fbb4-0x40fbbd); a tree root keeps A_up.  The head's parent value: normally the row
// A[parent] holds (a cut piece's head: whatever its neighbour piece has written so far, a guess);
// REPAIR: yin, the exact row of the piece above, with A_up read from ub (the rows' backup, since the
// speculative walk overwrote them) and the walk stopping at the first all-lanes bitwise agreement.
// The next chunk's A_up rows and weights are loaded while the current chunk runs.
template <bool REPAIR>
__device__ bool down_walk(const PmsDev& d, const double* __restrict__ sS, const double* __restrict__ sS2, int phase,
                          int t, int top, int bot, int chunk, double yin, const double* __restrict__ ub) {
    int P, base;
    phase_labels(d, phase, t, P, base);
    (void)base;
    const int j = chunk * 64 + (int)(threadIdx.x & 63);
    if (chunk * 64 >= P) return true;
    const bool act = j < P;
    const int ts = d.tree_start[t], pt = d.tree_pt[t];
    double* __restrict__ A = d.A + d.tree_abase[t] + j;
    const double* __restrict__ Al = d.A + d.tree_abase[t] + (act ? j : 0);  // loads: every lane in bounds,
    const int jl = act ? j : 0;                                               // no selects (see up_walk)
    const int row0 = top, len = bot - top + 1;
    const int parent = REPAIR ? row0 - 1 : uni(d.rows[row0].parent);
    const int lane = (int)(threadIdx.x & 63);
    // weights of a chunk: lane k holds rows[row0 + i0 + k].w
    auto wload = [&](int i0, int n) {
        const int r = row0 + (i0 < len ? i0 + (lane < n ? lane : 0) : 0);
        return (int)d.rows[r].w;
    };
    auto uload = [&](double (&u)[PMS_CH], double (&o)[PMS_CH], int i0, int n) {
#pragma unroll
        for (int k = 0; k < PMS_CH; ++k) {
            const int i = i0 < len ? i0 + (k < n ? k : 0) : 0;  // clamped: unconditional loads (see label_cost)
            u[k] = REPAIR ? ub[(size_t)i * pt + jl] : Al[(size_t)(row0 + i - ts) * pt];
            if (REPAIR) o[k] = Al[(size_t)(row0 + i - ts) * pt];
        }
    };
    double y = REPAIR ? yin : 0.0;
    if (!REPAIR && parent >= 0) y = Al[(size_t)(parent - ts) * pt];
    int i0 = 0, n = len < PMS_CH ? len : PMS_CH;
    double uc[PMS_CH], oc[PMS_CH];
    uload(uc, oc, 0, n);
    int wl = wload(0, n);
    while (i0 < len) {
        const int i0n = i0 + n, nn = len - i0n < PMS_CH ? len - i0n : PMS_CH;
        double un[PMS_CH], on[PMS_CH];
        uload(un, on, i0n, nn);  // past the bottom: dummy reloads of row0 (no branch before the serial part)
        const int wn = wload(i0n, nn);
#pragma unroll
        for (int k = 0; k < PMS_CH; ++k) {
            if (k >= n) break;
            const int w = __builtin_amdgcn_readlane(wl, k);
            const double S = sS[w], S2 = sS2[w];
            if (i0 + k == 0) {
                y = parent >= 0 ? fma(S, y, S2 * uc[0]) : uc[0];
            } else {
                y = fma(S, y, S2 * uc[k]);
            }
            if (REPAIR) {
                const bool same = !act || __double_as_longlong(y) == __double_as_longlong(oc[k]);
                if (__all(same)) return true;
                if (!same) A[(size_t)(row0 + i0 + k - ts) * pt] = y;
            } else if (act) {
                A[(size_t)(row0 + i0 + k - ts) * pt] = y;
            }
        }
#pragma unroll
        for (int k = 0; k < PMS_CH; ++k) {
            uc[k] = un[k];
            if (REPAIR) oc[k] = on[k];
        }
        wl = wn;
        i0 = i0n;
        n = nn;
    }
    return !REPAIR;  // a repair that never agreed rewrote the bottom row
}

__device__ void down_item(const PmsDev& d, const double* __restrict__ sS, const double* __restrict__ sS2, int phase,
                          int path, int chunk) {
    const PmsPath pa = d.paths[path];
    down_walk<false>(d, sS, sS2, phase, uni(pa.tree), uni(pa.row), uni(pa.row) + uni(pa.len) - 1, chunk, 0.0, nullptr);
}

// the S / S2 tables (766 weight codes) into LDS
#define PMS_NW 766
__device__ __forceinline__ void load_luts(const PmsDev& d, double* sS, double* sS2) {
    for (int i = threadIdx.x; i < PMS_NW; i += blockDim.x) {
        sS[i] = d.slut[i];
        sS2[i] = d.s2lut[i];
    }
    __syncthreads();
}

// strict-< update of one row's pixel over the phase's proposals in order (:173-185)
__device__ void update_row(const PmsDev& d, int phase, int row, int t) {
    int P, base;
    phase_labels(d, phase, t, P, base);
    if (P <= 0) return;
    const int pix = d.rows[row].pix;
    const double* a = d.A + d.tree_abase[t] + (size_t)(row - d.tree_start[t]) * d.tree_pt[t];
    double m = d.minc[pix];
    int best = -1;
    for (int j = 0; j < P; ++j) {
        const double v = a[j];
        if (v < m) {
            m = v;
            best = j;
        }
    }
    if (best >= 0) {
        const float4 L = d.lab[base + best];
        d.minc[pix] = m;
        d.abc[3 * (size_t)pix] = L.x;
        d.abc[3 * (size_t)pix + 1] = L.y;
        d.abc[3 * (size_t)pix + 2] = L.z;
    }
}

// propagation label j of tree t whose draws start at offset o (:567-573): the neighbour's BFS node
// (int)(((dice + 1) * 0.5f) * size) (0x40ff6b-0x40ff9a), and that pixel's current label
__device__ void prop_label(const PmsDev& d, int t, long long o, int j) {
    const int u = d.nb[d.nb_start[t] + j];
    const long long k = o + j;
    float r = 0.0f;
    if (k < d.dice_n) r = d.dice[k];
    else atomicOr(d.err, 4u);
    const int us = d.tree_start[u], sz = d.tree_start[u + 1] - us;
    int i = cvtt(((r + 1.0f) * 0.5f) * (float)sz);
    if (i < 0 || i >= sz) {  // the reference would read outside mst_vertices_vec[u]
        atomicOr(d.err, 2u);
        i = i < 0 ? 0 : sz - 1;
    }
    const int q = d.bfs_pix[us + i];
    const int slot = d.tree_lab[t] + j;
    // serial order: a higher neighbour has not run yet in this call
    const float* src = d.hi_bak && u > t ? d.abc_bak : d.abc;
    d.lab[slot] = make_float4(src[3 * (size_t)q], src[3 * (size_t)q + 1], src[3 * (size_t)q + 2], 0.0f);
    d.labq[slot] = q;
}

// Random refinement of tree t (:582-625) with its draws from offset o: the labels of the in-range levels
// (written compacted when `write`) and the number of draws.  The test pixel's label is read as it is now.
// the refinement's starting disparity dd of tree t (its test pixel's current plane at that pixel)
__device__ float ref_dd(const PmsDev& d, int t) {
    const int ts = d.tree_start[t], sz = d.tree_start[t + 1] - ts;
    const int tp = d.bfs_pix[ts + (int)((uint32_t)d.rnd[t] % (uint32_t)sz)];
    const float px = (float)(tp % d.W), py = (float)(tp / d.W);
    return fmaf(d.abc[3 * (size_t)tp], px, d.abc[3 * (size_t)tp + 1] * py) + d.abc[3 * (size_t)tp + 2];
}

// draws of tree t's refinement from offset o given dd (ref_levels without the labels); dice(k) reads
// the stream
template <class Dice>
__device__ int ref_count(const PmsDev& d, float dd, long long o, Dice dice) {
    const float fmax = (float)d.Dmax;
    float max_d = 0.5f * fmax;
    long long k = o;
    for (; max_d > 0.1f; max_d *= 0.5f) {
        if (k + 4 > d.dice_n) {
            atomicOr(d.err, 4u);
            break;
        }
        const float rd = fmaf(dice(k++), max_d, dd);
        if (rd < 0.0f || rd > fmax) continue;
        k += 3;
    }
    return (int)(k - o);
}

// dice(k): the stream's draw k (global memory, or a window staged in LDS)
template <class Dice>
__device__ int ref_levels_d(const PmsDev& d, int t, long long o, bool write, Dice dice) {
    const int ts = d.tree_start[t], sz = d.tree_start[t + 1] - ts;
    const int tp = d.bfs_pix[ts + (int)((uint32_t)d.rnd[t] % (uint32_t)sz)];  // std::rand() % size()
    const float px = (float)(tp % d.W), py = (float)(tp / d.W);
    const float la = d.abc[3 * (size_t)tp], lb = d.abc[3 * (size_t)tp + 1], lc = d.abc[3 * (size_t)tp + 2];
    const float nz = div_rn(1.0f, sqrt_rn(fmaf(la, la, lb * lb) + 1.0f));  // 0x410139-0x410170
    const float nx = -la * nz, ny = -lb * nz;
    const float dd = fmaf(la, px, lb * py) + lc;
    const float fmax = (float)d.Dmax;
    float max_n = 1.0f, max_d = 0.5f * fmax;
    long long k = o;
    int nv = 0;
    const int base = d.tree_lab[t] + (d.nb_start[t + 1] - d.nb_start[t]);
    for (; max_d > 0.1f; max_d *= 0.5f, max_n *= 0.5f) {
        if (k + 4 > d.dice_n) {
            atomicOr(d.err, 4u);
            break;
        }
        const float rd = fmaf(dice(k++), max_d, dd);  // 0x410247
        if (rd < 0.0f || rd > fmax) continue;           // :604
        float rnx = fmaf(max_n, dice(k++), nx);
        float rny = fmaf(max_n, dice(k++), ny);
        float rnz = fmaf(max_n, dice(k++), nz);
        if (!write) continue;
        const float ni = div_rn(1.0f, sqrt_rn(fmaf(rnz, rnz, fmaf(rnx, rnx, rny * rny))));  // 0x41037b-0x4103c9
        rnx *= ni;
        rny *= ni;
        rnz = fabsf(rnz * ni);
        const float a = div_rn(-rnx, rnz), b = div_rn(-rny, rnz);
        const float c = div_rn(fmaf(rd, rnz, fmaf(rnx, px, rny * py)), rnz);  // 0x41041f-0x41043d
        d.lab[base + nv++] = make_float4(a, b, c, 0.0f);
    }
    if (write) d.nref[t] = nv;
    return (int)(k - o);
}

__device__ int ref_levels(const PmsDev& d, int t, long long o, bool write) {
    return ref_levels_d(d, t, o, write, [&d](long long k) { return d.dice[k]; });
}

// ----------------------------------------------------------------------------- serial mode
constexpr int PMS_SER_MAXP = 1024;  // paths of a round that k_pms_serial sorts into lane groups
// A path of at least PMS_GLONG rows goes to the wave walker whatever its P: its walk is a latency chain,
// and the wave walker issues PMS_CH nodes per memory round trip against the group walker's PMS_GCH.
constexpr int PMS_GLONG = 48;
template <int GW>
__device__ void up_group(const PmsDev& d, const double* __restrict__ sS, int phase, int path);
template <int GW>
__device__ void down_group(const PmsDev& d, const double* __restrict__ sS, const double* __restrict__ sS2, int phase,
                           int path);
// NT threads: 1024 caps a lane at 128 registers (4 waves per SIMD), below what the inlined walkers
// hold; 768 gives 168 (SM_PMS_SER_NT A/B)
template <int NT>
__global__ void __launch_bounds__(NT, 1) k_pms_serial(PmsDev d, int t0, int t1) {
    __shared__ long long s_off;
    __shared__ int s_n, s_ns, s_nl;
    __shared__ float s_dice[64];
    __shared__ int s_short[PMS_SER_MAXP], s_long[PMS_SER_MAXP];
    __shared__ double sS[PMS_NW], sS2[PMS_NW];
    load_luts(d, sS, sS2);
    const int tid = threadIdx.x, nt = blockDim.x;
    const int wave = tid >> 6, nwaves = nt >> 6, lane = tid & 63;
    // SM_PMS_PROF builds: per-segment wall-clock totals (100 MHz ticks) of thread 0
    long long tick = 0;
    auto seg = [&](int k) __attribute__((always_inline)) {
        if (d.prof && tid == 0) {
            const long long now = (long long)wall_clock64();
            if (k >= 0) atomicAdd((unsigned long long*)&d.prof[k], (unsigned long long)(now - tick));
            tick = now;
        }
    };
    if (tid == 0) s_off = d.off[0];
    __syncthreads();
    seg(-1);
    for (int t = t0; t < t1; ++t) {
        const int deg = tree_deg(d, t);
        const int R = d.tree_rounds[t];
        const int ts = d.tree_start[t], te = d.tree_start[t + 1];
        const long long o = s_off;
        for (int phase = 0; phase < 2; ++phase) {
            if (phase == 0) {
                for (int j = tid; j < deg; j += nt) prop_label(d, t, o, j);
            } else {
                // the refinement's draws (at most 4 per level) staged in LDS first: thread 0's level loop then
                // reads LDS instead of one dependent global load per level
                const long long o1 = o + deg;
                if (tid < 64) s_dice[tid] = o1 + tid < d.dice_n ? d.dice[o1 + tid] : 0.0f;
                __syncthreads();
                if (tid == 0)
                    s_n = ref_levels_d(d, t, o1, true, [&](long long k) { return k - o1 < 64 ? s_dice[k - o1] : d.dice[k]; });
            }
            __threadfence_block();
            __syncthreads();
            seg(4 * phase + 0);
            const int P = phase == 0 ? deg : d.nref[t];
            if (P > 0) {
                const int base = d.tree_lab[t] + (phase == 0 ? 0 : deg);
                if (P <= 16) {
                    for (int row = ts + tid; row < te; row += nt) cost_row(d, row, t, P, base, 0, 1);
                } else {
                    for (int row = ts + wave; row < te; row += nwaves) cost_row(d, row, t, P, base, tid & 63, 64);
                }
                __threadfence_block();
                __syncthreads();
                const int32_t* rt = phase == 0 ? d.rt_item : d.rt_path;
                int Pw, bw;
                phase_labels(d, phase, t, Pw, bw);  // the walkers' proposal count
                // A round of a tree with few proposals (P <= 8): its short paths (< PMS_GLONG rows) in lane
                // groups, 32 (P <= 2) or 8 paths per wave (the planned walks' up_group / down_group), the long
                // ones by the wave walker -- instead of one wave per path, which left a round with many short
                // paths waiting on 16 waves.  Otherwise one wave per (path, 64-proposal chunk) item.
                auto round = [&](int r, bool up) __attribute__((always_inline)) {  // (inlined: no captures in scratch)
                    const int plo = d.rt_path[(size_t)r * (d.K + 1) + t], phi = d.rt_path[(size_t)r * (d.K + 1) + t + 1];
                    const int np = phi - plo;
                    if (Pw <= 8 && np <= PMS_SER_MAXP) {
                        if (tid == 0) {
                            s_ns = 0;
                            s_nl = 0;
                        }
                        __syncthreads();
                        for (int k = tid; k < np; k += nt) {
                            if (d.paths[plo + k].len < PMS_GLONG) s_short[atomicAdd(&s_ns, 1)] = plo + k;
                            else s_long[atomicAdd(&s_nl, 1)] = plo + k;
                        }
                        __syncthreads();
                        const int ns = s_ns, nl = s_nl, GP = Pw <= 2 ? 32 : 8, ng = (ns + GP - 1) / GP;
                        for (int w = wave; w < ng + nl; w += nwaves) {
                            if (w < ng) {
                                if (GP == 32) {
                                    const int k = w * 32 + lane / 2;
                                    const int path = k < ns ? s_short[k] : -1;
                                    if (up) up_group<2>(d, sS, phase, path);
                                    else down_group<2>(d, sS, sS2, phase, path);
                                } else {
                                    const int k = w * 8 + lane / 8;
                                    const int path = k < ns ? s_short[k] : -1;
                                    if (up) up_group<8>(d, sS, phase, path);
                                    else down_group<8>(d, sS, sS2, phase, path);
                                }
                            } else {
                                const int path = s_long[w - ng];
                                if (up) up_item(d, sS, phase, path, 0);
                                else down_item(d, sS, sS2, phase, path, 0);
                            }
                        }
                    } else {
                        const int lo = rt[(size_t)r * (d.K + 1) + t], hi = rt[(size_t)r * (d.K + 1) + t + 1];
                        for (int it = lo + wave; it < hi; it += nwaves) {
                            const int path = phase == 0 ? d.items[it].path : it, chunk = phase == 0 ? d.items[it].chunk : 0;
                            if (up) up_item(d, sS, phase, path, chunk);
                            else down_item(d, sS, sS2, phase, path, chunk);
                        }
                    }
                    __threadfence_block();
                    __syncthreads();
                };
                for (int r = R - 1; r >= 0; --r) round(r, true);  // leaf -> root: deepest light depth first
                seg(4 * phase + 1);
                for (int r = 0; r < R; ++r) round(r, false);  // root -> leaf
                seg(4 * phase + 2);
                if (d.evals && tid == 0) atomicAdd(d.evals, (unsigned long long)(te - ts) * (unsigned long long)P);
                for (int row = ts + tid; row < te; row += nt) update_row(d, phase, row, t);
                __threadfence_block();
                __syncthreads();
                seg(4 * phase + 3);
            }
        }
        if (tid == 0) {
            s_off = o + deg + s_n;
            if (d.prof) atomicAdd((unsigned long long*)&d.prof[8], (unsigned long long)R);
        }
        __syncthreads();
    }
    if (tid == 0) d.off[0] = s_off;
}

// ----------------------------------------------------------------------------- speculation
// Guessed offsets of trees [t_lo, K) from the exact offset of t_lo (off[0]): each tree's refinement
// draws counted from the label its test pixel has now, i.e. assuming propagation leaves it unchanged.
// The offsets are a serial chain (a tree's draws depend on the dice at its offset), so the rest is
// taken off it: every tree's starting disparity in parallel, and the stream window the chain can
// reach (wn floats, when it fits) staged in LDS, so each link reads LDS instead of global memory.
template <bool STAGED>
__global__ void __launch_bounds__(1024) k_pms_guess(PmsDev d, int t_lo, long long wn) {
    extern __shared__ float gsm[];
    const int nt = d.K - t_lo, tid = threadIdx.x;
    const long long o0 = d.off[0];
    const long long tks = d.prof && tid == 0 ? (long long)wall_clock64() : 0;
    // STAGED: per-tree dd, degree and result offset, and the reachable stream window (wn floats), in
    // LDS -- the chain then touches no global memory (a global access would make every link wait on
    // the previous links' traffic)
    float* sdd = gsm;
    int* sdeg = reinterpret_cast<int*>(gsm + nt);
    long long* sog = reinterpret_cast<long long*>(gsm + ((3 * nt + 1) & ~1));
    float* sdice = reinterpret_cast<float*>(sog + nt);
    if (STAGED) {
        // Per tree, in parallel: each refinement level's range test rd = fmaf(dice, max_d, dd) is monotone in
        // the draw (dice in [-1, 1], one rounding), so a level whose two extreme rd are both in [0, Dmax] is
        // in range whatever it draws (4 draws), one whose extremes are both below 0 or both above Dmax is out
        // (1 draw); only the others read the stream.  sdeg holds the degree and the level classes, 2 bits
        // per level (1 always in, 0 always out, 2 draw-dependent).  The serial chain then reads one LDS
        // word per draw-dependent level instead of one per level: the same offsets as ref_count.
        const float fmax = (float)d.Dmax;
        for (int i = tid; i < nt; i += blockDim.x) {
            const float dd = ref_dd(d, t_lo + i);
            sdd[i] = dd;
            uint32_t cls = 0;
            int l = 0;
            for (float md = 0.5f * fmax; md > 0.1f; md *= 0.5f, ++l) {
                const float lo = fmaf(-1.0f, md, dd), hi = fmaf(1.0f, md, dd);
                const bool lo_in = !(lo < 0.0f || lo > fmax), hi_in = !(hi < 0.0f || hi > fmax);
                const uint32_t c = (lo_in && hi_in) ? 1u : (hi < 0.0f || lo > fmax) ? 0u : 2u;
                cls |= c << (2 * l);
            }
            sdeg[2 * i] = tree_deg(d, t_lo + i);
            sdeg[2 * i + 1] = (int)cls;
        }
        for (long long i = tid; i < wn; i += blockDim.x) sdice[i] = o0 + i < d.dice_n ? d.dice[o0 + i] : 0.0f;
        __syncthreads();
        long long tk0 = 0;  // SM_PMS_PROF builds: staging / chain wall-clock split (100 MHz ticks)
        if (d.prof && tid == 0) {
            tk0 = (long long)wall_clock64();
            atomicAdd((unsigned long long*)&d.prof[9], (unsigned long long)(tk0 - tks));
        }
        if (tid < 64) {
            // The chain on one wave with wave-uniform (scalar) state: each tree's degree, classes and dd come
            // from a 64-tree register window and each draw-dependent level's draw from a 64-draw register
            // window, both by readlane, so a link costs no LDS round trip unless a window is refilled.  Only
            // the draw-dependent (class 2) levels are visited: the fixed levels between them advance the
            // offset by popcounts (4 draws per always-in level, 1 per always-out one), and level i's
            // max_d = (Dmax / 2) * 2^-i exactly (the loop's halvings).  A tree whose draws could pass the end
            // of the stream takes the level-by-level loop with ref_count's checks.
            const int lane = tid;
            int nlev = 0;
            for (float md = 0.5f * fmax; md > 0.1f; md *= 0.5f) ++nlev;
            const uint32_t lvmask = nlev >= 16 ? 0xFFFFFFFFu : (1u << (2 * nlev)) - 1u;
            long long o = o0, og_w = 0;
            int tw = -64, wdeg = 0, wcls = 0, wdd = 0;
            long long kw = LLONG_MIN / 2;
            float wdice = 0.0f;
            auto draw = [&](long long k) {
                if (k >= kw + 64) {  // the next 64 draws from k
                    kw = k;
                    const long long q = k - o0 + lane;
                    wdice = q < wn ? sdice[q] : 0.0f;
                }
                return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wdice), (int)(k - kw)));
            };
            for (int t = 0; t < nt; ++t) {
                if (t - tw >= 64) {  // the next 64 trees (the finished window's offsets to LDS)
                    if (tw >= 0 && tw + lane < nt) sog[tw + lane] = og_w;
                    tw = t;
                    const int ti = t + lane;
                    wdeg = ti < nt ? sdeg[2 * ti] : 0;
                    wcls = ti < nt ? sdeg[2 * ti + 1] : 0;
                    wdd = ti < nt ? __float_as_int(sdd[ti]) : 0;
                }
                if (lane == t - tw) og_w = o;
                const int deg = __builtin_amdgcn_readlane(wdeg, t - tw);
                const uint32_t cls = (uint32_t)__builtin_amdgcn_readlane(wcls, t - tw) & lvmask;
                const float dd = __int_as_float(__builtin_amdgcn_readlane(wdd, t - tw));
                long long k = o + deg;
                if (k + 4ll * nlev > d.dice_n) {  // near the end of the stream: ref_count's checks level by level
                    uint32_t c2 = cls;
                    for (float md = 0.5f * fmax; md > 0.1f; md *= 0.5f, c2 >>= 2) {
                        if (k + 4 > d.dice_n) {
                            if (lane == 0) atomicOr(d.err, 4u);
                            break;
                        }
                        const uint32_t c = c2 & 3u;
                        bool in = c == 1u;
                        if (c == 2u) {
                            const float rd = fmaf(draw(k), md, dd);
                            in = !(rd < 0.0f || rd > fmax);
                        }
                        k += in ? 4 : 1;
                    }
                    o = k;
                    continue;
                }
                // per level 2 bits: 01 in, 00 out, 10 draw-dependent; odd bits mark class 2, even bits class 1
                const uint32_t hi = cls & 0xAAAAAAAAu, lo = cls & 0x55555555u;
                uint32_t c2 = hi;
                int lvl = 0;  // the next level not yet counted (bit 2 * lvl)
                while (c2) {
                    const int b = __builtin_ctz(c2);  // bit 2i + 1 of class-2 level i
                    const int i = b >> 1;
                    const uint32_t below = (1u << (2 * i)) - (1u << (2 * lvl));  // levels [lvl, i), both bits
                    const int nin = __builtin_popcount(lo & below), nfix = i - lvl;
                    k += 4 * nin + (nfix - nin);
                    const float md = ldexpf(0.5f * fmax, -i);
                    const float rd = fmaf(draw(k), md, dd);
                    k += !(rd < 0.0f || rd > fmax) ? 4 : 1;
                    lvl = i + 1;
                    c2 &= c2 - 1;
                }
                const uint32_t rest = lvmask & ~((1u << (2 * lvl)) - 1u);  // levels [lvl, nlev)
                const int nin = __builtin_popcount(lo & rest), nfix = nlev - lvl;
                k += 4 * nin + (nfix - nin);
                o = k;
            }
            if (tw >= 0 && tw + lane < nt) sog[tw + lane] = og_w;
        }
        __syncthreads();
        if (d.prof && tid == 0) atomicAdd((unsigned long long*)&d.prof[10], (unsigned long long)((long long)wall_clock64() - tk0));
        for (int i = tid; i < nt; i += blockDim.x) d.oguess[t_lo + i] = sog[i];
        return;
    }
    if (tid != 0) return;
    long long o = o0;
    for (int t = t_lo; t < d.K; ++t) {
        d.oguess[t] = o;
        const int deg = tree_deg(d, t);
        o += deg + ref_count(d, ref_dd(d, t), o + deg, [&](long long k) { return d.dice[k]; });
    }
}

// serial mode, one large tree with the whole GPU: after its propagation update, its refinement labels, which
// advance the offset (its propagation labels: k_pms_prop_tree below)
__global__ void k_pms_ref_one(PmsDev d, int t) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    const int deg = tree_deg(d, t);
    const long long o = d.off[0];
    d.off[0] = o + deg + ref_levels(d, t, o + deg, true);
}

__global__ void k_pms_prop_setup(PmsDev d, int t_lo) {
    // one thread per (tree, neighbour): nb entries from nb_start[t_lo]
    const int e = d.nb_start[t_lo] + (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (e >= d.nb_start[d.K]) return;
    // tree of entry e: binary search in nb_start
    int lo = t_lo, hi = d.K - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (d.nb_start[mid] <= e) lo = mid;
        else hi = mid - 1;
    }
    prop_label(d, lo, d.oguess[lo], e - d.nb_start[lo]);
}

// Propagation proposals of trees [t_lo, t_hi) without repeats, one wave per tree: the first occurrence of
// each bitwise-distinct label, in proposal order, into labu, and their count into nprop.  A repeated
// label has the same data terms and aggregates to bitwise the same costs as its first occurrence, which
// comes earlier in the strict-< scan (:173-185), so it can never win: the pass runs on labu / nprop
// with every pixel's result unchanged.  (In later calls many neighbour trees propose the same plane.)
__global__ void __launch_bounds__(256) k_pms_prop_dedupe(PmsDev d, int t_lo, int t_hi) {
    const int t = t_lo + (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    if (t >= t_hi) return;
    const int lane = (int)(threadIdx.x & 63);
    const int deg = tree_deg(d, t), base = d.tree_lab[t];
    int n = 0;
    for (int j0 = 0; j0 < deg; j0 += 64) {
        const int j = j0 + lane;
        bool keep = false;
        float4 L = make_float4(0.f, 0.f, 0.f, 0.f);
        if (j < deg) {
            L = d.lab[base + j];
            keep = true;
            for (int i = 0; i < j; ++i) {
                const float4 M = d.lab[base + i];
                if (__float_as_uint(M.x) == __float_as_uint(L.x) && __float_as_uint(M.y) == __float_as_uint(L.y) &&
                    __float_as_uint(M.z) == __float_as_uint(L.z)) {
                    keep = false;
                    break;
                }
            }
        }
        const unsigned long long m = __ballot(keep);
        if (keep) d.labu[base + n + __popcll(m & ((1ull << lane) - 1ull))] = L;
        n += __popcll(m);
    }
    if (lane == 0) d.nprop[t] = n;
}

// serial mode, one large tree: its propagation labels from the running offset and k_pms_prop_dedupe of that
// tree in one block (round 5: k_pms_prop_one and the dedupe were two launches per large tree; the first
// call is bound by its ~10k launches): the labels, a block barrier, then wave 0 keeps the first occurrence
// of each distinct label, as k_pms_prop_dedupe does
__global__ void __launch_bounds__(256) k_pms_prop_tree(PmsDev d, int t) {
    const int deg = tree_deg(d, t);
    const long long o = d.off[0];
    for (int j = (int)threadIdx.x; j < deg; j += (int)blockDim.x) prop_label(d, t, o, j);
    __threadfence_block();
    __syncthreads();
    if (threadIdx.x >= 64) return;
    const int lane = (int)threadIdx.x, base = d.tree_lab[t];
    int n = 0;
    for (int j0 = 0; j0 < deg; j0 += 64) {
        const int j = j0 + lane;
        bool keep = false;
        float4 L = make_float4(0.f, 0.f, 0.f, 0.f);
        if (j < deg) {
            L = d.lab[base + j];
            keep = true;
            for (int i = 0; i < j; ++i) {
                const float4 M = d.lab[base + i];
                if (__float_as_uint(M.x) == __float_as_uint(L.x) && __float_as_uint(M.y) == __float_as_uint(L.y) &&
                    __float_as_uint(M.z) == __float_as_uint(L.z)) {
                    keep = false;
                    break;
                }
            }
        }
        const unsigned long long m = __ballot(keep);
        if (keep) d.labu[base + n + __popcll(m & ((1ull << lane) - 1ull))] = L;
        n += __popcll(m);
    }
    if (lane == 0) d.nprop[t] = n;
}

// The data term of every row of [row_lo, row_hi) for the phase's proposals, into the A rows (the up
// walks' PRE input): rows with few proposals one per lane, wider ones by the whole wave.
__global__ void __launch_bounds__(256) k_pms_cost(PmsDev d, int phase, int row_lo, int row_hi) {
    const int lane = (int)(threadIdx.x & 63);
    const int base_row = row_lo + (int)((blockIdx.x * blockDim.x + threadIdx.x) & ~63u);
    const int row = base_row + lane;
    const bool valid = row < row_hi;
    int t = 0, P = 0, lb = 0;
    if (valid) {
        t = d.rtree[row];
        phase_labels(d, phase, t, P, lb);
    }
    const bool wide = valid && P > 16;
    if (valid && !wide) cost_row(d, row, t, P, lb, 0, 1);
    unsigned long long m = __ballot(wide);
    while (m) {
        const int b = __ffsll((long long)m) - 1;
        m &= m - 1;
        cost_row(d, base_row + b, __shfl(t, b), __shfl(P, b), __shfl(lb, b), lane, 64);
    }
}


// ----------------------------------------------------------------------------- per-phase layout
// The A rows of a phase hold its P proposals per node.  The static layout (tree_pt / tree_abase) has
// room for the most a tree can have (max(deg, L) + 1: the first call's propagation), but a later call's
// propagation keeps a handful of distinct labels per tree (C2: ~2 on average), so its rows were mostly
// air: the big tree's 618k rows at 238 doubles spread a phase over 1.2 GB.  k_pms_layout packs the
// phase's rows with a stride of P rounded up to even (16-byte rows), per tree an exclusive scan of
// size x stride, into pt_out / ab_out, which the phase's kernels then take as tree_pt / tree_abase.
// A rows are scratch of one phase (the outputs are minc and abc), so each phase may lay them out anew.
__global__ void __launch_bounds__(1024) k_pms_layout(PmsDev d, int phase, int t_lo, int t_hi, int32_t* pt_out,
                                                     long long* ab_out, int32_t* zero, int nzero) {
    __shared__ long long s_w[16];
    const int tid = (int)threadIdx.x, lane = tid & 63, wv = tid >> 6;
    for (int i = tid; i < nzero; i += 1024) zero[i] = 0;  // the phase's plan counters (k_pms_plan), one launch fewer
    long long base = 0;
    for (int t0 = t_lo; t0 < t_hi; t0 += 1024) {
        const int t = t0 + tid;
        long long v = 0;
        int stride = 2;
        if (t < t_hi) {
            int P, lb;
            phase_labels(d, phase, t, P, lb);
            stride = P > 2 ? (P + 1) & ~1 : 2;
            v = (long long)(d.tree_start[t + 1] - d.tree_start[t]) * stride;
        }
        long long incl = v;
#pragma unroll
        for (int k = 1; k < 64; k <<= 1) {
            const long long u = __shfl_up(incl, k);
            if (lane >= k) incl += u;
        }
        if (lane == 63) s_w[wv] = incl;
        __syncthreads();
        long long pre = 0, tot = 0;
        for (int k = 0; k < 16; ++k) {
            if (k < wv) pre += s_w[k];
            tot += s_w[k];
        }
        if (t < t_hi) {
            pt_out[t] = stride;
            ab_out[t] = base + pre + incl - v;
        }
        base += tot;
        __syncthreads();
    }
}

// ----------------------------------------------------------------------------- planned walks
// In the later (speculative) calls the propagation dedupe leaves a tree only a few distinct labels (C2:
// ~2.4 node-label evaluations per node and call over both phases), yet a wave per (path, 64-proposal
// chunk) walks every path: up to 350k waves per round for a handful of active lanes each.  The plan
// (k_pms_plan) sorts a round's paths by their tree's proposal count P into lane-group classes, and the
// walk kernel (k_pms_walk_plan, a persistent grid) lets GW lanes walk one path: lane j of the group
// evaluates proposal j < P, so one wave walks 64 / GW paths.  Paths with P > 8 keep the wave walker
// (up_walk / down_walk, one wave per 64-proposal chunk).  Each lane performs exactly the wave walker's
// operations on its (path, proposal) -- the same fma order, the same guesses at cut pieces -- so the A
// rows are bitwise the same whichever walker ran.
constexpr int PMS_GCH = 4;  // nodes whose loads a group walker issues together

__device__ __forceinline__ int pms_class_gw(int c) { return c == 0 ? 2 : 8; }
__device__ __forceinline__ int pms_class_of(int P) { return P <= 2 ? 0 : P <= 8 ? 1 : 2; }

// the up-walk fields of row r: words 2..9 of the PmsRow (children, w | nch | hk, child weights, x | y)
struct GMeta {
    uint2 c01, c23, w6, w8;
};
__device__ __forceinline__ GMeta gmeta_load(const PmsRow* rows, int r) {
    const uint2* b = reinterpret_cast<const uint2*>(reinterpret_cast<const uint32_t*>(rows + r) + 2);
    GMeta m;
    m.c01 = b[0];
    m.c23 = b[1];
    m.w6 = b[2];
    m.w8 = b[3];
    return m;
}

// Leaf->root walk of path `path` (rows [row, row + len), bottom to head, from x = 0 below the bottom: a
// leaf, or a cut piece's guess) for proposal j of the lane's group; the up_walk<false, true> recurrence
// per lane.  Chunks of PMS_GCH nodes: a chunk's child and cost rows are loaded together, its successor's
// metadata behind them.
template <int GW>
__device__ void up_group(const PmsDev& d, const double* __restrict__ sS, int phase, int path) {
    const int j = (int)(threadIdx.x & 63) % GW;
    int P = 0, base = 0, t = 0, r0 = 0, len = 0;
    if (path >= 0) {
        const PmsPath pa = d.paths[path];
        t = pa.tree;
        r0 = pa.row;
        len = pa.len;
        phase_labels(d, phase, t, P, base);
    }
    if (j >= P) return;
    const int ts = d.tree_start[t], pt = d.tree_pt[t];
    double* __restrict__ A = d.A + d.tree_abase[t] + j;
    double x = 0.0;
    int i0 = len - 1;
    GMeta mc[PMS_GCH];
#pragma unroll
    for (int k = 0; k < PMS_GCH; ++k) mc[k] = gmeta_load(d.rows, r0 + (i0 - k >= 0 ? i0 - k : 0));
    while (i0 >= 0) {
        const int n = i0 + 1 < PMS_GCH ? i0 + 1 : PMS_GCH;
        double cv[PMS_GCH][4], cost[PMS_GCH];
#pragma unroll
        for (int k = 0; k < PMS_GCH; ++k) {
            const int row = r0 + i0 - (k < n ? k : 0);
            const int nch = (int)((mc[k].w6.x >> 16) & 255u), hk = (int)(mc[k].w6.x >> 24);
            const uint32_t ch[4] = {mc[k].c01.x, mc[k].c01.y, mc[k].c23.x, mc[k].c23.y};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                cv[k][q] = 0.0;  // only the light children's rows (no dummy loads of absent ones)
                if (q < nch && q != hk) cv[k][q] = A[(size_t)((int)ch[q] - ts) * pt];
            }
            cost[k] = A[(size_t)(row - ts) * pt];
        }
        const int i0n = i0 - n;
        GMeta mn[PMS_GCH];
#pragma unroll
        for (int k = 0; k < PMS_GCH; ++k) mn[k] = gmeta_load(d.rows, r0 + (i0n - k >= 0 ? i0n - k : 0));
#pragma unroll
        for (int k = 0; k < PMS_GCH; ++k) {
            if (k >= n) break;
            const int nch = (int)((mc[k].w6.x >> 16) & 255u), hk = (int)(mc[k].w6.x >> 24);
            const int wc[4] = {(int)(mc[k].w6.y & 0xFFFFu), (int)(mc[k].w6.y >> 16), (int)(mc[k].w8.x & 0xFFFFu),
                               (int)(mc[k].w8.x >> 16)};
            double acc = 0.0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (q >= nch) break;
                const double v = q == hk ? x : cv[k][q];
                acc = fma(v, sS[wc[q]], acc);  // as up_walk (0x40fad5)
            }
            x = cost[k] + acc;
            A[(size_t)(r0 + i0 - k - ts) * pt] = x;
        }
#pragma unroll
        for (int k = 0; k < PMS_GCH; ++k) mc[k] = mn[k];
        i0 = i0n;
    }
}

// Root->leaf walk of path `path`, head to bottom, A(c) = fma(S_c, A(p), S2_c * A_up(c)) per lane (the
// down_walk<false> recurrence); the next chunk's A_up rows and weights are loaded while one runs.
template <int GW>
__device__ void down_group(const PmsDev& d, const double* __restrict__ sS, const double* __restrict__ sS2, int phase,
                           int path) {
    const int j = (int)(threadIdx.x & 63) % GW;
    int P = 0, base = 0, t = 0, r0 = 0, len = 0;
    if (path >= 0) {
        const PmsPath pa = d.paths[path];
        t = pa.tree;
        r0 = pa.row;
        len = pa.len;
        phase_labels(d, phase, t, P, base);
    }
    if (j >= P) return;
    const int ts = d.tree_start[t], pt = d.tree_pt[t];
    double* __restrict__ A = d.A + d.tree_abase[t] + j;
    const int parent = d.rows[r0].parent;
    double y = parent >= 0 ? A[(size_t)(parent - ts) * pt] : 0.0;
    auto ld = [&](double (&u)[PMS_GCH], int (&w)[PMS_GCH], int i0) {
#pragma unroll
        for (int k = 0; k < PMS_GCH; ++k) {
            const int i = i0 + k < len ? i0 + k : 0;  // clamped: every load from a valid row
            u[k] = A[(size_t)(r0 + i - ts) * pt];
            w[k] = (int)(d.rows[r0 + i].w);
        }
    };
    double uc[PMS_GCH];
    int wc[PMS_GCH];
    ld(uc, wc, 0);
    for (int i0 = 0; i0 < len; i0 += PMS_GCH) {
        double un[PMS_GCH];
        int wn[PMS_GCH];
        ld(un, wn, i0 + PMS_GCH);
#pragma unroll
        for (int k = 0; k < PMS_GCH; ++k) {
            if (i0 + k >= len) break;
            const double S = sS[wc[k]], S2 = sS2[wc[k]];
            if (i0 + k == 0) y = parent >= 0 ? fma(S, y, S2 * uc[0]) : uc[0];
            else y = fma(S, y, S2 * uc[k]);
            A[(size_t)(r0 + i0 + k - ts) * pt] = y;
        }
#pragma unroll
        for (int k = 0; k < PMS_GCH; ++k) {
            uc[k] = un[k];
            wc[k] = wn[k];
        }
    }
}

// The plan of trees [t_lo, t_hi) for one phase: blockIdx.y = round r, one thread per path of the round.
constexpr int PMS_CHAIN_LEN = SM_PMS_CHAIN_LEN;  // from here on: k_pms_chain

__global__ void __launch_bounds__(1024) k_pms_plan(PmsDev d, int phase, int t_lo, int t_hi, int chain_len) {
    __shared__ int s_n[PMS_NCNT], s_base[PMS_NCNT];
    const int r = (int)blockIdx.y, K1 = d.K + 1;
    const int p0 = d.rt_path[(size_t)r * K1 + t_lo], p1 = d.rt_path[(size_t)r * K1 + t_hi];
    const int p = p0 + (int)(blockIdx.x * blockDim.x + threadIdx.x);
    const int lane = (int)(threadIdx.x & 63);
    if (threadIdx.x < PMS_NCNT) s_n[threadIdx.x] = 0;
    __syncthreads();
    int P = 0, base = 0, len = 0;
    if (p < p1) {
        const PmsPath pa = d.paths[p];
        len = pa.len;
        phase_labels(d, phase, pa.tree, P, base);
    }
    // classes: 0 / 1 lane groups, 2 wave items, 3 chain items (k_pms_chain)
    const int c = P <= 0 ? -1 : len >= chain_len ? 3 : len >= PMS_GLONG ? 2 : pms_class_of(P);
    const int nchunk = c >= 2 ? (P + 63) / 64 : 1;
    // block-aggregated appends: wave offsets in LDS, one global atomic per class and block
    int wpos[PMS_NCNT];
#pragma unroll
    for (int k = 0; k < PMS_NCNT; ++k) {
        int v = c == k ? nchunk : 0, incl = v;  // an exclusive wave scan of the entries of class k
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int t = __shfl_up(incl, o);
            if (lane >= o) incl += t;
        }
        const int cnt_w = __shfl(incl, 63);
        int wb = 0;
        if (lane == 0 && cnt_w) wb = atomicAdd(&s_n[k], cnt_w);
        wpos[k] = __shfl(wb, 0) + incl - v;
    }
    __syncthreads();
    if (threadIdx.x < PMS_NCNT)
        s_base[threadIdx.x] = s_n[threadIdx.x] ? atomicAdd(d.plan_cnt + r * PMS_NCNT + threadIdx.x, s_n[threadIdx.x]) : 0;
    __syncthreads();
    if (c < 0) return;
    const int pos = s_base[c] + wpos[c];
    if (c < 2) {
        d.plan_path[(size_t)c * d.npaths_total + d.plan_base[r] + pos] = p;
    } else {
        PmsItem* out = d.plan_item + (c == 3 ? (size_t)d.item_cap : 0) + d.plan_ibase[r] + pos;
        for (int k = 0; k < nchunk; ++k) out[k] = PmsItem{p, k};
    }
}

// One round's planned walk over a persistent grid: wave w takes virtual tasks w, w + waves, ...: first
// the class-0 waves (32 paths each), then class 1 (8 paths each), then one (path, chunk) item each.
__global__ void __launch_bounds__(256) k_pms_walk_plan(PmsDev d, int phase, int up, int r) {
    __shared__ double sS[PMS_NW], sS2[PMS_NW];
    for (int i = threadIdx.x; i < PMS_NW; i += blockDim.x) {
        sS[i] = d.slut[i];
        sS2[i] = d.s2lut[i];
    }
    __syncthreads();
    const int* cnt = d.plan_cnt + r * PMS_NCNT;
    const int n0 = cnt[0], n1 = cnt[1], n2 = cnt[2];
    const int T0 = (n0 + 31) / 32, T1 = (n1 + 7) / 8, T = T0 + T1 + n2;
    const int lane = (int)(threadIdx.x & 63);
    const int nw = (int)(gridDim.x * (blockDim.x >> 6));
    for (int w = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6); w < T; w += nw) {
        if (w < T0) {
            const int k = w * 32 + lane / 2;
            const int path = k < n0 ? d.plan_path[d.plan_base[r] + k] : -1;
            if (up) up_group<2>(d, sS, phase, path);
            else down_group<2>(d, sS, sS2, phase, path);
        } else if (w < T0 + T1) {
            const int k = (w - T0) * 8 + lane / 8;
            const int path = k < n1 ? d.plan_path[(size_t)d.npaths_total + d.plan_base[r] + k] : -1;
            if (up) up_group<8>(d, sS, phase, path);
            else down_group<8>(d, sS, sS2, phase, path);
        } else {
            const PmsItem it = d.plan_item[d.plan_ibase[r] + (w - T0 - T1)];
            if (up) up_item(d, sS, phase, uni(it.path), uni(it.chunk));
            else down_item(d, sS, sS2, phase, uni(it.path), uni(it.chunk));
        }
    }
}

// ----------------------------------------------------------------------------- chains (long paths)
// A path (or piece) of at least PMS_CHAIN_LEN rows is a long latency chain for the walkers: each PMS_CH
// nodes cost a memory round trip (~3 us at C2 in rounds with many walkers).  k_pms_chain walks it with
// one workgroup per (path, 64-proposal chunk): PC_LW loader waves take the groups of PC_G nodes in turn,
// load everything a node needs and stage it in an LDS ring of PC_NS slots; the chain wave runs the
// recurrence from LDS and only stores.  Up (bottom to head): a loader folds the light children that
// precede the heavy one in fold order into pre (from +0, as the walkers do), and stages the post-heavy
// light rows and the cost; the chain then does acc = fma(x, S_heavy, pre), the post children in order,
// x = cost + acc -- up_walk's operations, the fold split at the heavy child.  A node with a third
// post-heavy child (only a tree root can have one) has the chain read that row itself.  Down (head to
// bottom): a loader stages T = S2 * A_up and S, the chain does y = fma(S, y, T); the head reads its
// parent row (or keeps A_up at a tree root) -- down_walk's operations.  Same bits as the walkers.
constexpr int PC_G = 8;        // nodes per group

// a[i] of a 4-element register array by selects: a runtime index into a local array would put the array
// in scratch memory (the up loaders had 272 bytes of it per lane)
__device__ __forceinline__ double pc_sel(const double (&a)[4], int i) {
    return i == 0 ? a[0] : i == 1 ? a[1] : i == 2 ? a[2] : a[3];
}
__device__ __forceinline__ int pc_sel(const int (&a)[4], int i) { return i == 0 ? a[0] : i == 1 ? a[1] : i == 2 ? a[2] : a[3]; }
// up ring slots (2 KB per node): 6 = ~100 KB, one workgroup per CU.  4 (67 KB, two per CU) was faster while
// the loaders' rows sat in scratch memory; without it 6 is: 100-call C2 frame 487-491 -> 473 ms (profiles/r04/nsu/)
constexpr int PC_NSU = 6;
constexpr int PC_NSU_MAX = 8;  // SM_PMS_CHAIN_NSU up to this: 133 KB, one workgroup per CU
constexpr int PC_NSD = 14;     // down ring slots (0.5 KB per node): 58 KB, two workgroups per CU
constexpr int PC_LW = 7;       // loader waves (+ the chain wave: 512 threads)

struct PcUpSlot {
    double2 pc[PC_G][64];  // (pre, cost): one 16-byte LDS read per node and lane
    double2 pp[PC_G][64];  // (post1, post2)
    double sh[PC_G], s1[PC_G], s2[PC_G];
    double s3;   // the group's node with a third post-heavy child (a tree root; at most one): its S,
    int k3, p3;  // its index in the group (-1: none) and the child's row
};
struct PcDnSlot {
    double T[PC_G][64];
    double S[PC_G];
};

__device__ __forceinline__ void pc_publish(int* p, int v) {  // after this wave's LDS writes have landed
    __builtin_amdgcn_s_waitcnt(0xC07F);                       // lgkmcnt(0)
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}
__device__ __forceinline__ void pc_publish_ordered(int* p, int v) {  // LDS reads issued before complete first
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}
__device__ __forceinline__ void pc_wait_ge(int* p, int v) {
    while (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < v) __builtin_amdgcn_s_sleep(1);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// (512, 2): two workgroups per CU -- 4 waves per SIMD, so up to 128 VGPRs.  With the bare bound the compiler
// aimed at 8 waves per SIMD, gave the kernel 64 VGPRs and spilled the up loaders' rows to scratch.
template <bool UP>
__global__ void __launch_bounds__(512, 2) k_pms_chain(PmsDev d, int phase, int r, int ns) {
    extern __shared__ double2 pc_lds[];  // 16-byte aligned: the up ring is read as double2
    __shared__ double sS[PMS_NW], sS2[PMS_NW];
    __shared__ int s_staged[PC_NSD], s_freed;
    const int tid = (int)threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int NS = ns;  // ring slots (<= PC_NSU / PC_NSD): fewer slots, more workgroups per CU
    // the grid is the schedule's bound (paths of >= SM_PMS_CHAIN_LEN rows); blocks past the plan's chain
    // items leave before touching anything
    if ((int)blockIdx.x >= d.plan_cnt[r * PMS_NCNT + PMS_NCLS]) return;
    for (int i = tid; i < PMS_NW; i += blockDim.x) {
        sS[i] = d.slut[i];
        sS2[i] = d.s2lut[i];
    }
    if (tid < PC_NSD) s_staged[tid] = 0;
    if (tid == 0) s_freed = 0;
    __syncthreads();
    const PmsItem it = d.plan_item[(size_t)d.item_cap + d.plan_ibase[r] + blockIdx.x];
    const PmsPath pa = d.paths[it.path];
    const int t = pa.tree, r0 = pa.row, len = pa.len;
    int P, base;
    phase_labels(d, phase, t, P, base);
    const int j = it.chunk * 64 + lane;
    const bool act = j < P;
    const int ts = d.tree_start[t], pt = d.tree_pt[t];
    double* __restrict__ A = d.A + d.tree_abase[t] + j;
    const double* __restrict__ Al = d.A + d.tree_abase[t] + (act ? j : 0);
    const int ngroups = (len + PC_G - 1) / PC_G;
    if (UP) {
        PcUpSlot* ring = reinterpret_cast<PcUpSlot*>(pc_lds);
        if (wave > 0) {  // loaders: groups wave - 1, wave - 1 + PC_LW, ...
            // a group's metadata is loaded during the previous group (after its row loads), so each group
            // costs one memory round trip (metadata -> rows was two)
            auto gmeta = [&](int gg) {
                const int it = len - 1 - gg * PC_G, il = it - PC_G + 1 > 0 ? it - PC_G + 1 : 0;
                return meta_load(d.rows, r0 + il, it - il + 1);
            };
            ChunkMeta m = gmeta(wave - 1 < ngroups ? wave - 1 : 0);  // unconditional (clamped)
            for (int g = wave - 1; g < ngroups; g += PC_LW) {
                const int itop = len - 1 - g * PC_G;                 // the group's first (lowest) node
                const int ilo = itop - PC_G + 1 > 0 ? itop - PC_G + 1 : 0;
                const int n = itop - ilo + 1;
                double cv[PC_G][4], cost[PC_G];
#pragma unroll
                for (int k = 0; k < PC_G; ++k) {
                    const int kk = k < n ? k : 0;
                    const int row = r0 + itop - kk, w0 = (itop - kk - ilo) * 10;
                    const uint32_t w6 = meta_dw(m, w0 + 6);
                    const int nch = (int)((w6 >> 16) & 255u), hk = (int)(w6 >> 24);
                    // only the light children's rows (wave-uniform tests): most nodes have none, and the
                    // dummy reloads of absent children made the up loaders 5 row loads per node
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        cv[k][q] = 0.0;
                        if (q < nch && q != hk) cv[k][q] = Al[(size_t)((int)meta_dw(m, w0 + 2 + q) - ts) * pt];
                    }
                    cost[k] = Al[(size_t)(row - ts) * pt];
                }
                const ChunkMeta mn = gmeta(g + PC_LW < ngroups ? g + PC_LW : g);  // the next group's (clamped)
                const int s = g % NS;
                pc_wait_ge(&s_freed, g - NS + 1);  // the slot's previous group is consumed
                PcUpSlot& sl = ring[s];
                int k3 = -1, p3 = 0;
                double s3 = 0.0;
#pragma unroll
                for (int k = 0; k < PC_G; ++k) {
                    if (k >= n) break;
                    const int w0 = (itop - k - ilo) * 10;
                    const uint32_t w6 = meta_dw(m, w0 + 6), w7 = meta_dw(m, w0 + 7), w8 = meta_dw(m, w0 + 8);
                    const int nch = (int)((w6 >> 16) & 255u), hk = (int)(w6 >> 24);
                    const int wc[4] = {(int)(w7 & 0xFFFFu), (int)(w7 >> 16), (int)(w8 & 0xFFFFu), (int)(w8 >> 16)};
                    const int h = hk == 0xFF ? nch : hk;  // fold position of the heavy child (a leaf: none)
                    double pre = 0.0;
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        if (q < h) pre = fma(cv[k][q], sS[wc[q]], pre);
                    sl.pc[k][lane] = make_double2(pre, cost[k]);
                    const int np = hk == 0xFF ? 0 : nch - 1 - hk;
                    sl.pp[k][lane] = make_double2(np >= 1 ? pc_sel(cv[k], (hk + 1) & 3) : 0.0,
                                                  np >= 2 ? pc_sel(cv[k], (hk + 2) & 3) : 0.0);
                    if (lane == 0) {
                        sl.sh[k] = hk == 0xFF ? 0.0 : sS[pc_sel(wc, hk & 3)];
                        sl.s1[k] = np >= 1 ? sS[pc_sel(wc, (hk + 1) & 3)] : 0.0;
                        sl.s2[k] = np >= 2 ? sS[pc_sel(wc, (hk + 2) & 3)] : 0.0;
                    }
                    if (np >= 3) {
                        k3 = k;
                        p3 = (int)meta_dw(m, w0 + 5);
                        s3 = sS[wc[3]];
                    }
                }
                if (lane == 0) {
                    sl.k3 = k3;
                    sl.p3 = p3;
                    sl.s3 = s3;
                }
                pc_publish(&s_staged[s], g + 1);
                m = mn;
            }
        } else {  // the chain wave
            double x = 0.0;  // the bottom row's heavy child: a leaf's none, a cut piece's guess 0
            const long long tc0 = d.prof ? (long long)wall_clock64() : 0;  // SM_PMS_PROF: per-item timing
            for (int g = 0; g < ngroups; ++g) {
                const int s = g % NS;
                pc_wait_ge(&s_staged[s], g + 1);
                const PcUpSlot& sl = ring[s];
                const int itop = len - 1 - g * PC_G;
                const int n = itop + 1 < PC_G ? itop + 1 : PC_G;
                // the whole group from LDS in one batch, then the recurrence from registers (absent posts
                // were staged as 0 with S = 0: fma(0, 0, acc) == acc, aggregates are finite and >= +0)
                double pre[PC_G], p1[PC_G], p2[PC_G], cst[PC_G], sh[PC_G], s1[PC_G], s2[PC_G];
#pragma unroll
                for (int k = 0; k < PC_G; ++k) {
                    const double2 pc = sl.pc[k][lane], pp = sl.pp[k][lane];
                    pre[k] = pc.x;
                    cst[k] = pc.y;
                    p1[k] = pp.x;
                    p2[k] = pp.y;
                    sh[k] = sl.sh[k];
                    s1[k] = sl.s1[k];
                    s2[k] = sl.s2[k];
                }
                // a tree root's third post-heavy child (rare): read with the group, before the slot is released
                const int k3 = sl.k3, p3row = sl.p3;
                const double s3 = sl.s3;
                pc_publish_ordered(&s_freed, g + 1);  // the slot's reads are issued: free it
                const int np3 = k3 >= 0 ? 1 << k3 : 0;
#pragma unroll
                for (int k = 0; k < PC_G; ++k) {
                    if (k >= n) break;
                    double acc = fma(x, sh[k], pre[k]);  // a leaf: fma(0, 0, +0) = +0
                    acc = fma(p1[k], s1[k], acc);
                    acc = fma(p2[k], s2[k], acc);
                    if (__builtin_expect((np3 >> k) & 1, 0))  // a tree root's third post-heavy child
                        acc = fma(Al[(size_t)(p3row - ts) * pt], s3, acc);
                    x = cst[k] + acc;
                    if (act) A[(size_t)(r0 + itop - k - ts) * pt] = x;
                }
            }
            if (d.prof && lane == 0) {  // the call's longest up item (ticks << 24 | rows), totals
                const long long dt = (long long)wall_clock64() - tc0;
                atomicMax((unsigned long long*)&d.prof[11], (unsigned long long)((dt << 24) | (long long)len));
                atomicAdd((unsigned long long*)&d.prof[12], (unsigned long long)dt);
                atomicAdd((unsigned long long*)&d.prof[13], (unsigned long long)len);
                atomicAdd((unsigned long long*)&d.prof[14], 1ull);
            }
        }
    } else {
        PcDnSlot* ring = reinterpret_cast<PcDnSlot*>(pc_lds);
        if (wave > 0) {
            for (int g = wave - 1; g < ngroups; g += PC_LW) {
                const int i0 = g * PC_G;
                const int n = len - i0 < PC_G ? len - i0 : PC_G;
                double u[PC_G];
                int w[PC_G];
#pragma unroll
                for (int k = 0; k < PC_G; ++k) {
                    const int i = i0 + (k < n ? k : 0);
                    u[k] = Al[(size_t)(r0 + i - ts) * pt];
                    w[k] = (int)d.rows[r0 + i].w;
                }
                const int s = g % NS;
                pc_wait_ge(&s_freed, g - NS + 1);
                PcDnSlot& sl = ring[s];
#pragma unroll
                for (int k = 0; k < PC_G; ++k) {
                    if (k >= n) break;
                    sl.T[k][lane] = sS2[w[k]] * u[k];
                    if (lane == 0) sl.S[k] = sS[w[k]];
                }
                pc_publish(&s_staged[s], g + 1);
            }
        } else {
            const int parent = d.rows[r0].parent;
            // the head: fma(S, A(parent), S2 * A_up), or A_up itself at a tree root -- loaded before any store
            double y = parent >= 0 ? Al[(size_t)(parent - ts) * pt] : Al[(size_t)(r0 - ts) * pt];
            for (int g = 0; g < ngroups; ++g) {
                const int s = g % NS;
                pc_wait_ge(&s_staged[s], g + 1);
                const PcDnSlot& sl = ring[s];
                const int i0 = g * PC_G;
                const int n = len - i0 < PC_G ? len - i0 : PC_G;
                double T[PC_G], S[PC_G];
#pragma unroll
                for (int k = 0; k < PC_G; ++k) {
                    T[k] = sl.T[k][lane];
                    S[k] = sl.S[k];
                }
                pc_publish_ordered(&s_freed, g + 1);
#pragma unroll
                for (int k = 0; k < PC_G; ++k) {
                    if (k >= n) break;
                    if (!(i0 + k == 0 && parent < 0)) y = fma(S[k], y, T[k]);  // a tree root keeps A_up
                    if (act) A[(size_t)(r0 + i0 + k - ts) * pt] = y;
                }
            }
        }
    }
}

// Pieces (sm_pms_host.h PmsCut): one wave per repair item (cut path, chunk) re-walks the guessed
// pieces in dependency order from their exact neighbours -- up: from the piece above the exact bottom
// piece to the head; down: from the piece below the exact head piece to the bottom.
// gated (the parallel repair ran first): only items whose flag word is set -- a piece's repair rewrote
// the boundary row its neighbour had started from -- run, and clear the word
__global__ void __launch_bounds__(256) k_pms_repair(PmsDev d, int phase, int up, int lo, int hi, int gated) {
    __shared__ double sS[PMS_NW], sS2[PMS_NW];
    load_luts(d, sS, sS2);
    const int it = lo + (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    if (it >= hi) return;
    if (gated) {
        if (uni(d.rep_flag[it]) == 0) return;
        if ((threadIdx.x & 63) == 0) d.rep_flag[it] = 0;
    }
    const PmsRep rp = d.reps[it];
    const PmsCut c = d.cuts[uni(rp.cut)];
    const int t = uni(c.tree), Pn = d.piece, np = uni(c.npieces), row = uni(c.row), len = uni(c.len);
    int P, base;
    phase_labels(d, phase, t, P, base);
    const int j = uni(rp.chunk) * 64 + (int)(threadIdx.x & 63);
    if (uni(rp.chunk) * 64 >= P) return;
    const bool act = j < P;
    const int ts = d.tree_start[t], pt = d.tree_pt[t];
    const double* A = d.A + d.tree_abase[t] + j;
    if (up) {
        for (int i = np - 2; i >= 0; --i) {
            const int top = row + i * Pn, bot = top + Pn - 1;
            const double x0 = act ? A[(size_t)(bot + 1 - ts) * pt] : 0.0;  // the exact head row of the piece below
            up_walk<true, false>(d, sS, phase, t, top, bot, rp.chunk, x0);
        }
    } else {
        const double* ub = d.Abak + d.cut_bak[uni(rp.cut)];  // A_up of rows [row + Pn, row + len)
        for (int i = 1; i < np; ++i) {
            const int top = row + i * Pn, bot = i + 1 < np ? top + Pn - 1 : row + len - 1;
            const double y0 = act ? A[(size_t)(top - 1 - ts) * pt] : 0.0;  // the exact bottom row of the piece above
            down_walk<true>(d, sS, sS2, phase, t, top, bot, rp.chunk, y0, ub + (size_t)(top - row - Pn) * pt);
        }
    }
}

// Parallel repair: one wave per (repair item, piece): every guessed piece re-walks at once from its
// neighbour's boundary row as the speculative walk left it -- up: the head row of the piece below, down:
// the bottom row of the piece above.  That row is usually exact already: the neighbour's own guess error
// has decayed within its >= 512 rows.  A piece whose repair reaches its far end without agreeing has
// rewritten that boundary row, so its neighbour may have started from a stale value: the item's flag word
// gets the piece's bit, and the gated sequential repair (k_pms_repair) redoes that item in order.
__global__ void __launch_bounds__(256) k_pms_repair_par(PmsDev d, int phase, int up, int lo, int hi, int maxp) {
    __shared__ double sS[PMS_NW], sS2[PMS_NW];
    load_luts(d, sS, sS2);
    const int g = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const int it = lo + g / maxp, i = g % maxp;
    if (it >= hi) return;
    const PmsRep rp = d.reps[it];
    const PmsCut c = d.cuts[uni(rp.cut)];
    const int t = uni(c.tree), Pn = d.piece, np = uni(c.npieces), row = uni(c.row), len = uni(c.len);
    int P, base;
    phase_labels(d, phase, t, P, base);
    const int j = uni(rp.chunk) * 64 + (int)(threadIdx.x & 63);
    if (uni(rp.chunk) * 64 >= P) return;
    const bool act = j < P;
    const int ts = d.tree_start[t], pt = d.tree_pt[t];
    const double* A = d.A + d.tree_abase[t] + j;
    bool ok;
    if (up) {
        if (i > np - 2) return;  // the bottom piece (np - 1) starts from the path's leaf: exact
        const int top = row + i * Pn, bot = top + Pn - 1;
        const double x0 = act ? A[(size_t)(bot + 1 - ts) * pt] : 0.0;
        ok = up_walk<true, false>(d, sS, phase, t, top, bot, rp.chunk, x0);
    } else {
        if (i < 1 || i >= np) return;  // the head piece (0) starts from the path's exact parent
        const double* ub = d.Abak + d.cut_bak[uni(rp.cut)];
        const int top = row + i * Pn, bot = i + 1 < np ? top + Pn - 1 : row + len - 1;
        const double y0 = act ? A[(size_t)(top - 1 - ts) * pt] : 0.0;
        ok = down_walk<true>(d, sS, sS2, phase, t, top, bot, rp.chunk, y0, ub + (size_t)(top - row - Pn) * pt);
    }
    // the far boundary changed: the neighbour that read it (up: piece i - 1, down: i + 1) may be stale
    const bool neighbour = up ? i > 0 : i + 1 < np;
    if (!ok && neighbour && (threadIdx.x & 63) == 0) atomicOr(&d.rep_flag[it], 1u << (i & 31));
}

// A_up rows of the non-head pieces of cuts [c_lo, c_hi) -> Abak (blockIdx.y = cut - c_lo)
__global__ void k_pms_cut_backup(PmsDev d, int c_lo) {
    const int ci = c_lo + (int)blockIdx.y;
    const PmsCut c = d.cuts[ci];
    const int t = c.tree, pt = d.tree_pt[t];
    const size_t n = (size_t)(c.len - d.piece) * pt;
    const double* src = d.A + d.tree_abase[t] + (size_t)(c.row + d.piece - d.tree_start[t]) * pt;
    double* dst = d.Abak + d.cut_bak[ci];
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) dst[i] = src[i];
}

// Rows with few proposals (P <= 16) are updated one per lane (update_row); a row with more is updated
// by the whole wave, lanes over its proposals (coalesced A reads), then a wave reduction to the
// minimum value and, among equal values, the smallest index -- the same winner as the serial strict-<
// scan from index 0 (:173-185) -- then the strict-< test against the pixel's current minimum.
__global__ void __launch_bounds__(256) k_pms_update(PmsDev d, int phase, int row_lo, int row_hi) {
    const int lane = (int)(threadIdx.x & 63);
    const int base_row = row_lo + (int)((blockIdx.x * blockDim.x + threadIdx.x) & ~63u);
    const int row = base_row + lane;
    const bool valid = row < row_hi;
    int t = 0, P = 0, lb = 0;
    if (valid) {
        t = d.rtree[row];
        phase_labels(d, phase, t, P, lb);
    }
    const bool wide = valid && P > 16;
    if (d.evals) {  // node-label evaluations: one atomic per block (same-address atomics serialise in L2)
        __shared__ int s_sum;
        if (threadIdx.x == 0) s_sum = 0;
        __syncthreads();
        int sum = valid ? P : 0;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) sum += __shfl_xor(sum, o);
        if (lane == 0 && sum) atomicAdd(&s_sum, sum);
        __syncthreads();
        if (threadIdx.x == 0 && s_sum) atomicAdd(d.evals, (unsigned long long)s_sum);
    }
    if (valid && !wide) update_row(d, phase, row, t);
    unsigned long long m = __ballot(wide);
    while (m) {
        const int b = __ffsll((long long)m) - 1;
        m &= m - 1;
        const int r = base_row + b;
        const int tr = __shfl(t, b), Pr = __shfl(P, b), br = __shfl(lb, b);
        const double* a = d.A + d.tree_abase[tr] + (size_t)(r - d.tree_start[tr]) * d.tree_pt[tr];
        double mv = 0.0;
        int mi = INT_MAX;
        for (int j = lane; j < Pr; j += 64) {  // per lane: the first minimum of its indices
            const double v = a[j];
            if (mi == INT_MAX || v < mv) {
                mv = v;
                mi = j;
            }
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {  // (value, index) minimum over the wave
            const double ov = __shfl_xor(mv, o);
            const int oi = __shfl_xor(mi, o);
            if (oi != INT_MAX && (mi == INT_MAX || ov < mv || (ov == mv && oi < mi))) {
                mv = ov;
                mi = oi;
            }
        }
        if (lane == 0) {
            const int pix = d.rows[r].pix;
            if (mv < d.minc[pix]) {
                const float4 L = d.lab[br + mi];
                d.minc[pix] = mv;
                d.abc[3 * (size_t)pix] = L.x;
                d.abc[3 * (size_t)pix + 1] = L.y;
                d.abc[3 * (size_t)pix + 2] = L.z;
            }
        }
    }
}

__global__ void k_pms_ref_setup(PmsDev d, int t_lo) {
    const int t = t_lo + (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (t >= d.K) return;
    const int deg = tree_deg(d, t);
    d.cnt[t] = deg + ref_levels(d, t, d.oguess[t] + deg, true);
}

// Per tree: a propagation label taken from a lower neighbour differs from that pixel's label after the
// neighbour ran (the serial order would have read the new one).  Then the scan: the first tree whose
// guessed offset or inputs are wrong; every tree before it is exact.
__global__ void k_pms_flags(PmsDev d, int t_lo) {
    const int t = t_lo + (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (t >= d.K) return;
    int f = 0;
    const int deg = tree_deg(d, t), base = d.tree_lab[t];
    for (int j = 0; j < deg && !f; ++j) {
        if (d.nb[d.nb_start[t] + j] >= t) continue;
        const int q = d.labq[base + j];
        const float4 L = d.lab[base + j];
        f = __float_as_uint(L.x) != __float_as_uint(d.abc[3 * (size_t)q]) ||
            __float_as_uint(L.y) != __float_as_uint(d.abc[3 * (size_t)q + 1]) ||
            __float_as_uint(L.z) != __float_as_uint(d.abc[3 * (size_t)q + 2]);
    }
    d.flag[t] = f;
}

// One workgroup, 1024 trees per step: the exact offsets are the running offset plus an exclusive scan of
// the counts; the first tree whose guess differs or whose flag is set (a block minimum) ends the scan.
__global__ void __launch_bounds__(1024) k_pms_scan(PmsDev d, int t_lo) {
    __shared__ long long s_w[16];
    __shared__ int s_first;
    const int tid = (int)threadIdx.x, lane = tid & 63, wv = tid >> 6;
    long long o = d.off[0];
    for (int t0 = t_lo; t0 < d.K; t0 += 1024) {
        const int t = t0 + tid;
        const long long c = t < d.K ? (long long)d.cnt[t] : 0;
        long long incl = c;  // wave inclusive scan, then across the 16 waves
#pragma unroll
        for (int k = 1; k < 64; k <<= 1) {
            const long long v = __shfl_up(incl, k);
            if (lane >= k) incl += v;
        }
        if (lane == 63) s_w[wv] = incl;
        if (tid == 0) s_first = INT_MAX;
        __syncthreads();
        long long pre = 0;
        for (int k = 0; k < wv; ++k) pre += s_w[k];
        const long long ex = o + pre + incl - c;  // the exact offset of tree t
        int why = 0;
        if (t < d.K) why = d.oguess[t] != ex ? 1 : d.flag[t] ? 2 : 0;
        if (why) atomicMin(&s_first, t);
        __syncthreads();
        const int first = s_first;
        if (first != INT_MAX) {
            if (t == first) {
                d.result[0] = t;
                d.result[1] = why;  // 1: wrong offset (every later tree drew from the wrong place); 2: stale inputs only
                *reinterpret_cast<long long*>(d.result + 2) = ex;
            }
            return;
        }
        long long tot = 0;
        for (int k = 0; k < 16; ++k) tot += s_w[k];
        o += tot;
        __syncthreads();
    }
    if (tid == 0) {
        d.result[0] = d.K;
        d.result[1] = 0;
        *reinterpret_cast<long long*>(d.result + 2) = o;
    }
}

__global__ void k_pms_restore(PmsDev d, int row_lo, int row_hi) {
    const int row = row_lo + (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (row >= row_hi) return;
    const size_t p = (size_t)d.rows[row].pix;
    d.minc[p] = d.minc_bak[p];
    d.abc[3 * p] = d.abc_bak[3 * p];
    d.abc[3 * p + 1] = d.abc_bak[3 * p + 1];
    d.abc[3 * p + 2] = d.abc_bak[3 * p + 2];
}

__global__ void k_pms_vol_rows(const float* __restrict__ in, size_t N, int D, int Dv, int clamp, float* __restrict__ out) {
    // 32 x 32 tile transpose through LDS: in [D][N] -> out [N][Dv]
    __shared__ float tile[32][33];
    const size_t p0 = (size_t)blockIdx.x * 32;
    const int d0 = blockIdx.y * 32;
    for (int k = threadIdx.y; k < 32; k += blockDim.y) {
        const int dd = d0 + k;
        const size_t p = p0 + threadIdx.x;
        float v = 0.0f;
        if (dd < D && p < N) {
            v = in[(size_t)dd * N + p];
            if (clamp) v = isnan(v) ? 0.5f : (v < 0.5f ? v : 0.5f);  // std::min(0.5f, v)
        }
        tile[k][threadIdx.x] = v;
    }
    __syncthreads();
    for (int k = threadIdx.y; k < 32; k += blockDim.y) {
        const size_t p = p0 + k;
        const int dd = d0 + threadIdx.x;
        if (p < N && dd < Dv) out[p * Dv + dd] = dd < D ? tile[threadIdx.x][k] : 0.0f;
    }
}

__global__ void k_pms_disp(const float* __restrict__ abc, int W, size_t N, float* __restrict__ disp) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const float xf = (float)(int)(i % (size_t)W), yf = (float)(int)(i / (size_t)W);
    disp[i] = fmaf(xf, abc[3 * i], yf * abc[3 * i + 1]) + abc[3 * i + 2];  // 0x40fdbe-0x40fdd0
}

__global__ void k_pms_backup(PmsDev d, size_t N) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    d.minc_bak[i] = d.minc[i];
    d.abc_bak[3 * i] = d.abc[3 * i];
    d.abc_bak[3 * i + 1] = d.abc[3 * i + 1];
    d.abc_bak[3 * i + 2] = d.abc[3 * i + 2];
}

// Per tree (one wave): the distinct propagation labels of the call (lab holds every tree's exact
// sampled labels once the call is done, in both device modes) and the refinement labels (nref), times
// the tree's size -- the node-label evaluations the call needed (acc[0]; repeats of a label cannot win,
// k_pms_prop_dedupe) and the reference's count, every sampled label (acc[1]).
__global__ void __launch_bounds__(256) k_pms_count(PmsDev d, unsigned long long* acc) {
    const int t = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    if (t >= d.K) return;
    const int lane = (int)(threadIdx.x & 63);
    const int deg = tree_deg(d, t), base = d.tree_lab[t];
    int n = 0;
    // a speculative call leaves every tree's distinct count in nprop (k_pms_prop_dedupe ran on the exact
    // labels of every tree: the validated pass or the tree's serial re-run)
    for (int j0 = d.nprop ? deg : 0; j0 < deg; j0 += 64) {
        const int j = j0 + lane;
        bool keep = false;
        if (j < deg) {
            const float4 L = d.lab[base + j];
            keep = true;
            for (int i = 0; i < j && keep; ++i) {
                const float4 M = d.lab[base + i];
                keep = !(__float_as_uint(M.x) == __float_as_uint(L.x) && __float_as_uint(M.y) == __float_as_uint(L.y) &&
                         __float_as_uint(M.z) == __float_as_uint(L.z));
            }
        }
        n += __popcll(__ballot(keep));
    }
    if (d.nprop) n = d.nprop[t];
    if (lane == 0) {
        const unsigned long long sz = (unsigned long long)(d.tree_start[t + 1] - d.tree_start[t]);
        const unsigned long long nr = (unsigned long long)d.nref[t];
        atomicAdd(acc, sz * ((unsigned long long)n + nr));
        atomicAdd(acc + 1, sz * ((unsigned long long)deg + nr));
    }
}

inline unsigned blocks(size_t n, unsigned b) { return (unsigned)((n + b - 1) / b); }

}  // namespace

hipError_t launch_pms_serial(hipStream_t st, const PmsDev& d, int t0, int t1) {
    if (t1 <= t0) return hipSuccess;
    // 768 threads: 1024 spilled VGPRs; 512 / 768 / 1024 within noise once it did not (round 4)
    hipLaunchKernelGGL(k_pms_serial<768>, dim3(1), dim3(768), 0, st, d, t0, t1);
    return hipGetLastError();
}


hipError_t launch_pms_prop_tree(hipStream_t st, const PmsDev& d, int t) {
    hipLaunchKernelGGL(k_pms_prop_tree, dim3(1), dim3(256), 0, st, d, t);
    return hipGetLastError();
}

hipError_t launch_pms_ref_one(hipStream_t st, const PmsDev& d, int t) {
    hipLaunchKernelGGL(k_pms_ref_one, dim3(1), dim3(64), 0, st, d, t);
    return hipGetLastError();
}

hipError_t launch_pms_guess(hipStream_t st, const PmsDev& d, int t_lo, long long wn) {
    // wn covers every draw trees [t_lo, K) can consume (the host's bound), so a staged chain never
    // reads past the window; otherwise (too many trees / draws for the LDS) it reads global memory
    const size_t nt = (size_t)(d.K - t_lo);
    constexpr size_t cap = 150 * 1024;  // LDS bytes
    const size_t lds = 4 * ((3 * nt + 1) & ~(size_t)1) + 8 * nt + 4 * (size_t)wn;
    static const hipError_t attr =  // once per process (thread-safe static initialisation)
        hipFuncSetAttribute((const void*)k_pms_guess<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)cap);
    if (attr != hipSuccess) return attr;
    if (lds <= cap)
        hipLaunchKernelGGL(k_pms_guess<true>, dim3(1), dim3(1024), lds, st, d, t_lo, wn);
    else
        hipLaunchKernelGGL(k_pms_guess<false>, dim3(1), dim3(64), 0, st, d, t_lo, 0ll);
    return hipGetLastError();
}

hipError_t launch_pms_prop_setup(hipStream_t st, const PmsDev& d, int t_lo, int total_deg) {
    if (total_deg <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_pms_prop_setup, dim3(blocks((size_t)total_deg, 256)), dim3(256), 0, st, d, t_lo);
    return hipGetLastError();
}

hipError_t launch_pms_prop_dedupe(hipStream_t st, const PmsDev& d, int t_lo, int t_hi) {
    if (t_hi <= t_lo) return hipSuccess;
    hipLaunchKernelGGL(k_pms_prop_dedupe, dim3(blocks((size_t)(t_hi - t_lo) * 64, 256)), dim3(256), 0, st, d, t_lo, t_hi);
    return hipGetLastError();
}

hipError_t launch_pms_layout(hipStream_t st, const PmsDev& d, int phase, int t_lo, int t_hi, int32_t* pt_out,
                             long long* ab_out, int32_t* zero, int nzero) {
    if (t_hi <= t_lo) return hipSuccess;
    hipLaunchKernelGGL(k_pms_layout, dim3(1), dim3(1024), 0, st, d, phase, t_lo, t_hi, pt_out, ab_out, zero, nzero);
    return hipGetLastError();
}

hipError_t launch_pms_plan(hipStream_t st, const PmsDev& d, int phase, int t_lo, int t_hi, int nrounds, int max_paths,
                           int chain_len, bool zeroed) {
    if (t_hi <= t_lo || nrounds <= 0) return hipSuccess;
    if (!zeroed) {  // (k_pms_layout zeroes the counters when it runs first)
        hipError_t e = hipMemsetAsync(d.plan_cnt, 0, sizeof(int32_t) * PMS_NCNT * (size_t)nrounds, st);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_pms_plan, dim3(blocks((size_t)std::max(max_paths, 1), 1024), (unsigned)nrounds), dim3(1024), 0, st, d,
                       phase, t_lo, t_hi, chain_len > 0 ? std::max(chain_len, PMS_CHAIN_LEN) : INT_MAX);
    return hipGetLastError();
}

hipError_t launch_pms_chain(hipStream_t st, const PmsDev& d, int phase, bool up, int r, int items) {
    if (items <= 0) return hipSuccess;
    // SM_PMS_CHAIN_NSU / _NSD: ring slots of the up / down chain (LDS per workgroup, so workgroups per CU)
    const char* eu = sm_knob("SM_PMS_CHAIN_NSU");
    const char* ed = sm_knob("SM_PMS_CHAIN_NSD");
    const int nsu = eu ? std::min(std::max(atoi(eu), 1), PC_NSU_MAX) : PC_NSU;
    const int nsd = ed ? std::min(std::max(atoi(ed), 1), PC_NSD) : PC_NSD;
    const int ns = up ? nsu : nsd;
    const size_t lds = up ? ns * sizeof(PcUpSlot) : ns * sizeof(PcDnSlot);
    static const hipError_t a0 = hipFuncSetAttribute((const void*)k_pms_chain<true>,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)(PC_NSU_MAX * sizeof(PcUpSlot)));
    static const hipError_t a1 = hipFuncSetAttribute((const void*)k_pms_chain<false>,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)(PC_NSD * sizeof(PcDnSlot)));
    if (a0 != hipSuccess) return a0;
    if (a1 != hipSuccess) return a1;
    if (up) hipLaunchKernelGGL(k_pms_chain<true>, dim3((unsigned)items), dim3(64 * (PC_LW + 1)), lds, st, d, phase, r, ns);
    else hipLaunchKernelGGL(k_pms_chain<false>, dim3((unsigned)items), dim3(64 * (PC_LW + 1)), lds, st, d, phase, r, ns);
    return hipGetLastError();
}

hipError_t launch_pms_walk_plan(hipStream_t st, const PmsDev& d, int phase, bool up, int r, int waves) {
    if (waves <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_pms_walk_plan, dim3(blocks((size_t)waves, 4)), dim3(256), 0, st, d, phase, up ? 1 : 0, r);
    return hipGetLastError();
}

hipError_t launch_pms_cost(hipStream_t st, const PmsDev& d, int phase, int row_lo, int row_hi) {
    if (row_hi <= row_lo) return hipSuccess;
    hipLaunchKernelGGL(k_pms_cost, dim3(blocks((size_t)(row_hi - row_lo), 256)), dim3(256), 0, st, d, phase, row_lo, row_hi);
    return hipGetLastError();
}

hipError_t launch_pms_update(hipStream_t st, const PmsDev& d, int phase, int row_lo, int row_hi) {
    if (row_hi <= row_lo) return hipSuccess;
    hipLaunchKernelGGL(k_pms_update, dim3(blocks((size_t)(row_hi - row_lo), 256)), dim3(256), 0, st, d, phase, row_lo, row_hi);
    return hipGetLastError();
}

hipError_t launch_pms_repair(hipStream_t st, const PmsDev& d, int phase, bool up, int lo, int hi, int maxp) {
    if (hi <= lo) return hipSuccess;
    if (maxp > 0)  // parallel over pieces, then the gated sequential pass
        hipLaunchKernelGGL(k_pms_repair_par, dim3(blocks((size_t)(hi - lo) * maxp * 64, 256)), dim3(256), 0, st, d, phase,
                           up ? 1 : 0, lo, hi, maxp);
    hipLaunchKernelGGL(k_pms_repair, dim3(blocks((size_t)(hi - lo) * 64, 256)), dim3(256), 0, st, d, phase, up ? 1 : 0, lo, hi,
                       maxp > 0 ? 1 : 0);
    return hipGetLastError();
}

hipError_t launch_pms_cut_backup(hipStream_t st, const PmsDev& d, int c_lo, int c_hi) {
    if (c_hi <= c_lo) return hipSuccess;
    hipLaunchKernelGGL(k_pms_cut_backup, dim3(64, (unsigned)(c_hi - c_lo)), dim3(256), 0, st, d, c_lo);
    return hipGetLastError();
}

hipError_t launch_pms_ref_setup(hipStream_t st, const PmsDev& d, int t_lo) {
    if (t_lo >= d.K) return hipSuccess;
    hipLaunchKernelGGL(k_pms_ref_setup, dim3(blocks((size_t)(d.K - t_lo), 256)), dim3(256), 0, st, d, t_lo);
    return hipGetLastError();
}

hipError_t launch_pms_validate(hipStream_t st, const PmsDev& d, int t_lo) {
    if (t_lo < d.K) hipLaunchKernelGGL(k_pms_flags, dim3(blocks((size_t)(d.K - t_lo), 256)), dim3(256), 0, st, d, t_lo);
    hipLaunchKernelGGL(k_pms_scan, dim3(1), dim3(1024), 0, st, d, t_lo);
    return hipGetLastError();
}

hipError_t launch_pms_restore(hipStream_t st, const PmsDev& d, int row_lo, int row_hi) {
    if (row_hi <= row_lo) return hipSuccess;
    hipLaunchKernelGGL(k_pms_restore, dim3(blocks((size_t)(row_hi - row_lo), 256)), dim3(256), 0, st, d, row_lo, row_hi);
    return hipGetLastError();
}

hipError_t launch_pms_backup(hipStream_t st, const PmsDev& d, size_t N) {
    hipLaunchKernelGGL(k_pms_backup, dim3(blocks(N, 256)), dim3(256), 0, st, d, N);
    return hipGetLastError();
}

hipError_t launch_pms_count(hipStream_t st, const PmsDev& d, unsigned long long* acc) {
    if (d.K <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_pms_count, dim3(blocks((size_t)d.K * 64, 256)), dim3(256), 0, st, d, acc);
    return hipGetLastError();
}

hipError_t launch_pms_vol_rows(hipStream_t st, const float* in, size_t N, int D, int Dv, int clamp, float* out) {
    hipLaunchKernelGGL(k_pms_vol_rows, dim3(blocks(N, 32), (unsigned)((Dv + 31) / 32)), dim3(32, 8), 0, st, in, N, D, Dv,
                       clamp, out);
    return hipGetLastError();
}

hipError_t launch_pms_disp(hipStream_t st, const float* abc, int W, size_t N, float* disp) {
    hipLaunchKernelGGL(k_pms_disp, dim3(blocks(N, 256)), dim3(256), 0, st, abc, W, N, disp);
    return hipGetLastError();
}
