// sm_kernels.hip -- hand-written CDNA4 (gfx950) kernels of the Stereo3DMST path.
//
// Compiled with -ffp-contract=off: every fused multiply-add below is an explicit
// __builtin_fma, mirroring exactly the ones the shipped reference binary performs
// (DESIGN.md "Shipped arithmetic"); all other float/double ops round individually.
//
// Kernels (v = view: 0 left, 1 right; both views run in one launch via blockIdx.z):
//   k_prep          packed BGR u8 -> bgrx u32 + gray f32 planes             (prep)
//   k_median        3x3 median per channel, replicate border               (Stereo3DMST.cpp:226-228)
//   k_weights       L1-RGB edge weights of the median image                 (:83-94, :242-262)
//   k_cost_volume   AGD cost volume [d][y][x] from LDS-staged row tiles      (PatchMatchStereoGPU.cu:1482-1550)
//   k_bor_*         Boruvka MST in (w,a,b) order: LDS tile phase + global    (segment-graph.h:54-89, c=+inf)
//   (tree-filter walkers: sm_walk.hip)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdint.h>

#include "sm_common.h"
#include "sm_reduce_rule.h"

#define WAVE 64

// ---------------------------------------------------------------------------------------------
// small device helpers
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ float sm_gray(uint32_t bgrx) {
    // 0.114f*B + 0.587f*G + 0.299f*R, left to right, no contraction (PatchMatchStereoGPU.cu:1529)
    const float b = (float)(bgrx & 255u), g = (float)((bgrx >> 8) & 255u), r = (float)((bgrx >> 16) & 255u);
    float t = 0.114f * b;
    t = t + 0.587f * g;
    t = t + 0.299f * r;
    return t;
}

// AGD cost of right pixel x at disparity d: r0=right(x) r1=right(x+1) l0=left(x+d) l1=left(x+d+1)
// (PatchMatchStereoGPU.cu:1518-1543).  color_l1 is an exact integer -> SAD + table.
__device__ __forceinline__ float sm_agd(uint32_t r0, uint32_t l0, float gr0, float gr1, float gl0, float gl1,
                                        const float* __restrict__ atab) {
    const uint32_t l1 = __builtin_amdgcn_sad_u8(r0, l0, 0u);
    const float a = atab[l1];
    float g = gl0 - gr0;
    g = g + (gr1 - gl1);
    const float b = 0.89f * fminf(fabsf(g), 2.0f);
    return a + b;
}

// ---------------------------------------------------------------------------------------------
// prep / median / weights
// ---------------------------------------------------------------------------------------------
struct ImgPair {
    const uint8_t* src[2];  // packed BGR rows (device)
    uint32_t* bgrx[2];      // W*H
    float* gray[2];         // W*H
    uint2* rec[2];          // W*H {bgrx, gray bits}: one 8-byte load per pixel (chain helpers)
    uint32_t* rec4[2];      // W*H bgrx, padded like rec (the up walker recomputes the gray)
};

__global__ void k_prep(ImgPair P, int W, int H, int stride) {
    const int v = blockIdx.z;
    const int y = blockIdx.y;
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= W) return;
    const uint8_t* s = P.src[v] + (size_t)y * stride + 3 * (size_t)x;
    const uint32_t w = (uint32_t)s[0] | ((uint32_t)s[1] << 8) | ((uint32_t)s[2] << 16);
    const size_t p = (size_t)y * W + x;
    const float g = sm_gray(w);
    P.bgrx[v][p] = w;
    P.gray[v][p] = g;
    P.rec[v][p] = make_uint2(w, __float_as_uint(g));
    P.rec4[v][p] = w;
}

__device__ __forceinline__ void cswap(int& a, int& b) {
    const int lo = min(a, b), hi = max(a, b);
    a = lo;
    b = hi;
}

__device__ __forceinline__ int median9(int p0, int p1, int p2, int p3, int p4, int p5, int p6, int p7, int p8) {
    // 19-exchange median network (same network as OpenCV's medianBlur_SortNet m=3).
    cswap(p1, p2); cswap(p4, p5); cswap(p7, p8); cswap(p0, p1);
    cswap(p3, p4); cswap(p6, p7); cswap(p1, p2); cswap(p4, p5);
    cswap(p7, p8); cswap(p0, p3); cswap(p5, p8); cswap(p4, p7);
    cswap(p3, p6); cswap(p1, p4); cswap(p2, p5); cswap(p4, p7);
    cswap(p4, p2); cswap(p6, p4); cswap(p4, p2);
    return p4;
}

struct MedPair {
    const uint32_t* bgrx[2];
    uint32_t* med[2];
};

__global__ void k_median(MedPair P, int W, int H) {
    const int v = blockIdx.z;
    const int y = blockIdx.y;
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= W) return;
    const uint32_t* img = P.bgrx[v];
    const int ys[3] = {y > 0 ? y - 1 : 0, y, y < H - 1 ? y + 1 : H - 1};
    const int xs[3] = {x > 0 ? x - 1 : 0, x, x < W - 1 ? x + 1 : W - 1};
    uint32_t q[9];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) q[3 * i + j] = img[(size_t)ys[i] * W + xs[j]];
    uint32_t out = 0;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const int sh = 8 * c;
        const int m = median9((q[0] >> sh) & 255, (q[1] >> sh) & 255, (q[2] >> sh) & 255, (q[3] >> sh) & 255,
                              (q[4] >> sh) & 255, (q[5] >> sh) & 255, (q[6] >> sh) & 255, (q[7] >> sh) & 255,
                              (q[8] >> sh) & 255);
        out |= (uint32_t)m << sh;
    }
    P.med[v][(size_t)y * W + x] = out;
}

struct WeightPair {
    const uint32_t* med[2];
    uint16_t* wR[2];
    uint16_t* wD[2];
};

__global__ void k_weights(WeightPair P, int W, int H) {
    const int v = blockIdx.z;
    const int y = blockIdx.y;
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= W) return;
    const size_t p = (size_t)y * W + x;
    const uint32_t a = P.med[v][p];
    P.wR[v][p] = x < W - 1 ? (uint16_t)__builtin_amdgcn_sad_u8(a, P.med[v][p + 1], 0u) : (uint16_t)SM_WEIGHT_NONE;
    P.wD[v][p] = y < H - 1 ? (uint16_t)__builtin_amdgcn_sad_u8(a, P.med[v][p + W], 0u) : (uint16_t)SM_WEIGHT_NONE;
}

// ---------------------------------------------------------------------------------------------
// K1: AGD cost volume, [d][y][x], both volumes (the sm_cost_volume entry / MC-CNN-shaped path)
// block = 256 threads = one row segment of 256 pixels; grid = (ceil(W/256), H, ceil(D/DC)).
// LDS holds the right row segment [x0-DC-d0', x0+256] and the left row segment
// [x0+dc, x0+256+dc+DC] so every (x, d) pair is served from LDS; stores are coalesced rows.
// ---------------------------------------------------------------------------------------------
#define CV_TX 256
#define CV_DC 64

__global__ __launch_bounds__(CV_TX) void k_cost_volume(const uint32_t* __restrict__ Lb, const float* __restrict__ Lg,
                                                       const uint32_t* __restrict__ Rb, const float* __restrict__ Rg,
                                                       const float* __restrict__ atab_g, int W, int H, int d0, int D,
                                                       float* __restrict__ lvol, float* __restrict__ rvol) {
    __shared__ float atab[SM_MAX_W + 1];
    __shared__ uint32_t sRb[CV_TX + 2 * CV_DC + 2];
    __shared__ float sRg[CV_TX + 2 * CV_DC + 2];
    __shared__ uint32_t sLb[CV_TX + 2 * CV_DC + 2];
    __shared__ float sLg[CV_TX + 2 * CV_DC + 2];
    for (int i = threadIdx.x; i <= SM_MAX_W; i += CV_TX) atab[i] = atab_g[i];
    const int x0 = blockIdx.x * CV_TX;
    const int y = blockIdx.y;
    const int dc = d0 + blockIdx.z * CV_DC;               // first global disparity of this block
    const int nd = min(CV_DC, d0 + D - dc);
    const size_t row = (size_t)y * W;
    // right segment for the left volume: xr in [x0 - (dc+nd-1), x0 + 256]   (+1 for the gradient)
    const int rbeg = x0 - (dc + nd - 1);
    const int rlen = CV_TX + nd + 1;
    for (int i = threadIdx.x; i < rlen; i += CV_TX) {
        const int xr = rbeg + i;
        const bool ok = xr >= 0 && xr < W;
        sRb[i] = ok ? Rb[row + xr] : 0u;
        sRg[i] = ok ? Rg[row + xr] : 0.f;
    }
    // left segment for the right volume: xl in [x0 + dc, x0 + 256 + dc + nd]
    const int lbeg = x0 + dc;
    const int llen = CV_TX + nd + 1;
    for (int i = threadIdx.x; i < llen; i += CV_TX) {
        const int xl = lbeg + i;
        const bool ok = xl >= 0 && xl < W;
        sLb[i] = ok ? Lb[row + xl] : 0u;
        sLg[i] = ok ? Lg[row + xl] : 0.f;
    }
    __syncthreads();
    const int x = x0 + threadIdx.x;
    if (x >= W) return;
    // own pixels of both images (x is a right pixel for rvol and a left pixel for lvol)
    const uint32_t Rx = Rb[row + x];
    const float gRx = Rg[row + x], gRx1 = x + 1 < W ? Rg[row + x + 1] : 0.f;
    const uint32_t Lx = Lb[row + x];
    const float gLx = Lg[row + x], gLx1 = x + 1 < W ? Lg[row + x + 1] : 0.f;
    const size_t N = (size_t)W * H;
    for (int k = 0; k < nd; ++k) {
        const int d = dc + k;
        const size_t o = (size_t)(d - d0) * N + row + x;
        // right reference: right(x) vs left(x+d)
        float cr = 3.0f;
        if (x + d + 1 < W) {
            const int li = threadIdx.x + k;  // (x+d) - lbeg
            cr = sm_agd(Rx, sLb[li], gRx, gRx1, sLg[li], sLg[li + 1], atab);
        }
        rvol[o] = cr;
        // left pixel x: cost(x - d, d); invalid (x<d) and the column W-1 the reference never writes -> 3.0
        float cl = 3.0f;
        if (x - d >= 0 && x + 1 < W) {
            const int ri = threadIdx.x + (nd - 1 - k);  // (x-d) - rbeg
            cl = sm_agd(sRb[ri], Lx, sRg[ri], sRg[ri + 1], gLx, gLx1, atab);
        }
        lvol[o] = cl;
    }
}

// ---------------------------------------------------------------------------------------------
// Boruvka MST (MST mode of segment_graph: every edge whose endpoints are in different trees is
// taken in (w,a,b) order -> the unique MST under that total order).  A component's minimum
// incident edge (by the 64-bit key) is always an MST edge (cut property), so:
//   k_bor_local : per 32x32 tile, in LDS, hook components through their minimum edge while that
//                 edge is inside the tile; a component whose minimum edge leaves the tile freezes.
//   k_bor_min / k_bor_hook / k_bor_root / k_bor_relabel : global rounds on the remaining labels.
// Mask output: mR[p]=1 <=> edge (p,p+1) in MST, mD[p]=1 <=> edge (p,p+W) in MST.
// ---------------------------------------------------------------------------------------------
#define BT 64                 // tile side
#define BTN (BT * BT)         // 4096 pixels per tile
#define BTHREADS 1024

struct MstView {
    const uint16_t* wR;
    const uint16_t* wD;
    uint32_t* comp;           // component label (global pixel index of the representative)
    unsigned long long* best; // per representative: min incident key
    uint32_t* root;           // per representative: final root after hooking
    uint8_t* mR;
    uint8_t* mD;
    int* flags;               // flags[r] = 1 if global round r hooked anything
    uint32_t* ccount;         // contracted rounds: [0] K, and root[] = the representatives' compact ids
                              // (k_bor_local assigns them: k_cid folded in, round 5); null otherwise
    uint32_t* clab;           // contracted rounds: compact id -> label (k_bor_local starts it at the id)
    size_t bstride;           // contracted rounds: the second minima array is best + bstride
};
struct MstPair {
    MstView v[2];
};

__device__ __forceinline__ uint64_t key_of(const uint16_t* wR, const uint16_t* wD, int W, int p, int k) {
    // k: 0 right, 1 down, 2 left, 3 up (caller guarantees existence)
    switch (k) {
        case 0: return sm_edge_key(wR[p], (uint32_t)p, 0u);
        case 1: return sm_edge_key(wD[p], (uint32_t)p, 1u);
        case 2: return sm_edge_key(wR[p - 1], (uint32_t)(p - 1), 0u);
        default: return sm_edge_key(wD[p - W], (uint32_t)(p - W), 1u);
    }
}

// Tile keys: inside one tile every candidate edge (a, a+1 or a+W) has its lower endpoint a in the
// tile, its left column or the row above, so (w, a, vertical) order is the order of the 32-bit
//   w << 14 | ((ly_a + 1) * 66 + (lx_a + 1)) << 1 | vertical
// (a = y*W + x is lexicographic in (y, x), and w <= SM_MAX_W < 2^18).  Each thread keeps its 4
// pixels' 4 edge keys in registers across the iterations, and the LDS minima are 32-bit.
#define TK_NONE 0xFFFFFFFFu
__device__ __forceinline__ uint32_t tile_key(uint32_t w, int lxa, int lya, uint32_t vert) {
    return (w << 14) | ((uint32_t)((lya + 1) * 66 + (lxa + 1)) << 1) | vert;
}

__global__ __launch_bounds__(BTHREADS) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_bor_local(MstPair P, int W, int H, int max_iter) {
    const MstView V = P.v[blockIdx.z];
    __shared__ uint32_t best[BTN];
    __shared__ uint16_t comp[BTN];
    __shared__ uint16_t hk[BTN];
    __shared__ int flag;
    const int tx0 = blockIdx.x * BT, ty0 = blockIdx.y * BT;
    const int tw = min(BT, W - tx0), th = min(BT, H - ty0);
    const int n = tw * th;
    for (int i = threadIdx.x; i < BTN; i += BTHREADS) comp[i] = (uint16_t)i;
    // the tile's mask bytes start at 0 here (round 5: no separate zero-fill): only this block writes
    // them before the global rounds, because it hooks intra-tile edges only (a, b both in the tile)
    for (int i = threadIdx.x; i < n; i += BTHREADS) {
        const size_t p = (size_t)(ty0 + i / tw) * W + tx0 + i % tw;
        V.mR[p] = 0;
        V.mD[p] = 0;
    }
    __syncthreads();
    constexpr int PPT = BTN / BTHREADS;  // thread t, slot j: tile pixel (lx, ly) = ((t + 1024 j) % 64, (t + 1024 j) / 64)
    uint32_t ek[PPT][4];
#pragma unroll
    for (int j = 0; j < PPT; ++j) {
        const int t = threadIdx.x + j * BTHREADS;
        const int lx = t & (BT - 1), ly = t / BT;
        const int x = tx0 + lx, y = ty0 + ly;
        const bool ok = lx < tw && ly < th;
        const int p = y * W + x;
        ek[j][0] = ok && x + 1 < W ? tile_key(V.wR[p], lx, ly, 0u) : TK_NONE;
        ek[j][1] = ok && y + 1 < H ? tile_key(V.wD[p], lx, ly, 1u) : TK_NONE;
        ek[j][2] = ok && x > 0 ? tile_key(V.wR[p - 1], lx - 1, ly, 0u) : TK_NONE;
        ek[j][3] = ok && y > 0 ? tile_key(V.wD[p - W], lx, ly - 1, 1u) : TK_NONE;
    }
    __syncthreads();
    for (int iter = 0; iter < max_iter; ++iter) {
        for (int i = threadIdx.x; i < BTN; i += BTHREADS) best[i] = TK_NONE;
        if (threadIdx.x == 0) flag = 0;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < PPT; ++j) {
            const int t = threadIdx.x + j * BTHREADS;
            const int lx = t & (BT - 1), ly = t / BT;
            if (lx >= tw || ly >= th) continue;
            const int i = ly * tw + lx;
            const int c = comp[i];
            uint32_t mk = TK_NONE;
            if (ek[j][0] != TK_NONE && (lx + 1 >= tw || comp[i + 1] != c)) mk = min(mk, ek[j][0]);
            if (ek[j][1] != TK_NONE && (ly + 1 >= th || comp[i + tw] != c)) mk = min(mk, ek[j][1]);
            if (ek[j][2] != TK_NONE && (lx == 0 || comp[i - 1] != c)) mk = min(mk, ek[j][2]);
            if (ek[j][3] != TK_NONE && (ly == 0 || comp[i - tw] != c)) mk = min(mk, ek[j][3]);
            if (mk != TK_NONE) atomicMin(&best[c], mk);
        }
        __syncthreads();
        for (int c = threadIdx.x; c < n; c += BTHREADS) {
            hk[c] = (uint16_t)c;
            if (comp[c] != c) continue;
            const uint32_t k = best[c];
            if (k == TK_NONE) continue;
            const uint32_t vert = k & 1u, idx = (k >> 1) & 0x1FFFu;
            const int lya = (int)(idx / 66u) - 1, lxa = (int)(idx % 66u) - 1;
            const int lyb = lya + (int)vert, lxb = lxa + 1 - (int)vert;
            const bool ain = lxa >= 0 && lxa < tw && lya >= 0 && lya < th;
            const bool bin = lxb >= 0 && lxb < tw && lyb >= 0 && lyb < th;
            if (!ain || !bin) continue;  // minimum edge leaves the tile: frozen this phase
            const int la = lya * tw + lxa, lb = lyb * tw + lxb;
            const int ca = comp[la];
            const int c2 = (ca == c) ? comp[lb] : ca;
            if (best[c2] == k && c < c2) continue;  // mutual choice: the smaller label stays root
            hk[c] = (uint16_t)c2;
            const uint32_t a = (uint32_t)((ty0 + lya) * W + tx0 + lxa);
            if (vert) V.mD[a] = 1; else V.mR[a] = 1;
            flag = 1;
        }
        __syncthreads();
        if (flag == 0) break;
        // pointer jumping to the roots of the hook forest
        for (;;) {
            __syncthreads();
            int again = 0;
            for (int c = threadIdx.x; c < n; c += BTHREADS) {
                const int h = hk[c];
                const int hh = hk[h];
                if (hh != h) { hk[c] = (uint16_t)hh; again = 1; }
            }
            again = __syncthreads_or(again);
            if (!again) break;
        }
        for (int i = threadIdx.x; i < n; i += BTHREADS) comp[i] = hk[comp[i]];
        __syncthreads();
    }
    constexpr int IPT = BTN / BTHREADS;  // (i = threadIdx.x + BTHREADS j below)
    uint32_t reps = 0;
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        const int i = threadIdx.x + j * BTHREADS;
        if (i >= n) break;
        const int lx = i % tw, ly = i / tw;
        const int r = comp[i];
        const uint32_t gr = (uint32_t)((ty0 + r / tw) * W + tx0 + r % tw);
        V.comp[(size_t)(ty0 + ly) * W + tx0 + lx] = gr;
        if (r == i) reps |= 1u << j;
    }
    if (V.ccount == nullptr) return;  // (uniform: the pixel-round engine)
    // compact ids of the tile's components: a block scan of the representative counts, one atomic per
    // tile (any id order is fine: ids only name components; the mutual-choice tie-break on ids picks
    // which of two components stays root, never which edge joins the MST)
    __shared__ uint32_t s_w[BTHREADS / 64], s_base;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t c = (uint32_t)__builtin_popcount(reps);
    uint32_t x = c;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    if (lane == 63) s_w[wv] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int k = 0; k < BTHREADS / 64; ++k) {
            const uint32_t u = s_w[k];
            s_w[k] = t;
            t += u;
        }
        s_base = atomicAdd(V.ccount, t);
    }
    __syncthreads();
    uint32_t id = s_base + s_w[wv] + x - c;
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        if (!((reps >> j) & 1u)) continue;
        const int i = threadIdx.x + j * BTHREADS;
        V.root[(size_t)(ty0 + i / tw) * W + tx0 + i % tw] = id;
        // the contracted rounds' initial state of component id (round 5: k_cinit folded in)
        V.clab[id] = id;
        V.best[id] = SM_KEY_NONE;
        V.best[V.bstride + id] = SM_KEY_NONE;
        ++id;
    }
}

__device__ __forceinline__ bool round_done(const MstView& V, int r) { return r > 0 && V.flags[r - 1] == 0; }

__global__ void k_bor_min(MstPair P, int W, int H, int rnd) {
    const MstView V = P.v[blockIdx.z];
    if (round_done(V, rnd)) return;
    const int y = blockIdx.y;
    const int x0 = blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = x0 < W;
    const int x = live ? x0 : W - 1;
    const int p = y * W + x;
    const uint32_t c = V.comp[p];
    unsigned long long mk = SM_KEY_NONE;
    if (x + 1 < W && V.comp[p + 1] != c) mk = min(mk, (unsigned long long)key_of(V.wR, V.wD, W, p, 0));
    if (y + 1 < H && V.comp[p + W] != c) mk = min(mk, (unsigned long long)key_of(V.wR, V.wD, W, p, 1));
    if (x > 0 && V.comp[p - 1] != c) mk = min(mk, (unsigned long long)key_of(V.wR, V.wD, W, p, 2));
    if (y > 0 && V.comp[p - W] != c) mk = min(mk, (unsigned long long)key_of(V.wR, V.wD, W, p, 3));
    // wave-aggregated atomics: one atomicMin per distinct component among the lanes
    bool active = live && mk != SM_KEY_NONE;
    const int lane = threadIdx.x & 63;
    while (true) {
        const unsigned long long act = __ballot(active);
        if (!act) break;
        const int leader = __builtin_ctzll(act);
        const uint32_t c0 = __shfl(c, leader);
        const bool mine = active && c == c0;
        unsigned long long v = mine ? mk : SM_KEY_NONE;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const unsigned long long o = __shfl_xor(v, off);
            v = o < v ? o : v;
        }
        if (lane == leader) atomicMin(&V.best[c0], v);
        active = active && !mine;
    }
}

__global__ void k_bor_hook(MstPair P, int W, int H, int rnd) {
    const MstView V = P.v[blockIdx.z];
    if (round_done(V, rnd)) return;
    const int y = blockIdx.y;
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= W) return;
    const uint32_t c = (uint32_t)(y * W + x);
    if (V.comp[c] != c) return;
    uint32_t h = c;
    const unsigned long long k = V.best[c];
    if (k != SM_KEY_NONE) {
        const uint32_t a = (uint32_t)(k >> 1) & 0xFFFFFFFFu;
        const uint32_t vert = (uint32_t)(k & 1ull);
        const uint32_t b = a + (vert ? (uint32_t)W : 1u);
        const uint32_t ca = V.comp[a];
        const uint32_t c2 = (ca == c) ? V.comp[b] : ca;
        if (!(V.best[c2] == k && c < c2)) {
            h = c2;
            if (vert) V.mD[a] = 1; else V.mR[a] = 1;
            V.flags[rnd] = 1;
        }
    }
    V.root[c] = h;
}

__global__ void k_bor_root(MstPair P, int W, int H, int rnd) {
    // chase hook pointers to the root of each hook tree (hooks only point between old roots)
    const MstView V = P.v[blockIdx.z];
    if (round_done(V, rnd) || V.flags[rnd] == 0) return;
    const int y = blockIdx.y;
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= W) return;
    const uint32_t c = (uint32_t)(y * W + x);
    if (V.comp[c] != c) return;
    uint32_t r = V.root[c];
    for (int it = 0; it < (1 << 26); ++it) {
        const uint32_t rr = V.root[r];
        if (rr == r) break;
        r = rr;
    }
    V.best[c] = SM_KEY_NONE;  // reset for the next round
    V.root[c] = r;            // in-place shortcut: concurrent chasers still reach the same root
}

__global__ void k_bor_relabel(MstPair P, int W, int H, int rnd) {
    const MstView V = P.v[blockIdx.z];
    if (round_done(V, rnd) || V.flags[rnd] == 0) return;
    const int y = blockIdx.y;
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= W) return;
    const int p = y * W + x;
    V.comp[p] = V.root[V.comp[p]];
}

// ---------------------------------------------------------------------------------------------
// Contracted Boruvka.  After k_bor_local most pixels share a tile component; the remaining rounds
// run on the component graph: compact component ids (k_bor_local), the list of inter-component pixel
// edges (k_cedges, same 64-bit keys), then per round min over edges (k_cmin), hook (k_chook),
// root chase (k_croot) and relabel (k_crelabel) over K components / E' edges instead of N pixels.
// The keys and the mutual-choice rule are those of the pixel rounds, so the MST is identical.
// ---------------------------------------------------------------------------------------------
struct CEdge {
    unsigned long long key;
    uint32_t u, v;  // compact ids of the endpoint components after the tile phase
};

struct CView {
    const uint16_t* wR;
    const uint16_t* wD;
    const uint32_t* comp;  // pixel -> tile-phase representative pixel
    uint32_t* cid;         // representative pixel -> compact id (only at representatives)
    uint32_t* counts;      // [0] K components, [1] / [2] live edges in list 0 / 1
    CEdge* edges;          // two lists of emax edges
    size_t emax;
    uint32_t* lab;         // compact id -> current root id
    uint32_t* hook;        // root id -> hooked root
    unsigned long long* best;  // two arrays: round r uses best + (r & 1) * bstride
    size_t bstride;
    uint8_t* mR;
    uint8_t* mD;
    int* flags;
};
struct CPair {
    CView v[2];
};

// Compaction appends: every block reserves its whole range with ONE atomic (same-address
// atomics serialise in L2 at ~10 ns each; a per-wave append over 2.3M pixels cost 0.6-1.5 ms).
#define CBLK 256   // threads per compaction block
#define EPT 4      // edges per thread (k_cmin: latency-bound, wants more waves)

// exclusive block scan of cnt + one atomicAdd on counter: returns this thread's first slot
__device__ __forceinline__ uint32_t block_append(uint32_t cnt, uint32_t* counter) {
    __shared__ uint32_t s_w[CBLK / 64];
    __shared__ uint32_t s_base;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t x = cnt;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    if (lane == 63) s_w[wave] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
#pragma unroll
        for (int w = 0; w < CBLK / 64; ++w) {
            const uint32_t u = s_w[w];
            s_w[w] = t;
            t += u;
        }
        s_base = t ? atomicAdd(counter, t) : 0u;
    }
    __syncthreads();
    return s_base + s_w[wave] + x - cnt;
}

// One block per BT x BT tile of the tile phase.  Tile-phase components never cross a tile border,
// so all parallel pixel edges between two components inside the tile (~3-5 per pair: a boundary
// several pixels long) meet in this block: they are merged in an LDS hash table keyed by the
// unordered component pair, keeping the minimum key, and only one edge per pair is listed.  Every
// round's minimum per component is a minimum over whole pairs, so the MST is unchanged, and every
// round sweeps ~3x fewer edges.  Pairs that find no slot (tile caps of 0/1 make ~4k components per
// tile) are listed unmerged.
#define EH 1024                      // hash slots per block (~500 pairs per tile at C2; 16 KB of LDS)
#define EH_EMPTY 0xFFFFFFFFFFFFFFFFull
__global__ __launch_bounds__(CBLK) void k_cedges(CPair P, int W, int H) {
    const CView V = P.v[blockIdx.y];
    const int ntx = (W + BT - 1) / BT;
    const int tx0 = (blockIdx.x % ntx) * BT, ty0 = (blockIdx.x / ntx) * BT;
    const int lx = threadIdx.x & (BT - 1);
    __shared__ unsigned long long hpair[EH], hmin[EH];
    for (int i = threadIdx.x; i < EH; i += CBLK) { hpair[i] = EH_EMPTY; hmin[i] = SM_KEY_NONE; }
    __syncthreads();
    constexpr int RPT = BT * BT / CBLK;  // rows per thread: tile row (threadIdx.x / BT) + i * CBLK / BT
    uint32_t ovf = 0;                   // bit 2i / 2i+1: right / down edge of row i listed unmerged
    const int x = tx0 + lx;
#pragma unroll 4
    for (int i = 0; i < RPT; ++i) {
        const int y = ty0 + (int)(threadIdx.x / BT) + i * (CBLK / BT);
        if (x >= W || y >= H) continue;
        const uint32_t p = (uint32_t)y * (uint32_t)W + (uint32_t)x;
        const uint32_t c = V.comp[p];
#pragma unroll
        for (int d = 0; d < 2; ++d) {
            if (d == 0 ? x + 1 >= W : y + 1 >= H) continue;
            const uint32_t q = d == 0 ? p + 1 : p + (uint32_t)W;
            const uint32_t cq = V.comp[q];
            if (cq == c) continue;
            const uint32_t cu = V.cid[c], cv = V.cid[cq];
            const unsigned long long pr = cu < cv ? ((unsigned long long)cu << 32) | cv : ((unsigned long long)cv << 32) | cu;
            const unsigned long long key = sm_edge_key(d == 0 ? V.wR[p] : V.wD[p], p, (uint32_t)d);
            uint32_t h = (uint32_t)((pr * 0x9E3779B97F4A7C15ull) >> 54);  // 10 bits
            bool done = false;
            for (int probe = 0; probe < 8 && !done; ++probe) {
                const unsigned long long old = atomicCAS(&hpair[h], EH_EMPTY, pr);
                if (old == EH_EMPTY || old == pr) {
                    atomicMin(&hmin[h], key);
                    done = true;
                }
                h = (h + 1) & (EH - 1);
            }
            if (!done) ovf |= 1u << (2 * i + d);
        }
    }
    __syncthreads();
    constexpr int SPT = EH / CBLK;
    uint32_t occ = 0;
#pragma unroll
    for (int j = 0; j < SPT; ++j)
        if (hpair[threadIdx.x + j * CBLK] != EH_EMPTY) occ |= 1u << j;
    // Round 0 of the contracted rounds happens here (round 5: its k_cmin is not launched): every listed
    // edge joins two distinct components (labels are the ids), so the list is round 0's output list
    // (list 1) as it stands, and each edge offers its key to both endpoints' round-0 minima
    CEdge* out = V.edges + V.emax;
    uint32_t slot = block_append(__builtin_popcount(occ) + __builtin_popcount(ovf), &V.counts[2]);
    auto emit = [&](const CEdge& E) __attribute__((always_inline)) {
        out[slot++] = E;
        atomicMin(&V.best[E.u], E.key);
        atomicMin(&V.best[E.v], E.key);
    };
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
        if (!(occ & (1u << j))) continue;
        const unsigned long long pr = hpair[threadIdx.x + j * CBLK];
        emit(CEdge{hmin[threadIdx.x + j * CBLK], (uint32_t)(pr >> 32), (uint32_t)pr});
    }
    while (ovf) {
        const int b = __builtin_ctz(ovf);
        ovf &= ovf - 1;
        const int i = b >> 1, d = b & 1;
        const int y = ty0 + (int)(threadIdx.x / BT) + i * (CBLK / BT);
        const uint32_t p = (uint32_t)y * (uint32_t)W + (uint32_t)x;
        const uint32_t q = d == 0 ? p + 1 : p + (uint32_t)W;
        emit(CEdge{sm_edge_key(d == 0 ? V.wR[p] : V.wD[p], p, (uint32_t)d), V.cid[V.comp[p]], V.cid[V.comp[q]]});
    }
}

__device__ __forceinline__ bool cround_done(const CView& V, int r) { return r > 0 && V.flags[r - 1] == 0; }

// Segmented min over runs of equal target among consecutive lanes (shfl_up scan where a lane
// only folds in a value from a lane with the same target: any such subset is valid, and a run's
// last lane ends up with the whole run's minimum).  True on the lanes holding a run's minimum.
__device__ __forceinline__ bool wave_seg_min(bool active, uint32_t& c, unsigned long long& k) {
    const int lane = threadIdx.x & 63;
    if (!active) { c = 0xFFFFFFFFu; k = SM_KEY_NONE; }
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const unsigned long long y = __shfl_up(k, off);
        const uint32_t cy = __shfl_up(c, off);
        if (lane >= off && cy == c && y < k) k = y;
    }
    const uint32_t cn = __shfl_down(c, 1);
    return active && (lane == 63 || cn != c);
}

// Per-block direct-mapped LDS table of component minima: late rounds have few components with
// thousands of incident edges each, and global atomics on one best[] word serialise in L2.  A
// slot is claimed by CAS on its tag; a collision falls through to the global atomic.
#define CTAB 1024  // (12 KB: 8 waves per SIMD; 2048 slots held k_cmin to 6)
struct CTable {
    uint32_t tag[CTAB];
    unsigned long long mn[CTAB];
};
__device__ __forceinline__ void ctab_min(CTable& T, uint32_t c, unsigned long long k, unsigned long long* best) {
    const uint32_t slot = (c * 2654435761u) >> 22;  // 10-bit multiplicative hash
    const uint32_t old = atomicCAS(&T.tag[slot], 0xFFFFFFFFu, c);
    if (old == 0xFFFFFFFFu || old == c) atomicMin(&T.mn[slot], k);
    else atomicMin(&best[c], k);
}

// Round r reads edge list (r & 1) and appends the edges that still join two components, with
// relabelled endpoints, to list (r & 1) ^ 1, so each round sweeps only live edges.  Grid-stride
// over a fixed grid: the host never needs the edge count.
__global__ __launch_bounds__(CBLK) void k_cmin(CPair P, int rnd) {
    const CView V = P.v[blockIdx.y];
    if (cround_done(V, rnd)) return;
    __shared__ CTable T;
    const int ib = rnd & 1;
    const uint32_t ne = V.counts[1 + ib];
    if (blockIdx.x * (CBLK * EPT) >= ne) return;  // block-uniform
    unsigned long long* best = V.best + (size_t)ib * V.bstride;
    for (int i = threadIdx.x; i < CTAB; i += CBLK) {
        T.tag[i] = 0xFFFFFFFFu;
        T.mn[i] = SM_KEY_NONE;
    }
    __syncthreads();
    const CEdge* in = V.edges + (size_t)ib * V.emax;
    CEdge* out = V.edges + (size_t)(ib ^ 1) * V.emax;
    for (uint32_t b0 = blockIdx.x * (CBLK * EPT); b0 < ne; b0 += gridDim.x * (CBLK * EPT)) {
        uint32_t bits = 0;
        CEdge keep[EPT];
#pragma unroll
        for (int i = 0; i < EPT; ++i) {
            const uint32_t e = b0 + i * CBLK + threadIdx.x;
            const bool live = e < ne;
            CEdge E{SM_KEY_NONE, 0u, 0u};
            if (live) E = in[e];
            uint32_t lu = live ? V.lab[E.u] : 0u, lv = live ? V.lab[E.v] : 0u;
            const bool act = live && lu != lv;
            keep[i] = CEdge{E.key, lu, lv};
            if (act) bits |= 1u << i;
            unsigned long long ku = E.key, kv = E.key;
            if (wave_seg_min(act, lu, ku)) ctab_min(T, lu, ku, best);
            if (wave_seg_min(act, lv, kv)) ctab_min(T, lv, kv, best);
        }
        uint32_t slot = block_append(__builtin_popcount(bits), &V.counts[2 - ib]);
#pragma unroll
        for (int i = 0; i < EPT; ++i)
            if (bits & (1u << i)) out[slot++] = keep[i];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < CTAB; i += CBLK)
        if (T.tag[i] != 0xFFFFFFFFu) atomicMin(&best[T.tag[i]], T.mn[i]);
}

__global__ void k_chook(CPair P, int W, int rnd) {
    const CView V = P.v[blockIdx.y];
    if (cround_done(V, rnd)) return;
    const int ib = rnd & 1;
    const unsigned long long* best = V.best + (size_t)ib * V.bstride;
    unsigned long long* best_next = V.best + (size_t)(ib ^ 1) * V.bstride;
    if (blockIdx.x == 0 && threadIdx.x == 0) V.counts[1 + ib] = 0;  // list k_cmin just read: next output
    const uint32_t K = V.counts[0];
    for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < K; c += gridDim.x * blockDim.x) {
        if (V.lab[c] != c) continue;  // current roots only
        uint32_t h = c;
        const unsigned long long k = best[c];
        if (k != SM_KEY_NONE) {
            const uint32_t a = (uint32_t)(k >> 1) & 0xFFFFFFFFu;
            const uint32_t vert = (uint32_t)(k & 1ull);
            const uint32_t b = a + (vert ? (uint32_t)W : 1u);
            const uint32_t la = V.lab[V.cid[V.comp[a]]];
            const uint32_t c2 = la == c ? V.lab[V.cid[V.comp[b]]] : la;
            if (!(best[c2] == k && c < c2)) {  // mutual choice: the smaller id stays root
                h = c2;
                if (vert) V.mD[a] = 1; else V.mR[a] = 1;
                V.flags[rnd] = 1;
            }
        }
        V.hook[c] = h;
        best_next[c] = SM_KEY_NONE;  // next round's roots are a subset of this round's
    }
}

// Chase every label to the root of its hook tree; shortcut the old root's hook in place
// (concurrent chasers then still reach the same root).
__global__ void k_crelabel(CPair P, int rnd) {
    const CView V = P.v[blockIdx.y];
    if (cround_done(V, rnd) || V.flags[rnd] == 0) return;
    const uint32_t K = V.counts[0];
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < K; i += gridDim.x * blockDim.x) {
        const uint32_t l = V.lab[i];
        uint32_t r = V.hook[l];
        for (int it = 0; it < (1 << 26); ++it) {
            const uint32_t rr = V.hook[r];
            if (rr == r) break;
            r = rr;
        }
        if (r != l) V.hook[l] = r;
        V.lab[i] = r;
    }
}

// cross-rank WTA helpers: candidate index where this rank holds the global minimum
__global__ void k_cand(const double* __restrict__ minc, const double* __restrict__ gmin, const int32_t* __restrict__ idx,
                       int32_t* __restrict__ cand, size_t N) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < N) cand[i] = sm_rule_cand32(minc[i], gmin[i], idx[i]);
}

__global__ void k_finalize(const double* __restrict__ gmin, const int32_t* __restrict__ gidx, double* __restrict__ minc,
                           int32_t* __restrict__ idx, float* __restrict__ disp, size_t N) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < N) sm_rule_finalize32(gmin[i], gidx[i], minc[i], idx[i], disp[i]);
}

// subpixel variant: the candidate carries the rank's subpixel disparity in its low word
__global__ void k_cand64(const double* __restrict__ minc, const double* __restrict__ gmin, const int32_t* __restrict__ idx,
                         const float* __restrict__ disp, unsigned long long* __restrict__ cand, size_t N) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < N) cand[i] = sm_rule_cand64(minc[i], gmin[i], idx[i], __float_as_uint(disp[i]));
}

__global__ void k_finalize64(const double* __restrict__ gmin, const unsigned long long* __restrict__ gkey,
                             double* __restrict__ minc, int32_t* __restrict__ idx, float* __restrict__ disp, size_t N) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < N) {
        uint32_t bits;
        sm_rule_finalize64(gmin[i], gkey[i], minc[i], idx[i], bits);
        disp[i] = __uint_as_float(bits);
    }
}

// MC-CNN ingest (Stereo3DMST.cpp:764-803): slices [d0, d0 + D) of a caller-supplied raw volume
// [Dv][H][W] -> f32 cost rows Cst[slot][Dpad] after the reference's clamp, NaN -> 0.5 else
// min(0.5, x) (:785-803; std::min(0.5f, x) returns 0.5 unless x < 0.5).  Row padding (d >= D)
// gets 3.0, like the AGD path's out-of-range slices (finite; never reaches the WTA).  A block
// moves 64 consecutive pixels x 64 slices through LDS: 256-B coalesced reads along x per slice,
// one 256-B row segment written per pixel at its slot.
__global__ __launch_bounds__(256) void k_vol_rows(const float* __restrict__ vin, size_t N, int d0, int D, int Dpad,
                                                  const uint32_t* __restrict__ slotpix, float* __restrict__ Cst) {
    __shared__ float t[64][65];
    const size_t p0 = (size_t)blockIdx.x * 64;
    const int dc = blockIdx.y * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int dd = ty; dd < 64; dd += 4) {
        const int d = dc + dd;
        float v = 3.0f;
        if (d < D && p0 + tx < N) {
            const float r = vin[(size_t)(d0 + d) * N + p0 + tx];
            v = r != r ? 0.5f : (r < 0.5f ? r : 0.5f);
        }
        t[dd][tx] = v;
    }
    __syncthreads();
    for (int px = ty; px < 64; px += 4) {
        if (p0 + px >= N) break;
        if (dc + tx < Dpad) Cst[(size_t)slotpix[p0 + px] * Dpad + dc + tx] = t[tx][px];
    }
}

hipError_t launch_vol_rows(hipStream_t st, const float* vin, size_t N, int d0, int D, int Dpad, const uint32_t* slotpix,
                           float* Cst) {
    const dim3 g((unsigned)((N + 63) / 64), (unsigned)((Dpad + 63) / 64));
    hipLaunchKernelGGL(k_vol_rows, g, dim3(256), 0, st, vin, N, d0, D, Dpad, slotpix, Cst);
    return hipGetLastError();
}

// debug: scatter the fp64 rows of slices [0, D) back to [d][y][x]
__global__ void k_rows_to_volume(const SmMeta* __restrict__ meta, const double* __restrict__ U, int nslots, int Dpad,
                                 int D, size_t N, double* __restrict__ out) {
    const int s = blockIdx.x;
    if (s >= nslots) return;
    const uint32_t pix = meta[s].pix;
    for (int d = threadIdx.x; d < D; d += blockDim.x) out[(size_t)d * N + pix] = U[(size_t)s * Dpad + d];
}

// ---------------------------------------------------------------------------------------------
// host-callable launchers (extern "C++" within the library)
// ---------------------------------------------------------------------------------------------
#include <cstdlib>
#include "sm_launch.h"
#include "sm_knob.h"

hipError_t launch_prep(hipStream_t st, const uint8_t* l, const uint8_t* r, int W, int H, int stride, uint32_t* lb,
                       float* lg, uint32_t* rb, float* rg, uint2* lrec, uint2* rrec, uint32_t* lrec4, uint32_t* rrec4) {
    ImgPair P{{l, r}, {lb, rb}, {lg, rg}, {lrec, rrec}, {lrec4, rrec4}};
    dim3 g((W + 255) / 256, H, 2);
    hipLaunchKernelGGL(k_prep, g, dim3(256), 0, st, P, W, H, stride);
    return hipGetLastError();
}

hipError_t launch_median_weights(hipStream_t st, const uint32_t* lb, const uint32_t* rb, uint32_t* lmed, uint32_t* rmed,
                                 uint16_t* lwR, uint16_t* lwD, uint16_t* rwR, uint16_t* rwD, int W, int H) {
    MedPair M{{lb, rb}, {lmed, rmed}};
    dim3 g((W + 255) / 256, H, 2);
    hipLaunchKernelGGL(k_median, g, dim3(256), 0, st, M, W, H);
    WeightPair P{{lmed, rmed}, {lwR, rwR}, {lwD, rwD}};
    hipLaunchKernelGGL(k_weights, g, dim3(256), 0, st, P, W, H);
    return hipGetLastError();
}

hipError_t launch_cost_volume(hipStream_t st, const uint32_t* lb, const float* lg, const uint32_t* rb, const float* rg,
                              const float* atab, int W, int H, int d0, int D, float* lvol, float* rvol) {
    dim3 g((W + CV_TX - 1) / CV_TX, H, (D + CV_DC - 1) / CV_DC);
    hipLaunchKernelGGL(k_cost_volume, g, dim3(CV_TX), 0, st, lb, lg, rb, rg, atab, W, H, d0, D, lvol, rvol);
    return hipGetLastError();
}

hipError_t launch_bor_local(hipStream_t st, const MstArgs& a, int W, int H, uint32_t* const ccount[2],
                            uint32_t* const clab[2], size_t bstride) {
    MstPair P;
    for (int v = 0; v < 2; ++v)
        P.v[v] = MstView{a.wR[v], a.wD[v], a.comp[v], a.best[v], a.root[v], a.mR[v], a.mD[v], a.flags[v], ccount[v],
                         clab[v], bstride};
    dim3 g((W + BT - 1) / BT, (H + BT - 1) / BT, a.nviews);
    // Tile-phase Boruvka iterations: any cap is exact (unfinished components continue in the
    // contracted rounds); 4 is the measured optimum at C2 (tools/gpu_mst_sweep.sh).
    const char* e = sm_knob("SM_MST_LOCAL_ITERS");
    const int max_iter = e ? atoi(e) : 4;
    hipLaunchKernelGGL(k_bor_local, g, dim3(BTHREADS), 0, st, P, W, H, max_iter);
    return hipGetLastError();
}

hipError_t launch_bor_round(hipStream_t st, const MstArgs& a, int W, int H, int r) {
    MstPair P;
    for (int v = 0; v < 2; ++v)
        P.v[v] = MstView{a.wR[v], a.wD[v], a.comp[v], a.best[v], a.root[v], a.mR[v], a.mD[v], a.flags[v], nullptr,
                         nullptr, 0};
    dim3 g((W + 255) / 256, H, a.nviews);
    hipLaunchKernelGGL(k_bor_min, g, dim3(256), 0, st, P, W, H, r);
    hipLaunchKernelGGL(k_bor_hook, g, dim3(256), 0, st, P, W, H, r);
    hipLaunchKernelGGL(k_bor_root, g, dim3(256), 0, st, P, W, H, r);
    hipLaunchKernelGGL(k_bor_relabel, g, dim3(256), 0, st, P, W, H, r);
    return hipGetLastError();
}

// MST completeness word read by every layout kernel: the last enqueued contracted round r hooked
// nothing in any view (stage_mst enqueues rounds without a host check)
__global__ void k_mst_done(const int* __restrict__ f0, const int* __restrict__ f1, int r, int nviews, int* ok) {
    if (threadIdx.x == 0) *ok = (f0[r] == 0 && (nviews < 2 || f1[r] == 0)) ? 1 : 0;
}

// one launch for a frame stage's zero-fills (each hipMemsetAsync is its own dispatch)
__global__ __launch_bounds__(256) void k_zero(ZeroList z) {
    uint8_t* p = static_cast<uint8_t*>(z.p[blockIdx.y]);
    const size_t n = z.n[blockIdx.y], n16 = n / 16;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256)
        reinterpret_cast<uint4*>(p)[i] = make_uint4(0u, 0u, 0u, 0u);
    if (blockIdx.x == 0 && threadIdx.x < n - n16 * 16) p[n16 * 16 + threadIdx.x] = 0;
}

hipError_t launch_zero(hipStream_t st, const ZeroList& z) {
    if (z.count <= 0) return hipSuccess;
    size_t mx = 0;
    for (int i = 0; i < z.count; ++i) {
        if (reinterpret_cast<uintptr_t>(z.p[i]) & 15u) return hipErrorInvalidValue;
        mx = mx > z.n[i] ? mx : z.n[i];
    }
    const unsigned gx = (unsigned)std::min<size_t>(std::max<size_t>((mx / 16 + 255) / 256, 1), 512);
    hipLaunchKernelGGL(k_zero, dim3(gx, z.count), dim3(256), 0, st, z);
    return hipGetLastError();
}

hipError_t launch_mst_done(hipStream_t st, const MstArgs& a, int r, int* ok) {
    hipLaunchKernelGGL(k_mst_done, dim3(1), dim3(64), 0, st, a.flags[0], a.flags[1], r, a.nviews, ok);
    return hipGetLastError();
}

hipError_t launch_cand(hipStream_t st, const double* minc, const double* gmin, const int32_t* idx, int32_t* cand, size_t N) {
    hipLaunchKernelGGL(k_cand, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, st, minc, gmin, idx, cand, N);
    return hipGetLastError();
}

hipError_t launch_finalize(hipStream_t st, const double* gmin, const int32_t* gidx, double* minc, int32_t* idx, float* disp,
                           size_t N) {
    hipLaunchKernelGGL(k_finalize, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, st, gmin, gidx, minc, idx, disp, N);
    return hipGetLastError();
}

hipError_t launch_cand64(hipStream_t st, const double* minc, const double* gmin, const int32_t* idx, const float* disp,
                         unsigned long long* cand, size_t N) {
    hipLaunchKernelGGL(k_cand64, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, st, minc, gmin, idx, disp, cand, N);
    return hipGetLastError();
}

hipError_t launch_finalize64(hipStream_t st, const double* gmin, const unsigned long long* gkey, double* minc, int32_t* idx,
                             float* disp, size_t N) {
    hipLaunchKernelGGL(k_finalize64, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, st, gmin, gkey, minc, idx, disp, N);
    return hipGetLastError();
}

hipError_t launch_rows_to_volume(hipStream_t st, const SmMeta* meta, const double* U, int nslots, int Dpad, int D,
                                 size_t N, double* out) {
    hipLaunchKernelGGL(k_rows_to_volume, dim3(nslots), dim3(64), 0, st, meta, U, nslots, Dpad, D, N, out);
    return hipGetLastError();
}

static CPair make_cpair(const MstArgs& a, const MstCompact& c) {
    CPair P;
    for (int v = 0; v < 2; ++v)
        P.v[v] = CView{a.wR[v], a.wD[v], a.comp[v], c.cid[v], c.counts[v], reinterpret_cast<CEdge*>(c.edges[v]), c.emax,
                       c.lab[v], c.hook[v], a.best[v], c.bstride, a.mR[v], a.mD[v], a.flags[v]};
    return P;
}

hipError_t launch_bor_compact(hipStream_t st, const MstArgs& a, const MstCompact& c, int W, int H) {
    const CPair P = make_cpair(a, c);
    const dim3 gt((unsigned)(((W + BT - 1) / BT) * ((H + BT - 1) / BT)), a.nviews);
    hipLaunchKernelGGL(k_cedges, gt, dim3(CBLK), 0, st, P, W, H);
    return hipGetLastError();
}

// fixed grids (grid-stride kernels): K and E' stay on the device
#define CGRID_K 256    // blocks of 256 over components
#define CGRID_E 512    // blocks of CBLK * EPT over edges


hipError_t launch_bor_cround(hipStream_t st, const MstArgs& a, const MstCompact& c, int W, int r) {
    const CPair P = make_cpair(a, c);
    if (r > 0) hipLaunchKernelGGL(k_cmin, dim3(CGRID_E, a.nviews), dim3(CBLK), 0, st, P, r);  // (round 0: k_cedges)
    hipLaunchKernelGGL(k_chook, dim3(CGRID_K, a.nviews), dim3(256), 0, st, P, W, r);
    hipLaunchKernelGGL(k_crelabel, dim3(CGRID_K, a.nviews), dim3(256), 0, st, P, r);
    return hipGetLastError();
}
