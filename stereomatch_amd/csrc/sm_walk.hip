// sm_walk.hip -- tree-filter walkers: leaf->root (up) and root->leaf (down) passes over the
// heavy paths of one light-depth round, for both views in one launch (blockIdx.y = view).
//
// Aggregation rows U[slot][Dpad] are fp64; lane l owns slices [l*SPL, l*SPL+SPL) of this call.
// One wave walks one heavy path; a 256-thread block runs four independent paths.  A path is
// processed in chunks of CH consecutive nodes with a two-stage software pipeline:
//   * the metadata of chunk c+1 (CH x 32 B, one dword per lane: lane 8j+f holds word f of node j)
//     is in flight while chunk c computes;
//   * all row / image loads of chunk c are issued together, then one wait;
//   * off-chain work (AGD costs, edge-weight lookups in LDS tables) is done for the whole chunk
//     before the serial recurrence, which is then only fma/add on registers;
//   * the down pass keeps the chunk's CH results in registers and runs the CH WTA reductions
//     interleaved (DPP), writing one output store per array per chunk.
//
// Per node the arithmetic is exactly the shipped reference's (DESIGN.md "Shipped arithmetic"):
//   up  : acc = 0; for children c in descending (w,a,b) key order: acc = fma(S_c, A_up(c), acc);
//         A_up(v) = acc + C(v)                                     (Stereo3DMST.cpp:125-137)
//   down: A(v) = fma(S_v, A(parent), S2_v * A_up(v)); A(root) = A_up(root)   (:145-157)
//   WTA : strict-< first minimum over ascending d                  (:173-185, .cu:1700-1717)
// with C(v) the AGD cost of PatchMatchStereoGPU.cu:1482-1550 computed on the fly, so the result
// does not depend on the schedule (rounds, paths, chunks, waves).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "sm_common.h"
#include "sm_launch.h"

// per-view mutable state; the read-only metadata and path lists are separate __restrict__ kernel
// arguments (kernarg-derived, provably unclobbered)
struct WalkView {
    int npaths;
    double* U;             // [slots][Dpad]
    int32_t* idx;          // W*H   (down pass)
    double* minc;          // W*H   (down pass)
    float* disp;           // W*H   (down pass)
};

#define SM_NUM_W 766
#define S_ZERO SM_NUM_W    // LDS S-table entry holding 0.0 (absent children)

__device__ __forceinline__ uint32_t uniform(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ float rgray(uint2 r) { return __uint_as_float(r.y); }

// AGD cost (PatchMatchStereoGPU.cu:1518-1543) from {bgrx, gray} records:
// r0 = right(x), l0 = left(x+d), gr1 = gray(right(x+1)), gl1 = gray(left(x+d+1))
__device__ __forceinline__ float agd_rec(uint2 r0, uint2 l0, float gr1, float gl1, const float* __restrict__ atab) {
    const uint32_t l1 = __builtin_amdgcn_sad_u8(r0.x, l0.x, 0u);  // exact integer colour L1
    const float a = atab[l1];
    float g = rgray(l0) - rgray(r0);
    g = g + (gr1 - gl1);
    const float b = 0.89f * fminf(fabsf(g), 2.0f);
    return a + b;
}

template <int SPL>
__device__ __forceinline__ void load_row(const double* __restrict__ U, uint32_t slot, int Dpad, int lane, double (&r)[SPL]) {
    const double* p = U + (size_t)slot * Dpad + lane * SPL;
    if constexpr (SPL == 1) {
        r[0] = p[0];
    } else {
#pragma unroll
        for (int k = 0; k < SPL; k += 2) {
            const double2 t = *reinterpret_cast<const double2*>(p + k);
            r[k] = t.x;
            r[k + 1] = t.y;
        }
    }
}

template <int SPL>
__device__ __forceinline__ void store_row(double* __restrict__ U, uint32_t slot, int Dpad, int lane, const double (&r)[SPL]) {
    double* p = U + (size_t)slot * Dpad + lane * SPL;
    if constexpr (SPL == 1) {
        p[0] = r[0];
    } else {
#pragma unroll
        for (int k = 0; k < SPL; k += 2) *reinterpret_cast<double2*>(p + k) = make_double2(r[k], r[k + 1]);
    }
}

// lane-distributed metadata of CH nodes: lane 8j+f holds word f of node j (8 nodes per VGPR)
template <int CH>
struct MetaVec {
    uint32_t w[(CH + 7) / 8];
};

template <int CH>
__device__ __forceinline__ void load_meta(MetaVec<CH>& mv, const uint32_t* __restrict__ meta32, int lane, int first,
                                          int step, int n) {
    // node j of the chunk = first + step*j (clamped to the chunk's valid nodes)
#pragma unroll
    for (int q = 0; q < (CH + 7) / 8; ++q) {
        const int j = q * 8 + (lane >> 3);
        const int jj = j < n ? j : n - 1;
        mv.w[q] = meta32[(size_t)(first + step * jj) * 8 + (lane & 7)];
    }
}

template <int CH>
__device__ __forceinline__ uint32_t mfield(const MetaVec<CH>& mv, int j, int f) {
    return __builtin_amdgcn_readlane(mv.w[j >> 3], ((j & 7) << 3) + f);
}

// SmMeta words: 0 pix, 1 parent, 2 lo (wp|cw0|cw1), 3 hi (cw2|cw3|nch|hidx|has_light), 4..7 cslot
__device__ __forceinline__ uint32_t lo_wp(uint32_t lo) { return lo & 1023u; }
__device__ __forceinline__ uint32_t cw_of(uint32_t lo, uint32_t hi, int i) {
    return i == 0 ? (lo >> 10) & 1023u : i == 1 ? (lo >> 20) & 1023u : i == 2 ? hi & 1023u : (hi >> 10) & 1023u;
}
__device__ __forceinline__ uint32_t hi_nch(uint32_t hi) { return (hi >> 20) & 7u; }
__device__ __forceinline__ uint32_t hi_hidx(uint32_t hi) { return (hi >> 23) & 3u; }
__device__ __forceinline__ uint32_t hi_light(uint32_t hi) { return (hi >> 25) & 1u; }

struct WalkShared {
    float atab[SM_MAX_W + 1];
    double slut[SM_NUM_W + 1];  // [SM_NUM_W] = 0.0
    double s2lut[SM_NUM_W];
};

__device__ __forceinline__ void load_tables(WalkShared& sh, const float* atab_g, const double* slut_g, const double* s2lut_g) {
    for (int i = threadIdx.x; i <= SM_MAX_W; i += blockDim.x) sh.atab[i] = atab_g[i];
    for (int i = threadIdx.x; i < SM_NUM_W; i += blockDim.x) {
        sh.slut[i] = slut_g[i];
        sh.s2lut[i] = s2lut_g[i];
    }
    if (threadIdx.x == 0) sh.slut[SM_NUM_W] = 0.0;
    __syncthreads();
}

// ---------------------------------------------------------------------------------------------
// up pass
// ---------------------------------------------------------------------------------------------
template <int SPL, int CH>
__device__ __forceinline__ void up_chunk(const MetaVec<CH>& mv, int n, int top, int view, int lane, int W, int Dpad,
                                         int dbase, int dend, const uint2* __restrict__ own, const uint2* __restrict__ oth,
                                         double* __restrict__ U, const WalkShared& sh, double (&xc)[SPL]) {
    // ---- all vector loads of the chunk
    double lr[CH][2][SPL];
    uint2 ob[CH][SPL + 1], o0[CH], o1[CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) {
        if (j < n) {
            const uint32_t hi = mfield(mv, j, 3);
            const uint32_t nch = hi_nch(hi), hidx = hi_hidx(hi);
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const uint32_t i = (uint32_t)k + ((uint32_t)k >= hidx ? 1u : 0u);  // child position of light slot k
                if (i < nch) load_row<SPL>(U, mfield(mv, j, 4 + (int)i), Dpad, lane, lr[j][k]);
            }
            const int pix = (int)mfield(mv, j, 0);
            const int y = pix / W;
            const int x = pix - y * W;
            const size_t row = (size_t)y * W;
            // own pixels x, x+1 through a lane-dependent (vector) load: a uniform address would become
            // a scalar-cache load whose lgkmcnt waits serialise with the LDS table reads
            const uint2 t = own[row + x + (lane & 1)];  // x+1 == W reads the next row / the pad: masked below
            o0[j] = make_uint2(__builtin_amdgcn_readlane(t.x, 0), __builtin_amdgcn_readlane(t.y, 0));
            o1[j] = make_uint2(__builtin_amdgcn_readlane(t.x, 1), __builtin_amdgcn_readlane(t.y, 1));
            const long long base = view ? (long long)(row + x) + dbase : (long long)(row + x) - dbase - (SPL - 1);
#pragma unroll
            for (int q = 0; q <= SPL; ++q) ob[j][q] = oth[base + q];
        }
    }
    // ---- off-chain work: costs and edge factors of every node of the chunk
    double c[CH][SPL], Sv[CH][4];
#pragma unroll
    for (int j = 0; j < CH; ++j) {
        const uint32_t lo = mfield(mv, j, 2), hi = mfield(mv, j, 3);
        const uint32_t nch = hi_nch(hi);
#pragma unroll
        for (int i = 0; i < 4; ++i) Sv[j][i] = sh.slut[(uint32_t)i < nch ? cw_of(lo, hi, i) : (uint32_t)S_ZERO];
        const int pix = (int)mfield(mv, j, 0);
        const int y = pix / W;
        const int x = pix - y * W;
#pragma unroll
        for (int k = 0; k < SPL; ++k) {
            const int d = dbase + k;
            float v;
            bool ok;
            if (view) {  // right reference: right(x) vs left(x+d)
                ok = d < dend && x + d + 1 < W;
                v = agd_rec(o0[j], ob[j][k], rgray(o1[j]), rgray(ob[j][k + 1]), sh.atab);
            } else {     // left pixel x at d: cost(x-d, d); x-d<0 and column W-1 -> 3.0
                ok = d < dend && x - d >= 0 && x + 1 < W;
                v = agd_rec(ob[j][SPL - 1 - k], o0[j], rgray(ob[j][SPL - k]), rgray(o1[j]), sh.atab);
            }
            c[j][k] = (double)(ok ? v : 3.0f);
        }
    }
    // ---- serial recurrence along the path (bottom -> top)
#pragma unroll
    for (int j = 0; j < CH; ++j) {
        if (j < n) {
            const uint32_t hi = mfield(mv, j, 3);
            const uint32_t nch = hi_nch(hi), hidx = hi_hidx(hi);
            double acc[SPL];
#pragma unroll
            for (int k = 0; k < SPL; ++k) acc[k] = 0.0;
#pragma unroll
            for (uint32_t i = 0; i < 4; ++i) {
                if (i < nch) {
                    double v[SPL];
                    if (i == hidx) {
#pragma unroll
                        for (int k = 0; k < SPL; ++k) v[k] = xc[k];
                    } else {
                        const uint32_t kk = i - (i > hidx ? 1u : 0u);
                        if (kk == 0) {
#pragma unroll
                            for (int k = 0; k < SPL; ++k) v[k] = lr[j][0][k];
                        } else if (kk == 1) {
#pragma unroll
                            for (int k = 0; k < SPL; ++k) v[k] = lr[j][1][k];
                        } else {
                            load_row<SPL>(U, mfield(mv, j, 4 + (int)i), Dpad, lane, v);  // root's third light child
                        }
                    }
#pragma unroll
                    for (int k = 0; k < SPL; ++k) acc[k] = __builtin_fma(Sv[j][i], v[k], acc[k]);
                }
            }
#pragma unroll
            for (int k = 0; k < SPL; ++k) xc[k] = acc[k] + c[j][k];
            store_row<SPL>(U, (uint32_t)(top - j), Dpad, lane, xc);
        }
    }
}

template <int SPL, int CH>
__global__ __launch_bounds__(256) void k_up_walk(WalkView V0, WalkView V1, const uint32_t* __restrict__ meta0,
                                                 const uint32_t* __restrict__ meta1, const SmPath* __restrict__ paths0,
                                                 const SmPath* __restrict__ paths1, const uint2* __restrict__ Lrec,
                                                 const uint2* __restrict__ Rrec, const float* __restrict__ atab_g,
                                                 const double* __restrict__ slut_g, const double* __restrict__ s2lut_g,
                                                 int W, int Dpad, int dcall, int dglob0) {
    __shared__ WalkShared sh;
    load_tables(sh, atab_g, slut_g, s2lut_g);
    const int view = blockIdx.y;
    const WalkView& V = view ? V1 : V0;
    const uint32_t* __restrict__ meta32 = view ? meta1 : meta0;
    const int lane = threadIdx.x & 63;
    const int pi = (int)uniform(blockIdx.x * 4 + (threadIdx.x >> 6));
    if (pi >= V.npaths) return;
    const SmPath path = (view ? paths1 : paths0)[pi];
    const int head = (int)uniform(path.head), len = (int)uniform(path.len);
    const int dbase = dglob0 + lane * SPL;  // global disparity of this lane's first slice
    const int dend = dglob0 + dcall;
    const uint2* __restrict__ own = view ? Rrec : Lrec;  // the view's reference image
    const uint2* __restrict__ oth = view ? Lrec : Rrec;  // the matched image
    double xc[SPL];
#pragma unroll
    for (int k = 0; k < SPL; ++k) xc[k] = 0.0;
    // chunk c covers nodes top_c, top_c-1, ... (bottom of the path first)
    int top = head + len - 1;
    int n = min(CH, top - head + 1);
    MetaVec<CH> cur;
    load_meta<CH>(cur, meta32, lane, top, -1, n);
    while (true) {
        const int ntop = top - CH;
        const int nn = ntop >= head ? min(CH, ntop - head + 1) : 0;
        MetaVec<CH> nxt;
        if (nn > 0) load_meta<CH>(nxt, meta32, lane, ntop, -1, nn);  // prefetch the next chunk's metadata
        up_chunk<SPL, CH>(cur, n, top, view, lane, W, Dpad, dbase, dend, own, oth, V.U, sh, xc);
        if (nn == 0) break;
        cur = nxt;
        top = ntop;
        n = nn;
    }
}

// ---------------------------------------------------------------------------------------------
// down pass + WTA
// ---------------------------------------------------------------------------------------------
// min of a double with the value DPP-moved from another lane (both 32-bit halves moved)
template <int CTRL>
__device__ __forceinline__ double dpp_min(double v) {
    const int lo = __double2loint(v), hi = __double2hiint(v);
    const int lo2 = __builtin_amdgcn_update_dpp(lo, lo, CTRL, 0xF, 0xF, false);
    const int hi2 = __builtin_amdgcn_update_dpp(hi, hi, CTRL, 0xF, 0xF, false);
    return fmin(v, __hiloint2double(hi2, lo2));
}

__device__ __forceinline__ double readlane_f64(double v, int l) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), l), hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
    return __hiloint2double(hi, lo);
}

// CH strict-< first-minimum reductions at once (independent -> their latencies overlap).
// Returns, in lane j < CH, node j's argmin (slice index of this call) and minimum.
template <int SPL, int CH>
__device__ __forceinline__ void wta_chunk(const double (&x)[CH][SPL], int lane, int dloc0, int dcall, double& out_min,
                                          int& out_idx) {
    double bv[CH], g[CH];
    int bi[CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) {
        bv[j] = __builtin_huge_val();
        bi[j] = 0x7fffffff;
#pragma unroll
        for (int k = 0; k < SPL; ++k) {
            if (dloc0 + k < dcall && x[j][k] < bv[j]) { bv[j] = x[j][k]; bi[j] = dloc0 + k; }
        }
        g[j] = bv[j];
    }
#pragma unroll
    for (int j = 0; j < CH; ++j) g[j] = dpp_min<0xB1>(g[j]);   // quad_perm [1,0,3,2]
#pragma unroll
    for (int j = 0; j < CH; ++j) g[j] = dpp_min<0x4E>(g[j]);   // quad_perm [2,3,0,1]
#pragma unroll
    for (int j = 0; j < CH; ++j) g[j] = dpp_min<0x141>(g[j]);  // row_half_mirror
#pragma unroll
    for (int j = 0; j < CH; ++j) g[j] = dpp_min<0x140>(g[j]);  // row_mirror
    out_min = 0.0;
    out_idx = 0;
#pragma unroll
    for (int j = 0; j < CH; ++j) {
        const double m = fmin(fmin(readlane_f64(g[j], 0), readlane_f64(g[j], 16)),
                              fmin(readlane_f64(g[j], 32), readlane_f64(g[j], 48)));
        const unsigned long long ball = __ballot(bv[j] == m && bi[j] != 0x7fffffff);
        const int win = ball ? (int)__builtin_ctzll(ball) : 0;
        const int gi = ball ? __builtin_amdgcn_readlane(bi[j], win) : 0;
        if (lane == j) { out_min = m; out_idx = gi; }
    }
}

template <int SPL, int CH>
__global__ __launch_bounds__(256) void k_down_walk(WalkView V0, WalkView V1, const uint32_t* __restrict__ meta0,
                                                   const uint32_t* __restrict__ meta1, const SmPath* __restrict__ paths0,
                                                   const SmPath* __restrict__ paths1, const float* __restrict__ atab_g,
                                                   const double* __restrict__ slut_g, const double* __restrict__ s2lut_g,
                                                   int Dpad, int dcall, int dglob0, int store_all) {
    __shared__ WalkShared sh;
    load_tables(sh, atab_g, slut_g, s2lut_g);
    const int view = blockIdx.y;
    const WalkView& V = view ? V1 : V0;
    const uint32_t* __restrict__ meta32 = view ? meta1 : meta0;
    const int lane = threadIdx.x & 63;
    const int pi = (int)uniform(blockIdx.x * 4 + (threadIdx.x >> 6));
    if (pi >= V.npaths) return;
    const SmPath path = (view ? paths1 : paths0)[pi];
    const int head = (int)uniform(path.head), len = (int)uniform(path.len);
    const int dloc0 = lane * SPL;
    const uint32_t hparent = uniform(meta32[(size_t)head * 8 + 1]);
    double xc[SPL];
    int c0 = head;
    int n = min(CH, len);
    MetaVec<CH> cur;
    load_meta<CH>(cur, meta32, lane, c0, 1, n);
    bool first = true;
    while (true) {
        const int nc0 = c0 + CH;
        const int nn = nc0 < head + len ? min(CH, head + len - nc0) : 0;
        MetaVec<CH> nxt;
        if (nn > 0) load_meta<CH>(nxt, meta32, lane, nc0, 1, nn);  // prefetch the next chunk's metadata
        // rows of the chunk (contiguous slots) + the parent's A row for the path head
        double u[CH][SPL], xp[SPL];
#pragma unroll
        for (int j = 0; j < CH; ++j)
            if (j < n) load_row<SPL>(V.U, (uint32_t)(c0 + j), Dpad, lane, u[j]);
        if (first && hparent != SM_NONE) load_row<SPL>(V.U, hparent, Dpad, lane, xp);
        double S[CH], S2[CH];
#pragma unroll
        for (int j = 0; j < CH; ++j) {
            const uint32_t wp = lo_wp(mfield(cur, j, 2));
            S[j] = sh.slut[wp];
            S2[j] = sh.s2lut[wp];
        }
        double xs[CH][SPL];
#pragma unroll
        for (int j = 0; j < CH; ++j) {
            if (j < n) {
                const bool is_head = first && j == 0;
                if (is_head) {
                    if (hparent == SM_NONE) {
#pragma unroll
                        for (int k = 0; k < SPL; ++k) xc[k] = u[j][k];  // A(root) = A_up(root)
                    } else {
#pragma unroll
                        for (int k = 0; k < SPL; ++k) xc[k] = __builtin_fma(S[j], xp[k], S2[j] * u[j][k]);
                    }
                } else {
#pragma unroll
                    for (int k = 0; k < SPL; ++k) xc[k] = __builtin_fma(S[j], xc[k], S2[j] * u[j][k]);
                }
                const uint32_t hi = mfield(cur, j, 3);
                if (store_all || (hi_light(hi) && !(is_head && hparent == SM_NONE)))
                    store_row<SPL>(V.U, (uint32_t)(c0 + j), Dpad, lane, xc);
            }
#pragma unroll
            for (int k = 0; k < SPL; ++k) xs[j][k] = xc[k];
        }
        double mn;
        int mi;
        wta_chunk<SPL, CH>(xs, lane, dloc0, dcall, mn, mi);
        if (lane < n) {
            const uint32_t pix = meta32[(size_t)(c0 + lane) * 8];  // lane j stores node j's result
            V.idx[pix] = dglob0 + mi;
            V.minc[pix] = mn;
            V.disp[pix] = (float)(dglob0 + mi);
        }
        if (nn == 0) break;
        cur = nxt;
        c0 = nc0;
        n = nn;
        first = false;
    }
}

// ---------------------------------------------------------------------------------------------
static WalkView to_view(const WalkArgs& a, int v) { return WalkView{a.npaths[v], a.U[v], a.idx[v], a.minc[v], a.disp[v]}; }

template <int SPL, int CH>
static void up_launch(hipStream_t st, dim3 g, const WalkArgs& a) {
    hipLaunchKernelGGL((k_up_walk<SPL, CH>), g, dim3(256), 0, st, to_view(a, 0), to_view(a, 1),
                       reinterpret_cast<const uint32_t*>(a.meta[0]), reinterpret_cast<const uint32_t*>(a.meta[1]),
                       a.paths[0], a.paths[1], a.Lrec, a.Rrec, a.atab, a.slut, a.s2lut, a.W, a.Dpad, a.dcall, a.dglob0);
}

template <int SPL, int CH>
static void down_launch(hipStream_t st, dim3 g, const WalkArgs& a, int store_all) {
    hipLaunchKernelGGL((k_down_walk<SPL, CH>), g, dim3(256), 0, st, to_view(a, 0), to_view(a, 1),
                       reinterpret_cast<const uint32_t*>(a.meta[0]), reinterpret_cast<const uint32_t*>(a.meta[1]),
                       a.paths[0], a.paths[1], a.atab, a.slut, a.s2lut, a.Dpad, a.dcall, a.dglob0, store_all);
}

hipError_t launch_up(hipStream_t st, const WalkArgs& a, int spl, bool long_paths) {
    const int np = a.npaths[0] > a.npaths[1] ? a.npaths[0] : a.npaths[1];
    if (np == 0) return hipSuccess;
    const dim3 g((np + 3) / 4, 2);
    if (long_paths) {
        switch (spl) {
            case 1: up_launch<1, 8>(st, g, a); break;
            case 2: up_launch<2, 8>(st, g, a); break;
            default: up_launch<4, 4>(st, g, a); break;
        }
    } else {
        switch (spl) {
            case 1: up_launch<1, 4>(st, g, a); break;
            case 2: up_launch<2, 4>(st, g, a); break;
            default: up_launch<4, 2>(st, g, a); break;
        }
    }
    return hipGetLastError();
}

static hipError_t launch_down_impl(hipStream_t st, const WalkArgs& a, int spl, int store_all, bool long_paths) {
    const int np = a.npaths[0] > a.npaths[1] ? a.npaths[0] : a.npaths[1];
    if (np == 0) return hipSuccess;
    const dim3 g((np + 3) / 4, 2);
    if (long_paths) {
        switch (spl) {
            case 1: down_launch<1, 16>(st, g, a, store_all); break;
            case 2: down_launch<2, 16>(st, g, a, store_all); break;
            default: down_launch<4, 8>(st, g, a, store_all); break;
        }
    } else {
        switch (spl) {
            case 1: down_launch<1, 4>(st, g, a, store_all); break;
            case 2: down_launch<2, 4>(st, g, a, store_all); break;
            default: down_launch<4, 4>(st, g, a, store_all); break;
        }
    }
    return hipGetLastError();
}

hipError_t launch_down(hipStream_t st, const WalkArgs& a, int spl, bool long_paths) {
    return launch_down_impl(st, a, spl, 0, long_paths);
}
hipError_t launch_down_debug(hipStream_t st, const WalkArgs& a, int spl, bool long_paths) {
    return launch_down_impl(st, a, spl, 1, long_paths);
}
