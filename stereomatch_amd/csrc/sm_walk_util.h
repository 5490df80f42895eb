// sm_walk_util.h -- device helpers shared by the tree-filter walkers (sm_walk.hip) and the
// long-path chain engine (sm_chain.hip): metadata access, row I/O, the on-the-fly AGD cost, the
// LDS weight tables and the batched strict-< WTA reduction.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sm_common.h"
#include "sm_launch.h"      // UpPreArgs
#include "sm_layout_gpu.h"  // sm_piece_cut

// per-view mutable state; the read-only metadata and path lists are separate __restrict__ kernel
// arguments (kernarg-derived, provably unclobbered)
struct WalkView {
    int npaths;
    double* U;             // [slots][Dpad]: A_up (the up pass writes, the down pass reads)
    int32_t* idx;          // W*H   (down pass)
    double* minc;          // W*H   (down pass)
    float* disp;           // W*H   (down pass)
    double* A;             // [n_has_light][Dpad]: A rows of the down pass for the parents of light
                           // children (row = SmMeta::cslot[3]; a head reads sm_arow(parent word));
                           // separate from U so A_up stays intact (down repair)
    double* Adbg;          // [slots][Dpad]: every node's A row (debug calls, store_all), else unused
};

#define SM_NUM_W 766
#define S_ZERO SM_NUM_W    // LDS S-table entry holding 0.0 (absent children)

__device__ __forceinline__ uint32_t uniform(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ float rgray(uint2 r) { return __uint_as_float(r.y); }

// AGD cost (PatchMatchStereoGPU.cu:1518-1543) from {bgrx, gray} records:
// r0 = right(x), l0 = left(x+d), gr1 = gray(right(x+1)), gl1 = gray(left(x+d+1))
__device__ __forceinline__ float agd_rec(uint2 r0, uint2 l0, float gr1, float gl1, const float* __restrict__ atab) {
    const uint32_t l1 = __builtin_amdgcn_sad_u8(r0.x, l0.x, 0u);  // exact integer colour L1
#ifdef SM_AGD_NO_TABLE
    const float a = 0.11f * fminf((float)((double)(float)l1 * 0.33333333333), 7.0f);
#else
    const float a = atab[l1];
#endif
    float g = rgray(l0) - rgray(r0);
    g = g + (gr1 - gl1);
    const float b = 0.89f * fminf(fabsf(g), 2.0f);
    return a + b;
}

// Rows are Dpad doubles: 64*SPL, or 32 at SPL = 1 for calls of <= 32 slices (a 32-slice shard then
// moves 32 slices of rows, not 64).  At SPL = 1 lanes >= Dpad neither load (they read +0, outside the
// WTA's range) nor store.
template <int SPL>
__device__ __forceinline__ bool row_lane(int lane, int Dpad) {
    if constexpr (SPL == 1) return lane < Dpad;
    return true;
}

template <int SPL>
__device__ __forceinline__ void load_row(const double* __restrict__ U, uint32_t slot, int Dpad, int lane, double (&r)[SPL]) {
    const double* p = U + (size_t)slot * Dpad + lane * SPL;
    if constexpr (SPL == 1) {
        r[0] = lane < Dpad ? p[0] : 0.0;
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
        if (lane < Dpad) p[0] = r[0];
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

// lane j (< CH) gets node j's pixel (word 0) from the lane-distributed metadata, no memory access.
// Call with every lane active: ds_bpermute reads nothing from inactive source lanes.
template <int CH>
__device__ __forceinline__ uint32_t meta_pix_of_lane(const MetaVec<CH>& mv, int lane) {
    const int src = ((lane & 7) << 3) << 2;  // byte address of lane 8*(lane%8)
    uint32_t r = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)mv.w[0]);
#pragma unroll
    for (int q = 1; q < (CH + 7) / 8; ++q) {
        const uint32_t t = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)mv.w[q]);
        r = (lane >> 3) == q ? t : r;
    }
    return r;
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
    double s2lut[SM_NUM_W + 1];  // [SM_NUM_W] = 1.0 (segment mode's virtual edges: S = 0, S2 = 1)
};

__device__ __forceinline__ void load_tables(WalkShared& sh, const float* atab_g, const double* slut_g, const double* s2lut_g) {
    for (int i = threadIdx.x; i <= SM_MAX_W; i += blockDim.x) sh.atab[i] = atab_g[i];
    for (int i = threadIdx.x; i < SM_NUM_W; i += blockDim.x) {
        sh.slut[i] = slut_g[i];
        sh.s2lut[i] = s2lut_g[i];
    }
    if (threadIdx.x == 0) {
        sh.slut[SM_NUM_W] = 0.0;
        sh.s2lut[SM_NUM_W] = 1.0;
    }
    __syncthreads();
}

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

// CH strict-< first-minimum reductions at once (independent -> their latencies overlap), over the
// slices [lo, hi) of this call (slices outside: padding, or a shard's subpixel halo).
// Returns, in lane j < CH, node j's argmin (slice index of this call) and minimum.
template <int SPL, int CH>
__device__ __forceinline__ void wta_chunk(const double (&x)[CH][SPL], int lane, int dloc0, int lo, int hi, double& out_min,
                                          int& out_idx) {
    double bv[CH], g[CH];
    int bi[CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) {
        bv[j] = __builtin_huge_val();
        bi[j] = 0x7fffffff;
#pragma unroll
        for (int k = 0; k < SPL; ++k) {
            const int d = dloc0 + k;
            if (d >= lo && d < hi && x[j][k] < bv[j]) { bv[j] = x[j][k]; bi[j] = d; }
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

// WTA configuration of a down-pass launch: the call computes slices [dglob0, dglob0 + dcall) (local
// 0 ..), the WTA takes local slices [lo, hi); dtot = the total disparity range (subpixel edge rule)
#ifndef SM_WTACFG_DEFINED
#define SM_WTACFG_DEFINED
struct WtaCfg {
    int lo, hi, dglob0, dtot, sub;
};
#endif

// slice k of lane l's row (k and l wave-uniform): every slice is read at lane l and the scalars are
// selected -- a select among the row's registers by a run-time k can be folded into one load at a
// computed index, which puts the whole row array in scratch memory (seen at SPL = 4)
template <int SPL>
__device__ __forceinline__ double readlane_slice(const double (&r)[SPL], int k, int l) {
    double v = readlane_f64(r[0], l);
#pragma unroll
    for (int q = 1; q < SPL; ++q) {
        const double t = readlane_f64(r[q], l);
        v = k == q ? t : v;
    }
    return v;
}

// WTA of CH nodes: lane j < CH gets node j's global index, minimum and float disparity.  With w.sub
// the disparity gets selectDisparity's parabola (PatchMatchStereoGPU.cu:1726-1736) through the
// neighbouring slices' aggregated costs rounded to float (pre / next = 0 at the ends of the total
// range): s = (next - pre) * 0.5f / (next - 2 cur + pre); disp = d - s if |s| < 1, else d.  The
// neighbours sit in other lanes (lane t / SPL, element t % SPL): one readlane each.
template <int SPL, int CH>
__device__ __forceinline__ void wta_nodes(const double (&x)[CH][SPL], int lane, const WtaCfg& w, double& mn, int& gi,
                                          float& disp) {
    int mi;
    wta_chunk<SPL, CH>(x, lane, lane * SPL, w.lo, w.hi, mn, mi);
    gi = w.dglob0 + mi;
    disp = (float)gi;
    if (w.sub) {
#pragma unroll
        for (int j = 0; j < CH; ++j) {
            const int m = __builtin_amdgcn_readlane(mi, j);
            const int g = w.dglob0 + m;
            const float cur = (float)readlane_f64(mn, j);
            float pre = 0.0f, nxt = 0.0f;
            if (g > 0) {
                const int t = m - 1;
                pre = (float)readlane_slice<SPL>(x[j], t % SPL, t / SPL);
            }
            if (g < w.dtot - 1) {
                const int t = m + 1;
                nxt = (float)readlane_slice<SPL>(x[j], t % SPL, t / SPL);
            }
            const float s = (nxt - pre) * 0.5f / (nxt - 2.0f * cur + pre);
            const float dj = fabsf(s) < 1.0f ? (float)g - s : (float)g;
            if (lane == j) disp = dj;
        }
    }
}


// A heavy leaf's slot in U holds its f32 cost row (the first half of the slot; WalkArgs::leaf_cost):
// store_leaf_row writes it, load_leaf_row loads its bits into the registers of a double row, and
// widen_leaf_row turns them into the doubles 0.0 + (double)C the up walker computed.
template <int SPL>
__device__ __forceinline__ void store_leaf_row(double* __restrict__ U, uint32_t slot, int Dpad, int lane, const float (&c)[SPL]) {
    float* p = reinterpret_cast<float*>(U + (size_t)slot * Dpad) + lane * SPL;
    if constexpr (SPL == 1) {
        if (lane < Dpad) p[0] = c[0];
    } else if constexpr (SPL == 2) {
        *reinterpret_cast<float2*>(p) = make_float2(c[0], c[1]);
    } else {
        *reinterpret_cast<float4*>(p) = make_float4(c[0], c[1], c[2], c[3]);
    }
}
template <int SPL>
__device__ __forceinline__ void load_leaf_row(const double* __restrict__ U, uint32_t slot, int Dpad, int lane, double (&r)[SPL]) {
    const float* p = reinterpret_cast<const float*>(U + (size_t)slot * Dpad) + lane * SPL;
    if constexpr (SPL == 1) {
        r[0] = __longlong_as_double((long long)(lane < Dpad ? __float_as_uint(p[0]) : 0u));
    } else if constexpr (SPL == 2) {
        const uint2 t = *reinterpret_cast<const uint2*>(p);
        r[0] = __longlong_as_double((long long)(((unsigned long long)t.y << 32) | t.x));
        r[1] = 0.0;
    } else {
        const uint4 t = *reinterpret_cast<const uint4*>(p);
        r[0] = __longlong_as_double((long long)(((unsigned long long)t.y << 32) | t.x));
        r[1] = __longlong_as_double((long long)(((unsigned long long)t.w << 32) | t.z));
        r[2] = 0.0;
        r[3] = 0.0;
    }
}
template <int SPL>
__device__ __forceinline__ void widen_leaf_row(double (&r)[SPL]) {
    float f[SPL];
#pragma unroll
    for (int q = 0; q < SPL; ++q) {
        const unsigned long long b = (unsigned long long)__double_as_longlong(r[q / 2]);
        f[q] = __uint_as_float((uint32_t)(q & 1 ? b >> 32 : b));
    }
#pragma unroll
    for (int q = 0; q < SPL; ++q) r[q] = 0.0 + (double)f[q];  // the up walker's acc + C
}

// f32 cost row of one slot (this lane's SPL slices): MC-CNN ingest rows, or the chain staging rows
template <int SPL>
__device__ __forceinline__ void load_cost_row(const float* __restrict__ C, uint32_t slot, int Dpad, int lane, float (&c)[SPL]) {
    const float* p = C + (size_t)slot * Dpad + lane * SPL;
    if constexpr (SPL == 1) {
        c[0] = lane < Dpad ? p[0] : 0.0f;
    } else if constexpr (SPL == 2) {
        const float2 t = *reinterpret_cast<const float2*>(p);
        c[0] = t.x;
        c[1] = t.y;
    } else {
        const float4 t = *reinterpret_cast<const float4*>(p);
        c[0] = t.x;
        c[1] = t.y;
        c[2] = t.z;
        c[3] = t.w;
    }
}

// column of pixel index pix: a float estimate of pix / W is off by at most one while pix < 2^24
// (exact in float; W <= 2 exact, W >= 3: |error| <= 2^24/W * 2^-22 < 1), fixed with one compare
// each way -- an integer division costs ~25 VALU per node.  Larger images take the division.
__device__ __forceinline__ int pix_col(int pix, int W) {
    if (pix >= (1 << 24)) return pix % W;
    const int y = (int)((float)pix * __builtin_amdgcn_rcpf((float)W));
    int x = pix - y * W;
    x = x < 0 ? x + W : x;
    x = x >= W ? x - W : x;
    return x;
}

// image records of CH path nodes: own(x), own(x+1) of all CH nodes in ONE lane-distributed load
// (lane j: node j's x, lane 32 + j: its x+1; one VMEM instruction instead of CH) and the SPL+1
// matched-image records a lane needs per node (of the last one only its gray word).  All loads are
// unconditional (rows of absent nodes are clamped to the last valid one) and nothing reads the
// loaded values here, so a chunk's loads are all in flight before the first wait.
template <int SPL, int CH>
struct ImgRecs {
    uint2 ob[CH][SPL], own;
    float obg[CH];  // gray of the matched record after the last one (only its gray is used)
};

template <int SPL, int CH>
__device__ __forceinline__ void load_recs(const MetaVec<CH>& mv, int n, int view, int lane, int W, int dbase,
                                          const uint2* __restrict__ own, const uint2* __restrict__ oth, ImgRecs<SPL, CH>& r) {
    static_assert(CH <= 32, "own records: lanes j and 32 + j hold node j");
    {
        // lane l: node min(l & 31, n - 1), by selects over the uniform pixels (a ds_bpermute would
        // queue the address behind LDS traffic, heavy in the chain helpers); x+1 == W reads the
        // next row / the pad: masked in chunk_costs
        const int node = min(lane & 31, n - 1);
        uint32_t pl = mfield(mv, 0, 0);
#pragma unroll
        for (int j = 1; j < CH; ++j) pl = node == j ? mfield(mv, j, 0) : pl;
#ifdef SM_EXP_NO_OWN  // timing experiment only (wrong results): no own-record loads
        r.own = make_uint2(pl, (uint32_t)lane);
#else
        r.own = own[(long long)pl + (lane >> 5)];
#endif
    }
#pragma unroll
    for (int j = 0; j < CH; ++j) {
        const int jj = j < n ? j : n - 1;
        const long long pix = (long long)mfield(mv, jj, 0);  // = y*W + x: no division needed here
        const long long base = view ? pix + dbase : pix - dbase - (SPL - 1);
#pragma unroll
        for (int q = 0; q < SPL; ++q) r.ob[j][q] = oth[base + q];
        r.obg[j] = __uint_as_float(reinterpret_cast<const uint32_t*>(oth + base + SPL)[1]);
    }
}

// The up walker's 4-byte records: bgrx alone, the gray recomputed as k_prep computes it
// (sm_kernels.hip sm_gray: 0.114f*B + 0.587f*G + 0.299f*R, left to right, no contraction), so the
// costs are bit-identical.  Per node a lane loads SPL + 1 dwords instead of SPL {bgrx, gray}
// pairs and one gray word: 0.5 KB instead of 1.3 KB per node through L1 / L2 / the Infinity Cache.
__device__ __forceinline__ float gray4(uint32_t bgrx) {
    const float b = (float)(bgrx & 255u), g = (float)((bgrx >> 8) & 255u), r = (float)((bgrx >> 16) & 255u);
    float t = 0.114f * b;
    t = t + 0.587f * g;
    t = t + 0.299f * r;
    return t;
}
// agd_rec with the grays given: r0 = right(x), l0 = left(x+d) (bgrx), their grays gr0 / gl0, and
// gr1 = gray(right(x+1)), gl1 = gray(left(x+d+1)); same operations in the same order
__device__ __forceinline__ float agd4(uint32_t r0, uint32_t l0, float gr0, float gl0, float gr1, float gl1,
                                      const float* __restrict__ atab) {
    const uint32_t l1 = __builtin_amdgcn_sad_u8(r0, l0, 0u);
#ifdef SM_AGD_NO_TABLE
    const float a = 0.11f * fminf((float)((double)(float)l1 * 0.33333333333), 7.0f);
#else
    const float a = atab[l1];
#endif
    float g = gl0 - gr0;
    g = g + (gr1 - gl1);
    const float b = 0.89f * fminf(fabsf(g), 2.0f);
    return a + b;
}

template <int SPL, int CH>
struct ImgRecs4 {
    uint32_t ob[CH][SPL + 1];  // matched-image bgrx, records base .. base + SPL
    uint2 own;
};

template <int SPL, int CH>
__device__ __forceinline__ void load_recs4(const MetaVec<CH>& mv, int n, int view, int lane, int dbase,
                                           const uint2* __restrict__ own, const uint32_t* __restrict__ oth,
                                           ImgRecs4<SPL, CH>& r) {
    static_assert(CH <= 32, "own records: lanes j and 32 + j hold node j");
    {
        const int node = min(lane & 31, n - 1);
        uint32_t pl = mfield(mv, 0, 0);
#pragma unroll
        for (int j = 1; j < CH; ++j) pl = node == j ? mfield(mv, j, 0) : pl;
        r.own = own[(long long)pl + (lane >> 5)];
    }
#pragma unroll
    for (int j = 0; j < CH; ++j) {
        const int jj = j < n ? j : n - 1;
        const long long pix = (long long)mfield(mv, jj, 0);
        const long long base = view ? pix + dbase : pix - dbase - (SPL - 1);
#pragma unroll
        for (int q = 0; q <= SPL; ++q) r.ob[j][q] = oth[base + q];
    }
}

template <int SPL, int CH, class T>
__device__ __forceinline__ void chunk_costs4(const MetaVec<CH>& mv, int view, int W, int dbase, int dend,
                                             const ImgRecs4<SPL, CH>& r, const float* __restrict__ atab, T (&c)[CH][SPL]) {
#pragma unroll
    for (int j = 0; j < CH; ++j) {
        const int x = pix_col((int)mfield(mv, j, 0), W);
        const uint2 o0 = make_uint2(__builtin_amdgcn_readlane(r.own.x, j), __builtin_amdgcn_readlane(r.own.y, j));
        const uint2 o1 = make_uint2(__builtin_amdgcn_readlane(r.own.x, 32 + j), __builtin_amdgcn_readlane(r.own.y, 32 + j));
        float g[SPL + 1];
#pragma unroll
        for (int q = 0; q <= SPL; ++q) g[q] = gray4(r.ob[j][q]);
#pragma unroll
        for (int k = 0; k < SPL; ++k) {
            const int d = dbase + k;
            float v;
            bool ok;
            if (view) {  // right reference: right(x) vs left(x+d)
                ok = d < dend && x + d + 1 < W;
                v = agd4(o0.x, r.ob[j][k], rgray(o0), g[k], rgray(o1), g[k + 1], atab);
            } else {     // left pixel x at d: cost(x-d, d); x-d<0 and column W-1 -> 3.0
                ok = d < dend && x - d >= 0 && x + 1 < W;
                v = agd4(r.ob[j][SPL - 1 - k], o0.x, g[SPL - 1 - k], rgray(o0), g[SPL - k], rgray(o1), atab);
            }
            c[j][k] = (T)(ok ? v : 3.0f);
        }
    }
}

// AGD costs C(v, d) of the chunk's nodes for this lane's SPL slices; invalid (x-d<0, column W-1,
// d beyond the call's range) -> 3.0 as the reference (PatchMatchStereoGPU.cu:1501-1549)
template <int SPL, int CH, class T>
__device__ __forceinline__ void chunk_costs(const MetaVec<CH>& mv, int view, int W, int dbase, int dend,
                                            const ImgRecs<SPL, CH>& r, const float* __restrict__ atab, T (&c)[CH][SPL]) {
#pragma unroll
    for (int j = 0; j < CH; ++j) {
        const int x = pix_col((int)mfield(mv, j, 0), W);
        const uint2 o0 = make_uint2(__builtin_amdgcn_readlane(r.own.x, j), __builtin_amdgcn_readlane(r.own.y, j));
        const uint2 o1 = make_uint2(__builtin_amdgcn_readlane(r.own.x, 32 + j), __builtin_amdgcn_readlane(r.own.y, 32 + j));
#pragma unroll
        for (int k = 0; k < SPL; ++k) {
            const int d = dbase + k;
            float v;
            bool ok;
            if (view) {  // right reference: right(x) vs left(x+d)
                ok = d < dend && x + d + 1 < W;
                v = agd_rec(o0, r.ob[j][k], rgray(o1), k + 1 < SPL ? rgray(r.ob[j][k + 1 < SPL ? k + 1 : 0]) : r.obg[j], atab);
            } else {     // left pixel x at d: cost(x-d, d); x-d<0 and column W-1 -> 3.0
                ok = d < dend && x - d >= 0 && x + 1 < W;
                v = agd_rec(r.ob[j][SPL - 1 - k], o0, k > 0 ? rgray(r.ob[j][k > 0 ? SPL - k : 0]) : r.obg[j], rgray(o1), atab);
            }
#ifdef SM_EXP_COST_CHEAP  // timing experiment only (wrong results): the records' loads, trivial arithmetic
            v = rgray(r.ob[j][k]) + rgray(o0) + r.obg[j] + rgray(o1);
            ok = true;
#endif
            c[j][k] = (T)(ok ? v : 3.0f);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Segment aggregates of the up pass (the pieces' guessed inputs, sm_chain.hip "Pieces"): the
// affine map x_first = P * x_below + B of one SM_PRE_SEG-node segment of a cut long path, with
// b = Pre + sum(S_post * A_post) + C per node and x = S_heavy * x_below + b.  Approximate (any
// rounding only moves a guess; the chains' results are repaired exactly).  Four waves of
// CH * NSUB nodes each; run by k_up_pre or by the extra blocks of the round's fused walker launch.
// ---------------------------------------------------------------------------------------------

// scratch: >= 6 * 64 doubles of LDS (the up pass's idle s2lut table)
template <int SPL, int CH, int NSUB, bool VOL>
__device__ __forceinline__ void up_pre_segment(const UpPreArgs& pa, int view, int sidx, const double* __restrict__ U,
                                               const uint32_t* __restrict__ meta32, const float* __restrict__ Cst,
                                               const uint2* __restrict__ own, const uint2* __restrict__ oth, int W, int Dpad,
                                               int dcall, int dglob0, const WalkShared& sh, double* scratch, int lane, int wv) {
    static_assert(CH * NSUB * 4 == SM_PRE_SEG, "four waves per segment");
    const uint2 sg = pa.seg[view][sidx];
    const SmPath path = pa.paths[view][uniform(sg.x)];
    const int head = (int)uniform(path.head), len = (int)uniform(path.len);
    double* __restrict__ agg = pa.agg[view];
    if (agg == nullptr || !sm_piece_cut((uint32_t)len, (uint32_t)pa.plen[view])) return;  // uniform over the block
    const int dbase = dglob0 + lane * SPL;
    const int dend = dglob0 + dcall;
    double P[SPL], B[SPL];
#pragma unroll
    for (int k = 0; k < SPL; ++k) {
        P[k] = 1.0;
        B[k] = 0.0;
    }
#pragma unroll
    for (int s = NSUB - 1; s >= 0; --s) {  // bottom-most nodes first
        const int first = (int)uniform(sg.y * SM_PRE_SEG + (wv * NSUB + s) * CH);
        const int n = max(0, min(CH, len - first));
        if (n == 0) continue;  // uniform
        MetaVec<CH> mv;
        load_meta<CH>(mv, meta32, lane, head + first, 1, n);
        float c[CH][SPL];
        if constexpr (VOL) {
#pragma unroll
            for (int j = 0; j < CH; ++j) load_cost_row<SPL>(Cst, (uint32_t)(head + first + (j < n ? j : n - 1)), Dpad, lane, c[j]);
        } else {
            ImgRecs<SPL, CH> rec;
            load_recs<SPL, CH>(mv, n, view, lane, W, dbase, own, oth, rec);
            chunk_costs<SPL, CH>(mv, view, W, dbase, dend, rec, sh.atab, c);
        }
#pragma unroll
        for (int j = CH - 1; j >= 0; --j) {
            if (j < n) {
                const uint32_t lo = mfield(mv, j, 2), hi = mfield(mv, j, 3);
                const uint32_t nch = hi_nch(hi), hidx = hi_hidx(hi);
                const double Sh = nch > 0 ? readlane_f64(sh.slut[cw_of(lo, hi, (int)hidx)], 0) : 0.0;
                double b[SPL];
#pragma unroll
                for (int k = 0; k < SPL; ++k) b[k] = 0.0;
#pragma unroll
                for (int i = 0; i < 4; ++i) {  // every light child, in key order (rows loaded where used)
                    if ((uint32_t)i < nch && (uint32_t)i != hidx) {
                        const double S = readlane_f64(sh.slut[cw_of(lo, hi, i)], 0);
                        double r[SPL];
                        load_row<SPL>(U, mfield(mv, j, 4 + i), Dpad, lane, r);
#pragma unroll
                        for (int k = 0; k < SPL; ++k) b[k] = __builtin_fma(S, r[k], b[k]);
                    }
                }
#pragma unroll
                for (int k = 0; k < SPL; ++k) {
                    B[k] = __builtin_fma(Sh, B[k], b[k] + (double)c[j][k]);
                    P[k] = Sh * P[k];
                }
            }
        }
    }
    // segment = wave 0 o wave 1 o wave 2 o wave 3 (wave 3 holds the bottom-most nodes), one slice
    // column at a time through the scratch
    double* out = agg + (size_t)sidx * 2 * Dpad;  // segment index within the bucket
#pragma unroll
    for (int k = 0; k < SPL; ++k) {
        if (wv > 0) {
            scratch[(wv - 1) * 128 + lane] = P[k];
            scratch[(wv - 1) * 128 + 64 + lane] = B[k];
        }
        __syncthreads();
        if (wv == 0) {
            double Pr = scratch[2 * 128 + lane], Br = scratch[2 * 128 + 64 + lane];  // wave 3
#pragma unroll
            for (int w = 2; w >= 1; --w) {
                const double Pw = scratch[(w - 1) * 128 + lane], Bw = scratch[(w - 1) * 128 + 64 + lane];
                Br = __builtin_fma(Pw, Br, Bw);
                Pr = Pw * Pr;
            }
            Br = __builtin_fma(P[k], Br, B[k]);
            Pr = P[k] * Pr;
            if (row_lane<SPL>(lane, Dpad)) {
                out[lane * SPL + k] = Pr;
                out[Dpad + lane * SPL + k] = Br;
            }
        }
        __syncthreads();
    }
}
