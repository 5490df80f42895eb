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
#include "sm_walk_util.h"
#include "sm_knob.h"

// segment blocks of the fused up launch (up_pre_segment): 4 waves x CH x NSUB nodes
#define UP_PRE_CH(SPL) ((SPL) == 4 ? 4 : 8)
#define UP_PRE_NSUB(SPL) ((SPL) == 4 ? 2 : 1)
// paths per wave work item (a bucket's paths occupy consecutive slots: one contiguous range)
#ifndef WALK_PPW_UP
#define WALK_PPW_UP 6
#endif
#ifndef WALK_PPW_DN
#define WALK_PPW_DN 4
#endif
// chunk sizes (nodes per software-pipeline stage) of the short-path walkers, per SPL
#ifndef WALK_UP_CH2
#define WALK_UP_CH2 3
#endif
#ifndef WALK_UP_CH4
#define WALK_UP_CH4 3
#endif
#ifndef WALK_DN_CH4
#define WALK_DN_CH4 4
#endif
#ifndef WALK_DN_CH2
#define WALK_DN_CH2 4  // round 5: 6 -> 4 (81 -> 64 VGPRs, 5 -> 8 waves per SIMD): the same kernel time one
                       // frame at a time, C2 4.37 -> 4.30 ms/frame with frames in flight (5: 7 waves, 4.30-4.34)
#endif
#ifndef WALK_UP_CH1
#define WALK_UP_CH1 4
#endif
#ifndef WALK_DN_CH1
#define WALK_DN_CH1 4
#endif


// One explicit vmcnt(0) per chunk, right after the chunk's loads (rows, image records, next
// metadata) are issued.  gfx9 counts loads and stores in one counter and the compiler treats
// their completion as unordered: any wait for a load while a store is pending becomes vmcnt(0).
// Letting the compiler place the waits put such full waits behind the chunk's own stores (and
// behind a metadata prefetch issued first), i.e. two memory latencies per chunk.  Draining here
// costs one: the previous chunk's stores were issued a whole chunk earlier.
__device__ __forceinline__ void walk_vm_drain() {
#ifndef SM_WALK_NO_DRAIN
    __builtin_amdgcn_s_waitcnt(0x0F70);
#endif
}

// ---------------------------------------------------------------------------------------------
// up pass
// ---------------------------------------------------------------------------------------------
// Light-child rows of a chunk are compacted: the chunk's light children, in node order and key
// order within a node, take row registers 0 .. LR-1 (wave-uniform bookkeeping from the metadata).
// ~75% of nodes have none, so LR = 2 register rows cover almost every chunk; the rest (and a
// tree root's third light child) are loaded where the recurrence uses them.  Holding CH x 2 rows
// instead cost 16 VGPRs at SPL = 2, i.e. two of eight waves per SIMD.
#ifndef WALK_UP_LR
#define WALK_UP_LR 2
#endif
// VOL: the costs are caller-supplied volume rows (MC-CNN ingest, k_vol_rows) instead of the AGD
// cost computed from the image records
template <int SPL, int CH, bool VOL>
__device__ __forceinline__ void up_chunk(const MetaVec<CH>& mv, int n, int top, int view, int lane, int W, int Dpad,
                                         int dbase, int dend, const uint2* __restrict__ own, const uint2* __restrict__ oth,
                                         const uint32_t* __restrict__ oth4, double* __restrict__ U, const float* __restrict__ Cv, const WalkShared& sh,
                                         double (&xc)[SPL], MetaVec<CH>& nxt, const uint32_t* __restrict__ meta32, int ntop,
                                         int nn, int leaf_cost) {
    constexpr int LR = WALK_UP_LR;
    // ---- light-row bookkeeping (uniform): node j's light children are compact rows off[j] ..
    int off[CH];
    int tot = 0;
#pragma unroll
    for (int j = 0; j < CH; ++j) {
        const uint32_t nch = j < n ? hi_nch(mfield(mv, j, 3)) : 0u;
        off[j] = tot;
        tot += nch > 0 ? (int)nch - 1 : 0;
    }
    // ---- all vector loads of the chunk
    double lr[LR][SPL];
#pragma unroll
    for (int q = 0; q < LR; ++q) {
#ifdef SM_EXP_UP_NO_LIGHT  // timing experiment only (wrong results): no light-child row loads
        if (false) {
#else
        if (q < tot) {  // wave-uniform: only present rows travel through L1
#endif
            // the node j and light index kk of compact row q
            int jq = 0;
#pragma unroll
            for (int j = 1; j < CH; ++j) jq = off[j] <= q ? j : jq;
            const uint32_t hidx = hi_hidx(mfield(mv, jq, 3));
            const int kk = q - off[jq];
            const int pos = kk + (kk >= (int)hidx ? 1 : 0);
            load_row<SPL>(U, mfield(mv, jq, 4 + min(pos, 3)), Dpad, lane, lr[q]);
        } else {
#pragma unroll
            for (int k = 0; k < SPL; ++k) lr[q][k] = 0.0;
        }
    }
    // ---- off-chain work: costs and edge factors of every node of the chunk
    float c[CH][SPL];  // float until the add: half the registers of the converted values
    double Sv[CH][4];
    if constexpr (VOL) {
#pragma unroll
        for (int j = 0; j < CH; ++j) load_cost_row<SPL>(Cv, (uint32_t)(top - (j < n ? j : n - 1)), Dpad, lane, c[j]);
        if (nn > 0) load_meta<CH>(nxt, meta32, lane, ntop, -1, nn);
        walk_vm_drain();
    } else {
#ifdef SM_EXP_UP_NO_COST  // timing experiment only (wrong results): no image records, constant cost
        if (nn > 0) load_meta<CH>(nxt, meta32, lane, ntop, -1, nn);
        walk_vm_drain();
#pragma unroll
        for (int j = 0; j < CH; ++j)
#pragma unroll
            for (int k = 0; k < SPL; ++k) c[j][k] = 0.25f;
#elif defined(SM_WALK_REC8)  // A/B: {bgrx, gray} records (2.5x the record bytes)
        (void)oth4;
        ImgRecs<SPL, CH> rec;
        load_recs<SPL, CH>(mv, n, view, lane, W, dbase, own, oth, rec);
        if (nn > 0) load_meta<CH>(nxt, meta32, lane, ntop, -1, nn);
        walk_vm_drain();
        chunk_costs<SPL, CH>(mv, view, W, dbase, dend, rec, sh.atab, c);
#else
        (void)oth;
        ImgRecs4<SPL, CH> rec;
        load_recs4<SPL, CH>(mv, n, view, lane, dbase, own, oth4, rec);
        // the next chunk's metadata, issued behind this chunk's loads: it completes with them, so
        // the next chunk starts without a wait (a prefetch issued first made the chunk's first
        // wait a vmcnt(0) over the prefetch and the previous chunk's stores)
        if (nn > 0) load_meta<CH>(nxt, meta32, lane, ntop, -1, nn);
        walk_vm_drain();
        chunk_costs4<SPL, CH>(mv, view, W, dbase, dend, rec, sh.atab, c);
#endif
    }
#pragma unroll
    for (int j = 0; j < CH; ++j) {
        const uint32_t lo = mfield(mv, j, 2), hi = mfield(mv, j, 3);
        const uint32_t nch = hi_nch(hi);
#pragma unroll
        for (int i = 0; i < 4; ++i)  // uniform: SGPR pairs (v_fma_f64 takes one), not 2 VGPRs each
#ifdef SM_WALK_SV_VGPR
            Sv[j][i] = sh.slut[(uint32_t)i < nch ? cw_of(lo, hi, i) : (uint32_t)S_ZERO];
#else
            Sv[j][i] = readlane_f64(sh.slut[(uint32_t)i < nch ? cw_of(lo, hi, i) : (uint32_t)S_ZERO], 0);
#endif
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
                        const int q = off[j] + (int)i - (i > hidx ? 1 : 0);  // compact light row
                        bool held = false;
#pragma unroll
                        for (int r = 0; r < LR; ++r) {
                            if (q == r) {
#pragma unroll
                                for (int k = 0; k < SPL; ++k) v[k] = lr[r][k];
                                held = true;
                            }
                        }
                        if (!held) load_row<SPL>(U, mfield(mv, j, 4 + (int)i), Dpad, lane, v);  // rare: loaded here
                    }
#pragma unroll
                    for (int k = 0; k < SPL; ++k) acc[k] = __builtin_fma(Sv[j][i], v[k], acc[k]);
                }
            }
#pragma unroll
            for (int k = 0; k < SPL; ++k) xc[k] = acc[k] + (double)c[j][k];
#ifdef SM_EXP_UP_HEADS_ONLY  // timing experiment only (wrong results): store path heads' rows only
            if (mfield(mv, j, 1) != (uint32_t)(top - j) - 1u)
#endif
            // a heavy leaf (no children, its parent the previous slot): only the down walker reads its
            // row, and its A_up is exactly (double)C: the f32 cost row, half the bytes
            // (WalkArgs::leaf_cost)
            const uint32_t par = mfield(mv, j, 1);
            if (leaf_cost && nch == 0 && par != SM_NONE && par == (uint32_t)(top - j) - 1u)
                store_leaf_row<SPL>(U, (uint32_t)(top - j), Dpad, lane, c[j]);
            else
                store_row<SPL>(U, (uint32_t)(top - j), Dpad, lane, xc);
        }
    }
}

template <int SPL, int CH, bool VOL>
__global__ __launch_bounds__(256) void k_up_walk(WalkView V0, WalkView V1, const uint32_t* __restrict__ meta0,
                                                 const uint32_t* __restrict__ meta1, const SmPath* __restrict__ paths0,
                                                 const SmPath* __restrict__ paths1, const uint2* __restrict__ Lrec,
                                                 const uint2* __restrict__ Rrec, const uint32_t* __restrict__ Lrec4,
                                                 const uint32_t* __restrict__ Rrec4, const float* __restrict__ atab_g,
                                                 const double* __restrict__ slut_g, const double* __restrict__ s2lut_g,
                                                 int W, int Dpad, int dcall, int dglob0, const float* __restrict__ Cv0,
                                                 const float* __restrict__ Cv1, int ppw, int leaf_cost, UpPreArgs pa) {
    // issue priority 1 (chain waves run at 3, everything else at 0): where a walker wave shares a SIMD
    // with another frame's tree-stage waves, the filter's latency chains issue first.  Round 5, C2, 7
    // interleaved pairs: 4.288 -> 4.257 ms/frame (priority 2: no gain); profiles/r05/walk_prio/
    __builtin_amdgcn_s_setprio(1);
    __shared__ WalkShared sh;
    load_tables(sh, atab_g, slut_g, s2lut_g);
    const int view = blockIdx.y;
    const WalkView& V = view ? V1 : V0;
    const uint32_t* __restrict__ meta32 = view ? meta1 : meta0;
    const int lane = threadIdx.x & 63;
#ifdef SM_PRE_FUSED  // A/B (sm_api.cpp up_round): the round's segment aggregates as extra blocks
    if ((int)blockIdx.x >= pa.walk_blocks) {  // uniform: a segment of the round's cut long paths
        const int sidx = (int)blockIdx.x - pa.walk_blocks;
        if (sidx < pa.nseg[view])
            up_pre_segment<SPL, UP_PRE_CH(SPL), UP_PRE_NSUB(SPL), VOL>(
                pa, view, sidx, V.U, meta32, view ? Cv1 : Cv0, view ? Rrec : Lrec, view ? Lrec : Rrec, W, Dpad, dcall,
                dglob0, sh, sh.s2lut, lane, (int)uniform(threadIdx.x >> 6));  // s2lut: unused by the up pass
        return;
    }
#else
    (void)pa;
#endif
    // work item: ppw consecutive paths of the bucket = one contiguous slot range (the recurrence
    // restarts by itself at every path bottom: a leaf has no heavy child)
    const int pi0 = (int)uniform((blockIdx.x * 4 + (threadIdx.x >> 6)) * ppw);
    if (pi0 >= V.npaths) return;
    const int pi1 = min(pi0 + ppw, V.npaths);
    const SmPath* __restrict__ pp = view ? paths1 : paths0;
    const int head = (int)uniform(pp[pi0].head);
    const int len = (int)uniform(pp[pi1 - 1].head + pp[pi1 - 1].len) - head;
    const int dbase = dglob0 + lane * SPL;  // global disparity of this lane's first slice
    const int dend = dglob0 + dcall;
    const uint2* __restrict__ own = view ? Rrec : Lrec;  // the view's reference image
    const uint2* __restrict__ oth = view ? Lrec : Rrec;  // the matched image
    const uint32_t* __restrict__ oth4 = view ? Lrec4 : Rrec4;
    double xc[SPL];
#pragma unroll
    for (int k = 0; k < SPL; ++k) xc[k] = 0.0;
    // chunk c covers nodes top_c, top_c-1, ... (bottom of the path first)
    int top = head + len - 1;
    int n = min(CH, top - head + 1);
    MetaVec<CH> cur;
    load_meta<CH>(cur, meta32, lane, top, -1, n);
    walk_vm_drain();  // nothing pending on loop entry: the loop top then needs no wait at all
    while (true) {
        const int ntop = top - CH;
        const int nn = ntop >= head ? min(CH, ntop - head + 1) : 0;
        MetaVec<CH> nxt;  // the next chunk's metadata: loaded inside up_chunk
        const float* __restrict__ Cv = view ? Cv1 : Cv0;
        up_chunk<SPL, CH, VOL>(cur, n, top, view, lane, W, Dpad, dbase, dend, own, oth, oth4, V.U, Cv, sh, xc, nxt, meta32, ntop, nn,
                               VOL ? 0 : leaf_cost);
        if (nn == 0) break;
        cur = nxt;
        top = ntop;
        n = nn;
    }
}

// ---------------------------------------------------------------------------------------------
// Half-wave walkers (SPL = 1 calls with 64-double rows, e.g. a 64-slice view-group shard at N = 8).
// At SPL = 1 a node step costs a wave the same instructions as at SPL = 2: the per-node metadata,
// LUT and branch work does not shrink with the slices.  Here each half-wave of 32 lanes walks its
// own work item with 2 slices per lane, i.e. two paths per wave-step.  Values the full-wave
// walkers keep wave-uniform are per half (two readlanes and a select, or a ds_bpermute); rows are
// the same [slot][64] rows (lane l of a half holds slices 2(l%32), 2(l%32)+1) and the arithmetic
// is the full-wave walkers' exactly.  A half whose item is finished (or empty) re-reads its last
// chunk and stores nothing.  Metadata: lane 32h + 8j + f holds word f of half h's node j.
// ---------------------------------------------------------------------------------------------
template <int CH>
__device__ __forceinline__ uint32_t hfield(uint32_t w, int hl, int j, int f) {
    const uint32_t a = __builtin_amdgcn_readlane(w, 8 * j + f), b = __builtin_amdgcn_readlane(w, 32 + 8 * j + f);
    return hl ? b : a;
}
// word f of node j of this lane's half, j and f per lane (call with every lane active)
__device__ __forceinline__ uint32_t hfield_v(uint32_t w, int hl, int j, int f) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute(((hl << 5) + 8 * j + f) << 2, (int)w);
}

#ifndef WALK_UP_CHH
#define WALK_UP_CHH 2  // round 5: 3 -> 2 (76 -> 72 VGPRs, 6 -> 7 waves per SIMD), with WALK_DN_CHH 4 -> 3
                       // (5 -> 7): the N = 8 share 2.009-2.016 -> 1.967-1.987 ms/frame
#endif
#ifndef WALK_UP_CHH1
#define WALK_UP_CHH1 2  // 32-slice rows (1 slice per half-lane)
#endif

template <int CH, int SH>
__device__ __forceinline__ void up_chunk_h2(uint32_t mv, int n, int top, int view, int lane, int W, int dbase, int dend,
                                            const uint2* __restrict__ own, const uint32_t* __restrict__ oth4,
                                            double* __restrict__ U, const WalkShared& sh, double (&xc)[SH], uint32_t& nxt,
                                            const uint32_t* __restrict__ meta32, int mtop, int mn, int leaf_cost) {
    static_assert(CH <= 4, "lane 32h + 8j + f holds word f of half h's node j");
    constexpr int LR = WALK_UP_LR;
    constexpr int DP = 32 * SH;  // row length: 64 doubles (2 slices per half-lane) or 32 (1)
    const int hl = lane >> 5, hlane = lane & 31;
    const int nv = n > 0 ? n : 1;  // rows / records of a finished half: its chunk's first node
    // ---- light-row bookkeeping (per half): node j's light children are compact rows off[j] ..
    int off[CH];
    int tot = 0;
#pragma unroll
    for (int j = 0; j < CH; ++j) {
        const uint32_t nch = j < n ? hi_nch(hfield<CH>(mv, hl, j, 3)) : 0u;
        off[j] = tot;
        tot += nch > 0 ? (int)nch - 1 : 0;
    }
    double lr[LR][SH];
#pragma unroll
    for (int q = 0; q < LR; ++q) {
        int jq = 0, oq = off[0];
#pragma unroll
        for (int j = 1; j < CH; ++j) {
            jq = off[j] <= q ? j : jq;
            oq = off[j] <= q ? off[j] : oq;
        }
        const uint32_t hidx = hi_hidx(hfield_v(mv, hl, jq, 3));
        const int kk = q - oq;
        const int pos = kk + (kk >= (int)hidx ? 1 : 0);
        const uint32_t slot = hfield_v(mv, hl, jq, 4 + min(max(pos, 0), 3));
        if (q < tot) {
            load_row<SH>(U, slot, DP, hlane, lr[q]);
        } else {
#pragma unroll
            for (int k = 0; k < SH; ++k) lr[q][k] = 0.0;
        }
    }
    // ---- image records: lane 32h + i (i < 16) own(x) of node min(i, n-1), lane 32h + 16 + i own(x+1)
    uint2 ownr;
    {
        const int node = min(hlane & 15, nv - 1);
        uint32_t pl = hfield<CH>(mv, hl, 0, 0);
#pragma unroll
        for (int j = 1; j < CH; ++j) pl = node == j ? hfield<CH>(mv, hl, j, 0) : pl;
        ownr = own[(long long)pl + (hlane >> 4)];
    }
    // matched-image records x + dbase .. x + dbase + SH (right view) or x - dbase - (SH - 1) .. x - dbase + 1
    // (left view): slice k reads records q = k, k + 1 (right) or SH - 1 - k, SH - k (left)
    uint32_t ob[CH][SH + 1];
#pragma unroll
    for (int j = 0; j < CH; ++j) {
        // node j >= n: its metadata lanes already hold node n - 1's words (clamped load); the
        // readlane index must stay uniform
        const long long pix = (long long)hfield<CH>(mv, hl, j, 0);
        const long long base = view ? pix + dbase : pix - dbase - (SH - 1);
#pragma unroll
        for (int q = 0; q <= SH; ++q) ob[j][q] = oth4[base + q];
    }
    nxt = meta32[(size_t)(mtop - min(hlane >> 3, mn - 1)) * 8 + (lane & 7)];
    walk_vm_drain();
    // ---- costs (chunk_costs4 at SPL = SH, per half) and edge factors
    float c[CH][SH];
#pragma unroll
    for (int j = 0; j < CH; ++j) {
        const int x = pix_col((int)hfield<CH>(mv, hl, j, 0), W);
        // own(x) of node j at lane 32h + j, own(x+1) (only its gray) at lane 32h + 16 + j
        const uint32_t ox0 = hfield<CH>(ownr.x, hl, 0, j), oy0 = hfield<CH>(ownr.y, hl, 0, j);
        const uint32_t oy1 = hfield<CH>(ownr.y, hl, 2, j);
        const float go0 = __uint_as_float(oy0), go1 = __uint_as_float(oy1);
        float g[SH + 1];
#pragma unroll
        for (int q = 0; q <= SH; ++q) g[q] = gray4(ob[j][q]);
#pragma unroll
        for (int k = 0; k < SH; ++k) {
            const int d = dbase + k;
            float v;
            bool ok;
            if (view) {
                ok = d < dend && x + d + 1 < W;
                v = agd4(ox0, ob[j][k], go0, g[k], go1, g[k + 1], sh.atab);
            } else {
                ok = d < dend && x - d >= 0 && x + 1 < W;
                v = agd4(ob[j][SH - 1 - k], ox0, g[SH - 1 - k], go0, g[SH - k], go1, sh.atab);
            }
            c[j][k] = ok ? v : 3.0f;
        }
    }
    // edge factors of the first two children up front (per lane: LDS reads); a third or fourth
    // child (rare) reads its factor where the recurrence uses it
    double Sv[CH][2];
#pragma unroll
    for (int j = 0; j < CH; ++j) {
        const uint32_t lo = hfield<CH>(mv, hl, j, 2), hi = hfield<CH>(mv, hl, j, 3);
        const uint32_t nch = hi_nch(hi);
#pragma unroll
        for (int i = 0; i < 2; ++i) Sv[j][i] = sh.slut[(uint32_t)i < nch ? cw_of(lo, hi, i) : (uint32_t)S_ZERO];
    }
    // ---- serial recurrence along the path (bottom -> top)
#pragma unroll
    for (int j = 0; j < CH; ++j) {
        const uint32_t hi = hfield<CH>(mv, hl, j, 3);
        const uint32_t par = hfield<CH>(mv, hl, j, 1);
        uint32_t cs[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) cs[i] = hfield<CH>(mv, hl, j, 4 + i);
        if (j < n) {
            const uint32_t nch = hi_nch(hi), hidx = hi_hidx(hi);
            double acc[SH];
#pragma unroll
            for (int k = 0; k < SH; ++k) acc[k] = 0.0;
#pragma unroll
            for (uint32_t i = 0; i < 4; ++i) {
                if (i < nch) {
                    double v[SH];
                    if (i == hidx) {
#pragma unroll
                        for (int k = 0; k < SH; ++k) v[k] = xc[k];
                    } else {
                        const int q = off[j] + (int)i - (i > hidx ? 1 : 0);
                        bool held = false;
#pragma unroll
                        for (int r = 0; r < LR; ++r) {
                            if (q == r) {
#pragma unroll
                                for (int k = 0; k < SH; ++k) v[k] = lr[r][k];
                                held = true;
                            }
                        }
                        if (!held) load_row<SH>(U, cs[i], DP, hlane, v);  // rare: loaded here
                    }
                    const double S = i < 2 ? Sv[j][i < 2 ? i : 0] : sh.slut[cw_of(hfield<CH>(mv, hl, j, 2), hi, (int)i)];
#pragma unroll
                    for (int k = 0; k < SH; ++k) acc[k] = __builtin_fma(S, v[k], acc[k]);
                }
            }
#pragma unroll
            for (int k = 0; k < SH; ++k) xc[k] = acc[k] + (double)c[j][k];
            if (leaf_cost && nch == 0 && par != SM_NONE && par == (uint32_t)(top - j) - 1u)
                store_leaf_row<SH>(U, (uint32_t)(top - j), DP, hlane, c[j]);
            else
                store_row<SH>(U, (uint32_t)(top - j), DP, hlane, xc);
        }
    }
}

template <int CH, int SH>
__global__ __launch_bounds__(256) void k_up_walk_h2(WalkView V0, WalkView V1, const uint32_t* __restrict__ meta0,
                                                    const uint32_t* __restrict__ meta1, const SmPath* __restrict__ paths0,
                                                    const SmPath* __restrict__ paths1, const uint2* __restrict__ Lrec,
                                                    const uint2* __restrict__ Rrec, const uint32_t* __restrict__ Lrec4,
                                                    const uint32_t* __restrict__ Rrec4, const float* __restrict__ atab_g,
                                                    const double* __restrict__ slut_g, const double* __restrict__ s2lut_g,
                                                    int W, int dcall, int dglob0, int ppw, int leaf_cost) {
    __shared__ WalkShared sh;
    load_tables(sh, atab_g, slut_g, s2lut_g);
    const int view = blockIdx.y;
    const WalkView& V = view ? V1 : V0;
    const uint32_t* __restrict__ meta32 = view ? meta1 : meta0;
    const int lane = threadIdx.x & 63, hl = lane >> 5, hlane = lane & 31;
    const int wave = (int)uniform(blockIdx.x * 4 + (threadIdx.x >> 6));
    if (2 * wave * ppw >= V.npaths) return;  // uniform: both halves empty
    const SmPath* __restrict__ pp = view ? paths1 : paths0;
    const int pi0 = (2 * wave + hl) * ppw;
    int head = 0, len = 0;
    if (pi0 < V.npaths) {
        const int pi1 = min(pi0 + ppw, V.npaths);
        head = (int)pp[pi0].head;
        len = (int)(pp[pi1 - 1].head + pp[pi1 - 1].len) - head;
    }
    const int dbase = dglob0 + hlane * SH;
    const int dend = dglob0 + dcall;
    const uint2* __restrict__ own = view ? Rrec : Lrec;
    const uint32_t* __restrict__ oth4 = view ? Lrec4 : Rrec4;
    double xc[SH];
#pragma unroll
    for (int k = 0; k < SH; ++k) xc[k] = 0.0;
    int top = len > 0 ? head + len - 1 : 0;
    int n = min(CH, len);
    uint32_t cur = meta32[(size_t)(top - min(hlane >> 3, max(n, 1) - 1)) * 8 + (lane & 7)];
    walk_vm_drain();
    while (true) {
        const int ntop = top - CH;
        const int nn = (n > 0 && ntop >= head) ? min(CH, ntop - head + 1) : 0;
        uint32_t nxt;
        up_chunk_h2<CH, SH>(cur, n, top, view, lane, W, dbase, dend, own, oth4, V.U, sh, xc, nxt, meta32, nn > 0 ? ntop : top,
                        nn > 0 ? nn : max(n, 1), leaf_cost);
        if (__ballot(nn > 0) == 0) break;
        cur = nxt;
        if (nn > 0) {
            top = ntop;
            n = nn;
        } else {
            n = 0;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// down pass + WTA
// ---------------------------------------------------------------------------------------------
template <int SPL, int CH>
__global__ __launch_bounds__(256) void k_down_walk(WalkView V0, WalkView V1, const uint32_t* __restrict__ meta0,
                                                   const uint32_t* __restrict__ meta1, const SmPath* __restrict__ paths0,
                                                   const SmPath* __restrict__ paths1, const float* __restrict__ atab_g,
                                                   const double* __restrict__ slut_g, const double* __restrict__ s2lut_g,
                                                   int Dpad, WtaCfg w, int store_all, int ppw, int leaf_cost) {
    __builtin_amdgcn_s_setprio(1);  // as k_up_walk
    __shared__ WalkShared sh;
    load_tables(sh, atab_g, slut_g, s2lut_g);
    const int view = blockIdx.y;
    const WalkView& V = view ? V1 : V0;
    const uint32_t* __restrict__ meta32 = view ? meta1 : meta0;
    const int lane = threadIdx.x & 63;
    // work item: ppw consecutive paths = one contiguous slot range, root side first; a node is a
    // path head iff its parent is not the previous slot
    const int pi0 = (int)uniform((blockIdx.x * 4 + (threadIdx.x >> 6)) * ppw);
    if (pi0 >= V.npaths) return;
    const int pi1 = min(pi0 + ppw, V.npaths);
    const SmPath* __restrict__ pp = view ? paths1 : paths0;
    const int head = (int)uniform(pp[pi0].head);
    const int len = (int)uniform(pp[pi1 - 1].head + pp[pi1 - 1].len) - head;
    double xc[SPL];
#pragma unroll
    for (int k = 0; k < SPL; ++k) xc[k] = 0.0;
    int c0 = head;
    int n = min(CH, len);
    MetaVec<CH> cur;
    load_meta<CH>(cur, meta32, lane, c0, 1, n);
    walk_vm_drain();  // nothing pending on loop entry: the loop top then needs no wait at all
    while (true) {
        const int nc0 = c0 + CH;
        const int nn = nc0 < head + len ? min(CH, head + len - nc0) : 0;
        MetaVec<CH> nxt;
        // rows of the chunk (contiguous slots) and, for path heads, the parent's finished A row
        // (earlier round)
        double u[CH][SPL], xp[CH][SPL];
        uint32_t par[CH];
        // heavy leaves (WalkArgs::leaf_cost): their slot holds the f32 cost row (A_up = (double)C)
        bool leaf[CH];
#pragma unroll
        for (int j = 0; j < CH; ++j) {
            const int jj = j < n ? j : n - 1;
            const uint32_t slot = (uint32_t)(c0 + jj);
            par[j] = mfield(cur, jj, 1);
            const bool head_j = par[j] == SM_NONE || par[j] != slot - 1u;
            leaf[j] = leaf_cost && !head_j && hi_nch(mfield(cur, jj, 3)) == 0u;
#ifdef SM_EXP_DN_HEADS_ONLY  // timing experiment only (wrong results): read path heads' rows only
            if (head_j) load_row<SPL>(V.U, slot, Dpad, lane, u[j]); else for (int q = 0; q < SPL; ++q) u[j][q] = 0.0;
#else
            if (!leaf[j])  // uniform
                load_row<SPL>(V.U, slot, Dpad, lane, u[j]);
            else
                load_leaf_row<SPL>(V.U, slot, Dpad, lane, u[j]);  // f32 bits in u[j]'s registers
#endif
            if (head_j && par[j] != SM_NONE) {  // wave-uniform: only path heads read their parent's row
                load_row<SPL>(V.A, sm_arow(par[j]), Dpad, lane, xp[j]);
            } else {
#pragma unroll
                for (int q = 0; q < SPL; ++q) xp[j][q] = 0.0;
            }

        }
        // the next chunk's metadata, behind this chunk's row loads (see up_chunk)
        if (nn > 0) load_meta<CH>(nxt, meta32, lane, nc0, 1, nn);
        walk_vm_drain();
#pragma unroll
        for (int j = 0; j < CH; ++j)
            if (leaf[j]) widen_leaf_row<SPL>(u[j]);  // uniform
        double S[CH], S2[CH];
#pragma unroll
        for (int j = 0; j < CH; ++j) {
            const uint32_t wp = lo_wp(mfield(cur, j, 2));
            S[j] = readlane_f64(sh.slut[wp], 0);  // uniform: SGPR pairs
            S2[j] = readlane_f64(sh.s2lut[wp], 0);
        }
        // the chunk's recurrence first (registers only), then its stores: no store sits between
        // two uses of loaded rows, so the loads are waited for once
        double xs[CH][SPL];
#pragma unroll
        for (int j = 0; j < CH; ++j) {
            if (j < n) {
                // branch-free (selects): every loaded row is used on every path, so the compiler
                // keeps the loads in the chunk's batch instead of sinking them into a branch
                const uint32_t slot = (uint32_t)(c0 + j);
                const bool root = par[j] == SM_NONE;
                const bool head = !root && par[j] != slot - 1u;  // parent from an earlier round
#pragma unroll
                for (int k = 0; k < SPL; ++k) {
                    const double b = head ? xp[j][k] : xc[k];
                    const double f = __builtin_fma(S[j], b, S2[j] * u[j][k]);
                    xc[k] = root ? u[j][k] : f;  // A(root) = A_up(root)
                }
            }
#pragma unroll
            for (int k = 0; k < SPL; ++k) xs[j][k] = xc[k];
        }
#pragma unroll
        for (int j = 0; j < CH; ++j) {
            // light children's parents (the root too: A is a separate buffer) at their compact row
            if (j < n && hi_light(mfield(cur, j, 3))) store_row<SPL>(V.A, mfield(cur, j, 7), Dpad, lane, xs[j]);
            if (j < n && store_all) store_row<SPL>(V.Adbg, (uint32_t)(c0 + j), Dpad, lane, xs[j]);
        }
        double mn;
        int gi;
        float dsp;
#ifdef SM_EXP_DN_NO_WTA  // timing experiment only (wrong results): no WTA reduction
        mn = xs[0][0];
        gi = 0;
        dsp = 0.0f;
#else
        wta_nodes<SPL, CH>(xs, lane, w, mn, gi, dsp);
#endif
        const uint32_t pix = meta_pix_of_lane<CH>(cur, lane);  // all lanes active: bpermute sources
        if (lane < n) {  // lane j stores node j's result
            V.idx[pix] = gi;
            V.minc[pix] = mn;
            V.disp[pix] = dsp;
        }
        if (nn == 0) break;
        cur = nxt;
        c0 = nc0;
        n = nn;
    }
}

// ---------------------------------------------------------------------------------------------
// Half-wave down walker: SPL = 1 calls with 64-double rows (a 64-slice shard, e.g. a view-group
// rank at N = 8).  At SPL = 1 a node step costs a wave the same instructions as at SPL = 2 (the
// per-node metadata, LUT and branch work does not shrink with the slices), so here each half-wave
// of 32 lanes walks its own work item with 2 slices per lane: two paths per wave-step.  Per-node
// values that k_down_walk keeps wave-uniform are per half (two readlanes and a select); rows are
// the same [slot][64] rows (lane l of a half holds slices 2(l%32), 2(l%32)+1), the arithmetic is
// k_down_walk's exactly.  A half whose item is finished keeps re-reading its last chunk and stores
// nothing.
// wta_chunk per half-wave: lane 32h + j (< CH) gets node j of half h's strict-< first minimum
template <int CH, int SH>
__device__ __forceinline__ void wta_half(const double (&x)[CH][SH], int lane, int lo, int hi, double& out_min, int& out_idx) {
    const int hl = lane >> 5, hlane = lane & 31, dloc0 = hlane * SH;
    double bv[CH], g[CH];
    int bi[CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) {
        bv[j] = __builtin_huge_val();
        bi[j] = 0x7fffffff;
#pragma unroll
        for (int k = 0; k < SH; ++k) {
            const int d = dloc0 + k;
            if (d >= lo && d < hi && x[j][k] < bv[j]) { bv[j] = x[j][k]; bi[j] = d; }
        }
        g[j] = bv[j];
    }
#pragma unroll
    for (int j = 0; j < CH; ++j) g[j] = dpp_min<0xB1>(g[j]);
#pragma unroll
    for (int j = 0; j < CH; ++j) g[j] = dpp_min<0x4E>(g[j]);
#pragma unroll
    for (int j = 0; j < CH; ++j) g[j] = dpp_min<0x141>(g[j]);
#pragma unroll
    for (int j = 0; j < CH; ++j) g[j] = dpp_min<0x140>(g[j]);  // min over each row of 16 lanes
    out_min = 0.0;
    out_idx = 0;
#pragma unroll
    for (int j = 0; j < CH; ++j) {
        const double m0 = fmin(readlane_f64(g[j], 0), readlane_f64(g[j], 16));
        const double m1 = fmin(readlane_f64(g[j], 32), readlane_f64(g[j], 48));
        const double m = hl ? m1 : m0;
        const unsigned long long ball = __ballot(bv[j] == m && bi[j] != 0x7fffffff);
        const uint32_t b0 = (uint32_t)ball, b1 = (uint32_t)(ball >> 32);
        const int g0 = b0 ? __builtin_amdgcn_readlane(bi[j], (int)__builtin_ctz(b0)) : 0;
        const int g1 = b1 ? __builtin_amdgcn_readlane(bi[j], 32 + (int)__builtin_ctz(b1)) : 0;
        if (hlane == j) { out_min = m; out_idx = hl ? g1 : g0; }
    }
}

template <int CH, int SH>
__global__ __launch_bounds__(256) void k_down_walk_h2(WalkView V0, WalkView V1, const uint32_t* __restrict__ meta0,
                                                      const uint32_t* __restrict__ meta1, const SmPath* __restrict__ paths0,
                                                      const SmPath* __restrict__ paths1, const float* __restrict__ atab_g,
                                                      const double* __restrict__ slut_g, const double* __restrict__ s2lut_g,
                                                      WtaCfg w, int store_all, int ppw, int leaf_cost) {
    static_assert(CH <= 4, "lane 32h + 8j + f holds word f of half h's node j");
    constexpr int DP = 32 * SH;  // row length (doubles): 2 slices per half-lane, or 1 (32-slice rows)
    __shared__ WalkShared sh;
    load_tables(sh, atab_g, slut_g, s2lut_g);
    const int view = blockIdx.y;
    const WalkView& V = view ? V1 : V0;
    const uint32_t* __restrict__ meta32 = view ? meta1 : meta0;
    const int lane = threadIdx.x & 63, hl = lane >> 5, hlane = lane & 31;
    // work items 2*wave (lanes 0-31) and 2*wave+1 (lanes 32-63); an empty half has len 0
    const int wave = (int)uniform(blockIdx.x * 4 + (threadIdx.x >> 6));
    if (2 * wave * ppw >= V.npaths) return;  // uniform: both halves empty
    const SmPath* __restrict__ pp = view ? paths1 : paths0;
    const int pi0 = (2 * wave + hl) * ppw;
    int head = 0, len = 0;
    if (pi0 < V.npaths) {
        const int pi1 = min(pi0 + ppw, V.npaths);
        head = (int)pp[pi0].head;
        len = (int)(pp[pi1 - 1].head + pp[pi1 - 1].len) - head;
    }
    double xc[SH];
#pragma unroll
    for (int k = 0; k < SH; ++k) xc[k] = 0.0;
    int c0 = head;
    int n = min(CH, len);  // 0: this half is finished (or empty)
    // metadata: lane 32h + 8j + f holds word f of node j of half h (clamped to a valid node)
    uint32_t cur = meta32[(size_t)(c0 + min(hlane >> 3, max(n, 1) - 1)) * 8 + (lane & 7)];
    walk_vm_drain();
    while (true) {
        const int nc0 = c0 + CH;
        const int nn = (n > 0 && nc0 < head + len) ? min(CH, head + len - nc0) : 0;
        double u[CH][SH], xp[CH][SH];
        uint32_t par[CH], hiw[CH];
        bool leaf[CH];
#pragma unroll
        for (int j = 0; j < CH; ++j) {
            // node j >= n: the metadata lanes of node j already hold node n - 1's words (clamped
            // load), so readlane indices stay uniform; only the slot is clamped per lane
            const uint32_t slot = (uint32_t)(c0 + min(j, max(n, 1) - 1));
            par[j] = hfield<CH>(cur, hl, j, 1);
            hiw[j] = hfield<CH>(cur, hl, j, 3);
            const bool head_j = par[j] == SM_NONE || par[j] != slot - 1u;
            leaf[j] = leaf_cost && !head_j && hi_nch(hiw[j]) == 0u;
            if (!leaf[j])
                load_row<SH>(V.U, slot, DP, hlane, u[j]);
            else
                load_leaf_row<SH>(V.U, slot, DP, hlane, u[j]);
            // a finished half's re-read chunk pairs node j's words with slot c0: no A row is read
            // there (its parent word may be a slot, not a compact A row)
            if (n > 0 && head_j && par[j] != SM_NONE) {
                load_row<SH>(V.A, sm_arow(par[j]), DP, hlane, xp[j]);
            } else {
#pragma unroll
                for (int k = 0; k < SH; ++k) xp[j][k] = 0.0;
            }
        }
        // the next chunk's metadata behind the rows (a finished half re-reads its last chunk's)
        const int mc0 = nn > 0 ? nc0 : c0;
        const int mn_ = nn > 0 ? nn : max(n, 1);
        const uint32_t nxt = meta32[(size_t)(mc0 + min(hlane >> 3, mn_ - 1)) * 8 + (lane & 7)];
        walk_vm_drain();
#pragma unroll
        for (int j = 0; j < CH; ++j)
            if (leaf[j]) widen_leaf_row<SH>(u[j]);
        double S[CH], S2[CH];
#pragma unroll
        for (int j = 0; j < CH; ++j) {
            const uint32_t wp = lo_wp(hfield<CH>(cur, hl, j, 2));
            S[j] = sh.slut[wp];
            S2[j] = sh.s2lut[wp];
        }
        double xs[CH][SH];
#pragma unroll
        for (int j = 0; j < CH; ++j) {
            if (j < n) {
                const uint32_t slot = (uint32_t)(c0 + j);
                const bool root = par[j] == SM_NONE;
                const bool hd = !root && par[j] != slot - 1u;
#pragma unroll
                for (int k = 0; k < SH; ++k) {
                    const double b = hd ? xp[j][k] : xc[k];
                    const double f = __builtin_fma(S[j], b, S2[j] * u[j][k]);
                    xc[k] = root ? u[j][k] : f;
                }
            }
#pragma unroll
            for (int k = 0; k < SH; ++k) xs[j][k] = xc[k];
        }
#pragma unroll
        for (int j = 0; j < CH; ++j) {
            if (j < n && hi_light(hiw[j])) store_row<SH>(V.A, hfield<CH>(cur, hl, j, 7), DP, hlane, xs[j]);
            if (j < n && store_all) store_row<SH>(V.Adbg, (uint32_t)(c0 + j), DP, hlane, xs[j]);
        }
        double mn;
        int mi;
        wta_half<CH, SH>(xs, lane, w.lo, w.hi, mn, mi);
        const int gi = w.dglob0 + mi;
        // lane 32h + j (< CH) stores node j of half h: its pixel is word 0 at lane 32h + 8j
        const int src = ((hl << 5) + ((hlane & 3) << 3)) << 2;
        const uint32_t pix = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)cur);
        if (hlane < n) {
            V.idx[pix] = gi;
            V.minc[pix] = mn;
            V.disp[pix] = (float)gi;
        }
        if (__ballot(nn > 0) == 0) break;
        cur = nxt;
        if (nn > 0) {
            c0 = nc0;
            n = nn;
        } else {
            n = 0;
        }
    }
}

// ---------------------------------------------------------------------------------------------
static WalkView to_view(const WalkArgs& a, int v) {
    return WalkView{a.npaths[v], a.U[v], a.idx[v], a.minc[v], a.disp[v], a.A[v], a.Adbg[v]};
}

// A/B knob: extra dynamic LDS per block (limits walker occupancy; experiments only)
static size_t walk_lds_pad() {
    static const char* e = sm_dev_knob("SM_WALK_LDS_PAD");
    return e ? (size_t)atoi(e) : 0;
}

// Paths per work item.  A round whose items at the default size would not give the GPU ~8k
// waves (a small, deep round: its time is the latency of its longest item, not bytes) gets fewer
// paths per item, down to one.  SM_WALK_FILL / SM_WALK_FILL_DN: the target item count of the up /
// down walker (0: always the default).
static int walk_ppw(int np, int dflt, bool down) {
    static const int fill_up = [] {
        const char* e = sm_dev_knob("SM_WALK_FILL");
        return e ? atoi(e) : 8192;
    }();
    static const int fill_dn = [] {
        const char* e = sm_dev_knob("SM_WALK_FILL_DN");
        return e ? atoi(e) : 8192;
    }();
    const int fill = down ? fill_dn : fill_up;
    if (fill <= 0 || (np + dflt - 1) / dflt >= fill) return dflt;
    const int p = (np + fill - 1) / fill;
    return p < 1 ? 1 : p;
}

template <int SPL, int CH>
static void up_launch(hipStream_t st, dim3 g, const WalkArgs& a, int ppw, const UpPreArgs& pa) {
    if (a.vol)
        hipLaunchKernelGGL((k_up_walk<SPL, CH, true>), g, dim3(256), walk_lds_pad(), st, to_view(a, 0), to_view(a, 1),
                           reinterpret_cast<const uint32_t*>(a.meta[0]), reinterpret_cast<const uint32_t*>(a.meta[1]),
                           a.paths[0], a.paths[1], a.Lrec, a.Rrec, a.Lrec4, a.Rrec4, a.atab, a.slut, a.s2lut, a.W, a.Dpad, a.dcall,
                           a.dglob0, a.Cst[0], a.Cst[1], ppw, a.leaf_cost, pa);
    else
        hipLaunchKernelGGL((k_up_walk<SPL, CH, false>), g, dim3(256), walk_lds_pad(), st, to_view(a, 0), to_view(a, 1),
                           reinterpret_cast<const uint32_t*>(a.meta[0]), reinterpret_cast<const uint32_t*>(a.meta[1]),
                           a.paths[0], a.paths[1], a.Lrec, a.Rrec, a.Lrec4, a.Rrec4, a.atab, a.slut, a.s2lut, a.W, a.Dpad, a.dcall,
                           a.dglob0, a.Cst[0], a.Cst[1], ppw, a.leaf_cost, pa);
}

template <int SPL, int CH>
static void down_launch(hipStream_t st, dim3 g, const WalkArgs& a, int store_all, int ppw) {
    hipLaunchKernelGGL((k_down_walk<SPL, CH>), g, dim3(256), walk_lds_pad(), st, to_view(a, 0), to_view(a, 1),
                       reinterpret_cast<const uint32_t*>(a.meta[0]), reinterpret_cast<const uint32_t*>(a.meta[1]),
                       a.paths[0], a.paths[1], a.atab, a.slut, a.s2lut, a.Dpad, a.wta, store_all, ppw,
                       store_all ? 0 : a.leaf_cost);
}

// SPL = 1 calls take the half-wave walkers: 64-double rows with 2 slices per half-lane, 32-double rows
// (a call of <= 32 slices, e.g. a d-shard rank at N = 8) with 1 (dev builds: SM_NO_HALF_WAVE for A/B)
static bool half_wave(const WalkArgs& a, int spl) {
    static const bool off = sm_dev_knob("SM_NO_HALF_WAVE") != nullptr;
    return !off && spl == 1 && (a.Dpad == 64 || a.Dpad == 32);
}

hipError_t launch_up(hipStream_t st, const WalkArgs& a, int spl, bool long_paths, const WalkArgs* pre) {
    const int np = a.npaths[0] > a.npaths[1] ? a.npaths[0] : a.npaths[1];
    if (!long_paths && !pre && !a.vol && half_wave(a, spl)) {
        if (np == 0) return hipSuccess;
        const int ppw = walk_ppw(np, WALK_PPW_UP, false);
        const int items = (np + ppw - 1) / ppw;
        const int waves = (items + 1) / 2;
        const dim3 g((waves + 3) / 4, 2);
        if (a.Dpad == 64)
            hipLaunchKernelGGL((k_up_walk_h2<WALK_UP_CHH, 2>), g, dim3(256), walk_lds_pad(), st, to_view(a, 0), to_view(a, 1),
                               reinterpret_cast<const uint32_t*>(a.meta[0]), reinterpret_cast<const uint32_t*>(a.meta[1]),
                               a.paths[0], a.paths[1], a.Lrec, a.Rrec, a.Lrec4, a.Rrec4, a.atab, a.slut, a.s2lut, a.W, a.dcall,
                               a.dglob0, ppw, a.leaf_cost);
        else
            hipLaunchKernelGGL((k_up_walk_h2<WALK_UP_CHH1, 1>), g, dim3(256), walk_lds_pad(), st, to_view(a, 0), to_view(a, 1),
                               reinterpret_cast<const uint32_t*>(a.meta[0]), reinterpret_cast<const uint32_t*>(a.meta[1]),
                               a.paths[0], a.paths[1], a.Lrec, a.Rrec, a.Lrec4, a.Rrec4, a.atab, a.slut, a.s2lut, a.W, a.dcall,
                               a.dglob0, ppw, a.leaf_cost);
        return hipGetLastError();
    }
    const int ppw = walk_ppw(np, WALK_PPW_UP, false);
    const int items = (np + ppw - 1) / ppw;
    UpPreArgs pa{};
    if (pre) pa = up_pre_args(*pre);
    pa.walk_blocks = (items + 3) / 4;
    const int ns = pa.nseg[0] > pa.nseg[1] ? pa.nseg[0] : pa.nseg[1];
    if (pa.walk_blocks + ns == 0) return hipSuccess;
    const dim3 g(pa.walk_blocks + ns, 2);
    if (long_paths) {
        switch (spl) {
            case 1: up_launch<1, 8>(st, g, a, ppw, pa); break;
            case 2: up_launch<2, 8>(st, g, a, ppw, pa); break;
            default: up_launch<4, 4>(st, g, a, ppw, pa); break;
        }
    } else {
        switch (spl) {
            case 1: up_launch<1, WALK_UP_CH1>(st, g, a, ppw, pa); break;
            case 2: up_launch<2, WALK_UP_CH2>(st, g, a, ppw, pa); break;
            default: up_launch<4, WALK_UP_CH4>(st, g, a, ppw, pa); break;
        }
    }
    return hipGetLastError();
}

// SPL = 1 calls with 64-double rows take the half-wave down walker (env SM_NO_HALF_WAVE: A/B)
#ifndef WALK_DN_CHH
#define WALK_DN_CHH 3
#endif
#ifndef WALK_DN_CHH1
#define WALK_DN_CHH1 3  // 32-slice rows (1 slice per half-lane)
#endif
static bool half_wave_down(const WalkArgs& a, int spl) { return half_wave(a, spl) && !a.wta.sub; }

static hipError_t launch_down_impl(hipStream_t st, const WalkArgs& a, int spl, int store_all, bool long_paths) {
    const int np = a.npaths[0] > a.npaths[1] ? a.npaths[0] : a.npaths[1];
    if (np == 0) return hipSuccess;
    if (!long_paths && half_wave_down(a, spl)) {
        const int ppw = walk_ppw(np, WALK_PPW_DN, true);
        const int items = (np + ppw - 1) / ppw;
        const int waves = (items + 1) / 2;
        const dim3 g((waves + 3) / 4, 2);
        if (a.Dpad == 64)
            hipLaunchKernelGGL((k_down_walk_h2<WALK_DN_CHH, 2>), g, dim3(256), walk_lds_pad(), st, to_view(a, 0), to_view(a, 1),
                               reinterpret_cast<const uint32_t*>(a.meta[0]), reinterpret_cast<const uint32_t*>(a.meta[1]),
                               a.paths[0], a.paths[1], a.atab, a.slut, a.s2lut, a.wta, store_all, ppw, store_all ? 0 : a.leaf_cost);
        else
            hipLaunchKernelGGL((k_down_walk_h2<WALK_DN_CHH1, 1>), g, dim3(256), walk_lds_pad(), st, to_view(a, 0), to_view(a, 1),
                               reinterpret_cast<const uint32_t*>(a.meta[0]), reinterpret_cast<const uint32_t*>(a.meta[1]),
                               a.paths[0], a.paths[1], a.atab, a.slut, a.s2lut, a.wta, store_all, ppw, store_all ? 0 : a.leaf_cost);
        return hipGetLastError();
    }
    const int ppw = walk_ppw(np, WALK_PPW_DN, true);
    const int items = (np + ppw - 1) / ppw;
    const dim3 g((items + 3) / 4, 2);
    if (long_paths) {
        switch (spl) {
            case 1: down_launch<1, 16>(st, g, a, store_all, ppw); break;
            case 2: down_launch<2, 16>(st, g, a, store_all, ppw); break;
            default: down_launch<4, 8>(st, g, a, store_all, ppw); break;
        }
    } else {
        switch (spl) {
            case 1: down_launch<1, WALK_DN_CH1>(st, g, a, store_all, ppw); break;
            case 2: down_launch<2, WALK_DN_CH2>(st, g, a, store_all, ppw); break;
            default: down_launch<4, WALK_DN_CH4>(st, g, a, store_all, ppw); break;
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
