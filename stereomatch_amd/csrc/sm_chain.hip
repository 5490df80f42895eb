// sm_chain.hip -- long-path engine of the tree filter.
//
// A heavy path of L nodes is a serial recurrence of L steps per disparity slice; in the chunked
// walkers (sm_walk.hip) every step also waits for its own row/image loads, so a long path costs
// ~L x (memory latency / chunk).  For paths of >= SM_LONG_PATH nodes the work is split so that the
// serial chain touches only LDS and registers:
//
//   k_up_pre    (grid-wide, fully parallel over the long paths' nodes)
//               Pre(v) = fold of the light children that come BEFORE the heavy child in the
//               reference's descending-key order, written into U[slot(v)]; the AGD cost C(v) is
//               written to the float staging row Cst[slot(v)].
//   k_up_chain  (one 1024-thread workgroup per long path)
//               wave 0 runs  acc = fma(S_h, x, Pre); acc = fma(S_p, A_p, acc) for the children
//               AFTER the heavy one; x = acc + C   out of an LDS ring; waves 1..15 stream Pre, C,
//               the post-heavy child rows and the weights into the ring ahead of it and store the
//               finished rows back to U.
//   k_down_chain (one workgroup per long path)
//               helpers stage T(v) = S2_v * A_up(v) and S_v; wave 0 runs x = fma(S_v, x, T(v));
//               helpers then do the strict-< WTA of each finished row (batched DPP), write
//               idx/minc/disp and store the rows that light children (or the debug path) need.
//
// Every value is produced by the same fp64 operations in the same order as the shipped
// reference (Stereo3DMST.cpp:125-157, DESIGN.md "Shipped arithmetic"): splitting the fold at the
// heavy child only moves the pre-heavy fmas (whose inputs are final before the round starts) off
// the chain; T(v) = S2*A_up is the product the reference rounds before its fma.  Results stay
// bit-identical to the oracle and independent of the schedule.
//
// Group ring (see "Group ring" below): one state word per group of G nodes; a wave's LDS
// operations complete in issue order, so a state word observed after data written before it
// (or a state written after data read before it) orders the hand-off without extra waits.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "sm_common.h"
#include "sm_launch.h"
#include "sm_layout_gpu.h"
#include "sm_walk_util.h"


// -DSM_CHAIN_PROF: the first path of each launch prints chain-wave cycles / failed polls and helper
// wait cycles (device printf) -- a diagnostic build only (tools/chain_prof.sh)
#ifdef SM_CHAIN_PROF
#include <stdio.h>
#endif
#ifdef SM_CHAIN_TIMES
// diagnostic build: every chain workgroup appends {tag | view | M | len, start, end, item} (100 MHz
// s_memrealtime) to a device log, read by sm_chain_times_dump (tools/chain_times.py)
#define SM_CT_CAP 65536
__device__ unsigned long long g_ct[4 * SM_CT_CAP];
__device__ unsigned int g_ct_n;
__device__ __forceinline__ void ct_log(int down, int view, int M, int len, int item, unsigned long long t0,
                                       unsigned long long t1 = 0) {
    const unsigned k = atomicAdd(&g_ct_n, 1u);
    if (k < SM_CT_CAP) {
        g_ct[4 * k] = (unsigned long long)down | ((unsigned long long)view << 2) | ((unsigned long long)M << 8) |
                      ((unsigned long long)len << 32);
        g_ct[4 * k + 1] = t0;
        g_ct[4 * k + 2] = t1 ? t1 : __builtin_amdgcn_s_memrealtime();
        g_ct[4 * k + 3] = (unsigned long long)item;
    }
}
extern "C" int sm_chain_times_dump(unsigned long long* out, int cap) {
    unsigned n = 0;
    if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(g_ct_n), sizeof(n)) != hipSuccess) return -1;
    n = n < SM_CT_CAP ? n : SM_CT_CAP;
    n = (int)n < cap ? n : (unsigned)cap;
    if (n && hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ct), (size_t)n * 32) != hipSuccess) return -1;
    const unsigned z = 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_ct_n), &z, sizeof(z)) != hipSuccess) return -1;
    return (int)n;
}
#endif
#ifdef SM_CHAIN_PROF
__device__ unsigned long long g_spins;
#define PROF_SPIN(x) (x)
#else
#define PROF_SPIN(x) ((void)0)
#endif

// chain-side publish: LDS operations of one wave complete in issue order, so the result rows
// written before this store are visible to any wave that observes the new state
__device__ __forceinline__ void lds_publish_ordered(int* p, int v) {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

__device__ __forceinline__ int lds_state(int* p) {
    const int v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    return v;
}

__device__ __forceinline__ void lds_publish(int* p, int v) {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS writes have landed
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// all of this wave's vector-memory loads have returned (stores issued later are not waited for)
__device__ __forceinline__ void vm_drain() { __builtin_amdgcn_s_waitcnt(0x0F70); }  // vmcnt(0)

// Cross-workgroup hand-off (status words of pieces), the agent-scope release/acquire protocol:
//   producer: its stores (rows: agent-scope stores) -> release fence at agent scope (writes back the
//             XCD's L2) -> s_waitcnt vmcnt(0) in asm (ROCm 7.2 can drop the fence's own wait) ->
//             relaxed agent-scope store of the word;
//   consumer: relaxed agent-scope polls of the word -> one acquire fence at agent scope (invalidates
//             this CU's L1) -> s_waitcnt vmcnt(0) -> its loads (rows: agent-scope loads).
// A wait gives up after SM_WAIT_ITERS polls (~1 s by default; tests lower it): it then sets the
// call's device error word, which sm_synchronize turns into an error status -- a missed publication
// can never return SM_OK with wrong disparities.
__device__ __forceinline__ uint32_t wait_word(const uint32_t* p, uint32_t lo, uint32_t hi, uint32_t* err, int iters) {
    uint32_t v = 0;
    for (int it = 0; it < iters; ++it) {
        v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (v >= lo && v <= hi) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            return v;
        }
        __builtin_amdgcn_s_sleep(2);
    }
    __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return v;
}
__device__ __forceinline__ void publish_word(uint32_t* p, uint32_t v) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void lds_wait(int* p, int v, bool sleep, unsigned* spins = nullptr) {
    while (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != v) {
        PROF_SPIN(spins && ++*spins);
        if (sleep) __builtin_amdgcn_s_sleep(1);
    }
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

template <int SPL>
__device__ __forceinline__ void lds_row_read(const double* row, int lane, double (&r)[SPL]) {
#pragma unroll
    for (int k = 0; k < SPL; ++k) r[k] = row[lane * SPL + k];
}
template <int SPL>
__device__ __forceinline__ void lds_row_write(double* row, int lane, const double (&r)[SPL]) {
#pragma unroll
    for (int k = 0; k < SPL; ++k) row[lane * SPL + k] = r[k];
}

template <int SPL>
__device__ __forceinline__ void load_crow(const float* __restrict__ C, uint32_t slot, int Dpad, int lane, float (&c)[SPL]) {
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
// ---------------------------------------------------------------------------------------------
// k_up_pre: the segment aggregates of the round's cut long paths (up_pre_segment) in a launch of
// their own, before the round's chains.  -DSM_PRE_FUSED (A/B) runs them as extra blocks of the
// round's walker launch instead (sm_walk.hip).
// ---------------------------------------------------------------------------------------------
template <int SPL, int CH, int NSUB, bool VOL>
__global__ __launch_bounds__(256) void k_up_pre(WalkView V0, WalkView V1, const uint32_t* __restrict__ meta0,
                                                const uint32_t* __restrict__ meta1, UpPreArgs pa,
                                                const float* __restrict__ Cst0, const float* __restrict__ Cst1,
                                                const uint2* __restrict__ Lrec, const uint2* __restrict__ Rrec,
                                                const float* __restrict__ atab_g, const double* __restrict__ slut_g,
                                                const double* __restrict__ s2lut_g, int W, int Dpad, int dcall, int dglob0) {
    const int view = blockIdx.y;
    if ((int)blockIdx.x >= pa.nseg[view]) return;  // uniform over the block
    __shared__ WalkShared sh;
    load_tables(sh, atab_g, slut_g, s2lut_g);
    up_pre_segment<SPL, CH, NSUB, VOL>(pa, view, (int)blockIdx.x, view ? V1.U : V0.U, view ? meta1 : meta0, view ? Cst1 : Cst0,
                                       view ? Rrec : Lrec, view ? Lrec : Rrec, W, Dpad, dcall, dglob0, sh, sh.s2lut,
                                       threadIdx.x & 63, (int)uniform(threadIdx.x >> 6));
}

// ---------------------------------------------------------------------------------------------
// Group ring.  Chain node j (0 = first node the chain visits) belongs to group g = j / G; group g
// is staged in LDS slot g % NS by helper (g % NH), which holds its next group's rows in registers
// while it waits for the slot -- so the lead time of the global loads is ~NH groups of chain time,
// independent of the LDS capacity.  The serial recurrence is split over NCW chain waves by slice
// range (slices are independent chains): a lone wave's cost per node is dominated by the bytes it
// moves through LDS, so each chain wave moves 1/NCW of the row.  Chain wave w, lane l owns slice
// elements [(64w + l) * CS, +CS) of every row.
// ---------------------------------------------------------------------------------------------
#ifndef CHN_WAVES
#define CHN_WAVES 16
#endif
#define CHN_THREADS (64 * CHN_WAVES)

template <int SPL>
struct Split {
    static constexpr int NCW = SPL == 1 ? 1 : 2;  // chain waves
    static constexpr int CS = SPL / NCW;          // slices per chain lane
#ifdef SM_CHAIN_EXCL
    // chain waves own their SIMDs (wave w runs on SIMD w % 4): helpers only on the other SIMDs
    static constexpr int NH = CHN_WAVES / 4 * (4 - NCW);
    // role of wave w: chain wave w (w < NCW), helper index, or -1 (idle)
    __device__ static int helper_of(int w) { return (w & 3) < NCW ? -1 : (w >> 2) * (4 - NCW) + (w & 3) - NCW; }
#else
    static constexpr int NH = CHN_WAVES - NCW;    // helper waves
    __device__ static int helper_of(int w) { return w - NCW; }
#endif
};

template <int CS>
__device__ __forceinline__ void lds_read_at(const double* row, int e0, double (&r)[CS]) {
#pragma unroll
    for (int q = 0; q < CS; ++q) r[q] = row[e0 + q];
}
template <int CS>
__device__ __forceinline__ void lds_write_at(double* row, int e0, const double (&r)[CS]) {
#pragma unroll
    for (int q = 0; q < CS; ++q) row[e0 + q] = r[q];
}
template <int CS>
__device__ __forceinline__ void global_read_at(const double* __restrict__ U, uint32_t slot, int Dpad, int e0, double (&r)[CS]) {
    const double* p = U + (size_t)slot * Dpad + e0;
    if constexpr (CS == 1) {
        r[0] = p[0];
    } else {
        const double2 t = *reinterpret_cast<const double2*>(p);
        r[0] = t.x;
        r[1] = t.y;
    }
}
template <int CS>
__device__ __forceinline__ void global_write_at(double* __restrict__ U, uint32_t slot, int Dpad, int e0, const double (&r)[CS]) {
    double* p = U + (size_t)slot * Dpad + e0;
    if constexpr (CS == 1)
        p[0] = r[0];
    else
        *reinterpret_cast<double2*>(p) = make_double2(r[0], r[1]);
}

__device__ __forceinline__ void lds_wait_all(int* p, int n, int v) {  // p[0..n) == v
    for (int w = 0; w < n; ++w) lds_wait(&p[w], v, true);
}

// ---------------------------------------------------------------------------------------------
// k_up_chain
//
// Branch-free node step:  acc = fma(Sh, x, Pre); acc = fma(Sp1, P1, acc); acc = fma(Sp2, P2, acc);
// x = acc + C.  Absent children carry S = 0 and a dummy row: every aggregate is finite and >= +0,
// so fma(0, r, acc) == acc exactly and the step equals the reference's fold with only the
// children present (the bottom node has Sh = 0 and x = 0, i.e. acc = Pre).  A tree root may have a
// third post-heavy child: its group takes the node-by-node path with one more fma.
// ---------------------------------------------------------------------------------------------
#ifndef UP_NS2
#define UP_NS2 9
#endif
#ifndef UP_G4
#define UP_G4 2
#endif
#ifndef UP_NS4
#define UP_NS4 8
#endif
#ifndef UP_G1
#define UP_G1 4  // SPL = 1 (one-view 64-slice shares, D <= 64); 6 x 10 -> 4 x 18: k_up_chain 0.529 -> 0.504 ms at the N = 8 share
#endif
#ifndef UP_NS1
#define UP_NS1 10  // round 5: 18 -> 10 slots (150 -> ~85 KB of LDS, so other frames' walker blocks fit beside
                   // a chain workgroup): the N = 8 share 1.945-1.948 -> 1.907-1.918 ms/frame, the kernel itself
                   // unchanged (SPL = 2's ring at 5 / 6 slots did not help C2: DESIGN.md 5.-2)
#endif
#ifndef UP_G2
#define UP_G2 4  // even: the chain's two-half pipeline
#endif
#ifndef UP_STORERS
#define UP_STORERS 2  // helper waves that only store the chain's results (the others load and stage)
#endif
template <int SPL>
struct UpCfg {
    static constexpr int G = SPL == 1 ? UP_G1 : SPL == 2 ? UP_G2 : UP_G4;  // nodes per group (helper registers)
    static constexpr int NS = SPL == 1 ? UP_NS1 : SPL == 2 ? UP_NS2 : UP_NS4;  // LDS slots (the ring: static_assert below)
};

struct UpNodeS {
    double Sh, Sp1, Sp2, pad;
};

template <int SPL>
struct UpSlot {
    static constexpr int G = UpCfg<SPL>::G;
    double pre[G][64 * SPL];    // Pre (pre-heavy fold) in; the chain's A_up rows out
    double post1[G][64 * SPL];  // first post-heavy child row (dummy if absent)
    double post2[G][64 * SPL];  // second post-heavy child row (dummy if absent)
    double post3[64 * SPL];     // a root's third post-heavy child
    float c[G][64 * SPL];       // AGD cost
    UpNodeS s[G];
    double S3;
    int k3;                     // node of the group with a third post-heavy child, or -1
    int done[2];                // g+1: chain wave w finished group g  (chain wave -> owner helper)
    int freed;                  // g+1: slot of group g reusable        (owner helper -> next helper)
    unsigned long long staged;  // (flags << 32) | (g+1): group g staged (helper -> chain waves);
                                // flags: 3 bits per node (Pre, post1, post2 rows present) + UP_F3
};
#define UP_F_PRE 1u
#define UP_F_P1 2u
#define UP_F_P2 4u
#define UP_F3 (1u << 31)  // the group has a third post-heavy child (node-by-node path)

__device__ __forceinline__ unsigned long long lds_state64(unsigned long long* p) {
    const unsigned long long v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    return v;
}

template <int SPL>
struct UpRing {
    UpSlot<SPL> s[UpCfg<SPL>::NS];
    double slut[SM_NUM_W + 1];
    float atab[SM_MAX_W + 1];  // AGD colour term by integer L1 (helpers compute the cost rows)
};
// LDS budget of k_up_chain (gfx950: 160 KB per workgroup): the ring, the pieces' guess row and a few
// words of scalars.  UP_G*/UP_NS* are A/B macros; a geometry that does not fit fails here, not at launch.
#define SM_LDS_BYTES (160 * 1024)
static_assert(sizeof(UpRing<1>) + 64 * 1 * 8 + 64 <= SM_LDS_BYTES, "UpRing<1> (UP_G1 x UP_NS1) exceeds the LDS");
static_assert(sizeof(UpRing<2>) + 64 * 2 * 8 + 64 <= SM_LDS_BYTES, "UpRing<2> (UP_G2 x UP_NS2) exceeds the LDS");
static_assert(sizeof(UpRing<4>) + 64 * 4 * 8 + 64 <= SM_LDS_BYTES, "UpRing<4> (UP_G4 x UP_NS4) exceeds the LDS");

// where the up chain's cost rows come from: computed by the helpers from the image records (the
// AGD cost, PatchMatchStereoGPU.cu:1482-1550), or read from the f32 rows k_vol_rows filled
// (MC-CNN ingest)
struct UpCost {
    const uint2* own;      // the view's reference image records
    const uint2* oth;      // the matched image's records
    const uint32_t* oth4;  // the matched image's 4-byte records (bgrx; the gray is recomputed)
    const float* Cst;      // cost rows [slot][Dpad] (ingest)
    int W, dbase, dend, view;
};

// The up chain's image records (helpers and repair walks).  Round 6: the walkers' 4-byte records (bgrx
// alone, the gray recomputed in k_prep's operation order, so the costs are bit-identical): per node a
// lane loads SPL + 1 dwords instead of SPL {bgrx, gray} pairs and a gray word.  At C2 the chain's
// fetched bytes were ~1 KB per node, mostly these windows missing L2.  -DSM_CHAIN_REC8: the 8-byte
// records (A/B).
#ifdef SM_CHAIN_REC8
template <int SPL, int CH>
using ChainRecs = ImgRecs<SPL, CH>;
template <int SPL, int CH>
__device__ __forceinline__ void chain_load_recs(const MetaVec<CH>& mv, int n, int lane, const UpCost& cs, ChainRecs<SPL, CH>& r) {
    load_recs<SPL, CH>(mv, n, cs.view, lane, cs.W, cs.dbase, cs.own, cs.oth, r);
}
template <int SPL, int CH, class T>
__device__ __forceinline__ void chain_costs(const MetaVec<CH>& mv, const UpCost& cs, const ChainRecs<SPL, CH>& r,
                                            const float* __restrict__ atab, T (&c)[CH][SPL]) {
    chunk_costs<SPL, CH>(mv, cs.view, cs.W, cs.dbase, cs.dend, r, atab, c);
}
#else
template <int SPL, int CH>
using ChainRecs = ImgRecs4<SPL, CH>;
template <int SPL, int CH>
__device__ __forceinline__ void chain_load_recs(const MetaVec<CH>& mv, int n, int lane, const UpCost& cs, ChainRecs<SPL, CH>& r) {
    load_recs4<SPL, CH>(mv, n, cs.view, lane, cs.dbase, cs.own, cs.oth4, r);
}
template <int SPL, int CH, class T>
__device__ __forceinline__ void chain_costs(const MetaVec<CH>& mv, const UpCost& cs, const ChainRecs<SPL, CH>& r,
                                            const float* __restrict__ atab, T (&c)[CH][SPL]) {
    chunk_costs4<SPL, CH>(mv, cs.view, cs.W, cs.dbase, cs.dend, r, atab, c);
}
#endif

// NN consecutive nodes k0.. of a staged group; NN is a compile-time count so the LDS waits are
// exact; THIRD = the node-by-node path that also applies a root's third post-heavy child.
// Every row is read unconditionally (the ring is zeroed at kernel start, so rows a helper did
// not stage are stale-but-finite): absent posts carry S = 0, and an absent Pre is replaced by +0
// through a select on the presence flags -- exact, and off the serial chain.
template <int SPL, int NN, bool THIRD>
__device__ __forceinline__ void up_group(UpSlot<SPL>& sl, uint32_t flags, int k0, int j0, int top, int e0,
                                         double (&x)[Split<SPL>::CS], double* __restrict__ U, int Dpad) {
    constexpr int CS = Split<SPL>::CS;
    double pr[NN][CS], p1[NN][CS], p2[NN][CS], Sh[NN], Sp1[NN], Sp2[NN];
    float cv[NN][CS];
#pragma unroll
    for (int k = 0; k < NN; ++k) {
        Sh[k] = sl.s[k0 + k].Sh;
        Sp1[k] = sl.s[k0 + k].Sp1;
        Sp2[k] = sl.s[k0 + k].Sp2;
#ifdef SM_PROF_NOROWS
#pragma unroll
        for (int q = 0; q < CS; ++q) {
            pr[k][q] = 0.25 * (k + q);
            p1[k][q] = 0.5 * (k + q);
            p2[k][q] = 0.125 * (k + q);
            cv[k][q] = 0.75f;
        }
#else
        lds_read_at<CS>(sl.pre[k0 + k], e0, pr[k]);
        lds_read_at<CS>(sl.post1[k0 + k], e0, p1[k]);
        lds_read_at<CS>(sl.post2[k0 + k], e0, p2[k]);
#pragma unroll
        for (int q = 0; q < CS; ++q) cv[k][q] = sl.c[k0 + k][e0 + q];
#endif
    }
#pragma unroll
    for (int k = 0; k < NN; ++k) {
        const bool hpre = (flags >> (3 * (k0 + k))) & UP_F_PRE;
        double acc[CS];
#pragma unroll
        for (int q = 0; q < CS; ++q) {
            acc[q] = __builtin_fma(Sh[k], x[q], hpre ? pr[k][q] : 0.0);  // select: exact +0 whatever the stale row holds
            acc[q] = __builtin_fma(Sp1[k], p1[k][q], acc[q]);
            acc[q] = __builtin_fma(Sp2[k], p2[k][q], acc[q]);
        }
        if (THIRD && k0 + k == sl.k3) {
            double r[CS];
            lds_read_at<CS>(sl.post3, e0, r);
#pragma unroll
            for (int q = 0; q < CS; ++q) acc[q] = __builtin_fma(sl.S3, r[q], acc[q]);
        }
#pragma unroll
        for (int q = 0; q < CS; ++q) x[q] = acc[q] + (double)cv[k][q];
        // the result row goes back through LDS and the owner helper stores it: a global store per
        // node on the chain wave makes the chain wait on store completions (vmcnt), which are slow
        // whenever the rest of the GPU is busy
        lds_write_at<CS>(sl.pre[k0 + k], e0, x);
        (void)U;
        (void)top;
        (void)j0;
        (void)Dpad;
    }
}

// Software-pipelined chain (even G): a group is two halves of H = G/2 nodes held in two register
// sets A and B.  The LDS reads of the next half are issued before the current half's recurrence,
// so their latency hides behind it; the loop is unrolled by one group so A and B swap roles
// without register copies, and every read is unconditional (exact lgkm counts).
template <int SPL, int H>
struct UpHalf {
    static constexpr int CS = Split<SPL>::CS;
    double pr[H][CS], p1[H][CS], p2[H][CS], S[H][3];
    float cv[H][CS];
};

template <int SPL, int H>
__device__ __forceinline__ void up_half_read(const UpSlot<SPL>& sl, int k0, int e0, UpHalf<SPL, H>& r) {
    constexpr int CS = Split<SPL>::CS;
#pragma unroll
    for (int k = 0; k < H; ++k) {
        r.S[k][0] = sl.s[k0 + k].Sh;
        r.S[k][1] = sl.s[k0 + k].Sp1;
        r.S[k][2] = sl.s[k0 + k].Sp2;
        lds_read_at<CS>(sl.pre[k0 + k], e0, r.pr[k]);
        lds_read_at<CS>(sl.post1[k0 + k], e0, r.p1[k]);
        lds_read_at<CS>(sl.post2[k0 + k], e0, r.p2[k]);
#pragma unroll
        for (int q = 0; q < CS; ++q) r.cv[k][q] = sl.c[k0 + k][e0 + q];
    }
}

template <int SPL, int H>
__device__ __forceinline__ void up_half_step(UpSlot<SPL>& sl, uint32_t flags, int k0, int e0, const UpHalf<SPL, H>& r,
                                             double (&x)[Split<SPL>::CS]) {
    constexpr int CS = Split<SPL>::CS;
#pragma unroll
    for (int k = 0; k < H; ++k) {
        const bool hpre = (flags >> (3 * (k0 + k))) & UP_F_PRE;
        double acc[CS];
#pragma unroll
        for (int q = 0; q < CS; ++q) {
            acc[q] = __builtin_fma(r.S[k][0], x[q], hpre ? r.pr[k][q] : 0.0);
            acc[q] = __builtin_fma(r.S[k][1], r.p1[k][q], acc[q]);
            acc[q] = __builtin_fma(r.S[k][2], r.p2[k][q], acc[q]);
        }
#pragma unroll
        for (int q = 0; q < CS; ++q) x[q] = acc[q] + (double)r.cv[k][q];
        lds_write_at<CS>(sl.pre[k0 + k], e0, x);
    }
}

template <int SPL>
__device__ __forceinline__ void up_chain_wave(UpRing<SPL>& ring, int w, int head, int len, int lane,
                                              double* __restrict__ U, int Dpad, const double* x0) {
    constexpr int G = UpCfg<SPL>::G, NS = UpCfg<SPL>::NS, CS = Split<SPL>::CS;
    __builtin_amdgcn_s_setprio(3);
    unsigned spins = 0;
#ifdef SM_CHAIN_PROF
    const long long t0 = clock64();
    long long tr = 0, tc = 0;
#endif
    const int e0 = (w * 64 + lane) * CS;
    const int top = head + len - 1;  // chain node j sits at slot top - j (bottom first)
    const int ngroups = (len + G - 1) / G;
    double x[CS];
#pragma unroll
    for (int q = 0; q < CS; ++q) x[q] = x0 ? x0[e0 + q] : 0.0;  // a piece with a lower piece: its guessed input
    unsigned long long st = lds_state64(&ring.s[0].staged);  // poll-ahead: the next group's state
    int g0 = 0;
#ifdef SM_NO_PIPE
    if constexpr (false) {
#else
    if constexpr (G % 2 == 0) {
#endif
        // all full groups but the last through the pipeline; the last group (partial, or the tree
        // root's with a third post-heavy child) takes the generic path below
        constexpr int H = G / 2;
        UpHalf<SPL, H> A, B;
        while ((uint32_t)st != 1u) st = lds_state64(&ring.s[0].staged);
        uint32_t flags = uniform((uint32_t)(st >> 32));
        up_half_read<SPL, H>(ring.s[0], 0, e0, A);
        for (int g = 0; g + 1 < ngroups; ++g) {
            UpSlot<SPL>& sl = ring.s[g % NS];
            UpSlot<SPL>& sn = ring.s[(g + 1) % NS];
            st = lds_state64(&sn.staged);  // poll-ahead for group g+1
            up_half_read<SPL, H>(sl, H, e0, B);
            up_half_step<SPL, H>(sl, flags, 0, e0, A, x);
            while ((uint32_t)st != (uint32_t)(g + 2)) {
                PROF_SPIN(++spins);
                st = lds_state64(&sn.staged);
            }
            const uint32_t fnext = uniform((uint32_t)(st >> 32));
            up_half_read<SPL, H>(sn, 0, e0, A);
            up_half_step<SPL, H>(sl, flags, H, e0, B, x);
            lds_publish_ordered(&sl.done[w], g + 1);
            flags = fnext;
        }
        g0 = ngroups - 1;
        st = lds_state64(&ring.s[g0 % NS].staged);
    }
    for (int g = g0; g < ngroups; ++g) {
        UpSlot<SPL>& sl = ring.s[g % NS];
        const int n = min(G, len - g * G);
#ifdef SM_CHAIN_PROF
        const long long ta = clock64();
#endif
        while ((uint32_t)st != (uint32_t)(g + 1)) {
            PROF_SPIN(++spins);
            st = lds_state64(&sl.staged);
        }
        const uint32_t flags = uniform((uint32_t)(st >> 32));
#ifdef SM_CHAIN_PROF
        const long long tb = clock64();
        tr += tb - ta;
#endif
        // issued now, consumed after this group: its latency hides behind the group's work
        st = lds_state64(&ring.s[(g + 1) % NS].staged);
        if (n == G && !(flags & UP_F3)) {
            up_group<SPL, G, false>(sl, flags, 0, g * G, top, e0, x, U, Dpad);
        } else {
            for (int k = 0; k < n; ++k) up_group<SPL, 1, true>(sl, flags, k, g * G + k, top, e0, x, U, Dpad);
        }
        lds_publish_ordered(&sl.done[w], g + 1);
#ifdef SM_CHAIN_PROF
        tc += clock64() - tb;
#endif
    }
#ifdef SM_PROF_NOSTORE
    global_write_at<CS>(U, (uint32_t)top, Dpad, e0, x);  // keeps the recurrence alive
#endif
#ifdef SM_CHAIN_PROF
    if (blockIdx.x == 0 && lane == 0 && w == 0)
        printf("up chain view %d len %d cycles %lld spins %u wait %lld compute %lld\n", (int)blockIdx.y, len,
               clock64() - t0, spins, tr, tc);
#endif
    (void)spins;
}

// Helper waves: every global load of a group is unconditional (indices clamped, absent children
// read the path head's rows as L2-resident dummies), so the compiler's vmcnt bookkeeping stays
// exact and the loads stay in flight while the helper waits for its slot.  Per node a helper loads
// the light children's rows (at most two; a tree root's third through one row per group) and the
// image records, and computes off the chain, in registers:
//   Pre = the fold of the light children before the heavy one, from +0 in key order
//         (Stereo3DMST.cpp:125-137: acc = fma(S_c, A_up(c), acc));
//   C   = the AGD cost of the node's slices (or its ingested cost row);
// then stages Pre, the post-heavy rows, C and the weights into the slot.  Nothing of the up pass
// makes an HBM round trip other than the A_up rows themselves.
template <int SPL, bool AGD>
__device__ __forceinline__ void up_helper_wave(UpRing<SPL>& ring, int hh, int head, int len, int lane,
                                               const uint32_t* __restrict__ meta32, double* __restrict__ U,
                                               const UpCost& cs, int Dpad, bool lower, uint32_t* done_word,
                                               uint32_t epoch) {
    constexpr int G = UpCfg<SPL>::G, NS = UpCfg<SPL>::NS;
    constexpr int NCW = Split<SPL>::NCW;
    constexpr int NST = UP_STORERS, NL = Split<SPL>::NH - NST;  // storer / loader waves
    const int top = head + len - 1;
    const int ngroups = (len + G - 1) / G;
    if (hh >= NL) {
        // ---- storer: the chain's results of groups hh - NL (mod NST) go back to U, then the slot
        // is freed.  Its waves hold no loads, so its stores never delay a loader's load wait (gfx9
        // counts loads and stores in one vmcnt: a wave with both pending must wait for all of them)
#ifdef SM_CHAIN_PROF
        long long h_done = 0, h_t0 = clock64();
#endif
        for (int g = hh - NL; g < ngroups; g += NST) {
            const int n = min(G, len - g * G);
            UpSlot<SPL>& sl = ring.s[g % NS];
#ifdef SM_CHAIN_PROF
            long long h_d = clock64();
#endif
            lds_wait_all(sl.done, NCW, g + 1);
#ifdef SM_CHAIN_PROF
            h_done += clock64() - h_d;
#endif
#pragma unroll
            for (int k = 0; k < G; ++k) {  // unconditional (clamped rows are stored twice, same value)
                double xr[SPL];
                lds_row_read<SPL>(sl.pre[min(k, n - 1)], lane, xr);
                store_row<SPL>(U, (uint32_t)(top - (g * G + min(k, n - 1))), Dpad, lane, xr);
            }
            if (done_word && g == ngroups - 1) {
                // the piece's top row is the next piece's input: written through at device scope,
                // then its done word
                double xr[SPL];
                lds_row_read<SPL>(sl.pre[n - 1], lane, xr);
                double* row = U + (size_t)head * Dpad + lane * SPL;
                if (row_lane<SPL>(lane, Dpad))
#pragma unroll
                    for (int q = 0; q < SPL; ++q) __hip_atomic_store(row + q, xr[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                vm_drain();
                if (lane == 0) publish_word(done_word, epoch);
            }
            lds_publish(&sl.freed, g + 1);  // the rows are in flight from registers
        }
#ifdef SM_CHAIN_PROF
        if (blockIdx.x == 0 && lane == 0 && hh == NL)
            printf("up storer view %d len %d cycles %lld done %lld\n", (int)blockIdx.y, len, clock64() - h_t0, h_done);
#endif
        return;
    }
    // ---- loader: groups hh, hh + NL, ...
    int g = hh;
    if (g >= ngroups) return;
    // meta runs two groups ahead of the rows
    auto meta_of = [&](MetaVec<G>& m, int gg) {
        const int gc = gg < ngroups ? gg : g;  // unconditional prefetch (clamped)
        load_meta<G>(m, meta32, lane, top - gc * G, -1, min(G, len - gc * G));
    };
    MetaVec<G> mv, mnext;
    meta_of(mv, g);
    meta_of(mnext, g + NL);
    // light children of node k in key order: l0, l1; a third one (only a tree root with four
    // children) in l2 -- at most one such node per group
    double l0[G][SPL], l1[G][SPL], l2[SPL];
    float cr[G][SPL];
    ChainRecs<SPL, G> rec;
    auto issue = [&](int gg, const MetaVec<G>& m) {
        const int n = min(G, len - gg * G);
        uint32_t s2 = (uint32_t)head;
#pragma unroll
        for (int k = 0; k < G; ++k) {
            const int kk = min(k, n - 1);
            const uint32_t slot = (uint32_t)(top - (gg * G + kk));
            const uint32_t hi = mfield(m, kk, 3);
            const uint32_t nch = hi_nch(hi), hidx = hi_hidx(hi);
            const uint32_t nl = nch > 0 ? nch - 1u : 0u;
            const uint32_t c0 = nl >= 1 ? mfield(m, kk, hidx == 0 ? 5 : 4) : (uint32_t)head;
            const uint32_t c1 = nl >= 2 ? mfield(m, kk, hidx <= 1 ? 6 : 5) : (uint32_t)head + 1u;
            load_row<SPL>(U, c0, Dpad, lane, l0[k]);
            load_row<SPL>(U, c1, Dpad, lane, l1[k]);
            if constexpr (!AGD) load_crow<SPL>(cs.Cst, slot, Dpad, lane, cr[k]);
            if (nl >= 3) s2 = mfield(m, kk, hidx == 3 ? 6 : 7);
        }
        load_row<SPL>(U, s2, Dpad, lane, l2);
        if constexpr (AGD) chain_load_recs<SPL, G>(m, n, lane, cs, rec);
    };
    issue(g, mv);
#ifdef SM_CHAIN_PROF
    long long h_cost = 0, h_slot = 0, h_rest = 0, h_t0 = clock64();
#endif
    for (;;) {
        const int n = min(G, len - g * G);
#ifdef SM_CHAIN_PROF
        long long h_a = clock64();
#endif
        // ---- weights and presence flags (meta + LDS table only): before waiting for the slot;
        // lane q < 3 holds S of the heavy child (q = 0) / post q of node k
        double Sl[G];
        int k3 = -1;
        double S3 = 0.0;
        uint32_t flags = 0;
#pragma unroll
        for (int k = 0; k < G; ++k) {
            const uint32_t lo = mfield(mv, k, 2), hi = mfield(mv, k, 3);
            const uint32_t nch = hi_nch(hi), hidx = hi_hidx(hi);
            const uint32_t np = nch > 0 ? nch - 1u - hidx : 0u;
            const uint32_t i = hidx + (uint32_t)min(lane, 2);
            const bool live = lane == 0 ? (nch > 0 && (g * G + k > 0 || lower)) : (uint32_t)lane <= np;
            Sl[k] = ring.slut[live && lane < 3 ? cw_of(lo, hi, (int)min(i, 3u)) : (uint32_t)S_ZERO];
            if (k < n) {
                flags |= ((hidx > 0 ? UP_F_PRE : 0u) | (np >= 1 ? UP_F_P1 : 0u) | (np >= 2 ? UP_F_P2 : 0u)) << (3 * k);
                if (np >= 3) {
                    k3 = k;
                    S3 = ring.slut[cw_of(lo, hi, 3)];
                }
            }
        }
        MetaVec<G> mnn;
        meta_of(mnn, g + 2 * NL);
        const int gn = g + NL;
        const int gl = gn < ngroups ? gn : g;
        // ---- Pre and C of the group (registers; the loads have landed by now in all but the
        // first group, whose wait is here)
        if constexpr (AGD) chain_costs<SPL, G>(mv, cs, rec, ring.atab, cr);
        // Pre replaces l0 (with hidx >= 1 the first light child is a pre-heavy one, folded here)
#pragma unroll
        for (int k = 0; k < G; ++k) {
            const uint32_t lo = mfield(mv, k, 2), hi = mfield(mv, k, 3);
            const uint32_t hidx = hi_hidx(hi);
            if (hidx >= 1) {  // uniform: positions 0 .. hidx-1 are the light children l0, l1, l2
                const double S0 = ring.slut[cw_of(lo, hi, 0)];
#pragma unroll
                for (int q = 0; q < SPL; ++q) l0[k][q] = __builtin_fma(S0, l0[k][q], 0.0);
                if (hidx >= 2) {
                    const double S1 = ring.slut[cw_of(lo, hi, 1)];
#pragma unroll
                    for (int q = 0; q < SPL; ++q) l0[k][q] = __builtin_fma(S1, l1[k][q], l0[k][q]);
                    if (hidx >= 3) {
                        const double S2 = ring.slut[cw_of(lo, hi, 2)];
#pragma unroll
                        for (int q = 0; q < SPL; ++q) l0[k][q] = __builtin_fma(S2, l2[q], l0[k][q]);
                    }
                }
            }
        }
#ifdef SM_CHAIN_PROF
        {
            double t = 0;
#pragma unroll
            for (int k = 0; k < G; ++k) t += l0[k][0] + (double)cr[k][0];
            if (t == -1.0) h_rest += 1;  // keeps the stamp after the values are ready
        }
        long long h_b = clock64();
        h_cost += h_b - h_a;
#endif
        // ---- wait for the slot, fill it, publish
        UpSlot<SPL>& sl = ring.s[g % NS];
        if (g >= NS) lds_wait(&sl.freed, g - NS + 1, true);
#ifdef SM_CHAIN_PROF
        long long h_c = clock64();
        h_slot += h_c - h_b;
#endif
#pragma unroll
        for (int k = 0; k < G; ++k) {
            if (k < n) {
                const uint32_t f = flags >> (3 * k);
                const uint32_t hidx = hi_hidx(mfield(mv, k, 3));
                if (f & UP_F_PRE) lds_row_write<SPL>(sl.pre[k], lane, l0[k]);
                // post-heavy rows: the light children from index hidx on
                if (f & UP_F_P1) {
                    if (hidx == 0)
                        lds_row_write<SPL>(sl.post1[k], lane, l0[k]);
                    else if (hidx == 1)
                        lds_row_write<SPL>(sl.post1[k], lane, l1[k]);
                    else
                        lds_row_write<SPL>(sl.post1[k], lane, l2);
                }
                if (f & UP_F_P2) {
                    if (hidx == 0)
                        lds_row_write<SPL>(sl.post2[k], lane, l1[k]);
                    else
                        lds_row_write<SPL>(sl.post2[k], lane, l2);
                }
#pragma unroll
                for (int q = 0; q < SPL; ++q) sl.c[k][lane * SPL + q] = cr[k][q];
                if (lane < 3) (&sl.s[k].Sh)[lane] = Sl[k];
            }
        }
        if (k3 >= 0) {  // a third post-heavy child: hidx == 0 and three light children
            lds_row_write<SPL>(sl.post3, lane, l2);
            flags |= UP_F3;
        }
        if (lane == 0) {
            sl.k3 = k3;
            sl.S3 = S3;
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the group's rows have landed
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        __hip_atomic_store(&sl.staged, ((unsigned long long)flags << 32) | (unsigned)(g + 1), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        // ---- the next group's loads go out now
        issue(gl, mnext);
        if (gn >= ngroups) break;
        g = gn;
        mv = mnext;
        mnext = mnn;
    }
#ifdef SM_CHAIN_PROF
    if (blockIdx.x == 0 && lane == 0 && hh == 0)
        printf("up loader view %d len %d cycles %lld cost+loads %lld slot %lld\n", (int)blockIdx.y, len, clock64() - h_t0,
               h_cost, h_slot);
#endif
}

// ---------------------------------------------------------------------------------------------
// Pieces.  A long path of L >= 2*SM_PIECE nodes is cut into M = L / SM_PIECE pieces (piece 0 at
// the head; the bottom piece takes the remainder), one workgroup each, so the serial critical
// path of a round is ~SM_PIECE nodes instead of L.  A piece other than the bottom one does not
// know its input (the top row of the piece below) when it starts, so:
//   1. guess: k_up_pre left per-segment affine aggregates (x_top = P * x_below + B, approximate)
//      for the path; the piece folds those of every segment below it into a guessed input;
//   2. speculate: the chain runs the piece from the guess with the exact per-node arithmetic,
//      and the piece's top row goes out at device scope with a done word;
//   3. repair: once the piece below is done, one wave re-runs the piece's first nodes from the
//      true input with the same operations and compares bitwise with the stored rows.  Two
//      trajectories of the same deterministic recurrence that agree at one node agree from there
//      on, so the first node whose recomputed row equals the stored row ends the repair (the
//      guess is within a few ulp, so this takes a handful of nodes);
//   4. decoupled look-back: the repair is exact iff the input was, i.e. iff every piece below
//      merged.  Each piece publishes merged / not merged, then reads the words of the pieces
//      below: all merged -> commit the buffered corrections.  Otherwise (never seen; correctness
//      only) it waits for the piece below to be final and re-walks the whole piece from the now
//      exact input, writing through, and publishes final.
// A piece waits only on pieces of lower block index (listed bottom first), so the lowest
// unfinished piece always progresses.  All waits are bounded (~1 s): a bug shows up as a parity
// failure, not a hang.  Status words hold the filter call's epoch, so nothing is reset per call.
// ---------------------------------------------------------------------------------------------

// rows of a cut path's nodes (the fix buffer, 32 rows per segment, WalkArgs::fix): node slot s of the
// path whose first segment is f (bucket-relative, the piece entry's .w) has row s + off, off = 32 f - head
struct FixRows {
    double* p;      // the bucket's first row (nullptr: write through / none)
    long long off;  // row = slot + off
    __device__ uint32_t row(uint32_t slot) const { return (uint32_t)((long long)slot + off); }
};

struct PieceView {
    const uint4* pieces;  // {path, j, M, first segment of the path} per piece, bottom piece first
    int npieces;
    const double* agg;    // per bucket segment: [P row | B row]
    double* fix;          // the bucket's fix rows (FixRows): up repair corrections, down pieces' last rows
    uint32_t* stat;       // done [i], merged [i + stride], final [i + 2 * stride]
    int stride;
    int plen;             // nodes per piece
    int rmax;             // nodes a fast repair may take (tests: force the slow path)
    unsigned long long* dbg;  // SM_PIECE_DEBUG: [fast, slow, sum of repair nodes, max, guess cycles, finish cycles]
    uint32_t* err;        // the call's error word (host-mapped): bit 0 = a cross-workgroup wait timed out
    int wait_iters;       // polls before a wait gives up
};

template <int SPL>
__device__ __forceinline__ void agent_row_read(const double* U, uint32_t slot, int Dpad, int lane, double (&r)[SPL]) {
    const double* p = U + (size_t)slot * Dpad + lane * SPL;
#pragma unroll
    for (int q = 0; q < SPL; ++q)
        r[q] = row_lane<SPL>(lane, Dpad) ? __hip_atomic_load(p + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0;
}
template <int SPL>
__device__ __forceinline__ void agent_row_write(double* U, uint32_t slot, int Dpad, int lane, const double (&r)[SPL]) {
    double* p = U + (size_t)slot * Dpad + lane * SPL;
    if (row_lane<SPL>(lane, Dpad))
#pragma unroll
        for (int q = 0; q < SPL; ++q) __hip_atomic_store(p + q, r[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// guessed input of a piece: fold of the ns segment aggregates below it (agg = the first of them,
// the top-most), split over the 16 waves and combined in LDS (scratch: 16 x 2 rows).  Ends with a
// barrier; the result row is in guess[].
template <int SPL>
__device__ void up_guess(double* scratch, double* guess, const double* __restrict__ agg, int ns, int Dpad, int wave,
                         int lane) {
    const int per = (ns + CHN_WAVES - 1) / CHN_WAVES;
    const int s0 = min(ns, wave * per), s1 = min(ns, s0 + per);
    double P[SPL], B[SPL];
#pragma unroll
    for (int k = 0; k < SPL; ++k) {
        P[k] = 1.0;
        B[k] = 0.0;
    }
    for (int s = s1 - 1; s >= s0; s -= 4) {  // bottom up, 4 segments' loads at a time
        double pr[4][SPL], br[4][SPL];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int ss = max(s - q, s0);
            load_row<SPL>(agg + (size_t)ss * 2 * Dpad, 0, Dpad, lane, pr[q]);
            load_row<SPL>(agg + (size_t)ss * 2 * Dpad + Dpad, 0, Dpad, lane, br[q]);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (s - q >= s0) {
#pragma unroll
                for (int k = 0; k < SPL; ++k) {
                    B[k] = __builtin_fma(pr[q][k], B[k], br[q][k]);
                    P[k] = pr[q][k] * P[k];
                }
            }
        }
    }
    double* my = scratch + (size_t)wave * 2 * 64 * SPL;
#pragma unroll
    for (int k = 0; k < SPL; ++k) {
        my[lane * SPL + k] = P[k];
        my[64 * SPL + lane * SPL + k] = B[k];
    }
    __syncthreads();
    if (wave == 0) {
        double x[SPL];
#pragma unroll
        for (int k = 0; k < SPL; ++k) x[k] = 0.0;
        for (int w = CHN_WAVES - 1; w >= 0; --w) {
            const double* t = scratch + (size_t)w * 2 * 64 * SPL;
#pragma unroll
            for (int k = 0; k < SPL; ++k) x[k] = __builtin_fma(t[lane * SPL + k], x[k], t[64 * SPL + lane * SPL + k]);
        }
#pragma unroll
        for (int k = 0; k < SPL; ++k) guess[lane * SPL + k] = x[k];
    }
    __syncthreads();
}

// Exact re-walk of a piece's chain nodes 0 .. nmax-1 (slot top - n, bottom first) from the input
// row x (lane * SPL layout), with the reference's operations in the chain engine's order:
// the light children before the heavy one folded from +0 (k_up_pre's Pre), acc = fma(S_h, x, .),
// the light children after it, x = acc + C.  Compares every node with the stored row; returns the
// first node where all lanes agree (the nodes before it were corrected), or -1.  Corrections go
// to the same slot of fix[] or, with fix == nullptr, straight to U at device scope.  Batches of
// CHR nodes: the next batch's metadata is in flight during a batch, the first light child row of
// every node is loaded with the batch, further light children (rare) on demand.
#ifndef UP_WALK_CH
#define UP_WALK_CH(SPL) ((SPL) == 4 ? 2 : 6)  // nodes per repair batch (registers: the image records)
#endif
template <int SPL, int CHR, bool AGD>
__device__ __forceinline__ int up_exact_walk(const uint32_t* __restrict__ meta32, double* __restrict__ U,
                                          const UpCost& cs, const double* slut, const float* atab, int top, int nmax,
                                          int Dpad, int lane, double* xio, FixRows fix, bool write,
                                          double* lfix = nullptr, int lcap = 0) {
    double x[SPL];
#pragma unroll
    for (int q = 0; q < SPL; ++q) x[q] = xio[q];
    MetaVec<CHR> mv;
    load_meta<CHR>(mv, meta32, lane, top, -1, min(CHR, nmax));
    for (int n0 = 0; n0 < nmax; n0 += CHR) {
        const int nb = min(CHR, nmax - n0);
        MetaVec<CHR> mn;
        const int n1 = n0 + CHR < nmax ? n0 + CHR : n0;
        load_meta<CHR>(mn, meta32, lane, top - n1, -1, min(CHR, nmax - n1));
        double spec[CHR][SPL], r0[CHR][SPL];
        float cr[CHR][SPL];
        ChainRecs<SPL, CHR> rec;
#pragma unroll
        for (int k = 0; k < CHR; ++k) {
            const int kk = min(k, nb - 1);
            const uint32_t slot = (uint32_t)(top - (n0 + kk));
            const uint32_t hi = mfield(mv, kk, 3);
            const int nch = (int)hi_nch(hi), hidx = (int)hi_hidx(hi);
            load_row<SPL>(U, nch >= 2 ? mfield(mv, kk, hidx > 0 ? 4 : 5) : slot, Dpad, lane, r0[k]);  // first light child
            if constexpr (!AGD) load_crow<SPL>(cs.Cst, slot, Dpad, lane, cr[k]);
            agent_row_read<SPL>(U, slot, Dpad, lane, spec[k]);  // own piece's rows (this launch)
        }
        if constexpr (AGD) {
            chain_load_recs<SPL, CHR>(mv, nb, lane, cs, rec);
            chain_costs<SPL, CHR>(mv, cs, rec, atab, cr);
        }
#pragma unroll
        for (int k = 0; k < CHR; ++k) {
            if (k >= nb) break;
            const uint32_t lo = mfield(mv, k, 2), hi = mfield(mv, k, 3);
            const int nch = (int)hi_nch(hi), hidx = (int)hi_hidx(hi);
            double acc[SPL];
#pragma unroll
            for (int q = 0; q < SPL; ++q) acc[q] = 0.0;
            bool first = true;
#pragma unroll
            for (int pos = 0; pos < 4; ++pos) {
                if (pos >= nch) break;
                const double S = slut[cw_of(lo, hi, pos)];
                if (pos == hidx) {
#pragma unroll
                    for (int q = 0; q < SPL; ++q) acc[q] = __builtin_fma(S, x[q], acc[q]);
                } else {
                    double r[SPL];
                    if (first) {
#pragma unroll
                        for (int q = 0; q < SPL; ++q) r[q] = r0[k][q];
                        first = false;
                    } else {
                        load_row<SPL>(U, mfield(mv, k, 4 + pos), Dpad, lane, r);
                    }
#pragma unroll
                    for (int q = 0; q < SPL; ++q) acc[q] = __builtin_fma(S, r[q], acc[q]);
                }
            }
            bool eq = true;
#pragma unroll
            for (int q = 0; q < SPL; ++q) {
                x[q] = acc[q] + (double)cr[k][q];
                // lanes beyond a 32-double row hold nothing (cost 3.0 there, stored rows read 0)
                eq = eq && (!row_lane<SPL>(lane, Dpad) || __double_as_longlong(x[q]) == __double_as_longlong(spec[k][q]));
            }
            if (__all(eq)) return n0 + k;
            if (!write) continue;
            const uint32_t slot = (uint32_t)(top - (n0 + k));
            if (n0 + k < lcap)  // buffered in LDS (the free ring): no global store between the batches'
                lds_row_write<SPL>(lfix + (size_t)(n0 + k) * 64 * SPL, lane, x);  // loads and their waits
            else if (fix.p)
                store_row<SPL>(fix.p, fix.row(slot), Dpad, lane, x);
            else
                agent_row_write<SPL>(U, slot, Dpad, lane, x);
        }
        mv = mn;
    }
    return -1;
}

// ---------------------------------------------------------------------------------------------
// Cooperative up repair (round 2).  A piece's repair re-walks its first nodes from the true input
// until the trajectory meets the stored one (see "Pieces").  One wave doing that alone pays a
// memory round trip per batch of nodes (loads, costs, then the recurrence): ~0.6 us per node, and a
// 210-node repair set the end of its whole round.  Here all 16 waves of the workgroup (idle once
// the chain is done) stage the inputs of B nodes at a time into the free ring's LDS -- exactly
// what the loaders stage for the chain: Pre, the post-heavy rows, the cost row, the weights, plus
// the stored row to compare with -- and wave 0 runs the recurrence over them from LDS.
// ---------------------------------------------------------------------------------------------
template <int SPL>
struct RepNode {
    double pre[64 * SPL];   // Pre (pre-heavy fold), valid iff flags & UP_F_PRE
    double p1[64 * SPL];    // first post-heavy row (iff UP_F_P1)
    double p2[64 * SPL];    // second post-heavy row (iff UP_F_P2)
    double spec[64 * SPL];  // the row the chain stored (speculative trajectory)
    float c[64 * SPL];      // cost row
    double S[4];            // S of the heavy child (0 if none), post 1, post 2, post 3
    uint32_t flags;         // UP_F_PRE | UP_F_P1 | UP_F_P2 | UP_F3 (third post row: loaded by wave 0)
    uint32_t c3;            // slot of the third post-heavy child (UP_F3)
};

template <int SPL>
struct RepCfg {
    static constexpr size_t RING = sizeof(UpRing<SPL>::s);
    static constexpr int B0 = (int)(RING / sizeof(RepNode<SPL>));
    static constexpr int BB = B0 / 2 < 16 ? B0 / 2 : 16;  // nodes per pass; two passes' buffers
    // waves 1 .. 15 stage (wave 0's correction stores then never share a vmcnt with loads)
    static constexpr int NSW = CHN_WAVES - 1;
    static constexpr int CHR = (BB + NSW - 1) / NSW;  // nodes staged per wave and pass
    static_assert(BB >= 4, "repair pass");
};
// the repair batch follows the ring's size; its value at the shipped geometries is pinned here, so a
// ring sweep that changes it is visible (SPL=1 4 x 10 ring, 78 KB -> still 16-node passes)
static_assert(UP_G1 != 4 || UP_NS1 != 10 || RepCfg<1>::BB == 16, "RepCfg<1>::BB changed with the SPL=1 ring");

// one wave stages nodes k0 .. k0+nb-1 (node k = slot top - k; metadata in mv) into rn[k - kb]
template <int SPL, bool AGD, int CHR>
__device__ __forceinline__ void up_repair_stage(RepNode<SPL>* rn, int kb, int k0, int nb, const MetaVec<CHR>& mv,
                                                int top, int lane, const double* __restrict__ U, const UpCost& cs,
                                                const double* slut, const float* atab, int Dpad, int head) {
    double l0[CHR][SPL], l1[CHR][SPL], l2[SPL], sp[CHR][SPL];
    float cr[CHR][SPL];
    ChainRecs<SPL, CHR> rec;
    uint32_t s2 = (uint32_t)head;
#pragma unroll
    for (int k = 0; k < CHR; ++k) {
        const int kk = min(k, nb - 1);
        const uint32_t slot = (uint32_t)(top - (k0 + kk));
        const uint32_t hi = mfield(mv, kk, 3);
        const uint32_t nch = hi_nch(hi), hidx = hi_hidx(hi);
        const uint32_t nl = nch > 0 ? nch - 1u : 0u;
        load_row<SPL>(U, nl >= 1 ? mfield(mv, kk, hidx == 0 ? 5 : 4) : (uint32_t)head, Dpad, lane, l0[k]);
        load_row<SPL>(U, nl >= 2 ? mfield(mv, kk, hidx <= 1 ? 6 : 5) : (uint32_t)head, Dpad, lane, l1[k]);
        if constexpr (!AGD) load_crow<SPL>(cs.Cst, slot, Dpad, lane, cr[k]);
        agent_row_read<SPL>(U, slot, Dpad, lane, sp[k]);  // this launch's stored rows
        if (nl >= 3) s2 = mfield(mv, kk, hidx == 3 ? 6 : 7);  // a root's third light row
    }
    load_row<SPL>(U, s2, Dpad, lane, l2);
    if constexpr (AGD) {
        chain_load_recs<SPL, CHR>(mv, nb, lane, cs, rec);
        chain_costs<SPL, CHR>(mv, cs, rec, atab, cr);
    }
#pragma unroll
    for (int k = 0; k < CHR; ++k) {
        if (k >= nb) break;
        RepNode<SPL>& r = rn[k0 + k - kb];
        const uint32_t lo = mfield(mv, k, 2), hi = mfield(mv, k, 3);
        const uint32_t nch = hi_nch(hi), hidx = hi_hidx(hi);
        const uint32_t np = nch > 0 ? nch - 1u - hidx : 0u;
        // Pre: the light children before the heavy one, from +0 in key order (uniform branches)
        double pre[SPL];
#pragma unroll
        for (int q = 0; q < SPL; ++q) pre[q] = 0.0;
        if (hidx >= 1) {
            const double S0 = slut[cw_of(lo, hi, 0)];
#pragma unroll
            for (int q = 0; q < SPL; ++q) pre[q] = __builtin_fma(S0, l0[k][q], 0.0);
            if (hidx >= 2) {
                const double S1 = slut[cw_of(lo, hi, 1)];
#pragma unroll
                for (int q = 0; q < SPL; ++q) pre[q] = __builtin_fma(S1, l1[k][q], pre[q]);
                if (hidx >= 3) {
                    const double S2 = slut[cw_of(lo, hi, 2)];
#pragma unroll
                    for (int q = 0; q < SPL; ++q) pre[q] = __builtin_fma(S2, l2[q], pre[q]);
                }
            }
        }
        uint32_t flags = (hidx > 0 ? UP_F_PRE : 0u) | (np >= 1 ? UP_F_P1 : 0u) | (np >= 2 ? UP_F_P2 : 0u);
        if (flags & UP_F_PRE) lds_row_write<SPL>(r.pre, lane, pre);
        if (np >= 1) {
            if (hidx == 0)
                lds_row_write<SPL>(r.p1, lane, l0[k]);
            else if (hidx == 1)
                lds_row_write<SPL>(r.p1, lane, l1[k]);
            else
                lds_row_write<SPL>(r.p1, lane, l2);
        }
        if (np >= 2) {
            if (hidx == 0)
                lds_row_write<SPL>(r.p2, lane, l1[k]);
            else
                lds_row_write<SPL>(r.p2, lane, l2);
        }
        lds_row_write<SPL>(r.spec, lane, sp[k]);
#pragma unroll
        for (int q = 0; q < SPL; ++q) r.c[lane * SPL + q] = cr[k][q];
        if (lane < 4) {
            // lane 0: the heavy child (always live here: a repaired piece has a lower piece), 1..3:
            // the post-heavy children
            const bool live = lane == 0 ? nch > 0 : (uint32_t)lane <= np;
            const uint32_t pos = min(hidx + (uint32_t)lane, 3u);
            r.S[lane] = slut[live ? cw_of(lo, hi, (int)pos) : (uint32_t)S_ZERO];
        }
        if (np >= 3) flags |= UP_F3;
        if (lane == 0) {
            r.flags = flags;
            r.c3 = np >= 3 ? mfield(mv, k, 7) : 0u;
        }
    }
}

// All waves: the repair walk of nodes 0 .. nmax-1.  Waves 1 .. 15 stage pass p+1 (metadata one
// pass further ahead, so one memory round trip per pass) while wave 0 runs the recurrence over
// pass p from LDS; pass 0 is staged while wave 0 runs pro(x), which produces the input row (the
// wait for the piece below).  Corrections go to fix[] (write == 1) or through U at device scope
// (write == 2), none with write == 0 (probe).  Returns (to every wave) the first node where the
// recomputed row equals the stored one, or -1.
template <int SPL, bool AGD, class Pro>
__device__ int up_repair_coop(UpRing<SPL>& ring, int* res2, const uint32_t* __restrict__ meta32, double* __restrict__ U,
                              FixRows fix, const UpCost& cs, int Dpad, int wave, int lane, int top, int nmax,
                              int head, int write, Pro&& pro) {
    constexpr int BB = RepCfg<SPL>::BB, CHR = RepCfg<SPL>::CHR;
    RepNode<SPL>* rn = reinterpret_cast<RepNode<SPL>*>(ring.s);
    const int npass = (nmax + BB - 1) / BB;
    const int sw = (wave - 1) * CHR;  // a stager's first node within a pass
    MetaVec<CHR> mv, mn;
    auto meta = [&](MetaVec<CHR>& m, int p) {
        const int n = min(CHR, min(nmax, (p + 1) * BB) - (p * BB + sw));
        if (p < npass && n > 0) load_meta<CHR>(m, meta32, lane, top - (p * BB + sw), -1, n);
    };
    auto stage = [&](int p) {
        const int n = min(CHR, min(nmax, (p + 1) * BB) - (p * BB + sw));
        if (n > 0)
            up_repair_stage<SPL, AGD, CHR>(rn + (p & 1) * BB, p * BB, p * BB + sw, n, mv, top, lane, U, cs, ring.slut,
                                           ring.atab, Dpad, head);
    };
    double x[SPL];
    if (wave > 0) {
        meta(mv, 0);
        meta(mn, 1);
        stage(0);
        mv = mn;
    } else {
        pro(x);
    }
    __syncthreads();
    int out = -1;
    for (int p = 0; p < npass; ++p) {
        if (wave == 0) {
            const int n0 = p * BB, nb = min(BB, nmax - n0);
            const RepNode<SPL>* rb = rn + (p & 1) * BB;
            int m = -1;
            for (int k = 0; k < nb; ++k) {
                const RepNode<SPL>& r = rb[k];
                const uint32_t flags = uniform(r.flags);
                const double Sh = r.S[0], S1 = r.S[1], S2 = r.S[2];
                double acc[SPL];
#pragma unroll
                for (int q = 0; q < SPL; ++q) {
                    acc[q] = __builtin_fma(Sh, x[q], (flags & UP_F_PRE) ? r.pre[lane * SPL + q] : 0.0);
                    acc[q] = __builtin_fma(S1, (flags & UP_F_P1) ? r.p1[lane * SPL + q] : 0.0, acc[q]);
                    acc[q] = __builtin_fma(S2, (flags & UP_F_P2) ? r.p2[lane * SPL + q] : 0.0, acc[q]);
                }
                if (flags & UP_F3) {  // a tree root's third post-heavy child (rare): loaded here
                    double r3[SPL];
                    load_row<SPL>(U, uniform(r.c3), Dpad, lane, r3);
#pragma unroll
                    for (int q = 0; q < SPL; ++q) acc[q] = __builtin_fma(r.S[3], r3[q], acc[q]);
                }
                bool eq = true;
#pragma unroll
                for (int q = 0; q < SPL; ++q) {
                    x[q] = acc[q] + (double)r.c[lane * SPL + q];
                    eq = eq && (!row_lane<SPL>(lane, Dpad) ||
                                __double_as_longlong(x[q]) == __double_as_longlong(r.spec[lane * SPL + q]));
                }
                if (__all(eq)) {
                    m = n0 + k;
                    break;
                }
                const uint32_t slot = (uint32_t)(top - (n0 + k));
                if (write == 1)
                    store_row<SPL>(fix.p, fix.row(slot), Dpad, lane, x);
                else if (write == 2)
                    agent_row_write<SPL>(U, slot, Dpad, lane, x);
            }
            // res2[p & 1]: rewritten two passes later, after every wave has passed the barrier below
            if (lane == 0) res2[p & 1] = m >= 0 ? m : (p + 1 >= npass ? -1 : -2);
        } else if (p + 1 < npass) {
            meta(mn, p + 2);
            stage(p + 1);
            mv = mn;
        }
        __syncthreads();
        const int r = res2[p & 1];
        if (r != -2) {
            out = r;
            break;
        }
    }
    if (wave == 0) vm_drain();  // corrections stored
    return out;
}

// Repair + look-back of piece e (one wave, after its chain).  j of M, bottom piece first: the
// pieces below are entries e - (M-1-j) .. e - 1, the bottom one exact by construction.  A piece
// "merged" iff its repair met the stored trajectory below its top node, i.e. its top row (the
// next piece's input) never changes; every input of a piece is then exact iff all pieces below
// merged.
template <int SPL, bool AGD>
__device__ void up_finish(UpRing<SPL>& ring, int* hdone, const uint32_t* __restrict__ meta32, double* __restrict__ U,
                          FixRows fix, const UpCost& cs, int Dpad, int lane, int head, int len, int j, int M,
                          int e, const PieceView& Q, uint32_t epoch) {
    uint32_t* done = Q.stat;
    uint32_t* merged = Q.stat + Q.stride;
    uint32_t* fin = Q.stat + 2 * Q.stride;
    if (j + 1 == M) {  // bottom piece
        if (lane == 0) publish_word(fin + e, epoch);
        return;
    }
    // the helpers are done: this piece's rows are stored
    while (__hip_atomic_load(hdone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < Split<SPL>::NH) __builtin_amdgcn_s_sleep(1);
    const int top = head + len - 1;
    const uint32_t below = (uint32_t)(head + len);  // top node of the piece below
    double x[SPL];
#ifdef SM_CHAIN_TIMES
    const unsigned long long tf0 = __builtin_amdgcn_s_memrealtime();
#endif
    wait_word(done + e - 1, epoch, epoch, Q.err, Q.wait_iters);
    vm_drain();
    agent_row_read<SPL>(U, below, Dpad, lane, x);
    vm_drain();
#ifdef SM_CHAIN_TIMES
    const unsigned long long tf1 = __builtin_amdgcn_s_memrealtime();
#endif
    if (Q.dbg && Q.dbg[15] == 1) {  // probe (SM_PIECE_DEBUG=2): merge distance histogram, no writes
        const int mp = up_exact_walk<SPL, UP_WALK_CH(SPL), AGD>(meta32, U, cs, ring.slut, ring.atab, top, len, Dpad, lane, x, FixRows{nullptr, 0}, false);
        int b = 8;  // 8: < 8 nodes, 9: < 16, ... 13: >= 128 (merged), 14: never merged
        while (b < 13 && mp >= (8 << (b - 8))) ++b;
        if (lane == 0) atomicAdd(Q.dbg + (mp < 0 ? 14 : b), 1ull);
    }
    // corrections of the first lcap nodes stay in the ring's LDS (free now: the helpers are done);
    // a global store per corrected node made every batch's loads wait for the previous batch's
    // stores (one vmcnt for both), two memory latencies per batch on the round's critical path
    double* lfix = reinterpret_cast<double*>(ring.s);
    constexpr int lcap = (int)(sizeof(ring.s) / (64 * SPL * sizeof(double)));
    const int m = up_exact_walk<SPL, UP_WALK_CH(SPL), AGD>(meta32, U, cs, ring.slut, ring.atab, top, min(Q.rmax, len), Dpad, lane, x,
                                                           fix, true, lfix, lcap);
    if (lane == 0) publish_word(merged + e, 2u * epoch + (m >= 0 ? 0u : 1u));
#ifdef SM_CHAIN_TIMES
    const unsigned long long tf2 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
        ct_log(2, (int)blockIdx.y, M, m, e, tf0, tf1);  // waiting for the piece below
        ct_log(3, (int)blockIdx.y, M, m, e, tf1, tf2);  // the repair walk (len field: merge node)
    }
#endif
    bool all = m >= 0;
    for (int q = e - 1; all && q > e - (M - 1 - j); --q) all = wait_word(merged + q, 2u * epoch, 2u * epoch + 1u, Q.err, Q.wait_iters) == 2u * epoch;
    if (Q.dbg && lane == 0) {
        atomicAdd(Q.dbg + (all ? 0 : 1), 1ull);
        if (m >= 0) {
            atomicAdd(Q.dbg + 2, (unsigned long long)m);
            atomicMax(Q.dbg + 3, (unsigned long long)m);
        }
    }
    if (all) {  // commit the corrections
        for (int k = 0; k < m; ++k) {
            double r[SPL];
            if (k < lcap)
                lds_row_read<SPL>(lfix + (size_t)k * 64 * SPL, lane, r);
            else
                load_row<SPL>(fix.p, fix.row((uint32_t)(top - k)), Dpad, lane, r);
            store_row<SPL>(U, (uint32_t)(top - k), Dpad, lane, r);
        }
        if (lane == 0) publish_word(fin + e, epoch);
        return;
    }
    // slow path: the piece below is final (exact); repair again from its final top row, writing
    // through (the stored rows are still the chain's trajectory: nothing was committed)
    wait_word(fin + e - 1, epoch, epoch, Q.err, Q.wait_iters);
    vm_drain();
    agent_row_read<SPL>(U, below, Dpad, lane, x);
    vm_drain();
    up_exact_walk<SPL, UP_WALK_CH(SPL), AGD>(meta32, U, cs, ring.slut, ring.atab, top, len, Dpad, lane, x, FixRows{nullptr, 0}, true);
    vm_drain();
    if (lane == 0) publish_word(fin + e, epoch);
}

// Repair + look-back of piece e with all waves (see up_finish for the protocol; wave 0 handles the
// status words, the walk is up_repair_coop).  xin: the guess buffer, free after the chain.
template <int SPL, bool AGD>
__device__ void up_finish_coop(UpRing<SPL>& ring, double* xin, const uint32_t* __restrict__ meta32, double* __restrict__ U,
                               FixRows fix, const UpCost& cs, int Dpad, int wave, int lane, int head, int len,
                               int j, int M, int e, const PieceView& Q, uint32_t epoch) {
    uint32_t* done = Q.stat;
    uint32_t* merged = Q.stat + Q.stride;
    uint32_t* fin = Q.stat + 2 * Q.stride;
    __shared__ int res2[2];
    if (j + 1 == M) {  // bottom piece
        if (wave == 0 && lane == 0) publish_word(fin + e, epoch);
        return;
    }
    const int top = head + len - 1;
    const uint32_t below = (uint32_t)(head + len);  // top node of the piece below
#ifdef SM_CHAIN_TIMES
    const unsigned long long tf0 = __builtin_amdgcn_s_memrealtime();
    unsigned long long tf1 = tf0;
#endif
    // wave 0: the true input, the final row of the piece below's top node once it is stored
    auto input = [&](double (&x)[SPL], const uint32_t* word) {
        wait_word(word, epoch, epoch, Q.err, Q.wait_iters);
        vm_drain();
        agent_row_read<SPL>(U, below, Dpad, lane, x);
        vm_drain();
#ifdef SM_CHAIN_TIMES
        tf1 = __builtin_amdgcn_s_memrealtime();
#endif
    };
    const bool probe = Q.dbg && Q.dbg[15] == 1;  // SM_PIECE_DEBUG=2: merge distance histogram, no writes
    if (probe) {
        const int mp = up_repair_coop<SPL, AGD>(ring, res2, meta32, U, fix, cs, Dpad, wave, lane, top, len, head, 0,
                                                [&](double (&x)[SPL]) {
                                                    input(x, done + e - 1);
                                                    lds_row_write<SPL>(xin, lane, x);
                                                });
        int b = 8;  // 8: < 8 nodes, 9: < 16, ... 13: >= 128 (merged), 14: never merged
        while (b < 13 && mp >= (8 << (b - 8))) ++b;
        if (wave == 0 && lane == 0) atomicAdd(Q.dbg + (mp < 0 ? 14 : b), 1ull);
    }
    const int m = up_repair_coop<SPL, AGD>(ring, res2, meta32, U, fix, cs, Dpad, wave, lane, top, min(Q.rmax, len), head, 1,
                                           [&](double (&x)[SPL]) {
                                               if (probe)
                                                   lds_row_read<SPL>(xin, lane, x);
                                               else
                                                   input(x, done + e - 1);
                                           });
#ifdef SM_CHAIN_TIMES
    if (wave == 0 && lane == 0) {
        const unsigned long long tf2 = __builtin_amdgcn_s_memrealtime();
        ct_log(2, (int)blockIdx.y, M, m, e, tf0, tf1);  // waiting for the piece below
        ct_log(3, (int)blockIdx.y, M, m, e, tf1, tf2);  // the repair walk (len field: merge node)
    }
#endif
    __shared__ int all_s;
    if (wave == 0) {
        if (lane == 0) publish_word(merged + e, 2u * epoch + (m >= 0 ? 0u : 1u));
        bool all = m >= 0;
        for (int q = e - 1; all && q > e - (M - 1 - j); --q)
            all = wait_word(merged + q, 2u * epoch, 2u * epoch + 1u, Q.err, Q.wait_iters) == 2u * epoch;
        if (Q.dbg && lane == 0) {
            atomicAdd(Q.dbg + (all ? 0 : 1), 1ull);
            if (m >= 0) {
                atomicAdd(Q.dbg + 2, (unsigned long long)m);
                atomicMax(Q.dbg + 3, (unsigned long long)m);
            }
        }
        if (lane == 0) all_s = all ? 1 : 0;
    }
    __syncthreads();
    if (all_s) {  // commit the corrections: rows 0 .. m-1 from fix, spread over the waves
        for (int k = wave; k < m; k += CHN_WAVES) {
            double r[SPL];
            load_row<SPL>(fix.p, fix.row((uint32_t)(top - k)), Dpad, lane, r);
            store_row<SPL>(U, (uint32_t)(top - k), Dpad, lane, r);
        }
        vm_drain();
        __syncthreads();
        if (wave == 0 && lane == 0) publish_word(fin + e, epoch);
        return;
    }
    // slow path: the piece below is final (exact); repair again from its final top row, writing
    // through (the stored rows are still the chain's trajectory: nothing was committed)
    up_repair_coop<SPL, AGD>(ring, res2, meta32, U, fix, cs, Dpad, wave, lane, top, len, head, 2,
                             [&](double (&x)[SPL]) { input(x, fin + e - 1); });
    __syncthreads();
    if (wave == 0 && lane == 0) publish_word(fin + e, epoch);
}

template <int SPL, bool AGD>
__global__ __launch_bounds__(CHN_THREADS) void k_up_chain(WalkView V0, WalkView V1, const uint32_t* __restrict__ meta0,
                                                          const uint32_t* __restrict__ meta1,
                                                          const SmPath* __restrict__ paths0,
                                                          const SmPath* __restrict__ paths1,
                                                          const float* __restrict__ Cst0, const float* __restrict__ Cst1,
                                                          const uint2* __restrict__ Lrec, const uint2* __restrict__ Rrec,
                                                          const uint32_t* __restrict__ Lrec4,
                                                          const uint32_t* __restrict__ Rrec4,
                                                          const float* __restrict__ atab_g, int W, int dcall, int dglob0,
                                                          const double* __restrict__ slut_g, int Dpad, PieceView Q0,
                                                          PieceView Q1, uint32_t epoch) {
    __shared__ UpRing<SPL> ring;
    __shared__ double guess[64 * SPL];
    __shared__ int hdone;
    const int view = blockIdx.y;
    const WalkView V{view ? V1.npaths : V0.npaths, view ? V1.U : V0.U, nullptr, nullptr, nullptr, nullptr};
    // field-wise select: a reference to one of two by-value kernel arguments would copy both to
    // scratch
    PieceView Q;
    Q.pieces = view ? Q1.pieces : Q0.pieces;
    Q.npieces = view ? Q1.npieces : Q0.npieces;
    Q.agg = view ? Q1.agg : Q0.agg;
    Q.fix = view ? Q1.fix : Q0.fix;
    Q.stat = view ? Q1.stat : Q0.stat;
    Q.stride = Q0.stride;
    Q.plen = view ? Q1.plen : Q0.plen;
    Q.rmax = Q0.rmax;
    Q.dbg = Q0.dbg;
    Q.err = Q0.err;
    Q.wait_iters = Q0.wait_iters;
    const int e = blockIdx.x;
    uint4 pc = make_uint4((uint32_t)e, 0u, 1u, 0u);  // without pieces: block = path, one piece
    if (Q.pieces) {
        if (e >= Q.npieces) return;  // uniform over the block
        pc = Q.pieces[e];
    } else if (e >= V.npaths) {
        return;
    }
    const SmPath* __restrict__ pp = view ? paths1 : paths0;
    const SmPath path = pp[uniform(pc.x)];
    const int j = (int)uniform(pc.y), M = (int)uniform(pc.z);
    int plen = (int)uniform(path.len);
    if (Q.pieces && M == 1) {  // a run of consecutive paths: one contiguous slot range (every path's
                               // bottom node has S_heavy = 0, which restarts the recurrence)
        const SmPath last = pp[uniform(pc.x + pc.w - 1u)];
        plen = (int)uniform(last.head + last.len - path.head);
    }
    const int o0 = (int)sm_piece_begin_p((uint32_t)plen, (uint32_t)M, (uint32_t)j, (uint32_t)Q.plen);
    const int o1 = (int)sm_piece_begin_p((uint32_t)plen, (uint32_t)M, (uint32_t)j + 1u, (uint32_t)Q.plen);
    const int head = (int)uniform(path.head) + o0, len = o1 - o0;
    const bool lower = j + 1 < M;
    // a cut path's repair rows: 32 per segment of the path, from its first segment pc.w
    const FixRows fx{Q.fix, (long long)pc.w * SM_PRE_SEG - (long long)path.head};
    const int wave = (int)uniform(threadIdx.x >> 6), lane = threadIdx.x & 63;
#ifdef SM_CHAIN_TIMES  // diagnostic build: per-workgroup start / end (100 MHz) of every chain launch
    const unsigned long long tt0 = __builtin_amdgcn_s_memrealtime();
#endif
    static_assert(sizeof(ring.s) >= (size_t)CHN_WAVES * 2 * 64 * SPL * sizeof(double), "prologue scratch");
    if (lower) {  // guessed input: the aggregates of the segments below the piece
        const int sb = o1 / SM_PRE_SEG, ns = (plen + SM_PRE_SEG - 1) / SM_PRE_SEG - sb;
        up_guess<SPL>(reinterpret_cast<double*>(ring.s), guess, Q.agg + (size_t)(pc.w + sb) * 2 * Dpad, ns, Dpad, wave, lane);
    }
    // zero the ring: rows a helper does not stage are then always finite (see up_group)
    for (int i = threadIdx.x; i < (int)(sizeof(ring.s) / 4); i += CHN_THREADS) reinterpret_cast<uint32_t*>(ring.s)[i] = 0u;
    for (int i = threadIdx.x; i < SM_NUM_W; i += CHN_THREADS) ring.slut[i] = slut_g[i];
    if constexpr (AGD)
        for (int i = threadIdx.x; i <= SM_MAX_W; i += CHN_THREADS) ring.atab[i] = atab_g[i];
    if (threadIdx.x == 0) {
        ring.slut[SM_NUM_W] = 0.0;
        hdone = 0;
    }
    __syncthreads();
    const uint32_t* __restrict__ meta32 = view ? meta1 : meta0;
    UpCost cs;
    cs.own = view ? Rrec : Lrec;
    cs.oth = view ? Lrec : Rrec;
    cs.oth4 = view ? Lrec4 : Rrec4;
    cs.Cst = view ? Cst1 : Cst0;
    cs.W = W;
    cs.dbase = dglob0 + lane * SPL;
    cs.dend = dglob0 + dcall;
    cs.view = view;
    if (wave < Split<SPL>::NCW) {
        up_chain_wave<SPL>(ring, wave, head, len, lane, V.U, Dpad, lower ? guess : nullptr);
#ifdef SM_UP_SOLO_REPAIR  // A/B: round 1's repair, wave 0 alone
        if (wave == 0 && M > 1)
            up_finish<SPL, AGD>(ring, &hdone, meta32, V.U, fx, cs, Dpad, lane, head, len, j, M, e, Q, epoch);
#endif
    } else if (Split<SPL>::helper_of(wave) >= 0) {
        up_helper_wave<SPL, AGD>(ring, Split<SPL>::helper_of(wave), head, len, lane, meta32, V.U, cs, Dpad, lower,
                                 j > 0 ? Q.stat + e : nullptr, epoch);
        vm_drain();  // this helper's stores are complete before the repair reads or overwrites them
        if (lane == 0) atomicAdd(&hdone, 1);
    }
#ifndef SM_UP_SOLO_REPAIR
    if (M > 1) {  // uniform over the block
        __syncthreads();  // the chain is done and every helper's stores have completed (vm_drain)
        up_finish_coop<SPL, AGD>(ring, guess, meta32, V.U, fx, cs, Dpad, wave, lane, head, len, j, M, e, Q, epoch);
    }
#endif
#ifdef SM_CHAIN_TIMES
    __syncthreads();
    if (threadIdx.x == 0) ct_log(0, (int)blockIdx.y, M, len, e, tt0);
#endif
}

// ---------------------------------------------------------------------------------------------
// k_down_chain.  Chain node j = slot head + j (root side first).
// ---------------------------------------------------------------------------------------------
#ifndef DN_G1
#define DN_G1 8  // SPL = 1
#endif
#ifndef DN_NS1
#define DN_NS1 10
#endif
#ifndef DN_G2
#define DN_G2 6
#endif
#ifndef DN_NS2
#define DN_NS2 12
#endif
#ifndef DN_G4
#define DN_G4 3  // SPL = 4 (C3 / C4): 4 x 8 -> 3 x 20, k_down_chain 5.76 -> 5.43 ms at C3, 1.91 -> 1.79 ms at C4 size
#endif
#ifndef DN_NS4
#define DN_NS4 20
#endif
template <int SPL>
struct DownCfg {
    static constexpr int G = SPL == 4 ? DN_G4 : SPL == 2 ? DN_G2 : DN_G1;  // helper registers: next group's rows + WTA rows
    static constexpr int NS = SPL == 4 ? DN_NS4 : SPL == 2 ? DN_NS2 : DN_NS1;
};

template <int SPL>
struct DownSlot {
    static constexpr int G = DownCfg<SPL>::G;
    double x[G][64 * SPL];  // T = S2 * A_up in, A out
    double S[G];
    uint32_t pix[G];
    uint32_t st[G];         // 1 + compact A row of a light children's parent, else 0
    int staged;             // g+1: group g staged          (helper -> chain waves)
    int done[2];            // g+1: chain wave w computed g (chain wave -> owner helper)
    int freed;              // g+1: slot of group g free     (owner helper -> next helper)
};

template <int SPL>
struct DownRing {
    DownSlot<SPL> s[DownCfg<SPL>::NS];
    double slut[SM_NUM_W + 1];
    double s2lut[SM_NUM_W + 1];  // [SM_NUM_W]: S = 0, S2 = 1 (absent children; segment mode's virtual edges)
};
static_assert(sizeof(DownRing<1>) + 64 * 1 * 8 + 64 <= SM_LDS_BYTES, "DownRing<1> exceeds the LDS");
static_assert(sizeof(DownRing<2>) + 64 * 2 * 8 + 64 <= SM_LDS_BYTES, "DownRing<2> exceeds the LDS");
static_assert(sizeof(DownRing<4>) + 64 * 4 * 8 + 64 <= SM_LDS_BYTES, "DownRing<4> exceeds the LDS");

template <int SPL, int NN>
__device__ __forceinline__ void down_group(DownSlot<SPL>& sl, int k0, int e0, double (&x)[Split<SPL>::CS]) {
    constexpr int CS = Split<SPL>::CS;
    double t[NN][CS], S[NN];
#pragma unroll
    for (int k = 0; k < NN; ++k) {
        S[k] = sl.S[k0 + k];
        lds_read_at<CS>(sl.x[k0 + k], e0, t[k]);
    }
#pragma unroll
    for (int k = 0; k < NN; ++k) {
#pragma unroll
        for (int q = 0; q < CS; ++q) x[q] = __builtin_fma(S[k], x[q], t[k][q]);
        lds_write_at<CS>(sl.x[k0 + k], e0, x);
    }
}

// rows and S of a full group, read from its slot into registers
template <int SPL>
struct DownRegs {
    static constexpr int G = DownCfg<SPL>::G, CS = Split<SPL>::CS;
    double t[G][CS], S[G];
};
template <int SPL>
__device__ __forceinline__ void down_read(const DownSlot<SPL>& sl, int e0, DownRegs<SPL>& r) {
#pragma unroll
    for (int k = 0; k < DownRegs<SPL>::G; ++k) {
        r.S[k] = sl.S[k];
        lds_read_at<Split<SPL>::CS>(sl.x[k], e0, r.t[k]);
    }
}
template <int SPL>
__device__ __forceinline__ void down_step(DownSlot<SPL>& sl, int e0, const DownRegs<SPL>& r, double (&x)[Split<SPL>::CS]) {
    constexpr int CS = Split<SPL>::CS;
#pragma unroll
    for (int k = 0; k < DownRegs<SPL>::G; ++k) {
#pragma unroll
        for (int q = 0; q < CS; ++q) x[q] = __builtin_fma(r.S[k], x[q], r.t[k][q]);
        lds_write_at<CS>(sl.x[k], e0, x);
    }
}

// The chain wave reads a full group's rows one group ahead: when the next group is already staged
// at the top of a group, its LDS reads are issued before the group's recurrence and complete
// behind it (otherwise right after it).  Two register sets, the loop unrolled by two groups.
template <int SPL>
__device__ __forceinline__ void down_chain_wave(DownRing<SPL>& ring, int w, int len, int lane, const double* x0) {
    constexpr int G = DownCfg<SPL>::G, NS = DownCfg<SPL>::NS, CS = Split<SPL>::CS;
    __builtin_amdgcn_s_setprio(3);
    unsigned spins = 0;
#ifdef SM_CHAIN_PROF
    const long long t0 = clock64();
    long long tr = 0, tc = 0;
#endif
    const int e0 = (w * 64 + lane) * CS;
    // a piece below the path's first piece starts from its guessed input (the repair follows);
    // otherwise the first node is a path head or the root, staged with S = 0
    double x[CS];
#pragma unroll
    for (int q = 0; q < CS; ++q) x[q] = x0 ? x0[e0 + q] : 0.0;
    const int ngroups = (len + G - 1) / G;
    const int nfull = len / G;  // full groups take the pipeline; a partial last one node by node
    auto wait_staged = [&](int g) {
#ifdef SM_CHAIN_PROF
        const long long ta = clock64();
#endif
        while (lds_state(&ring.s[g % NS].staged) != g + 1) PROF_SPIN(++spins);
#ifdef SM_CHAIN_PROF
        tr += clock64() - ta;
#endif
    };
    DownRegs<SPL> A, B;
    int g = 0;
    if (nfull > 0) {
        wait_staged(0);
        down_read<SPL>(ring.s[0], e0, A);
    }
    // invariant at the top: group g (< nfull) is in A
    while (g < nfull) {
        // ---- group g (A); group g+1 into B, ahead when it is staged already
        bool ahead = false;
        if (g + 1 < nfull && lds_state(&ring.s[(g + 1) % NS].staged) == g + 2) {
            down_read<SPL>(ring.s[(g + 1) % NS], e0, B);
            ahead = true;
        }
        down_step<SPL>(ring.s[g % NS], e0, A, x);
        lds_publish_ordered(&ring.s[g % NS].done[w], g + 1);
        ++g;
        if (g >= nfull) break;
        if (!ahead) {
            wait_staged(g);
            down_read<SPL>(ring.s[g % NS], e0, B);
        }
        // ---- group g (B); group g+1 into A
        ahead = false;
        if (g + 1 < nfull && lds_state(&ring.s[(g + 1) % NS].staged) == g + 2) {
            down_read<SPL>(ring.s[(g + 1) % NS], e0, A);
            ahead = true;
        }
        down_step<SPL>(ring.s[g % NS], e0, B, x);
        lds_publish_ordered(&ring.s[g % NS].done[w], g + 1);
        ++g;
        if (g >= nfull) break;
        if (!ahead) {
            wait_staged(g);
            down_read<SPL>(ring.s[g % NS], e0, A);
        }
    }
    if (nfull < ngroups) {  // the partial last group
        DownSlot<SPL>& sl = ring.s[nfull % NS];
        wait_staged(nfull);
        for (int k = 0; k < len - nfull * G; ++k) down_group<SPL, 1>(sl, k, e0, x);
        lds_publish_ordered(&sl.done[w], nfull + 1);
    }
#ifdef SM_CHAIN_PROF
    if (blockIdx.x == 0 && lane == 0 && w == 0)
        printf("down chain view %d len %d cycles %lld spins %u wait %lld compute %lld\n", (int)blockIdx.y, len,
               clock64() - t0, spins, tr, tc);
#endif
    (void)spins;
}

// Helper waves of the down chain, split like the up chain's: loaders (load A_up rows + metadata,
// stage T and S) and storers (WTA of the chain's results, output and row stores, free the slot).
// A loader then never waits on store completions (gfx9: one vmcnt for loads and stores).
#ifndef DN_STORERS
#define DN_STORERS 8
#endif
template <int SPL>
__device__ __forceinline__ void down_helper_wave(DownRing<SPL>& ring, int hh, int head, int len, int lane,
                                                 const uint32_t* __restrict__ meta32, const WalkView& V, int Dpad,
                                                 const WtaCfg& w, int store_all, uint32_t epoch,
                                                 uint32_t* done_word, double* last_row) {
    constexpr int G = DownCfg<SPL>::G, NS = DownCfg<SPL>::NS, NCW = Split<SPL>::NCW;
    constexpr int NST = DN_STORERS, NL = Split<SPL>::NH - NST;
    const int ngroups = (len + G - 1) / G;
    if (hh >= NL) {
        // ---- storer: groups hh - NL (mod NST)
        for (int g = hh - NL; g < ngroups; g += NST) {
            const int n = min(G, len - g * G);
            DownSlot<SPL>& sl = ring.s[g % NS];
            lds_wait_all(sl.done, NCW, g + 1);
            double xs[G][SPL];
#pragma unroll
            for (int k = 0; k < G; ++k) {
                if (k < n) {
                    lds_row_read<SPL>(sl.x[k], lane, xs[k]);
                } else {
#pragma unroll
                    for (int q = 0; q < SPL; ++q) xs[k][q] = 0.0;
                }
            }
            const uint32_t pix = sl.pix[min(lane, G - 1)];
            uint32_t st[G];
#pragma unroll
            for (int k = 0; k < G; ++k) st[k] = sl.st[k];
            lds_publish(&sl.freed, g + 1);
            double mn;
            int gi;
            float dsp;
            wta_nodes<SPL, G>(xs, lane, w, mn, gi, dsp);
#pragma unroll
            for (int k = 0; k < G; ++k) {
                if (k < n && st[k]) store_row<SPL>(V.A, st[k] - 1u, Dpad, lane, xs[k]);
                if (k < n && store_all) store_row<SPL>(V.Adbg, (uint32_t)(head + g * G + k), Dpad, lane, xs[k]);
            }
            if (lane < n) {
                V.idx[pix] = gi;
                V.minc[pix] = mn;
                V.disp[pix] = dsp;
            }
            if (done_word && g == ngroups - 1) {
                // the piece's last row is the next piece's input: device scope, then the done word
                double* row = last_row + lane * SPL;
#pragma unroll
                for (int k = 0; k < G; ++k)
                    if (k == n - 1 && row_lane<SPL>(lane, Dpad))
#pragma unroll
                        for (int q = 0; q < SPL; ++q) __hip_atomic_store(row + q, xs[k][q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                vm_drain();
                if (lane == 0) publish_word(done_word, epoch);
            }
        }
        return;
    }
    // ---- loader: groups hh, hh + NL, ...
    int g = hh;
    if (g >= ngroups) return;
    double* __restrict__ U = V.U;
    double u[G][SPL];
    MetaVec<G> mv;
    auto issue = [&](int gg) {
        const int n = min(G, len - gg * G);
#pragma unroll
        for (int k = 0; k < G; ++k) load_row<SPL>(U, (uint32_t)(head + gg * G + min(k, n - 1)), Dpad, lane, u[k]);
        load_meta<G>(mv, meta32, lane, head + gg * G, 1, n);
    };
    issue(g);
    for (;;) {
        const int n = min(G, len - g * G);
        DownSlot<SPL>& sl = ring.s[g % NS];
        // ---- stage T = S2 * A_up and S.  A path head (its parent finished in an earlier round)
        // folds its parent row here: T = fma(S, A(parent), S2 * A_up), staged with S = 0, so the
        // chain's fma(0, x, T) == T exactly; the root: T = A_up, S = 0.
        double t[G][SPL], Sk[G];
#pragma unroll
        for (int k = 0; k < G; ++k) {
            const uint32_t par = mfield(mv, k, 1);
            const uint32_t slot = (uint32_t)(head + g * G + k);
            const uint32_t wp = lo_wp(mfield(mv, k, 2));
            const double S = ring.slut[wp], S2 = ring.s2lut[wp];
            const bool root = par == SM_NONE, phead = !root && par != slot - 1u;
#pragma unroll
            for (int q = 0; q < SPL; ++q) t[k][q] = root ? u[k][q] : S2 * u[k][q];
            Sk[k] = root || phead ? 0.0 : S;
            if (k < n && phead) {  // uniform; one node per path
                double ap[SPL];
                load_row<SPL>(V.A, sm_arow(par), Dpad, lane, ap);
#pragma unroll
                for (int q = 0; q < SPL; ++q) t[k][q] = __builtin_fma(S, ap[q], t[k][q]);
            }
        }
        uint32_t pixk[G], stk[G];
#pragma unroll
        for (int k = 0; k < G; ++k) {
            pixk[k] = mfield(mv, k, 0);
            stk[k] = hi_light(mfield(mv, k, 3)) ? mfield(mv, k, 7) + 1u : 0u;
        }
        // ---- next group's loads go out now (unconditional, clamped)
        const int gn = g + NL;
        issue(gn < ngroups ? gn : g);
        if (g >= NS) lds_wait(&sl.freed, g - NS + 1, true);
#pragma unroll
        for (int k = 0; k < G; ++k) {
            if (k < n) {
                lds_row_write<SPL>(sl.x[k], lane, t[k]);
                if (lane == 0) {
                    sl.S[k] = Sk[k];
                    sl.pix[k] = pixk[k];
                    sl.st[k] = stk[k];
                }
            }
        }
        lds_publish(&sl.staged, g + 1);
        if (gn >= ngroups) break;
        g = gn;
    }
}

// ---------------------------------------------------------------------------------------------
// Down-pass pieces (see "Pieces" above; pieces top first).  The guess of piece i is the fold of
// the piece-level affine aggregates of pieces 0 .. i-1 (A(last) = P * A(before) + B, with the
// reference's per-node map A = S * A(parent) + S2 * A_up) applied to the path's input row; every
// piece computes its own aggregate in the prologue (16 waves in parallel) and publishes it, so
// the guess waits for no chain.  The repair re-runs the piece's first nodes from the true input
// and compares at the nodes whose rows are stored (light children's parents, the piece's last
// node): equal there -> equal from there on.  Corrections (WTA outputs, stored rows) are written
// directly; when the look-back finds a piece above that did not merge, the piece is re-walked
// completely from the final input (correctness only), overwriting everything it wrote.
// ---------------------------------------------------------------------------------------------
// per-piece aggregate: all 16 waves fold a contiguous node range (top first), combined in LDS;
// ends with a barrier, the result (P row | B row) is in scratch[0 .. 2 * 64 * SPL)
template <int SPL>
__device__ void down_piece_agg(double* scratch, const uint32_t* __restrict__ meta32, const double* __restrict__ U,
                               const double* slut, const double* s2lut, int head, int len, int Dpad, int wave, int lane) {
    const int per = (len + CHN_WAVES - 1) / CHN_WAVES;
    const int n0 = min(len, wave * per), n1 = min(len, n0 + per);
    double P[SPL], B[SPL];
#pragma unroll
    for (int k = 0; k < SPL; ++k) {
        P[k] = 1.0;
        B[k] = 0.0;
    }
    for (int n = n0; n < n1; n += 8) {
        const int nb = min(8, n1 - n);
        MetaVec<8> mv;
        load_meta<8>(mv, meta32, lane, head + n, 1, nb);
        double u[8][SPL];
#pragma unroll
        for (int k = 0; k < 8; ++k) load_row<SPL>(U, (uint32_t)(head + n + min(k, nb - 1)), Dpad, lane, u[k]);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (k < nb) {
                const bool root = mfield(mv, k, 1) == SM_NONE;
                const uint32_t wp = lo_wp(mfield(mv, k, 2));
                const double S = root ? 0.0 : slut[wp], S2 = s2lut[wp];
#pragma unroll
                for (int q = 0; q < SPL; ++q) {
                    B[q] = __builtin_fma(S, B[q], root ? u[k][q] : S2 * u[k][q]);
                    P[q] = S * P[q];
                }
            }
        }
    }
    double* my = scratch + (size_t)wave * 2 * 64 * SPL;
#pragma unroll
    for (int k = 0; k < SPL; ++k) {
        my[lane * SPL + k] = P[k];
        my[64 * SPL + lane * SPL + k] = B[k];
    }
    __syncthreads();
    if (wave == 0) {
#pragma unroll
        for (int q = 0; q < SPL; ++q) {
            double p = scratch[lane * SPL + q], b = scratch[64 * SPL + lane * SPL + q];
            for (int w = 1; w < CHN_WAVES; ++w) {
                const double* t = scratch + (size_t)w * 2 * 64 * SPL;
                b = __builtin_fma(t[lane * SPL + q], b, t[64 * SPL + lane * SPL + q]);
                p = t[lane * SPL + q] * p;
            }
            scratch[lane * SPL + q] = p;
            scratch[64 * SPL + lane * SPL + q] = b;
        }
    }
    __syncthreads();
}

// guessed input of piece e (index i >= 1 within its path): x_path (the path's input row: A of
// the head's parent) through the aggregates of the pieces above, entries e - i .. e - 1, split
// over the 16 waves.  Ends with a barrier; the result is in guess[].
template <int SPL>
__device__ void down_guess(double* scratch, double* guess, const double* __restrict__ A, const double* __restrict__ agg,
                           const uint32_t* aggw, uint32_t hp, int e, int i, int Dpad, int wave, int lane,
                           uint32_t epoch, uint32_t* err, int wait_iters) {
    const int per = (i + CHN_WAVES - 1) / CHN_WAVES;
    const int q0 = min(i, wave * per), q1 = min(i, q0 + per);
    double P[SPL], B[SPL];
#pragma unroll
    for (int k = 0; k < SPL; ++k) {
        P[k] = 1.0;
        B[k] = 0.0;
    }
    for (int q = q0; q < q1; ++q) {
        const int eq = e - i + q;
        wait_word(aggw + eq, epoch, epoch, err, wait_iters);
        vm_drain();
        double p[SPL], b[SPL];
        agent_row_read<SPL>(agg + (size_t)eq * 2 * Dpad, 0, Dpad, lane, p);
        agent_row_read<SPL>(agg + (size_t)eq * 2 * Dpad + Dpad, 0, Dpad, lane, b);
#pragma unroll
        for (int k = 0; k < SPL; ++k) {
            B[k] = __builtin_fma(p[k], B[k], b[k]);
            P[k] = p[k] * P[k];
        }
    }
    double* my = scratch + (size_t)wave * 2 * 64 * SPL;
#pragma unroll
    for (int k = 0; k < SPL; ++k) {
        my[lane * SPL + k] = P[k];
        my[64 * SPL + lane * SPL + k] = B[k];
    }
    __syncthreads();
    if (wave == 0) {
        double x[SPL];
        if (hp != SM_NONE) {
            load_row<SPL>(A, sm_arow(hp), Dpad, lane, x);  // finished in an earlier launch
        } else {
#pragma unroll
            for (int k = 0; k < SPL; ++k) x[k] = 0.0;  // the root's S is 0
        }
        for (int w = 0; w < CHN_WAVES; ++w) {
            const double* t = scratch + (size_t)w * 2 * 64 * SPL;
#pragma unroll
            for (int k = 0; k < SPL; ++k) x[k] = __builtin_fma(t[lane * SPL + k], x[k], t[64 * SPL + lane * SPL + k]);
        }
#pragma unroll
        for (int k = 0; k < SPL; ++k) guess[lane * SPL + k] = x[k];
    }
    __syncthreads();
}

// Exact re-walk of a down piece's nodes 0 .. nmax-1 (slot head + n) from the input row x:
// A = fma(S, x, S2 * A_up) as the chain, WTA outputs and the stored rows (light children's
// parents, every row with store_all, the piece's last node at device scope when last_pub) of
// every node before the merge.  check: compare at stored nodes and return the first node equal
// in all lanes (nothing is written from there on); otherwise / no merge: -1.
template <int SPL, int CHR>
__device__ __forceinline__ int down_exact_walk(const uint32_t* __restrict__ meta32, const double* __restrict__ U,
                                               const WalkView& V, const double* slut, const double* s2lut, int head,
                                               int len, int nmax, int Dpad, int lane, double* xio, const WtaCfg& w,
                                               int store_all, const double* last_row, bool check) {
    const bool last_pub = last_row != nullptr;
    double x[SPL];
#pragma unroll
    for (int q = 0; q < SPL; ++q) x[q] = xio[q];
    MetaVec<CHR> mv;
    load_meta<CHR>(mv, meta32, lane, head, 1, min(CHR, nmax));
    for (int n0 = 0; n0 < nmax; n0 += CHR) {
        const int nb = min(CHR, nmax - n0);
        MetaVec<CHR> mn;
        const int n1 = n0 + CHR < nmax ? n0 + CHR : n0;
        load_meta<CHR>(mn, meta32, lane, head + n1, 1, min(CHR, nmax - n1));
        double u[CHR][SPL], spec[CHR][SPL], ys[CHR][SPL];
#pragma unroll
        for (int k = 0; k < CHR; ++k) {
            const int kk = min(k, nb - 1);
            const uint32_t slot = (uint32_t)(head + n0 + kk);
            load_row<SPL>(U, slot, Dpad, lane, u[k]);
            // the row stored for this node, if any: every row (debug), the piece's last row, or the
            // compact A row of a light children's parent; another node reads its own U row (never
            // compared).  Scalar selects and one unconditional load: the batch's loads stay one batch
            if (check) {
                const double* src = store_all ? V.Adbg + (size_t)slot * Dpad
                                    : (last_pub && n0 + kk == len - 1) ? last_row
                                    : hi_light(mfield(mv, kk, 3)) ? V.A + (size_t)mfield(mv, kk, 7) * Dpad
                                    : U + (size_t)slot * Dpad;
                agent_row_read<SPL>(src, 0, Dpad, lane, spec[k]);
            }
        }
        int mk = nb;  // nodes of this batch before the merge
#pragma unroll
        for (int k = 0; k < CHR; ++k) {
            if (k < mk) {
                const uint32_t wp = lo_wp(mfield(mv, k, 2));
                const double S = slut[wp], S2 = s2lut[wp];
                bool eq = true;
#pragma unroll
                for (int q = 0; q < SPL; ++q) {
                    x[q] = __builtin_fma(S, x[q], S2 * u[k][q]);
                    ys[k][q] = x[q];
                    // lanes beyond a 32-double row hold nothing (cost 3.0 there, stored rows read 0)
                eq = eq && (!row_lane<SPL>(lane, Dpad) || __double_as_longlong(x[q]) == __double_as_longlong(spec[k][q]));
                }
                const bool stored = store_all || hi_light(mfield(mv, k, 3)) || (last_pub && n0 + k == len - 1);
                if (check && stored && __all(eq)) mk = k;
            } else {
#pragma unroll
                for (int q = 0; q < SPL; ++q) ys[k][q] = 0.0;
            }
        }
        double mnv;
        int gi;
        float dsp;
        wta_nodes<SPL, CHR>(ys, lane, w, mnv, gi, dsp);
        const uint32_t pix = meta_pix_of_lane<CHR>(mv, lane);
        if (lane < mk) {
            V.idx[pix] = gi;
            V.minc[pix] = mnv;
            V.disp[pix] = dsp;
        }
#pragma unroll
        for (int k = 0; k < CHR; ++k) {
            if (k < mk) {
                const uint32_t slot = (uint32_t)(head + n0 + k);
                if (last_pub && n0 + k == len - 1) agent_row_write<SPL>(const_cast<double*>(last_row), 0, Dpad, lane, ys[k]);
                if (hi_light(mfield(mv, k, 3))) store_row<SPL>(V.A, mfield(mv, k, 7), Dpad, lane, ys[k]);
                if (store_all) store_row<SPL>(V.Adbg, slot, Dpad, lane, ys[k]);
            }
        }
        if (mk < nb) return n0 + mk;
        mv = mn;
    }
    return -1;
}

#ifndef DN_WALK_CH
#define DN_WALK_CH(SPL) ((SPL) == 4 ? 4 : 8)  // nodes per down-repair batch (registers)
#endif

// Repair + look-back of down piece e (index i of M, pieces top first: the pieces above are
// entries e - i .. e - 1, the top one exact by construction).
template <int SPL>
__device__ void down_finish(DownRing<SPL>& ring, int* hdone, const uint32_t* __restrict__ meta32, const WalkView& V,
                            int Dpad, const WtaCfg& w, int store_all, int lane, int head, int len, int i, int M,
                            int e, const PieceView& Q, uint32_t epoch, FixRows fx) {
    uint32_t* done = Q.stat;
    uint32_t* merged = Q.stat + Q.stride;
    uint32_t* fin = Q.stat + 2 * Q.stride;
    if (i == 0) {
        if (lane == 0) publish_word(fin + e, epoch);
        return;
    }
    while (__hip_atomic_load(hdone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < Split<SPL>::NH) __builtin_amdgcn_s_sleep(1);
    // this piece's published last row (none for the bottom piece) and the piece above's
    const double* last_row = i + 1 < M ? fx.p + (size_t)fx.row((uint32_t)(head + len - 1)) * Dpad : nullptr;
    const double* above = fx.p + (size_t)fx.row((uint32_t)(head - 1)) * Dpad;
    double x[SPL];
#ifdef SM_CHAIN_TIMES
    const unsigned long long tf0 = __builtin_amdgcn_s_memrealtime();
#endif
    wait_word(done + e - 1, epoch, epoch, Q.err, Q.wait_iters);
    vm_drain();
    agent_row_read<SPL>(above, 0, Dpad, lane, x);
    vm_drain();
#ifdef SM_CHAIN_TIMES
    const unsigned long long tf1 = __builtin_amdgcn_s_memrealtime();
#endif
    const int m = down_exact_walk<SPL, DN_WALK_CH(SPL)>(meta32, V.U, V, ring.slut, ring.s2lut, head, len, min(Q.rmax, len), Dpad,
                                                        lane, x, w, store_all, last_row, true);
    vm_drain();
#ifdef SM_CHAIN_TIMES
    if (lane == 0) {
        ct_log(2 | 8, (int)blockIdx.y, M, m, e, tf0, tf1);  // waiting for the piece above
        ct_log(3 | 8, (int)blockIdx.y, M, m, e, tf1);       // the repair walk (len field: merge node)
    }
#endif
    if (lane == 0) publish_word(merged + e, 2u * epoch + (m >= 0 ? 0u : 1u));
    bool all = m >= 0;
    for (int q = e - 1; all && q > e - i; --q) all = wait_word(merged + q, 2u * epoch, 2u * epoch + 1u, Q.err, Q.wait_iters) == 2u * epoch;
    if (Q.dbg && lane == 0) {
        atomicAdd(Q.dbg + (all ? 4 : 5), 1ull);
        if (m >= 0) {
            atomicAdd(Q.dbg + 6, (unsigned long long)m);
            atomicMax(Q.dbg + 7, (unsigned long long)m);
        }
    }
    if (all) {
        if (lane == 0) publish_word(fin + e, epoch);
        return;
    }
    wait_word(fin + e - 1, epoch, epoch, Q.err, Q.wait_iters);
    vm_drain();
    agent_row_read<SPL>(above, 0, Dpad, lane, x);
    vm_drain();
    down_exact_walk<SPL, DN_WALK_CH(SPL)>(meta32, V.U, V, ring.slut, ring.s2lut, head, len, len, Dpad, lane, x, w,
                                          store_all, last_row, false);
    vm_drain();
    if (lane == 0) publish_word(fin + e, epoch);
}

template <int SPL>
__global__ __launch_bounds__(CHN_THREADS) void k_down_chain(WalkView V0, WalkView V1,
                                                            const uint32_t* __restrict__ meta0,
                                                            const uint32_t* __restrict__ meta1,
                                                            const SmPath* __restrict__ paths0,
                                                            const SmPath* __restrict__ paths1,
                                                            const double* __restrict__ slut_g,
                                                            const double* __restrict__ s2lut_g, int Dpad, WtaCfg w,
                                                            int store_all, uint32_t epoch, PieceView Q0,
                                                            PieceView Q1) {
    __shared__ DownRing<SPL> ring;
    __shared__ double guess[64 * SPL];
    __shared__ int hdone;
    const int view = blockIdx.y, pidx = blockIdx.x;
    // field-wise selects (a reference to one of two by-value arguments would go to scratch)
    WalkView V;
    V.npaths = view ? V1.npaths : V0.npaths;
    V.U = view ? V1.U : V0.U;
    V.idx = view ? V1.idx : V0.idx;
    V.minc = view ? V1.minc : V0.minc;
    V.disp = view ? V1.disp : V0.disp;
    V.A = view ? V1.A : V0.A;
    V.Adbg = view ? V1.Adbg : V0.Adbg;
    PieceView Q;
    Q.pieces = view ? Q1.pieces : Q0.pieces;
    Q.npieces = view ? Q1.npieces : Q0.npieces;
    Q.agg = view ? Q1.agg : Q0.agg;
    Q.fix = view ? Q1.fix : Q0.fix;  // the pieces' published last rows
    Q.stat = view ? Q1.stat : Q0.stat;
    Q.stride = Q0.stride;
    Q.plen = view ? Q1.plen : Q0.plen;
    Q.rmax = Q0.rmax;
    Q.dbg = Q0.dbg;
    Q.err = Q0.err;
    Q.wait_iters = Q0.wait_iters;
    // work item: piece i of M of a cut path (entries list a path's pieces bottom first with index
    // j: i = M - 1 - j, pieces top first), or a run of w whole paths (M == 1)
    uint4 pc = make_uint4((uint32_t)pidx, 0u, 1u, 1u);
    if (Q.pieces) {
        if (pidx >= Q.npieces) return;  // uniform over the block
        pc = Q.pieces[pidx];
    } else if (pidx >= V.npaths) {
        return;
    }
    const int M = (int)uniform(pc.z), i = M - 1 - (int)uniform(pc.y);
    const uint32_t* __restrict__ meta32 = view ? meta1 : meta0;
    const SmPath* __restrict__ pp = view ? paths1 : paths0;
    const SmPath path = pp[uniform(pc.x)];
    int plen = (int)uniform(path.len);
    if (M == 1) {  // a run: slots of consecutive paths are contiguous
        const SmPath last = pp[uniform(pc.x + pc.w - 1u)];
        plen = (int)uniform(last.head + last.len - path.head);
    }
    const int o0 = (int)sm_piece_begin_dn((uint32_t)plen, (uint32_t)M, (uint32_t)i, (uint32_t)Q.plen);
    const int o1 = (int)sm_piece_begin_dn((uint32_t)plen, (uint32_t)M, (uint32_t)i + 1u, (uint32_t)Q.plen);
    const int head = (int)uniform(path.head) + o0, len = o1 - o0;
    const FixRows fx{Q.fix, (long long)pc.w * SM_PRE_SEG - (long long)path.head};  // (cut paths: M > 1)
#ifdef SM_CHAIN_TIMES
    const unsigned long long tt0 = __builtin_amdgcn_s_memrealtime();
#endif
    const int wave = (int)uniform(threadIdx.x >> 6), lane = threadIdx.x & 63;
    for (int k = threadIdx.x; k < SM_NUM_W; k += CHN_THREADS) {
        ring.slut[k] = slut_g[k];
        ring.s2lut[k] = s2lut_g[k];
    }
    if (threadIdx.x == 0) {
        ring.slut[SM_NUM_W] = 0.0;
        ring.s2lut[SM_NUM_W] = 1.0;
    }
    __syncthreads();
    if (M > 1) {
        uint32_t* aggw = Q.stat + 3 * Q.stride;
        double* scratch = reinterpret_cast<double*>(ring.s);
        static_assert(sizeof(ring.s) >= (size_t)CHN_WAVES * 2 * 64 * SPL * sizeof(double), "prologue scratch");
        if (i + 1 < M) {  // this piece's aggregate, for the pieces below
            down_piece_agg<SPL>(scratch, meta32, V.U, ring.slut, ring.s2lut, head, len, Dpad, wave, lane);
            if (wave == 0) {
                double p[SPL], b[SPL];
#pragma unroll
                for (int q = 0; q < SPL; ++q) {
                    p[q] = scratch[lane * SPL + q];
                    b[q] = scratch[64 * SPL + lane * SPL + q];
                }
                double* out = const_cast<double*>(Q.agg) + (size_t)pidx * 2 * Dpad;
                agent_row_write<SPL>(out, 0, Dpad, lane, p);
                agent_row_write<SPL>(out + Dpad, 0, Dpad, lane, b);
                vm_drain();
                if (lane == 0) publish_word(aggw + pidx, epoch);
            }
            __syncthreads();
        }
#ifdef SM_CHAIN_TIMES
        if (threadIdx.x == 0) ct_log(1 | 8, (int)blockIdx.y, M, len, pidx, tt0);  // tables + own aggregate published
#endif
        if (i > 0)
            down_guess<SPL>(scratch, guess, V.A, Q.agg, aggw, uniform(meta32[(size_t)path.head * 8 + 1]), pidx, i, Dpad, wave,
                            lane, epoch, Q.err, Q.wait_iters);
    }
    for (int k = threadIdx.x; k < DownCfg<SPL>::NS; k += CHN_THREADS) {
        ring.s[k].staged = ring.s[k].freed = 0;
        ring.s[k].done[0] = ring.s[k].done[1] = 0;
    }
    if (threadIdx.x == 0) hdone = 0;
    __syncthreads();
#ifdef SM_CHAIN_TIMES
    if (threadIdx.x == 0 && M > 1) ct_log(0 | 8, (int)blockIdx.y, M, len, pidx, tt0);  // prologue: aggregate + guess
#endif
    if (wave < Split<SPL>::NCW) {
        down_chain_wave<SPL>(ring, wave, len, lane, i > 0 ? guess : nullptr);
        if (wave == 0 && M > 1)
            down_finish<SPL>(ring, &hdone, meta32, V, Dpad, w, store_all, lane, head, len, i, M, pidx, Q, epoch, fx);
    } else if (Split<SPL>::helper_of(wave) >= 0) {
        const bool pub = M > 1 && i + 1 < M;
        down_helper_wave<SPL>(ring, Split<SPL>::helper_of(wave), head, len, lane, meta32, V, Dpad, w, store_all, epoch,
                              pub ? Q.stat + pidx : nullptr, pub ? Q.fix + (size_t)fx.row((uint32_t)(head + len - 1)) * Dpad : nullptr);
        vm_drain();  // this helper's stores are complete before the repair overwrites them
        if (lane == 0) atomicAdd(&hdone, 1);
    }
#ifdef SM_CHAIN_TIMES
    __syncthreads();
    if (threadIdx.x == 0) ct_log(1, (int)blockIdx.y, M, len, pidx, tt0);
#endif
}

// ---------------------------------------------------------------------------------------------
static WalkView chain_view(const WalkArgs& a, int v) {
    return WalkView{a.npaths[v], a.U[v], a.idx[v], a.minc[v], a.disp[v], a.A[v], a.Adbg[v]};
}

UpPreArgs up_pre_args(const WalkArgs& a) {
    UpPreArgs pa{};
    for (int v = 0; v < 2; ++v) {
        pa.paths[v] = a.paths[v];
        pa.seg[v] = a.segtab[v];
        pa.nseg[v] = a.nseg[v];
        pa.agg[v] = a.pieces[v] ? a.agg[v] : nullptr;
        pa.plen[v] = a.bucket_plen[v];
    }
    return pa;
}

template <int SPL, int CH, int NSUB, bool VOL>
static void up_pre_launch_k(hipStream_t st, const WalkArgs& a) {
    const int ns = a.nseg[0] > a.nseg[1] ? a.nseg[0] : a.nseg[1];
    if (ns == 0) return;
    hipLaunchKernelGGL((k_up_pre<SPL, CH, NSUB, VOL>), dim3(ns, 2), dim3(256), 0, st, chain_view(a, 0), chain_view(a, 1),
                       reinterpret_cast<const uint32_t*>(a.meta[0]), reinterpret_cast<const uint32_t*>(a.meta[1]),
                       up_pre_args(a), a.Cst[0], a.Cst[1], a.Lrec, a.Rrec, a.atab, a.slut, a.s2lut, a.W, a.Dpad, a.dcall,
                       a.dglob0);
}

template <int SPL, int CH, int NSUB>
static void up_pre_launch(hipStream_t st, const WalkArgs& a) {
    if (a.vol)  // cost rows in Cst (k_vol_rows)
        up_pre_launch_k<SPL, CH, NSUB, true>(st, a);
    else
        up_pre_launch_k<SPL, CH, NSUB, false>(st, a);
}

static PieceView piece_view(const WalkArgs& a, int v) {
    return PieceView{a.pieces[v], a.npieces[v], a.agg[v], a.fix[v], a.pstat[v], a.pstride, a.bucket_plen[v], a.repair_max, a.piece_dbg,
                     a.err, a.wait_iters};
}

template <int SPL, bool AGD>
static void up_chain_launch_k(hipStream_t st, const WalkArgs& a, int np) {
    hipLaunchKernelGGL((k_up_chain<SPL, AGD>), dim3(np, 2), dim3(CHN_THREADS), 0, st, chain_view(a, 0), chain_view(a, 1),
                       reinterpret_cast<const uint32_t*>(a.meta[0]), reinterpret_cast<const uint32_t*>(a.meta[1]),
                       a.paths[0], a.paths[1], a.Cst[0], a.Cst[1], a.Lrec, a.Rrec, a.Lrec4, a.Rrec4, a.atab, a.W, a.dcall,
                       a.dglob0, a.slut, a.Dpad, piece_view(a, 0), piece_view(a, 1), a.epoch);
}
template <int SPL>
static void up_chain_launch(hipStream_t st, const WalkArgs& a, int np) {
    if (a.vol)
        up_chain_launch_k<SPL, false>(st, a, np);
    else
        up_chain_launch_k<SPL, true>(st, a, np);
}

template <int SPL>
static void down_chain_launch(hipStream_t st, const WalkArgs& a, int np, int store_all) {
    const dim3 grid(np, 2);
    PieceView q0 = piece_view(a, 0), q1 = piece_view(a, 1);
    for (PieceView* q : {&q0, &q1})  // the down pass's status words: arrays 3..6 (up: 0..2)
        if (q->stat) q->stat += 3 * (size_t)q->stride;
    hipLaunchKernelGGL((k_down_chain<SPL>), grid, dim3(CHN_THREADS), 0, st, chain_view(a, 0), chain_view(a, 1),
                       reinterpret_cast<const uint32_t*>(a.meta[0]), reinterpret_cast<const uint32_t*>(a.meta[1]),
                       a.paths[0], a.paths[1], a.slut, a.s2lut, a.Dpad, a.wta, store_all, a.epoch, q0, q1);
}

hipError_t launch_up_pre(hipStream_t st, const WalkArgs& a, int spl) {
    switch (spl) {
        case 1: up_pre_launch<1, 8, 1>(st, a); break;
        case 2: up_pre_launch<2, 8, 1>(st, a); break;
        default: up_pre_launch<4, 4, 2>(st, a); break;
    }
    return hipGetLastError();
}

hipError_t launch_up_chain(hipStream_t st, const WalkArgs& a, int spl) {
    int np = 0;
    for (int v = 0; v < 2; ++v) np = std::max(np, a.pieces[v] ? a.npieces[v] : a.npaths[v]);
    if (np == 0) return hipSuccess;
    switch (spl) {
        case 1: up_chain_launch<1>(st, a, np); break;
        case 2: up_chain_launch<2>(st, a, np); break;
        default: up_chain_launch<4>(st, a, np); break;
    }
    return hipGetLastError();
}

hipError_t launch_down_long(hipStream_t st, const WalkArgs& a, int spl, int store_all) {
    int np = 0;
    for (int v = 0; v < 2; ++v) np = std::max(np, a.pieces[v] ? a.npieces[v] : a.npaths[v]);
    if (np == 0) return hipSuccess;
    switch (spl) {
        case 1: down_chain_launch<1>(st, a, np, store_all); break;
        case 2: down_chain_launch<2>(st, a, np, store_all); break;
        default: down_chain_launch<4>(st, a, np, store_all); break;
    }
    return hipGetLastError();
}
