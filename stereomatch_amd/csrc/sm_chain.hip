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
// Ring protocol (per entry e, node j of the path, entry = j mod R):
//   state[e] = 2j+1 : helper has written node j's inputs      (helper -> chain)
//   state[e] = 2j+2 : chain has written node j's result       (chain  -> helper)
// Entry e is owned by helper e / E, so the only cross-wave traffic is these two hand-offs.  LDS
// operations of one wave complete in order; a publish is preceded by lgkmcnt(0) so the entry's
// data is in LDS before its state word changes.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sm_common.h"
#include "sm_launch.h"
#include "sm_layout_gpu.h"
#include "sm_walk_util.h"

#define CHN_HELPERS 15
#define CHN_THREADS (64 * (CHN_HELPERS + 1))
#define CHN_G 8  // nodes per chain group (one LDS round trip per group)

// -DSM_CHAIN_PROF: the first path of each launch prints chain-wave cycles / failed polls and helper
// wait cycles (device printf) -- a diagnostic build only (tools/chain_prof.sh)
#ifdef SM_CHAIN_PROF
#include <stdio.h>
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
        c[0] = p[0];
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
template <int SPL>
__device__ __forceinline__ void store_crow(float* __restrict__ C, uint32_t slot, int Dpad, int lane, const double (&c)[SPL]) {
    float* p = C + (size_t)slot * Dpad + lane * SPL;
    if constexpr (SPL == 1) {
        p[0] = (float)c[0];
    } else if constexpr (SPL == 2) {
        *reinterpret_cast<float2*>(p) = make_float2((float)c[0], (float)c[1]);
    } else {
        *reinterpret_cast<float4*>(p) = make_float4((float)c[0], (float)c[1], (float)c[2], (float)c[3]);
    }
}

// ---------------------------------------------------------------------------------------------
// k_up_pre: one block per SM_PRE_SEG-node segment of a long path (segment table from the layout),
// SM_PRE_SEG / CH waves of CH nodes each; grid.y = view
// ---------------------------------------------------------------------------------------------
template <int SPL, int CH>
__global__ __launch_bounds__(64 * SM_PRE_SEG / CH) void k_up_pre(
    WalkView V0, WalkView V1, const uint32_t* __restrict__ meta0, const uint32_t* __restrict__ meta1,
    const SmPath* __restrict__ paths0, const SmPath* __restrict__ paths1, const uint2* __restrict__ seg0,
    const uint2* __restrict__ seg1, int nseg0, int nseg1, float* __restrict__ Cst0, float* __restrict__ Cst1,
    const uint2* __restrict__ Lrec, const uint2* __restrict__ Rrec, const float* __restrict__ atab_g,
    const double* __restrict__ slut_g, const double* __restrict__ s2lut_g, int W, int Dpad, int dcall, int dglob0) {
    const int view = blockIdx.y;
    if ((int)blockIdx.x >= (view ? nseg1 : nseg0)) return;  // uniform over the block
    __shared__ WalkShared sh;
    load_tables(sh, atab_g, slut_g, s2lut_g);
    const WalkView& V = view ? V1 : V0;
    const uint32_t* __restrict__ meta32 = view ? meta1 : meta0;
    const int lane = threadIdx.x & 63;
    const uint2 sg = (view ? seg1 : seg0)[blockIdx.x];
    const SmPath path = (view ? paths1 : paths0)[uniform(sg.x)];
    const int head = (int)uniform(path.head), len = (int)uniform(path.len);
    const int first = (int)uniform(sg.y * SM_PRE_SEG + (threadIdx.x >> 6) * CH);
    if (first >= len) return;
    const int n = min(CH, len - first);
    const int dbase = dglob0 + lane * SPL;
    const int dend = dglob0 + dcall;
    const uint2* __restrict__ own = view ? Rrec : Lrec;
    const uint2* __restrict__ oth = view ? Lrec : Rrec;
    double* __restrict__ U = V.U;
    float* __restrict__ Cst = view ? Cst1 : Cst0;
    MetaVec<CH> mv;
    load_meta<CH>(mv, meta32, lane, head + first, 1, n);
    // pre-heavy light child rows (positions 0 .. hidx-1; up to 3 at a tree root)
    double lr[CH][3][SPL];
#pragma unroll
    for (int j = 0; j < CH; ++j) {
        if (j < n) {
            const uint32_t hidx = hi_hidx(mfield(mv, j, 3));
#pragma unroll
            for (int i = 0; i < 3; ++i)
                if ((uint32_t)i < hidx) load_row<SPL>(U, mfield(mv, j, 4 + i), Dpad, lane, lr[j][i]);
        }
    }
    ImgRecs<SPL, CH> rec;
    load_recs<SPL, CH>(mv, n, view, lane, W, dbase, own, oth, rec);
    double c[CH][SPL];
    chunk_costs<SPL, CH>(mv, view, W, dbase, dend, rec, sh.atab, c);
#pragma unroll
    for (int j = 0; j < CH; ++j) {
        if (j < n) {
            const uint32_t lo = mfield(mv, j, 2), hi = mfield(mv, j, 3);
            const uint32_t hidx = hi_hidx(hi);
            double acc[SPL];
#pragma unroll
            for (int k = 0; k < SPL; ++k) acc[k] = 0.0;
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                if ((uint32_t)i < hidx) {
                    const double S = sh.slut[cw_of(lo, hi, i)];
#pragma unroll
                    for (int k = 0; k < SPL; ++k) acc[k] = __builtin_fma(S, lr[j][i][k], acc[k]);
                }
            }
            const uint32_t slot = (uint32_t)(head + first + j);
            store_row<SPL>(U, slot, Dpad, lane, acc);
            store_crow<SPL>(Cst, slot, Dpad, lane, c[j]);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// k_up_chain
// ---------------------------------------------------------------------------------------------
template <int SPL>
struct UpCfg {
    static constexpr int E = SPL == 1 ? 4 : SPL == 2 ? 2 : 1;  // ring entries per helper wave
    static constexpr int R = CHN_HELPERS * E;
};

// entry header: the state word sits next to the weights so one read batch fetches both
struct UpHdr {
    int state;
    uint32_t fl;   // npost | has_heavy << 2
    double s[4];   // S of the heavy child and of posts 0..2
};

template <int SPL>
struct UpRing {
    static constexpr int R = UpCfg<SPL>::R;
    double x[R][64 * SPL];        // Pre in, A_up out
    double post[R][2][64 * SPL];  // rows of the light children after the heavy one
    float c[R][64 * SPL];         // AGD cost
    UpHdr h[R];
    double post3[64 * SPL];       // a tree root's third post-heavy child
    double slut[SM_NUM_W + 1];
};

// The chain wave reads a whole group (state words first, then the rows: in-order LDS execution
// makes rows read after a matching state current) with one wait, re-reading the group in the
// rare case a helper is late.
template <int SPL>
__device__ __forceinline__ void up_chain_wave(UpRing<SPL>& ring, int len, int lane) {
    constexpr int R = UpCfg<SPL>::R;
    constexpr int G = SPL == 1 ? 8 : SPL == 2 ? 6 : 3;  // nodes per group (register budget: 128 VGPRs)
    __builtin_amdgcn_s_setprio(3);
    unsigned spins = 0;
#ifdef SM_CHAIN_PROF
    const long long t0 = clock64();
    long long tr = 0, tc = 0;
#endif
    double x[SPL];
#pragma unroll
    for (int k = 0; k < SPL; ++k) x[k] = 0.0;
    int e0 = 0;  // entry of node j0
    for (int j0 = 0; j0 < len; j0 += G) {
        const int ng = min(G, len - j0);
        int eg[G];
#pragma unroll
        for (int g = 0; g < G; ++g) eg[g] = e0 + g < R ? e0 + g : e0 + g - R;
        double pr[G][SPL], p0[G][SPL], S[G][2];
        float cv[G][SPL];
        uint32_t fl[G];
        bool ok;
#ifdef SM_CHAIN_PROF
        const long long ta = clock64();
#endif
        do {
            int st[G];
#pragma unroll
            for (int g = 0; g < G; ++g)
                if (g < ng) st[g] = lds_state(&ring.h[eg[g]].state);
#pragma unroll
            for (int g = 0; g < G; ++g) {
                if (g < ng) {
                    const int e = eg[g];
                    fl[g] = ring.h[e].fl;
                    S[g][0] = ring.h[e].s[0];
                    S[g][1] = ring.h[e].s[1];
                    lds_row_read<SPL>(ring.x[e], lane, pr[g]);
                    lds_row_read<SPL>(ring.post[e][0], lane, p0[g]);
#pragma unroll
                    for (int k = 0; k < SPL; ++k) cv[g][k] = ring.c[e][lane * SPL + k];
                }
            }
            ok = true;
#pragma unroll
            for (int g = 0; g < G; ++g)
                if (g < ng) ok &= st[g] == 2 * (j0 + g) + 1;
            PROF_SPIN(spins += ok ? 0 : 1);
        } while (!ok);
#ifdef SM_CHAIN_PROF
        const long long tb = clock64();
        tr += tb - ta;
#endif
#pragma unroll
        for (int g = 0; g < G; ++g) {
            if (g < ng) {
                const int e = eg[g];
                const uint32_t npost = fl[g] & 3u;
                double acc[SPL];
                if (fl[g] & 4u) {
#pragma unroll
                    for (int k = 0; k < SPL; ++k) acc[k] = __builtin_fma(S[g][0], x[k], pr[g][k]);
                } else {
#pragma unroll
                    for (int k = 0; k < SPL; ++k) acc[k] = pr[g][k];
                }
                if (npost) {
#pragma unroll
                    for (int k = 0; k < SPL; ++k) acc[k] = __builtin_fma(S[g][1], p0[g][k], acc[k]);
                    if (npost > 1) {  // rare (a few % of nodes): one extra LDS round trip
                        double p[SPL];
                        const double S2 = ring.h[e].s[2];
                        lds_row_read<SPL>(ring.post[e][1], lane, p);
#pragma unroll
                        for (int k = 0; k < SPL; ++k) acc[k] = __builtin_fma(S2, p[k], acc[k]);
                        if (npost > 2) {
                            const double S3 = ring.h[e].s[3];
                            lds_row_read<SPL>(ring.post3, lane, p);
#pragma unroll
                            for (int k = 0; k < SPL; ++k) acc[k] = __builtin_fma(S3, p[k], acc[k]);
                        }
                    }
                }
#pragma unroll
                for (int k = 0; k < SPL; ++k) x[k] = acc[k] + (double)cv[g][k];
                lds_row_write<SPL>(ring.x[e], lane, x);
            }
        }
#pragma unroll
        for (int g = 0; g < G; ++g)
            if (g < ng) lds_publish_ordered(&ring.h[eg[g]].state, 2 * (j0 + g) + 2);
#ifdef SM_CHAIN_PROF
        tc += clock64() - tb;
#endif
        e0 = e0 + G < R ? e0 + G : e0 + G - R;
    }
#ifdef SM_CHAIN_PROF
    if (blockIdx.x == 0 && lane == 0)
        printf("up chain view %d len %d cycles %lld spins %u read %lld compute %lld\n", (int)blockIdx.y, len, clock64() - t0, spins, tr, tc);
#endif
    (void)spins;
}

// Helper waves: every global load of a batch is unconditional (indices clamped into the batch) and
// all conditional stores come last in the iteration, so the compiler's vmcnt bookkeeping stays
// exact and a batch's loads remain in flight while the helper waits for the chain.
template <int SPL>
__device__ __forceinline__ void up_helper_wave(UpRing<SPL>& ring, int hh, int head, int len, int lane,
                                               const uint32_t* __restrict__ meta32, double* __restrict__ U,
                                               const float* __restrict__ Cst, int Dpad) {
    constexpr int E = UpCfg<SPL>::E, R = UpCfg<SPL>::R;
    const int top = head + len - 1;  // node j of the chain sits at slot top - j (bottom first)
    const int b0 = hh * E;
    if (b0 >= len) return;
    MetaVec<E> mv;
    load_meta<E>(mv, meta32, lane, top - b0, -1, min(E, len - b0));
    double rp[E][SPL];  // finished rows of the previous occupants
    int base = b0;
    for (;;) {
        const int n = min(E, len - base);
        // ---- this batch's loads: Pre and C rows (slot-addressed), then the post-heavy children
        double xr[E][SPL], p0[E][SPL], p1[E][SPL];
        float cr[E][SPL];
#pragma unroll
        for (int k = 0; k < E; ++k) {
            const int kk = min(k, n - 1);
            const uint32_t slot = (uint32_t)(top - (base + kk));
            load_row<SPL>(U, slot, Dpad, lane, xr[k]);
            load_crow<SPL>(Cst, slot, Dpad, lane, cr[k]);
        }
        uint32_t npost[E];
#pragma unroll
        for (int k = 0; k < E; ++k) {
            const int kk = min(k, n - 1);
            const uint32_t hi = mfield(mv, kk, 3);
            const uint32_t nch = hi_nch(hi), hidx = hi_hidx(hi);
            npost[k] = base + kk > 0 ? nch - 1u - hidx : 0u;
            // absent posts load the path head's rows (L2-resident dummies): a dummy equal to a
            // slot loaded above would be folded into a register copy that waits for that load
            const uint32_t s0 = npost[k] >= 1 ? mfield(mv, kk, 4 + (int)min(hidx + 1u, 3u)) : (uint32_t)head;
            const uint32_t s1 = npost[k] >= 2 ? mfield(mv, kk, 4 + (int)min(hidx + 2u, 3u)) : (uint32_t)head + 1u;
            load_row<SPL>(U, s0, Dpad, lane, p0[k]);
            load_row<SPL>(U, s1, Dpad, lane, p1[k]);
        }
        // ---- previous occupants of this helper's entries (all E existed): wait, read back
        if (base >= R) {
#pragma unroll
            for (int k = 0; k < E; ++k) {
                const int e = b0 + k;
                lds_wait(&ring.h[e].state, 2 * (base - R + k) + 2, true);
                lds_row_read<SPL>(ring.x[e], lane, rp[k]);
            }
        }
        // ---- fill the entries and publish
        vm_drain();
#pragma unroll
        for (int k = 0; k < E; ++k) {
            if (k < n) {
                const int e = b0 + k;
                lds_row_write<SPL>(ring.x[e], lane, xr[k]);
#pragma unroll
                for (int q = 0; q < SPL; ++q) ring.c[e][lane * SPL + q] = cr[k][q];
                if (npost[k] >= 1) lds_row_write<SPL>(ring.post[e][0], lane, p0[k]);
                if (npost[k] >= 2) lds_row_write<SPL>(ring.post[e][1], lane, p1[k]);
                const uint32_t lo = mfield(mv, k, 2), hi = mfield(mv, k, 3);
                const uint32_t nch = hi_nch(hi), hidx = hi_hidx(hi);
                if (npost[k] >= 3) {  // a tree root: one synchronous load per tree
                    double p3[SPL];
                    load_row<SPL>(U, mfield(mv, k, 7), Dpad, lane, p3);
                    lds_row_write<SPL>(ring.post3, lane, p3);
                }
                const bool has_heavy = base + k > 0;
                if (lane < 4) {
                    const uint32_t i = hidx + (uint32_t)lane;  // lane 0: heavy child, lanes 1..3: posts
                    const bool live = has_heavy && i < nch;
                    ring.h[e].s[lane] = ring.slut[live ? cw_of(lo, hi, (int)i) : (uint32_t)S_ZERO];
                }
                if (lane == 0) ring.h[e].fl = npost[k] | (has_heavy ? 4u : 0u);
            }
        }
#pragma unroll
        for (int k = 0; k < E; ++k)
            if (k < n) lds_publish(&ring.h[b0 + k].state, 2 * (base + k) + 1);
        // ---- store the previous occupants' A_up rows
        if (base >= R) {
#pragma unroll
            for (int k = 0; k < E; ++k) store_row<SPL>(U, (uint32_t)(top - (base - R + k)), Dpad, lane, rp[k]);
        }
        const int nb = base + R;
        if (nb >= len) break;
        load_meta<E>(mv, meta32, lane, top - nb, -1, min(E, len - nb));
        base = nb;
    }
    // ---- retire the last batch
    const int n = min(E, len - base);
#pragma unroll
    for (int k = 0; k < E; ++k) {
        if (k < n) {
            const int e = b0 + k;
            lds_wait(&ring.h[e].state, 2 * (base + k) + 2, true);
            lds_row_read<SPL>(ring.x[e], lane, rp[k]);
            store_row<SPL>(U, (uint32_t)(top - (base + k)), Dpad, lane, rp[k]);
        }
    }
}

template <int SPL>
__global__ __launch_bounds__(CHN_THREADS) void k_up_chain(WalkView V0, WalkView V1, const uint32_t* __restrict__ meta0,
                                                          const uint32_t* __restrict__ meta1,
                                                          const SmPath* __restrict__ paths0,
                                                          const SmPath* __restrict__ paths1,
                                                          const float* __restrict__ Cst0, const float* __restrict__ Cst1,
                                                          const double* __restrict__ slut_g, int Dpad) {
    __shared__ UpRing<SPL> ring;
    const int view = blockIdx.y;
    const WalkView& V = view ? V1 : V0;
    if ((int)blockIdx.x >= V.npaths) return;  // uniform over the block
    const SmPath path = (view ? paths1 : paths0)[blockIdx.x];
    const int head = (int)uniform(path.head), len = (int)uniform(path.len);
    for (int i = threadIdx.x; i < UpCfg<SPL>::R; i += CHN_THREADS) ring.h[i].state = 0;
    for (int i = threadIdx.x; i < SM_NUM_W; i += CHN_THREADS) ring.slut[i] = slut_g[i];
    if (threadIdx.x == 0) ring.slut[SM_NUM_W] = 0.0;
    __syncthreads();
    const int wave = (int)uniform(threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (wave == 0)
        up_chain_wave<SPL>(ring, len, lane);
    else
        up_helper_wave<SPL>(ring, wave - 1, head, len, lane, view ? meta1 : meta0, V.U, view ? Cst1 : Cst0, Dpad);
}

// ---------------------------------------------------------------------------------------------
// k_down_chain
// ---------------------------------------------------------------------------------------------
template <int SPL>
struct DownCfg {
    static constexpr int E = SPL == 1 ? 8 : SPL == 2 ? 6 : 3;
    static constexpr int R = CHN_HELPERS * E;
};

struct DownHdr {
    int state;
    uint32_t pix;
    uint32_t store;  // row needed by light children (or the debug path)
    uint32_t pad;
    double S;
};

template <int SPL>
struct DownRing {
    static constexpr int R = DownCfg<SPL>::R;
    double x[R][64 * SPL];  // T = S2 * A_up in, A out
    DownHdr h[R];
    double slut[SM_NUM_W + 1];
    double s2lut[SM_NUM_W];
};

template <int SPL>
__device__ __forceinline__ void down_chain_wave(DownRing<SPL>& ring, int len, int lane, const double* __restrict__ U,
                                                uint32_t hparent, int Dpad) {
    constexpr int R = DownCfg<SPL>::R;
    __builtin_amdgcn_s_setprio(3);
    unsigned spins = 0;
#ifdef SM_CHAIN_PROF
    const long long t0 = clock64();
    long long tr = 0, tc = 0;
#endif
    double x[SPL];
    if (hparent != SM_NONE) {
        load_row<SPL>(U, hparent, Dpad, lane, x);  // A(parent): finished in an earlier round
    } else {
#pragma unroll
        for (int k = 0; k < SPL; ++k) x[k] = 0.0;  // root: S = 0, T = A_up -> A(root) = A_up(root)
    }
    int e0 = 0;
    for (int j0 = 0; j0 < len; j0 += CHN_G) {
        const int ng = min(CHN_G, len - j0);
        int eg[CHN_G];
#pragma unroll
        for (int g = 0; g < CHN_G; ++g) eg[g] = e0 + g < R ? e0 + g : e0 + g - R;
        double t[CHN_G][SPL], S[CHN_G];
        bool ok;
#ifdef SM_CHAIN_PROF
        const long long ta = clock64();
#endif
        do {
            int st[CHN_G];
#pragma unroll
            for (int g = 0; g < CHN_G; ++g)
                if (g < ng) st[g] = lds_state(&ring.h[eg[g]].state);
#pragma unroll
            for (int g = 0; g < CHN_G; ++g) {
                if (g < ng) {
                    S[g] = ring.h[eg[g]].S;
                    lds_row_read<SPL>(ring.x[eg[g]], lane, t[g]);
                }
            }
            ok = true;
#pragma unroll
            for (int g = 0; g < CHN_G; ++g)
                if (g < ng) ok &= st[g] == 2 * (j0 + g) + 1;
            PROF_SPIN(spins += ok ? 0 : 1);
        } while (!ok);
#ifdef SM_CHAIN_PROF
        const long long tb = clock64();
        tr += tb - ta;
#endif
#pragma unroll
        for (int g = 0; g < CHN_G; ++g) {
            if (g < ng) {
#pragma unroll
                for (int k = 0; k < SPL; ++k) x[k] = __builtin_fma(S[g], x[k], t[g][k]);
                lds_row_write<SPL>(ring.x[eg[g]], lane, x);
            }
        }
#pragma unroll
        for (int g = 0; g < CHN_G; ++g)
            if (g < ng) lds_publish_ordered(&ring.h[eg[g]].state, 2 * (j0 + g) + 2);
#ifdef SM_CHAIN_PROF
        tc += clock64() - tb;
#endif
        e0 = e0 + CHN_G < R ? e0 + CHN_G : e0 + CHN_G - R;
    }
#ifdef SM_CHAIN_PROF
    if (blockIdx.x == 0 && lane == 0)
        printf("down chain view %d len %d cycles %lld spins %u read %lld compute %lld\n", (int)blockIdx.y, len, clock64() - t0, spins, tr, tc);
#endif
    (void)spins;
}

// finished entries of a helper: wait, read back, WTA (lane k < n gets node k's result)
template <int SPL>
struct DownDone {
    double xs[DownCfg<SPL>::E][SPL];
    double mn;
    int mi;
};

template <int SPL>
__device__ __forceinline__ void down_collect(DownRing<SPL>& ring, int b0, int jbase, int n, int lane, int dcall,
                                             DownDone<SPL>& d) {
    constexpr int E = DownCfg<SPL>::E;
#pragma unroll
    for (int k = 0; k < E; ++k) {
        if (k < n) {
            lds_wait(&ring.h[b0 + k].state, 2 * (jbase + k) + 2, true);
            lds_row_read<SPL>(ring.x[b0 + k], lane, d.xs[k]);
        } else {
#pragma unroll
            for (int q = 0; q < SPL; ++q) d.xs[k][q] = 0.0;
        }
    }
    wta_chunk<SPL, E>(d.xs, lane, lane * SPL, dcall, d.mn, d.mi);
}

// stores of collected entries (must read ring.pix/store before the entries are refilled)
template <int SPL>
__device__ __forceinline__ void down_store(const DownDone<SPL>& d, int head, int jbase, int n, int lane,
                                           const uint32_t (&st)[DownCfg<SPL>::E], uint32_t pix, double* __restrict__ U,
                                           const WalkView& V, int Dpad, int dglob0, int store_all) {
    constexpr int E = DownCfg<SPL>::E;
#pragma unroll
    for (int k = 0; k < E; ++k)
        if (k < n && (store_all || st[k])) store_row<SPL>(U, (uint32_t)(head + jbase + k), Dpad, lane, d.xs[k]);
    if (lane < n) {
        V.idx[pix] = dglob0 + d.mi;
        V.minc[pix] = d.mn;
        V.disp[pix] = (float)(dglob0 + d.mi);
    }
}

template <int SPL>
__device__ __forceinline__ void down_helper_wave(DownRing<SPL>& ring, int hh, int head, int len, int lane,
                                                 uint32_t hparent, const uint32_t* __restrict__ meta32,
                                                 const WalkView& V, int Dpad, int dcall, int dglob0, int store_all) {
    constexpr int E = DownCfg<SPL>::E, R = DownCfg<SPL>::R;
    const int b0 = hh * E;
    if (b0 >= len) return;
    double* __restrict__ U = V.U;
    DownDone<SPL> done;
    uint32_t st[E], pix = 0;
    int base = b0;
    for (;;) {
        const int n = min(E, len - base);
        // ---- this batch's loads (unconditional): A_up rows and metadata
        double u[E][SPL];
#pragma unroll
        for (int k = 0; k < E; ++k) load_row<SPL>(U, (uint32_t)(head + base + min(k, n - 1)), Dpad, lane, u[k]);
        MetaVec<E> mv;
        load_meta<E>(mv, meta32, lane, head + base, 1, n);
        // ---- previous occupants: wait, read back, WTA; keep their store flags and pixels
        if (base >= R) {
            down_collect<SPL>(ring, b0, base - R, E, lane, dcall, done);
#pragma unroll
            for (int k = 0; k < E; ++k) st[k] = ring.h[b0 + k].store;
            pix = ring.h[b0 + min(lane, E - 1)].pix;
        }
        // ---- fill and publish
        vm_drain();
#pragma unroll
        for (int k = 0; k < E; ++k) {
            if (k < n) {
                const int e = b0 + k;
                const bool root = base + k == 0 && hparent == SM_NONE;
                const uint32_t wp = lo_wp(mfield(mv, k, 2));
                const double S = root ? 0.0 : ring.slut[wp];
                const double S2 = ring.s2lut[wp];
                double t[SPL];
#pragma unroll
                for (int q = 0; q < SPL; ++q) t[q] = root ? u[k][q] : S2 * u[k][q];
                lds_row_write<SPL>(ring.x[e], lane, t);
                if (lane == 0) {
                    ring.h[e].S = S;
                    ring.h[e].pix = mfield(mv, k, 0);
                    ring.h[e].store = hi_light(mfield(mv, k, 3));
                }
            }
        }
#pragma unroll
        for (int k = 0; k < E; ++k)
            if (k < n) lds_publish(&ring.h[b0 + k].state, 2 * (base + k) + 1);
        // ---- the previous occupants' stores
        if (base >= R) down_store<SPL>(done, head, base - R, E, lane, st, pix, U, V, Dpad, dglob0, store_all);
        if (base + R >= len) break;
        base += R;
    }
    const int n = min(E, len - base);
    down_collect<SPL>(ring, b0, base, n, lane, dcall, done);
#pragma unroll
    for (int k = 0; k < E; ++k) st[k] = ring.h[b0 + k].store;
    pix = ring.h[b0 + min(lane, E - 1)].pix;
    down_store<SPL>(done, head, base, n, lane, st, pix, U, V, Dpad, dglob0, store_all);
}

template <int SPL>
__global__ __launch_bounds__(CHN_THREADS) void k_down_chain(WalkView V0, WalkView V1,
                                                            const uint32_t* __restrict__ meta0,
                                                            const uint32_t* __restrict__ meta1,
                                                            const SmPath* __restrict__ paths0,
                                                            const SmPath* __restrict__ paths1,
                                                            const double* __restrict__ slut_g,
                                                            const double* __restrict__ s2lut_g, int Dpad, int dcall,
                                                            int dglob0, int store_all) {
    __shared__ DownRing<SPL> ring;
    const int view = blockIdx.y;
    const WalkView& V = view ? V1 : V0;
    if ((int)blockIdx.x >= V.npaths) return;
    const uint32_t* __restrict__ meta32 = view ? meta1 : meta0;
    const SmPath path = (view ? paths1 : paths0)[blockIdx.x];
    const int head = (int)uniform(path.head), len = (int)uniform(path.len);
    const uint32_t hparent = uniform(meta32[(size_t)head * 8 + 1]);
    for (int i = threadIdx.x; i < DownCfg<SPL>::R; i += CHN_THREADS) ring.h[i].state = 0;
    for (int i = threadIdx.x; i < SM_NUM_W; i += CHN_THREADS) {
        ring.slut[i] = slut_g[i];
        ring.s2lut[i] = s2lut_g[i];
    }
    if (threadIdx.x == 0) ring.slut[SM_NUM_W] = 0.0;
    __syncthreads();
    const int wave = (int)uniform(threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (wave == 0)
        down_chain_wave<SPL>(ring, len, lane, V.U, hparent, Dpad);
    else
        down_helper_wave<SPL>(ring, wave - 1, head, len, lane, hparent, meta32, V, Dpad, dcall, dglob0, store_all);
}

// ---------------------------------------------------------------------------------------------
static WalkView chain_view(const WalkArgs& a, int v) { return WalkView{a.npaths[v], a.U[v], a.idx[v], a.minc[v], a.disp[v]}; }

template <int SPL, int CH>
static void up_pre_launch(hipStream_t st, const WalkArgs& a) {
    const int ns = a.nseg[0] > a.nseg[1] ? a.nseg[0] : a.nseg[1];
    if (ns == 0) return;
    hipLaunchKernelGGL((k_up_pre<SPL, CH>), dim3(ns, 2), dim3(64 * SM_PRE_SEG / CH), 0, st, chain_view(a, 0),
                       chain_view(a, 1), reinterpret_cast<const uint32_t*>(a.meta[0]),
                       reinterpret_cast<const uint32_t*>(a.meta[1]), a.paths[0], a.paths[1], a.segtab[0], a.segtab[1],
                       a.nseg[0], a.nseg[1], a.Cst[0], a.Cst[1], a.Lrec, a.Rrec, a.atab, a.slut, a.s2lut, a.W, a.Dpad,
                       a.dcall, a.dglob0);
}

template <int SPL>
static void up_chain_launch(hipStream_t st, const WalkArgs& a, int np) {
    hipLaunchKernelGGL((k_up_chain<SPL>), dim3(np, 2), dim3(CHN_THREADS), 0, st, chain_view(a, 0), chain_view(a, 1),
                       reinterpret_cast<const uint32_t*>(a.meta[0]), reinterpret_cast<const uint32_t*>(a.meta[1]),
                       a.paths[0], a.paths[1], a.Cst[0], a.Cst[1], a.slut, a.Dpad);
}

template <int SPL>
static void down_chain_launch(hipStream_t st, const WalkArgs& a, int np, int store_all) {
    hipLaunchKernelGGL((k_down_chain<SPL>), dim3(np, 2), dim3(CHN_THREADS), 0, st, chain_view(a, 0), chain_view(a, 1),
                       reinterpret_cast<const uint32_t*>(a.meta[0]), reinterpret_cast<const uint32_t*>(a.meta[1]),
                       a.paths[0], a.paths[1], a.slut, a.s2lut, a.Dpad, a.dcall, a.dglob0, store_all);
}

hipError_t launch_up_long(hipStream_t st, const WalkArgs& a, int spl) {
    const int np = a.npaths[0] > a.npaths[1] ? a.npaths[0] : a.npaths[1];
    if (np == 0) return hipSuccess;
    switch (spl) {
        case 1: up_pre_launch<1, 8>(st, a); up_chain_launch<1>(st, a, np); break;
        case 2: up_pre_launch<2, 8>(st, a); up_chain_launch<2>(st, a, np); break;
        default: up_pre_launch<4, 4>(st, a); up_chain_launch<4>(st, a, np); break;
    }
    return hipGetLastError();
}

hipError_t launch_down_long(hipStream_t st, const WalkArgs& a, int spl, int store_all) {
    const int np = a.npaths[0] > a.npaths[1] ? a.npaths[0] : a.npaths[1];
    if (np == 0) return hipSuccess;
    switch (spl) {
        case 1: down_chain_launch<1>(st, a, np, store_all); break;
        case 2: down_chain_launch<2>(st, a, np, store_all); break;
        default: down_chain_launch<4>(st, a, np, store_all); break;
    }
    return hipGetLastError();
}
