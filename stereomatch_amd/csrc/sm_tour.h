// sm_tour.h -- list ranking of Euler tours over grid arcs (arc a = 4p + k; k: 0 right, 1 down,
// 2 left, 3 up), shared by the tree layout (sm_layout_gpu.hip: one tour of the MST) and the MST_PMS
// schedule forest (sm_pms_forest.hip: one tour per tree, two child orders).  Library-internal.
//
// A graph G supplies has(p, k) (arc 4p+k exists) and succ(a) (the next arc of a's list, SM_NONE at
// the end of a list).  Three levels:
//   L1 tour_tile       : per 32x32 tile, LDS pointer jumping contracts every maximal run of a list
//                        inside the tile into one chain (distance to the chain end, chain id)
//   L2 tour_chain_init : chain successor + length; tour_chain_rank: in-place pointer jumping over the
//                        chains, cnw[c] >> 32 = arcs from chain c's head to the end of its list
//   L3 (caller)        : arcs from arc a to its list's end, inclusive =
//                        (cnw[c] >> 32) - (c_len[c] - a_dist[a]), c = a_cid[a]
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sm_common.h"

#define TL 32                 // tile side
#define TLP (TL * TL)         // pixels per tile
#define TLS (4 * TLP)         // arc slots per tile
#define TL_THREADS 256
#define L_EXIT 0xFFFFu        // successor leaves the tile
#define L_NIL 0xFFFEu         // end of a list

struct TourBufs {
    // per arc (4N)
    uint16_t* a_dist;   // arcs from the arc to its chain's end, inclusive
    uint32_t* a_cid;    // the arc's chain
    // per chain
    uint32_t* nchains;  // device counter
    uint32_t* c_last;
    uint32_t* c_len;
    uint64_t* cnw;      // successor chain (low 32 bits) | arcs to it (high 32 bits)
};

__device__ __forceinline__ uint32_t tour_nbr(uint32_t p, int k, int W) {
    return k == 0 ? p + 1 : k == 1 ? p + (uint32_t)W : k == 2 ? p - 1 : p - (uint32_t)W;
}

// L1: contract the lists inside the 32x32 tile at (tx0, ty0).  One 64-bit LDS word per arc
// slot, nxt | dist << 16 | last << 32, so a jump is one gathered word; every thread keeps its 16 words
// in registers.
template <class G>
__device__ __forceinline__ void tour_tile(const G& g, const TourBufs& T, int W, int H, int tx0, int ty0) {
    __shared__ union {
        uint64_t w[TLS];
        uint16_t h[4 * TLS];  // once the jumping is done, h[4*s + 2]: the tile-local id of the chain whose
                              // last slot is s (bits 32..47 of w[s], which nobody reads any more)
    } st;
    __shared__ uint8_t haspred[TLS];
    constexpr int PER = TLS / TL_THREADS;  // 16 slots per thread
    for (int i = 0; i < PER; ++i) haspred[threadIdx.x + i * TL_THREADS] = 0;
    __syncthreads();
    uint64_t own[PER];
    for (int i = 0; i < PER; ++i) {
        const int s = threadIdx.x + i * TL_THREADS;
        const int lp = s >> 2, k = s & 3;
        const int lx = lp % TL, ly = lp / TL;
        const int x = tx0 + lx, y = ty0 + ly;
        uint32_t n = L_NIL, dd = 0;
        if (x < W && y < H) {
            const uint32_t p = (uint32_t)(y * W + x);
            if (g.has(p, k)) {
                dd = 1;
                const uint32_t sa = g.succ(4u * p + (uint32_t)k);
                if (sa != SM_NONE) {
                    // the successor leaves from q = the neighbour of p in direction k: its tile
                    // coordinates follow from p's without a division by W
                    const int qx = lx + (k == 0 ? 1 : k == 2 ? -1 : 0), qy = ly + (k == 1 ? 1 : k == 3 ? -1 : 0);
                    if (qx >= 0 && qx < TL && qy >= 0 && qy < TL) {
                        n = (uint32_t)(4 * (qy * TL + qx) + (int)(sa & 3u));
                        haspred[n] = 1;
                    } else {
                        n = L_EXIT;
                    }
                }
            }
        }
        own[i] = (uint64_t)n | ((uint64_t)dd << 16) | ((uint64_t)s << 32);
        st.w[s] = own[i];
    }
    __syncthreads();
    // pointer jumping: dist -> arcs to chain end (inclusive), last -> chain's last slot.  Only the words
    // that moved are written back (a word that reached its chain's end is final in LDS already): the
    // loop is bound by LDS traffic, and most chains finish long before the tile's longest
    for (int it = 0; it < 13; ++it) {
        uint32_t moved = 0;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const uint32_t n = (uint32_t)own[i] & 0xFFFFu;
            if (n < L_NIL) {
                const uint64_t nb = st.w[n];
                const uint32_t d = (uint32_t)(own[i] >> 16) + (uint32_t)(nb >> 16);  // low 16 bits: the sum
                own[i] = (nb & 0xFFFF0000FFFFull) | ((uint64_t)(d & 0xFFFFu) << 16);
                moved |= 1u << i;
            }
        }
        if (!__syncthreads_or(moved != 0)) break;
#pragma unroll
        for (int i = 0; i < PER; ++i)
            if ((moved >> i) & 1u) st.w[threadIdx.x + i * TL_THREADS] = own[i];
        __syncthreads();
    }
    // heads: existing arcs without an in-tile predecessor; register chains
    __shared__ uint32_t nheads, cbase;
    if (threadIdx.x == 0) nheads = 0;
    __syncthreads();
    uint32_t myhead[PER];
    for (int i = 0; i < PER; ++i) {
        const int s = threadIdx.x + i * TL_THREADS;
        const uint32_t dist = (uint32_t)(own[i] >> 16) & 0xFFFFu, last = (uint32_t)(own[i] >> 32) & 0xFFFFu;
        myhead[i] = SM_NONE;
        if (dist != 0 && !haspred[s]) {
            myhead[i] = atomicAdd(&nheads, 1u);  // LDS atomic: rank of this chain inside the tile
            st.h[4 * last + 2] = (uint16_t)myhead[i];
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) cbase = atomicAdd(T.nchains, nheads);  // one global atomic per tile
    __syncthreads();
    for (int i = 0; i < PER; ++i) {
        const int s = threadIdx.x + i * TL_THREADS;
        const uint32_t dist = (uint32_t)(own[i] >> 16) & 0xFFFFu, last = (uint32_t)(own[i] >> 32) & 0xFFFFu;
        if (dist == 0) continue;
        const int lp = s >> 2, k = s & 3;
        const uint32_t p = (uint32_t)((ty0 + lp / TL) * W + tx0 + lp % TL);
        const uint32_t a = 4u * p + (uint32_t)k;
        const uint32_t cid = cbase + st.h[4 * last + 2];  // every arc its chain's id
        T.a_dist[a] = (uint16_t)dist;
        T.a_cid[a] = cid;
        if (myhead[i] != SM_NONE) {
            const int llp = (int)last >> 2;
            const uint32_t lpix = (uint32_t)((ty0 + llp / TL) * W + tx0 + llp % TL);
            T.c_last[cid] = 4u * lpix + (last & 3u);
            T.c_len[cid] = dist;
        }
    }
}

// L2 init: chain successor + weight (one thread per chain)
template <class G>
__device__ __forceinline__ void tour_chain_init(const G& g, const TourBufs& T, uint32_t c) {
    if (c >= *T.nchains) return;
    const uint32_t s = g.succ(T.c_last[c]);
    const uint32_t n = s == SM_NONE ? SM_NONE : T.a_cid[s];
    T.cnw[c] = ((uint64_t)T.c_len[c] << 32) | n;
}

// L2: suffix sums over the chain lists by in-place pointer jumping, one launch.  Every word {n, w}
// satisfies "w = arcs from this chain up to (not including) chain n" whichever update of it a reader
// sees (the pair is one 64-bit access), so no step needs a grid barrier.  The grid must be at most
// co-resident size, and every thread sweeps its chains, one jump each per sweep, until all have
// reached their list's end: with one thread per chain, threads that were not yet resident left the
// resident ones reading never-updated words, i.e. advancing one chain per step (19.7 ms at
// 3840x2160).  Every jump moves strictly forward along an acyclic list, so the loop ends (the caller
// guarantees the lists are acyclic: a tree's Euler tour); with fresh words it takes ~log2(chains)
// sweeps.  Integer sums: the result is exact.
__device__ __forceinline__ void tour_chain_rank(const TourBufs& T) {
    const uint32_t nch = *T.nchains;
    uint64_t* nw = T.cnw;
    const uint32_t stride = gridDim.x * blockDim.x;
    for (;;) {
        bool any = false;
        for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < nch; c += stride) {
            const uint64_t me = __hip_atomic_load(nw + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t n = (uint32_t)me;
            if (n == SM_NONE) continue;
            const uint64_t nb = __hip_atomic_load(nw + n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t w = (uint32_t)(me >> 32) + (uint32_t)(nb >> 32);
            __hip_atomic_store(nw + c, ((uint64_t)w << 32) | (uint32_t)nb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            any = true;
        }
        if (!any) break;
    }
}

// L3: arcs from arc a to the end of its list, inclusive
__device__ __forceinline__ uint32_t tour_suffix(const TourBufs& T, uint32_t a) {
    const uint32_t c = T.a_cid[a];
    return (uint32_t)(T.cnw[c] >> 32) - (T.c_len[c] - T.a_dist[a]);
}
