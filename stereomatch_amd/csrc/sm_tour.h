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
//                        (cnw[c] >> 32) - (c_len[c] - a_dist[a]), c = a_cid[a]; tour_chain_rank leaves
//                        the first two terms folded in c_len, so this is one gather
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
// arcs leaving a tile's pixels along a forest: 2 per edge inside the tile (<= TLP - 1 edges) plus one per
// edge across its border (<= 4 TL): the compact word array's size (round 5: 18 KB of LDS instead of 32,
// 7 blocks per CU instead of 4)
#define TL_ARCS (2 * (TLP - 1) + 4 * TL)

struct TourBufs {
    // per arc (4N)
    uint16_t* a_dist;   // arcs from the arc to its chain's end, inclusive
    uint32_t* a_cid;    // the arc's chain
    // per chain
    uint32_t* nchains;  // device counter
    uint32_t* c_last;
    uint32_t* c_len;    // the chain's arcs; after tour_chain_rank its suffix base: (arcs from its head to
                        // its list's end) - (its arcs), so an arc's suffix is one gather (tour_suffix)
    uint64_t* cnw;      // successor chain (low 32 bits) | arcs to it (high 32 bits)
    int32_t* err;       // a tile with more than TL_ARCS arcs (not a forest) ORs errv in here
    int32_t errv;
};

__device__ __forceinline__ uint32_t tour_nbr(uint32_t p, int k, int W) {
    return k == 0 ? p + 1 : k == 1 ? p + (uint32_t)W : k == 2 ? p - 1 : p - (uint32_t)W;
}

// L1: contract the lists inside the 32x32 tile at (tx0, ty0).  One 64-bit LDS word per arc,
// nxt | dist << 16 | last << 32 | slot << 48, so a jump is one gathered word; every thread keeps its words
// in registers.  The tile's arcs that exist (about half of its 4096 slots: a tree has ~2 arcs per pixel)
// are first compacted in slot order (round 5: the jumping loop issued all 16 slots per thread every
// iteration, live or not), so the loop runs over ceil(arcs / 256) words per thread.
template <class G>
__device__ __forceinline__ void tour_tile(const G& g, const TourBufs& T, int W, int H, int tx0, int ty0) {
    __shared__ union {
        uint64_t w[TL_ARCS];
        uint16_t h[4 * TL_ARCS];  // h[s] (s < TLS) during the compaction: slot s's compact index; once the
                                  // jumping is done, h[4*j + 2]: the tile-local id of the chain whose last
                                  // arc is j (bits 32..47 of w[j], which nobody reads any more), h[4*j + 3]:
                                  // j's slot
    } st;
    static_assert(4 * TL_ARCS >= TLS, "the compaction's index table fits the word array");
    __shared__ uint32_t haspred[(TL_ARCS + 31) / 32];  // a bit per arc (bytes held the block to 7 per CU)
    __shared__ uint32_t s_cnt[64];
    constexpr int PER = TLS / TL_THREADS;  // 16 slots per thread
    static_assert(PER * (TL_THREADS / 64) == 64, "one wave scans the per-(slot row, wave) counts");
    const int lane = (int)threadIdx.x & 63, wave = (int)threadIdx.x >> 6;
    for (int i = threadIdx.x; i < (TL_ARCS + 31) / 32; i += TL_THREADS) haspred[i] = 0u;
    // successors in slot space; compact ranks in slot order: slot s = threadIdx.x + 256 i, so for each i
    // the waves hold consecutive runs of 64 slots
    uint32_t nxt[PER], rk[PER], live = 0;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int s = threadIdx.x + i * TL_THREADS;
        const int lp = s >> 2, k = s & 3;
        const int lx = lp % TL, ly = lp / TL;
        const int x = tx0 + lx, y = ty0 + ly;
        uint32_t n = L_NIL;
        bool has = false;
        if (x < W && y < H) {
            const uint32_t p = (uint32_t)(y * W + x);
            if (g.has(p, k)) {
                has = true;
                const uint32_t sa = g.succ(4u * p + (uint32_t)k);
                if (sa != SM_NONE) {
                    // the successor leaves from q = the neighbour of p in direction k: its tile
                    // coordinates follow from p's without a division by W
                    const int qx = lx + (k == 0 ? 1 : k == 2 ? -1 : 0), qy = ly + (k == 1 ? 1 : k == 3 ? -1 : 0);
                    n = (qx >= 0 && qx < TL && qy >= 0 && qy < TL) ? (uint32_t)(4 * (qy * TL + qx) + (int)(sa & 3u)) : L_EXIT;
                }
            }
        }
        nxt[i] = n;
        const uint64_t b = __ballot(has);
        rk[i] = (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
        if (has) live |= 1u << i;
        if (lane == 0) s_cnt[i * (TL_THREADS / 64) + wave] = (uint32_t)__popcll(b);
    }
    __syncthreads();
    __shared__ uint32_t s_base[64], s_count;
    if (wave == 0) {
        const uint32_t c = s_cnt[lane];
        uint32_t x = c;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(x, off);
            if (lane >= off) x += y;
        }
        s_base[lane] = x - c;
        if (lane == 63) s_count = x;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        rk[i] += s_base[i * (TL_THREADS / 64) + wave];
        if ((live >> i) & 1u) st.h[threadIdx.x + i * TL_THREADS] = (uint16_t)rk[i];
    }
    const uint32_t count = s_count;
    if (count > (uint32_t)TL_ARCS) {  // (block-uniform) not a forest: never write past the LDS arrays
        if (threadIdx.x == 0 && T.err) atomicOr(T.err, T.errv);
        return;
    }
    __syncthreads();
    // the compact words: successor remapped, distance 1, last = itself, slot
    uint64_t nw[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        nw[i] = 0;
        if (!((live >> i) & 1u)) continue;
        const uint32_t n = nxt[i];
        const uint32_t nc = n < L_NIL ? (uint32_t)st.h[n] : n;
        if (n < L_NIL) atomicOr(&haspred[nc >> 5], 1u << (nc & 31u));
        nw[i] = (uint64_t)nc | (1ull << 16) | ((uint64_t)rk[i] << 32) | ((uint64_t)(threadIdx.x + i * TL_THREADS) << 48);
    }
    __syncthreads();  // (h read: now the words overwrite it)
#pragma unroll
    for (int i = 0; i < PER; ++i)
        if ((live >> i) & 1u) st.w[rk[i]] = nw[i];
    __syncthreads();
    // compact word j is owned by thread j % 256
    const int nper = (int)((count + TL_THREADS - 1) / TL_THREADS);
    uint64_t own[PER];
#pragma unroll
    for (int m = 0; m < PER; ++m) {
        const uint32_t j = threadIdx.x + m * TL_THREADS;
        own[m] = (m < nper && j < count) ? st.w[j] : (uint64_t)L_NIL;  // (dist 0: no arc)
    }
    // pointer jumping: dist -> arcs to chain end (inclusive), last -> chain's last arc.  Only the words
    // that moved are written back (a word that reached its chain's end is final in LDS already)
    for (int it = 0; it < 13; ++it) {
        uint32_t moved = 0;
#pragma unroll
        for (int m = 0; m < PER; ++m) {
            if (m >= nper) break;  // (block-uniform)
            const uint32_t n = (uint32_t)own[m] & 0xFFFFu;
            if (n < L_NIL) {
                const uint64_t nb = st.w[n];
                const uint32_t d = (uint32_t)(own[m] >> 16) + (uint32_t)(nb >> 16);  // low 16 bits: the sum
                own[m] = (nb & 0x0000FFFF0000FFFFull) | ((uint64_t)(d & 0xFFFFu) << 16) | (own[m] & 0xFFFF000000000000ull);
                moved |= 1u << m;
            }
        }
        if (!__syncthreads_or(moved != 0)) break;
#pragma unroll
        for (int m = 0; m < PER; ++m)
            if ((moved >> m) & 1u) st.w[threadIdx.x + m * TL_THREADS] = own[m];
        __syncthreads();
    }
    // heads: arcs without an in-tile predecessor; register chains
    __shared__ uint32_t nheads, cbase;
    if (threadIdx.x == 0) nheads = 0;
    __syncthreads();
    uint32_t myhead[PER];
#pragma unroll
    for (int m = 0; m < PER; ++m) {
        const uint32_t j = threadIdx.x + m * TL_THREADS;
        const uint32_t dist = (uint32_t)(own[m] >> 16) & 0xFFFFu, last = (uint32_t)(own[m] >> 32) & 0xFFFFu;
        myhead[m] = SM_NONE;
        if (m < nper && dist != 0 && !((haspred[j >> 5] >> (j & 31u)) & 1u)) {
            myhead[m] = atomicAdd(&nheads, 1u);  // LDS atomic: rank of this chain inside the tile
            st.h[4 * last + 2] = (uint16_t)myhead[m];
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) cbase = atomicAdd(T.nchains, nheads);  // one global atomic per tile
    __syncthreads();
#pragma unroll
    for (int m = 0; m < PER; ++m) {
        const uint32_t dist = (uint32_t)(own[m] >> 16) & 0xFFFFu, last = (uint32_t)(own[m] >> 32) & 0xFFFFu;
        if (m >= nper || dist == 0) continue;
        const int s = (int)(own[m] >> 48);
        const int lp = s >> 2, k = s & 3;
        const uint32_t p = (uint32_t)((ty0 + lp / TL) * W + tx0 + lp % TL);
        const uint32_t a = 4u * p + (uint32_t)k;
        const uint32_t cid = cbase + st.h[4 * last + 2];  // every arc its chain's id
        T.a_dist[a] = (uint16_t)dist;
        T.a_cid[a] = cid;
        if (myhead[m] != SM_NONE) {
            const int ls = (int)st.h[4 * last + 3];  // the last arc's slot
            const int llp = ls >> 2;
            const uint32_t lpix = (uint32_t)((ty0 + llp / TL) * W + tx0 + llp % TL);
            T.c_last[cid] = 4u * lpix + (uint32_t)(ls & 3);
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
    // every chain of this thread has reached its list's end: its word is final
    for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < nch; c += stride)
        T.c_len[c] = (uint32_t)(__hip_atomic_load(nw + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> 32) - T.c_len[c];
}

// L3: arcs from arc a to the end of its list, inclusive
__device__ __forceinline__ uint32_t tour_suffix(const TourBufs& T, uint32_t a) {
    const uint32_t c = T.a_cid[a];
    return T.c_len[c] + T.a_dist[a];  // (c_len: the suffix base after tour_chain_rank)
}
