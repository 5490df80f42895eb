// sm_seg_gpu.hip -- segment mode's Felzenszwalb segmentation (c finite) on the GPU, bucket by bucket.
// The argument that makes it exact is in sm_seg_gpu.h; DESIGN.md 4.5 has the measurements.
//
// Per view and frame:
//   k_seg_init      union-find reset, masks cleared, weight histogram (LDS, one atomic per bin and block)
//   k_seg_scan      bucket starts (one block)
//   k_seg_scatter   edge ids into their weight bucket (order inside a bucket is free: Boruvka keys by id)
//   per non-empty bucket w, in ascending order:
//     k_seg_classify  roots of both ends; open-open edges between two components -> candidate list
//                     (and the first Boruvka selection), other edges between two components -> rejected
//     k_seg_best / k_seg_hook   global Boruvka rounds (big buckets): each root's minimum-id crossing
//                     edge, then hooks along those edges (mutual pairs: the larger root onto the smaller)
//     k_seg_tail      the remaining rounds in one workgroup, until no candidate crosses two components
//     k_seg_sizes     sizes of the joined components, last-join weight w
//     (k_seg_small: all of it in one workgroup, for a run of buckets of at most SM_SEG_SMALL edges)
//   k_seg_minsize   rejected edges with an end smaller than min_size, radix-sorted into (w, id) order
//                   (hipcub) and gathered (k_seg_gather); k_seg_pairkey .. k_seg_dense keep the first
//                   candidate of each pair of roots, with dense root ids -> the host's serial merge
//   k_seg_apply     the host's merges (root hooks, marked edges)
//   k_seg_first / k_seg_virtual   first pixel of each tree, virtual edges to link the forest (sm_segment.cpp)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include <hipcub/device/device_radix_sort.hpp>
#include <hipcub/device/device_scan.hpp>
#include <rocprim/device/device_radix_sort.hpp>

#include "sm_seg_gpu.h"
#include "sm_segment.h"
#include "sm_knob.h"

namespace {

__device__ __forceinline__ uint32_t seg_find(uint32_t* par, uint32_t x) {
    // path halving; a concurrent writer only ever stores an ancestor, so every value read is valid
    // (plain accesses: parents only change by plain stores -- hooks and halving -- which a wave of the
    // same workgroup sees through the CU's L1 after a barrier, and other kernels after their launch)
    for (;;) {
        const uint32_t p = par[x];
        if (p == x) return x;
        const uint32_t g = par[p];
        if (g == p) return p;
        par[x] = g;
        x = g;
    }
}

__device__ __forceinline__ uint32_t edge_b(uint32_t id, int W) { return (id >> 1) + ((id & 1u) ? (uint32_t)W : 1u); }

// the reference's acceptance test at the bucket's start: (double)w <= w_last + (double)(c / (float)size)
// (sizes grow by L2 atomics, which a CU's L1 does not see: read them at agent scope)
__device__ __forceinline__ bool seg_open(const SegView& v, uint32_t r, double wd, float c) {
    const uint32_t sz = __hip_atomic_load(v.sz + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return wd <= (double)v.wl[r] + (double)__fdiv_rn(c, (float)sz);
}

// wave-aggregated append: returns this lane's slot (valid where pred)
__device__ __forceinline__ uint32_t wave_append(uint32_t* counter, bool pred) {
    const unsigned long long m = __ballot(pred);
    if (m == 0) return 0;
    const int lane = __lane_id();
    const int leader = __ffsll((long long)m) - 1;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(counter, (uint32_t)__popcll(m));
    base = __shfl(base, leader);
    return base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
}

// block-aggregated appends to K counters: every thread of the block calls it (it has barriers); one global
// atomic per counter and block instead of one per wave.  Every wave appending to one counter serialised the
// appends at the L2 (~6-10 ns per atomic on one address: 11-25k of them per launch in the big buckets of
// synthetic C2 made k_seg_hook / k_seg_best / k_seg_classify 0.1-0.16 ms).  Returns each lane's slots (valid
// where pred).
template <int K>
__device__ __forceinline__ void block_append(uint32_t* const (&counter)[K], const bool (&pred)[K], uint32_t (&slot)[K]) {
    __shared__ uint32_t s_cnt[K][16], s_base[K];
    const int lane = __lane_id(), wv = (int)(threadIdx.x >> 6), nw = (int)((blockDim.x + 63) >> 6);
    unsigned long long m[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        m[k] = __ballot(pred[k]);
        if (lane == 0) s_cnt[k][wv] = (uint32_t)__popcll(m[k]);
    }
    __syncthreads();
    if ((int)threadIdx.x < K) {  // thread k: the waves' offsets (exclusive scan) and the block's base
        const int k = (int)threadIdx.x;
        uint32_t run = 0;
        for (int j = 0; j < nw; ++j) {
            const uint32_t c = s_cnt[k][j];
            s_cnt[k][j] = run;
            run += c;
        }
        uint32_t* ctr = counter[0];
#pragma unroll
        for (int q = 1; q < K; ++q) ctr = k == q ? counter[q] : ctr;
        s_base[k] = run ? atomicAdd(ctr, run) : 0u;
    }
    __syncthreads();
    const unsigned long long lt = (1ull << lane) - 1ull;
#pragma unroll
    for (int k = 0; k < K; ++k) slot[k] = s_base[k] + s_cnt[k][wv] + (uint32_t)__popcll(m[k] & lt);
    __syncthreads();  // s_cnt / s_base free for the next call
}

__global__ void __launch_bounds__(256) k_seg_init(SegPair sp) {
    const SegView& v = sp.v[blockIdx.y];
    __shared__ uint32_t hist[SM_SEG_NB];
    const uint32_t N = (uint32_t)v.W * (uint32_t)v.H;
    for (int i = threadIdx.x; i < SM_SEG_NB; i += 256) hist[i] = 0;
    __syncthreads();
    const uint32_t p0 = blockIdx.x * SM_SEG_TILE;
    for (uint32_t k = threadIdx.x; k < SM_SEG_TILE; k += 256) {
        const uint32_t p = p0 + k;
        if (p >= N) break;
        v.par[p] = p;
        v.sz[p] = 1;
        v.wl[p] = 0;
        v.first[p] = 0xFFFFFFFFu;
        v.mR[p] = 0;
        v.mD[p] = 0;
        const uint32_t x = p % (uint32_t)v.W, y = p / (uint32_t)v.W;
        if (x + 1 < (uint32_t)v.W) atomicAdd(&hist[v.wR[p]], 1u);
        if (y + 1 < (uint32_t)v.H) atomicAdd(&hist[v.wD[p]], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < SM_SEG_NB; i += 256)
        if (hist[i]) atomicAdd(&v.bcnt[i], hist[i]);
}

__global__ void __launch_bounds__(1024) k_seg_scan(SegPair sp) {
    const SegView& v = sp.v[blockIdx.x];
    // exclusive scan of SM_SEG_NB counts -> starts (NB + 1) and cursors
    __shared__ uint32_t s[1024];
    const int t = threadIdx.x;
    uint32_t x = t < SM_SEG_NB ? v.bcnt[t] : 0u;
    s[t] = x;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const uint32_t y = t >= o ? s[t - o] : 0u;
        __syncthreads();
        s[t] += y;
        __syncthreads();
    }
    uint32_t* start = v.bcnt + SM_SEG_NB;
    uint32_t* cur = v.bcnt + 2 * SM_SEG_NB + 1;
    if (t < SM_SEG_NB) {
        start[t] = s[t] - x;
        cur[t] = s[t] - x;
    }
    if (t == SM_SEG_NB - 1) start[SM_SEG_NB] = s[t];
}

__global__ void __launch_bounds__(256) k_seg_scatter(SegPair sp) {
    const SegView& v = sp.v[blockIdx.y];
    __shared__ uint32_t hist[SM_SEG_NB];
    const uint32_t N = (uint32_t)v.W * (uint32_t)v.H;
    for (int i = threadIdx.x; i < SM_SEG_NB; i += 256) hist[i] = 0;
    __syncthreads();
    const uint32_t p0 = blockIdx.x * SM_SEG_TILE;
    for (uint32_t k = threadIdx.x; k < SM_SEG_TILE; k += 256) {
        const uint32_t p = p0 + k;
        if (p >= N) break;
        const uint32_t x = p % (uint32_t)v.W, y = p / (uint32_t)v.W;
        if (x + 1 < (uint32_t)v.W) atomicAdd(&hist[v.wR[p]], 1u);
        if (y + 1 < (uint32_t)v.H) atomicAdd(&hist[v.wD[p]], 1u);
    }
    __syncthreads();
    uint32_t* cur = v.bcnt + 2 * SM_SEG_NB + 1;
    for (int i = threadIdx.x; i < SM_SEG_NB; i += 256)
        if (hist[i]) hist[i] = atomicAdd(&cur[i], hist[i]);  // this block's range in bucket i
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < SM_SEG_TILE; k += 256) {
        const uint32_t p = p0 + k;
        if (p >= N) break;
        const uint32_t x = p % (uint32_t)v.W, y = p / (uint32_t)v.W;
        if (x + 1 < (uint32_t)v.W) v.ebuf[atomicAdd(&hist[v.wR[p]], 1u)] = 2u * p;
        if (y + 1 < (uint32_t)v.H) v.ebuf[atomicAdd(&hist[v.wD[p]], 1u)] = 2u * p + 1u;
    }
}

constexpr uint32_t SEG_EMPTY = 0xFFFFFFFFu;  // an empty LDS hash slot

__device__ __forceinline__ unsigned long long seg_key(uint32_t gen, uint32_t id) {
    return ((unsigned long long)(0xFFFFFFFFu - gen) << 32) | id;
}

// a bucket's edges: candidates (open-open, two components) -> list lout with their roots, and the
// first Boruvka selection (generation gen) over them; the other two-component edges -> rejected
__global__ void __launch_bounds__(256) k_seg_classify(SegPair sp, int w, float c, int lout, uint32_t gen) {
    const SegView& v = sp.v[blockIdx.y];
    const uint32_t s = v.bcnt[SM_SEG_NB + w], m = v.bcnt[SM_SEG_NB + w + 1] - s;
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i == 0) v.cnt[SM_SEG_C_BUCKET + w] = v.cnt[SM_SEG_C_HOOK];  // first hooked root of this bucket
    bool cand = false, rej = false;
    uint32_t id = 0, ra = 0, rb = 0;
    if (i < m) {
        id = v.ebuf[s + i];
        ra = seg_find(v.par, id >> 1);
        rb = seg_find(v.par, edge_b(id, v.W));
        if (ra != rb) {
            const double wd = (double)w;
            cand = seg_open(v, ra, wd, c) && seg_open(v, rb, wd, c);
            rej = !cand;
            if (cand) {
                const unsigned long long key = seg_key(gen, id);
                atomicMin(v.best + ra, key);
                atomicMin(v.best + rb, key);
            }
        }
    }
    uint32_t* const ctr[2] = {v.cnt + SM_SEG_C_LIST + lout, v.cnt + SM_SEG_C_REJ};
    const bool pred[2] = {cand, rej};
    uint32_t slot[2];
    block_append<2>(ctr, pred, slot);
    if (cand) v.list[lout & 1][slot[0]] = make_uint4(id, ra, rb, 0u);
    if (rej) v.rej[slot[1]] = id;
}

// one Boruvka selection over list lin: crossing edges -> list lout with their current roots, and each
// root's minimum key
__global__ void __launch_bounds__(256) k_seg_best(SegPair sp, int lin, int lout, uint32_t gen) {
    const SegView& v = sp.v[blockIdx.y];
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    const uint32_t n = v.cnt[SM_SEG_C_LIST + lin];
    if (blockIdx.x * 256 >= n) return;  // block-uniform: the grid covers the bucket, the list is shorter
    bool cross = false;
    uint4 e = make_uint4(0, 0, 0, 0);
    if (i < n) {
        e = v.list[lin & 1][i];
        e.y = seg_find(v.par, e.y);
        e.z = seg_find(v.par, e.z);
        cross = e.y != e.z;
        if (cross) {
            const unsigned long long key = seg_key(gen, e.x);
            atomicMin(v.best + e.y, key);
            atomicMin(v.best + e.z, key);
        }
    }
    uint32_t* const ctr[1] = {v.cnt + SM_SEG_C_LIST + lout};
    const bool pred[1] = {cross};
    uint32_t po[1];
    block_append<1>(ctr, pred, po);
    if (cross) v.list[lout & 1][po[0]] = e;
}

__device__ __forceinline__ void seg_hook_edge(const SegView& v, uint4 e, uint32_t gen, bool pred) {
    uint32_t child = 0, parent = 0;
    bool hook = false;
    if (pred) {
        const unsigned long long key = seg_key(gen, e.x);
        const bool ba = __hip_atomic_load(v.best + e.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == key;
        const bool bb = __hip_atomic_load(v.best + e.z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == key;
        if (ba || bb) {
            hook = true;
            if (ba && bb) {  // mutual minimum: one hook, the larger root onto the smaller
                child = e.y > e.z ? e.y : e.z;
                parent = e.y > e.z ? e.z : e.y;
            } else if (ba) {
                child = e.y;
                parent = e.z;
            } else {
                child = e.z;
                parent = e.y;
            }
        }
    }
    uint32_t* const ctr[1] = {v.cnt + SM_SEG_C_HOOK};
    const bool hk[1] = {hook};
    uint32_t ph[1];
    block_append<1>(ctr, hk, ph);  // (every thread of the block calls seg_hook_edge)
    if (hook) {
        v.par[child] = parent;
        v.hooked[ph[0]] = child;
        const uint32_t a = e.x >> 1;
        if (e.x & 1u)
            v.mD[a] = 1;
        else
            v.mR[a] = 1;
    }
}

__global__ void __launch_bounds__(256) k_seg_hook(SegPair sp, int lout, uint32_t gen) {
    const SegView& v = sp.v[blockIdx.y];
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    const uint32_t n = v.cnt[SM_SEG_C_LIST + lout];
    if (blockIdx.x * 256 >= n) return;  // block-uniform (as k_seg_best)
    uint4 e = make_uint4(0, 0, 0, 0);
    if (i < n) e = v.list[lout & 1][i];
    seg_hook_edge(v, e, gen, i < n);
}

// workgroup barrier: the waves of one workgroup share the CU's L1, so plain global stores before it
// are visible to plain loads after it (workgroup scope).  Values changed by atomics (keys, sizes,
// counters) live in L2 and are read with agent-scope atomic loads.
__device__ __forceinline__ void seg_wg_sync() { __syncthreads(); }

// the rest of a bucket's Boruvka rounds in one workgroup: n candidates in buffer b ping-pong with the
// other buffer; gens gen0, gen0 + 1, ... (at most SM_SEG_TAIL_GENS).  Returns the rounds run, or -1 if
// they did not converge.
__device__ int seg_wg_rounds(const SegView& v, int b, uint32_t n, uint32_t gen0, uint32_t* s_out, bool pre) {
    uint32_t g = 0;
    if (pre && n > 0) {  // generation gen0's keys were selected while classifying: hook straight away
        for (uint32_t i0 = 0; i0 < n; i0 += 1024) {
            const uint32_t i = i0 + threadIdx.x;
            uint4 e = make_uint4(0, 0, 0, 0);
            if (i < n) e = v.list[b][i];
            seg_hook_edge(v, e, gen0, i < n);
        }
        seg_wg_sync();
        g = 1;
    }
    for (; n > 0; ++g) {
        if (g == SM_SEG_TAIL_GENS) {  // cannot happen (Boruvka halves the components each round)
            if (threadIdx.x == 0) atomicOr(v.cnt + SM_SEG_C_ERR, 1u);
            return -1;
        }
        const uint32_t gen = gen0 + g;
        if (threadIdx.x == 0) *s_out = 0;
        seg_wg_sync();
        const uint4* in = v.list[b];
        uint4* out = v.list[b ^ 1];
        for (uint32_t i0 = 0; i0 < n; i0 += 1024) {
            const uint32_t i = i0 + threadIdx.x;
            bool cross = false;
            uint4 e = make_uint4(0, 0, 0, 0);
            if (i < n) {
                e = in[i];
                e.y = seg_find(v.par, e.y);
                e.z = seg_find(v.par, e.z);
                cross = e.y != e.z;
                if (cross) {
                    const unsigned long long key = seg_key(gen, e.x);
                    atomicMin(v.best + e.y, key);
                    atomicMin(v.best + e.z, key);
                }
            }
            const uint32_t po = wave_append(s_out, cross);
            if (cross) out[po] = e;
        }
        seg_wg_sync();
        const uint32_t m = *s_out;
        for (uint32_t i0 = 0; i0 < m; i0 += 1024) {
            const uint32_t i = i0 + threadIdx.x;
            uint4 e = make_uint4(0, 0, 0, 0);
            if (i < m) e = out[i];
            seg_hook_edge(v, e, gen, i < m);
        }
        seg_wg_sync();
        n = m;
        b ^= 1;
    }
    return (int)g;
}

// The tail's rounds on an LDS union-find (big buckets): the n (<= SEG_TAIL_MAX) crossing candidates left
// after the global rounds, their current roots hashed into LDS slots, then Boruvka rounds with LDS atomics
// (keys (~round << 32) | id, never reset) until no candidate crosses two components; the bucket's minimum
// spanning forest keyed by id is unique, so these rounds mark the same edges as the global ones.  Then every
// joined root goes onto its final root in the global union-find and into `hooked` (k_seg_sizes adds the
// sizes).  Synthetic C2: at most 2.7k candidates; the global-memory rounds took up to 120 us per bucket
// (several dependent global round trips and barriers per round).  Returns false, having written nothing
// global, when the roots overflow the table (then the global rounds run).
constexpr int SEG_TAIL_MAX = 4096;    // crossing candidates an LDS tail holds
constexpr int SEG_TAIL_RS = 6144;     // its root slots
constexpr uint32_t SEG_TAIL_MIN = 256;  // shorter lists keep the global-memory rounds (the LDS setup costs more)
constexpr uint16_t SEG_NOSLOT = 0xFFFFu;
__device__ __forceinline__ int seg_tslot(uint32_t* hk, uint16_t* used, uint32_t* nused, uint32_t root, uint32_t* full) {
    int h = (int)(((root * 2654435761u) >> 8) % (uint32_t)SEG_TAIL_RS);
    for (int probe = 0; probe < 256; ++probe) {
        const uint32_t prev = atomicCAS(hk + h, SEG_EMPTY, root);
        if (prev == SEG_EMPTY) used[atomicAdd(nused, 1u)] = (uint16_t)h;  // (at most RS inserts)
        if (prev == SEG_EMPTY || prev == root) return h;
        h = h + 1 == SEG_TAIL_RS ? 0 : h + 1;
    }
    atomicAdd(full, 1u);
    return 0;
}
__device__ bool seg_tail_lds(const SegView& v, int b, uint32_t n) {
    __shared__ uint32_t s_id[SEG_TAIL_MAX];
    __shared__ uint16_t s_a[SEG_TAIL_MAX], s_b[SEG_TAIL_MAX];
    __shared__ uint32_t s_hk[SEG_TAIL_RS];
    __shared__ uint16_t s_par[SEG_TAIL_RS], s_used[SEG_TAIL_RS];
    __shared__ unsigned long long s_best[SEG_TAIL_RS];
    __shared__ uint32_t s_full, s_cross, s_m, s_nused;
    const int tid = (int)threadIdx.x;
    for (int i = tid; i < SEG_TAIL_RS; i += 1024) {
        s_hk[i] = SEG_EMPTY;
        s_par[i] = (uint16_t)i;
        s_best[i] = ~0ull;
    }
    if (tid == 0) {
        s_full = 0;
        s_m = 0;
        s_nused = 0;
    }
    __syncthreads();
    // the list's edges that still cross two components (after the last global hooks), roots hashed
    for (uint32_t k = tid; k < n; k += 1024) {
        const uint4 e = v.list[b][k];
        const uint32_t ra = seg_find(v.par, e.y), rb = seg_find(v.par, e.z);
        if (ra == rb) continue;
        const uint32_t pos = atomicAdd(&s_m, 1u);
        if (pos >= (uint32_t)SEG_TAIL_MAX) continue;  // (overflow: the global rounds run)
        s_id[pos] = e.x;
        s_a[pos] = (uint16_t)seg_tslot(s_hk, s_used, &s_nused, ra, &s_full);
        s_b[pos] = (uint16_t)seg_tslot(s_hk, s_used, &s_nused, rb, &s_full);
    }
    __syncthreads();
    const uint32_t m = s_m;
    if (s_full || m > (uint32_t)SEG_TAIL_MAX) return false;  // block-uniform, nothing global written
    for (uint32_t round = 0;; ++round) {
        if (tid == 0) s_cross = 0;
        __syncthreads();
        // each root's minimum crossing key; the edge's slots become its current roots (s_par is only read
        // in this phase), which the hook phase then uses as they are -- finds there would race the hooks
        for (uint32_t k = tid; k < m; k += 1024) {
            if (s_a[k] == SEG_NOSLOT) continue;
            int a = s_a[k], c = s_b[k];
            while (s_par[a] != a) a = s_par[a];
            while (s_par[c] != c) c = s_par[c];
            if (a == c) {  // internal for good
                s_a[k] = SEG_NOSLOT;
                continue;
            }
            s_a[k] = (uint16_t)a;
            s_b[k] = (uint16_t)c;
            const unsigned long long key = ((unsigned long long)(0xFFFFFFFFu - round) << 32) | s_id[k];
            atomicMin(&s_best[a], key);
            atomicMin(&s_best[c], key);
            s_cross = 1;
        }
        __syncthreads();
        if (!s_cross) break;  // block-uniform
        for (uint32_t k = tid; k < m; k += 1024) {  // hooks along those keys (mutual pairs: larger slot onto smaller)
            if (s_a[k] == SEG_NOSLOT) continue;
            const int a = s_a[k], c = s_b[k];  // roots at the selection
            const unsigned long long key = ((unsigned long long)(0xFFFFFFFFu - round) << 32) | s_id[k];
            const bool ba = s_best[a] == key, bc = s_best[c] == key;
            if (!ba && !bc) continue;
            const int child = ba && bc ? (a > c ? a : c) : ba ? a : c;
            const int parent = ba && bc ? (a > c ? c : a) : ba ? c : a;
            s_par[child] = (uint16_t)parent;
            const uint32_t id = s_id[k];
            if (id & 1u)
                v.mD[id >> 1] = 1;
            else
                v.mR[id >> 1] = 1;
        }
        __syncthreads();
        if (round + 1 >= (uint32_t)SM_SEG_TAIL_GENS) {  // cannot happen (Boruvka halves the components)
            if (tid == 0) atomicOr(v.cnt + SM_SEG_C_ERR, 1u);
            break;
        }
    }
    // joined roots onto their final roots (global), and into `hooked` for k_seg_sizes
    const uint32_t nu = s_nused;
    for (uint32_t u0 = 0; u0 < nu; u0 += 1024) {
        const uint32_t u = u0 + tid;
        int i = 0, f = 0;
        if (u < nu) {
            i = s_used[u];
            f = i;
            while (s_par[f] != f) f = s_par[f];
        }
        const bool joined = u < nu && f != i;
        uint32_t* const ctr[1] = {v.cnt + SM_SEG_C_HOOK};
        const bool pred[1] = {joined};
        uint32_t slot[1];
        block_append<1>(ctr, pred, slot);
        if (joined) {
            const uint32_t r = s_hk[i];
            v.par[r] = s_hk[f];
            v.hooked[slot[0]] = r;
        }
    }
    return true;
}

// lds: try seg_tail_lds first (SM_SEG_TAIL_GLOBAL=1: always the global-memory rounds)
__global__ void __launch_bounds__(1024) k_seg_tail(SegPair sp, int lin, uint32_t gen0, int lds, uint32_t tmin) {
    const SegView& v = sp.v[blockIdx.x];
    __shared__ uint32_t s_out;
    const uint32_t n = v.cnt[SM_SEG_C_LIST + lin];
    if (lds && n >= tmin && seg_tail_lds(v, lin & 1, n)) return;
    seg_wg_rounds(v, lin & 1, n, gen0, &s_out, false);
}

// hooked root i (valid lanes) adds its size to its component's root, whose last-join weight becomes w.
// r's size is its size at the bucket's start (only roots grow; r is no root any more, so no lane adds into
// it); agent scope: sizes change in L2.  Call with the whole wave: lanes with the same root add their sizes
// in one atomic -- one join of synthetic C2 (w = 9) hooks 25.6k roots into one component, i.e. 25.6k
// atomics on one address (0.24 ms) without it.
__device__ __forceinline__ void seg_size_update(const SegView& v, uint32_t i, int w, bool valid) {
    uint32_t t = 0, sz = 0;
    if (valid) {
        const uint32_t r = v.hooked[i];
        t = seg_find(v.par, r);
        sz = __hip_atomic_load(v.sz + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    unsigned long long act = __ballot(valid);
    const int lane = __lane_id();
    // up to 8 distinct roots of the wave one group at a time (a wave whose first lane is in a small
    // component still folds the giant one's lanes), then one atomic per remaining lane
    for (int it = 0; act && it < 8; ++it) {
        const int leader = __ffsll((long long)act) - 1;
        const uint32_t tl = __shfl(t, leader);
        const unsigned long long m = __ballot(valid && t == tl) & act;
        uint32_t sum = ((m >> lane) & 1ull) ? sz : 0u;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) sum += __shfl_xor(sum, o);
        if (lane == leader) {
            atomicAdd(v.sz + tl, sum);
            v.wl[tl] = (uint16_t)w;
        }
        act &= ~m;
    }
    if ((act >> lane) & 1ull) {
        atomicAdd(v.sz + t, sz);
        v.wl[t] = (uint16_t)w;
    }
}

// a run of small buckets [w0, w1) (each of at most SM_SEG_SMALL edges) in one workgroup, one bucket
// after the other.  A bucket's candidates (open-open edges between two components) are few (at most 163
// per bucket at C2): when they fit in LDS (SEG_LC), the bucket's marked edges -- the minimum spanning
// forest of its candidates keyed by edge id -- are Kruskal's in id order over the
// candidates' roots in an LDS union-find (roots hashed to slots), and the joins go back to the global
// union-find at once: each joined root hooks onto its component's final root, whose size grows by the
// joined sizes and whose last-join weight becomes w.  Only the candidate scan and that write-back touch
// global memory (the Boruvka rounds cost several dependent global-atomic phases per bucket).  A bucket
// with more candidates takes the Boruvka rounds (seg_wg_rounds) and the hooked-root size update; gens
// from gen0, at most SM_SEG_TAIL_GENS per such bucket.
constexpr int SEG_LC = 1024;         // candidates of an LDS bucket
constexpr int SEG_LH = 4096;         // hash slots (power of two, >= 2 SEG_LC)

__device__ __forceinline__ int seg_lfind(uint16_t* par, int x) {
    while (par[x] != x) {
        const int g = par[par[x]];
        par[x] = (uint16_t)g;
        x = g;
    }
    return x;
}
__device__ __forceinline__ int seg_lfind_ro(const uint16_t* par, int x) {
    while (par[x] != x) x = par[x];
    return x;
}
__device__ __forceinline__ int seg_lslot(uint32_t* hk, uint32_t root) {
    int h = (int)((root * 2654435761u) >> 20) & (SEG_LH - 1);
    for (;;) {
        const uint32_t prev = atomicCAS(hk + h, SEG_EMPTY, root);
        if (prev == SEG_EMPTY || prev == root) return h;
        h = (h + 1) & (SEG_LH - 1);
    }
}

constexpr uint32_t SEG_DONE = 0x80000000u;  // an ebuf entry k_seg_split rejected already (ids < 2^31)
constexpr int SEG_ACT_MAX = 4096;           // active edges of a run that k_seg_small buckets in LDS

// The start of a run of small buckets [w0, w1), over the whole GPU.  An edge whose ends are in one component
// stays internal for the rest of the sweep.  An edge with an end that is closed at w0 is rejected now: a
// closed component never joins again (a join needs its own acceptance, and its threshold only changes by
// joining), so in its own bucket the edge still joins two components, one of them closed.  The rest (both
// ends open at w0: 538 of the 48k small-bucket edges of a synthetic C2 view) go to the active list, the
// only edges k_seg_small then walks.  Rejected ebuf entries get SEG_DONE (its full-scan fallback skips them).
__global__ void __launch_bounds__(256) k_seg_split(SegPair sp, int w0, int w1, float c) {
    const SegView& v = sp.v[blockIdx.y];
    const uint32_t s = v.bcnt[SM_SEG_NB + w0], e = v.bcnt[SM_SEG_NB + w1];
    const uint32_t j = s + blockIdx.x * 256 + threadIdx.x;
    bool act = false, rej = false;
    uint32_t id = 0;
    if (j < e) {
        id = v.ebuf[j];
        const uint32_t ra = seg_find(v.par, id >> 1), rb = seg_find(v.par, edge_b(id, v.W));
        if (ra != rb) {
            const double wd = (double)w0;
            act = seg_open(v, ra, wd, c) && seg_open(v, rb, wd, c);
            rej = !act;
        }
    }
    uint32_t* const ctr[2] = {v.cnt + SM_SEG_C_ACT, v.cnt + SM_SEG_C_REJ};
    const bool pred[2] = {act, rej};
    uint32_t slot[2];
    block_append<2>(ctr, pred, slot);
    if (act) v.act[slot[0]] = id;
    if (rej) {
        v.rej[slot[1]] = id;
        v.ebuf[j] = id | SEG_DONE;
    }
}

// split: k_seg_split ran first; its active edges (at most amax) are bucketed by weight in LDS and walked
// instead of the run's ebuf ranges (otherwise the full scan, skipping the entries it rejected)
constexpr int SEG_PROF_SLOT = 60000;  // SM_SEG_PROF: k_seg_small's timings at cnt[SM_SEG_C_LIST + 60000 ..]
constexpr int SEG_RUN_DONE = 59990;   // cnt[SM_SEG_C_LIST + 59990]: k_seg_run did the run (k_seg_small skips it)
constexpr int SEG_RUN_MAX = 6144;     // active edges of a run that k_seg_run holds in LDS
constexpr int SEG_RUN_RS = 6144;      // its root slots

__device__ __forceinline__ int seg_rslot(uint32_t* hk, uint32_t root, uint32_t* nfull) {
    int h = (int)(((root * 2654435761u) >> 8) % (uint32_t)SEG_RUN_RS);
    for (int probe = 0; probe < 256; ++probe) {
        const uint32_t prev = atomicCAS(hk + h, SEG_EMPTY, root);
        if (prev == SEG_EMPTY || prev == root) return h;
        h = h + 1 == SEG_RUN_RS ? 0 : h + 1;
    }
    atomicAdd(nfull, 1u);  // (table too full: the run falls back to k_seg_small)
    return 0;
}

// A run of small buckets [w0, w1) after k_seg_split, entirely in LDS.  Only the run's active edges (both
// ends open at w0) can join anything (k_seg_split), and they only join components that were open at w0, so
// the run's whole union-find state lives in LDS: the active edges bucketed by weight and sorted by id
// within a bucket, and their roots at the run's start (hashed slots with size and last-join weight).  Per
// bucket: every edge's current roots and the acceptance test at the bucket's start in parallel, then the
// candidates' Kruskal in id order (thread 0): the minimum spanning forest keyed by id of the bucket's open-open
// edges, sizes summed, last-join weight w.  No global memory is touched between buckets --
// k_seg_small's buckets each paid ~5 dependent global round trips (4-8 us; 250 buckets in one synthetic C2
// view).  At the end: joined roots' parents, the roots' sizes and weights, and the rejected edges go back.
// A run that does not fit (more than SEG_RUN_MAX active edges, or its roots overflow the table) sets no done
// flag and k_seg_small runs it instead (nothing global was written).
__global__ void __launch_bounds__(1024) k_seg_run(SegPair sp, int w0, int w1, float c) {
    const SegView& v = sp.v[blockIdx.x];
    const int tid = (int)threadIdx.x, nb = w1 - w0;
    __shared__ uint32_t s_start[SM_SEG_NB + 1], s_wc[SM_SEG_NB + 1];
    __shared__ uint32_t s_aid[SEG_RUN_MAX];
    __shared__ uint16_t s_ea[SEG_RUN_MAX], s_eb[SEG_RUN_MAX], s_ord[SEG_RUN_MAX];
    __shared__ uint8_t s_fl[SEG_RUN_MAX];
    __shared__ uint32_t s_hk[SEG_RUN_RS], s_sz[SEG_RUN_RS];
    __shared__ uint16_t s_par[SEG_RUN_RS], s_wl[SEG_RUN_RS];
    __shared__ uint32_t s_full;
    const uint32_t na = __hip_atomic_load(v.cnt + SM_SEG_C_ACT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (na > (uint32_t)SEG_RUN_MAX) return;  // block-uniform: k_seg_small runs it
    for (int i = tid; i <= nb; i += 1024) s_wc[i] = 0;
    for (int i = tid; i < SEG_RUN_RS; i += 1024) {
        s_hk[i] = SEG_EMPTY;
        s_par[i] = (uint16_t)i;
    }
    if (tid == 0) s_full = 0;
    __syncthreads();
    // the active edges by weight: counts, exclusive offsets (s_start), scatter
    for (uint32_t k = tid; k < na; k += 1024) {
        const uint32_t id = v.act[k], a = id >> 1;
        atomicAdd(&s_wc[((id & 1u) ? v.wD[a] : v.wR[a]) - w0], 1u);
    }
    __syncthreads();
    if (tid < 64) {
        uint32_t run = 0;
        for (int b = 0; b <= nb; b += 64) {
            const int i = b + tid;
            const uint32_t x = i <= nb ? s_wc[i] : 0u;
            uint32_t incl = x;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(incl, o);
                if (tid >= o) incl += y;
            }
            if (i <= nb) s_start[i] = run + incl - x;
            run += __shfl(incl, 63);
        }
    }
    __syncthreads();
    for (int i = tid; i <= nb; i += 1024) s_wc[i] = s_start[i];
    __syncthreads();
    for (uint32_t k = tid; k < na; k += 1024) {
        const uint32_t id = v.act[k], a = id >> 1;
        s_aid[atomicAdd(&s_wc[((id & 1u) ? v.wD[a] : v.wR[a]) - w0], 1u)] = id;
    }
    __syncthreads();
    // per edge: its rank by id within its bucket (Kruskal's order), and its ends' roots at the run's start
    for (uint32_t k = tid; k < na; k += 1024) {
        const uint32_t id = s_aid[k], a = id >> 1;
        const int wb = ((id & 1u) ? v.wD[a] : v.wR[a]) - w0;
        const uint32_t lo = s_start[wb], hi = s_start[wb + 1];
        uint32_t r = 0;
        for (uint32_t j = lo; j < hi; ++j) r += s_aid[j] < id;
        s_ord[lo + r] = (uint16_t)k;
        s_ea[k] = (uint16_t)seg_rslot(s_hk, seg_find(v.par, a), &s_full);
        s_eb[k] = (uint16_t)seg_rslot(s_hk, seg_find(v.par, edge_b(id, v.W)), &s_full);
        s_fl[k] = 0;
    }
    __syncthreads();
    if (s_full) return;  // block-uniform (nothing global written): k_seg_small runs it
    for (int i = tid; i < SEG_RUN_RS; i += 1024) {
        const uint32_t r = s_hk[i];
        if (r != SEG_EMPTY) {
            s_sz[i] = __hip_atomic_load(v.sz + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_wl[i] = v.wl[r];
        }
    }
    __syncthreads();
    // the sweep on wave 0 alone (no workgroup barriers between buckets): its lanes take a bucket's edges in
    // id order, 64 at a time -- current roots and the acceptance test at the bucket's start, all chunks of
    // the bucket first -- then lane 0 joins the candidates in id order (Kruskal)
    if (tid < 64) {
        const int lane = tid;
        for (int w = w0; w < w1; ++w) {
            const uint32_t lo = s_start[w - w0], hi = s_start[w + 1 - w0];
            if (lo == hi) continue;  // uniform
            const double wd = (double)w;
            for (uint32_t q0 = lo; q0 < hi; q0 += 64) {
                const uint32_t q = q0 + lane;
                if (q < hi) {
                    const uint32_t k = s_ord[q];
                    int a = s_ea[k], b = s_eb[k];
                    while (s_par[a] != a) a = s_par[a];
                    while (s_par[b] != b) b = s_par[b];
                    uint8_t f = 0;
                    if (a != b) {
                        const bool oa = wd <= (double)s_wl[a] + (double)__fdiv_rn(c, (float)s_sz[a]);
                        const bool ob = wd <= (double)s_wl[b] + (double)__fdiv_rn(c, (float)s_sz[b]);
                        f = (oa && ob) ? 1 : 2;  // candidate / rejected
                    }
                    s_fl[k] = f;
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            for (uint32_t q0 = lo; q0 < hi; q0 += 64) {
                const uint32_t q = q0 + lane;
                const uint32_t k = q < hi ? s_ord[q] : 0u;
                const bool cnd = q < hi && s_fl[k] == 1;
                // the candidate's id and its ends' slots, loaded by its own lane (lane 0 then reads them by
                // readlane instead of one LDS round trip after another)
                const uint32_t kid = cnd ? s_aid[k] : 0u;
                const int ka = cnd ? (int)s_ea[k] : 0, kb = cnd ? (int)s_eb[k] : 0;
                unsigned long long m = __ballot(cnd);
                while (m) {  // uniform: the candidates of this chunk in id order
                    const int j = __ffsll((long long)m) - 1;
                    m &= m - 1ull;
                    const int a0 = __builtin_amdgcn_readlane(ka, j), b0 = __builtin_amdgcn_readlane(kb, j);
                    const uint32_t id = (uint32_t)__builtin_amdgcn_readlane((int)kid, j);
                    if (lane == 0) {
                        const int a = seg_lfind(s_par, a0), b = seg_lfind(s_par, b0);
                        if (a != b) {
                            s_par[b] = (uint16_t)a;
                            s_sz[a] += s_sz[b];
                            s_wl[a] = (uint16_t)w;
                            if (id & 1u)
                                v.mD[id >> 1] = 1;
                            else
                                v.mR[id >> 1] = 1;
                        }
                    }
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        }
    }
    __syncthreads();
    // write-back: joined roots onto their final roots, the roots' sizes and last-join weights
    for (int i = tid; i < SEG_RUN_RS; i += 1024) {
        const uint32_t r = s_hk[i];
        if (r == SEG_EMPTY) continue;
        int f = i;
        while (s_par[f] != f) f = s_par[f];
        if (f != i) {
            v.par[r] = s_hk[f];
        } else {
            v.sz[r] = s_sz[i];
            v.wl[r] = s_wl[i];
        }
    }
    // the rejected edges (flag 2)
    for (uint32_t k0 = 0; k0 < na; k0 += 1024) {
        const uint32_t k = k0 + tid;
        const bool rj = k < na && s_fl[k] == 2;
        uint32_t* const ctr[1] = {v.cnt + SM_SEG_C_REJ};
        const bool pred[1] = {rj};
        uint32_t slot[1];
        block_append<1>(ctr, pred, slot);
        if (rj) v.rej[slot[0]] = s_aid[k];
    }
    if (tid == 0) {
        v.cnt[SM_SEG_C_ACT] = 0;
        v.cnt[SM_SEG_C_LIST + SEG_RUN_DONE] = 1;
    }
}
__global__ void __launch_bounds__(1024) k_seg_small(SegPair sp, int w0, int w1, float c, uint32_t gen0, uint32_t lc,
                                                    int split, uint32_t amax, int prof_on) {
    const unsigned long long tk0 = prof_on && threadIdx.x == 0 ? wall_clock64() : 0ull;
    const SegView& v = sp.v[blockIdx.x];
    if (split && __hip_atomic_load(v.cnt + SM_SEG_C_LIST + SEG_RUN_DONE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        __syncthreads();  // every thread has read the flag
        if (threadIdx.x == 0) v.cnt[SM_SEG_C_LIST + SEG_RUN_DONE] = 0;
        return;  // k_seg_run did this run
    }
    __shared__ uint32_t s_n, s_out, s_h0;
    __shared__ uint32_t s_cid[SEG_LC], s_ord[SEG_LC];
    __shared__ uint16_t s_sa[SEG_LC], s_sb[SEG_LC];
    __shared__ uint8_t s_mk[SEG_LC];
    __shared__ uint32_t s_hk[SEG_LH];
    __shared__ uint16_t s_par[SEG_LH];
    const int tid = (int)threadIdx.x;
    for (int i = tid; i < SEG_LH; i += 1024) {
        s_hk[i] = SEG_EMPTY;
        s_par[i] = (uint16_t)i;
    }
    // the run's bucket starts in LDS: most buckets of a run are empty (synthetic C2: 24 of ~740 hold edges),
    // and a global load per bucket just to skip it cost ~1 us each, one after the other
    __shared__ uint32_t s_start[SM_SEG_NB + 1];
    __shared__ uint32_t s_wc[SM_SEG_NB + 1];
    __shared__ uint32_t s_aid[SEG_ACT_MAX];
    const int nb = w1 - w0;
    const uint32_t na = split ? __hip_atomic_load(v.cnt + SM_SEG_C_ACT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    const bool lact = split && na <= amax && na <= (uint32_t)SEG_ACT_MAX;  // block-uniform
    if (lact) {  // the active edges bucketed by weight: counts, exclusive offsets (s_start), scatter (s_aid)
        for (int i = tid; i <= nb; i += 1024) s_wc[i] = 0;
        seg_wg_sync();
        for (uint32_t k = tid; k < na; k += 1024) {
            const uint32_t id = v.act[k], a = id >> 1;
            atomicAdd(&s_wc[((id & 1u) ? v.wD[a] : v.wR[a]) - w0], 1u);
        }
        seg_wg_sync();
        if (tid < 64) {  // one wave: exclusive scan of nb + 1 <= 767 counts, 64 at a time
            uint32_t run = 0;
            for (int b = 0; b <= nb; b += 64) {
                const int i = b + tid;
                const uint32_t x = i <= nb ? s_wc[i] : 0u;
                uint32_t incl = x;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const uint32_t y = __shfl_up(incl, o);
                    if (tid >= o) incl += y;
                }
                if (i <= nb) s_start[i] = run + incl - x;
                run += __shfl(incl, 63);
            }
        }
        seg_wg_sync();
        for (int i = tid; i <= nb; i += 1024) s_wc[i] = s_start[i];  // cursors
        seg_wg_sync();
        for (uint32_t k = tid; k < na; k += 1024) {
            const uint32_t id = v.act[k], a = id >> 1;
            s_aid[atomicAdd(&s_wc[((id & 1u) ? v.wD[a] : v.wR[a]) - w0], 1u)] = id;
        }
    } else {
        for (int i = w0 + tid; i <= w1; i += 1024) s_start[i - w0] = v.bcnt[SM_SEG_NB + i];
    }
    seg_wg_sync();
    if (split && tid == 0) v.cnt[SM_SEG_C_ACT] = 0;  // for the next run (read above by every thread, before the barrier)
    // SM_SEG_PROF builds: wall-clock ticks (100 MHz) of the prologue and of each bucket in spare list counters
    uint32_t* const prof = prof_on ? v.cnt + SM_SEG_C_LIST + SEG_PROF_SLOT : nullptr;
    unsigned long long tk = prof && tid == 0 ? wall_clock64() : 0ull;
    if (prof && tid == 0) {
        prof[0] = (uint32_t)(tk - tk0);
        prof[1] = na;
    }
    uint32_t gen = gen0;
    for (int w = w0; w < w1; ++w) {
        const uint32_t s = s_start[w - w0], m = s_start[w + 1 - w0] - s;
        if (m == 0) continue;
        if (tid == 0) {
            s_n = 0;
            s_h0 = __hip_atomic_load(v.cnt + SM_SEG_C_HOOK, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        seg_wg_sync();
        const double wd = (double)w;
        for (uint32_t i0 = 0; i0 < m; i0 += 1024) {
            const uint32_t i = i0 + tid;
            bool cand = false, rej = false;
            uint32_t id = 0, ra = 0, rb = 0;
            if (i < m) id = lact ? s_aid[s + i] : v.ebuf[s + i];
            if (i < m && !(id & SEG_DONE)) {
                ra = seg_find(v.par, id >> 1);
                rb = seg_find(v.par, edge_b(id, v.W));
                if (ra != rb) {
                    cand = seg_open(v, ra, wd, c) && seg_open(v, rb, wd, c);
                    rej = !cand;
                }
            }
            const uint32_t pc = wave_append(&s_n, cand);
            if (cand) {
                v.list[0][pc] = make_uint4(id, ra, rb, 0u);
                if (pc < lc) {  // the LDS copy: id and the roots' hash slots
                    s_cid[pc] = id;
                    s_sa[pc] = (uint16_t)seg_lslot(s_hk, ra);
                    s_sb[pc] = (uint16_t)seg_lslot(s_hk, rb);
                }
            }
            uint32_t* const ctr[1] = {v.cnt + SM_SEG_C_REJ};
            const bool pred[1] = {rej};
            uint32_t pr[1];
            block_append<1>(ctr, pred, pr);
            if (rej) v.rej[pr[0]] = id;
        }
        seg_wg_sync();
        const uint32_t n = s_n;
        if (n <= lc) {
            // Kruskal's order: each candidate's rank among the bucket's ids (distinct)
            for (uint32_t t = tid; t < n; t += 1024) {
                const uint32_t id = s_cid[t];
                uint32_t r = 0;
                for (uint32_t j = 0; j < n; ++j) r += s_cid[j] < id;
                s_ord[r] = t;
            }
            seg_wg_sync();
            if (tid == 0)
                for (uint32_t k = 0; k < n; ++k) {
                    const uint32_t t = s_ord[k];
                    const int a = seg_lfind(s_par, s_sa[t]), b = seg_lfind(s_par, s_sb[t]);
                    s_mk[t] = a != b;
                    if (a != b) s_par[b] = (uint16_t)a;
                }
            seg_wg_sync();
            // write-back: marked edges; every joined root onto its final root, sizes, last-join weights
            for (uint32_t t = tid; t < n; t += 1024)
                if (s_mk[t]) {
                    const uint32_t id = s_cid[t];
                    if (id & 1u)
                        v.mD[id >> 1] = 1;
                    else
                        v.mR[id >> 1] = 1;
                }
            for (int l = tid; l < SEG_LH; l += 1024) {
                const uint32_t r = s_hk[l];
                if (r == SEG_EMPTY) continue;
                const int f = seg_lfind_ro(s_par, l);
                if (f == l) continue;
                const uint32_t rf = s_hk[f];
                v.par[r] = rf;
                // r's size is its size at the bucket's start (r was a root); rf is never a joined root
                atomicAdd(v.sz + rf, __hip_atomic_load(v.sz + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                v.wl[rf] = (uint16_t)w;
            }
            seg_wg_sync();
            for (int l = tid; l < SEG_LH; l += 1024) {  // the table back to empty for the next bucket
                s_hk[l] = SEG_EMPTY;
                s_par[l] = (uint16_t)l;
            }
            seg_wg_sync();  // sizes final before the next bucket's acceptance tests
            if (prof && tid == 0) {
                const unsigned long long t = wall_clock64();
                prof[2 + w] = (uint32_t)(t - tk);
                tk = t;
            }
            continue;
        }
        // more candidates than the LDS holds: the table back to empty, then the Boruvka rounds
        for (int l = tid; l < SEG_LH; l += 1024) s_hk[l] = SEG_EMPTY;
        const int r = seg_wg_rounds(v, 0, n, gen, &s_out, false);
        if (r < 0) return;
        gen += (uint32_t)r;
        const uint32_t h1 = __hip_atomic_load(v.cnt + SM_SEG_C_HOOK, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (uint32_t i0 = s_h0; i0 < h1; i0 += 1024) seg_size_update(v, i0 + tid, w, i0 + tid < h1);
        seg_wg_sync();  // sizes final before the next bucket's acceptance tests
        if (prof && tid == 0) {
            const unsigned long long t = wall_clock64();
            prof[2 + w] = (uint32_t)(t - tk) | 0x80000000u;  // (Boruvka rounds)
            tk = t;
        }
    }
}

__global__ void __launch_bounds__(256) k_seg_sizes(SegPair sp, int w) {
    const SegView& v = sp.v[blockIdx.y];
    const uint32_t h0 = v.cnt[SM_SEG_C_BUCKET + w], h1 = v.cnt[SM_SEG_C_HOOK];
    const uint32_t i = h0 + blockIdx.x * 256 + threadIdx.x;
    if (h0 + blockIdx.x * 256 >= h1) return;  // block-uniform
    seg_size_update(v, i, w, i < h1);
}

__global__ void __launch_bounds__(256) k_seg_minsize(SegPair sp, uint32_t ms) {
    const SegView& v = sp.v[blockIdx.y];
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    const uint32_t n = v.cnt[SM_SEG_C_REJ];
    bool keep = false;
    SegMin r{};
    if (i < n) {
        const uint32_t id = v.rej[i];
        const uint32_t a = id >> 1;
        r.id = id;
        r.w = (id & 1u) ? v.wD[a] : v.wR[a];
        r.ra = seg_find(v.par, a);
        r.rb = seg_find(v.par, edge_b(id, v.W));
        r.sa = v.sz[r.ra];
        r.sb = v.sz[r.rb];
        keep = r.sa < ms || r.sb < ms;
    }
    uint32_t* const ctr[1] = {v.cnt + SM_SEG_C_MIN};
    const bool pred[1] = {keep};
    uint32_t ps[1];
    block_append<1>(ctr, pred, ps);
    const uint32_t p = ps[0];
    if (keep) {
        v.mlist[p] = r;
        v.mkey[0][p] = ((unsigned long long)r.w << 32) | r.id;  // the merge's (w, a, b) order
        v.mval[0][p] = p;
    }
}

// the min-size candidates in (w, id) order, for the host
__global__ void __launch_bounds__(256) k_seg_gather(SegPair sp) {
    const SegView& v = sp.v[blockIdx.y];
    const uint32_t n = v.nmin;
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) v.msorted[i] = v.mlist[v.mval[1][i]];
}

// Pair dedupe.  A candidate whose pair of sweep roots {ra, rb} already occurred earlier in (w, id) order
// can never join: if the first occurrence joined, the two are one set from then on; if it did not, they
// were one set already or both had min_size pixels, and sizes only grow.  So only the first of each pair
// goes to the host (~23k of ~260k per C2 view).  Keys: lo * N + hi; the radix sort is stable, so the
// first of a run of equal keys is the earliest position.
__global__ void __launch_bounds__(256) k_seg_pairkey(SegPair sp) {
    const SegView& v = sp.v[blockIdx.y];
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= v.nmin) return;
    const SegMin m = v.msorted[i];
    const unsigned long long N = (unsigned long long)v.W * (unsigned long long)v.H;
    const uint32_t lo = m.ra < m.rb ? m.ra : m.rb, hi = m.ra < m.rb ? m.rb : m.ra;
    v.mkey[0][i] = (unsigned long long)lo * N + hi;
    v.mval[0][i] = i;
}

__global__ void __launch_bounds__(256) k_seg_keep(SegPair sp) {
    const SegView& v = sp.v[blockIdx.y];
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i == 0) v.keep[v.nmin] = 0;
    if (i >= v.nmin) return;
    v.keep[v.mval[1][i]] = (i == 0 || v.mkey[1][i] != v.mkey[1][i - 1]) ? 1u : 0u;
}

__global__ void __launch_bounds__(256) k_seg_mark(SegPair sp) {
    const SegView& v = sp.v[blockIdx.y];
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= v.nmin || !v.keep[i]) return;
    const SegMin m = v.msorted[i];
    v.lmark[m.ra] = 1;
    v.lmark[m.rb] = 1;
}

__global__ void __launch_bounds__(256) k_seg_dense(SegPair sp) {
    const SegView& v = sp.v[blockIdx.y];
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i == 0) {
        v.cnt[SM_SEG_C_UNIQ] = v.kpos[v.nmin];
        v.cnt[SM_SEG_C_LOCAL] = v.lid[(size_t)v.W * v.H];
    }
    if (i >= v.nmin || !v.keep[i]) return;
    const SegMin m = v.msorted[i];
    const uint32_t la = v.lid[m.ra], lb = v.lid[m.rb];
    v.dense[v.kpos[i]] = SegEdge{la, lb, m.id, m.w};
    v.lsize[la] = m.sa;  // (every candidate of a root writes the same values)
    v.lroot[la] = m.ra;
    v.lsize[lb] = m.sb;
    v.lroot[lb] = m.rb;
}

// Pair dedupe by hashing (seg_launch_dedupe_hash): the pair key lo * N + hi of each candidate into an
// open-addressing table (keys in mkey[0], each pair's minimum (w, id) key in mkey[1]), the slot kept in mval[0]
__global__ void __launch_bounds__(256) k_seg_hins(SegPair sp, uint32_t cap) {
    const SegView& v = sp.v[blockIdx.y];
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= v.nmin) return;
    const SegMin m = v.mlist[i];
    const unsigned long long N = (unsigned long long)v.W * (unsigned long long)v.H;
    const uint32_t lo = m.ra < m.rb ? m.ra : m.rb, hi = m.ra < m.rb ? m.rb : m.ra;
    const unsigned long long pk = (unsigned long long)lo * N + hi;
    uint32_t h = (uint32_t)((pk * 0x9E3779B97F4A7C15ull) >> 32) & (cap - 1u);
    for (uint32_t probe = 0; probe < cap; ++probe) {  // load <= 1/2: a few probes
        const unsigned long long prev = atomicCAS(v.mkey[0] + h, ~0ull, pk);
        if (prev == ~0ull || prev == pk) break;
        h = (h + 1u) & (cap - 1u);
    }
    atomicMin(v.mkey[1] + h, ((unsigned long long)m.w << 32) | m.id);
    v.mval[0][i] = h;
}

// a candidate is kept iff it holds its pair's minimum key; its roots get dense ids (lmark)
__global__ void __launch_bounds__(256) k_seg_hkeep(SegPair sp) {
    const SegView& v = sp.v[blockIdx.y];
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i == 0) v.keep[v.nmin] = 0;
    if (i >= v.nmin) return;
    const SegMin m = v.mlist[i];
    const bool k = v.mkey[1][v.mval[0][i]] == (((unsigned long long)m.w << 32) | m.id);
    v.keep[i] = k ? 1u : 0u;
    if (k) {
        v.lmark[m.ra] = 1;
        v.lmark[m.rb] = 1;
    }
}

// k_seg_dense over the unsorted candidates
__global__ void __launch_bounds__(256) k_seg_hdense(SegPair sp) {
    const SegView& v = sp.v[blockIdx.y];
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i == 0) {
        v.cnt[SM_SEG_C_UNIQ] = v.kpos[v.nmin];
        v.cnt[SM_SEG_C_LOCAL] = v.lid[(size_t)v.W * v.H];
    }
    if (i >= v.nmin || !v.keep[i]) return;
    const SegMin m = v.mlist[i];
    const uint32_t la = v.lid[m.ra], lb = v.lid[m.rb];
    v.dense[v.kpos[i]] = SegEdge{la, lb, m.id, m.w};
    v.lsize[la] = m.sa;
    v.lroot[la] = m.ra;
    v.lsize[lb] = m.sb;
    v.lroot[lb] = m.rb;
}

// every pixel's parent set to its root (chains grow by one level per join; the one-workgroup kernels pay
// each level as a dependent load)
__global__ void __launch_bounds__(256) k_seg_flatten(SegPair sp) {
    const SegView& v = sp.v[blockIdx.y];
    const uint32_t p = blockIdx.x * 256 + threadIdx.x;
    if (p >= (uint32_t)v.W * (uint32_t)v.H) return;
    const uint32_t r = seg_find(v.par, p);
    if (v.par[p] != r) v.par[p] = r;
}

// hooks[2k] = child root, hooks[2k + 1] = parent root (0xFFFFFFFF: none) ; marked edge ids after the
// pairs: hooks[2 * nhooks + k]
__global__ void __launch_bounds__(256) k_seg_apply(SegPair sp) {
    const SegView& v = sp.v[blockIdx.y];
    const uint32_t* hooks = v.hooks;
    const int nhooks = v.nhooks;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= nhooks) return;
    v.par[hooks[2 * i]] = hooks[2 * i + 1];
    const uint32_t id = hooks[2 * nhooks + i];
    if (id & 1u)
        v.mD[id >> 1] = 1;
    else
        v.mR[id >> 1] = 1;
}

__global__ void __launch_bounds__(256) k_seg_first(SegPair sp) {
    const SegView& v = sp.v[blockIdx.y];
    const uint32_t p = blockIdx.x * 256 + threadIdx.x;
    const uint32_t N = (uint32_t)v.W * (uint32_t)v.H;
    const uint32_t r = p < N ? seg_find(v.par, p) : 0xFFFFFFFFu;
    if (p < N && v.par[p] != r) v.par[p] = r;  // flattened: k_seg_virtual's finds take one step
    // one atomic per run of equal roots in the wave (rows are mostly long runs of one tree), and none
    // where the tree's first pixel is already known to be smaller
    const uint32_t rprev = __shfl_up(r, 1);
    if (p >= N) return;
    if ((__lane_id() == 0 || rprev != r) && v.first[r] > p) atomicMin(v.first + r, p);
    v.fwR[p] = v.wR[p];
    v.fwD[p] = v.wD[p];
}

__global__ void __launch_bounds__(256) k_seg_virtual(SegPair sp) {
    const SegView& v = sp.v[blockIdx.y];
    const uint32_t p = blockIdx.x * 256 + threadIdx.x;
    const uint32_t N = (uint32_t)v.W * (uint32_t)v.H;
    const bool root = p < N && v.first[seg_find(v.par, p)] == p;
    wave_append(v.cnt + SM_SEG_C_TREES, root);
    if (!root || p == 0) return;
    // the tree's first pixel links to its left neighbour, in column 0 to its upper one (sm_segment.cpp)
    if (p % (uint32_t)v.W > 0) {
        v.mR[p - 1] = 1;
        v.fwR[p - 1] = SM_VIRTUAL_W;
    } else {
        v.mD[p - (uint32_t)v.W] = 1;
        v.fwD[p - (uint32_t)v.W] = SM_VIRTUAL_W;
    }
}

unsigned blocks_of(size_t n, unsigned per) { return (unsigned)((n + per - 1) / per); }

constexpr int SEG_KEY_BITS = 42;  // (w << 32) | edge id, w < 1024

}  // namespace

hipError_t seg_launch_init(hipStream_t st, const SegPair& p) {
    const size_t N = (size_t)p.v[0].W * p.v[0].H;
    hipLaunchKernelGGL(k_seg_init, dim3(blocks_of(N, SM_SEG_TILE), p.nv), dim3(256), 0, st, p);
    hipLaunchKernelGGL(k_seg_scan, dim3(p.nv), dim3(1024), 0, st, p);
    return hipGetLastError();
}

hipError_t seg_launch_scatter(hipStream_t st, const SegPair& p) {
    const size_t N = (size_t)p.v[0].W * p.v[0].H;
    hipLaunchKernelGGL(k_seg_scatter, dim3(blocks_of(N, SM_SEG_TILE), p.nv), dim3(256), 0, st, p);
    return hipGetLastError();
}

hipError_t seg_launch_classify(hipStream_t st, const SegPair& p, int w, uint32_t m, float c, int lout, uint32_t gen) {
    hipLaunchKernelGGL(k_seg_classify, dim3(blocks_of(m, 256), p.nv), dim3(256), 0, st, p, w, c, lout, gen);
    hipLaunchKernelGGL(k_seg_hook, dim3(blocks_of(m, 256), p.nv), dim3(256), 0, st, p, lout, gen);
    return hipGetLastError();
}

hipError_t seg_launch_round(hipStream_t st, const SegPair& p, uint32_t m, int lin, int lout, uint32_t gen) {
    hipLaunchKernelGGL(k_seg_best, dim3(blocks_of(m, 256), p.nv), dim3(256), 0, st, p, lin, lout, gen);
    hipLaunchKernelGGL(k_seg_hook, dim3(blocks_of(m, 256), p.nv), dim3(256), 0, st, p, lout, gen);
    return hipGetLastError();
}

hipError_t seg_launch_tail(hipStream_t st, const SegPair& p, int lin, uint32_t gen0) {
    const int lds = sm_knob("SM_SEG_TAIL_GLOBAL") ? 0 : 1;
    const uint32_t tmin = sm_knob("SM_SEG_TAIL_MIN") ? (uint32_t)atoi(sm_knob("SM_SEG_TAIL_MIN")) : SEG_TAIL_MIN;
    hipLaunchKernelGGL(k_seg_tail, dim3(p.nv), dim3(1024), 0, st, p, lin, gen0, lds, tmin);
    return hipGetLastError();
}

hipError_t seg_launch_small(hipStream_t st, const SegPair& p, int w0, int w1, float c, uint32_t gen0, bool split) {
    // SM_SEG_ACT_MAX: the most active edges bucketed in LDS (0: always the full scan; tests)
    const uint32_t lc = (uint32_t)SEG_LC;
    const uint32_t amax = sm_knob("SM_SEG_ACT_MAX") ? (uint32_t)atoi(sm_knob("SM_SEG_ACT_MAX")) : (uint32_t)SEG_ACT_MAX;
    const int prof = sm_knob("SM_SEG_PROF") ? 1 : 0;
    // SM_SEG_NORUN=1: no k_seg_run (every split run through k_seg_small)
    if (split && !sm_knob("SM_SEG_NORUN")) hipLaunchKernelGGL(k_seg_run, dim3(p.nv), dim3(1024), 0, st, p, w0, w1, c);
    hipLaunchKernelGGL(k_seg_small, dim3(p.nv), dim3(1024), 0, st, p, w0, w1, c, gen0, lc, split ? 1 : 0, amax, prof);
    return hipGetLastError();
}

hipError_t seg_launch_split(hipStream_t st, const SegPair& p, int w0, int w1, float c, uint32_t nedges) {
    if (nedges) hipLaunchKernelGGL(k_seg_split, dim3(blocks_of(nedges, 256), p.nv), dim3(256), 0, st, p, w0, w1, c);
    return hipGetLastError();
}

hipError_t seg_launch_flatten(hipStream_t st, const SegPair& p) {
    const size_t N = (size_t)p.v[0].W * p.v[0].H;
    hipLaunchKernelGGL(k_seg_flatten, dim3(blocks_of(N, 256), p.nv), dim3(256), 0, st, p);
    return hipGetLastError();
}

hipError_t seg_launch_sizes(hipStream_t st, const SegPair& p, int w, uint32_t m) {
    hipLaunchKernelGGL(k_seg_sizes, dim3(blocks_of(m, 256), p.nv), dim3(256), 0, st, p, w);
    return hipGetLastError();
}

hipError_t seg_launch_minsize(hipStream_t st, const SegPair& p, int min_size, uint32_t nrej_max) {
    const uint32_t ms = (uint32_t)(min_size < 2 ? 2 : min_size);
    if (nrej_max) hipLaunchKernelGGL(k_seg_minsize, dim3(blocks_of(nrej_max, 256), p.nv), dim3(256), 0, st, p, ms);
    return hipGetLastError();
}

// The min-size candidates' sorts (~260k pairs per C2 view): rocprim's onesweep radix sort (one histogram
// launch + one launch per 8-bit digit, stable) instead of hipcub's choice below 2^20 items, the merge-sort
// path (~20 launches per sort, 0.2-0.36 ms each at C2).  (Only when the hashed pair dedupe's table does
// not fit: the default dedupe sorts nothing.)
using SegOnesweep = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config, rocprim::default_config, 0>;
hipError_t seg_sort_pairs(void* temp, size_t& bytes, const unsigned long long* kin, unsigned long long* kout,
                          const uint32_t* vin, uint32_t* vout, uint32_t n, int bits, hipStream_t st) {
    return rocprim::radix_sort_pairs<SegOnesweep>(temp, bytes, kin, kout, vin, vout, n, 0u, (unsigned)bits, st);
}

size_t seg_sort_temp_bytes(uint32_t n) {
    size_t a = 0, b = 0, c = 0, d = 0, e = 0;
    (void)rocprim::radix_sort_pairs<SegOnesweep>(nullptr, d, (const unsigned long long*)nullptr, (unsigned long long*)nullptr,
                                                 (const uint32_t*)nullptr, (uint32_t*)nullptr, n, 0u, 64u);
    (void)rocprim::radix_sort_pairs<SegOnesweep>(nullptr, e, (const unsigned long long*)nullptr, (unsigned long long*)nullptr,
                                                 (const uint32_t*)nullptr, (uint32_t*)nullptr, n, 0u, (unsigned)SEG_KEY_BITS);
    a = std::max(a, std::max(d, e));
    // the scans: E + 1 candidate flags, N + 1 root marks (n = E = 2N)
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, c, (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n + 1);
    return std::max(a, std::max(b, c));
}

// per view: its nmin candidates sorted by key (temp: that view's scratch), then one gather launch
hipError_t seg_launch_sort(hipStream_t st, const SegPair& p, void* const* temp, const size_t* temp_bytes) {
    uint32_t nmax = 0;
    for (int i = 0; i < p.nv; ++i) {
        const SegView& v = p.v[i];
        if (v.nmin == 0) continue;
        nmax = v.nmin > nmax ? v.nmin : nmax;
        size_t tb = temp_bytes[i];
        hipError_t e = seg_sort_pairs(temp[i], tb, v.mkey[0], v.mkey[1], v.mval[0], v.mval[1], v.nmin, SEG_KEY_BITS, st);
        if (e != hipSuccess) return e;
    }
    if (nmax) hipLaunchKernelGGL(k_seg_gather, dim3(blocks_of(nmax, 256), p.nv), dim3(256), 0, st, p);
    return hipGetLastError();
}

hipError_t seg_launch_dedupe(hipStream_t st, const SegPair& p, void* const* temp, const size_t* temp_bytes) {
    const size_t N = (size_t)p.v[0].W * p.v[0].H;
    int bits = 1;
    while (bits < 64 && (1ull << bits) <= (unsigned long long)N * N) ++bits;
    uint32_t nmax = 0;
    for (int i = 0; i < p.nv; ++i) nmax = p.v[i].nmin > nmax ? p.v[i].nmin : nmax;
    const unsigned nb = blocks_of(nmax ? nmax : 1, 256);
    hipLaunchKernelGGL(k_seg_pairkey, dim3(nb, p.nv), dim3(256), 0, st, p);
    for (int i = 0; i < p.nv; ++i) {
        const SegView& v = p.v[i];
        hipError_t e = hipMemsetAsync(v.lmark, 0, (N + 1) * 4, st);
        if (e != hipSuccess) return e;
        if (v.nmin == 0) continue;
        size_t tb = temp_bytes[i];
        if ((e = seg_sort_pairs(temp[i], tb, v.mkey[0], v.mkey[1], v.mval[0], v.mval[1], v.nmin, bits, st)) != hipSuccess)
            return e;
    }
    hipLaunchKernelGGL(k_seg_keep, dim3(nb, p.nv), dim3(256), 0, st, p);
    hipLaunchKernelGGL(k_seg_mark, dim3(nb, p.nv), dim3(256), 0, st, p);
    for (int i = 0; i < p.nv; ++i) {
        const SegView& v = p.v[i];
        size_t tb = temp_bytes[i];
        hipError_t e = hipcub::DeviceScan::ExclusiveSum(temp[i], tb, v.keep, v.kpos, (int)v.nmin + 1, st);
        if (e != hipSuccess) return e;
        tb = temp_bytes[i];
        if ((e = hipcub::DeviceScan::ExclusiveSum(temp[i], tb, v.lmark, v.lid, (int)N + 1, st)) != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_seg_dense, dim3(nb, p.nv), dim3(256), 0, st, p);
    return hipGetLastError();
}

hipError_t seg_launch_dedupe_hash(hipStream_t st, const SegPair& p, void* const* temp, const size_t* temp_bytes,
                                  uint32_t cap) {
    const size_t N = (size_t)p.v[0].W * p.v[0].H;
    uint32_t nmax = 0;
    for (int i = 0; i < p.nv; ++i) {
        const SegView& v = p.v[i];
        nmax = v.nmin > nmax ? v.nmin : nmax;
        hipError_t e;
        if ((e = hipMemsetAsync(v.mkey[0], 0xFF, (size_t)cap * 8, st)) != hipSuccess) return e;
        if ((e = hipMemsetAsync(v.mkey[1], 0xFF, (size_t)cap * 8, st)) != hipSuccess) return e;
        if ((e = hipMemsetAsync(v.lmark, 0, (N + 1) * 4, st)) != hipSuccess) return e;
    }
    const unsigned nb = blocks_of(nmax ? nmax : 1, 256);
    hipLaunchKernelGGL(k_seg_hins, dim3(nb, p.nv), dim3(256), 0, st, p, cap);
    hipLaunchKernelGGL(k_seg_hkeep, dim3(nb, p.nv), dim3(256), 0, st, p);
    for (int i = 0; i < p.nv; ++i) {
        const SegView& v = p.v[i];
        size_t tb = temp_bytes[i];
        hipError_t e = hipcub::DeviceScan::ExclusiveSum(temp[i], tb, v.keep, v.kpos, (int)v.nmin + 1, st);
        if (e != hipSuccess) return e;
        tb = temp_bytes[i];
        if ((e = hipcub::DeviceScan::ExclusiveSum(temp[i], tb, v.lmark, v.lid, (int)N + 1, st)) != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_seg_hdense, dim3(nb, p.nv), dim3(256), 0, st, p);
    return hipGetLastError();
}

hipError_t seg_launch_apply(hipStream_t st, const SegPair& p) {
    int nmax = 0;
    for (int i = 0; i < p.nv; ++i) nmax = p.v[i].nhooks > nmax ? p.v[i].nhooks : nmax;
    if (nmax) hipLaunchKernelGGL(k_seg_apply, dim3(blocks_of((size_t)nmax, 256), p.nv), dim3(256), 0, st, p);
    return hipGetLastError();
}

hipError_t seg_launch_trees(hipStream_t st, const SegPair& p) {
    const size_t N = (size_t)p.v[0].W * p.v[0].H;
    hipLaunchKernelGGL(k_seg_first, dim3(blocks_of(N, 256), p.nv), dim3(256), 0, st, p);
    hipLaunchKernelGGL(k_seg_virtual, dim3(blocks_of(N, 256), p.nv), dim3(256), 0, st, p);
    return hipGetLastError();
}
