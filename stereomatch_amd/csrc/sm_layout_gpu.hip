// sm_layout_gpu.hip -- tree layout on the GPU: rooting at pixel 0, subtree sizes, heavy-light
// decomposition, heavy-first preorder slots, light depth, per-slot metadata and per-round
// heavy-path lists, from the MST edge mask produced by Boruvka.
//
// Method: Euler tour of the MST (arc a = 4*p + k, k: 0 right, 1 down, 2 left, 3 up; the tour
// leaves a pixel through the next MST direction after the one it arrived from), ranked by
//   L1  k_tour_tile   : per 32x32 tile, LDS pointer jumping contracts every maximal run of the
//                       tour inside the tile into one chain (distance-to-chain-end, chain id)
//   L2  k_chain_*     : in-place pointer jumping over the ~1e5 chains in global memory
//   L3  (k_orient)    : arc rank = tour length - arcs to the tour end (sm_tour.h)
// then orientation (an arc is "down" iff it precedes its reverse), subtree size
// (rank distance / 2), heavy child (max size, ties -> smallest direction), and a single int64
// prefix sum over the tour of (light<<32 | preorder offset) that yields every node's heavy-first
// preorder number and light depth at once.  Slot = preorder.  This reproduces the rooting and
// child order of Stereo3DMST.cpp:450-522 (root = first pixel; children by edge key), which is all
// the exact arithmetic depends on; the heavy-light choice only schedules the work.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <stdint.h>

#include <algorithm>

#include "sm_common.h"
#include "sm_layout_gpu.h"
#include "sm_tour.h"
#include "sm_knob.h"

#ifndef SM_RUN_DIV
#define SM_RUN_DIV 384  // run window = bucket nodes / SM_RUN_DIV (~3 runs per CU, both views)
#endif
__device__ __forceinline__ uint32_t nbr_of(uint32_t p, int k, int W) { return tour_nbr(p, k, W); }

// next MST direction of pixel q after direction j, cyclic (j itself if q is a leaf)
__device__ __forceinline__ int next_dir(uint32_t adjq, int j) {
#pragma unroll
    for (int t = 1; t <= 4; ++t) {
        const int k = (j + t) & 3;
        if (adjq & (1u << k)) return k;
    }
    return j;
}

__device__ __forceinline__ uint64_t key_dir(const uint16_t* wR, const uint16_t* wD, int W, uint32_t p, int k) {
    switch (k) {
        case 0: return sm_edge_key(wR[p], p, 0u);
        case 1: return sm_edge_key(wD[p], p, 1u);
        case 2: return sm_edge_key(wR[p - 1], p - 1, 0u);
        default: return sm_edge_key(wD[p - W], p - (uint32_t)W, 1u);
    }
}

// ------------------------------------------------------------------------------------------
// 32x32 pixel tiles of the layout's per-pixel kernels, XCD-aware (round 5): block b of the 1D grid
// (8 x per blocks, per = ceil(tiles / 8)) takes tile (b % 8) * per + b / 8.  Blocks b and b + 8 share an
// XCD (round-robin dispatch), so each XCD takes a band of consecutive tiles, and a tile sits on the same
// XCD in every kernel.  A tile touches the arrays indexed by tour rank (its chains are tile runs of the
// tour, sm_tour.h), by preorder or by slot in a few contiguous runs, which then stay in that XCD's L2;
// in row order the same passes were scattered over every L2.  Placement is for speed only: nothing
// depends on it.
struct TileRef {
    int x0, y0;
    bool ok;
};
__device__ __forceinline__ TileRef layout_tile(int W, int H, int b) {
    const int ntx = (W + TL - 1) / TL, nt = ntx * ((H + TL - 1) / TL);
    const int per = (nt + 7) / 8;
    const int t = (b & 7) * per + (b >> 3);
    return TileRef{(t % ntx) * TL, (t / ntx) * TL, t < nt};
}
__host__ __device__ inline int layout_tile_blocks(int W, int H) {
    const int nt = ((W + TL - 1) / TL) * ((H + TL - 1) / TL);
    return 8 * ((nt + 7) / 8);
}
// f(pixel) over tile t's pixels: 256 threads x 4 rows of 32 (a wave: two 32-pixel row segments)
template <class F>
__device__ __forceinline__ void tile_pixels(const TileRef& t, int W, int H, F&& f) {
    if (!t.ok) return;
    const int lx = (int)threadIdx.x & 31, ly = (int)threadIdx.x >> 5;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int x = t.x0 + lx, y = t.y0 + ly + 8 * i;
        if (x < W && y < H) f((uint32_t)(y * W + x));
    }
}
// ... with the pixel's coordinates: f(pixel, x, y)
template <class F>
__device__ __forceinline__ void tile_pixels_xy(const TileRef& t, int W, int H, F&& f) {
    if (!t.ok) return;
    const int lx = (int)threadIdx.x & 31, ly = (int)threadIdx.x >> 5;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int x = t.x0 + lx, y = t.y0 + ly + 8 * i;
        if (x < W && y < H) f((uint32_t)(y * W + x), (uint32_t)x, (uint32_t)y);
    }
}

__global__ void k_adj(LayoutPair LP, int W, int H) {
    if (*LP.mst_ok == 0) return;  // the MST is still a forest: nothing to lay out yet (stage_layout redoes it)
    const LayoutView& V = LP.v[blockIdx.z];
    const int y = blockIdx.y, x = blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= W) return;
    const uint32_t p = (uint32_t)(y * W + x);
    uint32_t a = 0;
    if (V.mR[p]) a |= 1u;
    if (V.mD[p]) a |= 2u;
    if (x > 0 && V.mR[p - 1]) a |= 4u;
    if (y > 0 && V.mD[p - W]) a |= 8u;
    V.adj[p] = (uint8_t)a;
}

// the global tour start: first MST direction out of pixel 0 (direction order 0..3)
__device__ __forceinline__ uint32_t start_arc(const uint8_t* adj) {
    const uint32_t a0 = adj[0];
    for (int k = 0; k < 4; ++k)
        if (a0 & (1u << k)) return (uint32_t)k;
    return SM_NONE;
}

__device__ __forceinline__ uint32_t succ_arc(const uint8_t* adj, int W, uint32_t a, uint32_t start) {
    const uint32_t p = a >> 2;
    const int k = (int)(a & 3u);
    const uint32_t q = nbr_of(p, k, W);
    const int k2 = next_dir(adj[q], (k + 2) & 3);
    const uint32_t s = 4u * q + (uint32_t)k2;
    return s == start ? SM_NONE : s;
}

// The MST's tour as a tour_tile graph (sm_tour.h): arcs along MST edges, the successor leaves a
// pixel through the next MST direction after the one it arrived from; one list, cut before the start
struct MstTour {
    const uint8_t* adj;
    int W;
    uint32_t start;
    __device__ bool has(uint32_t p, int k) const { return (adj[p] >> k) & 1u; }
    __device__ uint32_t succ(uint32_t a) const { return succ_arc(adj, W, a, start); }
};

__device__ __forceinline__ TourBufs tour_bufs(const LayoutView& V) {
    return TourBufs{V.a_dist, V.a_cid, V.nchains, V.c_last, V.c_len, V.cnw, nullptr, 0};
}

// L1: contract the tour inside each 32x32 tile (sm_tour.h)
// (waves_per_eu 8: 66 -> 64 VGPRs, no scratch; with the bit-packed predecessor flags the LDS fits 8 per CU)
__global__ __launch_bounds__(TL_THREADS) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_tour_tile(LayoutPair LP, int W, int H) {
    if (*LP.mst_ok == 0) return;  // the MST is still a forest: nothing to lay out yet (stage_layout redoes it)
    const LayoutView& V = LP.v[blockIdx.z];
    const TileRef t = layout_tile(W, H, (int)blockIdx.x);
    if (!t.ok) return;  // (block-uniform)
    TourBufs T = tour_bufs(V);
    T.err = reinterpret_cast<int32_t*>(LP.scan.err);  // the layout's error bit
    T.errv = 2;
    tour_tile(MstTour{V.adj, W, start_arc(V.adj)}, T, W, H, t.x0, t.y0);
}

// L2 init: chain successor + weight
__global__ void k_chain_init(LayoutPair LP, int W) {
    if (*LP.mst_ok == 0) return;  // the MST is still a forest: nothing to lay out yet (stage_layout redoes it)
    const LayoutView& V = LP.v[blockIdx.y];
    tour_chain_init(MstTour{V.adj, W, start_arc(V.adj)}, tour_bufs(V), blockIdx.x * blockDim.x + threadIdx.x);
}

// L2: suffix sums over the chain list by in-place pointer jumping, one launch (sm_tour.h).  The grid
// is at most CR_BLOCKS blocks (co-resident).
#define CR_BLOCKS 256  // per view, 256 threads each (1024 / 256 / 128: the same frame rate at C2, round 5;
                       // the smaller grid leaves the other frames' kernels room)

__global__ __launch_bounds__(256) void k_chain_rank(LayoutPair LP) {
    if (*LP.mst_ok == 0) return;  // the MST is still a forest: nothing to lay out yet (stage_layout redoes it)
    tour_chain_rank(tour_bufs(LP.v[blockIdx.y]));
}

// Tour values are 32-bit, light << 27 | preorder offset, summed mod 2^32 (round 5; int64 before): a
// prefix sum is (light depth) << 27 | (preorder), exactly, while N <= 2^27 (the host checks) and the
// light depth < 32 (SM_MAX_ROUNDS); an up arc's value, the negation, is >= 2^31 and a down arc's < 2^28.
#define TOUR_SHIFT 27
#define TOUR_LIGHT (1u << TOUR_SHIFT)
// a path head's preorder record: (1 + position) << 5 | light depth (32 bits while N < 2^27; the max-scan
// carries it to the path's other positions, which hold 0)
#define HK_REC(pre, ld) ((((pre) + 1u) << 5) | (ld))

// L3 + orientation + heavy child, one pass per pixel v: an arc's rank is the tour length minus its
// suffix (sm_tour.h); an arc precedes its reverse iff it goes down, and the rank distance between the
// two is twice the subtree size below it.  From the two suffixes of each tree edge at v, v knows its
// parent direction and its own subtree size, and every child's subtree size and arc ranks.  So it picks its heavy child (max size, ties -> smallest
// direction) and writes the tour values of its children's edges straight at their ranks: down arc into
// child c +(light << 27 | preorder offset of c within v's subtree, heavy child first), up arc out of c
// the negation, and c itself at the down arc's rank (arcpix).  (Round 5: k_orient and k_heavy fused;
// k_heavy had re-read every child's size and ranks.)
__global__ void k_orient(LayoutPair LP, int W, int H) {
    if (*LP.mst_ok == 0) return;  // the MST is still a forest: nothing to lay out yet (stage_layout redoes it)
    const LayoutView& V = LP.v[blockIdx.z];
    const TileRef tr = layout_tile(W, H, (int)blockIdx.x);
    const unsigned long long below = (1ull << (threadIdx.x & 63)) - 1ull;
    uint32_t wacc = 0;  // this wave's light children's parents so far (every active lane holds it)
    tile_pixels(tr, W, H, [&](uint32_t v) {
        const uint32_t adj = V.adj[v];
        const uint32_t total = 2u * (uint32_t)(W * H) - 2u;
        const TourBufs T = tour_bufs(V);
        int pd = -1, heavy = -1;
        uint32_t sz = (uint32_t)(W * H), best = 0;
        uint32_t csz[4] = {0u, 0u, 0u, 0u};
        uint2 crio[4];
        bool bad = false;
        // v's own four arcs are one 16-byte chain-id record and one 8-byte distance record
        const uint4 oc = *reinterpret_cast<const uint4*>(V.a_cid + 4u * v);
        const uint2 od = *reinterpret_cast<const uint2*>(V.a_dist + 4u * v);
        const uint32_t ocid[4] = {oc.x, oc.y, oc.z, oc.w};
        const uint32_t odist[4] = {od.x & 0xFFFFu, od.x >> 16, od.y & 0xFFFFu, od.y >> 16};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            crio[k] = make_uint2(0u, 0u);
            if (!(adj & (1u << k))) continue;
            const uint32_t n = nbr_of(v, k, W);
            const uint32_t si = tour_suffix(T, 4u * n + (uint32_t)((k + 2) & 3));  // n -> v
            const uint32_t so = T.c_len[ocid[k]] + odist[k];                       // v -> n (tour_suffix)
            bad |= si - 1u >= total || so - 1u >= total;  // (never for a spanning tree's tour)
            if (si > so) {  // rank(n -> v) < rank(v -> n): n is the parent
                pd = k;
                sz = (si - so + 1u) / 2u;
            } else {        // n is a child
                csz[k] = (so - si + 1u) / 2u;
                crio[k] = make_uint2(total - so, total - si);
                if (csz[k] > best) { best = csz[k]; heavy = k; }
            }
        }
        // compact A row, part 1 (SmMeta::cslot[3]): a node of >= 2 children has a light one; its rank
        // among its tile wave's (the wave's lanes active here were active in every earlier pass)
        const int nc = __popc(adj & 15u) - (pd >= 0 ? 1 : 0);
        const unsigned long long bal = __ballot(!bad && nc >= 2);
        if (!bad && nc >= 2) V.lrank[v] = (uint8_t)(wacc + (uint32_t)__popcll(bal & below));
        wacc += (uint32_t)__popcll(bal);
        if (bad) {
            __hip_atomic_fetch_or(LP.scan.err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            return;
        }
        V.pdir[v] = (int8_t)pd;
        if (LP.want_size) V.size[v] = sz;  // (only sm_build_tree reports subtree sizes)
        V.heavy[v] = (int8_t)heavy;
        if (pd < 0) {  // the root: preorder 0, light depth 0, a path head (the tour scan writes the others)
            V.hk[0] = HK_REC(0u, 0u);
            V.pixpre[0] = v;
        }
        uint32_t off = 1u + (heavy >= 0 ? csz[heavy] : 0u);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (!(adj & (1u << k)) || k == pd) continue;
            uint32_t val = 1u;  // the heavy child: offset 1, not light
            if (k != heavy) {
                val = TOUR_LIGHT + off;
                off += csz[k];
            }
            V.tour[crio[k].x] = val;
            V.tour[crio[k].y] = 0u - val;
            V.arcpix[crio[k].x] = nbr_of(v, k, W);  // the child, for the scan's epilogue
        }
    });
    // the wave's count (lane 0 is active wherever any lane of its wave is), scanned after this pass
    if (tr.ok && (threadIdx.x & 63) == 0)
        V.wrow[4 * ((tr.y0 / TL) * ((W + TL - 1) / TL) + tr.x0 / TL) + (threadIdx.x >> 6)] = wacc;
}

// ---- inclusive scans: reduce, then scan (round 5).  A tile is SP_TILE elements (4096 of 32 bits, 2048 of 64) per 256-thread block,
// each wave 16 chunks of 64 consecutive elements (coalesced).  k_scan_reduce writes every tile's total;
// k_scan_tiles re-reads its tile, takes its exclusive prefix as the reduction of the lower tiles' totals
// (<= a few thousand L2-resident words per block, so no third launch scans the totals), scans in
// registers and writes in place.  Nothing waits on another block.  (A single-pass decoupled look-back
// was tried this round: its status words cross XCDs, so each look-back hop is an agent-scope round trip,
// and the int64 scan took 193 us at C2 against 89 for the old 3-phase scan; this one reads its data
// twice but never serialises.)
#define SP_THREADS 256
// items per thread: 16 of 32 bits, 8 of 64 bits (16 64-bit items and their interleaved shuffles took
// 120 VGPRs: 4 waves per SIMD)
// (an epilogue may ask for fewer: Out::kItems, e.g. the path histogram's, whose 16 unrolled items took 95
// VGPRs)
template <class T> struct SpItems { static constexpr int n = sizeof(T) == 8 ? 8 : 16; };
template <class T, class Out> struct SpItemsOut { static constexpr int n = Out::kItems ? Out::kItems : SpItems<T>::n; };
#define SP_ITEMS IT
#define SP_TILE (SP_THREADS * IT)

struct OpAdd {
    template <class T> __device__ static T apply(T a, T b) { return a + b; }
    template <class T> __device__ static T ident() { return T(0); }
};
struct OpMax {
    template <class T> __device__ static T apply(T a, T b) { return a > b ? a : b; }
    template <class T> __device__ static T ident() { return T(0); }
};

// block-wide exclusive scan of one value per thread (SCAN_BLOCK threads; k_long_segments)
#define SCAN_BLOCK 1024

template <class T, class Op>
__device__ __forceinline__ T block_exclusive_scan(T v, T* sh, T* total) {
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    T x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const T y = __shfl_up(x, off);
        if (lane >= off) x = Op::apply(x, y);
    }
    if (lane == 63) sh[wid] = x;
    __syncthreads();
    if (wid == 0) {
        T s2 = lane < (SCAN_BLOCK / 64) ? sh[lane] : Op::template ident<T>();
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const T y = __shfl_up(s2, off);
            if (lane >= off) s2 = Op::apply(s2, y);
        }
        if (lane < (SCAN_BLOCK / 64)) sh[lane] = s2;
    }
    __syncthreads();
    const T wpre = wid ? sh[wid - 1] : Op::template ident<T>();
    if (total) *total = sh[SCAN_BLOCK / 64 - 1];
    // exclusive: combine warp prefix with the lane's exclusive prefix
    T lex = __shfl_up(x, 1);
    if (lane == 0) lex = Op::template ident<T>();
    const T r = Op::apply(wpre, lex);
    __syncthreads();
    return r;
}

template <class T>
struct ScanBufs {
    T* data[2];
    const uint32_t* len[2];  // optional: the element count, read on the device (min with nelem)
};
template <class T>
__device__ __forceinline__ int scan_len(const ScanBufs<T>& B, int v, int nelem) {
    return B.len[v] ? min(nelem, (int)*B.len[v]) : nelem;
}

// block-wide reduction of one value per thread (SP_THREADS threads), the result on every thread
template <class T, class Op>
__device__ __forceinline__ T sp_block_reduce(T x, T* sh) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) x = Op::apply(x, __shfl_xor(x, off));  // (add / max: order-free)
    const int lane = (int)threadIdx.x & 63, w = (int)threadIdx.x >> 6;
    __syncthreads();  // sh may still be read by a previous call
    if (lane == 0) sh[w] = x;
    __syncthreads();
    T r = sh[0];
#pragma unroll
    for (int k = 1; k < SP_THREADS / 64; ++k) r = Op::apply(r, sh[k]);
    return r;
}

template <class T, class Op, int IT>
__global__ __launch_bounds__(SP_THREADS) void k_scan_reduce(ScanBufs<T> B, ScanState S, int nelem) {
    const int v = blockIdx.y;
    nelem = scan_len(B, v, nelem);
    __shared__ T sh[SP_THREADS / 64];
    const T* d = B.data[v];
    const int lane = (int)threadIdx.x & 63, w = (int)threadIdx.x >> 6;
    const size_t wbase = (size_t)blockIdx.x * SP_TILE + (size_t)w * 64 * SP_ITEMS;
    T x = Op::template ident<T>();
#pragma unroll
    for (int j = 0; j < SP_ITEMS; ++j) {
        const size_t i = wbase + (size_t)j * 64 + lane;
        if (i < (size_t)nelem) x = Op::apply(x, d[i]);
    }
    const T tot = sp_block_reduce<T, Op>(x, sh);
    if (threadIdx.x == 0) reinterpret_cast<T*>(S.part[v])[blockIdx.x] = tot;
}

// the scans' outputs: in place (the max-scan of hk, the add-scan of the path lengths) ...
struct ScanInPlace {
    static constexpr int kItems = 0;      // items per thread (0: by element size)
    static constexpr bool kNext = false;  // the epilogue needs the next element's tag bit 0
    __device__ bool active() const { return true; }
    __device__ void begin() const {}
    __device__ void end(int) const {}
    template <class T> __device__ static uint32_t tag(T) { return 0u; }
    template <class T> __device__ void operator()(T* d, int, size_t i, T incl, uint32_t, bool) const { d[i] = incl; }
};
// ... or, for the tour, the preorder records: at the down arc into node q (orig < 2^31) the inclusive sum is
// (light depth of q) << 27 | (heavy-first preorder of q), and orig == 1 iff q is its parent's heavy child,
// so hk[pre] = HK_REC(pre, light depth) at a path head (0 elsewhere: after the inclusive
// max-scan of hk every position holds its path's head and that head's light depth) and pixpre[pre] = q.
// The root's record comes from k_orient.  (Round 5: this epilogue replaces k_assign, which re-read each
// pixel's parent arc rank, its tour sum and its parent's heavy child; the tour itself is not written back.)
struct ScanTourOut {
    LayoutPair LP;
    int N;
    static constexpr int kItems = 0;
    static constexpr bool kNext = false;
    // an incomplete MST (k_orient wrote nothing: the tour holds a previous call's values) has no records
    __device__ bool active() const { return *LP.mst_ok != 0; }
    __device__ void begin() const {}
    __device__ void end(int) const {}
    // what the epilogue needs of an element's own value, 2 bits (kept in one register for all 16 items
    // instead of a copy of the items): 1 = a down arc, 2 = the heavy child's
    __device__ static uint32_t tag(uint32_t orig) { return orig < 0x80000000u ? (orig == 1u ? 3u : 1u) : 0u; }
    __device__ void operator()(uint32_t*, int v, size_t i, uint32_t incl, uint32_t tg, bool) const {
        if (!(tg & 1u)) return;  // an up arc
        const LayoutView& V = LP.v[v];
        const uint32_t pre = incl & (TOUR_LIGHT - 1u), ld = incl >> TOUR_SHIFT;
        if (pre >= (uint32_t)N || ld >= (uint32_t)SM_MAX_ROUNDS) {  // never for a spanning tree's tour (defensive)
            __hip_atomic_fetch_or(LP.scan.err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            return;
        }
        V.hk[pre] = !(tg & 2u) ? HK_REC(pre, ld) : 0u;
        V.pixpre[pre] = V.arcpix[i];
    }
};

// ... or, for the max-scan of the path records, in place plus the path histogram (round 5: replaces
// k_path_count): position s ends its path iff s + 1 is a head (tag: the raw record is not 0), and its
// scanned record names the path's head and light depth -> per (light depth, long / short) bucket the
// paths, their nodes and the longest, block-aggregated in LDS.
struct ScanPathCount {
    static constexpr int kItems = 8;
    static constexpr bool kNext = true;
    LayoutPair LP;
    __device__ bool active() const { return *LP.mst_ok != 0; }
    __device__ static uint32_t* lds() {
        __shared__ uint32_t h[3 * SM_NBUCKETS];  // paths, nodes, longest
        return h;
    }
    __device__ void begin() const {
        for (int i = threadIdx.x; i < 3 * SM_NBUCKETS; i += blockDim.x) lds()[i] = 0;
        __syncthreads();
    }
    __device__ static uint32_t tag(uint32_t raw) { return raw != 0u ? 1u : 0u; }
    // another wave's element k, raw or already scanned (in place) by now: a head's record names k itself
    // either way, any other position holds 0 or an earlier head's record
    __device__ static bool tag_of_stored(uint32_t stored, size_t k) { return (stored >> 5) == (uint32_t)k + 1u; }
    __device__ void operator()(uint32_t* d, int v, size_t i, uint32_t incl, uint32_t, bool next_head) const {
        d[i] = incl;
        if (!next_head) return;
        const uint32_t s = (uint32_t)i, head = (incl >> 5) - 1u, ld = incl & 31u;
        if (head > s) {  // (never for a spanning tree's tour: defensive)
            __hip_atomic_fetch_or(LP.scan.err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            return;
        }
        const uint32_t len = s - head + 1u, b = 2u * ld + (len >= SM_LONG_PATH ? 0u : 1u);
        uint32_t* h = lds();
        atomicAdd(&h[b], 1u);
        atomicAdd(&h[SM_NBUCKETS + b], len);
        if (len >= SM_LONG_PATH) atomicMax(&h[2 * SM_NBUCKETS + b], len);
        (void)v;
    }
    __device__ void end(int v) const {
        __syncthreads();
        const LayoutView& V = LP.v[v];
        const uint32_t* h = lds();
        const int b = threadIdx.x;
        if (b < SM_NBUCKETS && h[b]) {
            atomicAdd(&V.round_count[b], h[b]);
            atomicAdd(&V.round_nodes[b], h[SM_NBUCKETS + b]);
            if (h[2 * SM_NBUCKETS + b]) atomicMax(&V.round_maxlen[b], h[2 * SM_NBUCKETS + b]);
        }
    }
};

template <class T, class Op, class Out, int IT>
__global__ __launch_bounds__(SP_THREADS) void k_scan_tiles(ScanBufs<T> B, ScanState S, int nelem, Out out) {
    if (!out.active()) return;  // (block-uniform)
    const int v = blockIdx.y;
    nelem = scan_len(B, v, nelem);
    if ((size_t)blockIdx.x * SP_TILE >= (size_t)nelem) return;  // (block-uniform) past a dynamic length
    const uint32_t tile = blockIdx.x;
    __shared__ T s_w[SP_THREADS / 64];
    T* d = B.data[v];
    const int lane = (int)threadIdx.x & 63, w = (int)threadIdx.x >> 6;
    const size_t wbase = (size_t)tile * SP_TILE + (size_t)w * 64 * SP_ITEMS;
    T x[SP_ITEMS];
    uint32_t tags = 0;  // 2 bits per item (Out::tag)
#pragma unroll
    for (int j = 0; j < SP_ITEMS; ++j) {
        const size_t i = wbase + (size_t)j * 64 + lane;
        x[j] = i < (size_t)nelem ? d[i] : Op::template ident<T>();
        tags |= Out::tag(x[j]) << (2 * j);
    }
    // the tile's exclusive prefix: the lower tiles' totals (loads in flight with the tile's)
    const T* part = reinterpret_cast<const T*>(S.part[v]);
    T pre = Op::template ident<T>();
    for (uint32_t t = threadIdx.x; t < tile; t += SP_THREADS) pre = Op::apply(pre, part[t]);
#pragma unroll
    for (int off = 1; off < 64; off <<= 1)
#pragma unroll
        for (int j = 0; j < SP_ITEMS; ++j) {
            const T y = __shfl_up(x[j], off);
            if (lane >= off) x[j] = Op::apply(y, x[j]);
        }
    T carry = Op::template ident<T>();
#pragma unroll
    for (int j = 0; j < SP_ITEMS; ++j) {
        const T tot = __shfl(x[j], 63);
        x[j] = Op::apply(carry, x[j]);
        carry = Op::apply(carry, tot);
    }
    pre = sp_block_reduce<T, Op>(pre, s_w);
    __syncthreads();
    if (lane == 0) s_w[w] = carry;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < SP_THREADS / 64; ++k)
        if (k < w) pre = Op::apply(pre, s_w[k]);
    out.begin();
#pragma unroll
    for (int j = 0; j < SP_ITEMS; ++j) {
        const size_t i = wbase + (size_t)j * 64 + lane;
        bool nxt = false;
        if constexpr (Out::kNext) {  // the next element's tag bit 0: a neighbour lane, the next chunk, or memory
            const uint32_t t0 = (tags >> (2 * j)) & 1u;
            const uint32_t dn = __shfl_down(t0, 1);
            uint32_t t1 = 0;
            if (j + 1 < SP_ITEMS) t1 = __shfl((tags >> (2 * (j + 1))) & 1u, 0);
            if (lane < 63) nxt = dn != 0u;
            else if (j + 1 < SP_ITEMS) nxt = t1 != 0u;
            else if (i + 1 < (size_t)nelem) nxt = Out::tag_of_stored(d[i + 1], i + 1);
            if (i + 1 == (size_t)nelem) nxt = true;  // the last element ends its path
        }
        if (i < (size_t)nelem) out(d, v, i, Op::apply(pre, x[j]), (tags >> (2 * j)) & 3u, nxt);  // inclusive
    }
    out.end(v);
}

template <class T, class Op, class Out = ScanInPlace>
static void launch_scan(hipStream_t st, const ScanBufs<T>& B, const ScanState& S, int nviews, int nelem, Out out = Out{}) {
    if (nelem <= 0) return;
    constexpr int IT = SpItemsOut<T, Out>::n;
    const int ntiles = (nelem + SP_TILE - 1) / SP_TILE;
    hipLaunchKernelGGL((k_scan_reduce<T, Op, IT>), dim3(ntiles, nviews), dim3(SP_THREADS), 0, st, B, S, nelem);
    hipLaunchKernelGGL((k_scan_tiles<T, Op, Out, IT>), dim3(ntiles, nviews), dim3(SP_THREADS), 0, st, B, S, nelem, out);
}

// Per-slot metadata: pixel, parent slot, child weights and slots in descending (w,a,b) key order (the
// reference's fold order), heavy-child position, light flag.  Round 5: computed in pixel order, where a
// node's tree neighbours are its grid neighbours (local reads), and written to its slot (one random
// 32-byte store) -- in slot order it had gathered a packed record of the node and of every neighbour.
// Round 6: compact A rows (SmMeta::cslot[3], sm_common.h) without atomics: a light children's parent's
// row is its tile wave's first row (wrow, exclusive) plus its rank in the wave (lrank, k_orient), so a
// path head writes its parent's row into its own parent word here too (SM_HEAD | row).
#define META_BLOCKS 1024  // blocks per view (grid-stride)

// the first compact row of pixel (x, y)'s tile wave; ntx tiles per image row
__device__ __forceinline__ uint32_t wave_row0(const LayoutView& V, uint32_t x, uint32_t y, uint32_t ntx) {
    const uint32_t k = 4u * ((y / TL) * ntx + x / TL) + ((y & 7u) >> 1);
    return k ? V.wrow[k - 1u] : 0u;
}

__global__ __launch_bounds__(256) void k_meta(LayoutPair LP, int W, int H) {
    if (*LP.mst_ok == 0) return;  // the MST is still a forest: nothing to lay out yet (stage_layout redoes it)
    const LayoutView& V = LP.v[blockIdx.y];
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // the rows' total: the scan's last entry
        const uint32_t nw = 4u * (uint32_t)(((W + TL - 1) / TL) * ((H + TL - 1) / TL));
        *V.n_has_light = V.wrow[nw - 1u];
    }
    // tiles in the XCD-aware order, grid-stride (META_BLOCKS is a multiple of 8: a block keeps its XCD band)
    const int nb = layout_tile_blocks(W, H);
    const uint32_t ntx = (uint32_t)(W + TL - 1) / TL;
    for (int b = (int)blockIdx.x; b < nb; b += META_BLOCKS) tile_pixels_xy(layout_tile(W, H, b), W, H, [&](uint32_t v, uint32_t px, uint32_t py) {
        const uint32_t adj = V.adj[v];
        const int pd = V.pdir[v], hv = V.heavy[v];
        const uint32_t slot = V.slotpix[v];
        // compact rows: v's own and its parent's inputs, loaded up front (unconditional: a root or a
        // node without light children reads its own words and ignores them)
        const uint32_t pn = pd >= 0 ? nbr_of(v, pd, W) : v;
        const uint32_t pnx = pd == 0 ? px + 1u : pd == 2 ? px - 1u : px, pny = pd == 1 ? py + 1u : pd == 3 ? py - 1u : py;
        const int par_heavy = V.heavy[pn];
        const uint32_t par_row = wave_row0(V, pnx, pny, ntx) + V.lrank[pn];
        const uint32_t own_row = wave_row0(V, px, py, ntx) + V.lrank[v];
        if (slot >= (uint32_t)(W * H)) {  // (never for a spanning tree's tour: defensive, err set)
            __hip_atomic_fetch_or(LP.scan.err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            return;
        }
        // the children in descending key order by a fixed 5-comparator network over the 4 directions
        // (absent ones sort last; keys are unique): no local array is indexed at run time, which
        // would put them in scratch memory
        uint32_t ck[4];
        uint32_t cs[4], cw[4];
        int cq[4];
        bool cv[4];
        uint32_t wp = 0, parent = SM_NONE;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const bool in = (adj & (1u << k)) != 0;
            const uint32_t n = in ? nbr_of(v, k, W) : v;
            // right / down edges are v's own, left / up the neighbour's
            const uint32_t w = k == 0 ? V.wR[v] : k == 1 ? V.wD[v] : k == 2 ? V.wR[n] : V.wD[n];
            // the (w, a, vertical) key order among v's own edges: for equal w, up (a = v - W) < left
            // (a = v - 1) < right (a = v, horizontal) < down (a = v, vertical), so a 32-bit key
            // w << 2 | that rank orders them as sm_edge_key does (round 5: 64-bit keys in the network)
            const uint32_t key = ((w & 1023u) << 2) | (k == 3 ? 0u : k == 2 ? 1u : k == 0 ? 2u : 3u);
            const uint32_t ns = in ? V.slotpix[n] : SM_NONE;
            if (in && k == pd) {
                wp = key >> 2;
                // a path head (not its parent's heavy child): SM_HEAD | the parent's compact A row
                parent = par_heavy == ((k + 2) & 3) ? ns : (SM_HEAD | par_row);
            }
            ck[k] = key;
            cq[k] = k;
            cs[k] = ns;
            cv[k] = in && k != pd;
        }
        auto cswap = [&](int i, int j) __attribute__((always_inline)) {  // i, j constants after unrolling
            const bool sw = cv[j] && (!cv[i] || ck[j] > ck[i]);
            const uint32_t tk = ck[i]; const int tq = cq[i]; const uint32_t ts = cs[i]; const bool tv = cv[i];
            ck[i] = sw ? ck[j] : ck[i]; cq[i] = sw ? cq[j] : cq[i]; cs[i] = sw ? cs[j] : cs[i]; cv[i] = sw ? cv[j] : cv[i];
            ck[j] = sw ? tk : ck[j]; cq[j] = sw ? tq : cq[j]; cs[j] = sw ? ts : cs[j]; cv[j] = sw ? tv : cv[j];
        };
        cswap(0, 1);
        cswap(2, 3);
        cswap(0, 2);
        cswap(1, 3);
        cswap(1, 2);
        int nch = 0;
        uint32_t hidx = 0, has_light = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            nch += cv[i] ? 1 : 0;
            cw[i] = cv[i] ? ck[i] >> 2 : 0u;
            cs[i] = cv[i] ? cs[i] : SM_NONE;
            if (cv[i]) {
                if (cq[i] == hv) hidx = (uint32_t)i; else has_light = 1;
            }
        }
        if (has_light) {
            // a light children's parent has at most 3 children (sm_common.h): its fourth child word is free
            if (nch > 3) __hip_atomic_fetch_or(LP.scan.err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            cs[3] = own_row;
        }
        V.meta[slot] = sm_make_meta(v, parent, wp, cw, (uint32_t)nch, hidx, has_light, cs);
    });
}

// heads in preorder -> path lengths -> bucketed by light depth (order inside a round is free).
// After the inclusive max-scan of hk (ScanTourOut), hk[s] >> 5 is 1 + the preorder position of the head
// of s's path (heavy paths are contiguous in preorder) and its low word 1 + that head's light depth;
// s is the last node of its path iff s + 1 is a head.
__device__ __forceinline__ bool path_last(const LayoutView& V, uint32_t s, int N) {
    return s + 1 == (uint32_t)N || (V.hk[s + 1] >> 5) == s + 2u;
}
// the path ending at s: its head and (light depth, long/short) bucket; false (and the error word set)
// only for a corrupt layout (defensive) -- nothing is then written out of range
__device__ __forceinline__ bool path_of(const LayoutPair& LP, const LayoutView& V, uint32_t s, uint32_t& head, uint32_t& b) {
    const uint32_t h = V.hk[s];
    head = (h >> 5) - 1u;
    const uint32_t ld = h & 31u;
    if (head > s) {
        __hip_atomic_fetch_or(LP.scan.err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return false;
    }
    b = 2u * ld + (s - head + 1u >= SM_LONG_PATH ? 0u : 1u);
    return true;
}
#define PATH_BLOCK 1024
#define PATH_ITEMS 8   // slots per thread -> 8192 per block (few global atomics per round bin)

__global__ __launch_bounds__(PATH_BLOCK) void k_path_emit(LayoutPair LP, int N) {
    if (*LP.mst_ok == 0) return;  // the MST is still a forest: nothing to lay out yet (stage_layout redoes it)
    const LayoutView& V = LP.v[blockIdx.y];
    __shared__ uint32_t hist[SM_NBUCKETS], gbase[SM_NBUCKETS], begin[SM_NBUCKETS + 1];
    if (threadIdx.x < SM_NBUCKETS) hist[threadIdx.x] = 0;
    static_assert(SM_NBUCKETS <= 64, "one wave scans the bucket counts");
    // every block derives the bucket offsets from the final counts (round 5: no k_path_offsets launch);
    // block 0 publishes them and the round count
    if (threadIdx.x < 64) {
        const int b = (int)threadIdx.x;
        const uint32_t c = b < SM_NBUCKETS ? V.round_count[b] : 0u;
        uint32_t x = c;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(x, off);
            if (b >= off) x += y;
        }
        if (b < SM_NBUCKETS) begin[b] = x - c;
        if (b == SM_NBUCKETS - 1) begin[SM_NBUCKETS] = x;
        const uint64_t nz = __ballot(c != 0u);
        if (blockIdx.x == 0) {
            if (b < SM_NBUCKETS) V.round_begin[b] = x - c;
            if (b == SM_NBUCKETS - 1) V.round_begin[SM_NBUCKETS] = x;
            if (b == 0) *V.nrounds = nz ? (uint32_t)(63 - __builtin_clzll(nz)) / 2u + 1u : 0u;
        }
    }
    __syncthreads();
    const uint32_t base = blockIdx.x * PATH_BLOCK * PATH_ITEMS;
    uint32_t myr[PATH_ITEMS], myrank[PATH_ITEMS], myhead[PATH_ITEMS];
    for (int i = 0; i < PATH_ITEMS; ++i) {
        const uint32_t s = base + i * PATH_BLOCK + threadIdx.x;
        myr[i] = SM_NONE;
        if (s >= (uint32_t)N) continue;
        uint32_t head, b;
        if (!path_last(V, s, N) || !path_of(LP, V, s, head, b)) continue;
        myhead[i] = head;
        myr[i] = b;
        myrank[i] = atomicAdd(&hist[myr[i]], 1u);
    }
    __syncthreads();
    if (threadIdx.x < SM_NBUCKETS && hist[threadIdx.x])
        gbase[threadIdx.x] = begin[threadIdx.x] + atomicAdd(&V.round_cursor[threadIdx.x], hist[threadIdx.x]);
    __syncthreads();
    for (int i = 0; i < PATH_ITEMS; ++i) {
        if (myr[i] == SM_NONE) continue;
        const uint32_t s = base + i * PATH_BLOCK + threadIdx.x;
        const uint32_t P = gbase[myr[i]] + myrank[i];
        const uint32_t len = s - myhead[i] + 1u;
        V.paths[P] = SmPath{myhead[i], len};  // head in preorder numbering until k_newslot
        V.pathpos[myhead[i]] = P;
        V.plen[P] = len;
    }
}

// Slots, in preorder order (coalesced): the paths of one (light depth, long/short) bucket occupy a
// contiguous slot range, each path contiguous from its head, in paths[] order; plen holds the inclusive
// scan of the lengths, i.e. the end slot of a path.  slotpix is the pass's one (random) store (round 5: the
// inverse slot2pix, which no pass read, is gone).
__global__ void k_newslot(LayoutPair LP, int N) {
    if (*LP.mst_ok == 0) return;  // the MST is still a forest: nothing to lay out yet (stage_layout redoes it)
    const LayoutView& V = LP.v[blockIdx.y];
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= (uint32_t)N) return;
    const uint32_t head = (V.hk[s] >> 5) - 1u;
    // every index below comes from the scans: a corrupt layout (err set) must not write out of range
    // (round 5: a look-back scan that gave up did)
    const uint32_t P = head <= s ? V.pathpos[head] : SM_NONE;
    const uint32_t len = P < (uint32_t)N ? V.paths[P].len : 0u;
    const uint32_t nh = P < (uint32_t)N ? V.plen[P] - len : SM_NONE;
    const uint32_t slot = nh + (s - head);
    const uint32_t pix = V.pixpre[s];
    if (P >= (uint32_t)N || slot >= (uint32_t)N || pix >= (uint32_t)N) {
        __hip_atomic_fetch_or(LP.scan.err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
    }
    V.slotpix[pix] = slot;
    if (s == head) V.paths[P].head = nh;  // (other threads read .len only)
}

// segment table of the long-path buckets: segment i of bucket b -> {path within b, SM_PRE_SEG-node
// segment of that path}, so k_up_pre launches exactly one block per segment; and the chain work
// items of the bucket ("pieces"):
//  * a path of len > plen nodes gives M = ceil(len / plen) balanced pieces {path, j, M, first segment of the
//    path}, listed bottom piece first (the chain launches wait only on lower entries);
//  * the other paths are packed into runs of consecutive paths (one contiguous slot range): a
//    path starts a new run when its bucket slot offset enters a new window of rwin nodes (or
//    after a cut path) -> item {first path, 0, 1, number of paths}.
// One block per view.
__global__ __launch_bounds__(1024) void k_long_segments(LayoutPair LP, uint32_t plen, uint32_t rdiv, uint32_t rcap) {
    if (*LP.mst_ok == 0) return;  // the MST is still a forest: nothing to lay out yet (stage_layout redoes it)
    const LayoutView& V = LP.v[blockIdx.x];
    __shared__ unsigned long long sc[SCAN_BLOCK / 64];  // the block scan's per-wave totals
    __shared__ uint32_t sp[1024];
    __shared__ uint32_t prev_win, prev_cut;
    // the bucket tables and each long bucket's first head, loaded once (a dependent global load
    // per bucket made this single-block kernel latency-bound: 89 us at C2)
    __shared__ uint32_t rb[SM_NBUCKETS + 1], rn[SM_NBUCKETS], hb[SM_NBUCKETS];
    if (threadIdx.x <= SM_NBUCKETS) rb[threadIdx.x] = V.round_begin[threadIdx.x];
    if (threadIdx.x < SM_NBUCKETS) rn[threadIdx.x] = V.round_nodes[threadIdx.x];
    __syncthreads();
    if (threadIdx.x < SM_NBUCKETS)
        hb[threadIdx.x] = rb[threadIdx.x] < rb[threadIdx.x + 1] ? V.paths[rb[threadIdx.x]].head : 0u;
    __syncthreads();
    uint32_t running = 0, prun = 0;
    for (int b = 0; b < SM_NBUCKETS; ++b) {
        if (threadIdx.x == 0) {
            V.seg_begin[b] = running;
            V.piece_begin[b] = prun;
        }
        if (b & 1) continue;  // short buckets have no segments
        const uint32_t p0 = rb[b], p1 = rb[b + 1];
        if (p0 == p1) continue;  // uniform
        const uint32_t sbase = running;  // the bucket's first segment
        const uint32_t ibase = prun;     // and its first work item
        const uint32_t hbase = hb[b];
        const uint32_t pl = sm_bucket_piece_len(rn[b], plen);  // this bucket's piece length
        // run window: ~3 runs per CU over both views (256 CUs), 64 .. plen nodes
        const uint32_t rwin = min(rcap, max(64u, rn[b] / rdiv));
        if (threadIdx.x == 0) {
            prev_win = 0xFFFFFFFFu;
            prev_cut = 1u;
        }
        __syncthreads();
        // chunks of 4096 paths, 4 consecutive paths per thread, one shuffle-based block scan of
        // (segments << 32 | items) per chunk
        for (uint32_t c = p0; c < p1; c += 4 * 1024) {
            const uint32_t pb = c + 4u * threadIdx.x;
            uint32_t len[4], ns[4], np[4], win[4];
            bool cut[4], start[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint32_t p = pb + (uint32_t)i;
                const SmPath path = p < p1 ? V.paths[p] : SmPath{hbase, 0u};
                len[i] = path.len;
                cut[i] = sm_piece_cut(len[i], pl);
                // segments (k_up_pre / k_dn_pre aggregates, the pieces' guesses): cut paths only
                ns[i] = cut[i] ? (len[i] + SM_PRE_SEG - 1) / SM_PRE_SEG : 0u;
                win[i] = (path.head - hbase) / rwin;
            }
            // previous path's window / alone flag (thread 0: the last path of the previous chunk).
            // A path is alone -- never shares a run -- when it is cut or longer than the run window:
            // a long uncut path then is one item, not the tail of a run of up to 2.5 windows
            bool alone[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) alone[i] = cut[i] || len[i] > rwin;
            sp[threadIdx.x] = (win[3] << 1) | (alone[3] ? 1u : 0u);
            __syncthreads();
            uint32_t pv = threadIdx.x ? sp[threadIdx.x - 1] : ((prev_win << 1) | prev_cut);
            uint32_t tns = 0, tnp = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                start[i] = !cut[i] && (alone[i] || (pv & 1u) || (pv >> 1) != win[i]);
                np[i] = pb + (uint32_t)i < p1 ? (cut[i] ? sm_piece_count(len[i], pl) : (start[i] ? 1u : 0u)) : 0u;
                pv = (win[i] << 1) | (alone[i] ? 1u : 0u);
                tns += ns[i];
                tnp += np[i];
            }
            unsigned long long tot;
            const unsigned long long ex = block_exclusive_scan<unsigned long long, OpAdd>(
                ((unsigned long long)tns << 32) | tnp, sc, &tot);
            if (threadIdx.x == 1023) {
                prev_win = win[3];
                prev_cut = alone[3] ? 1u : 0u;
            }
            uint32_t seg = running + (uint32_t)(ex >> 32), item = prun + (uint32_t)ex;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint32_t p = pb + (uint32_t)i;
                if (p >= p1) break;
                for (uint32_t q = 0; q < ns[i]; ++q) V.segtab[seg + q] = make_uint2(p - p0, q);
                if (cut[i]) {
                    for (uint32_t j = 0; j < np[i]; ++j) V.pieces[item + j] = make_uint4(p - p0, np[i] - 1u - j, np[i], seg - sbase);
                } else if (start[i]) {
                    V.pieces[item] = make_uint4(p - p0, 0u, 1u, 0u);
                }
                seg += ns[i];
                item += np[i];
            }
            running += (uint32_t)(tot >> 32);
            prun += (uint32_t)tot;
            __syncthreads();
            // count the paths of each run: every uncut path adds itself to the run it belongs to
            // (the latest item, which is a run start since this path is not cut)
            item = prun - (uint32_t)tot + (uint32_t)ex;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                item += np[i];
                if (pb + (uint32_t)i < p1 && !cut[i]) atomicAdd(reinterpret_cast<uint32_t*>(V.pieces + (item - 1u)) + 3, 1u);
            }
            __syncthreads();
        }
        // Longest first: a chain launch runs one workgroup per CU and the CUs take items in index
        // order, so a long item that starts late sets the round's end.  Items are regrouped as
        // [pieces of cut paths, in their order (the look-back needs a path's pieces contiguous,
        // bottom first) | runs longer than the run window | the other runs], each group stable.
        {
            const uint32_t ib = ibase, ie = prun;
            auto klass = [&](uint32_t it) -> uint32_t {
                const uint4 pc = V.pieces[it];
                if (pc.z > 1u) return 0u;
                const SmPath f = V.paths[p0 + pc.x], l = V.paths[p0 + pc.x + pc.w - 1u];
                return (l.head + l.len - f.head) > rwin ? 1u : 2u;
            };
            // pass 1: class totals; pass 2: stable scatter into the scratch; then copy back
            unsigned long long tall = 0;
            for (uint32_t c = ib; c < ie; c += 1024) {
                const uint32_t it = c + threadIdx.x;
                const unsigned long long f = it < ie ? 1ull << (21 * klass(it)) : 0ull;
                unsigned long long t;
                block_exclusive_scan<unsigned long long, OpAdd>(f, sc, &t);
                tall += t;
            }
            const uint32_t n0 = (uint32_t)(tall & 0x1FFFFF), n1 = (uint32_t)((tall >> 21) & 0x1FFFFF);
            unsigned long long run = 0;
            for (uint32_t c = ib; c < ie; c += 1024) {
                const uint32_t it = c + threadIdx.x;
                const uint32_t k = it < ie ? klass(it) : 3u;
                const unsigned long long f = k < 3u ? 1ull << (21 * k) : 0ull;
                unsigned long long t;
                const unsigned long long e = run + block_exclusive_scan<unsigned long long, OpAdd>(f, sc, &t);
                run += t;
                if (k < 3u) {
                    const uint32_t r = (uint32_t)((e >> (21 * k)) & 0x1FFFFF);
                    const uint32_t dst = k == 0u ? r : k == 1u ? n0 + r : n0 + n1 + r;
                    V.pieces_tmp[ib + dst] = V.pieces[it];
                }
            }
            __threadfence_block();
            __syncthreads();
            for (uint32_t it = ib + threadIdx.x; it < ie; it += 1024) V.pieces[it] = V.pieces_tmp[it];
            __threadfence_block();
            __syncthreads();
        }
    }
    if (threadIdx.x == 0) {
        V.seg_begin[SM_NBUCKETS] = running;
        V.piece_begin[SM_NBUCKETS] = prun;
    }
}

// ------------------------------------------------------------------------------------------
static dim3 pix_grid(int W, int H, int nv) { return dim3((W + 255) / 256, H, nv); }

hipError_t launch_layout(hipStream_t st, const LayoutPair& LP, int nviews, int W, int H, uint32_t max_chains,
                         uint32_t piece_len) {
    const int N = W * H;
    const dim3 pg = pix_grid(W, H, nviews);
    hipLaunchKernelGGL(k_adj, pg, dim3(256), 0, st, LP, W, H);
    const dim3 tg(layout_tile_blocks(W, H), 1, nviews);  // XCD-aware 32x32 tiles (layout_tile)
    hipLaunchKernelGGL(k_tour_tile, tg, dim3(TL_THREADS), 0, st, LP, W, H);
    const dim3 cg((max_chains + 255) / 256, nviews);
    hipLaunchKernelGGL(k_chain_init, cg, dim3(256), 0, st, LP, W);
    hipLaunchKernelGGL(k_chain_rank, dim3(std::min<uint32_t>((max_chains + 255) / 256, CR_BLOCKS), nviews), dim3(256), 0, st, LP);
    hipLaunchKernelGGL(k_orient, tg, dim3(256), 0, st, LP, W, H);
    ScanBufs<uint32_t> wb{{LP.v[0].wrow, LP.v[1].wrow}, {nullptr, nullptr}};  // compact A rows per tile wave
    launch_scan<uint32_t, OpAdd>(st, wb, LP.scan, nviews, 4 * ((W + TL - 1) / TL) * ((H + TL - 1) / TL));
    ScanBufs<uint32_t> tb{{LP.v[0].tour, LP.v[1].tour}, {nullptr, nullptr}};
    launch_scan<uint32_t, OpAdd>(st, tb, LP.scan, nviews, 2 * N - 2, ScanTourOut{LP, N});
    const dim3 sg((N + PATH_BLOCK * PATH_ITEMS - 1) / (PATH_BLOCK * PATH_ITEMS), nviews);
    ScanBufs<uint32_t> hb{{LP.v[0].hk, LP.v[1].hk}, {nullptr, nullptr}};
    launch_scan<uint32_t, OpMax>(st, hb, LP.scan, nviews, N, ScanPathCount{LP});
    hipLaunchKernelGGL(k_path_emit, sg, dim3(PATH_BLOCK), 0, st, LP, N);
    // contiguous bucket slots: scan of path lengths in paths[] order (plen past the last path is not read
    // path), slot of every preorder position, then the metadata in slot numbering
    // (only the paths' lengths: the path count, round_begin[SM_NBUCKETS], is read on the device)
    ScanBufs<uint32_t> lb{{LP.v[0].plen, LP.v[1].plen}, {LP.v[0].round_begin + SM_NBUCKETS, LP.v[1].round_begin + SM_NBUCKETS}};
    launch_scan<uint32_t, OpAdd>(st, lb, LP.scan, nviews, N);
    hipLaunchKernelGGL(k_newslot, dim3((N + 255) / 256, nviews), dim3(256), 0, st, LP, N);
    hipLaunchKernelGGL(k_meta, dim3(META_BLOCKS, nviews), dim3(256), 0, st, LP, W, H);
    // run sizing (A/B knobs: SM_RUN_DIV, SM_RUN_CAP = the window cap in nodes)
    const char* ed = sm_dev_knob("SM_RUN_DIV");
    const char* ec = sm_dev_knob("SM_RUN_CAP");
    const uint32_t rdiv = ed && atoi(ed) > 0 ? (uint32_t)atoi(ed) : (uint32_t)SM_RUN_DIV;
    const uint32_t rcap = ec && atoi(ec) >= 64 ? (uint32_t)atoi(ec) : piece_len;
    hipLaunchKernelGGL(k_long_segments, dim3(nviews), dim3(1024), 0, st, LP, piece_len, rdiv, rcap);
    return hipGetLastError();
}
