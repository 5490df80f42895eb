// sm_pms_forest.hip -- the MST_PMS schedule forest on the GPU (round 4).  The host construction
// (pms_build_forest, sm_pms_host.cpp) walks each tree sequentially; at C2 the largest tree (618k nodes)
// alone took ~90 ms of it.  Here, for one view:
//   pf_trees : union-find over the forest's real edges with the smaller root always the parent, so a
//              tree's root is its first pixel in raster order; a scan of the root flags numbers the
//              trees as the reference does (Stereo3DMST.cpp:342-384), a scan of their sizes places them
//   pf_bfs   : one workgroup runs the BFS of every tree at once, level by level (children of a node in
//              ascending (w, a, b) key order, Stereo3DMST.cpp:450-522); within a level the nodes are
//              ordered by tree and, per tree, in its BFS order, so a stable sort of the level order by
//              tree gives every tree's BFS numbering.  The same workgroup then sweeps the levels bottom
//              up for subtree sizes and heavy children (the largest subtree, ties: the smallest BFS id);
//              pointer jumping gives each node its heavy path's head and its offset on it, Jacobi
//              iterations over the heads the light depths
//   pf_lists : heads sorted by (tree, light depth, BFS id) place the rows (each path head first on
//              consecutive rows); the tree graph from the grid's inter-tree edges (sorted, unique);
//              heads sorted by (light depth, tree, BFS id) count the round-major paths, items, repair
//              items and chain items
//   pf_fill  : the lists themselves and the per-(round, tree) tables as prefix sums of counts.
// Every array equals the host construction's (tests/test_pms_gpu.py, SM_PMS_FOREST_CHECK).
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdlib>

#include <hipcub/device/device_radix_sort.hpp>
#include <hipcub/device/device_scan.hpp>

#include "sm_pms_forest.h"
#include "sm_segment.h"
#include "sm_tour.h"
#include "sm_knob.h"

#define SM_VIRTUAL_W_PF SM_VIRTUAL_W

namespace {

inline unsigned nblk(size_t n, unsigned b) { return (unsigned)((n + b - 1) / b); }

__device__ __forceinline__ unsigned long long pf_ekey(uint32_t w, uint32_t a, uint32_t vert) {
    return ((unsigned long long)w << 33) | ((unsigned long long)a << 1) | vert;
}

// real forest edges of pixel p (the segment forest's virtual links excluded): bit 0 (p, p+1), bit 1 (p, p+W)
__device__ __forceinline__ uint32_t pf_real(const PfView& v, int p) {
    uint32_t r = 0;
    if (v.mR[p] && v.fwR[p] != SM_VIRTUAL_W_PF) r |= 1u;
    if (v.mD[p] && v.fwD[p] != SM_VIRTUAL_W_PF) r |= 2u;
    return r;
}

// neighbour lists in key order; union-find init
__global__ void k_pf_prep(PfView v) {
    const int p = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (p >= v.N) return;
    const int W = v.W, x = p % W;
    unsigned long long key[4];
    int nb[4], w[4], k = 0;
    const uint32_t rp = pf_real(v, p);
    if (rp & 1u) { key[k] = pf_ekey(v.wR[p], (uint32_t)p, 0); nb[k] = p + 1; w[k++] = v.wR[p]; }
    if (rp & 2u) { key[k] = pf_ekey(v.wD[p], (uint32_t)p, 1); nb[k] = p + W; w[k++] = v.wD[p]; }
    if (x > 0 && (pf_real(v, p - 1) & 1u)) { key[k] = pf_ekey(v.wR[p - 1], (uint32_t)(p - 1), 0); nb[k] = p - 1; w[k++] = v.wR[p - 1]; }
    if (p >= W && (pf_real(v, p - W) & 2u)) { key[k] = pf_ekey(v.wD[p - W], (uint32_t)(p - W), 1); nb[k] = p - W; w[k++] = v.wD[p - W]; }
    for (int i = 1; i < k; ++i)
        for (int j = i; j > 0 && key[j] < key[j - 1]; --j) {
            const unsigned long long tk = key[j]; key[j] = key[j - 1]; key[j - 1] = tk;
            const int tn = nb[j]; nb[j] = nb[j - 1]; nb[j - 1] = tn;
            const int tw = w[j]; w[j] = w[j - 1]; w[j - 1] = tw;
        }
    for (int i = k; i < 4; ++i) { nb[i] = -1; w[i] = 0; }
    v.nbr[p] = make_int4(nb[0], nb[1], nb[2], nb[3]);
    v.nbw[p] = make_uint2((uint32_t)w[0] | ((uint32_t)w[1] << 16), (uint32_t)w[2] | ((uint32_t)w[3] << 16));
    v.par[p] = p;
}

__device__ __forceinline__ int uf_find(const int32_t* par, int x) {
    int p = par[x];
    while (p != x) {
        x = p;
        p = par[x];
    }
    return x;
}

// the same with path halving (k_pf_link: the largest tree's chains are long; every value written is an
// ancestor, so concurrent halving and linking stay valid)
__device__ __forceinline__ int uf_find_halve(int32_t* par, int x) {
    for (;;) {
        const int p = par[x];
        if (p == x) return x;
        const int g = par[p];
        if (g != p) par[x] = g;
        x = g;
    }
}

// wave-aggregated atomicAdd of `add` to cnt[key] over the lanes with `valid` (lanes sharing a key --
// consecutive pixels of one tree, heads of one (round, tree) -- make one atomic)
__device__ __forceinline__ void wave_add_by_key(int32_t* cnt, long long key, int add, bool valid) {
    unsigned long long act = __ballot(valid);
    const int lane = __lane_id();
    while (act) {
        const int leader = __ffsll((long long)act) - 1;
        const long long kl = __shfl(key, leader);
        const unsigned long long m = __ballot(valid && key == kl) & act;
        int sum = ((m >> lane) & 1ull) ? add : 0;  // the group's sum: a full wave reduction, others zero
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) sum += __shfl_xor(sum, o);
        if (lane == leader && sum) atomicAdd(cnt + kl, sum);
        act &= ~m;
    }
}

// link the larger root under the smaller one (the root of a tree ends as its smallest pixel)
__device__ void uf_union(int32_t* par, int a, int b) {
    for (;;) {
        a = uf_find_halve(par, a);
        b = uf_find_halve(par, b);
        if (a == b) return;
        if (a < b) {
            const int t = a;
            a = b;
            b = t;
        }
        const int old = atomicCAS(&par[a], a, b);
        if (old == a) return;
        a = old;  // a was linked meanwhile (to a smaller root): continue from there, never from a stale read
    }
}

__global__ void k_pf_link(PfView v) {
    const int p = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (p >= v.N) return;
    const uint32_t r = pf_real(v, p);
    if (r & 1u) uf_union(v.par, p, p + 1);
    if (r & 2u) uf_union(v.par, p, p + v.W);
}

__global__ void k_pf_compress(PfView v) {
    const int p = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (p > v.N) return;
    if (p == v.N) {
        v.flag[p] = 0;
        return;
    }
    const int r = uf_find(v.par, p);
    v.par[p] = r;
    v.flag[p] = r == p ? 1 : 0;
}

// tid (the flags' exclusive scan, in gpix) -> tree of every pixel, root pixels, sizes
__global__ void k_pf_trees(PfView v) {
    const int p = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    const bool valid = p < v.N;
    int t = 0;
    if (valid) {
        const int r = v.par[p];
        t = v.gpix[r];
        v.tree_of[p] = t;
        if (r == p) v.root_pix[t] = p;
    }
    wave_add_by_key(v.tsize, t, 1, valid);  // one atomic per tree in the wave (not 618k on one counter)
}

// ---------------------------------------------------------------------------------------- BFS
// Every tree's BFS numbering (Stereo3DMST.cpp:450-522: root first, then level by level, a node's
// children in ascending (w, a, b) key order after the children of the nodes before it) in O(log) depth,
// from two Euler tours per tree (sm_tour.h list ranking; round 5, replacing a level-synchronous BFS in
// one workgroup that took ~2.5 us per level: 26 ms for the 8.6k-level tree at C2):
//   tour 1 : the successor leaves a node through its next neighbour in cyclic key order; ranked per
//            tree, an arc p->q precedes its reverse iff p is q's parent (orientation), and the distance
//            between the two is twice q's subtree size
//   tour 2 : children in key order, then back to the parent: a depth-first order whose preorder, among
//            the nodes of one depth, is the lexicographic order of their root paths' key ranks -- i.e.
//            the BFS order.  An int64 prefix sum over the tours (+1 | +1 down, -1 | 0 up) gives every
//            node's depth and preorder, and a stable radix sort of the preorder sequence by (tree, depth)
//            is the BFS numbering of every tree at once.
// Rotation words (rot): bits 0..3 the node's real tree edges by direction; nibble 1 + j: the direction
// the tour leaves by after arriving from direction j (PF_END: the end of the tree's list).
#define PF_END 4u

struct PfTourG {
    const uint32_t* rot;
    int W;
    __device__ bool has(uint32_t p, int k) const { return (rot[p] >> k) & 1u; }
    __device__ uint32_t succ(uint32_t a) const {
        const uint32_t q = tour_nbr(a >> 2, (int)(a & 3u), W);
        const uint32_t nd = (rot[q] >> (4 + 4 * (((a & 3u) + 2u) & 3u))) & 0xFu;
        return nd == PF_END ? SM_NONE : 4u * q + nd;
    }
};

__device__ __forceinline__ TourBufs pf_tour_bufs(const PfView& v) {
    return TourBufs{v.a_dist, v.a_cid, v.nchains, v.c_last, v.c_len, v.cnw, v.tot + 7, 4};  // (4: an inconsistent tour)
}

// direction from p to its grid neighbour n
__device__ __forceinline__ int pf_dir(int p, int n, int W) { return n == p + 1 ? 0 : n == p + W ? 1 : n == p - 1 ? 2 : 3; }

// the real tree neighbours' directions in key order (nbr, k_pf_prep); returns their count
__device__ __forceinline__ int pf_dirs(const PfView& v, int p, int (&d)[4]) {
    const int4 n4 = v.nbr[p];
    const int nn[4] = {n4.x, n4.y, n4.z, n4.w};
    int c = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        d[i] = nn[i] >= 0 ? pf_dir(p, nn[i], v.W) : 0;
        c += nn[i] >= 0 ? 1 : 0;
    }
    return c;
}

// tour 1's rotation: cyclic key order; a tree's list starts at root -> its first neighbour, so the root
// ends it after its last one
__global__ void k_pf_rot1(PfView v) {
    const int p = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (p >= v.N) return;
    int d[4];
    const int c = pf_dirs(v, p, d);
    const bool root = v.par[p] == p;
    uint32_t r = 0;
    for (int i = 0; i < c; ++i) {
        r |= 1u << d[i];
        const uint32_t nx = (root && i == c - 1) ? PF_END : (uint32_t)d[(i + 1) % c];
        r |= nx << (4 + 4 * d[i]);
    }
    v.rot[p] = r;
}

// tour 2's rotation from tour 1's orientation: arriving from the parent, the first child in key order;
// from a child, the next child, then the parent (the root: the end of the list)
__global__ void k_pf_rot2(PfView v) {
    const int p = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (p >= v.N) return;
    int d[4];
    const int c = pf_dirs(v, p, d);
    const int pd = v.pdir[p];
    uint32_t r = 0;
    int prev = pd;  // the direction whose successor is set next (the parent's arrival first)
    for (int i = 0; i < c; ++i) {
        r |= 1u << d[i];
        if (d[i] == pd) continue;
        if (prev >= 0) r |= (uint32_t)d[i] << (4 + 4 * prev);
        prev = d[i];
    }
    if (prev >= 0) r |= (pd >= 0 ? (uint32_t)pd : PF_END) << (4 + 4 * prev);  // a leaf: straight back up
    v.rot[p] = r;
}

__global__ void k_pf_tour_tile(PfView v) {
    tour_tile(PfTourG{v.rot, v.W}, pf_tour_bufs(v), v.W, v.H, (int)blockIdx.x * TL, (int)blockIdx.y * TL);
}

__global__ void k_pf_chain_init(PfView v) {
    tour_chain_init(PfTourG{v.rot, v.W}, pf_tour_bufs(v), blockIdx.x * blockDim.x + threadIdx.x);
}

constexpr int PF_CR_BLOCKS = 512;  // per view (the two views' forests build concurrently)
__global__ __launch_bounds__(256) void k_pf_chain_rank(PfView v) { tour_chain_rank(pf_tour_bufs(v)); }

// tour 1: orientation (pdir: direction to the parent, -1 at a root) and subtree sizes.  Arc ranks per
// tree are its list length minus the suffix, so rank(p->q) < rank(q->p) iff suffix(p->q) > suffix(q->p)
__global__ void k_pf_orient(PfView v) {
    const int q = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (q >= v.N) return;
    const uint32_t adj = v.rot[q] & 0xFu;
    int pd = -1;
    int sz = v.tsize[v.tree_of[q]];  // a root: its tree
    const TourBufs T = pf_tour_bufs(v);
    for (int k = 0; k < 4; ++k) {
        if (!((adj >> k) & 1u)) continue;
        const uint32_t p = tour_nbr((uint32_t)q, k, v.W);
        const uint32_t si = tour_suffix(T, 4u * p + (uint32_t)((k + 2) & 3)), so = tour_suffix(T, 4u * (uint32_t)q + (uint32_t)k);
        if (si > so) {
            pd = k;
            sz = (int)((si - so + 1u) / 2u);
        }
    }
    v.pdir[q] = (int8_t)pd;
    v.psize[q] = sz;
}

// tour 2: the arcs' +-1 values at their positions in the concatenation of the trees' lists (tree t's
// 2(|t| - 1) arcs start at 2(tree_start[t] - t)): down (1 << 32 | 1), up -(1 << 32)
__global__ void k_pf_tourval(PfView v) {
    const int p = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (p >= v.N) return;
    const uint32_t adj = v.rot[p] & 0xFu;
    if (!adj) return;
    const int t = v.tree_of[p];
    const uint32_t len = 2u * (uint32_t)(v.tsize[t] - 1);
    const uint32_t base = 2u * (uint32_t)(v.tree_start[t] - t);
    const TourBufs T = pf_tour_bufs(v);
    for (int k = 0; k < 4; ++k) {
        if (!((adj >> k) & 1u)) continue;
        const uint32_t a = 4u * (uint32_t)p + (uint32_t)k;
        const uint32_t q = tour_nbr((uint32_t)p, k, v.W);
        const bool down = v.pdir[q] == ((k + 2) & 3);
        const uint32_t rank = len - tour_suffix(T, a);
        v.tval[base + rank] = down ? (long long)((1ull << 32) | 1ull) : -(long long)(1ull << 32);
    }
}

// depth and preorder of every node from the scanned values at its down arc; the sort input: key
// (tree, depth) at the node's global preorder position (trees in order), value the pixel
__global__ void k_pf_depth(PfView v, int dbits) {
    const int q = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (q >= v.N) return;
    const int t = v.tree_of[q], pd = v.pdir[q];
    long long depth = 0, pre = 0;
    if (pd >= 0) {
        const uint32_t p = tour_nbr((uint32_t)q, pd, v.W);
        const uint32_t a = 4u * p + (uint32_t)((pd + 2) & 3);
        const uint32_t len = 2u * (uint32_t)(v.tsize[t] - 1);
        const uint32_t pos = 2u * (uint32_t)(v.tree_start[t] - t) + len - tour_suffix(pf_tour_bufs(v), a);
        const long long s = v.tval_s[pos];
        depth = s >> 32;
        pre = (s & 0xFFFFFFFFll) - (long long)(v.tree_start[t] - t);
    }
    const int g = v.tree_start[t] + (int)pre;
    if (g < v.tree_start[t] || g >= v.tree_start[t + 1] || depth < 0 || depth >= (1ll << dbits)) {
        v.tot[7] = 4;  // an inconsistent tour: flag it, never write out of range
        return;
    }
    v.tkey[0][g] = ((unsigned long long)t << dbits) | (unsigned long long)depth;
    v.tpix[0][g] = q;
}

// BFS position of every pixel, tree of every BFS node
__global__ void k_pf_bpos(PfView v) {
    const int n = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (n >= v.N) return;
    const int q = v.gpix[n];
    v.bpos[q] = n;
    v.gtree[n] = v.tree_of[q];
}

// the BFS-numbered node fields the rest of the build reads (as the level-order arrays of the round-4
// BFS, whose level order is now the BFS order itself): parent, edge weight to it, children (consecutive
// in BFS order, key order), subtree size, heavy child (the largest subtree, ties: the smallest BFS id)
__global__ void k_pf_fields(PfView v) {
    const int n = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (n >= v.N) return;
    const int q = v.gpix[n], pd = v.pdir[q];
    const int4 n4 = v.nbr[q];
    const uint2 w4 = v.nbw[q];
    const int nn[4] = {n4.x, n4.y, n4.z, n4.w};
    const uint32_t ww[4] = {w4.x & 0xFFFFu, w4.x >> 16, w4.y & 0xFFFFu, w4.y >> 16};
    const int par = pd >= 0 ? (int)tour_nbr((uint32_t)q, pd, v.W) : -1;
    int nc = 0, fc = -1, best = -1, bs = 0;
    for (int i = 0; i < 4; ++i) {
        if (nn[i] < 0 || nn[i] == par) continue;
        if (nc == 0) fc = v.bpos[nn[i]];
        const int sk = v.psize[nn[i]];
        if (sk > bs) {
            bs = sk;
            best = nc;
        }
        ++nc;
    }
    uint32_t w = 0;  // the weight code of the edge to the parent
    for (int i = 0; i < 4; ++i)
        if (par >= 0 && nn[i] == par) w = ww[i];
    v.gpar[n] = par >= 0 ? v.bpos[par] : -1;
    v.gw[n] = (uint16_t)w;
    v.gnc[n] = (uint8_t)nc;
    v.gfc[n] = nc ? fc : n;
    v.gsize[n] = v.psize[q];
    v.ghk[n] = (int8_t)best;
}

// test hook (SM_TEST_PMS_CYCLE=1, tests/test_pms_gpu.py): the square of pixels 0, 1, W, W + 1 becomes four
// real edges -- a cycle, which the build must refuse (k_pf_edges) rather than tour
__global__ void k_pf_test_cycle(PfView v) {
    if (threadIdx.x != 0 || v.W < 2 || v.H < 2) return;
    uint8_t* mR = const_cast<uint8_t*>(v.mR);
    uint8_t* mD = const_cast<uint8_t*>(v.mD);
    uint16_t* fwR = const_cast<uint16_t*>(v.fwR);
    uint16_t* fwD = const_cast<uint16_t*>(v.fwD);
    mR[0] = mD[0] = mR[v.W] = mD[1] = 1;
    fwR[0] = v.wR[0];
    fwD[0] = v.wD[0];
    fwR[v.W] = v.wR[v.W];
    fwD[1] = v.wD[1];
}

// real tree edges of the view (a forest of N nodes in K trees has exactly N - K)
__global__ void k_pf_edges(PfView v) {
    const int p = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    int c = p < v.N ? __popc(pf_real(v, p)) : 0;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) c += __shfl_xor(c, o);
    if (__lane_id() == 0 && c) atomicAdd(v.tot + 8, c);
}

__global__ void k_pf_iota(int32_t* a, int n) {
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i < n) a[i] = i;
}

__global__ void k_pf_fill1(int32_t* a, int n) {
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i < n) a[i] = 1;
}

__global__ void k_pf_g2b(PfView v) {
    const int n = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (n < v.N) v.g2b[v.bglob[n]] = n;
}

// wave-aggregated atomicMax of `val` into cnt[key] (as wave_add_by_key)
__device__ __forceinline__ void wave_max_by_key(int32_t* cnt, int key, int val, bool valid) {
    unsigned long long act = __ballot(valid);
    const int lane = __lane_id();
    while (act) {
        const int leader = __ffsll((long long)act) - 1;
        const int kl = __shfl(key, leader);
        const unsigned long long m = __ballot(valid && key == kl) & act;
        int mx = ((m >> lane) & 1ull) ? val : INT_MIN;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) mx = max(mx, __shfl_xor(mx, o));
        if (lane == leader) atomicMax(cnt + kl, mx);
        act &= ~m;
    }
}

// BFS-numbered node fields; the heavy path's up-link for the pointer jumping
__global__ void k_pf_nodes(PfView v) {
    const int n = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (n >= v.N) return;
    const int i = v.bglob[n], gp = v.gpar[i];
    v.bfs_pix[n] = v.gpix[i];
    v.bpar[n] = gp >= 0 ? v.g2b[gp] : n;
    v.bch0[n] = v.gnc[i] ? v.g2b[v.gfc[i]] : -1;
    const bool heavy = gp >= 0 && v.ghk[gp] >= 0 && v.gfc[gp] + v.ghk[gp] == i;
    v.J[0][n] = heavy ? v.g2b[gp] : n;
    v.Dj[0][n] = heavy ? 1 : 0;
}

__global__ void k_pf_jump(const int32_t* J0, const int32_t* D0, int32_t* J1, int32_t* D1, int N) {
    const int n = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (n >= N) return;
    const int j = J0[n];
    J1[n] = J0[j];
    D1[n] = D0[n] + D0[j];
}

// path lengths at the heads (a path ends at a leaf); light depth 0 at tree roots, unknown (-1) at the
// other heads; head flags
__global__ void k_pf_heads(PfView v, const int32_t* J, const int32_t* D) {
    const int n = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (n > v.N) return;
    if (n == v.N) {
        v.hflag[n] = 0;
        return;
    }
    if (v.bch0[n] < 0) v.plen[J[n]] = D[n] + 1;
    const bool head = J[n] == n;
    v.hflag[n] = head ? 1 : 0;
    v.ld[n] = head ? (v.bpar[n] == n ? 0 : -1) : -2;
}

// one Jacobi step of ld(head) = ld(head of its parent's path) + 1 (values only ever go from -1 to final)
__global__ void k_pf_ld_step(PfView v, const int32_t* J) {
    const int n = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (n >= v.N || v.ld[n] != -1) return;
    const int hp = J[v.bpar[n]];
    const int l = __hip_atomic_load(&v.ld[hp], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (l >= 0) __hip_atomic_store(&v.ld[n], l + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// every node's light depth, the trees' round counts, the view's, and the heads' sort keys
__global__ void k_pf_ld_all(PfView v, const int32_t* J) {
    const int n = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    bool head = false;
    int t = 0, l = 0;
    if (n < v.N && J[n] == n) {
        t = v.gtree_s[n];
        l = v.ld[n];
        head = true;
        if (l < 0 || l > 255) {  // unresolved light depth: an inconsistent schedule, flag it (never key on it)
            v.tot[7] = 2;
            head = false;
        }
    }
    // one atomic per tree and wave, one per wave for the view's rounds (a tree's heads are contiguous)
    wave_max_by_key(v.tree_rounds, t, l + 1, head);
    wave_max_by_key(v.tot, 5, l + 1, head);
}

// head keys: A = (tree, light depth, BFS id within the tree): the rows' order; B = (light depth,
// tree, BFS id): the round-major lists' order
__global__ void k_pf_hkeys(PfView v, int which) {
    const int n = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (n >= v.N || !v.hflag[n]) return;
    const unsigned long long t = (unsigned long long)v.gtree_s[n], l = (unsigned long long)v.ld[n];
    const unsigned long long loc = (unsigned long long)(n - v.tree_start[t]);
    v.hkey[0][v.hidx[n]] = which == 0 ? (t << 40) | (l << 32) | loc : (l << 56) | (t << 32) | loc;
}

__device__ __forceinline__ int head_of_a(const PfView& v, unsigned long long k) {
    const int t = (int)(k >> 40);
    return v.tree_start[t] + (int)(k & 0xFFFFFFFFull);
}

// A order: path lengths (the rows' scan input) and cut flags (the cuts' scan input)
__global__ void k_pf_rows_in(PfView v, int nh) {
    const int j = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (j > nh) return;
    if (j == nh) {
        v.hcnt[0][j] = 0;
        v.hcnt[1][j] = 0;
        return;
    }
    const int len = v.plen[head_of_a(v, v.hkey[1][j])];
    v.hcnt[0][j] = len;
    v.hcnt[1][j] = v.piece > 0 && len >= 2 * v.piece ? 1 : 0;
}

// rows of the heads, the cuts (tree order), cut counts per tree
__global__ void k_pf_rows_out(PfView v, int nh) {
    const int j = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (j >= nh) return;
    const unsigned long long k = v.hkey[1][j];
    const int t = (int)(k >> 40), h = head_of_a(v, k);
    const int row = v.hoff[0][j];
    v.rowstart[h] = row;
    if (v.hcnt[1][j]) {
        const int c = v.hoff[1][j], len = v.plen[h];
        v.cutof[h] = c;
        v.cuts[c] = PmsCut{t, row, len, len / v.piece};
        v.cut_round[c] = (int)((k >> 32) & 0xFFu);
        atomicAdd(&v.nbcnt[t], 1);  // (nbcnt: the cuts per tree here; zeroed again for the tree graph)
    } else {
        v.cutof[h] = -1;
    }
}

__global__ void k_pf_rowof(PfView v) {
    const int n = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (n < v.N) v.rowof[n] = v.rowstart[v.J[0][n]] + v.Dj[0][n];
}

// the PmsRow of every node at its row (sm_pms_host.cpp's fill, children in descending BFS id)
__global__ void k_pf_rows(PfView v) {
    const int n = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (n >= v.N) return;
    const int row = v.rowof[n];
    if (row < 0 || row >= v.N) {  // guard: an inconsistent schedule is flagged, never written out of bounds
        v.tot[7] = 3;
        return;
    }
    const int i = v.bglob[n];
    const int p = v.gpix[i];
    PmsRow R;
    R.pix = p;
    R.x = (uint16_t)(p % v.W);
    R.y = (uint16_t)(p / v.W);
    R.parent = v.bpar[n] == n ? -1 : v.rowof[v.bpar[n]];
    R.w = v.gw[i];
    const int nch = v.gnc[i], c0 = v.bch0[n], hk = v.ghk[i];
    R.nch = (uint8_t)nch;
    R.hk = 0xFF;
    for (int q = 0; q < 4; ++q) {
        R.child[q] = -1;
        R.wch[q] = 0;
    }
    for (int q = 0; q < nch; ++q) {
        const int ci = nch - 1 - q;  // descending BFS id: the up pass's fold order (:125)
        R.child[q] = v.rowof[c0 + ci];
        R.wch[q] = v.gw[v.gfc[i] + ci];
        if (ci == hk) R.hk = (uint8_t)q;
    }
    v.rows[row] = R;
    v.rtree[row] = v.gtree_s[n];
}

// the grid's inter-tree edges as (tree, tree) pairs, both directions (tree_g, :377-384)
__global__ void k_pf_pairs(PfView v) {
    const int p = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    const int W = v.W, x = p % W, a = p < v.N ? v.tree_of[p] : 0;
    unsigned long long out[4];
    int c = 0;
    if (p < v.N && x + 1 < W) {
        const int b = v.tree_of[p + 1];
        if (a != b) {
            out[c++] = ((unsigned long long)a << 32) | (uint32_t)b;
            out[c++] = ((unsigned long long)b << 32) | (uint32_t)a;
        }
    }
    if (p < v.N && p + W < v.N) {
        const int b = v.tree_of[p + W];
        if (a != b) {
            out[c++] = ((unsigned long long)a << 32) | (uint32_t)b;
            out[c++] = ((unsigned long long)b << 32) | (uint32_t)a;
        }
    }
    // one append per wave: an exclusive wave scan of the lanes' pair counts
    const int lane = __lane_id();
    int incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
    }
    const int total = __shfl(incl, 63);
    int base = 0;
    if (lane == 63 && total) base = atomicAdd(v.npairs, total);
    base = __shfl(base, 63);
    const int pos = base + incl - c;
    for (int k = 0; k < c; ++k) v.pairs[0][pos + k] = out[k];
}

__global__ void k_pf_uniq_flag(PfView v, int np) {
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i > np) return;
    v.uflag[i] = i < np && (i == 0 || v.pairs[1][i] != v.pairs[1][i - 1]) ? 1 : 0;
}

__global__ void k_pf_uniq_emit(PfView v, int np) {
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= np || !v.uflag[i]) return;
    const unsigned long long k = v.pairs[1][i];
    v.nb[v.uidx[i]] = (int32_t)(k & 0xFFFFFFFFull);
    atomicAdd(&v.nbcnt[(int)(k >> 32)], 1);
}

__device__ __forceinline__ void head_of_b(const PfView& v, unsigned long long k, int& r, int& t, int& h) {
    r = (int)(k >> 56);
    t = (int)((k >> 32) & 0xFFFFFFu);
    h = v.tree_start[t] + (int)(k & 0xFFFFFFFFull);
}

// B order: per head its pieces, prop items, repair items and chain items (sm_pms_host.cpp's counts), and
// the per-(round, tree) counts of the four tables
__device__ long long pf_count_head(const PfView& v, int j, int K, int* cout);

__global__ void k_pf_counts(PfView v, int nh, int K) {
    const int j = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (j == nh)
        for (int q = 0; q < 4; ++q) v.hcnt[q][j] = 0;
    const bool valid = j < nh;
    int c[4] = {0, 0, 0, 0};
    long long k = 0;
    if (valid) k = pf_count_head(v, j, K, c);
    // heads are in (round, tree) order: one atomic per (round, tree) and wave
    for (int q = 0; q < 4; ++q) wave_add_by_key(v.rtc[q], k, c[q], valid && c[q] != 0);
}

__device__ long long pf_count_head(const PfView& v, int j, int K, int* cout) {
    int r, t, h;
    head_of_b(v, v.hkey[1][j], r, t, h);
    const int len = v.plen[h];
    const bool cut = v.cutof[h] >= 0;
    const int np = cut ? len / v.piece : 1;
    const int chunks = (v.nb_start[t + 1] - v.nb_start[t] + 63) / 64;
    int lg = 0;
    for (int q = 0; q < np; ++q) {
        const int lq = !cut ? len : (q + 1 < np ? v.piece : len - q * v.piece);
        if (lq >= SM_PMS_CHAIN_LEN) lg += chunks > 1 ? chunks : 1;
    }
    const int c[4] = {np, np * chunks, cut ? (chunks > 1 ? chunks : 1) : 0, lg};
    for (int q = 0; q < 4; ++q) {
        v.hcnt[q][j] = c[q];
        cout[q] = c[q];
    }
    return (long long)r * (K + 1) + t;
}

// the lists: paths (pieces head first), items, repair items
__global__ void k_pf_emit(PfView v, int nh) {
    const int j = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (j >= nh) return;
    int r, t, h;
    head_of_b(v, v.hkey[1][j], r, t, h);
    const int len = v.plen[h], row = v.rowstart[h];
    const int c = v.cutof[h];
    const bool cut = c >= 0;
    const int np = cut ? len / v.piece : 1;
    const int chunks = (v.nb_start[t + 1] - v.nb_start[t] + 63) / 64;
    int pi = v.hoff[0][j], ii = v.hoff[1][j];
    for (int q = 0; q < np; ++q, ++pi) {
        const int r0 = row + q * v.piece;
        const int lq = !cut ? len : (q + 1 < np ? v.piece : row + len - r0);
        v.paths[pi] = PmsPath{t, cut ? r0 : row, lq, 0};
        for (int k = 0; k < chunks; ++k) v.items[ii++] = PmsItem{pi, k};
    }
    if (cut) {
        int ri = v.hoff[2][j];
        for (int k = 0; k < (chunks > 1 ? chunks : 1); ++k) v.reps[ri++] = PmsRep{c, k};
    }
}

}  // namespace

size_t pf_temp_bytes(int N) {
    size_t a = 0, b = 0, c = 0, d = 0, f = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, d, (const unsigned long long*)nullptr, (unsigned long long*)nullptr,
                                             (const int32_t*)nullptr, (int32_t*)nullptr, N, 0, 64);
    (void)hipcub::DeviceScan::InclusiveSum(nullptr, f, (const long long*)nullptr, (long long*)nullptr, 2 * N);
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, a, (const int32_t*)nullptr, (int32_t*)nullptr, (const int32_t*)nullptr,
                                             (int32_t*)nullptr, N, 0, 32);
    (void)hipcub::DeviceRadixSort::SortKeys(nullptr, b, (const unsigned long long*)nullptr, (unsigned long long*)nullptr,
                                            4 * N, 0, 64);
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, c, (const int32_t*)nullptr, (int32_t*)nullptr, 32 * N + 1);
    return std::max(std::max(a, std::max(b, c)), std::max(d, f)) + 256;
}

static int bits_for(int n) {
    int b = 1;
    while ((1ll << b) <= n) ++b;
    return b;
}

hipError_t pf_trees(hipStream_t st, PfView& v, int* K_out) {
    const int N = v.N;
    if (sm_knob("SM_TEST_PMS_CYCLE") && atoi(sm_knob("SM_TEST_PMS_CYCLE")) == 1)
        hipLaunchKernelGGL(k_pf_test_cycle, dim3(1), dim3(64), 0, st, v);
    hipLaunchKernelGGL(k_pf_prep, dim3(nblk(N, 256)), dim3(256), 0, st, v);
    hipLaunchKernelGGL(k_pf_link, dim3(nblk(N, 256)), dim3(256), 0, st, v);
    hipLaunchKernelGGL(k_pf_compress, dim3(nblk(N + 1, 256)), dim3(256), 0, st, v);
    size_t tb = v.temp_bytes;
    hipError_t e = hipcub::DeviceScan::ExclusiveSum(v.temp, tb, v.flag, v.gpix, N + 1, st);  // gpix: tid scratch
    if (e != hipSuccess) return e;
    int32_t K = 0;
    if ((e = hipMemcpyAsync(&K, v.gpix + N, 4, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(v.tsize, 0, (K + 1) * 4, st)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_pf_trees, dim3(nblk(N, 256)), dim3(256), 0, st, v);
    tb = v.temp_bytes;
    if ((e = hipcub::DeviceScan::ExclusiveSum(v.temp, tb, v.tsize, v.tree_start, K + 1, st)) != hipSuccess) return e;
    *K_out = K;
    return hipGetLastError();
}

// one tree tour (rotation words in v.rot): contraction, chain ranking (sm_tour.h)
static hipError_t pf_tour(hipStream_t st, PfView& v) {
    hipError_t e = hipMemsetAsync(v.nchains, 0, 4, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_pf_tour_tile, dim3((v.W + TL - 1) / TL, (v.H + TL - 1) / TL), dim3(TL_THREADS), 0, st, v);
    hipLaunchKernelGGL(k_pf_chain_init, dim3(nblk(v.max_chains, 256)), dim3(256), 0, st, v);
    hipLaunchKernelGGL(k_pf_chain_rank, dim3(PF_CR_BLOCKS), dim3(256), 0, st, v);
    return hipGetLastError();
}

size_t pf_max_chains(int W, int H, int K) {
    // a chain head enters its 32x32 tile across the border (<= 128 per tile) or starts a tree's list
    return (size_t)((W + TL - 1) / TL) * ((H + TL - 1) / TL) * 129 + (size_t)K + 1;
}

hipError_t pf_bfs(hipStream_t st, PfView& v, int K, int* out) {
    const int N = v.N;
    out[0] = out[1] = out[2] = 0;
    hipError_t e = hipMemsetAsync(v.tot, 0, 16 * 4, st);
    if (e != hipSuccess) return e;
    // a forest of N nodes in K trees has N - K edges; anything else has a cycle, whose tour would not
    // be a list (the chain ranking would never reach an end): refuse before any tour
    hipLaunchKernelGGL(k_pf_edges, dim3(nblk(N, 256)), dim3(256), 0, st, v);
    int32_t E = 0;
    if ((e = hipMemcpyAsync(&E, v.tot + 8, 4, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
    if (E != N - K) {
        out[2] = 1;
        return hipSuccess;
    }
    const int dbits = bits_for(N), tbits = bits_for(K);
    if (N - K > 0) {
        hipLaunchKernelGGL(k_pf_rot1, dim3(nblk(N, 256)), dim3(256), 0, st, v);
        if ((e = pf_tour(st, v)) != hipSuccess) return e;
        hipLaunchKernelGGL(k_pf_orient, dim3(nblk(N, 256)), dim3(256), 0, st, v);
        hipLaunchKernelGGL(k_pf_rot2, dim3(nblk(N, 256)), dim3(256), 0, st, v);
        if ((e = pf_tour(st, v)) != hipSuccess) return e;
        hipLaunchKernelGGL(k_pf_tourval, dim3(nblk(N, 256)), dim3(256), 0, st, v);
        size_t tb = v.temp_bytes;
        if ((e = hipcub::DeviceScan::InclusiveSum(v.temp, tb, v.tval, v.tval_s, 2 * (N - K), st)) != hipSuccess) return e;
    } else {  // single-pixel trees only: no arcs, every node a root
        if ((e = hipMemsetAsync(v.pdir, 0xFF, (size_t)N, st)) != hipSuccess) return e;
        hipLaunchKernelGGL(k_pf_fill1, dim3(nblk(N, 256)), dim3(256), 0, st, v.psize, N);
    }
    hipLaunchKernelGGL(k_pf_depth, dim3(nblk(N, 256)), dim3(256), 0, st, v, dbits);
    {
        // an inconsistent tour (a tile over TL_ARCS arcs, or k_pf_depth's range check) leaves positions of
        // the sort input unwritten: stop here, before the sort and the gathers that would read them
        int32_t bad = 0;
        if ((e = hipMemcpyAsync(&bad, v.tot + 7, 4, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
        if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
        if (bad) {
            out[2] = bad;
            return hipSuccess;
        }
    }
    {
        size_t tb = v.temp_bytes;
        if ((e = hipcub::DeviceRadixSort::SortPairs(v.temp, tb, v.tkey[0], v.tkey[1], v.tpix[0], v.gpix, N, 0, tbits + dbits,
                                                    st)) != hipSuccess)
            return e;
    }
    hipLaunchKernelGGL(k_pf_bpos, dim3(nblk(N, 256)), dim3(256), 0, st, v);
    hipLaunchKernelGGL(k_pf_fields, dim3(nblk(N, 256)), dim3(256), 0, st, v);
    // the BFS order is final: identity maps where the round-4 build sorted the level order by tree
    hipLaunchKernelGGL(k_pf_iota, dim3(nblk(N, 256)), dim3(256), 0, st, v.bglob, N);
    hipLaunchKernelGGL(k_pf_iota, dim3(nblk(N, 256)), dim3(256), 0, st, v.g2b, N);
    if ((e = hipMemcpyAsync(v.gtree_s, v.gtree, (size_t)N * 4, hipMemcpyDeviceToDevice, st)) != hipSuccess) return e;
    size_t tb;
    hipLaunchKernelGGL(k_pf_nodes, dim3(nblk(N, 256)), dim3(256), 0, st, v);
    int c = 0;
    for (int it = 0; it < 24; ++it, c ^= 1)  // 2^24 > any depth of a <= 2^24-pixel image
        hipLaunchKernelGGL(k_pf_jump, dim3(nblk(N, 256)), dim3(256), 0, st, v.J[c], v.Dj[c], v.J[c ^ 1], v.Dj[c ^ 1], N);
    if (c) {  // results in J[0] / Dj[0]
        if ((e = hipMemcpyAsync(v.J[0], v.J[1], (size_t)N * 4, hipMemcpyDeviceToDevice, st)) != hipSuccess) return e;
        if ((e = hipMemcpyAsync(v.Dj[0], v.Dj[1], (size_t)N * 4, hipMemcpyDeviceToDevice, st)) != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_pf_heads, dim3(nblk(N + 1, 256)), dim3(256), 0, st, v, v.J[0], v.Dj[0]);
    for (int it = 0; it < 26; ++it)  // light depth <= log2(N) < 25
        hipLaunchKernelGGL(k_pf_ld_step, dim3(nblk(N, 256)), dim3(256), 0, st, v, v.J[0]);
    if ((e = hipMemsetAsync(v.tree_rounds, 0, (size_t)K * 4, st)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_pf_ld_all, dim3(nblk(N, 256)), dim3(256), 0, st, v, v.J[0]);
    tb = v.temp_bytes;
    if ((e = hipcub::DeviceScan::ExclusiveSum(v.temp, tb, v.hflag, v.hidx, N + 1, st)) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(v.tot + 6, v.hidx + N, 4, hipMemcpyDeviceToDevice, st)) != hipSuccess) return e;
    int32_t h[8];
    if ((e = hipMemcpyAsync(h, v.tot, 32, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
    out[0] = h[5];  // rounds
    out[1] = h[6];  // heads
    out[2] = h[7];  // 2: an unresolved light depth, 4: an inconsistent tour (1, above: not a forest)
    return hipGetLastError();
}

hipError_t pf_lists(hipStream_t st, PfView& v, int K, int R, int nh, int* counts) {
    const int N = v.N;
    hipError_t e;
    size_t tb;
    // A order: rows and cuts
    hipLaunchKernelGGL(k_pf_hkeys, dim3(nblk(N, 256)), dim3(256), 0, st, v, 0);
    tb = v.temp_bytes;
    if ((e = hipcub::DeviceRadixSort::SortKeys(v.temp, tb, v.hkey[0], v.hkey[1], nh, 0, 64, st)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_pf_rows_in, dim3(nblk(nh + 1, 256)), dim3(256), 0, st, v, nh);
    for (int q = 0; q < 2; ++q) {
        tb = v.temp_bytes;
        if ((e = hipcub::DeviceScan::ExclusiveSum(v.temp, tb, v.hcnt[q], v.hoff[q], nh + 1, st)) != hipSuccess) return e;
    }
    if ((e = hipMemsetAsync(v.nbcnt, 0, (size_t)(K + 1) * 4, st)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_pf_rows_out, dim3(nblk(nh, 256)), dim3(256), 0, st, v, nh);
    tb = v.temp_bytes;
    if ((e = hipcub::DeviceScan::ExclusiveSum(v.temp, tb, v.nbcnt, v.tree_cut, K + 1, st)) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(v.tot + 4, v.hoff[1] + nh, 4, hipMemcpyDeviceToDevice, st)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_pf_rowof, dim3(nblk(N, 256)), dim3(256), 0, st, v);
    hipLaunchKernelGGL(k_pf_rows, dim3(nblk(N, 256)), dim3(256), 0, st, v);
    // tree graph
    if ((e = hipMemsetAsync(v.npairs, 0, 8, st)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_pf_pairs, dim3(nblk(N, 256)), dim3(256), 0, st, v);
    int32_t np = 0;
    if ((e = hipMemcpyAsync(&np, v.npairs, 4, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
    if (np > 0) {
        tb = v.temp_bytes;
        if ((e = hipcub::DeviceRadixSort::SortKeys(v.temp, tb, v.pairs[0], v.pairs[1], np, 0, 64, st)) != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_pf_uniq_flag, dim3(nblk(np + 1, 256)), dim3(256), 0, st, v, np);
    tb = v.temp_bytes;
    if ((e = hipcub::DeviceScan::ExclusiveSum(v.temp, tb, v.uflag, v.uidx, np + 1, st)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(v.nbcnt, 0, (size_t)(K + 1) * 4, st)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_pf_uniq_emit, dim3(nblk(np, 256) ? nblk(np, 256) : 1), dim3(256), 0, st, v, np);
    tb = v.temp_bytes;
    if ((e = hipcub::DeviceScan::ExclusiveSum(v.temp, tb, v.nbcnt, v.nb_start, K + 1, st)) != hipSuccess) return e;
    // B order: the round-major counts
    hipLaunchKernelGGL(k_pf_hkeys, dim3(nblk(N, 256)), dim3(256), 0, st, v, 1);
    tb = v.temp_bytes;
    if ((e = hipcub::DeviceRadixSort::SortKeys(v.temp, tb, v.hkey[0], v.hkey[1], nh, 0, 64, st)) != hipSuccess) return e;
    const size_t T = (size_t)R * (K + 1);
    for (int q = 0; q < 4; ++q)
        if ((e = hipMemsetAsync(v.rtc[q], 0, (T + 1) * 4, st)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_pf_counts, dim3(nblk(nh + 1, 256)), dim3(256), 0, st, v, nh, K);
    for (int q = 0; q < 4; ++q) {
        tb = v.temp_bytes;
        if ((e = hipcub::DeviceScan::ExclusiveSum(v.temp, tb, v.hcnt[q], v.hoff[q], nh + 1, st)) != hipSuccess) return e;
        tb = v.temp_bytes;
        if ((e = hipcub::DeviceScan::ExclusiveSum(v.temp, tb, v.rtc[q], v.rt[q], T + 1, st)) != hipSuccess) return e;
        if ((e = hipMemcpyAsync(v.tot + q, v.hoff[q] + nh, 4, hipMemcpyDeviceToDevice, st)) != hipSuccess) return e;
    }
    int32_t h[8];
    if ((e = hipMemcpyAsync(h, v.tot, 32, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
    for (int q = 0; q < 5; ++q) counts[q] = h[q];  // paths, items, reps, chain items, cuts
    counts[5] = np;
    counts[6] = h[7];  // != 0: the schedule was inconsistent (rows out of range)
    return hipGetLastError();
}

hipError_t pf_fill(hipStream_t st, PfView& v, int nh) {
    hipLaunchKernelGGL(k_pf_emit, dim3(nblk(nh, 256) ? nblk(nh, 256) : 1), dim3(256), 0, st, v, nh);
    return hipGetLastError();
}
