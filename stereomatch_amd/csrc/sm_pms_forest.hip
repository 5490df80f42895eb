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

#include <hipcub/device/device_radix_sort.hpp>
#include <hipcub/device/device_scan.hpp>

#include "sm_pms_forest.h"
#include "sm_segment.h"

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
constexpr int BT = 1024;  // threads of the BFS workgroup

// exclusive block scan of c (all BT threads), returns the thread's offset; *total the sum
__device__ __forceinline__ int block_scan(int c, int* s_w, int* total) {
    const int tid = (int)threadIdx.x, lane = tid & 63, wv = tid >> 6;
    int incl = c;
#pragma unroll
    for (int k = 1; k < 64; k <<= 1) {
        const int u = __shfl_up(incl, k);
        if (lane >= k) incl += u;
    }
    if (lane == 63) s_w[wv] = incl;
    __syncthreads();
    int pre = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < BT / 64; ++k) {
        const int x = s_w[k];
        if (k < wv) pre += x;
        tot += x;
    }
    __syncthreads();
    *total = tot;
    return pre + incl - c;
}

// the children of a node (its tree neighbours but the parent, in key order) compacted into q / wv by static
// selects: a runtime index into the local arrays (q[c++] = ...) would put them in scratch memory
__device__ __forceinline__ void pf_children(const int (&nn)[4], const uint32_t (&ww)[4], int pp, int (&q)[4], uint32_t (&wv)[4],
                                            int& c) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const bool keep = nn[k] >= 0 && nn[k] != pp;
#pragma unroll
        for (int s = 0; s < 4; ++s)
            if (keep && c == s) {
                q[s] = nn[k];
                wv[s] = ww[k];
            }
        c += keep ? 1 : 0;
    }
}

// Narrow levels (at most 64 nodes: the deep tails of the largest trees, thousands of levels at C2) run on
// wave 0 alone, level after level without workgroup barriers: the frontier stays in registers, the next
// one is handed over through LDS (one wave's LDS operations complete in order).  Entered at level d =
// [a, b) whose nodes are in global memory; leaves at the first level wider than 64 (or the end) with
// s_state = {a, b, d}.
__device__ void bfs_narrow(const PfView& v, int a, int b, int d, int* s_q, int* s_pp, int* s_tr, int* s_state) {
    const int lane = (int)threadIdx.x;
    int n = b - a, i = a + lane;
    bool val = lane < n;
    int p = 0, pp = -1, tr = 0;
    if (val) {
        p = v.gpix[i];
        const int gp = v.gpar[i];
        pp = gp >= 0 ? v.gpix[gp] : -1;
        tr = v.gtree[i];
    }
    while (n > 0 && n <= 64) {
        if (lane == 0) v.glev[d] = a;
        int q[4] = {-1, -1, -1, -1}, c = 0;
        uint32_t wv[4] = {0, 0, 0, 0};
        if (val) {
            const int4 n4 = v.nbr[p];
            const uint2 w4 = v.nbw[p];
            const int nn[4] = {n4.x, n4.y, n4.z, n4.w};
            const uint32_t ww[4] = {w4.x & 0xFFFFu, w4.x >> 16, w4.y & 0xFFFFu, w4.y >> 16};
            pf_children(nn, ww, pp, q, wv, c);
        }
        int incl = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int u = __shfl_up(incl, o);
            if (lane >= o) incl += u;
        }
        const int total = __shfl(incl, 63), pos = incl - c;
        if (val) {
            v.gfc[i] = b + pos;
            v.gnc[i] = (uint8_t)c;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (k >= c) break;
                const int j = b + pos + k;
                if (j >= v.N) {  // only masks with a cycle get here (as in the workgroup levels)
                    v.tot[7] = 1;
                    break;
                }
                v.gpix[j] = q[k];
                v.gpar[j] = i;
                v.gtree[j] = tr;
                v.gw[j] = (uint16_t)wv[k];
                if (pos + k < 64) {
                    s_q[pos + k] = q[k];
                    s_pp[pos + k] = p;
                    s_tr[pos + k] = tr;
                }
            }
        }
        const int nb = b + total < v.N ? b + total : v.N;
        a = b;
        b = nb;
        ++d;
        n = b - a;
        i = a + lane;
        val = lane < n;
        __atomic_signal_fence(__ATOMIC_SEQ_CST);  // the LDS writes above stay before the reads below
        __builtin_amdgcn_wave_barrier();
        if (n <= 64 && val) {
            p = s_q[lane];
            pp = s_pp[lane];
            tr = s_tr[lane];
        }
        __atomic_signal_fence(__ATOMIC_SEQ_CST);  // and these reads before the next level's writes
        __builtin_amdgcn_wave_barrier();
    }
    if (lane == 0) {
        s_state[0] = a;
        s_state[1] = b;
        s_state[2] = d;
    }
}

// Narrow levels of the bottom-up sweep on wave 0, from level l down while levels have at most 64 nodes;
// a level's sizes stay in LDS for its parents' level.  s_state[3] = the first level left (or -1).
__device__ void sweep_narrow(const PfView& v, int l, int* s_sz, int* s_state) {
    const int lane = (int)threadIdx.x;
    int pbase = -1;  // the start of level l + 1 when its sizes are in s_sz
    for (; l >= 0; --l) {
        const int la = min(max(v.glev[l], 0), v.N), lb = min(max(v.glev[l + 1], la), v.N);
        const int n = lb - la;
        if (n > 64) break;
        const int i = la + lane;
        int s = 1, best = -1, bs = 0;
        if (lane < n) {
            const int f = v.gfc[i], c = min((int)v.gnc[i], v.N - f);
            for (int k = 0; k < c; ++k) {
                const int o = f + k - pbase;
                const int sk = pbase >= 0 && o >= 0 && o < 64 ? s_sz[o] : v.gsize[f + k];
                s += sk;
                if (sk > bs) {  // strictly larger: ties keep the smallest BFS id
                    bs = sk;
                    best = k;
                }
            }
            v.gsize[i] = s;
            v.ghk[i] = (int8_t)best;
        }
        __atomic_signal_fence(__ATOMIC_SEQ_CST);  // this level's reads of s_sz before its writes
        __builtin_amdgcn_wave_barrier();
        if (lane < n) s_sz[lane] = s;
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        __builtin_amdgcn_wave_barrier();
        pbase = la;
    }
    if (lane == 0) s_state[3] = l;
}

// One workgroup: the BFS of every tree of the view at once, then the bottom-up sweep.  Level 0 is the
// roots in tree order; a node's children follow, in key order, at the next level, after the children
// of the nodes before it.
constexpr int PF_FC = 4096;  // a level of at most this many nodes is handed to the next one in LDS

__global__ void __launch_bounds__(BT) k_pf_bfs(PfView v, int K) {
    __shared__ int s_w[BT / 64];
    __shared__ int s_q[64], s_pp[64], s_tr[64], s_sz[64], s_state[4];
    // the frontier of a level (pixel, its parent's pixel, tree), double-buffered: a level's children are
    // written there too, so the next level reads LDS instead of three dependent global loads
    __shared__ int s_fp[2][PF_FC], s_fpp[2][PF_FC], s_ftr[2][PF_FC];
    const int tid = (int)threadIdx.x;
    for (int t = tid; t < K; t += BT) {
        v.gpix[t] = v.root_pix[t];
        v.gpar[t] = -1;
        v.gtree[t] = t;
        v.gw[t] = 0;
    }
    __syncthreads();
    int a = 0, b = K, next = K, d = 0, cur = 0;
    bool in_lds = false;  // the roots are in global memory
    while (a < b) {
        if (b - a <= 64) {  // narrow levels on wave 0 (next == b at a level's start)
            if (tid < 64) bfs_narrow(v, a, b, d, s_q, s_pp, s_tr, s_state);
            __syncthreads();
            a = s_state[0];
            b = s_state[1];
            d = s_state[2];
            next = b;
            in_lds = false;
            __syncthreads();  // s_state read by every wave before it is written again
            continue;
        }
        if (tid == 0) v.glev[d] = a;
        for (int base = a; base < b; base += BT) {
            const int i = base + tid;
            int q[4] = {-1, -1, -1, -1}, c = 0;
            uint32_t wv[4] = {0, 0, 0, 0};
            int tr = 0;
            int p = 0;
            if (i < b) {
                int pp;
                if (in_lds) {
                    p = s_fp[cur][i - a];
                    pp = s_fpp[cur][i - a];
                    tr = s_ftr[cur][i - a];
                } else {
                    p = v.gpix[i];
                    const int gp = v.gpar[i];
                    pp = gp >= 0 ? v.gpix[gp] : -1;
                    tr = v.gtree[i];
                }
                const int4 n4 = v.nbr[p];
                const uint2 w4 = v.nbw[p];
                const int nn[4] = {n4.x, n4.y, n4.z, n4.w};
                const uint32_t ww[4] = {w4.x & 0xFFFFu, w4.x >> 16, w4.y & 0xFFFFu, w4.y >> 16};
                pf_children(nn, ww, pp, q, wv, c);  // every tree neighbour but the parent is a child
            }
            int total;
            const int pos = block_scan(c, s_w, &total);
            if (i < b) {
                v.gfc[i] = next + pos;
                v.gnc[i] = (uint8_t)c;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    if (k >= c) break;
                    const int j = next + pos + k;
                    if (j >= v.N) {  // only masks with a cycle (not a forest) get here: flag, never write out of bounds
                        v.tot[7] = 1;
                        break;
                    }
                    v.gpix[j] = q[k];
                    v.gpar[j] = i;
                    v.gtree[j] = tr;
                    v.gw[j] = (uint16_t)wv[k];
                    if (j - b < PF_FC) {
                        s_fp[cur ^ 1][j - b] = q[k];
                        s_fpp[cur ^ 1][j - b] = p;
                        s_ftr[cur ^ 1][j - b] = tr;
                    }
                }
            }
            next = next + total < v.N ? next + total : v.N;
        }
        __syncthreads();  // this level's writes are visible to the next one's reads
        in_lds = next - b <= PF_FC;
        cur ^= 1;
        a = b;
        b = next;
        ++d;
    }
    if (tid == 0) {
        v.glev[d] = a;
        v.nlev[0] = d;
    }
    __syncthreads();  // the last boundary is read by every wave below
    // bottom up: subtree sizes and heavy children, a level at a time
    for (int l = d - 1; l >= 0; --l) {
        const int la = min(max(v.glev[l], 0), v.N), lb = min(max(v.glev[l + 1], la), v.N);
        if (lb - la <= 64) {  // narrow levels on wave 0
            if (tid < 64) sweep_narrow(v, l, s_sz, s_state);
            __syncthreads();
            l = s_state[3] + 1;  // the loop's decrement gives the first level left
            __syncthreads();
            continue;
        }
        for (int i = la + tid; i < lb; i += BT) {
            const int f = v.gfc[i], c = min((int)v.gnc[i], v.N - f);  // clamp: only a cycle overflows
            int s = 1, best = -1, bs = 0;
            for (int k = 0; k < c; ++k) {
                const int sk = v.gsize[f + k];
                s += sk;
                if (sk > bs) {  // strictly larger: ties keep the smallest BFS id (children are in BFS order)
                    bs = sk;
                    best = k;
                }
            }
            v.gsize[i] = s;
            v.ghk[i] = (int8_t)best;
        }
        __syncthreads();
    }
}

__global__ void k_pf_iota(int32_t* a, int n) {
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i < n) a[i] = i;
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
    size_t a = 0, b = 0, c = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, a, (const int32_t*)nullptr, (int32_t*)nullptr, (const int32_t*)nullptr,
                                             (int32_t*)nullptr, N, 0, 32);
    (void)hipcub::DeviceRadixSort::SortKeys(nullptr, b, (const unsigned long long*)nullptr, (unsigned long long*)nullptr,
                                            4 * N, 0, 64);
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, c, (const int32_t*)nullptr, (int32_t*)nullptr, 32 * N + 1);
    return std::max(a, std::max(b, c)) + 256;
}

static int bits_for(int n) {
    int b = 1;
    while ((1ll << b) <= n) ++b;
    return b;
}

hipError_t pf_trees(hipStream_t st, PfView& v, int* K_out) {
    const int N = v.N;
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

hipError_t pf_bfs(hipStream_t st, PfView& v, int K, int* out) {
    const int N = v.N;
    hipError_t e0 = hipMemsetAsync(v.tot, 0, 8 * 4, st);
    if (e0 != hipSuccess) return e0;
    hipLaunchKernelGGL(k_pf_bfs, dim3(1), dim3(BT), 0, st, v, K);
    hipLaunchKernelGGL(k_pf_iota, dim3(nblk(N, 256)), dim3(256), 0, st, v.iota, N);
    size_t tb = v.temp_bytes;
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(v.temp, tb, v.gtree, v.gtree_s, v.iota, v.bglob, N, 0, bits_for(K), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_pf_g2b, dim3(nblk(N, 256)), dim3(256), 0, st, v);
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
    out[2] = h[7];  // 1: the masks were not a forest
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
