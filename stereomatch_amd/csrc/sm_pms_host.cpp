// sm_pms_host.cpp -- host side of the MST_PMS label search: the forest in the reference's numbering,
// its tree graph, the heavy-path schedule the GPU walkers follow, and the random streams.
//
// Reference (src/Stereo3DMST.cpp):
//   * trees are numbered by their first pixel in raster order and rooted there (:342-384, :454-467);
//     BFS from the root gives the node ids (mst_vertices_vec[t]), siblings in Boost vecS adjacency order
//     = ascending (w, a, b) edge key, since MST edges are inserted in sorted-edge order (:436-446, 492-516);
//   * tree_g links trees that share a 4-connected grid edge; boost setS keeps one entry per neighbour in
//     ascending id (:46, :377-384), the order MST_PMS visits them (:563-580);
//   * dice = uniform_real_distribution<float> bound to a COPY of a default-seeded minstd_rand0 (:390-392,
//     :554, :851-852): every segment_image_other_init and every MST_PMS call replays one stream;
//   * rand() (glibc, shared with random()): random_rgb's 3 draws per pixel of each view (:72-80, :316)
//     come before MST_PMS's one draw per tree (:584).
// The schedule is this library's own: every tree is cut into heavy paths; a path's light children are
// heads of paths one light depth deeper, so the up pass runs light depths deepest first and the down
// pass root first, each depth one round of independent paths (DESIGN.md "MST_PMS").
#include "sm_pms_host.h"
#include "sm_knob.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <chrono>
#include <cstdio>

namespace {

// the (w, a, b) edge order as a key: b = a+1 or a+W, so (w, a, vertical) is order-isomorphic
inline uint64_t ekey(uint32_t w, uint32_t a, uint32_t vert) { return ((uint64_t)w << 33) | ((uint64_t)a << 1) | vert; }

struct Bfs {
    std::vector<int32_t> tree_start, pix, parent, nodeof;
    std::vector<uint16_t> w;
    std::vector<uint8_t> nch;
    std::vector<int32_t> child;  // 4 per node, ascending BFS id
};

// forest masks -> BFS numbering of every tree (mR / mD: real edges only)
void bfs_forest(int W, int H, const uint16_t* wR, const uint16_t* wD, const uint8_t* mR, const uint8_t* mD, Bfs& b) {
    const int N = W * H;
    b.pix.resize(N);
    b.parent.resize(N);
    b.nodeof.assign(N, -1);
    b.w.resize(N);
    b.nch.resize(N);
    b.child.assign(4 * (size_t)N, -1);
    b.tree_start.clear();
    int tail = 0;
    for (int r = 0; r < N; ++r) {
        if (b.nodeof[r] >= 0) continue;  // the first unvisited pixel in raster order roots a new tree
        b.tree_start.push_back(tail);
        int head = tail;
        b.pix[tail] = r;
        b.parent[tail] = tail;
        b.w[tail] = 0;
        b.nodeof[r] = tail++;
        while (head < tail) {
            const int n = head++;
            const int p = b.pix[n];
            const int x = p % W;
            uint64_t key[4];
            int nb[4], k = 0;
            if (x + 1 < W && mR[p]) { key[k] = ekey(wR[p], (uint32_t)p, 0); nb[k++] = p + 1; }
            if (p + W < N && mD[p]) { key[k] = ekey(wD[p], (uint32_t)p, 1); nb[k++] = p + W; }
            if (x > 0 && mR[p - 1]) { key[k] = ekey(wR[p - 1], (uint32_t)(p - 1), 0); nb[k++] = p - 1; }
            if (p >= W && mD[p - W]) { key[k] = ekey(wD[p - W], (uint32_t)(p - W), 1); nb[k++] = p - W; }
            for (int i = 1; i < k; ++i)  // ascending key (insertion sort of <= 4)
                for (int j = i; j > 0 && key[j] < key[j - 1]; --j) {
                    std::swap(key[j], key[j - 1]);
                    std::swap(nb[j], nb[j - 1]);
                }
            int c = 0;
            for (int i = 0; i < k; ++i) {
                const int q = nb[i];
                if (b.nodeof[q] >= 0) continue;  // the parent
                b.pix[tail] = q;
                b.parent[tail] = n;
                b.w[tail] = (uint16_t)(key[i] >> 33);
                b.nodeof[q] = tail;
                b.child[4 * (size_t)n + c++] = tail++;
            }
            b.nch[n] = (uint8_t)c;
        }
    }
    b.tree_start.push_back(tail);
}

// tree_g as CSR: neighbours ascending, no duplicates
void tree_graph(int W, int H, const Bfs& b, std::vector<int32_t>& nb_start, std::vector<int32_t>& nb) {
    const int N = W * H;
    const int K = (int)b.tree_start.size() - 1;
    std::vector<int32_t> cc(N);
    for (int t = 0; t < K; ++t)
        for (int n = b.tree_start[t]; n < b.tree_start[t + 1]; ++n) cc[b.pix[n]] = t;
    std::vector<uint64_t> pr;
    for (int p = 0; p < N; ++p) {
        const int x = p % W;
        if (x + 1 < W && cc[p] != cc[p + 1]) {
            pr.push_back(((uint64_t)cc[p] << 32) | (uint32_t)cc[p + 1]);
            pr.push_back(((uint64_t)cc[p + 1] << 32) | (uint32_t)cc[p]);
        }
        if (p + W < N && cc[p] != cc[p + W]) {
            pr.push_back(((uint64_t)cc[p] << 32) | (uint32_t)cc[p + W]);
            pr.push_back(((uint64_t)cc[p + W] << 32) | (uint32_t)cc[p]);
        }
    }
    std::sort(pr.begin(), pr.end());
    pr.erase(std::unique(pr.begin(), pr.end()), pr.end());
    nb_start.assign(K + 1, 0);
    nb.resize(pr.size());
    for (size_t i = 0; i < pr.size(); ++i) {
        nb_start[(pr[i] >> 32) + 1]++;
        nb[i] = (int32_t)(pr[i] & 0xffffffffu);
    }
    for (int t = 0; t < K; ++t) nb_start[t + 1] += nb_start[t];
}

uint32_t minstd_next(uint32_t s) { return (uint32_t)(((uint64_t)s * 16807u) % 2147483647u); }
// generate_canonical<float, 24> of the shipped libstdc++ (GCC 5.4): one engine call, (float)(u - 1) /
// 2^31 as a multiply by 2^-31, no clamp below 1 (build/StereoYin 0x40ff38-0x40ff63)
float canon(uint32_t u) { return (float)(int32_t)(u - 1u) * 0x1p-31f; }

}  // namespace

// Runs fn(i) for i in [0, n) over nthreads host threads, indices handed out in order (dynamic).
template <class F>
void parallel_for(int n, int nthreads, F&& fn) {
    if (nthreads <= 1 || n <= 1) {
        for (int i = 0; i < n; ++i) fn(i);
        return;
    }
    std::atomic<int> next{0};
    auto work = [&] {
        for (int i; (i = next.fetch_add(1, std::memory_order_relaxed)) < n;) fn(i);
    };
    std::vector<std::thread> th;
    const int nt = std::min(nthreads, n);
    for (int k = 1; k < nt; ++k) th.emplace_back(work);
    work();
    for (auto& x : th) x.join();
}

int pms_prep_threads() {
    const char* e = sm_knob("SM_PREP_THREADS");
    if (e) return std::max(1, atoi(e));
    const unsigned hc = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(8u, hc / 2));  // two views build at once
}

// The forest in the reference's numbering, built tree by tree on `nthreads` host threads:
//   1. union-find over the forest edges, each root the smallest pixel, so the raster-order scan meets every
//      tree at its first pixel and numbers the trees as the reference does (:342-384);
//   2. per tree (in parallel, largest first): the BFS from that pixel (bfs_forest's order, :450-522), subtree
//      sizes, heavy children, light depths, heads by (light depth, BFS id) and the rows;
//   3. tree_g from per-band pair lists; the cuts and the round-major lists by counting and prefix sums.
// The result is the sequential construction's, array for array (tests/test_pms_host.py).
int pms_build_forest(int W, int H, const uint16_t* wR, const uint16_t* wD, const uint8_t* mR, const uint8_t* mD,
                     PmsForest& f, int piece, int nthreads) {
    const int N = W * H;
    if (nthreads <= 0) nthreads = pms_prep_threads();
    const bool dbg = sm_knob("SM_PREP_DEBUG") != nullptr;  // phase times on stderr (diagnostics)
    auto now = [] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    const double tp0 = dbg ? now() : 0.0;
    // 1. trees
    std::vector<int32_t> uf(N), tree_of(N);
    for (int p = 0; p < N; ++p) uf[p] = p;
    auto find = [&uf](int x) {
        while (uf[x] != x) {
            uf[x] = uf[uf[x]];
            x = uf[x];
        }
        return x;
    };
    auto unite = [&](int a, int c) {
        const int ra = find(a), rc = find(c);
        if (ra < rc) uf[rc] = ra;
        else if (rc < ra) uf[ra] = rc;
    };
    for (int p = 0; p < N; ++p) {
        if (p % W + 1 < W && mR[p]) unite(p, p + 1);
        if (p + W < N && mD[p]) unite(p, p + W);
    }
    std::vector<int32_t> root_pix, tsize;
    for (int p = 0; p < N; ++p) {
        const int r = find(p);
        if (r == p) {
            tree_of[p] = (int32_t)root_pix.size();
            root_pix.push_back(p);
            tsize.push_back(0);
        } else {
            tree_of[p] = tree_of[r];
        }
        ++tsize[tree_of[p]];
    }
    const int K = (int)root_pix.size();
    f.W = W;
    f.H = H;
    f.K = K;
    f.tree_start.assign(K + 1, 0);
    for (int t = 0; t < K; ++t) f.tree_start[t + 1] = f.tree_start[t] + tsize[t];
    std::vector<int> order(K);
    for (int t = 0; t < K; ++t) order[t] = t;
    std::stable_sort(order.begin(), order.end(), [&](int a, int c) { return tsize[a] > tsize[c]; });
    const double tp1 = dbg ? now() : 0.0;
    // 2. per tree: BFS, heavy paths, rows
    Bfs b;
    b.pix.resize(N);
    b.parent.resize(N);
    b.nodeof.assign(N, -1);
    b.w.resize(N);
    b.nch.resize(N);
    b.child.resize(4 * (size_t)N);
    std::vector<int32_t> size(N), heavy(N), ld(N), rowof(N), tmaxld(K, 0), hd(N), off(N), plen(N), rowstart(N);
    std::vector<std::vector<PmsPath>> tp(K);
    std::vector<std::vector<int32_t>> tpld(K);
    f.rows.resize(N);
    parallel_for(K, nthreads, [&](int oi) {
        const int t = order[oi];
        const int ts = f.tree_start[t], te = f.tree_start[t + 1];
        int tail = ts, head = ts;
        b.pix[tail] = root_pix[t];
        b.parent[tail] = tail;
        b.w[tail] = 0;
        b.nodeof[root_pix[t]] = tail++;
        while (head < tail) {  // bfs_forest's visit, confined to the tree
            const int n = head++;
            const int p = b.pix[n];
            const int x = p % W;
            uint64_t key[4];
            int nb[4], k = 0;
            if (x + 1 < W && mR[p]) { key[k] = ekey(wR[p], (uint32_t)p, 0); nb[k++] = p + 1; }
            if (p + W < N && mD[p]) { key[k] = ekey(wD[p], (uint32_t)p, 1); nb[k++] = p + W; }
            if (x > 0 && mR[p - 1]) { key[k] = ekey(wR[p - 1], (uint32_t)(p - 1), 0); nb[k++] = p - 1; }
            if (p >= W && mD[p - W]) { key[k] = ekey(wD[p - W], (uint32_t)(p - W), 1); nb[k++] = p - W; }
            for (int i = 1; i < k; ++i)
                for (int j = i; j > 0 && key[j] < key[j - 1]; --j) {
                    std::swap(key[j], key[j - 1]);
                    std::swap(nb[j], nb[j - 1]);
                }
            int c = 0;
            for (int i = 0; i < k; ++i) {
                const int q = nb[i];
                if (b.nodeof[q] >= 0) continue;  // the parent (pixels of this tree only: no other thread's)
                b.pix[tail] = q;
                b.parent[tail] = n;
                b.w[tail] = (uint16_t)(key[i] >> 33);
                b.nodeof[q] = tail;
                b.child[4 * (size_t)n + c++] = tail++;
            }
            for (int i = c; i < 4; ++i) b.child[4 * (size_t)n + i] = -1;
            b.nch[n] = (uint8_t)c;
        }
        // subtree sizes (children have larger BFS ids), heavy child = the largest subtree (ties: the
        // smallest BFS id), light depth
        for (int n = ts; n < te; ++n) size[n] = 1;
        for (int n = te - 1; n > ts; --n) size[b.parent[n]] += size[n];
        ld[ts] = 0;
        int mld = 0;
        for (int n = ts; n < te; ++n) {
            int best = -1;
            for (int i = 0; i < b.nch[n]; ++i) {
                const int c = b.child[4 * (size_t)n + i];
                if (best < 0 || size[c] > size[best]) best = c;
            }
            heavy[n] = best;
            for (int i = 0; i < b.nch[n]; ++i) {
                const int c = b.child[4 * (size_t)n + i];
                ld[c] = ld[n] + (c == best ? 0 : 1);
                mld = std::max(mld, ld[c]);
            }
        }
        tmaxld[t] = mld;
        // heads by (light depth, BFS id): a counting sort; each path head-first on consecutive rows.  In
        // BFS order (parents first) every node learns its path's head and its offset on the path, so the
        // rows come from forward passes instead of walking each heavy chain (pointer chasing)
        std::vector<int32_t> cnt(mld + 2, 0);
        for (int n = ts; n < te; ++n) {
            const bool head = n == ts || heavy[b.parent[n]] != n;
            hd[n] = head ? n : hd[b.parent[n]];
            off[n] = head ? 0 : off[b.parent[n]] + 1;
            plen[hd[n]] = off[n] + 1;  // the chain's nodes come in increasing offset
            if (head) ++cnt[ld[n] + 1];
        }
        for (int l = 0; l <= mld; ++l) cnt[l + 1] += cnt[l];
        std::vector<int32_t> heads(cnt[mld + 1]);
        for (int n = ts; n < te; ++n)
            if (hd[n] == n) heads[cnt[ld[n]]++] = n;
        int row = ts;
        tp[t].reserve(heads.size());
        tpld[t].reserve(heads.size());
        for (int h : heads) {
            rowstart[h] = row;
            tp[t].push_back(PmsPath{t, row, plen[h], 0});
            tpld[t].push_back(ld[h]);
            row += plen[h];
        }
        for (int n = ts; n < te; ++n) rowof[n] = rowstart[hd[n]] + off[n];
        for (int n = ts; n < te; ++n) {
            PmsRow& R = f.rows[rowof[n]];
            const int p = b.pix[n];
            R.pix = p;
            R.x = (uint16_t)(p % W);
            R.y = (uint16_t)(p / W);
            R.parent = n == ts ? -1 : rowof[b.parent[n]];
            R.w = b.w[n];
            R.nch = b.nch[n];
            R.hk = 0xFF;
            for (int i = 0; i < 4; ++i) {
                R.child[i] = -1;
                R.wch[i] = 0;
            }
            for (int i = 0; i < b.nch[n]; ++i) {  // descending BFS id: the up pass's fold order (:125)
                const int c = b.child[4 * (size_t)n + (b.nch[n] - 1 - i)];
                R.child[i] = rowof[c];
                R.wch[i] = b.w[c];
                if (c == heavy[n]) R.hk = (uint8_t)i;
            }
        }
    });
    const double tp2 = dbg ? now() : 0.0;
    f.bfs_pix = std::move(b.pix);
    // 3. tree_g: inter-tree grid edges of row bands, both directions, sorted and deduplicated
    {
        const int nb = std::max(1, std::min(nthreads * 4, H));
        std::vector<std::vector<uint64_t>> pr(nb);
        parallel_for(nb, nthreads, [&](int k) {
            const int y0 = (int)((long long)H * k / nb), y1 = (int)((long long)H * (k + 1) / nb);
            std::vector<uint64_t>& v = pr[k];
            for (int p = y0 * W; p < y1 * W; ++p) {
                const int x = p % W;
                if (x + 1 < W && tree_of[p] != tree_of[p + 1]) {
                    v.push_back(((uint64_t)tree_of[p] << 32) | (uint32_t)tree_of[p + 1]);
                    v.push_back(((uint64_t)tree_of[p + 1] << 32) | (uint32_t)tree_of[p]);
                }
                if (p + W < N && tree_of[p] != tree_of[p + W]) {
                    v.push_back(((uint64_t)tree_of[p] << 32) | (uint32_t)tree_of[p + W]);
                    v.push_back(((uint64_t)tree_of[p + W] << 32) | (uint32_t)tree_of[p]);
                }
            }
            std::sort(v.begin(), v.end());
            v.erase(std::unique(v.begin(), v.end()), v.end());
        });
        std::vector<uint64_t> all;
        for (auto& v : pr) all.insert(all.end(), v.begin(), v.end());
        std::sort(all.begin(), all.end());
        all.erase(std::unique(all.begin(), all.end()), all.end());
        f.nb_start.assign(K + 1, 0);
        f.nb.resize(all.size());
        for (size_t i = 0; i < all.size(); ++i) {
            f.nb_start[(all[i] >> 32) + 1]++;
            f.nb[i] = (int32_t)(all[i] & 0xffffffffu);
        }
        for (int t = 0; t < K; ++t) f.nb_start[t + 1] += f.nb_start[t];
    }
    // cut paths, in tree order
    f.piece = piece > 0 ? piece : 0;
    f.tree_cut.assign(K + 1, 0);
    for (int t = 0; t < K; ++t) {
        int nc = 0;
        if (f.piece > 0)
            for (const PmsPath& pa : tp[t]) nc += pa.len >= 2 * f.piece;
        f.tree_cut[t + 1] = f.tree_cut[t] + nc;
    }
    f.cuts.resize(f.tree_cut[K]);
    f.cut_round.resize(f.tree_cut[K]);
    // round-major path, item and repair lists: counts per (round, tree), prefix sums, then each tree fills its
    // slots (a tree's paths are in light-depth order)
    int rmax = 0;
    for (int t = 0; t < K; ++t) rmax = std::max(rmax, tmaxld[t] + 1);
    f.nrounds = rmax;
    f.tree_rounds.resize(K);
    for (int t = 0; t < K; ++t) f.tree_rounds[t] = tmaxld[t] + 1;
    const size_t K1 = (size_t)K + 1;
    std::vector<int32_t> cp((size_t)rmax * K1, 0), ci((size_t)rmax * K1, 0), cr((size_t)rmax * K1, 0),
        cl((size_t)rmax * K1, 0);
    auto chunks_of = [&f](int t) { return (f.nb_start[t + 1] - f.nb_start[t] + 63) / 64; };
    parallel_for(K, nthreads, [&](int t) {
        const int chunks = chunks_of(t);
        for (size_t i = 0; i < tp[t].size(); ++i) {
            const PmsPath& pa = tp[t][i];
            const bool cut = f.piece > 0 && pa.len >= 2 * f.piece;
            const int np = cut ? pa.len / f.piece : 1;
            const size_t k = (size_t)tpld[t][i] * K1 + t;
            cp[k] += np;
            ci[k] += np * chunks;
            if (cut) cr[k] += std::max(chunks, 1);
            for (int q = 0; q < np; ++q) {  // the pieces' lengths (as the fill below)
                const int len = !cut ? pa.len : (q + 1 < np ? f.piece : pa.len - q * f.piece);
                if (len >= SM_PMS_CHAIN_LEN) cl[k] += std::max(chunks, 1);
            }
        }
    });
    f.rt_path.assign((size_t)rmax * K1, 0);
    f.rt_item.assign((size_t)rmax * K1, 0);
    f.rt_rep.assign((size_t)rmax * K1, 0);
    f.rt_long.assign((size_t)rmax * K1, 0);
    int32_t sp = 0, si = 0, sr = 0, sl = 0;
    for (int r = 0; r < rmax; ++r)
        for (int t = 0; t <= K; ++t) {
            const size_t k = (size_t)r * K1 + t;
            f.rt_path[k] = sp;
            f.rt_item[k] = si;
            f.rt_rep[k] = sr;
            f.rt_long[k] = sl;
            if (t < K) {
                sp += cp[k];
                si += ci[k];
                sr += cr[k];
                sl += cl[k];
            }
        }
    f.paths.resize(sp);
    f.items.resize(si);
    f.reps.resize(sr);
    parallel_for(K, nthreads, [&](int t) {
        const int chunks = chunks_of(t);
        int c = f.tree_cut[t];
        for (size_t i = 0; i < tp[t].size(); ++i) {
            const PmsPath pa = tp[t][i];
            const int r = tpld[t][i];
            const size_t k = (size_t)r * K1 + t;
            const bool cut = f.piece > 0 && pa.len >= 2 * f.piece;
            const int np = cut ? pa.len / f.piece : 1;
            if (cut) {
                f.cuts[c] = PmsCut{t, pa.row, pa.len, np};
                f.cut_round[c] = r;
            }
            for (int q = 0; q < np; ++q) {  // the pieces, head first
                const int r0 = pa.row + q * f.piece;
                const int len = !cut ? pa.len : (q + 1 < np ? f.piece : pa.row + pa.len - r0);
                const int pi = f.rt_path[k]++;
                f.paths[pi] = PmsPath{t, r0, len, 0};
                for (int h = 0; h < chunks; ++h) f.items[f.rt_item[k]++] = PmsItem{pi, h};
            }
            if (cut) {
                for (int h = 0; h < std::max(chunks, 1); ++h) f.reps[f.rt_rep[k]++] = PmsRep{c, h};
                ++c;
            }
        }
    });
    if (dbg)
        fprintf(stderr, "pms_build_forest %dx%d K %d threads %d: trees (union-find) %.1f ms, BFS + paths + rows %.1f ms, "
                "tree graph + lists %.1f ms (largest tree %d nodes)\n", W, H, K, nthreads, tp1 - tp0, tp2 - tp1, now() - tp2,
                K ? tsize[order[0]] : 0);
    f.npaths = (int)f.paths.size();
    f.nitems = (int)f.items.size();
    f.on_device = false;
    // the fills advanced each (round, tree) start to the next one's: shift back
    for (auto* v : {&f.rt_path, &f.rt_item, &f.rt_rep}) {
        std::vector<int32_t>& a = *v;
        for (size_t k = a.size(); k-- > 1;) a[k] = a[k - 1];
        if (!a.empty()) a[0] = 0;
    }
    return K;
}

// TYPE_3 additive feedback generator (degree 31, separation 3): srandom_r fills the state with
// 16807 * x mod (2^31 - 1) (Schrage), then discards 310 outputs; each output is the new state word
// shifted right by one.
void GlibcRandom::seed_skip(unsigned seed, long skip) {
    if (seed == 0) seed = 1;
    st[0] = (int32_t)seed;
    long word = (long)seed;
    for (int i = 1; i < 31; ++i) {
        const long hi = word / 127773, lo = word % 127773;
        word = 16807 * lo - 2836 * hi;
        if (word < 0) word += 2147483647;
        st[i] = (int32_t)word;
    }
    f = 3;
    r = 0;
    const long total = 310 + skip;
    for (long k = 0; k < total; ++k) {
        st[f] = (int32_t)((uint32_t)st[f] + (uint32_t)st[r]);
        if (++f >= 31) {
            f = 0;
            ++r;
        } else if (++r >= 31) {
            r = 0;
        }
    }
}

void GlibcRandom::draw(long n, int32_t* out) {
    for (long k = 0; k < n; ++k) {
        const uint32_t v = (uint32_t)st[f] + (uint32_t)st[r];
        st[f] = (int32_t)v;
        out[k] = (int32_t)(v >> 1);
        if (++f >= 31) {
            f = 0;
            ++r;
        } else if (++r >= 31) {
            r = 0;
        }
    }
}

// FNV-1a digests of the built forest's arrays (tests: the build is the same for any thread count)
static uint64_t fnv(const void* p, size_t n, uint64_t h = 1469598103934665603ull) {
    const unsigned char* c = static_cast<const unsigned char*>(p);
    for (size_t i = 0; i < n; ++i) h = (h ^ c[i]) * 1099511628211ull;
    return h;
}
template <class T>
static uint64_t fnv_vec(const std::vector<T>& v) { return fnv(v.data(), v.size() * sizeof(T)); }

extern "C" {

int sm_pms_forest_bfs(int W, int H, const uint16_t* wR, const uint16_t* wD, const uint8_t* mask, int32_t* tree_start,
                      int32_t* node_pix, int32_t* node_parent, uint16_t* node_w, uint8_t* node_nch, int32_t* node_child) {
    const int N = W * H;
    std::vector<uint8_t> mR(N), mD(N);
    for (int p = 0; p < N; ++p) {
        mR[p] = mask[p] & 1;
        mD[p] = (mask[p] >> 1) & 1;
    }
    Bfs b;
    bfs_forest(W, H, wR, wD, mR.data(), mD.data(), b);
    const int K = (int)b.tree_start.size() - 1;
    std::memcpy(tree_start, b.tree_start.data(), (K + 1) * sizeof(int32_t));
    std::memcpy(node_pix, b.pix.data(), N * sizeof(int32_t));
    std::memcpy(node_parent, b.parent.data(), N * sizeof(int32_t));
    std::memcpy(node_w, b.w.data(), N * sizeof(uint16_t));
    std::memcpy(node_nch, b.nch.data(), N);
    std::memcpy(node_child, b.child.data(), 4 * (size_t)N * sizeof(int32_t));
    return K;
}

int sm_pms_tree_graph(int W, int H, const uint8_t* mask, const uint16_t* wR, const uint16_t* wD, int32_t* nb_start,
                      int32_t* nb, int nb_cap) {
    const int N = W * H;
    std::vector<uint8_t> mR(N), mD(N);
    for (int p = 0; p < N; ++p) {
        mR[p] = mask[p] & 1;
        mD[p] = (mask[p] >> 1) & 1;
    }
    Bfs b;
    bfs_forest(W, H, wR, wD, mR.data(), mD.data(), b);
    std::vector<int32_t> s, n;
    tree_graph(W, H, b, s, n);
    if ((int)n.size() > nb_cap) return -1;
    std::memcpy(nb_start, s.data(), s.size() * sizeof(int32_t));
    std::memcpy(nb, n.data(), n.size() * sizeof(int32_t));
    return (int)n.size();
}

int sm_pms_forest_digest(int W, int H, const uint16_t* wR, const uint16_t* wD, const uint8_t* mask, int piece, int nthreads,
                         uint64_t* out, int32_t* tree_start, int32_t* bfs_pix) {
    const int N = W * H;
    std::vector<uint8_t> mR(N), mD(N);
    for (int p = 0; p < N; ++p) {
        mR[p] = mask[p] & 1;
        mD[p] = (mask[p] >> 1) & 1;
    }
    PmsForest f;
    const int K = pms_build_forest(W, H, wR, wD, mR.data(), mD.data(), f, piece, nthreads);
    out[0] = fnv_vec(f.rows);
    out[1] = fnv_vec(f.paths);
    out[2] = fnv_vec(f.items);
    out[3] = fnv_vec(f.rt_path) ^ (fnv_vec(f.rt_item) * 3) ^ (fnv_vec(f.rt_rep) * 5);
    out[4] = fnv_vec(f.cuts) ^ (fnv_vec(f.reps) * 3) ^ (fnv_vec(f.tree_cut) * 5) ^ (fnv_vec(f.cut_round) * 7);
    out[5] = fnv_vec(f.nb_start) ^ (fnv_vec(f.nb) * 3) ^ (fnv_vec(f.tree_rounds) * 5) ^ (uint64_t)f.nrounds;
    if (tree_start) std::memcpy(tree_start, f.tree_start.data(), (K + 1) * sizeof(int32_t));
    if (bfs_pix) std::memcpy(bfs_pix, f.bfs_pix.data(), N * sizeof(int32_t));
    return K;
}

void sm_pms_dice(long n, float* out) {
    uint32_t s = 1u;
    for (long k = 0; k < n; ++k) {
        s = minstd_next(s);
        out[k] = std::fma(canon(s), 2.0f, -1.0f);  // fma(r, b - a, a) (build/StereoYin 0x40ff6b)
    }
}

void sm_pms_glibc_random(unsigned seed, long skip, long n, int32_t* out) {
    GlibcRandom g;
    g.seed_skip(seed, skip);
    g.draw(n, out);
}

void sm_pms_init_labels(int W, int H, int max_disp, float* abc) {
    // :397-430 with distribution(0, 1) over a fresh default-seeded engine; arithmetic of
    // build/StereoYin 0x4125ea-0x4127f7 (squares reused, nz^2 by two fnma, c by two fma)
    uint32_t s = 1u;
    const float fmax = (float)max_disp;
    auto dice = [&s]() {
        s = minstd_next(s);
        return canon(s);
    };
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const size_t i = (size_t)y * W + x;
            const float d = dice() * fmax;
            float x1, x2, s1, s2;
            for (;;) {
                x1 = dice();
                x2 = dice();
                s1 = x1 * x1;
                s2 = x2 * x2;
                if (s1 + s2 < 1.0f) break;
            }
            const float root = std::sqrt((1.0f - s1) - s2);
            const float nx = (x1 + x1) * root, ny = (x2 + x2) * root;
            const float nz = std::sqrt(std::fma(-ny, ny, std::fma(-nx, nx, 1.0f)));
            abc[3 * i] = -nx / nz;
            abc[3 * i + 1] = -ny / nz;
            abc[3 * i + 2] = std::fma(nz, d, std::fma((float)x, nx, ny * (float)y)) / nz;
        }
}

int sm_pms_levels(int max_disp) {
    int n = 0;
    for (float md = 0.5f * (float)max_disp; md > 0.1f; md *= 0.5f) ++n;
    return n;
}

}  // extern "C"
