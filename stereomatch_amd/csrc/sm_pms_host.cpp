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

#include <algorithm>
#include <cmath>
#include <cstring>

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

int pms_build_forest(int W, int H, const uint16_t* wR, const uint16_t* wD, const uint8_t* mR, const uint8_t* mD,
                     PmsForest& f, int piece) {
    const int N = W * H;
    Bfs b;
    bfs_forest(W, H, wR, wD, mR, mD, b);
    const int K = (int)b.tree_start.size() - 1;
    f.W = W;
    f.H = H;
    f.K = K;
    f.tree_start = b.tree_start;
    f.bfs_pix = b.pix;
    tree_graph(W, H, b, f.nb_start, f.nb);

    // heavy paths: subtree sizes (children have larger BFS ids), heavy child = the largest subtree
    // (ties: the smallest BFS id), light depth
    std::vector<int32_t> size(N, 1), heavy(N, -1), ld(N, 0);
    for (int n = N - 1; n >= 0; --n)
        if (b.parent[n] != n) size[b.parent[n]] += size[n];
    for (int n = 0; n < N; ++n) {
        int best = -1;
        for (int i = 0; i < b.nch[n]; ++i) {
            const int c = b.child[4 * (size_t)n + i];
            if (best < 0 || size[c] > size[best]) best = c;
        }
        heavy[n] = best;
        for (int i = 0; i < b.nch[n]; ++i) {
            const int c = b.child[4 * (size_t)n + i];
            ld[c] = ld[n] + (c == best ? 0 : 1);
        }
    }
    // rows: per tree, heads by (light depth, BFS id), each path head-first
    std::vector<int32_t> rowof(N, -1), tmaxld(K, 0);
    std::vector<int32_t> heads;
    std::vector<PmsPath> tpaths;  // per-tree paths in row order (by light depth)
    std::vector<int32_t> tpath_start(K + 1, 0), path_ld;
    f.rows.resize(N);
    for (int t = 0; t < K; ++t) {
        const int ts = b.tree_start[t], te = b.tree_start[t + 1];
        heads.clear();
        int mld = 0;
        for (int n = ts; n < te; ++n)
            if (n == ts || heavy[b.parent[n]] != n) {
                heads.push_back(n);
                mld = std::max(mld, ld[n]);
            }
        tmaxld[t] = mld;
        std::stable_sort(heads.begin(), heads.end(), [&](int a, int c) { return ld[a] < ld[c]; });
        int row = ts;
        for (int h : heads) {
            const int r0 = row;
            for (int n = h; n >= 0; n = heavy[n]) rowof[n] = row++;
            tpaths.push_back(PmsPath{t, r0, row - r0, 0});
            path_ld.push_back(ld[h]);
        }
        tpath_start[t + 1] = (int32_t)tpaths.size();
    }
    for (int n = 0; n < N; ++n) {
        PmsRow& R = f.rows[rowof[n]];
        const int p = b.pix[n];
        R.pix = p;
        R.x = (uint16_t)(p % W);
        R.y = (uint16_t)(p / W);
        R.parent = b.parent[n] == n ? -1 : rowof[b.parent[n]];
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
    // cut paths (tree order)
    f.piece = piece > 0 ? piece : 0;
    f.cuts.clear();
    f.cut_round.clear();
    f.tree_cut.assign(K + 1, 0);
    std::vector<int32_t> cut_of(tpaths.size(), -1);
    for (int t = 0; t < K; ++t) {
        f.tree_cut[t] = (int32_t)f.cuts.size();
        if (f.piece == 0) continue;
        for (int i = tpath_start[t]; i < tpath_start[t + 1]; ++i)
            if (tpaths[i].len >= 2 * f.piece) {
                cut_of[i] = (int32_t)f.cuts.size();
                f.cuts.push_back(PmsCut{t, tpaths[i].row, tpaths[i].len, tpaths[i].len / f.piece});
                f.cut_round.push_back(path_ld[i]);
            }
    }
    f.tree_cut[K] = (int32_t)f.cuts.size();
    // round-major path, item and repair lists
    int rmax = 0;
    for (int t = 0; t < K; ++t) rmax = std::max(rmax, tmaxld[t] + 1);
    f.nrounds = rmax;
    f.tree_rounds.resize(K);
    for (int t = 0; t < K; ++t) f.tree_rounds[t] = tmaxld[t] + 1;
    f.rt_path.assign((size_t)rmax * (K + 1), 0);
    f.rt_item.assign((size_t)rmax * (K + 1), 0);
    f.rt_rep.assign((size_t)rmax * (K + 1), 0);
    f.paths.clear();
    f.items.clear();
    f.reps.clear();
    std::vector<int32_t> cur(tpath_start.begin(), tpath_start.end() - 1);
    for (int r = 0; r < rmax; ++r)
        for (int t = 0; t <= K; ++t) {
            f.rt_path[(size_t)r * (K + 1) + t] = (int32_t)f.paths.size();
            f.rt_item[(size_t)r * (K + 1) + t] = (int32_t)f.items.size();
            f.rt_rep[(size_t)r * (K + 1) + t] = (int32_t)f.reps.size();
            if (t == K) break;
            const int deg = f.nb_start[t + 1] - f.nb_start[t];
            const int chunks = (deg + 63) / 64;
            for (; cur[t] < tpath_start[t + 1] && path_ld[cur[t]] == r; ++cur[t]) {
                const PmsPath pa = tpaths[cur[t]];
                const int c = cut_of[cur[t]];
                const int np = c < 0 ? 1 : f.cuts[c].npieces;
                for (int i = 0; i < np; ++i) {  // the pieces, head first
                    const int r0 = pa.row + i * f.piece;
                    const int len = c < 0 ? pa.len : (i + 1 < np ? f.piece : pa.row + pa.len - r0);
                    const int pi = (int)f.paths.size();
                    f.paths.push_back(PmsPath{t, r0, len, 0});
                    for (int k = 0; k < chunks; ++k) f.items.push_back(PmsItem{pi, k});
                }
                if (c >= 0)
                    for (int k = 0; k < std::max(chunks, 1); ++k) f.reps.push_back(PmsRep{c, k});
            }
        }
    return K;
}

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

void sm_pms_dice(long n, float* out) {
    uint32_t s = 1u;
    for (long k = 0; k < n; ++k) {
        s = minstd_next(s);
        out[k] = std::fma(canon(s), 2.0f, -1.0f);  // fma(r, b - a, a) (build/StereoYin 0x40ff6b)
    }
}

void sm_pms_glibc_random(unsigned seed, long skip, long n, int32_t* out) {
    // TYPE_3 additive feedback generator (degree 31, separation 3): srandom_r fills the state with
    // 16807 * x mod (2^31 - 1) (Schrage), then discards 310 outputs; each output is the new state
    // word shifted right by one.
    int32_t st[31];
    if (seed == 0) seed = 1;
    st[0] = (int32_t)seed;
    long word = (long)seed;
    for (int i = 1; i < 31; ++i) {
        const long hi = word / 127773, lo = word % 127773;
        word = 16807 * lo - 2836 * hi;
        if (word < 0) word += 2147483647;
        st[i] = (int32_t)word;
    }
    int f = 3, r = 0;
    const long first = 310 + skip, total = first + n;
    for (long k = 0; k < total; ++k) {
        const uint32_t v = (uint32_t)st[f] + (uint32_t)st[r];
        st[f] = (int32_t)v;
        if (k >= first) out[k - first] = (int32_t)(v >> 1);
        if (++f >= 31) {
            f = 0;
            ++r;
        } else if (++r >= 31) {
            r = 0;
        }
    }
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
