// sm_segment.cpp -- segment mode (finite c): the reference's Felzenszwalb segmentation of the
// 4-connected grid graph, on the host, and its embedding into one spanning tree for the GPU layout.
//
// Reference semantics (include/segment-graph.h:54-89, src/Stereo3DMST.cpp:242-307):
//   * edges (w, a, b): for each pixel a = y*W + x in raster order its right edge (b = a+1), then its
//     down edge (b = a+W); w = |dR|+|dG|+|dB| of the median image (an integer in [0, 765]);
//   * std::sort by (w, a, b); thresholds start at c/1; an edge joins two components iff
//     w <= thr(a) and w <= thr(b), and the joined component's threshold becomes w + c/size
//     (THRESHOLD(size, c) = c/size: float c over an int size, in float; added to the double w);
//   * then the min-size pass over the same sorted edges: two different components are joined when
//     either has fewer than max(2, min_size) pixels (:293-307).
// The joined edges form a forest; Stereo3DMST roots each tree at its first pixel in raster order
// (:342-384, :450-467) and filters every tree on its own.
//
// The order-dependent segmentation is inherently serial (each decision depends on every earlier
// one), so it runs here, on the host: a stable counting sort of the edge ids by weight (the emission
// order is ascending (a, b), so stable by w == std::sort's (w, a, b)), then two union-find sweeps,
// the second over the first's rejected edges only.  The sweep is bound by the latency of its random
// node visits: 8-byte nodes, a weight read off the bucket instead of the pixel, and prefetches of the
// nodes (and their parents) of the edges a few places ahead.
//
// GPU embedding.  The tree layout and filter engine work on one spanning tree rooted at pixel 0.
// For every tree T other than pixel 0's, its root r_T (the first pixel of T in raster order) gets a
// VIRTUAL edge to its left neighbour (x > 0) or, in column 0, to its upper neighbour: both come
// before r_T in raster order, so they lie in other trees whose roots come earlier -- the virtual
// edges link the forest into one tree rooted at pixel 0 in which every T hangs from r_T, i.e. every
// real edge keeps the orientation of T's own rooting.  A virtual edge carries weight code
// SM_VIRTUAL_W = 766, whose tables hold S = 0 and S2 = 1: the up pass folds fma(0, A_up, acc) == acc
// (aggregates are finite and >= +0) and the down pass gives A(r_T) = fma(0, A(p), 1 * A_up(r_T)) ==
// A_up(r_T), the reference's root rule -- the forest filter, bit for bit, with the tree engine
// unchanged.
#include <cstdint>
#include <cstring>
#include <utility>
#include <vector>

#include "sm_segment.h"

namespace {

// union-find node: parent and component size (8 B: the nodes of a 1920x1200 view stay in one CCD's
// L3 together with the last-join weights); roots have parent == self
struct Node {
    uint32_t parent, size;
};

uint32_t find(Node* u, uint32_t x) {
    while (u[x].parent != x) {
        u[x].parent = u[u[x].parent].parent;  // path halving
        x = u[x].parent;
    }
    return x;
}

uint32_t unite(Node* u, uint32_t a, uint32_t b) {  // a, b roots; union by size
    if (u[a].size < u[b].size) std::swap(a, b);
    u[b].parent = a;
    u[a].size += u[b].size;
    return a;
}

}  // namespace

int sm_segment_forest(const uint16_t* wR, const uint16_t* wD, int W, int H, float c, int min_size, uint8_t* mR,
                      uint8_t* mD, uint16_t* fwR, uint16_t* fwD) {
    const uint32_t N = (uint32_t)W * (uint32_t)H;
    // edge id e = 2p + vertical; ids ascend in the reference's emission order
    std::vector<uint32_t> count(SM_VIRTUAL_W + 1, 0u);
    for (uint32_t y = 0, p = 0; y < (uint32_t)H; ++y)
        for (uint32_t x = 0; x < (uint32_t)W; ++x, ++p) {
            if (x + 1 < (uint32_t)W) ++count[wR[p] + 1u];
            if (y + 1 < (uint32_t)H) ++count[wD[p] + 1u];
        }
    for (int w = 0; w < SM_VIRTUAL_W; ++w) count[w + 1] += count[w];
    const uint32_t E = count[SM_VIRTUAL_W];
    std::vector<uint32_t> order(E);
    for (uint32_t y = 0, p = 0; y < (uint32_t)H; ++y)
        for (uint32_t x = 0; x < (uint32_t)W; ++x, ++p) {
            if (x + 1 < (uint32_t)W) order[count[wR[p]]++] = 2u * p;
            if (y + 1 < (uint32_t)H) order[count[wD[p]]++] = 2u * p + 1u;
        }
    // count[w] is now the end of weight w's bucket: the sweep reads an edge's weight off its bucket
    const uint32_t step[2] = {1u, (uint32_t)W};

    std::memset(mR, 0, N);
    std::memset(mD, 0, N);
    uint8_t* mk[2] = {mR, mD};
    std::vector<Node> nodes(N);
    std::vector<uint16_t> wl(N, 0);  // per root: the weight of its last join (thr = wl + c/size)
    Node* u = nodes.data();
    for (uint32_t i = 0; i < N; ++i) u[i] = Node{i, 1u};
    // Threshold of a root: w_last + c/size, the reference's w + THRESHOLD(size, c) set at the root's
    // last join (each join sets it from the joined size; a singleton's is 0 + c/1).  Edges rejected
    // here are the only ones the min-size pass can join (an edge whose ends were one component stays
    // inside one), so they are kept, in order, for it.
    std::vector<uint32_t> rejected;
    rejected.reserve(E / 8);
    uint32_t sets = N, w = 0;
    constexpr uint32_t PF = 16;  // prefetch distance (edges): nodes at PF, their parents at PF/2
    for (uint32_t i = 0; i < E; ++i) {
        if (i + PF < E) {
            const uint32_t e2 = order[i + PF], p2 = e2 >> 1;
            __builtin_prefetch(&u[p2]);
            __builtin_prefetch(&u[p2 + step[e2 & 1u]]);
        }
        if (i + PF / 2 < E) {
            const uint32_t e2 = order[i + PF / 2], p2 = e2 >> 1;
            __builtin_prefetch(&u[u[p2].parent]);
            __builtin_prefetch(&u[u[p2 + step[e2 & 1u]].parent]);
        }
        while (i >= count[w]) ++w;
        const uint32_t e = order[i], pa = e >> 1;
        const uint32_t a = find(u, pa), b = find(u, pa + step[e & 1u]);
        if (a == b) continue;
        const double wd = (double)w;
        const bool ja = wd <= (double)wl[a] + (double)(c / (float)u[a].size);
        const bool jb = wd <= (double)wl[b] + (double)(c / (float)u[b].size);
        if (ja & jb) {
            wl[unite(u, a, b)] = (uint16_t)w;
            mk[e & 1u][pa] = 1;
            --sets;
        } else {
            rejected.push_back(e);
        }
    }
    const uint32_t ms = (uint32_t)(min_size < 2 ? 2 : min_size);
    for (size_t i = 0; i < rejected.size() && sets > 1; ++i) {
        const uint32_t e = rejected[i], pa = e >> 1;
        const uint32_t a = find(u, pa), b = find(u, pa + step[e & 1u]);
        if (a != b && (u[a].size < ms || u[b].size < ms)) {
            unite(u, a, b);
            mk[e & 1u][pa] = 1;
            --sets;
        }
    }
    // layout weights: the real weights, and SM_VIRTUAL_W on the edges that link each tree's root to
    // an earlier tree
    std::memcpy(fwR, wR, N * sizeof(uint16_t));
    std::memcpy(fwD, wD, N * sizeof(uint16_t));
    std::vector<uint8_t> seen(N, 0);
    int ntrees = 0;
    for (uint32_t p = 0; p < N; ++p) {
        const uint32_t r = find(u, p);
        if (seen[r]) continue;
        seen[r] = 1;
        ++ntrees;
        if (p == 0) continue;
        if (p % (uint32_t)W > 0) {
            mR[p - 1] = 1;
            fwR[p - 1] = SM_VIRTUAL_W;
        } else {
            mD[p - (uint32_t)W] = 1;
            fwD[p - (uint32_t)W] = SM_VIRTUAL_W;
        }
    }
    return ntrees;
}
