// sm_layout.cpp -- tree layout (rooting, heavy-light decomposition, slot order, per-slot
// metadata, per-round heavy-path lists) computed from an MST edge mask.
//
// This is the host-side layout stage: the GPU produces the MST (Boruvka) and the edge
// weights; this code roots each tree at its first raster pixel (Stereo3DMST.cpp:454-467),
// orders children by edge key (:436-446, :492-516), and emits the layout the walker kernels
// consume.  It is O(N) and deterministic; DESIGN.md lists moving it onto the GPU
// (Euler tour + list ranking) as the next step for the MST/layout budget.
#include <algorithm>
#include <cstring>
#include <vector>

#include "sm_common.h"
#include "sm_layout.h"

namespace {

inline uint32_t nbr(uint32_t p, int k, int W) {
    switch (k) {
        case 0: return p + 1;
        case 1: return p + (uint32_t)W;
        case 2: return p - 1;
        default: return p - (uint32_t)W;
    }
}

}  // namespace

void sm_build_layout(int W, int H, const uint8_t* mR, const uint8_t* mD, const uint16_t* wR, const uint16_t* wD,
                     SmLayout& L) {
    const uint32_t N = (uint32_t)W * (uint32_t)H;
    // adjacency bits per pixel: bit k set if the MST edge in direction k exists
    std::vector<uint8_t> adj(N, 0);
    for (uint32_t p = 0; p < N; ++p) {
        if (mR[p]) { adj[p] |= 1; adj[p + 1] |= 4; }
        if (mD[p]) { adj[p] |= 2; adj[p + W] |= 8; }
    }
    auto key = [&](uint32_t p, int k) -> uint64_t {
        switch (k) {
            case 0: return sm_edge_key(wR[p], p, 0);
            case 1: return sm_edge_key(wD[p], p, 1);
            case 2: return sm_edge_key(wR[p - 1], p - 1, 0);
            default: return sm_edge_key(wD[p - W], p - W, 1);
        }
    };
    auto wgt = [&](uint32_t p, int k) -> uint32_t { return (uint32_t)(key(p, k) >> 33); };

    // BFS from each root (first raster pixel of each tree) -> parent, order
    std::vector<uint32_t> parent(N, SM_NONE), order;
    std::vector<int8_t> pdir(N, -1);  // direction from node to its parent
    order.reserve(N);
    std::vector<uint8_t> seen(N, 0);
    std::vector<uint32_t> roots;
    for (uint32_t r = 0; r < N; ++r) {
        if (seen[r]) continue;
        roots.push_back(r);
        seen[r] = 1;
        size_t head = order.size();
        order.push_back(r);
        while (head < order.size()) {
            const uint32_t v = order[head++];
            for (int k = 0; k < 4; ++k) {
                if (!(adj[v] & (1u << k))) continue;
                const uint32_t q = nbr(v, k, W);
                if (seen[q]) continue;
                seen[q] = 1;
                parent[q] = v;
                pdir[q] = (int8_t)((k + 2) & 3);
                order.push_back(q);
            }
        }
    }
    // subtree sizes and heavy child (max size; ties -> smallest direction index)
    std::vector<uint32_t> size(N, 1);
    for (size_t i = N; i-- > 0;) {
        const uint32_t v = order[i];
        if (parent[v] != SM_NONE) size[parent[v]] += size[v];
    }
    std::vector<int8_t> heavy(N, -1);
    for (uint32_t v = 0; v < N; ++v) {
        uint32_t best = 0;
        for (int k = 0; k < 4; ++k) {
            if (!(adj[v] & (1u << k)) || k == pdir[v]) continue;
            const uint32_t q = nbr(v, k, W);
            if (size[q] > best) { best = size[q]; heavy[v] = (int8_t)k; }
        }
    }
    // heavy-first preorder and light depth
    std::vector<uint32_t> pre(N), ld(N, 0), stack;
    stack.reserve(1024);
    uint32_t counter = 0;
    uint32_t maxld = 0;
    for (uint32_t r : roots) {
        stack.push_back(r);
        while (!stack.empty()) {
            const uint32_t v = stack.back();
            stack.pop_back();
            pre[v] = counter++;
            // push lights in descending direction (so ascending pops), heavy last (popped first)
            for (int k = 3; k >= 0; --k) {
                if (!(adj[v] & (1u << k)) || k == pdir[v] || k == heavy[v]) continue;
                const uint32_t q = nbr(v, k, W);
                ld[q] = ld[v] + 1;
                maxld = std::max(maxld, ld[q]);
                stack.push_back(q);
            }
            if (heavy[v] >= 0) {
                const uint32_t q = nbr(v, heavy[v], W);
                ld[q] = ld[v];
                stack.push_back(q);
            }
        }
    }
    // slot = rank in (ld, preorder): counting sort by ld over nodes in preorder
    std::vector<uint32_t> by_pre(N);
    for (uint32_t v = 0; v < N; ++v) by_pre[pre[v]] = v;
    const uint32_t nr = maxld + 1;
    std::vector<uint32_t> cnt(nr + 1, 0);
    for (uint32_t v = 0; v < N; ++v) cnt[ld[v] + 1]++;
    for (uint32_t r = 0; r < nr; ++r) cnt[r + 1] += cnt[r];
    L.round_slot_begin.assign(cnt.begin(), cnt.end());
    std::vector<uint32_t> slot(N);
    {
        std::vector<uint32_t> pos(cnt.begin(), cnt.end() - 1);
        for (uint32_t i = 0; i < N; ++i) {
            const uint32_t v = by_pre[i];
            slot[v] = pos[ld[v]]++;
        }
    }
    // per-slot metadata
    L.meta.resize(N);
    L.n_light = 0;
    for (uint32_t v = 0; v < N; ++v) {
        uint64_t ck[4];
        uint32_t cq[4];
        int nch = 0;
        for (int k = 0; k < 4; ++k) {
            if (!(adj[v] & (1u << k)) || k == pdir[v]) continue;
            ck[nch] = key(v, k);
            cq[nch] = (uint32_t)k;
            nch++;
        }
        // descending key order (the reference's up-pass fold order)
        for (int i = 1; i < nch; ++i)
            for (int j = i; j > 0 && ck[j] > ck[j - 1]; --j) { std::swap(ck[j], ck[j - 1]); std::swap(cq[j], cq[j - 1]); }
        uint32_t cw[4] = {0, 0, 0, 0}, cs[4] = {SM_NONE, SM_NONE, SM_NONE, SM_NONE};
        uint32_t hidx = 0, has_light = 0;
        for (int i = 0; i < nch; ++i) {
            cw[i] = (uint32_t)(ck[i] >> 33);
            cs[i] = slot[nbr(v, (int)cq[i], W)];
            if ((int)cq[i] == heavy[v]) hidx = (uint32_t)i; else has_light = 1;
        }
        L.n_light += (uint32_t)(nch - (heavy[v] >= 0 ? 1 : 0));
        const uint32_t wp = parent[v] == SM_NONE ? 0u : wgt(v, pdir[v]);
        L.meta[slot[v]] = sm_make_meta(v, parent[v] == SM_NONE ? SM_NONE : slot[parent[v]], wp, cw, (uint32_t)nch, hidx,
                                       has_light, cs);
    }
    // heavy paths per round: heads are roots and light children; len by following heavy chains
    std::vector<std::vector<SmPath>> per_round(nr);
    for (uint32_t v = 0; v < N; ++v) {
        bool is_head;
        if (parent[v] == SM_NONE) {
            is_head = true;
        } else {
            const uint32_t p = parent[v];
            is_head = heavy[p] < 0 || nbr(p, heavy[p], W) != v;
        }
        if (!is_head) continue;
        uint32_t len = 1, u = v;
        while (heavy[u] >= 0) { u = nbr(u, heavy[u], W); ++len; }
        per_round[ld[v]].push_back(SmPath{slot[v], len});
    }
    L.paths.clear();
    L.round_path_begin.assign(nr + 1, 0);
    L.max_path_len.assign(nr, 0);
    for (uint32_t r = 0; r < nr; ++r) {
        auto& P = per_round[r];
        std::stable_sort(P.begin(), P.end(), [](const SmPath& a, const SmPath& b) { return a.len > b.len; });
        L.round_path_begin[r] = (uint32_t)L.paths.size();
        if (!P.empty()) L.max_path_len[r] = P[0].len;
        L.paths.insert(L.paths.end(), P.begin(), P.end());
    }
    L.round_path_begin[nr] = (uint32_t)L.paths.size();
    L.nrounds = nr;
    L.nroots = (uint32_t)roots.size();
    L.parent_pix.assign(parent.begin(), parent.end());
    L.subtree_size.assign(size.begin(), size.end());
    L.slot_of_pix.assign(slot.begin(), slot.end());
}
