// min-size merge microbench (host only): the merge over every candidate (loc table) vs dense ids vs the first
// candidate of each root pair, on synthetic C2 weights dumped to /tmp/segmb.
// g++ -O2 -march=native tools/microbench/seg_merge_mb.cpp -o /tmp/segmb/mb
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>
struct SegMin { uint32_t id, w, ra, rb, sa, sb; };
struct Node { uint32_t parent, size; };
static uint32_t find(Node* u, uint32_t x) { while (u[x].parent != x) { u[x].parent = u[u[x].parent].parent; x = u[x].parent; } return x; }
static double now() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int merge_loc(const SegMin* e, uint32_t n, uint32_t ms, uint32_t* out, std::vector<uint32_t>& loc) {
    std::vector<uint32_t> par, size, root;
    par.reserve(2 * (size_t)n); size.reserve(2 * (size_t)n); root.reserve(2 * (size_t)n);
    auto local = [&](uint32_t r, uint32_t s) { uint32_t& l = loc[r]; if (l == 0xFFFFFFFFu) { l = (uint32_t)par.size(); par.push_back(l); size.push_back(s); root.push_back(r); } return l; };
    auto fnd = [&](uint32_t x) { while (par[x] != x) x = par[x] = par[par[x]]; return x; };
    std::vector<uint32_t> ids; int k = 0;
    for (uint32_t j = 0; j < n; ++j) {
        const SegMin& m = e[j];
        uint32_t a = fnd(local(m.ra, m.sa)), b = fnd(local(m.rb, m.sb));
        if (a == b || (size[a] >= ms && size[b] >= ms)) continue;
        if (size[a] < size[b]) std::swap(a, b);
        par[b] = a; size[a] += size[b];
        out[2 * k] = root[b]; out[2 * k + 1] = root[a]; ids.push_back(m.id); ++k;
    }
    for (int i = 0; i < k; ++i) out[2 * k + i] = ids[i];
    for (uint32_t r : root) loc[r] = 0xFFFFFFFFu;
    return k;
}
struct Dense { uint32_t la, lb, id; };
// dense: la/lb local ids from the GPU; lsize[nl] initial sizes; lroot[nl] roots
int merge_dense(const Dense* e, uint32_t n, uint32_t nl, const uint32_t* lsize, const uint32_t* lroot, uint32_t ms, uint32_t* out,
                std::vector<uint32_t>& par, std::vector<uint32_t>& size) {
    par.resize(nl); size.assign(lsize, lsize + nl);
    for (uint32_t i = 0; i < nl; ++i) par[i] = i;
    uint32_t* P = par.data(); uint32_t* S = size.data();
    auto fnd = [&](uint32_t x) { while (P[x] != x) x = P[x] = P[P[x]]; return x; };
    int k = 0;
    uint32_t* ids = out + 2 * (size_t)n;  // scratch after the pairs' maximum
    for (uint32_t j = 0; j < n; ++j) {
        if (j + 16 < n) { __builtin_prefetch(&P[e[j + 16].la]); __builtin_prefetch(&P[e[j + 16].lb]); }
        uint32_t a = fnd(e[j].la), b = fnd(e[j].lb);
        if (a == b) continue;
        uint32_t sa = S[a], sb = S[b];
        if (sa >= ms && sb >= ms) continue;
        if (sa < sb) { std::swap(a, b); std::swap(sa, sb); }
        P[b] = a; S[a] = sa + sb;
        out[2 * k] = lroot[b]; out[2 * k + 1] = lroot[a]; ids[k] = e[j].id; ++k;
    }
    memmove(out + 2 * k, ids, k * 4);
    return k;
}

int main(int argc, char** argv) {
    const int W = 1920, H = 1200; const uint32_t N = W * H; const float c = 5000; const uint32_t ms = 200;
    for (const char* v : {"l", "r"}) {
        std::vector<uint16_t> wR(N), wD(N);
        char fn[64];
        snprintf(fn, 64, "/tmp/segmb/wR_%s", v); FILE* f = fopen(fn, "rb"); fread(wR.data(), 2, N, f); fclose(f);
        snprintf(fn, 64, "/tmp/segmb/wD_%s", v); f = fopen(fn, "rb"); fread(wD.data(), 2, N, f); fclose(f);
        std::vector<uint32_t> ids;
        for (uint32_t p = 0; p < N; ++p) { if (p % W + 1 < (uint32_t)W) ids.push_back(2 * p); if (p / W + 1 < (uint32_t)H) ids.push_back(2 * p + 1); }
        auto wof = [&](uint32_t e) { return (e & 1) ? wD[e >> 1] : wR[e >> 1]; };
        std::stable_sort(ids.begin(), ids.end(), [&](uint32_t a, uint32_t b) { return wof(a) < wof(b); });
        std::vector<Node> u(N); for (uint32_t i = 0; i < N; ++i) u[i] = {i, 1};
        std::vector<uint16_t> wl(N, 0); std::vector<uint32_t> rej;
        for (uint32_t e : ids) {
            uint32_t pa = e >> 1, a = find(u.data(), pa), b = find(u.data(), pa + ((e & 1) ? W : 1));
            if (a == b) continue; uint32_t w = wof(e);
            bool ja = (double)w <= (double)wl[a] + (double)(c / (float)u[a].size), jb = (double)w <= (double)wl[b] + (double)(c / (float)u[b].size);
            if (ja && jb) { if (u[a].size < u[b].size) std::swap(a, b); u[b].parent = a; u[a].size += u[b].size; wl[a] = w; } else rej.push_back(e);
        }
        std::vector<SegMin> cand;
        for (uint32_t e : rej) {
            uint32_t pa = e >> 1, a = find(u.data(), pa), b = find(u.data(), pa + ((e & 1) ? W : 1));
            SegMin m{e, wof(e), a, b, u[a].size, u[b].size};
            if (m.sa < ms || m.sb < ms) cand.push_back(m);
        }
        std::sort(cand.begin(), cand.end(), [](const SegMin& a, const SegMin& b) { return a.w != b.w ? a.w < b.w : a.id < b.id; });
        const uint32_t n = cand.size();
        // dense ids (as the GPU would: mark + scan over N)
        std::vector<uint32_t> mark(N + 1, 0);
        for (auto& m : cand) { mark[m.ra] = 1; mark[m.rb] = 1; }
        std::vector<uint32_t> lid(N + 1); uint32_t nl = 0; for (uint32_t i = 0; i < N; ++i) { lid[i] = nl; nl += mark[i]; }
        std::vector<uint32_t> lsize(nl), lroot(nl); std::vector<Dense> de(n);
        for (uint32_t j = 0; j < n; ++j) { auto& m = cand[j]; de[j] = {lid[m.ra], lid[m.rb], m.id}; lsize[lid[m.ra]] = m.sa; lsize[lid[m.rb]] = m.sb; lroot[lid[m.ra]] = m.ra; lroot[lid[m.rb]] = m.rb; }
        std::vector<uint32_t> loc(N, 0xFFFFFFFFu), o1(3 * n + 1), o2(3 * n + 1), par, size;
        int k1 = 0, k2 = 0; double t1 = 1e9, t2 = 1e9;
        for (int rep = 0; rep < 7; ++rep) {
            double t = now(); k1 = merge_loc(cand.data(), n, ms, o1.data(), loc); t1 = std::min(t1, now() - t);
            t = now(); k2 = merge_dense(de.data(), n, nl, lsize.data(), lroot.data(), ms, o2.data(), par, size); t2 = std::min(t2, now() - t);
        }
        // first occurrence of each unordered local pair, in order
        std::vector<Dense> uq; {
            std::vector<unsigned long long> key(n); for (uint32_t j = 0; j < n; ++j) { uint32_t x = std::min(de[j].la, de[j].lb), y = std::max(de[j].la, de[j].lb); key[j] = ((unsigned long long)x << 32) | y; }
            std::vector<uint32_t> ord(n); for (uint32_t j = 0; j < n; ++j) ord[j] = j;
            std::stable_sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) { return key[a] < key[b]; });
            std::vector<uint8_t> keep(n, 0); for (uint32_t i = 0; i < n; ++i) if (i == 0 || key[ord[i]] != key[ord[i - 1]]) keep[ord[i]] = 1;
            for (uint32_t j = 0; j < n; ++j) if (keep[j]) uq.push_back(de[j]);
        }
        std::vector<uint32_t> o3(3 * n + 1); int k3 = 0; double t3 = 1e9;
        for (int rep = 0; rep < 7; ++rep) { double t = now(); k3 = merge_dense(uq.data(), uq.size(), nl, lsize.data(), lroot.data(), ms, o3.data(), par, size); t3 = std::min(t3, now() - t); }
        printf("  unique pairs %zu: dense-unique %.3f ms, same %d\n", uq.size(), t3, k3 == k1 && !memcmp(o1.data(), o3.data(), 3 * (size_t)k1 * 4));
        // compare: the joined edge id sets and the hooks (pairs may differ only by tie order? they should be identical)
        bool same = k1 == k2 && !memcmp(o1.data(), o2.data(), 3 * (size_t)k1 * 4);
        printf("view %s: rejected %zu candidates %u local %u joins %d | loc-table %.2f ms, dense %.2f ms, same %d\n", v, rej.size(), n, nl, k1, t1, t2, same);
    }
}
