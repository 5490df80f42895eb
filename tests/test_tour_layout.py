"""CPU check of the arithmetic behind the tree layout's preorder (stereomatch_amd/csrc/sm_layout_gpu.hip,
round 5): on random spanning trees of small grids, the MST tour (k_tour_tile's successor rule: leave a pixel
through the next tree direction after the one it arrived from, cut before the start arc), ranks from
suffixes, k_orient's orientation / subtree sizes / heavy child and its 32-bit tour values
(light << 27 | preorder offset, negated going up, summed mod 2^32), the tour scan's epilogue
(ScanTourOut: hk = (1 + position) << 5 | light depth at a path head, 0 elsewhere), the 32-bit max-scan
of hk and the path histogram's end-of-path rule (ScanPathCount) give exactly the heavy-first preorder of
the tree rooted at pixel 0 (Stereo3DMST.cpp:454-467's root), its light depths and its heavy paths.
A pure-Python restatement of the kernels' index arithmetic; the GPU build itself is checked end to end
by the -m gpu parity tests (bit-exact matches need the exact layout)."""
import random

import pytest

MASK = 0xFFFFFFFF
SHIFT = 27


def nbr(p, k, W):
    return p + 1 if k == 0 else p + W if k == 1 else p - 1 if k == 2 else p - W


def random_tree(W, H, seed):
    """Kruskal over random small-integer weights (ties by edge id): a spanning tree of the grid, as
    adjacency bits (1 right, 2 down, 4 left, 8 up)."""
    rng = random.Random(seed)
    N = W * H
    edges = []
    for p in range(N):
        if p % W + 1 < W:
            edges.append((rng.randrange(8), p, 0))
        if p + W < N:
            edges.append((rng.randrange(8), p, 1))
    edges.sort()
    par = list(range(N))

    def find(a):
        while par[a] != a:
            par[a] = par[par[a]]
            a = par[a]
        return a
    adj = [0] * N
    for _, a, vert in edges:
        b = a + (W if vert else 1)
        ra, rb = find(a), find(b)
        if ra == rb:
            continue
        par[ra] = rb
        adj[a] |= 2 if vert else 1
        adj[b] |= 8 if vert else 4
    return adj


def gpu_layout(adj, W, H):
    N = W * H
    start = next(k for k in range(4) if adj[0] >> k & 1)

    def succ(a):
        p, k = a >> 2, a & 3
        q = nbr(p, k, W)
        j = (k + 2) & 3
        kk = j
        for t in range(1, 5):
            if adj[q] >> ((j + t) & 3) & 1:
                kk = (j + t) & 3
                break
        s = 4 * q + kk
        return None if s == start else s
    order, a = [], start
    while a is not None:
        order.append(a)
        a = succ(a)
    total = 2 * N - 2
    assert len(order) == total
    suffix = {arc: total - i for i, arc in enumerate(order)}
    tour, arcpix = [0] * total, [0] * total
    hk, pixpre = [None] * N, [None] * N
    for v in range(N):  # k_orient
        pd, heavy, best, csz, crio = -1, -1, 0, [0] * 4, [None] * 4
        for k in range(4):
            if not adj[v] >> k & 1:
                continue
            n = nbr(v, k, W)
            si, so = suffix[4 * n + ((k + 2) & 3)], suffix[4 * v + k]
            if si > so:
                pd = k
            else:
                csz[k] = (so - si + 1) // 2
                crio[k] = (total - so, total - si)
                if csz[k] > best:
                    best, heavy = csz[k], k
        if pd < 0:
            hk[0], pixpre[0] = (1 << 5) | 0, v
        off = 1 + (csz[heavy] if heavy >= 0 else 0)
        for k in range(4):
            if not adj[v] >> k & 1 or k == pd:
                continue
            val = 1
            if k != heavy:
                val = (1 << SHIFT) + off
                off += csz[k]
            tour[crio[k][0]] = val
            tour[crio[k][1]] = (-val) & MASK
            arcpix[crio[k][0]] = nbr(v, k, W)
    acc = 0
    for i, x in enumerate(tour):  # the 32-bit add-scan and ScanTourOut
        acc = (acc + x) & MASK
        if x >= 1 << 31:
            continue
        pre, ld = acc & ((1 << SHIFT) - 1), acc >> SHIFT
        assert pre < N and ld < 32 and hk[pre] is None
        hk[pre] = ((pre + 1) << 5 | ld) if x != 1 else 0
        pixpre[pre] = arcpix[i]
    raw = list(hk)
    m = 0
    for i in range(N):  # the max-scan (in place)
        m = max(m, hk[i])
        hk[i] = m
    paths = []
    for s in range(N):  # ScanPathCount's rule: s ends its path iff s + 1 holds a head's record
        nxt = s + 1 == N or raw[s + 1] != 0
        assert nxt == (s + 1 == N or (hk[s + 1] >> 5) == s + 2)  # the stored-value test, either state
        if nxt:
            head, ld = (hk[s] >> 5) - 1, hk[s] & 31
            paths.append((head, s - head + 1, ld))
    return pixpre, paths


def reference_layout(adj, W, H):
    """Heavy-first preorder from pixel 0 by DFS: the heavy child (largest subtree, ties to the smallest
    direction) right after its parent, then the light children in direction order."""
    N = W * H
    parent, kids, order = [-1] * N, [[] for _ in range(N)], []
    stack, seen = [0], [False] * N
    seen[0] = True
    while stack:
        v = stack.pop()
        order.append(v)
        for k in range(4):
            if adj[v] >> k & 1:
                c = nbr(v, k, W)
                if not seen[c]:
                    seen[c] = True
                    parent[c] = v
                    kids[v].append((k, c))
                    stack.append(c)
    size = [1] * N
    for v in reversed(order):
        if parent[v] >= 0:
            size[parent[v]] += size[v]
    pre, ldepth, paths = [], {}, []

    def visit(v, ld, head):
        pre.append(v)
        ldepth[v] = ld
        ks = sorted(kids[v])
        heavy = None
        for k, c in ks:
            if heavy is None or size[c] > size[heavy[1]]:
                heavy = (k, c)
        if heavy is None:
            paths.append(head)
        else:
            visit(heavy[1], ld, head)
        for k, c in ks:
            if (k, c) != heavy:
                visit(c, ld + 1, (len(pre), ld + 1))
    import sys
    sys.setrecursionlimit(10000)
    visit(0, 0, (0, 0))
    # paths as (head position, length, light depth), in preorder of their heads
    heads = sorted(set(paths))
    bounds = [h[0] for h in heads] + [N]
    return pre, [(h[0], bounds[i + 1] - h[0], h[1]) for i, h in enumerate(heads)]


@pytest.mark.parametrize("W,H,seed", [(5, 4, 1), (16, 9, 2), (13, 11, 3), (40, 3, 4), (1, 17, 5), (23, 1, 6),
                                      (33, 34, 7), (64, 48, 8)])
def test_tour_layout_matches_heavy_first_preorder(W, H, seed):
    if W * H < 2:
        pytest.skip("one pixel: no tour")
    adj = random_tree(W, H, seed)
    pixpre, paths = gpu_layout(adj, W, H)
    pre, ref_paths = reference_layout(adj, W, H)
    assert pixpre == pre
    assert paths == ref_paths
