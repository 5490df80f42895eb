"""CPU check of the argument behind the MST_PMS forest's BFS numbering by Euler tours
(stereomatch_amd/csrc/sm_pms_forest.hip, "BFS"): on random spanning forests of small grids, the two
tours with the kernels' rotation words, the per-tree list ranks, the int64 prefix sum (+1|+1 down,
-1 up) and a stable sort of the preorder sequence by (tree, depth) give exactly the reference's BFS
(Stereo3DMST.cpp:450-522: root = first raster pixel, children in ascending (w, a, b) key order),
plus subtree sizes and parents.  A pure-Python restatement of the kernels' index arithmetic; the GPU
build itself is checked array by array against the host construction in tests/test_pms_gpu.py."""
import random
from collections import deque

import pytest

END = 4


def nbr(p, k, W):
    return p + 1 if k == 0 else p + W if k == 1 else p - 1 if k == 2 else p - W


def direction(p, n, W):
    return 0 if n == p + 1 else 1 if n == p + W else 2 if n == p - 1 else 3


def random_forest(W, H, seed, keep=0.9):
    """Kruskal on random weights (ties by id) over the grid, each MST edge kept with prob `keep`:
    a spanning forest; weights are small integers so ties are frequent (the key breaks them)."""
    rng = random.Random(seed)
    N = W * H
    edges = []
    for p in range(N):
        x = p % W
        if x + 1 < W:
            edges.append((rng.randrange(6), p, 0))
        if p + W < N:
            edges.append((rng.randrange(6), p, 1))
    edges.sort()
    par = list(range(N))

    def find(a):
        while par[a] != a:
            par[a] = par[par[a]]
            a = par[a]
        return a
    adj = [[] for _ in range(N)]  # (key, neighbour)
    for w, a, vert in edges:
        b = a + (W if vert else 1)
        ra, rb = find(a), find(b)
        if ra == rb or rng.random() > keep:
            continue
        par[ra] = rb
        key = (w, a, vert)
        adj[a].append((key, b))
        adj[b].append((key, a))
    for lst in adj:
        lst.sort()
    return [[n for _, n in lst] for lst in adj]


def reference_bfs(nb, N):
    """Trees in first-pixel order; per tree its BFS list (children in key order)."""
    seen = [False] * N
    trees = []
    for r in range(N):
        if seen[r]:
            continue
        seen[r] = True
        order, q = [], deque([(r, -1)])
        while q:
            v, p = q.popleft()
            order.append(v)
            for c in nb[v]:
                if c != p:
                    seen[c] = True
                    q.append((c, v))
        trees.append(order)
    return trees


def rank_lists(rot, N, W):
    """List ranking of the tour given by rotation words: rot[q] = {arrival dir: next dir or END}.
    Returns suffix[a] = arcs from a to its list's end, inclusive (what tour_suffix computes)."""
    succ = {}
    for p in range(N):
        for k in rot[p]:
            q = nbr(p, k, W)
            nd = rot[q][(k + 2) & 3]
            succ[4 * p + k] = None if nd == END else 4 * q + nd
    pred = {s: a for a, s in succ.items() if s is not None}
    suffix = {}
    for a in succ:
        if a in pred:
            continue
        lst, x = [], a
        while x is not None:
            lst.append(x)
            x = succ[x]
        for i, y in enumerate(lst):
            suffix[y] = len(lst) - i
    return suffix


def tour_bfs(nb, N, W):
    # union-find roots: a tree's first pixel; tree ids in root order
    root_of = [-1] * N
    for r in range(N):
        if root_of[r] >= 0:
            continue
        stack = [r]
        root_of[r] = r
        while stack:
            v = stack.pop()
            for c in nb[v]:
                if root_of[c] < 0:
                    root_of[c] = r
                    stack.append(c)
    roots = sorted(set(root_of))
    tid = {r: i for i, r in enumerate(roots)}
    tree_of = [tid[root_of[p]] for p in range(N)]
    K = len(roots)
    tsize = [0] * K
    for p in range(N):
        tsize[tree_of[p]] += 1
    tree_start = [0] * (K + 1)
    for t in range(K):
        tree_start[t + 1] = tree_start[t] + tsize[t]
    dirs = [[direction(p, n, W) for n in nb[p]] for p in range(N)]
    # tour 1 (k_pf_rot1): cyclic key order, the root ends its list after its last neighbour
    rot1 = []
    for p in range(N):
        d, c, r = dirs[p], len(dirs[p]), {}
        for i in range(c):
            r[d[i]] = END if (root_of[p] == p and i == c - 1) else d[(i + 1) % c]
        rot1.append(r)
    suf = rank_lists(rot1, N, W)
    # k_pf_orient
    pdir, psize = [-1] * N, [0] * N
    for q in range(N):
        psize[q] = tsize[tree_of[q]]
        for k in dirs[q]:
            p = nbr(q, k, W)
            si, so = suf[4 * p + ((k + 2) & 3)], suf[4 * q + k]
            if si > so:
                pdir[q] = k
                psize[q] = (si - so + 1) // 2
    # tour 2 (k_pf_rot2): children in key order, then the parent (the root: the end)
    rot2 = []
    for p in range(N):
        r, prev, pd = {}, pdir[p], pdir[p]
        for k in dirs[p]:
            if k == pd:
                continue
            if prev >= 0:
                r[prev] = k
            prev = k
        if prev >= 0:
            r[prev] = pd if pd >= 0 else END
        rot2.append(r)
    suf2 = rank_lists(rot2, N, W)
    # k_pf_tourval + the inclusive scan
    tval = [0] * (2 * (N - K))
    for p in range(N):
        t = tree_of[p]
        ln, base = 2 * (tsize[t] - 1), 2 * (tree_start[t] - t)
        for k in dirs[p]:
            q = nbr(p, k, W)
            down = pdir[q] == ((k + 2) & 3)
            tval[base + ln - suf2[4 * p + k]] = (1 << 32) | 1 if down else -(1 << 32)
    s, scan = 0, []
    for x in tval:
        s += x
        scan.append(s)
    # k_pf_depth, then the stable sort by (tree, depth)
    seq = [None] * N
    for q in range(N):
        t, pd = tree_of[q], pdir[q]
        depth = pre = 0
        if pd >= 0:
            p = nbr(q, pd, W)
            pos = 2 * (tree_start[t] - t) + 2 * (tsize[t] - 1) - suf2[4 * p + ((pd + 2) & 3)]
            v = scan[pos]
            depth, pre = v >> 32, (v & 0xFFFFFFFF) - (tree_start[t] - t)
        g = tree_start[t] + pre
        assert seq[g] is None
        seq[g] = ((t, depth), q)
    order = [q for _, q in sorted(seq, key=lambda e: e[0])]  # Python's sort is stable
    parent = [nbr(q, pdir[q], W) if pdir[q] >= 0 else -1 for q in range(N)]
    return order, tree_start, psize, parent


def subtree_sizes(nb, trees, N):
    size, parent = [1] * N, [-1] * N
    for order in trees:
        pos = {v: i for i, v in enumerate(order)}
        for v in order:
            for c in nb[v]:
                if pos[c] > pos[v]:
                    parent[c] = v
        for v in reversed(order):
            if parent[v] >= 0:
                size[parent[v]] += size[v]
    return size, parent


@pytest.mark.parametrize("W,H,keep,seed", [(7, 5, 1.0, 1), (16, 9, 0.9, 2), (13, 11, 0.6, 3), (40, 3, 0.95, 4),
                                           (1, 17, 1.0, 5), (23, 1, 0.8, 6), (33, 34, 0.97, 7), (9, 9, 0.0, 8)])
def test_tour_bfs_matches_reference_bfs(W, H, keep, seed):
    N = W * H
    nb = random_forest(W, H, seed, keep)
    trees = reference_bfs(nb, N)
    order, tree_start, psize, parent = tour_bfs(nb, N, W)
    assert order == [v for t in trees for v in t]
    assert tree_start[1:] == [sum(len(t) for t in trees[:i + 1]) for i in range(len(trees))]
    size, par = subtree_sizes(nb, trees, N)
    assert psize == size
    assert parent == par
