"""How much of the short-path (walker) work sits in subtrees that contain no long path (CPU only).

Such a subtree needs nothing from the chain engine in either pass, so a walker could process all of its
light-depth rounds on its own, deepest first (verdict item 1).  Builds one view's MST with
the oracle (oracle/oracle.py build_tree: median, edge weights, Kruskal, BFS rooting), decomposes it into
heavy paths as the layout does (heavy child = largest subtree), and reports:
  * the short-path nodes inside maximal long-path-free subtrees, their count and sizes;
  * per light depth, the short nodes whose path has a long path below it ("late": they need the chains).

    python tools/subtree_stats.py [W H]      (default 1920 1200: C2, the left view of tools/synth's pair)
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O  # noqa: E402  (test infrastructure: a statistics tool, not the product)
from tools.synth import make_pair  # noqa: E402

LONG = 32  # SM_LONG_PATH


def main():
    W, H = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (1920, 1200)
    left, _, _ = make_pair(W, H, 128, index=0)
    t = O.build_tree(left)
    assert t["ntrees"] == 1
    N = W * H
    par = t["node_parent"]
    nch = t["node_nch"]
    ch = t["node_child"].reshape(N, 4)
    size = np.ones(N, np.int64)
    for v in range(N - 1, 0, -1):  # BFS order: children after parents
        size[par[v]] += size[v]
    heavy = np.full(N, -1, np.int64)
    for v in np.nonzero(nch)[0]:
        cs = ch[v, :nch[v]]
        heavy[v] = cs[np.argmax(size[cs])]
    head = np.zeros(N, np.int64)
    ld = np.zeros(N, np.int64)
    for v in range(N):  # BFS order: a parent's head and light depth are final before its children's
        if v == 0:
            continue
        p = par[v]
        if heavy[p] == v:
            head[v], ld[v] = head[p], ld[p]
        else:
            head[v], ld[v] = v, ld[p] + 1
    plen = np.bincount(head, minlength=N)
    onlong = plen[head] >= LONG
    # long nodes below (or at) each node
    below = onlong.astype(np.int64)
    for v in range(N - 1, 0, -1):
        below[par[v]] += below[v]
    free = below == 0  # the node's subtree has no long-path node
    short = ~onlong
    roots = np.nonzero(free & (np.arange(N) > 0) & ~free[np.maximum(par, 0)])[0]
    sz = np.sort(size[roots])[::-1]
    ns, nf = int(short.sum()), int((short & free).sum())
    print("%dx%d: %d nodes, %d short-path nodes, %d of them (%.3f%%) in %d long-path-free subtrees" %
          (W, H, N, ns, nf, 100.0 * nf / ns, len(roots)))
    print("subtree sizes: largest %s, mean %.1f" % ([int(x) for x in sz[:8]], sz.mean()))
    for r in range(int(ld.max()) + 1):
        m = (ld == r) & short
        print("  light depth %2d: short nodes %8d, late (a long path below) %6d" % (r, int(m.sum()), int((m & ~free).sum())))


if __name__ == "__main__":
    main()
