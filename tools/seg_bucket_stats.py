"""Analysis only (CPU, not part of any GPU run): per weight bucket of segment mode's sweep,
the bucket's edges, its candidates (open-open edges between two components) and the crossing candidates
left after each Boruvka round, on the bench's synthetic C2 left image -- i.e. how much work the
one-workgroup tail (k_seg_tail) gets after the global rounds.  Vectorised Boruvka with id keys (the same
selection as k_seg_classify / k_seg_best / k_seg_hook); sizes and last-join weights as seg_size_update.

    python tools/seg_bucket_stats.py [W H] [--c 5000] [--small 16384]
"""
import argparse
import os
import sys

import numpy as np
from scipy.sparse import coo_matrix
from scipy.sparse.csgraph import connected_components

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from oracle import oracle as O  # noqa: E402
from tools.synth import make_pair  # noqa: E402


def roots_of(par):
    r = par.copy()
    while True:
        n = r[r]
        if np.array_equal(n, r):
            return r
        r = n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("W", type=int, nargs="?", default=1920)
    ap.add_argument("H", type=int, nargs="?", default=1200)
    ap.add_argument("--c", type=float, default=5000.0)
    ap.add_argument("--small", type=int, default=16384)
    ap.add_argument("--view", default="left", choices=["left", "right"])
    a = ap.parse_args()
    W, H = a.W, a.H
    left, right, _ = make_pair(W, H, 128, index=0)
    wR, wD = O.edge_weights(O.median3(left if a.view == "left" else right))
    wR = np.asarray(wR, dtype=np.int64).reshape(-1)
    wD = np.asarray(wD, dtype=np.int64).reshape(-1)
    N = W * H
    p = np.arange(N, dtype=np.int64)
    x, y = p % W, p // W
    ids, ea, eb, ew = [], [], [], []
    mr = x + 1 < W
    ids.append(2 * p[mr]); ea.append(p[mr]); eb.append(p[mr] + 1); ew.append(wR[mr])
    md = y + 1 < H
    ids.append(2 * p[md] + 1); ea.append(p[md]); eb.append(p[md] + W); ew.append(wD[md])
    ids, ea, eb, ew = (np.concatenate(t) for t in (ids, ea, eb, ew))
    order = np.lexsort((ids, ew))
    ids, ea, eb, ew = ids[order], ea[order], eb[order], ew[order]
    bstart = np.searchsorted(ew, np.arange(767))
    par = np.arange(N, dtype=np.int64)
    sz = np.ones(N, dtype=np.int64)
    wl = np.zeros(N, dtype=np.int64)
    tot_tail = 0
    small = dict(buckets=0, live=0, cand=0, edges=0, live_edges=0, cand_edges=0, open_end=0, open_end_edges=0)
    w_first, thr0 = None, None
    print("   w      edges  candidates  crossing after rounds 1, 2, ...")
    for w in range(766):
        s, e = bstart[w], bstart[w + 1]
        m = e - s
        if m == 0:
            continue
        ra, rb = par[ea[s:e]], par[eb[s:e]]  # par is kept fully compressed (roots)
        two = ra != rb
        thr = lambda r: w <= wl[r] + (np.float32(a.c) / sz[r].astype(np.float32)).astype(np.float64)  # noqa: E731
        cand = two & thr(ra) & thr(rb)
        ca, cb, cid = ra[cand], rb[cand], ids[s:e][cand]
        n = len(cid)
        if m <= a.small:  # small buckets: live (two-component) edges, and those with both ends open at the
            # first small bucket (the others are rejected whatever happens: a closed component never joins)
            if w_first is None:
                w_first = w
                thr0 = wl + (np.float32(a.c) / sz.astype(np.float32)).astype(np.float64)
            small["buckets"] += 1
            small["edges"] += m
            nl = int(two.sum())
            small["live"] += nl > 0
            small["live_edges"] += nl
            small["cand"] += n > 0
            small["cand_edges"] += n
            oo = two & (thr0[ra] >= w_first) & (thr0[rb] >= w_first)
            small["open_end"] += int(oo.sum()) > 0
            small["open_end_edges"] += int(oo.sum())
        if n == 0:
            continue
        # Boruvka rounds over the candidates' roots (components relabelled after each round)
        uniq, inv = np.unique(np.concatenate([ca, cb]), return_inverse=True)
        la, lb = inv[:n], inv[n:]
        k = len(uniq)
        lab = np.arange(k)
        left_n, rounds = [], 0
        xa, xb, xid = la, lb, cid
        while len(xid):
            rounds += 1
            best = np.full(k, np.iinfo(np.int64).max)
            np.minimum.at(best, xa, xid)
            np.minimum.at(best, xb, xid)
            sel = (best[xa] == xid) | (best[xb] == xid)
            g = coo_matrix((np.ones(int(sel.sum())), (xa[sel], xb[sel])), shape=(k, k))
            _, comp = connected_components(g, directed=False)
            lab = comp[lab]
            xa, xb = comp[xa], comp[xb]
            keep = xa != xb
            xa, xb, xid = xa[keep], xb[keep], xid[keep]
            k = comp.max() + 1
            left_n.append(len(xid))
        # joins: every candidate root onto its component's representative (the smallest root id)
        groups = lab
        rep = np.full(groups.max() + 1, np.iinfo(np.int64).max)
        np.minimum.at(rep, groups, uniq)
        tgt = rep[groups]
        gsz = np.zeros(groups.max() + 1, dtype=np.int64)
        np.add.at(gsz, groups, sz[uniq])
        moved = tgt != uniq
        par[uniq] = tgt
        sz[rep] = gsz
        wl[rep[np.unique(groups[moved])]] = w
        par = par[par]  # keep compressed
        par = roots_of(par)
        if m > a.small:
            tail = sum(left_n[1:])  # edges the tail's rounds scan after 2 global rounds (classify+hook, best+hook)
            tot_tail += tail
            # contention: candidates per root (classify's atomicMin on both ends), roots per joined component
            # (the size update's atomicAdd), and per wave of 64 consecutive candidates the distinct roots
            inc = np.bincount(np.concatenate([la, lb]))
            per = np.bincount(groups)
            nw = (n + 63) // 64
            dist = [len(np.unique(np.concatenate([la[i:i + 64], lb[i:i + 64]]))) for i in range(0, n, 64)]
            print("%4d %10d %11d  %-28s max cand/root %7d  max roots/comp %7d  distinct roots/wave %.1f (of 128)"
                  % (w, m, n, left_n[:8], inc.max(), per.max(), float(np.mean(dist)) if nw else 0.0))
    print("big-bucket tail scans (sum over rounds >= 3 of the crossing candidates): %d" % tot_tail)
    print("small buckets (from w = %s): %s" % (w_first, small))


if __name__ == "__main__":
    main()
