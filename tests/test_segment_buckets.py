"""The argument behind the GPU segmentation (sm_seg_gpu.h), checked on the CPU: the
reference's serial Felzenszwalb sweep (segment-graph.h:54-89) plus its min-size merge
(Stereo3DMST.cpp:293-307) equals a bucket-synchronous restatement in which, per weight bucket,

  * a component is open iff w <= w_last + c/size at the bucket's start (closed ones reject the
    whole bucket, joined ones accept the rest of it),
  * the bucket's marked edges are the minimum spanning forest, keyed by edge id, of its open-open
    edges between components (any order gives the same partition), and
  * from any bucket w0 on (the GPU: the start of a run of small buckets, k_seg_split), every later edge can
    be classified once against the state at w0's start: internal ones stay internal, one with an end
    closed at w0 is rejected (a closed component never joins again: a join needs its own acceptance), and
    only the rest (both ends open at w0) need the per-bucket sweep,
  * the rejected edges are its other two-component edges; the min-size merge only needs those whose
    end is smaller than min_size after the sweep, in (w, id) order, and of those only the first of each
    pair of sweep roots (the GPU's pair dedupe, seg_launch_dedupe: a later edge of the same pair finds
    the two joined, or both of at least min_size pixels, for good).

The restatement below is plain Python over small images; the oracle (oracle/sm_oracle.c
orc_segment, itself pinned to the reference's segment-graph.h) is the serial sweep."""
import numpy as np
import pytest

from oracle import oracle as O
from tools.synth import make_pair


def bucket_segment(W, H, wR, wD, c, min_size, dedupe=False, split_at=None):
    N = W * H
    p = np.arange(N)
    x, y = p % W, p // W
    e = np.concatenate([2 * p[x + 1 < W], 2 * p[y + 1 < H] + 1])
    w = np.concatenate([wR[x + 1 < W], wD[y + 1 < H]]).astype(np.int64)
    par = list(range(N))
    size = [1] * N
    wl = [0] * N

    def find(a):
        while par[a] != a:
            par[a] = par[par[a]]
            a = par[a]
        return a

    mask = np.zeros(N, np.uint8)
    rejected = []
    cf = np.float32(c)
    active = None  # after the split: the edges still to sweep
    for wv in np.unique(w):
        if split_at is not None and active is None and wv >= split_at:
            # the split at this bucket's start (k_seg_split): every edge of weight >= wv classified once
            active = set()
            for i in e[w >= wv]:
                ra, rb = find(i >> 1), find((i >> 1) + (W if i & 1 else 1))
                if ra == rb:
                    continue
                if all(float(wv) <= float(wl[r]) + float(np.float32(cf / np.float32(size[r]))) for r in (ra, rb)):
                    active.add(int(i))
                else:
                    rejected.append((int(w[e == i][0]), int(i)))
        ids = np.sort(e[w == wv])
        if active is not None:
            ids = np.array([i for i in ids if int(i) in active], dtype=np.int64)
        roots = [(find(i >> 1), find((i >> 1) + (W if i & 1 else 1))) for i in ids]
        opened = {}

        def is_open(r):
            if r not in opened:  # the acceptance test at the bucket's start (float c / size, double sum)
                opened[r] = float(wv) <= float(wl[r]) + float(np.float32(cf / np.float32(size[r])))
            return opened[r]

        cand = []
        for i, (ra, rb) in zip(ids, roots):
            if ra == rb:
                continue
            if is_open(ra) and is_open(rb):
                cand.append((int(i), ra, rb))
            else:
                rejected.append((int(wv), int(i)))
        # id-keyed minimum spanning forest of the candidates over the components: Kruskal in id order
        joined = set()
        for i, ra, rb in cand:
            a, b = find(ra), find(rb)
            if a == b:
                continue
            if size[a] < size[b]:
                a, b = b, a
            par[b] = a
            size[a] += size[b]
            joined.add(a)
            mask[i >> 1] |= 2 if i & 1 else 1
        for r in joined:
            if find(r) == r:
                wl[r] = int(wv)
    # a rejected edge still joins two components after the sweep (one end's component is closed)
    assert all(find(i >> 1) != find((i >> 1) + (W if i & 1 else 1)) for _, i in rejected)
    ms = max(2, min_size)
    ends = lambda i: (find(i >> 1), find((i >> 1) + (W if i & 1 else 1)))
    cands = [(wv, i) for wv, i in sorted(rejected) if min(size[r] for r in ends(i)) < ms]
    if dedupe:  # the first candidate of each unordered pair of sweep roots
        seen, kept = set(), []
        for wv, i in cands:
            key = tuple(sorted(ends(i)))
            if key not in seen:
                seen.add(key)
                kept.append((wv, i))
        assert len(kept) <= len(cands)
        cands = kept
    for wv, i in cands:
        a, b = find(i >> 1), find((i >> 1) + (W if i & 1 else 1))
        if a != b and (size[a] < ms or size[b] < ms):
            if size[a] < size[b]:
                a, b = b, a
            par[b] = a
            size[a] += size[b]
            mask[i >> 1] |= 2 if i & 1 else 1
    return mask, len({find(q) for q in range(N)})


@pytest.mark.parametrize("W,H,c,min_size,index", [(64, 48, 5000.0, 200, 0), (64, 48, 300.0, 20, 1),
                                                  (80, 40, 40.0, 5, 2), (48, 64, 0.0, 2, 3), (72, 54, 1000.0, 60, 4)])
@pytest.mark.parametrize("dedupe", [False, True])
def test_bucket_sweep_equals_serial_sweep(W, H, c, min_size, index, dedupe):
    left, _, _ = make_pair(W, H, 32, index=index)
    wR, wD = O.edge_weights(O.median3(left))
    ref, n = O.segment(W, H, wR, wD, c, min_size)
    got, k = bucket_segment(W, H, wR, wD, c, min_size, dedupe)
    np.testing.assert_array_equal(got, ref)
    assert k == n


@pytest.mark.parametrize("W,H,c,min_size,index", [(64, 48, 5000.0, 200, 0), (64, 48, 300.0, 20, 1),
                                                  (80, 40, 40.0, 5, 2), (72, 54, 1000.0, 60, 4)])
@pytest.mark.parametrize("q", [0.0, 0.3, 0.6, 0.9])
def test_split_sweep_equals_serial_sweep(W, H, c, min_size, index, q):
    """k_seg_split's argument: the sweep split at the bucket holding the q-quantile of the weights."""
    left, _, _ = make_pair(W, H, 32, index=index)
    wR, wD = O.edge_weights(O.median3(left))
    ref, n = O.segment(W, H, wR, wD, c, min_size)
    ws = np.sort(np.concatenate([wR.reshape(H, W)[:, :-1].ravel(), wD.reshape(H, W)[:-1, :].ravel()]))
    got, k = bucket_segment(W, H, wR, wD, c, min_size, True, split_at=int(ws[int(q * (len(ws) - 1))]))
    np.testing.assert_array_equal(got, ref)
    assert k == n
