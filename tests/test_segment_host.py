"""CPU: segment mode's host segmentation (stereomatch_amd/csrc/sm_segment.cpp, in the product
library; no GPU involved) against the oracle's restatement of segment_graph + the min-size merge
(segment-graph.h:54-89, Stereo3DMST.cpp:242-307), which is itself pinned to the reference's own
segment-graph.h on the golden fixtures (test_oracle_golden.py); plus the virtual-edge embedding."""
import ctypes

import numpy as np
import pytest

from conftest import golden_cases, load_case
from oracle import oracle as O

VIRTUAL_W = 766


def segment_forest(wR, wD, W, H, c, min_size):
    import stereomatch_amd as sm
    L = sm.lib()
    f = L.sm_segment_forest
    f.restype = ctypes.c_int
    N = W * H
    mR = np.zeros(N, np.uint8)
    mD = np.zeros(N, np.uint8)
    fwR = np.zeros(N, np.uint16)
    fwD = np.zeros(N, np.uint16)
    P = lambda a: np.ascontiguousarray(a).ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    wR = np.ascontiguousarray(wR, np.uint16)
    wD = np.ascontiguousarray(wD, np.uint16)
    nt = f(P(wR), P(wD), ctypes.c_int(W), ctypes.c_int(H), ctypes.c_float(c), ctypes.c_int(min_size), P(mR), P(mD),
           P(fwR), P(fwD))
    return nt, mR, mD, fwR, fwD


def check(wR, wD, W, H, c, min_size):
    nt, mR, mD, fwR, fwD = segment_forest(wR, wD, W, H, c, min_size)
    vR, vD = fwR == VIRTUAL_W, fwD == VIRTUAL_W
    mask = ((mR.astype(bool) & ~vR) * 1 | (mD.astype(bool) & ~vD) * 2).astype(np.uint8)
    ref, nref = O.segment(W, H, wR, wD, c, min_size)
    np.testing.assert_array_equal(mask, ref)
    assert nt == nref
    # real weights untouched; one virtual edge per tree but pixel 0's, at the root's left / upper edge
    np.testing.assert_array_equal(fwR[~vR], wR[~vR])
    np.testing.assert_array_equal(fwD[~vD], wD[~vD])
    assert int(vR.sum() + vD.sum()) == nt - 1
    # forest + virtual edges = one spanning tree (N - 1 edges, connected)
    assert int(mR.sum()) + int(mD.sum()) == W * H - 1
    t = O.bfs(W, H, wR, wD, (mR | (mD << 1)).astype(np.uint8))
    assert t["ntrees"] == 1
    # every virtual edge hangs a tree root (its first pixel in raster order) from an earlier pixel
    tb = O.bfs(W, H, wR, wD, ref)
    roots = set(int(tb["node_pix"][s]) for s in tb["tree_start"][:-1])
    for p in np.nonzero(vR)[0]:
        assert p + 1 in roots
    for p in np.nonzero(vD)[0]:
        assert p + W in roots and (p + W) % W == 0
    return nt


@pytest.mark.parametrize("name", golden_cases())
@pytest.mark.parametrize("c,min_size", [(5000.0, 200), (5000.0, 0), (300.0, 20), (0.0, 2)])
def test_segment_forest_matches_oracle_golden(name, c, min_size):
    z = load_case(name)
    H, W, _ = z["left"].shape
    for v in ("left", "right"):
        check(z[v + "_wR"], z[v + "_wD"], W, H, c, min_size)


@pytest.mark.parametrize("W,H,seed", [(200, 150, 1), (333, 7, 2), (1, 50, 3), (64, 64, 4)])
def test_segment_forest_matches_oracle_random(W, H, seed):
    from tools.synth import make_pair
    left, _, _ = make_pair(W, H, 16, index=seed)
    wR, wD = O.edge_weights(O.median3(left))
    nt = check(wR, wD, W, H, 5000.0, 200)
    assert nt >= 1
