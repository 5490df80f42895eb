"""Degenerate trees at full size: the tree layout's 27-bit preorder packing
(sm_layout_gpu.hip ScanTourOut / path records) and the long-path piece / repair engine on shapes the
textured pairs never produce.

* all-ties constant image at C2: every weight is 0, so Kruskal's (w, a, b) tie order makes a comb
  (row 0 plus every column): 1919 light paths of 1199 nodes, each cut into pieces, under a root
  path of 3119 nodes.  Costs from random MC-CNN-like volumes, so the WTA is not degenerate;
* a serpentine of 4-row bands at C2, each band a different grey and every band joined to the next
  through a mid-grey block at alternating ends: one heavy path of 576 598 nodes (1 126 pieces of
  512) with every other path 3-7 nodes, all hanging off it;
* a single row of 2^20 pixels and a single column of 2^20 pixels: the whole tree one path;
* 16384 x 8191 pixels (N = 2^27 - 16384), a constant image: preorder positions up to the top of the
  27-bit field.  With w = 0 everywhere S = 1 and S2 = 0, so every A row of a tree is the sum of the
  whole tree's costs; the AGD costs of a constant image are 0 or 3 (invalid positions), all sums
  are integers below 2^53 and exact in any order: every pixel's minimum is 3 H at slice 0;
* N >= 2^27 is refused with SM_ERR_ARG before anything is uploaded.

All but the last two compare idx / minc bitwise with the oracle (reference order, fp64)."""
import ctypes

import numpy as np
import pytest

from oracle import oracle as O
from tools.synth import make_pair

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a).view(np.uint64)


def heavy_paths(tree):
    """Lengths of the heavy paths of an oracle tree (BFS order: parents before children)."""
    par = tree["node_parent"]
    n = len(par)
    size = np.ones(n, np.int64)
    for i in range(n - 1, 0, -1):
        size[par[i]] += size[i]
    heavy = np.full(n, -1, np.int64)
    best = np.zeros(n, np.int64)
    for i in range(1, n):
        p = par[i]
        if size[i] > best[p]:
            best[p], heavy[p] = size[i], i
    head = np.ones(n, bool)
    head[heavy[heavy >= 0]] = False
    lens = []
    for h in np.nonzero(head)[0]:
        k, v = 1, h
        while heavy[v] >= 0:
            v, k = heavy[v], k + 1
        lens.append(k)
    return np.array(lens)


def serpentine(W, H, band=4):
    """Bands of `band` rows in greys 0 / 100 / 200 (cycling); band b and b+1 meet through a 3 x 3
    mid-grey block at the right end (b even) or the left end (b odd), which survives the 3x3 median."""
    img = np.zeros((H, W, 3), np.uint8)
    vals = (0, 100, 200)
    nb = (H + band - 1) // band
    for b in range(nb):
        img[b * band:(b + 1) * band, :, 0] = vals[b % 3]
    for b in range(nb - 1):
        r = (b + 1) * band
        c0 = W - 3 if b % 2 == 0 else 0
        img[r - 1:r + 2, c0:c0 + 3, 0] = (vals[b % 3] + vals[(b + 1) % 3]) // 2
    return img


def _check(out, ref, views=("left", "right")):
    for v in views:
        np.testing.assert_array_equal(out[v]["idx"].ravel(), ref[v]["idx"])
        assert np.array_equal(bits(out[v]["minc"].ravel()), bits(ref[v]["minc"]))


def test_constant_image_comb_c2(gpu_ctx):
    import stereomatch_amd as sm
    W, H, D = 1920, 1200, 128
    img = np.full((H, W, 3), 128, np.uint8)
    t = O.build_tree(img)
    lens = heavy_paths(t)
    assert (lens == H - 1).sum() == W - 1 and lens.max() == W + H - 1  # the comb
    rng = np.random.default_rng(61)
    lv = rng.random((D, H, W), dtype=np.float32)
    rv = rng.random((D, H, W), dtype=np.float32)
    gpu_ctx.upload_cost_volumes(lv, rv)
    out = gpu_ctx.match(img, img, D, sm.default_params(cost_kind=sm.SM_COST_VOLUME))
    ref = {v: O.tree_filter(W, H, t, O.mccnn_clamp(vol), 0, True, False, 16) for v, vol in (("left", lv), ("right", rv))}
    _check(out, ref)
    # the AGD cost too (0 at valid positions, 3 elsewhere: ties everywhere in the WTA)
    _check(gpu_ctx.match(img, img, D), O.match(img, img, D, nthreads=16))


def test_serpentine_single_heavy_path_c2(gpu_ctx):
    W, H, D = 1920, 1200, 128
    img = serpentine(W, H)
    lens = heavy_paths(O.build_tree(img))
    assert lens.max() > W * H // 4 and (lens >= 32).sum() == 1  # one heavy path of a quarter of the image
    _, right, _ = make_pair(W, H, D, index=11)
    _check(gpu_ctx.match(img, right, D), O.match(img, right, D, nthreads=16))


@pytest.mark.parametrize("W,H,D", [(1 << 20, 1, 64), (1, 1 << 20, 32)])
def test_single_path_2p20(gpu_ctx, W, H, D):
    rng = np.random.default_rng(W)
    left = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    right = np.roll(left, 3, axis=1) if W > 1 else left[::-1].copy()
    ref = O.match(left, right, D, nthreads=16)
    assert heavy_paths(ref["left"]["tree"]).max() == W * H
    _check(gpu_ctx.match(left, right, D), ref)


def test_constant_image_near_2p27_exact():
    """N = 2^27 - 16384, one view, 32 slices: every preorder position up to the 27-bit field's top."""
    import stereomatch_amd as sm
    W, H, D = 16384, 8191, 32
    img = np.full((H, W, 3), 77, np.uint8)
    ctx = sm.Context(0)
    try:
        out = ctx.match(img, img, D, sm.default_params(views=1))
        assert np.all(out["left"]["idx"] == 0)
        assert np.all(out["left"]["minc"] == 3.0 * H)
    finally:
        ctx.close()


def test_2p27_pixels_refused():
    import stereomatch_amd as sm
    from stereomatch_amd._lib import SM_ERR_ARG, lib
    L = lib()
    ctx = sm.Context(0)
    try:
        W, H = 16384, 8192  # 2^27 pixels
        tiny = np.zeros(16, np.uint8)
        vp = ctypes.c_void_p(tiny.ctypes.data)  # never read: the size check comes first
        p = sm.default_params()
        assert L.sm_match(ctx.h, vp, vp, W, H, 3 * W, 8, ctypes.byref(p), None, None, None, None, None, None) == SM_ERR_ARG
        assert L.sm_build_tree(ctx.h, vp, W, H, 3 * W, None, None, None, None) == SM_ERR_ARG
        assert L.sm_aggregate_debug(ctx.h, vp, vp, W, H, 3 * W, 0, 0, 8, None, None) == SM_ERR_ARG
        # the device-resident path: the images upload (up to 2^30 pixels), the match refuses them
        img = np.zeros((H, W, 3), np.uint8)
        ctx.upload(img, img)
        with pytest.raises(sm.StereoMSTError, match="SM_ERR_ARG"):
            ctx.match_async(8, p)
        del img
        # the context stays usable
        left, right, _ = make_pair(96, 64, 16, index=1)
        _check(ctx.match(left, right, 16), O.match(left, right, 16, nthreads=16))
    finally:
        ctx.close()
