"""CPU: the oracle's colour guided-filter aggregator (PatchMatchStereoGPU.cu:8251-8470, box means
:495-580, selectDisparity :1688-1737).  The literal float restatement is checked against
(1) a float64 textbook guided filter (He et al., colour guide) within a float tolerance -- the
formulas are the right ones -- and (2) its own box mean against a pure-Python transcription of the
reference's 32-block sliding sums, bitwise."""
import numpy as np

from oracle import oracle as O
from tools.synth import make_pair


def box_ref(a, r):
    """float64 box mean with zero padding outside, divided by the full window (2r+1)^2 (the
    reference's boxes divide by the window size everywhere)."""
    H, W = a.shape
    p = np.zeros((H + 2 * r, W + 2 * r))
    p[r:r + H, r:r + W] = a
    c = p.cumsum(0).cumsum(1)
    c = np.pad(c, ((1, 0), (1, 0)))
    k = 2 * r + 1
    s = c[k:, k:] - c[:-k, k:] - c[k:, :-k] + c[:-k, :-k]
    return s / (k * k)


def guided_ref(img, p, r, eps):
    I = img.astype(np.float64)[:, :, ::-1]  # r, g, b planes
    mI = [box_ref(I[:, :, c], r) for c in range(3)]
    mp = box_ref(p, r)
    cov = [box_ref(I[:, :, c] * p, r) - mI[c] * mp for c in range(3)]
    S = np.empty(p.shape + (3, 3))
    for i in range(3):
        for j in range(3):
            S[..., i, j] = box_ref(I[:, :, i] * I[:, :, j], r) - mI[i] * mI[j] + (eps if i == j else 0)
    a = np.linalg.solve(S, np.stack(cov, -1)[..., None])[..., 0]
    b = mp - sum(a[..., c] * mI[c] for c in range(3))
    return sum(box_ref(a[..., c], r) * I[:, :, c] for c in range(3)) + box_ref(b, r)


def test_guided_filter_matches_textbook():
    left, right, _ = make_pair(80, 56, 8, index=3)
    lv, _ = O.cost_agd(left, right, 0, 8)
    out = O.guided_filter(left, lv, 4, 6.5025)
    for d in (0, 3, 7):
        ref = guided_ref(left, lv[d].astype(np.float64), 4, 6.5025)
        np.testing.assert_allclose(out[d], ref, rtol=2e-3, atol=2e-3)


def _box_x_py(a, r):
    H, W = a.shape
    out = np.empty_like(a)
    sc = np.float32(1.0) / np.float32(2 * r + 1)
    for y in range(H):
        for x0 in range(0, W, 32):
            t = np.float32(0)
            for i in range(x0 - r, x0 + r + 1):
                t = np.float32(t + (np.float32(0) if (i < 0 or i >= W) else a[y, i]))
            out[y, x0] = np.float32(t * sc)
            for x in range(x0 + 1, min(W, x0 + 32)):
                t = np.float32(t + (np.float32(0) if x + r >= W else a[y, x + r]))
                t = np.float32(t - (np.float32(0) if x - r - 1 < 0 else a[y, x - r - 1]))
                out[y, x] = np.float32(t * sc)
    return out


def test_box_mean_is_the_sliding_block_sum():
    """The oracle's box mean, bitwise against a pure-Python transcription of the reference's
    32-block sliding sums (x pass, then the same on the transpose for y)."""
    rng = np.random.default_rng(4)
    for H, W, r in ((40, 70, 5), (33, 65, 9), (7, 3, 2)):
        p = (rng.random((H, W)) * 3 - 1).astype(np.float32)
        exp = _box_x_py(_box_x_py(p, r).T.copy(), r).T
        np.testing.assert_array_equal(O.box_mean(p, r), exp)


def test_select_disparity_rules():
    v = np.array([[[3.0]], [[1.0]], [[1.0]], [[2.0]]], np.float32)  # tie at d=1,2: first wins
    idx, mn, disp = O.select_disparity(v, 0, 4, True)
    assert idx[0] == 1 and mn[0] == 1.0
    s = (np.float32(1.0) - np.float32(3.0)) * np.float32(0.5) / (np.float32(1.0) - np.float32(2.0) + np.float32(3.0))
    assert disp[0] == np.float32(1.0) - s
    idx, mn, disp = O.select_disparity(np.full((3, 1, 1), 2e10, np.float32), 0, 3, True)
    assert idx[0] == 0 and disp[0] == 0.0  # nothing below 1e10: -1 -> 0


def test_contraction_whatif_is_separate_from_the_shipped_arithmetic():
    """orc_set_gf_contract(1) (tools/gf_contraction.py's nvcc --fmad=true what-if) changes the filtered
    costs but stays within float rounding of the shipped result, and setting it back restores the
    shipped bits."""
    left, right, _ = make_pair(96, 64, 16, index=4)
    lv, _ = O.cost_agd(left, right, 0, 16)
    base = O.guided_filter(left, lv)
    try:
        O.set_gf_contract(1)
        fused = O.guided_filter(left, lv)
    finally:
        O.set_gf_contract(0)
    again = O.guided_filter(left, lv)
    assert np.array_equal(again.view(np.uint32), base.view(np.uint32))
    assert not np.array_equal(fused, base)
    np.testing.assert_allclose(fused, base, rtol=1e-3, atol=1e-3)
