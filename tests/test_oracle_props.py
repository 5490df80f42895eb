"""CPU: size-independent properties of the oracle (edge cases of the reference path)."""
import numpy as np

from oracle import oracle as O


def test_constant_image_aggregates_to_slice_sum():
    # all edge weights 0 -> S=1, S2=0 -> every pixel's A equals the slice's total cost
    H, W, D = 9, 13, 5
    img = np.full((H, W, 3), 42, np.uint8)
    res = O.match(img, img, D, want_volumes=True)
    for v in ("left", "right"):
        A, vol = res[v]["A"], res[v]["vol"]
        for d in range(D):
            tot = float(np.sum(vol[d].astype(np.float64)))
            assert np.allclose(A[d], tot, rtol=1e-12)


def test_wta_first_minimum_on_ties():
    # identical slices: strict < keeps the lowest disparity (Stereo3DMST.cpp:177)
    H, W = 6, 7
    img = np.random.default_rng(3).integers(0, 256, (H, W, 3), dtype=np.uint8)
    t = O.build_tree(img)
    vol = np.ones((4, H, W), np.float32)
    r = O.tree_filter(W, H, t, vol, 0, True, False, 1)
    assert (r["idx"] == 0).all()


def test_cost_volume_borders():
    H, W, D = 5, 11, 6
    rng = np.random.default_rng(7)
    L = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    R = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    lv, rv = O.cost_agd(L, R, 0, D)
    for d in range(D):
        assert (rv[d][:, W - 1 - d:] == 3.0).all()           # x + d + 1 >= W
        assert (lv[d][:, :d] == 3.0).all()                   # x - d < 0
        assert (lv[d][:, W - 1] == 3.0).all()                # column the reference never writes
        if W - 1 - d > 0:
            np.testing.assert_array_equal(lv[d][:, d:W - 1], rv[d][:, :W - 1 - d])  # mirrored store (.cu:1543)
    assert (lv <= 3.0).all() and (lv >= 0).all()


def test_tree_filter_is_linear_and_normalised_when_costs_constant():
    # A = sum_q w(p,q) C(q) with w in (0,1]; constant C=c gives A between c and N*c
    H, W = 8, 10
    img = np.random.default_rng(11).integers(0, 256, (H, W, 3), dtype=np.uint8)
    t = O.build_tree(img)
    vol = np.full((2, H, W), 0.5, np.float32)
    r = O.tree_filter(W, H, t, vol, 0, False, True, 1)
    assert (r["A"] >= 0.5 - 1e-12).all() and (r["A"] <= 0.5 * H * W + 1e-9).all()
    r2 = O.tree_filter(W, H, t, vol * 2, 0, False, True, 1)
    np.testing.assert_allclose(r2["A"], 2 * r["A"], rtol=1e-12)


def test_bfs_children_in_ascending_key_order():
    H, W = 7, 9
    img = np.random.default_rng(5).integers(0, 256, (H, W, 3), dtype=np.uint8)
    t = O.build_tree(img)
    N = W * H
    assert t["ntrees"] == 1 and t["node_pix"][0] == 0
    # BFS ids are a permutation; parents precede children
    assert sorted(t["node_pix"].tolist()) == list(range(N))
    assert (t["node_parent"][1:] < np.arange(1, N)).all()
    # siblings: ascending edge weight (ties by a, dir)
    for n in range(N):
        k = t["node_nch"][n]
        ch = t["node_child"][4 * n:4 * n + k]
        ws = [int(t["node_w"][c]) for c in ch]
        assert ws == sorted(ws)


def test_lr_check_semantics():
    """Stereo3DMST.cpp:632-662 (fill=false): out-of-range / inconsistent left pixels -> 0."""
    L = np.array([[0, 1, 2, 5], [3, 0, 1, 1], [1.5, 2.5, 0.5, 2]], np.float32)
    R = np.array([[0, 1, 1, 2], [0, 0, 0, 1], [1, 1, 0, 2]], np.float32)
    out = O.lr_check(L, R, 4)
    # row 0: d=2 at x=2 reads R(0)=0 (|2-0|>1); d=5 >= max_disp
    # row 1: x=0, d=3 -> x-d < 0
    # row 2: round(1.5)=2 -> x-d<0; round(2.5)=3 -> x-d<0; round(0.5)=1 -> R(1)=1, |0.5-1|<=1; x=3,d=2 -> R(1)=1
    exp = np.array([[0, 1, 0, 0], [0, 0, 1, 1], [0, 0, 0.5, 2]], np.float32)
    np.testing.assert_array_equal(out, exp)


def test_mccnn_clamp_follows_reference():
    """Stereo3DMST.cpp:785-803: NaN -> 0.5, otherwise std::min(0.5f, x) (returns 0.5 unless x < 0.5)."""
    x = np.array([np.nan, -1.0, 0.25, 0.5, 0.7, np.inf, -np.inf, -0.0, 0.49999997], np.float32)
    y = O.mccnn_clamp(x)
    exp = np.array([0.5, -1.0, 0.25, 0.5, 0.5, 0.5, -np.inf, -0.0, 0.49999997], np.float32)
    assert y.dtype == np.float32
    np.testing.assert_array_equal(y.view(np.uint32), exp.view(np.uint32))


# ---- output step (Stereo3DMST.cpp:189-201, 632-709, 900-904; PatchMatchStereoGPU.cu:1128-1288) ----
def test_label_to_disp_float_roundtrip():
    """numpy float32 arithmetic (IEEE, one rounding per op) restates LabelToDisp + *= (Dmax-1.f);
    the integers that do not survive the round trip at the caller's Dmax=100 (stereo_Yin.cpp:207)."""
    for D in (16, 48, 64, 100, 128, 200, 256):
        d = np.arange(-2, D + 3, dtype=np.float32)
        dm1 = np.float32(D) - np.float32(1)
        q = d / dm1
        q = np.where(q < np.float32(1), q, np.float32(1)).astype(np.float32)
        q = np.where(np.float32(0) < q, q, np.float32(0)).astype(np.float32)
        np.testing.assert_array_equal(O.label_to_disp(d, D), (q * dm1).astype(np.float32))
    changed = np.nonzero(O.label_to_disp(np.arange(100, dtype=np.float32), 100) != np.arange(100))[0]
    assert list(changed) == [7, 14, 25, 28, 31, 50, 55, 56, 61, 62]
    changed = np.nonzero(O.label_to_disp(np.arange(48, dtype=np.float32), 48) != np.arange(48))[0]
    assert list(changed) == [1, 2, 4, 8, 16, 32]


def _lr_fill_py(left, right, max_disp, fill):
    """Literal pure-Python transcription of leftRightConsistencyCheck (:632-709)."""
    L = left.astype(np.float32).copy()
    H, W = L.shape
    mask = np.zeros((H, W), np.uint8)
    for y in range(H):
        for x in range(W):
            df = L[y, x]
            a = abs(float(df))  # float64: a + 0.5 is exact for a float32 a
            d = int(np.floor(a + 0.5)) * (1 if df >= 0 else -1)  # std::round: half away from zero
            if x - d >= 0 and 0 <= d < max_disp:
                if abs(np.float32(df - right[y, x - d])) > 1.0:
                    mask[y, x] = 1
                    L[y, x] = 0.0
            else:
                mask[y, x] = 1
                L[y, x] = 0.0
    if not fill:
        return L
    for y in range(H):
        for x in range(W):
            if mask[y, x] == 0:
                continue
            i = 1
            while x - i >= 0:
                if mask[y, x - i] == 0:
                    L[y, x] = L[y, x - i]
                    mask[y, x] = 0
                    break
                i += 1
            i = 1
            while x + i < W:
                if mask[y, x + i] == 0:
                    if L[y, x + i] < L[y, x] or mask[y, x] == 1:
                        L[y, x] = L[y, x + i]
                    break
                i += 1
    return L


def test_lr_check_and_fill_match_literal_python():
    rng = np.random.default_rng(21)
    for H, W, D in ((5, 17, 8), (3, 40, 16), (1, 9, 4), (6, 1, 3)):
        for trial in range(4):
            ld = rng.integers(0, D, (H, W)).astype(np.float32)
            rd = rng.integers(0, D, (H, W)).astype(np.float32)
            if trial == 1:
                rd = ld.copy()  # mostly consistent maps
            if trial == 2:
                ld = O.label_to_disp(ld, D)
                rd = O.label_to_disp(rd, D)
            for fill in (False, True):
                np.testing.assert_array_equal(O.lr_check(ld, rd, D, fill), _lr_fill_py(ld, rd, D, fill))


def _occlusion_py(L, R, min_disp, thresh, remove):
    """pure-Python restatement of handleOcclusionSharedMemory with the marks complete before the search."""
    L = L.astype(np.float32).copy()
    R = R.astype(np.float32).copy()
    H, W = L.shape
    inv = np.float32(1e18)
    for y in range(H):
        oL, oR = L[y].copy(), R[y].copy()
        mL, mR = np.zeros(W, bool), np.zeros(W, bool)
        for x in range(W):
            rx = int(np.float32(x) - oL[x])  # truncation toward zero
            mL[x] = rx < 0 or abs(oR[rx] - oL[x]) > thresh
            lx = int(np.float32(x) + oR[x])
            mR[x] = lx >= W or abs(oR[x] - oL[lx]) > thresh
        for orig, m, out in ((oL, mL, L[y]), (oR, mR, R[y])):
            for x in range(W):
                if not m[x]:
                    continue
                if remove:
                    out[x] = min_disp
                    continue
                ls = next((orig[q] for q in range(x - 1, -1, -1) if not m[q]), inv)
                rs = next((orig[q] for q in range(x + 1, W) if not m[q]), inv)
                out[x] = np.float32(255) if (ls == inv and rs == inv) else min(ls, rs)
    return L, R


def test_occlusion_matches_python():
    rng = np.random.default_rng(5)
    for H, W, D in ((4, 23, 8), (2, 64, 20), (3, 5, 3)):
        for sub in (False, True):
            L = rng.integers(0, D, (H, W)).astype(np.float32)
            R = rng.integers(0, D, (H, W)).astype(np.float32)
            if sub:
                L += rng.random((H, W)).astype(np.float32) * 0.9
                R += rng.random((H, W)).astype(np.float32) * 0.9
            for remove in (False, True):
                a = O.occlusion(L, R, 0, 1.0, remove)
                b = _occlusion_py(L, R, 0, 1.0, remove)
                np.testing.assert_array_equal(a[0], b[0])
                np.testing.assert_array_equal(a[1], b[1])
