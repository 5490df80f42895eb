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
