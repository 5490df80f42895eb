"""MST_PMS on the CPU: the oracle's random streams against the pinned fixture (tests/golden/pms,
made by tests/golden/make_rng_golden.py from this container's libstdc++ and glibc), the library's
host-side forest / tree graph / streams (stereomatch_amd/csrc/sm_pms_host.cpp) against the oracle,
and the oracle's MST_PMS against a literal pure-Python transcription of Stereo3DMST.cpp:546-629 on
tiny images."""
import os
from fractions import Fraction

import numpy as np
import pytest

import stereomatch_amd._lib as L
from conftest import GOLDEN, golden_cases, load_case
from oracle import oracle as O
from tools.synth import make_pair

RNG = os.path.join(GOLDEN, "pms", "rng_streams.npz")


def u32(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def test_oracle_streams_match_pinned_fixture():
    z = np.load(RNG)
    np.testing.assert_array_equal(u32(O.pms_dice(8192)), u32(z["dice"]))
    np.testing.assert_array_equal(O.glibc_random(1, 0, 8192), z["glibc"])
    np.testing.assert_array_equal(O.glibc_random(1, 40000, 1000), z["glibc_skip40000"])
    np.testing.assert_array_equal(u32(O.pms_init_labels(16, 12, 64)), u32(z["init_16x12_d64"]))


def test_library_streams_match_oracle():
    np.testing.assert_array_equal(u32(L.pms_dice(100000)), u32(O.pms_dice(100000)))
    np.testing.assert_array_equal(L.pms_glibc_random(1, 6 * 97 * 61, 5000), O.glibc_random(1, 6 * 97 * 61, 5000))
    for W, H, D in ((97, 61, 64), (33, 7, 100), (5, 3, 2)):
        np.testing.assert_array_equal(u32(L.pms_init_labels(W, H, D)), u32(O.pms_init_labels(W, H, D)))
    for D in (2, 16, 64, 100, 128, 256, 1000):
        assert L.pms_levels(D) == O.pms_levels(D)


@pytest.mark.parametrize("name", golden_cases())
@pytest.mark.parametrize("c,min_size", [(5000.0, 200), (300.0, 20), (float("inf"), 200), (0.0, 2)])
def test_library_forest_bfs_matches_oracle(name, c, min_size):
    """The reference numbering (Stereo3DMST.cpp:342-384, 450-522) and tree_g (:377-384) of the
    library's host code against the oracle's, for the segment forest of every golden image."""
    z = load_case(name)
    for img in (z["left"], z["right"]):
        H, W, _ = img.shape
        med = O.median3(img)
        wR, wD = O.edge_weights(med)
        mask, _ = O.segment(W, H, wR, wD, c, min_size)
        ref = O.bfs(W, H, wR, wD, mask)
        got = L.pms_forest_bfs(W, H, wR, wD, mask)
        assert got["ntrees"] == ref["ntrees"]
        for k in ("tree_start", "node_pix", "node_parent", "node_w", "node_nch"):
            np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
        np.testing.assert_array_equal(got["node_child"], ref["node_child"])
        s, nb = L.pms_tree_graph(W, H, wR, wD, mask)
        rs, rnb = O.tree_graph(W, H, ref)
        np.testing.assert_array_equal(s[:ref["ntrees"] + 1], rs)
        np.testing.assert_array_equal(nb, rnb)


@pytest.mark.parametrize("src,c,min_size,piece", [("smooth_97x61", 5000.0, 200, 16), ("rand_37x23", 0.0, 2, 4),
                                                  ("synth", 300.0, 20, 64), ("synth", 5000.0, 200, 8),
                                                  ("synth", float("inf"), 200, 512)])
def test_schedule_forest_threads_invariant(src, c, min_size, piece):
    """The schedule forest (rows, paths, items, round lists, cuts, tree graph) built tree by tree on 1, 3
    and 8 host threads is the same, and its numbering is the oracle's BFS (Stereo3DMST.cpp:342-384,
    450-522)."""
    img = load_case(src)["left"] if src != "synth" else make_pair(640, 480, 32, index=3)[0]
    H, W, _ = img.shape
    wR, wD = O.edge_weights(O.median3(img))
    mask, _ = O.segment(W, H, wR, wD, c, min_size)
    ref = O.bfs(W, H, wR, wD, mask)
    outs = [L.pms_forest_digest(W, H, wR, wD, mask, piece, nt) for nt in (1, 3, 8)]
    for o in outs:
        assert o["ntrees"] == ref["ntrees"]
        np.testing.assert_array_equal(o["tree_start"], ref["tree_start"])
        np.testing.assert_array_equal(o["bfs_pix"], ref["node_pix"])
        np.testing.assert_array_equal(o["digest"], outs[0]["digest"])


# ---------------------------------------------------------------- literal transcription of MST_PMS
def _r32(fr):
    c = np.float32(float(fr))
    best = None
    for cand in (np.nextafter(c, np.float32(-np.inf)), c, np.nextafter(c, np.float32(np.inf))):
        if not np.isfinite(cand):
            continue
        e = abs(Fraction(float(cand)) - fr)
        key = (e, int(np.array(cand, np.float32).view(np.uint32)) & 1)
        if best is None or key < best[0]:
            best = (key, cand)
    return np.float32(best[1])


def fmaf(a, b, c):
    return _r32(Fraction(float(a)) * Fraction(float(b)) + Fraction(float(c)))


def fma64(a, b, c):
    return float(Fraction(a) * Fraction(b) + Fraction(c))  # Fraction -> float rounds correctly


def _cvtt(f):
    f = float(f)
    return int(f) if -2147483648.0 <= f < 2147483648.0 else -(2 ** 31)


def py_mst_pms(W, H, Dmax, tree, nb_start, nb, vol, abc, minc, dice, rnd):
    """Stereo3DMST.cpp:546-629 line by line (serial), float32 steps with the shipped binary's fmas."""
    f32 = np.float32
    S, S2 = O.s_lut(), O.s2_lut()
    N = W * H
    ts_, pix_, par_, w_, nch_, ch_ = (tree[k] for k in ("tree_start", "node_pix", "node_parent", "node_w",
                                                         "node_nch", "node_child"))

    def cost(lab, p):  # compute3DLabelCost (:103-118)
        d = f32(fmaf(f32(p % W), lab[0], f32(f32(p // W) * lab[1])) + lab[2])
        dc, df = f32(np.ceil(d)), f32(np.floor(d))
        if _cvtt(dc) >= Dmax or _cvtt(df) < 0:
            return f32(0.5)
        return fmaf(f32(dc - d), vol[_cvtt(df) * N + p], f32(f32(d - df) * vol[_cvtt(dc) * N + p]))

    def update(t, lab):  # MSTCostAggregationAndLabelUpdate (:160-186)
        agg = {}
        nodes = range(ts_[t], ts_[t + 1])
        for n in nodes:
            agg[pix_[n]] = 0.0
        for n in reversed(nodes[1:]):
            p, pp = pix_[n], pix_[par_[n]]
            agg[p] = float(cost(lab, p)) + agg[p]
            agg[pp] = fma64(agg[p], S[w_[n]], agg[pp])
        r = pix_[ts_[t]]
        agg[r] = float(cost(lab, r)) + agg[r]
        for n in nodes:
            for i in range(nch_[n]):
                c = ch_[4 * n + i]
                agg[pix_[c]] = fma64(S[w_[c]], agg[pix_[n]], S2[w_[c]] * agg[pix_[c]])
        for n in nodes:
            p = pix_[n]
            if agg[p] < minc[p]:
                minc[p] = agg[p]
                abc[p] = lab
    k = 0
    for t in range(tree["ntrees"]):
        for u in nb[nb_start[t]:nb_start[t + 1]]:
            sz = ts_[u + 1] - ts_[u]
            i = _cvtt(f32(f32(f32(dice[k] + f32(1.0)) * f32(0.5)) * f32(sz)))
            k += 1
            q = pix_[ts_[u] + i]
            update(t, abc[q].copy())
        sz = ts_[t + 1] - ts_[t]
        tp = pix_[ts_[t] + int(rnd[t]) % sz]
        px, py = f32(tp % W), f32(tp // W)
        la, lb, lc = abc[tp]
        nz = _r32(Fraction(1) / Fraction(float(f32(np.sqrt(np.float64(f32(fmaf(la, la, f32(lb * lb)) + f32(1.0))))))))
        nx, ny = f32(-la * nz), f32(-lb * nz)
        d = f32(fmaf(la, px, f32(lb * py)) + lc)
        max_n, max_d = f32(1.0), f32(f32(0.5) * f32(Dmax))
        while max_d > f32(0.1):
            rd = fmaf(dice[k], max_d, d)
            k += 1
            if not (rd < f32(0.0) or rd > f32(Dmax)):
                rnx = fmaf(max_n, dice[k], nx)
                rny = fmaf(max_n, dice[k + 1], ny)
                rnz = fmaf(max_n, dice[k + 2], nz)
                k += 3
                ss = fmaf(rnz, rnz, fmaf(rnx, rnx, f32(rny * rny)))
                ni = _r32(Fraction(1) / Fraction(float(f32(np.sqrt(np.float64(ss))))))
                rnx, rny, rnz = f32(rnx * ni), f32(rny * ni), abs(f32(rnz * ni))
                lab = np.array([_r32(Fraction(float(-rnx)) / Fraction(float(rnz))),
                                _r32(Fraction(float(-rny)) / Fraction(float(rnz))),
                                _r32(Fraction(float(fmaf(rd, rnz, fmaf(rnx, px, f32(rny * py))))) / Fraction(float(rnz)))],
                               np.float32)
                update(t, lab)
            max_d, max_n = f32(max_d * f32(0.5)), f32(max_n * f32(0.5))
    return k


@pytest.mark.parametrize("W,H,D,c,ms,idx", [(20, 14, 12, 150.0, 8, 0), (17, 9, 9, 300.0, 5, 2), (12, 10, 6, float("inf"), 200, 1)])
def test_oracle_mst_pms_matches_literal_transcription(W, H, D, c, ms, idx):
    left, right, _ = make_pair(W, H, D, index=idx)
    tree = O.build_tree(left, c, ms)
    nb_start, nb = O.tree_graph(W, H, tree)
    vol = O.cost_agd(left, right, 0, D)[0]
    dice = O.pms_dice(O.dice_budget(tree, nb_start, D))
    rnd = O.glibc_random(1, 6 * W * H, 2 * tree["ntrees"])
    abc = O.pms_init_labels(W, H, D)
    minc = np.full(W * H, np.finfo(np.float64).max)
    pa, pm = abc.copy(), minc.copy()
    flat = vol.reshape(-1)
    for it in range(2):
        K = tree["ntrees"]
        k = O.mst_pms(W, H, D, tree, nb_start, nb, vol, abc, minc, dice, rnd[it * K:(it + 1) * K])
        kp = py_mst_pms(W, H, D, tree, nb_start, nb, flat, pa, pm, dice, rnd[it * K:(it + 1) * K])
        assert k == kp
        np.testing.assert_array_equal(u32(abc), u32(pa))
        np.testing.assert_array_equal(minc.view(np.uint64), pm.view(np.uint64))
