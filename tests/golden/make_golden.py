#!/usr/bin/env python3
"""Generate the committed golden fixtures (run in the build container only).

Sources of truth, per fixture field:
  ref_mst_mask / ref_seg_mask : the reference's OWN include/segment-graph.h +
      include/disjoint-set.h, compiled from /root/reference into oracle/_ref
      (oracle/ref_segment_probe.cpp), run on the 4-connected edges of each image --
      real reference outputs.  ref_seg_* use c=5000 (Stereo3DMST.cpp:831) without the
      min-size merge (segment_graph alone).
  everything else (median, weights, bfs tree, cost volumes, idx/minc, Aup/A slices):
      the oracle restatement (oracle/sm_oracle.c), kept as regression vectors for the
      GPU parity tests; the tests also recompute them live.

Inputs: seeded synthetic BGR images (random, smooth, constant = all ties, 1-row,
1-column) and a 256x192 crop of the reference's FLIR pair build/000020_19140004{2,39}.jpg
(left = ..042, right = ..039, stereo_Yin.cpp:122-123), decoded here with PIL.  The full
FLIR JPEGs are copied as data into tests/golden/flir/ for the C1 (2048x1536, D=64) case.

Usage: make -C oracle && python3 tests/golden/make_golden.py
"""
import os
import shutil
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402

REF = "/root/reference"
D_SMALL = 16


def smooth_noise(rng, H, W):
    base = rng.integers(0, 256, (H // 8 + 2, W // 8 + 2, 3)).astype(np.float64)
    ys = np.linspace(0, base.shape[0] - 1.001, H)
    xs = np.linspace(0, base.shape[1] - 1.001, W)
    y0 = ys.astype(int); x0 = xs.astype(int)
    fy = (ys - y0)[:, None, None]; fx = (xs - x0)[None, :, None]
    b = base
    img = (b[y0][:, x0] * (1 - fy) * (1 - fx) + b[y0 + 1][:, x0] * fy * (1 - fx)
           + b[y0][:, x0 + 1] * (1 - fy) * fx + b[y0 + 1][:, x0 + 1] * fy * fx)
    img += rng.integers(-4, 5, img.shape)
    return np.clip(img, 0, 255).astype(np.uint8)


def shifted_pair(rng, H, W, maxd, smooth=True):
    """left texture; right(x) = left(x + d) with a per-row-smooth disparity; holes = noise."""
    big = smooth_noise(rng, H, W + maxd + 2) if smooth else rng.integers(0, 256, (H, W + maxd + 2, 3), dtype=np.uint8)
    left = big[:, :W].copy()
    right = np.empty_like(left)
    d = (np.arange(H)[:, None] * 0 + (np.arange(W)[None, :] * maxd // (2 * max(W, 1))) + maxd // 3)
    for y in range(H):
        for x in range(W):
            right[y, x] = big[y, x + int(d[y, x])]
    return left, right


def load_flir():
    from PIL import Image
    L = np.array(Image.open(os.path.join(REF, "build/000020_191400042.jpg")).convert("RGB"))[:, :, ::-1]
    R = np.array(Image.open(os.path.join(REF, "build/000020_191400039.jpg")).convert("RGB"))[:, :, ::-1]
    return np.ascontiguousarray(L), np.ascontiguousarray(R)


def case(name, left, right, D, out):
    H, W, _ = left.shape
    rec = dict(left=left, right=right, D=np.int32(D))
    res = O.match(left, right, D, want_volumes=(W * H * D <= 64 * 48 * 16))
    for view in ("left", "right"):
        r = res[view]
        t = r["tree"]
        ref = O.ref_segment_graph(W, H, t["wR"], t["wD"], float("inf"))
        refseg = O.ref_segment_graph(W, H, t["wR"], t["wD"], 5000.0)
        assert ref is not None, "oracle/_ref not built"
        m, _ = O.segment(W, H, t["wR"], t["wD"], float("inf"), 200)
        assert (m == ref["mask"]).all(), (name, view, "oracle MST != reference segment_graph")
        ms, _ = O.segment(W, H, t["wR"], t["wD"], 5000.0, -1)
        assert (ms == refseg["mask"]).all(), (name, view, "oracle segments != reference segment_graph")
        pfx = view + "_"
        rec[pfx + "median"] = t["med"]
        rec[pfx + "wR"] = t["wR"]
        rec[pfx + "wD"] = t["wD"]
        rec[pfx + "ref_mst_mask"] = ref["mask"]
        rec[pfx + "ref_seg_mask"] = refseg["mask"]
        rec[pfx + "ref_seg_nsets"] = np.int32(refseg["nsets"])
        rec[pfx + "node_pix"] = t["node_pix"]
        rec[pfx + "node_parent"] = t["node_parent"]
        rec[pfx + "vol"] = r["vol"]
        rec[pfx + "idx"] = r["idx"]
        rec[pfx + "minc"] = r["minc"]
        if r["Aup"] is not None:
            rec[pfx + "Aup"] = r["Aup"]
            rec[pfx + "A"] = r["A"]
    np.savez_compressed(os.path.join(out, name + ".npz"), **rec)
    print("wrote", name, W, H, D)


def main():
    out = HERE
    rng = np.random.default_rng(20261015)
    cases = []
    cases.append(("rand_8x6", rng.integers(0, 256, (6, 8, 3), dtype=np.uint8), rng.integers(0, 256, (6, 8, 3), dtype=np.uint8), 4))
    l, r = shifted_pair(rng, 23, 37, 8, smooth=False); cases.append(("rand_37x23", l, r, 8))
    l, r = shifted_pair(rng, 48, 64, 16); cases.append(("smooth_64x48", l, r, D_SMALL))
    l, r = shifted_pair(rng, 61, 97, 24); cases.append(("smooth_97x61", l, r, D_SMALL))
    c = np.full((12, 16, 3), 77, np.uint8); c2 = c.copy(); c2[:, 8:] = 80
    cases.append(("const_16x12", c, c2, 6))
    cases.append(("row_20x1", rng.integers(0, 256, (1, 20, 3), dtype=np.uint8), rng.integers(0, 256, (1, 20, 3), dtype=np.uint8), 5))
    cases.append(("col_1x15", rng.integers(0, 256, (15, 1, 3), dtype=np.uint8), rng.integers(0, 256, (15, 1, 3), dtype=np.uint8), 3))
    L, R = load_flir()
    y0, x0 = 700, 900
    cases.append(("flir_crop_256x192", L[y0:y0 + 192, x0:x0 + 256].copy(), R[y0:y0 + 192, x0:x0 + 256].copy(), D_SMALL))
    for name, left, right, D in cases:
        case(name, left, right, D, out)
    flir = os.path.join(out, "flir")
    os.makedirs(flir, exist_ok=True)
    for f in ("000020_191400042.jpg", "000020_191400039.jpg"):
        shutil.copyfile(os.path.join(REF, "build", f), os.path.join(flir, f))
    # pixel checksum of the PIL decode, so the box can verify it decodes identically
    np.savez_compressed(os.path.join(flir, "decode_check.npz"),
                        left_sum=np.int64(L.astype(np.int64).sum()), right_sum=np.int64(R.astype(np.int64).sum()),
                        left_row0=L[0].copy(), right_row0=R[0].copy())
    print("copied FLIR pair")


if __name__ == "__main__":
    main()
