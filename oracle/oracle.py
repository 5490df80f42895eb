"""oracle.py -- TEST INFRASTRUCTURE ONLY.

ctypes bindings for oracle/liboracle.so (the CPU restatement of the Stereo3DMST path,
see sm_oracle.h) and for oracle/_ref/libref_segment.so (the reference's own
segment-graph.h compiled from /root/reference, present only in the build container).

Allowed importers: tests/, __graft_entry__.smoke(), bench.py's cpu_baseline leg.
The product package stereomatch_amd never imports this module.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None
_REF = None

u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
u16p = np.ctypeslib.ndpointer(np.uint16, flags="C_CONTIGUOUS")
i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
c_int, c_float, vp = ctypes.c_int, ctypes.c_float, ctypes.c_void_p


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError("oracle not built: run `make -C oracle` (liboracle.so missing)")
        L = ctypes.CDLL(path)
        L.orc_median3.argtypes = [u8p, c_int, c_int, c_int, u8p]
        L.orc_edge_weights.argtypes = [u8p, c_int, c_int, u16p, u16p]
        L.orc_segment.argtypes = [c_int, c_int, u16p, u16p, c_float, c_int, u8p]
        L.orc_segment.restype = c_int
        L.orc_bfs.argtypes = [c_int, c_int, u16p, u16p, u8p, i32p, i32p, i32p, u16p, u8p, i32p]
        L.orc_bfs.restype = c_int
        L.orc_cost_agd.argtypes = [u8p, u8p, c_int, c_int, c_int, c_int, c_int, vp, vp, c_int]
        L.orc_tree_filter.argtypes = [c_int, c_int, c_int, c_int, c_int, i32p, i32p, i32p, u16p, u8p,
                                      i32p, f32p, vp, vp, vp, vp, c_int]
        L.orc_s_lut.restype = ctypes.POINTER(ctypes.c_double)
        L.orc_s2_lut.restype = ctypes.POINTER(ctypes.c_double)
        L.orc_agd_color_term.argtypes = [c_int]
        L.orc_agd_color_term.restype = c_float
        L.orc_lr_check.argtypes = [vp, vp, c_int, c_int, c_int]
        L.orc_lr_check_fill.argtypes = [vp, vp, c_int, c_int, c_int, c_int]
        L.orc_label_to_disp.argtypes = [vp, ctypes.c_long, c_int]
        L.orc_set_agd_contract.argtypes = [c_int]
        L.orc_set_gf_contract.argtypes = [c_int]
        L.orc_guided_filter.argtypes = [u8p, c_int, c_int, c_int, vp, c_int, c_int, c_float, vp, c_int]
        L.orc_box_mean.argtypes = [vp, vp, c_int, c_int, c_int]
        L.orc_select_disparity.argtypes = [vp, c_int, c_int, c_int, ctypes.c_size_t, c_int, vp, vp, vp]
        L.orc_occlusion.argtypes = [vp, vp, c_int, c_int, c_int, c_float, c_int]
        L.orc_pms_dice.argtypes = [ctypes.c_long, f32p]
        L.orc_glibc_random.argtypes = [ctypes.c_uint, ctypes.c_long, ctypes.c_long, i32p]
        L.orc_pms_init_labels.argtypes = [c_int, c_int, c_int, f32p]
        L.orc_label_cost.argtypes = [f32p, c_float, c_float, c_float, c_int, c_int, c_int, ctypes.c_size_t]
        L.orc_label_cost.restype = c_float
        L.orc_pms_label_to_disp.argtypes = [f32p, c_int, c_int, c_int, f32p]
        L.orc_pms_plane_disp.argtypes = [f32p, c_int, c_int, f32p]
        L.orc_tree_graph.argtypes = [c_int, c_int, c_int, i32p, i32p, i32p, i32p, c_int]
        L.orc_tree_graph.restype = c_int
        L.orc_mst_pms.argtypes = [c_int, c_int, c_int, c_int, i32p, i32p, i32p, u16p, u8p, i32p, i32p, i32p, f32p,
                                  f32p, f64p, f32p, ctypes.c_long, i32p, vp]
        L.orc_mst_pms.restype = ctypes.c_long
        _LIB = L
    return _LIB


def ref_lib():
    """The reference's segment_graph (oracle/_ref); None when not built (e.g. on the GPU box)."""
    global _REF
    if _REF is None:
        path = os.path.join(HERE, "_ref", "libref_segment.so")
        if not os.path.exists(path):
            return None
        R = ctypes.CDLL(path)
        R.ref_segment_graph.argtypes = [c_int, c_int, i32p, i32p, f64p, c_float, i32p, i32p, f64p, i32p]
        R.ref_segment_graph.restype = c_int
        _REF = R
    return _REF


def _ptr(a):
    return None if a is None else a.ctypes.data_as(vp)


def s_lut():
    L = lib()
    return np.ctypeslib.as_array(L.orc_s_lut(), shape=(766,)).copy()


def s2_lut():
    L = lib()
    return np.ctypeslib.as_array(L.orc_s2_lut(), shape=(766,)).copy()


def median3(img):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    H, W, _ = img.shape
    out = np.empty((H, W, 3), np.uint8)
    lib().orc_median3(img, W, H, W * 3, out)
    return out


def edge_weights(med):
    med = np.ascontiguousarray(med, dtype=np.uint8)
    H, W, _ = med.shape
    wR = np.empty(H * W, np.uint16)
    wD = np.empty(H * W, np.uint16)
    lib().orc_edge_weights(med, W, H, wR, wD)
    return wR, wD


def segment(W, H, wR, wD, c=float("inf"), min_size=200):
    mask = np.empty(H * W, np.uint8)
    n = lib().orc_segment(W, H, wR, wD, c, min_size, mask)
    return mask, n


def bfs(W, H, wR, wD, mask):
    N = W * H
    tree_start = np.empty(N + 1, np.int32)
    node_pix = np.empty(N, np.int32)
    node_parent = np.empty(N, np.int32)
    node_w = np.empty(N, np.uint16)
    node_nch = np.empty(N, np.uint8)
    node_child = np.empty(4 * N, np.int32)
    nt = lib().orc_bfs(W, H, wR, wD, mask, tree_start, node_pix, node_parent, node_w, node_nch, node_child)
    return dict(ntrees=nt, tree_start=tree_start[:nt + 1].copy(), node_pix=node_pix, node_parent=node_parent,
                node_w=node_w, node_nch=node_nch, node_child=node_child)


def set_gf_contract(mode):
    """1: the guided filter's helper kernels contracted as nvcc's default --fmad=true would (what-if
    for tools/gf_contraction.py); 0: the shipped, uncontracted restatement."""
    lib().orc_set_gf_contract(int(mode))


def set_agd_contract(mode):
    """Oracle-only switch: 1 = the AGD cost with the FMAs nvcc's default --fmad=true forms."""
    lib().orc_set_agd_contract(int(mode))


def cost_agd(left, right, d0, d1, nthreads=0):
    left = np.ascontiguousarray(left, dtype=np.uint8)
    right = np.ascontiguousarray(right, dtype=np.uint8)
    H, W, _ = left.shape
    lv = np.empty((d1 - d0, H, W), np.float32)
    rv = np.empty((d1 - d0, H, W), np.float32)
    lib().orc_cost_agd(left, right, W, H, W * 3, d0, d1, _ptr(lv), _ptr(rv), int(nthreads))
    return lv, rv


def tree_filter(W, H, tree, vol, d0=0, want_idx=True, want_volumes=False, nthreads=0):
    nd = vol.shape[0]
    N = W * H
    idx = np.empty(N, np.int32) if want_idx else None
    minc = np.empty(N, np.float64) if want_idx else None
    Aup = np.empty((nd, H, W), np.float64) if want_volumes else None
    A = np.empty((nd, H, W), np.float64) if want_volumes else None
    lib().orc_tree_filter(W, H, nd, d0, tree["ntrees"], tree["tree_start"], tree["node_pix"], tree["node_parent"],
                          tree["node_w"], tree["node_nch"], tree["node_child"],
                          np.ascontiguousarray(vol, dtype=np.float32),
                          _ptr(idx), _ptr(minc), _ptr(Aup), _ptr(A), nthreads)
    return dict(idx=idx, minc=minc, Aup=Aup, A=A)


def mccnn_clamp(vol):
    """MC-CNN ingest clamp of Stereo3DMST.cpp:785-803: NaN -> 0.5, else min(0.5f, x)
    (std::min(a, b) returns b only if b < a)."""
    v = np.asarray(vol, dtype=np.float32)
    return np.where(np.isnan(v), np.float32(0.5), np.where(v < np.float32(0.5), v, np.float32(0.5))).astype(np.float32)


def build_tree(img, c=float("inf"), min_size=200):
    """median -> edge weights -> segment/MST -> BFS rooting, for one view."""
    H, W, _ = img.shape
    med = median3(img)
    wR, wD = edge_weights(med)
    mask, ncomp = segment(W, H, wR, wD, c, min_size)
    tree = bfs(W, H, wR, wD, mask)
    tree.update(med=med, wR=wR, wD=wD, mask=mask)
    return tree


def match(left, right, D, c=float("inf"), min_size=200, want_volumes=False, nthreads=0):
    """The whole path on the CPU: both views, slices 0..D-1.  Returns per-view dicts."""
    H, W, _ = left.shape
    lv, rv = cost_agd(left, right, 0, D, nthreads)
    out = {}
    for name, img, vol in (("left", left, lv), ("right", right, rv)):
        tree = build_tree(img, c, min_size)
        res = tree_filter(W, H, tree, vol, 0, True, want_volumes, nthreads)
        res["tree"] = tree
        res["vol"] = vol
        out[name] = res
    return out


def ref_segment_graph(W, H, wR, wD, c):
    """Run the reference's own segment_graph on the 4-connected edges of (wR, wD).
    Returns the per-pixel mask in ORC_EDGE_* encoding and num_sets, or None if _ref is absent."""
    R = ref_lib()
    if R is None:
        return None
    a, b, w = [], [], []
    for p in range(W * H):  # emission order of Stereo3DMST.cpp:244-262
        x, y = p % W, p // W
        if x < W - 1:
            a.append(p); b.append(p + 1); w.append(float(wR[p]))
        if y < H - 1:
            a.append(p); b.append(p + W); w.append(float(wD[p]))
    E = len(a)
    a = np.array(a, np.int32); b = np.array(b, np.int32); w = np.array(w, np.float64)
    oa = np.empty(E, np.int32); ob = np.empty(E, np.int32); ow = np.empty(E, np.float64); om = np.empty(E, np.int32)
    nsets = R.ref_segment_graph(W * H, E, a, b, w, c, oa, ob, ow, om)
    mask = np.zeros(W * H, np.uint8)
    sel = om == 1
    right = sel & (ob == oa + 1) & (W > 1)
    down = sel & ~right
    np.bitwise_or.at(mask, oa[right], 1)
    np.bitwise_or.at(mask, oa[down], 2)
    return dict(mask=mask, nsets=nsets, sorted_a=oa, sorted_b=ob, sorted_w=ow, sorted_mask=om)


def lr_check(left_disp, right_disp, max_disp, fill=False):
    """Stereo3DMST.cpp:632-709 (fill=false as at :904); returns a new left map."""
    left = np.ascontiguousarray(left_disp, dtype=np.float32).copy()
    right = np.ascontiguousarray(right_disp, dtype=np.float32)
    H, W = left.shape
    lib().orc_lr_check_fill(_ptr(left), _ptr(right), W, H, int(max_disp), 1 if fill else 0)
    return left


def label_to_disp(disp, dmax):
    """LabelToDisp of the label (0, 0, d) + the *= (Dmax-1) scaling (Stereo3DMST.cpp:189-201, 900-902)."""
    d = np.ascontiguousarray(disp, dtype=np.float32).copy()
    lib().orc_label_to_disp(_ptr(d), d.size, int(dmax))
    return d


def stereo3dmst_output(left_idx, right_idx, dmax, fill=False):
    """stereo3dmst's output step on the per-slice WTA maps: LabelToDisp + scaling of both maps, then
    the L-R check of the left map (Stereo3DMST.cpp:900-904).  Returns (left_disp, right_disp)."""
    ld = label_to_disp(np.asarray(left_idx).astype(np.float32), dmax)
    rd = label_to_disp(np.asarray(right_idx).astype(np.float32), dmax)
    return lr_check(ld, rd, dmax, fill), rd


def subpixel(A, idx, dglob0, dtot):
    """selectDisparity's parabola (PatchMatchStereoGPU.cu:1726-1736) on the WTA winners, float32:
    A = [nd][H][W] fp64 aggregated costs of global slices dglob0.., idx = global winners; the
    neighbours' costs as float (0 at the ends of [0, dtot)); disp = d - s if |s| < 1 else d."""
    nd = A.shape[0]
    flat = A.reshape(nd, -1)
    i = np.asarray(idx).ravel().astype(np.int64)
    m = i - dglob0
    p = np.arange(flat.shape[1])
    f32 = np.float32
    cur = flat[m, p].astype(f32)
    pre = np.where(i > 0, flat[np.clip(m - 1, 0, nd - 1), p].astype(f32), f32(0))
    nxt = np.where(i < dtot - 1, flat[np.clip(m + 1, 0, nd - 1), p].astype(f32), f32(0))
    with np.errstate(all="ignore"):
        s = ((nxt - pre) * f32(0.5) / ((nxt - f32(2.0) * cur) + pre)).astype(f32)
    g = i.astype(f32)
    return np.where(np.abs(s) < f32(1.0), g - s, g).astype(f32)


def guided_filter(img, vol, radius=9, eps=6.5025, nthreads=0):
    """Colour guided filter of a [nd][H][W] float cost volume, guided by the view's BGR image
    (PatchMatchStereoGPU.cu:8251-8470)."""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    H, W, _ = img.shape
    v = np.ascontiguousarray(vol, dtype=np.float32)
    out = np.empty_like(v)
    lib().orc_guided_filter(img, W, H, W * 3, _ptr(v), v.shape[0], int(radius), float(eps), _ptr(out), int(nthreads))
    return out


def box_mean(a, r):
    a = np.ascontiguousarray(a, dtype=np.float32)
    out = np.empty_like(a)
    lib().orc_box_mean(_ptr(a), _ptr(out), a.shape[1], a.shape[0], int(r))
    return out


def select_disparity(vol, d0=0, dtot=None, sub=False):
    """selectDisparity (PatchMatchStereoGPU.cu:1688-1737) of a float [nd][H][W] volume."""
    v = np.ascontiguousarray(vol, dtype=np.float32)
    nd = v.shape[0]
    N = v[0].size
    idx = np.empty(N, np.int32)
    mn = np.empty(N, np.float32)
    disp = np.empty(N, np.float32)
    lib().orc_select_disparity(_ptr(v), nd, int(d0), int(dtot if dtot else d0 + nd), N, 1 if sub else 0, _ptr(idx),
                               _ptr(mn), _ptr(disp))
    return idx, mn, disp


def guided_match(left, right, D, radius=9, eps=6.5025, sub=False, nthreads=0):
    """The guided-filter aggregator end to end: AGD cost, colour guided filter per view (guide: the
    view's own image), selectDisparity.  Returns per-view dicts idx / minc / disp / vol."""
    lv, rv = cost_agd(left, right, 0, D, nthreads)
    out = {}
    for name, img, vol in (("left", left, lv), ("right", right, rv)):
        f = guided_filter(img, vol, radius, eps, nthreads)
        idx, mn, disp = select_disparity(f, 0, D, sub)
        out[name] = dict(idx=idx, minc=mn, disp=disp, vol=f)
    return out


def occlusion(left_disp, right_disp, min_disp=0, thresh=1.0, remove=False):
    """handleOcclusionSharedMemory (PatchMatchStereoGPU.cu:1128-1288); returns new (left, right)."""
    L = np.ascontiguousarray(left_disp, dtype=np.float32).copy()
    R = np.ascontiguousarray(right_disp, dtype=np.float32).copy()
    H, W = L.shape
    lib().orc_occlusion(_ptr(L), _ptr(R), W, H, int(min_disp), float(thresh), 1 if remove else 0)
    return L, R


# ---------------------------------------------------------------- MST_PMS (Stereo3DMST.cpp:546-629)
def pms_dice(n):
    """The (-1, 1) dice stream every MST_PMS call replays (minstd_rand0 seed 1, :554 / :851-852)."""
    out = np.empty(int(n), np.float32)
    lib().orc_pms_dice(int(n), out)
    return out


def glibc_random(seed, skip, n):
    """glibc random()/rand() outputs skip..skip+n-1 after srandom(seed) (TYPE_3)."""
    out = np.empty(int(n), np.int32)
    lib().orc_glibc_random(int(seed), int(skip), int(n), out)
    return out


def pms_init_labels(W, H, max_disp):
    """segment_image_other_init's random plane labels (:390-430): [H*W, 3] float (a, b, c)."""
    abc = np.empty((H * W, 3), np.float32)
    lib().orc_pms_init_labels(W, H, int(max_disp), abc)
    return abc


def pms_levels(max_disp):
    """Refinement levels per tree (:597-600): max_d = 0.5*Dmax halved while > 0.1f."""
    md, n = np.float32(0.5) * np.float32(max_disp), 0
    while md > np.float32(0.1):
        n += 1
        md = np.float32(md * np.float32(0.5))
    return n


def tree_graph(W, H, tree):
    """tree_g (:377-384) as CSR (nb_start, nb), neighbours ascending."""
    nt = tree["ntrees"]
    nb_start = np.empty(nt + 1, np.int32)
    cap = 4 * W * H + 4
    nb = np.empty(cap, np.int32)
    n = lib().orc_tree_graph(W, H, nt, tree["tree_start"], tree["node_pix"], nb_start, nb, cap)
    if n < 0:
        raise RuntimeError("tree_graph: capacity")
    return nb_start, nb[:n].copy()


def dice_budget(tree, nb_start, max_disp):
    """Upper bound of the dice values one MST_PMS call consumes: deg(t) + 4 per refinement level."""
    return int(nb_start[-1]) + 4 * pms_levels(max_disp) * int(tree["ntrees"]) + 4


def mst_pms(W, H, max_disp, tree, nb_start, nb, vol, abc, min_cost, dice, rnd, stats=False):
    """One MST_PMS call over one view, in place on abc [N,3] f32 and min_cost [N] f64.  Returns the dice
    values consumed (and per-tree stats {dice, prop changes, refinement changes, test pixel})."""
    st = np.empty((tree["ntrees"], 4), np.int32) if stats else None
    k = lib().orc_mst_pms(W, H, int(max_disp), tree["ntrees"], tree["tree_start"], tree["node_pix"],
                          tree["node_parent"], tree["node_w"], tree["node_nch"], tree["node_child"], nb_start, nb,
                          np.ascontiguousarray(vol, dtype=np.float32), abc, min_cost, dice, dice.size,
                          np.ascontiguousarray(rnd, dtype=np.int32), _ptr(st))
    if k < 0:
        raise RuntimeError("mst_pms: dice stream exhausted or a propagation index out of its tree")
    return (k, st) if stats else k


def pms_label_to_disp(abc, W, H, max_disp):
    """LabelToDisp (:189-201) + *= (Dmax-1.f) (:900-902) of plane labels: [H, W] float."""
    out = np.empty(W * H, np.float32)
    lib().orc_pms_label_to_disp(np.ascontiguousarray(abc, dtype=np.float32), W, H, int(max_disp), out)
    return out.reshape(H, W)


def pms_plane_disp(abc, W, H):
    """fma(x, a, y*b) + c per pixel (LabelToDisp's plane value before its clamp, :197): [H, W] float."""
    out = np.empty(W * H, np.float32)
    lib().orc_pms_plane_disp(np.ascontiguousarray(abc, dtype=np.float32), W, H, out)
    return out.reshape(H, W)


def stereo3dmst_pms(left, right, max_disp, iters=100, vols=None, c=5000.0, min_size=200, stats=False):
    """The reference's stereo3dmst() after the cost volume (Stereo3DMST.cpp:805-904): segment forests
    of both views, random plane init, `iters` MST_PMS calls on the left view then on the right, plane
    LabelToDisp + scaling, L-R check of the left map (no fill).  vols: (left, right) [Dmax][H][W] data
    costs (default: the AGD volumes).  glibc's rand() stream starts after random_rgb's 3 draws per pixel
    of both views (:316)."""
    H, W, _ = left.shape
    if vols is None:
        vols = cost_agd(left, right, 0, max_disp)
    out = {}
    trees = [build_tree(img, c, min_size) for img in (left, right)]
    nbs = [tree_graph(W, H, t) for t in trees]
    K = [t["ntrees"] for t in trees]
    rnd = glibc_random(1, 6 * W * H, iters * (K[0] + K[1]))
    dice = pms_dice(max(dice_budget(t, nb[0], max_disp) for t, nb in zip(trees, nbs)))
    abc0 = pms_init_labels(W, H, max_disp)
    off = 0
    for v, name in enumerate(("left", "right")):
        abc = abc0.copy()
        minc = np.full(W * H, np.finfo(np.float64).max)
        st_all = []
        for _ in range(iters):
            r = mst_pms(W, H, max_disp, trees[v], nbs[v][0], nbs[v][1], vols[v], abc, minc, dice,
                        rnd[off:off + K[v]], stats)
            if stats:
                st_all.append(r[1])
            off += K[v]
        out[name] = dict(abc=abc, minc=minc, tree=trees[v], nb=nbs[v], disp=pms_label_to_disp(abc, W, H, max_disp))
        if stats:
            out[name]["stats"] = st_all
    out["left"]["disp_checked"] = lr_check(out["left"]["disp"], out["right"]["disp"], max_disp, False)
    out["abc0"] = abc0
    return out
