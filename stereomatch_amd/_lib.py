"""ctypes binding of libstereomst.so (include/stereomst.h).

The HIP library is the only compute path: if it is missing or no GPU is present the
calls raise -- there is no CPU fallback in this package.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# SM_LIB: an alternative build of the same library (diagnostic builds, tools/chain_prof.sh)
LIB_PATH = os.environ.get("SM_LIB") or os.path.join(HERE, "libstereomst.so")

SM_OK, SM_ERR_ARG, SM_ERR_HIP, SM_ERR_OOM, SM_ERR_RCCL, SM_ERR_STATE, SM_ERR_NODEVICE = range(7)
STATUS_NAMES = {0: "SM_OK", 1: "SM_ERR_ARG", 2: "SM_ERR_HIP", 3: "SM_ERR_OOM", 4: "SM_ERR_RCCL",
                5: "SM_ERR_STATE", 6: "SM_ERR_NODEVICE"}
SM_COST_AGD, SM_COST_VOLUME = 0, 1
SM_POST_LR_CHECK, SM_POST_LABEL_TO_DISP, SM_POST_LR_FILL, SM_POST_OCCLUSION, SM_POST_OCCLUSION_ZERO = 1, 2, 4, 8, 16
SM_POST_SUBPIXEL = 32
SM_AGG_TREE, SM_AGG_GUIDED, SM_AGG_PMS = 0, 1, 2
SM_UNIQUE_ID_BYTES = 128


class SmConfig(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int), ("max_width", ctypes.c_int), ("max_height", ctypes.c_int),
                ("max_disp", ctypes.c_int)]


class SmParams(ctypes.Structure):
    _fields_ = [("gamma", ctypes.c_float), ("c", ctypes.c_float), ("min_size", ctypes.c_int),
                ("median_ksize", ctypes.c_int), ("cost_kind", ctypes.c_int), ("disp_begin", ctypes.c_int),
                ("disp_total", ctypes.c_int), ("post", ctypes.c_int), ("aggregator", ctypes.c_int),
                ("gf_radius", ctypes.c_int), ("gf_eps", ctypes.c_float), ("views", ctypes.c_int),
                ("pms_iters", ctypes.c_int)]


class SmPmsStats(ctypes.Structure):
    _fields_ = [("iters", ctypes.c_int), ("ntrees", ctypes.c_int * 2), ("spec_rounds", ctypes.c_int),
                ("serial_trees", ctypes.c_int), ("prep_ms", ctypes.c_double), ("setup_ms", ctypes.c_double),
                ("iter0_ms", ctypes.c_double), ("iters_ms", ctypes.c_double), ("total_ms", ctypes.c_double),
                ("calls_ms", ctypes.c_double), ("concurrent_views", ctypes.c_int),
                ("first_ms_view", ctypes.c_double * 2), ("later_ms_view", ctypes.c_double * 2),
                ("evals_first", ctypes.c_double), ("evals_first_ref", ctypes.c_double),
                ("evals_first_run", ctypes.c_double), ("evals_later", ctypes.c_double),
                ("evals_later_ref", ctypes.c_double), ("evals_later_run", ctypes.c_double),
                ("prep_seg_ms", ctypes.c_double), ("prep_forest_ms", ctypes.c_double)]


class SmFilterStats(ctypes.Structure):
    _fields_ = [("up_ms", ctypes.c_double), ("down_ms", ctypes.c_double), ("up_bytes", ctypes.c_double),
                ("down_bytes", ctypes.c_double), ("up_launches", ctypes.c_int), ("down_launches", ctypes.c_int)]


class SmKernelStat(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * 32), ("launches", ctypes.c_int), ("ms", ctypes.c_double),
                ("voxels", ctypes.c_double), ("bytes_per_voxel", ctypes.c_double)]


class StereoMSTError(RuntimeError):
    def __init__(self, status, msg):
        super().__init__("%s: %s" % (STATUS_NAMES.get(status, str(status)), msg))
        self.status = status


_lib = None
vp = ctypes.c_void_p
ci = ctypes.c_int


def lib():
    """Load the in-tree HIP library (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError("stereomatch_amd HIP library missing (%s): run __graft_entry__.build() or "
                           "`make -C stereomatch_amd/csrc`" % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    sigs = {
        "sm_version": ([], ctypes.c_char_p),
        "sm_default_params": ([ctypes.POINTER(SmParams)], None),
        "sm_device_count": ([ctypes.POINTER(ci)], ci),
        "sm_create": ([ctypes.POINTER(vp), ctypes.POINTER(SmConfig)], ci),
        "sm_destroy": ([vp], None),
        "sm_last_error": ([vp], ctypes.c_char_p),
        "sm_match": ([vp, vp, vp, ci, ci, ci, ci, ctypes.POINTER(SmParams), vp, vp, vp, vp, vp, vp], ci),
        "sm_upload_images": ([vp, vp, vp, ci, ci, ci], ci),
        "sm_upload_cost_volumes": ([vp, vp, vp, ci, ci, ci], ci),
        "sm_match_async": ([vp, ci, ctypes.POINTER(SmParams)], ci),
        "sm_match_begin": ([vp, ci, ctypes.POINTER(SmParams)], ci),
        "sm_match_finish": ([vp], ci),
        "sm_synchronize": ([vp], ci),
        "sm_download_results": ([vp, vp, vp, vp, vp, vp, vp], ci),
        "sm_cost_volume": ([vp, vp, vp, ci, ci, ci, ci, ci, vp, vp], ci),
        "sm_build_tree": ([vp, vp, ci, ci, ci, vp, vp, vp, vp], ci),
        "sm_build_tree_p": ([vp, vp, ci, ci, ci, ctypes.POINTER(SmParams), vp, vp, vp, vp, vp], ci),
        "sm_aggregate_debug": ([vp, vp, vp, ci, ci, ci, ci, ci, ci, vp, vp], ci),
        "sm_aggregate_debug_p": ([vp, vp, vp, ci, ci, ci, ctypes.POINTER(SmParams), ci, ci, ci, vp, vp], ci),
        "sm_stage_times": ([vp, vp, ci], ci),
        "sm_get_filter_stats": ([vp, ctypes.POINTER(SmFilterStats)], ci),
        "sm_get_kernel_stats": ([vp, ctypes.POINTER(SmKernelStat), ci], ci),
        "sm_set_kernel_timing": ([vp, ctypes.c_uint], ci),
        "sm_download_labels": ([vp, vp, vp], ci),
        "sm_get_pms_stats": ([vp, ctypes.POINTER(SmPmsStats)], ci),
        "sm_get_pms_stats_n": ([vp, ctypes.POINTER(SmPmsStats), ctypes.c_size_t], ci),
        "sm_labels_extent": ([vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)], ci),
        "sm_pms_forest_bfs": ([ci, ci, vp, vp, vp, vp, vp, vp, vp, vp, vp], ci),
        "sm_pms_forest_digest": ([ci, ci, vp, vp, vp, ci, ci, vp, vp, vp], ci),
        "sm_pms_tree_graph": ([ci, ci, vp, vp, vp, vp, vp, ci], ci),
        "sm_pms_dice": ([ctypes.c_long, vp], None),
        "sm_pms_glibc_random": ([ctypes.c_uint, ctypes.c_long, ctypes.c_long, vp], None),
        "sm_pms_init_labels": ([ci, ci, ci, vp], None),
        "sm_pms_levels": ([ci], ci),
        "sm_reduce_candidates": ([vp, vp, vp, vp, ci, vp, ctypes.c_size_t], None),
        "sm_reduce_finalize": ([vp, vp, ci, vp, vp, vp, ctypes.c_size_t], None),
        "sm_comm_unique_id": ([vp], ci),
        "sm_comm_init": ([vp, ci, ci, vp], ci),
        "sm_comm_destroy": ([vp], ci),
        "sm_start_timer": ([ctypes.POINTER(ctypes.c_double)], None),
        "sm_get_timer_ms": ([ctypes.POINTER(ctypes.c_double)], ctypes.c_double),
        "sm_set_knob": ([ctypes.c_char_p, ctypes.c_char_p], ci),
        "sm_knob_names": ([ctypes.POINTER(ctypes.c_char_p), ci], ci),
    }
    for name, (args, res) in sigs.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def set_knob(name, value):
    """sm_set_knob: a tuning / diagnostic knob of the library (include/stereomst.h); value None restores
    the default.  Knobs are never read from the environment by the product library."""
    st = lib().sm_set_knob(name.encode(), None if value is None else str(value).encode())
    if st != SM_OK:
        raise StereoMSTError(st, "sm_set_knob(%s): not a knob" % name)


def knob_names():
    n = lib().sm_knob_names(None, 0)
    buf = (ctypes.c_char_p * n)()
    lib().sm_knob_names(buf, n)
    return [buf[i].decode() for i in range(n)]


def default_params(**overrides):
    p = SmParams()
    lib().sm_default_params(ctypes.byref(p))
    for k, v in overrides.items():
        setattr(p, k, v)
    return p


def _active(out, views):
    """The views a call computed (sm_params.views: 1 left, 2 right, 3 both)."""
    return {v: out[v] for i, v in enumerate(("left", "right")) if (views >> i) & 1}


def device_count():
    n = ci(0)
    lib().sm_device_count(ctypes.byref(n))
    return n.value


def ptr(a):
    return None if a is None else a.ctypes.data_as(vp)


def as_image(img):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    if img.ndim != 3 or img.shape[2] != 3:
        raise ValueError("expected an HxWx3 uint8 BGR image")
    return img


class Context:
    """One sm_ctx (one HIP device, one stream).  Not thread-safe: one per host thread."""

    def __init__(self, device=0, max_width=0, max_height=0, max_disp=0):
        L = lib()
        cfg = SmConfig(device, max_width, max_height, max_disp)
        h = vp()
        st = L.sm_create(ctypes.byref(h), ctypes.byref(cfg))
        if st != SM_OK:
            raise StereoMSTError(st, "sm_create failed (no HIP device?)")
        self.h = h
        self.device = device

    def close(self):
        if getattr(self, "h", None):
            lib().sm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, st):
        if st != SM_OK:
            msg = lib().sm_last_error(self.h)
            raise StereoMSTError(st, msg.decode() if msg else "")

    # -- whole path --------------------------------------------------------------------
    def match(self, left, right, D, params=None):
        left, right = as_image(left), as_image(right)
        H, W, _ = left.shape
        if right.shape != left.shape:
            raise ValueError("left/right shapes differ")
        p = params or default_params()
        out = {v: dict(disp=np.empty((H, W), np.float32), idx=np.empty((H, W), np.int32),
                       minc=np.empty((H, W), np.float64)) for v in ("left", "right")}
        self._views = p.views or 3
        self.shape = (H, W)
        self._check(lib().sm_match(self.h, ptr(left), ptr(right), W, H, W * 3, D, ctypes.byref(p),
                                   ptr(out["left"]["disp"]), ptr(out["right"]["disp"]), ptr(out["left"]["idx"]),
                                   ptr(out["right"]["idx"]), ptr(out["left"]["minc"]), ptr(out["right"]["minc"])))
        return _active(out, self._views)

    def upload(self, left, right):
        left, right = as_image(left), as_image(right)
        H, W, _ = left.shape
        self.shape = (H, W)
        self._check(lib().sm_upload_images(self.h, ptr(left), ptr(right), W, H, W * 3))

    def upload_cost_volumes(self, left_vol, right_vol):
        """Raw [D][H][W] float32 matching-cost volumes (MC-CNN left.bin / right.bin layout) for
        matches with cost_kind=SM_COST_VOLUME (clamped as Stereo3DMST.cpp:785-803 on the GPU)."""
        lv = np.ascontiguousarray(left_vol, dtype=np.float32)
        rv = np.ascontiguousarray(right_vol, dtype=np.float32)
        if lv.ndim != 3 or lv.shape != rv.shape:
            raise ValueError("expected two same-shaped [D][H][W] volumes")
        D, H, W = lv.shape
        self._check(lib().sm_upload_cost_volumes(self.h, ptr(lv), ptr(rv), W, H, D))

    def match_async(self, D, params=None):
        p = params or default_params()
        self._views = p.views or 3
        self._check(lib().sm_match_async(self.h, D, ctypes.byref(p)))

    def match_begin(self, D, params=None):
        """sm_match_begin: enqueue prep, MST and layout; the filter follows in match_finish."""
        p = params or default_params()
        self._views = p.views or 3
        self._check(lib().sm_match_begin(self.h, D, ctypes.byref(p)))

    def match_finish(self):
        """sm_match_finish: wait for the layout's round counts, enqueue filter, reduce, output step."""
        self._check(lib().sm_match_finish(self.h))

    def synchronize(self):
        self._check(lib().sm_synchronize(self.h))

    def results(self):
        H, W = self.shape
        out = {v: dict(disp=np.empty((H, W), np.float32), idx=np.empty((H, W), np.int32),
                       minc=np.empty((H, W), np.float64)) for v in ("left", "right")}
        self._check(lib().sm_download_results(self.h, ptr(out["left"]["disp"]), ptr(out["right"]["disp"]),
                                              ptr(out["left"]["idx"]), ptr(out["right"]["idx"]),
                                              ptr(out["left"]["minc"]), ptr(out["right"]["minc"])))
        return _active(out, getattr(self, "_views", 3))

    def stage_times(self):
        buf = (ctypes.c_float * 7)()
        n = lib().sm_stage_times(self.h, buf, 7)
        names = ["prep_ms", "mst_ms", "layout_ms", "up_ms", "down_ms", "reduce_ms", "total_ms"]
        return {names[i]: float(buf[i]) for i in range(n)}

    def filter_stats(self):
        s = SmFilterStats()
        self._check(lib().sm_get_filter_stats(self.h, ctypes.byref(s)))
        return {k: getattr(s, k) for k, _ in SmFilterStats._fields_}

    def kernel_stats(self):
        """Per kernel family of the tree filter (last call): launches, ms, voxels, bytes/voxel."""
        buf = (SmKernelStat * 8)()
        n = lib().sm_get_kernel_stats(self.h, buf, 8)
        return {buf[i].name.decode(): dict(launches=buf[i].launches, ms=buf[i].ms, voxels=buf[i].voxels,
                                           bytes_per_voxel=buf[i].bytes_per_voxel) for i in range(n)}

    def set_kernel_timing(self, families=None):
        """Time only these kernel families with HIP events (names as in kernel_stats(); None = all)."""
        mask = 0xFFFFFFFF
        if families is not None:
            names = list(self.kernel_stats().keys())
            mask = 0
            for f in families:
                mask |= 1 << names.index(f)
        self._check(lib().sm_set_kernel_timing(self.h, ctypes.c_uint(mask)))

    # -- MST_PMS (SM_AGG_PMS) -------------------------------------------------------------
    def labels(self):
        """Plane labels (a, b, c) of every pixel after the last SM_AGG_PMS call: {view: [H*W, 3] float32}."""
        # sized from the library's own record of the SM_AGG_PMS call (not Python-side bookkeeping: a
        # match_begin / match_async call or a later upload must not change what this allocates)
        w, h = ctypes.c_int(0), ctypes.c_int(0)
        self._check(lib().sm_labels_extent(self.h, ctypes.byref(w), ctypes.byref(h)))
        H, W = h.value, w.value
        out = {v: np.empty((H * W, 3), np.float32) for v in ("left", "right")}
        self._check(lib().sm_download_labels(self.h, ptr(out["left"]), ptr(out["right"])))
        return out

    def pms_stats(self):
        s = SmPmsStats()
        self._check(lib().sm_get_pms_stats_n(self.h, ctypes.byref(s), ctypes.sizeof(s)))
        d = {k: getattr(s, k) for k, _ in SmPmsStats._fields_}
        d["ntrees"] = list(s.ntrees)
        d["first_ms_view"] = list(s.first_ms_view)
        d["later_ms_view"] = list(s.later_ms_view)
        return d

    # -- stages ---------------------------------------------------------------------------
    def cost_volume(self, left, right, d0, D):
        left, right = as_image(left), as_image(right)
        H, W, _ = left.shape
        lv = np.empty((D, H, W), np.float32)
        rv = np.empty((D, H, W), np.float32)
        self._check(lib().sm_cost_volume(self.h, ptr(left), ptr(right), W, H, W * 3, d0, D, ptr(lv), ptr(rv)))
        return lv, rv

    def build_tree(self, img, params=None):
        """The tree of one view: the MST, or with params.c finite the segment forest (roots: parent -1)."""
        img = as_image(img)
        H, W, _ = img.shape
        mask = np.empty(H * W, np.uint8)
        parent = np.empty(H * W, np.int32)
        size = np.empty(H * W, np.int32)
        slot = np.empty(H * W, np.int32)
        nt = ctypes.c_int32(0)
        if params is None:
            self._check(lib().sm_build_tree(self.h, ptr(img), W, H, W * 3, ptr(mask), ptr(parent), ptr(size), ptr(slot)))
            nt.value = 1
        else:
            self._check(lib().sm_build_tree_p(self.h, ptr(img), W, H, W * 3, ctypes.byref(params), ptr(mask), ptr(parent),
                                              ptr(size), ptr(slot), ctypes.byref(nt)))
        return dict(mask=mask, parent_pix=parent, subtree_size=size, slot_of_pix=slot, ntrees=nt.value)

    def aggregate_debug(self, left, right, view, d0, D, params=None):
        left, right = as_image(left), as_image(right)
        H, W, _ = left.shape
        Aup = np.empty((D, H, W), np.float64)
        A = np.empty((D, H, W), np.float64)
        if params is None:
            self._check(lib().sm_aggregate_debug(self.h, ptr(left), ptr(right), W, H, W * 3, view, d0, D, ptr(Aup),
                                                 ptr(A)))
        else:
            self._check(lib().sm_aggregate_debug_p(self.h, ptr(left), ptr(right), W, H, W * 3, ctypes.byref(params), view,
                                                   d0, D, ptr(Aup), ptr(A)))
        return Aup, A

    # -- multi-GPU ------------------------------------------------------------------------
    @staticmethod
    def unique_id():
        buf = (ctypes.c_uint8 * SM_UNIQUE_ID_BYTES)()
        st = lib().sm_comm_unique_id(buf)
        if st != SM_OK:
            raise StereoMSTError(st, "sm_comm_unique_id failed")
        return bytes(buf)

    def comm_init(self, nranks, rank, uid):
        buf = (ctypes.c_uint8 * SM_UNIQUE_ID_BYTES).from_buffer_copy(uid)
        self._check(lib().sm_comm_init(self.h, nranks, rank, buf))

    def comm_destroy(self):
        self._check(lib().sm_comm_destroy(self.h))


# -- host-side MST_PMS helpers of the library (CPU; tests compare them with the oracle) -----------------
def pms_forest_bfs(W, H, wR, wD, mask):
    N = W * H
    ts = np.empty(N + 1, np.int32); pix = np.empty(N, np.int32); par = np.empty(N, np.int32)
    w = np.empty(N, np.uint16); nch = np.empty(N, np.uint8); ch = np.empty(4 * N, np.int32)
    k = lib().sm_pms_forest_bfs(W, H, ptr(np.ascontiguousarray(wR, np.uint16)), ptr(np.ascontiguousarray(wD, np.uint16)),
                                ptr(np.ascontiguousarray(mask, np.uint8)), ptr(ts), ptr(pix), ptr(par), ptr(w), ptr(nch),
                                ptr(ch))
    return dict(ntrees=k, tree_start=ts[:k + 1].copy(), node_pix=pix, node_parent=par, node_w=w, node_nch=nch,
                node_child=ch)



def pms_forest_digest(W, H, wR, wD, mask, piece, nthreads):
    """The MST_PMS schedule forest (sm_pms_host.cpp pms_build_forest) on `nthreads` host threads: digests
    of its arrays, tree_start and bfs_pix (test hook)."""
    N = W * H
    dig = np.zeros(6, np.uint64)
    ts = np.empty(N + 1, np.int32)
    pix = np.empty(N, np.int32)
    k = lib().sm_pms_forest_digest(W, H, ptr(np.ascontiguousarray(wR, np.uint16)), ptr(np.ascontiguousarray(wD, np.uint16)),
                                   ptr(np.ascontiguousarray(mask, np.uint8)), piece, nthreads, ptr(dig), ptr(ts), ptr(pix))
    return dict(ntrees=k, digest=dig, tree_start=ts[:k + 1].copy(), bfs_pix=pix)

def pms_tree_graph(W, H, wR, wD, mask):
    N = W * H
    s = np.empty(N + 1, np.int32); nb = np.empty(4 * N + 4, np.int32)
    n = lib().sm_pms_tree_graph(W, H, ptr(np.ascontiguousarray(mask, np.uint8)), ptr(np.ascontiguousarray(wR, np.uint16)),
                                ptr(np.ascontiguousarray(wD, np.uint16)), ptr(s), ptr(nb), nb.size)
    if n < 0:
        raise RuntimeError("sm_pms_tree_graph: capacity")
    return s, nb[:n].copy()


def pms_dice(n):
    out = np.empty(int(n), np.float32)
    lib().sm_pms_dice(int(n), ptr(out))
    return out


def pms_glibc_random(seed, skip, n):
    out = np.empty(int(n), np.int32)
    lib().sm_pms_glibc_random(int(seed), int(skip), int(n), ptr(out))
    return out


def pms_init_labels(W, H, max_disp):
    out = np.empty((W * H, 3), np.float32)
    lib().sm_pms_init_labels(W, H, int(max_disp), ptr(out))
    return out


def pms_levels(max_disp):
    return lib().sm_pms_levels(int(max_disp))


# -- the cross-rank WTA exchange rule (sm_reduce_rule.h), host form; the CPU tests' gloo exchange ---------
def reduce_candidates(minc, gmin, idx, disp=None, sub=False):
    """Per-pixel candidate of this rank after the MIN all-reduce of the minima: int32 index (or INT_MAX),
    or with sub the uint64 (index << 32 | disparity bits) (or ~0)."""
    minc = np.ascontiguousarray(minc, np.float64)
    gmin = np.ascontiguousarray(gmin, np.float64)
    idx = np.ascontiguousarray(idx, np.int32)
    N = minc.size
    cand = np.empty(N, np.uint64 if sub else np.int32)
    d = np.ascontiguousarray(disp, np.float32) if sub else None
    lib().sm_reduce_candidates(ptr(minc), ptr(gmin), ptr(idx), ptr(d), 1 if sub else 0, ptr(cand), N)
    return cand


def reduce_finalize(gmin, gcand, sub=False):
    """The global (minimum, index, disparity) from the reduced minima and candidates."""
    gmin = np.ascontiguousarray(gmin, np.float64)
    gcand = np.ascontiguousarray(gcand, np.uint64 if sub else np.int32)
    N = gmin.size
    minc = np.empty(N, np.float64)
    idx = np.empty(N, np.int32)
    disp = np.empty(N, np.float32)
    lib().sm_reduce_finalize(ptr(gmin), ptr(gcand), 1 if sub else 0, ptr(minc), ptr(idx), ptr(disp), N)
    return minc, idx, disp
