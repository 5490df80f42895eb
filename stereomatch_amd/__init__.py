"""stereomatch_amd -- MI355X-native Stereo3DMST cost-aggregation path.

Python mirror of the reference's entry surface (include/Stereo3DMST.h:7-11):

    stereo3dmst(left_name, right_name, left_img, right_img, data_cost, Dmax)
        -> (left_disp, right_disp)                 # src/Stereo3DMST.cpp:714
    startTimer() / getTimer()                      # src/Stereo3DMST.cpp:15-26

backed by the HIP library libstereomst.so (C-ABI in include/stereomst.h).  The compute
runs only on the GPU; a missing library or device raises.
"""
import ctypes
import os

import numpy as np

from ._lib import (SM_AGG_GUIDED, SM_AGG_PMS, SM_AGG_TREE, SM_COST_AGD, SM_COST_VOLUME, SM_POST_LABEL_TO_DISP, SM_POST_LR_CHECK, SM_POST_LR_FILL,  # noqa: F401
                   SM_POST_OCCLUSION, SM_POST_OCCLUSION_ZERO, SM_POST_SUBPIXEL, Context, StereoMSTError, default_params, device_count, lib,
                   knob_names, set_knob)

# stereo3dmst's output step: LabelToDisp + *= (Dmax-1) on both maps, then the fill-less L-R check of
# the left map (Stereo3DMST.cpp:189-201, 900-904)
STEREO3DMST_POST = SM_POST_LABEL_TO_DISP | SM_POST_LR_CHECK

__all__ = ["stereo3dmst", "startTimer", "getTimer", "Context", "default_params", "StereoMSTError", "device_count",
           "shard_range", "partition", "STEREO3DMST_POST", "SM_AGG_PMS"]


def shard_range(d_total, nranks, rank):
    """Contiguous ascending disparity shard of `rank`: (d0, D).  Ranks take
    [g*Dt/G, (g+1)*Dt/G) so the cross-rank (cost, global d) minimum reproduces the strict-<
    first minimum over ascending d (PatchMatchStereoGPU.cu:1712)."""
    if nranks < 1 or not 0 <= rank < nranks or d_total < nranks:
        raise ValueError("need 0 <= rank < nranks <= d_total")
    d0 = rank * d_total // nranks
    d1 = (rank + 1) * d_total // nranks
    return d0, d1 - d0


def partition(d_total, nranks, rank, split_views=True):
    """The share of one frame (both views, d_total disparities each) that `rank` of `nranks` owns
    (DESIGN.md 7).  With split_views, an even nranks and at most 128 slices per rank after the
    split, the ranks form two view groups -- ranks [0, N/2) the left view, [N/2, N) the right view
    -- and each group D-shards its view over its N/2 ranks: a rank builds one tree and filters
    d_total / (N/2) slices of one view, and the WTA reduce runs inside its group.  Otherwise every
    rank takes both views and d_total / N slices (measured at C4: one view of 256 slices is slower
    than both views of 128, so N = 2 keeps both views).
    Returns dict(views, d0, D, group, group_size, group_rank): views is the sm_params.views mask."""
    if split_views and nranks >= 2 and nranks % 2 == 0 and -(-d_total // (nranks // 2)) <= 128:
        half = nranks // 2
        group, grank = divmod(rank, half)
        d0, D = shard_range(d_total, half, grank)
        return dict(views=1 << group, d0=d0, D=D, group=group, group_size=half, group_rank=grank)
    d0, D = shard_range(d_total, nranks, rank)
    return dict(views=3, d0=d0, D=D, group=0, group_size=nranks, group_rank=rank)


_default_ctx = None
_timer = ctypes.c_double(0.0)


def _ctx():
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context(0)
    return _default_ctx


# stereo3dmst's own algorithm (Stereo3DMST.cpp:830-832, 854): the Felzenszwalb forest with c = 5000 and
# min_size = 200, random plane labels, 100 MST_PMS calls per view
PMS_C, PMS_MIN_SIZE, PMS_ITERS = 5000.0, 200, 100


def stereo3dmst(left_name, right_name, left_img, right_img, data_cost="AGD", Dmax=100, algorithm=None,
                iters=PMS_ITERS):
    """Reference-compatible entry (src/Stereo3DMST.cpp:714-912).

    left_img/right_img: HxWx3 uint8 BGR (cv::Mat CV_8UC3).  Returns (left_disp, right_disp), float32 HxW
    in [0, Dmax-1], after the reference's output step: both maps through LabelToDisp's
    clamp(d/(Dmax-1.f), 0, 1) and *= (Dmax-1.f) in float (:189-201, :900-902), then the left map
    left-right checked without fill (:904, :632-662); the right map is unchecked.

    algorithm "pms" (default; env SM_STEREO3DMST_ALGO overrides): the reference's own label search --
    segment forest (c=5000, min_size=200), random slanted-plane labels, `iters` MST_PMS calls per view
    (:546-629, :851-889), LabelToDisp of the plane labels.  "slices": this framework's per-slice
    restatement -- the MST tree filter of every disparity slice and a strict-< WTA.
    data_cost "AGD" builds the cost on the GPU; "MCCNN_fst"/"MCCNN_acrt" take the MC-CNN volumes
    from mc-cnn-master/{left,right}.bin (after running the network there, as the reference does).
    Like the reference, an unsupported data_cost prints a message and returns
    allocated-but-unset maps (:756-759); the names are only forwarded to the cost source.
    """
    algorithm = algorithm or os.environ.get("SM_STEREO3DMST_ALGO", "pms")
    if algorithm not in ("pms", "slices"):
        raise ValueError("algorithm must be 'pms' or 'slices'")
    H, W = left_img.shape[:2]
    left_disp = np.empty((H, W), np.float32)
    right_disp = np.empty((H, W), np.float32)
    p = default_params(post=STEREO3DMST_POST, disp_total=int(Dmax))
    if algorithm == "pms":
        p.aggregator = SM_AGG_PMS
        p.c = PMS_C
        p.min_size = PMS_MIN_SIZE
        p.pms_iters = int(iters)
    if data_cost in ("MCCNN_fst", "MCCNN_acrt"):
        # reference: without an mc-cnn-master folder MCCNN_fst prints and returns (:727-731),
        # MCCNN_acrt returns silently (:744-745); otherwise it runs the network (./main.lua, a
        # subprocess: :733-750) and maps mc-cnn-master/{left,right}.bin, [Dmax][rows][cols] float
        # (:764-775), whose clamp and filter run here on the GPU (SM_COST_VOLUME)
        if not os.path.isdir("mc-cnn-master"):
            if data_cost == "MCCNN_fst":
                print("no mc-cnn-master folder")
            return left_disp, right_disp
        vols = _mccnn_volumes(left_name, right_name, data_cost, H, W, int(Dmax))
        if vols is None:
            return left_disp, right_disp
        ctx = _ctx()
        ctx.upload_cost_volumes(*vols)
        p.cost_kind = SM_COST_VOLUME
        out = ctx.match(left_img, right_img, int(Dmax), p)
        left_disp[...] = out["left"]["disp"]
        right_disp[...] = out["right"]["disp"]
        return left_disp, right_disp
    if data_cost != "AGD":
        print("wrong data cost")
        return left_disp, right_disp
    out = _ctx().match(left_img, right_img, int(Dmax), p)
    left_disp[...] = out["left"]["disp"]
    right_disp[...] = out["right"]["disp"]
    return left_disp, right_disp


def _mccnn_volumes(left_name, right_name, data_cost, H, W, Dmax):
    """The reference's MC-CNN step (Stereo3DMST.cpp:725-775): run mc-cnn-master/main.lua when it
    is present (its failure is ignored, as system()'s exit status is), then read left.bin and
    right.bin.  Returns the two [Dmax][H][W] volumes, or None (message printed) without them."""
    import subprocess
    net = "fast" if data_cost == "MCCNN_fst" else "slow"
    if os.path.exists(os.path.join("mc-cnn-master", "main.lua")):
        cmd = ["./main.lua", "mb", net, "-a", "predict", "-net_fname", "net/net_mb_%s_-a_train_all.t7" % net,
               "-left", "../" + left_name, "-right", "../" + right_name, "-disp_max", str(Dmax), "-sm_terminate", "cnn"]
        try:
            subprocess.run(cmd, cwd="mc-cnn-master", check=False)
        except OSError:
            pass
    n = Dmax * H * W
    vols = []
    for side in ("left", "right"):
        path = os.path.join("mc-cnn-master", side + ".bin")
        if not os.path.exists(path) or os.path.getsize(path) < 4 * n:
            print("stereo3dmst: %s missing or shorter than %d x %d x %d floats" % (path, Dmax, H, W))
            return None
        vols.append(np.fromfile(path, dtype=np.float32, count=n).reshape(Dmax, H, W))
    return vols


def startTimer():
    lib().sm_start_timer(ctypes.byref(_timer))


def getTimer():
    return lib().sm_get_timer_ms(ctypes.byref(_timer))
