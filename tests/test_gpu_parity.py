"""GPU parity: the HIP path through the C-ABI against the oracle restatement and the
reference-derived golden fixtures.  Integer/index outputs and the fp64 aggregated costs
are compared BIT-EXACT (the kernels perform the shipped reference's exact operation
sequence); the north-star tolerance (1e-4 relative on aggregated costs) is
therefore met with zero slack."""

import numpy as np
import pytest

from conftest import flir_pair, golden_cases, load_case
from oracle import oracle as O
from tools.synth import make_pair

pytestmark = pytest.mark.gpu
CASES = golden_cases()
REL_TOL = 1e-4  # north_star: aggregated float costs within 1e-4 relative (we assert bitwise)


def bits(a):
    return np.ascontiguousarray(a).view(np.uint64)


@pytest.mark.parametrize("name", CASES)
def test_cost_volume_bitexact_golden(gpu_ctx, name):
    z = load_case(name)
    D = int(z["D"])
    lv, rv = gpu_ctx.cost_volume(z["left"], z["right"], 0, D)
    np.testing.assert_array_equal(lv, z["left_vol"])
    np.testing.assert_array_equal(rv, z["right_vol"])


@pytest.mark.parametrize("W,H,d0,D", [(300, 200, 0, 64), (257, 61, 37, 100), (64, 16, 0, 90)])
def test_cost_volume_bitexact_synthetic(gpu_ctx, W, H, d0, D):
    left, right, _ = make_pair(W, H, d0 + D, index=1)
    lv, rv = gpu_ctx.cost_volume(left, right, d0, D)
    olv, orv = O.cost_agd(left, right, d0, d0 + D)
    np.testing.assert_array_equal(lv, olv)
    np.testing.assert_array_equal(rv, orv)


@pytest.mark.parametrize("name", CASES)
def test_mst_matches_reference_segment_graph(gpu_ctx, name):
    z = load_case(name)
    H, W, _ = z["left"].shape
    for v in ("left", "right"):
        t = gpu_ctx.build_tree(z[v])
        np.testing.assert_array_equal(t["mask"], z[v + "_ref_mst_mask"])
        # rooted at pixel 0 exactly like the BFS of Stereo3DMST.cpp:450-522
        par = np.full(W * H, -1, np.int32)
        pix, parent = z[v + "_node_pix"], z[v + "_node_parent"]
        par[pix[1:]] = pix[parent[1:]]
        np.testing.assert_array_equal(t["parent_pix"], par)
        assert t["subtree_size"][0] == W * H


@pytest.mark.parametrize("iters", ["0", "1", "64"])
@pytest.mark.parametrize("pixel_rounds", [False, True])
def test_mst_phase_split_exact(gpu_ctx, knobs, iters, pixel_rounds):
    """Any tile-phase iteration cap (SM_MST_LOCAL_ITERS: 0 = pure global Boruvka, 64 = tile
    phase to completion) and either global-round engine (contracted component graph, or the
    pixel rounds kept as the SM_MST_PIXEL_ROUNDS A/B path) gives the reference's MST."""
    knobs.setenv("SM_MST_LOCAL_ITERS", iters)
    if pixel_rounds:
        knobs.setenv("SM_MST_PIXEL_ROUNDS", "1")
    else:
        knobs.delenv("SM_MST_PIXEL_ROUNDS", raising=False)
    z = load_case(CASES[-1])
    for v in ("left", "right"):
        t = gpu_ctx.build_tree(z[v])
        np.testing.assert_array_equal(t["mask"], z[v + "_ref_mst_mask"])


@pytest.mark.parametrize("name", CASES)
def test_aggregate_bitexact_golden(gpu_ctx, name):
    z = load_case(name)
    D = int(z["D"])
    if "left_Aup" not in z:
        pytest.skip("no stored volumes (large case): covered by test_match_bitexact_golden")
    for vi, v in enumerate(("left", "right")):
        Aup, A = gpu_ctx.aggregate_debug(z["left"], z["right"], vi, 0, D)
        assert np.array_equal(bits(Aup), bits(z[v + "_Aup"]))
        assert np.array_equal(bits(A), bits(z[v + "_A"]))


@pytest.mark.parametrize("name", CASES)
def test_match_bitexact_golden(gpu_ctx, name):
    z = load_case(name)
    D = int(z["D"])
    out = gpu_ctx.match(z["left"], z["right"], D)
    for v in ("left", "right"):
        np.testing.assert_array_equal(out[v]["idx"].ravel(), z[v + "_idx"])
        assert np.array_equal(bits(out[v]["minc"].ravel()), bits(z[v + "_minc"]))
        np.testing.assert_array_equal(out[v]["disp"].ravel(), z[v + "_idx"].astype(np.float32))


@pytest.mark.parametrize("W,H,D", [(320, 240, 64), (200, 150, 128), (160, 90, 256), (97, 61, 33), (333, 7, 200)])
def test_match_bitexact_synthetic(gpu_ctx, W, H, D):
    left, right, _ = make_pair(W, H, D, index=2)
    out = gpu_ctx.match(left, right, D)
    ref = O.match(left, right, D, nthreads=16)
    for v in ("left", "right"):
        np.testing.assert_array_equal(out[v]["idx"].ravel(), ref[v]["idx"])
        assert np.array_equal(bits(out[v]["minc"].ravel()), bits(ref[v]["minc"]))


@pytest.mark.parametrize("plen,rmax", [("64", None), ("96", None), ("64", "1"), ("128", "2")])
@pytest.mark.parametrize("W,H,D", [(320, 240, 64), (256, 160, 128), (200, 120, 200)])
def test_pieces_match_bitexact(gpu_ctx, knobs, plen, rmax, W, H, D):
    """Long heavy paths cut into pieces of SM_PIECE_LEN nodes that run from guessed inputs and are
    repaired exactly (sm_chain.hip "Pieces"); SM_REPAIR_MAX=1/2 makes most repairs give up, which
    sends those pieces through the serial slow path.  SPL = 1, 2, 4."""
    knobs.setenv("SM_PIECE_LEN", plen)
    if rmax:
        knobs.setenv("SM_REPAIR_MAX", rmax)
    else:
        knobs.delenv("SM_REPAIR_MAX", raising=False)
    left, right, _ = make_pair(W, H, D, index=4)
    out = gpu_ctx.match(left, right, D)
    ref = O.match(left, right, D, nthreads=16)
    for v in ("left", "right"):
        np.testing.assert_array_equal(out[v]["idx"].ravel(), ref[v]["idx"])
        assert np.array_equal(bits(out[v]["minc"].ravel()), bits(ref[v]["minc"]))


@pytest.mark.parametrize("plen,rmax", [("64", None), ("64", "1")])
def test_pieces_rows_bitexact(gpu_ctx, knobs, plen, rmax):
    """Every fp64 A_up / A value of 4 slices with short pieces, bitwise."""
    knobs.setenv("SM_PIECE_LEN", plen)
    if rmax:
        knobs.setenv("SM_REPAIR_MAX", rmax)
    else:
        knobs.delenv("SM_REPAIR_MAX", raising=False)
    W, H, d0, D = 400, 300, 20, 4
    left, right, _ = make_pair(W, H, 64, index=5)
    lv, rv = O.cost_agd(left, right, d0, d0 + D)
    for vi, (img, vol) in enumerate(((left, lv), (right, rv))):
        Aup, A = gpu_ctx.aggregate_debug(left, right, vi, d0, D)
        t = O.build_tree(img)
        r = O.tree_filter(W, H, t, vol, d0, False, True, 16)
        assert np.array_equal(bits(Aup), bits(r["Aup"]))
        assert np.array_equal(bits(A), bits(r["A"]))


@pytest.mark.parametrize("plen", ["64", "512"])
@pytest.mark.parametrize("D", [32, 64, 100, 200])
def test_chain_helper_costs_bitexact(gpu_ctx, knobs, plen, D):
    """The up chain's helpers fold the pre-heavy children and compute the AGD cost rows from the
    image records themselves (SPL 1, 2, 4; 32-double rows at D=32): bit-exact against the oracle,
    cut paths (k_up_pre's aggregates and the repair walks compute costs too) included."""
    knobs.setenv("SM_PIECE_LEN", plen)
    W, H = 400, 300
    left, right, _ = make_pair(W, H, D, index=6)
    ref = O.match(left, right, D, nthreads=16)
    out = gpu_ctx.match(left, right, D)
    for v in ("left", "right"):
        np.testing.assert_array_equal(out[v]["idx"].ravel(), ref[v]["idx"])
        assert np.array_equal(bits(out[v]["minc"].ravel()), bits(ref[v]["minc"]))


@pytest.mark.parametrize("D", [32, 64, 128, 256])
def test_leaf_f32_rows_bitexact(gpu_ctx, knobs, D):
    """Heavy leaves keep an f32 cost row in their U slot (WalkArgs::leaf_cost): the walkers' results
    with it equal the full-row path (SM_NO_LEAF_COST=1) and the oracle bitwise (SPL 1, 2, 4; 32-double
    rows at D=32; segment forest too)."""
    import stereomatch_amd as sm
    W, H = 320, 240
    left, right, _ = make_pair(W, H, D, index=7)
    for params, ref in ((None, O.match(left, right, D, nthreads=16)),
                        (sm.default_params(c=5000.0, min_size=200), O.match(left, right, D, c=5000.0, nthreads=16))):
        out = gpu_ctx.match(left, right, D, params)
        knobs.setenv("SM_NO_LEAF_COST", "1")
        full = gpu_ctx.match(left, right, D, params)
        knobs.delenv("SM_NO_LEAF_COST")
        for v in ("left", "right"):
            np.testing.assert_array_equal(out[v]["idx"], full[v]["idx"])
            assert np.array_equal(bits(out[v]["minc"]), bits(full[v]["minc"]))
            np.testing.assert_array_equal(out[v]["idx"].ravel(), ref[v]["idx"])
            assert np.array_equal(bits(out[v]["minc"].ravel()), bits(ref[v]["minc"]))


def test_kernel_timing_mask(gpu_ctx):
    """sm_set_kernel_timing: untimed families report no launches, timed ones do; the results do
    not depend on the timing."""
    W, H, D = 160, 120, 32
    left, right, _ = make_pair(W, H, D, index=2)
    base = gpu_ctx.match(left, right, D)
    gpu_ctx.set_kernel_timing(["k_up_walk"])
    try:
        out = gpu_ctx.match(left, right, D)
        ks = gpu_ctx.kernel_stats()
    finally:
        gpu_ctx.set_kernel_timing(None)
    assert ks["k_up_walk"]["launches"] > 0 and ks["k_up_walk"]["ms"] > 0
    assert all(v["launches"] == 0 for k, v in ks.items() if k != "k_up_walk")
    for v in ("left", "right"):
        np.testing.assert_array_equal(out[v]["idx"], base[v]["idx"])
    ks = None
    gpu_ctx.match(left, right, D)
    assert sum(v["launches"] for v in gpu_ctx.kernel_stats().values()) > 0


def test_match_shard_offset_bitexact(gpu_ctx):
    """A disparity shard [d0, d0+D) (what one rank computes under D sharding)."""
    import stereomatch_amd as sm
    W, H, d0, D = 240, 160, 24, 40
    left, right, _ = make_pair(W, H, d0 + D, index=3)
    out = gpu_ctx.match(left, right, D, sm.default_params(disp_begin=d0))
    lv, rv = O.cost_agd(left, right, d0, d0 + D)
    for v, vol in (("left", lv), ("right", rv)):
        t = O.build_tree(left if v == "left" else right)
        r = O.tree_filter(W, H, t, vol, d0, True, False, 16)
        np.testing.assert_array_equal(out[v]["idx"].ravel(), r["idx"])
        assert np.array_equal(bits(out[v]["minc"].ravel()), bits(r["minc"]))


def test_full_size_c2_slices_bitexact(gpu_ctx):
    """1920x1200 (BASELINE config 1): every fp64 A_up/A value of 4 slices, bitwise."""
    W, H, d0, D = 1920, 1200, 60, 4
    left, right, _ = make_pair(W, H, 128, index=0)
    lv, rv = O.cost_agd(left, right, d0, d0 + D)
    for vi, (img, vol) in enumerate(((left, lv), (right, rv))):
        Aup, A = gpu_ctx.aggregate_debug(left, right, vi, d0, D)
        t = O.build_tree(img)
        r = O.tree_filter(W, H, t, vol, d0, False, True, 16)
        assert np.array_equal(bits(Aup), bits(r["Aup"]))
        assert np.array_equal(bits(A), bits(r["A"]))


def test_full_size_c4_match_bitexact(gpu_ctx):
    """1920x1200 D=256 (BASELINE config C4 unsharded; SPL=4, cut root paths), bitwise."""
    W, H, D = 1920, 1200, 256
    left, right, _ = make_pair(W, H, D, index=11)
    out = gpu_ctx.match(left, right, D)
    ref = O.match(left, right, D, nthreads=16)
    for v in ("left", "right"):
        np.testing.assert_array_equal(out[v]["idx"].ravel(), ref[v]["idx"])
        assert np.array_equal(bits(out[v]["minc"].ravel()), bits(ref[v]["minc"]))


def test_full_size_c2_match_bitexact(gpu_ctx):
    """1920x1200 D=128 (the headline config): WTA indices and fp64 minima, bitwise."""
    W, H, D = 1920, 1200, 128
    left, right, _ = make_pair(W, H, D, index=0)
    out = gpu_ctx.match(left, right, D)
    ref = O.match(left, right, D, nthreads=16)
    for v in ("left", "right"):
        np.testing.assert_array_equal(out[v]["idx"].ravel(), ref[v]["idx"])
        assert np.array_equal(bits(out[v]["minc"].ravel()), bits(ref[v]["minc"]))
    # determinism: a second run is bit-identical
    out2 = gpu_ctx.match(left, right, D)
    for v in ("left", "right"):
        assert np.array_equal(bits(out2[v]["minc"]), bits(out[v]["minc"]))


def test_full_size_c3_match_bitexact(gpu_ctx):
    """3840x2160 D=256 (BASELINE config C3: SPL=4, ~30k-node cut root paths, 4K MST and layout):
    full WTA indices and fp64 minima of both views, bitwise against the oracle."""
    W, H, D = 3840, 2160, 256
    left, right, _ = make_pair(W, H, D, index=12)
    out = gpu_ctx.match(left, right, D)
    ref = O.match(left, right, D, nthreads=16)
    for v in ("left", "right"):
        np.testing.assert_array_equal(out[v]["idx"].ravel(), ref[v]["idx"])
        assert np.array_equal(bits(out[v]["minc"].ravel()), bits(ref[v]["minc"]))


def test_full_size_c3_slices_bitexact(gpu_ctx):
    """C3 size: every fp64 A_up / A value of 4 slices (SPL=1 rows over the C3 tree), bitwise."""
    W, H, d0, D = 3840, 2160, 150, 4
    left, right, _ = make_pair(W, H, 256, index=12)
    lv, rv = O.cost_agd(left, right, d0, d0 + D)
    for vi, (img, vol) in enumerate(((left, lv), (right, rv))):
        Aup, A = gpu_ctx.aggregate_debug(left, right, vi, d0, D)
        r = O.tree_filter(W, H, O.build_tree(img), vol, d0, False, True, 16)
        assert np.array_equal(bits(Aup), bits(r["Aup"]))
        assert np.array_equal(bits(A), bits(r["A"]))


@pytest.mark.parametrize("rank", [0, 3, 7])
def test_full_size_c4_shard_with_reduce_bitexact(rank):
    """BASELINE C4 as sharded: one 32-slice shard of 1920x1200 D=256 (rank r of 8 owns
    [32r, 32r+32)), at full size, through a one-rank RCCL communicator so that the cross-rank
    exchange (grouped all-reduce MIN of the fp64 minima, k_cand, all-reduce MIN of the candidate
    index, k_finalize; sm_api.cpp stage_reduce) runs on the GPU.  With one rank the exchange must
    return the shard's own strict-< minimum, so the result equals the oracle's tree filter over the
    shard's slices, bitwise; the output step then scales with the TOTAL range (Dmax = 256)."""
    import stereomatch_amd as sm
    W, H, Dt = 1920, 1200, 256
    d0, D = sm.shard_range(Dt, 8, rank)
    left, right, _ = make_pair(W, H, Dt, index=13)
    ctx = sm.Context(0)
    try:
        ctx.comm_init(1, 0, sm.Context.unique_id())
        out = ctx.match(left, right, D, sm.default_params(disp_begin=d0, disp_total=Dt))
        outp = ctx.match(left, right, D, sm.default_params(disp_begin=d0, disp_total=Dt, post=sm.STEREO3DMST_POST))
        assert ctx.stage_times()["reduce_ms"] > 0
    finally:
        ctx.close()
    lv, rv = O.cost_agd(left, right, d0, d0 + D)
    ref = {}
    for v, img, vol in (("left", left, lv), ("right", right, rv)):
        r = O.tree_filter(W, H, O.build_tree(img), vol, d0, True, False, 16)
        ref[v] = r["idx"].reshape(H, W)
        np.testing.assert_array_equal(out[v]["idx"], ref[v])
        assert np.array_equal(bits(out[v]["minc"].ravel()), bits(r["minc"]))
        np.testing.assert_array_equal(out[v]["disp"], ref[v].astype(np.float32))
    lref, rref = O.stereo3dmst_output(ref["left"], ref["right"], Dt)
    np.testing.assert_array_equal(outp["left"]["disp"], lref)
    np.testing.assert_array_equal(outp["right"]["disp"], rref)


@pytest.mark.parametrize("c", [float("inf"), 5000.0])
@pytest.mark.parametrize("W,H,D,plen", [(320, 240, 64, "64"), (256, 160, 128, None), (160, 90, 200, "64"), (200, 150, 32, None)])
def test_one_view_calls_bitexact(gpu_ctx, knobs, W, H, D, plen, c):
    """sm_params.views = 1 / 2: a call builds and filters only that view (the multi-GPU view
    groups); bit-exact against the oracle, MST and segment forest, cut paths too."""
    import stereomatch_amd as sm
    if plen:
        knobs.setenv("SM_PIECE_LEN", plen)
    else:
        knobs.delenv("SM_PIECE_LEN", raising=False)
    left, right, _ = make_pair(W, H, D, index=9)
    ref = O.match(left, right, D, nthreads=16, c=c)
    for views, v in ((1, "left"), (2, "right")):
        out = gpu_ctx.match(left, right, D, sm.default_params(views=views, c=c))
        assert list(out) == [v]
        np.testing.assert_array_equal(out[v]["idx"].ravel(), ref[v]["idx"])
        assert np.array_equal(bits(out[v]["minc"].ravel()), bits(ref[v]["minc"]))


@pytest.mark.parametrize("n,rank", [(8, 0), (8, 6), (4, 1), (4, 2)])
def test_full_size_c4_view_group_shard_with_reduce(n, rank):
    """BASELINE C4 frame under the view-group partition (stereomatch_amd.partition, bench.py
    --shard vd): rank r of n filters 256 / (n/2) slices of ONE view at full size and reduces
    through a one-rank RCCL communicator (stage_reduce over its view only); bitwise equal to the
    oracle's tree filter over that view's shard.  n = 4 is also the share of a rank at N = 8 with 2
    frame groups (bench.py --frame-groups, the N = 8 default)."""
    import stereomatch_amd as sm
    W, H, Dt = 1920, 1200, 256
    part = sm.partition(Dt, n, rank)
    d0, D, views = part["d0"], part["D"], part["views"]
    v = "left" if views == 1 else "right"
    left, right, _ = make_pair(W, H, Dt, index=13)
    ctx = sm.Context(0)
    try:
        ctx.comm_init(1, 0, sm.Context.unique_id())
        out = ctx.match(left, right, D, sm.default_params(disp_begin=d0, disp_total=Dt, views=views))
        assert ctx.stage_times()["reduce_ms"] > 0
    finally:
        ctx.close()
    lv, rv = O.cost_agd(left, right, d0, d0 + D)
    r = O.tree_filter(W, H, O.build_tree(left if v == "left" else right), lv if v == "left" else rv, d0, True, False, 16)
    assert list(out) == [v]
    np.testing.assert_array_equal(out[v]["idx"].ravel(), r["idx"])
    assert np.array_equal(bits(out[v]["minc"].ravel()), bits(r["minc"]))


def test_one_view_rejects_two_map_post(gpu_ctx):
    import stereomatch_amd as sm
    left, right, _ = make_pair(64, 48, 16, index=2)
    for post in (sm.STEREO3DMST_POST, 8):
        with pytest.raises(sm.StereoMSTError):
            gpu_ctx.match(left, right, 16, sm.default_params(views=1, post=post))
    with pytest.raises(sm.StereoMSTError):
        gpu_ctx.match(left, right, 16, sm.default_params(views=4))


def test_chain_wait_timeout_is_an_error(knobs):
    """A cross-workgroup wait of the chain engine that never sees its status word must not return
    SM_OK: SM_WAIT_ITERS=0 makes every such wait give up at once, which sets the call's device error
    word; sm_synchronize reports SM_ERR_STATE.  The next call (normal waits) is exact again."""
    import stereomatch_amd as sm
    knobs.setenv("SM_PIECE_LEN", "64")  # cut paths: pieces wait for their neighbours
    W, H, D = 320, 240, 64
    left, right, _ = make_pair(W, H, D, index=4)
    ctx = sm.Context(0)
    try:
        knobs.setenv("SM_WAIT_ITERS", "0")
        with pytest.raises(sm.StereoMSTError, match="SM_ERR_STATE.*timed out"):
            ctx.match(left, right, D)
        knobs.delenv("SM_WAIT_ITERS")
        out = ctx.match(left, right, D)
    finally:
        ctx.close()
    ref = O.match(left, right, D, nthreads=16)
    for v in ("left", "right"):
        np.testing.assert_array_equal(out[v]["idx"].ravel(), ref[v]["idx"])
        assert np.array_equal(bits(out[v]["minc"].ravel()), bits(ref[v]["minc"]))


def test_large_disp_begin_pads(gpu_ctx):
    """A shard far into the disparity range (disp_begin + 64*SPL > the default 1024-record image
    pad): the record pad grows with the call's range, results stay exact."""
    import stereomatch_amd as sm
    W, H, d0, D = 1400, 40, 1100, 24
    left, right, _ = make_pair(W, H, 64, index=3)
    out = gpu_ctx.match(left, right, D, sm.default_params(disp_begin=d0))
    lv, rv = O.cost_agd(left, right, d0, d0 + D)
    for v, vol in (("left", lv), ("right", rv)):
        r = O.tree_filter(W, H, O.build_tree(left if v == "left" else right), vol, d0, True, False, 16)
        np.testing.assert_array_equal(out[v]["idx"].ravel(), r["idx"])
        assert np.array_equal(bits(out[v]["minc"].ravel()), bits(r["minc"]))


def test_flir_c1_bitexact(gpu_ctx):
    """BASELINE config 0: the FLIR 000020 pair, 2048x1536, D=64."""
    L, R = flir_pair()
    D = 64
    out = gpu_ctx.match(L, R, D)
    ref = O.match(L, R, D, nthreads=16)
    for v in ("left", "right"):
        np.testing.assert_array_equal(out[v]["idx"].ravel(), ref[v]["idx"])
        assert np.array_equal(bits(out[v]["minc"].ravel()), bits(ref[v]["minc"]))


def test_errors_are_loud(gpu_ctx):
    import stereomatch_amd as sm
    left, right, _ = make_pair(32, 16, 8)
    with pytest.raises(sm.StereoMSTError):
        gpu_ctx.match(left, right, 0)
    with pytest.raises(sm.StereoMSTError):  # negative / NaN segment threshold
        gpu_ctx.match(left, right, 8, sm.default_params(c=-1.0))
    with pytest.raises(sm.StereoMSTError):
        gpu_ctx.match(left, right, 8, sm.default_params(c=float("nan")))
    with pytest.raises(sm.StereoMSTError):  # shard beyond the declared total range
        gpu_ctx.match(left, right, 8, sm.default_params(disp_begin=4, disp_total=8))
    with pytest.raises(sm.StereoMSTError):  # fill without the check
        gpu_ctx.match(left, right, 8, sm.default_params(post=sm.SM_POST_LR_FILL))
    with pytest.raises(sm.StereoMSTError):
        gpu_ctx.match(left, right, 8, sm.default_params(post=sm.SM_POST_OCCLUSION | sm.SM_POST_OCCLUSION_ZERO))


@pytest.mark.parametrize("Dmax", [16, 48, 100, 128])
def test_reference_surface(gpu_ctx, Dmax):
    """stereo3dmst's output contract: LabelToDisp + *= (Dmax-1.f) in float on both maps, then the
    fill-less L-R check of the left map (Stereo3DMST.cpp:189-201, 900-904).  At Dmax = 48 / 100 the
    float round trip moves some integer disparities by an ulp, which the check then sees."""
    import stereomatch_amd as sm
    left, right, _ = make_pair(160, 96, Dmax, index=4)
    sm.startTimer()
    ld, rd = sm.stereo3dmst("l.png", "r.png", left, right, "AGD", Dmax, algorithm="slices")
    assert sm.getTimer() >= 0
    ref = O.match(left, right, Dmax, nthreads=16)
    H, W = left.shape[:2]
    lref, rref = O.stereo3dmst_output(ref["left"]["idx"].reshape(H, W), ref["right"]["idx"].reshape(H, W), Dmax)
    np.testing.assert_array_equal(ld, lref)
    np.testing.assert_array_equal(rd, rref)


@pytest.mark.parametrize("W,H,D", [(200, 120, 48), (301, 47, 100), (256, 128, 128)])
@pytest.mark.parametrize("fill", [False, True])
def test_output_step_bitexact(gpu_ctx, W, H, D, fill):
    """SM_POST_LABEL_TO_DISP | SM_POST_LR_CHECK [| SM_POST_LR_FILL] against the oracle's literal
    restatement of :189-201, :632-709, :900-904; idx stays the integral WTA index."""
    import stereomatch_amd as sm
    post = sm.SM_POST_LABEL_TO_DISP | sm.SM_POST_LR_CHECK | (sm.SM_POST_LR_FILL if fill else 0)
    left, right, _ = make_pair(W, H, D, index=5)
    out = gpu_ctx.match(left, right, D, sm.default_params(post=post, disp_total=D))
    ref = O.match(left, right, D, nthreads=16)
    li, ri = ref["left"]["idx"].reshape(H, W), ref["right"]["idx"].reshape(H, W)
    lref, rref = O.stereo3dmst_output(li, ri, D, fill)
    np.testing.assert_array_equal(out["left"]["disp"], lref)
    np.testing.assert_array_equal(out["right"]["disp"], rref)
    np.testing.assert_array_equal(out["left"]["idx"], li)


@pytest.mark.parametrize("remove", [False, True])
@pytest.mark.parametrize("W,H,D", [(200, 120, 48), (1500, 16, 64)])
def test_occlusion_post_bitexact(gpu_ctx, W, H, D, remove):
    """SM_POST_OCCLUSION[_ZERO] = handleOcclusionSharedMemory (PatchMatchStereoGPU.cu:1128-1288) on the
    WTA maps, against the oracle (rows wider than the reference's 1024-thread limit included)."""
    import stereomatch_amd as sm
    post = sm.SM_POST_OCCLUSION_ZERO if remove else sm.SM_POST_OCCLUSION
    left, right, _ = make_pair(W, H, D, index=6)
    out = gpu_ctx.match(left, right, D, sm.default_params(post=post))
    ref = O.match(left, right, D, nthreads=16)
    Lr, Rr = O.occlusion(ref["left"]["idx"].reshape(H, W).astype(np.float32),
                         ref["right"]["idx"].reshape(H, W).astype(np.float32), 0, 1.0, remove)
    np.testing.assert_array_equal(out["left"]["disp"], Lr)
    np.testing.assert_array_equal(out["right"]["disp"], Rr)


@pytest.mark.parametrize("W,H,D", [(128, 80, 32), (301, 47, 100), (64, 9, 200)])
def test_lr_check_post_bitexact(gpu_ctx, W, H, D):
    import stereomatch_amd as sm
    left, right, _ = make_pair(W, H, D, index=5)
    out = gpu_ctx.match(left, right, D, sm.default_params(post=sm.SM_POST_LR_CHECK))
    ref = O.match(left, right, D, nthreads=16)
    lref = ref["left"]["idx"].astype(np.float32).reshape(H, W)
    rref = ref["right"]["idx"].astype(np.float32).reshape(H, W)
    np.testing.assert_array_equal(out["left"]["disp"], O.lr_check(lref, rref, D))
    np.testing.assert_array_equal(out["right"]["disp"], rref)
    np.testing.assert_array_equal(out["left"]["idx"].reshape(H, W), lref.astype(np.int32))  # idx untouched


def expected_layout(W, H, node_pix, node_parent):
    """Subtree sizes and heavy-first preorder (ties: smallest direction R,D,L,U) from the
    oracle's BFS tree -- the schedule layout the GPU builds (DESIGN.md "Tree layout")."""
    N = W * H
    parent = np.full(N, -1, np.int64)
    parent[node_pix[1:]] = node_pix[node_parent[1:]]
    size = np.ones(N, np.int64)
    for n in range(N - 1, 0, -1):
        size[node_pix[node_parent[n]]] += size[node_pix[n]]
    children = [[] for _ in range(N)]
    for q in range(N):
        p = parent[q]
        if p >= 0:
            d = q - p
            k = 0 if d == 1 else 1 if d == W else 2 if d == -1 else 3
            children[p].append((k, q))
    pre = np.zeros(N, np.int64)
    stack, cnt = [0], 0
    while stack:
        v = stack.pop()
        pre[v] = cnt
        cnt += 1
        ch = sorted(children[v])
        heavy = None
        for k, q in ch:
            if heavy is None or size[q] > size[heavy]:
                heavy = q
        lights = [q for k, q in ch if q != heavy]
        for q in reversed(lights):
            stack.append(q)
        if heavy is not None:
            stack.append(heavy)
    return size, pre


def expected_paths(W, H, node_pix, node_parent):
    """Heavy child (largest subtree, ties: smallest direction R,D,L,U), light depth and heavy
    paths restated from the oracle's BFS tree."""
    N = W * H
    parent = np.full(N, -1, np.int64)
    parent[node_pix[1:]] = node_pix[node_parent[1:]]
    size = np.ones(N, np.int64)
    for n in range(N - 1, 0, -1):
        size[node_pix[node_parent[n]]] += size[node_pix[n]]
    heavy = np.full(N, -1, np.int64)
    best = np.zeros(N, np.int64)
    for q in range(N):
        p = parent[q]
        if p < 0:
            continue
        d = q - p
        k = 0 if d == 1 else 1 if d == W else 2 if d == -1 else 3
        key = size[q] * 4 + (3 - k)  # larger subtree wins, then the smaller direction
        if key > best[p]:
            best[p], heavy[p] = key, q
    ld = np.zeros(N, np.int64)
    for n in range(1, N):  # BFS order: parents first
        q = node_pix[n]
        p = parent[q]
        ld[q] = ld[p] + (0 if heavy[p] == q else 1)
    heads = [q for q in range(N) if parent[q] < 0 or heavy[parent[q]] != q]
    paths = []
    for h in heads:
        nodes = [h]
        while heavy[nodes[-1]] >= 0:
            nodes.append(heavy[nodes[-1]])
        paths.append((h, nodes))
    return size, ld, paths


@pytest.mark.parametrize("name", ["rand_37x23", "smooth_97x61", "flir_crop_256x192", "const_16x12", "col_1x15"])
def test_gpu_layout_matches_restated_schedule(gpu_ctx, name):
    """The GPU schedule layout: subtree sizes; every heavy path on consecutive
    slots from its head; the paths of one (light depth, long/short) bucket on one contiguous
    slot range, buckets in increasing order (order of paths inside a bucket is free)."""
    z = load_case(name)
    H, W, _ = z["left"].shape
    t = gpu_ctx.build_tree(z["left"])
    size, ld, paths = expected_paths(W, H, z["left_node_pix"], z["left_node_parent"])
    np.testing.assert_array_equal(t["subtree_size"], size)
    slot = t["slot_of_pix"].astype(np.int64)
    assert np.array_equal(np.sort(slot), np.arange(W * H))
    spans = []
    for h, nodes in paths:
        np.testing.assert_array_equal(slot[nodes], slot[h] + np.arange(len(nodes)))
        bucket = 2 * ld[h] + (0 if len(nodes) >= 32 else 1)
        spans.append((slot[h], len(nodes), bucket))
    spans.sort()
    buckets = [b for _, _, b in spans]
    assert buckets == sorted(buckets)


# ---- MC-CNN volume ingest (SM_COST_VOLUME; Stereo3DMST.cpp:764-803) ----
def _mccnn_like(Dv, H, W, seed):
    """Raw volumes like MC-CNN's accurate output (0..1) with NaNs and values above the 0.5 clamp."""
    rng = np.random.default_rng(seed)
    v = rng.random((Dv, H, W), dtype=np.float32)
    v[rng.random(v.shape) < 0.01] = np.nan
    v[rng.random(v.shape) < 0.01] = np.float32(0.5)
    return v


@pytest.mark.parametrize("W,H,D,Dv,d0", [(200, 150, 64, 64, 0), (160, 120, 100, 128, 20), (97, 61, 33, 40, 5),
                                         (256, 160, 128, 128, 0), (120, 80, 200, 256, 56)])
def test_volume_ingest_bitexact(gpu_ctx, W, H, D, Dv, d0):
    """Costs from caller volumes: the GPU's clamp + tree filter + WTA equal the oracle's tree filter
    over the reference clamp of the same slices, bitwise (SPL 1, 2, 4; shard offsets)."""
    import stereomatch_amd as sm
    left, right, _ = make_pair(W, H, 64, index=8)
    lv, rv = _mccnn_like(Dv, H, W, 1), _mccnn_like(Dv, H, W, 2)
    gpu_ctx.upload_cost_volumes(lv, rv)
    out = gpu_ctx.match(left, right, D, sm.default_params(cost_kind=sm.SM_COST_VOLUME, disp_begin=d0))
    for v, img, vol in (("left", left, lv), ("right", right, rv)):
        t = O.build_tree(img)
        r = O.tree_filter(W, H, t, O.mccnn_clamp(vol[d0:d0 + D]), d0, True, False, 16)
        np.testing.assert_array_equal(out[v]["idx"].ravel(), r["idx"])
        assert np.array_equal(bits(out[v]["minc"].ravel()), bits(r["minc"]))


def test_volume_ingest_pieces_bitexact(gpu_ctx, knobs):
    """Volume costs through cut paths (64-node pieces) and runs."""
    import stereomatch_amd as sm
    knobs.setenv("SM_PIECE_LEN", "64")
    W, H, D = 320, 240, 64
    left, right, _ = make_pair(W, H, D, index=9)
    lv, rv = _mccnn_like(D, H, W, 3), _mccnn_like(D, H, W, 4)
    gpu_ctx.upload_cost_volumes(lv, rv)
    out = gpu_ctx.match(left, right, D, sm.default_params(cost_kind=sm.SM_COST_VOLUME))
    for v, img, vol in (("left", left, lv), ("right", right, rv)):
        r = O.tree_filter(W, H, O.build_tree(img), O.mccnn_clamp(vol), 0, True, False, 16)
        np.testing.assert_array_equal(out[v]["idx"].ravel(), r["idx"])
        assert np.array_equal(bits(out[v]["minc"].ravel()), bits(r["minc"]))


def test_volume_ingest_errors():
    import stereomatch_amd as sm
    ctx = sm.Context(0)
    left, right, _ = make_pair(40, 30, 8, index=1)
    p = sm.default_params(cost_kind=sm.SM_COST_VOLUME)
    with pytest.raises(sm.StereoMSTError, match="SM_ERR_STATE"):  # nothing uploaded
        ctx.match(left, right, 8, p)
    ctx.upload_cost_volumes(np.zeros((8, 30, 40), np.float32), np.zeros((8, 30, 40), np.float32))
    with pytest.raises(sm.StereoMSTError, match="SM_ERR_ARG"):  # beyond the uploaded slices
        ctx.match(left, right, 8, sm.default_params(cost_kind=sm.SM_COST_VOLUME, disp_begin=1))
    l2, r2, _ = make_pair(41, 30, 8, index=1)
    with pytest.raises(sm.StereoMSTError, match="SM_ERR_ARG"):  # size mismatch
        ctx.match(l2, r2, 8, p)
    ctx.close()


def test_stereo3dmst_mccnn_ingest(gpu_ctx, tmp_path, monkeypatch):
    """The reference surface with data_cost="MCCNN_acrt": volumes read from
    mc-cnn-master/{left,right}.bin ([Dmax][rows][cols] float, Stereo3DMST.cpp:769-775; no network
    present, so the main.lua step is skipped), clamped and filtered on the GPU, then the output
    step (left map L-R checked without fill, :900-904)."""
    import stereomatch_amd as sm
    W, H, D = 120, 90, 48
    left, right, _ = make_pair(W, H, D, index=10)
    lv, rv = _mccnn_like(D, H, W, 5), _mccnn_like(D, H, W, 6)
    (tmp_path / "mc-cnn-master").mkdir()
    lv.tofile(str(tmp_path / "mc-cnn-master" / "left.bin"))
    rv.tofile(str(tmp_path / "mc-cnn-master" / "right.bin"))
    monkeypatch.chdir(tmp_path)
    ld, rd = sm.stereo3dmst("l.png", "r.png", left, right, "MCCNN_acrt", D, algorithm="slices")
    ref = {}
    for v, img, vol in (("left", left, lv), ("right", right, rv)):
        ref[v] = O.tree_filter(W, H, O.build_tree(img), O.mccnn_clamp(vol), 0, True, False, 16)["idx"]
    lref, rref = O.stereo3dmst_output(ref["left"].reshape(H, W), ref["right"].reshape(H, W), D)
    np.testing.assert_array_equal(rd, rref)
    np.testing.assert_array_equal(ld, lref)


# ---- segment mode: the Felzenszwalb forest (c, min_size) filtered per tree (SURVEY.md 8f rank 1;
# segment-graph.h:54-89, Stereo3DMST.cpp:242-384, 120-158 per tree) ----
SEG = [(5000.0, 200), (300.0, 20), (0.0, 2)]


def _forest_parent(W, H, t):
    """parent pixel per pixel from the oracle's per-tree BFS (roots: -1)."""
    par = np.full(W * H, -1, np.int32)
    pix, parent = t["node_pix"], t["node_parent"]
    roots = set(int(x) for x in t["tree_start"][:-1])
    for n in range(W * H):
        if n not in roots:
            par[pix[n]] = pix[parent[n]]
    return par


@pytest.mark.parametrize("name", ["rand_37x23", "smooth_97x61", "flir_crop_256x192", "const_16x12", "col_1x15"])
@pytest.mark.parametrize("c,min_size", SEG)
def test_segment_forest_tree(gpu_ctx, name, c, min_size):
    """The GPU path's forest (host segmentation, virtual links removed) and per-tree rooting against
    the oracle's segmentation and BFS (each tree rooted at its first raster pixel)."""
    import stereomatch_amd as sm
    z = load_case(name)
    H, W, _ = z["left"].shape
    for v in ("left", "right"):
        t = gpu_ctx.build_tree(z[v], sm.default_params(c=c, min_size=min_size))
        ot = O.build_tree(z[v], c, min_size)
        np.testing.assert_array_equal(t["mask"], ot["mask"])
        assert t["ntrees"] == ot["ntrees"]
        np.testing.assert_array_equal(t["parent_pix"], _forest_parent(W, H, ot))


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("c,min_size", SEG)
def test_segment_match_bitexact_golden(gpu_ctx, name, c, min_size):
    import stereomatch_amd as sm
    z = load_case(name)
    D = int(z["D"])
    out = gpu_ctx.match(z["left"], z["right"], D, sm.default_params(c=c, min_size=min_size))
    ref = O.match(z["left"], z["right"], D, c=c, min_size=min_size, nthreads=16)
    for v in ("left", "right"):
        np.testing.assert_array_equal(out[v]["idx"].ravel(), ref[v]["idx"])
        assert np.array_equal(bits(out[v]["minc"].ravel()), bits(ref[v]["minc"]))


@pytest.mark.parametrize("c,min_size", SEG)
def test_segment_aggregate_bitexact(gpu_ctx, c, min_size):
    """Every fp64 A_up / A value of the forest filter (4 slices), bitwise: virtual links carry S = 0,
    S2 = 1, so each tree's root gets A = A_up as in the reference."""
    import stereomatch_amd as sm
    W, H, d0, D = 320, 240, 30, 4
    left, right, _ = make_pair(W, H, 64, index=5)
    lv, rv = O.cost_agd(left, right, d0, d0 + D)
    for vi, (img, vol) in enumerate(((left, lv), (right, rv))):
        Aup, A = gpu_ctx.aggregate_debug(left, right, vi, d0, D, sm.default_params(c=c, min_size=min_size))
        r = O.tree_filter(W, H, O.build_tree(img, c, min_size), vol, d0, False, True, 16)
        assert np.array_equal(bits(Aup), bits(r["Aup"]))
        assert np.array_equal(bits(A), bits(r["A"]))


@pytest.mark.parametrize("W,H,D,c", [(320, 240, 64, 5000.0), (200, 150, 128, 5000.0), (160, 90, 256, 5000.0),
                                     (256, 160, 128, 800.0)])
def test_segment_match_bitexact_synthetic(gpu_ctx, knobs, W, H, D, c):
    """Segment mode at SPL 1 / 2 / 4 with short pieces (cut paths inside the trees)."""
    import stereomatch_amd as sm
    knobs.setenv("SM_PIECE_LEN", "64")
    left, right, _ = make_pair(W, H, D, index=7)
    out = gpu_ctx.match(left, right, D, sm.default_params(c=c, min_size=200))
    ref = O.match(left, right, D, c=c, min_size=200, nthreads=16)
    for v in ("left", "right"):
        np.testing.assert_array_equal(out[v]["idx"].ravel(), ref[v]["idx"])
        assert np.array_equal(bits(out[v]["minc"].ravel()), bits(ref[v]["minc"]))


@pytest.mark.parametrize("src,c,min_size", [("synth", 5000.0, 200), ("synth", 300.0, 20), ("synth", 40.0, 5),
                                            ("flir", 5000.0, 200), ("flir", 150.0, 50)])
def test_full_size_segment_forest(gpu_ctx, src, c, min_size):
    """The GPU segmentation (sm_seg_gpu.hip, bucket-synchronous Boruvka + host min-size merge) at full
    size: forest masks and tree count equal to the oracle's serial segment_graph + min-size merge, on a
    synthetic C2 view and on the FLIR pair's 2048x1536 left image (a broad weight histogram)."""
    import stereomatch_amd as sm
    if src == "synth":
        img, _, _ = make_pair(1920, 1200, 128, index=0)
    else:
        img = flir_pair()[0]
    H, W, _ = img.shape
    t = gpu_ctx.build_tree(img, sm.default_params(c=c, min_size=min_size))
    wR, wD = O.edge_weights(O.median3(img))
    mask, n = O.segment(W, H, wR, wD, c, min_size)
    np.testing.assert_array_equal(t["mask"], mask)
    assert t["ntrees"] == n


def test_full_size_c3_segment_forest_and_match(gpu_ctx):
    """BASELINE C3 size (3840x2160) in segment mode: the GPU segmentation's forest against the oracle's
    serial sweep, then a 32-slice match of the same pair bit-exact against the oracle's forest filter
    (the largest edge lists, bucket counts and sort keys of the GPU segmentation)."""
    import stereomatch_amd as sm
    W, H, d0, D = 3840, 2160, 96, 32
    left, right, _ = make_pair(W, H, 256, index=4)
    t = gpu_ctx.build_tree(left, sm.default_params(c=5000.0, min_size=200))
    wR, wD = O.edge_weights(O.median3(left))
    mask, n = O.segment(W, H, wR, wD, 5000.0, 200)
    np.testing.assert_array_equal(t["mask"], mask)
    assert t["ntrees"] == n
    out = gpu_ctx.match(left, right, D, sm.default_params(c=5000.0, min_size=200, disp_begin=d0, disp_total=d0 + D))
    lv, rv = O.cost_agd(left, right, d0, d0 + D)
    for v, img, vol in (("left", left, lv), ("right", right, rv)):
        r = O.tree_filter(W, H, O.build_tree(img, 5000.0, 200), vol, d0, True, False, 16)
        np.testing.assert_array_equal(out[v]["idx"].ravel(), r["idx"])
        assert np.array_equal(bits(out[v]["minc"].ravel()), bits(r["minc"]))


@pytest.mark.parametrize("env", [{"SM_SEG_SMALL": "0"}, {"SM_SEG_SMALL": "0", "SM_SEG_GLOBAL_ROUNDS": "0"},
                                 {"SM_SEG_SMALL": "100000000"}, {"SM_SEG_GLOBAL_ROUNDS": "7"}, {"SM_SEG_HOST": "1"},
                                 {"SM_SEG_FLATTEN": "0"}, {"SM_SEG_FLATTEN": "3"},
                                 {"SM_SEG_NOSPLIT": "1"}, {"SM_SEG_NORUN": "1"}, {"SM_SEG_NORUN": "1", "SM_SEG_ACT_MAX": "0"},
                                 {"SM_SEG_TAIL_GLOBAL": "1"}, {"SM_SEG_GLOBAL_ROUNDS": "1"},
                                 {"SM_SEG_TAIL_MIN": "0"}, {"SM_SEG_TAIL_MIN": "0", "SM_SEG_GLOBAL_ROUNDS": "1"}])
def test_segment_forest_schedules(gpu_ctx, knobs, env):
    """The GPU segmentation's launch schedules give the same forest: every bucket over the whole GPU
    (with and without global Boruvka rounds before the one-workgroup tail), every bucket in one
    workgroup, more global rounds; the host sweep (SM_SEG_HOST); no root flattening, or flattening
    before every bucket (SM_SEG_FLATTEN); small-bucket runs without the k_seg_split pre-pass
    (SM_SEG_NOSPLIT), or with it but without the LDS-resident run (SM_SEG_NORUN: k_seg_small over the
    LDS-bucketed active edges, or with SM_SEG_ACT_MAX=0 the full scan, which skips the edges the pre-pass
    rejected); the big buckets' tails by global-memory rounds instead of the LDS rounds (SM_SEG_TAIL_GLOBAL),
    or after one global round (SM_SEG_GLOBAL_ROUNDS=1: larger tails), or in LDS whatever their length
    (SM_SEG_TAIL_MIN=0; the default keeps lists under 256 edges on the global rounds).  (The pair
    dedupe's sort fallback, for tables that do not fit, runs on the smallest golden images.)"""
    import stereomatch_amd as sm
    for k, val in env.items():
        knobs.setenv(k, val)
    img, _, _ = make_pair(640, 480, 64, index=3)
    H, W, _ = img.shape
    wR, wD = O.edge_weights(O.median3(img))
    for c, ms in ((5000.0, 200), (120.0, 30)):
        t = gpu_ctx.build_tree(img, sm.default_params(c=c, min_size=ms))
        mask, n = O.segment(W, H, wR, wD, c, ms)
        np.testing.assert_array_equal(t["mask"], mask)
        assert t["ntrees"] == n


def test_full_size_c2_segment_match_bitexact(gpu_ctx):
    """1920x1200 D=128 in Stereo3DMST's own segment mode (c = 5000, min_size = 200; :831-832)."""
    import stereomatch_amd as sm
    W, H, D = 1920, 1200, 128
    left, right, _ = make_pair(W, H, D, index=0)
    out = gpu_ctx.match(left, right, D, sm.default_params(c=5000.0, min_size=200))
    ref = O.match(left, right, D, c=5000.0, min_size=200, nthreads=16)
    for v in ("left", "right"):
        assert ref[v]["tree"]["ntrees"] > 1
        np.testing.assert_array_equal(out[v]["idx"].ravel(), ref[v]["idx"])
        assert np.array_equal(bits(out[v]["minc"].ravel()), bits(ref[v]["minc"]))


# ---- subpixel WTA (SM_POST_SUBPIXEL; PatchMatchStereoGPU.cu:1726-1736) ----
@pytest.mark.parametrize("W,H,D", [(160, 120, 48), (200, 96, 100), (256, 128, 128), (128, 64, 200)])
def test_subpixel_bitexact(gpu_ctx, knobs, W, H, D):
    """Subpixel disparities of both views (SPL 1 / 2 / 4, cut paths through the chain engine and
    its repair walks) against the oracle's parabola over its own aggregated volumes; idx / min are
    the integral WTA's."""
    import stereomatch_amd as sm
    knobs.setenv("SM_PIECE_LEN", "64")
    left, right, _ = make_pair(W, H, D, index=9)
    out = gpu_ctx.match(left, right, D, sm.default_params(post=sm.SM_POST_SUBPIXEL))
    ref = O.match(left, right, D, want_volumes=True, nthreads=16)
    for v in ("left", "right"):
        np.testing.assert_array_equal(out[v]["idx"].ravel(), ref[v]["idx"])
        assert np.array_equal(bits(out[v]["minc"].ravel()), bits(ref[v]["minc"]))
        exp = O.subpixel(ref[v]["A"], ref[v]["idx"], 0, D)
        np.testing.assert_array_equal(out[v]["disp"].ravel(), exp)
        assert np.count_nonzero(exp != ref[v]["idx"].astype(np.float32)) > 0


@pytest.mark.parametrize("d0,D,Dt", [(0, 32, 96), (32, 32, 96), (64, 32, 96), (40, 30, 100)])
def test_subpixel_shard_halo_with_reduce(d0, D, Dt):
    """A subpixel shard through a one-rank communicator: the shard computes a 1-slice halo on each
    inner side, the WTA covers [d0, d0+D) only, the parabola of its winner uses the halo slices, and
    the 64-bit (index, disparity) exchange carries the disparity (stage_reduce)."""
    import stereomatch_amd as sm
    W, H = 180, 120
    left, right, _ = make_pair(W, H, Dt, index=11)
    ctx = sm.Context(0)
    try:
        ctx.comm_init(1, 0, sm.Context.unique_id())
        out = ctx.match(left, right, D, sm.default_params(disp_begin=d0, disp_total=Dt, post=sm.SM_POST_SUBPIXEL))
    finally:
        ctx.close()
    lo, hi = max(0, d0 - 1), min(Dt, d0 + D + 1)
    lv, rv = O.cost_agd(left, right, lo, hi)
    for v, img, vol in (("left", left, lv), ("right", right, rv)):
        r = O.tree_filter(W, H, O.build_tree(img), vol, lo, False, True, 16)
        A = r["A"]
        sh = A[d0 - lo:d0 - lo + D].reshape(D, -1)
        am = np.argmin(sh, axis=0)  # first minimum over the shard = strict-< over ascending d
        idx = (d0 + am).astype(np.int32)
        np.testing.assert_array_equal(out[v]["idx"].ravel(), idx)
        np.testing.assert_array_equal(out[v]["disp"].ravel(), O.subpixel(A, idx, lo, Dt))


# ---- 32-slice rows (Dpad = 32 for calls of <= 32 slices: a C4 shard moves 32 slices of rows) ----
@pytest.mark.parametrize("W,H,D,plen", [(320, 240, 32, "64"), (256, 160, 17, "64"), (200, 150, 32, None)])
def test_dpad32_match_bitexact(gpu_ctx, knobs, W, H, D, plen):
    """Calls of <= 32 slices use 32-double rows (lanes 32..63 load nothing, store nothing): matches
    with cut paths (fast and forced-slow repair) against the oracle, bitwise."""
    if plen:
        knobs.setenv("SM_PIECE_LEN", plen)
    left, right, _ = make_pair(W, H, D, index=12)
    ref = O.match(left, right, D, nthreads=16)
    for rmax in (None, "1"):
        if rmax:
            knobs.setenv("SM_REPAIR_MAX", rmax)
        out = gpu_ctx.match(left, right, D)
        for v in ("left", "right"):
            np.testing.assert_array_equal(out[v]["idx"].ravel(), ref[v]["idx"])
            assert np.array_equal(bits(out[v]["minc"].ravel()), bits(ref[v]["minc"]))


def test_dpad32_volume_ingest_and_rows(gpu_ctx, knobs):
    """MC-CNN volume rows and every A_up / A value at 32-slice rows, with 64-node pieces."""
    import stereomatch_amd as sm
    knobs.setenv("SM_PIECE_LEN", "64")
    W, H, D, d0 = 240, 160, 30, 2
    left, right, _ = make_pair(W, H, 64, index=13)
    lv, rv = _mccnn_like(40, H, W, 7), _mccnn_like(40, H, W, 8)
    gpu_ctx.upload_cost_volumes(lv, rv)
    out = gpu_ctx.match(left, right, D, sm.default_params(cost_kind=sm.SM_COST_VOLUME, disp_begin=d0))
    for v, img, vol in (("left", left, lv), ("right", right, rv)):
        r = O.tree_filter(W, H, O.build_tree(img), O.mccnn_clamp(vol[d0:d0 + D]), d0, True, False, 16)
        np.testing.assert_array_equal(out[v]["idx"].ravel(), r["idx"])
        assert np.array_equal(bits(out[v]["minc"].ravel()), bits(r["minc"]))
    cl, cr = O.cost_agd(left, right, 5, 5 + 20)
    for vi, (img, vol) in enumerate(((left, cl), (right, cr))):
        Aup, A = gpu_ctx.aggregate_debug(left, right, vi, 5, 20)
        r = O.tree_filter(W, H, O.build_tree(img), vol, 5, False, True, 16)
        assert np.array_equal(bits(Aup), bits(r["Aup"]))
        assert np.array_equal(bits(A), bits(r["A"]))


# ---- guided-filter aggregator (SM_AGG_GUIDED; PatchMatchStereoGPU.cu:8251-8470) ----
@pytest.mark.parametrize("W,H,D,rad", [(160, 120, 32, 9), (203, 97, 48, 4), (70, 33, 40, 9), (256, 64, 100, 9)])
@pytest.mark.parametrize("sub", [False, True])
def test_guided_match_bitexact(gpu_ctx, W, H, D, rad, sub):
    """The colour guided filter of the AGD cost (each view guided by its own image) + selectDisparity,
    against the oracle's literal float restatement: indices, minima and disparities bitwise (ragged
    32-pixel blocks, batches of 32 slices with a partial last one, radius 4 and 9)."""
    import stereomatch_amd as sm
    left, right, _ = make_pair(W, H, D, index=14)
    post = sm.SM_POST_SUBPIXEL if sub else 0
    out = gpu_ctx.match(left, right, D, sm.default_params(aggregator=sm.SM_AGG_GUIDED, gf_radius=rad, post=post))
    ref = O.guided_match(left, right, D, radius=rad, sub=sub, nthreads=16)
    for v in ("left", "right"):
        np.testing.assert_array_equal(out[v]["idx"].ravel(), ref[v]["idx"])
        np.testing.assert_array_equal(out[v]["minc"].ravel(), ref[v]["minc"].astype(np.float64))
        np.testing.assert_array_equal(out[v]["disp"].ravel(), ref[v]["disp"])


def test_guided_match_full_size_c2(gpu_ctx):
    """1920x1200 D=128 through the guided aggregator, bitwise against the oracle."""
    import stereomatch_amd as sm
    W, H, D = 1920, 1200, 128
    left, right, _ = make_pair(W, H, D, index=0)
    out = gpu_ctx.match(left, right, D, sm.default_params(aggregator=sm.SM_AGG_GUIDED, post=sm.SM_POST_SUBPIXEL))
    ref = O.guided_match(left, right, D, sub=True, nthreads=16)
    for v in ("left", "right"):
        np.testing.assert_array_equal(out[v]["idx"].ravel(), ref[v]["idx"])
        np.testing.assert_array_equal(out[v]["disp"].ravel(), ref[v]["disp"])


def test_guided_direct_x_pass(gpu_ctx, knobs):
    """The direct x box pass (the path for rows too wide for the LDS tile) gives the same bits as the
    LDS-tiled one; a 7 px wide and a 1 px high image exercise the tile edges."""
    import stereomatch_amd as sm
    for W, H, D in ((203, 97, 24), (7, 40, 4), (90, 1, 16)):
        left, right, _ = make_pair(W, H, D, index=3)
        p = sm.default_params(aggregator=sm.SM_AGG_GUIDED, gf_radius=5, post=sm.SM_POST_SUBPIXEL)
        a = gpu_ctx.match(left, right, D, p)
        knobs.setenv("SM_GF_DIRECT_X", "1")
        b = gpu_ctx.match(left, right, D, p)
        knobs.delenv("SM_GF_DIRECT_X")
        ref = O.guided_match(left, right, D, radius=5, sub=True, nthreads=16)
        for v in ("left", "right"):
            np.testing.assert_array_equal(a[v]["idx"].ravel(), ref[v]["idx"])
            np.testing.assert_array_equal(a[v]["disp"].ravel(), ref[v]["disp"])
            np.testing.assert_array_equal(b[v]["idx"], a[v]["idx"])
            np.testing.assert_array_equal(b[v]["disp"], a[v]["disp"])


def test_guided_fused_tiles_match_unfused(gpu_ctx, knobs):
    """Radius 9 with W % 4 == 0 runs the fused tile kernels (k_gf_box1_ab / k_gf_box2_q / k_gf_wta);
    SM_GF_UNFUSED=1 (and any other width or radius) the unfused chain.  Same bits, and the oracle's, on
    images narrower than a tile, one row high, ragged in both 32-pixel block directions, and with
    partial slice batches."""
    import stereomatch_amd as sm
    for W, H, D in ((8, 40, 4), (92, 1, 16), (204, 97, 40), (68, 33, 33), (132, 70, 24), (7, 20, 8)):
        left, right, _ = make_pair(W, H, D, index=5)
        p = sm.default_params(aggregator=sm.SM_AGG_GUIDED, post=sm.SM_POST_SUBPIXEL)
        a = gpu_ctx.match(left, right, D, p)
        knobs.setenv("SM_GF_UNFUSED", "1")
        b = gpu_ctx.match(left, right, D, p)
        knobs.delenv("SM_GF_UNFUSED")
        ref = O.guided_match(left, right, D, sub=True, nthreads=16)
        for v in ("left", "right"):
            np.testing.assert_array_equal(a[v]["idx"].ravel(), ref[v]["idx"])
            np.testing.assert_array_equal(a[v]["minc"].ravel(), ref[v]["minc"].astype(np.float64))
            np.testing.assert_array_equal(a[v]["disp"].ravel(), ref[v]["disp"])
            for k in ("idx", "minc", "disp"):
                np.testing.assert_array_equal(b[v][k], a[v][k])


def test_guided_errors(gpu_ctx):
    import stereomatch_amd as sm
    left, right, _ = make_pair(40, 30, 8)
    for bad in (dict(gf_radius=0), dict(gf_eps=0.0), dict(cost_kind=sm.SM_COST_VOLUME),
                dict(post=sm.SM_POST_SUBPIXEL, disp_begin=2, disp_total=16)):
        with pytest.raises(sm.StereoMSTError):
            gpu_ctx.match(left, right, 8, sm.default_params(aggregator=sm.SM_AGG_GUIDED, **bad))


def test_split_calls_interleaved_bitexact():
    """sm_match_begin / sm_match_finish interleaved over two contexts (frame i+1's tree enqueued
    before frame i's filter, as bench.py streams frames) give the oracle's answer bitwise; a
    finish without a begin and a second begin are SM_ERR_STATE."""
    import stereomatch_amd as sm
    from stereomatch_amd._lib import SM_ERR_STATE, StereoMSTError
    pairs = [make_pair(256, 160, D, index=i) for i, D in ((3, 64), (4, 128))]
    ctxs = [sm.Context(0), sm.Context(0)]
    try:
        for c, (l, r, _) in zip(ctxs, pairs):
            c.upload(l, r)
        Ds = (64, 128)
        ctxs[0].match_begin(Ds[0])
        ctxs[1].match_begin(Ds[1])
        with pytest.raises(StereoMSTError) as e:
            ctxs[1].match_begin(Ds[1])
        assert e.value.status == SM_ERR_STATE
        # every entry point that would read or replace the begun call's state refuses until its finish
        l0, r0, _ = pairs[0]
        for call in (ctxs[0].synchronize, ctxs[0].results, lambda: ctxs[0].upload(l0, r0),
                     lambda: ctxs[0].cost_volume(l0, r0, 0, 8), lambda: ctxs[0].build_tree(l0),
                     lambda: ctxs[0].aggregate_debug(l0, r0, 0, 0, 4),
                     lambda: ctxs[0].upload_cost_volumes(np.zeros((2, 160, 256), np.float32), np.zeros((2, 160, 256), np.float32))):
            with pytest.raises(StereoMSTError) as e:
                call()
            assert e.value.status == SM_ERR_STATE
        ctxs[0].match_finish()
        ctxs[1].match_finish()
        with pytest.raises(StereoMSTError) as e:
            ctxs[0].match_finish()
        assert e.value.status == SM_ERR_STATE
        for c, (l, r, _), D in zip(ctxs, pairs, Ds):
            c.synchronize()
            out = c.results()
            ref = O.match(l, r, D, nthreads=16)
            for v in ("left", "right"):
                np.testing.assert_array_equal(out[v]["idx"].ravel(), ref[v]["idx"])
                assert np.array_equal(bits(out[v]["minc"].ravel()), bits(ref[v]["minc"]))
    finally:
        for c in ctxs:
            c.close()


def test_guided_subpixel_with_one_rank_comm():
    """SM_AGG_GUIDED + SM_POST_SUBPIXEL on a context with a (one-rank) communicator: the exchange carries
    the guided WTA's subpixel disparities (64-bit candidates), so the result equals the call without one."""
    import stereomatch_amd as sm
    left, right, _ = make_pair(160, 96, 32, index=2)
    p = sm.default_params(aggregator=sm.SM_AGG_GUIDED, post=sm.SM_POST_SUBPIXEL, disp_total=32)
    ctx = sm.Context(0)
    try:
        ref = ctx.match(left, right, 32, p)
        ctx.comm_init(1, 0, sm.Context.unique_id())
        out = ctx.match(left, right, 32, p)
        for v in ("left", "right"):
            np.testing.assert_array_equal(out[v]["disp"], ref[v]["disp"])
            np.testing.assert_array_equal(out[v]["idx"], ref[v]["idx"])
            assert np.array_equal(bits(out[v]["minc"].ravel()), bits(ref[v]["minc"].ravel()))
        assert not np.array_equal(out["left"]["disp"], out["left"]["idx"].astype(np.float32))  # subpixel survived
    finally:
        ctx.close()


@pytest.mark.timeout(600)
def test_segment_mode_begin_on_many_contexts_bitexact():
    """Segment mode (c finite) with begin/finish interleaved over 4 contexts, as bench.py streams segment
    frames (lag inflight - 2): every context's segmentation runs on its own worker thread concurrently
    (hipcub sorts, host waits, pinned min-size buffers of several contexts at once) before any finish.
    Each frame's forest and match against the oracle's serial segment_graph + min-size merge."""
    import stereomatch_amd as sm
    cases = [(320, 200, 48, 5000.0, 200, 1), (288, 176, 64, 300.0, 20, 2), (320, 200, 32, 5000.0, 200, 3),
             (256, 160, 48, 40.0, 5, 4)]
    ctxs = [sm.Context(0) for _ in cases]
    try:
        pairs = []
        for c, (W, H, D, cc, ms, idx) in zip(ctxs, cases):
            l, r, _ = make_pair(W, H, D, index=idx)
            pairs.append((l, r))
            c.upload(l, r)
        for c, (W, H, D, cc, ms, idx) in zip(ctxs, cases):
            c.match_begin(D, sm.default_params(c=cc, min_size=ms))
        for c in ctxs:
            c.match_finish()
        for c, (l, r), (W, H, D, cc, ms, idx) in zip(ctxs, pairs, cases):
            c.synchronize()
            out = c.results()
            ref = O.match(l, r, D, c=cc, min_size=ms, nthreads=16)
            for v in ("left", "right"):
                np.testing.assert_array_equal(out[v]["idx"].ravel(), ref[v]["idx"], err_msg="%dx%d c=%g %s" % (W, H, cc, v))
                assert np.array_equal(bits(out[v]["minc"].ravel()), bits(ref[v]["minc"]))
    finally:
        for c in ctxs:
            c.close()
