"""GPU parity of MST_PMS (SM_AGG_PMS), Stereo3DMST's slanted-plane label search
(src/Stereo3DMST.cpp:546-629, driven at :851-889), through the C-ABI against the oracle's serial
restatement (oracle/sm_oracle_pms.c).  Labels (a, b, c), the per-pixel aggregated minima and the
plane disparities are compared BIT-EXACT after 1 and 3 calls per view, in both device modes (the
first call of a view serial, later calls speculative with validation; SM_PMS_SERIAL=1 runs every
call serially)."""
import numpy as np
import pytest

import stereomatch_amd as sm
from conftest import golden_cases, load_case
from oracle import oracle as O
from tools.synth import make_pair

pytestmark = pytest.mark.gpu


def u32(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def u64(a):
    return np.ascontiguousarray(a, dtype=np.float64).view(np.uint64)


def run_gpu(ctx, left, right, D, iters, c=5000.0, min_size=200, post=0, vols=None):
    p = sm.default_params(aggregator=sm.SM_AGG_PMS, c=c, min_size=min_size, pms_iters=iters, post=post,
                          disp_total=D)
    if vols is not None:
        ctx.upload_cost_volumes(*vols)
        p.cost_kind = sm.SM_COST_VOLUME
    out = ctx.match(left, right, D, p)
    return out, ctx.labels(), ctx.pms_stats()


def check_view(out, labs, ref, v):
    np.testing.assert_array_equal(u32(labs[v]), u32(ref[v]["abc"]), err_msg="%s labels" % v)
    np.testing.assert_array_equal(u64(out[v]["minc"].ravel()), u64(ref[v]["minc"]), err_msg="%s minima" % v)
    np.testing.assert_array_equal(u32(out[v]["disp"].ravel()), u32(plane_disp(ref[v]["abc"], out[v]["disp"].shape)),
                                  err_msg="%s plane disparities" % v)
    assert (out[v]["idx"] == -1).all()


def plane_disp(abc, shape):
    H, W = shape
    return O.pms_plane_disp(abc, W, H).ravel()


SMALL = [n for n in golden_cases() if n in ("smooth_64x48", "rand_37x23", "smooth_97x61", "const_16x12")]


@pytest.mark.parametrize("name", SMALL)
@pytest.mark.parametrize("c,min_size", [(5000.0, 200), (300.0, 20)])
@pytest.mark.parametrize("iters", [1, 3])
def test_pms_golden_bitexact(gpu_ctx, name, c, min_size, iters):
    z = load_case(name)
    D = int(z["D"])
    ref = O.stereo3dmst_pms(z["left"], z["right"], D, iters=iters, c=c, min_size=min_size)
    out, labs, st = run_gpu(gpu_ctx, z["left"], z["right"], D, iters, c, min_size)
    for v in ("left", "right"):
        check_view(out, labs, ref, v)
    assert st["iters"] == iters and st["ntrees"] == [ref["left"]["tree"]["ntrees"], ref["right"]["tree"]["ntrees"]]


@pytest.mark.parametrize("mode", ["spec", "serial", "chain48", "nsu4", "nsu8"])
def test_pms_synthetic_modes_bitexact(gpu_ctx, knobs, mode):
    """Many trees (c=300, min_size 20) and 4 calls: the speculative passes meet stale inputs (one
    tree re-run serially, later trees kept and re-validated, higher neighbours sampled from the
    call's starting labels) and wrong offsets (a new pass); SM_PMS_SERIAL=1 is the plain serial order;
    SM_PMS_CHAIN_MIN=48 sends paths of >= 48 rows to the chain kernel; SM_PMS_CHAIN_NSU=4 / 8 gives the
    up chain that many ring slots (default 6)."""
    knobs.setenv("SM_PMS_SERIAL", "1" if mode == "serial" else "0")
    if mode in ("chain48", "nsu4", "nsu8"):
        knobs.setenv("SM_PMS_CHAIN_MIN", "48")  # (more chain items at this size)
    else:
        knobs.delenv("SM_PMS_CHAIN_MIN", raising=False)
    if mode in ("nsu4", "nsu8"):
        knobs.setenv("SM_PMS_CHAIN_NSU", mode[3:])
    else:
        knobs.delenv("SM_PMS_CHAIN_NSU", raising=False)
    left, right, _ = make_pair(160, 120, 48, index=3)
    ref = O.stereo3dmst_pms(left, right, 48, iters=4, c=300.0, min_size=20)
    out, labs, st = run_gpu(gpu_ctx, left, right, 48, 4, 300.0, 20)
    for v in ("left", "right"):
        check_view(out, labs, ref, v)
    if mode != "serial":
        assert st["spec_rounds"] >= 6  # calls 2..4 of both views: one pass each at least
        assert st["serial_trees"] > 2 * ref["left"]["tree"]["ntrees"] - 50  # first calls + the failures


@pytest.mark.parametrize("piece,serial", [("16", "0"), ("8", "1"), ("64", "0"), ("8", "0")])
def test_pms_pieces_bitexact(gpu_ctx, knobs, piece, serial):
    """Long heavy paths cut into pieces of SM_PMS_PIECE rows: every piece runs from a guessed input; the
    parallel repair (k_pms_repair_par) re-walks every piece at once from its neighbour's boundary row until
    the rows agree, and the gated sequential pass redoes the cuts where a piece's repair rewrote the row
    its neighbour started from (8-row pieces mostly re-walk whole pieces, so they take it).  First call serial (cut trees take the whole-GPU launches), later
    calls speculative; SM_PMS_SERIAL=1 all serial."""
    knobs.setenv("SM_PMS_PIECE", piece)
    knobs.setenv("SM_PMS_SERIAL", serial)
    left, right, _ = make_pair(192, 128, 48, index=7)
    ref = O.stereo3dmst_pms(left, right, 48, iters=3, c=5000.0, min_size=200)
    out, labs, st = run_gpu(gpu_ctx, left, right, 48, 3, 5000.0, 200)
    for v in ("left", "right"):
        check_view(out, labs, ref, v)


def test_pms_many_trees_bitexact(gpu_ctx):
    """79k trees (c=5, min_size 2): the speculative offset chain (k_pms_guess) too large to stage its
    per-tree values in LDS takes them from global memory."""
    left, right, _ = make_pair(640, 480, 32, index=9)
    ref = O.stereo3dmst_pms(left, right, 32, iters=2, c=5.0, min_size=2)
    assert ref["left"]["tree"]["ntrees"] > 20000
    out, labs, st = run_gpu(gpu_ctx, left, right, 32, 2, 5.0, 2)
    for v in ("left", "right"):
        check_view(out, labs, ref, v)
    assert st["spec_rounds"] >= 2


def test_pms_max_rounds_fallback(gpu_ctx, knobs):
    """SM_PMS_MAX_ROUNDS=1: a call whose first speculative pass fails finishes in serial order."""
    knobs.setenv("SM_PMS_MAX_ROUNDS", "1")
    left, right, _ = make_pair(128, 96, 40, index=4)
    ref = O.stereo3dmst_pms(left, right, 40, iters=3, c=200.0, min_size=10)
    out, labs, _ = run_gpu(gpu_ctx, left, right, 40, 3, 200.0, 10)
    for v in ("left", "right"):
        check_view(out, labs, ref, v)


def test_pms_mccnn_volumes_bitexact(gpu_ctx):
    """MC-CNN ingest (:764-803) as the data term: NaNs and values above the clamp."""
    left, right, _ = make_pair(96, 64, 32, index=5)
    rng = np.random.default_rng(7)
    vols = [rng.uniform(-0.2, 0.8, (32, 64, 96)).astype(np.float32) for _ in range(2)]
    for v in vols:
        v[rng.uniform(size=v.shape) < 0.01] = np.nan
    ref = O.stereo3dmst_pms(left, right, 32, iters=2, vols=[O.mccnn_clamp(v) for v in vols], c=500.0, min_size=30)
    out, labs, _ = run_gpu(gpu_ctx, left, right, 32, 2, 500.0, 30, vols=vols)
    for v in ("left", "right"):
        check_view(out, labs, ref, v)


def test_pms_output_step(gpu_ctx):
    """stereo3dmst's output step on the plane labels: LabelToDisp + *= (Dmax-1.f), then the L-R check of
    the left map (:189-201, :900-904)."""
    left, right, _ = make_pair(128, 80, 40, index=6)
    D = 40
    ref = O.stereo3dmst_pms(left, right, D, iters=2, c=1000.0, min_size=50)
    out, labs, _ = run_gpu(gpu_ctx, left, right, D, 2, 1000.0, 50, post=sm.STEREO3DMST_POST)
    np.testing.assert_array_equal(u32(out["right"]["disp"]), u32(ref["right"]["disp"]))
    np.testing.assert_array_equal(u32(out["left"]["disp"]), u32(ref["left"]["disp_checked"]))


def test_pms_bad_params(gpu_ctx):
    left, right, _ = make_pair(32, 24, 16, index=1)
    for kw in (dict(disp_begin=4), dict(views=1), dict(post=sm.SM_POST_SUBPIXEL), dict(pms_iters=-1)):
        p = sm.default_params(aggregator=sm.SM_AGG_PMS, c=100.0, min_size=10, pms_iters=1)
        for k, val in kw.items():
            setattr(p, k, val)
        with pytest.raises(sm.StereoMSTError) as e:
            gpu_ctx.match(left, right, 16, p)
        assert e.value.status == 1
    with pytest.raises(sm.StereoMSTError) as e:  # labels after a non-PMS call
        gpu_ctx.match(left, right, 16)
        gpu_ctx.labels()
    assert e.value.status == 5


def test_pms_forest_cycle_is_an_error(gpu_ctx, knobs):
    """Masks that are not a forest (SM_TEST_PMS_CYCLE=1 turns the square of pixels 0, 1, W, W + 1 into
    four real edges) are refused before any Euler tour -- whose list ranking would never end -- with
    SM_ERR_STATE; the next call on the same context is exact again."""
    left, right, _ = make_pair(96, 64, 24, index=2)
    knobs.setenv("SM_TEST_PMS_CYCLE", "1")
    with pytest.raises(sm.StereoMSTError, match="cycle") as e:
        run_gpu(gpu_ctx, left, right, 24, 1, 300.0, 20)
    assert e.value.status == 5
    knobs.delenv("SM_TEST_PMS_CYCLE")
    ref = O.stereo3dmst_pms(left, right, 24, iters=1, c=300.0, min_size=20)
    out, labs, st = run_gpu(gpu_ctx, left, right, 24, 1, 300.0, 20)
    for v in ("left", "right"):
        check_view(out, labs, ref, v)


@pytest.mark.timeout(600)
def test_pms_full_c2_one_call_bitexact(gpu_ctx):
    """Full C2 (1920x1200, Dmax 128), the reference's segment mode (c=5000, min_size 200), one MST_PMS
    call per view."""
    left, right, _ = make_pair(1920, 1200, 128, index=0)
    ref = O.stereo3dmst_pms(left, right, 128, iters=1, c=5000.0, min_size=200)
    out, labs, st = run_gpu(gpu_ctx, left, right, 128, 1)
    for v in ("left", "right"):
        np.testing.assert_array_equal(u32(labs[v]), u32(ref[v]["abc"]))
        np.testing.assert_array_equal(u64(out[v]["minc"].ravel()), u64(ref[v]["minc"]))


def test_pms_reference_surface_100_calls(gpu_ctx):
    """The Python mirror of stereo3dmst() with the reference's own algorithm and constants (c=5000,
    min_size 200, 100 MST_PMS calls per view, Stereo3DMST.cpp:830-832, 854) against the oracle."""
    left, right, _ = make_pair(128, 96, 48, index=8)
    sm.startTimer()
    ld, rd = sm.stereo3dmst("l.png", "r.png", left, right, "AGD", 48)
    assert sm.getTimer() >= 0
    ref = O.stereo3dmst_pms(left, right, 48, iters=100)
    np.testing.assert_array_equal(u32(ld), u32(ref["left"]["disp_checked"]))
    np.testing.assert_array_equal(u32(rd), u32(ref["right"]["disp"]))


_FULL_C2_REF = {}


@pytest.mark.timeout(900)
@pytest.mark.parametrize("chain_min", [None, "48"])
def test_pms_full_c2_speculative_bitexact(gpu_ctx, knobs, chain_min):
    """Full C2 (1920x1200, Dmax 128), c=5000, min_size 200, THREE MST_PMS calls per view: calls 2-3 take
    the speculative path (guessed offsets, every tree at once, validation, single-tree repairs) with the
    default 512-row pieces, propagation dedupe and whole-GPU launches -- the mode the reference's 99 later
    calls per view run in (Stereo3DMST.cpp:546-629, 854-889).  Labels, fp64 minima and plane disparities
    bitwise against the oracle's serial restatement.  chain_min 48: paths of >= 48 rows on the chain kernel
    (SM_PMS_CHAIN_MIN)."""
    for k in ("SM_PMS_SERIAL", "SM_PMS_PIECE", "SM_PMS_MAX_ROUNDS", "SM_PMS_CHAIN_MIN"):
        knobs.delenv(k, raising=False)
    if chain_min:
        knobs.setenv("SM_PMS_CHAIN_MIN", chain_min)
    left, right, _ = make_pair(1920, 1200, 128, index=0)
    if "ref" not in _FULL_C2_REF:  # the oracle's three calls once for both cases
        _FULL_C2_REF["ref"] = O.stereo3dmst_pms(left, right, 128, iters=3, c=5000.0, min_size=200)
    ref = _FULL_C2_REF["ref"]
    out, labs, st = run_gpu(gpu_ctx, left, right, 128, 3)
    for v in ("left", "right"):
        check_view(out, labs, ref, v)
    assert st["spec_rounds"] >= 4  # calls 2..3 of both views: at least one speculative pass each
    assert st["ntrees"] == [ref["left"]["tree"]["ntrees"], ref["right"]["tree"]["ntrees"]]


@pytest.mark.timeout(900)
def test_pms_flir_c1_two_calls_output_step(gpu_ctx, knobs):
    """BASELINE config C1's pair (FLIR 000020, 2048x1536, Dmax 64), the reference's own constants, two
    MST_PMS calls per view (the second speculative) and stereo3dmst's output step (LabelToDisp, *= Dmax-1,
    L-R check of the left map; :189-201, :900-904), bitwise against the oracle."""
    from conftest import flir_pair
    for k in ("SM_PMS_SERIAL", "SM_PMS_PIECE", "SM_PMS_MAX_ROUNDS"):
        knobs.delenv(k, raising=False)
    L, R = flir_pair()
    D = 64
    ref = O.stereo3dmst_pms(L, R, D, iters=2, c=5000.0, min_size=200)
    out, labs, st = run_gpu(gpu_ctx, L, R, D, 2, post=sm.STEREO3DMST_POST)
    for v in ("left", "right"):
        np.testing.assert_array_equal(u32(labs[v]), u32(ref[v]["abc"]), err_msg="%s labels" % v)
        np.testing.assert_array_equal(u64(out[v]["minc"].ravel()), u64(ref[v]["minc"]), err_msg="%s minima" % v)
    np.testing.assert_array_equal(u32(out["right"]["disp"].ravel()), u32(ref["right"]["disp"].ravel()))
    np.testing.assert_array_equal(u32(out["left"]["disp"].ravel()), u32(ref["left"]["disp_checked"].ravel()))
    assert st["spec_rounds"] >= 2


@pytest.mark.timeout(600)
@pytest.mark.parametrize("case", ["golden5000", "golden300", "synth300", "many_trees", "pieces16", "mst_mode", "one_pixel",
                                  "full_c2"])
def test_pms_gpu_forest_matches_host_build(gpu_ctx, knobs, case):
    """The schedule forest built on the GPU (sm_pms_forest.hip: union-find tree numbering, the level-order
    BFS of every tree, heavy paths, rows, tree graph, round lists) against the host construction
    (pms_build_forest), array by array (SM_PMS_FOREST_CHECK=1 makes the call fail on any difference), then
    the call's labels against the oracle.  "one_pixel": a 1 x 1 image, the only forest of single-pixel trees
    the reference's min-size merge (min_size >= 2, Stereo3DMST.cpp:293) lets through (N - K == 0: no tour)."""
    knobs.setenv("SM_PMS_FOREST_CHECK", "1")
    knobs.delenv("SM_PMS_HOST_FOREST", raising=False)
    if case == "pieces16":
        knobs.setenv("SM_PMS_PIECE", "16")
    else:
        knobs.delenv("SM_PMS_PIECE", raising=False)
    if case.startswith("golden"):
        z = load_case("smooth_97x61")
        left, right, D = z["left"], z["right"], int(z["D"])
        c, ms = (5000.0, 200) if case == "golden5000" else (300.0, 20)
    elif case == "synth300":
        (left, right, _), D, c, ms = make_pair(160, 120, 48, index=3), 48, 300.0, 20
    elif case == "many_trees":
        (left, right, _), D, c, ms = make_pair(640, 480, 32, index=9), 32, 5.0, 2
    elif case == "pieces16":
        (left, right, _), D, c, ms = make_pair(192, 128, 48, index=7), 48, 5000.0, 200
    elif case == "one_pixel":
        rng = np.random.default_rng(5)
        left, right = (rng.integers(0, 256, (1, 1, 3), dtype=np.uint8) for _ in range(2))
        D, c, ms = 4, 5000.0, 200
    elif case == "mst_mode":
        (left, right, _), D, c, ms = make_pair(200, 150, 32, index=2), 32, float("inf"), 200
    else:
        (left, right, _), D, c, ms = make_pair(1920, 1200, 128, index=0), 128, 5000.0, 200
    iters = 1 if case == "full_c2" else 2
    ref = O.stereo3dmst_pms(left, right, D, iters=iters, c=c, min_size=ms)
    out, labs, st = run_gpu(gpu_ctx, left, right, D, iters, c, ms)
    for v in ("left", "right"):
        check_view(out, labs, ref, v)
